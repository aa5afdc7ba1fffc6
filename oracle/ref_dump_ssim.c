/*
 * ref_dump_ssim.c -- SSIM golden-vector generator linked against the
 * UNMODIFIED reference objects (TEST INFRASTRUCTURE; built by oracle/Makefile
 * into oracle/_ref/, never shipped).
 *
 * Calls the reference's own createPredictionFrame (src/common/prediction_frame.c:3)
 * and findBestBlkSSIM (src/cpu/main_ssim.c:15) for every block,
 * single-threaded, and writes one record per block in raster order:
 *     int32 mvx, int32 mvy, float32 ssim     (little endian, 12 bytes)
 * main_ssim.c is compiled with -Dmain=reference_ssim_main; nothing else in
 * the reference is changed.  findBestMatchSSIM (src/common/ssim.c:83-108)
 * leaves the MV uninitialised when no candidate scores above 0; such blocks
 * are reported on stderr (count) so the generator can exclude those cases.
 *
 * usage: ref_dump_ssim <cur.yuv> <ref.yuv> <W> <H> <blk> <span> <out.bin>
 */
#include <stdio.h>
#include <stdlib.h>

#include "prediction_frame.h"
#include "utils.h"

float findBestBlkSSIM(predictionFrame pf, int* referenceFrame, block* blk, int extraSpan);

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: ref_dump_ssim cur ref W H blk span out.bin\n");
    return 2;
  }
  int W = atoi(argv[3]), H = atoi(argv[4]);
  int blk = atoi(argv[5]), span = atoi(argv[6]);
  int n = W * H;
  int* cur = (int*)malloc(sizeof(int) * (size_t)n);
  int* ref = (int*)malloc(sizeof(int) * (size_t)n);
  if (!yuvReadFrame(argv[1], cur, n) || !yuvReadFrame(argv[2], ref, n)) return 1;
  predictionFrame p;
  createPredictionFrame(&p, cur, W, H, blk);
  FILE* f = fopen(argv[7], "wb");
  if (!f) return 1;
  int unset = 0;
  for (int i = 0; i < p.num_blks; i++) {
    float s = findBestBlkSSIM(p, ref, &p.blks[i], span);
    if (!(s > 0)) unset++;
    int rec[2] = {p.blks[i].motion_vectorX, p.blks[i].motion_vectorY};
    fwrite(rec, sizeof(int), 2, f);
    fwrite(&s, sizeof(float), 1, f);
  }
  fclose(f);
  fprintf(stderr, "blocks without a positive score: %d\n", unset);
  return 0;
}
