/*
 * ref_dump.c -- golden-vector generator linked against the UNMODIFIED
 * reference objects (TEST INFRASTRUCTURE; built by oracle/Makefile into
 * oracle/_ref/, never shipped).
 *
 * The reference never prints its MVs (src/cpu/main.c:160-178 only writes the
 * MC plane and PSNR), so this driver calls the reference's own
 * createPredictionFrame (src/common/prediction_frame.c:3) and
 * findBestBlkMse (src/cpu/main.c:67) for every block, single-threaded, and
 * writes one record per block in raster order:
 *     int32 mvx, int32 mvy, float32 mse     (little endian, 12 bytes)
 * main.c is compiled with -Dmain=reference_main so its driver is not linked
 * as the entry point; nothing else in the reference is changed.
 *
 * usage: ref_dump <cur.yuv> <ref.yuv> <W> <H> <blk> <span> <out.bin> [begin end]
 * The optional raster block range [begin, end) lets a large frame (8K 8x8
 * +-128: ~30 CPU-minutes) be dumped as parallel slabs that concatenate to the
 * whole-frame record stream (tests/golden/make_golden.py --big).
 */
#include <stdio.h>
#include <stdlib.h>

#include "prediction_frame.h"
#include "utils.h"

float findBestBlkMse(predictionFrame pf, int* referenceFrame, block* blk,
                     int extraSpan);

int main(int argc, char** argv) {
  if (argc != 8 && argc != 10) {
    fprintf(stderr, "usage: ref_dump cur ref W H blk span out.bin [begin end]\n");
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
  int begin = 0, end = p.num_blks;
  if (argc == 10) {
    begin = atoi(argv[8]);
    end = atoi(argv[9]);
    if (begin < 0 || end > p.num_blks || begin > end) return 2;
  }
  for (int i = begin; i < end; i++) {
    float mse = findBestBlkMse(p, ref, &p.blks[i], span);
    int rec[2] = {p.blks[i].motion_vectorX, p.blks[i].motion_vectorY};
    fwrite(rec, sizeof(int), 2, f);
    fwrite(&mse, sizeof(float), 1, f);
  }
  fclose(f);
  return 0;
}
