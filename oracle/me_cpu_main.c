/*
 * me_cpu -- the CPU restatement as a command line tool (TEST ORACLE / CPU
 * baseline).  Same positional argv and stdout lines as the reference driver
 * src/cpu/main.c:109-179:
 *   me_cpu <current_frame> <reference_frame> <output_dir> [blk] [span] [W] [H]
 * Extra trailing options (not in the reference):
 *   --cost mse|ssd|sad   (default mse = the reference arithmetic)
 *   --threads N          (default 100, as main.c:144)
 *   --mv FILE            dump int16 (mvx, mvy) per block, raster order
 * Writes <output_dir>/output_<blk>_<span>.yuv = [ref, cur, mc, |ref-cur|, |mc-cur|].
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "me_oracle.h"

static int read_plane(const char* path, uint8_t* buf, size_t n) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    printf("yuvOpenInputFile: Could not open the file %s\n", path);
    return 0;
  }
  size_t got = fread(buf, 1, n, f);
  fclose(f);
  if (got != n) {
    printf("yuvReadFrame: The read was failed!\n");
    return 0;
  }
  return 1;
}

int main(int argc, char** argv) {
  const char* pos[7] = {0};
  int npos = 0, kind = ORC_MSE_FLOAT, threads = 100;
  const char* mv_path = NULL;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--cost") && i + 1 < argc) {
      const char* c = argv[++i];
      kind = !strcmp(c, "sad") ? ORC_SAD : !strcmp(c, "ssd") ? ORC_SSD : ORC_MSE_FLOAT;
    } else if (!strcmp(argv[i], "--threads") && i + 1 < argc) {
      threads = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--mv") && i + 1 < argc) {
      mv_path = argv[++i];
    } else if (npos < 7) {
      pos[npos++] = argv[i];
    }
  }
  if (npos < 3) {
    printf("Error: wrong number of argument. Usage: <current_frame> <reference_frame> <output_dir> [<blk_dim>] [<extra_span>] [<width>] [<height>]\n");
    return 0;
  }
  int blk = npos > 3 ? atoi(pos[3]) : 8;
  int span = npos > 4 ? atoi(pos[4]) : 12;
  int W = npos > 5 ? atoi(pos[5]) : 352;
  int H = npos > 6 ? atoi(pos[6]) : 288;
  printf("[\n  Current Frame: %s\n  Reference Frame: %s\n  Output Dir: %s\n  BlkDim: %d\n  ExtraSpan: %d\n  FrameWidth: %d\n  FrameHeight: %d\n]\n",
         pos[0], pos[1], pos[2], blk, span, W, H);
  size_t n = (size_t)W * H;
  uint8_t* out = (uint8_t*)calloc(5 * n, 1);
  uint8_t *ref = out, *cur = out + n, *mc = out + 2 * n;
  if (!read_plane(pos[0], cur, n) || !read_plane(pos[1], ref, n)) return 1;
  int nb = orc_num_blocks(W, H, blk);
  int16_t* mv = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)(nb ? nb : 1));
  double t0 = orc_now();
  if (orc_full_search(ref, cur, W, H, W, blk, span, kind, threads, 0, nb, mv,
                      NULL, NULL) != 0) {
    printf("Error: invalid arguments\n");
    return 1;
  }
  double t1 = orc_now();
  orc_motion_compensate(ref, W, H, blk, mv, mc);
  orc_frame_diff(ref, cur, (int)n, out + 3 * n);
  orc_frame_diff(mc, cur, (int)n, out + 4 * n);
  double psnr = orc_psnr(mc, cur, W, H);
  printf("PSNR: %.6f\n", psnr);
  printf("Output file dimensions: (%d x %d)\n", W, 5 * H);
  char path[4096];
  snprintf(path, sizeof path, "%s/output_%d_%d.yuv", pos[2], blk, span);
  FILE* f = fopen(path, "wb");
  if (f) {
    fwrite(out, 1, 5 * n, f);
    fclose(f);
  } else {
    printf("yuvWriteToFile: Could not open the file %s\n", path);
  }
  if (mv_path) {
    FILE* g = fopen(mv_path, "wb");
    if (g) {
      fwrite(mv, sizeof(int16_t), 2 * (size_t)nb, g);
      fclose(g);
    }
  }
  printf("Computation time: %.lf ms\n", (t1 - t0) * 1000);
  printf("PSNR: %.lf \n", psnr);
  free(mv);
  free(out);
  return 0;
}
