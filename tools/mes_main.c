/*
 * mes_hip -- the reference's command-line driver on the GPU engine.
 *
 * Same positional argv and stdout lines as src/cpu/main.c:109-179:
 *   mes_hip <current_frame> <reference_frame> <output_dir> [blk] [span] [W] [H]
 * with the thread-pool dispatch (main.c:144-158) replaced by one
 * me_full_search() call through include/me.h, and the post-processing
 * (main.c:160-178) by me_compensate_planes().  Extra trailing options:
 *   --cost ssd|sad|ssim (default ssd = the reference's MSE choice; ssim = the
 *                       reference's SSIM driver src/cpu/main_ssim.c, whose
 *                       stdout -- score lines instead of PSNR -- is mirrored)
 *   --gpus N            stripe the search over devices 0..N-1 (RCCL gather)
 *   --mv FILE           MV field + costs as a MEMV file (include/me.h, me_mv_write)
 * Errors print a message and return 1 (no exit() inside the library).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "me.h"

static double now(void) {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return (double)tv.tv_sec + (double)tv.tv_usec / 1e6;
}

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
  int npos = 0, gpus = 1;
  me_cost cost = ME_COST_SSD;
  const char* mv_path = NULL;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--cost") && i + 1 < argc) {
      ++i;
      cost = !strcmp(argv[i], "sad") ? ME_COST_SAD : !strcmp(argv[i], "ssim") ? ME_COST_SSIM : ME_COST_SSD;
    } else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) {
      gpus = atoi(argv[++i]);
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
  uint8_t* ref = (uint8_t*)malloc(n);
  uint8_t* cur = (uint8_t*)malloc(n);
  uint8_t* out = (uint8_t*)malloc(5 * n);
  if (!ref || !cur || !out) return 1;
  if (!read_plane(pos[0], cur, n) || !read_plane(pos[1], ref, n)) return 1;

  int ids[64];
  if (gpus < 1) gpus = 1;
  if (gpus > 64) gpus = 64;
  for (int i = 0; i < gpus; i++) ids[i] = i;
  me_ctx* ctx = NULL;
  me_status s = me_create(&ctx, ids, gpus);
  if (s != ME_OK) {
    printf("Error: me_create: %s\n", me_status_str(s));
    return 1;
  }
  int nb = me_num_blocks(W, H, blk);
  int16_t* mv = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)(nb > 0 ? nb : 1));
  uint32_t* bc = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(nb > 0 ? nb : 1));
  /* first call allocates device buffers; time a second call like main.c:151-157 */
  s = me_full_search(ctx, ref, cur, W, H, W, blk, span, cost, mv, bc);
  double t0 = now();
  if (s == ME_OK) s = me_full_search(ctx, ref, cur, W, H, W, blk, span, cost, mv, bc);
  double t1 = now();
  if (s != ME_OK) {
    printf("Error: me_full_search: %s (%s)\n", me_status_str(s), me_last_error(ctx));
    me_destroy(ctx);
    return 1;
  }
  double psnr = 0;
  s = me_compensate_planes(ctx, ref, cur, W, H, blk, mv, out, &psnr);
  if (s != ME_OK) {
    printf("Error: me_compensate_planes: %s (%s)\n", me_status_str(s), me_last_error(ctx));
    me_destroy(ctx);
    return 1;
  }
  if (cost == ME_COST_SSIM) {
    /* main_ssim.c:83-96: float sums of squared differences, pixel order */
    float comp = 0.0f, orig = 0.0f;
    for (size_t i = 0; i < n; i++) {
      const int m = out[2 * n + i], c = out[n + i], r = out[i];
      comp += (m - c) * (m - c);
      orig += (c - r) * (c - r);
    }
    printf("Original Score: %.4f, Compensated Score: %.4f\n", orig / (int)n, comp / (int)n);
  } else {
    printf("PSNR: %.6f\n", psnr);
  }
  printf("Output file dimensions: (%d x %d)\n", W, 5 * H);
  char path[4096];
  snprintf(path, sizeof path, "%s/output_%d_%d.yuv", pos[2], blk, span);
  if (me_yuv_write(path, out, 5 * n, 0) != ME_OK)
    printf("yuvWriteToFile: Could not open the file %s\n", path);
  if (mv_path && me_mv_write(mv_path, W, H, blk, span, cost, NULL, 1, mv, bc) != ME_OK)
    printf("Error: could not write %s\n", mv_path);
  printf("Computation time: %.lf ms\n", (t1 - t0) * 1000);
  if (cost != ME_COST_SSIM) printf("PSNR: %.lf \n", psnr);
  me_destroy(ctx);
  free(mv);
  free(bc);
  free(ref);
  free(cur);
  free(out);
  return 0;
}
