/*
 * mes_seq -- multi-frame driver: search every frame pair of a YUV sequence in
 * one pipelined call (me_search_pairs) and write the MV fields as one MEMV
 * file.  The reference handles one pair per process (src/cpu/main.c:109-179);
 * this is SURVEY §8f-3 (frame-pair streaming, multi-reference) end to end in
 * u8 (§8f-2).
 *
 *   mes_seq <sequence.yuv> <width> <height> <blk> <span> [options]
 *     --layout luma|i420   frame layout in the file (default luma: W*H per frame)
 *     --frames N           first N frames (default: all whole frames)
 *     --ref prev|first     pair k = (k, k+1) (default) or (0, k+1)
 *     --cost ssd|sad|ssim  default ssd (the reference's MSE choice)
 *     --gpus N             devices 0..N-1, pairs split in contiguous runs
 *     --repeat R           time R calls after a warm-up call (default 1)
 *     --mv FILE            write the MV fields + costs (MEMV, include/me.h)
 * Frames are read straight into pinned host memory (me_host_alloc), so their
 * upload is a direct DMA that overlaps the search of the previous pair.
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

int main(int argc, char** argv) {
  const char* pos[5] = {0};
  int npos = 0, gpus = 1, nframes = -1, first_ref = 0, repeat = 1;
  me_yuv_layout layout = ME_YUV_LUMA;
  me_cost cost = ME_COST_SSD;
  const char* mv_path = NULL;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--layout") && i + 1 < argc) {
      layout = !strcmp(argv[++i], "i420") ? ME_YUV_I420 : ME_YUV_LUMA;
    } else if (!strcmp(argv[i], "--frames") && i + 1 < argc) {
      nframes = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--ref") && i + 1 < argc) {
      first_ref = !strcmp(argv[++i], "first");
    } else if (!strcmp(argv[i], "--cost") && i + 1 < argc) {
      ++i;
      cost = !strcmp(argv[i], "sad") ? ME_COST_SAD : !strcmp(argv[i], "ssim") ? ME_COST_SSIM : ME_COST_SSD;
    } else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) {
      gpus = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--repeat") && i + 1 < argc) {
      repeat = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--mv") && i + 1 < argc) {
      mv_path = argv[++i];
    } else if (npos < 5) {
      pos[npos++] = argv[i];
    }
  }
  if (npos < 5) {
    printf("Usage: mes_seq <sequence.yuv> <width> <height> <blk> <span> [--layout luma|i420] "
           "[--frames N] [--ref prev|first] [--cost ssd|sad|ssim] [--gpus N] [--repeat R] [--mv FILE]\n");
    return 1;
  }
  const int W = atoi(pos[1]), H = atoi(pos[2]), blk = atoi(pos[3]), span = atoi(pos[4]);
  const int64_t avail = me_yuv_frame_count(pos[0], W, H, layout);
  if (avail < 0) {
    printf("Error: cannot open %s as %dx%d frames\n", pos[0], W, H);
    return 1;
  }
  if (nframes < 0 || nframes > avail) nframes = (int)avail;
  if (nframes < 2) {
    printf("Error: %s holds %d whole frame(s); need 2\n", pos[0], nframes);
    return 1;
  }
  if (repeat < 1) repeat = 1;
  const size_t plane = (size_t)W * H;
  uint8_t* pix = (uint8_t*)me_host_alloc(plane * nframes);
  const uint8_t** frames = (const uint8_t**)malloc(sizeof(uint8_t*) * nframes);
  const int npairs = nframes - 1;
  int* pairs = (int*)malloc(sizeof(int) * 2 * npairs);
  const int nb = me_num_blocks(W, H, blk);
  int16_t* mv = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)(nb > 0 ? nb : 1) * npairs);
  uint32_t* bc = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(nb > 0 ? nb : 1) * npairs);
  if (!pix || !frames || !pairs || !mv || !bc) {
    printf("Error: out of host memory\n");
    return 1;
  }
  for (int k = 0; k < nframes; k++) {
    frames[k] = pix + plane * k;
    me_status s = me_yuv_read_luma(pos[0], W, H, layout, k, pix + plane * k, W);
    if (s != ME_OK) {
      printf("Error: reading frame %d: %s\n", k, me_status_str(s));
      return 1;
    }
  }
  for (int k = 0; k < npairs; k++) {
    pairs[2 * k] = first_ref ? 0 : k;
    pairs[2 * k + 1] = k + 1;
  }
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
  /* warm-up call allocates the device slots; then time `repeat` calls */
  s = me_search_pairs(ctx, frames, nframes, W, H, W, blk, span, cost, pairs, npairs, mv, bc);
  const double t0 = now();
  for (int r = 0; r < repeat && s == ME_OK; r++)
    s = me_search_pairs(ctx, frames, nframes, W, H, W, blk, span, cost, pairs, npairs, mv, bc);
  const double t1 = now();
  if (s != ME_OK) {
    printf("Error: me_search_pairs: %s (%s)\n", me_status_str(s), me_last_error(ctx));
    me_destroy(ctx);
    return 1;
  }
  const double per_call = (t1 - t0) / repeat;
  const double cand = (double)me_candidate_count(W, H, blk, span) * npairs;
  printf("Frames: %d, pairs: %d (%s), %dx%d, blk %d, span %d, %s, gpus %d\n", nframes, npairs,
         first_ref ? "first" : "prev", W, H, blk, span, cost == ME_COST_SAD ? "sad" : cost == ME_COST_SSIM ? "ssim" : "ssd", gpus);
  printf("Computation time: %.3f ms per sequence (%.1f pairs/s, %.3e candidates/s incl. upload)\n",
         per_call * 1e3, npairs / per_call, cand / per_call);
  if (mv_path) {
    s = me_mv_write(mv_path, W, H, blk, span, cost, pairs, npairs, mv, bc);
    if (s != ME_OK) printf("Error: writing %s: %s\n", mv_path, me_status_str(s));
  }
  me_destroy(ctx);
  me_host_free(pix);
  free(frames);
  free(pairs);
  free(mv);
  free(bc);
  return s == ME_OK ? 0 : 1;
}
