/*
 * me_oracle.h -- CPU restatement of the reference's full-search block matcher.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the timed CPU baseline.  The product path
 * (motionestimation_amd, libme_hip.so) never links or calls it.
 *
 * Restated from souravBhat/MotionEstimation (paths relative to the reference):
 *   block tiling            src/common/prediction_frame.c:3-25, src/common/block.c:3-13
 *   candidate cost (MSE)    src/cpu/main.c:18-36   (float accumulate of int squares, / (w*h))
 *   raster search, strict < src/cpu/main.c:39-64
 *   frame-clamped window    src/cpu/main.c:67-82
 *   per-block dispatch      src/cpu/main.c:141-158 (thread pool, one job per block)
 *   MC / diff / PSNR        src/common/utils.c:94-164
 *   SSIM cost (maximised)   src/common/ssim.c:3-62 (score), :83-108 (raster
 *                           search, strict > from 0), src/cpu/main_ssim.c:15-29
 * Pinned against the real reference: tests/golden/ holds MV fields dumped by
 * oracle/_ref/ref_dump (the unmodified reference objects), and the published
 * results/cpu/foreman/output_4_{7,15}.yuv planes.
 */
#ifndef ME_ORACLE_H
#define ME_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Cost kinds.  ORC_MSE_FLOAT replays the reference arithmetic literally
 * (float accumulation, float divide); ORC_SSD / ORC_SAD use exact integer
 * accumulation with the same loop order and tie rule.  ORC_SSIM replays
 * src/common/ssim.c: the first candidate in raster order whose float score
 * is strictly greater than every earlier one and than 0; the returned "cost"
 * is the score's float bits, *mse the score.  If no candidate scores above 0
 * the reference leaves its MV uninitialised (ssim.c:87-104); here it is
 * (0, 0) with score 0. */
enum { ORC_SSD = 0, ORC_SAD = 1, ORC_MSE_FLOAT = 2, ORC_SSIM = 3 };

typedef struct orc_block {
  int idx_x, idx_y;
  int top_left_x, top_left_y;
  int bottom_right_x, bottom_right_y;
  int width, height;
} orc_block;

int orc_num_blocks(int width, int height, int blk);
void orc_block_at(int i, int width, int height, int blk, orc_block* out);

/* One block, one cost kind.  Writes the MV of the first minimum in raster
 * order.  Returns the integer cost (SSD or SAD); for ORC_MSE_FLOAT also
 * stores the reference's float score in *mse (may be NULL). */
uint32_t orc_search_block(const uint8_t* ref, const uint8_t* cur, int width,
                          int height, int stride, const orc_block* b,
                          int range, int kind, int* mvx, int* mvy, float* mse);

/* Frame level, blocks [blk_begin, blk_end) in raster order, nthreads pthreads
 * pulling block indices from a shared counter.  mv_xy[2*i], cost[i], mse[i]
 * are written for i in the range (cost / mse may be NULL).
 * Returns 0, or -1 on invalid arguments. */
int orc_full_search(const uint8_t* ref, const uint8_t* cur, int width,
                    int height, int stride, int blk, int range, int kind,
                    int nthreads, int blk_begin, int blk_end, int16_t* mv_xy,
                    uint32_t* cost, float* mse);

/* Exact candidate count under the reference's clamping rules. */
uint64_t orc_candidate_count(int width, int height, int blk, int range);

/* Post-processing, src/common/utils.c:94-164 semantics, u8 planes. */
void orc_motion_compensate(const uint8_t* ref, int width, int height, int blk,
                           const int16_t* mv_xy, uint8_t* mc);
void orc_frame_diff(const uint8_t* a, const uint8_t* b, int n, uint8_t* out);
double orc_psnr(const uint8_t* a, const uint8_t* b, int width, int height);

/* Wall-clock seconds (gettimeofday, as src/common/utils.c:23-27). */
double orc_now(void);

#ifdef __cplusplus
}
#endif
#endif
