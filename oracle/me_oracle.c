/*
 * me_oracle.c -- CPU restatement of the reference full search (TEST ORACLE).
 * See me_oracle.h for the reference lines each function follows.
 * Build: gcc -O2 (no -ffast-math: ORC_MSE_FLOAT must round like the reference).
 */
#include "me_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

double orc_now(void) {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return (double)tv.tv_sec + (double)tv.tv_usec / 1e6;
}

/* prediction_frame.c:9-11 -- ceil tiling. */
int orc_num_blocks(int width, int height, int blk) {
  if (width <= 0 || height <= 0 || blk <= 0) return 0;
  return ((width + blk - 1) / blk) * ((height + blk - 1) / blk);
}

/* prediction_frame.c:15-23 + block.c:3-13 -- raster index -> block, partial
 * blocks on the right / bottom edges. */
void orc_block_at(int i, int width, int height, int blk, orc_block* o) {
  int nbx = (width + blk - 1) / blk;
  o->idx_x = i % nbx;
  o->idx_y = i / nbx;
  o->top_left_x = o->idx_x * blk;
  o->top_left_y = o->idx_y * blk;
  o->width = (o->top_left_x + blk) < width ? blk : width - o->top_left_x;
  o->height = (o->top_left_y + blk) < height ? blk : height - o->top_left_y;
  o->bottom_right_x = o->top_left_x + o->width - 1;
  o->bottom_right_y = o->top_left_y + o->height - 1;
}

/* main.c:73-76 -- search window clamped to the frame, no padding. */
static void window_of(const orc_block* b, int width, int height, int range,
                      int* wx0, int* wy0, int* wx1, int* wy1) {
  *wx0 = b->top_left_x - range < 0 ? 0 : b->top_left_x - range;
  *wy0 = b->top_left_y - range < 0 ? 0 : b->top_left_y - range;
  *wx1 = b->bottom_right_x + range >= width ? width - 1 : b->bottom_right_x + range;
  *wy1 = b->bottom_right_y + range >= height ? height - 1 : b->bottom_right_y + range;
}

/* main.c:18-27 literally: float += int square, then float / int. */
static float mse_float(const uint8_t* ref, const uint8_t* cur, int stride,
                       const orc_block* b, int cx, int cy) {
  float sum = 0;
  for (int oy = 0; oy < b->height; oy++) {
    const uint8_t* c = cur + (size_t)(b->top_left_y + oy) * stride + b->top_left_x;
    const uint8_t* r = ref + (size_t)(cy + oy) * stride + cx;
    for (int ox = 0; ox < b->width; ox++) {
      int d = (int)c[ox] - (int)r[ox];
      sum += d * d;
    }
  }
  return sum / (b->width * b->height);
}

static uint32_t cost_int(const uint8_t* ref, const uint8_t* cur, int stride,
                         const orc_block* b, int cx, int cy, int kind) {
  uint32_t s = 0;
  for (int oy = 0; oy < b->height; oy++) {
    const uint8_t* c = cur + (size_t)(b->top_left_y + oy) * stride + b->top_left_x;
    const uint8_t* r = ref + (size_t)(cy + oy) * stride + cx;
    if (kind == ORC_SAD) {
      for (int ox = 0; ox < b->width; ox++) {
        int d = (int)c[ox] - (int)r[ox];
        s += (uint32_t)(d < 0 ? -d : d);
      }
    } else {
      for (int ox = 0; ox < b->width; ox++) {
        int d = (int)c[ox] - (int)r[ox];
        s += (uint32_t)(d * d);
      }
    }
  }
  return s;
}

/* ssim.c:3-62 restated on u8 planes: means as float sums of ints (exact) over
 * w*h; variances as float sums of (float(p) - mean)^2 in raster order; the
 * cross term with the means truncated to int (computeCrossVar takes int
 * means) accumulated in float from int products (exact: |sum| < 2^24); the
 * standard deviations through double sqrt; then the three factors in float,
 * left to right, no contraction (build with -ffp-contract=off). */
static void ssim_stats(const uint8_t* p, int stride, int x0, int y0, int w, int h, float* mean,
                       float* var) {
  const int n = w * h;
  float s = 0;
  for (int oy = 0; oy < h; oy++)
    for (int ox = 0; ox < w; ox++) s += (int)p[(size_t)(y0 + oy) * stride + x0 + ox];
  const float m = s / n;
  float v = 0;
  for (int oy = 0; oy < h; oy++)
    for (int ox = 0; ox < w; ox++) {
      const int q = p[(size_t)(y0 + oy) * stride + x0 + ox];
      v += (q - m) * (q - m);
    }
  *mean = m;
  *var = v / n;
}

static float ssim_score(const uint8_t* ref, const uint8_t* cur, int stride, const orc_block* b,
                        int cx, int cy) {
  const int w = b->width, h = b->height, n = w * h;
  const float C1 = 0.01f, C2 = 0.09f, C3 = 0.045f;  /* ssim.c:48, float from double */
  float mr, vr, mp, vp;
  ssim_stats(ref, stride, cx, cy, w, h, &mr, &vr);
  ssim_stats(cur, stride, b->top_left_x, b->top_left_y, w, h, &mp, &vp);
  const float sr = (float)sqrt((double)vr), sp = (float)sqrt((double)vp);
  const int imr = (int)mr, imp = (int)mp;
  float cv = 0;
  for (int oy = 0; oy < h; oy++)
    for (int ox = 0; ox < w; ox++) {
      const int r = ref[(size_t)(cy + oy) * stride + cx + ox];
      const int c = cur[(size_t)(b->top_left_y + oy) * stride + b->top_left_x + ox];
      cv += (r - imr) * (c - imp);
    }
  cv = cv / n;
  const float lum = (2 * mr * mp + C1) / (mr * mr + mp * mp + C1);
  const float con = (2 * sr * sp + C2) / (sr * sr + sp * sp + C2);
  const float str = (cv + C3) / (sr * sp + C3);
  return lum * con * str;
}

/* main.c:39-64 + 67-82: y outer, x inner, keep the first strict minimum. */
uint32_t orc_search_block(const uint8_t* ref, const uint8_t* cur, int width,
                          int height, int stride, const orc_block* b,
                          int range, int kind, int* mvx, int* mvy, float* mse) {
  int wx0, wy0, wx1, wy1;
  window_of(b, width, height, range, &wx0, &wy0, &wx1, &wy1);
  int best_x = 0, best_y = 0;
  if (kind == ORC_MSE_FLOAT) {
    float best = INFINITY;
    for (int y = wy0; y <= wy1 - b->height + 1; y++)
      for (int x = wx0; x <= wx1 - b->width + 1; x++) {
        float m = mse_float(ref, cur, stride, b, x, y);
        if (m < best) {
          best = m;
          best_x = x - b->top_left_x;
          best_y = y - b->top_left_y;
        }
      }
    if (mse) *mse = best;
    *mvx = best_x;
    *mvy = best_y;
    return cost_int(ref, cur, stride, b, b->top_left_x + best_x,
                    b->top_left_y + best_y, ORC_SSD);
  }
  if (kind == ORC_SSIM) {  /* ssim.c:83-108: maximise, strict > from 0 */
    float best = 0;
    for (int y = wy0; y <= wy1 - b->height + 1; y++)
      for (int x = wx0; x <= wx1 - b->width + 1; x++) {
        const float sc = ssim_score(ref, cur, stride, b, x, y);
        if (sc > best) {
          best = sc;
          best_x = x - b->top_left_x;
          best_y = y - b->top_left_y;
        }
      }
    if (mse) *mse = best;
    *mvx = best_x;
    *mvy = best_y;
    uint32_t bits;
    memcpy(&bits, &best, 4);
    return bits;
  }
  uint32_t best = 0xFFFFFFFFu;
  int found = 0;
  for (int y = wy0; y <= wy1 - b->height + 1; y++)
    for (int x = wx0; x <= wx1 - b->width + 1; x++) {
      uint32_t c = cost_int(ref, cur, stride, b, x, y, kind);
      if (!found || c < best) {
        found = 1;
        best = c;
        best_x = x - b->top_left_x;
        best_y = y - b->top_left_y;
      }
    }
  if (mse) *mse = (float)best / (float)(b->width * b->height);
  *mvx = best_x;
  *mvy = best_y;
  return best;
}

typedef struct {
  const uint8_t *ref, *cur;
  int width, height, stride, blk, range, kind;
  int next, end;
  pthread_mutex_t mu;
  int16_t* mv_xy;
  uint32_t* cost;
  float* mse;
  int base;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->end) break;
    orc_block b;
    orc_block_at(i, j->width, j->height, j->blk, &b);
    int mx, my;
    float m;
    uint32_t c = orc_search_block(j->ref, j->cur, j->width, j->height, j->stride,
                                  &b, j->range, j->kind, &mx, &my, &m);
    int k = i - j->base;
    j->mv_xy[2 * k] = (int16_t)mx;
    j->mv_xy[2 * k + 1] = (int16_t)my;
    if (j->cost) j->cost[k] = c;
    if (j->mse) j->mse[k] = m;
  }
  return NULL;
}

/* main.c:141-158: the timed dispatch region, one job per block. */
int orc_full_search(const uint8_t* ref, const uint8_t* cur, int width,
                    int height, int stride, int blk, int range, int kind,
                    int nthreads, int blk_begin, int blk_end, int16_t* mv_xy,
                    uint32_t* cost, float* mse) {
  if (!ref || !cur || !mv_xy || width <= 0 || height <= 0 || blk <= 0 ||
      range < 0 || stride < width)
    return -1;
  int n = orc_num_blocks(width, height, blk);
  if (blk_begin < 0 || blk_end > n || blk_begin > blk_end) return -1;
  if (nthreads < 1) nthreads = 1;
  job_t j = {ref, cur, width, height, stride, blk, range, kind,
             blk_begin, blk_end, PTHREAD_MUTEX_INITIALIZER, mv_xy, cost, mse,
             blk_begin};
  if (nthreads == 1) {
    worker(&j);
    return 0;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  int started = 0;
  for (int t = 0; t < nthreads; t++)
    if (pthread_create(&th[t], NULL, worker, &j) == 0) started++;
    else break;
  if (started == 0) worker(&j);
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  free(th);
  return 0;
}

uint64_t orc_candidate_count(int width, int height, int blk, int range) {
  uint64_t total = 0;
  int n = orc_num_blocks(width, height, blk);
  for (int i = 0; i < n; i++) {
    orc_block b;
    orc_block_at(i, width, height, blk, &b);
    int wx0, wy0, wx1, wy1;
    window_of(&b, width, height, range, &wx0, &wy0, &wx1, &wy1);
    uint64_t nx = (uint64_t)(wx1 - b.width + 1 - wx0 + 1);
    uint64_t ny = (uint64_t)(wy1 - b.height + 1 - wy0 + 1);
    total += nx * ny;
  }
  return total;
}

/* utils.c:102-134: copy ref[p + mv] into every pixel of each block. */
void orc_motion_compensate(const uint8_t* ref, int width, int height, int blk,
                           const int16_t* mv_xy, uint8_t* mc) {
  int n = orc_num_blocks(width, height, blk);
  memset(mc, 0, (size_t)width * height);
  for (int i = 0; i < n; i++) {
    orc_block b;
    orc_block_at(i, width, height, blk, &b);
    int mx = mv_xy[2 * i], my = mv_xy[2 * i + 1];
    for (int ox = 0; ox < b.width; ox++)
      for (int oy = 0; oy < b.height; oy++) {
        int cx = b.top_left_x + ox, cy = b.top_left_y + oy;
        int px = cx + mx, py = cy + my;
        if (px >= 0 && py >= 0 && px < width && py < height)
          mc[cy * width + cx] = ref[py * width + px];
      }
  }
}

/* utils.c:94-100 */
void orc_frame_diff(const uint8_t* a, const uint8_t* b, int n, uint8_t* out) {
  for (int i = 0; i < n; i++) {
    int d = (int)a[i] - (int)b[i];
    out[i] = (uint8_t)(d < 0 ? -d : d);
  }
}

/* utils.c:137-164: MAX is the largest pixel of either frame, not 255. */
double orc_psnr(const uint8_t* f1, const uint8_t* f2, int x, int y) {
  double mse = 0.0;
  int mx = 0;
  for (int i = 0; i < x * y; i++) {
    if (mx < f1[i]) mx = f1[i];
    if (mx < f2[i]) mx = f2[i];
    double t = abs((int)f1[i] - (int)f2[i]);
    mse += t * t;
  }
  mse /= x * y;
  if (mse == 0) return 99.0;
  return 20 * log10(mx) - 10 * log10(mse);
}
