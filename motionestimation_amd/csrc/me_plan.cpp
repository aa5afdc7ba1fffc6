// me_plan.cpp -- host-only geometry of the search (include/me.h): block
// tiling, exact candidate counts under the reference's clamping, and the
// stripe planner of the multi-GPU split.  Plain C++ with no HIP
// dependency, so the CPU sanitizer harness (oracle/Makefile asan, tsan) links
// it as it is.
#include <stdint.h>

#include <vector>

#include "me.h"

namespace {

uint64_t row_candidates(int width, int height, int blk, int range, int by) {
  const int nbx = (width + blk - 1) / blk;
  const int tly = by * blk;
  const int h = height - tly < blk ? height - tly : blk;
  const int dymin = -range > -tly ? -range : -tly;
  const int dymax = range < height - h - tly ? range : height - h - tly;
  uint64_t ny = (uint64_t)(dymax - dymin + 1), total = 0;
  for (int bx = 0; bx < nbx; bx++) {
    const int tlx = bx * blk;
    const int w = width - tlx < blk ? width - tlx : blk;
    const int dxmin = -range > -tlx ? -range : -tlx;
    const int dxmax = range < width - w - tlx ? range : width - w - tlx;
    total += (uint64_t)(dxmax - dxmin + 1) * ny;
  }
  return total;
}

}  // namespace

extern "C" {

int me_num_blocks(int width, int height, int blk) {
  if (width <= 0 || height <= 0 || blk <= 0) return 0;
  // 64-bit: a hostile MEMV header must not overflow the count (0 = invalid)
  const int64_t n = ((int64_t)width + blk - 1) / blk * (((int64_t)height + blk - 1) / blk);
  return n > INT32_MAX ? 0 : (int)n;
}

uint64_t me_candidate_count(int width, int height, int blk, int range) {
  if (width <= 0 || height <= 0 || blk <= 0 || range < 0) return 0;
  uint64_t t = 0;
  const int nby = (height + blk - 1) / blk;
  for (int by = 0; by < nby; by++) t += row_candidates(width, height, blk, range, by);
  return t;
}

me_status me_plan_stripes(int width, int height, int blk, int range, int n, int* bounds) {
  if (!bounds || n < 1 || width <= 0 || height <= 0 || blk <= 0 || range < 0) return ME_EINVAL;
  const int nby = (height + blk - 1) / blk;
  // Row cost (include/me.h): nbx * (3 (2S + 1) + ny) -- an exact-candidate
  // balance gave the 4K +-64 edge stripes 18 block rows against 16-17 inside,
  // and 2,160 two-block tiles take three rounds of the chip's 1,024 workgroup
  // slots where 2,040 take two (8-way 4K edge stripe 0.200 vs 0.153 ms,
  // profiles/r02i_stripe_4k.jsonl).
  std::vector<uint64_t> cum(nby + 1, 0);
  const uint64_t nbx = (uint64_t)((width + blk - 1) / blk);
  for (int by = 0; by < nby; by++) {
    const int tly = by * blk;
    const int h = height - tly < blk ? height - tly : blk;
    const int dymin = -range > -tly ? -range : -tly;
    const int dymax = range < height - h - tly ? range : height - h - tly;
    const uint64_t ny = (uint64_t)(dymax - dymin + 1);
    cum[by + 1] = cum[by] + nbx * (3 * (uint64_t)(2 * range + 1) + ny);
  }
  bounds[0] = 0;
  int r = 0;
  for (int i = 1; i < n; i++) {
    const double target = (double)cum[nby] * i / n;
    while (r < nby && (double)cum[r + 1] <= target) r++;
    // pick the nearer boundary
    if (r < nby && target - (double)cum[r] > (double)cum[r + 1] - target) r++;
    if (r < bounds[i - 1]) r = bounds[i - 1];
    bounds[i] = r;
  }
  bounds[n] = nby;
  return ME_OK;
}

}  // extern "C"
