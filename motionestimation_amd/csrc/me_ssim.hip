// me_ssim.hip -- SSIM-cost full search, bit-exact with the
// reference's CPU SSIM search (souravBhat/MotionEstimation src/common/ssim.c:3-108,
// src/cpu/main_ssim.c:15-29).
//
// The reference maximises a float SSIM score per candidate (first strict
// maximum above 0 in raster order).  Every float operation is replayed in the
// reference's order with round-to-nearest intrinsics, and the file is built
// with -ffp-contract=off (csrc/Makefile: the intrinsics are plain operators
// here, and a fused d*d + v rounds once where the reference rounds twice):
//   mean   = (float) sum(p) / (float)(w*h)       sum of ints is exact in float
//   var    = float chain sum((float)p - mean)^2 in raster order, / (w*h)
//   cross  = float chain of int products (p - (int)mean_r)(c - (int)mean_c)
//            (computeCrossVar takes int means), / (w*h)
//   stddev = (float) sqrt((double) var)
//   score  = lum * con * str, each factor as written in ssim.c:53-56
// The argmax is a min over 64-bit keys (0x7FFFFFFF - bits(score)) << 32 |
// (dy, dx): scores > 0 are ordered by their bits, ties go to the smallest
// (dy, dx) -- the reference's first strict maximum.  Blocks with no score
// above 0 get MV (0, 0) and cost 0 (the reference leaves them uninitialised).
// block_cost carries the float bits of the best score.
//
// One workgroup per block, SSIM_Q adjacent candidates per lane per step; the
// block and its window are staged in LDS when they fit.  Float-chain bound
// (two dependent w*h chains per candidate, 2*SSIM_Q of them interleaved per
// lane), not a hot path of the headline metric.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_kernels.h"

namespace me {

namespace {

constexpr int SSIM_THREADS = 256;
constexpr int SSIM_Q = 4;  // adjacent candidates per lane

__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

// ssim.c:3-28 for one w x h patch at p (row pitch `pitch`): mean and variance.
__device__ __forceinline__ void patch_stats(const uint8_t* p, int pitch, int w, int h, float nf,
                                            float* mean, float* var) {
  int s = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) s += p[y * pitch + x];
  const float m = __fdiv_rn((float)s, nf);
  float v = 0.f;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const float d = __fsub_rn((float)p[y * pitch + x], m);
      v = __fadd_rn(v, __fmul_rn(d, d));
    }
  *mean = m;
  *var = __fdiv_rn(v, nf);
}

__device__ __forceinline__ float sqrt_via_double(float v) {
  return __double2float_rn(__dsqrt_rn((double)v));
}

}  // namespace

__global__ __launch_bounds__(SSIM_THREADS) void me_ssim_kernel(SearchArgs p, int row0,
                                                               int win_lds_bytes) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[SSIM_THREADS / 64];
  const int tid = threadIdx.x;
  const int bx = (int)(blockIdx.x % (unsigned)p.nbx);
  const int by = row0 + (int)(blockIdx.x / (unsigned)p.nbx);
  const int B = p.blk, S = p.range;
  const int tlx = bx * B, tly = by * B;
  const int w = min(B, p.width - tlx), h = min(B, p.height - tly);
  const int wx0 = max(tlx - S, 0), wy0 = max(tly - S, 0);
  const int wx1 = min(tlx + w - 1 + S, p.width - 1), wy1 = min(tly + h - 1 + S, p.height - 1);
  const int ncx = wx1 - w + 1 - wx0 + 1, ncy = wy1 - h + 1 - wy0 + 1;
  const int ww = wx1 - wx0 + 1, wh = wy1 - wy0 + 1;

  uint8_t* cblk = smem;                        // w*h bytes, pitch w
  uint8_t* win = smem + ((B * B + 15) & ~15);  // ww*wh bytes when staged
  const bool staged = win_lds_bytes >= ww * wh;
  for (int i = tid; i < w * h; i += SSIM_THREADS) {
    const int oy = i / w, ox = i - oy * w;
    cblk[i] = p.cur[(ptrdiff_t)(tly + oy - p.cur_row0) * p.stride + tlx + ox];
  }
  if (staged)
    for (int i = tid; i < ww * wh; i += SSIM_THREADS) {
      const int oy = i / ww, ox = i - oy * ww;
      win[i] = p.ref[(ptrdiff_t)(wy0 + oy - p.ref_row0) * p.stride + wx0 + ox];
    }
  __syncthreads();

  const float nf = (float)(w * h);
  const float C1 = 0.01f, C2 = 0.09f, C3 = 0.045f;  // ssim.c:48
  // Statistics of the current block (the reference recomputes them for every
  // candidate; they are the same numbers).
  float mp, vp;
  patch_stats(cblk, w, w, h, nf, &mp, &vp);
  const float sp = sqrt_via_double(vp);
  const int imp = (int)mp;  // truncation, as the int parameter of computeCrossVar

  // Lane = Q horizontally adjacent candidates: one cur byte and one ref byte
  // per pixel step feed all Q (a sliding register window of ref bytes), and
  // the 2Q float chains are independent (each still in raster order).
  uint64_t best = ~0ull;
  const int ngx = (ncx + SSIM_Q - 1) / SSIM_Q;
  const int ngroups = ngx * ncy;
  for (int t = tid; t < ngroups; t += SSIM_THREADS) {
    const int cy = t / ngx, cx0 = (t - cy * ngx) * SSIM_Q;
    const uint8_t* r = staged ? win + cy * ww + cx0
                              : p.ref + (ptrdiff_t)(wy0 + cy - p.ref_row0) * p.stride + wx0 + cx0;
    const int rp = staged ? ww : p.stride;
    // Columns past the window (candidates cx0 + k >= ncx of the last group)
    // are read but never used: padded in LDS, clamped in global memory.
    const int lim = staged ? 0x7FFFFFFF : ww - 1 - cx0;
    auto rb = [&](int y, int x) -> int { return r[y * rp + min(x, lim)]; };

    int s[SSIM_Q];
#pragma unroll
    for (int k = 0; k < SSIM_Q; k++) s[k] = 0;
    for (int y = 0; y < h; y++) {
      int rw[SSIM_Q];
#pragma unroll
      for (int k = 0; k < SSIM_Q - 1; k++) rw[k + 1] = rb(y, k);
      for (int x = 0; x < w; x++) {
#pragma unroll
        for (int k = 0; k < SSIM_Q - 1; k++) rw[k] = rw[k + 1];
        rw[SSIM_Q - 1] = rb(y, x + SSIM_Q - 1);
#pragma unroll
        for (int k = 0; k < SSIM_Q; k++) s[k] += rw[k];
      }
    }
    float mr[SSIM_Q], vr[SSIM_Q], cv[SSIM_Q];
    int imr[SSIM_Q];
#pragma unroll
    for (int k = 0; k < SSIM_Q; k++) {
      mr[k] = __fdiv_rn((float)s[k], nf);
      imr[k] = (int)mr[k];
      vr[k] = 0.f;
      cv[k] = 0.f;
    }
    for (int y = 0; y < h; y++) {
      int rw[SSIM_Q];
#pragma unroll
      for (int k = 0; k < SSIM_Q - 1; k++) rw[k + 1] = rb(y, k);
      for (int x = 0; x < w; x++) {
#pragma unroll
        for (int k = 0; k < SSIM_Q - 1; k++) rw[k] = rw[k + 1];
        rw[SSIM_Q - 1] = rb(y, x + SSIM_Q - 1);
        const int cc = cblk[y * w + x] - imp;
#pragma unroll
        for (int k = 0; k < SSIM_Q; k++) {
          const float d = __fsub_rn((float)rw[k], mr[k]);
          vr[k] = __fadd_rn(vr[k], __fmul_rn(d, d));
          cv[k] = __fadd_rn(cv[k], (float)((rw[k] - imr[k]) * cc));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < SSIM_Q; k++) {
      if (cx0 + k >= ncx) break;
      const float sr = sqrt_via_double(__fdiv_rn(vr[k], nf));
      const float cvk = __fdiv_rn(cv[k], nf);
      const float m = mr[k];
      const float lum = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, m), mp), C1),
                                  __fadd_rn(__fadd_rn(__fmul_rn(m, m), __fmul_rn(mp, mp)), C1));
      const float con = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, sr), sp), C2),
                                  __fadd_rn(__fadd_rn(__fmul_rn(sr, sr), __fmul_rn(sp, sp)), C2));
      const float str = __fdiv_rn(__fadd_rn(cvk, C3), __fadd_rn(__fmul_rn(sr, sp), C3));
      const float score = __fmul_rn(__fmul_rn(lum, con), str);
      if (score > 0.f) {
        const int dx = wx0 + cx0 + k - tlx, dy = wy0 + cy - tly;
        const uint64_t key = ((uint64_t)(0x7FFFFFFFu - __float_as_uint(score)) << 32) |
                             ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
        best = key < best ? key : best;
      }
    }
  }
  best = wave_min(best);
  if ((tid & 63) == 0) red[tid >> 6] = best;
  __syncthreads();
  if (tid == 0) {
    uint64_t b = red[0];
#pragma unroll
    for (int i = 1; i < SSIM_THREADS / 64; i++) b = red[i] < b ? red[i] : b;
    int dx = 0, dy = 0;
    uint32_t bits = 0;
    if (b != ~0ull) {
      dx = (int)(b & 0xFFFF) - 32768;
      dy = (int)((b >> 16) & 0xFFFF) - 32768;
      bits = 0x7FFFFFFFu - (uint32_t)(b >> 32);
    }
    const int out = (by - p.block_row_begin) * p.nbx + bx;
    p.mv[2 * out] = (int16_t)dx;
    p.mv[2 * out + 1] = (int16_t)dy;
    if (p.cost) p.cost[out] = bits;
  }
}

hipError_t launch_ssim(const SearchArgs& p, hipStream_t stream) {
  const int rows = p.block_row_end - p.block_row_begin;
  if (rows <= 0 || p.nbx <= 0) return hipSuccess;
  const int B = p.blk;
  long win = (long)(B + 2 * p.range) * (B + 2 * p.range);
  const int cur = (B * B + 15) & ~15;
  if (cur + win + SSIM_Q > GENERIC_LDS_BUDGET) win = 0;  // read the window from global memory
  // + SSIM_Q bytes: the last candidate group of the last row reads past the window
  hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(rows * p.nbx)), dim3(SSIM_THREADS),
                     cur + (int)win + SSIM_Q, stream, p, p.block_row_begin, (int)win);
  return hipGetLastError();
}

}  // namespace me
