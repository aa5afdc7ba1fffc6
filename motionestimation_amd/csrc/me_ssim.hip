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
// block and its window are staged in LDS when they fit.  Float-chain bound,
// not a hot path of the headline metric.
//
// Patch statistics prepass (round 3): a ref patch's mean and stddev depend on
// its position only, yet every block whose window covers the position
// recomputed them (about (2S/B + 1)^2 = 25 times at B = 16, S = 32).
// me_ssim_stats_kernel computes them once per position of the full B x B
// patches with the same float operations in the same order (ssim.c:3-28, the
// same patch_stats as below), so they are the same bits; the search then runs
// only the cross-term chain per candidate.  Blocks of a partial right column or
// bottom row (w or h < B) keep the in-kernel statistics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_kernels.h"

namespace me {

namespace {

constexpr int SSIM_THREADS = 256;
constexpr int SSIM_Q = 4;   // adjacent candidates per lane (in-kernel statistics)
constexpr int SSIM_QP = 8;  // ... with the statistics plane (one cross chain each)
constexpr int SSIM_Q16 = 12; // ... 16 x 16 blocks (1080p +-32: 6: 1.27 ms, 8: 0.88, 12: 0.72, 16: 0.81; profiles/r03bc_*, r03bd_*)
// LDS bytes past the window: the last row's last candidate group reads up to
// SSIM_QP (8-candidate groups) or SSIM_Q16 - 1 (16x16 register rows) bytes past it
constexpr int SSIM_PAD = SSIM_QP > SSIM_Q16 - 1 ? SSIM_QP : SSIM_Q16 - 1;

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

// Statistics plane: entry (rr, x) = (mean, stddev) of the B x B ref patch at
// frame row ylo + rr, column x (x in [0, W - B]), for every position a full
// block of block rows [block_row_begin, block_row_end) can meet.
struct SsimPlane {
  int ylo, rows, pitch;
};

static bool ssim_plane(const SearchArgs& p, SsimPlane* s) {
  const int B = p.blk, S = p.range, W = p.width, H = p.height;
  if (W < B || H < B || B > 64) return false;
  const int r0 = p.block_row_begin;
  int r1 = p.block_row_end;
  if (r1 * B > H) r1--;  // the partial bottom block row keeps the in-kernel statistics
  if (r1 <= r0) return false;
  s->ylo = max(r0 * B - S, 0);
  s->rows = min((r1 - 1) * B + S, H - B) - s->ylo + 1;
  s->pitch = W - B + 1;
  return s->rows > 0;
}

size_t ssim_scratch(const SearchArgs& p) {
  SsimPlane s;
  if (p.cost_kind != COST_SSIM || !ssim_plane(p, &s)) return 0;
  return (size_t)s.rows * (size_t)s.pitch * sizeof(float2);
}

// Workgroup = 64 columns x 16 rows of positions: the 16 + B - 1 ref rows they
// read are staged once in LDS; thread (column c, row group g) then computes
// positions (c, 4 g .. 4 g + 3), each as patch_stats does: the integer sum, then
// the float chain over the patch in raster order, a row's bytes taken four at
// a time from two aligned LDS words (v_alignbyte, v_cvt_f32_ubyte).  One thread
// per position straight from global memory took 226 us at 1080p (byte loads).
constexpr int STATS_TR = 16 + 63;  // staged rows for B <= 64
constexpr int STATS_TW = 33;       // staged words per row: 64 + 63 bytes + an aligned tail word

template <int BT>
__device__ __forceinline__ void stats_at(const uint32_t* t, int pr, int c, int Bdyn, float* m,
                                         float* v) {
  const int B = BT > 0 ? BT : Bdyn;
  const int a = c & 3, wb = c >> 2, G = (B + 3) >> 2;
  const float nf = (float)(B * B);
  auto word = [&](int i, int q) -> uint32_t {
    const uint32_t* row = t + (pr + i) * STATS_TW + wb + q;
    return __builtin_amdgcn_alignbyte(row[1], row[0], (uint32_t)a);
  };
  // raster order: rows i, then the row's groups q of four bytes (the compile-
  // time B are fully unrolled; a runtime B loops)
  auto rows = [&](auto&& body) {
    if constexpr (BT > 0) {
#pragma unroll
      for (int i = 0; i < BT; i++)
#pragma unroll
        for (int q = 0; q < (BT + 3) / 4; q++) body(i, q);
    } else {
      for (int i = 0; i < B; i++)
        for (int q = 0; q < G; q++) body(i, q);
    }
  };
  uint32_t s = 0;
  rows([&](int i, int q) {
    uint32_t w = word(i, q);
    const int nb = B - 4 * q;
    if (nb < 4) w &= (1u << (8 * nb)) - 1u;
    s = __builtin_amdgcn_sad_u8(w, 0u, s);
  });
  const float mf = __fdiv_rn((float)s, nf);
  float acc = 0.f;
  rows([&](int i, int q) {
    const uint32_t w = word(i, q);
#pragma unroll
    for (int b = 0; b < 4; b++) {
      if (4 * q + b < B) {
        const float d = __fsub_rn((float)((w >> (8 * b)) & 255u), mf);
        acc = __fadd_rn(acc, __fmul_rn(d, d));
      }
    }
  });
  *m = mf;
  *v = __fdiv_rn(acc, nf);
}

__global__ __launch_bounds__(256) void me_ssim_stats_kernel(SearchArgs p, SsimPlane s,
                                                            float2* plane) {
  __shared__ uint32_t t[STATS_TR * STATS_TW];
  const int B = p.blk;
  const int x0 = (int)blockIdx.x * 64, y0 = (int)blockIdx.y * 16;
  const int tid = (int)threadIdx.x;
  uint8_t* tb = reinterpret_cast<uint8_t*>(t);
  const int rows = 16 + B - 1;
  // row r, byte col <- ref(ylo + y0 + r, x0 + col); 0 past the frame or the
  // resident rows (never read by a position inside the plane)
  for (int i = tid; i < rows * STATS_TW * 4; i += 256) {
    const int r = i / (STATS_TW * 4), col = i - r * (STATS_TW * 4);
    const int y = s.ylo + y0 + r, xx = x0 + col;
    tb[i] = (xx < p.width && y < s.ylo + s.rows + B - 1)
                ? p.ref[(ptrdiff_t)(y - p.ref_row0) * p.stride + xx] : 0;
  }
  __syncthreads();
  const int c = tid & 63, g = tid >> 6, x = x0 + c;
  if (x >= s.pitch) return;
#pragma unroll 1
  for (int j = 0; j < 4; j++) {
    const int pr = 4 * g + j, rr = y0 + pr;
    if (rr >= s.rows) break;
    float m, v;
    switch (B) {
      case 16: stats_at<16>(t, pr, c, B, &m, &v); break;
      case 8: stats_at<8>(t, pr, c, B, &m, &v); break;
      default: stats_at<0>(t, pr, c, B, &m, &v); break;
    }
    plane[(size_t)rr * s.pitch + x] = make_float2(m, sqrt_via_double(v));
  }
}

__global__ __launch_bounds__(SSIM_THREADS) void me_ssim_kernel(SearchArgs p, int row0,
                                                               int win_lds_bytes,
                                                               const float2* stats, SsimPlane pg) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[SSIM_THREADS / 64];
  __shared__ float ccl[256];  // 16 x 16 blocks with the statistics plane: (c - imc) as floats
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
  // ssim.c:53-56 for candidate (cx0 + k, cy) of a group: the key, or ~0
  auto key_of = [&](float m, float sr, float cvsum, int cx, int cy) -> uint64_t {
    const float cvk = __fdiv_rn(cvsum, nf);
    const float lum = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, m), mp), C1),
                                __fadd_rn(__fadd_rn(__fmul_rn(m, m), __fmul_rn(mp, mp)), C1));
    const float con = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, sr), sp), C2),
                                __fadd_rn(__fadd_rn(__fmul_rn(sr, sr), __fmul_rn(sp, sp)), C2));
    const float str = __fdiv_rn(__fadd_rn(cvk, C3), __fadd_rn(__fmul_rn(sr, sp), C3));
    const float score = __fmul_rn(__fmul_rn(lum, con), str);
    if (!(score > 0.f)) return ~0ull;
    const int dx = wx0 + cx - tlx, dy = wy0 + cy - tly;
    return ((uint64_t)(0x7FFFFFFFu - __float_as_uint(score)) << 32) |
           ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
  };
  if (stats != nullptr && B == 16 && w == 16 && h == 16 && staged) {
    // 16 x 16 blocks, window in LDS: per window row the lane's SSIM_Q16
    // candidates' 16 + SSIM_Q16 - 1 ref bytes as floats in registers, the
    // block's (c - imc) as floats in LDS (broadcast reads), the row's 16 pixels
    // unrolled (no register shifts).  The same chains as below, in the same order.
    constexpr int Q = SSIM_Q16;
    for (int i = tid; i < 256; i += SSIM_THREADS) ccl[i] = (float)(cblk[i] - imp);
    __syncthreads();
    const int ngq = (ncx + Q - 1) / Q, ng = ngq * ncy;
    for (int t = tid; t < ng; t += SSIM_THREADS) {
      const int cy = t / ngq, cx0 = (t - cy * ngq) * Q;
      const uint8_t* r = win + cy * ww + cx0;  // past the window: the launch's SSIM_PAD bytes
      const float2* st = stats + (size_t)(wy0 + cy - pg.ylo) * pg.pitch;
      float fimr[Q], cv[Q];
#pragma unroll
      for (int k = 0; k < Q; k++) {
        fimr[k] = (float)(int)st[min(wx0 + cx0 + k, pg.pitch - 1)].x;
        cv[k] = 0.f;
      }
#pragma unroll 1
      for (int y = 0; y < 16; y++) {
        float rf[16 + Q - 1];
#pragma unroll
        for (int j = 0; j < 16 + Q - 1; j++) rf[j] = (float)r[y * ww + j];
#pragma unroll
        for (int x = 0; x < 16; x++) {
          const float c = ccl[y * 16 + x];
#pragma unroll
          for (int k = 0; k < Q; k++) cv[k] = __fmaf_rn(__fsub_rn(rf[x + k], fimr[k]), c, cv[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < Q; k++) {
        if (cx0 + k >= ncx) break;
        const float2 v = st[wx0 + cx0 + k];
        const uint64_t key = key_of(v.x, v.y, cv[k], cx0 + k, cy);
        best = key < best ? key : best;
      }
    }
  } else if (stats != nullptr && w == B && h == B) {
    // Full block: patch statistics from the prepass plane; per candidate only
    // the cross chain fl(cv + (r - imr)(c - imc)) in raster order.  The product
    // is an exact integer below 2^24, so fma(r - imr, c - imc, cv) (operands
    // exact in float) rounds once, exactly where the reference's add rounds.
    const int ngx8 = (ncx + SSIM_QP - 1) / SSIM_QP;
    const int ngroups8 = ngx8 * ncy;
    for (int t = tid; t < ngroups8; t += SSIM_THREADS) {
      const int cy = t / ngx8, cx0 = (t - cy * ngx8) * SSIM_QP;
      const uint8_t* r = staged ? win + cy * ww + cx0
                                : p.ref + (ptrdiff_t)(wy0 + cy - p.ref_row0) * p.stride + wx0 + cx0;
      const int rp = staged ? ww : p.stride;
      const int lim = staged ? 0x7FFFFFFF : ww - 1 - cx0;
      auto rb = [&](int y, int x) -> float { return (float)r[y * rp + min(x, lim)]; };
      const float2* st = stats + (size_t)(wy0 + cy - pg.ylo) * pg.pitch;
      float fimr[SSIM_QP], cv[SSIM_QP];
#pragma unroll
      for (int k = 0; k < SSIM_QP; k++) {
        // past ncx: read (clamped), never used
        fimr[k] = (float)(int)st[min(wx0 + cx0 + k, pg.pitch - 1)].x;
        cv[k] = 0.f;
      }
      for (int y = 0; y < h; y++) {
        float rf[SSIM_QP];
#pragma unroll
        for (int k = 0; k < SSIM_QP - 1; k++) rf[k + 1] = rb(y, k);
        for (int x = 0; x < w; x++) {
#pragma unroll
          for (int k = 0; k < SSIM_QP - 1; k++) rf[k] = rf[k + 1];
          rf[SSIM_QP - 1] = rb(y, x + SSIM_QP - 1);
          const float ccf = (float)(cblk[y * w + x] - imp);
#pragma unroll
          for (int k = 0; k < SSIM_QP; k++)
            cv[k] = __fmaf_rn(__fsub_rn(rf[k], fimr[k]), ccf, cv[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < SSIM_QP; k++) {
        if (cx0 + k >= ncx) break;
        const float2 v = st[wx0 + cx0 + k];
        const uint64_t key = key_of(v.x, v.y, cv[k], cx0 + k, cy);
        best = key < best ? key : best;
      }
    }
  } else
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
      const uint64_t key =
          key_of(mr[k], sqrt_via_double(__fdiv_rn(vr[k], nf)), cv[k], cx0 + k, cy);
      best = key < best ? key : best;
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
  note_path(7);
  const int rows = p.block_row_end - p.block_row_begin;
  if (rows <= 0 || p.nbx <= 0) return hipSuccess;
  const int B = p.blk;
  long win = (long)(B + 2 * p.range) * (B + 2 * p.range);
  const int cur = (B * B + 15) & ~15;
  if (cur + win + SSIM_PAD > GENERIC_LDS_BUDGET) win = 0;  // read the window from global memory
  // Patch statistics plane in the context scratch when it holds one (attach_scratch
  // sizes it with ssim_scratch); otherwise every block computes its own.
  SsimPlane sp{0, 0, 0};
  const float2* stats = nullptr;
  const size_t need = ssim_scratch(p);
  if (need && p.scratch && p.scratch_bytes >= need && ssim_plane(p, &sp)) {
    float2* plane = reinterpret_cast<float2*>(p.scratch);
    hipLaunchKernelGGL(me_ssim_stats_kernel, dim3((unsigned)((sp.pitch + 63) / 64),
                                                  (unsigned)((sp.rows + 15) / 16)),
                       dim3(256), 0, stream, p, sp, plane);
    stats = plane;
  }
  // + SSIM_PAD bytes: the last candidate group of the last row reads past the window
  hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(rows * p.nbx)), dim3(SSIM_THREADS),
                     cur + (int)win + SSIM_PAD, stream, p, p.block_row_begin, (int)win, stats, sp);
  return hipGetLastError();
}

}  // namespace me
