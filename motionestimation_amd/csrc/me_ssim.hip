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
// (packed fp32: one v_pk_add + one v_pk_fma per two candidate pixels), not a
// hot path of the headline metric.
//
// Patch statistics prepass (round 3): a ref patch's mean and stddev depend on
// its position only, yet every block whose window covers the position
// recomputed them (about (2S/B + 1)^2 = 25 times at B = 16, S = 32).
// me_ssim_stats_kernel computes them once per position of the full B x B
// patches with the same float operations in the same order (ssim.c:3-28, the
// same patch_stats as below), so they are the same bits; the search then runs
// only the cross-term chain per candidate.  Blocks of a partial right column or
// bottom row (w or h < B) keep the in-kernel statistics, except for 16 x 16
// blocks (round 6): the full-width blocks of the partial bottom row get a
// plane of 16 x (H % 16) patches and run on the matrix cores with the rest
// (me_ssim_mfma_kernel below).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "me_kernels.h"
#include "me_mfma_util.h"

namespace me {

namespace {

constexpr int SSIM_THREADS = 256;
constexpr int SSIM_Q = 4;   // adjacent candidates per lane (in-kernel statistics)
constexpr int SSIM_QP = 8;  // ... with the statistics plane (one cross chain each)
// ... 16 x 16 blocks with the statistics plane on the float path (1080p +-32:
// 6: 1.27 ms, 8: 0.88, 12: 0.72, 16: 0.81; profiles/r03bc_*, r03bd_*; 13 and
// workgroups sized to one round of lane-tasks: slower, profiles/r06k_*)
constexpr int SSIM_Q16 = 12;
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

// ssim.c:53-56 for one candidate: the ref patch's mean m and stddev sr, the
// cross variance cvk, the current block's mean mp and stddev sp -> the key
// (0x7FFFFFFF - bits(score)) << 32 | (dy, dx), or ~0 for a score <= 0.
__device__ __forceinline__ uint64_t ssim_key(float m, float sr, float cvk, float mp, float sp,
                                             int dx, int dy) {
  const float C1 = 0.01f, C2 = 0.09f, C3 = 0.045f;  // ssim.c:48
  const float lum = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, m), mp), C1),
                              __fadd_rn(__fadd_rn(__fmul_rn(m, m), __fmul_rn(mp, mp)), C1));
  const float con = __fdiv_rn(__fadd_rn(__fmul_rn(__fmul_rn(2.f, sr), sp), C2),
                              __fadd_rn(__fadd_rn(__fmul_rn(sr, sr), __fmul_rn(sp, sp)), C2));
  const float str = __fdiv_rn(__fadd_rn(cvk, C3), __fadd_rn(__fmul_rn(sr, sp), C3));
  const float score = __fmul_rn(__fmul_rn(lum, con), str);
  if (!(score > 0.f)) return ~0ull;
  return ((uint64_t)(0x7FFFFFFFu - __float_as_uint(score)) << 32) |
         ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
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

// The partial bottom block row's plane (16 x 16 blocks, S <= 64, the row in
// the search): entry (rr, x) = (mean, stddev) of the 16 x hbh ref patch at
// row ylo + rr, column x, for every position its blocks can meet; the
// matrix-core SSIM kernel runs that row too.
static bool ssim_hb_plane(const SearchArgs& p, SsimPlane* s, int* hbh) {
  const int S = p.range, W = p.width, H = p.height;
  if (p.blk != 16 || S > 64 || W < 16 || H < 16 || H % 16 == 0) return false;
  const int hb_row = H / 16;
  if (hb_row < p.block_row_begin || hb_row >= p.block_row_end) return false;
  *hbh = H - 16 * hb_row;
  s->ylo = max(16 * hb_row - S, 0);
  s->rows = H - *hbh - s->ylo + 1;
  s->pitch = W - 15;
  return s->rows > 0;
}

static size_t ssim_plane_bytes(const SsimPlane& s) {
  return ((size_t)s.rows * (size_t)s.pitch * sizeof(float2) + 255) & ~(size_t)255;
}

size_t ssim_scratch(const SearchArgs& p) {
  if (p.cost_kind != COST_SSIM) return 0;
  SsimPlane s, h;
  int hbh;
  size_t n = ssim_plane(p, &s) ? ssim_plane_bytes(s) : 0;
  if (ssim_hb_plane(p, &h, &hbh)) n += ssim_plane_bytes(h);
  return n;
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

// patch_stats of a 16-wide, hgt-row patch (the partial bottom row's, hgt < 16):
// stats_at's operations with a runtime row count.
__device__ __forceinline__ void stats_w16(const uint32_t* t, int pr, int c, int hgt, float* m,
                                          float* v) {
  const int a = c & 3, wb = c >> 2;
  const float nf = (float)(16 * hgt);
  auto word = [&](int i, int q) -> uint32_t {
    const uint32_t* row = t + (pr + i) * STATS_TW + wb + q;
    return __builtin_amdgcn_alignbyte(row[1], row[0], (uint32_t)a);
  };
  uint32_t s = 0;
  for (int i = 0; i < hgt; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) s = __builtin_amdgcn_sad_u8(word(i, q), 0u, s);
  const float mf = __fdiv_rn((float)s, nf);
  float acc = 0.f;
  for (int i = 0; i < hgt; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t w = word(i, q);
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const float d = __fsub_rn((float)((w >> (8 * b)) & 255u), mf);
        acc = __fadd_rn(acc, __fmul_rn(d, d));
      }
    }
  *m = mf;
  *v = __fdiv_rn(acc, nf);
}

// ph: the patches' height (p.blk; the partial bottom row's plane: hbh < 16)
__global__ __launch_bounds__(256) void me_ssim_stats_kernel(SearchArgs p, SsimPlane s,
                                                            float2* plane, int ph) {
  __shared__ uint32_t t[STATS_TR * STATS_TW];
  const int B = p.blk;
  const int x0 = (int)blockIdx.x * 64, y0 = (int)blockIdx.y * 16;
  const int tid = (int)threadIdx.x;
  uint8_t* tb = reinterpret_cast<uint8_t*>(t);
  const int rows = 16 + ph - 1;
  // row r, byte col <- ref(ylo + y0 + r, x0 + col); 0 past the frame or the
  // resident rows (never read by a position inside the plane)
  for (int i = tid; i < rows * STATS_TW * 4; i += 256) {
    const int r = i / (STATS_TW * 4), col = i - r * (STATS_TW * 4);
    const int y = s.ylo + y0 + r, xx = x0 + col;
    tb[i] = (xx < p.width && y < s.ylo + s.rows + ph - 1)
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
    if (ph != B)
      stats_w16(t, pr, c, ph, &m, &v);
    else
      switch (B) {
        case 16: stats_at<16>(t, pr, c, B, &m, &v); break;
        case 8: stats_at<8>(t, pr, c, B, &m, &v); break;
        default: stats_at<0>(t, pr, c, B, &m, &v); break;
      }
    plane[(size_t)rr * s.pitch + x] = make_float2(m, sqrt_via_double(v));
  }
}

// Blocks [row0, ..) x [col0, nbx) of the launch's rows (grid = rows x (nbx - col0)).
__global__ __launch_bounds__(SSIM_THREADS) void me_ssim_kernel(SearchArgs p, int row0, int col0,
                                                               int win_lds_bytes,
                                                               const float2* stats, SsimPlane pg) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[SSIM_THREADS / 64];
  __shared__ float ccl[256];  // 16 x 16 blocks with the statistics plane: (c - imc) as floats
  __shared__ float cstat[2];  // the current block's mean and variance
  const int tid = threadIdx.x, nt = (int)blockDim.x;
  const int ncol = p.nbx - col0;
  const int bx = col0 + (int)(blockIdx.x % (unsigned)ncol);
  const int by = row0 + (int)(blockIdx.x / (unsigned)ncol);
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
  for (int i = tid; i < w * h; i += nt) {
    const int oy = i / w, ox = i - oy * w;
    cblk[i] = p.cur[(ptrdiff_t)(tly + oy - p.cur_row0) * p.stride + tlx + ox];
  }
  if (staged)
    for (int i = tid; i < ww * wh; i += nt) {
      const int oy = i / ww, ox = i - oy * ww;
      win[i] = p.ref[(ptrdiff_t)(wy0 + oy - p.ref_row0) * p.stride + wx0 + ox];
    }
  __syncthreads();

  const float nf = (float)(w * h);
  // Statistics of the current block (the reference recomputes them for every
  // candidate; they are the same numbers): one serial float chain, run by
  // wave 0 alone (every wave running it cost ~1/6 of a 16 x 16 workgroup's
  // VALU issue) and handed over in LDS.
  if (tid < 64) {
    float m0, v0;
    patch_stats(cblk, w, w, h, nf, &m0, &v0);
    if (tid == 0) {
      cstat[0] = m0;
      cstat[1] = v0;
    }
  }
  __syncthreads();
  const float mp = cstat[0], vp = cstat[1];
  const float sp = sqrt_via_double(vp);
  const int imp = (int)mp;  // truncation, as the int parameter of computeCrossVar

  // Lane = Q horizontally adjacent candidates: one cur byte and one ref byte
  // per pixel step feed all Q (a sliding register window of ref bytes), and
  // the 2Q float chains are independent (each still in raster order).
  uint64_t best = ~0ull;
  const int ngx = (ncx + SSIM_Q - 1) / SSIM_Q;
  const int ngroups = ngx * ncy;
  // ssim.c:53-56 for candidate (cx0 + k, cy) of a group: the key, or ~0
  // cv / nf: nf = w h a power of two (the full 16 x 16 and 8 x 8 blocks)
  // divides exactly as a multiplication by 1 / nf (both are the correctly
  // rounded x 2^-k); the 10-instruction division otherwise
  const int nfi = w * h;
  const bool pow2 = (nfi & (nfi - 1)) == 0;
  const float inv_nf = 1.0f / nf;  // exact when nf is a power of two
  auto key_of = [&](float m, float sr, float cvsum, int cx, int cy) -> uint64_t {
    const float cvk = pow2 ? __fmul_rn(cvsum, inv_nf) : __fdiv_rn(cvsum, nf);
    return ssim_key(m, sr, cvk, mp, sp, wx0 + cx - tlx, wy0 + cy - tly);
  };
  if (stats != nullptr && B == 16 && w == 16 && h == 16 && staged) {
    // 16 x 16 blocks, window in LDS: per window row the lane's SSIM_Q16
    // candidates' 16 + SSIM_Q16 - 1 ref bytes as floats in registers, the
    // block's (c - imc) as floats in LDS (broadcast reads), the row's 16 pixels
    // unrolled (no register shifts).  The same chains as below, in the same order.
    constexpr int Q = SSIM_Q16;
    for (int i = tid; i < 256; i += nt) ccl[i] = (float)(cblk[i] - imp);
    __syncthreads();
    const int ngq = (ncx + Q - 1) / Q, ng = ngq * ncy;
    for (int t = tid; t < ng; t += nt) {
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
    for (int t = tid; t < ngroups8; t += nt) {
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
  for (int t = tid; t < ngroups; t += nt) {
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
    for (int i = 1; i < nt / 64; i++) b = red[i] < b ? red[i] : b;
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

// ---------------------------------------------------------------------------
// 16 x 16 blocks on the matrix cores.  The reference's cross variance is an
// exact integer for a 16 x 16 block: each term (r - imr)(c - imc) is an int
// with |term| <= 255^2, so every partial sum of the float chain
// (computeCrossVar, ssim.c:30-42) is an integer below 256 * 255^2 =
// 16,646,400 < 2^24 and exactly representable: the chain's result does not
// depend on its order.  So
//   cv = sum r c - imc S1r - imr S1c + 256 imr imc,
//   sum r c = 127 S1r + 128 S1c - 4161536 - X,  X = sum (127 - c)(r - 128)
// (S1r / S1c the patch / block byte sums, imr = S1r >> 8 = (int) mean_r, imc
// likewise), and X is the i8 GEMM the SSD path already runs on
// v_mfma_i32_16x16x64_i8 in the block-major layout (me_band.hip /
// me_mfma.hip): one workgroup per block, 16 x 16 candidate tiles (16 x
// positions by 16 y positions, 8 MFMAs each, K = two block rows in a 32-byte
// span), and per candidate only the score's float operations in the
// reference's order (ssim_key, as the float path) from the statistics plane's
// mean and stddev.  The float path spent ~128 VALU per candidate on the chain.
constexpr int SSIM_CREC = 48;                                // row record: 0^16, c ^ 0x7F, 0^16

__host__ __device__ inline int ssim_mfma_lp(int S) { return 16 * ((2 * S + 15) / 16 + 3); }
__host__ __device__ inline int ssim_mfma_rows(int S) { return 16 * ((2 * S + 1 + 15) / 16) + 15; }
__host__ __device__ inline int ssim_mfma_lds(int S) {
  return 256 + 16 * SSIM_CREC + ssim_mfma_rows(S) * ssim_mfma_lp(S);
}

// bh: the blocks' height -- 16, or the partial bottom row's H % 16 (its own
// statistics plane; N = 16 bh pixels <= 256, so the identity above holds with
// 256 -> N and 4161536 -> 16256 N; record rows >= bh are zero)
__global__ __launch_bounds__(256) void me_ssim_mfma_kernel(SearchArgs p, int row0, int nbxf,
                                                           const float2* stats, SsimPlane pg,
                                                           int aligned16, int bh) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[4];
  __shared__ float cstat[2];
  __shared__ int csum;
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const uint32_t lds_c32;
  typedef __attribute__((address_space(3))) const v4i lds_cv4i;
  auto lds_addr = [](const void* q) {
    return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)q);
  };
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, hh = lane >> 4;
  const int bx = (int)(blockIdx.x % (unsigned)nbxf), by = row0 + (int)(blockIdx.x / (unsigned)nbxf);
  const int S = p.range, W = p.width, H = p.height;
  const int tlx = 16 * bx, tly = 16 * by;
  const int wx0 = max(tlx - S, 0), wy0 = max(tly - S, 0);
  const int ncx = min(tlx + S, W - 16) - wx0 + 1, ncy = min(tly + S, H - bh) - wy0 + 1;
  const int i0 = wx0 >> 4, ni = ((wx0 + ncx - 1) >> 4) - i0 + 1, nj = (ncy + 15) >> 4;
  const int LP = ssim_mfma_lp(S), R = 16 * nj + 15;
  uint8_t* cblk = smem;                        // the block, raw
  uint8_t* crec = smem + 256;                  // 16 row records
  uint8_t* win = crec + 16 * SSIM_CREC;        // rows wy0 .., columns 16 i0 ..: r ^ 0x80
  for (int i = tid; i < 256; i += 256) {
    const int oy = i >> 4, ox = i & 15;
    const uint8_t c = oy < bh ? p.cur[(ptrdiff_t)(tly + oy - p.cur_row0) * p.stride + tlx + ox] : 0;
    cblk[i] = c;
    crec[oy * SSIM_CREC + 16 + ox] = oy < bh ? c ^ 0x7F : 0;
    crec[oy * SSIM_CREC + ox] = 0;
    crec[oy * SSIM_CREC + 32 + ox] = 0;
  }
  // (columns and rows past the frame: zeros or the next bytes of the plane;
  // only masked candidates read them)
  if (aligned16) {
    // 16-byte granules through a buffer resource over the resident rows
    // (reads past it return 0)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    const __amdgpu_buffer_rsrc_t rref =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.ref, (short)0, p.ref_bytes, 0x00020000);
    const int G = LP >> 4;
    for (int i = tid; i < R * G; i += 256) {
      const int rr = i / G, gq = i - rr * G;
      const uint32_t off = (uint32_t)((wy0 + rr - p.ref_row0) * p.stride + 16 * (i0 + gq));
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rref, off, 0, 0));
      *reinterpret_cast<lds_u32x4*>((uintptr_t)(lds_addr(win) + 16u * (uint32_t)i)) = v ^ 0x80808080u;
    }
  } else {
    for (int i = tid; i < R * LP; i += 256) {
      const int rr = i / LP, col = i - rr * LP;
      const int y = wy0 + rr, x = 16 * i0 + col;
      win[i] = (y < H && x < W) ? (uint8_t)(p.ref[(ptrdiff_t)(y - p.ref_row0) * p.stride + x] ^ 0x80) : 0;
    }
  }
  __syncthreads();
  // the block's statistics (ssim.c:3-28 as the float path: one serial chain,
  // wave 0) and byte sum
  const int N = 16 * bh;
  if (tid < 64) {
    float m0, v0;
    patch_stats(cblk, 16, 16, bh, (float)N, &m0, &v0);
    int cs = 0;
    for (int i = lane; i < 256; i += 64) cs += cblk[i];  // rows >= bh: 0
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cs += __shfl_xor(cs, off, 64);
    if (tid == 0) {
      cstat[0] = m0;
      cstat[1] = v0;
      csum = cs;
    }
  }
  // A fragments (me_band.hip's enter): lane (m = n, K group hh), fragment q =
  // bytes o .. o + 15 of record row 2 q + (hh >> 1), o = 16 + 16 (hh & 1) - m
  v4i A[8];
  {
    const int o = 16 + 16 * (hh & 1) - n, sh = o & 3;
    const uint32_t lb = lds_addr(crec) + (uint32_t)((hh >> 1) * SSIM_CREC + (o & ~3));
#pragma unroll
    for (int q = 0; q < 8; q++) {
      uint32_t d[5];
#pragma unroll
      for (int e = 0; e < 5; e++)
        d[e] = *reinterpret_cast<lds_c32*>((uintptr_t)(lb + (uint32_t)(2 * q * SSIM_CREC + 4 * e)));
#pragma unroll
      for (int e = 0; e < 4; e++) A[q][e] = (int)__builtin_amdgcn_alignbyte(d[e + 1], d[e], sh);
    }
  }
  __syncthreads();
  const float mp = cstat[0], sp = sqrt_via_double(cstat[1]);
  // (int) mp = S1c / N: the rounded quotient stays below the next integer
  // (1 - frac >= 1 / N is far above its ulp)
  const int S1c = csum, imc = (int)mp;
  const int kc = 128 * S1c - 16256 * N;
  const float nf = (float)N, inv_nf = 1.0f / nf;  // exact when N is a power of two
  const bool pow2 = (N & (N - 1)) == 0;
  uint64_t best = ~0ull;
  const uint32_t xb0 = lds_addr(win) + (uint32_t)((n + (hh >> 1)) * LP + 16 * (hh & 1));
#pragma unroll 1
  for (int t = wave; t < ni * nj; t += 4) {
    const int tj = t / ni, ti = t - tj * ni;
    // B fragment q: window row 16 tj + n + 2 q + (hh >> 1), column 16 ti + 16 (hh & 1)
    const uint32_t xb = xb0 + (uint32_t)(16 * tj * LP + 16 * ti);
    v4i f[8];
#pragma unroll
    for (int q = 0; q < 8; q++) f[q] = *reinterpret_cast<lds_cv4i*>((uintptr_t)(xb + (uint32_t)(2 * q * LP)));
    v4i acc = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 8; q++) acc = MFMA16(A[q], f[q], acc, 0, 0, 0);
    // lane (n, hh): X of positions x = 16 (i0 + ti) + 4 hh + r, y = wy0 + 16 tj + n
    const int cy = 16 * tj + n, cx0 = 16 * (i0 + ti) + 4 * hh - wx0;
    if (cy < ncy) {
      const float2* st = stats + (size_t)(wy0 + cy - pg.ylo) * pg.pitch + wx0;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int cx = cx0 + r;
        if (cx < 0 || cx >= ncx) continue;
        const float2 v = st[cx];
        // mean_r = fl(S1r / N): N mean_r is within N ulp / 2 < 1/2 of S1r
        const int S1r = __float2int_rn(__fmul_rn(v.x, nf));
        const int imr = (int)v.x;
        const int cv = 127 * S1r + kc - acc[r] - imc * S1r - imr * S1c + N * imr * imc;
        const float cvk = pow2 ? __fmul_rn((float)cv, inv_nf) : __fdiv_rn((float)cv, nf);
        const uint64_t key = ssim_key(v.x, v.y, cvk, mp, sp, wx0 + cx - tlx, wy0 + cy - tly);
        best = key < best ? key : best;
      }
    }
  }
  best = wave_min(best);
  if (lane == 0) red[wave] = best;
  __syncthreads();
  if (tid == 0) {
    uint64_t b = red[0];
#pragma unroll
    for (int i = 1; i < 4; i++) b = red[i] < b ? red[i] : b;
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
  // Patch statistics planes in the context scratch when it holds them
  // (attach_scratch sizes it with ssim_scratch); otherwise every block computes
  // its own.  The full rows' plane first, then the partial bottom row's.
  SsimPlane sp{0, 0, 0}, hp{0, 0, 0};
  const float2* stats = nullptr;
  const float2* hstats = nullptr;
  int hbh = 0;
  const size_t need = ssim_scratch(p);
  if (need && p.scratch && p.scratch_bytes >= need) {
    uint8_t* base = reinterpret_cast<uint8_t*>(p.scratch);
    if (ssim_plane(p, &sp)) {
      float2* plane = reinterpret_cast<float2*>(base);
      hipLaunchKernelGGL(me_ssim_stats_kernel, dim3((unsigned)((sp.pitch + 63) / 64),
                                                    (unsigned)((sp.rows + 15) / 16)),
                         dim3(256), 0, stream, p, sp, plane, B);
      stats = plane;
      base += ssim_plane_bytes(sp);
    }
    if (ssim_hb_plane(p, &hp, &hbh)) {
      float2* plane = reinterpret_cast<float2*>(base);
      hipLaunchKernelGGL(me_ssim_stats_kernel, dim3((unsigned)((hp.pitch + 63) / 64),
                                                    (unsigned)((hp.rows + 15) / 16)),
                         dim3(256), 0, stream, p, hp, plane, hbh);
      hstats = plane;
    }
  }
  // 16 x 16 blocks with the statistics planes, S <= 64: the full-width columns
  // on the matrix cores (full rows, then the partial bottom row with its own
  // plane); the partial right column on the float path
  const int a16 = p.stride % 16 == 0 && (uintptr_t)p.ref % 16 == 0 && p.ref_bytes > 0;
  const int nbxf = B == 16 && p.range <= 64 ? p.width / 16 : 0;
  int r_full = 0;
  if (stats && nbxf > 0) {
    r_full = std::max(0, std::min(p.block_row_end, p.height / 16) - p.block_row_begin);
    if (r_full > 0)
      hipLaunchKernelGGL(me_ssim_mfma_kernel, dim3((unsigned)(r_full * nbxf)), dim3(256),
                         ssim_mfma_lds(p.range), stream, p, p.block_row_begin, nbxf, stats, sp, a16,
                         16);
  }
  const bool hb_mfma = hstats && nbxf > 0;
  if (hb_mfma)
    hipLaunchKernelGGL(me_ssim_mfma_kernel, dim3((unsigned)nbxf), dim3(256), ssim_mfma_lds(p.range),
                       stream, p, p.height / 16, nbxf, hstats, hp, a16, hbh);
  // + SSIM_PAD bytes: the last candidate group of the last row reads past the window
  const int lds = cur + (int)win + SSIM_PAD;
  if (r_full == 0 && !hb_mfma) {
    hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(rows * p.nbx)), dim3(SSIM_THREADS), lds, stream,
                       p, p.block_row_begin, 0, (int)win, stats, sp);
  } else {
    // the rest: the partial right column of the full rows, then the partial
    // bottom row (its right-column block only when the row ran on the matrix cores)
    if (r_full > 0 && nbxf < p.nbx)
      hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(r_full * (p.nbx - nbxf))), dim3(SSIM_THREADS),
                         lds, stream, p, p.block_row_begin, nbxf, (int)win, stats, sp);
    const int rb = p.block_row_begin + r_full;
    if (rb < p.block_row_end) {
      const int col0 = hb_mfma ? nbxf : 0;
      if (col0 < p.nbx)
        hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)((p.block_row_end - rb) * (p.nbx - col0))),
                           dim3(SSIM_THREADS), lds, stream, p, rb, col0, (int)win, stats, sp);
    }
  }
  return hipGetLastError();
}

}  // namespace me
