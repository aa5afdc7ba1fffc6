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

typedef float f2v __attribute__((ext_vector_type(2)));

// a / b for two lane-halves, correctly rounded: the compiler's f32 division
// (v_div_scale, v_rcp_f32, the Newton / residual fma chain, v_div_fmas,
// v_div_fixup) without the scaling and fix-up steps.  Those are the identity
// when |a| and |b| lie in [2^-40, 2^40]: v_div_scale scales only for an
// exponent gap >= 96, a denormal or near-denormal numerator, or a denominator
// whose reciprocal is denormal, and v_div_fixup changes only NaN / inf / zero /
// overflowed results.  So these are __fdiv_rn's bits, two quotients per packed
// fma, for the SSIM score's operands, which stay in that range whatever the
// frame (means in [0, 255], stddevs in [0, 127.5], C1..C3 > 0.009):
//   lum  (2m mp + C1) / (m^2 + mp^2 + C1)       both in [0.01, 130051]
//   con  (2sr sp + C2) / (sr^2 + sp^2 + C2)     both in [0.09, 32514]
//   str  (cv / N + C3) / (sr sp + C3)           |cv / N + C3| in [2^-17, 2^27]
// (cv an integer: cv / N + 0.045 is never 0 for N = 16 k <= 256 and stays
// above 2^-17 in magnitude; |cv| < 2^31).  tests/test_gpu_ssim.py and the
// reference's goldens pin the bits.
__device__ __forceinline__ f2v div_rn2(f2v a, f2v b) {
  const f2v one = {1.f, 1.f};
  f2v y = {__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  const f2v e = __builtin_elementwise_fma(-b, y, one);
  y = __builtin_elementwise_fma(e, y, y);
  f2v q = a * y;
  f2v r = __builtin_elementwise_fma(-b, q, a);
  q = __builtin_elementwise_fma(r, y, q);
  r = __builtin_elementwise_fma(-b, q, a);
  return __builtin_elementwise_fma(r, y, q);
}

}  // namespace

// Statistics plane: entry (rr, x) = (mean, stddev) of the B x B ref patch at
// frame row ylo + rr, column x (x in [0, W - B]), for every position a full
// block of block rows [block_row_begin, block_row_end) can meet.
// 16 x 16 blocks with S <= 64 (the matrix-core kernel reads the plane) store
// it compact: stddev as float [rows][ld], then the patch byte sum S1r as u16
// [rows][ld] (the mean is S1r / N, exact for N = 256, and fl(S1r / N)
// otherwise), ld a multiple of 64 entries: a lane's four adjacent candidates
// are one 16-byte and one 8-byte load (float2 entries took four 8-byte loads,
// 32 tag lookups per wave each: ~49 of the kernel's 115 us at 1080p,
// profiles/r06q_*).  Other shapes: float2 (mean, stddev) [rows][ld = pitch].
struct SsimPlane {
  int ylo, rows, pitch, ld, compact;
};

static bool ssim_compact(const SearchArgs& p) { return p.blk == 16 && p.range <= 64; }

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
  s->compact = ssim_compact(p);
  s->ld = s->compact ? (s->pitch + 15 + 63) & ~63 : s->pitch;  // >= W: a tile's last column
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
  s->compact = 1;
  s->ld = (s->pitch + 15 + 63) & ~63;
  return s->rows > 0;
}

static size_t ssim_plane_bytes(const SsimPlane& s) {
  return ((size_t)s.rows * (size_t)s.ld * (s.compact ? 6 : sizeof(float2)) + 255) & ~(size_t)255;
}

// 16 x 16 blocks on the matrix cores: (mean, stddev, byte sum) of each
// full-width current block of the launch's rows
static size_t ssim_cur_stats_bytes(const SearchArgs& p) {
  if (p.blk != 16 || p.range > 64 || p.width < 16) return 0;
  return (size_t)(p.block_row_end - p.block_row_begin) * (size_t)(p.width / 16) * sizeof(float4);
}

size_t ssim_scratch(const SearchArgs& p) {
  if (p.cost_kind != COST_SSIM) return 0;
  SsimPlane s, h;
  int hbh;
  size_t n = ssim_plane(p, &s) ? ssim_plane_bytes(s) : 0;
  if (ssim_hb_plane(p, &h, &hbh)) n += ssim_plane_bytes(h);
  return n ? n + ssim_cur_stats_bytes(p) : 0;
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

// One launch for every statistic the search reads: grid rows [0, gy[0]) the
// current blocks' (mean, stddev, byte sum) for the matrix-core kernel, then
// gy[2] rows of tiles of plane 2 (the partial bottom row's, patch height
// ph[2] < 16), then gy[1] of plane 1 (the full rows').
struct SsimStatsJob {
  SsimPlane pl[3];
  float2* out[3];
  int ph[3], gy[3];
  float4* cst;      // current blocks: (by - block_row_begin) nbxf + bx
  int cst_n, nbxf;  // entries, full-width columns
  int cur_a4;       // current rows 4-byte aligned
};

// The current block at (bx, by) from global memory: ssim.c:3-28 in the float
// path's order (patch_stats), and the integer byte sum.
__device__ __forceinline__ float4 cur_block_stats(const SearchArgs& p, int bx, int by, int a4) {
  const int bh = min(16, p.height - 16 * by);
  const uint8_t* src = p.cur + (ptrdiff_t)(16 * by - p.cur_row0) * p.stride + 16 * bx;
  uint32_t w[16][4];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint8_t* row = src + (ptrdiff_t)min(i, bh - 1) * p.stride;
    if (a4) {
#pragma unroll
      for (int q = 0; q < 4; q++) w[i][q] = reinterpret_cast<const uint32_t*>(row)[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++)
        w[i][q] = (uint32_t)row[4 * q] | (uint32_t)row[4 * q + 1] << 8 |
                  (uint32_t)row[4 * q + 2] << 16 | (uint32_t)row[4 * q + 3] << 24;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++)
    if (i < bh)
#pragma unroll
      for (int q = 0; q < 4; q++) s = __builtin_amdgcn_sad_u8(w[i][q], 0u, s);
  const float nf = (float)(16 * bh);
  const float m = __fdiv_rn((float)s, nf);
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i++)
    if (i < bh)
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const float d = __fsub_rn((float)((w[i][q] >> (8 * b)) & 255u), m);
          acc = __fadd_rn(acc, __fmul_rn(d, d));
        }
  return make_float4(m, sqrt_via_double(__fdiv_rn(acc, nf)), __int_as_float((int)s), 0.f);
}

__global__ __launch_bounds__(256) void me_ssim_stats_kernel(SearchArgs p, SsimStatsJob J) {
  __shared__ uint32_t t[STATS_TR * STATS_TW];
  const int B = p.blk;
  const int tid = (int)threadIdx.x;
  // grid rows: the current blocks' statistics, then the partial row's plane
  // (its workgroups run the longest scalar chains: first, not as a tail),
  // then the full rows' plane
  int yb = (int)blockIdx.y, k;
  if (yb < J.gy[0]) {
    k = 0;
  } else if ((yb -= J.gy[0]) < J.gy[2]) {
    k = 2;
  } else {
    yb -= J.gy[2];
    k = 1;
  }
  if (k == 0) {
    const int e = (yb * (int)gridDim.x + (int)blockIdx.x) * 256 + tid;
    if (e < J.cst_n)
      J.cst[e] = cur_block_stats(p, e % J.nbxf, p.block_row_begin + e / J.nbxf, J.cur_a4);
    return;
  }
  const SsimPlane s = J.pl[k];
  float2* const plane = J.out[k];
  const int ph = J.ph[k];
  const int x0 = (int)blockIdx.x * 64, y0 = yb * 16;
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
  const float nfp = (float)(B * ph);
  auto put = [&](int rr, int x, float m, float v) {
    const size_t e = (size_t)rr * s.ld + x;
    if (s.compact) {
      float* sd = reinterpret_cast<float*>(plane);
      sd[e] = sqrt_via_double(v);
      // m = fl(S1r / N): N m is within N ulp / 2 < 1/2 of the integer S1r
      reinterpret_cast<uint16_t*>(sd + (size_t)s.rows * s.ld)[e] = (uint16_t)__float2int_rn(__fmul_rn(m, nfp));
    } else {
      plane[e] = make_float2(m, sqrt_via_double(v));
    }
  };
  if (B == 16 && ph == 16) {
    // 16 x 16 patches (the full rows' plane): the staged bytes once more as
    // float pairs (column j, column j + 32) of each row, and 16-row column
    // sums.  Thread (cc, rg) then runs the positions (cc, cc + 32) of rows
    // 2 rg and 2 rg + 1: per pixel one aligned 8-byte LDS read feeds one
    // packed chain step of two positions (v_pk_add / v_pk_mul, each half
    // rounded as the scalar op, in patch_stats' raster order), and the two
    // rows' chains interleave.  (Bytes converted per read with two positions
    // per chain, round 6's first form: 57.4 against 52.2 us at 1080p,
    // profiles/r06zv_*.)
    typedef float f2v_ __attribute__((ext_vector_type(2)));
    __shared__ f2v_ pf[31 * 47];
    __shared__ int cs[16 * 79];
    constexpr int TB = STATS_TW * 4;  // staged bytes per row
    for (int i = tid; i < 31 * 47; i += 256) {
      const int r = i / 47, j = i - r * 47;
      pf[i] = f2v_{(float)tb[r * TB + j], (float)tb[r * TB + j + 32]};
    }
    for (int i = tid; i < 16 * 79; i += 256) {
      const int r = i / 79, col = i - r * 79;
      int sum = 0;
#pragma unroll
      for (int q = 0; q < 16; q++) sum += tb[(r + q) * TB + col];
      cs[i] = sum;
    }
    __syncthreads();
    const int cc = tid & 31, rg = tid >> 5, r0 = 2 * rg;
    f2v_ mf[2];
#pragma unroll
    for (int rw = 0; rw < 2; rw++) {
      int sa = 0, sb = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        sa += cs[(r0 + rw) * 79 + cc + k];
        sb += cs[(r0 + rw) * 79 + cc + 32 + k];
      }
      // byte sums / 256: exact, as __fdiv_rn(s, 256.f)
      mf[rw] = f2v_{__fmul_rn((float)sa, 1.0f / 256.0f), __fmul_rn((float)sb, 1.0f / 256.0f)};
    }
    f2v_ acc[2] = {f2v_{0.f, 0.f}, f2v_{0.f, 0.f}};
#pragma unroll 1
    for (int i = 0; i < 16; i++) {
      const f2v_* ra = pf + (r0 + i) * 47 + cc;
      const f2v_* rb = ra + 47;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const f2v_ da = ra[k] - mf[0], db = rb[k] - mf[1];
        acc[0] = acc[0] + da * da;
        acc[1] = acc[1] + db * db;
      }
    }
#pragma unroll
    for (int rw = 0; rw < 2; rw++) {
      const int rr = y0 + r0 + rw;
      if (rr >= s.rows) continue;
#pragma unroll
      for (int hh = 0; hh < 2; hh++) {
        const int x = x0 + cc + 32 * hh;
        if (x < s.pitch) put(rr, x, mf[rw][hh], __fmul_rn(acc[rw][hh], 1.0f / 256.0f));
      }
    }
    return;
  }
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
    put(rr, x, m, v);
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
      const float2* st = stats + (size_t)(wy0 + cy - pg.ylo) * pg.ld;
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
      const float2* st = stats + (size_t)(wy0 + cy - pg.ylo) * pg.ld;
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
#ifndef ME_SSIM_ABL
#define ME_SSIM_ABL 0  // A/B ablations (tools/dbg/ssim_variants.sh); 0 in the product
#endif
constexpr int SSIM_CREC = 48;                                // row record: 0^16, c ^ 0x7F, 0^16

__host__ __device__ inline int ssim_mfma_lp(int S) { return 16 * ((2 * S + 15) / 16 + 3); }
__host__ __device__ inline int ssim_mfma_rows(int S) { return 16 * ((2 * S + 1 + 15) / 16) + 15; }
__host__ __device__ inline int ssim_mfma_lds(int S) {
  return 16 * SSIM_CREC + ssim_mfma_rows(S) * ssim_mfma_lp(S);
}

// bh: the blocks' height -- 16, or the partial bottom row's H % 16 (its own
// statistics plane; N = 16 bh pixels <= 256, so the identity above holds with
// 256 -> N and 4161536 -> 16256 N; record rows >= bh are zero)
// Grid: the full rows' full-width blocks (plane 1), then the partial bottom
// row's (plane 2, bh = H % 16), J's current-block statistics for each.
__global__ __launch_bounds__(256) void me_ssim_mfma_kernel(SearchArgs p, SsimStatsJob J,
                                                           int aligned16) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[4];
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const uint32_t lds_c32;
  typedef __attribute__((address_space(3))) const v4i lds_cv4i;
  auto lds_addr = [](const void* q) {
    return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)q);
  };
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, hh = lane >> 4;
  const int nbxf = J.nbxf;
  // XCD-aware order: workgroup i runs on XCD i % 8, and XCD x takes a
  // contiguous run of raster-order blocks, so the blocks sharing plane and
  // window lines share that XCD's L2 (round robin sent horizontal neighbours
  // to different XCDs: ~276 MB of plane reads from the Infinity cache at 1080p)
  const int G = (int)gridDim.x, wg = (int)blockIdx.x;
  const int xq = G >> 3, xr = G & 7, xcd = wg & 7, xk = wg >> 3;
  const int blk = xcd < xr ? xcd * (xq + 1) + xk : xr * (xq + 1) + (xcd - xr) * xq + xk;
  const int bx = blk % nbxf;
  const int by = p.block_row_begin + blk / nbxf;
  const int S = p.range, W = p.width, H = p.height;
  const int bh = min(16, H - 16 * by);
  const int k = bh < 16 ? 2 : 1;
  const float2* const stats = J.out[k];
  const SsimPlane pg = J.pl[k];
  // the block's mean, stddev and byte sum (me_ssim_stats_kernel)
  const float4 cs = J.cst[blk];
  const int tlx = 16 * bx, tly = 16 * by;
  const int wx0 = max(tlx - S, 0), wy0 = max(tly - S, 0);
  const int ncx = min(tlx + S, W - 16) - wx0 + 1, ncy = min(tly + S, H - bh) - wy0 + 1;
  const int i0 = wx0 >> 4, ni = ((wx0 + ncx - 1) >> 4) - i0 + 1, nj = (ncy + 15) >> 4;
  const int LP = ssim_mfma_lp(S), R = 16 * nj + 15;
  uint8_t* crec = smem;                        // 16 row records
  uint8_t* win = crec + 16 * SSIM_CREC;        // rows wy0 .., columns 16 i0 ..: r ^ 0x80
  for (int i = tid; i < 256; i += 256) {
    const int oy = i >> 4, ox = i & 15;
    const uint8_t c = oy < bh ? p.cur[(ptrdiff_t)(tly + oy - p.cur_row0) * p.stride + tlx + ox] : 0;
    crec[oy * SSIM_CREC + 16 + ox] = oy < bh ? c ^ 0x7F : 0;
    crec[oy * SSIM_CREC + ox] = 0;
    crec[oy * SSIM_CREC + 32 + ox] = 0;
  }
  // (columns and rows past the frame: zeros or the next bytes of the plane;
  // only masked candidates read them)
  if (ME_SSIM_ABL & 4) {
  } else if (aligned16) {
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
  const int N = 16 * bh;
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
  const float mp = cs.x, sp = cs.y;
  const float mp2 = __fmul_rn(mp, mp), sp2 = __fmul_rn(sp, sp);
  // S1c: the block's byte sum; imc = (int) mp = S1c / N (the rounded quotient
  // stays below the next integer: 1 - frac >= 1 / N is far above its ulp)
  const int S1c = __float_as_int(cs.z), imc = (int)mp;
  // S1r < 2^16, imr < 256: with ka = 127 - imc and kb = S1c - N imc (in [0, N))
  // every factor fits v_mul_i32_i24
  const int ka = 127 - imc, kb = S1c - N * imc;
  const int kc = 128 * S1c - 16256 * N;
  const float nf = (float)N, inv_nf = 1.0f / nf;  // exact when N is a power of two
  const bool pow2 = (N & (N - 1)) == 0;
  uint64_t best = ~0ull;
  const uint32_t xb0 = lds_addr(win) + (uint32_t)((n + (hh >> 1)) * LP + 16 * (hh & 1));
  const int nt = ni * nj;
  // the compact plane's entries of tile t's lane candidates: stddevs as one
  // 16-byte load, byte sums as one 8-byte load (absolute columns 16 (i0 + ti)
  // + 4 hh .. + 3, inside the padded row; masked candidates read row-clamped
  // or padding entries, never used), loaded one tile ahead of their use
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
  const float* sdp = reinterpret_cast<const float*>(stats);
  const unsigned short* s1p = reinterpret_cast<const unsigned short*>(sdp + (size_t)pg.rows * pg.ld);
  auto load_st = [&](int t, f4v* sd, u16x4* s1) {
    const int tj = t / ni, ti = t - tj * ni;
    const size_t e = (size_t)(wy0 + min(16 * tj + n, ncy - 1) - pg.ylo) * pg.ld + 16 * (i0 + ti) + 4 * hh;
    *sd = *reinterpret_cast<const f4v*>(sdp + e);
    *s1 = *reinterpret_cast<const u16x4*>(s1p + e);
  };
  f4v nsd = {0.f, 0.f, 0.f, 0.f};
  u16x4 ns1 = {0, 0, 0, 0};
  if (!(ME_SSIM_ABL & 2) && wave < nt) load_st(wave, &nsd, &ns1);
#pragma unroll 1
  for (int t = wave; t < nt; t += 4) {
    const int tj = t / ni, ti = t - tj * ni;
    const f4v csd = nsd;
    const u16x4 cs1 = ns1;
    if (!(ME_SSIM_ABL & 2) && t + 4 < nt) load_st(t + 4, &nsd, &ns1);
    // B fragment q: window row 16 tj + n + 2 q + (hh >> 1), column 16 ti + 16 (hh & 1)
    const uint32_t xb = xb0 + (uint32_t)(16 * tj * LP + 16 * ti);
    v4i f[8];
#pragma unroll
    for (int q = 0; q < 8; q++) f[q] = *reinterpret_cast<lds_cv4i*>((uintptr_t)(xb + (uint32_t)(2 * q * LP)));
    v4i acc = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 8; q++) acc = (ME_SSIM_ABL & 8) ? acc + f[q] : MFMA16(A[q], f[q], acc, 0, 0, 0);
    // lane (n, hh): X of positions x = 16 (i0 + ti) + 4 hh + r, y = wy0 + 16 tj + n
    const int cy = 16 * tj + n, cx0 = 16 * (i0 + ti) + 4 * hh - wx0;
    if (ME_SSIM_ABL & 3) {
      uint64_t k = 0;
#pragma unroll
      for (int r = 0; r < 4; r++) k += (uint32_t)acc[r] ^ __float_as_uint(csd[r]) ^ cs1[r];
      best = k < best ? k : best;
    } else {
      // ssim.c:53-56 for the lane's four candidates, two per packed
      // instruction (each half rounded as ssim_key's scalar operation)
      const float C1 = 0.01f, C2 = 0.09f, C3 = 0.045f;  // ssim.c:48
#pragma unroll
      for (int h2 = 0; h2 < 2; h2++) {
        f2v m, cvf;
        const f2v sr = {csd[2 * h2], csd[2 * h2 + 1]};
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int S1r = cs1[2 * h2 + e];
          // the reference's mean: fl(S1r / N) (exact for N = 256); imr = (int) mean
          m[e] = pow2 ? __fmul_rn((float)S1r, inv_nf) : __fdiv_rn((float)S1r, nf);
          const int imr = (int)m[e];
          // = 127 S1r + kc - X - imc S1r - imr S1c + N imr imc, 24-bit products
          cvf[e] = (float)(__mul24(S1r, ka) + kc - acc[2 * h2 + e] - __mul24(imr, kb));
        }
        const f2v cvk = pow2 ? cvf * inv_nf : f2v{__fdiv_rn(cvf.x, nf), __fdiv_rn(cvf.y, nf)};
        const f2v lum = div_rn2((2.f * m) * mp + C1, (m * m + mp2) + C1);
        const f2v con = div_rn2((2.f * sr) * sp + C2, (sr * sr + sp2) + C2);
        const f2v str = div_rn2(cvk + C3, sr * sp + C3);
        const f2v score = (lum * con) * str;
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int cx = cx0 + 2 * h2 + e;
          const bool ok = cy < ncy && cx >= 0 && cx < ncx && score[e] > 0.f;
          const uint64_t key = ((uint64_t)(0x7FFFFFFFu - __float_as_uint(score[e])) << 32) |
                               ((uint32_t)(wy0 + cy - tly + 32768) << 16) |
                               (uint32_t)(wx0 + cx - tlx + 32768);
          best = ok && key < best ? key : best;
        }
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
  // its own.  The full rows' plane, the partial bottom row's, then the current
  // blocks' statistics for the matrix-core kernel -- all from one launch.
  SsimStatsJob J{};
  SsimPlane& sp = J.pl[1];
  int hbh = 0;
  const float2* stats = nullptr;
  bool hb = false;
  const size_t need = ssim_scratch(p);
  if (need && p.scratch && p.scratch_bytes >= need) {
    uint8_t* base = reinterpret_cast<uint8_t*>(p.scratch);
    if (ssim_plane(p, &sp)) {
      J.out[1] = reinterpret_cast<float2*>(base);
      J.ph[1] = B;
      J.gy[1] = (sp.rows + 15) / 16;
      stats = J.out[1];
      base += ssim_plane_bytes(sp);
    }
    if (ssim_hb_plane(p, &J.pl[2], &hbh)) {
      J.out[2] = reinterpret_cast<float2*>(base);
      J.ph[2] = hbh;
      J.gy[2] = (J.pl[2].rows + 15) / 16;
      base += ssim_plane_bytes(J.pl[2]);
      hb = true;
    }
    // 16 x 16 blocks, S <= 64: full-width columns on the matrix cores
    J.nbxf = ssim_cur_stats_bytes(p) ? p.width / 16 : 0;
    if (J.nbxf > 0) {
      J.cst = reinterpret_cast<float4*>(base);
      J.cst_n = rows * J.nbxf;
      J.cur_a4 = p.stride % 4 == 0 && (uintptr_t)p.cur % 4 == 0;
    }
    const int gx = std::max((std::max(sp.pitch, J.pl[2].pitch) + 63) / 64, 1);
    J.gy[0] = J.nbxf > 0 ? (J.cst_n + 256 * gx - 1) / (256 * gx) : 0;
    hipLaunchKernelGGL(me_ssim_stats_kernel, dim3((unsigned)gx, (unsigned)(J.gy[0] + J.gy[1] + J.gy[2])),
                       dim3(256), 0, stream, p, J);
  }
  // The matrix cores: the full rows (plane 1) and the partial bottom row (plane 2)
  // of the full-width columns; the partial right column on the float path
  int r_full = 0;
  const bool hb_mfma = hb && J.nbxf > 0;
  if (J.nbxf > 0 && (stats || hb)) {
    r_full = stats ? std::max(0, std::min(p.block_row_end, p.height / 16) - p.block_row_begin) : 0;
    const int a16 = p.stride % 16 == 0 && (uintptr_t)p.ref % 16 == 0 && p.ref_bytes > 0;
    const int nrow = r_full + (hb_mfma ? 1 : 0);
    hipLaunchKernelGGL(me_ssim_mfma_kernel, dim3((unsigned)(nrow * J.nbxf)), dim3(256),
                       ssim_mfma_lds(p.range), stream, p, J, a16);
  }
  const int nbxf = hb_mfma || r_full > 0 ? J.nbxf : 0;
  // the float kernel reads only a float2 plane (a compact one serves the matrix cores)
  const float2* fstats = sp.compact ? nullptr : stats;
  // + SSIM_PAD bytes: the last candidate group of the last row reads past the window
  const int lds = cur + (int)win + SSIM_PAD;
  if (r_full == 0 && !hb_mfma) {
    hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(rows * p.nbx)), dim3(SSIM_THREADS), lds, stream,
                       p, p.block_row_begin, 0, (int)win, fstats, sp);
  } else {
    // the rest: the partial right column of the full rows, then the partial
    // bottom row (its right-column block only when the row ran on the matrix cores)
    if (r_full > 0 && nbxf < p.nbx)
      hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)(r_full * (p.nbx - nbxf))), dim3(SSIM_THREADS),
                         lds, stream, p, p.block_row_begin, nbxf, (int)win, fstats, sp);
    const int rb = p.block_row_begin + r_full;
    if (rb < p.block_row_end) {
      const int col0 = hb_mfma ? nbxf : 0;
      if (col0 < p.nbx)
        hipLaunchKernelGGL(me_ssim_kernel, dim3((unsigned)((p.block_row_end - rb) * (p.nbx - col0))),
                           dim3(SSIM_THREADS), lds, stream, p, rb, col0, (int)win, fstats, sp);
    }
  }
  return hipGetLastError();
}

}  // namespace me
