// me_band.hip -- 16x16 SSD (the reference's MSE cost, souravBhat/MotionEstimation
// src/cpu/main.c:18-36, argmin with raster-first ties main.c:53-60, window
// clamp main.c:73-76) on the matrix cores, walking bands.
//
// The decomposition is me_mfma.hip's (SSD = Cc_m + S2(x, y) + 2 X_m(x, y), X_m
// an i8 GEMM on v_mfma_i32_16x16x64_i8 with the block-major operand layout of
// me_mfma_bm16_kernel: one block per 16x16 output tile of 16 x positions by 16
// y positions).  What differs is where S2 = sum over the 16x16 window of
// (r - 127)^2 comes from.  The block-major kernel reads it from a prepass plane
// (7.5x the algorithmic HBM bytes at 1080p); me_mfma_bmv_kernel forms it per
// workgroup and band, once for every block row whose range covers the band
// (~5x at S = 32).  Here a workgroup owns a strip of C block columns and walks
// DOWN a segment of block rows band by band: a band is the 16 candidate rows
// [16 b, 16 b + 16), its S2 is formed once, and every block row in flight (the
// rows whose search range meets the band: 2 ceil(S/16) + 1 of them) runs its
// MFMA tiles on it with the same B fragments.  A block row enters at its first
// band and leaves after its last, so the A fragments of the rows in flight
// stay in registers (a ring of NS slots per searcher wave).
//
//   waves      8 (512 threads, one workgroup per CU), two roles, one of each
//              per SIMD (waves w and w + 4 share SIMD w):
//   searchers  waves 0..3: block column w % C of the strip, row class w / C
//              (4 / C classes split a column's rows in flight).  Per band and
//              tile: 8 B fragments (ds_read_b128, two fragments ahead) and one
//              P0 vector; 8 MFMAs per row in flight, the rows interleaved
//              (independent accumulation chains); keys as the block-major
//              kernel's.  Nothing else but the rows' entries and exits.
//   producers  waves 4..7: the window slabs (LDS DMA), the XOR-ed copy, and
//              S2: band m is produced by producer (m - first band) % 4 during
//              the 4 iterations before it is searched (46 steps of a sliding
//              16-row sum, 12 per iteration), lane = 4 positions (one v_dot4
//              per window row of 4 bytes), the 16-wide horizontal sum by DPP
//              within 16-lane rows, the result stored as the key's position
//              term P0 = (S2 << 6) + 2^29 + 64 + (x & 3).  Their VALU work
//              runs beside the searchers' MFMAs on the same SIMDs.
//   LDS        the window in 16-row slabs: a raw ring (6 slabs ahead) read by
//              the producers, and the slabs XOR-ed with 0x80 (the MFMA B
//              operand r - 128) in a ring of 3 + a mirror of slot 0, so a
//              band's 31 rows are contiguous; 5 P0 planes (the band searched +
//              the 4 in production)
//
// HBM: the reference rows of the strip window, once per workgroup (adjacent
// strips share them through the XCD's L2: consecutive workgroups are adjacent
// strips, dealt to one XCD), the cur rows once, 8 bytes per block out.  No
// context scratch.  Rows are walked full height, so no band is formed twice
// within a workgroup; a frame is split into segments of block rows only when
// the frames' strips alone do not fill the CUs (each segment re-forms the
// 2 ceil(S/16) bands above and below it).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "me_kernels.h"
#include "me_mfma_util.h"
#include "me_tuning.h"

namespace me {

namespace {

using mfma::v4i;
using mfma::lshl6_add;
using mfma::mfma_job;
using mfma::opaque;
using mfma::umin3;

constexpr int BW_NW = 8;             // waves per workgroup: 4 searchers, 4 producers
constexpr int BW_T = 64 * BW_NW;     // threads
constexpr int BW_RAWN = 6;           // raw slab ring (slabs b + 1 .. b + 6 at band b)
constexpr int BW_P0N = 5;            // P0 planes: the band searched + 4 in production
constexpr int BW_XN = 4;             // XOR-ed slabs: ring of 3 + the mirror of slot 0
constexpr int BW_OPS = 46;           // producer steps per band: 16 rows in, then 15 x (out, in)
constexpr int BW_OPS_IT = 12;        // producer steps per iteration (4 iterations per band)
constexpr int BW_CREC = 48;          // cur row record: 16 zero bytes, the row (c ^ 0x7F), 16 zero bytes

#ifdef ME_STAMPS
// Diagnostic build only (libme_hip_stamps.so): per workgroup and wave, the
// s_memtime cycles spent in each phase of the band loop, summed over the
// iterations: [prologue, entries / slab DMA + XOR, fetch, tiles, band end,
// production, barrier wait, iterations] (tools/bw_stamps.py).
__device__ unsigned long long g_bwstamps[8 * 8 * 4096];
#define BW_T0() unsigned long long bw_t = __builtin_amdgcn_s_memtime()
#define BW_ACC(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); bw_acc[k] += t_ - bw_t; bw_t = t_; } while (0)
#else
#define BW_T0() do { } while (0)
#define BW_ACC(k) do { } while (0)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t lds_c32;
typedef __attribute__((address_space(3))) const v4i lds_cv4i;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)p);
}
__device__ __forceinline__ uint32_t ld32(uint32_t a) {
  return *reinterpret_cast<lds_c32*>((uintptr_t)a);
}
__device__ __forceinline__ v4i ldv4(uint32_t a) {
  return *reinterpret_cast<lds_cv4i*>((uintptr_t)a);
}
// (a << 7) + b in one instruction
__device__ __forceinline__ uint32_t lshl7_add(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_lshl_add_u32 %0, %1, 7, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

// LDS layout (bytes): XN slabs | RAWN slabs | P0N planes | crec (searchers) | keys
__host__ __device__ constexpr int bw_slab(int lp) { return 16 * lp; }
__host__ __device__ inline int bw_lds_bytes(int lp, int pp, int ns) {
  return (BW_XN + BW_RAWN) * bw_slab(lp) + BW_P0N * 16 * pp * 4 + 4 * 16 * BW_CREC + 4 * ns * 8;
}

template <int C, int NS, int LP>
__global__ __launch_bounds__(BW_T) void me_mfma_bw_kernel(SearchArgs p, MfmaGeom g, MfmaJobs jb) {
  constexpr int WPC = 4 / C;  // row classes per column
  constexpr int SLAB = bw_slab(LP);
  extern __shared__ __align__(16) uint8_t smem[];
  const int PP = g.bw_pp;
  const int P0PLANE = 16 * PP;  // ints
  uint8_t* xw = smem;
  uint8_t* raw = xw + BW_XN * SLAB;
  int* p0 = reinterpret_cast<int*>(raw + BW_RAWN * SLAB);
  uint8_t* crec_all = reinterpret_cast<uint8_t*>(p0 + BW_P0N * P0PLANE);
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(crec_all + 4 * 16 * BW_CREC);

  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool searcher = wave < 4;
  const int col = wave % C, cls = (wave & 3) / C;  // searchers
  const int pw = wave & 3, ptid = tid & 255;       // producers: index, thread within the role
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  int lin = mfma::xcd_banded_index();
  {  // batched launch: jobs are consecutive runs of jb.wgs workgroups
    const int j = lin / jb.wgs;
    lin -= j * jb.wgs;
    mfma_job(jb, j, p, g);
  }
  const int seg = lin / g.bw_strips, strip = lin - seg * g.bw_strips;
  const int r0 = g.row0 + seg * g.bw_seg_rows;
  const int r1 = min(r0 + g.bw_seg_rows, g.row0 + g.nrows);
  const int bc0 = strip * C, ncol = min(C, g.nbx - bc0);
  const int tc0 = max(16 * bc0 - S, 0) >> 4;  // first tile column of the strip window
  const int tcl = min(16 * (bc0 + ncol - 1) + S, W - 16) >> 4;
  const int npos = 16 * (tcl - tc0 + 1);  // positions of the window's tiles
  const int Sc = (S + 15) >> 4;
  auto lo = [&](int br) { return max(16 * br - S, 0) >> 4; };      // first band of row br
  auto hi = [&](int br) { return min(16 * br + S, H - 16) >> 4; };  // last band of row br
  auto E = [&](int b) { return b <= 0 ? 0 : b + Sc; };              // first row with lo >= b
  const int bfirst = lo(r0), blast = hi(r1 - 1);
  const int bend = blast + 1;  // slabs bfirst .. bend are read (band blast's window reaches slab bend)

  // ================================ producers
  // the window: raw slabs by LDS DMA (frame rows [16 s, 16 s + 16) x columns
  // [16 tc0, 16 tc0 + LP)).  Rows outside the resident ones are outside the
  // buffer range and read as 0 (their positions are masked).
  const __amdgpu_buffer_rsrc_t rref =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ref, (short)0, p.ref_bytes, 0x00020000);
  auto dma_slab = [&](int s) {
    uint8_t* dst = raw + (s % BW_RAWN) * SLAB;
    const int rowb = 16 * s - p.ref_row0;
    for (int s0 = pw * 1024; s0 < SLAB; s0 += 4 * 1024) {
      const int d = s0 + 16 * lane;
      if (d < SLAB) {
        const int rho = d / LP, k = d - rho * LP;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rref, (__attribute__((address_space(3))) void*)(dst + s0), 16,
            (uint32_t)((rowb + rho) * p.stride + 16 * tc0 + k), 0, 0, 0);
      }
    }
  };
  // slab s XOR-ed (r ^ 0x80 = r - 128 as i8, the B operand) into ring slot s % 3
  // and, for slot 0, its mirror after slot 2: band b's rows 16 b .. 16 b + 30
  // are then contiguous from slot b % 3
  auto xor_slab = [&](int s) {
    const u32x4* src = reinterpret_cast<const u32x4*>(raw + (s % BW_RAWN) * SLAB);
    const int slot = s % 3;
    u32x4* dst = reinterpret_cast<u32x4*>(xw + slot * SLAB);
    u32x4* mir = reinterpret_cast<u32x4*>(xw + 3 * SLAB);
    for (int t = ptid; t < SLAB / 16; t += 256) {
      const u32x4 v = src[t] ^ 0x80808080u;
      dst[t] = v;
      if (slot == 0) mir[t] = v;
    }
  };
  // V(row) = sum of 16 window rows of H, H(row, x) = sum over the 4 bytes at
  // x of (r - 127)^2 (u = r ^ 0x7F = 127 - r as an i8: one v_dot4 per 4
  // bytes).  Lane (row R, l) owns the 4 positions of group pg = 13 R + l: the
  // 16-lane rows overlap by 3 groups, so a group's three right neighbours are
  // in its own row (l < 13 outputs).
  const int pg = 13 * (lane >> 4) + (lane & 15);
  const bool pout = (lane & 15) < 13 && 4 * pg < npos;
  v4i V = {0, 0, 0, 0};
  auto h_acc = [&](uint32_t w0, uint32_t w1, v4i acc) {  // acc + H of the bytes (w0, w1)
    const uint32_t u0 = w0 ^ 0x7F7F7F7Fu, u1 = w1 ^ 0x7F7F7F7Fu;
    const uint32_t u[4] = {u0, __builtin_amdgcn_alignbyte(u1, u0, 1),
                           __builtin_amdgcn_alignbyte(u1, u0, 2),
                           __builtin_amdgcn_alignbyte(u1, u0, 3)};
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = __builtin_amdgcn_sdot4((int)u[r], (int)u[r], acc[r], false);
    return acc;
  };
  // row j of band m: S2(x) = V(x) + V(x + 4) + V(x + 8) + V(x + 12), the
  // neighbours by DPP row_shl 1 then 2; stored as the key's position term
  auto out_row = [&](int m, int j) {
    v4i T, Q;
#pragma unroll
    for (int r = 0; r < 4; r++) T[r] = V[r] + __builtin_amdgcn_update_dpp(0, V[r], 0x101, 0xF, 0xF, false);
#pragma unroll
    for (int r = 0; r < 4; r++) Q[r] = T[r] + __builtin_amdgcn_update_dpp(0, T[r], 0x102, 0xF, 0xF, false);
    if (pout) {
      v4i o;
#pragma unroll
      for (int r = 0; r < 4; r++) o[r] = (int)lshl6_add((uint32_t)Q[r], (1u << 29) + 64u + (uint32_t)r);
      *reinterpret_cast<v4i*>(p0 + (m % BW_P0N) * P0PLANE + j * PP + 4 * pg) = o;
    }
  };
  // steps [o0, o1) of band m (at most BW_OPS_IT): 0..15 add rows 0..15 (row
  // 0 out after 15), then for j = 1..15: remove row j - 1, add row j + 15,
  // row j out.  The window rows of all the steps are read first: one LDS
  // latency per call.
  auto produce = [&](int m, int o0, int o1) {
    uint32_t w0[BW_OPS_IT], w1[BW_OPS_IT];
#pragma unroll
    for (int k = 0; k < BW_OPS_IT; k++) {
      const int o = min(o0 + k, o1 - 1), q = o - 16;
      const int rho = o < 16 ? o : (q & 1) ? (q >> 1) + 16 : (q >> 1);
      const uint32_t a = lds_addr(raw + ((m + (rho >> 4)) % BW_RAWN) * SLAB + (rho & 15) * LP) +
                         4u * (uint32_t)pg;
      w0[k] = ld32(a);
      w1[k] = ld32(a + 4);
    }
#pragma unroll
    for (int k = 0; k < BW_OPS_IT; k++) {
      const int o = o0 + k;
      if (o >= o1) break;
      if (o < 16) {
        const v4i z = {0, 0, 0, 0};
        V = h_acc(w0[k], w1[k], o == 0 ? z : V);
        if (o == 15) out_row(m, 0);
      } else {
        const int q = o - 16, j = (q >> 1) + 1;
        if ((q & 1) == 0) {
          const v4i z = {0, 0, 0, 0};
          V -= h_acc(w0[k], w1[k], z);
        } else {
          V = h_acc(w0[k], w1[k], V);
          out_row(m, j);
        }
      }
    }
  };

  // ================================ searchers
  // block rows in flight: a ring of NS slots (this searcher's class)
  int srow[NS];  // row of the slot, -1: free (wave-uniform)
  v4i A[NS][8];
  int cc[NS];
  uint32_t bk[NS], bcur[NS];
  int bb[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) {
    srow[s] = -1;
    cc[s] = 0;
    bk[s] = bcur[s] = ~0u;
    bb[s] = 0;
  }
  const bool hascol = searcher && col < ncol;
  const int bx = 16 * (bc0 + col);
  const int xlo = max(bx - S, 0), xhi = min(bx + S, W - 16);
  const int i0c = xlo >> 4, i1c = xhi >> 4;
  uint8_t* crec = crec_all + (wave & 3) * 16 * BW_CREC;
  const uint8_t* cur_lane = p.cur + (ptrdiff_t)(lane - p.cur_row0) * p.stride + 16 * (bc0 + col);

  // The first row entering at band b (this column and class) is prefetched
  // into pf0 one iteration ahead; further ones (frame top, segment starts)
  // are loaded when they enter.
  u32x4 pf0 = {0u, 0u, 0u, 0u};
  int pe0 = 0, pe1 = 0;  // this class's entering rows: pe0, pe0 + WPC, ... < pe1
  auto fetch = [&](int b) {
    const int e0 = max(E(b), r0), e1 = min(E(b + 1), r1);
    pe0 = e0 + ((cls - (e0 - r0)) % WPC + WPC) % WPC;
    pe1 = e1;
    if (hascol && lane < 16 && pe0 < pe1)
      pf0 = *reinterpret_cast<const u32x4*>(cur_lane + (ptrdiff_t)(16 * pe0) * p.stride);
  };
  // A fragments of an entering row: bytes o .. o + 15 of record row
  // 2 q + (h >> 1), o = 16 + 16 (h & 1) - m (me_mfma_bm16_kernel's layout);
  // Cc = sum (c''^2 + 2 c'') over the block
  auto enter = [&](int br, u32x4 v) {
    const int slot = ((br - r0) / WPC) % NS;
    const u32x4 x = v ^ 0x7F7F7F7Fu;
    int part = 0;
    if (lane < 16) {
      const u32x4 z = {0u, 0u, 0u, 0u};
      u32x4* rec = reinterpret_cast<u32x4*>(crec + lane * BW_CREC);
      rec[0] = z;
      rec[1] = x;
      rec[2] = z;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        part = __builtin_amdgcn_sdot4((int)x[e], (int)x[e], part, false);
        part = __builtin_amdgcn_sdot4((int)x[e], 0x02020202, part, false);
      }
    }
    // Cc: the sum over lanes 0..15 (DPP row_shr 1, 2, 4, 8 with zeros shifted
    // in: lane 15 holds it; no LDS atomic, which would wait for the slab DMA)
    part += __builtin_amdgcn_update_dpp(0, part, 0x111, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x112, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x114, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x118, 0xF, 0xF, false);
    const int ccv = __builtin_amdgcn_readlane(part, 15);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int o = 16 + 16 * (h & 1) - n, sh = o & 3;
    const uint32_t lb = lds_addr(crec) + (uint32_t)((h >> 1) * BW_CREC + (o & ~3));
    uint32_t d[8][5];  // every record read first: one LDS latency
#pragma unroll
    for (int q = 0; q < 8; q++)
#pragma unroll
      for (int e = 0; e < 5; e++) d[q][e] = ld32(lb + (uint32_t)(2 * q * BW_CREC + 4 * e));
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (s != slot) continue;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        v4i f;
#pragma unroll
        for (int e = 0; e < 4; e++) f[e] = (int)__builtin_amdgcn_alignbyte(d[q][e + 1], d[q][e], sh);
        A[s][q] = f;
      }
      srow[s] = br;
      cc[s] = ccv;
      bk[s] = bcur[s] = ~0u;
      bb[s] = 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // record reads done before the next entry
  };
  // a row's last band is done: its best over the lanes (cost, dy, dx) -> record
  auto emit = [&](int s) {
    const int br = srow[s];
    const uint32_t kb = bk[s], hk = kb >> 6;
    unsigned long long* kp = keys + (wave & 3) * NS + s;
    if (hk < (1u << 25)) {
      const uint32_t cost = hk - 1u - (1u << 23) + (uint32_t)cc[s];
      const int idx = (int)(kb & 63u);
      const int dx = 16 * (i0c + (idx >> 2)) + 4 * h + (idx & 3) - bx;
      const int dy = 16 * bb[s] + n - 16 * br;
      const unsigned long long key = ((unsigned long long)cost << 32) |
                                     ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
      asm volatile("ds_min_u64 %0, %1" : : "v"(lds_addr(kp)), "v"(key) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) {
      const unsigned long long kk = *kp;
      const int out = (br - p.block_row_begin) * p.nbx + bc0 + col;
      store_mv(p.mv, out, kk);
      if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
      *kp = ~0ull;
    }
  };

#ifdef ME_STAMPS
  unsigned long long bw_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  BW_T0();
  // ---- prologue: the first slabs, the keys, the first two XOR-ed slabs, the
  // production steps the schedule puts before iteration 0, the first rows
  if (!searcher)
    for (int s = bfirst; s < bfirst + BW_RAWN && s <= bend; s++) dma_slab(s);
  if (tid < 4 * NS) keys[tid] = ~0ull;
  if (searcher) fetch(bfirst);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!searcher) {
    xor_slab(bfirst);
    if (bfirst + 1 <= bend) xor_slab(bfirst + 1);
    if (bfirst + pw <= blast && !(g.bw_abl & 1)) {
      const int oend = min(BW_OPS_IT * (4 - pw), BW_OPS);
      for (int o = 0; o < oend; o += BW_OPS_IT) produce(bfirst + pw, o, min(o + BW_OPS_IT, oend));
    }
  }
  __syncthreads();
  BW_ACC(0);

  const int nit = blast - bfirst + 1;
  for (int it = 0; it < nit; it++) {
    const int b = bfirst + it;
    if (!searcher) {
      if (b + BW_RAWN <= bend) dma_slab(b + BW_RAWN);
      if (b + 2 <= bend && !(g.bw_abl & 8)) xor_slab(b + 2);
      BW_ACC(1);
      // band first + m', m' = it + 1 + ((pw - it - 1) & 3), its steps of this iteration
      const int d = (pw - it - 1) & 3;
      const int m = b + 1 + d, t = 3 - d;
      if (m <= blast && !(g.bw_abl & 1)) produce(m, BW_OPS_IT * t, min(BW_OPS_IT * (t + 1), BW_OPS));
      BW_ACC(5);
    } else if (hascol) {
      if (!(g.bw_abl & 4))
        for (int br = pe0; br < pe1; br += WPC)
          enter(br, br == pe0 ? pf0 : *reinterpret_cast<const u32x4*>(cur_lane + (ptrdiff_t)(16 * br) * p.stride));
      BW_ACC(1);
      fetch(b + 1);
      BW_ACC(2);
      if (!(g.bw_abl & 2)) {
        // y validity of the band's rows per row in flight: bit 31 on the keys
        // of rows outside the row's range (partial bands only)
        uint32_t ym[NS];
        bool act[NS], ypart[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) {
          act[s] = srow[s] >= 0;
          const int ylo = max(16 * srow[s] - S, 0), yhi = min(16 * srow[s] + S, H - 16);
          const int y = 16 * b + n;
          ym[s] = (y < ylo || y > yhi) ? 0x80000000u : 0u;
          ypart[s] = 16 * b < ylo || 16 * b + 15 > yhi;
        }
        const uint32_t xb = lds_addr(xw + (b % 3) * SLAB) +
                            (uint32_t)((n + (h >> 1)) * LP + 16 * (h & 1) - 16 * tc0);
        const uint32_t pb = lds_addr(p0 + (b % BW_P0N) * P0PLANE) + (uint32_t)((n * PP + 4 * h - 16 * tc0) * 4);
        // fragments through a ring of 4 registers, two fragments ahead
        // (fragment q of tile i: window row n + 2 q + (h >> 1), column 16 i + 16 (h & 1))
        v4i f[4];
        {
          const uint32_t l0 = (uint32_t)opaque((int)(xb + (uint32_t)(16 * i0c)));
          f[0] = ldv4(l0);
          f[1] = ldv4(l0 + (uint32_t)(2 * LP));
        }
        const v4i zero4 = {0, 0, 0, 0};
#pragma unroll 1
        for (int i = i0c; i <= i1c; i++) {
          const int inx = i < i1c ? i + 1 : i;  // the last tile prefetches itself (unused)
          const uint32_t lcur = (uint32_t)opaque((int)(xb + (uint32_t)(16 * i)));
          const uint32_t lnext = (uint32_t)opaque((int)(xb + (uint32_t)(16 * inx)));
          const v4i pv = ldv4(pb + (uint32_t)(64 * i));
          v4i acc[NS];
#pragma unroll
          for (int q = 0; q < 8; q++) {
            const int qn = q + 2;
            f[qn & 3] = ldv4(qn < 8 ? lcur + (uint32_t)(2 * qn * LP) : lnext + (uint32_t)(2 * (qn - 8) * LP));
#pragma unroll
            for (int s = 0; s < NS; s++) acc[s] = MFMA16(A[s][q], f[q & 3], q == 0 ? zero4 : acc[s], 0, 0, 0);
          }
          const uint32_t rel4 = 4u * (uint32_t)(i - i0c);
          uint32_t P[4];
#pragma unroll
          for (int r = 0; r < 4; r++) P[r] = (uint32_t)pv[r] + rel4;
          // x validity on the column's first / last tile: bit 31
          const bool edge = i == i0c || i == i1c;
          uint32_t mk[4] = {0u, 0u, 0u, 0u};
          if (edge) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
              const int x = 16 * i + 4 * h + r;
              mk[r] = (x < xlo || x > xhi) ? 0x80000000u : 0u;
            }
          }
#pragma unroll
          for (int s = 0; s < NS; s++) {
            uint32_t k[4];
#pragma unroll
            for (int r = 0; r < 4; r++) k[r] = lshl7_add((uint32_t)acc[s][r], P[r]);
            if (edge) {
#pragma unroll
              for (int r = 0; r < 4; r++) k[r] |= mk[r];
            }
            if (ypart[s]) {
#pragma unroll
              for (int r = 0; r < 4; r++) k[r] |= ym[s];
            }
            bcur[s] = umin3(umin3(bcur[s], k[0], k[1]), k[2], k[3]);
          }
        }
        BW_ACC(3);
        // band end: the lane's best of the band into the row's best (an earlier
        // band keeps ties: smaller dy); rows whose last band this was leave
#pragma unroll
        for (int s = 0; s < NS; s++) {
          if (!act[s]) continue;
          if ((bcur[s] >> 6) < (bk[s] >> 6)) {
            bk[s] = bcur[s];
            bb[s] = b;
          }
          bcur[s] = ~0u;
          if (hi(srow[s]) == b) {
            emit(s);
            srow[s] = -1;
          }
        }
        BW_ACC(4);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMA'd slab and fetched cur rows landed
    __syncthreads();
    BW_ACC(6);
  }
#ifdef ME_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    bw_acc[7] = (unsigned long long)nit;
    for (int k = 0; k < 8; k++) g_bwstamps[(blockIdx.x * 8 + wave) * 8 + k] = bw_acc[k];
  }
#endif
}

static int bw_cu_count() {
  static const int cus = []() {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  return cus;
}

// Smallest pitch >= need with pitch = r (mod m): the conflict-free classes of
// the tiles' ds_read_b128 lane groups (window LP = 32 mod 64 bytes, P0 PP = 8
// mod 16 ints; checked for every group of 16 lanes).
static int pitch_at_least(int need, int r, int m) {
  int p = need + ((r - need) % m + m) % m;
  return p;
}

}  // namespace

bool plan_bw(const SearchArgs& p, MfmaGeom* g, int jobs) {
  const int S = p.range;
  g->bw = 0;
  if (p.blk != 16 || S < 1 || S > 64 || tuning().bw == 0) return false;
  if (p.stride % 16 || (uintptr_t)p.cur % 16) return false;  // 16-byte cur row loads
  const int rows = g->nrows - (g->hb_row >= 0 ? 1 : 0);       // full-height rows
  if (rows < 1 || g->nbx < 1) return false;
  // Three ring slots per searcher (A fragments of 3 rows: 96 VGPRs): the
  // 2 ceil(S/16) + 1 rows in flight of a column split over 4 / C searchers.
  // S <= 16: 4 columns, one searcher each (3 rows); S <= 32: 2 columns, two
  // searchers each (5 rows); S <= 64: 1 column, four searchers (9 rows).
  const int C = S <= 16 ? 4 : S <= 32 ? 2 : 1;
  const int ns = 3;
  const int npos_max = 16 * ((16 * (C - 1) + 2 * S) / 16 + 2);
  const int lp = C == 1 ? 224 : 160;
  if (npos_max + 16 > lp || npos_max / 4 > 52) return false;  // 4 lane rows x 13 output groups
  const int pp = pitch_at_least(npos_max, 8, 16);
  g->bw_wpc = 4 / C;
  g->bw_ns = ns;
  g->bw_cols = C;
  g->bw_lp = lp;
  g->bw_pp = pp;
  g->bw_strips = (g->nbx + C - 1) / C;
  // Segment rows: a workgroup per CU; rounds of workgroups x (segment bands +
  // the 2 ceil(S/16) extra bands + ~2 bands of prologue), the smallest
  int best_t = 1 << 30, best_l = rows;
  const int cus = bw_cu_count(), extra = 2 * ((S + 15) / 16) + 2;
  const long per = (long)std::max(jobs, 1) * g->bw_strips;
  for (int L = rows; L >= 4; L--) {
    const long segs = (rows + L - 1) / L;
    if ((rows + segs - 1) / segs != L) continue;  // even splits only
    const long rounds = (per * segs + cus - 1) / cus;
    const long t = rounds * (L + extra);
    if (t < best_t) {
      best_t = (int)t;
      best_l = L;
    }
  }
  if (tuning().bw_seg > 0) best_l = std::min(rows, tuning().bw_seg);
  g->bw_seg_rows = best_l;
  g->bw_abl = tuning().bw_abl;
  g->bw_segs = (rows + best_l - 1) / best_l;
  g->lds = bw_lds_bytes(lp, pp, ns);
  if (g->lds > 160 * 1024) return false;
  g->bw = 1;
  return true;
}

hipError_t launch_bw(const SearchArgs& p, const MfmaGeom& g0, const MfmaJobs& jb0, hipStream_t stream) {
  MfmaGeom g = g0;
  g.nrows = g0.nrows - (g0.hb_row >= 0 ? 1 : 0);  // full-height rows: the kernel's
  MfmaJobs jb = jb0;
  jb.wgs = g.bw_strips * g.bw_segs;
  const dim3 grid((unsigned)(jb.n * jb.wgs)), blk(BW_T);
  hipError_t e;
#define ME_BW_CASE(C, NS, LP)                                                            \
  if (g.bw_cols == C && g.bw_ns == NS && g.bw_lp == LP) {                                \
    e = lds_attr((const void*)me_mfma_bw_kernel<C, NS, LP>, g.lds);                      \
    if (e != hipSuccess) return e;                                                       \
    hipLaunchKernelGGL((me_mfma_bw_kernel<C, NS, LP>), grid, blk, g.lds, stream, p, g, jb); \
    return hipGetLastError();                                                            \
  }
  ME_BW_CASE(4, 3, 160) ME_BW_CASE(2, 3, 160) ME_BW_CASE(1, 3, 224)
#undef ME_BW_CASE
  return hipErrorInvalidValue;
}

}  // namespace me

#ifdef ME_STAMPS
extern "C" int me_debug_bw_stamps(unsigned long long* out, int n_words) {
  if (n_words > 8 * 8 * 4096) n_words = 8 * 8 * 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_bwstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
