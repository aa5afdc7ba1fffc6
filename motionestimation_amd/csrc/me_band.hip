// me_band.hip -- 16x16 SSD (the reference's MSE cost, souravBhat/MotionEstimation
// src/cpu/main.c:18-36, argmin with raster-first ties main.c:53-60, window
// clamp main.c:73-76) on the matrix cores, walking bands.
//
// The decomposition is me_mfma.hip's: SSD(block m, x, y) = Cc_m + S2(x, y) +
// 2 X_m(x, y) with c'' = 127 - c and r' = r - 128 (both exact i8: c ^ 0x7F,
// r ^ 0x80), X_m = sum c'' r' an i8 GEMM on v_mfma_i32_16x16x64_i8 with the
// block-major operand layout of me_mfma_bm16_kernel (one block per 16x16
// output tile of 16 x positions by 16 y positions), Cc_m = sum (c''^2 + 2 c'')
// per block and S2 = sum (r - 127)^2 over the 16x16 window per position.
// What differs from the block-major kernel is where S2 comes from: that
// kernel reads a prepass plane (7.5x the algorithmic HBM bytes at 1080p).
// Here a workgroup owns a strip of C block columns and walks DOWN a segment of
// block rows band by band: a band is the 16 candidate rows [16 b, 16 b + 16), its S2 is
// formed once in LDS, and every block row in flight (the rows whose search
// range meets the band: 2 ceil(S/16) + 1 of them) runs its MFMA tiles on it
// with the same B fragments.  A block row enters at its first band and leaves
// after its last, so the A fragments of the rows in flight stay in registers
// (a ring of NS slots per searcher wave).
//
//   waves      16 (1,024 threads, one workgroup per CU, <= 128 VGPRs): 12
//              searchers and 4 producers, three searchers and one producer
//              per SIMD.
//   searchers  waves 0..11: block column w % C of the strip, row class w / C
//              (12 / C classes split a column's rows in flight, two ring slots
//              each: A fragments of 2 rows = 64 VGPRs).  Per band and tile: 8 B
//              fragments (ds_read_b128, three ahead through a ring of 4) and
//              one P0 vector; 8 MFMAs per row in flight, no MFMA for a free
//              slot; keys (X << 7) + P0 and a v_min3 per two keys.
//   producers  waves 12..15: producer p forms bands first + p, + 4, ...: it
//              DMAs the band's 31 window rows into the band's ring slot,
//              XORs them with 0x80 in place (b128 LDS ops: the MFMA B operand
//              r'), then 46 steps of a sliding 16-row sum (16 rows in, then
//              15 x (row out, row in)), lane = 4 positions (one v_dot4 of
//              u = 127 - r = ~r' with itself per 4 bytes), the 16-wide
//              horizontal sum by DPP within 16-lane rows, stored as the key's
//              position term P0 = (S2 << 6) + 2^29 + 64 + idx.  Their VALU work runs
//              beside the searchers' MFMAs on the same SIMDs.
//   hand-off   a ring of BW_K = 8 band slots (window + P0 plane each), no
//              barrier after the start: the producer publishes ready[k] =
//              band, the searchers bump done[k] when they are through with
//              it, and the producer of band b + 8 waits for every searcher
//              before reusing the slot (bounded waits: ME_EDEVICE, never a
//              hang).
//   partial    a partial bottom block row (height < 16) is searched by the
//   bottom row producers of the last segment after their bands, on hb-row
//              S2 planes they form beside the bands.
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
#include <type_traits>

#include "me_kernels.h"
#include "me_mfma_util.h"
#include "me_tuning.h"

namespace me {

namespace {

using mfma::v4i;
using mfma::mfma_job;
using mfma::opaque;
using mfma::umin3;

constexpr int BW_OPS = 46;           // producer steps per band: 16 rows in, then 15 x (out, in)
constexpr int BW_CREC = 48;          // cur row record: 16 zero bytes, the row (c ^ 0x7F), 16 zero bytes
constexpr int BW_NSW = 12;           // searcher waves per workgroup (three per SIMD)
constexpr int BW_PW = 4;             // producer waves per workgroup (one per SIMD)

#ifdef ME_STAMPS
// Diagnostic build only (libme_hip_stamps.so): per workgroup and wave, the
// s_memtime cycles spent in each phase, summed over the bands: searchers
// [start, entries, fetch, tiles, band end, -, ready wait, bands], producers
// [start, slot wait + DMA issue, DMA wait, partial-row S2, publish,
// production, partial-row search, bands] (tools/bw_stamps.py).
constexpr int BW_STW = 16;  // waves per workgroup slot
__device__ unsigned long long g_bwstamps[BW_STW * 8 * 4096];
// per workgroup and wave: s_memrealtime (100 MHz) at its start and end
__device__ unsigned long long g_bwtimes[BW_STW * 2 * 4096];
#define BW_T0() unsigned long long bw_t = __builtin_amdgcn_s_memtime()
#define BW_ACC(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); bw_acc[k] += t_ - bw_t; bw_t = t_; } while (0)
#else
#define BW_T0() do { } while (0)
#define BW_ACC(k) do { } while (0)
#endif

constexpr int BW_K = 8;              // band ring: the bands in flight (window + P0 plane each)

constexpr int BW_WIN_ROWS = 31;      // window rows of a band: 16 b .. 16 b + 30

// Producer -> searcher handshake per band slot (LDS): ready[k] = the band
// whose window and P0 plane slot k holds (published after they are written);
// done[k] = searcher waves finished with it (the producer of band b + K
// waits for all of them, then reuses the slot).
struct BwCtl {
  uint32_t trash[4];  // (16-byte aligned) the P0 store of producer lanes without an output
  int ready[BW_K];
  int done[BW_K];
  int hbready[BW_K];  // the partial row's plane of band lo_h + i formed
  int hbcnt[BW_K];    // the partial row's bands searched, per block column
};

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

// LDS layout (bytes): K windows | K P0 planes | crec (searchers) | staged cur
// rows (searchers) | keys | ctl
__host__ __device__ constexpr int bw_win(int lp) { return BW_WIN_ROWS * lp; }
__host__ __device__ inline int bw_lds_bytes(int lp, int pp, int ns, int nsw) {
  return BW_K * bw_win(lp) + BW_K * 16 * pp * 4 + nsw * 16 * BW_CREC + nsw * 256 + nsw * ns * 8 +
         (int)sizeof(BwCtl);
}
// the partial bottom row's extra LDS: its nhb S2 planes and a key per block
// column of the strip
__host__ __device__ inline int bw_lds_hb_bytes(int pp, int ns, int nhb) {
  (void)ns;
  return nhb ? nhb * 16 * pp * 4 + BW_K * 8 : 0;  // its planes, a key per block column
}

// Bounded spin on an LDS word (the handshake's ordering argument says it
// ends; the bound keeps a broken invariant from hanging the GPU: an expired
// wait sets the context's error word, read back as ME_EDEVICE).
template <typename Pred>
__device__ __forceinline__ bool bw_wait(const SearchArgs& p, int lane, Pred ok) {
  int spins = 0;
  while (!ok()) {
    if (++spins >= (1 << 22)) {
      if (lane == 0 && p.sched)
        __hip_atomic_store(p.sched + SCHED_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// NSW searcher waves + PW producer waves, <= 128 VGPRs (four waves per SIMD).
// No workgroup barrier after the start: bands flow through a ring of BW_K
// slots, each published by its producer and released by its searchers, so a
// wave's band-end work and its waits overlap the MFMAs of the SIMD's other
// waves instead of every wave meeting at a barrier each band.
// Workgroup -> (strip item, segment).  Items u = job * strips + strip.
// Uniform (bw_xt = 0): XCD-banded workgroup index, segment-major in a job.
// Per-XCD tail split (bw_xt = 1): XCD x = blockIdx & 7 owns a contiguous run
// of the items (neighbouring strips share window rows in its L2) and walks
// them whole, one per CU per round; the last partial round's kx items
// (kx = items mod CUs per XCD) are cut into st segments each so that round
// fills the XCD's CUs too (a whole strip item takes rows + 2 ceil(S/16) + 2
// band times; its st segments ~ rows / st + that).  Launch order within an
// XCD is blockIdx order, so the segments run last.
struct BwItem {
  int u, seg, rows;  // segment seg of item u: block rows [seg rows, + rows), clipped to the job's
};
__host__ __device__ inline void bw_xcd_split(int nx, int cx, int rows, int* main, int* kx, int* st,
                                             int* L) {
  int k = nx % cx, s = 1;
  if (k) s = max(1, min(cx / k, rows / 4));
  const int l = (rows + s - 1) / s;
  *kx = k;
  *L = l;
  *st = (rows + l - 1) / l;
  *main = nx - k;
}
__device__ __forceinline__ BwItem bw_item(const MfmaGeom& g, int jobs) {
  if (!g.bw_xt) {
    int lin = mfma::xcd_banded_index();
    const int per = g.bw_strips * g.bw_segs, j = lin / per;
    lin -= j * per;
    const int seg = lin / g.bw_strips;
    return {j * g.bw_strips + lin - seg * g.bw_strips, seg, g.bw_seg_rows};
  }
  const int b = (int)blockIdx.x, x = b & 7, m = b >> 3;
  const int U = jobs * g.bw_strips, q = U >> 3, rem = U & 7;
  const int nx = q + (x < rem ? 1 : 0), u0 = x * q + min(x, rem);
  int mainx, kx, st, L;
  bw_xcd_split(nx, g.bw_cx, g.bw_seg_rows, &mainx, &kx, &st, &L);
  if (m < mainx) return {u0 + m, 0, g.bw_seg_rows};
  const int t = m - mainx;
  if (t >= kx * st) return {-1, 0, 0};
  return {u0 + mainx + t % kx, t / kx, L};
}

template <int C, int NS, int LP, int NSW, int PW, bool ABL>
__global__ __launch_bounds__(64 * (NSW + PW), 4) void me_mfma_bw_kernel(SearchArgs p, MfmaGeom g, MfmaJobs jb) {
  constexpr int WPC = NSW / C;  // row classes per column
  constexpr int WIN = bw_win(LP);
  extern __shared__ __align__(16) uint8_t smem[];
  const int PP = g.bw_pp;
  const int P0PLANE = 16 * PP;  // ints
  uint8_t* xw = smem;
  int* p0 = reinterpret_cast<int*>(xw + BW_K * WIN);
  // (the partial bottom row's S2 planes, g.bw_hb of them, follow the ring)
  const int nkeys = NSW * NS + (g.bw_hb ? BW_K : 0);  // the searchers' slots, the partial row's columns
  uint8_t* crec_all = reinterpret_cast<uint8_t*>(p0 + (BW_K + g.bw_hb) * P0PLANE);
  uint8_t* stage_all = crec_all + NSW * 16 * BW_CREC;
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(stage_all + NSW * 256);
  BwCtl* ctl = reinterpret_cast<BwCtl*>(keys + nkeys);

  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool searcher = wave < NSW;
  const int col = wave % C, cls = wave / C;  // searchers
  const int pw = wave - NSW;                 // producers: index
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  int strip, r0, r1;
  {
    const BwItem it = bw_item(g, jb.n);
    if (it.u < 0) return;  // a slot past its XCD's items (whole workgroup)
    const int j = it.u / g.bw_strips;
    strip = it.u - j * g.bw_strips;
    mfma_job(jb, j, p, g);
    r0 = g.row0 + it.seg * it.rows;
    r1 = min(r0 + it.rows, g.row0 + g.nrows);
  }
  const int bc0 = strip * C, ncol = min(C, g.nbx - bc0);
  const int tc0 = max(16 * bc0 - S, 0) >> 4;  // first tile column of the strip window
  const int tcl = min(16 * (bc0 + ncol - 1) + S, W - 16) >> 4;
  const int npos = 16 * (tcl - tc0 + 1);  // positions of the window's tiles
  const int Sc = (S + 15) >> 4;
  auto lo = [&](int br) { return max(16 * br - S, 0) >> 4; };      // first band of row br
  auto hi = [&](int br) { return min(16 * br + S, H - 16) >> 4; };  // last band of row br
  auto E = [&](int b) { return b <= 0 ? 0 : b + Sc; };              // first row with lo >= b
  const int bfirst = lo(r0), blast = hi(r1 - 1);
  // A partial bottom block row (height hbh < 16) is searched here when the
  // planner gave it S2 planes (g.bw_hb > 0): by the producers of the job's
  // last segment, after their bands, over bands lo_h .. hbrow (its last
  // candidate row is H - hbh = 16 hbrow), with an hbh-row S2 they form with
  // those bands.
  const bool hbk = g.bw_hb > 0 && g.hb_row >= 0 && r1 == g.row0 + g.nrows;
  const int hbrow = hbk ? g.hb_row : -1, hbh = g.hb;
  const int lo_h = hbk ? lo(hbrow) : 0;
  const int blast_p = hbk ? max(blast, hbrow) : blast;  // the bands the producers form
  const int nact = WPC * ncol;  // searcher waves that walk the bands (a column each)

  // ================================ producers
  // Window rows straight from global memory (8 bytes per lane: the 4
  // positions of group pg and the 4 bytes after them), rows outside the
  // resident ones outside the buffer range (read as 0; their positions are
  // masked).
  const __amdgpu_buffer_rsrc_t rref =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ref, (short)0, p.ref_bytes, 0x00020000);
  // V(row) = sum of 16 window rows of H, H(row, x) = sum over the 4 bytes at
  // x of (r - 127)^2 (u = 127 - r = ~(r ^ 0x80) as an i8, from the XOR-ed
  // window byte: one v_dot4 per 4 bytes).  Lane (row R, l) owns the 4 positions of group pg = 13 R + l: the
  // 16-lane rows overlap by 3 groups, so a group's three right neighbours are
  // in its own row (l < 13 outputs).
  const int pg = 13 * (lane >> 4) + (lane & 15);
  const bool pout = (lane & 15) < 13 && 4 * pg < npos;
  v4i V = {0, 0, 0, 0}, R = {0, 0, 0, 0};  // sums of the rows added / removed
  auto h_acc = [&](uint32_t w0, uint32_t w1, v4i acc) {  // acc + H of the XOR-ed window bytes (w0, w1)
    const uint32_t u0 = ~w0, u1 = ~w1;  // u = 127 - r = ~(r - 128)
    const uint32_t u[4] = {u0, __builtin_amdgcn_alignbyte(u1, u0, 1),
                           __builtin_amdgcn_alignbyte(u1, u0, 2),
                           __builtin_amdgcn_alignbyte(u1, u0, 3)};
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = __builtin_amdgcn_sdot4((int)u[r], (int)u[r], acc[r], false);
    return acc;
  };
  // row j of the band in slot k: with D = V - R (the rows added minus the
  // rows removed), S2(x) = D(x) + D(x + 4) + D(x + 8) + D(x + 12), the
  // neighbours by DPP row_shl 1 then 2; stored as the key's position term
  // P0 = (S2 << 6) + 2^29 + 64 + idx, idx = 4 (tile - tc0) + (x & 3): the
  // strip-relative tile, so the search adds nothing per tile (a lane's keys
  // share its x & 12, and idx orders its candidates by x)
  const uint32_t p0k = (1u << 29) + 64u + 4u * (uint32_t)(pg >> 2);
  // Every lane stores (no exec-mask branch per row, and the DPP adds fuse):
  // a lane without an output (the 3 overlap lanes of each 16-lane row, groups
  // past the window) stores into ctl->trash.
  auto out_row = [&](int k, int j) {
    v4i T, Q, D;
#pragma unroll
    for (int r = 0; r < 4; r++) D[r] = V[r] - R[r];
#pragma unroll
    for (int r = 0; r < 4; r++) T[r] = D[r] + __builtin_amdgcn_update_dpp(0, D[r], 0x101, 0xF, 0xF, true);
#pragma unroll
    for (int r = 0; r < 4; r++) Q[r] = T[r] + __builtin_amdgcn_update_dpp(0, T[r], 0x102, 0xF, 0xF, true);
    v4i o;
#pragma unroll
    for (int r = 0; r < 4; r++) o[r] = (int)(((uint32_t)Q[r] << 6) + p0k + (uint32_t)r);
    // the lane's base recomputed per row (opaque): hoisted, the 16 row
    // addresses pinned 16 VGPRs and spilled
    typedef __attribute__((address_space(3))) v4i lds_v4i;
    const uint32_t pa = pout ? (uint32_t)opaque((int)lds_addr(p0 + 4 * pg)) + 4u * (uint32_t)(k * P0PLANE + j * PP)
                             : lds_addr(ctl->trash);
    *reinterpret_cast<lds_v4i*>((uintptr_t)pa) = o;
  };
  // The band's window rows (16 m .. 16 m + 30, LP bytes from column 16 tc0)
  // by LDS DMA straight into its slot, then XOR-ed there in place by the
  // production below.  DMA_N instructions of 64 lanes x 16 bytes per window.
  constexpr int DMA_N = (WIN + 1023) / 1024;
  auto dma_win = [&](int m, int k) __attribute__((always_inline)) {
    uint8_t* dst = xw + k * WIN;
    const int rowb = 16 * m - p.ref_row0;
#pragma unroll
    for (int i = 0; i < DMA_N; i++) {
      const int d = 1024 * i + 16 * lane;
      if (d < WIN) {  // lane 0 always: every instruction issues (vmcnt counts DMA_N)
        const int rho = d / LP, kk = d - rho * LP;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rref, (__attribute__((address_space(3))) void*)(dst + 1024 * i), 16,
            (uint32_t)((rowb + rho) * p.stride + 16 * tc0 + kk), 0, 0, 0);
      }
    }
  };
  // Band m's 46 steps: 0..15 add window rows 0..15 (row 0 out after 15), then
  // for j = 1..15: remove row j - 1, add row j + 15, row j out.  Every step
  // reads its row XOR-ed (xor_win ran first: u = 127 - r = ~w).  Steps
  // [O0, O1) (compile-time, at most 12): the rows of all the steps are read
  // first (one LDS latency).
  auto step_row = [](int o) { return o < 16 ? o : ((o - 16) & 1) ? ((o - 16) >> 1) + 16 : ((o - 16) >> 1); };
  // A batch of steps [O0, O1) (compile-time, at most 12) reads the rows of
  // all its steps first (one LDS round trip), then computes them.  (Reading
  // batch i + 1 before computing batch i measured the same:
  // profiles/r06g_bw_ab.jsonl.)
  auto load = [&](auto c0, auto c1, int k, uint32_t (&w0)[12], uint32_t (&w1)[12]) __attribute__((always_inline)) {
    constexpr int O0 = decltype(c0)::value, O1 = decltype(c1)::value;
    const uint32_t xa = (uint32_t)opaque((int)lds_addr(xw + k * WIN)) + 4u * (uint32_t)pg;
#pragma unroll
    for (int o = O0; o < O1; o++) {
      w0[o - O0] = ld32(xa + (uint32_t)(step_row(o) * LP));
      w1[o - O0] = ld32(xa + (uint32_t)(step_row(o) * LP + 4));
    }
  };
  auto steps = [&](auto c0, auto c1, int k, const uint32_t (&w0)[12], const uint32_t (&w1)[12]) __attribute__((always_inline)) {
    constexpr int O0 = decltype(c0)::value, O1 = decltype(c1)::value;
#pragma unroll
    for (int o = O0; o < O1; o++) {
      const bool add = o < 16 || ((o - 16) & 1);
      // the window is XOR-ed already (xor_win): w = r ^ 0x80 (h_acc takes ~w)
      const uint32_t x0 = w0[o - O0], x1 = w1[o - O0];
      if (o < 16) {
        const v4i z = {0, 0, 0, 0};
        V = h_acc(x0, x1, o == 0 ? z : V);
        if (o == 0) R = z;
        if (o == 15) out_row(k, 0);
      } else if (!add) {
        R = h_acc(x0, x1, R);
      } else {
        V = h_acc(x0, x1, V);
        out_row(k, ((o - 16) >> 1) + 1);
      }
    }
  };
  // The partial row's S2 over hbh rows for band m into plane BW_K + (m - lo_h):
  // the same sliding sum with an hbh-row window over the band's window rows
  // (XOR-ed by produce already: u = w ^ 0xFF); runtime steps, a few bands per
  // job.
  auto produce_hb = [&](int m) {
    const int k = BW_K + (m - lo_h);
    const uint32_t xa = (uint32_t)opaque((int)lds_addr(xw + (m % BW_K) * WIN)) + 4u * (uint32_t)pg;
    const v4i z = {0, 0, 0, 0};
    V = z;
    R = z;
    // rows in groups of 4 (one LDS round trip per group, not per row: this
    // runs before the band is published)
#pragma unroll 1
    for (int t0 = 0; t0 < hbh; t0 += 4) {  // t0 + 3 <= 15: inside the window
      uint32_t a0[4], a1[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        a0[i] = ld32(xa + (uint32_t)((t0 + i) * LP));
        a1[i] = ld32(xa + (uint32_t)((t0 + i) * LP + 4));
      }
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (t0 + i < hbh) V = h_acc(a0[i], a1[i], V);
    }
    out_row(k, 0);
#pragma unroll 1
    for (int j0 = 1; j0 < 16; j0 += 4) {  // rows j - 1 and j + hbh - 1 <= 29
      uint32_t r0w[4], r1w[4], a0[4], a1[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int j = min(j0 + i, 15);
        r0w[i] = ld32(xa + (uint32_t)((j - 1) * LP));
        r1w[i] = ld32(xa + (uint32_t)((j - 1) * LP + 4));
        a0[i] = ld32(xa + (uint32_t)((j + hbh - 1) * LP));
        a1[i] = ld32(xa + (uint32_t)((j + hbh - 1) * LP + 4));
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (j0 + i > 15) break;
        R = h_acc(r0w[i], r1w[i], R);
        V = h_acc(a0[i], a1[i], V);
        out_row(k, j0 + i);
      }
    }
  };
  // The band's window XOR-ed with 0x80 in place (r - 128 as an i8: the MFMA
  // B operand), 16 bytes per lane, before the production reads it: one pass
  // of b128 LDS ops instead of a masked 4-byte write per lane and window row
  // inside the steps (31 exec-mask branches per band).
  constexpr int XN = (WIN + 1023) / 1024;
  static_assert(WIN % 16 == 0, "window slots of whole 16-byte granules");
  auto xor_win = [&](int k) __attribute__((always_inline)) {
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    const uint32_t base = (uint32_t)opaque((int)lds_addr(xw + k * WIN)) + 16u * (uint32_t)lane;
    u32x4 v[XN];
#pragma unroll
    for (int i = 0; i < XN; i++)
      if (i < XN - 1 || 1024 * i + 16 * lane < WIN) v[i] = *reinterpret_cast<lds_u32x4*>((uintptr_t)(base + 1024u * i));
#pragma unroll
    for (int i = 0; i < XN; i++)
      if (i < XN - 1 || 1024 * i + 16 * lane < WIN)
        *reinterpret_cast<lds_u32x4*>((uintptr_t)(base + 1024u * i)) = v[i] ^ 0x80808080u;
  };
  auto produce = [&](int k) __attribute__((always_inline)) {
    using I0 = std::integral_constant<int, 0>;
    using I12 = std::integral_constant<int, 12>;
    using I24 = std::integral_constant<int, 24>;
    using I36 = std::integral_constant<int, 36>;
    using IE = std::integral_constant<int, BW_OPS>;
    xor_win(k);
    uint32_t w0[12], w1[12];
    load(I0{}, I12{}, k, w0, w1);
    steps(I0{}, I12{}, k, w0, w1);
    load(I12{}, I24{}, k, w0, w1);
    steps(I12{}, I24{}, k, w0, w1);
    load(I24{}, I36{}, k, w0, w1);
    steps(I24{}, I36{}, k, w0, w1);
    load(I36{}, IE{}, k, w0, w1);
    steps(I36{}, IE{}, k, w0, w1);
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
  uint8_t* crec = crec_all + wave * 16 * BW_CREC;

  // The first row entering at band b (this column and class) is prefetched a
  // band ahead by LDS DMA into the wave's 256-byte stage (16 lanes x 16
  // bytes: no VGPRs live across the band); further ones (frame top, segment
  // starts) are loaded when they enter.
  uint8_t* stage = stage_all + wave * 256;
  const __amdgpu_buffer_rsrc_t rcur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.cur, (short)0, p.cur_bytes, 0x00020000);
  int pe0 = 0, pe1 = 0;  // this class's entering rows: pe0, pe0 + WPC, ... < pe1
  auto fetch = [&](int b) {
    const int e0 = max(E(b), r0), e1 = min(E(b + 1), r1);
    pe0 = e0 + ((cls - (e0 - r0)) % WPC + WPC) % WPC;
    pe1 = e1;
    if (hascol && lane < 16 && pe0 < pe1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rcur, (__attribute__((address_space(3))) void*)stage, 16,
          (uint32_t)((16 * pe0 + lane - p.cur_row0) * p.stride + 16 * (bc0 + col)), 0, 0, 0);
  };
  auto staged = [&]() {  // the prefetched row (lanes 0..15)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return *reinterpret_cast<const u32x4*>(stage + 16 * (lane & 15));
  };
  auto cur_row = [&](int br) {  // block row br's cur rows (lane < 16: row 16 br + lane), loaded now
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
        rcur, (uint32_t)opaque((16 * br + (lane & 15) - p.cur_row0) * p.stride + 16 * (bc0 + col)), 0, 0));
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
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (s != slot) continue;
#pragma unroll
      for (int q0 = 0; q0 < 8; q0 += 4) {  // half the records read at a time: one LDS latency each
        uint32_t d[4][5];
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
          for (int e = 0; e < 5; e++) d[q][e] = ld32(lb + (uint32_t)(2 * (q0 + q) * BW_CREC + 4 * e));
#pragma unroll
        for (int q = 0; q < 4; q++) {
          v4i f;
#pragma unroll
          for (int e = 0; e < 4; e++) f[e] = (int)__builtin_amdgcn_alignbyte(d[q][e + 1], d[q][e], sh);
          A[s][q0 + q] = f;
        }
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
    unsigned long long* kp = keys + wave * NS + s;
    if (hk < (1u << 25)) {
      const uint32_t cost = hk - 1u - (1u << 23) + (uint32_t)cc[s];
      const int idx = (int)(kb & 63u);
      const int dx = 16 * (tc0 + (idx >> 2)) + 4 * h + (idx & 3) - bx;
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
      *kp = ((unsigned long long)(uint32_t)opaque(-1) << 32) | (uint32_t)opaque(-1);  // (no pinned -1 pair)
    }
  };

  // The partial bottom row (block row hbrow, hbh < 16 rows) at block column
  // c of the strip and band b, one of its bands lo_h .. hbrow: a searcher
  // wave once its own walk is done (the pairs are dealt over all searcher
  // waves: 12 at 1080p, one each).  Its A fragments from its hbh cur rows
  // (rows below as c'' = 0: they add nothing to X or Cc), one MFMA slot, the
  // keys on the band's hbh-row S2 plane; the band's best over the lanes into
  // the column's 64-bit key, and the column's last band to finish writes its
  // record.
  auto hb_pair = [&](int c, int b, int nbh) {
    const int bxc = 16 * (bc0 + c);
    const int xl = max(bxc - S, 0), xh = min(bxc + S, W - 16);
    const int ia = xl >> 4, ib = xh >> 4;
    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
        rcur, (uint32_t)((16 * hbrow + (lane & 15) - p.cur_row0) * p.stride + bxc), 0, 0));
    const u32x4 x = (lane & 15) < hbh ? v ^ 0x7F7F7F7Fu : u32x4{0u, 0u, 0u, 0u};
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
    part += __builtin_amdgcn_update_dpp(0, part, 0x111, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x112, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x114, 0xF, 0xF, false);
    part += __builtin_amdgcn_update_dpp(0, part, 0x118, 0xF, 0xF, false);
    const int ccv = __builtin_amdgcn_readlane(part, 15);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int o = 16 + 16 * (h & 1) - n, sh = o & 3;
    const uint32_t lb = lds_addr(crec) + (uint32_t)((h >> 1) * BW_CREC + (o & ~3));
    v4i Ah[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      uint32_t d[5];
#pragma unroll
      for (int e = 0; e < 5; e++) d[e] = ld32(lb + (uint32_t)(2 * q * BW_CREC + 4 * e));
#pragma unroll
      for (int e = 0; e < 4; e++) Ah[q][e] = (int)__builtin_amdgcn_alignbyte(d[e + 1], d[e], sh);
    }
    // the band's window (slot b % K: no later band of this segment reuses
    // it) and hbh-row plane, published by its producer
    const int kw = b % BW_K;
    if (!bw_wait(p, lane, [&] {
          return __hip_atomic_load(&ctl->hbready[b - lo_h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
        }))
      return false;
    const uint32_t xb = lds_addr(xw + kw * WIN) + (uint32_t)((n + (h >> 1)) * LP + 16 * (h & 1) - 16 * tc0);
    const uint32_t pb = lds_addr(p0 + (BW_K + b - lo_h) * P0PLANE) + (uint32_t)((n * PP + 4 * h - 16 * tc0) * 4);
    uint32_t bc = ~0u;
#pragma unroll 1
    for (int i = ia; i <= ib; i++) {
      // the tile's 8 fragments and P0 vector read first: one LDS round trip
      v4i f[8];
#pragma unroll
      for (int q = 0; q < 8; q++) f[q] = ldv4(xb + (uint32_t)(16 * i + 2 * q * LP));
      const v4i pv = ldv4(pb + (uint32_t)(64 * i));
      v4i acc = {0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < 8; q++) acc = MFMA16(Ah[q], f[q], acc, 0, 0, 0);
      uint32_t k[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int xx = 16 * i + 4 * h + r;
        k[r] = ((uint32_t)acc[r] << 7) + ((uint32_t)pv[r] | ((xx < xl || xx > xh) ? 0x80000000u : 0u));
      }
      bc = umin3(umin3(bc, k[0], k[1]), k[2], k[3]);
    }
    const int ylo = max(16 * hbrow - S, 0), yhi = H - hbh;
    const int y = 16 * b + n;
    // the band's best over the lanes -> the column's key (cost, dy, dx)
    unsigned long long* kp = keys + NSW * NS + c;
    const uint32_t hk = bc >> 6;
    if (y >= ylo && y <= yhi && hk < (1u << 25)) {
      const uint32_t cost = hk - 1u - (1u << 23) + (uint32_t)ccv;
      const int idx = (int)(bc & 63u);
      const int dx = 16 * (tc0 + (idx >> 2)) + 4 * h + (idx & 3) - bxc;
      const int dy = y - 16 * hbrow;
      const unsigned long long key = ((unsigned long long)cost << 32) |
                                     ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
      asm volatile("ds_min_u64 %0, %1" : : "v"(lds_addr(kp)), "v"(key) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0 &&
        __hip_atomic_fetch_add(&ctl->hbcnt[c], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == nbh - 1) {
      const unsigned long long kk = *kp;  // every band of the column folded in
      const int out = (hbrow - p.block_row_begin) * p.nbx + bc0 + c;
      store_mv(p.mv, out, kk);
      if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
    }
    return true;
  };

#ifdef ME_STAMPS
  unsigned long long bw_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long bw_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  BW_T0();
  if (tid < nkeys) keys[tid] = ~0ull;
  if (tid < BW_K) {
    ctl->ready[tid] = -(1 << 30);
    ctl->done[tid] = 0;
    ctl->hbready[tid] = 0;
    ctl->hbcnt[tid] = 0;
  }
  __syncthreads();  // the only barrier: keys and handshake words initialised
  BW_ACC(0);

  if (!searcher) {
    // Producer pw: bands bfirst + pw, + PW, ... in order, each into slot
    // m % K.  Band m + PW's window is DMA'd (its slot released by every
    // searcher first) before band m is produced, so the DMA latency hides
    // behind one band's production.
    auto claim = [&](int m) {  // wait until slot m % K is free, then DMA band m into it
      const int k = m % BW_K;
      if (m - BW_K >= bfirst) {
        if (!bw_wait(p, lane, [&] {
              return __hip_atomic_load(&ctl->done[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= nact;
            }))
          return false;
        if (lane == 0) __hip_atomic_store(&ctl->done[k], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      dma_win(m, k);
      return true;
    };
    // (tuning build: bit 16 raises the producers' issue priority for the
    // whole walk, bit 32 for the first ring of bands only)
    if (ABL && (g.bw_abl & 48)) __builtin_amdgcn_s_setprio(2);
    // Band m + PW's window is DMA'd (its slot released by every searcher
    // first) before band m is produced, so the DMA latency hides behind one
    // band's production.  (Claiming it only when already free, else after band
    // m is published, measured the same: profiles/r06g_bw_ab.jsonl.)
    bool ok = bfirst + pw > blast_p || claim(bfirst + pw);
#pragma unroll 1
    for (int m = bfirst + pw; ok && m <= blast_p; m += PW) {
      const int k = m % BW_K;
      if (ABL && (g.bw_abl & 32) && m >= bfirst + BW_K) __builtin_amdgcn_s_setprio(0);
      const bool next = m + PW <= blast_p;
      if (next) ok = claim(m + PW);
      BW_ACC(1);
      // band m's window landed (band m + PW's DMA may still be in flight)
      if (next)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_N) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BW_ACC(2);  // (stamps, producers: DMA wait)
      if (!(ABL && (g.bw_abl & 1))) produce(k);
      BW_ACC(5);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the window and P0 stores landed
      if (lane == 0) __hip_atomic_store(&ctl->ready[k], m, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      BW_ACC(4);  // (stamps, producers: publish)
      // the partial row's plane of this band, after the band is published
      // (the searchers go on with it meanwhile)
      if (hbk && m >= lo_h) {
        if (!(ABL && (g.bw_abl & 1))) produce_hb(m);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&ctl->hbready[m - lo_h], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        BW_ACC(3);  // (stamps, producers: the partial row's S2)
      }
    }
  } else {
   if (hascol) {
    fetch(bfirst);
    if (!(ABL && (g.bw_abl & 4)))
      for (int br = pe0; br < pe1; br += WPC)
        enter(br, br == pe0 ? staged() : cur_row(br));
#pragma unroll 1
    for (int b = bfirst; b <= blast; b++) {
      const int k = b % BW_K;
      // the rows entering at band b + 1: their cur rows load during this
      // band's tiles, they enter after its end
      if (b + 1 <= blast) fetch(b + 1);
      BW_ACC(2);
      if (!bw_wait(p, lane, [&] {
            return __hip_atomic_load(&ctl->ready[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == b;
          }))
        break;
      BW_ACC(6);
      // y validity per row in flight: a lane forms the keys of one candidate
      // row (y = 16 b + n) only, so a row outside the block's range (the
      // range's partial bands) drops the lane's band best at the band end
      bool act[NS], yok[NS];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        act[s] = srow[s] >= 0;
        const int ylo = max(16 * srow[s] - S, 0), yhi = min(16 * srow[s] + S, H - 16);
        const int y = 16 * b + n;
        yok[s] = y >= ylo && y <= yhi;
      }
      if (!(ABL && (g.bw_abl & 2))) {
        // the tiles of the band for the active slots M (compile-time: no MFMA
        // for a free slot)
        auto tiles = [&](auto mc) __attribute__((always_inline)) {
          constexpr int M = decltype(mc)::value;
          const uint32_t xb = lds_addr(xw + k * WIN) + (uint32_t)((n + (h >> 1)) * LP + 16 * (h & 1) - 16 * tc0);
          const uint32_t pb = lds_addr(p0 + k * P0PLANE) + (uint32_t)((n * PP + 4 * h - 16 * tc0) * 4);
          // fragments through a ring of 4 registers, three fragments ahead
          // (fragment q of tile i: window row n + 2 q + (h >> 1), column 16 i + 16 (h & 1))
          v4i f[4];
          {
            const uint32_t l0 = (uint32_t)opaque((int)(xb + (uint32_t)(16 * i0c)));
            f[0] = ldv4(l0);
            f[1] = ldv4(l0 + (uint32_t)(2 * LP));
            f[2] = ldv4(l0 + (uint32_t)(4 * LP));
          }
          const v4i zero4 = {0, 0, 0, 0};
          // tile i, prefetching tile inx; E: the column's first or last tile,
          // where the block's x range may end (bit 31 on the position term)
          auto tile = [&](auto ec, int i, int inx) __attribute__((always_inline)) {
            constexpr bool E = decltype(ec)::value;
            const uint32_t lcur = (uint32_t)opaque((int)(xb + (uint32_t)(16 * i)));
            const uint32_t lnext = (uint32_t)opaque((int)(xb + (uint32_t)(16 * inx)));
            const v4i pv = ldv4(pb + (uint32_t)(64 * i));
            v4i acc[NS];
#pragma unroll
            for (int q = 0; q < 8; q++) {
              const int qn = q + 3;
              if (!(ABL && (g.bw_abl & 128)))
                f[qn & 3] = ldv4(qn < 8 ? lcur + (uint32_t)(2 * qn * LP) : lnext + (uint32_t)(2 * (qn - 8) * LP));
#pragma unroll
              for (int s = 0; s < NS; s++)
                if ((M >> s) & 1) acc[s] = MFMA16(A[s][q], f[q & 3], q == 0 ? zero4 : acc[s], 0, 0, 0);
            }
            uint32_t P[4];
#pragma unroll
            for (int r = 0; r < 4; r++) P[r] = (uint32_t)pv[r];
            if constexpr (E) {
              // (x opaque: hoisted out of the band loop, the masks pinned
              // VGPRs and spilled)
              const int x0 = opaque(16 * i + 4 * h);
#pragma unroll
              for (int r = 0; r < 4; r++) {
                const int x = x0 + r;
                P[r] |= (x < xlo || x > xhi) ? 0x80000000u : 0u;
              }
            }
            if (ABL && (g.bw_abl & 64)) {  // timing only: no key epilogue
#pragma unroll
              for (int s = 0; s < NS; s++)
                if ((M >> s) & 1) bcur[s] ^= (uint32_t)acc[s][0];
              return;
            }
#pragma unroll
            for (int s = 0; s < NS; s++) {
              if (!((M >> s) & 1)) continue;
              uint32_t k[4];
#pragma unroll
              // plain C, not inline asm: the compiler must see this read of the
              // MFMA result to insert the wait states the hardware does not
              // interlock (an asm read right after the MFMA read stale values)
              for (int r = 0; r < 4; r++) k[r] = ((uint32_t)acc[s][r] << 7) + P[r];
              bcur[s] = umin3(umin3(bcur[s], k[0], k[1]), k[2], k[3]);
            }
          };
          tile(std::true_type{}, i0c, min(i0c + 1, i1c));
#pragma unroll 1
          for (int i = i0c + 1; i < i1c; i++) tile(std::false_type{}, i, i + 1);
          if (i1c > i0c) tile(std::true_type{}, i1c, i1c);
        };
        int am = 0;
#pragma unroll
        for (int s = 0; s < NS; s++) am |= act[s] ? 1 << s : 0;
        am = __builtin_amdgcn_readfirstlane(am);
        if (ABL && (g.bw_abl & 256)) am &= 1;  // timing only: slot 0's MFMAs only
        if constexpr (NS == 2) {
          if (am == 3) tiles(std::integral_constant<int, 3>{});
          else if (am == 1) tiles(std::integral_constant<int, 1>{});
          else if (am == 2) tiles(std::integral_constant<int, 2>{});
        } else {
          if (am) tiles(std::integral_constant<int, (1 << NS) - 1>{});
        }
      }
      // band b's LDS reads are done: release the slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(&ctl->done[k], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      BW_ACC(3);
      // band end: the lane's best of the band into the row's best (an earlier
      // band keeps ties: smaller dy); rows whose last band this was leave
#pragma unroll
      for (int s = 0; s < NS; s++) {
        if (!act[s]) continue;
        if (yok[s] && (bcur[s] >> 6) < (bk[s] >> 6)) {
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
      if (b + 1 <= blast && !(ABL && (g.bw_abl & 4)))
        for (int br = pe0; br < pe1; br += WPC)
          enter(br, br == pe0 ? staged() : cur_row(br));
      BW_ACC(1);
    }
   }
    // then the partial bottom row: its (column, band) pairs over every
    // searcher wave
    if (hbk) {
      const int nbh = hbrow - lo_h + 1;
#pragma unroll 1
      for (int t = wave; t < ncol * nbh; t += NSW)
        if (!hb_pair(t % ncol, lo_h + t / ncol, nbh)) break;
      BW_ACC(5);  // (stamps, searchers: the partial row's search)
    }
  }
#ifdef ME_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    bw_acc[7] = (unsigned long long)(blast - bfirst + 1);
    for (int k = 0; k < 8; k++) g_bwstamps[(blockIdx.x * BW_STW + wave) * 8 + k] = bw_acc[k];
    g_bwtimes[(blockIdx.x * BW_STW + wave) * 2] = bw_rt0;
    g_bwtimes[(blockIdx.x * BW_STW + wave) * 2 + 1] = __builtin_amdgcn_s_memrealtime();
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
  // Two ring slots per searcher wave (A fragments of 2 rows: 64 VGPRs): the
  // 2 ceil(S/16) + 1 rows in flight of a column split over 12 / C searchers,
  // the widest strip whose column fits its rows: S <= 16: 6 columns (3 rows
  // on 4 slots); S <= 32: 4 (5 on 6); S <= 48: 3 (7 on 8); S <= 64: 2 (9 on
  // 12).  One workgroup of 12 searchers + 4 producers per CU (four waves per
  // SIMD at <= 128 VGPRs).
  const int nsw = BW_NSW, npw = BW_PW, ns = 2, wgs_cu = 1;
  const int inflight = 2 * ((S + 15) / 16) + 1;
  int C = 0;
  for (int c : {6, 4, 3, 2, 1})
    if (nsw % c == 0 && (nsw / c) * ns >= inflight) {
      C = c;
      break;
    }
  if (C == 0) return false;
  const int npos_max = 16 * ((16 * (C - 1) + 2 * S) / 16 + 2);
  const int lp = npos_max + 16 <= 160 ? 160 : 224;
  if (npos_max + 16 > lp || npos_max / 4 > 52) return false;  // 4 lane rows x 13 output groups
  const int pp = pitch_at_least(npos_max, 8, 16);
  g->bw_wpc = nsw / C;
  g->bw_ns = ns;
  g->bw_nsw = nsw;
  g->bw_pw = npw;
  g->bw_cols = C;
  g->bw_lp = lp;
  g->bw_pp = pp;
  g->bw_strips = (g->nbx + C - 1) / C;
  // Segments: rounds of resident workgroups x (the most bands one segment
  // walks + ~2 bands of prologue), the smallest.  A segment of rows [r0, r1)
  // walks bands lo(r0) .. hi(r1 - 1); even splits, the last segment the
  // rest.  (Uneven splits -- a longer first segment, which walks ceil(S/16)
  // fewer bands, the partial row's segment shorter -- measured 1.5 % slower
  // at 1080p: profiles/r06g_bw_ab.jsonl; longer first and last segments with
  // shorter middle ones, 12 bands worst instead of 13 at 1080p one frame,
  // 1.5 % slower again: 38.6 against 38.0 us per call, r06zl_bw_seg.jsonl.
  // The segments' band counts do not set the time alone.)
  const int cus = bw_cu_count() * wgs_cu;
  const int nfull = g->row0 + rows;  // (rows from row0: the job's full-height rows)
  auto lo_b = [&](int br) { return std::max(16 * br - S, 0) >> 4; };
  auto hi_b = [&](int br) { return std::min(16 * br + S, p.height - 16) >> 4; };
  const long per = (long)std::max(jobs, 1) * g->bw_strips;
  long best_t = 1L << 40;
  int best_l = rows, best_segs = 1;
  for (int segs = 1; segs <= std::max(1, rows / 4); segs++) {
    const int L = (rows + segs - 1) / segs;
    if ((rows + L - 1) / L != segs) continue;  // (an empty last segment)
    const long rounds = (per * segs + cus - 1) / cus;
    int worst = 0;  // bands of the longest segment
    for (int r0 = g->row0; r0 < nfull; r0 += L)
      worst = std::max(worst, hi_b(std::min(r0 + L, nfull) - 1) - lo_b(r0) + 1);
    const long t = rounds * (worst + 2);
    if (t < best_t) {
      best_t = t;
      best_l = L;
      best_segs = segs;
    }
  }
  if (tuning().bw_seg > 0) {
    best_l = std::min(rows, tuning().bw_seg);
    best_segs = (rows + best_l - 1) / best_l;
  }
  g->bw_seg_rows = best_l;
  g->bw_abl = tuning().bw_abl;
  g->bw_segs = best_segs;
  // Launches of whole rounds of strips take the per-XCD tail split instead.
  g->bw_xt = 0;
  g->bw_cx = bw_cu_count() / 8;
  if (tuning().bw_xt != 0 && tuning().bw_seg == 0 && per >= cus && g->bw_cx > 0) {
    g->bw_xt = 1;
    g->bw_seg_rows = rows;
    g->bw_segs = 1;
  }
  g->lds = bw_lds_bytes(lp, pp, ns, nsw);
  if (g->lds > 160 * 1024 / wgs_cu) return false;
  // A partial bottom block row (rows H - hb .. H - 1) joins the walk when its
  // hb-row S2 planes fit in LDS beside the ring: one per band it meets, bands
  // lo .. hb_row (its last candidate row is H - hb = 16 hb_row); otherwise it
  // is a second launch of the lean kernel (launch_bw_jobs).
  g->bw_hb = 0;
  if (g->hb_row >= 0 && tuning().bw_hb != 0) {
    const int nhb = g->hb_row - (std::max(16 * g->hb_row - S, 0) >> 4) + 1;
    const int lds_hb = g->lds + bw_lds_hb_bytes(pp, ns, nhb);
    if (lds_hb <= 160 * 1024 / wgs_cu) {
      g->bw_hb = nhb;
      g->lds = lds_hb;
    }
  }
  g->bw = 1;
  return true;
}

bool bw_one_round(const MfmaGeom& g, int jobs) {
  return (long)std::max(jobs, 1) * g.bw_strips * g.bw_segs <= (long)bw_cu_count();
}

hipError_t launch_bw(const SearchArgs& p, const MfmaGeom& g0, const MfmaJobs& jb0, hipStream_t stream) {
  MfmaGeom g = g0;
  g.nrows = g0.nrows - (g0.hb_row >= 0 ? 1 : 0);  // full-height rows: the kernel's
  MfmaJobs jb = jb0;
  jb.wgs = g.bw_strips * g.bw_segs;
  long wgs = (long)jb.n * jb.wgs;
  if (g.bw_xt) {  // 8 XCDs x the most slots one of them needs (bw_item)
    const long per = (long)jb.n * g.bw_strips;
    int wmax = 0;
    for (int nx : {(int)(per / 8), (int)((per + 7) / 8)}) {
      int mainx, kx, st, L;
      bw_xcd_split(nx, g.bw_cx, g.bw_seg_rows, &mainx, &kx, &st, &L);
      wmax = std::max(wmax, mainx + kx * st);
    }
    wgs = 8L * wmax;
  }
  const dim3 grid((unsigned)wgs), blk(64 * (g.bw_nsw + g.bw_pw));
  hipError_t e;
  // ablation instances (tuning build only: ME_BW_ABL) are separate kernels
#define ME_BW_CASE(C, NS, LP, NSW, PW)                                                          \
  if (g.bw_cols == C && g.bw_ns == NS && g.bw_lp == LP && g.bw_nsw == NSW && g.bw_pw == PW) {   \
    const void* k = g.bw_abl ? (const void*)me_mfma_bw_kernel<C, NS, LP, NSW, PW, true>         \
                             : (const void*)me_mfma_bw_kernel<C, NS, LP, NSW, PW, false>;       \
    e = lds_attr(k, g.lds);                                                                     \
    if (e != hipSuccess) return e;                                                              \
    if (g.bw_abl)                                                                               \
      hipLaunchKernelGGL((me_mfma_bw_kernel<C, NS, LP, NSW, PW, true>), grid, blk, g.lds, stream, p, g, jb); \
    else                                                                                        \
      hipLaunchKernelGGL((me_mfma_bw_kernel<C, NS, LP, NSW, PW, false>), grid, blk, g.lds, stream, p, g, jb); \
    return hipGetLastError();                                                                   \
  }
  ME_BW_CASE(6, 2, 160, 12, 4) ME_BW_CASE(4, 2, 160, 12, 4) ME_BW_CASE(3, 2, 160, 12, 4)
  ME_BW_CASE(3, 2, 224, 12, 4) ME_BW_CASE(2, 2, 160, 12, 4) ME_BW_CASE(2, 2, 224, 12, 4)
#undef ME_BW_CASE
  return hipErrorInvalidValue;
}

}  // namespace me

#ifdef ME_STAMPS
extern "C" int me_debug_bw_times(unsigned long long* out, int n_words) {
  if (n_words > me::BW_STW * 2 * 4096) n_words = me::BW_STW * 2 * 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_bwtimes), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int me_debug_bw_stamps(unsigned long long* out, int n_words) {
  if (n_words > me::BW_STW * 8 * 4096) n_words = me::BW_STW * 8 * 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_bwstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
