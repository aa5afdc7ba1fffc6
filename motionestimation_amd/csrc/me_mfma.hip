// me_mfma.hip -- the reference's cost (float MSE = SSD / (w*h), souravBhat/
// MotionEstimation src/cpu/main.c:18-36) on the CDNA4 matrix cores, for 16x16
// and 8x8 blocks.  SAD stays on the VALU (|a - b| is no contraction); SSD is one:
//
//   SSD(block m, candidate top-left (x, y))
//     = sum (c - r)^2 = Cc_m + S2(x, y) + 2 X_m(x, y)
//   c'' = 127 - c, r' = r - 128      (both in i8: bytes c ^ 0x7F and r ^ 0x80)
//   X_m(x, y) = sum_{i,j} c''_m[i][j] * r'[y + i][x + j]   (v_mfma_i32_16x16x64_i8)
//   Cc_m      = sum (c''^2 + 2 c'')  = sum (128 - c)^2 - 256     (per block)
//   S2(x, y)  = sum (r - 127)^2 over the 16x16 window at (x, y)  (per position)
// Everything is exact integer arithmetic, so the argmin (raster-first ties,
// main.c:53-60) and the reported SSD are the VALU kernels' bit for bit, and
// through them the reference's float-MSE choice.
//
// Three kernels share this decomposition and the prepass (plan_mfma_ssd picks):
//   me_mfma_bm16_kernel   16x16: block-major GEMMs (one block per output
//                         tile, see its comment) -- the default path
//   me_mfma_ssd16_kernel  16x16, S <= 103, rows not 16-byte aligned: 4x4-block tiles
//   me_mfma_ssd8_kernel   8x8: one MFMA per 4x4-block tile and position row
//
// 4x4-block tiles: M = 16 blocks of a 4x4 block tile, N = 16 candidate positions,
// K = 64 = 4 block rows x 16 columns; four MFMAs (q = 0..3, block rows 4q..4q+3)
// complete one 16x16 output tile (16 positions at one y, 16 blocks).  The B
// operand of lane (n, h) is window row R + h at position x_n, and it feeds
// the tiles y = R, R-4, R-8, R-12 (q = 0..3): one 16-byte LDS fragment per
// four MFMAs.  Positions of a wave are x_n = xbase + 4n + s (stride 4): all
// its lanes share the byte alignment of x_n, and the window is held in LDS as
// four copies shifted by 0..3 bytes (copy 0 by LDS DMA, copies 1..3 built
// from it with v_alignbyte), so every fragment read is dword aligned and the
// loop needs no realignment.
//
// Epilogue per output tile, per lane (position n, block row h, block column r
// in result register r): 32-bit keys
//   key = (SSD - p_m + 1) << 6 | (y - y0)          (p_m = Cc_m & 1)
//       = ((S2 + 1) << 6) + (y - y0) + (acc << 7),   acc = X + Cc_m >> 1
// so one v_lshl_add per candidate and an unsigned min.  Invalid pairs cannot
// win: x out of block m's window -> acc starts 2^23 higher (key in [2^30,
// 2^31)); y out of block row h's window -> bit 31 set on the lane's position
// term.  The lane's best key per block is widened to the (cost, dy, dx) key of
// the VALU kernels and merged with one LDS atomicMin per block per task.
//
// The window bytes r ^ 0x80 and the S2 plane come from a prepass kernel over
// the reference plane (me_ssd_prep_kernel): 5 bytes per pixel of scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "me_kernels.h"
#include "me_mfma_util.h"
#include "me_tuning.h"

// Steps between a row's last MFMA and its epilogue (the 16-register accumulator
// ring holds 13 + DLY rows); 2 and 3 measured slower (DESIGN.md, 8x8 blocks).
constexpr int MFMA_DLY = 1;
#ifndef ME_SSD8_KM
#define ME_SSD8_KM 3  // 8x8 chunk length L = 16 KM: 48 rows (8K +-128: 64 rows 7.12 ms, 48 6.95-7.0, 32 8.3)
#endif
#ifndef SSD8_STRIP
#define SSD8_STRIP 32  // 8x8 kernel: tile columns per strip of the workgroup order (1,024 pixels)
#endif
#ifndef ME_SSD8_ABL
#define ME_SSD8_ABL 0  // A/B ablations of the 8x8 kernel (1: no steps, 2: no re-staging); 0 in the product
#endif
#ifndef ME_SSD8_WPE
#define ME_SSD8_WPE 4  // 8x8: waves per SIMD the register budget targets (<= 128 VGPRs)
#endif
#ifndef ME_SSD8_NT
#define ME_SSD8_NT 2  // 8x8: horizontally adjacent 4x4-block tiles per workgroup (1 or 2)
#endif
#ifndef ME_SSD8_S2PERM
#define ME_SSD8_S2PERM 1  // 8x8: S2 table rows permuted in LDS (bank-conflict-free reads)
#endif
#ifndef ME_SSD8_WP
#define ME_SSD8_WP 80  // 8x8 window copy pitch: 4 x (L + 8 = 56) x 80 + S2 table (L + 1) x 256 = 30 KB at L = 48
#endif

namespace me {

namespace {

using mfma::v4i;
using mfma::opaque;
using mfma::mfma_job;
using mfma::umin3;
using mfma::lshl6_add;
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

#ifdef ME_STAMPS
// Diagnostic build only: per workgroup [start, staged, chunk 0 done, end,
// hw_id, xcc_id, realtime start, realtime end] (tools/mfma_stamps.py).
__device__ unsigned long long g_mstamps[8 << 14];
#define MS_STAMP(slot, v) do { if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) g_mstamps[8 * blockIdx.x + (slot)] = (v); } while (0)
// block-major kernel: per workgroup and band, [wave 0 compute done, barrier passed]
__device__ unsigned long long g_bstamps[32 << 12];
#define BS_STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < (1u << 12) && (slot) < 32) \
  g_bstamps[32 * blockIdx.x + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
// prepass: [start, staged, rp done, end] per workgroup, after the main kernel's slots
__device__ unsigned long long g_pstamps[6 << 14];
#define PS_STAMP(slot) do { const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x; \
  if (threadIdx.x == 0 && b_ < (1u << 14)) { g_pstamps[6 * b_ + (slot)] = __builtin_amdgcn_s_memtime(); \
    if ((slot) == 0 || (slot) == 3) g_pstamps[6 * b_ + 4 + ((slot) == 3)] = __builtin_amdgcn_s_memrealtime(); } } while (0)
#else
#define MS_STAMP(slot, v) do { } while (0)
#define BS_STAMP(slot) do { } while (0)
#define PS_STAMP(slot) do { } while (0)
#endif


// -------------------------------------------------------------- prepass
// Plane row rr is frame row ya0 + rr; every plane holds rows_alloc rows of
// `pitch` entries, all written (the main kernel's masked candidates read the
// padding, and its keys stay ordered only while every S2 it reads is < 2^23):
//   rp [rr][x]  = ref ^ 0x80 (the i8 value r - 128), 0 outside the frame
//   s2 [rr][x]  = sum_{i < 16, j < 16} (ref[ya0 + rr + i][x + j] - 127)^2,
//                 0 where the 16x16 window leaves the resident rows / frame
//   s2h[rr][x]  = the same over hb rows (the partial bottom block row, block
//                 height hb), rows >= s2h_row0 only (the last tile row's range)
// One workgroup: 64 x 64 outputs, 320 threads = 80 columns (64 + 15 halo)
// x 4 segments of 16 output rows.  Each thread loads its column's 15 + BH
// rows straight from global memory (byte loads: a wave reads consecutive
// bytes of a row, all loads of a thread independent), slides the BH-row sums
// down them into LDS and stores its rp bytes; after one barrier, 256 threads
// slide the BW-column sums along 16 outputs each.  (A staged 79 x 80 window in
// LDS, then the same two passes, took twice as long: one more global-latency
// phase and barrier per workgroup.)
constexpr int PREP_W = 64 + 16;  // columns of vertical sums (64 + 15, padded)
constexpr int VS_P = 84;         // ints per row of the vertical sums (16-byte rows, bank spread)
constexpr int PREP_T = 4 * PREP_W;  // threads per workgroup

__device__ __forceinline__ int sq127(int v) {
  v -= 127;
  return v * v;
}

constexpr int RPT_P = 80;  // bytes per row of the rp tile (16-byte aligned rows)

template <int BH, int BW>
__device__ __forceinline__ void prep_tile(const SearchArgs& p, const MfmaGeom& g, int* vs, uint8_t* rpt,
                                          int* plane, int x0, int r0, int row_lo, bool write_rp) {
  const int tid = (int)threadIdx.x;
  const int W = p.width;
  {
    const int c = tid % PREP_W, y0 = 16 * (tid / PREP_W);
    const int x = x0 + c;
    const bool xin = x < W;
    // frame row ya0 + rr; bytes outside the frame / resident rows read as 127
    // (square term 0: they only feed outputs that are zeroed)
    const uint8_t* col = p.ref + (ptrdiff_t)(g.ya0 - p.ref_row0) * p.stride + x;
    int v[16 + BH - 1];
#pragma unroll
    for (int i = 0; i < 16 + BH - 1; i++) {
      const int rr = r0 + y0 + i;
      v[i] = (xin && rr < g.rp_rows) ? (int)col[(ptrdiff_t)rr * p.stride] : 127;
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < BH; i++) s += sq127(v[i]);
#pragma unroll
    for (int j = 0; j < 16; j++) {
      vs[(y0 + j) * VS_P + c] = s;
      if (j < 15) s += sq127(v[j + BH]) - sq127(v[j]);
    }
    PS_STAMP(1);
    if (write_rp && c < 64) {  // rp bytes via LDS: stored as whole 16-byte groups below
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int rr = r0 + y0 + j;
        rpt[(y0 + j) * RPT_P + c] = (uint8_t)((xin && rr < g.rp_rows) ? (v[j] ^ 0x80) : 0);
      }
    }
  }
  __syncthreads();
  PS_STAMP(2);
  if (write_rp) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (int t = tid; t < 64 * 4; t += PREP_T) {
      const int y = t >> 2, xs = 16 * (t & 3);
      const int rr = r0 + y;
      if (rr < g.rows_alloc && x0 + xs < g.pitch)
        __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(rpt + y * RPT_P + xs),
                                    reinterpret_cast<u32x4*>(g.rp + (ptrdiff_t)rr * g.pitch + x0 + xs));
    }
  }
  // Horizontal sums, 4 outputs per task: consecutive lanes store consecutive
  // 16-byte groups (a wave's store covers 1 KB of whole lines; 16-output tasks
  // wrote 16 bytes per 64 and measured half the write bandwidth).
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  for (int t = tid; t < 64 * 16; t += PREP_T) {
    const int y = t >> 4, xs = 4 * (t & 15);
    const int yy = r0 + y;
    if (yy < g.rows_alloc && yy >= row_lo && x0 + xs < g.pitch) {
      const i32x4* v4 = reinterpret_cast<const i32x4*>(vs + y * VS_P + xs);
      int v[20];
#pragma unroll
      for (int k = 0; k < 5; k++) {
        const i32x4 qq = v4[k];
        v[4 * k] = qq[0]; v[4 * k + 1] = qq[1]; v[4 * k + 2] = qq[2]; v[4 * k + 3] = qq[3];
      }
      int sacc = 0;
#pragma unroll
      for (int j = 0; j < BW; j++) sacc += v[j];
      const bool yok = yy <= g.rp_rows - BH;
      i32x4 o;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        o[j] = (yok && x0 + xs + j <= W - BW) ? sacc : 0;
        if (j < 3) sacc += v[j + BW] - v[j];
      }
      // non-temporal: the planes are read by the next kernel, not this one
      __builtin_nontemporal_store(o, reinterpret_cast<i32x4*>(plane + (ptrdiff_t)yy * g.pitch + x0 + xs));
    }
  }
}

template <int B>
__global__ __launch_bounds__(PREP_T) void me_ssd_prep_kernel(SearchArgs p, MfmaGeom g, MfmaJobs jb) {
  // Tiles (tx, ty, job) in XCD bands: XCD k (dispatch order, bid % 8) takes
  // the k-th eighth of the row-major tile order, so the 128-byte lines two
  // neighbouring tiles share (a tile reads 80 columns) and the 7 halo rows
  // between tile rows are fetched into one L2 (round-robin tiles over the
  // XCDs fetched each line into two or three: 3x the plane's bytes).
  int bx, by, bz;
  {
    const int gx = (int)gridDim.x, gxy = gx * (int)gridDim.y;
    const int nwg = gxy * (int)gridDim.z;
    const int bid = (int)blockIdx.x + gx * ((int)blockIdx.y + (int)gridDim.y * (int)blockIdx.z);
    const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
    const int lin = x * q + min(x, rem) + m;
    bz = lin / gxy;
    by = (lin - bz * gxy) / gx;
    bx = lin - bz * gxy - by * gx;
  }
  mfma_job(jb, bz, p, g);  // z: the job of a batched launch
  __shared__ __align__(16) int vs[64 * VS_P];
  __shared__ __align__(16) uint8_t rpt[64 * RPT_P];
  // by < nmain: rp and s2 rows [64 by, +64); past it: s2h rows from s2h_row0
  // (B = 8: no rp plane, the search kernel stages the reference itself)
  const int nmain = (g.rows_alloc + 63) / 64;
  const bool hpass = by >= nmain;
  const int x0 = bx * 64;
  PS_STAMP(0);
  if (hpass) {  // hb-row sums for the partial bottom block row's lanes
    const int r0 = g.s2h_row0 + 64 * (by - nmain);
    switch (g.hb) {
#define ME_HB(k) case k: if constexpr (k < B) prep_tile<k, B>(p, g, vs, rpt, g.s2h, x0, r0, g.s2h_row0, false); break;
      ME_HB(1) ME_HB(2) ME_HB(3) ME_HB(4) ME_HB(5) ME_HB(6) ME_HB(7) ME_HB(8)
      ME_HB(9) ME_HB(10) ME_HB(11) ME_HB(12) ME_HB(13) ME_HB(14) ME_HB(15)
#undef ME_HB
      default: break;
    }
    return;
  }
  prep_tile<B, B>(p, g, vs, rpt, g.s2, x0, 64 * by, 0, B == 16);
  PS_STAMP(3);
}

// LDS DMA with 16-byte granules from any byte offset (unaligned sources probed
// exact on gfx950: tools/mfma_probe.hip); bytes is a multiple of 16.
template <typename F>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_dst, int bytes,
                                      F src_off) {
  const int tid = opaque((int)threadIdx.x);
  const int lane = tid & 63, wave = tid >> 6, nw = (int)blockDim.x >> 6;
  for (int s0 = wave * 1024; s0 < bytes; s0 += nw * 1024) {
    const int d = s0 + 16 * lane;
    if (d < bytes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(lds_dst + s0), 16, src_off(d), 0, 0, 0);
  }
}

#ifndef ME_ABL
#define ME_ABL 0  // diagnostic ablations of the block-major kernel (never in libme_hip.so)
#endif
__device__ __forceinline__ uint32_t sad_u32(uint32_t a_sgpr, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "s"(a_sgpr), "v"(b), "v"(c));
  return d;
}

// ------------------------------------------------------------------ main
// One workgroup per 4x4 block tile; 4 * NGX waves, wave w = x-subtile
// (group w >> 2 of 64 positions, phase s = w & 3).  The tile's candidate rows
// are walked in chunks of L = 13 + 16 * KM rows; per chunk the window rows
// [y0, y0 + L + 15) are staged as four shifted copies.  Step t of a chunk
// reads fragment F(t) (window row t + h) -- issued one step ahead -- and runs
// the MFMAs of output rows t - 4q; the epilogue of row t - 13 follows (its
// last MFMA ran one step earlier).
template <int NGX, int KM>
__global__ __launch_bounds__(256 * NGX)
__attribute__((amdgpu_waves_per_eu(4))) void me_mfma_ssd16_kernel(SearchArgs p, MfmaGeom g) {
  // NGX 64-position groups per workgroup (4 waves each)
  constexpr int WP = 64 * NGX + 32;  // bytes per copy row
  constexpr int DLY = MFMA_DLY;         // steps between a row's last MFMA and its epilogue
  constexpr int P0 = 12 + DLY;         // prologue steps (= epilogue lag)
  constexpr int L = P0 + 16 * KM;      // candidate rows per chunk
  constexpr int CROWS = L + 15;
  constexpr int COPY = CROWS * WP;
  extern __shared__ __align__(16) uint8_t smem[];
  constexpr int RB = 256 * NGX;        // bytes per S2 table row (64 NGX positions)
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem + 4 * COPY);
  int* cc = reinterpret_cast<int*>(smem + 4 * COPY + 16 * 8);
  uint8_t* s2t = smem + 4 * COPY + 16 * 8 + 16 * 4;  // S2 of the chunk: [L][64 NGX] ints

  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
  // (bid % 8, a speed heuristic only), so XCD x gets one contiguous band of
  // tiles and its L2 holds that band's window and S2 rows.
  // Workgroup = (tile, wg-th run of NGX groups of 64 candidate columns); a
  // tile's workgroups are adjacent in this order, so they share an XCD band.
  const int wpt = (g.ngx + NGX - 1) / NGX;  // workgroups per tile (launch-wide)
  int tile, wg;
  {
    const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
    const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
    const int lin = x * q + min(x, rem) + m;
    tile = lin / wpt;
    wg = lin - tile * wpt;
  }
  const int tx = tile % g.tiles_x, ty = tile / g.tiles_x;
  const int bc0 = 4 * tx, br0 = g.row0 + 4 * ty;
  const int nbc = min(4, g.nbx - bc0), nbr = min(4, g.row0 + g.nrows - br0);
  const int tlx0 = 16 * bc0, tly0 = 16 * br0;
  // block heights: 16, or hb for the frame's partial bottom block row
  auto bh_of = [&](int br) { return br == g.hb_row ? g.hb : 16; };
  const int xa = max(tlx0 - S, 0), xb = min(tlx0 + 16 * (nbc - 1) + S, W - 16);
  const int ya = max(tly0 - S, 0);
  const int yb = min(tly0 + 16 * (nbr - 1) + S, H - bh_of(br0 + nbr - 1));
  const int ngx = (xb - xa + 1 + 63) >> 6;  // groups this tile needs (<= g.ngx)
  const int nwt = (ngx + NGX - 1) / NGX;     // workgroups this tile needs
  if (wg >= nwt) return;  // uniform; the tile's arrival count is nwt
  const int gx0 = wg * NGX;                  // first group of this workgroup
  // tiles holding the frame's partial bottom block row read S2 from global
  // memory (see chunk()); they walk shorter chunks (L - 16) to finish with the rest
  const bool tile_hb = g.hb_row >= br0 && g.hb_row < br0 + nbr;
  const int Lt = (tile_hb && KM > 2) ? L - 16 : L;
  const int nch = (yb - ya + 1 + Lt - 1) / Lt;
  const int X0 = (xa + 64 * gx0) & ~3;  // window column origin of this workgroup

  const __amdgpu_buffer_rsrc_t rrp =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.rp, (short)0, g.rp_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.s2, (short)0, g.s2_bytes, 0x00020000);

  // Copy 0 of the window arrives by LDS DMA; copies 1..3 (shifted by 1..3
  // bytes) are built from it in LDS (v_alignbyte), not fetched again.
  auto stage = [&](int y0) {
    const int base = (y0 - g.ya0) * g.pitch + X0;
    dma16(rrp, smem, (Lt + 15) * WP, [&](int d) {
      const int rho = d / WP, k = d - rho * WP;
      return (uint32_t)(base + rho * g.pitch + k);
    });
    // S2 rows [y0, y0 + L) x this workgroup's positions [xa + 64 gx0, +64 NGX) (16-row plane)
    if (tile_hb) return;
    const int sbase = ((y0 - g.ya0) * g.pitch + xa + 64 * gx0) * 4;
    dma16(rs2, s2t, L * RB, [&](int d) {
      const int rho = d / RB, k = d - rho * RB;
      return (uint32_t)(sbase + rho * g.pitch * 4 + k);
    });
  };

  auto shift_copies = [&]() {
    typedef __attribute__((address_space(3))) uint32_t lds_w32;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) u32x4 lds_w128;
    constexpr int QW = WP / 16;  // 16-byte groups per row
    const int nq = (Lt + 15) * QW;
    for (int i = opaque(tid); i < nq; i += (int)blockDim.x) {
      const int rho = i / QW, c = i - rho * QW;
      const uint32_t off = (uint32_t)(rho * WP + 16 * c);
      const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)smem);
      const u32x4 w = *reinterpret_cast<lds_w128*>((uintptr_t)(lbase + off));
      const uint32_t nx = c + 1 < QW ? *reinterpret_cast<lds_w32*>((uintptr_t)(lbase + off + 16)) : 0u;
      sfor<1, 4>([&](auto SG) {
        constexpr int sg = decltype(SG)::value;
        const u32x4 o = {__builtin_amdgcn_alignbyte(w[1], w[0], sg), __builtin_amdgcn_alignbyte(w[2], w[1], sg),
                         __builtin_amdgcn_alignbyte(w[3], w[2], sg), __builtin_amdgcn_alignbyte(nx, w[3], sg)};
        *reinterpret_cast<lds_w128*>((uintptr_t)(lbase + sg * COPY + off)) = o;
      });
    }
  };

  MS_STAMP(0, __builtin_amdgcn_s_memtime());
  MS_STAMP(6, __builtin_amdgcn_s_memrealtime());
  if (tid < 16) {
    keys[tid] = ~0ull;
    cc[tid] = 0;
  }
  stage(ya);
  __syncthreads();

  // A fragments: lane (n, h) holds block n's rows 4q + h as c'' = c ^ 0x7F
  // (rows past the block height: 0, so they add nothing to X or Cc).
  v4i a[4];
  {
    const int br = n >> 2, bc = n & 3;
    const bool present = br < nbr && bc < nbc;
    const int bh = bh_of(br0 + br);
    int part = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      v4i v = {0, 0, 0, 0};
      if (present && 4 * q + h < bh) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(
            p.cur + (ptrdiff_t)(tly0 + 16 * br + 4 * q + h - p.cur_row0) * p.stride + tlx0 + 16 * bc);
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = (int)(src[e] ^ 0x7F7F7F7Fu);
      }
      a[q] = v;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        part = __builtin_amdgcn_sdot4(v[e], v[e], part, false);
        part = __builtin_amdgcn_sdot4(v[e], 0x02020202, part, false);
      }
    }
    if (wave == 0 && present) atomicAdd(&cc[n], part);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  shift_copies();
  __syncthreads();
  MS_STAMP(1, __builtin_amdgcn_s_memtime());

  // Per lane: block row h (y validity, S2 plane), block columns r = 0..3
  // (x validity through the accumulator start value).
  uint32_t sumLH, Cv, s2_voff;
  const int gx = gx0 + (wave >> 2), s = wave & 3;  // positions x_n = xa + 64 gx + 4n + s
  const int xn = xa + 64 * gx + 4 * n + s;
  {
    const int tly = tly0 + 16 * h;
    const int bh = bh_of(br0 + h);
    int lo = max(tly - S, 0), hi = min(tly + S, H - bh);
    if (h >= nbr) { lo = 1; hi = 0; }
    sumLH = (uint32_t)(lo + hi);
    Cv = 0x80000000u - (uint32_t)(hi - lo) - 1u;
    s2_voff = (uint32_t)xn * 4u + (bh < 16 ? g.s2h_off : 0u);
  }
  const int u = xn - X0, sig = u & 3, ccol = u - sig;
  v4i initv;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int tlx = tlx0 + 16 * r;
    const int dx = xn - tlx;
    const bool ok = r < nbc && dx >= max(-S, -tlx) && dx <= min(S, W - 16 - tlx);
    const int c = cc[4 * h + r];
    initv[r] = ok ? (c >> 1) : (c >> 1) + (1 << 23);
  }
  const uint32_t lds_lane = (uint32_t)(uintptr_t)(
      (__attribute__((address_space(3))) uint8_t*)smem) + (uint32_t)(sig * COPY + h * WP + ccol);
  const uint32_t s2t_lane = (uint32_t)(uintptr_t)(
      (__attribute__((address_space(3))) uint8_t*)s2t) + (uint32_t)(64 * (gx - gx0) + 4 * n + s) * 4u;
  const bool active = gx < ngx;

  for (int ch = 0; ch < nch; ch++) {
    const int y0 = ya + ch * Lt;
    if (ch > 0) {
      __syncthreads();  // every wave done with the previous chunk's copies
      if (ch == 1) MS_STAMP(2, __builtin_amdgcn_s_memtime());
      stage(y0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      shift_copies();
      __syncthreads();
    }
    auto chunk = [&](auto HBC) {
      constexpr int KMc = (decltype(HBC)::value && KM > 2) ? KM - 1 : KM;  // = (Lt - P0) / 16
    uint32_t best[4] = {~0u, ~0u, ~0u, ~0u};
    v4i acc[16];
    v4i fr[2];
    int sv[4];
    uint32_t lp = lds_lane;  // window row 4j of the fragments being loaded (advanced every 4 rows)
    const int s2row0 = (y0 - g.ya0) * g.pitch * 4;  // bytes, row y0 of the S2 planes

    // F(row): row & 3 is static at every call site; lp moves on at rows = 0 mod 4
    // (two ds_read2_b32 with constant offsets from one base per 4 rows).
    auto load_row = [&](v4i& dst, auto ROW) {
      constexpr int row = decltype(ROW)::value;
      if constexpr ((row & 3) == 0 && row > 0) {
        lp += 4 * WP;
        asm volatile("" : "+v"(lp));
      }
      lds_u32* w = reinterpret_cast<lds_u32*>((uintptr_t)lp + (row & 3) * WP);
      dst[0] = (int)w[0]; dst[1] = (int)w[1]; dst[2] = (int)w[2]; dst[3] = (int)w[3];
    };
    uint32_t sp = s2t_lane;  // S2 table row 16k of the main loop
    auto s2load = [&](int yrel_static_off, int yrel) -> int {
      if constexpr (decltype(HBC)::value) {
        // the lanes' S2 planes differ (s2 / s2h): straight from global memory
        (void)yrel_static_off;
        return (int)__builtin_amdgcn_raw_buffer_load_b32(rs2, s2_voff, s2row0 + yrel * g.pitch * 4, 0);
      } else {
        typedef __attribute__((address_space(3))) const int lds_i32;
        (void)yrel;
        return *reinterpret_cast<lds_i32*>((uintptr_t)(sp + (uint32_t)yrel_static_off * RB));
      }
    };
    auto epi = [&](int yrel, const v4i& av, int s2v) {
      const uint32_t P = lshl6_add((uint32_t)s2v, (uint32_t)(64 + yrel));
      const uint32_t Wd = sad_u32((uint32_t)(2 * (y0 + yrel)), sumLH, Cv);
      const uint32_t Pf = (Wd & 0x80000000u) | P;
      const uint32_t k0 = ((uint32_t)av[0] << 7) + Pf, k1 = ((uint32_t)av[1] << 7) + Pf;
      const uint32_t k2 = ((uint32_t)av[2] << 7) + Pf, k3 = ((uint32_t)av[3] << 7) + Pf;
      best[0] = min(best[0], k0);
      best[1] = min(best[1], k1);
      best[2] = min(best[2], k2);
      best[3] = min(best[3], k3);
    };

    load_row(fr[0], std::integral_constant<int, 0>{});
    // prologue: steps t = 0 .. P0-1
    sfor<0, P0>([&](auto TT) {
      constexpr int t = decltype(TT)::value;
      load_row(fr[(t + 1) & 1], std::integral_constant<int, t + 1>{});
      const v4i f = fr[t & 1];
      sfor<0, 4>([&](auto QQ) {
        constexpr int q = decltype(QQ)::value;
        if constexpr (t - 4 * q >= 0) {
          constexpr int i = (t - 4 * q) & 15;
          acc[i] = MFMA16(a[q], f, q == 0 ? initv : acc[i], 0, 0, 0);
        }
      });
      if constexpr (t >= P0 - 4) sv[(t - P0 + 4) & 3] = s2load(t - P0 + 4, t - P0 + 4);
    });
    // main: t = P0 + 16k + i, every MFMA and the epilogue of y = t - P0
    // (its last MFMA ran DLY steps earlier)
    for (int k = 0; k < KMc; k++) {
      sfor<0, 16>([&](auto II) {
        constexpr int i = decltype(II)::value;
        constexpr int t = P0 + i;  // mod 16
        const int yrel = 16 * k + i;
        load_row(fr[(t + 1) & 1], std::integral_constant<int, t + 1>{});
        const v4i f = fr[t & 1];
        sfor<0, 4>([&](auto QQ) {
          constexpr int q = decltype(QQ)::value;
          constexpr int j = (t - 4 * q) & 15;
          acc[j] = MFMA16(a[q], f, q == 0 ? initv : acc[j], 0, 0, 0);
        });
        epi(yrel, acc[i], sv[i & 3]);
        sv[i & 3] = s2load(i + 4, yrel + 4);
      });
      sp += 16 * RB;
      asm volatile("" : "+v"(sp));
    }
    // tail: t = L + e, e = 0 .. P0-1
    sfor<0, P0>([&](auto EE) {
      constexpr int e = decltype(EE)::value;
      constexpr int t = P0 + e;  // mod 16
      const int yrel = 16 * KMc + e;
      if constexpr (e < 12) {
        if constexpr (e < 11) load_row(fr[(t + 1) & 1], std::integral_constant<int, t + 1>{});
        const v4i f = fr[t & 1];
        sfor<0, 4>([&](auto QQ) {
          constexpr int q = decltype(QQ)::value;
          if constexpr (e < 4 * q) {
            constexpr int j = (t - 4 * q) & 15;
            acc[j] = MFMA16(a[q], f, acc[j], 0, 0, 0);
          }
        });
      }
      epi(yrel, acc[e], sv[e & 3]);
      if constexpr (e < P0 - 4) sv[e & 3] = s2load(e + 4, yrel + 4);
    });

    // lane bests -> (cost, dy, dx) keys of the tile's blocks
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t b = best[r];
      if (b < (1u << 30)) {
        const int m = 4 * h + r;
        const uint32_t cost = (b >> 6) - 1u + (uint32_t)(cc[m] & 1);
        const int dy = y0 + (int)(b & 63u) - (tly0 + 16 * h);
        const int dx = xn - (tlx0 + 16 * r);
        const unsigned long long key = ((unsigned long long)cost << 32) |
                                       ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
        atomicMin(&keys[m], key);
      }
    }
    };
    if (active) {
      if (tile_hb) chunk(std::true_type{});
      else chunk(std::false_type{});
    }
  }
  __syncthreads();
#ifdef ME_STAMPS
  if (tid == 0 && blockIdx.x < (1u << 14)) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_mstamps[8 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    g_mstamps[8 * blockIdx.x + 4] = hw;
    g_mstamps[8 * blockIdx.x + 5] = xcc;
    g_mstamps[8 * blockIdx.x + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  // Merge the tile's groups: with one group the keys are final; otherwise each
  // group folds its keys into the tile's global keys (device-scope atomicMin)
  // and the last group to arrive writes the outputs and resets the keys and
  // its counter for the next launch (self-resetting scratch, me_internal.h).
  const int br = tid >> 2, bc = tid & 3;
  const bool outb = tid < 16 && br < nbr && bc < nbc;
  unsigned long long* gk = g.mkeys + 16 * (size_t)tile + tid;
  // Only atomics carry data between the groups (all at the device coherence
  // point), so completion order is enough: each group waits for its returning
  // atomicMins before its arrival increment; no fences (a device-scope release
  // writes back L2).
  bool last = nwt == 1;
  if (!last) {
    int* flag = reinterpret_cast<int*>(keys + 16);  // scratch word past the keys
    if (outb) {
      const unsigned long long old = __hip_atomic_fetch_min(gk, keys[tid], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" : : "v"((uint32_t)old) : "memory");
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned arrived = __hip_atomic_fetch_add(g.mcnt + tile, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = arrived == (unsigned)nwt - 1u;
    }
    __syncthreads();
    last = flag[0] != 0;
  }
  if (last && outb) {
    const unsigned long long kk =
        nwt == 1 ? keys[tid]
                 : __hip_atomic_exchange(gk, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int out = (br0 + br - p.block_row_begin) * p.nbx + bc0 + bc;
    store_mv(p.mv, out, kk);
    if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
  }
  if (last && nwt > 1 && tid == 0)
    __hip_atomic_store(g.mcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------- 8x8 blocks
// B = 8: K = 64 is a whole block, so one MFMA finishes an output tile (16
// positions at one y x the 16 blocks of a 4x4-block tile): lane (n, h) holds
// block rows 2h, 2h+1 (A) and window rows y + 2h, y + 2h + 1 at x_n (B).  No
// accumulator ring; per step one fragment (two ds_read2_b32), one MFMA and the
// same 32-bit key epilogue as the 16x16 kernel:
//   key = ((S2 + 1) << 6) + (y - y0) + (acc << 7) = (SSD - p + 1) << 6 | (y - y0)
// SSD <= 64 * 255^2 < 2^22, so valid keys < 2^28; x out of window: acc + 2^22
// (keys in [2^29, 2^30)); y out of window: bit 31.  Chunks of L = 16 KM8 rows (48).
// Workgroup = NT horizontally adjacent tiles (ME_SSD8_NT), 4 waves (phase s),
// walking the union of the tiles' groups of 64 candidate columns one after
// another: the (cost, dy, dx) keys meet in LDS and leave once, with no
// cross-workgroup merge (per-group workgroups merged through device-scope
// atomics that reach memory: 35 MB of the 8K search's writes).  Round 6: two
// tiles share every staged window row and S2 row and every B fragment -- one
// MFMA per tile per step on the same f -- so the staging (L2 / Infinity-cache
// reads of window and S2, the copy pass, the barriers: 44 of 107 ms per 16 8K
// frames with the steps switched off) is paid once per two tiles; their
// candidate ranges overlap in all but 32 columns.
template <int KM8>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(ME_SSD8_WPE))) void me_mfma_ssd8_kernel(SearchArgs p, MfmaGeom g) {
  constexpr int WP = ME_SSD8_WP;   // bytes per copy row (64 positions + 7 + align, 16-byte granules)
  constexpr int L = 16 * KM8;      // candidate rows per chunk (yidx < 64)
  constexpr int CROWS = L + 8;     // rows y0 .. y0 + L + 6, + the last (unused) prefetch
  constexpr int COPY = CROWS * WP;
  constexpr int RB = 256;          // bytes per S2 table row (L + 1 rows: one prefetch past)
  static_assert(L <= 64, "6-bit row index");
  constexpr int NT = ME_SSD8_NT;   // tiles per workgroup
  static_assert(NT >= 1 && NT <= 4, "1 to 4 tiles per workgroup");
  extern __shared__ __align__(16) uint8_t smem[];
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem + 4 * COPY);  // [NT][16]
  int* cc = reinterpret_cast<int*>(smem + 4 * COPY + 16 * NT * 8);                     // [NT][16]
  uint8_t* s2t = smem + 4 * COPY + 16 * NT * 12;  // [L][64] ints
  constexpr int QW = WP / 16;                        // 16-byte granules per copy row
  uint8_t* nxt = s2t + (L + 1) * RB;                 // [CROWS][QW] words: the 4 bytes after each granule

  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  int wcol, ty;  // the workgroup's column of NT tiles, its tile row
  {
    // Workgroups in vertical strips of SSD8_STRIP tile columns, each strip
    // walked down its tile rows (then across the strip, then the groups); each
    // XCD (bid % 8, a speed heuristic only) takes one contiguous run of that
    // order, so its L2 sweeps one strip top to bottom: a window / S2 row stays
    // resident while the 9 tile rows that read it pass (tile-row-major order
    // re-fetched it once per tile row: 8K +-128 1.56 GB per launch).
    const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
    const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
    const int lin = x * q + min(x, rem) + m;
    const int wcols = (g.tiles_x + NT - 1) / NT;
    const int sw = min(SSD8_STRIP / NT, wcols);
    const int per_strip = g.tiles_y * sw;
    const int st = lin / per_strip, r = lin - st * per_strip;
    const int sws = min(sw, wcols - st * sw);  // the last strip may be narrower
    ty = r / sws;
    wcol = st * sw + (r - ty * sws);
  }
  // tile k of the workgroup: tile column NT wcol + k (none past the last)
  int bc0[NT], nbc[NT], tlx0[NT];
#pragma unroll
  for (int k = 0; k < NT; k++) {
    bc0[k] = 4 * (NT * wcol + k);
    nbc[k] = NT * wcol + k < g.tiles_x ? min(4, g.nbx - bc0[k]) : 0;
    tlx0[k] = 8 * bc0[k];
  }
  int kl = 0;  // the last tile present
#pragma unroll
  for (int k = 1; k < NT; k++)
    if (nbc[k] > 0) kl = k;
  const int br0 = g.row0 + 4 * ty;
  const int nbr = min(4, g.row0 + g.nrows - br0);
  const int tly0 = 8 * br0;
  const int xa = max(tlx0[0] - S, 0), xb = min(tlx0[kl] + 8 * (nbc[kl] - 1) + S, W - 8);
  const int ya = max(tly0 - S, 0), yb = min(tly0 + 8 * (nbr - 1) + S, H - 8);
  const int ngx = (xb - xa + 1 + 63) >> 6;  // groups of 64 positions this tile needs
  const int nch = (yb - ya + 1 + L - 1) / L;
  int gx = 0;                 // the group being searched
  int X0 = xa & ~3;           // its window column origin

  // The window straight from the reference plane into copy 0 (rows past the
  // resident ones read as 0 through the buffer range; bytes past W belong to
  // masked candidates only); the copy pass turns it into r ^ 0x80 in place and
  // writes the shifted copies.  (A separate raw-row region cost the fifth
  // workgroup per CU -- 35 KB -- and 3 % at 8K; prefetching it did not help.)
  const __amdgpu_buffer_rsrc_t rref =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ref, (short)0, p.ref_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.s2, (short)0, g.s2_bytes, 0x00020000);

  auto stage = [&](int y0) {
    const int base = (y0 - p.ref_row0) * p.stride + X0;
    dma16(rref, smem, COPY, [&](int d) {
      const int rho = d / WP, k = d - rho * WP;
      return (uint32_t)(base + rho * p.stride + k);
    });
    // and the word after every granule, apart: the copy pass then reads no
    // byte it (or another thread) overwrites, so it needs no barrier between
    // its reads and its writes
    {
      const int t = opaque(tid), ln = t & 63, wv = t >> 6;
      for (int s0 = 64 * wv; s0 < CROWS * QW; s0 += 256) {
        const int d = s0 + ln, rho = d / QW, c = d - rho * QW;
        if (d < CROWS * QW)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rref, (__attribute__((address_space(3))) void*)(nxt + 4 * s0), 4,
              (uint32_t)(base + rho * p.stride + 16 * (c + 1)), 0, 0, 0);
      }
    }
    const int sbase = ((y0 - g.ya0) * g.pitch + xa + 64 * gx) * 4;
#if ME_SSD8_S2PERM
    // S2 rows permuted in LDS: position p of the group at dword (p & 3) 16 +
    // (p >> 2), so the 16 positions 4 n + s one wave reads per step are 16
    // adjacent banks (in order, p = 4 n + s sat on banks 4 n + s: n and n + 8
    // collided, a 2-way conflict on every step's S2 read).  One wave-wide
    // 4-byte LDS DMA per row: lane i lands at dword i and loads position
    // 4 (i & 15) + (i >> 4) -- the row's 256 bytes, read once.
    {
      const int t = opaque(tid), ln = t & 63, wv = t >> 6;
      const uint32_t src = (uint32_t)(sbase + 4 * (4 * (ln & 15) + (ln >> 4)));
      for (int rho = wv; rho < L; rho += 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs2, (__attribute__((address_space(3))) void*)(s2t + rho * RB), 4,
            src + (uint32_t)(rho * g.pitch * 4), 0, 0, 0);
    }
#else
    dma16(rs2, s2t, L * RB, [&](int d) {
      const int rho = d / RB, k = d - rho * RB;
      return (uint32_t)(sbase + rho * g.pitch * 4 + k);
    });
#endif
  };
  auto shift_copies = [&]() {
    typedef __attribute__((address_space(3))) uint32_t lds_w32;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) u32x4 lds_w128;
    const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)smem);
    const uint32_t nbase = lbase + (uint32_t)(nxt - smem);
    // a thread's granule of copy 0 is read and rewritten by that thread only;
    // the word after it comes from the nxt table (the granule's last shifted
    // bytes beyond the 71 the lanes read are don't-cares)
    for (int i = opaque(tid); i < CROWS * QW; i += 256) {
      const int rho = i / QW, c = i - rho * QW;
      const uint32_t off = (uint32_t)(rho * WP + 16 * c);
      const u32x4 w = *reinterpret_cast<lds_w128*>((uintptr_t)(lbase + off)) ^ 0x80808080u;
      const uint32_t nx = *reinterpret_cast<lds_w32*>((uintptr_t)(nbase + 4u * (uint32_t)i)) ^ 0x80808080u;
      *reinterpret_cast<lds_w128*>((uintptr_t)(lbase + off)) = w;
      sfor<1, 4>([&](auto SG) {
        constexpr int sg = decltype(SG)::value;
        const u32x4 o = {__builtin_amdgcn_alignbyte(w[1], w[0], sg), __builtin_amdgcn_alignbyte(w[2], w[1], sg),
                         __builtin_amdgcn_alignbyte(w[3], w[2], sg), __builtin_amdgcn_alignbyte(nx, w[3], sg)};
        *reinterpret_cast<lds_w128*>((uintptr_t)(lbase + sg * COPY + off)) = o;
      });
    }
  };

  if (tid < 16 * NT) {
    keys[tid] = ~0ull;
    cc[tid] = 0;
  }
  stage(ya);
  __syncthreads();
  // A fragments: lane (n, h) holds block n's rows 2h, 2h+1 of each tile as c'' = c ^ 0x7F
  v4i a[NT];
#pragma unroll
  for (int k = 0; k < NT; k++) {
    const int br = n >> 2, bc = n & 3;
    const bool present = br < nbr && bc < nbc[k];
    v4i v = {0, 0, 0, 0};
    if (present) {
      const uint8_t* row = p.cur + (ptrdiff_t)(tly0 + 8 * br + 2 * h - p.cur_row0) * p.stride + tlx0[k] + 8 * bc;
      const uint32_t* r0 = reinterpret_cast<const uint32_t*>(row);
      const uint32_t* r1 = reinterpret_cast<const uint32_t*>(row + p.stride);
      v[0] = (int)(r0[0] ^ 0x7F7F7F7Fu); v[1] = (int)(r0[1] ^ 0x7F7F7F7Fu);
      v[2] = (int)(r1[0] ^ 0x7F7F7F7Fu); v[3] = (int)(r1[1] ^ 0x7F7F7F7Fu);
    }
    a[k] = v;
    int part = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      part = __builtin_amdgcn_sdot4(v[e], v[e], part, false);
      part = __builtin_amdgcn_sdot4(v[e], 0x02020202, part, false);
    }
    if (wave == 0 && present) atomicAdd(&cc[16 * k + n], part);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  shift_copies();
  __syncthreads();

  uint32_t sumLH, Cv;
  const int s = wave;
  {
    const int tly = tly0 + 8 * h;
    int lo = max(tly - S, 0), hi = min(tly + S, H - 8);
    if (h >= nbr) { lo = 1; hi = 0; }
    sumLH = (uint32_t)(lo + hi);
    Cv = 0x80000000u - (uint32_t)(hi - lo) - 1u;
  }
  // x_n - X0 = (xa & 3) + 4n + s whatever the group: fixed LDS lane offsets
  const int u = (xa & 3) + 4 * n + s, sig = u & 3, ccol = u - sig;
  const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)smem);
  const uint32_t lds_lane = lbase + (uint32_t)(sig * COPY + 2 * h * WP + ccol);
  const uint32_t s2t_lane = (uint32_t)(uintptr_t)(
      (__attribute__((address_space(3))) uint8_t*)s2t) +
      (uint32_t)(ME_SSD8_S2PERM ? 16 * s + n : 4 * n + s) * 4u;
  typedef __attribute__((address_space(3))) const int lds_i32;

  for (; gx < ngx; gx++) {
  X0 = (xa + 64 * gx) & ~3;
  const int xn = xa + 64 * gx + 4 * n + s;
  v4i initv[NT];
#pragma unroll
  for (int k = 0; k < NT; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int tlx = tlx0[k] + 8 * r;
      const int dx = xn - tlx;
      const bool ok = r < nbc[k] && dx >= max(-S, -tlx) && dx <= min(S, W - 8 - tlx);
      const int c = cc[16 * k + 4 * h + r];
      initv[k][r] = ok ? (c >> 1) : (c >> 1) + (1 << 22);
    }
  for (int ch = 0; ch < nch; ch++) {
    const int y0 = ya + ch * L;
    if (!(ME_SSD8_ABL & 2) && (ch > 0 || gx > 0)) {
      __syncthreads();
      stage(y0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      shift_copies();
      __syncthreads();
    }
    uint32_t best[NT][4];
#pragma unroll
    for (int k = 0; k < NT; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) best[k][r] = ~0u;
    uint32_t lp = lds_lane, sp = s2t_lane;
    // One window row (8 bytes at x_n) of lane group h: window row row + 2h.  Step
    // t's fragment is rows t + 2h, t + 2h + 1, so consecutive steps share a row:
    // one new row per step (row & 3 static at every call; lp moves every 4 rows).
    typedef int v2i __attribute__((ext_vector_type(2)));
    auto load_row = [&](v2i& dst, auto ROW) {
      constexpr int row = decltype(ROW)::value;
      if constexpr ((row & 3) == 0 && row > 0) {
        lp += 4 * WP;
        asm volatile("" : "+v"(lp));
      }
      lds_u32* w0 = reinterpret_cast<lds_u32*>((uintptr_t)lp + (row & 3) * WP);
      dst[0] = (int)w0[0]; dst[1] = (int)w0[1];
    };
    // Keys of one step; steps pair up into one v_min3 per block.  MASKED = false
    // on chunks where every lane group's block row is valid for every row
    // (the middle of a tile's range): no y test at all.
    // (the position term Pf is the same for every tile: S2 is the window's)
    auto pos_term = [&](int yrel, int s2v, auto MASKED) -> uint32_t {
      uint32_t Pf = lshl6_add((uint32_t)s2v, (uint32_t)(64 + yrel));
      if constexpr (decltype(MASKED)::value) {
        const uint32_t Wd = sad_u32((uint32_t)(2 * (y0 + yrel)), sumLH, Cv);
        Pf = (Wd & 0x80000000u) | Pf;
      }
      return Pf;
    };
    auto keys_of = [&](const v4i& av, uint32_t Pf, uint32_t (&k)[4]) {
#pragma unroll
      for (int r = 0; r < 4; r++) k[r] = ((uint32_t)av[r] << 7) + Pf;
    };
    auto body = [&](auto MASKED) {
      v2i rw[3];  // window rows t+2h (older), t+2h+1, and the prefetched t+2h+2
      int sv[2];
      uint32_t kp[NT][4];
      load_row(rw[0], std::integral_constant<int, 0>{});
      load_row(rw[1], std::integral_constant<int, 1>{});
      sv[0] = *reinterpret_cast<lds_i32*>((uintptr_t)sp);
      // fully unrolled: the 3-row ring index t % 3 must be static.  (Issuing
      // step t's MFMA before step t - 1's keys, and the position term
      // precomputed in the S2 table, measured the same or slower:
      // profiles/r06k_ssd8_ab.jsonl)
      sfor<0, L>([&](auto TT) {
        constexpr int t = decltype(TT)::value;
        // rows t+2h in rw[t % 3], t+2h+1 in rw[(t+1) % 3]; prefetch t+2h+2
        load_row(rw[(t + 2) % 3], std::integral_constant<int, t + 2>{});
        if constexpr (t + 1 < L)
          sv[(t + 1) & 1] = *reinterpret_cast<lds_i32*>((uintptr_t)(sp + (uint32_t)(t + 1) * RB));
        const v2i r0 = rw[t % 3], r1 = rw[(t + 1) % 3];
        const v4i f = {r0[0], r0[1], r1[0], r1[1]};
        v4i acc[NT];
#pragma unroll
        for (int k = 0; k < NT; k++) acc[k] = MFMA16(a[k], f, initv[k], 0, 0, 0);
        const uint32_t Pf = pos_term(t, sv[t & 1], MASKED);
#pragma unroll
        for (int k = 0; k < NT; k++) {
          if constexpr ((t & 1) == 0) {
            keys_of(acc[k], Pf, kp[k]);
          } else {
            uint32_t kc[4];
            keys_of(acc[k], Pf, kc);
#pragma unroll
            for (int r = 0; r < 4; r++) best[k][r] = umin3(best[k][r], kp[k][r], kc[r]);
          }
        }
      });
    };
    // every block row present and valid on all L rows of this chunk?
    bool full = nbr == 4;
#pragma unroll
    for (int hh = 0; hh < 4; hh++) {
      const int tly = tly0 + 8 * hh;
      full = full && max(tly - S, 0) <= y0 && min(tly + S, H - 8) >= y0 + L - 1;
    }
    if (ME_SSD8_ABL & 1) {
    } else if (full) body(std::false_type{});
    else body(std::true_type{});
#pragma unroll
    for (int k = 0; k < NT; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t b = best[k][r];
        if (b < (1u << 29)) {
          const int m = 16 * k + 4 * h + r;
          const uint32_t cost = (b >> 6) - 1u + (uint32_t)(cc[m] & 1);
          const int dy = y0 + (int)(b & 63u) - (tly0 + 8 * h);
          const int dx = xn - (tlx0[k] + 8 * r);
          const unsigned long long key = ((unsigned long long)cost << 32) |
                                         ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
          atomicMin(&keys[m], key);
        }
      }
  }
  }  // groups
  __syncthreads();
  const int kt = tid >> 4, br = (tid >> 2) & 3, bc = tid & 3;
  if (tid < 16 * NT) {
    int nbck = nbc[0], bc0k = bc0[0];
#pragma unroll
    for (int k = 1; k < NT; k++)
      if (kt == k) {
        nbck = nbc[k];
        bc0k = bc0[k];
      }
    if (br < nbr && bc < nbck) {
      const unsigned long long kk = keys[tid];
      const int out = (br0 + br - p.block_row_begin) * p.nbx + bc0k + bc;
      store_mv(p.mv, out, kk);
      if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
    }
  }
}

// ------------------------------------------------- 16x16, block-major tiles
// One block per GEMM instead of 16: the output tile is 16 x positions (M,
// x = 16 i + m) by 16 y positions (N, y = Ys + n) of ONE block, so every output
// is a candidate of that block (the 4x4-block tiles above compute 27 % useful
// outputs at S = 32; here the waste is only the range's 16-alignment).  K = 64
// = 2 block rows x a 32-byte window span: lane (m, h) of A holds block row
// 2q + (h >> 1) shifted right by m bytes inside the span (bytes 16 (h & 1) ..
// +15 of [0^m, c''_row, 0...]), so half of K is zero -- 8 MFMAs per output
// tile.  B is 16 window bytes at row Ys + n + 2q + (h >> 1), column 16 i +
// 16 (h & 1): one aligned ds_read_b128, no shifted copies.  A wave holds two
// horizontally adjacent blocks (A in 64 VGPRs) that share each B fragment and
// each S2 load; a workgroup = 4 waves = 8 blocks of one block row, whose
// window (rows [ylo, ylo + 16 Ty + 15), 16-aligned columns) is DMA'd once:
// no chunks, no cross-workgroup merge.
//   lane (n, h), result r: position x = 16 i + 4 h + r, y = Ys + n
//   key = ((2 X + S2 + 1 + 2^23) << 6) + 4 ((i - iu0) & 15) + r
//       = (X << 7) + ((S2 << 6) + 2^29 + 64 + 4 ((i - iu0) & 15) + r)
// 2 X + S2 = SSD - Cc with Cc <= 2^22, so valid keys lie in (0, 2^31), and any
// window content keeps 2 X + S2 + 1 + 2^23 in (0, 2^25): positions outside
// the block's x range get 2^24 added to the accumulator (key + 2^31, first and
// last tile only) and can never win.  y bands of 16 rows; the last band ends at
// the range's last row (overlapping its predecessor), so no y mask.  Per band
// the lane's best is widened to (key >> 6, s << 6 | idx), which orders by SSD,
// then dy, then dx (the raster-first rule); the lanes meet in a 64-bit LDS min.
// Window row pitch LP = 288 (S <= 64) or 544 (S <= 192): LP = 32 (mod 256) puts
// the 16-byte slots 2n + (h & 1) (mod 16) of a ds_read_b128 lane group on
// distinct banks.
constexpr int BM_CREC = 48;   // cur row record: 16 zero bytes, the row (c ^ 0x7F), 16 zero bytes
constexpr int BM_HDR = 8 * 16 * BM_CREC + 8 * 8 + 8 * 4;  // records, keys, cc

template <int LP>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(4))) void me_mfma_bm16_kernel(SearchArgs p, MfmaGeom g, MfmaJobs jb) {
  constexpr int BM_LP = LP;
  constexpr int BM_WINB = 31 * LP;  // one band's window rows
  extern __shared__ __align__(16) uint8_t smem[];
  uint8_t* crec = smem;
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem + 8 * 16 * BM_CREC);
  int* cc = reinterpret_cast<int*>(smem + 8 * 16 * BM_CREC + 64);
  uint8_t* win = smem + BM_HDR;

  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  int lin;
  {  // XCD-banded: XCD x walks one contiguous run of strips
    const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
    const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
    lin = x * q + min(x, rem) + m;
  }
  {  // batched launch: jobs are consecutive runs of jb.wgs workgroups
    const int j = lin / jb.wgs;
    lin -= j * jb.wgs;
    mfma_job(jb, j, p, g);
  }
  const int brl = lin / g.bm_wpr, sx = lin - brl * g.bm_wpr;
  const int br = g.row0 + brl;
  const int bc0 = 8 * sx, nb = min(8, g.nbx - bc0);
  const int by = 16 * br, bh = br == g.hb_row ? g.hb : 16;
  const int ylo = max(by - S, 0), yhi = min(by + S, H - bh);
  const int Ty = (yhi - ylo + 16) >> 4;
  const int tc0 = max(16 * bc0 - S, 0) >> 4;
  // y bands of 16 rows; when the range has >= 16 rows the last band ends at yhi
  // (it overlaps the one before: no row past yhi is ever computed)
  const bool yover = yhi - ylo >= 15;
  auto band_y = [&](int s) { return yover ? min(ylo + 16 * s, yhi - 15) : ylo + 16 * s; };
  // band window: frame rows [Ys, Ys + 31) x columns [16 tc0, 16 tc0 + BM_LP),
  // double-buffered (band s + 1 arrives by LDS DMA while band s computes)
  const __amdgpu_buffer_rsrc_t rrp =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.rp, (short)0, g.rp_bytes, 0x00020000);
  auto stage_band = [&](int s) {
    const int gbase = (band_y(s) - g.ya0) * g.pitch + 16 * tc0;
    dma16(rrp, win + (s & 1) * BM_WINB, BM_WINB, [&](int d) {
      const int rho = d / BM_LP, k = d - rho * BM_LP;
      return (uint32_t)(gbase + rho * g.pitch + k);
    });
  };

  MS_STAMP(0, __builtin_amdgcn_s_memtime());
  MS_STAMP(6, __builtin_amdgcn_s_memrealtime());
  if (tid < 8) {
    keys[tid] = ~0ull;
    cc[tid] = 0;
  }
  stage_band(0);
  __syncthreads();  // keys / cc initialised
  if (tid < 128) {  // cur row records and Cc = sum(c''^2 + 2 c'')
    const int j = tid >> 4, rho = tid & 15;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {0u, 0u, 0u, 0u};
    if (j < nb && rho < bh) {
      const u32x4* src = reinterpret_cast<const u32x4*>(
          p.cur + (ptrdiff_t)(by + rho - p.cur_row0) * p.stride + 16 * (bc0 + j));
      v = *src ^ 0x7F7F7F7Fu;
    }
    const u32x4 z = {0u, 0u, 0u, 0u};
    u32x4* rec = reinterpret_cast<u32x4*>(crec + (16 * j + rho) * BM_CREC);
    rec[0] = z;
    rec[1] = v;
    rec[2] = z;
    int part = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      part = __builtin_amdgcn_sdot4((int)v[e], (int)v[e], part, false);
      part = __builtin_amdgcn_sdot4((int)v[e], 0x02020202, part, false);
    }
    if (j < nb) atomicAdd(&cc[j], part);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int j0 = 2 * wave, j1 = j0 + 1;
  const bool hasA = j0 < nb, hasB = j1 < nb;
  // per block: tile range [i0, i1] (16-aligned positions) and x range [xlo, xhi]
  const int bxA = 16 * (bc0 + j0), bxB = bxA + 16;
  const int xloA = max(bxA - S, 0), xhiA = min(bxA + S, W - 16);
  const int xloB = max(bxB - S, 0), xhiB = min(bxB + S, W - 16);
  const int i0A = xloA >> 4, i1A = xhiA >> 4, i0B = xloB >> 4, i1B = xhiB >> 4;
  const int iu0 = i0A, iu1 = hasB ? i1B : i1A;

  // A fragments: bytes o .. o + 15 of record row 2q + (h >> 1), o = 16 + 16 (h & 1) - m
  v4i aA[8], aB[8];
  {
    const int o = 16 + 16 * (h & 1) - n, sh = o & 3;
    typedef __attribute__((address_space(3))) const uint32_t lds_c32;
    const uint32_t lb = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)crec) +
                        (uint32_t)((h >> 1) * BM_CREC + (o & ~3));
#pragma unroll
    for (int q = 0; q < 8; q++) {
#pragma unroll
      for (int bsel = 0; bsel < 2; bsel++) {
        const uint32_t a0 = lb + (uint32_t)(((2 * wave + bsel) * 16 + 2 * q) * BM_CREC);
        uint32_t d[5];
#pragma unroll
        for (int e = 0; e < 5; e++) d[e] = *reinterpret_cast<lds_c32*>((uintptr_t)(a0 + 4 * e));
        v4i f;
#pragma unroll
        for (int e = 0; e < 4; e++) f[e] = (int)__builtin_amdgcn_alignbyte(d[e + 1], d[e], sh);
        if (bsel == 0) aA[q] = f; else aB[q] = f;
      }
    }
  }
  MS_STAMP(1, __builtin_amdgcn_s_memtime());
  const int ccA = hasA ? cc[j0] : 0, ccB = hasB ? cc[j1] : 0;
  // Masks of a block's first / last tile: 2^24 on the accumulator of positions
  // outside [xlo, xhi] (bit 31 of the key).
  // Bit 4 e + r of mbits: result r of edge e (A first, A last, B first, B last).
  uint32_t mbits = 0;
  {
    auto xmask = [&](int e, int i, int xlo, int xhi) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int x = 16 * i + 4 * h + r;
        if (x < xlo || x > xhi) mbits |= 1u << (4 * e + r);
      }
    };
    xmask(0, i0A, xloA, xhiA);
    xmask(1, i1A, xloA, xhiA);
    xmask(2, i0B, xloB, xhiB);
    xmask(3, i1B, xloB, xhiB);
  }
  const uint32_t ym = (!yover && n > yhi - ylo) ? 0x80000000u : 0u;  // OR-ed into the key
  // Interior pairs (both blocks' x ranges inside the frame, >= 3 tiles each,
  // full 16-row bands) take the mask-free fast path; their only invalid
  // positions are the range ends inside the first and the last tile, the
  // same lanes for every such block: m < (bx - S) & 15, m > (bx + S) & 15.
  const bool fast = hasB && yover && bxA - S >= 0 && bxB + S <= W - 16 && i1A - i0A >= 2;
  const int mfa = (bxA - S) & 15, mlb = (bxA + S) & 15;
  v4i mF, mL;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int m = 4 * h + r;
    mF[r] = m < mfa ? (1 << 24) : 0;
    mL[r] = m > mlb ? (1 << 24) : 0;
  }

  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.s2, (short)0, g.s2_bytes, 0x00020000);
  const int s2v = (n * g.pitch + 4 * h) * 4 + (br == g.hb_row ? (int)g.s2h_off : 0);
  const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)win) +
                         (uint32_t)((n + (h >> 1)) * BM_LP + 16 * (h & 1) - 16 * tc0);
  typedef __attribute__((address_space(3))) const v4i lds_v4i;
  const v4i zero4 = {0, 0, 0, 0};

  unsigned long long bestA = ~0ull, bestB = ~0ull;  // (key >> 6) << 32 | s << 6 | idx
  for (int s = 0; s < Ty; s++) {
    if (s + 1 < Ty) stage_band(s + 1);
    if (hasA) {
      const int Ys = band_y(s);
      const uint32_t lrow0 = lbase + (uint32_t)((s & 1) * BM_WINB);
      const int srow = (Ys - g.ya0) * g.pitch * 4;
      uint32_t bA = ~0u, bB = ~0u;
      // Widen the lane's 32-bit bests to (key >> 6, band << 8 | segment << 6 | idx):
      // a key's 6-bit index holds 16 tiles, so every 16 tiles of a band form a
      // segment.  The strictly better key wins: an earlier band (smaller dy) or
      // segment (smaller dx) keeps ties.
      auto widen = [&](int seg) {
        const uint32_t lo = ((uint32_t)s << 8) | ((uint32_t)seg << 6);
        const unsigned long long kA = ((unsigned long long)(bA >> 6) << 32) | lo | (bA & 63u);
        const unsigned long long kB = ((unsigned long long)(bB >> 6) << 32) | lo | (bB & 63u);
        bestA = (kA >> 32) < (bestA >> 32) ? kA : bestA;
        bestB = (kB >> 32) < (bestB >> 32) ? kB : bestB;
        bA = ~0u;
        bB = ~0u;
      };
      // One 16 x 16 output tile per block at window column 16 i.  MA / MB: the
      // mask of block A / B on this tile -- 0 none, 1 the first-tile mask mF, 2
      // the last-tile mask mL (both as the first MFMA's accumulator input, no
      // VALU), 3 the generic path (mbits, ym: frame-clipped pairs, tiny ranges).
      auto tile = [&](int i, auto DA, auto DB, auto MA, auto MB) {
        constexpr bool da = decltype(DA)::value, db = decltype(DB)::value;
        constexpr int ma = decltype(MA)::value, mb = decltype(MB)::value;
#if ME_ABL == 1  // diagnostic build: no S2 loads (timing only, keys wrong)
        const v4i s2c = {srow, s2v, i, 0};
#else
        const v4i s2c = __builtin_bit_cast(
            v4i, __builtin_amdgcn_raw_buffer_load_b128(rs2, s2v, srow + 64 * i, 0));
#endif
        // one base per tile, fragment rows at immediate offsets
        const uint32_t lrow = (uint32_t)opaque((int)(lrow0 + (uint32_t)(16 * i)));
        v4i accA = ma == 1 ? mF : ma == 2 ? mL : zero4;
        v4i accB = mb == 1 ? mF : mb == 2 ? mL : zero4;
        // Fragments in pairs, the next pair in flight during this pair's MFMAs
        // (four fragments live: the A fragments hold 64 VGPRs).
        auto ld = [&](int q) {
#if ME_ABL == 3  // diagnostic build: two fragment rows per tile (a quarter of the LDS reads)
          q &= 1;
#endif
          return *reinterpret_cast<lds_v4i*>((uintptr_t)(lrow + (uint32_t)(2 * q * BM_LP)));
        };
        v4i f0 = ld(0), f1 = ld(1);
#pragma unroll
        for (int qp = 0; qp < 4; qp++) {
          v4i n0 = f0, n1 = f1;
          if (qp < 3) {
            n0 = ld(2 * qp + 2);
            n1 = ld(2 * qp + 3);
          }
          if constexpr (da) accA = MFMA16(aA[2 * qp], f0, accA, 0, 0, 0);
          if constexpr (db) accB = MFMA16(aB[2 * qp], f0, accB, 0, 0, 0);
          if constexpr (da) accA = MFMA16(aA[2 * qp + 1], f1, accA, 0, 0, 0);
          if constexpr (db) accB = MFMA16(aB[2 * qp + 1], f1, accB, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          f0 = n0;
          f1 = n1;
        }
        // key = ((2 acc + S2 + 1 + 2^23) << 6) + 4 ((i - iu0) & 15) + r, acc = X (+ masks):
        // one v_lshl_add for the shared position term, one per key
        const int rel = i - iu0;
        const uint32_t kb = (1u << 29) + 64u + 4u * (uint32_t)(rel & 15);
        uint32_t P[4];
#pragma unroll
        for (int r = 0; r < 4; r++) P[r] = lshl6_add((uint32_t)s2c[r], kb + (uint32_t)r);
        auto keys_of = [&](v4i acc, uint32_t& best, int i0, int i1, int e0, auto GEN) {
#if ME_ABL == 2  // diagnostic build: no key epilogue (timing only)
          asm volatile("" : : "v"(acc), "v"(P[0]));
          best ^= (uint32_t)acc[0];
          return;
#endif
          if constexpr (decltype(GEN)::value) {
            if (i == i0 || i == i1) {
              const int e = i == i0 ? e0 : e0 + 1;
              const uint32_t mb4 = (uint32_t)opaque((int)mbits);  // not hoisted: no 16 VGPRs of masks
#pragma unroll
              for (int r = 0; r < 4; r++)
                acc[r] += (int)(__builtin_amdgcn_ubfe(mb4, (uint32_t)(4 * e + r), 1u) << 24);
            }
          }
          uint32_t k[4];
#pragma unroll
          for (int r = 0; r < 4; r++) k[r] = ((uint32_t)acc[r] << 7) + P[r];
          if constexpr (decltype(GEN)::value) {
#pragma unroll
            for (int r = 0; r < 4; r++) k[r] |= ym;
          }
          best = umin3(best, k[0], k[1]);
          best = umin3(best, k[2], k[3]);
        };
        if constexpr (da) keys_of(accA, bA, i0A, i1A, 0, std::integral_constant<bool, ma == 3>{});
        if constexpr (db) keys_of(accB, bB, i0B, i1B, 2, std::integral_constant<bool, mb == 3>{});
        if ((rel & 15) == 15 && i < iu1) widen(rel >> 4);  // S >= 113: a band spans > 16 tiles
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      using M0 = std::integral_constant<int, 0>;
      using M1 = std::integral_constant<int, 1>;
      using M2 = std::integral_constant<int, 2>;
      using M3 = std::integral_constant<int, 3>;
      if (fast) {
        // interior pair: A's tiles i0A .. i1A, B's one to the right
        tile(i0A, T_{}, F_{}, M1{}, M0{});
        tile(i0A + 1, T_{}, T_{}, M0{}, M1{});
        for (int i = i0A + 2; i < i1A; i++) tile(i, T_{}, T_{}, M0{}, M0{});
        tile(i1A, T_{}, T_{}, M2{}, M0{});
        tile(i1B, F_{}, T_{}, M0{}, M2{});
      } else {
        for (int i = iu0; i <= iu1; i++) {
          const bool useA = i <= i1A, useB = hasB && i >= i0B;
          if (useA && useB) tile(i, T_{}, T_{}, M3{}, M3{});
          else if (useA) tile(i, T_{}, F_{}, M3{}, M3{});
          else tile(i, F_{}, T_{}, M3{}, M3{});
        }
      }
      widen((iu1 - iu0) >> 4);  // end of the band
    }
    if (s == 0) MS_STAMP(2, __builtin_amdgcn_s_memtime());
    BS_STAMP(2 * s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // band s + 1 landed (this thread's pieces)
    __syncthreads();                                   // ... and everyone's; band s free
    BS_STAMP(2 * s + 1);
  }
  if (hasA) {
    auto emit = [&](unsigned long long b, int j, int ccj, int bx) {
      const uint32_t hi = (uint32_t)(b >> 32);
      if (hi < (1u << 25)) {
        const uint32_t lo = (uint32_t)b;
        const int sb = (int)(lo >> 8), seg = (int)((lo >> 6) & 3u), idx = (int)(lo & 63u);
        const uint32_t cost = hi - 1u - (1u << 23) + (uint32_t)ccj;
        const int dx = 16 * (iu0 + 16 * seg + (idx >> 2)) + 4 * h + (idx & 3) - bx;
        const int dy = band_y(sb) + n - by;
        const unsigned long long key = ((unsigned long long)cost << 32) |
                                       ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
        // per-lane LDS atomic (the compiler's wave-scan expansion of a
        // uniform-address atomicMin is a 64-step readlane loop)
        const uint32_t a = (uint32_t)(uintptr_t)(
            (__attribute__((address_space(3))) unsigned long long*)(keys + j));
        asm volatile("ds_min_u64 %0, %1" : : "v"(a), "v"(key) : "memory");
      }
    };
    emit(bestA, j0, ccA, bxA);
    if (hasB) emit(bestB, j1, ccB, bxB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();
#ifdef ME_STAMPS
  if (tid == 0 && blockIdx.x < (1u << 14)) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_mstamps[8 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    g_mstamps[8 * blockIdx.x + 4] = hw;
    g_mstamps[8 * blockIdx.x + 5] = xcc;
    g_mstamps[8 * blockIdx.x + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (tid < nb) {
    const unsigned long long kk = keys[tid];
    const int out = (br - p.block_row_begin) * p.nbx + bc0 + tid;
    store_mv(p.mv, out, kk);
    if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
  }
}

// --------------------------- 16x16, block-major, S2 formed in the workgroup
// me_mfma_bmv_kernel: the block-major kernel above without the prepass and its
// HBM planes (the rp bytes and the 4-byte S2 plane were 7.5x the algorithmic
// bytes of a 1080p search, DESIGN.md "SSD-path HBM traffic").  The band window
// is DMA'd from the reference plane itself, and every band's S2 is formed in
// LDS from the window the band already holds:
//   phase A  lane = position p: with u = r ^ 0x7F = 127 - r (an exact i8),
//            (r - 127)^2 = u^2, so H(row, p) = sum_{4 bytes} u^2 is ONE v_dot4
//            (plus the XOR and the v_alignbyte of the position's 4 bytes);
//            V(k, p) = sum_{i < hb} H(k + i, p) by a sliding sum down the
//            15 + hb window rows (raw bytes: it runs before the window is XOR-ed)
//   phase B  S2(k, x) = V(k, x) + V(k, x + 4) + V(k, x + 8) + V(k, x + 12), in place
//   the window's bytes are XOR-ed with 0x80 (r' = r - 128, the B operand)
// The tiles then read S2 from LDS instead of the plane.  crec (the cur row
// records) aliases the S2 plane: the A fragments are built before band 0.
// S <= 64 (window pitch 288): LDS 35 KB, four workgroups per CU as before.
constexpr int BMV_NP = 268;                // S2 / V plane row pitch (ints): 256 positions + 12 V; 67 * 4
constexpr int BMV_PLANE = 16 * BMV_NP * 4; // 17,152 bytes (>= the 6,144 of crec)
constexpr int BMV_LP = 288;
// acc + sum over the 4 bytes r of v of (r - 127)^2: u = r ^ 0x7F is 127 - r as
// an i8 (r in [0, 255] -> u in [-128, 127]), and u^2 = (r - 127)^2
__device__ __forceinline__ int h4acc(uint32_t v, int acc) {
  const int u = (int)(v ^ 0x7F7F7F7Fu);
  return __builtin_amdgcn_sdot4(u, u, acc, false);
}

// Phase A, 16-row blocks: V(k, p) for the 16 band rows k, position p (window
// column p), from window rows 0..30 (raw bytes, pitch LP); written to vcol[k * BMV_NP].
template <int LP>
__device__ __forceinline__ void bmv_vsum16(const uint8_t* win, int p, int* vcol) {
  typedef __attribute__((address_space(3))) const uint32_t lds_c32;
  // opaque: one base per call, the rows at immediate offsets (hoisted, the 31
  // row addresses were kept live across the band loop and spilled)
  const uint32_t a = (uint32_t)opaque(
      (int)((uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)win) +
            (uint32_t)(p & ~3)));
  const uint32_t sh = (uint32_t)(p & 3);
  auto row = [&](int k) {
    const uint32_t d0 = *reinterpret_cast<lds_c32*>((uintptr_t)(a + (uint32_t)(k * LP)));
    const uint32_t d1 = *reinterpret_cast<lds_c32*>((uintptr_t)(a + (uint32_t)(k * LP) + 4u));
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
  };
  // The column's own plane entries hold H(k) until V(k) replaces them (no
  // register array: the A fragments keep 64 VGPRs live across this phase).
  int v = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int nv = h4acc(row(k), v);
    if (k < 15) vcol[k * BMV_NP] = nv - v;  // H(k)
    v = nv;
  }
#pragma unroll
  for (int k = 1; k < 16; k++) {
    const int old = vcol[(k - 1) * BMV_NP];
    vcol[(k - 1) * BMV_NP] = v;
    v = h4acc(row(k + 15), v) - old;
  }
  vcol[15 * BMV_NP] = v;
}

// Phase A for a partial bottom block row (block height hb < 16): direct sums.
template <int LP>
__device__ __forceinline__ void bmv_vsum_hb(const uint8_t* win, int p, int hb, int* vcol) {
  typedef __attribute__((address_space(3))) const uint32_t lds_c32;
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)win) +
                     (uint32_t)(p & ~3);
  const uint32_t sh = (uint32_t)(p & 3);
  for (int k = 0; k < 16; k++) {
    int v = 0;
    for (int i = 0; i < hb; i++) {
      const uint32_t o = a + (uint32_t)((k + i) * LP);
      v = h4acc(__builtin_amdgcn_alignbyte(*reinterpret_cast<lds_c32*>((uintptr_t)(o + 4u)),
                                           *reinterpret_cast<lds_c32*>((uintptr_t)o), sh), v);
    }
    vcol[k * BMV_NP] = v;
  }
}

// Workgroup = R block rows (R = 1 or 2) x 8 blocks, 4 waves per row.  The y
// bands are the workgroup's: Y_s = ylo (of its first row) + 16 s, so a band's
// S2 is formed once for every row whose range it meets (R = 2: 6 bands for two
// rows at S = 32 instead of 5 + 5).  A row skips the bands outside its range
// and masks the rows of a band that leave it (bit 31 of the key).  A partial
// bottom block row (height hb) reads a second S2 plane of hb-row sums when it
// shares the workgroup with a full row.
template <int R>
constexpr int bmv_lds() {
  return R * (8 * 8 + 8 * 4) + (R == 2 ? 2 : 1) * BMV_PLANE + 2 * 31 * BMV_LP;
}

template <int R>
__global__ __launch_bounds__(256 * R)
__attribute__((amdgpu_waves_per_eu(4))) void me_mfma_bmv_kernel(SearchArgs p, MfmaGeom g, MfmaJobs jb) {
  constexpr int LP = BMV_LP;
  constexpr int WINB = 31 * LP;  // one band's window rows
  constexpr int NT = 256 * R;    // threads
  constexpr int KEYS = R * (8 * 8 + 8 * 4);
  static_assert(R * 8 * 16 * BM_CREC <= BMV_PLANE, "crec aliases the S2 plane");
  extern __shared__ __align__(16) uint8_t smem[];
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);  // [R * 8]
  int* cc = reinterpret_cast<int*>(smem + R * 64);                          // [R * 8]
  int* plane = reinterpret_cast<int*>(smem + KEYS);  // S2 (phase B) / V (phase A), [16][BMV_NP]
  int* plane2 = reinterpret_cast<int*>(smem + KEYS + BMV_PLANE);  // R = 2: hb-row sums
  uint8_t* crec = smem + KEYS;                                    // until the A fragments are built
  uint8_t* win = smem + KEYS + (R == 2 ? 2 : 1) * BMV_PLANE;

  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wave >> 2, wl = wave & 3;  // the wave's row in the workgroup, its place in the row
  const int n = lane & 15, h = lane >> 4;
  const int S = p.range, W = p.width, H = p.height;
  int lin;
  {  // XCD-banded: XCD x walks one contiguous run of strips
    const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
    const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
    lin = x * q + min(x, rem) + m;
  }
  {  // batched launch: jobs are consecutive runs of jb.wgs workgroups
    const int j = lin / jb.wgs;
    lin -= j * jb.wgs;
    mfma_job(jb, j, p, g);
  }
  const int grp = lin / g.bm_wpr, sx = lin - grp * g.bm_wpr;
  const int br0 = g.row0 + R * grp;
  const int nrw = min(R, g.row0 + g.nrows - br0);  // rows present (1 or R)
  const int bc0 = 8 * sx, nb = min(8, g.nbx - bc0);
  auto row_bh = [&](int r) { return br0 + r == g.hb_row ? g.hb : 16; };
  auto row_ylo = [&](int r) { return max(16 * (br0 + r) - S, 0); };
  auto row_yhi = [&](int r) { return min(16 * (br0 + r) + S, H - row_bh(r)); };
  const int ylo = row_ylo(0);
  const int yhi_w = row_yhi(nrw - 1) > row_yhi(0) ? row_yhi(nrw - 1) : row_yhi(0);
  const int T = (yhi_w - ylo + 16) >> 4;  // workgroup bands
  // S2 planes: plane for row 0's block height, plane2 for row 1's when it differs
  const int bh0 = row_bh(0);
  const bool two = R == 2 && nrw == 2 && row_bh(1) != bh0;
  const int tc0 = max(16 * bc0 - S, 0) >> 4;
  const int npos = 16 * ((min(16 * (bc0 + nb - 1) + S, W - 16) >> 4) - tc0 + 1);
  const int npv = npos + 12;
  auto band_y = [&](int s) { return ylo + 16 * s; };
  const __amdgpu_buffer_rsrc_t rref =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ref, (short)0, p.ref_bytes, 0x00020000);
  auto stage_band = [&](int s) {
    const int gbase = (band_y(s) - p.ref_row0) * p.stride + 16 * tc0;
    const int lane16 = opaque(tid);
    for (int s0 = (lane16 >> 6) * 1024; s0 < WINB; s0 += NT * 16) {
      const int d = s0 + 16 * (lane16 & 63);
      if (d < WINB) {
        const int rho = d / LP, k = d - rho * LP;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rref, (__attribute__((address_space(3))) void*)(win + (s & 1) * WINB + s0), 16,
            (uint32_t)(gbase + rho * p.stride + k), 0, 0, 0);
      }
    }
  };
  // S2 of band s (its window has landed in buffer s & 1; everyone is past the
  // previous band's tiles): V, then S2 in place, and the window XOR-ed for the MFMAs.
  auto band_s2 = [&](int s) {
    uint8_t* wb = win + (s & 1) * WINB;
#pragma unroll 1
    for (int pp = tid; pp < npv; pp += NT) {
      if (bh0 == 16) bmv_vsum16<LP>(wb, pp, plane + pp);
      else bmv_vsum_hb<LP>(wb, pp, bh0, plane + pp);
      if (two) bmv_vsum_hb<LP>(wb, pp, row_bh(1), plane2 + pp);
    }
    __syncthreads();
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr int QB = 64;            // 4-position groups per plane row (256 positions)
    constexpr int TPL = 1024 / NT;    // tasks per lane: 16 rows x 64 groups
    i32x4 o[TPL], o2[TPL];
    const int nq = npos >> 2;
#pragma unroll
    for (int t = 0; t < TPL; t++) {
      const int task = tid + NT * t, k = task / QB, q = task - k * QB;
      if (q < nq) {
        const i32x4* vr = reinterpret_cast<const i32x4*>(plane + k * BMV_NP + 4 * q);
        o[t] = vr[0] + vr[1] + vr[2] + vr[3];
        if (two) {
          const i32x4* v2 = reinterpret_cast<const i32x4*>(plane2 + k * BMV_NP + 4 * q);
          o2[t] = v2[0] + v2[1] + v2[2] + v2[3];
        }
      }
    }
    // the window's bytes become r' = r ^ 0x80 (the MFMA B operand)
    for (int d = tid; d < WINB / 16; d += NT) {
      u32x4* w4 = reinterpret_cast<u32x4*>(wb) + d;
      *w4 = *w4 ^ 0x80808080u;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TPL; t++) {
      const int task = tid + NT * t, k = task / QB, q = task - k * QB;
      if (q < nq) {
        *reinterpret_cast<i32x4*>(plane + k * BMV_NP + 4 * q) = o[t];
        if (two) *reinterpret_cast<i32x4*>(plane2 + k * BMV_NP + 4 * q) = o2[t];
      }
    }
    __syncthreads();
  };

  MS_STAMP(0, __builtin_amdgcn_s_memtime());
  MS_STAMP(6, __builtin_amdgcn_s_memrealtime());
  if (tid < 8 * R) {
    keys[tid] = ~0ull;
    cc[tid] = 0;
  }
  stage_band(0);
  __syncthreads();  // keys / cc initialised
  if (tid < 128 * R) {  // cur row records (c ^ 0x7F) and Cc = sum(c''^2 + 2 c'')
    const int jj = tid >> 4, rho = tid & 15, r = jj >> 3, j = jj & 7;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < nrw && j < nb && rho < row_bh(r)) {
      const u32x4* src = reinterpret_cast<const u32x4*>(
          p.cur + (ptrdiff_t)(16 * (br0 + r) + rho - p.cur_row0) * p.stride + 16 * (bc0 + j));
      v = *src ^ 0x7F7F7F7Fu;
    }
    const u32x4 z = {0u, 0u, 0u, 0u};
    u32x4* rec = reinterpret_cast<u32x4*>(crec + (16 * jj + rho) * BM_CREC);
    rec[0] = z;
    rec[1] = v;
    rec[2] = z;
    int part = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      part = __builtin_amdgcn_sdot4((int)v[e], (int)v[e], part, false);
      part = __builtin_amdgcn_sdot4((int)v[e], 0x02020202, part, false);
    }
    if (r < nrw && j < nb) atomicAdd(&cc[jj], part);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const bool rowok = rw < nrw;
  const int br = br0 + rw, by = 16 * br;
  const int rylo = rowok ? row_ylo(rw) : 0, ryhi = rowok ? row_yhi(rw) : -1;
  const int j0 = 2 * wl, j1 = j0 + 1;
  const bool hasA = rowok && j0 < nb, hasB = rowok && j1 < nb;
  const int bxA = 16 * (bc0 + j0), bxB = bxA + 16;
  const int xloA = max(bxA - S, 0), xhiA = min(bxA + S, W - 16);
  const int xloB = max(bxB - S, 0), xhiB = min(bxB + S, W - 16);
  const int i0A = xloA >> 4, i1A = xhiA >> 4, i0B = xloB >> 4, i1B = xhiB >> 4;
  const int iu0 = i0A, iu1 = hasB ? i1B : i1A;

  v4i aA[8], aB[8];
  {
    const int o = 16 + 16 * (h & 1) - n, sh = o & 3;
    typedef __attribute__((address_space(3))) const uint32_t lds_c32;
    const uint32_t lb = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)crec) +
                        (uint32_t)((h >> 1) * BM_CREC + (o & ~3));
#pragma unroll
    for (int q = 0; q < 8; q++) {
#pragma unroll
      for (int bsel = 0; bsel < 2; bsel++) {
        const uint32_t a0 = lb + (uint32_t)(((8 * rw + 2 * wl + bsel) * 16 + 2 * q) * BM_CREC);
        uint32_t d[5];
#pragma unroll
        for (int e = 0; e < 5; e++) d[e] = *reinterpret_cast<lds_c32*>((uintptr_t)(a0 + 4 * e));
        v4i f;
#pragma unroll
        for (int e = 0; e < 4; e++) f[e] = (int)__builtin_amdgcn_alignbyte(d[e + 1], d[e], sh);
        if (bsel == 0) aA[q] = f; else aB[q] = f;
      }
    }
  }
  MS_STAMP(1, __builtin_amdgcn_s_memtime());
  __syncthreads();  // crec read by every wave: the plane is free for band 0's S2
  band_s2(0);
  uint32_t mbits = 0;
  {
    auto xmask = [&](int e, int i, int xlo, int xhi) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int x = 16 * i + 4 * h + r;
        if (x < xlo || x > xhi) mbits |= 1u << (4 * e + r);
      }
    };
    xmask(0, i0A, xloA, xhiA);
    xmask(1, i1A, xloA, xhiA);
    xmask(2, i0B, xloB, xhiB);
    xmask(3, i1B, xloB, xhiB);
  }
  // interior pair in x: the mask-free tile sequence (y masks per band below)
  const bool fastx = hasB && bxA - S >= 0 && bxB + S <= W - 16 && i1A - i0A >= 2;
  const int mfa = (bxA - S) & 15, mlb = (bxA + S) & 15;
  int* splane = (two && rw == 1) ? plane2 : plane;
  const uint32_t s2base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) int*)splane) +
                          (uint32_t)((n * BMV_NP + 4 * h - 16 * tc0) * 4);
  const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)win) +
                         (uint32_t)((n + (h >> 1)) * LP + 16 * (h & 1) - 16 * tc0);
  typedef __attribute__((address_space(3))) const v4i lds_v4i;
  const v4i zero4 = {0, 0, 0, 0};

  unsigned long long bestA = ~0ull, bestB = ~0ull;
  for (int s = 0; s < T; s++) {
    if (s + 1 < T) stage_band(s + 1);
    const int Ys = band_y(s);
    if (hasA && Ys <= ryhi && Ys + 15 >= rylo) {
      // rows of the band outside this block row's range: bit 31 of the key
      const int yn = Ys + n;
      const uint32_t ym = (yn < rylo || yn > ryhi) ? 0x80000000u : 0u;
      const bool yfull = Ys >= rylo && Ys + 15 <= ryhi;
      const uint32_t lrow0 = lbase + (uint32_t)((s & 1) * WINB);
      uint32_t bA = ~0u, bB = ~0u;
      v4i mF, mL;
      const int h4b = opaque(4 * h);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int m = h4b + r;
        mF[r] = m < mfa ? (1 << 24) : 0;
        mL[r] = m > mlb ? (1 << 24) : 0;
      }
      auto widen = [&](int seg) {
        const uint32_t lo = ((uint32_t)s << 8) | ((uint32_t)seg << 6);
        const unsigned long long kA = ((unsigned long long)(bA >> 6) << 32) | lo | (bA & 63u);
        const unsigned long long kB = ((unsigned long long)(bB >> 6) << 32) | lo | (bB & 63u);
        bestA = (kA >> 32) < (bestA >> 32) ? kA : bestA;
        bestB = (kB >> 32) < (bestB >> 32) ? kB : bestB;
        bA = ~0u;
        bB = ~0u;
      };
      auto tile = [&](int i, auto DA, auto DB, auto MA, auto MB, auto YM) {
        constexpr bool da = decltype(DA)::value, db = decltype(DB)::value;
        constexpr int ma = decltype(MA)::value, mb = decltype(MB)::value;
        constexpr bool ymask = decltype(YM)::value;
        const v4i s2c = *reinterpret_cast<lds_v4i*>((uintptr_t)(s2base + (uint32_t)(64 * i)));
        const uint32_t lrow = (uint32_t)opaque((int)(lrow0 + (uint32_t)(16 * i)));
        v4i accA = ma == 1 ? mF : ma == 2 ? mL : zero4;
        v4i accB = mb == 1 ? mF : mb == 2 ? mL : zero4;
        auto ld = [&](int q) {
          return *reinterpret_cast<lds_v4i*>((uintptr_t)(lrow + (uint32_t)(2 * q * LP)));
        };
        v4i f0 = ld(0), f1 = ld(1);
#pragma unroll
        for (int qp = 0; qp < 4; qp++) {
          v4i n0 = f0, n1 = f1;
          if (qp < 3) {
            n0 = ld(2 * qp + 2);
            n1 = ld(2 * qp + 3);
          }
          if constexpr (da) accA = MFMA16(aA[2 * qp], f0, accA, 0, 0, 0);
          if constexpr (db) accB = MFMA16(aB[2 * qp], f0, accB, 0, 0, 0);
          if constexpr (da) accA = MFMA16(aA[2 * qp + 1], f1, accA, 0, 0, 0);
          if constexpr (db) accB = MFMA16(aB[2 * qp + 1], f1, accB, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          f0 = n0;
          f1 = n1;
        }
        // key = ((2 acc + S2 + 1 + 2^23) << 6) + 4 ((i - iu0) & 15) + r
        const int rel = i - iu0;
        const uint32_t kb = (1u << 29) + 64u + 4u * (uint32_t)(rel & 15);
        uint32_t P[4];
#pragma unroll
        for (int r = 0; r < 4; r++) P[r] = lshl6_add((uint32_t)s2c[r], kb + (uint32_t)r);
        auto keys_of = [&](v4i acc, uint32_t& best, int i0, int i1, int e0, auto GEN) {
          if constexpr (decltype(GEN)::value) {
            if (i == i0 || i == i1) {
              const int e = i == i0 ? e0 : e0 + 1;
              const uint32_t mb4 = (uint32_t)opaque((int)mbits);
#pragma unroll
              for (int r = 0; r < 4; r++)
                acc[r] += (int)(__builtin_amdgcn_ubfe(mb4, (uint32_t)(4 * e + r), 1u) << 24);
            }
          }
          uint32_t k[4];
#pragma unroll
          for (int r = 0; r < 4; r++) k[r] = ((uint32_t)acc[r] << 7) + P[r];
          if constexpr (ymask) {
#pragma unroll
            for (int r = 0; r < 4; r++) k[r] |= ym;
          }
          best = umin3(best, k[0], k[1]);
          best = umin3(best, k[2], k[3]);
        };
        if constexpr (da) keys_of(accA, bA, i0A, i1A, 0, std::integral_constant<bool, ma == 3>{});
        if constexpr (db) keys_of(accB, bB, i0B, i1B, 2, std::integral_constant<bool, mb == 3>{});
        if ((rel & 15) == 15 && i < iu1) widen(rel >> 4);
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      using M0 = std::integral_constant<int, 0>;
      using M1 = std::integral_constant<int, 1>;
      using M2 = std::integral_constant<int, 2>;
      using M3 = std::integral_constant<int, 3>;
      auto seq = [&](auto YM) {
        if (fastx) {
          tile(i0A, T_{}, F_{}, M1{}, M0{}, YM);
          tile(i0A + 1, T_{}, T_{}, M0{}, M1{}, YM);
          for (int i = i0A + 2; i < i1A; i++) tile(i, T_{}, T_{}, M0{}, M0{}, YM);
          tile(i1A, T_{}, T_{}, M2{}, M0{}, YM);
          tile(i1B, F_{}, T_{}, M0{}, M2{}, YM);
        } else {
          for (int i = iu0; i <= iu1; i++) {
            const bool useA = i <= i1A, useB = hasB && i >= i0B;
            if (useA && useB) tile(i, T_{}, T_{}, M3{}, M3{}, T_{});
            else if (useA) tile(i, T_{}, F_{}, M3{}, M3{}, T_{});
            else tile(i, F_{}, T_{}, M3{}, M3{}, T_{});
          }
        }
      };
      if (yfull) seq(F_{});
      else seq(T_{});
      widen((iu1 - iu0) >> 4);
    }
    if (s == 0) MS_STAMP(2, __builtin_amdgcn_s_memtime());
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // band s + 1 landed (this thread's pieces)
    __syncthreads();                                   // ... and everyone's; band s and its S2 free
    if (s + 1 < T) band_s2(s + 1);
  }
  if (hasA) {
    auto emit = [&](unsigned long long b, int j, int bx) {
      const uint32_t hi = (uint32_t)(b >> 32);
      if (hi < (1u << 25)) {
        const uint32_t lo = (uint32_t)b;
        const int sb = (int)(lo >> 8), seg = (int)((lo >> 6) & 3u), idx = (int)(lo & 63u);
        const uint32_t cost = hi - 1u - (1u << 23) + (uint32_t)cc[8 * rw + j];
        const int dx = 16 * (iu0 + 16 * seg + (idx >> 2)) + 4 * h + (idx & 3) - bx;
        const int dy = band_y(sb) + n - by;
        const unsigned long long key = ((unsigned long long)cost << 32) |
                                       ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
        const uint32_t a = (uint32_t)(uintptr_t)(
            (__attribute__((address_space(3))) unsigned long long*)(keys + 8 * rw + j));
        asm volatile("ds_min_u64 %0, %1" : : "v"(a), "v"(key) : "memory");
      }
    };
    emit(bestA, j0, bxA);
    if (hasB) emit(bestB, j1, bxB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();
#ifdef ME_STAMPS
  if (tid == 0 && blockIdx.x < (1u << 14)) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_mstamps[8 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    g_mstamps[8 * blockIdx.x + 4] = hw;
    g_mstamps[8 * blockIdx.x + 5] = xcc;
    g_mstamps[8 * blockIdx.x + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (tid < 8 * R) {
    const int r = tid >> 3, j = tid & 7;
    if (r < nrw && j < nb) {
      const unsigned long long kk = keys[tid];
      const int out = (br0 + r - p.block_row_begin) * p.nbx + bc0 + j;
      store_mv(p.mv, out, kk);
      if (p.cost) p.cost[out] = (uint32_t)(kk >> 32);
    }
  }
}

}  // namespace

// Process-wide path switch (me_set_kernel_path / ME_PATH, me_tuning.h).
bool mfma_disabled() { return kernel_path() == 1; }

// Tiles of a B = 16 search over block rows [begin, end) (the merge buffers' size).
size_t mfma_merge_tiles(const SearchArgs& p) {
  if (p.blk != 16 || p.width < p.blk) return 0;  // 8x8: no cross-workgroup merge
  const size_t tx = (size_t)((p.width / p.blk + 3) / 4);
  const size_t ty = (size_t)((p.block_row_end - p.block_row_begin + 3) / 4);
  return tx * ty;
}

// Scratch bytes the MFMA path needs for this search (0: path not applicable).
size_t mfma_ssd_scratch(const SearchArgs& p) {
  MfmaGeom g;
  return plan_mfma_ssd(p, &g) ? g.scratch_bytes : 0;
}

// Full-height block rows [row0, row0 + nrows) and full-width columns of a B = 16
// SSD search; the caller routes partial rows / columns to the VALU kernels.
static bool plan_mfma_ssd8(const SearchArgs& p, MfmaGeom* g);

// Block-major (me_mfma_bm16_kernel) or 4x4-block tiles (me_mfma_ssd16_kernel)?
// Block-major measured faster at every S (1080p, S = 2..103: tools/dbg/bm_sweep*.sh);
// the tile kernel remains for row pitches / cur pointers that are not 16-byte aligned.
static bool bm_auto(const SearchArgs& p) { return p.range <= 192; }

// The automatic path's choice for `jobs` frames of p's shape per launch:
// the band-walk kernel (lean: no prepass planes, ~1.0-1.3x the algorithmic
// HBM bytes against ~7x) when its plan runs in one round of workgroups or
// without splitting block rows into segments (each segment re-forms
// 2 ceil(S/16) bands around it).  A single 1080p frame is 8 segments of 9
// rows in one round: 37.5 against 37.8-38.8 us per call on the prepass pair;
// 4K +-64 (2 segments of 68 rows): 265.9 against 254 us, the price of ~18
// against ~122 MB of HBM traffic per search (profiles/r06h_ssd_ab.jsonl, one
// box).  The round-5 figure of 68.8 us was the partial bottom row's second
// launch, now searched inside the walk.
// ME_PATH_MFMA_LEAN (force) takes the band-walk kernel whenever it applies.
// g holds the block-major plan on entry and the band-walk plan on success.
static bool use_bw(const SearchArgs& p, MfmaGeom* g, int jobs, bool force = false) {
  if (!g->bm) return false;
  MfmaGeom t = *g;
  t.bmv = 0;
  if (!plan_bw(p, &t, jobs) || (!force && t.bw_segs != 1 && !bw_one_round(t, jobs))) return false;
  *g = t;
  g->bmv_r = 1;
  g->scratch_bytes = 0;
  g->rp = nullptr;
  g->s2 = g->s2h = nullptr;
  return true;
}

bool plan_mfma_ssd(const SearchArgs& p, MfmaGeom* g) {
  if (p.cost_kind != COST_SSD) return false;
  if (p.blk == 8) return plan_mfma_ssd8(p, g);
  if (p.blk != 16) return false;
  if (mfma_disabled()) return false;
  const int S = p.range, W = p.width, H = p.height;
  if (S < 1 || W < 16 || H < 16) return false;
  if (p.stride % 4 || (uintptr_t)p.cur % 4 || (uintptr_t)p.ref % 4) return false;
  // block-major kernel for S <= 192 (ME_MFMA_BM=0|1: tuning build override)
  const int force_bm = tuning().mfma_bm;
  g->bm = S <= 192 && kernel_path() != 2 && (force_bm == 1 || (force_bm == 2 && bm_auto(p)));
  // window row pitch: a workgroup's 8 blocks span 16 (tc1 - tc0) + 32 <= 16 (S / 8 + 8) + 32
  // bytes (<= 544 up to S = 192)
  g->bm_lp = S <= 64 ? 288 : 544;
  if (g->bm && (p.stride % 16 || (uintptr_t)p.cur % 16)) g->bm = 0;  // 16-byte cur row loads
  const int nxmax = min(48 + 2 * S + 1, W - 15);
  const int ngx = (nxmax + 63) / 64;
  if (ngx > 4 && !g->bm) return false;  // S > 103: the VALU kernels take it
  const int nby = (H + 15) / 16;
  const int r0 = p.block_row_begin, r1 = p.block_row_end;
  g->row0 = r0;
  g->nrows = r1 - r0;
  if (g->nrows <= 0) return false;
  // partial bottom block row (height hb): its lanes read the hb-row S2 plane
  g->hb = H - 16 * (nby - 1);
  g->hb_row = (g->hb < 16 && r1 == nby) ? nby - 1 : -1;
  if (g->hb_row < 0) g->hb = 16;
  g->nbx = W / 16;
  g->tiles_x = (g->nbx + 3) / 4;
  g->tiles_y = (g->nrows + 3) / 4;
  g->ngx = ngx;
  // chunk rows L = P0 + 16 KM: fewest (chunks x (L + P0)) steps on an interior tile
  const int ny = min(48 + 2 * S + 1, H - 15);
  int best = 1 << 30;
  const int force_km = tuning().mfma_km;  // ME_MFMA_KM=2|3: tuning build override
  for (int km = 2; km <= 3; km++) {  // km = 1 spills (its lone main-loop pass gets peeled)
    if (force_km && km != force_km) continue;
    const int L = 12 + MFMA_DLY + 16 * km, ch = (ny + L - 1) / L;
    const int cost = ch * (L + 12 + MFMA_DLY);
    if (cost < best) { best = cost; g->km = km; }
  }
  const int L = 12 + MFMA_DLY + 16 * g->km;
  // groups per workgroup: two when the tile needs an even number of groups
  // (whole tiles at 1080p +-32: no merge), else one (4K +-64: 3 workgroups)
  g->ngxw = ngx % 2 == 0 ? 2 : 1;
  if (tuning().mfma_ngxw) g->ngxw = tuning().mfma_ngxw;  // ME_MFMA_NGXW: tuning build
  if (!g->bm && (ngx + g->ngxw - 1) / g->ngxw > 1 &&
      (!p.mkeys || !p.mcnt || p.merge_tiles < mfma_merge_tiles(p)))
    return false;  // tiles span workgroups: needs the merge buffers
  g->lds = 4 * (L + 15) * (64 * g->ngxw + 32) + 16 * 8 + 16 * 4 + L * 256 * g->ngxw;
  g->bm_wpr = (g->nbx + 7) / 8;
  if (g->bm) g->lds = BM_HDR + 2 * 31 * g->bm_lp;
  // ME_PATH_MFMA_LEAN, S <= 64 (window pitch 288): S2 formed in the workgroup,
  // no prepass planes (ME_MFMA_S2K=0|1 overrides; tuning build)
  const int s2k = tuning().mfma_s2k >= 0 ? tuning().mfma_s2k : kernel_path() == 3;
  g->bmv = g->bm && g->bm_lp == BMV_LP && s2k;
  // block rows per workgroup (ME_MFMA_S2R=1|2 overrides; tuning build).  Two
  // rows share each band's S2 (6 bands for two rows at S = 32 instead of
  // 5 + 5; 10 instead of 9 + 9 at S = 64) but synchronise 8 waves per barrier
  // and leave a row idle in the other row's end bands: 16-frame batches, 1080p
  // +-32 35.9 us per frame against 33.8 with one row, 4K +-64 289 against 323
  // (profiles/r04f_ssd_ab.jsonl).  Two rows from S = 48 on.
  g->bmv_r = tuning().mfma_s2r > 0 ? tuning().mfma_s2r : (S >= 48 ? 2 : 1);
  if (g->bmv) g->lds = g->bmv_r == 2 ? bmv_lds<2>() : bmv_lds<1>();
  g->mkeys = p.mkeys;
  g->mcnt = p.mcnt;
  g->ya0 = max(r0 * 16 - S, 0);
  const int ya1 = min(r1 * 16 + S, H);
  g->rp_rows = ya1 - g->ya0;
  g->pitch = (W + 15) & ~15;
  // + 80 rows of slack: the last chunk of a tile reads (masked) window rows and
  // S2 entries up to L + 15 rows past the planes' last row.
  // (the block-major kernel reads at most 15 rows past them, and its buffer
  // loads are range-checked: 16 rows of slack)
  g->rows_alloc = g->rp_rows + (g->bm ? 16 : 80);
  // the last tile row's candidate rows start here (its lanes of the partial
  // block row read s2h from there on)
  const int tly_last = 16 * (r0 + 4 * (g->tiles_y - 1));
  g->s2h_row0 = max(tly_last - S, 0) - g->ya0;
  const size_t plane = (size_t)g->rows_alloc * g->pitch;
  const size_t rp_alloc = (plane + 255) & ~(size_t)255;
  const size_t s2_plane = plane * 4;
  const size_t n_s2 = g->hb < 16 ? 2 : 1;
  if (rp_alloc + n_s2 * s2_plane >= (1ull << 31)) return false;
  g->rp_bytes = (uint32_t)plane;
  g->s2_bytes = (uint32_t)(n_s2 * s2_plane);
  g->s2h_off = (uint32_t)s2_plane;
  g->scratch_bytes = rp_alloc + n_s2 * s2_plane;
  g->rp = reinterpret_cast<int8_t*>(p.scratch);
  g->s2 = p.scratch ? reinterpret_cast<int*>(p.scratch + rp_alloc) : nullptr;
  g->s2h = p.scratch ? reinterpret_cast<int*>(p.scratch + rp_alloc + s2_plane) : nullptr;
  // Automatic path, S <= 64: the band-walk kernel (me_band.hip) for the
  // full-height rows, me_mfma_bmv_kernel for a partial bottom row, neither
  // with scratch, when the frame's strips fill the CUs by themselves
  // (use_bw); ME_PATH_MFMA_PREPASS keeps the prepass + block-major pair.
  g->bw = 0;
  if (kernel_path() == 0 || kernel_path() == 3) use_bw(p, g, 1, kernel_path() == 3);
  if (g->bmv) {  // no planes: the kernel reads the reference plane
    g->scratch_bytes = 0;
    g->rp = nullptr;
    g->s2 = g->s2h = nullptr;
  }
  return true;
}

// 8x8 blocks: full-height block rows only (a partial bottom row goes to the
// VALU kernels), one workgroup per 4x4-block tile walking its 64-column groups,
// chunks of 16 ME_SSD8_KM rows.
static bool plan_mfma_ssd8(const SearchArgs& p, MfmaGeom* g) {
  if (mfma_disabled()) return false;
  const int S = p.range, W = p.width, H = p.height;
  if (S < 1 || W < 8 || H < 8) return false;
  if (p.stride % 4 || (uintptr_t)p.cur % 4 || (uintptr_t)p.ref % 4) return false;
  const int nby = (H + 7) / 8;
  const int r0 = p.block_row_begin;
  int r1 = p.block_row_end;
  if (r1 == nby && H % 8) r1--;
  g->row0 = r0;
  g->nrows = r1 - r0;
  if (g->nrows <= 0) return false;
  g->hb = 8;
  g->hb_row = -1;
  g->bm = 0;
  g->bmv = 0;
  g->bmv_r = 1;
  g->bw = 0;
  g->nbx = W / 8;
  g->tiles_x = (g->nbx + 3) / 4;
  g->tiles_y = (g->nrows + 3) / 4;
  const int nxmax = min(24 + 2 * S + 1, W - 7);
  g->ngx = (nxmax + 63) / 64;
  g->ngxw = g->ngx;  // one workgroup walks all of a tile's groups
  g->km = ME_SSD8_KM;  // L = 16 km candidate rows per chunk
  const int L = 16 * g->km;
  // 4 copies + keys + S2 table + the words after each copy granule: 31.9 KB (two tiles), 5 workgroups per CU
  g->lds = 4 * (L + 8) * ME_SSD8_WP + 16 * ME_SSD8_NT * 12 + (L + 1) * 256 + (L + 8) * (ME_SSD8_WP / 16) * 4;
  g->ya0 = max(r0 * 8 - S, 0);
  const int ya1 = min(r1 * 8 + S, H);
  g->rp_rows = ya1 - g->ya0;
  g->pitch = (W + 15) & ~15;
  g->rows_alloc = g->rp_rows + 80;
  g->s2h_row0 = 0;
  // S2 plane only: the kernel stages the reference rows itself (no r ^ 0x80 plane)
  const size_t plane = (size_t)g->rows_alloc * g->pitch;
  const size_t s2_plane = plane * 4;
  if (s2_plane >= (1ull << 31)) return false;
  g->rp_bytes = 0;
  g->s2_bytes = (uint32_t)s2_plane;
  g->s2h_off = 0;
  g->scratch_bytes = s2_plane;
  g->rp = nullptr;
  g->s2 = p.scratch ? reinterpret_cast<int*>(p.scratch) : nullptr;
  g->s2h = nullptr;
  g->mkeys = p.mkeys;
  g->mcnt = p.mcnt;
  return true;
}

// Main-kernel workgroups per job: a block row each, or R rows each on the
// lean path (me_mfma_bmv_kernel<R>).
static int wgs_per_job(const MfmaGeom& g) {
  return g.bmv ? (g.nrows + g.bmv_r - 1) / g.bmv_r * g.bm_wpr : g.nrows * g.bm_wpr;
}

// The one-job table of a single search (its own pointers, its own scratch).
static MfmaJobs single_job(const SearchArgs& p, const MfmaGeom& g) {
  MfmaJobs jb;
  jb.n = 1;
  jb.wgs = wgs_per_job(g);
  jb.scratch_stride = 0;
  jb.ref[0] = p.ref;
  jb.cur[0] = p.cur;
  jb.mv[0] = p.mv;
  jb.cost[0] = p.cost;
  return jb;
}

// Prepass over every job of the table (grid z = job).
static hipError_t launch_prep(const SearchArgs& p, const MfmaGeom& g, const MfmaJobs& jb,
                              hipStream_t stream) {
  const int nmain = (g.rows_alloc + 63) / 64;
  const int nh = g.hb_row >= 0 ? (g.rows_alloc - g.s2h_row0 + 63) / 64 : 0;
  dim3 pgrid((unsigned)((g.pitch + 63) / 64), (unsigned)(nmain + nh), (unsigned)jb.n);
  if (p.blk == 8)
    hipLaunchKernelGGL(me_ssd_prep_kernel<8>, pgrid, dim3(PREP_T), 0, stream, p, g, jb);
  else
    hipLaunchKernelGGL(me_ssd_prep_kernel<16>, pgrid, dim3(PREP_T), 0, stream, p, g, jb);
  return hipGetLastError();
}

static hipError_t launch_bm16(const SearchArgs& p, const MfmaGeom& g, const MfmaJobs& jb,
                              hipStream_t stream) {
  const dim3 gridb((unsigned)(jb.n * jb.wgs));
  if (g.bm_lp == 288)
    hipLaunchKernelGGL(me_mfma_bm16_kernel<288>, gridb, dim3(256), g.lds, stream, p, g, jb);
  else
    hipLaunchKernelGGL(me_mfma_bm16_kernel<544>, gridb, dim3(256), g.lds, stream, p, g, jb);
  return hipGetLastError();
}

static hipError_t launch_bmv(const SearchArgs& p, const MfmaGeom& g, const MfmaJobs& jb,
                             hipStream_t stream) {
  if (g.bmv_r == 2)
    hipLaunchKernelGGL(me_mfma_bmv_kernel<2>, dim3((unsigned)(jb.n * jb.wgs)), dim3(512), g.lds,
                       stream, p, g, jb);
  else
    hipLaunchKernelGGL(me_mfma_bmv_kernel<1>, dim3((unsigned)(jb.n * jb.wgs)), dim3(256), g.lds,
                       stream, p, g, jb);
  return hipGetLastError();
}

// The band-walk kernel over the full-height rows of every job of jb, then
// me_mfma_bmv_kernel over their partial bottom row (if any).
static hipError_t launch_bw_jobs(const SearchArgs& p, const MfmaGeom& g, const MfmaJobs& jb,
                                 hipStream_t stream) {
  hipError_t e = launch_bw(p, g, jb, stream);
  if (e != hipSuccess || g.hb_row < 0 || g.bw_hb > 0) return e;  // (bw_hb: the row ran in the walk)
  MfmaGeom t = g;
  t.bw = 0;
  t.bmv = 1;
  t.bmv_r = 1;
  t.row0 = g.hb_row;
  t.nrows = 1;
  t.lds = bmv_lds<1>();
  MfmaJobs tj = jb;
  tj.wgs = wgs_per_job(t);
  return launch_bmv(p, t, tj, stream);
}

static int mfma_path(const SearchArgs& p, const MfmaGeom& g) {
  return g.bw ? 3 : g.bmv ? 4 : p.blk == 8 ? 6 : g.bm ? 2 : 5;
}

hipError_t launch_mfma_ssd(const SearchArgs& p, const MfmaGeom& g, hipStream_t stream) {
  note_path(mfma_path(p, g));
  const MfmaJobs jb = single_job(p, g);
  if (g.bw) return launch_bw_jobs(p, g, jb, stream);
  if (g.bmv) return launch_bmv(p, g, jb, stream);
  hipError_t e = launch_prep(p, g, jb, stream);
  if (e != hipSuccess) return e;
  if (p.blk == 8) {
    const dim3 grid8((unsigned)((g.tiles_x + ME_SSD8_NT - 1) / ME_SSD8_NT * g.tiles_y));
    e = lds_attr((const void*)me_mfma_ssd8_kernel<ME_SSD8_KM>, g.lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(me_mfma_ssd8_kernel<ME_SSD8_KM>, grid8, dim3(256), g.lds, stream, p, g);
    return hipGetLastError();
  }
  if (g.bm) return launch_bm16(p, g, jb, stream);
  const int wpt = (g.ngx + g.ngxw - 1) / g.ngxw;
  const dim3 grid((unsigned)(g.tiles_x * g.tiles_y * wpt));
#define ME_MFMA_CASE(NG, KK)                                                              \
  if (g.ngxw == NG && g.km == KK) {                                                       \
    e = lds_attr((const void*)me_mfma_ssd16_kernel<NG, KK>, g.lds);                        \
    if (e != hipSuccess) return e;                                                        \
    hipLaunchKernelGGL((me_mfma_ssd16_kernel<NG, KK>), grid, dim3(256 * NG), g.lds, stream, p, g); \
    return hipGetLastError();                                                             \
  }
  ME_MFMA_CASE(1, 2) ME_MFMA_CASE(1, 3) ME_MFMA_CASE(2, 2) ME_MFMA_CASE(2, 3)
#undef ME_MFMA_CASE
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------------ batches
// A batch of frames with one geometry shares one prepass launch and one
// block-major launch: a 1080p search is one round of workgroups per CU, so a
// launch per frame pays the grid's fill and drain every frame.
static constexpr size_t MFMA_BATCH_SCRATCH = (size_t)1 << 30;  // prepass planes per launch

static size_t batch_stride(const MfmaGeom& g) { return (g.scratch_bytes + 255) & ~(size_t)255; }

// Jobs per batched launch for this geometry: 0 when the batch path does not
// apply (not the block-major kernel, or one job's planes alone exceed the cap).
static int batch_jobs(const MfmaGeom& g, int n) {
  if (!g.bm || n < 2) return 0;
  if (g.bmv || g.bw) return n < MAX_JOBS ? n : MAX_JOBS;  // no prepass planes
  const size_t per = MFMA_BATCH_SCRATCH / batch_stride(g);
  const int m = (int)(per < (size_t)MAX_JOBS ? per : (size_t)MAX_JOBS);
  return m >= 2 ? (n < m ? n : m) : 0;
}

size_t mfma_batch_scratch(const SearchArgs& p, int n) {
  MfmaGeom g;
  if (!plan_mfma_ssd(p, &g) || g.bmv || g.bw) return 0;
  // launch_mfma_jobs runs the batch job by job, each on its own single-frame
  // plan, when a job has a partial right column or its planes are not
  // aligned like job 0's: the scratch then has to hold one job's prepass
  // planes (a batch that fell back with none ran on the VALU kernels)
  const size_t one = g.scratch_bytes;
  if (g.nbx < p.nbx) return one;
  if (n >= 2 && kernel_path() == 0 && tuning().mfma_batch != 0 && use_bw(p, &g, n < MAX_JOBS ? n : MAX_JOBS))
    return one;  // the batch runs on the band-walk kernel (no planes) unless it falls back
  const int m = batch_jobs(g, n);
  return m ? ((size_t)m * batch_stride(g) > one ? (size_t)m * batch_stride(g) : one) : one;
}

bool launch_mfma_jobs(const SearchArgs& base, const SearchJob* jobs, int n, hipStream_t stream,
                      hipError_t* err) {
  *err = hipSuccess;
  if (base.cost_kind != COST_SSD || n < 2 || tuning().mfma_batch == 0) return false;
  for (int i = 1; i < n; i++)  // one geometry: the same rows of same-sized frames
    if (jobs[i].r0 != jobs[0].r0 || jobs[i].r1 != jobs[0].r1 ||
        jobs[i].ref_row0 != jobs[0].ref_row0 || jobs[i].cur_row0 != jobs[0].cur_row0)
      return false;
  SearchArgs p = base;
  p.ref = jobs[0].ref;
  p.ref_row0 = jobs[0].ref_row0;
  p.cur = jobs[0].cur;
  p.cur_row0 = jobs[0].cur_row0;
  p.block_row_begin = jobs[0].r0;
  p.block_row_end = jobs[0].r1;
  p.mv = jobs[0].mv;
  p.cost = jobs[0].cost;
  MfmaGeom g;
  if (jobs[0].r1 <= jobs[0].r0 || !plan_mfma_ssd(p, &g)) return false;
  // plan_mfma_ssd saw job 0's pointers only: every job's planes must meet the
  // same alignment (4-byte DMA sources; the block-major kernel's 16-byte cur
  // row loads), else the batch runs job by job, each planned on its own
  for (int i = 1; i < n; i++)
    if ((uintptr_t)jobs[i].ref % 4 || (uintptr_t)jobs[i].cur % (g.bm ? 16 : 4)) return false;
  // a launch of several frames may fill the CUs where one frame does not
  if (!g.bw && kernel_path() == 0) use_bw(p, &g, n < MAX_JOBS ? n : MAX_JOBS);
  const bool lean = g.bmv || g.bw;  // no prepass planes
  const size_t stride = lean ? 0 : batch_stride(g);
  int m = batch_jobs(g, n);
  if (!lean && (!base.scratch || (m && (size_t)m * stride > base.scratch_bytes)))
    m = base.scratch ? (int)(base.scratch_bytes / stride) : 0;
  if (g.bw) plan_bw(p, &g, m);  // segments sized for m jobs per launch
  if (m < 2 || g.nbx < p.nbx) return false;  // (a partial right column: job by job)
  note_path(mfma_path(p, g));
  for (int i0 = 0; i0 < n && *err == hipSuccess; i0 += m) {
    MfmaJobs jb;
    jb.n = n - i0 < m ? n - i0 : m;
    jb.wgs = wgs_per_job(g);
    jb.scratch_stride = stride;
    for (int j = 0; j < jb.n; j++) {
      const SearchJob& J = jobs[i0 + j];
      jb.ref[j] = J.ref;
      jb.cur[j] = J.cur;
      jb.mv[j] = J.mv;
      jb.cost[j] = J.cost;
    }
    if (g.bw) {
      *err = launch_bw_jobs(p, g, jb, stream);
    } else if (g.bmv) {
      *err = launch_bmv(p, g, jb, stream);
    } else {
      *err = launch_prep(p, g, jb, stream);
      if (*err == hipSuccess) *err = launch_bm16(p, g, jb, stream);
    }
  }
  return true;
}

}  // namespace me

#ifdef ME_STAMPS
extern "C" int me_debug_prep_stamps(unsigned long long* out, int n_words) {
  if (n_words > (6 << 14)) n_words = 6 << 14;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_pstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int me_debug_band_stamps(unsigned long long* out, int n_words) {
  if (n_words > (32 << 12)) n_words = 32 << 12;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_bstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int me_debug_mfma_stamps(unsigned long long* out, int n_words) {
  if (n_words > (8 << 14)) n_words = 8 << 14;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_mstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
