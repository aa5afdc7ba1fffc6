// me_kernels.hip -- CDNA4 (gfx950) full-search block-matching kernels.
//
// Semantics follow the reference CPU search exactly (souravBhat/MotionEstimation
// src/cpu/main.c:39-82): frame-clamped window (:73-76), candidates whose whole
// block fits the window (:53-54), the first minimum in raster order wins
// (:53-60, strict <).  Ties are made order-independent by reducing packed keys
//     key = cost << 32 | (dy + 32768) << 16 | (dx + 32768)
// with an unsigned min: the smallest key is the smallest cost and, among equal
// costs, the smallest (dy, dx) -- the reference's raster-first choice.
//
// Kernels (the matrix-core SSD kernels are in me_mfma.hip, SSIM in me_ssim.hip):
//   me_fast_kernel<COST, B, K, PC>
//                          SAD (qsad) or SSD (dot4), B in {8, 16}, full-width
//                          blocks.  Persistent and double-buffered: an item is
//                          (tile of TB blocks of one block row, pass of dy
//                          chunks); the union search window of the tile is
//                          staged once in LDS by LDS DMA; each SAD lane owns 4
//                          horizontal x K vertical candidates of one block and
//                          walks the window rows, 16 |a-b| per v_qsad_pk_u16_u8
//                          with the cur block held in VGPRs.
//   me_flow_kernel<B, K, PC>
//                          SAD, 16x16, S = 32 on frames with >= 2 tiles per CU
//                          (the 1080p headline): one 1,024-thread workgroup
//                          per CU, a ring of LDS slots, waves pulling 64-lane
//                          wave-tasks from one LDS counter (no item barriers).
//   me_generic_kernel      any B <= 64, any S, SSD or SAD, partial blocks; one
//                          workgroup per block, one candidate per lane.  SSD on
//                          blocks with w*h > 256 replays the reference's float
//                          accumulation (main.c:19-27) so the argmin is identical
//                          even when the float sum rounds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <type_traits>
#include <vector>

#include "me_kernels.h"
#include "me_tuning.h"


namespace me {

__device__ __forceinline__ uint64_t make_key(uint32_t cost, int dx, int dy) {
  return ((uint64_t)cost << 32) | ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
}

// Compile-time loop: every index is a constant, so register arrays indexed by
// it never fall back to scratch (plain #pragma unroll gives up on big bodies).
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ const uint8_t* row_ptr(const SearchArgs& p, const uint8_t* base,
                                                  int row0, int y) {
  return base + (ptrdiff_t)(y - row0) * p.stride;
}

// ------------------------------------------------------------------ generic
// One workgroup per block, GENERIC_THREADS lanes, one candidate per lane per
// step.  Window staged in LDS when it fits (win_lds_bytes > 0), else read from
// global memory.
template <int COST>
__global__ __launch_bounds__(GENERIC_THREADS) void me_generic_kernel(SearchArgs p, int bx0,
                                                                     int nbx_range, int row0,
                                                                     int win_lds_bytes) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[GENERIC_THREADS / 64];
  const int tid = threadIdx.x;
  const int bx = bx0 + (int)(blockIdx.x % nbx_range);
  const int by = row0 + (int)(blockIdx.x / nbx_range);
  const int B = p.blk, S = p.range;
  const int tlx = bx * B, tly = by * B;
  const int w = min(B, p.width - tlx), h = min(B, p.height - tly);
  const int wx0 = max(tlx - S, 0), wy0 = max(tly - S, 0);
  const int wx1 = min(tlx + w - 1 + S, p.width - 1), wy1 = min(tly + h - 1 + S, p.height - 1);
  const int ncx = wx1 - w + 1 - wx0 + 1, ncy = wy1 - h + 1 - wy0 + 1;
  const int ww = wx1 - wx0 + 1, wh = wy1 - wy0 + 1;

  uint8_t* cblk = smem;                       // w*h bytes
  uint8_t* win = smem + ((B * B + 15) & ~15); // ww*wh bytes when staged
  const bool staged = win_lds_bytes >= ww * wh;
  for (int i = tid; i < w * h; i += GENERIC_THREADS) {
    int oy = i / w, ox = i % w;
    cblk[i] = row_ptr(p, p.cur, p.cur_row0, tly + oy)[tlx + ox];
  }
  if (staged)
    for (int i = tid; i < ww * wh; i += GENERIC_THREADS) {
      int oy = i / ww, ox = i % ww;
      win[i] = row_ptr(p, p.ref, p.ref_row0, wy0 + oy)[wx0 + ox];
    }
  __syncthreads();

  // SSD on large blocks: key on the float MSE exactly as the reference rounds it.
  const bool float_key = (COST == COST_SSD) && (w * h > 256);
  uint64_t best = ~0ull;
  const int ncand = ncx * ncy;
  for (int t = tid; t < ncand; t += GENERIC_THREADS) {
    const int cy = t / ncx, cx = t % ncx;
    uint32_t acc = 0;
    float facc = 0.f;
    for (int oy = 0; oy < h; oy++) {
      const uint8_t* r = staged ? win + (cy + oy) * ww + cx
                                : row_ptr(p, p.ref, p.ref_row0, wy0 + cy + oy) + wx0 + cx;
      const uint8_t* c = cblk + oy * w;
      for (int ox = 0; ox < w; ox++) {
        int d = (int)c[ox] - (int)r[ox];
        if (COST == COST_SAD) {
          acc += (uint32_t)abs(d);
        } else if (float_key) {
          facc = __fadd_rn(facc, (float)(d * d));  // main.c:24, float += int
        } else {
          acc += (uint32_t)(d * d);
        }
      }
    }
    uint32_t k32 = acc;
    if (float_key) k32 = __float_as_uint(__fdiv_rn(facc, (float)(w * h)));  // main.c:27
    const int dx = wx0 + cx - tlx, dy = wy0 + cy - tly;
    uint64_t key = make_key(k32, dx, dy);
    best = key < best ? key : best;
  }
  best = wave_min_u64(best);
  if ((tid & 63) == 0) red[tid >> 6] = best;
  __syncthreads();
  if (tid == 0) {
    uint64_t b = red[0];
#pragma unroll
    for (int i = 1; i < GENERIC_THREADS / 64; i++) b = red[i] < b ? red[i] : b;
    const int dx = (int)(b & 0xFFFF) - 32768, dy = (int)((b >> 16) & 0xFFFF) - 32768;
    uint32_t cost = (uint32_t)(b >> 32);
    if (float_key) {  // report the integer SSD of the chosen vector
      cost = 0;
      for (int oy = 0; oy < h; oy++) {
        const uint8_t* r = row_ptr(p, p.ref, p.ref_row0, tly + dy + oy) + tlx + dx;
        for (int ox = 0; ox < w; ox++) {
          int d = (int)cblk[oy * w + ox] - (int)r[ox];
          cost += (uint32_t)(d * d);
        }
      }
    }
    const int out = (by - p.block_row_begin) * p.nbx + bx;
    p.mv[2 * out] = (int16_t)dx;
    p.mv[2 * out + 1] = (int16_t)dy;
    if (p.cost) p.cost[out] = cost;
  }
}

// --------------------------------------------------------------- qsad (SAD)
// Workgroup = TB consecutive full-width blocks of one block row; the union of
// their search windows is staged ONCE in LDS:
//   frame rows [Y0, Y0 + rows_alloc) x columns [X0, X0 + pitch), Y0 = tly - S,
//   X0 = tlx(b0) - S - a rounded down to a multiple of 4 (a = (tlx - S) mod 4),
//   zeros outside the frame (those candidates are masked).
// Each tile row is stored twice, the second copy shifted left by 4 bytes, so
// every 8-byte qsad operand (ref words w, w+1) is one aligned ds_read_b64 from
// one copy or the other -- gfx950 needs even-aligned VGPR pairs and unaligned
// overlapping pairs would cost a v_mov per qsad.
// Task t of the workgroup -> (dy chunk, block, dx group): the lane owns dx
// offsets q = 4g..4g+3 (dx = q - S - a) and dy offsets d = chunk*K .. +K-1
// (dy = d - S); it walks the K + H - 1 window rows once, each row feeding up
// to K accumulators (u16x4 packed, SAD <= 65280 fits) against the cur block
// held in VGPRs.
// Empty volatile asm on the accumulators row YY touched: orders that row's
// qsads before the next row's (volatile) address step.
template <int J, int K, int YY, int H>
__device__ __forceinline__ void pin_rows(uint64_t (&acc)[K]) {
  if constexpr (J < K) {
    if constexpr (YY - J >= 0 && YY - J < H) asm volatile("" : "+v"(acc[J]));
    pin_rows<J + 1, K, YY, H>(acc);
  }
}

template <int J, int K, int YY, int H>
__device__ __forceinline__ void pin_rows32(uint32_t (&acc)[K]) {
  if constexpr (J < K) {
    if constexpr (YY - J >= 0 && YY - J < H) asm volatile("" : "+v"(acc[J]));
    pin_rows32<J + 1, K, YY, H>(acc);
  }
}

// PC > 0: the pitch is that compile-time constant, and the rows of a group of
// RG share one base address (the row offset goes into the ds_read2 offset
// fields, <= 1020 bytes): one address add per group instead of per row.
// HK > 0: hook() runs at the start of every HK-th window row (the flow kernel's
// issue-priority check).
struct NoHook {
  __device__ void operator()() const {}
};
template <int B, int K, int H, int PC = 0, int HK = 0, typename Hook = NoHook>
__device__ __forceinline__ void qsad_lane(const uint8_t* __restrict__ tile, int pitch,
                                          uint32_t buf_off, int lrow, int w0,
                                          const uint32_t (&c)[B][B / 4], uint64_t (&acc)[K],
                                          Hook hook = Hook{}) {
  constexpr int CW = B / 4;
  constexpr int NR = K + H - 1;
  constexpr int RG = PC > 0 ? ((1020 - 4 * CW) / PC + 1 < 8 ? (1020 - 4 * CW) / PC + 1 : 8) : 1;
  // Operand pair k = ref words (w0 + k, w0 + k + 1) of the current row: one
  // ds_read2_b32 straight into an aligned VGPR pair.  Pairs 0, 2 come from
  // byte offset oe = 4*w0, pairs 1, 3 from oo = oe + 4; both advance through
  // an opaque asm, so the compiler neither hoists every row's address (spills)
  // nor merges the overlapping words of adjacent pairs (v_mov per qsad).
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)tile);
  uint32_t oe = lds0 + buf_off + (uint32_t)(lrow * pitch + 4 * w0);
  uint32_t oo = oe + 4;
  asm volatile("" : "+v"(oo));

#pragma unroll
  for (int j = 0; j < K; j++) acc[j] = 0;

  // LDS addresses as plain integers (address space 3, base folded into oe/oo
  // once) so no per-row add of the dynamic-LDS symbol survives.
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  auto load = [&](uint64_t (&dst)[CW], uint32_t ro) {
#pragma unroll
    for (int k = 0; k < CW; k++) {
      lds_u32* w = reinterpret_cast<lds_u32*>((uintptr_t)(((k & 1) ? oo : oe) + ro)) + 2 * (k >> 1);
      dst[k] = ((uint64_t)w[1] << 32) | w[0];
    }
  };
  uint64_t pr[CW], nx[CW];
  load(pr, 0);
  static_for<0, NR>([&](auto YY) {
    constexpr int yy = decltype(YY)::value;
    // one segment per window row: next row's loads, then this row's qsads.
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (HK > 0 && yy > 0 && yy % HK == 0) {
      hook();
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (yy + 1 < NR) {
      if constexpr (PC > 0) {
        constexpr int nr = yy + 1;
        if constexpr (nr % RG == 0) {
          oe += RG * PC;
          oo += RG * PC;
          asm volatile("" : "+v"(oe), "+v"(oo));
        }
        load(nx, (uint32_t)((nr % RG) * PC));
      } else {
        oe += pitch;
        oo += pitch;
        asm volatile("" : "+v"(oe), "+v"(oo));
        load(nx, 0);
      }
    }
    static_for<0, CW>([&](auto KK) {
      constexpr int k = decltype(KK)::value;
      static_for<0, K>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        constexpr int y = yy - j;
        if constexpr (y >= 0 && y < H)
          acc[j] = __builtin_amdgcn_qsad_pk_u16_u8(pr[k], c[y][k], acc[j]);
      });
    });
    // Pin this row's qsads inside its segment (readnone intrinsics are not
    // ordered by sched_barrier; the DAG would otherwise sink them past every
    // later row's loads and spill the loaded rows).
    pin_rows<0, K, yy, H>(acc);
    if constexpr (yy + 1 < NR) {
#pragma unroll
      for (int k = 0; k < CW; k++) pr[k] = nx[k];
    }
  });
}

#ifdef ME_STAMPS
// Diagnostic build only (-DME_STAMPS): per-workgroup s_memtime stamps
// [start, staged, computed, end, hw_id, xcc_id] for tools/stamps.py.
__device__ unsigned long long g_stamps[8 << 16];
#define ME_STAMP(slot, v) do { if (threadIdx.x == 0 && wid < (1 << 16)) g_stamps[8 * wid + (slot)] = (v); } while (0)
// ... and per wave of me_fast_kernel: [start, first item staged, last task
// loop done, end, hw_id, xcc_id, realtime start, realtime end] (tools/wave_stamps.py)
__device__ unsigned long long g_wstamps[8 << 14];
#define ME_WSTAMP(slot, v) do { if ((threadIdx.x & 63) == 0 && wwid < (1 << 14)) g_wstamps[8 * wwid + (slot)] = (v); } while (0)
#else
#define ME_WSTAMP(slot, v) do { } while (0)
#define ME_STAMP(slot, v) do { } while (0)
#endif

// 32-bit lane keys (sad << 16 | j*5 + i) ordered like (cost, dy, dx); i = 4 is
// the fold's dx = +S column (after every group dx of the same dy).  j*5 + i <=
// 64 for K <= 13 keeps every index an inline constant (VOP3 on gfx950 takes
// no literals: larger ones would each pin a VGPR and spill); invalid
// candidates forced to sad 0xFFFF (> any valid SAD: B*B*255 <= 65280).
// MASKJ = false on items whose whole dy range is valid (uniform per item).
// min(a, b, c) as one v_min3_u32 (ASM, K > 13: the 8x8 K = 26 lane-tasks):
// written as min(min(..)) the compiler reassociates the two key chains into
// trees of v_min + v_min3 (72 instead of 52 instructions for the 104 keys of
// an 8x8 lane-task).  The K <= 13 instances keep plain C: the asm operands
// pinned registers there and spilled 5 VGPRs of the 4K instance
// <SAD, 16, 13, 272> (24 bytes per lane of scratch, 32 MiB of writes per
// 16-frame launch; tests/test_kernel_resources.py guards it).
template <bool ASM>
__device__ __forceinline__ uint32_t min3u(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (ASM) {
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  } else {
    return min(min(a, b), c);
  }
}

template <int K, int J0, int J1, bool MASKJ>
__device__ __forceinline__ uint32_t lane_best_rows(const uint64_t (&acc)[K], uint32_t mlo,
                                                   uint32_t mhi, int jlo, int jhi) {
  // Two independent min3 chains (i = 0,1 and i = 2,3): the epilogues of all
  // waves on a SIMD tend to coincide (item barriers), so a single 2K-deep
  // dependent chain would run at VALU latency, not issue rate.
  uint32_t b01 = ~0u, b23 = ~0u;
#pragma unroll
  for (int j = J0; j < J1; j++) {
    uint32_t lo = (uint32_t)acc[j] | mlo, hi = (uint32_t)(acc[j] >> 32) | mhi;
    if (MASKJ) {
      const bool jv = j >= jlo && j <= jhi;
      lo = jv ? lo : ~0u;
      hi = jv ? hi : ~0u;
    }
    const uint32_t k0 = (lo << 16) | (uint32_t)(5 * (j - J0));
    const uint32_t k1 = (lo & 0xFFFF0000u) | (uint32_t)(5 * (j - J0) + 1);
    const uint32_t k2 = (hi << 16) | (uint32_t)(5 * (j - J0) + 2);
    const uint32_t k3 = (hi & 0xFFFF0000u) | (uint32_t)(5 * (j - J0) + 3);
    b01 = min3u<(K > 13)>(b01, k0, k1);
    b23 = min3u<(K > 13)>(b23, k2, k3);
  }
  return min(b01, b23);
}

// K > 13 (26: 8x8 SAD): two runs of 13 rows, each with inline-constant
// indices; the second's keys move past the first's (+ 5 * 13), so the min
// still orders by (sad, j, i).  A lane key's index is 5 j + i for every K.
template <int K, bool MASKJ>
__device__ __forceinline__ uint32_t lane_best(const uint64_t (&acc)[K], uint32_t mlo,
                                              uint32_t mhi, int jlo, int jhi) {
  if constexpr (K <= 13) {
    return lane_best_rows<K, 0, K, MASKJ>(acc, mlo, mhi, jlo, jhi);
  } else {
    const uint32_t a = lane_best_rows<K, 0, 13, MASKJ>(acc, mlo, mhi, jlo, jhi);
    uint32_t b = lane_best_rows<K, 13, K, MASKJ>(acc, mlo, mhi, jlo, jhi);
    b = b < 0xFFFF0000u ? b + 65u : b;  // (an all-masked run stays ~0)
    return min(a, b);
  }
}

// Fold column: SAD of the lane's one dx = +S candidate (window rows row..row+H-1,
// B bytes at byte offset `off` of the tile row, B-aligned) with v_sad_u8.
template <int B, int H>
__device__ __forceinline__ uint32_t tail_sad(const uint8_t* __restrict__ tile, int pitch,
                                             uint32_t off, const uint32_t (&c)[B][B / 4]) {
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)tile);
  uint32_t o = lds0 + off;
  uint32_t sad = 0;
#pragma unroll
  for (int y = 0; y < H; y++) {
    if constexpr (B == 16) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) const u32x4 lds_v4;
      const u32x4 w = *reinterpret_cast<lds_v4*>((uintptr_t)o);
      sad = __builtin_amdgcn_sad_u8(w[0], c[y][0], sad);
      sad = __builtin_amdgcn_sad_u8(w[1], c[y][1], sad);
      sad = __builtin_amdgcn_sad_u8(w[2], c[y][2], sad);
      sad = __builtin_amdgcn_sad_u8(w[3], c[y][3], sad);
    } else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      typedef __attribute__((address_space(3))) const u32x2 lds_v2;
      const u32x2 w = *reinterpret_cast<lds_v2*>((uintptr_t)o);
      sad = __builtin_amdgcn_sad_u8(w[0], c[y][0], sad);
      sad = __builtin_amdgcn_sad_u8(w[1], c[y][1], sad);
    }
    o += pitch;
  }
  return sad;
}

// --------------------------------------------------------------- dot4 (SSD)
// SSD of one dx and K dy candidates, exactly: SSD = sum c^2 + sum r^2 - 2 sum c*r
// in u32.  sum c*r: v_dot4_u32_u8 of the cur words with the ref words realigned
// to this lane's dx (v_alignbyte, shift sh); sum r^2: a running prefix P over
// the window rows (4 more dot4 per row), snapshotted when candidate j's first
// row arrives (pst[j] = P(j-1)) and closed after its last (pst[j] = P - pst[j]).
// Returns out[j] = sum r^2 - 2 sum c*r (mod 2^32; the caller adds sum c^2).
template <int B, int K, int H>
__device__ __forceinline__ void ssd_lane(const uint8_t* __restrict__ tile, int pitch,
                                         uint32_t buf_off, int lrow, int wb, int sh,
                                         const uint32_t (&c)[B][B / 4], uint32_t (&out)[K]) {
  constexpr int CW = B / 4;
  constexpr int NR = K + H - 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)tile);
  uint32_t o = lds0 + buf_off + (uint32_t)(lrow * pitch + 4 * wb);
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  auto load = [&](uint32_t (&dst)[CW + 1]) {
    lds_u32* w = reinterpret_cast<lds_u32*>((uintptr_t)o);
#pragma unroll
    for (int k = 0; k <= CW; k++) dst[k] = w[k];
  };
  uint32_t acc[K], pst[K];
#pragma unroll
  for (int j = 0; j < K; j++) { acc[j] = 0; pst[j] = 0; }
  uint32_t P = 0;
  uint32_t w[CW + 1], nw[CW + 1];
  load(w);
  static_for<0, NR>([&](auto YY) {
    constexpr int yy = decltype(YY)::value;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (yy + 1 < NR) {
      o += pitch;
      asm volatile("" : "+v"(o));
      load(nw);
    }
    uint32_t al[CW];
#pragma unroll
    for (int k = 0; k < CW; k++) al[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
    uint32_t rs = 0;
#pragma unroll
    for (int k = 0; k < CW; k++) rs = __builtin_amdgcn_udot4(al[k], al[k], rs, false);
    P += rs;
    static_for<0, CW>([&](auto KK) {
      constexpr int k = decltype(KK)::value;
      static_for<0, K>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        constexpr int y = yy - j;
        if constexpr (y >= 0 && y < H) acc[j] = __builtin_amdgcn_udot4(al[k], c[y][k], acc[j], false);
      });
    });
    if constexpr (yy + 1 < K) pst[yy + 1] = P;          // P(j - 1) for j = yy + 1
    if constexpr (yy - H + 1 >= 0 && yy - H + 1 < K)    // last row of j = yy - H + 1
      pst[yy - H + 1] = P - pst[yy - H + 1];
    pin_rows32<0, K, yy, H>(acc);
    if constexpr (yy + 1 < NR) {
#pragma unroll
      for (int k = 0; k <= CW; k++) w[k] = nw[k];
    }
  });
#pragma unroll
  for (int j = 0; j < K; j++) out[j] = pst[j] - 2u * acc[j];
}

// Lane key ((v + SSD_BIAS) << 5 | j) with v = sum r^2 - 2 sum c*r: SSD = v +
// sum c^2, and sum c^2 is the same for every candidate of a block, so v ranks
// them exactly; v >= -sum c^2 > -2^24 (B <= 16), so v + SSD_BIAS lies in
// [0, 2^25) and the key below 2^30 (j < 32).  Block costs get sum c^2 back
// once per block at output.
constexpr uint32_t SSD_BIAS = 1u << 24;

template <int K, bool MASKJ>
__device__ __forceinline__ uint32_t lane_best_ssd(const uint32_t (&v)[K], int jlo, int jhi) {
  static_assert(K < 32, "j field is 5 bits");
  uint32_t b0 = ~0u, b1 = ~0u;  // two chains (see lane_best)
#pragma unroll
  for (int j = 0; j < K; j++) {
    uint32_t key = ((v[j] + SSD_BIAS) << 5) | (uint32_t)j;
    if (MASKJ) key = (j >= jlo && j <= jhi) ? key : ~0u;
    if (j & 1) b1 = min(b1, key);
    else b0 = min(b0, key);
  }
  return min(b0, b1);
}

// LDS DMA of `bytes` (multiple of 16) into lds_dst: 16 bytes per lane, lane i
// of DMA step s covers bytes [1024 s + 16 i, +16) of the destination; src_off
// maps such a destination byte offset to the buffer offset (any uint32: the
// descriptor's range check returns zeros for offsets past the resident rows,
// including negative ones, which wrap).
// Lane index recomputed per call: an opaque copy of threadIdx.x keeps the
// compiler from hoisting lane-derived staging addresses out of the item loop,
// where they would stay live across the 128-VGPR task loop and spill.
__device__ __forceinline__ int fresh_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

template <typename F>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_dst, int bytes,
                                      F src_off) {
  const int tid = fresh_tid();
  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  for (int s0 = wave * 1024; s0 < bytes; s0 += nw * 1024) {
    const int d = s0 + 16 * lane;
    // lanes past the end must not execute: an out-of-range lane would still
    // write (zeros) to its LDS slot.
    if (d < bytes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(lds_dst + s0), 16, src_off(d), 0, 0, 0);
  }
}

// LDS DMA with 4-byte granules (256 bytes per wave step): used for the ref
// tile, whose left/top edges hang off the frame.  X0 is 4-aligned, so no
// granule straddles x = 0 or x = W (W % 4 == 0 on this path): every granule is
// either all in-frame or all masked, and the range check zeroes out-of-range
// ones (a 16-byte granule straddling x = 0 on row 0 would be zeroed whole).
template <typename F>
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_dst, int bytes,
                                     F src_off) {
  const int tid = fresh_tid();
  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  for (int s0 = wave * 256; s0 < bytes; s0 += nw * 256) {
    const int d = s0 + 4 * lane;
    if (d < bytes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(lds_dst + s0), 4, src_off(d), 0, 0, 0);
  }
}

// Geometry of one work item = (tile of TB blocks, dy pass); j: the flow
// kernel's job (FlowJobs) the tile belongs to.
struct Item {
  int bx0, by, nb, tly, h, a, X0, c0, nch, prow0, prows, j;
};

template <int B, int K>
__device__ __forceinline__ Item item_of(const SearchArgs& p, const QsadGeom& g, int tile,
                                        int pass) {
  Item it;
  it.j = 0;
  if (g.strip_w > 0) {
    // strip-major: strip s holds tile columns [s * sw, s * sw + its width),
    // walked row by row (the last strip may be narrower)
    const int sw = g.strip_w, per = sw * g.nrows;
    const int s = tile / per, r = tile - s * per;
    const int w = min(sw, g.wg_per_row - s * sw);
    const int row = r / w;
    it.bx0 = (s * sw + (r - row * w)) * g.tb;
    it.by = g.row0 + row;
  } else {
    // row-major; the division by a multiply-high (scalar) where the host
    // verified the magic: a VALU integer division here ran twice per item
    const int row = g.magic_wpr ? (int)__umulhi((uint32_t)tile, g.magic_wpr) : tile / g.wg_per_row;
    it.bx0 = (tile - row * g.wg_per_row) * g.tb;
    it.by = g.row0 + row;
  }
  it.nb = min(g.tb, g.nbx_full - it.bx0);
  it.tly = it.by * B;
  it.h = min(B, p.height - it.tly);
  it.a = ((it.bx0 * B - p.range) % 4 + 4) % 4;
  it.X0 = it.bx0 * B - p.range - it.a;
  it.c0 = pass * g.cpp;
  it.nch = min(g.cpp, g.chunks - it.c0);
  it.prow0 = it.tly - p.range + it.c0 * K;  // frame row of tile row 0
  it.prows = it.nch * K + B - 1;            // rows this item touches
  return it;
}

// Tile of a launch over a job table -> (job, tile of that job's rows): jobs
// are consecutive tile ranges (jb.tile_pre), every job the same frame
// geometry; a job's planes and records are its own.
template <int B, int K>
__device__ __forceinline__ Item job_item(const SearchArgs& p, const QsadGeom& g,
                                         const FlowJobs& jb, int tile, int pass) {
  int j = 0;
  while (j + 1 < jb.n && jb.tile_pre[j + 1] <= tile) j++;
  QsadGeom gj = g;
  gj.row0 = jb.r0[j];
  if (g.strip_w > 0) gj.nrows = (jb.tile_pre[j + 1] - jb.tile_pre[j]) / g.wg_per_row;  // strip walk
  Item it = item_of<B, K>(p, gj, tile - jb.tile_pre[j], pass);
  it.j = j;
  return it;
}

// Issue the staging of one item into an LDS buffer from its job's planes:
// asynchronous LDS DMA on the aligned path (no VGPR round trip, completes
// under the previous item's compute), synchronous byte copies otherwise.
template <int B>
__device__ __forceinline__ void stage_item(const SearchArgs& p, const QsadGeom& g, const Item& it,
                                           uint8_t* buf, const FlowJobs& jb) {
  uint8_t* tile = buf;
  uint8_t* cur = buf + g.tile_bytes;
  const int pitch = g.pitch, stride = p.stride;
  const int tid = fresh_tid(), nthr = blockDim.x;
  const int ref_row0 = jb.ref_row0[it.j], cur_row0 = jb.cur_row0[it.j];
  if (g.aligned) {
    const __amdgpu_buffer_rsrc_t rref = __builtin_amdgcn_make_buffer_rsrc(
        (void*)jb.ref[it.j], (short)0, jb.ref_bytes[it.j], 0x00020000);
    const __amdgpu_buffer_rsrc_t rcur = __builtin_amdgcn_make_buffer_rsrc(
        (void*)jb.cur[it.j], (short)0, jb.cur_bytes[it.j], 0x00020000);
    // tile byte (r, x) <- ref(prow0 + r, X0 + x); zeros outside the resident rows.
    const int base = (it.prow0 - ref_row0) * stride + it.X0;
    auto src = [&](int d) {
      const int r = (int)__umulhi((uint32_t)d, g.pitch_magic), x = d - r * pitch;
      return (uint32_t)(base + r * stride + x);
    };
    // 16-byte granules when X0, the frame width and the rows are 16-aligned:
    // no granule straddles x = 0 or x = W, and a quarter of the DMA steps.
    if (g.tile16)
      dma16(rref, tile, it.prows * pitch, src);
    else
      dma4(rref, tile, it.prows * pitch, src);
    // cur block b, row oy -> LDS bytes (b * B + oy) * B
    const int cbase = (it.tly - cur_row0) * stride + it.bx0 * B;
    if constexpr (B == 16) {
      dma16(rcur, cur, it.nb * B * B, [&](int d) {
        return (uint32_t)(cbase + ((d >> 4) & 15) * stride + (d >> 8) * B);
      });
    } else {
      dma4(rcur, cur, it.nb * B * B, [&](int d) {
        return (uint32_t)(cbase + ((d >> 3) & 7) * stride + (d >> 6) * B + (d & 4));
      });
    }
  } else {
    for (int i = tid; i < it.prows * pitch; i += nthr) {
      const int r = i / pitch, x = i - r * pitch;
      const int y = it.prow0 + r, xx = it.X0 + x;
      tile[i] = (y >= 0 && y < p.height && xx >= 0 && xx < p.width)
                    ? row_ptr(p, jb.ref[it.j], ref_row0, y)[xx] : 0;
    }
    for (int i = tid; i < it.nb * B * B; i += nthr) {
      const int b = i / (B * B), rem = i - b * B * B, oy = rem / B, x = rem - oy * B;
      cur[i] = oy < it.h ? row_ptr(p, jb.cur[it.j], cur_row0, it.tly + oy)[(it.bx0 + b) * B + x] : 0;
    }
  }
}

// Persistent, double-buffered search over a job table (one frame, or the
// frames / stripes of a batch: every job's tiles, job-major).  The grid is
// sized to what fits on the chip at once; workgroups sharing an XCD (bid % 8,
// a speed heuristic only) walk one contiguous band of tiles, so each XCD's L2
// holds one band of rows.  Item k of a workgroup = (its k / passes-th tile,
// pass k % passes); while item k is computed from LDS buffer k & 1, item k + 1
// streams into the other.
template <int COST, int B, int K, int PC = 0>
__global__ __launch_bounds__(1024) void me_fast_kernel(SearchArgs p, QsadGeom g, FlowJobs jb) {
  constexpr int CW = B / 4;
  extern __shared__ __align__(16) uint8_t smem[];
  const int buf_bytes = g.tile_bytes + g.tb * B * B;
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem + 2 * buf_bytes);
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int S = p.range;

  // Tiles of this workgroup come from the band of its XCD group x (bid % 8,
  // a speed heuristic only).  Dynamic (p.sched != null): the group's
  // workgroups pull whole tiles from one agent-scope counter, so faster CUs
  // take more; tile ids are pulled two tiles ahead into an LDS ring so the
  // double-buffered staging always knows its next item.  Static otherwise:
  // member m of n_x takes band tiles m, m + n_x, ...
  const int ntiles = jb.tile_pre[jb.n];
  const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
  const int ng = nwg < 8 ? nwg : 8;  // XCD groups that have workgroups
  const int x = bid % ng, m = bid / ng;
  const int n_x = nwg / ng + (x < nwg % ng ? 1 : 0);
  const int band0 = (int)((long)ntiles * x / ng), band1 = (int)((long)ntiles * (x + 1) / ng);
  const int passes = (g.chunks + g.cpp - 1) / g.cpp;
  // Dynamic only with enough tiles per workgroup (g.dyn_tiles, see plan_fast):
  // with few, the item-start pulls of all workgroups coincide and serialise.
  const bool dyn = p.sched != nullptr && g.dyn_tiles > 0 && ntiles >= g.dyn_tiles * nwg;
  int* tq = reinterpret_cast<int*>(smem + 2 * buf_bytes + 128);  // 4-slot ring of tile ids
#ifdef ME_STAMPS
  const int wid = bid;
  const int wwid = bid * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
#endif
  ME_STAMP(0, __builtin_amdgcn_s_memtime());
  ME_STAMP(6, __builtin_amdgcn_s_memrealtime());
  ME_WSTAMP(0, __builtin_amdgcn_s_memtime());
  ME_WSTAMP(6, __builtin_amdgcn_s_memrealtime());
  // Staging at raised issue priority: the SIMD arbiter otherwise favours the
  // oldest waves, so the co-resident workgroups already computing starve a
  // later one's staging address math and it gets its first item late (the
  // small-stripe "staircase" of DESIGN.md (e): per-wave stamps
  // profiles/r03c_wave_stamps.txt).
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  // Dynamic: each workgroup's first two tiles are its static ones (no atomic
  // storm at launch); band y's tiles past its first 2 * n_y are claimed from a
  // two-ended u64 counter: its own workgroups from the front (low half), once
  // their band is exhausted other XCD groups' workgroups from the back (high
  // half; clocks differ by several % between XCDs, so bands finish unevenly).
  // One atomic add per claim and the claim is valid iff lo + hi < avail of the
  // returned old value, so every tile is claimed once.  Thieves take the band's
  // LAST rows, contiguously, where front steals each re-read a whole window
  // (2S + B rows) on the thief's XCD for B rows of output; at 4K +-64 steals
  // are few and both measured alike (365 vs 368 MB per 16-frame launch,
  // profiles/r04i_*, r04j_*: the excess there was the claim distance, below).
  auto pull = [&]() -> int {
    for (int d = 0; d < ng; d++) {
      const int y = x + d < ng ? x + d : x + d - ng;
      const int b0 = (int)((long)ntiles * y / ng), b1 = (int)((long)ntiles * (y + 1) / ng);
      const int n_y = nwg / ng + (y < nwg % ng ? 1 : 0);
      const int first = min(b1 - b0, 2 * n_y), avail = b1 - b0 - first;
      if (avail <= 0) continue;
      const uint64_t o = __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(p.sched) + y,
                                                d == 0 ? 1ull : (1ull << 32), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const int lo = (int)(uint32_t)o, hi = (int)(o >> 32);
      if (lo + hi < avail) return d == 0 ? b0 + first + lo : b1 - 1 - hi;
    }
    return -1;
  };
  auto static_tile = [&](int i) -> int {  // i-th static tile of this workgroup
    const int t = band0 + m + i * n_x;
    return t < band1 ? t : -1;
  };
  auto tile_at = [&](int i) -> int {  // i-th tile of this workgroup, -1 = none
    return dyn ? tq[i & 3] : static_tile(i);
  };
  auto claim = [&](int i) -> int {  // tile i of this workgroup (dynamic)
    if (i < 2) {
      const int t = static_tile(i);
      if (t >= 0) return t;
    }
    return pull();
  };
  const int ahead = g.pull_ahead;
  if (dyn && tid == 0) {
    tq[0] = claim(0);
    if (ahead == 2) tq[1] = tq[0] >= 0 ? claim(1) : -1;
  }
  if (tid < g.tb) keys[tid] = ~0ull;
  __syncthreads();

  int ti = 0, pass = 0;
  int rot = bid % (nthr >> 6);
#ifdef ME_STAMPS
  int nitems = 0;
#endif
  int tile = tile_at(0);
  if (tile >= 0) stage_item<B>(p, g, job_item<B, K>(p, g, jb, tile, 0), smem, jb);
  const int G = g.groups;
  for (int k = 0; tile >= 0; k++) {
    const Item it = job_item<B, K>(p, g, jb, tile, pass);
    uint8_t* buf = smem + (k & 1) * buf_bytes;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // item k staged by every wave; item k-1 fully consumed
    if (k == 0) ME_STAMP(2, __builtin_amdgcn_s_memtime());  // first item staged
    if (k == 0) ME_WSTAMP(1, __builtin_amdgcn_s_memtime());
    if (dyn && pass == 0 && tid == 0) {  // starting tile ti: claim tile ti + ahead
      const int prev = tq[(ti + ahead - 1) & 3];
      tq[(ti + ahead) & 3] = prev >= 0 ? claim(ti + ahead) : -1;
    }
    {
      const int ntile = pass + 1 < passes ? tile : tile_at(ti + 1);
      const int npass = pass + 1 < passes ? pass + 1 : 0;
      if (g.prio) __builtin_amdgcn_s_setprio(3);
      if (ntile >= 0)
        stage_item<B>(p, g, job_item<B, K>(p, g, jb, ntile, npass),
                      smem + ((k + 1) & 1) * buf_bytes, jb);
      if (g.prio) __builtin_amdgcn_s_setprio(0);
    }
#ifdef ME_STAMPS
    nitems++;
#endif
    const uint32_t* cur_lds = reinterpret_cast<const uint32_t*>(buf + g.tile_bytes);
    const uint32_t tile_off = (uint32_t)((k & 1) * buf_bytes);
    const int dymin = max(-S, -it.tly), dymax = min(S, p.height - it.h - it.tly);
    // Chunks whose dy range lies wholly outside [dymin, dymax] (top / bottom
    // block rows) are skipped: tasks are chunk-major, so whole waves drop out.
    const int lc0 = max(0, (dymin + S) / K - it.c0);
    const int lc1 = min(it.nch, (dymax + S) / K + 1 - it.c0);
    // Every candidate row of this item valid -> no per-row masks (uniform).
    const bool full_rows = dymin + S <= it.c0 * K && dymax + S >= (it.c0 + it.nch) * K - 1;
    const int per_chunk = it.nb * G;
    const int T = (lc1 - lc0) * per_chunk;
    // task t -> (chunk, block, group) by multiply-high: t / G with the host's
    // verified magic, then / nb with a per-item magic (nb <= 16).
    const uint32_t magic_nb = it.nb == g.tb ? g.magic_tb : 0xFFFFFFFFu / (uint32_t)it.nb + 1u;
    // When T is not a multiple of the workgroup size the last round falls to
    // the first waves; rotate which wave that is from item to item so no SIMD
    // takes every extra round (rot == (bid + k) % waves, kept as a counter).
    int vt = fresh_tid() - 64 * rot;
    if (vt < 0) vt += nthr;
    rot = rot + 1 == (nthr >> 6) ? 0 : rot + 1;
    for (int t = vt; t < T; t += nthr) {
      const int bg = (int)__umulhi((uint32_t)t, g.magic_groups);  // t / G
      const int gi = t - bg * G;
      const int lcr = it.nb == 1 ? bg : (int)__umulhi((uint32_t)bg, magic_nb);  // bg / nb
      const int b = bg - lcr * it.nb;
      const int lc = lc0 + lcr;
      const int d0 = (it.c0 + lc) * K;
      const int tlx = (it.bx0 + b) * B;

      uint32_t c[B][CW];
#pragma unroll
      for (int y = 0; y < B; y++) {
        if constexpr (CW == 4) {
          const uint4 v = reinterpret_cast<const uint4*>(cur_lds)[b * B + y];
          c[y][0] = v.x; c[y][1] = v.y; c[y][2] = v.z; c[y][3] = v.w;
        } else {
          const uint2 v = reinterpret_cast<const uint2*>(cur_lds)[b * B + y];
          c[y][0] = v.x; c[y][1] = v.y;
        }
      }
      // Valid candidate ranges of this block (main.c:73-76 in closed form).
      const int dxmin = max(-S, -tlx), dxmax = min(S, p.width - B - tlx);
      const int jlo = dymin + S - d0, jhi = dymax + S - d0;
      if constexpr (COST == COST_SSD) {
        // lane = one dx (gi = dx + S); its column starts at tile byte b*B + a + gi
        const int q = b * B + it.a + gi, dx = gi - S;
        uint32_t v[K];
        if (it.h == B)
          ssd_lane<B, K, B>(smem, g.pitch, tile_off, lc * K, q >> 2, q & 3, c, v);
        else
          ssd_lane<B, K, B / 2>(smem, g.pitch, tile_off, lc * K, q >> 2, q & 3, c, v);
        uint32_t best = full_rows ? lane_best_ssd<K, false>(v, jlo, jhi)
                                  : lane_best_ssd<K, true>(v, jlo, jhi);
        if (dx < dxmin || dx > dxmax) best = ~0u;
        if (best != ~0u) {
          const int dy = d0 + (int)(best & 31u) - S;
          atomicMin(reinterpret_cast<unsigned long long*>(&keys[b]),
                    (unsigned long long)make_key(best >> 5, dx, dy));
        }
        continue;
      }
      const int w0 = (b * B) / 4 + gi;
      uint64_t acc[K];
      // fold: lane gi < K also owns candidate (dx = +S, dy index jt = gi)
      const int jt = gi < K ? gi : K - 1;
      const uint32_t toff = tile_off + (uint32_t)((lc * K + jt) * g.pitch + b * B + 2 * S);
      uint32_t tsad = 0;
      if (it.h == B) {
        qsad_lane<B, K, B, PC>(smem, g.pitch, tile_off, lc * K, w0, c, acc);
        if (g.fold) tsad = tail_sad<B, B>(smem, g.pitch, toff, c);
      } else {
        qsad_lane<B, K, B / 2, PC>(smem, g.pitch, tile_off, lc * K, w0, c, acc);
        if (g.fold) tsad = tail_sad<B, B / 2>(smem, g.pitch, toff, c);
      }
      // Waves with no frame-edge candidate (most of them) take the unmasked
      // epilogue: the test is wave-uniform, so there is no divergence.
      const int dxg = 4 * gi - S - it.a;  // dx of this lane's first candidate
      const bool edge = dxg < dxmin || dxg + 3 > dxmax;
      uint32_t best;
      const bool no_edge = __builtin_amdgcn_ballot_w64(edge) == 0;
      const int sjlo = __builtin_amdgcn_readfirstlane(jlo), sjhi = __builtin_amdgcn_readfirstlane(jhi);
      if (no_edge && (full_rows || __builtin_amdgcn_ballot_w64(jlo != sjlo || jhi != sjhi) == 0)) {
        // Rows partial only (the last dy chunk, the top and bottom block rows)
        // with one row range for the wave: park the invalid rows at SAD 0xFFFF
        // (scalar tests, a move only where a row is out) and take the unmasked
        // epilogue; the masked one tests every row of every lane.  (Testing
        // the row range only on partial-row tasks measured 0.7 % slower at 8K:
        // 271.7 vs 269.7 ms, profiles/r04y_ab.txt.)
        if (!full_rows) {
#pragma unroll
          for (int j = 0; j < K; j++)
            if (j < sjlo || j > sjhi) acc[j] = ~0ull;
        }
        best = lane_best<K, false>(acc, 0u, 0u, jlo, jhi);
      } else {
        uint32_t mlo = 0, mhi = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int dx = dxg + i;
          const uint32_t msk = (dx < dxmin || dx > dxmax) ? 0xFFFFu : 0u;
          if (i < 2) mlo |= msk << (16 * i);
          else mhi |= msk << (16 * (i - 2));
        }
        best = lane_best<K, true>(acc, mlo, mhi, jlo, jhi);
      }
      if (g.fold) {
        const bool tv = gi < K && jt >= jlo && jt <= jhi && S <= dxmax;
        best = min(best, tv ? (tsad << 16) | (uint32_t)(5 * jt + 4) : ~0u);
      }
      if (best < 0xFFFF0000u) {
        const int idx = (int)(best & 0xFFFFu), jj = idx / 5, i = idx - 5 * jj;
        const int dy = d0 + jj - S, dx = i == 4 ? S : 4 * gi + i - S - it.a;
        atomicMin(reinterpret_cast<unsigned long long*>(&keys[b]),
                  (unsigned long long)make_key(best >> 16, dx, dy));
      }
    }
    ME_WSTAMP(2, __builtin_amdgcn_s_memtime());  // this wave's tasks of item k done
    if (pass == passes - 1) {
      __syncthreads();  // every task of the tile has folded its key
      if (tid < it.nb) {
        const uint64_t kk = keys[tid];
        uint64_t none = ~0ull;  // materialised here, not kept live (it spilled)
        asm volatile("" : "+v"(none));
        keys[tid] = none;  // ready for this workgroup's next tile
        const int out = (it.by - jb.r0[it.j]) * p.nbx + it.bx0 + tid;
        int16_t* mv = jb.mv[it.j];
        store_mv(mv, out, kk);
        uint32_t cost = (uint32_t)(kk >> 32);
        if constexpr (COST == COST_SSD) {  // biased v -> SSD: + sum c^2 of the block
          const uint32_t* cb = reinterpret_cast<const uint32_t*>(buf + g.tile_bytes) + tid * B * CW;
          uint32_t csq = 0;
#pragma unroll 4
          for (int i = 0; i < B * CW; i++) csq = __builtin_amdgcn_udot4(cb[i], cb[i], csq, false);
          cost = cost - SSD_BIAS + csq;
        }
        if (jb.cost[it.j]) jb.cost[it.j][out] = cost;
      }
      ti++;
      pass = 0;
      tile = tile_at(ti);  // written >= one barrier ago
    } else {
      pass++;
    }
  }
  ME_STAMP(1, (unsigned long long)nitems);
#ifdef ME_STAMPS
  if ((threadIdx.x & 63) == 0 && wwid < (1 << 14)) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_wstamps[8 * wwid + 3] = __builtin_amdgcn_s_memtime();
    g_wstamps[8 * wwid + 4] = hw;
    g_wstamps[8 * wwid + 5] = xcc;
    g_wstamps[8 * wwid + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (dyn && tid == 0) {
    // The last workgroup out re-zeroes the counters for the next launch on
    // this stream (every other workgroup's final pull precedes its arrival).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t d = __hip_atomic_fetch_add(p.sched + SCHED_ARRIVE, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    if (d == (uint32_t)nwg - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
      for (int i = 0; i <= SCHED_ARRIVE; i++)
        __hip_atomic_store(p.sched + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#ifdef ME_STAMPS
  if (tid == 0 && wid < (1 << 16)) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_stamps[8 * wid + 3] = __builtin_amdgcn_s_memtime();
    g_stamps[8 * wid + 4] = hw;
    g_stamps[8 * wid + 5] = xcc;
    g_stamps[8 * wid + 7] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// --------------------------------------------------------------- flow (SAD)
// One workgroup per CU, 16 waves, no barriers after the start.  The
// workgroup's items (tiles of tb blocks with ALL their dy chunks) sit in a
// ring of NB LDS slots; the waves pull wave-tasks (64 consecutive lane-tasks
// of one item) from one LDS counter, so the 4 waves of every SIMD keep taking
// work until the workgroup's list is empty: no item barrier, no per-item
// partial last round of the workgroup (tb * G * chunks is a multiple of 64 on
// the shapes the planner gives this kernel: 1080p +-32 tb = 4 -> 320 lanes).
// The wave that finishes an item's last wave-task writes its blocks' vectors,
// then refills the slot with item k + NB (LDS DMA, its own vmcnt wait) and
// publishes it; a wave that pulls a task of an unpublished item sleeps on the
// slot's ready word.  Pulls are in order, so the items < k are all pulled
// before a wave waits on item k: the last of them to finish refills slot k % NB.
struct FlowCtl {
  uint32_t next;       // wave-tasks handed out
  uint32_t ready[16];  // item index + 1 published in the slot
  uint32_t done[16];   // wave-tasks of the slot's item finished
};

// Tile of the flow kernel's launch -> its item (all dy chunks: one pass).
template <int B, int K>
__device__ __forceinline__ Item flow_item(const SearchArgs& p, const QsadGeom& g,
                                          const FlowJobs& jb, int tile) {
  return job_item<B, K>(p, g, jb, tile, 0);
}

// Single-wave LDS DMA of one flow item (the aligned path): tile rows and cur
// blocks, from its job's planes.
template <int B>
__device__ __forceinline__ void stage_item_wave(const SearchArgs& p, const QsadGeom& g, const Item& it,
                                                uint8_t* buf, const FlowJobs& jb) {
  const __amdgpu_buffer_rsrc_t rref =
      __builtin_amdgcn_make_buffer_rsrc((void*)jb.ref[it.j], (short)0, jb.ref_bytes[it.j], 0x00020000);
  const __amdgpu_buffer_rsrc_t rcur =
      __builtin_amdgcn_make_buffer_rsrc((void*)jb.cur[it.j], (short)0, jb.cur_bytes[it.j], 0x00020000);
  // lane recomputed per call (fresh_tid): hoisted lane-derived offsets spilled
  const int lane = fresh_tid() & 63;
  uint8_t* tile = buf;
  uint8_t* cur = buf + g.tile_bytes;
  const int pitch = g.pitch, stride = p.stride;
  const uint32_t base = (uint32_t)((it.prow0 - jb.ref_row0[it.j]) * stride + it.X0);
  const int bytes = it.prows * pitch;
  for (int s0 = 0; s0 < bytes; s0 += 1024) {  // 16-byte granules (g.tile16)
    const int d = s0 + 16 * lane;
    const int r = (int)__umulhi((uint32_t)d, g.pitch_magic), x = d - r * pitch;
    if (d < bytes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rref, (__attribute__((address_space(3))) void*)(tile + s0), 16,
          base + (uint32_t)(r * stride + x), 0, 0, 0);
  }
  const uint32_t cbase = (uint32_t)((it.tly - jb.cur_row0[it.j]) * stride + it.bx0 * B);
  const int cb = it.nb * B * B;
  for (int s0 = 0; s0 < cb; s0 += 1024) {
    const int d = s0 + 16 * lane;
    if (d < cb)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rcur, (__attribute__((address_space(3))) void*)(cur + s0), 16,
          cbase + (uint32_t)(((d >> 4) & 15) * stride + (d >> 8) * B), 0, 0, 0);
  }
}

// Wave-tasks of one item: its lane-tasks (valid chunks x blocks x groups) / 64, rounded up.
template <int B, int K>
__device__ __forceinline__ int flow_tasks(const SearchArgs& p, const QsadGeom& g, const Item& it,
                                          int* lc0_out) {
  const int S = p.range;
  const int dymin = max(-S, -it.tly), dymax = min(S, p.height - it.h - it.tly);
  const int lc0 = max(0, (dymin + S) / K), lc1 = min(it.nch, (dymax + S) / K + 1);
  *lc0_out = lc0;
  return ((lc1 - lc0) * it.nb * g.groups + 63) >> 6;
}

template <int B, int K, int PC>
__global__ __launch_bounds__(1024) void me_flow_kernel(SearchArgs p, QsadGeom g, FlowJobs jb) {
  static_assert(B == 16, "cur-block DMA layout of stage_item_wave");
  constexpr int CW = B / 4;
  extern __shared__ __align__(16) uint8_t smem[];
  const int NB = g.flow_slots;
  const int slot_bytes = g.tile_bytes + g.tb * B * B;
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem + NB * slot_bytes);  // [NB][tb]
  FlowCtl* ctl = reinterpret_cast<FlowCtl*>(smem + NB * slot_bytes + NB * g.tb * 8);
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = p.range;

  // This workgroup's tiles: the XCD band of bid % 8 (a speed heuristic only),
  // member m takes tiles band0 + m, + n_x, ... (every job's tiles, job-major)
  const int ntiles = jb.tile_pre[jb.n];
  const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
  const int ng = nwg < 8 ? nwg : 8;
  const int x = bid % ng, m = bid / ng;
  const int n_x = nwg / ng + (x < nwg % ng ? 1 : 0);
  const int band0 = (int)((long)ntiles * x / ng), band1 = (int)((long)ntiles * (x + 1) / ng);
  const int nitems = band1 - band0 > m ? (band1 - band0 - m + n_x - 1) / n_x : 0;
  auto tile_of = [&](int k) { return band0 + m + k * n_x; };

  if (tid < 64) {
    if (tid == 0) ctl->next = 0;
    if (tid < 16) {
      ctl->ready[tid] = 0;
      ctl->done[tid] = 0;
    }
  }
  for (int i = tid; i < NB * g.tb; i += (int)blockDim.x) keys[i] = ~0ull;
  __syncthreads();
  // wave w < NB stages item w and publishes it
  if (wave < NB && wave < nitems) {
    // Staggered start (wave w waits w x 640 cycles): item 0's DMA gets the
    // CU's memory pipeline first and lands early instead of every item
    // landing together at the end of one burst (1080p, same box:
    // 78.4 -> 78.0 us; with the compile-time pitch 79.0 -> 77.3,
    // profiles/r02ae_ab_flow_start.txt).
    for (int i = 0; i < wave; i++) __builtin_amdgcn_s_sleep(10);
    if (g.prio) __builtin_amdgcn_s_setprio(3);  // see me_fast_kernel
    stage_item_wave<B>(p, g, flow_item<B, K>(p, g, jb, tile_of(wave)), smem + wave * slot_bytes, jb);
    if (g.prio) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(&ctl->ready[wave], (uint32_t)wave + 1u, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
  }

  int kc = 0, basec = 0, lc0c = 0, nwc = 0;  // this wave's view: item kc's first task, task count
  Item itc;
  bool have = false;
#ifdef ME_STAMPS
  // diagnostic build: per wave [start, first task, loop exit, spin cycles, tasks,
  // realtime start, realtime end, hw_id] (tools/flow_stamps.py)
  const int fw = bid * 16 + wave;
  unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_first = 0, st_spin = 0, st_n = 0;
  const unsigned long long st_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (;;) {
    uint32_t q = 0;
    if (lane == 0) q = __hip_atomic_fetch_add(&ctl->next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    q = (uint32_t)__builtin_amdgcn_readfirstlane((int)q);
    // advance to the item holding task q (pulls are in order: kc only grows)
    if (!have && kc < nitems) {
      itc = flow_item<B, K>(p, g, jb, tile_of(kc));
      nwc = flow_tasks<B, K>(p, g, itc, &lc0c);
      have = true;
    }
    while (kc < nitems && (int)q >= basec + nwc) {
      basec += nwc;
      kc++;
      if (kc < nitems) {
        itc = flow_item<B, K>(p, g, jb, tile_of(kc));
        nwc = flow_tasks<B, K>(p, g, itc, &lc0c);
      }
    }
    if (kc >= nitems) break;
    if (g.fair) __builtin_amdgcn_s_setprio(0);
    const int slot = kc % NB;
    // Bounded wait (the ordering argument above says it ends; the bound keeps a
    // broken invariant from hanging the GPU).  An expired wait is reported:
    // sched[SCHED_ERR] is set, and the host turns it into ME_EDEVICE
    // (device_status after the synchronous entry points, me_device_check).
    int spins = 0;
#ifdef ME_STAMPS
    const unsigned long long st_w0 = __builtin_amdgcn_s_memtime();
#endif
    while (__hip_atomic_load(&ctl->ready[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) !=
               (uint32_t)kc + 1u &&
           ++spins < (1 << 20))
      __builtin_amdgcn_s_sleep(2);
    if (spins >= (1 << 20)) {
      if (lane == 0 && p.sched)
        __hip_atomic_store(p.sched + SCHED_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
#ifdef ME_STAMPS
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_spin += now - st_w0;
      if (!st_first) st_first = now;
      st_n++;
    }
#endif
    const Item& it = itc;
    uint8_t* buf = smem + slot * slot_bytes;
    const uint32_t* cur_lds = reinterpret_cast<const uint32_t*>(buf + g.tile_bytes);
    const uint32_t tile_off = (uint32_t)(slot * slot_bytes);
    const int G = g.groups;
    const int t = (int)q - basec;
    const int i = 64 * t + lane;
    const int T = nwc * 64;  // lanes past the item's tasks are masked below
    const int dymin = max(-S, -it.tly), dymax = min(S, p.height - it.h - it.tly);
    const int lc1 = min(it.nch, (dymax + S) / K + 1);
    const int valid_lanes = (lc1 - lc0c) * it.nb * G;
    const bool live = i < valid_lanes;
    (void)T;
    const int ii = live ? i : 0;
    const int bg = (int)__umulhi((uint32_t)ii, g.magic_groups);  // ii / G
    const int gi = ii - bg * G;
    const uint32_t magic_nb = 0xFFFFFFFFu / (uint32_t)it.nb + 1u;
    const int lcr = it.nb == 1 ? bg : (int)__umulhi((uint32_t)bg, magic_nb);
    const int b = bg - lcr * it.nb;
    const int lc = lc0c + lcr;
    const int d0 = lc * K;
    const int tlx = (it.bx0 + b) * B;
    uint32_t c[B][CW];
#pragma unroll
    for (int y = 0; y < B; y++) {
      if constexpr (CW == 4) {
        const uint4 v = reinterpret_cast<const uint4*>(cur_lds)[b * B + y];
        c[y][0] = v.x; c[y][1] = v.y; c[y][2] = v.z; c[y][3] = v.w;
      } else {
        const uint2 v = reinterpret_cast<const uint2*>(cur_lds)[b * B + y];
        c[y][0] = v.x; c[y][1] = v.y;
      }
    }
    const int dxmin = max(-S, -tlx), dxmax = min(S, p.width - B - tlx);
    const int jlo = dymin + S - d0, jhi = dymax + S - d0;
    const bool full_rows = dymin + S <= 0 && dymax + S >= it.nch * K - 1;
    const int w0 = (b * B) / 4 + gi;
    uint64_t acc[K];
    const int jt = gi < K ? gi : K - 1;
    const uint32_t toff = tile_off + (uint32_t)((lc * K + jt) * g.pitch + b * B + 2 * S);
    uint32_t tsad = 0;
    // Fairness: the SIMD arbiter issues the oldest waves first, so a young
    // wave's wave-task lags while older waves run through later items (single
    // 1080p frames: per SIMD one wave ran ~6 wave-tasks, two ran 1 each), and
    // the slot refill that waits for it stalls every wave behind the ring.
    // Every 4 rows the wave compares its task with the pull counter and raises
    // its priority once lo / hi later tasks have been pulled (g.fair; back to
    // 0 at its next pull).  Only in launches with refills: without them (a
    // single 1080p frame, every tile staged at the start) the oldest-first
    // order ends the launch sooner (70.4 vs 74.7 us with the check on,
    // profiles/r03ad_*).  Tuning build, g.fair bits 16-17 (ME_FAIR): 2 = only
    // on items whose slot still gets a refill, 3 = on every item.
    const int fmode = g.fair >> 16;
    const bool fair = g.fair != 0 && (fmode == 3 || (fmode == 2 ? kc + NB < nitems : nitems > NB));
    // pull-counter values that raise the priority (two SGPRs across the rows)
    const int lim1 = __builtin_amdgcn_readfirstlane(fair ? (int)q + (g.fair & 255) : 0x7FFFFFFF);
    const int lim2 = __builtin_amdgcn_readfirstlane(fair ? (int)q + ((g.fair >> 8) & 255) : 0x7FFFFFFF);
    // The compare and s_setprio sit in one asm block: as C branches they split
    // the unrolled row loop into basic blocks, and it spilled 41 VGPRs.
    auto lag_check = [lim1, lim2, ctl]() {
      const int nx = __builtin_amdgcn_readfirstlane(
          (int)__hip_atomic_load(&ctl->next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      asm volatile(
          "s_cmp_ge_i32 %0, %2\n\t"
          "s_cbranch_scc0 1f\n\t"
          "s_setprio 2\n\t"
          "s_branch 2f\n"
          "1:\n\t"
          "s_cmp_ge_i32 %0, %1\n\t"
          "s_cbranch_scc0 2f\n\t"
          "s_setprio 1\n"
          "2:" ::"s"(nx), "s"(lim1), "s"(lim2) : "scc");
    };
    if (it.h == B) {
      qsad_lane<B, K, B, PC, 4>(smem, g.pitch, tile_off, lc * K, w0, c, acc, lag_check);
      if (g.fold) tsad = tail_sad<B, B>(smem, g.pitch, toff, c);
    } else {
      qsad_lane<B, K, B / 2, PC, 4>(smem, g.pitch, tile_off, lc * K, w0, c, acc, lag_check);
      if (g.fold) tsad = tail_sad<B, B / 2>(smem, g.pitch, toff, c);
    }
    const int dxg = 4 * gi - S - it.a;
    const bool edge = dxg < dxmin || dxg + 3 > dxmax || !live;
    uint32_t best;
    if (full_rows && __builtin_amdgcn_ballot_w64(edge) == 0) {
      best = lane_best<K, false>(acc, 0u, 0u, jlo, jhi);
    } else {
      uint32_t mlo = 0, mhi = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int dx = dxg + k;
        const uint32_t msk = (dx < dxmin || dx > dxmax) ? 0xFFFFu : 0u;
        if (k < 2) mlo |= msk << (16 * k);
        else mhi |= msk << (16 * (k - 2));
      }
      best = lane_best<K, true>(acc, mlo, mhi, jlo, jhi);
    }
    if (g.fold) {
      const bool tv = gi < K && jt >= jlo && jt <= jhi && S <= dxmax;
      best = min(best, tv ? (tsad << 16) | (uint32_t)(5 * jt + 4) : ~0u);
    }
    if (live && best < 0xFFFF0000u) {
      const int idx = (int)(best & 0xFFFFu), jj = idx / 5, k5 = idx - 5 * jj;
      const int dy = d0 + jj - S, dx = k5 == 4 ? S : 4 * gi + k5 - S - it.a;
      atomicMin(reinterpret_cast<unsigned long long*>(&keys[slot * g.tb + b]),
                (unsigned long long)make_key(best >> 16, dx, dy));
    }
    // this wave-task is done; the last one of the item writes and refills the slot
    uint32_t prev = 0;
    if (lane == 0)
      prev = __hip_atomic_fetch_add(&ctl->done[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = (uint32_t)__builtin_amdgcn_readfirstlane((int)prev);
    if ((int)prev + 1 == nwc) {
      if (lane < it.nb) {
        const uint64_t kk = keys[slot * g.tb + lane];
        keys[slot * g.tb + lane] = ~0ull;
        const int out = (it.by - jb.r0[it.j]) * p.nbx + it.bx0 + lane;
        int16_t* mv = jb.mv[it.j];
        store_mv(mv, out, kk);
        if (jb.cost[it.j]) jb.cost[it.j][out] = (uint32_t)(kk >> 32);
      }
      if (lane == 0) __hip_atomic_store(&ctl->done[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int kn = kc + NB;
      if (kn < nitems) {
        if (g.prio) __builtin_amdgcn_s_setprio(3);
        stage_item_wave<B>(p, g, flow_item<B, K>(p, g, jb, tile_of(kn)), buf, jb);
        if (g.prio) __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store(&ctl->ready[slot], (uint32_t)kn + 1u, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
#ifdef ME_STAMPS
  if (lane == 0 && fw < (1 << 16)) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned long long* o = g_stamps + 8 * fw;
    o[0] = st_t0; o[1] = st_first; o[2] = __builtin_amdgcn_s_memtime(); o[3] = st_spin;
    o[4] = st_n; o[5] = st_r0; o[6] = __builtin_amdgcn_s_memrealtime(); o[7] = hw;
  }
#endif
}

// ------------------------------------------------------------------ launch
static int generic_lds_bytes(const SearchArgs& p, int* win_bytes) {
  const int B = p.blk;
  long win = (long)(B + 2 * p.range) * (B + 2 * p.range);
  const int cur = (B * B + 15) & ~15;
  if (cur + win > GENERIC_LDS_BUDGET) win = 0;  // read the window from global memory
  *win_bytes = (int)win;
  return cur + (int)win;
}

hipError_t launch_generic(const SearchArgs& p, int bx0, int nbx_range, int row0, int nrows,
                          hipStream_t stream) {
  if (nbx_range <= 0 || nrows <= 0) return hipSuccess;
  int win = 0;
  const int lds = generic_lds_bytes(p, &win);
  dim3 grid((unsigned)(nbx_range * nrows)), block(GENERIC_THREADS);
  if (p.cost_kind == COST_SAD)
    hipLaunchKernelGGL(me_generic_kernel<COST_SAD>, grid, block, lds, stream, p, bx0, nbx_range,
                       row0, win);
  else
    hipLaunchKernelGGL(me_generic_kernel<COST_SSD>, grid, block, lds, stream, p, bx0, nbx_range,
                       row0, win);
  return hipGetLastError();
}

// Plan the fast kernels.  SAD lanes own 4 dx (one qsad group), SSD lanes one
// dx; both own K dy.  Search (fold, K, TB, chunks per pass) for the most
// useful work per wave-task (dy padding, the masked 4th column of the last
// SAD group or the fold's extra column, idle lanes of partly filled waves)
// within the LDS budget; then prefer fewer passes and smaller tiles (finer
// work items).  256 threads per workgroup: 4 workgroups of 4 waves per CU at
// the kernels' <= 128 VGPRs.
static int cu_count();

bool plan_fast(const SearchArgs& p, QsadGeom* g, int* k_out) {
  const int B = p.blk, S = p.range;
  if (B != 16 && B != 8) return false;
  if (S < 1 || S > 255) return false;
  g->nbx_full = p.width / B;
  if (g->nbx_full < 1) return false;
  const bool sad = p.cost_kind == COST_SAD;
  const int D = 2 * S + 1;
  const int CW = B / 4;
  // Fold needs a = 0 (S % 4 == 0) and the tail words of every block aligned
  // for one ds_read of B bytes (b*B + 2S multiple of B: S % 8 == 0 for B = 16).
  const bool fold_ok = sad && S % 4 == 0 && (B == 8 || S % 8 == 0);
  // SAD rows carry an alignment word for a = (tlx - S) mod 4 <= 3; with S % 4
  // == 0 (tlx a multiple of B) a = 0 and the lanes read exactly 4G + B bytes
  // past the block's first tile column: no word (1080p tb = 3 rows 112 instead
  // of 144 bytes; the 2- and 4-way stripe times moved within box-to-box
  // noise, profiles/r02al_stripe_sweeps.jsonl)
  const int aw = S % 4 == 0 ? 0 : 4;
  static const int Ks[] = {26, 13, 11, 8, 5};
  // K = 26 (8x8 SAD): twice the candidates per lane-task, so the task decode,
  // cur loads, fold column and key merge are paid per 104 candidates, not 52
  // (8K +-128: 18.23 -> 17.40 ms, tb 8 at the compiled pitch 336;
  // profiles/r03ar_plan_8k.jsonl)
  const bool k26_auto = sad && B == 8;
  // K = 5 (a quarter-size wave-task) only for SAD searches too small to give
  // every SIMD two K = 13 wave-tasks (an 8-way 1080p stripe: 1.25 per SIMD, so
  // a quarter of the SIMDs ran a second round); K >= 8 otherwise.
  bool small = false;
  if (sad) {
    const int G13 = S % 4 == 0 && (B == 8 || S % 8 == 0) ? S / 2 : (2 * S + 3 + 1 + 3) / 4;
    const double lanes = (double)(p.block_row_end - p.block_row_begin) * (p.width / B) * G13 *
                         ((D + 12) / 13);
    small = lanes / 64.0 < 2.0 * 4 * cu_count();
  }
  // Tuning build override (tools/plan_sweep.py): ME_PLAN="K,tb,cpp,threads[,fold]",
  // validated in me_api.hip; 0 = free (fold: -1 = free).
  const Tuning& tu = tuning();
  const int force[5] = {tu.plan_k, tu.plan_tb, tu.plan_cpp, tu.plan_threads, tu.plan_fold};
  const int thr = force[3] > 0 ? force[3] : 256;
  const int rows = p.block_row_end - p.block_row_begin;
  double best = -1;
  int bK = 13, bTB = 1, bC = 1, bF = 0, bG = 1;
  for (int fold = 0; fold <= 1; fold++) {
    if (fold && !fold_ok) continue;
    if (force[4] >= 0 && fold != force[4]) continue;
    // SAD: worst case a = 3 without fold
    const int G = sad ? (fold ? S / 2 : (2 * S + 3 + 1 + 3) / 4) : D;
    // useful share of a lane's candidates (the last group's padding), and the
    // fold's extra cost per task (one B-row v_sad_u8 column + its key)
    const double use_dx = sad ? (fold ? 1.0 : (double)D / (4.0 * G)) : 1.0;
    for (int K : Ks) {
      if (force[0] && K != force[0]) continue;
      // (K = 5 is instantiated for 16x16 SAD only: other small searches keep K >= 8;
      // K = 26 for 8x8 SAD only)
      if (K == 5 && (!sad || B != 16)) continue;
      if (K == 26 && (!sad || B != 8 || (!force[0] && !k26_auto))) continue;
      if (!force[0] && (K == 5) != (small && B == 16)) continue;
      if (fold && G < K) continue;
      const int chunks = (D + K - 1) / K;
      if (K == 5 && !force[0]) {
        // small search: one block per tile, every chunk in one pass, so each
        // block is its own workgroup item (1,020 of them in an 8-way 1080p
        // stripe: about one quarter-size wave-task per wave, all SIMDs busy).
        // No fold (17 groups): the fold's narrower rows measured slower here
        // (9-row stripe 20.2 vs 19.65 us, CIF +-16 12.4 vs 11.05 us,
        // profiles/r02am_small_plan_fold.txt).
        const int pt0 = ((sad ? 4 * G + B + aw : 2 * S + 1 + 3 + B + 4) + 15) & ~15;
        const int pt = ((pt0 >> 4) & 1) ? pt0 : pt0 + 16;
        const long lds = 128 + 2 * ((long)B * B + (long)(chunks * K + B - 1) * pt);
        if (lds <= QSAD_LDS_BUDGET && best < 0) {
          best = 1.0; bK = K; bTB = 1; bC = chunks; bF = fold; bG = G;
        }
        continue;
      }
      const double kpad = (double)D / (chunks * K);
      const double tail = fold ? 0.5 * (B * CW + 16) / (K * B * CW * 4 + 340) : 0.0;
      // Waves that hold whole (block, chunk) groups (64 % G == 0 or G % 64
      // == 0) read one cur block and share one row range per wave: measured
      // ~5 % faster than waves straddling blocks (8K B8: G 64 vs 65).
      const double wave_align = (64 % G == 0 || G % 64 == 0) ? 1.03 : 1.0;
      for (int tb = 1; tb <= 16; tb++) {
        if (force[1] && tb != force[1]) continue;
        // One-block tiles restage a whole window per block and leave waves of
        // every item part empty: measured slower than two-block tiles wherever
        // both fit (1080p: 171 vs 121 us static; 4K block rows 0..17, the edge
        // stripe of an 8-way split: 0.228 vs 0.188 ms; profiles/r02h_dyn.jsonl).
        if (tb == 1 && !force[1] && g->nbx_full >= 2) continue;
        // bytes the lanes touch per row (+ a <= 3, + alignment word)
        const int width = (tb - 1) * B + (sad ? 4 * G + B + aw : 2 * S + 1 + 3 + B + 4);
        int pt = (width + 15) & ~15;
        if (((pt >> 4) & 1) == 0) pt += 16;
        for (int cpp = chunks; cpp >= 1; cpp--) {
          if (force[2] && cpp != force[2]) continue;
          const long lds = 128 + 2 * ((long)tb * B * B + (long)(cpp * K + B - 1) * pt);
          if (lds > QSAD_LDS_BUDGET) continue;
          int passes = 0;
          for (int c0 = 0; c0 < chunks; c0 += cpp) passes++;
          const long items = (long)((g->nbx_full + tb - 1) / tb) * rows * passes;
          // Cost of an item in wave-tasks: its waves (a partly filled wave
          // costs a whole one), for SAD half of the wave slots its last round of
          // `thr` lanes leaves idle (the CU's other workgroups take up the
          // rest: 4K +-64, 68 block rows, tb 5 = 10 waves in rounds of 4:
          // 0.637 ms against tb 8's 0.570, profiles/r02aa_plan_sweep_4k_68rows.jsonl),
          // + ~0.45 for staging, barrier and output (fitted on
          // tools/plan_sweep.py runs).  With few items per workgroup (< 8 of
          // 1024) a partial last round is not amortised at all: whole rounds.
          const bool many = items >= 8L * 1024;
          double cost = 0, useful = 0;
          for (int c0 = 0; c0 < chunks; c0 += cpp) {
            const int t = tb * G * (chunks - c0 < cpp ? chunks - c0 : cpp);
            const int rounds = (t + thr - 1) / thr;
            const int waves = (t + 63) / 64, idle = rounds * (thr / 64) - waves;
            // few items: every extra round lengthens the kernel's tail too
            cost += (many ? waves + (sad ? 0.5 * idle : 0.0) : rounds * (thr / 64) + 0.5 * (rounds - 1)) + 0.45;
            useful += t / 64.0;
          }
          // Workgroups take whole tiles (every pass of a tile runs on the
          // workgroup holding its keys): too few tiles leave workgroup slots
          // idle (and nothing to prefetch): aim for >= 2 tiles per resident
          // workgroup (4 per CU).
          const long tiles = items / passes;
          const double fill = tiles >= 2048 ? 1.0 : (double)tiles / 2048;
          // K = 13 measured best wherever it fits (more candidates per row load
          // and per epilogue than the padding it costs).
          // K = 26 over K = 13 where it fits (8x8 SAD), at the compiled tile
          // pitch 336 if a tb gives it (tb 8: 17.40 ms; tb 12 / 16 at runtime
          // pitches 17.68 / 17.64 ms)
          const double kpref = K == 26 ? (pt == 336 ? 1.05 : 1.03) : K == 13 ? 1.0 : 0.95;
          // the last tile of a block row holds nbx_full % tb blocks
          const double tile_fill =
              (double)g->nbx_full / ((double)((g->nbx_full + tb - 1) / tb) * tb);
          const double score = kpad * kpref * wave_align * tile_fill * use_dx / (1.0 + tail) * useful / cost *
                               (0.7 + 0.3 * fill) - 0.002 * tb;
          if (score > best + 1e-9) {
            best = score; bK = K; bTB = tb; bC = cpp; bF = fold; bG = G;
          }
        }
      }
    }
  }
  if (best < 0) return false;  // nothing fits (only with an ME_PLAN override)
  g->fold = bF;
  g->groups = bG;
  // Dynamic tile pulls from this many tiles per workgroup on (ME_DYN overrides
  // in the tuning build; 0 = static bands only).
  {
    const int dyn_env = tu.dyn;
    // 3: measured (tools/dyn_sweep.sh) -- 4K (3.96 tiles/WG) and 8K gain
    // (8K -11 % with stealing), 1080p (2.7 tiles/WG) loses: its workgroups
    // start items in lockstep and the item-start pulls serialise on the
    // device-scope counters while wave 0 waits.
    g->dyn_tiles = dyn_env >= 0 ? dyn_env : 3;
    // ... and only for tiles of >= 16 wave-tasks: small tiles pay the pull per
    // few tasks (1080p tb = 2: 184 vs 121 us static; profiles/r02h_dyn.jsonl).
    const long tile_lanes = (long)bTB * bG * ((D + bK - 1) / bK);
    if (dyn_env < 0 && tile_lanes < 16L * 64) g->dyn_tiles = 0;
  }
  g->tb = bTB;
  g->cpp = bC;
  g->chunks = (D + bK - 1) / bK;
  // recompute the pitch of the chosen tb
  {
    const int width = (g->tb - 1) * B + (sad ? 4 * g->groups + B + aw : 2 * S + 1 + 3 + B + 4);
    int pt = (width + 15) & ~15;
    if (((pt >> 4) & 1) == 0) pt += 16;
    g->pitch = pt;
  }
  g->rows_alloc = g->cpp * bK + B - 1;
  g->tile_bytes = g->rows_alloc * g->pitch;
  g->threads = thr;
  g->lds = 2 * (g->tile_bytes + g->tb * B * B) + 128 + 16;
  // r = umulhi(d, magic) == d / pitch for every staged offset d (checked).
  g->pitch_magic = (uint32_t)(0x100000000ull / (uint64_t)g->pitch) + 1u;
  for (uint32_t d = 0; d < (uint32_t)g->tile_bytes; d += 4)
    if ((uint32_t)(((uint64_t)d * g->pitch_magic) >> 32) != d / (uint32_t)g->pitch) return false;
  g->wg_per_row = (g->nbx_full + g->tb - 1) / g->tb;
  {
    // t / wg_per_row by multiply-high for every tile index of these rows
    const uint32_t d = (uint32_t)g->wg_per_row, m = 0xFFFFFFFFu / d + 1u;
    const uint32_t nt = (uint32_t)g->wg_per_row * (uint32_t)(rows > 0 ? rows : 1);
    g->magic_wpr = m;
    for (uint32_t t = 0; t < nt; t++)
      if ((uint32_t)(((uint64_t)t * m) >> 32) != t / d) {
        g->magic_wpr = 0;
        break;
      }
    g->magic_tb = 0xFFFFFFFFu / (uint32_t)g->tb + 1u;
  }
  g->aligned = (p.stride % 4 == 0) && ((uintptr_t)p.ref % 4 == 0) && ((uintptr_t)p.cur % 4 == 0);
  // X0 = tb*B*t - S - a is 16-aligned for every tile when a = 0 (S % 4 == 0),
  // S % 16 == 0 and tb * B % 16 == 0; rows of the ref plane 16-aligned; W % 16
  // == 0 keeps the last in-frame granule of the last row inside the range.
  g->tile16 = g->aligned && S % 16 == 0 && (g->tb * B) % 16 == 0 && p.width % 16 == 0 &&
              p.stride % 16 == 0 && (uintptr_t)p.ref % 16 == 0;
  // umulhi(t, magic_groups) == t / groups for every task index of an item.
  g->magic_groups = 0xFFFFFFFFu / (uint32_t)g->groups + 1u;
  const uint32_t tmax = (uint32_t)(g->tb * g->groups * g->cpp);
  for (uint32_t t = 0; t < tmax; t++)
    if ((uint32_t)(((uint64_t)t * g->magic_groups) >> 32) != t / (uint32_t)g->groups) return false;
  for (uint32_t nb = 1; nb <= (uint32_t)g->tb; nb++) {  // per-item / nb, bg < tb * cpp
    const uint32_t m = 0xFFFFFFFFu / nb + 1u;
    for (uint32_t x = 0; x < (uint32_t)(g->tb * g->cpp); x++)
      if (nb > 1 && (uint32_t)(((uint64_t)x * m) >> 32) != x / nb) return false;
  }
  g->prio = tu.prio != 0;
  g->fair = 0;
  g->flow_slots = 0;
  // Wide frames: vertical strips of 16 tiles (8K 8x8: 1,024 pixels plus the
  // window's 2S), so an XCD's contiguous run of the order is a few whole
  // strips and its L2 holds a strip's window rows while they are reread
  // (the row-major order fetched 2.4x the algorithmic bytes at 8K SAD).
  g->strip_w = g->wg_per_row >= 32 && rows >= 32 ? 16 : 0;
  if (tu.strip >= 0) g->strip_w = tu.strip;
  // Dynamic pulls claim a workgroup's next tile when its current one starts if
  // a tile has >= 2 passes (the id is read at the last pass, a barrier later),
  // else two tiles ahead.  Claimed-but-unstarted tiles widen the band of rows
  // an XCD's workgroups touch at once: ahead = 2 at 4K +-64 (128 workgroups
  // per XCD, 3 passes) fetched 1.35x the compulsory bytes, ahead = 1
  // 1.11x, at the same time (profiles/r04l_variants_4k.txt).
  g->pull_ahead = (g->chunks + g->cpp - 1) / g->cpp >= 2 ? 1 : 2;
  if (tu.ahead > 0 && (tu.ahead == 2 || g->pull_ahead == 1)) g->pull_ahead = tu.ahead;
  *k_out = bK;
  return true;
}

// The flow kernel (SAD, 16x16, S = 32, one 1,024-thread workgroup per CU): tiles of tb
// blocks with all their dy chunks, tb * G * chunks a multiple of 64 (every
// wave-task full), a ring of >= 4 slots in LDS, the ref tile in 16-byte
// granules, and >= 2 tiles per CU (fewer leave most of the 16 waves idle: the
// persistent item kernel takes small stripes).
static constexpr int FLOW_LDS = 160 * 1024 - 1024;

static int cu_count();

bool plan_flow(const SearchArgs& p, QsadGeom* g) {
  const int B = p.blk, S = p.range;
  if (p.cost_kind != COST_SAD || B != 16) return false;
  // fold (S % 8) and 16-byte tile granules (S % 16).  S <= 32: at 4K +-64 the
  // item kernel's items are already whole waves (8 blocks x 4 chunks x 32
  // groups) and it measured faster (1.086 vs 1.12 ms, profiles/r02p_flow_sweep.txt).
  // The fold spreads the dx = +S column over lanes gi < K: G = S/2 >= K.
  if (S < 16 || S % 16 || S > 32) return false;
  if (tuning().flow == 0) return false;
  const int nbx_full = p.width / B;
  if (nbx_full < 1 || p.width % 16 || p.stride % 16 || (uintptr_t)p.ref % 16 || (uintptr_t)p.cur % 16)
    return false;
  const int D = 2 * S + 1, G = S / 2;
  const int rows = p.block_row_end - p.block_row_begin;  // launch_jobs: every job's rows
  const int cus = cu_count();
  auto pitch_of = [&](int tb) {
    int pt = ((tb - 1) * B + 4 * G + B + 4 + 15) & ~15;
    if (((pt >> 4) & 1) == 0) pt += 16;
    return pt;
  };
  auto slots_of = [&](int tb, int K) {
    const int chunks = (D + K - 1) / K;
    const int slot = (chunks * K + B - 1) * pitch_of(tb) + tb * B * B;
    return min(16, (FLOW_LDS - 16 * tb * 8 - (int)sizeof(int) * 40) / slot);
  };
  // K = 13, whole tiles per CU, XCD-banded: the widest tile that still gives
  // >= 6 tiles per CU (fine enough for the CUs to finish together), else the
  // narrowest with >= 2 per CU (fewer leave most of the 16 waves idle: the
  // persistent item kernel takes small stripes).
  const int K = 13;
  int best_tb = 0, best_ns = 0;
  if (G >= 13) {
    const int chunks = (D + 12) / 13;
    int fine_tb = 0, fine_ns = 0;
    for (int tb = 1; tb <= 8; tb++) {
      if ((tb * G * chunks) % 64) continue;
      if (tuning().plan_tb && tb != tuning().plan_tb) continue;  // tuning build
      const int ns = slots_of(tb, 13);
      const long tiles = (long)((nbx_full + tb - 1) / tb) * rows;
      if (ns < 4 || tiles < 2L * cus) continue;
      if (!best_tb) {
        best_tb = tb;
        best_ns = ns;
      }
      if (tiles >= 6L * cus) {
        fine_tb = tb;
        fine_ns = ns;
      }
    }
    if (fine_tb) {
      best_tb = fine_tb;
      best_ns = fine_ns;
    }
    // tb = 4 (the 144-byte pitch compiled into the kernel: row addresses in
    // the ds_read2 offsets) whenever it gives >= 6 tiles per CU: a batch of
    // 8 1080p frames took tb = 8 at the runtime pitch, 84 us per frame
    // against 69-78 for single frames (profiles/r03j_*)
    const long tiles4 = (long)((nbx_full + 3) / 4) * rows;
    if (best_tb != 4 && (4 * G * chunks) % 64 == 0 && pitch_of(4) == 144 && slots_of(4, 13) >= 4 &&
        tiles4 >= 6L * cus && !tuning().plan_tb) {
      best_tb = 4;
      best_ns = slots_of(4, 13);
    }
  }
  if (!best_tb) return false;
  const int chunks = (D + K - 1) / K;
  QsadGeom& q = *g;
  q.tb = best_tb;
  q.groups = G;
  q.chunks = chunks;
  q.cpp = chunks;
  q.fold = 1;
  q.nbx_full = nbx_full;
  q.pitch = pitch_of(q.tb);
  q.rows_alloc = chunks * K + B - 1;
  q.tile_bytes = q.rows_alloc * q.pitch;
  q.wg_per_row = (nbx_full + q.tb - 1) / q.tb;
  q.magic_wpr = 0;  // the flow kernel maps a tile once per item: plain division
  q.magic_tb = 0xFFFFFFFFu / (uint32_t)q.tb + 1u;
  q.aligned = 1;
  q.tile16 = 1;
  q.threads = 1024;
  q.dyn_tiles = 0;
  q.pull_ahead = 2;
  q.pitch_magic = (uint32_t)(0x100000000ull / (uint64_t)q.pitch) + 1u;
  for (uint32_t d = 0; d < (uint32_t)q.tile_bytes; d += 16)
    if ((uint32_t)(((uint64_t)d * q.pitch_magic) >> 32) != d / (uint32_t)q.pitch) return false;
  q.magic_groups = 0xFFFFFFFFu / (uint32_t)G + 1u;
  for (uint32_t t = 0; t < (uint32_t)(q.tb * G * chunks); t++)
    if ((uint32_t)(((uint64_t)t * q.magic_groups) >> 32) != t / (uint32_t)G) return false;
  for (uint32_t nb = 2; nb <= (uint32_t)q.tb; nb++) {
    const uint32_t mg = 0xFFFFFFFFu / nb + 1u;
    for (uint32_t xx = 0; xx < (uint32_t)(q.tb * chunks); xx++)
      if ((uint32_t)(((uint64_t)xx * mg) >> 32) != xx / nb) return false;
  }
  const int slot = q.tile_bytes + q.tb * B * B;
  if (tuning().flow_slots && tuning().flow_slots < best_ns) best_ns = tuning().flow_slots;
  q.flow_slots = best_ns;
  q.prio = tuning().prio != 0;
  q.fair = tuning().fair != 0
               ? (tuning().fair_lo | tuning().fair_hi << 8 | (tuning().fair > 1 ? tuning().fair : 1) << 16)
               : 0;
  q.strip_w = 0;
  q.lds = best_ns * slot + best_ns * q.tb * 8 + (int)sizeof(int) * 40;
  return q.lds <= 160 * 1024;
}

// Per-kernel launch facts, computed once per (kernel, device[, shape]) and
// shared by every host thread (a mutex-protected list: the per-device threads
// of multi_search and me_search_pairs plan and launch concurrently).  Setting
// the dynamic-LDS attribute and querying occupancy on every launch cost host
// time on the small-stripe step, which is host-bound.
namespace {
struct LaunchFact {
  const void* fn;
  int dev, threads, lds, value;  // threads == 0: the LDS attribute entry (value = max set)
};
std::mutex g_fact_mu;
std::vector<LaunchFact> g_facts;

int current_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}
}  // namespace

hipError_t lds_attr(const void* fn, int lds) {
  if (lds <= 64 * 1024) return hipSuccess;
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_fact_mu);
  for (LaunchFact& f : g_facts)
    if (f.fn == fn && f.dev == dev && f.threads == 0) {
      if (f.value >= lds) return hipSuccess;
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      if (e == hipSuccess) f.value = lds;
      return e;
    }
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e == hipSuccess) g_facts.push_back({fn, dev, 0, 0, lds});
  return e;
}

// Resident workgroups per CU for this kernel / block / LDS.
static int resident_wgs(const void* fn, int threads, int lds) {
  const int dev = current_device();
  {
    std::lock_guard<std::mutex> lk(g_fact_mu);
    for (const LaunchFact& f : g_facts)
      if (f.fn == fn && f.dev == dev && f.threads == threads && f.lds == lds) return f.value;
  }
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, lds) != hipSuccess || n < 1)
    n = 1;
  std::lock_guard<std::mutex> lk(g_fact_mu);
  g_facts.push_back({fn, dev, threads, lds, n});
  return n;
}

// CUs of the device (every device of a context is the same part): a C++11
// function-local static, initialised once and thread-safely (multi_search and
// me_search_pairs call the planners from one host thread per device).
static int cu_count() {
  static const int cus = []() {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  return cus;
}

// One item-kernel launch over the job table jb (full-height rows and h = B/2
// bottom rows; every job the geometry g was planned for).
static hipError_t launch_fast(const SearchArgs& p, QsadGeom g, int K, const FlowJobs& jb,
                              hipStream_t stream) {
  const int ntiles = jb.tile_pre[jb.n];
  if (ntiles <= 0) return hipSuccess;
  g.row0 = 0;
  g.nrows = 0;  // per job (jb.r0, jb.tile_pre)
  dim3 block((unsigned)g.threads);
// PP > 0: the instance with that compile-time tile pitch (row addresses in the
// ds_read2 offset fields), taken when the plan has exactly that pitch.
#define ME_FAST_CASE_P(CC, BB, KK, PP)                                                     \
  if (p.cost_kind == CC && p.blk == BB && K == KK && (PP == 0 || g.pitch == PP)) {         \
    const void* fn = (const void*)me_fast_kernel<CC, BB, KK, PP>;                         \
    const hipError_t e_ = lds_attr(fn, g.lds);                                             \
    if (e_ != hipSuccess) return e_;                                                       \
    int res = resident_wgs(fn, g.threads, g.lds);                                          \
    if (tuning().fast_res > 0 && tuning().fast_res < res) res = tuning().fast_res;         \
    const int nwg = ntiles < res * cu_count() ? ntiles : res * cu_count();                 \
    hipLaunchKernelGGL((me_fast_kernel<CC, BB, KK, PP>), dim3((unsigned)nwg), block, g.lds, stream, p, g, jb); \
    return hipGetLastError();                                                              \
  }
#define ME_FAST_CASE(CC, BB, KK) ME_FAST_CASE_P(CC, BB, KK, 0)
  // the plans' pitches of 4K +-64 (tb 8: 272; 1.098 -> 1.085 ms) and 8K 8x8
  // +-128 (tb 8: 336; 18.59 -> 18.19 ms); the 1080p stripes' pitches (144,
  // 112) measured no better (profiles/r02ah_ab_item_pitch.txt)
  ME_FAST_CASE_P(COST_SAD, 16, 13, 272) ME_FAST_CASE_P(COST_SAD, 8, 13, 336)
  ME_FAST_CASE(COST_SAD, 16, 13) ME_FAST_CASE(COST_SAD, 16, 11) ME_FAST_CASE(COST_SAD, 16, 8)
  ME_FAST_CASE(COST_SAD, 16, 5)
  ME_FAST_CASE(COST_SAD, 8, 13) ME_FAST_CASE(COST_SAD, 8, 11) ME_FAST_CASE(COST_SAD, 8, 8)
  ME_FAST_CASE_P(COST_SAD, 8, 26, 336) ME_FAST_CASE(COST_SAD, 8, 26)
  ME_FAST_CASE(COST_SSD, 16, 13) ME_FAST_CASE(COST_SSD, 16, 11) ME_FAST_CASE(COST_SSD, 16, 8)
  ME_FAST_CASE(COST_SSD, 8, 13) ME_FAST_CASE(COST_SSD, 8, 11) ME_FAST_CASE(COST_SSD, 8, 8)
#undef ME_FAST_CASE
#undef ME_FAST_CASE_P
  return hipErrorInvalidValue;
}

// Plans depend only on the search shape: cache them (process-wide, under a
// mutex: the per-device threads of multi_search and me_search_pairs share
// them) so a steady stream of same-shape searches pays the planner once.
struct PlanKey {
  int width, height, stride, blk, range, cost, rows, aligned;  // aligned: 1 (4 B) | 2 (16 B)
  bool operator==(const PlanKey& o) const {
    return width == o.width && height == o.height && stride == o.stride && blk == o.blk &&
           range == o.range && cost == o.cost && rows == o.rows && aligned == o.aligned;
  }
};
struct PlanEntry {
  PlanKey key;
  bool ok;
  QsadGeom g;
  int K;
};

static bool cached_plan(const SearchArgs& p, QsadGeom* g, int* K) {
  constexpr int N = 8;
  static PlanEntry cache[N];
  static int used = 0, next = 0;
  static std::mutex mu;
  const int aligned =
      ((p.stride % 4 == 0) && ((uintptr_t)p.ref % 4 == 0) && ((uintptr_t)p.cur % 4 == 0)) |
      (((p.stride % 16 == 0) && ((uintptr_t)p.ref % 16 == 0)) << 1);
  const PlanKey key{p.width, p.height, p.stride, p.blk, p.range, p.cost_kind,
                    p.block_row_end - p.block_row_begin, aligned};
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < used; i++)
    if (cache[i].key == key) {
      *g = cache[i].g;
      *K = cache[i].K;
      return cache[i].ok;
    }
  PlanEntry e;
  e.key = key;
  e.ok = plan_fast(p, &e.g, &e.K);
  cache[next] = e;
  next = (next + 1) % N;
  if (used < N) used++;
  *g = e.g;
  *K = e.K;
  return e.ok;
}

static bool cached_flow_plan(const SearchArgs& p, QsadGeom* g) {
  constexpr int N = 8;
  static PlanEntry cache[N];
  static int used = 0, next = 0;
  static std::mutex mu;
  const int aligned = ((p.stride % 16 == 0) && ((uintptr_t)p.ref % 16 == 0) &&
                       ((uintptr_t)p.cur % 16 == 0)) ? 3 : 0;
  const PlanKey key{p.width, p.height, p.stride, p.blk, p.range, p.cost_kind,
                    p.block_row_end - p.block_row_begin, aligned};
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < used; i++)
    if (cache[i].key == key) {
      *g = cache[i].g;
      return cache[i].ok;
    }
  PlanEntry e;
  e.key = key;
  e.ok = plan_flow(p, &e.g);
  e.K = 13;
  cache[next] = e;
  next = (next + 1) % N;
  if (used < N) used++;
  *g = e.g;
  return e.ok;
}

// The job table of jobs [0, n) (n <= MAX_JOBS; rows [r0, r1) each, already
// cut to what the kernel takes), wg_per_row tiles per block row.
static FlowJobs job_table(const SearchArgs& p, int wg_per_row, const SearchJob* jobs, int n) {
  FlowJobs jb;
  jb.n = 0;
  jb.tile_pre[0] = 0;
  const int B = p.blk, S = p.range, H = p.height;
  for (int i = 0; i < n; i++) {
    const SearchJob& J = jobs[i];
    if (J.r1 <= J.r0) continue;
    const int j = jb.n++;
    jb.r0[j] = J.r0;
    jb.ref_row0[j] = J.ref_row0;
    jb.cur_row0[j] = J.cur_row0;
    // bytes the job's descriptors may read: its resident rows (include/me.h)
    const int ref_end = J.r1 * B + S < H ? J.r1 * B + S : H, cur_end = J.r1 * B < H ? J.r1 * B : H;
    jb.ref_bytes[j] = (uint32_t)((long)(ref_end - J.ref_row0 - 1) * p.stride + p.width);
    jb.cur_bytes[j] = (uint32_t)((long)(cur_end - J.cur_row0 - 1) * p.stride + p.width);
    jb.ref[j] = J.ref;
    jb.cur[j] = J.cur;
    jb.mv[j] = J.mv;
    jb.cost[j] = J.cost;
    jb.tile_pre[j + 1] = jb.tile_pre[j] + wg_per_row * (J.r1 - J.r0);
  }
  return jb;
}

// One flow-kernel launch over jobs [0, n) (full-height rows and h = B/2
// bottom rows only; n <= MAX_JOBS).
static hipError_t launch_flow(const SearchArgs& p, QsadGeom g, const SearchJob* jobs, int n,
                              hipStream_t stream) {
  const FlowJobs jb = job_table(p, g.wg_per_row, jobs, n);
  const int ntiles = jb.tile_pre[jb.n];
  if (ntiles <= 0) return hipSuccess;
  g.row0 = 0;
  g.nrows = 0;  // per job (jb.r0)
  const int nwg = ntiles > cu_count() ? cu_count() : ntiles;  // one per CU, at most one per tile
  // 144: the pitch of the 4-block tiles 1080p +-32 gets (row addresses in
  // the ds_read2 offsets); any other pitch takes the runtime-pitch body
#define ME_FLOW_CASE(PP)                                                                        \
  if (PP == 0 || g.pitch == PP) {                                                               \
    const hipError_t e = lds_attr((const void*)me_flow_kernel<16, 13, PP>, g.lds);              \
    if (e != hipSuccess) return e;                                                              \
    hipLaunchKernelGGL((me_flow_kernel<16, 13, PP>), dim3((unsigned)nwg), dim3(1024), g.lds,    \
                       stream, p, g, jb);                                                       \
    return hipGetLastError();                                                                   \
  }
  ME_FLOW_CASE(144) ME_FLOW_CASE(0)
#undef ME_FLOW_CASE
  return hipErrorInvalidValue;
}

size_t merge_tiles_needed(const SearchArgs& p) {
  if (p.block_row_end <= p.block_row_begin) return 0;
  return p.cost_kind == COST_SSD ? mfma_merge_tiles(p) : 0;
}

// The single-job arguments of job J (geometry, cost and scratch from base).
static SearchArgs job_args(const SearchArgs& base, const SearchJob& J) {
  SearchArgs q = base;
  q.ref = J.ref;
  q.ref_row0 = J.ref_row0;
  q.cur = J.cur;
  q.cur_row0 = J.cur_row0;
  q.block_row_begin = J.r0;
  q.block_row_end = J.r1;
  q.mv = J.mv;
  q.cost = J.cost;
  const int B = base.blk, S = base.range, H = base.height;
  const int ref_end = J.r1 * B + S < H ? J.r1 * B + S : H, cur_end = J.r1 * B < H ? J.r1 * B : H;
  const long ref_rows = ref_end - J.ref_row0, cur_rows = cur_end - J.cur_row0;
  q.ref_bytes = ref_rows > 0 ? (uint32_t)((ref_rows - 1) * (long)base.stride + base.width) : 0;
  q.cur_bytes = cur_rows > 0 ? (uint32_t)((cur_rows - 1) * (long)base.stride + base.width) : 0;
  return q;
}

// End of the full-height (and h = B/2) rows of [.., r1) the qsad bodies take;
// a bottom row of another height goes to the generic kernel.
static int qsad_rows_end(const SearchArgs& p, int r1) {
  const int nby = (p.height + p.blk - 1) / p.blk;
  const int h_last = p.height - (nby - 1) * p.blk;
  return r1 == nby && h_last != p.blk && h_last != p.blk / 2 ? r1 - 1 : r1;
}

// The persistent item kernel (and the generic kernel for what it leaves).
static hipError_t launch_items(const SearchArgs& p, hipStream_t stream, int* used_fast) {
  const int r0 = p.block_row_begin, r1 = p.block_row_end;
  QsadGeom g;
  int K = 0;
  if (!cached_plan(p, &g, &K)) return launch_generic(p, 0, p.nbx, r0, r1 - r0, stream);
  const int rq1 = qsad_rows_end(p, r1);
  const SearchJob J{p.ref, p.ref_row0, p.cur, p.cur_row0, r0, rq1, p.mv, p.cost};
  hipError_t e = launch_fast(p, g, K, job_table(p, g.wg_per_row, &J, 1), stream);
  if (e != hipSuccess) return e;
  if (used_fast) *used_fast = 1;
  if (rq1 < r1) {
    e = launch_generic(p, 0, g.nbx_full, rq1, r1 - rq1, stream);
    if (e != hipSuccess) return e;
  }
  if (g.nbx_full < p.nbx)  // partial right column
    return launch_generic(p, g.nbx_full, p.nbx - g.nbx_full, r0, r1 - r0, stream);
  return hipSuccess;
}

// SAD jobs on the flow kernel where its plan (over every job's rows) takes
// them, all in one launch (MAX_JOBS jobs per launch).  Past the LDS ring a
// slot is refilled when its item's last wave-task ends; with the fairness
// check in the kernel (QsadGeom::fair) that wave-task no longer lags, and one
// launch of 8 1080p frames takes 62.5-63 us per frame against 71.4 for
// back-to-back single-frame launches on the same box (without the check:
// 80.9 us, waves spinning on unpublished slots; profiles/r03ac_fair_sweep.jsonl).
// Tuning build: ME_FLOW_ONE=0 cuts a batch into launches of about one ring.
// Returns false (nothing launched) when the flow kernel does not apply.
static bool launch_flow_jobs(const SearchArgs& base, const SearchJob* jobs, int n, hipStream_t stream,
                             hipError_t* err) {
  *err = hipSuccess;
  if (base.cost_kind != COST_SAD || n < 1) return false;
  int rows = 0;
  for (int i = 0; i < n; i++) {
    rows += jobs[i].r1 - jobs[i].r0;
    if ((uintptr_t)jobs[i].ref % 16 || (uintptr_t)jobs[i].cur % 16) return false;
  }
  SearchArgs probe = job_args(base, jobs[0]);
  probe.block_row_begin = 0;
  probe.block_row_end = rows;  // the planner counts tiles over every job's rows
  QsadGeom g;
  if (!cached_flow_plan(probe, &g)) return false;
  long total = 0;
  for (int i = 0; i < n; i++)
    total += (long)g.wg_per_row * (qsad_rows_end(base, jobs[i].r1) - jobs[i].r0);
  const long ring = tuning().flow_one != 0 ? (1L << 40) : (long)g.flow_slots * cu_count();
  const long nl = (total + ring - 1) / ring;  // launches of about total / nl tiles
  const long target = nl > 1 ? (total + nl - 1) / nl : total;
  SearchJob fj[MAX_JOBS];
  int m = 0;
  long tiles = 0;
  for (int i = 0; i < n && *err == hipSuccess; i++) {
    SearchJob J = jobs[i];
    J.r1 = qsad_rows_end(base, J.r1);
    const long t = (long)g.wg_per_row * (J.r1 - J.r0);
    if (m && (tiles + t > target || m == MAX_JOBS)) {
      *err = launch_flow(base, g, fj, m, stream);
      m = 0;
      tiles = 0;
    }
    fj[m++] = J;
    tiles += t;
  }
  if (m && *err == hipSuccess) *err = launch_flow(base, g, fj, m, stream);
  // the rows and columns the flow kernel leaves, job by job
  for (int i = 0; i < n && *err == hipSuccess; i++) {
    const SearchArgs q = job_args(base, jobs[i]);
    const int rq1 = qsad_rows_end(base, jobs[i].r1);
    if (rq1 < jobs[i].r1) *err = launch_generic(q, 0, g.nbx_full, rq1, jobs[i].r1 - rq1, stream);
    if (*err == hipSuccess && g.nbx_full < base.nbx)
      *err = launch_generic(q, g.nbx_full, base.nbx - g.nbx_full, jobs[i].r0,
                            jobs[i].r1 - jobs[i].r0, stream);
  }
  return true;
}

// Alignment class of a job's planes (the item planner's key, cached_plan).
static int align_class(const SearchArgs& p, const uint8_t* ref, const uint8_t* cur) {
  return ((p.stride % 4 == 0) && ((uintptr_t)ref % 4 == 0) && ((uintptr_t)cur % 4 == 0)) |
         (((p.stride % 16 == 0) && ((uintptr_t)ref % 16 == 0)) << 1);
}

// VALU jobs the item kernel takes (SAD, or SSD off the matrix cores) in one
// launch per MAX_JOBS: per-job launches each paid the persistent grid's fill
// and drain (8 stripes of a 4K frame: 1.165 ms against 1.047 for the frame).
// Returns false (nothing launched) when the jobs' planes differ in alignment
// class or the item kernel does not take the shape.
static bool launch_item_jobs(const SearchArgs& base, const SearchJob* jobs, int n,
                             hipStream_t stream, hipError_t* err) {
  *err = hipSuccess;
  if (n < 2 || (base.cost_kind != COST_SAD && base.cost_kind != COST_SSD)) return false;
  const int ac = align_class(base, jobs[0].ref, jobs[0].cur);
  int rows = 0;
  for (int i = 0; i < n; i++) {
    rows += jobs[i].r1 - jobs[i].r0;
    if (align_class(base, jobs[i].ref, jobs[i].cur) != ac) return false;
  }
  SearchArgs probe = job_args(base, jobs[0]);
  probe.block_row_begin = 0;
  probe.block_row_end = rows;  // the planner counts tiles over every job's rows
  QsadGeom g;
  int K = 0;
  if (!cached_plan(probe, &g, &K)) return false;
  // Every job shares the launch, however large: with whole frames per XCD band
  // the bands need no halo rows.  8K 8x8 +-128, 16 frames: 17.09 ms and 70.7 MB
  // read per frame in one row-major launch, against 17.26 ms and 89.9 MB one
  // launch per frame (profiles/r04m_variants_8k.txt; round 3 measured the
  // opposite, 124 vs 98 MB, with tiles claimed two ahead).  Row-major: the
  // strip walk, which keeps a single wide frame's window rows in L2, only
  // spreads a batch's working set (same run: strips of 16 tiles 87.9 MB).
  const int per = tuning().item_batch == 0 ? 1 : MAX_JOBS;  // tuning build: ME_ITEM_BATCH=0
  if (n > 1 && tuning().strip < 0) g.strip_w = 0;
  for (int i0 = 0; i0 < n && *err == hipSuccess; i0 += per) {
    const int m = n - i0 < per ? n - i0 : per;
    SearchJob fj[MAX_JOBS];
    for (int i = 0; i < m; i++) {
      fj[i] = jobs[i0 + i];
      fj[i].r1 = qsad_rows_end(base, fj[i].r1);
    }
    *err = launch_fast(base, g, K, job_table(base, g.wg_per_row, fj, m), stream);
  }
  // the rows and columns the item kernel leaves, job by job
  for (int i = 0; i < n && *err == hipSuccess; i++) {
    const SearchArgs q = job_args(base, jobs[i]);
    const int rq1 = qsad_rows_end(base, jobs[i].r1);
    if (rq1 < jobs[i].r1) *err = launch_generic(q, 0, g.nbx_full, rq1, jobs[i].r1 - rq1, stream);
    if (*err == hipSuccess && g.nbx_full < base.nbx)
      *err = launch_generic(q, g.nbx_full, base.nbx - g.nbx_full, jobs[i].r0,
                            jobs[i].r1 - jobs[i].r0, stream);
  }
  return true;
}

static hipError_t launch_valu(const SearchArgs& p, hipStream_t stream, int* used_fast) {
  note_path(1);
  if (p.block_row_end <= p.block_row_begin) return hipSuccess;
  const SearchJob J{p.ref, p.ref_row0, p.cur, p.cur_row0, p.block_row_begin, p.block_row_end, p.mv, p.cost};
  hipError_t e;
  if (launch_flow_jobs(p, &J, 1, stream, &e)) {
    if (used_fast) *used_fast = 3;
    return e;
  }
  return launch_items(p, stream, used_fast);
}

hipError_t launch_jobs(const SearchArgs& base, const SearchJob* jobs, int n, hipStream_t stream) {
  hipError_t e;
  if (n > 1 && launch_flow_jobs(base, jobs, n, stream, &e)) {
    note_path(1);
    return e;
  }
  // SSD jobs of one geometry share the matrix cores' launches (prepass planes
  // per job in the context scratch); others go one by one
  if (n > 1 && launch_mfma_jobs(base, jobs, n, stream, &e)) return e;
  MfmaGeom mg;
  const bool mfma = base.cost_kind == COST_SSD && plan_mfma_ssd(job_args(base, jobs[0]), &mg) &&
                    (mg.scratch_bytes == 0 || base.scratch);
  if (n > 1 && !mfma && launch_item_jobs(base, jobs, n, stream, &e)) {
    note_path(1);
    return e;
  }
  for (int i = 0; i < n; i++) {
    if (jobs[i].r1 <= jobs[i].r0) continue;
    e = launch_search(job_args(base, jobs[i]), stream, nullptr);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_search(const SearchArgs& p, hipStream_t stream, int* used_fast) {
  const int r0 = p.block_row_begin, r1 = p.block_row_end;
  if (r1 <= r0) return hipSuccess;
  if (used_fast) *used_fast = 0;
  if (p.cost_kind == COST_SSIM) return launch_ssim(p, stream);
  MfmaGeom mg;
  // (the band-walk and lean kernels need no context scratch: scratch_bytes 0)
  if (p.cost_kind == COST_SSD && plan_mfma_ssd(p, &mg) &&
      (mg.scratch_bytes == 0 || (p.scratch && p.scratch_bytes >= mg.scratch_bytes))) {
    // Matrix cores: every full-width block (the partial bottom row included);
    // the partial right column stays on the generic kernel.
    hipError_t e = launch_mfma_ssd(p, mg, stream);
    if (e != hipSuccess) return e;
    if (used_fast) *used_fast = 2;
    const int rest = mg.row0 + mg.nrows;  // < r1: a partial bottom row the MFMA kernel left (B = 8)
    if (mg.nbx < p.nbx) {
      e = launch_generic(p, mg.nbx, p.nbx - mg.nbx, r0, rest - r0, stream);
      if (e != hipSuccess) return e;
    }
    if (rest < r1) {
      SearchArgs q = p;
      q.block_row_begin = rest;
      q.mv = p.mv + 2 * (size_t)(rest - r0) * p.nbx;
      if (p.cost) q.cost = p.cost + (size_t)(rest - r0) * p.nbx;
      return launch_valu(q, stream, nullptr);
    }
    return hipSuccess;
  }
  return launch_valu(p, stream, used_fast);
}

}  // namespace me

#ifdef ME_STAMPS
// Diagnostic build only: copy the per-workgroup stamps to the host.
extern "C" int me_debug_wave_stamps(unsigned long long* out, int n_words) {
  if (n_words > (8 << 14)) n_words = 8 << 14;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_wstamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int me_debug_stamps(unsigned long long* out, int n_words) {
  if (n_words > (8 << 16)) n_words = 8 << 16;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(me::g_stamps), (size_t)n_words * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
