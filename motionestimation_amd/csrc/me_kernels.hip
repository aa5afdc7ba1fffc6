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
// Two kernels:
//   me_qsad_kernel<B, K>   SAD, B in {8, 16}, full-width blocks.  One workgroup
//                          per TB blocks of one block row; the union search
//                          window of those blocks is staged once in LDS; each
//                          lane owns 4 horizontal x K vertical candidates of one
//                          block and walks the window rows, 16 |a-b| per
//                          v_qsad_pk_u16_u8 with the cur block held in VGPRs.
//   me_generic_kernel      any B <= 64, any S, SSD or SAD, partial blocks; one
//                          workgroup per block, one candidate per lane.  SSD on
//                          blocks with w*h > 256 replays the reference's float
//                          accumulation (main.c:19-27) so the argmin is identical
//                          even when the float sum rounds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_kernels.h"

namespace me {

__device__ __forceinline__ uint64_t make_key(uint32_t cost, int dx, int dy) {
  return ((uint64_t)cost << 32) | ((uint32_t)(dy + 32768) << 16) | (uint32_t)(dx + 32768);
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
                                                                     int nbx_range,
                                                                     int win_lds_bytes) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint64_t red[GENERIC_THREADS / 64];
  const int tid = threadIdx.x;
  const int bx = bx0 + (int)(blockIdx.x % nbx_range);
  const int by = p.block_row_begin + (int)(blockIdx.x / nbx_range);
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
// Workgroup = TB consecutive full-width blocks of one block row.  LDS tile:
// frame rows [Y0, Y0 + 2S + B) x columns [X0, X0 + pitch), X0 = tlx(b0) - S - a
// rounded down to a multiple of 4 (a = (tlx - S) mod 4).  Task t of the
// workgroup -> (dy chunk, block, dx group): the lane evaluates dx offsets
// q = 4g..4g+3 (dx = q - S - a) and dy offsets d = chunk*K .. +K-1 (dy = d - S).
template <int B, int K>
__global__ __launch_bounds__(1024) void me_qsad_kernel(SearchArgs p, QsadGeom g) {
  constexpr int CW = B / 4;  // cur words per row
  extern __shared__ __align__(16) uint8_t smem[];
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem);            // TB keys
  uint32_t* cur_lds = reinterpret_cast<uint32_t*>(smem + 8 * 16);  // TB * B * CW words
  uint8_t* tile = smem + 8 * 16 + g.tb * B * B;                     // rows x pitch
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int S = p.range;
  const int wg_blocks = g.tb;
  const int bx0 = (int)(blockIdx.x % g.wg_per_row) * g.tb;
  const int by = p.block_row_begin + (int)(blockIdx.x / g.wg_per_row);
  const int nb = min(wg_blocks, g.nbx_full - bx0);
  const int tly = by * B;
  const int h = min(B, p.height - tly);
  const int a = ((bx0 * B - S) % 4 + 4) % 4;
  const int X0 = bx0 * B - S - a;
  const int Y0 = tly - S;
  const int rows = 2 * S + B;
  const int pw = g.pitch >> 2;

  if (tid < wg_blocks) keys[tid] = ~0ull;
  // Stage the ref tile (zeros outside the frame: those candidates are masked).
  for (int i = tid; i < rows * pw; i += nthr) {
    const int r = i / pw, q = i - r * pw;
    const int y = Y0 + r, x = X0 + 4 * q;
    uint32_t v = 0;
    if (y >= 0 && y < p.height) {
      const uint8_t* src = row_ptr(p, p.ref, p.ref_row0, y);
      if (x >= 0 && x + 3 < p.width && g.aligned) {
        v = *reinterpret_cast<const uint32_t*>(src + x);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (x + k >= 0 && x + k < p.width) v |= (uint32_t)src[x + k] << (8 * k);
      }
    }
    reinterpret_cast<uint32_t*>(tile)[i] = v;
  }
  // Stage the cur blocks: word (b, oy, k).
  for (int i = tid; i < nb * B * CW; i += nthr) {
    const int b = i / (B * CW), rem = i - b * B * CW, oy = rem / CW, k = rem - oy * CW;
    uint32_t v = 0;
    if (oy < h) {
      const uint8_t* src = row_ptr(p, p.cur, p.cur_row0, tly + oy) + (bx0 + b) * B + 4 * k;
      if (g.aligned) v = *reinterpret_cast<const uint32_t*>(src);
      else v = src[0] | (src[1] << 8) | (src[2] << 16) | ((uint32_t)src[3] << 24);
    }
    cur_lds[i] = v;
  }
  __syncthreads();

  const int G = g.groups;
  const int T = nb * G * g.chunks;
  for (int t = tid; t < T; t += nthr) {
    const int chunk = t / (nb * G);
    const int rem = t - chunk * nb * G;
    const int b = rem / G, gi = rem - b * G;
    const int d0 = chunk * K;

    uint32_t c[B][CW];
#pragma unroll
    for (int y = 0; y < B; y++)
#pragma unroll
      for (int k = 0; k < CW; k++) c[y][k] = cur_lds[(b * B + y) * CW + k];

    uint64_t acc[K];
#pragma unroll
    for (int j = 0; j < K; j++) acc[j] = 0;

    const uint32_t* rowp = reinterpret_cast<const uint32_t*>(tile) + d0 * pw + (b * B) / 4 + gi;
    if (h == B) {
#pragma unroll
      for (int yy = 0; yy < K + B - 1; yy++) {
        // rows beyond the tile are only reached by chunk padding (d > 2S):
        // clamp the address, the candidates are masked below.
        const int r = min(d0 + yy, rows - 1) - d0;
        uint32_t wv[CW + 1];
#pragma unroll
        for (int k = 0; k <= CW; k++) wv[k] = rowp[r * pw + k];
#pragma unroll
        for (int j = 0; j < K; j++) {
          const int y = yy - j;
          if (y >= 0 && y < B) {
#pragma unroll
            for (int k = 0; k < CW; k++)
              acc[j] = __builtin_amdgcn_qsad_pk_u16_u8(((uint64_t)wv[k + 1] << 32) | wv[k],
                                                       c[y][k], acc[j]);
          }
        }
      }
    } else {
#pragma unroll
      for (int yy = 0; yy < K + B - 1; yy++) {
        const int r = min(d0 + yy, rows - 1) - d0;
        uint32_t wv[CW + 1];
#pragma unroll
        for (int k = 0; k <= CW; k++) wv[k] = rowp[r * pw + k];
#pragma unroll
        for (int j = 0; j < K; j++) {
          const int y = yy - j;
          if (y >= 0 && y < B && y < h) {
#pragma unroll
            for (int k = 0; k < CW; k++)
              acc[j] = __builtin_amdgcn_qsad_pk_u16_u8(((uint64_t)wv[k + 1] << 32) | wv[k],
                                                       c[y][k], acc[j]);
          }
        }
      }
    }

    // Valid ranges of this block (main.c:73-76 closed form).
    const int tlx = (bx0 + b) * B;
    const int dxmin = max(-S, -tlx), dxmax = min(S, p.width - B - tlx);
    const int dymin = max(-S, -tly), dymax = min(S, p.height - h - tly);
    uint64_t best = ~0ull;
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int dy = d0 + j - S;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int dx = 4 * gi + i - S - a;
        const uint32_t sad = (uint32_t)(acc[j] >> (16 * i)) & 0xFFFFu;
        const bool ok = dx >= dxmin && dx <= dxmax && dy >= dymin && dy <= dymax;
        const uint64_t key = ok ? make_key(sad, dx, dy) : ~0ull;
        best = key < best ? key : best;
      }
    }
    atomicMin(reinterpret_cast<unsigned long long*>(&keys[b]), (unsigned long long)best);
  }
  __syncthreads();
  if (tid < nb) {
    const uint64_t k = keys[tid];
    const int out = (by - p.block_row_begin) * p.nbx + bx0 + tid;
    p.mv[2 * out] = (int16_t)((int)(k & 0xFFFF) - 32768);
    p.mv[2 * out + 1] = (int16_t)((int)((k >> 16) & 0xFFFF) - 32768);
    if (p.cost) p.cost[out] = (uint32_t)(k >> 32);
  }
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

hipError_t launch_generic(const SearchArgs& p, int bx0, int nbx_range, int nrows,
                          hipStream_t stream) {
  if (nbx_range <= 0 || nrows <= 0) return hipSuccess;
  int win = 0;
  const int lds = generic_lds_bytes(p, &win);
  dim3 grid((unsigned)(nbx_range * nrows)), block(GENERIC_THREADS);
  if (p.cost_kind == COST_SAD)
    hipLaunchKernelGGL(me_generic_kernel<COST_SAD>, grid, block, lds, stream, p, bx0, nbx_range, win);
  else
    hipLaunchKernelGGL(me_generic_kernel<COST_SSD>, grid, block, lds, stream, p, bx0, nbx_range, win);
  return hipGetLastError();
}

// Pick K (dy rows per lane) minimising chunk padding, and TB (blocks per
// workgroup) minimising idle lanes, within the LDS and 1024-thread limits.
bool plan_qsad(const SearchArgs& p, QsadGeom* g, int* k_out) {
  const int B = p.blk, S = p.range;
  if (p.cost_kind != COST_SAD || (B != 16 && B != 8)) return false;
  if (S < 1 || S > 255) return false;
  g->nbx_full = p.width / B;
  if (g->nbx_full < 1) return false;
  static const int Ks_16[] = {13, 11, 8};
  static const int Ks_8[] = {13, 11, 8};
  const int* Ks = B == 16 ? Ks_16 : Ks_8;
  const int D = 2 * S + 1;
  int bestK = Ks[0];
  double bestEff = -1;
  for (int i = 0; i < 3; i++) {
    const int K = Ks[i];
    const int ch = (D + K - 1) / K;
    const double eff = (double)D / (ch * K);
    if (eff > bestEff + 1e-9) { bestEff = eff; bestK = K; }
  }
  const int K = bestK;
  g->chunks = (D + K - 1) / K;
  // Groups: worst case a = 3 -> ceil((2S + 3 + 1) / 4).
  g->groups = (2 * S + 3 + 1 + 3) / 4;
  const int rows = 2 * S + B;
  int bestTB = 1;
  double bestUse = -1;
  for (int tb = 1; tb <= 16; tb++) {
    const int width = (tb - 1) * B + 4 * g->groups + 16;
    const int pitch = (width + 3) & ~3;
    const long lds = 8 * 16 + (long)tb * B * B + (long)rows * pitch;
    if (lds > QSAD_LDS_BUDGET) break;
    const int T = tb * g->groups * g->chunks;
    const int iters = (T + 1023) / 1024;
    const int thr = ((T + iters - 1) / iters + 63) & ~63;
    const double use = (double)T / (iters * thr);
    // prefer fuller waves; at equal use prefer fewer blocks (more workgroups).
    if (use > bestUse + 0.02) { bestUse = use; bestTB = tb; }
  }
  g->tb = bestTB;
  const int width = (g->tb - 1) * B + 4 * g->groups + 16;
  g->pitch = (width + 3) & ~3;
  const int T = g->tb * g->groups * g->chunks;
  const int iters = (T + 1023) / 1024;
  g->threads = ((T + iters - 1) / iters + 63) & ~63;
  g->lds = 8 * 16 + g->tb * B * B + rows * g->pitch;
  g->wg_per_row = (g->nbx_full + g->tb - 1) / g->tb;
  g->aligned = (p.stride % 4 == 0) && ((uintptr_t)p.ref % 4 == 0) && ((uintptr_t)p.cur % 4 == 0);
  *k_out = K;
  return true;
}

hipError_t launch_qsad(const SearchArgs& p, const QsadGeom& g, int K, int nrows,
                       hipStream_t stream) {
  dim3 grid((unsigned)(g.wg_per_row * nrows)), block((unsigned)g.threads);
#define ME_QSAD_CASE(BB, KK)                                                              \
  if (p.blk == BB && K == KK) {                                                           \
    if (g.lds > 64 * 1024) {                                                              \
      hipError_t e_ = hipFuncSetAttribute((const void*)me_qsad_kernel<BB, KK>,            \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, g.lds); \
      if (e_ != hipSuccess) return e_;                                                    \
    }                                                                                     \
    hipLaunchKernelGGL((me_qsad_kernel<BB, KK>), grid, block, g.lds, stream, p, g);       \
    return hipGetLastError();                                                             \
  }
  ME_QSAD_CASE(16, 13) ME_QSAD_CASE(16, 11) ME_QSAD_CASE(16, 8)
  ME_QSAD_CASE(8, 13) ME_QSAD_CASE(8, 11) ME_QSAD_CASE(8, 8)
#undef ME_QSAD_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_search(const SearchArgs& p, hipStream_t stream, int* used_fast) {
  const int nrows = p.block_row_end - p.block_row_begin;
  if (nrows <= 0) return hipSuccess;
  QsadGeom g;
  int K = 0;
  if (used_fast) *used_fast = 0;
  if (plan_qsad(p, &g, &K)) {
    hipError_t e = launch_qsad(p, g, K, nrows, stream);
    if (e != hipSuccess) return e;
    if (used_fast) *used_fast = 1;
    if (g.nbx_full < p.nbx)  // partial right column
      return launch_generic(p, g.nbx_full, p.nbx - g.nbx_full, nrows, stream);
    return hipSuccess;
  }
  return launch_generic(p, 0, p.nbx, nrows, stream);
}

}  // namespace me
