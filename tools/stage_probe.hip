// stage_probe.hip -- why do the small-stripe workgroups of a CU get their
// first item one after another?  (diagnostic; DESIGN.md (e) "staircase")
//
// 1,024 workgroups of 256 threads (4 per CU at 40 KB of LDS, or 1 per CU at
// 160 KB), each standing in for one one-block item of an 8-way 1080p stripe:
// stage an 80-row x 112-byte window of a 1920-byte-pitch plane into LDS (the
// real item's geometry; neighbouring workgroups' windows overlap like the real
// ones), then compute a qsad loop over LDS rows of about one K = 5 item.
// Every wave stamps (start, staged, end) with s_memtime plus its HW_ID, so the
// per-CU order of staging and the SIMD placement of each workgroup's waves can
// be read off directly.  Variants: LDS DMA or register staging, with or
// without the compute, 4 or 1 workgroups per CU.
//
//   hipcc --offload-arch=gfx950 -O3 -o bin/stage_probe tools/stage_probe.hip
//   bin/stage_probe > gpurun_out/stage_probe.jsonl
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

constexpr int PW = 1920, PH = 1088 + 128;  // plane (rows past the frame: slack)
constexpr int ROWS = 80, PITCH = 112, BYTES = ROWS * PITCH;

struct Args {
  const uint8_t* plane;
  uint32_t plane_bytes;
  int mode;  // bit0: LDS DMA (else register staging); bit1: no compute; bit2: disjoint windows
  int iters;
  unsigned long long* out;  // [wg][wave][4]
  uint32_t* sink;
};

__global__ __launch_bounds__(256) void probe(Args a) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int wg = (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // the item kernel's one-block windows: block (bx, by) of 120 per row
  int X0, Y0;
  if (a.mode & 4) {  // disjoint: every workgroup its own bytes
    X0 = (wg % 16) * 112;
    Y0 = (wg / 16) * 16 % (PH - ROWS);
  } else {
    X0 = (wg % 118) * 16;
    Y0 = (wg / 118) * 16;
  }
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.plane, (short)0, a.plane_bytes, 0x00020000);
  for (int s0 = wave * 1024; s0 < BYTES; s0 += 4 * 1024) {
    const int d = s0 + 16 * lane;
    const int r = d / PITCH, x = d - r * PITCH;
    const uint32_t src = (uint32_t)((Y0 + r) * PW + X0 + x);
    if (d < BYTES) {
      if (a.mode & 1) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(smem + s0), 16, src, 0, 0, 0);
      } else {
        const uint4 v = *reinterpret_cast<const uint4*>(a.plane + src);
        *reinterpret_cast<uint4*>(smem + d) = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint64_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
  if (!(a.mode & 2)) {
    const uint32_t c0 = 0x01020304u * (uint32_t)(lane + 1), c1 = c0 ^ 0x5a5a5a5au;
    typedef __attribute__((address_space(3))) const uint64_t lds_u64;
    uint32_t o = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)smem) +
                 (uint32_t)(4 * (lane & 15));
    for (int i = 0; i < a.iters; i++) {
      const uint64_t w0 = *reinterpret_cast<lds_u64*>((uintptr_t)o);
      const uint64_t w1 = *reinterpret_cast<lds_u64*>((uintptr_t)(o + 8));
      const uint64_t w2 = *reinterpret_cast<lds_u64*>((uintptr_t)(o + 16));
      const uint64_t w3 = *reinterpret_cast<lds_u64*>((uintptr_t)(o + 24));
#pragma unroll
      for (int j = 0; j < 4; j++) {
        acc0 = __builtin_amdgcn_qsad_pk_u16_u8(w0, j & 1 ? c0 : c1, acc0);
        acc1 = __builtin_amdgcn_qsad_pk_u16_u8(w1, j & 1 ? c1 : c0, acc1);
        acc2 = __builtin_amdgcn_qsad_pk_u16_u8(w2, j & 1 ? c0 : c1, acc2);
        acc3 = __builtin_amdgcn_qsad_pk_u16_u8(w3, j & 1 ? c1 : c0, acc3);
      }
      o += PITCH;
      if (o >= (uint32_t)BYTES - 64) o -= (uint32_t)(BYTES - 128);
      asm volatile("" : "+v"(o));
    }
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  if (((acc0 ^ acc1 ^ acc2 ^ acc3) & 0xFFFFFFFFFFull) == 0x123456789ull) a.sink[tid] = 1;
  if (lane == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* o = a.out + ((size_t)wg * 4 + wave) * 4;
    o[0] = t0;
    o[1] = t1;
    o[2] = t2;
    o[3] = ((unsigned long long)(xcc & 0xF) << 32) | hw;
  }
}

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[(size_t)((v.size() - 1) * p)];
}

int main() {
  uint8_t* plane;
  const size_t pb = (size_t)PW * PH;
  CK(hipMalloc(&plane, pb));
  std::vector<uint8_t> h(pb);
  for (size_t i = 0; i < pb; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  CK(hipMemcpy(plane, h.data(), pb, hipMemcpyHostToDevice));
  const int NWG = 1024;
  unsigned long long* out;
  uint32_t* sink;
  CK(hipMalloc(&out, (size_t)NWG * 16 * 8));
  CK(hipMalloc(&sink, 4096));
  CK(hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  struct V { const char* name; int mode, lds, iters, nwg; };
  const V vs[] = {
      {"dma+compute 4/CU", 1, 40 * 1024, 20, NWG},
      {"reg+compute 4/CU", 0, 40 * 1024, 20, NWG},
      {"dma only 4/CU", 3, 40 * 1024, 20, NWG},
      {"reg only 4/CU", 2, 40 * 1024, 20, NWG},
      {"dma+compute 4/CU disjoint", 5, 40 * 1024, 20, NWG},
      {"dma+compute 1/CU", 1, 150 * 1024, 20, 256},
      {"dma+compute 4/CU heavy", 1, 40 * 1024, 80, NWG},
  };
  std::vector<unsigned long long> st((size_t)NWG * 16);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const V& v : vs) {
    Args a{plane, (uint32_t)pb, v.mode, v.iters, out, sink};
    float ms = 0, best = 1e9;
    for (int rep = 0; rep < 6; rep++) {
      CK(hipMemset(out, 0, (size_t)NWG * 16 * 8));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(probe, dim3(v.nwg), dim3(256), v.lds, 0, a);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0) best = std::min(best, ms);
    }
    CK(hipMemcpy(st.data(), out, (size_t)v.nwg * 16 * 8, hipMemcpyDeviceToHost));
    // per-XCD time base: the earliest wave start of that XCD
    unsigned long long base[16];
    for (int x = 0; x < 16; x++) base[x] = ~0ull;
    for (int i = 0; i < v.nwg * 4; i++) {
      const int x = (int)(st[4 * i + 3] >> 32);
      base[x] = std::min(base[x], st[4 * i]);
    }
    std::vector<double> staged, lifew, ends, wg_staged;
    int same_simd_wgs = 0;
    // per CU: order of the workgroups' staging completion and ends
    std::vector<std::vector<std::pair<double, double>>> cu_wg(16 * 64 * 8);
    for (int g = 0; g < v.nwg; g++) {
      unsigned simds = 0;
      double gs = 0, ge = 0;
      unsigned long long hw = 0;
      int x = 0;
      for (int w = 0; w < 4; w++) {
        const unsigned long long* s = &st[((size_t)g * 4 + w) * 4];
        x = (int)(s[3] >> 32);
        hw = s[3] & 0xFFFFFFFFull;
        simds |= 1u << ((hw >> 4) & 3);
        staged.push_back((double)(s[1] - s[0]));
        gs = std::max(gs, (double)(s[1] - base[x]));
        ge = std::max(ge, (double)(s[2] - base[x]));
        ends.push_back((double)(s[2] - base[x]));
      }
      if (__builtin_popcount(simds) == 1) same_simd_wgs++;
      wg_staged.push_back(gs);
      const int cu = (x << 7) | (int)(((hw >> 13) & 7) << 4) | (int)(((hw >> 12) & 1) << 3) |
                     (int)((hw >> 8) & 0xF);
      if (cu < (int)cu_wg.size()) cu_wg[cu].push_back({gs, ge});
    }
    // staircase: per CU sorted staging times, averaged by rank
    double rank_staged[8] = {0}, rank_end[8] = {0};
    int rank_n[8] = {0};
    for (auto& c : cu_wg) {
      std::sort(c.begin(), c.end());
      for (size_t r = 0; r < c.size() && r < 8; r++) {
        rank_staged[r] += c[r].first;
        rank_end[r] += c[r].second;
        rank_n[r]++;
      }
    }
    printf("{\"variant\": \"%s\", \"kernel_us\": %.2f, \"wgs\": %d, \"staged_cyc\": [%.0f, %.0f, %.0f], "
           "\"wg_staged_cyc_p50_p90_max\": [%.0f, %.0f, %.0f], \"wave_end_cyc_p50_max\": [%.0f, %.0f], "
           "\"wgs_on_one_simd\": %d, \"per_cu_rank_staged_cyc\": [",
           v.name, best * 1e3, v.nwg, pct(staged, 0.5), pct(staged, 0.9), pct(staged, 1.0),
           pct(wg_staged, 0.5), pct(wg_staged, 0.9), pct(wg_staged, 1.0), pct(ends, 0.5),
           pct(ends, 1.0), same_simd_wgs);
    for (int r = 0; r < 8 && rank_n[r]; r++) printf("%s%.0f", r ? ", " : "", rank_staged[r] / rank_n[r]);
    printf("], \"per_cu_rank_end_cyc\": [");
    for (int r = 0; r < 8 && rank_n[r]; r++) printf("%s%.0f", r ? ", " : "", rank_end[r] / rank_n[r]);
    printf("]}\n");
    fflush(stdout);
  }
  return 0;
}
