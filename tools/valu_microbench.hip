// valu_microbench.hip -- issue-rate microbenchmark for the integer ops the
// block matcher can be built from (gfx950).  Each kernel runs 8 independent
// accumulation chains of ONE instruction with loop-invariant operands (no
// other VALU in the loop body), over the whole chip at 8 waves/SIMD, and
// stamps s_memtime / s_memrealtime to report the clock the chip actually held.
// Output: one JSON line per op with cycles per wave-instruction per SIMD.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o bin/valu_microbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 1024;
constexpr int UNROLL = 32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(256) void bench(const uint32_t* in, uint32_t* out, uint64_t* clk) {
  const int l = threadIdx.x & 63;
  uint32_t x[8], y[8], acc[8];
  uint64_t x64[8], acc64[8];
  float fx[8], fa[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x[i] = in[(l + i) & 63];
    y[i] = in[(l + 3 * i + 1) & 63];
    acc[i] = in[(l + 5 * i + 2) & 63];
    x64[i] = ((uint64_t)y[i] << 32) | x[i];
    acc64[i] = acc[i];
    fx[i] = (float)x[i];
    fa[i] = (float)acc[i];
  }
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if constexpr (OP == 0) acc[i] = acc[i] + x[i];
        if constexpr (OP == 1) acc[i] = __builtin_amdgcn_sad_u8(x[i], y[i], acc[i]);
        if constexpr (OP == 2) acc64[i] = __builtin_amdgcn_qsad_pk_u16_u8(x64[i], y[i], acc64[i]);
        if constexpr (OP == 3) acc[i] = __builtin_amdgcn_udot4(x[i], y[i], acc[i], false);
        if constexpr (OP == 4) acc[i] = __builtin_amdgcn_alignbyte(acc[i], x[i], y[i]);
        if constexpr (OP == 5) fa[i] = __builtin_fmaf(fa[i], fx[i], 0.5f);
        if constexpr (OP == 6) acc[i] = __builtin_amdgcn_sad_u16(x[i], y[i], acc[i]);
        if constexpr (OP == 7) acc[i] = __builtin_amdgcn_perm(acc[i], x[i], y[i]);
        if constexpr (OP == 8) acc[i] = __builtin_amdgcn_udot4(x[i], x[i], acc[i], false) - acc[i];
        if constexpr (OP == 9) acc[i] = min(acc[i], x[i]);
        if constexpr (OP == 10) {
          u32x4 v = __builtin_amdgcn_mqsad_u32_u8(x64[i], y[i], (u32x4){acc[i], x[i], y[i], acc[i]});
          acc[i] = v[0];
        }
      }
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i] + acc64[i] + (uint64_t)fa[i];
  if (s == 0x123456789ull) out[0] = (uint32_t)s;
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&clk[0], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long*)&clk[1], (unsigned long long)(r1 - r0));
    atomicAdd((unsigned long long*)&clk[2], 1ull);
  }
}

template <int OP>
static int run(const char* name, const uint32_t* d_in, uint32_t* d_out, uint64_t* d_clk, int blocks) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  bench<OP><<<blocks, 256>>>(d_in, d_out, d_clk);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipMemset(d_clk, 0, 24));
  CHK(hipEventRecord(e0));
  bench<OP><<<blocks, 256>>>(d_in, d_out, d_clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t c[3];
  CHK(hipMemcpy(c, d_clk, 24, hipMemcpyDeviceToHost));
  double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // memrealtime = 100 MHz
  double per_wave_instr = (double)ITERS * UNROLL * 8;
  double cyc_per_wave = (double)c[0] / c[2];
  // 8 waves per SIMD share the SIMD: cycles per wave-instruction per SIMD.
  double cyc_per_instr_simd = cyc_per_wave / per_wave_instr / 8.0;
  double winst = (double)blocks * 4 * per_wave_instr;
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"cyc_per_wave_instr_per_simd\": %.3f, "
         "\"wave_instr_per_s\": %.4g}\n", name, ms, ghz, cyc_per_instr_simd, winst / (ms / 1e3));
  return 0;
}

int main() {
  uint32_t h[64];
  for (int i = 0; i < 64; i++) h[i] = 0x9E3779B9u * (i + 1);
  uint32_t *d_in, *d_out;
  uint64_t* d_clk;
  CHK(hipMalloc(&d_in, sizeof h));
  CHK(hipMalloc(&d_out, 64));
  CHK(hipMalloc(&d_clk, 24));
  CHK(hipMemcpy(d_in, h, sizeof h, hipMemcpyHostToDevice));
  int blocks = 256 * 8;  // 8 WGs of 4 waves per CU = 8 waves per SIMD
  run<0>("v_add_u32", d_in, d_out, d_clk, blocks);
  run<5>("v_fma_f32", d_in, d_out, d_clk, blocks);
  run<9>("v_min_u32", d_in, d_out, d_clk, blocks);
  run<1>("v_sad_u8", d_in, d_out, d_clk, blocks);
  run<6>("v_sad_u16", d_in, d_out, d_clk, blocks);
  run<2>("v_qsad_pk_u16_u8", d_in, d_out, d_clk, blocks);
  run<10>("v_mqsad_u32_u8", d_in, d_out, d_clk, blocks);
  run<3>("v_dot4_u32_u8", d_in, d_out, d_clk, blocks);
  run<8>("v_dot4_u32_u8+v_sub", d_in, d_out, d_clk, blocks);
  run<4>("v_alignbyte_b32", d_in, d_out, d_clk, blocks);
  run<7>("v_perm_b32", d_in, d_out, d_clk, blocks);
  return 0;
}
