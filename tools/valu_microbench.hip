// valu_microbench.hip -- issue-rate microbenchmark for the integer ops the
// block matcher can be built from (gfx950).
//
// Each kernel runs 8 independent chains of ONE instruction over the whole chip.
// The instruction is emitted by `asm volatile` with its result fed back as an
// operand (a loop-carried, data-dependent chain), so the compiler can neither
// fold the loop (v_add / v_min: a builtin `acc += x` loop collapses to one
// multiply) nor schedule anything else into it.  Rates are taken from the whole
// launch: wave-instructions per second over the chip, and
//     cycles per wave-instruction per SIMD = clock * SIMDs / (wave-instr/s)
// with the clock the chip held (s_memtime / s_memrealtime) and SIMDs = 4 x CUs,
// so the result does not depend on how many waves were resident at once.
// Output: one JSON line per op.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o bin/valu_microbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 512;
constexpr int UNROLL = 16;

// One chain step of op OP: acc (32- or 64-bit) is both read and written.
template <int OP>
__device__ __forceinline__ void step(uint32_t& a, uint64_t& a64, uint32_t x, uint32_t y,
                                     uint64_t x64, float& fa, float fx) {
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 1) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 2) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(a64) : "v"(x64), "v"(y));
  if constexpr (OP == 3) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 4) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 5) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(fa) : "v"(fx));
  if constexpr (OP == 6) asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 7) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 8) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 9) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 11) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 12) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 13) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a) : "v"(x));
  if constexpr (OP == 14) asm volatile("v_msad_u8 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
  if constexpr (OP == 15) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a) : "v"(x) : "vcc");
  if constexpr (OP == 16) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(a64));
}

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
    fx[i] = (float)(x[i] >> 8) * 1e-7f;
    fa[i] = (float)(acc[i] >> 8);
  }
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
#pragma unroll
      for (int i = 0; i < 8; i++) step<OP>(acc[i], acc64[i], x[i], y[i], x64[i], fa[i], fx[i]);
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
static int run(const char* name, const uint32_t* d_in, uint32_t* d_out, uint64_t* d_clk,
               int blocks, int simds, int waves_per_simd = 0) {
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
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // memrealtime = 100 MHz
  const double per_wave = (double)ITERS * UNROLL * 8;
  const double winst = (double)blocks * 4 * per_wave;
  const double rate = winst / (ms / 1e3);                         // wave-instructions / s, chip
  const double cyc = ghz * 1e9 * simds / rate;                    // per wave-instruction per SIMD
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"cyc_per_wave_instr_per_simd\": %.2f, "
         "\"wave_instr_per_s\": %.4g, \"simds\": %d", name, ms, ghz, cyc, rate, simds);
  if (waves_per_simd) printf(", \"waves_per_simd\": %d", waves_per_simd);
  printf("}\n");
  return 0;
}

int main() {
  uint32_t h[64];
  for (int i = 0; i < 64; i++) h[i] = 0x9E3779B9u * (i + 1);
  uint32_t *d_in, *d_out;
  uint64_t* d_clk;
  int dev = 0, cus = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CHK(hipMalloc(&d_in, sizeof h));
  CHK(hipMalloc(&d_out, 64));
  CHK(hipMalloc(&d_clk, 24));
  CHK(hipMemcpy(d_in, h, sizeof h, hipMemcpyHostToDevice));
  const int blocks = cus * 8;  // 8 waves per SIMD when resident; rates do not assume it
  const int simds = 4 * cus;
  run<5>("v_fma_f32", d_in, d_out, d_clk, blocks, simds);
  run<0>("v_add_u32", d_in, d_out, d_clk, blocks, simds);
  run<15>("v_add_co_u32", d_in, d_out, d_clk, blocks, simds);
  run<8>("v_min_u32", d_in, d_out, d_clk, blocks, simds);
  run<9>("v_min3_u32", d_in, d_out, d_clk, blocks, simds);
  run<10>("v_lshl_or_b32", d_in, d_out, d_clk, blocks, simds);
  run<13>("v_pk_max_u16", d_in, d_out, d_clk, blocks, simds);
  run<16>("v_lshlrev_b64", d_in, d_out, d_clk, blocks, simds);
  run<11>("v_mul_lo_u32", d_in, d_out, d_clk, blocks, simds);
  run<12>("v_mul_hi_u32", d_in, d_out, d_clk, blocks, simds);
  run<1>("v_sad_u8", d_in, d_out, d_clk, blocks, simds);
  run<14>("v_msad_u8", d_in, d_out, d_clk, blocks, simds);
  run<6>("v_sad_u16", d_in, d_out, d_clk, blocks, simds);
  run<2>("v_qsad_pk_u16_u8", d_in, d_out, d_clk, blocks, simds);
  run<3>("v_dot4_u32_u8", d_in, d_out, d_clk, blocks, simds);
  run<4>("v_alignbyte_b32", d_in, d_out, d_clk, blocks, simds);
  run<7>("v_perm_b32", d_in, d_out, d_clk, blocks, simds);
  // Occupancy sweep: one 256-thread workgroup per CU puts one wave on each
  // SIMD, so `cus * w` workgroups (one wave of the grid resident) give w waves
  // per SIMD: what a SIMD sustains with that many waves to pick from.
  for (int w : {1, 2, 4}) {
    run<2>("v_qsad_pk_u16_u8", d_in, d_out, d_clk, cus * w, simds, w);
    run<1>("v_sad_u8", d_in, d_out, d_clk, cus * w, simds, w);
    run<9>("v_min3_u32", d_in, d_out, d_clk, cus * w, simds, w);
    run<0>("v_add_u32", d_in, d_out, d_clk, cus * w, simds, w);
  }
  return 0;
}
