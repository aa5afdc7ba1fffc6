// mfma_probe.hip -- hardware facts the MFMA SSD kernel relies on (diagnostic tool).
//   1. v_mfma_i32_16x16x64_i8 operand/result lane maps: lane l holds
//      A[row l&15][k = 16(l>>4) + e], B[k = 16(l>>4) + e][col l&15] (e = 0..15,
//      byte e of its 16-byte fragment) and C[row 4(l>>4) + r][col l&15] in reg r.
//   2. LDS DMA (buffer_load_dword ... lds) from byte offsets that are not
//      multiples of 4: does the granule come from the exact byte offset?
// Prints one JSON line per probe.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void mfma_i8_probe(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x;
  v4i a, b;
  int8_t* pa = reinterpret_cast<int8_t*>(&a);
  int8_t* pb = reinterpret_cast<int8_t*>(&b);
  for (int e = 0; e < 16; e++) {
    pa[e] = A[(l & 15) * 64 + 16 * (l >> 4) + e];
    pb[e] = B[(16 * (l >> 4) + e) * 16 + (l & 15)];
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; r++) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__global__ void dma_probe(const uint8_t* src, int nbytes, int shift, uint32_t* out) {
  __shared__ __align__(16) uint8_t lds[256];
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, 0x00020000);
  const int lane = threadIdx.x;
  // granule `lane` <- src bytes [shift + 4 lane, +4)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 4,
                                           (uint32_t)(shift + 4 * lane), 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  out[lane] = reinterpret_cast<const uint32_t*>(lds)[lane];
}

// 3. issue rate: 4 independent accumulators, back-to-back, one wave; cycles
//    per MFMA from s_memtime.
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
template <int KIND>
__global__ void mfma_rate(int iters, unsigned long long* out, int* sink) {
  v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  v4f f0 = {0, 0, 0, 0}, f1 = f0, f2 = f0, f3 = f0;
  v8bf ab = {}; 
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
    } else {
      f0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f0, 0, 0, 0);
      f1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f1, 0, 0, 0);
      f2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f2, 0, 0, 0);
      f3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f3, 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + (int)(f0[0] + f1[1] + f2[2] + f3[3]);
}

// 4. MFMA + N independent VALU ops per MFMA (one wave): does VALU issue
//    overlap the MFMA?  cycles per (MFMA + N VALU) from s_memtime.
template <int KIND, int NV>
__global__ void mfma_valu_mix(int iters, unsigned long long* out, int* sink) {
  // dense random operand bytes (an operand of mostly zero bytes may run faster)
  const uint32_t h0 = 0x9E3779B9u * (threadIdx.x + 1);
  v4i a = {(int)(h0 ^ 0x5bd1e995), (int)(h0 * 0x85ebca6b), (int)(h0 * 0xc2b2ae35), (int)(h0 + 0x27d4eb2f)};
  v4i b = {(int)(h0 * 0x165667b1), (int)(h0 ^ 0xd3a2646c), (int)(h0 * 0xfd7046c5), (int)(h0 + 0xb55a4f09)};
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = threadIdx.x * (i + 3);
  v8bf ab = {};
  v4f f0 = {0, 0, 0, 0}, f1 = f0, f2 = f0, f3 = f0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#define MIXV(j) if (NV > j) x[j] = __builtin_amdgcn_alignbyte(x[j], x[(j + 5) & 15], 1);
    if (KIND == 0) c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
    else f0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f0, 0, 0, 0);
    MIXV(0) MIXV(1) MIXV(2) MIXV(3)
    if (KIND == 0) c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
    else f1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f1, 0, 0, 0);
    MIXV(4) MIXV(5) MIXV(6) MIXV(7)
    if (KIND == 0) c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
    else f2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f2, 0, 0, 0);
    MIXV(8) MIXV(9) MIXV(10) MIXV(11)
    if (KIND == 0) c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
    else f3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, f3, 0, 0, 0);
    MIXV(12) MIXV(13) MIXV(14) MIXV(15)
#undef MIXV
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  // every wave's span: the SIMD's throughput is (last end - first start)
  if ((threadIdx.x & 63) == 0) {
    out[1 + 2 * (threadIdx.x >> 6)] = t0;
    out[2 + 2 * (threadIdx.x >> 6)] = t1;
  }
  uint32_t xs = 0;
  for (int i = 0; i < 16; i++) xs += x[i];
  sink[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + (int)xs + (int)(f0[0] + f1[1] + f2[2] + f3[3]);
}

// 5. dependent chains: D accumulators (D = 1: every MFMA waits for the one
//    before), 8 MFMAs per iteration, whole-workgroup span like 4.
template <int D>
__global__ void mfma_chain(int iters, unsigned long long* out, int* sink) {
  const uint32_t h0 = 0x9E3779B9u * (threadIdx.x + 1);
  v4i a = {(int)(h0 ^ 0x5bd1e995), (int)(h0 * 0x85ebca6b), (int)(h0 * 0xc2b2ae35), (int)(h0 + 0x27d4eb2f)};
  v4i b = {(int)(h0 * 0x165667b1), (int)(h0 ^ 0xd3a2646c), (int)(h0 * 0xfd7046c5), (int)(h0 + 0xb55a4f09)};
  v4i c[4] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int q = 0; q < 8; q++) c[q % D] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c[q % D], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    out[1 + 2 * (threadIdx.x >> 6)] = t0;
    out[2 + 2 * (threadIdx.x >> 6)] = t1;
  }
  sink[threadIdx.x] = c[0][0] + c[1 % 4][1] + c[2 % 4][2] + c[3][3];
}

__global__ void dma16_probe(const uint8_t* src, int nbytes, int shift, uint32_t* out) {
  __shared__ __align__(16) uint8_t lds[1024];
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, 0x00020000);
  const int lane = threadIdx.x;
  // granule `lane` (16 bytes) <- src bytes [shift + 16 lane, +16)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16,
                                           (uint32_t)(shift + 16 * lane), 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int k = 0; k < 4; k++) out[4 * lane + k] = reinterpret_cast<const uint32_t*>(lds)[4 * lane + k];
}

int main() {
  // 1. MFMA map
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; i++) hA[i] = (int8_t)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; i++) hB[i] = (int8_t)(rand() % 256 - 128);
  int hC[256], ref[256];
  for (int m = 0; m < 16; m++)
    for (int n = 0; n < 16; n++) {
      int s = 0;
      for (int k = 0; k < 64; k++) s += hA[m * 64 + k] * hB[k * 16 + n];
      ref[m * 16 + n] = s;
    }
  int8_t *dA, *dB;
  int* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, sizeof hC);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_i8_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; i++) bad += hC[i] != ref[i];
  printf("{\"probe\": \"mfma_i32_16x16x64_i8 map\", \"mismatches\": %d, \"C00\": %d, \"ref00\": %d}\n",
         bad, hC[0], ref[0]);

  // 2. unaligned LDS DMA
  uint8_t hs[1024];
  for (int i = 0; i < 1024; i++) hs[i] = (uint8_t)(i * 7 + 3);
  uint8_t* ds;
  uint32_t* dout;
  hipMalloc(&ds, sizeof hs);
  hipMalloc(&dout, 64 * 4);
  hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
  for (int shift = 0; shift < 4; shift++) {
    uint32_t hout[64];
    hipLaunchKernelGGL(dma_probe, dim3(1), dim3(64), 0, 0, ds, 1024, shift, dout);
    hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
    int exact = 0, floor4 = 0;
    for (int l = 0; l < 64; l++) {
      uint32_t e = 0, f = 0;
      for (int b = 0; b < 4; b++) {
        e |= (uint32_t)hs[shift + 4 * l + b] << (8 * b);
        f |= (uint32_t)hs[4 * l + b] << (8 * b);
      }
      exact += hout[l] == e;
      floor4 += hout[l] == f;
    }
    printf("{\"probe\": \"lds_dma_dword_unaligned\", \"shift\": %d, \"exact\": %d, \"rounded_down\": %d, \"of\": 64}\n",
           shift, exact, floor4);
  }
  {
    uint8_t* ds16;
    uint32_t* o16;
    uint8_t h16[2048];
    for (int i = 0; i < 2048; i++) h16[i] = (uint8_t)(i * 13 + 5);
    hipMalloc(&ds16, 2048);
    hipMalloc(&o16, 1024);
    hipMemcpy(ds16, h16, 2048, hipMemcpyHostToDevice);
    for (int shift : {0, 1, 2, 3, 4, 8}) {
      uint32_t ho[256];
      hipLaunchKernelGGL(dma16_probe, dim3(1), dim3(64), 0, 0, ds16, 2048, shift, o16);
      hipMemcpy(ho, o16, 1024, hipMemcpyDeviceToHost);
      int exact = 0;
      for (int w = 0; w < 256; w++) {
        uint32_t e = 0;
        for (int b = 0; b < 4; b++) e |= (uint32_t)h16[shift + 4 * w + b] << (8 * b);
        exact += ho[w] == e;
      }
      printf("{\"probe\": \"lds_dma_16B_unaligned\", \"shift\": %d, \"exact_dwords\": %d, \"of\": 256}\n", shift, exact);
    }
  }
  {
    unsigned long long* dt;
    int* sink;
    hipMalloc(&dt, 8);
    hipMalloc(&sink, 256);
    for (int kind = 0; kind < 2; kind++) {
      const int iters = 20000;
      unsigned long long cyc = 0;
      for (int rep = 0; rep < 2; rep++) {
        if (kind == 0) hipLaunchKernelGGL(mfma_rate<0>, dim3(1), dim3(64), 0, 0, iters, dt, sink);
        else hipLaunchKernelGGL(mfma_rate<1>, dim3(1), dim3(64), 0, 0, iters, dt, sink);
        hipMemcpy(&cyc, dt, 8, hipMemcpyDeviceToHost);
      }
      printf("{\"probe\": \"mfma issue\", \"kind\": \"%s\", \"cycles_per_mfma\": %.2f}\n",
             kind == 0 ? "i32_16x16x64_i8" : "f32_16x16x32_bf16", (double)cyc / (4.0 * iters));
    }
  }
  {
    unsigned long long* dt;
    int* sink;
    hipMalloc(&dt, 8);
    hipMalloc(&sink, 256);
    unsigned long long* dt2;
    hipMalloc(&dt2, 8 * (1 + 2 * 16));
    auto run = [&](auto kern, const char* name, int nv, int waves) {
      const int iters = 20000;
      unsigned long long cyc = 0, tt[1 + 2 * 16];
      for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64 * waves), 0, 0, iters, dt2, sink);
        hipMemcpy(tt, dt2, sizeof tt, hipMemcpyDeviceToHost);
      }
      unsigned long long lo = ~0ull, hi = 0;
      for (int w = 0; w < waves; w++) {
        lo = tt[1 + 2 * w] < lo ? tt[1 + 2 * w] : lo;
        hi = tt[2 + 2 * w] > hi ? tt[2 + 2 * w] : hi;
      }
      cyc = hi - lo;
      printf("{\"probe\": \"mfma+valu\", \"mfma\": \"%s\", \"valu_per_4mfma\": %d, \"waves_per_simd\": %d, \"simd_cycles_per_step\": %.1f}\n",
             name, nv, waves / 4, (double)cyc / iters / (waves / 4));
    };
    for (int waves : {4, 8, 16}) {
      run(mfma_valu_mix<0, 0>, "i8_16x16x64", 0, waves);
      run(mfma_valu_mix<0, 4>, "i8_16x16x64", 4, waves);
      run(mfma_valu_mix<0, 8>, "i8_16x16x64", 8, waves);
      run(mfma_valu_mix<0, 10>, "i8_16x16x64", 10, waves);
      run(mfma_valu_mix<0, 12>, "i8_16x16x64", 12, waves);
      run(mfma_valu_mix<0, 16>, "i8_16x16x64", 16, waves);
    }
  }
  {
    unsigned long long* dt2;
    int* sink;
    hipMalloc(&sink, 4096);
    hipMalloc(&dt2, 8 * (1 + 2 * 16));
    auto run = [&](auto kern, int d, int waves) {
      const int iters = 10000;
      unsigned long long tt[1 + 2 * 16];
      for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64 * waves), 0, 0, iters, dt2, sink);
        hipMemcpy(tt, dt2, sizeof tt, hipMemcpyDeviceToHost);
      }
      unsigned long long lo = ~0ull, hi = 0;
      for (int w = 0; w < waves; w++) {
        lo = tt[1 + 2 * w] < lo ? tt[1 + 2 * w] : lo;
        hi = tt[2 + 2 * w] > hi ? tt[2 + 2 * w] : hi;
      }
      printf("{\"probe\": \"mfma chain\", \"accumulators\": %d, \"waves_per_simd\": %d, \"simd_cycles_per_mfma\": %.2f}\n",
             d, waves / 4, (double)(hi - lo) / iters / 8 / (waves / 4));
    };
    for (int waves : {4, 8, 16}) {
      run(mfma_chain<1>, 1, waves);
      run(mfma_chain<2>, 2, waves);
      run(mfma_chain<4>, 4, waves);
    }
  }
  hipError_t e = hipDeviceSynchronize();
  printf("{\"probe\": \"done\", \"status\": \"%s\"}\n", hipGetErrorString(e));
  return 0;
}
