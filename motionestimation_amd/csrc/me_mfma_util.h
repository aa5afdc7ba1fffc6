// me_mfma_util.h -- device helpers shared by the matrix-core SSD kernels
// (me_mfma.hip: prepass + block-major / tile / 8x8 kernels; me_band.hip: the
// band-walk kernel).  Internal to libme_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_kernels.h"

namespace me {
namespace mfma {

typedef int v4i __attribute__((ext_vector_type(4)));

#define MFMA16 __builtin_amdgcn_mfma_i32_16x16x64_i8

// A value the compiler must treat as unknown (keeps one base per call instead
// of hoisting a set of derived addresses that then spill).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Job j of a batched launch: its planes, records and prepass planes.
__device__ __forceinline__ void mfma_job(const MfmaJobs& jb, int j, SearchArgs& p, MfmaGeom& g) {
  p.ref = jb.ref[j];
  p.cur = jb.cur[j];
  p.mv = jb.mv[j];
  p.cost = jb.cost[j];
  const size_t off = (size_t)j * jb.scratch_stride;
  g.rp += off;
  g.s2 = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(g.s2) + off);
  if (g.s2h) g.s2h = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(g.s2h) + off);
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t lshl6_add(uint32_t a, uint32_t b_sgpr) {
  uint32_t d;
  asm("v_lshl_add_u32 %0, %1, 6, %2" : "=v"(d) : "v"(a), "s"(b_sgpr));
  return d;
}

// XCD-banded workgroup order: the hardware deals blocks b, b + 8, ... to one
// XCD (a speed heuristic only, MI355X_MICROARCH.md), so XCD x walks one
// contiguous run of the linear work index.
__device__ __forceinline__ int xcd_banded_index() {
  const int nwg = (int)gridDim.x, bid = (int)blockIdx.x;
  const int x = bid & 7, m = bid >> 3, q = nwg >> 3, rem = nwg & 7;
  return x * q + min(x, rem) + m;
}

}  // namespace mfma
}  // namespace me
