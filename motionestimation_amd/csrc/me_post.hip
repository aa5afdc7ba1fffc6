// me_post.hip -- consumers of the MV field on the GPU.
//
// Reference: motionCompensatedFrame src/common/utils.c:102-134 (mc[p] =
// ref[p + mv(block of p)] when in frame), frameDiff :94-100, imagePSNR
// :137-164 (MAX = largest pixel of either frame), and the 5-plane output
// [ref, cur, mc, |ref-cur|, |mc-cur|] of src/cpu/main.c:161-168.
// One lane per 4 pixels; PSNR's sum of squares and MAX are reduced per wave and
// folded with one 64-bit atomic each (exact integers, order-independent).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_kernels.h"

namespace me {

__global__ __launch_bounds__(256) void me_compensate_kernel(const uint8_t* __restrict__ ref,
                                                            const uint8_t* __restrict__ cur,
                                                            int width, int height, int blk,
                                                            const int16_t* __restrict__ mv,
                                                            uint8_t* __restrict__ out5,
                                                            int write_planes,
                                                            unsigned long long* stats) {
  const size_t n = (size_t)width * height;
  const int nbx = (width + blk - 1) / blk;
  const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  unsigned long long sq = 0;
  uint32_t mx = 0;
  for (int k = 0; k < 4; k++) {
    const size_t i = i0 + k;
    if (i >= n) break;
    const int y = (int)(i / width), x = (int)(i % width);
    const int b = (y / blk) * nbx + x / blk;
    const int px = x + mv[2 * b], py = y + mv[2 * b + 1];
    const uint8_t r = ref[i], c = cur[i];
    uint8_t m = 0;
    if (px >= 0 && py >= 0 && px < width && py < height) m = ref[(size_t)py * width + px];
    const int d = (int)m - (int)c;
    sq += (unsigned long long)(d * d);
    mx = max(mx, (uint32_t)max(m, c));
    if (write_planes) {
      out5[i] = r;
      out5[n + i] = c;
      out5[2 * n + i] = m;
      out5[3 * n + i] = (uint8_t)abs((int)r - (int)c);
      out5[4 * n + i] = (uint8_t)abs(d);
    } else {
      out5[i] = m;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sq += __shfl_xor(sq, off, 64);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&stats[0], sq);
    atomicMax(&stats[1], (unsigned long long)mx);
  }
}

hipError_t launch_compensate(const uint8_t* ref, const uint8_t* cur, int width, int height,
                             int blk, const int16_t* mv, uint8_t* out5, int write_planes,
                             unsigned long long* stats, hipStream_t stream) {
  const size_t n = (size_t)width * height;
  const unsigned grid = (unsigned)((n + 4 * 256 - 1) / (4 * 256));
  hipLaunchKernelGGL(me_compensate_kernel, dim3(grid), dim3(256), 0, stream, ref, cur, width,
                     height, blk, mv, out5, write_planes, stats);
  return hipGetLastError();
}

}  // namespace me
