// Device-wide exclusive scan of 0/1 byte flags into int32 ranks (shared by frontend.hip and mesh.hip; kernels
// in an anonymous namespace: each translation unit gets its own copy).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ofx_common.h"

namespace ofx {
namespace {

// Device-wide exclusive scan of 0/1 byte flags into int32 ranks (total at out[n]); fixed order, no
// atomics. Tiles of 4096 flags: one 256-thread workgroup per tile, 16 flags per thread.
constexpr int kScanTile = 4096;

__device__ __forceinline__ int block_exscan256(int v, int& total) {
  __shared__ int s_w[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int base = 0;
  for (int q = 0; q < w; ++q) base += s_w[q];
  total = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
  __syncthreads();
  return base + x - v;
}

__device__ __forceinline__ int thread_flags(const uint8_t* __restrict__ in, int64_t n, int64_t i0, uint8_t f[16]) {
  int c = 0;
  if (i0 + 16 <= n && ((uintptr_t)(in + i0) & 15) == 0) {
    const uint4 q = *(const uint4*)(in + i0);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) { f[j] = (uint8_t)((w[j >> 2] >> (8 * (j & 3))) & 0xFF); c += f[j]; }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) { f[j] = i0 + j < n ? in[i0 + j] : 0; c += f[j]; }
  }
  return c;
}

__global__ __launch_bounds__(256) void k_scan_tiles(const uint8_t* __restrict__ in, int64_t n, int32_t* __restrict__ tsum) {
  uint8_t f[16];
  const int c = thread_flags(in, n, (int64_t)blockIdx.x * kScanTile + threadIdx.x * 16, f);
  int tot;
  (void)block_exscan256(c, tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of the tile sums in place; grand total at tsum[nt]
__global__ __launch_bounds__(256) void k_scan_tile_offsets(int32_t* __restrict__ tsum, int nt) {
  int carry = 0;
  for (int b = 0; b < nt; b += 256) {
    const int i = b + (int)threadIdx.x;
    const int v = i < nt ? tsum[i] : 0;
    int tot;
    const int e = block_exscan256(v, tot);
    if (i < nt) tsum[i] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) tsum[nt] = carry;
}

__global__ __launch_bounds__(256) void k_scan_apply(const uint8_t* __restrict__ in, int64_t n,
                                                    const int32_t* __restrict__ toff, int nt, int32_t* __restrict__ out) {
  uint8_t f[16];
  const int64_t i0 = (int64_t)blockIdx.x * kScanTile + threadIdx.x * 16;
  const int c = thread_flags(in, n, i0, f);
  int tot;
  int r = block_exscan256(c, tot) + toff[blockIdx.x];
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (i0 + j < n) { out[i0 + j] = r; r += f[j]; }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = toff[nt];
}

inline int64_t scan_tiles(int64_t n) { return (n + kScanTile - 1) / kScanTile; }

// out: int32[n+1]; tsum: int32[scan_tiles(n)+1] scratch
inline int scan_flags(const uint8_t* in, int64_t n, int32_t* out, int32_t* tsum, hipStream_t s) {
  const int64_t nt = scan_tiles(n);
  if (nt == 0) return hipMemsetAsync(out, 0, sizeof(int32_t), s) == hipSuccess ? OFX_OK : OFX_ERR_HIP;
  hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)nt), dim3(256), 0, s, in, n, tsum);
  hipLaunchKernelGGL(k_scan_tile_offsets, dim3(1), dim3(256), 0, s, tsum, (int)nt);
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nt), dim3(256), 0, s, in, n, (const int32_t*)tsum, (int)nt, out);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

}  // namespace
}  // namespace ofx
