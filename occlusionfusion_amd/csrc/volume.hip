// Volume storage kernels: reset, brick <-> C-order conversion, colour packing, node packing.
//   TSDFVolume.__init__ dense init        fusion_with_occlusion/tsdf.py:133-141
//   TSDFVolume.get_volume / load_volume   tsdf.py:673-702
//   TSDFVolume.update colour folding      tsdf.py:545-566
#include <stdarg.h>
#include <stdio.h>

#include "ofx_common.h"

namespace ofx {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

__global__ void k_fill3(float4* __restrict__ a, float va, float4* __restrict__ b, float vb,
                        float4* __restrict__ c, float vc, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    a[i] = make_float4(va, va, va, va);
    if (b) b[i] = make_float4(vb, vb, vb, vb);
    if (c) c[i] = make_float4(vc, vc, vc, vc);
  }
}

template <bool TO_DENSE>
__global__ void k_brick_dense(BrickGeom g, const float* __restrict__ src, float* __restrict__ dst, int32_t x_lo,
                              int32_t x_n) {
  const int64_t n = (int64_t)x_n * g.Dy * g.Dz;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = t % g.Dz;
    int64_t r = t / g.Dz;
    int64_t j = r % g.Dy;
    int64_t i = r / g.Dy + x_lo;
    int64_t b = ((i / kBrick - g.bx0) * g.nby + j / kBrick) * g.nbz + k / kBrick;
    int64_t l = ((i % kBrick) * kBrick + (j % kBrick)) * kBrick + (k % kBrick);
    if (TO_DENSE)
      dst[t] = src[b * kBrickVox + l];
    else
      dst[b * kBrickVox + l] = src[t];
  }
}

// tsdf.py:561-562 : c = 255*rgb (f32); floor(c_b*65536 + c_g*256 + c_r), left to right in f32.
__global__ void k_pack_color(const float* __restrict__ rgb, int64_t hw, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < hw; i += (int64_t)gridDim.x * blockDim.x) {
    float r = 255.0f * rgb[i];
    float gg = 255.0f * rgb[hw + i];
    float b = 255.0f * rgb[2 * hw + i];
    float s = b * 65536.0f + gg * 256.0f;
    s = s + r;
    out[i] = floorf(s);
  }
}

// packed node record (64 B): [R00 R01 R02 g0][R10 R11 R12 g1][R20 R21 R22 g2][t0 t1 t2 0]
__global__ void k_pack_nodes(const float* __restrict__ R, const float* __restrict__ T, const float* __restrict__ G,
                             int32_t n, float4* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = R + 9 * (int64_t)i;
  const float* g = G + 3 * (int64_t)i;
  const float* t = T + 3 * (int64_t)i;
  // pair-interleaved for packed-f32 warps: (R00,R10)(R01,R11) | (R02,R12)(g0,g1) | (t0,t1)(R20,R21) | R22 g2 t2 0
  out[4 * (int64_t)i + 0] = make_float4(r[0], r[3], r[1], r[4]);
  out[4 * (int64_t)i + 1] = make_float4(r[2], r[5], g[0], g[1]);
  out[4 * (int64_t)i + 2] = make_float4(t[0], t[1], r[6], r[7]);
  out[4 * (int64_t)i + 3] = make_float4(r[8], g[2], t[2], 0.f);
}

static int shard_x_range(const BrickGeom& g, int32_t* lo, int32_t* n) {
  *lo = g.bx0 * kBrick;
  int32_t hi = g.bx1 * kBrick;
  if (hi > g.Dx) hi = g.Dx;
  *n = hi - *lo;
  return OFX_OK;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

const char* ofx_last_error(void) { return ofx::g_err; }
int ofx_abi_version(void) { return OFX_ABI_VERSION; }

int ofx_volume_num_slots(const ofx_volume_desc* desc, int64_t* n_slots) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(n_slots, "null n_slots");
  *n_slots = g.n_bricks * kBrickVox;
  return OFX_OK;
}

int ofx_volume_reset(const ofx_volume_desc* desc, float* tsdf, float* weight, float* color, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(tsdf, "null tsdf");
  int64_t n4 = g.n_bricks * kBrickVox / 4;
  hipLaunchKernelGGL(k_fill3, dim3(grid_for(n4, 256, 8192)), dim3(256), 0, as_stream(s), (float4*)tsdf, 1.0f,
                     (float4*)weight, 0.0f, (float4*)color, 0.0f, n4);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_volume_to_dense(const ofx_volume_desc* desc, const float* bricked, float* dense, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(bricked && dense, "null buffer");
  int32_t lo, n;
  shard_x_range(g, &lo, &n);
  int64_t total = (int64_t)n * g.Dy * g.Dz;
  hipLaunchKernelGGL(k_brick_dense<true>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, as_stream(s), g, bricked,
                     dense, lo, n);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_volume_from_dense(const ofx_volume_desc* desc, const float* dense, float* bricked, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(bricked && dense, "null buffer");
  int32_t lo, n;
  shard_x_range(g, &lo, &n);
  int64_t total = (int64_t)n * g.Dy * g.Dz;
  hipLaunchKernelGGL(k_brick_dense<false>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, as_stream(s), g, dense,
                     bricked, lo, n);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_pack_color(const float* rgb, int32_t height, int32_t width, float* packed, ofx_stream_t s) {
  OFX_CHECK_ARG(rgb && packed && height > 0 && width > 0, "bad pack_color args");
  int64_t hw = (int64_t)height * width;
  hipLaunchKernelGGL(k_pack_color, dim3(grid_for(hw, 256, 4096)), dim3(256), 0, as_stream(s), rgb, hw, packed);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_pack_nodes(const float* R, const float* T, const float* G, int32_t n_nodes, float* packed, ofx_stream_t s) {
  OFX_CHECK_ARG(R && T && G && packed && n_nodes > 0, "bad pack_nodes args");
  hipLaunchKernelGGL(k_pack_nodes, dim3(grid_for(n_nodes, 256)), dim3(256), 0, as_stream(s), R, T, G, n_nodes,
                     (float4*)packed);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

}  // extern "C"
