// TSDF raycast: depth / normal / colour images of the fused volume seen from the camera (identity pose, the
// reference's convention, tsdf.py:329-336). New capability: the reference has no raycast (its surfaces come
// from marching cubes, tsdf.py:770-809; its only renderer is the pytorch3d point rasteriser,
// NonRigidICP/model/point_render.py:82, weighted 0 in NonRigidICP/config.yaml:6,10) — parity unpinned; the
// arithmetic below is restated op for op by oracle/fusion_oracle.py::raycast (f32, un-contracted).
//
// Per pixel (u, v): ray p(z) = z·(dx, dy, 1), dx = (u - cx)/fx, dy = (v - cy)/fy (correctly rounded f32).
// z runs from the entry into the volume box (and >= z_near) to the exit (and <= z_far), sampling the tsdf
// trilinearly (unobserved voxels — weight 0 — and voxels outside the volume count as +1, empty space) with a
// coarse step while the sample is truncated (>= 0.999) and a fine step (one voxel) otherwise. The first
// sign change + -> - between two taken samples is the surface: z* = z0 + (z1 - z0)·s0/(s0 - s1) (a ray whose
// first sample is already negative has no positive sample before it: no hit there). Normal: normalised central
// differences of the trilinear tsdf at p(z*) (+-1 voxel per axis). Colour: the packed colour of the voxel
// nearest p(z*). Misses give depth 0, normal 0, colour 0.
//
// MI355X layout: one thread per pixel, 256-thread workgroups of 16x16 pixel tiles (neighbouring rays walk
// neighbouring bricks: the trilinear gathers of a tile hit the same 2 KiB brick lines in L2).
#include "ofx_common.h"

namespace ofx {

struct RayGeom {
  BrickGeom g;
  float lo[3], hi[3], inv_vs, vs;
  float fx, fy, cx, cy;
  int W, H;
  float z_near, z_far, step_coarse, step_fine;
  int max_steps;
};

__device__ __forceinline__ float rdiv(float a, float b) { return (float)((double)a / (double)b); }

// tsdf value of voxel (i, j, k) for the raycast: +1 outside the volume or unobserved
__device__ __forceinline__ float ray_voxel(const RayGeom& r, const float* __restrict__ tsdf,
                                           const float* __restrict__ weight, int i, int j, int k) {
  const BrickGeom& g = r.g;
  if (i < 0 || j < 0 || k < 0 || i >= g.Dx || j >= g.Dy || k >= g.Dz) return 1.0f;
  const int64_t b = ((int64_t)(i >> 3) * g.nby + (j >> 3)) * g.nbz + (k >> 3);
  const int64_t s = b * kBrickVox + ((i & 7) * 8 + (j & 7)) * 8 + (k & 7);
  return weight[s] > 0.0f ? tsdf[s] : 1.0f;
}

// trilinear tsdf at grid coordinates q = (p - lo)·inv_vs (op order restated in the oracle)
__device__ __forceinline__ float ray_trilinear(const RayGeom& r, const float* __restrict__ tsdf,
                                               const float* __restrict__ weight, float qx, float qy, float qz) {
  const float fx0 = floorf(qx), fy0 = floorf(qy), fz0 = floorf(qz);
  const float ax = qx - fx0, ay = qy - fy0, az = qz - fz0;
  const int i = (int)fx0, j = (int)fy0, k = (int)fz0;
  const float t000 = ray_voxel(r, tsdf, weight, i, j, k), t100 = ray_voxel(r, tsdf, weight, i + 1, j, k);
  const float t010 = ray_voxel(r, tsdf, weight, i, j + 1, k), t110 = ray_voxel(r, tsdf, weight, i + 1, j + 1, k);
  const float t001 = ray_voxel(r, tsdf, weight, i, j, k + 1), t101 = ray_voxel(r, tsdf, weight, i + 1, j, k + 1);
  const float t011 = ray_voxel(r, tsdf, weight, i, j + 1, k + 1);
  const float t111 = ray_voxel(r, tsdf, weight, i + 1, j + 1, k + 1);
  const float bx = 1.0f - ax, by = 1.0f - ay, bz = 1.0f - az;
  const float c00 = t000 * bx + t100 * ax, c10 = t010 * bx + t110 * ax;
  const float c01 = t001 * bx + t101 * ax, c11 = t011 * bx + t111 * ax;
  const float c0 = c00 * by + c10 * ay, c1 = c01 * by + c11 * ay;
  return c0 * bz + c1 * az;
}

__device__ __forceinline__ float ray_sample(const RayGeom& r, const float* __restrict__ tsdf,
                                            const float* __restrict__ weight, float dx, float dy, float z) {
  const float qx = (z * dx - r.lo[0]) * r.inv_vs;
  const float qy = (z * dy - r.lo[1]) * r.inv_vs;
  const float qz = (z - r.lo[2]) * r.inv_vs;
  return ray_trilinear(r, tsdf, weight, qx, qy, qz);
}

__global__ __launch_bounds__(256) void k_raycast(RayGeom r, const float* __restrict__ tsdf,
                                                 const float* __restrict__ weight, const float* __restrict__ color,
                                                 float* __restrict__ depth, float* __restrict__ normal,
                                                 float* __restrict__ color_out) {
  const int u = blockIdx.x * 16 + (threadIdx.x & 15), v = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (u >= r.W || v >= r.H) return;
  const int64_t pix = (int64_t)v * r.W + u;
  const float dx = rdiv((float)u - r.cx, r.fx), dy = rdiv((float)v - r.cy, r.fy);
  // entry / exit depth of the volume box along the ray (slab test per axis, z-parameterised)
  float z0 = r.z_near, z1 = r.z_far;
  const float d[3] = {dx, dy, 1.0f};
  bool miss = false;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (d[a] == 0.0f) {
      if (!(0.0f >= r.lo[a] && 0.0f <= r.hi[a])) miss = true;
    } else {
      const float ta = rdiv(r.lo[a], d[a]), tb = rdiv(r.hi[a], d[a]);
      z0 = fmaxf(z0, fminf(ta, tb));
      z1 = fminf(z1, fmaxf(ta, tb));
    }
  }
  float hit = 0.0f;
  if (!miss && z0 <= z1) {
    // a sign change needs a real positive sample before it: a ray that enters the volume (or starts at z_near)
    // inside an observed negative region reports no surface at the entry plane
    float z = z0, zp = z0, sp = 1.0f;
    bool have_prev = false;
    for (int n = 0; n < r.max_steps && z <= z1; ++n) {
      const float s = ray_sample(r, tsdf, weight, dx, dy, z);
      if (have_prev && sp > 0.0f && s < 0.0f) {
        hit = zp + (z - zp) * rdiv(sp, sp - s);
        break;
      }
      have_prev = true;
      zp = z;
      sp = s;
      z = z + (s >= 0.999f ? r.step_coarse : r.step_fine);
    }
  }
  depth[pix] = hit;
  if (normal) {
    float nx = 0.0f, ny = 0.0f, nz = 0.0f;
    if (hit > 0.0f) {
      const float qx = (hit * dx - r.lo[0]) * r.inv_vs, qy = (hit * dy - r.lo[1]) * r.inv_vs;
      const float qz = (hit - r.lo[2]) * r.inv_vs;
      nx = ray_trilinear(r, tsdf, weight, qx + 1.0f, qy, qz) - ray_trilinear(r, tsdf, weight, qx - 1.0f, qy, qz);
      ny = ray_trilinear(r, tsdf, weight, qx, qy + 1.0f, qz) - ray_trilinear(r, tsdf, weight, qx, qy - 1.0f, qz);
      nz = ray_trilinear(r, tsdf, weight, qx, qy, qz + 1.0f) - ray_trilinear(r, tsdf, weight, qx, qy, qz - 1.0f);
      const float len = (float)sqrt((double)((nx * nx + ny * ny) + nz * nz));
      if (len > 0.0f) { nx = rdiv(nx, len); ny = rdiv(ny, len); nz = rdiv(nz, len); }
    }
    normal[3 * pix] = nx; normal[3 * pix + 1] = ny; normal[3 * pix + 2] = nz;
  }
  if (color_out) {
    float c = 0.0f;
    if (hit > 0.0f && color) {
      const int i = (int)floorf((hit * dx - r.lo[0]) * r.inv_vs + 0.5f);
      const int j = (int)floorf((hit * dy - r.lo[1]) * r.inv_vs + 0.5f);
      const int k = (int)floorf((hit - r.lo[2]) * r.inv_vs + 0.5f);
      const BrickGeom& g = r.g;
      if (i >= 0 && j >= 0 && k >= 0 && i < g.Dx && j < g.Dy && k < g.Dz) {
        const int64_t b = ((int64_t)(i >> 3) * g.nby + (j >> 3)) * g.nbz + (k >> 3);
        c = color[b * kBrickVox + ((i & 7) * 8 + (j & 7)) * 8 + (k & 7)];
      }
    }
    color_out[pix] = c;
  }
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_raycast(const ofx_volume_desc* desc, const ofx_camera* cam, const float* tsdf, const float* weight,
                const float* color, float z_near, float z_far, float* depth, float* normals, float* colors,
                ofx_stream_t s) {
  RayGeom r;
  int st = make_geom(desc, &r.g);
  if (st) return st;
  OFX_CHECK_ARG(r.g.bx0 == 0 && r.g.bx1 == r.g.nbx, "raycast needs the whole volume (brick range [0, nbx))");
  OFX_CHECK_ARG(cam && cam->width > 0 && cam->height > 0 && cam->fx != 0.f && cam->fy != 0.f, "bad camera");
  OFX_CHECK_ARG(tsdf && weight && depth, "null buffer");
  OFX_CHECK_ARG(z_far > z_near, "z_far <= z_near");
  const double vs = desc->voxel_size;
  for (int a = 0; a < 3; ++a) {
    r.lo[a] = desc->origin[a];
    r.hi[a] = (float)((double)desc->origin[a] + vs * (double)desc->dim[a]);
  }
  r.vs = (float)vs;
  r.inv_vs = (float)(1.0 / vs);
  r.fx = cam->fx; r.fy = cam->fy; r.cx = cam->cx; r.cy = cam->cy;
  r.W = cam->width; r.H = cam->height;
  r.z_near = z_near; r.z_far = z_far;
  r.step_coarse = (float)(0.8 * desc->trunc_margin);
  r.step_fine = (float)vs;
  r.max_steps = 1 << 16;
  dim3 grid((unsigned)((r.W + 15) / 16), (unsigned)((r.H + 15) / 16));
  hipLaunchKernelGGL(k_raycast, grid, dim3(256), 0, as_stream(s), r, tsdf, weight, color, depth, normals, colors);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

}  // extern "C"
