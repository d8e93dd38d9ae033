// Shared helpers of libofx: error plumbing, brick indexing, exact-arithmetic notes.
//
// Build contract: every translation unit is compiled with -ffp-contract=off so that
// f32/f64 expressions round exactly like the reference numpy/numba code they restate
// (no fused multiply-add contraction); see DESIGN.md §Numerics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/ofx.h"

namespace ofx {

void set_error(const char* fmt, ...);

#define OFX_CHECK_ARG(cond, ...)        \
  do {                                  \
    if (!(cond)) {                      \
      ::ofx::set_error(__VA_ARGS__);    \
      return OFX_ERR_ARG;               \
    }                                   \
  } while (0)

#define OFX_HIP(call)                                                               \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::ofx::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return OFX_ERR_HIP;                                                           \
    }                                                                               \
  } while (0)

#define OFX_LAUNCH_CHECK() OFX_HIP(hipGetLastError())

constexpr int kBrick = 8;            // brick edge (voxels)
constexpr int kBrickVox = 512;       // voxels per brick
constexpr uint16_t kNoAnchor = 0xFFFF;
constexpr int kPal = 64;             // node palette entries per brick (skin cache, integrate)
constexpr uint8_t kNoLocal = 0xFF;   // palette-local anchor of a skin-invalid voxel

// Brick geometry of one shard. Bricks are numbered brick-major in C order over the shard:
// b = ((bx - bx0) * nby + by) * nbz + bz ; voxel within brick l = (lx*8 + ly)*8 + lz.
struct BrickGeom {
  int32_t Dx, Dy, Dz;
  int32_t nbx, nby, nbz;   // full-volume brick counts
  int32_t bx0, bx1;        // shard range along x
  int32_t px0, px1;        // marching cubes: far corners processed along x (whole volume: [0, Dx))
  int64_t n_bricks;        // bricks in shard
  float ox, oy, oz;
  double vs;
};

inline int make_geom(const ofx_volume_desc* d, BrickGeom* g) {
  if (!d) { set_error("null volume desc"); return OFX_ERR_ARG; }
  if (d->dim[0] <= 0 || d->dim[1] <= 0 || d->dim[2] <= 0) { set_error("bad volume dims"); return OFX_ERR_ARG; }
  g->Dx = d->dim[0]; g->Dy = d->dim[1]; g->Dz = d->dim[2];
  g->nbx = (g->Dx + kBrick - 1) / kBrick;
  g->nby = (g->Dy + kBrick - 1) / kBrick;
  g->nbz = (g->Dz + kBrick - 1) / kBrick;
  g->bx0 = d->brick_x0; g->bx1 = d->brick_x1;
  if (g->bx0 < 0 || g->bx1 > g->nbx || g->bx0 >= g->bx1) { set_error("bad brick shard range [%d,%d) of %d", g->bx0, g->bx1, g->nbx); return OFX_ERR_ARG; }
  g->n_bricks = (int64_t)(g->bx1 - g->bx0) * g->nby * g->nbz;
  g->px0 = 0; g->px1 = g->Dx;
  g->ox = d->origin[0]; g->oy = d->origin[1]; g->oz = d->origin[2];
  g->vs = d->voxel_size;
  return OFX_OK;
}

// vox2world (tsdf.py:338-349): f32 origin + f64 voxel_size * coord, computed in f64, stored f32.
__device__ __forceinline__ float vox2world(float o, double vs, int i) {
  return (float)((double)o + vs * (double)i);
}

inline hipStream_t as_stream(ofx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace ofx
