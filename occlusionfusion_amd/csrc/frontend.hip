// Correspondence front-end plumbing: depth backprojection and the pixel-grid
// mesh of a point image, bit-exact with the reference C++ (csrc/cpu/image_proc.cpp).
//
//   ofx_backproject_depth   image_proc::backproject_depth_float / _ushort   csrc/cpu/image_proc.cpp:351-401
//                           (wrapper utils/image_proc.py:335-349)
//   ofx_depth_mesh_*        image_proc::compute_mesh_from_depth             csrc/cpu/image_proc.cpp:405-545
//                           (callers embedded_deformation_graph.py:95-151, warpfield.py:160-175)
//   ofx_depth_to_pc         depth_2_pc + masked compaction + map_pixel_to_pcd NonRigidICP/model/geometry.py:44-59,
//                           (Registration.optimize target cloud)            registration_fusion.py:104-109,388-395
//
// compute_mesh_from_depth numbers vertices in the order a sequential scan first uses them (quads in
// row-major order; per quad triangle A = (00, 01, 10) then B = (11, 10, 01)). Here every use of a
// pixel is a key (quad·6 + slot, slots A:00=0 01=1 10=2, B:11=3 10=4 01=5), each pixel finds its
// smallest key among the valid triangles that use it, and vertex ids are ranks of those keys (flags
// over the key space + one scan) — the sequential order, computed in parallel. Faces likewise are
// ranks of (quad·2 + triangle). Triangle test: all three z > 0 and every Eigen f32 edge length
// sqrt(dx²+(dy²+dz²)) <= max distance (Eigen's order).
#include "ofx_common.h"
#include "scan_flags.h"

namespace ofx {

__device__ __forceinline__ float fdiv(float a, float b) { return (float)((double)a / (double)b); }

template <bool U16>
__global__ __launch_bounds__(256) void k_backproject(const void* __restrict__ depth, int H, int W, float fx, float fy,
                                                      float cx, float cy, float normalizer, float* __restrict__ out) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int y = (int)(p / W), x = (int)(p % W);
  float d;
  if (U16) d = fdiv((float)((const uint16_t*)depth)[p], normalizer);
  else d = ((const float*)depth)[p];
  if (d > 0.f) {
    const int64_t hw = (int64_t)H * W;
    out[p] = fdiv(d * ((float)x - cx), fx);
    out[hw + p] = fdiv(d * ((float)y - cy), fy);
    out[2 * hw + p] = d;
  }
}

struct PImg {
  const float* p;
  int H, W;
  float maxd;
  __device__ __forceinline__ float3 at(int x, int y) const {
    const int64_t hw = (int64_t)H * W, i = (int64_t)y * W + x;
    return make_float3(p[i], p[hw + i], p[2 * hw + i]);
  }
};

__device__ __forceinline__ float dist3(float3 a, float3 b) {
  const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  // Eigen 3.3.7's unrolled redux sums a 3-vector as x0 + (x1 + x2) (Redux.h:92-104); checked against the
  // compiled csrc on threshold-straddling cases (tests/golden/make_golden.py).
  return (float)sqrt((double)(dx * dx + (dy * dy + dz * dz)));
}

// triangle t (0: A = 00,01,10; 1: B = 11,10,01) of quad (x, y) valid?
__device__ __forceinline__ bool tri_valid(const PImg& im, int x, int y, int t) {
  if (x < 0 || y < 0 || x >= im.W - 1 || y >= im.H - 1) return false;
  const float3 o01 = im.at(x, y + 1), o10 = im.at(x + 1, y);
  const float3 o = t == 0 ? im.at(x, y) : im.at(x + 1, y + 1);
  if (!(o.z > 0.f && o01.z > 0.f && o10.z > 0.f)) return false;
  if (t == 0) return dist3(o, o01) <= im.maxd && dist3(o, o10) <= im.maxd && dist3(o01, o10) <= im.maxd;
  return dist3(o10, o01) <= im.maxd && dist3(o10, o) <= im.maxd && dist3(o01, o) <= im.maxd;
}

// smallest key of pixel (x, y) over its uses by valid triangles, or -1
__device__ __forceinline__ int64_t pixel_key(const PImg& im, int x, int y) {
  const int QW = im.W - 1;
  auto key = [&](int qx, int qy, int slot) { return ((int64_t)qy * QW + qx) * 6 + slot; };
  if (tri_valid(im, x - 1, y - 1, 1)) return key(x - 1, y - 1, 3);   // as 11 of the quad up-left
  if (tri_valid(im, x, y - 1, 0)) return key(x, y - 1, 1);           // as 01 of the quad above (A)
  if (tri_valid(im, x, y - 1, 1)) return key(x, y - 1, 5);           //                        (B)
  if (tri_valid(im, x - 1, y, 0)) return key(x - 1, y, 2);           // as 10 of the quad left (A)
  if (tri_valid(im, x - 1, y, 1)) return key(x - 1, y, 4);           //                       (B)
  if (tri_valid(im, x, y, 0)) return key(x, y, 0);                   // as 00 of its own quad (A)
  return -1;
}

__global__ __launch_bounds__(256) void k_dm_flags(PImg im, uint8_t* __restrict__ kflag, uint8_t* __restrict__ tflag) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= (int64_t)im.H * im.W) return;
  const int y = (int)(p / im.W), x = (int)(p % im.W);
  const int64_t k = pixel_key(im, x, y);
  if (k >= 0) kflag[k] = 1;
  if (x < im.W - 1 && y < im.H - 1) {
    const int64_t q = (int64_t)y * (im.W - 1) + x;
    tflag[2 * q] = tri_valid(im, x, y, 0);
    tflag[2 * q + 1] = tri_valid(im, x, y, 1);
  }
}

__global__ __launch_bounds__(256) void k_dm_verts(PImg im, const int32_t* __restrict__ krank, int32_t* __restrict__ vid,
                                                   float* __restrict__ verts, int32_t* __restrict__ pixels) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= (int64_t)im.H * im.W) return;
  const int y = (int)(p / im.W), x = (int)(p % im.W);
  const int64_t k = pixel_key(im, x, y);
  if (k < 0) { vid[p] = -1; return; }
  const int32_t v = krank[k];
  vid[p] = v;
  const float3 o = im.at(x, y);
  verts[3 * (int64_t)v] = o.x; verts[3 * (int64_t)v + 1] = o.y; verts[3 * (int64_t)v + 2] = o.z;
  if (pixels) { pixels[2 * (int64_t)v] = x; pixels[2 * (int64_t)v + 1] = y; }
}

__global__ __launch_bounds__(256) void k_dm_faces(int H, int W, const uint8_t* __restrict__ tflag,
                                                   const int32_t* __restrict__ trank, const int32_t* __restrict__ vid,
                                                   int32_t* __restrict__ faces) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nq = (int64_t)(H - 1) * (W - 1);
  if (t >= 2 * nq || !tflag[t]) return;
  const int64_t q = t >> 1;
  const int y = (int)(q / (W - 1)), x = (int)(q % (W - 1));
  const int64_t i00 = (int64_t)y * W + x, i01 = i00 + W, i10 = i00 + 1, i11 = i00 + W + 1;
  const int64_t f = trank[t];
  if ((t & 1) == 0) { faces[3 * f] = vid[i00]; faces[3 * f + 1] = vid[i01]; faces[3 * f + 2] = vid[i10]; }
  else { faces[3 * f] = vid[i11]; faces[3 * f + 1] = vid[i10]; faces[3 * f + 2] = vid[i01]; }
}

struct DepthMesh {
  PImg im{};
  int64_t cap_px = 0;
  uint8_t *kflag = nullptr, *tflag = nullptr;
  int32_t *krank = nullptr, *trank = nullptr, *vid = nullptr, *tsum = nullptr;
  int64_t n_verts = 0, n_faces = 0;
  bool counted = false;
};

#define OFX_CHECK(call)            \
  do {                             \
    const int st_ = (call);        \
    if (st_ != OFX_OK) return st_; \
  } while (0)

// scratch for images of up to npx pixels: key flags/ranks (6 per pixel), triangle flags/ranks (2 per pixel)
inline int reserve(DepthMesh* m, int64_t npx) {
  if (npx <= m->cap_px) return OFX_OK;
  for (void** p : {(void**)&m->kflag, (void**)&m->tflag, (void**)&m->krank, (void**)&m->trank, (void**)&m->vid,
                   (void**)&m->tsum})
    if (*p) { OFX_HIP(hipFree(*p)); *p = nullptr; }
  m->cap_px = 0;
  OFX_HIP(hipMalloc((void**)&m->kflag, 6 * npx));
  OFX_HIP(hipMalloc((void**)&m->tflag, 2 * npx));
  OFX_HIP(hipMalloc((void**)&m->krank, (6 * npx + 1) * sizeof(int32_t)));
  OFX_HIP(hipMalloc((void**)&m->trank, (2 * npx + 1) * sizeof(int32_t)));
  OFX_HIP(hipMalloc((void**)&m->vid, npx * sizeof(int32_t)));
  OFX_HIP(hipMalloc((void**)&m->tsum, (scan_tiles(6 * npx) + 1) * sizeof(int32_t)));
  m->cap_px = npx;
  return OFX_OK;
}

// depth_2_pc (NonRigidICP/model/geometry.py:44-59) in float64 as numpy evaluates it — X = ((u - cx)·d)/fx,
// Y = ((v - cy)·d)/fy, Z = d — then rounded to f32 (`.float()`), compacted to the pixels with d > 0 in
// row-major order (registration_fusion.py:107-108); pix_map = map_pixel_to_pcd (registration_fusion.py:388-395).
__global__ __launch_bounds__(256) void k_pc_flags(const float* __restrict__ depth, int64_t n, uint8_t* __restrict__ flag) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p < n) flag[p] = depth[p] > 0.f;
}

__global__ __launch_bounds__(256) void k_pc_emit(const float* __restrict__ depth, int H, int W, double fx, double fy,
                                                 double cx, double cy, const int32_t* __restrict__ rank,
                                                 float* __restrict__ pts, int64_t* __restrict__ pix_map,
                                                 int32_t* __restrict__ n_points) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)H * W;
  if (p == 0 && n_points) *n_points = rank[n];
  if (p >= n) return;
  const float d = depth[p];
  const bool ok = d > 0.f;
  if (pix_map) pix_map[p] = ok ? (int64_t)rank[p] : -1;
  if (!ok) return;
  const int y = (int)(p / W), x = (int)(p % W);
  const double dd = (double)d;
  const int64_t r = rank[p];
  pts[3 * r] = (float)((((double)x - cx) * dd) / fx);
  pts[3 * r + 1] = (float)((((double)y - cy) * dd) / fy);
  pts[3 * r + 2] = d;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_backproject_depth(const void* depth, int32_t is_u16, int32_t height, int32_t width, float fx, float fy, float cx,
                          float cy, float normalizer, float* point_image, ofx_stream_t s) {
  OFX_CHECK_ARG(height >= 0 && width >= 0, "bad image size");
  if ((int64_t)height * width == 0) return OFX_OK;
  OFX_CHECK_ARG(depth && point_image, "null buffer");
  const int64_t n = (int64_t)height * width;
  if (is_u16)
    hipLaunchKernelGGL(k_backproject<true>, dim3(grid_for(n, 256, 1 << 30)), dim3(256), 0, as_stream(s), depth, height,
                       width, fx, fy, cx, cy, normalizer, point_image);
  else
    hipLaunchKernelGGL(k_backproject<false>, dim3(grid_for(n, 256, 1 << 30)), dim3(256), 0, as_stream(s), depth, height,
                       width, fx, fy, cx, cy, normalizer, point_image);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_depth_mesh_create(void** handle) {
  OFX_CHECK_ARG(handle, "null handle");
  *handle = new DepthMesh();
  return OFX_OK;
}

int ofx_depth_mesh_destroy(void* handle) {
  if (!handle) return OFX_OK;
  DepthMesh* m = (DepthMesh*)handle;
  (void)hipDeviceSynchronize();
  for (void* p : {(void*)m->kflag, (void*)m->tflag, (void*)m->krank, (void*)m->trank, (void*)m->vid, (void*)m->tsum})
    if (p) (void)hipFree(p);
  delete m;
  return OFX_OK;
}

int ofx_depth_mesh_count(void* handle, const float* point_image, int32_t height, int32_t width,
                         float max_triangle_distance, int64_t* n_verts, int64_t* n_faces, ofx_stream_t s) {
  DepthMesh* m = (DepthMesh*)handle;
  OFX_CHECK_ARG(m && point_image && n_verts && n_faces, "null argument");
  OFX_CHECK_ARG(height >= 2 && width >= 2, "point image must be at least 2x2");
  OFX_CHECK_ARG((int64_t)height * width < (int64_t)1 << 28, "point image too large (key space is int32)");
  hipStream_t hs = as_stream(s);
  const int64_t npx = (int64_t)height * width, nq = (int64_t)(height - 1) * (width - 1);
  OFX_CHECK(reserve(m, npx));
  m->im.p = point_image; m->im.H = height; m->im.W = width; m->im.maxd = max_triangle_distance;
  OFX_HIP(hipMemsetAsync(m->kflag, 0, 6 * nq, hs));
  hipLaunchKernelGGL(k_dm_flags, dim3(grid_for(npx, 256, 1 << 30)), dim3(256), 0, hs, m->im, m->kflag, m->tflag);
  OFX_CHECK(scan_flags(m->kflag, 6 * nq, m->krank, m->tsum, hs));
  OFX_CHECK(scan_flags(m->tflag, 2 * nq, m->trank, m->tsum, hs));
  OFX_LAUNCH_CHECK();
  int32_t nv = 0, nf = 0;
  OFX_HIP(hipMemcpyAsync(&nv, m->krank + 6 * nq, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipMemcpyAsync(&nf, m->trank + 2 * nq, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipStreamSynchronize(hs));
  m->n_verts = nv;
  m->n_faces = nf;
  *n_verts = nv;
  *n_faces = nf;
  m->counted = true;
  return OFX_OK;
}

int ofx_depth_mesh_emit(void* handle, float* vertices, int32_t* vertex_pixels, int32_t* faces, ofx_stream_t s) {
  DepthMesh* m = (DepthMesh*)handle;
  OFX_CHECK_ARG(m && m->counted, "ofx_depth_mesh_count not called");
  OFX_CHECK_ARG((m->n_verts == 0 || vertices) && (m->n_faces == 0 || faces), "null output");
  hipStream_t hs = as_stream(s);
  const int64_t npx = (int64_t)m->im.H * m->im.W, nq = (int64_t)(m->im.H - 1) * (m->im.W - 1);
  hipLaunchKernelGGL(k_dm_verts, dim3(grid_for(npx, 256, 1 << 30)), dim3(256), 0, hs, m->im, (const int32_t*)m->krank,
                     m->vid, vertices, vertex_pixels);
  hipLaunchKernelGGL(k_dm_faces, dim3(grid_for(2 * nq, 256, 1 << 30)), dim3(256), 0, hs, m->im.H, m->im.W,
                     (const uint8_t*)m->tflag, (const int32_t*)m->trank, (const int32_t*)m->vid, faces);
  OFX_LAUNCH_CHECK();
  m->counted = false;
  return OFX_OK;
}

int ofx_depth_to_pc(void* handle, const float* depth, int32_t height, int32_t width, double fx, double fy, double cx,
                    double cy, float* points, int64_t* pix_map, int32_t* n_points, ofx_stream_t s) {
  DepthMesh* m = (DepthMesh*)handle;
  OFX_CHECK_ARG(m && depth && points && n_points, "null argument");
  OFX_CHECK_ARG(height > 0 && width > 0, "bad image size");
  hipStream_t hs = as_stream(s);
  const int64_t npx = (int64_t)height * width;
  OFX_CHECK(reserve(m, npx));
  hipLaunchKernelGGL(k_pc_flags, dim3(grid_for(npx, 256, 1 << 30)), dim3(256), 0, hs, depth, npx, m->kflag);
  OFX_CHECK(scan_flags(m->kflag, npx, m->krank, m->tsum, hs));
  hipLaunchKernelGGL(k_pc_emit, dim3(grid_for(npx, 256, 1 << 30)), dim3(256), 0, hs, depth, height, width, fx, fy, cx,
                     cy, (const int32_t*)m->krank, points, pix_map, n_points);
  OFX_LAUNCH_CHECK();
  m->counted = false;
  return OFX_OK;
}

}  // extern "C"
