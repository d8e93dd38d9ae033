// Standalone skinning / anchor ops: the csrc pixel-anchor twins, a general k-NN
// query with distances, and anchor id remapping.
//
//   ofx_pixel_anchors_euclidean  graph_proc::compute_pixel_anchors_euclidean   csrc/cpu/graph_proc.cpp:610-709
//   ofx_pixel_anchors_geodesic   graph_proc::compute_pixel_anchors_geodesic    csrc/cpu/graph_proc.cpp:483-608
//   ofx_remap_anchors            graph_proc::update_pixel_anchors              csrc/cpu/graph_proc.cpp:934-961
//   ofx_knn_points               KDTree.query(points, k) (pykdtree)            warpfield.py:103-104,468-470
//                                (WarpField.find_unreachable_nodes, warpfield.py:462-485)
//
// csrc semantics reproduced exactly (tests/golden/anchors_csrc.npz holds the compiled reference's outputs):
//  * Eigen 3.3.7 squaredNorm of a Vector3f sums x0 + (x1 + x2) (unrolled redux, Redux.h:92-104);
//  * the Euclidean k-NN list inserts a node before the first entry with distance2 <= its own, so among equal
//    distances the LATER node id comes first; at most GRAPH_K = 4 entries; no cut-off;
//  * weights exp(-d2 / (2·c·c)) in f32 (std::exp(float); here the correctly rounded f32 of the f64 exp), summed
//    in f32 in list order, divided by the f32 sum (1/n when the sum is 0);
//  * geodesic: std::map<int, float> of valid nodes with dist >= 0, copied into a std::set ordered by distance
//    only — a node whose distance equals an earlier (lower id) node's is dropped — first GRAPH_K of the set.
#include "ofx_common.h"

namespace ofx {

constexpr int kGraphK = 4;   // GRAPH_K (csrc/cpu/graph_proc.h:8)

__device__ __forceinline__ float eigen_sqnorm(float dx, float dy, float dz) {
  const float a = dx * dx, b = dy * dy, c = dz * dz;
  return a + (b + c);
}

__device__ __forceinline__ float fdiv32(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float fexp32(float x) { return (float)exp((double)x); }

// weights of n anchors from their squared distances, csrc order (graph_proc.cpp:147-153, 672-696)
__device__ __forceinline__ void csrc_weights(const float* d2, int n, float two_c2, float* w) {
  float sum = 0.f;
  for (int i = 0; i < n; ++i) {
    w[i] = fexp32(fdiv32(-d2[i], two_c2));
    sum += w[i];
  }
  if (sum > 0.f) {
    for (int i = 0; i < n; ++i) w[i] = fdiv32(w[i], sum);
  } else if (n > 0) {
    for (int i = 0; i < n; ++i) w[i] = fdiv32(1.f, (float)n);
  }
}

__global__ __launch_bounds__(256) void k_fill_anchor_image(int64_t n, int32_t* __restrict__ a, float* __restrict__ w) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) { a[i] = -1; w[i] = 0.f; }
}

constexpr int kNodeTile = 512;

// one thread per pixel; node tiles through LDS
__global__ __launch_bounds__(256) void k_pixel_anchors_euclid(const float* __restrict__ img, int64_t hw,
                                                               const float* __restrict__ nodes, int n_nodes,
                                                               float two_c2, int32_t* __restrict__ anchors,
                                                               float* __restrict__ weights) {
  __shared__ float4 sn[kNodeTile];
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool act = p < hw;
  float x = 0.f, y = 0.f, z = 0.f;
  if (act) { x = img[p]; y = img[hw + p]; z = img[2 * hw + p]; }
  act = act && z > 0.f;
  // sorted list with +inf sentinels (registers); csrc inserts before the first entry >= d2 and drops the 5th
  float d[kGraphK];
  int id[kGraphK];
#pragma unroll
  for (int s = 0; s < kGraphK; ++s) { d[s] = __builtin_inff(); id[s] = -1; }
  for (int t0 = 0; t0 < n_nodes; t0 += kNodeTile) {
    const int nt = min(kNodeTile, n_nodes - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
      const float* q = nodes + 3 * (int64_t)(t0 + i);
      sn[i] = make_float4(q[0], q[1], q[2], 0.f);
    }
    __syncthreads();
    if (act)
      for (int i = 0; i < nt; ++i) {
        const float4 nd = sn[i];
        const float d2 = eigen_sqnorm(x - nd.x, y - nd.y, z - nd.z);
        if (!(d2 <= d[kGraphK - 1])) continue;
        d[kGraphK - 1] = d2;
        id[kGraphK - 1] = t0 + i;
        bool mv = true;                     // the new node moves before equal distances (ties: later id first)
#pragma unroll
        for (int s = kGraphK - 1; s > 0; --s)
          if (mv && d[s] <= d[s - 1]) {
            const float td = d[s]; d[s] = d[s - 1]; d[s - 1] = td;
            const int ti = id[s]; id[s] = id[s - 1]; id[s - 1] = ti;
          } else {
            mv = false;
          }
      }
  }
  int cnt = 0;
#pragma unroll
  for (int s = 0; s < kGraphK; ++s) cnt += id[s] >= 0 ? 1 : 0;
  if (!act) return;
  // weights use (node - pixel).squaredNorm(): the same squares, the same order
  float w[kGraphK];
  csrc_weights(d, cnt, two_c2, w);
  for (int s = 0; s < cnt; ++s) {
    anchors[p * kGraphK + s] = id[s];
    weights[p * kGraphK + s] = w[s];
  }
}

// one thread per vertex; node_to_vertex_distance is (N, V) row-major: lanes read consecutive vertices
__global__ __launch_bounds__(256) void k_pixel_anchors_geo(const float* __restrict__ dist, int n_nodes, int64_t n_verts,
                                                            const int32_t* __restrict__ valid_nodes,
                                                            const int32_t* __restrict__ vpix, int W, int H,
                                                            float cov, int32_t* __restrict__ anchors,
                                                            float* __restrict__ weights) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= n_verts) return;
  float d[kGraphK];
  int id[kGraphK];
  int cnt = 0;
  for (int n = 0; n < n_nodes; ++n) {
    if (valid_nodes[n] == 0) continue;
    const float dn = dist[(int64_t)n * n_verts + v];
    if (!(dn >= 0.f)) continue;
    // the set keeps the first node of every distinct distance, ordered by distance
    int pos = cnt;
    bool dup = false;
    for (int s = cnt - 1; s >= 0; --s) {
      if (d[s] == dn) dup = true;
      if (dn < d[s]) pos = s;
    }
    if (dup || pos >= kGraphK) continue;
    const int last = cnt < kGraphK ? cnt : kGraphK - 1;
    for (int s = last; s > pos; --s) { d[s] = d[s - 1]; id[s] = id[s - 1]; }
    d[pos] = dn;
    id[pos] = n;
    if (cnt < kGraphK) ++cnt;
  }
  const int u = vpix[2 * v], y = vpix[2 * v + 1];
  if (u < 0 || u >= W || y < 0 || y >= H) return;
  const float two_c2 = (2.f * cov) * cov;
  float d2[kGraphK], w[kGraphK];
  for (int s = 0; s < cnt; ++s) d2[s] = d[s] * d[s];
  csrc_weights(d2, cnt, two_c2, w);
  const int64_t o = ((int64_t)y * W + u) * kGraphK;
  for (int s = 0; s < cnt; ++s) { anchors[o + s] = id[s]; weights[o + s] = w[s]; }
}

__global__ __launch_bounds__(256) void k_remap_anchors(int32_t* __restrict__ a, int64_t n, const int32_t* __restrict__ map,
                                                        int32_t n_map, int32_t* __restrict__ n_missing) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t c = a[i];
  if (c == -1) return;
  const int32_t m = (c >= 0 && c < n_map) ? map[c] : -1;
  if (m < 0) { atomicAdd(n_missing, 1); return; }   // std::map::at would throw: reported, entry kept
  a[i] = m;
}

// general k-NN (k <= 8): ascending (squared distance, node id); squared distances as (dx²+dy²)+dz² in f32.
// K is a template parameter so the top-K lists stay in registers.
constexpr int kMaxK = 8;
template <int K>
__global__ __launch_bounds__(256) void k_knn(const float* __restrict__ pts, int64_t n_pts, const float* __restrict__ nodes,
                                             int n_nodes, int32_t* __restrict__ idx, float* __restrict__ sqd) {
  __shared__ float4 sn[kNodeTile];
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool act = p < n_pts;
  float x = 0.f, y = 0.f, z = 0.f;
  if (act) { x = pts[3 * p]; y = pts[3 * p + 1]; z = pts[3 * p + 2]; }
  float d[K];
  int id[K];
#pragma unroll
  for (int s = 0; s < K; ++s) { d[s] = __builtin_inff(); id[s] = 0x7fffffff; }
  for (int t0 = 0; t0 < n_nodes; t0 += kNodeTile) {
    const int nt = min(kNodeTile, n_nodes - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
      const float* q = nodes + 3 * (int64_t)(t0 + i);
      sn[i] = make_float4(q[0], q[1], q[2], 0.f);
    }
    __syncthreads();
    if (act)
      for (int i = 0; i < nt; ++i) {
        const float4 nd = sn[i];
        const float dx = x - nd.x, dy = y - nd.y, dz = z - nd.z;
        const float a = dx * dx, b = dy * dy, c = dz * dz;
        const float dn = (a + b) + c;
        const int in = t0 + i;
        if (!(dn < d[K - 1])) continue;          // ids ascend: an equal distance never displaces an earlier id
        d[K - 1] = dn;
        id[K - 1] = in;
#pragma unroll
        for (int s = K - 1; s > 0; --s)
          if (d[s] < d[s - 1]) {
            const float td = d[s]; d[s] = d[s - 1]; d[s - 1] = td;
            const int ti = id[s]; id[s] = id[s - 1]; id[s - 1] = ti;
          }
      }
  }
  if (!act) return;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const bool ok = id[s] != 0x7fffffff;
    idx[p * K + s] = ok ? id[s] : -1;
    sqd[p * K + s] = d[s];
  }
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_pixel_anchors_euclidean(const float* nodes, int32_t n_nodes, const float* point_image, int32_t height,
                                int32_t width, float node_coverage, int32_t* pixel_anchors, float* pixel_weights,
                                ofx_stream_t s) {
  OFX_CHECK_ARG(height >= 0 && width >= 0 && n_nodes >= 0, "bad sizes");
  const int64_t hw = (int64_t)height * width;
  if (hw == 0) return OFX_OK;
  OFX_CHECK_ARG(point_image && pixel_anchors && pixel_weights && (n_nodes == 0 || nodes), "null buffer");
  hipStream_t hs = as_stream(s);
  hipLaunchKernelGGL(k_fill_anchor_image, dim3(grid_for(hw * kGraphK, 256, 1 << 30)), dim3(256), 0, hs, hw * kGraphK,
                     pixel_anchors, pixel_weights);
  const float two_c2 = (2.f * node_coverage) * node_coverage;
  hipLaunchKernelGGL(k_pixel_anchors_euclid, dim3(grid_for(hw, 256, 1 << 30)), dim3(256), 0, hs, point_image, hw, nodes,
                     n_nodes, two_c2, pixel_anchors, pixel_weights);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_pixel_anchors_geodesic(const float* node_to_vertex_distance, const int32_t* valid_nodes_mask, int32_t n_nodes,
                               int64_t n_vertices, const int32_t* vertex_pixels, int32_t width, int32_t height,
                               float node_coverage, int32_t* pixel_anchors, float* pixel_weights, ofx_stream_t s) {
  OFX_CHECK_ARG(height >= 0 && width >= 0 && n_nodes >= 0 && n_vertices >= 0, "bad sizes");
  const int64_t hw = (int64_t)height * width;
  if (hw == 0) return OFX_OK;
  OFX_CHECK_ARG(pixel_anchors && pixel_weights, "null output");
  hipStream_t hs = as_stream(s);
  hipLaunchKernelGGL(k_fill_anchor_image, dim3(grid_for(hw * kGraphK, 256, 1 << 30)), dim3(256), 0, hs, hw * kGraphK,
                     pixel_anchors, pixel_weights);
  if (n_vertices > 0) {
    OFX_CHECK_ARG(vertex_pixels && (n_nodes == 0 || (node_to_vertex_distance && valid_nodes_mask)), "null input");
    hipLaunchKernelGGL(k_pixel_anchors_geo, dim3(grid_for(n_vertices, 256, 1 << 30)), dim3(256), 0, hs,
                       node_to_vertex_distance, n_nodes, n_vertices, valid_nodes_mask, vertex_pixels, width, height,
                       node_coverage, pixel_anchors, pixel_weights);
  }
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_remap_anchors(int32_t* anchors, int64_t n, const int32_t* id_map, int32_t n_map, int32_t* n_missing,
                      ofx_stream_t s) {
  OFX_CHECK_ARG(n >= 0 && n_map >= 0, "bad sizes");
  if (n == 0) return OFX_OK;
  OFX_CHECK_ARG(anchors && n_missing && (n_map == 0 || id_map), "null buffer");
  hipLaunchKernelGGL(k_remap_anchors, dim3(grid_for(n, 256, 1 << 30)), dim3(256), 0, as_stream(s), anchors, n, id_map,
                     n_map, n_missing);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_knn_points(const float* points, int64_t n_points, const float* nodes, int32_t n_nodes, int32_t k, int32_t* idx,
                   float* sq_dist, ofx_stream_t s) {
  OFX_CHECK_ARG(k >= 1 && k <= kMaxK, "k must be in [1, %d]", kMaxK);
  OFX_CHECK_ARG(n_points >= 0 && n_nodes >= 0, "bad sizes");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && idx && sq_dist && (n_nodes == 0 || nodes), "null buffer");
  const dim3 gr(grid_for(n_points, 256, 1 << 30));
  hipStream_t hs = as_stream(s);
  switch (k) {
#define OFX_KNN_CASE(KK) \
    case KK: hipLaunchKernelGGL(k_knn<KK>, gr, dim3(256), 0, hs, points, n_points, nodes, n_nodes, idx, sq_dist); break;
    OFX_KNN_CASE(1) OFX_KNN_CASE(2) OFX_KNN_CASE(3) OFX_KNN_CASE(4)
    OFX_KNN_CASE(5) OFX_KNN_CASE(6) OFX_KNN_CASE(7) OFX_KNN_CASE(8)
#undef OFX_KNN_CASE
  }
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

}  // extern "C"
