// Skinning: exact k-nearest-node search + Gaussian skinning weights.
//
// Restates WarpField.skin (fusion_with_occlusion/warpfield.py:83-129) over the voxel grid
// (skin_tsdf, :131-141) and over arbitrary points:
//   K = min(N,4) nearest nodes by f32 squared distance ((dx²+dy²)+dz², pykdtree order),
//   ties -> lower node index; dist = sqrt in f32; dist > 4σ (strict, f32) -> anchor -1,
//   w = exp(-dist²/(2σ²)) (f32 result of a f64 exp), valid = all K anchors >= 0,
//   w /= ((w0+w1)+w2)+w3 + 1e-6 (f32).
// csrc twin (no cut-off, no +1e-6): compute_pixel_anchors_euclidean, csrc/cpu/graph_proc.cpp:610-709.
//
// MI355X design: the volume pass first culls 8³ bricks whose AABB has fewer than K nodes within
// 4σ (no voxel in them can be valid), then one 256-thread workgroup per surviving brick streams
// the node set through LDS in 1024-node tiles, compacts each tile to the nodes that can reach the
// brick, and keeps a register top-K per voxel (2 voxels per thread). Exactness does not depend on
// the cull: any node within 4σ of a voxel is within 4σ of its brick.
#include "ofx_common.h"

namespace ofx {

constexpr int kTile = 1024;

struct TopK {
  float d[4];
  int id[4];
  __device__ void init() {
#pragma unroll
    for (int s = 0; s < 4; ++s) { d[s] = __builtin_inff(); id[s] = 0x7fffffff; }
  }
  __device__ __forceinline__ static bool less(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
  }
  __device__ __forceinline__ void insert(float dn, int in) {
    if (!less(dn, in, d[3], id[3])) return;
    // bubble into place
    d[3] = dn; id[3] = in;
#pragma unroll
    for (int s = 3; s > 0; --s) {
      if (less(d[s], id[s], d[s - 1], id[s - 1])) {
        float td = d[s]; d[s] = d[s - 1]; d[s - 1] = td;
        int ti = id[s]; id[s] = id[s - 1]; id[s - 1] = ti;
      }
    }
  }
};

__device__ __forceinline__ float sqdist(float px, float py, float pz, float nx, float ny, float nz) {
  float dx = px - nx, dy = py - ny, dz = pz - nz;
  float a = dx * dx;
  float b = dy * dy;
  float c = dz * dz;
  return (a + b) + c;
}

// Final anchors/weights for one point from its top-K (warpfield.py:104-124).
__device__ __forceinline__ void finish_skin(const TopK& tk, int K, float cutoff, float denom, int out_id[4],
                                            float out_w[4]) {
  float w[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    out_id[s] = -1;
    w[s] = 0.f;
    if (s < K && tk.id[s] != 0x7fffffff) {
      float dist = (float)sqrt((double)tk.d[s]);  // correctly rounded f32 sqrt
      if (!(dist > cutoff)) {
        out_id[s] = tk.id[s];
        float sq = dist * dist;
        float q = (float)((double)(-sq) / (double)denom);  // correctly rounded f32 division
        w[s] = (float)exp((double)q);
      }
    }
  }
  float wsum = w[0];
  for (int s = 1; s < K; ++s) wsum = wsum + w[s];
  float den = wsum + 1e-6f;
#pragma unroll
  for (int s = 0; s < 4; ++s) out_w[s] = (s < K) ? (float)((double)w[s] / (double)den) : 0.f;
}

// ---- brick cull: flag[b] = (#nodes within cull radius of brick AABB) >= K ----
__global__ __launch_bounds__(256) void k_brick_cull(BrickGeom g, const float* __restrict__ nodes, int n_nodes,
                                                     float cull_r2, int K, uint8_t* __restrict__ flags) {
  __shared__ float4 sn[kTile];
  int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool active = b < g.n_bricks;
  float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  if (active) {
    int64_t bz = b % g.nbz;
    int64_t r = b / g.nbz;
    int64_t by = r % g.nby;
    int64_t bx = r / g.nby + g.bx0;
    int i0 = (int)bx * kBrick, j0 = (int)by * kBrick, k0 = (int)bz * kBrick;
    int i1 = min(i0 + kBrick - 1, g.Dx - 1), j1 = min(j0 + kBrick - 1, g.Dy - 1), k1 = min(k0 + kBrick - 1, g.Dz - 1);
    lo[0] = vox2world(g.ox, g.vs, i0); hi[0] = vox2world(g.ox, g.vs, i1);
    lo[1] = vox2world(g.oy, g.vs, j0); hi[1] = vox2world(g.oy, g.vs, j1);
    lo[2] = vox2world(g.oz, g.vs, k0); hi[2] = vox2world(g.oz, g.vs, k1);
  }
  int count = 0;
  for (int t0 = 0; t0 < n_nodes; t0 += kTile) {
    int nt = min(kTile, n_nodes - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
      const float* p = nodes + 3 * (int64_t)(t0 + i);
      sn[i] = make_float4(p[0], p[1], p[2], 0.f);
    }
    __syncthreads();
    if (active && count < K) {
      for (int i = 0; i < nt; ++i) {
        float4 n = sn[i];
        float ex = fmaxf(fmaxf(lo[0] - n.x, n.x - hi[0]), 0.f);
        float ey = fmaxf(fmaxf(lo[1] - n.y, n.y - hi[1]), 0.f);
        float ez = fmaxf(fmaxf(lo[2] - n.z, n.z - hi[2]), 0.f);
        if (ex * ex + ey * ey + ez * ez <= cull_r2) ++count;
      }
    }
  }
  if (active) flags[b] = count >= K ? 1 : 0;
}

// ---- single-workgroup ordered compaction of a flag array into an index list ----
__global__ __launch_bounds__(1024) void k_compact(const uint8_t* __restrict__ flags, int64_t n,
                                                   int32_t* __restrict__ list, int32_t* __restrict__ count) {
  __shared__ int64_t part[1024];
  int64_t per = (n + blockDim.x - 1) / blockDim.x;
  int64_t s = threadIdx.x * per, e = min(n, s + per);
  int64_t c = 0;
  for (int64_t i = s; i < e; ++i) c += flags[i];
  part[threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) { int64_t v = part[i]; part[i] = acc; acc += v; }
    *count = (int32_t)acc;
  }
  __syncthreads();
  int64_t o = part[threadIdx.x];
  for (int64_t i = s; i < e; ++i)
    if (flags[i]) list[o++] = (int32_t)i;
}

// ---- per-voxel k-NN for listed bricks ----
__global__ __launch_bounds__(256) void k_skin_volume(BrickGeom g, const float* __restrict__ nodes, int n_nodes,
                                                      float cull_r2, float cutoff, float denom, int K,
                                                      const int32_t* __restrict__ list, ushort4* __restrict__ anchors,
                                                      float4* __restrict__ weights) {
  __shared__ float4 sc[kTile];
  __shared__ int s_nc;
  const int64_t slot = blockIdx.x;
  const int64_t b = list[slot];
  int64_t bz = b % g.nbz;
  int64_t r = b / g.nbz;
  int64_t by = r % g.nby;
  int64_t bx = r / g.nby + g.bx0;
  const int i0 = (int)bx * kBrick, j0 = (int)by * kBrick, k0 = (int)bz * kBrick;
  float lo[3], hi[3];
  lo[0] = vox2world(g.ox, g.vs, i0); hi[0] = vox2world(g.ox, g.vs, min(i0 + kBrick - 1, g.Dx - 1));
  lo[1] = vox2world(g.oy, g.vs, j0); hi[1] = vox2world(g.oy, g.vs, min(j0 + kBrick - 1, g.Dy - 1));
  lo[2] = vox2world(g.oz, g.vs, k0); hi[2] = vox2world(g.oz, g.vs, min(k0 + kBrick - 1, g.Dz - 1));

  float px[2], py[2], pz[2];
  TopK tk[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int l = threadIdx.x + h * 256;
    int lx = l >> 6, ly = (l >> 3) & 7, lz = l & 7;
    px[h] = vox2world(g.ox, g.vs, i0 + lx);
    py[h] = vox2world(g.oy, g.vs, j0 + ly);
    pz[h] = vox2world(g.oz, g.vs, k0 + lz);
    tk[h].init();
  }
  for (int t0 = 0; t0 < n_nodes; t0 += kTile) {
    int nt = min(kTile, n_nodes - t0);
    if (threadIdx.x == 0) s_nc = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
      const float* p = nodes + 3 * (int64_t)(t0 + i);
      float nx = p[0], ny = p[1], nz = p[2];
      float ex = fmaxf(fmaxf(lo[0] - nx, nx - hi[0]), 0.f);
      float ey = fmaxf(fmaxf(lo[1] - ny, ny - hi[1]), 0.f);
      float ez = fmaxf(fmaxf(lo[2] - nz, nz - hi[2]), 0.f);
      if (ex * ex + ey * ey + ez * ez <= cull_r2) {
        int pos = atomicAdd(&s_nc, 1);
        sc[pos] = make_float4(nx, ny, nz, __int_as_float(t0 + i));
      }
    }
    __syncthreads();
    int nc = s_nc;
    for (int i = 0; i < nc; ++i) {
      float4 n = sc[i];
      int id = __float_as_int(n.w);
#pragma unroll
      for (int h = 0; h < 2; ++h) tk[h].insert(sqdist(px[h], py[h], pz[h], n.x, n.y, n.z), id);
    }
    __syncthreads();
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int l = threadIdx.x + h * 256;
    int ids[4];
    float w[4];
    finish_skin(tk[h], K, cutoff, denom, ids, w);
    ushort4 a;
    a.x = ids[0] < 0 ? kNoAnchor : (uint16_t)ids[0];
    a.y = ids[1] < 0 ? kNoAnchor : (uint16_t)ids[1];
    a.z = ids[2] < 0 ? kNoAnchor : (uint16_t)ids[2];
    a.w = ids[3] < 0 ? kNoAnchor : (uint16_t)ids[3];
    anchors[slot * kBrickVox + l] = a;
    weights[slot * kBrickVox + l] = make_float4(w[0], w[1], w[2], w[3]);
  }
}

// ---- per-brick node palette of the skin cache ----
// Distinct anchors of the brick's skin-valid voxels, ascending node id (LDS bitmap over node ids +
// block scan of popcounts); each voxel's anchors re-expressed as palette ranks (uint8, kNoLocal for
// skin-invalid voxels and unused slots). pal_n > kPal marks an overflowing brick (palette unused).
__global__ __launch_bounds__(256) void k_skin_palette(const ushort4* __restrict__ anchors, int K, int n_nodes,
                                                       uint16_t* __restrict__ pal_ids, int32_t* __restrict__ pal_n,
                                                       uchar4* __restrict__ local) {
  __shared__ uint32_t s_bits[2048];
  __shared__ int s_pre[2048 + 1];
  __shared__ int s_tsum[256];
  const int64_t slot = blockIdx.x;
  const int nw = (n_nodes + 31) >> 5;
  for (int i = threadIdx.x; i < nw; i += 256) s_bits[i] = 0u;
  __syncthreads();
  int ids[2][4];
  bool val[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const ushort4 a = anchors[slot * kBrickVox + threadIdx.x + 256 * h];
    ids[h][0] = a.x; ids[h][1] = a.y; ids[h][2] = a.z; ids[h][3] = a.w;
    val[h] = ids[h][K - 1] != kNoAnchor;
    if (val[h])
      for (int s = 0; s < K; ++s) atomicOr(&s_bits[ids[h][s] >> 5], 1u << (ids[h][s] & 31));
  }
  __syncthreads();
  // exclusive prefix of word popcounts: contiguous chunk per thread, then a 256-entry scan
  const int chunk = (nw + 255) / 256;
  const int w0 = threadIdx.x * chunk, w1 = min(nw, w0 + chunk);
  int tsum = 0;
  for (int w = w0; w < w1; ++w) tsum += __popc(s_bits[w]);
  s_tsum[threadIdx.x] = tsum;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int v = threadIdx.x >= off ? s_tsum[threadIdx.x - off] : 0;
    __syncthreads();
    s_tsum[threadIdx.x] += v;
    __syncthreads();
  }
  int run = s_tsum[threadIdx.x] - tsum;
  for (int w = w0; w < w1; ++w) {
    s_pre[w] = run;
    const uint32_t bits = s_bits[w];
    uint32_t m = bits;
    int r = run;
    while (m) {
      const int bit = __ffs(m) - 1;
      if (r < kPal) pal_ids[slot * kPal + r] = (uint16_t)(w * 32 + bit);
      ++r;
      m &= m - 1;
    }
    run += __popc(bits);
  }
  if (threadIdx.x == 255) pal_n[slot] = s_tsum[255];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint8_t o[4] = {kNoLocal, kNoLocal, kNoLocal, kNoLocal};
    if (val[h])
      for (int s = 0; s < K; ++s) {
        const int id = ids[h][s];
        const int rk = s_pre[id >> 5] + __popc(s_bits[id >> 5] & ((1u << (id & 31)) - 1u));
        o[s] = rk < kPal ? (uint8_t)rk : kNoLocal;
      }
    local[slot * kBrickVox + threadIdx.x + 256 * h] = make_uchar4(o[0], o[1], o[2], o[3]);
  }
}

// ---- per-point k-NN (all nodes) ----
// kSP adjacent lanes per point, each scanning every kSP-th node of the LDS tile into its own top-K, then a butterfly
// merge over the kSP lanes (each round inserts the partner's K entries): the K smallest by (distance, id) are unique,
// so every lane ends with the single-thread scan's result, bit for bit. (One thread per point left 40 workgroups for
// 10k matches scanning 2k nodes each: ~330 us on the prefetch stream beside the solve.)
constexpr int kSP = 16;
static_assert(64 % kSP == 0, "a point's lanes within one wave");
__global__ __launch_bounds__(256) void k_skin_points(const float* __restrict__ pts, int64_t n_pts,
                                                      const float* __restrict__ nodes, int n_nodes, float cutoff,
                                                      float denom, int K, int32_t* __restrict__ anchors,
                                                      float* __restrict__ weights, uint8_t* __restrict__ valid) {
  __shared__ float4 sn[kTile];
  const int part = threadIdx.x % kSP;
  const int64_t p = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kSP;
  const bool act = p < n_pts;
  float x = 0, y = 0, z = 0;
  if (act) { x = pts[3 * p]; y = pts[3 * p + 1]; z = pts[3 * p + 2]; }
  TopK tk;
  tk.init();
  for (int t0 = 0; t0 < n_nodes; t0 += kTile) {
    int nt = min(kTile, n_nodes - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
      const float* q = nodes + 3 * (int64_t)(t0 + i);
      sn[i] = make_float4(q[0], q[1], q[2], 0.f);
    }
    __syncthreads();
    if (act)
      for (int i = part; i < nt; i += kSP) {
        float4 n = sn[i];
        tk.insert(sqdist(x, y, z, n.x, n.y, n.z), t0 + i);
      }
  }
#pragma unroll
  for (int o = 1; o < kSP; o <<= 1) {   // (every lane takes part: the shuffles precede any exit)
    float od[4];
    int oi[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) { od[s2] = __shfl_xor(tk.d[s2], o, 64); oi[s2] = __shfl_xor(tk.id[s2], o, 64); }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) tk.insert(od[s2], oi[s2]);
  }
  if (!act || part != 0) return;
  int ids[4];
  float w[4];
  finish_skin(tk, K, cutoff, denom, ids, w);
  for (int s = 0; s < K; ++s) {
    anchors[p * K + s] = ids[s];
    weights[p * K + s] = w[s];
  }
  valid[p] = ids[K - 1] >= 0 ? 1 : 0;
}

__global__ void k_slot_map(const int32_t* __restrict__ list, int n_list, int32_t* __restrict__ slot_of) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_list) slot_of[list[i]] = i;
}

__global__ void k_skin_to_dense(BrickGeom g, int32_t x_lo, int32_t x_n, const int32_t* __restrict__ slot_of,
                                const ushort4* __restrict__ anchors, const float4* __restrict__ weights, int K,
                                int32_t* __restrict__ a_out, float* __restrict__ w_out, uint8_t* __restrict__ v_out) {
  const int64_t n = (int64_t)x_n * g.Dy * g.Dz;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = t % g.Dz;
    int64_t r = t / g.Dz;
    int64_t j = r % g.Dy;
    int64_t i = r / g.Dy + x_lo;
    int64_t b = ((i / kBrick - g.bx0) * g.nby + j / kBrick) * g.nbz + k / kBrick;
    int64_t l = ((i % kBrick) * kBrick + (j % kBrick)) * kBrick + (k % kBrick);
    int32_t s = slot_of[b];
    int ids[4] = {-1, -1, -1, -1};
    float w[4] = {0, 0, 0, 0};
    if (s >= 0) {
      ushort4 a = anchors[(int64_t)s * kBrickVox + l];
      float4 ww = weights[(int64_t)s * kBrickVox + l];
      ids[0] = a.x == kNoAnchor ? -1 : a.x; ids[1] = a.y == kNoAnchor ? -1 : a.y;
      ids[2] = a.z == kNoAnchor ? -1 : a.z; ids[3] = a.w == kNoAnchor ? -1 : a.w;
      w[0] = ww.x; w[1] = ww.y; w[2] = ww.z; w[3] = ww.w;
    }
    for (int q = 0; q < K; ++q) { a_out[t * K + q] = ids[q]; w_out[t * K + q] = w[q]; }
    v_out[t] = ids[K - 1] >= 0 ? 1 : 0;
  }
}

struct SkinConsts {
  float cutoff, denom, cull_r2;
};

static SkinConsts skin_consts(double node_coverage) {
  SkinConsts c;
  c.cutoff = (float)(4.0 * node_coverage);                          // warpfield.py:109 (f64 product -> f32 compare)
  c.denom = (float)(2.0 * (node_coverage * node_coverage));         // warpfield.py:114
  double r = 4.0 * node_coverage * (1.0 + 1e-4) + 1e-6;             // conservative cull radius
  c.cull_r2 = (float)(r * r);
  return c;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_skin_volume_bricks(const ofx_volume_desc* desc, const float* nodes, int32_t n_nodes, double node_coverage,
                           int32_t k, int32_t* brick_list, int32_t* count, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(nodes && brick_list && count, "null buffer");
  OFX_CHECK_ARG(n_nodes > 0 && k >= 1 && k <= 4 && k <= n_nodes, "bad n_nodes/k");
  if (n_nodes >= 0xFFFF) { set_error("n_nodes %d exceeds 65534 (uint16 anchors)", n_nodes); return OFX_ERR_RANGE; }
  OFX_CHECK_ARG(node_coverage > 0, "node_coverage must be > 0");
  SkinConsts c = skin_consts(node_coverage);
  uint8_t* flags = nullptr;
  hipStream_t hs = as_stream(s);
  OFX_HIP(hipMallocAsync((void**)&flags, g.n_bricks, hs));
  hipLaunchKernelGGL(k_brick_cull, dim3(grid_for(g.n_bricks, 256, 1 << 30)), dim3(256), 0, hs, g, nodes, n_nodes,
                     c.cull_r2, k, flags);
  OFX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, hs, flags, g.n_bricks, brick_list, count);
  OFX_LAUNCH_CHECK();
  OFX_HIP(hipFreeAsync(flags, hs));
  return OFX_OK;
}

int ofx_skin_volume(const ofx_volume_desc* desc, const float* nodes, int32_t n_nodes, double node_coverage, int32_t k,
                    const int32_t* brick_list, int32_t n_list, uint16_t* anchors, float* weights, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(nodes && n_nodes > 0 && k >= 1 && k <= 4 && k <= n_nodes, "bad nodes/k");
  if (n_nodes >= 0xFFFF) { set_error("n_nodes %d exceeds 65534 (uint16 anchors)", n_nodes); return OFX_ERR_RANGE; }
  OFX_CHECK_ARG(n_list >= 0 && n_list <= g.n_bricks, "bad n_list");
  if (n_list == 0) return OFX_OK;
  OFX_CHECK_ARG(brick_list && anchors && weights, "null buffer");
  SkinConsts c = skin_consts(node_coverage);
  hipLaunchKernelGGL(k_skin_volume, dim3(n_list), dim3(256), 0, as_stream(s), g, nodes, n_nodes, c.cull_r2, c.cutoff,
                     c.denom, k, brick_list, (ushort4*)anchors, (float4*)weights);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_skin_palette(const uint16_t* anchors, int32_t n_list, int32_t k, int32_t n_nodes, uint16_t* pal_ids,
                     int32_t* pal_n, uint8_t* local_anchors, ofx_stream_t s) {
  OFX_CHECK_ARG(k >= 1 && k <= 4 && n_nodes >= k && n_list >= 0, "bad k/n_nodes/n_list");
  if (n_nodes > 65535) { set_error("n_nodes %d exceeds 65535 (palette bitmap)", n_nodes); return OFX_ERR_RANGE; }
  if (n_list == 0) return OFX_OK;
  OFX_CHECK_ARG(anchors && pal_ids && pal_n && local_anchors, "null buffer");
  hipLaunchKernelGGL(k_skin_palette, dim3(n_list), dim3(256), 0, as_stream(s), (const ushort4*)anchors, k, n_nodes,
                     pal_ids, pal_n, (uchar4*)local_anchors);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_skin_points(const float* points, int64_t n_points, const float* nodes, int32_t n_nodes, double node_coverage,
                    int32_t k, int32_t* anchors, float* weights, uint8_t* valid, ofx_stream_t s) {
  OFX_CHECK_ARG(n_points >= 0 && n_nodes > 0 && k >= 1 && k <= 4 && k <= n_nodes, "bad sizes");
  OFX_CHECK_ARG(node_coverage > 0, "node_coverage must be > 0");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && nodes && anchors && weights && valid, "null buffer");
  SkinConsts c = skin_consts(node_coverage);
  hipLaunchKernelGGL(k_skin_points, dim3(grid_for(n_points * kSP, 256, 1 << 30)), dim3(256), 0, as_stream(s), points,
                     n_points, nodes, n_nodes, c.cutoff, c.denom, k, anchors, weights, valid);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_skin_volume_to_dense(const ofx_volume_desc* desc, const int32_t* brick_list, int32_t n_list,
                             const uint16_t* anchors, const float* weights, int32_t k, int32_t* anchors_out,
                             float* weights_out, uint8_t* valid_out, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(k >= 1 && k <= 4 && anchors_out && weights_out && valid_out, "bad args");
  hipStream_t hs = as_stream(s);
  int32_t* slot_of = nullptr;
  OFX_HIP(hipMallocAsync((void**)&slot_of, g.n_bricks * sizeof(int32_t), hs));
  OFX_HIP(hipMemsetAsync(slot_of, 0xFF, g.n_bricks * sizeof(int32_t), hs));
  if (n_list > 0) {
    hipLaunchKernelGGL(k_slot_map, dim3(grid_for(n_list, 256)), dim3(256), 0, hs, brick_list, n_list, slot_of);
    OFX_LAUNCH_CHECK();
  }
  int32_t lo = g.bx0 * kBrick, hi = min(g.bx1 * kBrick, g.Dx);
  int64_t total = (int64_t)(hi - lo) * g.Dy * g.Dz;
  hipLaunchKernelGGL(k_skin_to_dense, dim3(grid_for(total, 256, 16384)), dim3(256), 0, hs, g, lo, hi - lo, slot_of,
                     (const ushort4*)anchors, (const float4*)weights, k, anchors_out, weights_out, valid_out);
  OFX_LAUNCH_CHECK();
  OFX_HIP(hipFreeAsync(slot_of, hs));
  return OFX_OK;
}

}  // extern "C"
