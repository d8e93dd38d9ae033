// Fused ED warp + TSDF integrate, plus point warp / visibility helpers.
//
// Per voxel (reference CPU path, fusion_with_occlusion/tsdf.py:378-494):
//   x  = vox2world(i,j,k)                                   (tsdf.py:338-349, f32)
//   x' = Σ_k w_k (R_k (x - g_k) + g_k + t_k)  if warp       (NonRigidICP/model/geometry.py:9-25, f32,
//                                                            registration_fusion.py:157-184; invalid skin -> skipped,
//                                                            tsdf.py:464)
//   u  = int(round_half_even((x'*fx)/z + cx)), v likewise   (tsdf.py:351-364, f64 with f32 intrinsics)
//   valid iff 0<=u<W, 0<=v<H, z>0, d=depth[v,u]>0, d-z >= -trunc        (tsdf.py:576-612)
//   dist = min(1,(d-z)/trunc); w' = f32(w+obs); tsdf' = f32((f32(w*tsdf) + obs*dist)/w')  (tsdf.py:366-376)
//   colour: per-channel running average in f32, rint, min 255  (tsdf.py:479-494)
//
// MI355X layout: tsdf/weight/colour are 8³ bricks (2 KiB contiguous per array per brick); one
// 256-thread workgroup owns one brick (2 voxels per thread, coalesced 4/8/16-B loads). For warped
// frames the grid is the compacted list of skinned bricks, and the skin cache of a brick is stored
// contiguously by list slot: anchors ushort4 (8 B) + weights float4 (16 B) per voxel. Node records
// (64 B) and the depth/colour images are gathered through L1/L2. Voxels with invalid skin read 8 B
// and stop. All arithmetic is un-contracted (-ffp-contract=off) so results are bit-identical to the
// oracle restatement.
#include <hip/hip_ext.h>
#include <stdlib.h>

#include <mutex>
#include <utility>
#include <vector>

#include "ofx_common.h"

namespace ofx {

struct CamD {
  double fx, fy, cx, cy;
  float fxf, fyf, cxf, cyf;   // the same intrinsics as f32 (exact: ofx_camera is f32)
  int W, H;
};

typedef float f2 __attribute__((ext_vector_type(2)));

// Warp one voxel position with its K anchors (f32, reference op order). Rows 0 and 1 of R(x-g)+g+t
// run as packed f32 pairs (v_pk_mul/add_f32; the same per-component rounding), row 2 scalar.
// Node record layout: see ofx_pack_nodes.
__device__ __forceinline__ void ed_warp(const float4* __restrict__ nodes, const int ids[4], const float w[4], int K,
                                        float& x, float& y, float& z) {
  f2 axy = {0.f, 0.f};
  float az = 0.f;
  const f2 xy = {x, y};
  for (int k = 0; k < K; ++k) {
    const float4* n = nodes + 4 * (int64_t)ids[k];
    const float4 a = n[0], b = n[1], c = n[2], d = n[3];
    const f2 P0 = {a.x, a.y}, P1 = {a.z, a.w}, P2 = {b.x, b.y}, G = {b.z, b.w}, T = {c.x, c.y};
    const f2 dxy = xy - G;
    const float dz = z - d.y;
    f2 r = P0 * dxy.x;
    r = r + P1 * dxy.y;
    r = r + P2 * dz;
    float rz = c.z * dxy.x;
    rz = rz + c.w * dxy.y;
    rz = rz + d.x * dz;
    const f2 yxy = ((r + G) + T) * w[k];
    const float yz = ((rz + d.y) + d.z) * w[k];
    if (k == 0) { axy = yxy; az = yz; }
    else { axy = axy + yxy; az = az + yz; }
  }
  x = axy.x; y = axy.y; z = az;
}

// Projection + visibility (tsdf.py:351-364, 576-612). Returns pixel index or -1.
__device__ __forceinline__ int64_t project(const CamD& c, float x, float y, float z, double& Z) {
  double X = x, Y = y;
  Z = z;
  double u = rint((X * c.fx) / Z + c.cx);
  double v = rint((Y * c.fy) / Z + c.cy);
  if (!(u >= 0.0 && u < (double)c.W && v >= 0.0 && v < (double)c.H && Z > 0.0)) return -1;
  return (int64_t)v * c.W + (int64_t)u;
}

__device__ __forceinline__ float cdiv(float a, float b) { return (float)((double)a / (double)b); }

// s lies within tol of a rounding tie of rint (a half-integer)
__device__ __forceinline__ bool near_half(double s, double tol) {
  return fabs((s - floor(s)) - 0.5) < tol;
}

// f32(t) for the exact f64 value t64 with |t - t64| <= err: returns false if t's f32 rounding could
// differ from t64's (t within err of a rounding boundary, or a zero / non-finite result)
__device__ __forceinline__ bool f32_round_safe(double t, double err, float& out) {
  const float f = (float)t;
  if (!(f != 0.f) || !isfinite(f)) return false;
  const int bits = __float_as_int(f);
  const float up = __int_as_float(bits + 1), dn = __int_as_float(bits - 1);   // magnitude up / down
  const double m1 = 0.5 * ((double)f + (double)up), m2 = 0.5 * ((double)f + (double)dn);
  const double lo = fmin(m1, m2), hi = fmax(m1, m2);
  out = f;
  return t - err > lo && t + err < hi;
}

// One voxel update; returns 1 if the voxel was integrated. Reference semantics (tsdf.py:351-376,
// 479-494; numba f64 promotion), with three of the seven f64 divisions replaced by products with a
// reciprocal: (X·fx)/Z and (Y·fy)/Z use 1/Z, dd/trunc uses 1/trunc, the SDF quotient uses 1/w_new.
// Each replacement perturbs the f64 value by a few ulp at most; the result is used only where that
// cannot change a rounding (pixel: not within 1e-9 of a half-integer; SDF: its f32 rounding interval
// contains the whole error bound) — otherwise the exact division path runs. Bit-identical results.
__device__ __forceinline__ int update_voxel(const CamD& c, const float* __restrict__ depth,
                                            const float* __restrict__ color_im, double trunc, double itrunc,
                                            double obs, float x, float y, float z, int64_t vi,
                                            float* __restrict__ tsdf, float* __restrict__ weight,
                                            float* __restrict__ color) {
  const double X = x, Y = y, Z = z;
  if (!(Z > 0.0)) return 0;
  const double nx = X * c.fx, ny = Y * c.fy;
  const double rz = 1.0 / Z;
  double qx = nx * rz, qy = ny * rz;
  double su = qx + c.cx, sv = qy + c.cy;
  if (near_half(su, 1e-9 * fmax(1.0, fmax(fabs(qx), fabs(su)))) ||
      near_half(sv, 1e-9 * fmax(1.0, fmax(fabs(qy), fabs(sv))))) {
    su = nx / Z + c.cx;
    sv = ny / Z + c.cy;
  }
  const double u = rint(su), v = rint(sv);
  if (!(u >= 0.0 && u < (double)c.W && v >= 0.0 && v < (double)c.H)) return 0;
  const int64_t pix = (int64_t)v * c.W + (int64_t)u;
  float d = depth[pix];
  double dd = (double)d - Z;
  if (!(d > 0.f && dd >= -trunc)) return 0;
  const float w_old = weight[vi];
  const float t_old = tsdf[vi];
  float w_new = (float)((double)w_old + obs);
  float prod = w_old * t_old;
  const double wn = (double)w_new;
  const double inv = 1.0 / wn;
  const double dist_a = fmin(1.0, dd * itrunc);
  const double num_a = (double)prod + obs * dist_a;
  const double t_a = num_a * inv;
  const double err = (fabs(obs) * 1e-15 + 1e-15 * fabs(num_a)) * inv + 1e-15 * fabs(t_a);
  float t_new;
  if (!f32_round_safe(t_a, err, t_new)) {
    const double dist = fmin(1.0, dd / trunc);
    t_new = (float)(((double)prod + obs * dist) / wn);
  }
  weight[vi] = w_new;
  tsdf[vi] = t_new;
  if (color) {
    const float C = 65536.0f;
    const float oc = color[vi];
    float ob = floorf(oc / C);
    float og = floorf((oc - ob * C) / 256.0f);
    float orr = (oc - ob * C) - og * 256.0f;
    float nc = color_im[pix];
    float nb = floorf(nc / C);
    float ng = floorf((nc - nb * C) / 256.0f);
    float nr = (nc - nb * C) - ng * 256.0f;
    float ow = (float)obs;
    // f32 quotients a/w_new as f32(a · f64(1/w_new)): for f32 a, b the f64 product is within 2^-52 of
    // a/b while a/b is never an f32 rounding midpoint and lies >= ~2^-49 (relative) from one, so the
    // rounding equals the correctly rounded f32 division (randomised check: 3.6e8 pairs, 0 diffs)
    float b2 = fminf(255.0f, rintf((float)((double)(w_old * ob + ow * nb) * inv)));
    float g2 = fminf(255.0f, rintf((float)((double)(w_old * og + ow * ng) * inv)));
    float r2 = fminf(255.0f, rintf((float)((double)(w_old * orr + ow * nr) * inv)));
    color[vi] = (b2 * C + g2 * 256.0f) + r2;
  }
  return 1;
}

// (int)f with the saturating conversion both CUDA (cvt.rzi.s32.f32) and CDNA (v_cvt_i32_f32) perform
// for the pycuda kernel's casts: NaN -> 0, out of range -> INT_MIN / INT_MAX.
__device__ __forceinline__ int cvt_sat_i32(float f) {
  if (f != f) return 0;
  if (f >= 2147483648.0f) return 2147483647;
  if (f <= -2147483648.0f) return (-2147483647 - 1);
  return (int)f;
}

// One voxel update with the pycuda kernel's arithmetic (OFX_SEM_PYCUDA, tsdf.py:192-288): f32
// throughout (correctly rounded divisions / sqrt via f64, exact by the double-rounding theorem), the
// identity cam_pose applied literally (tsdf.py:236-241), pixel = (int)roundf(f32(f·(x/z) + c) + 0.5)
// (the `+0.5` is a double literal: the sum is formed in f64 and narrowed to roundf's f32 argument),
// skip iff outside the image, z < 0 or depth == 0; depth difference scaled by the ray factor of the
// integer pixel; colours rounded half away from zero. Un-contracted (nvcc's default --fmad=true may
// fuse some of these products: the reference's last bits are not reproducible without nvcc).
__device__ __forceinline__ int update_voxel_pycuda(const CamD& c, const float* __restrict__ depth,
                                                   const float* __restrict__ color_im, float trunc, float obs,
                                                   float x, float y, float z, int64_t vi, float* __restrict__ tsdf,
                                                   float* __restrict__ weight, float* __restrict__ color) {
  const float one = 1.0f, zero = 0.0f;
  const float tx = x - zero, ty = y - zero, tz = z - zero;
  const float px_ = (one * tx + zero * ty) + zero * tz;
  const float py_ = (zero * tx + one * ty) + zero * tz;
  const float pz_ = (zero * tx + zero * ty) + one * tz;
  const float fx = (float)c.fx, fy = (float)c.fy, cx = (float)c.cx, cy = (float)c.cy;
  const float sx = fx * cdiv(px_, pz_) + cx;
  const float sy = fy * cdiv(py_, pz_) + cy;
  const int u = cvt_sat_i32(roundf((float)((double)sx + 0.5)));
  const int v = cvt_sat_i32(roundf((float)((double)sy + 0.5)));
  if (u < 0 || u >= c.W || v < 0 || v >= c.H || pz_ < 0.0f) return 0;
  const int64_t pix = (int64_t)v * c.W + u;
  const float d = depth[pix];
  if (d == 0.0f) return 0;
  float dd = d - pz_;
  const float mx = cdiv((float)u - cx, fx);
  const float my = cdiv((float)v - cy, fy);
  const float ss = (1.0f + mx * mx) + my * my;
  dd = dd * (float)sqrt((double)ss);
  if (dd < -trunc) return 0;
  const float dist = fminf(1.0f, cdiv(dd, trunc));
  const float w_old = weight[vi];
  const float w_new = w_old + obs;
  weight[vi] = w_new;
  tsdf[vi] = cdiv(tsdf[vi] * w_old + obs * dist, w_new);
  if (color) {
    const float C = 65536.0f;
    const float oc = color[vi];
    const float ob = floorf(cdiv(oc, C));
    const float og = floorf(cdiv(oc - ob * 256.0f * 256.0f, 256.0f));
    const float orr = (oc - ob * 256.0f * 256.0f) - og * 256.0f;
    const float nc = color_im[pix];
    const float nb = floorf(cdiv(nc, C));
    const float ng = floorf(cdiv(nc - nb * 256.0f * 256.0f, 256.0f));
    const float nr = (nc - nb * 256.0f * 256.0f) - ng * 256.0f;
    const float b2 = fminf(roundf(cdiv(ob * w_old + obs * nb, w_new)), 255.0f);
    const float g2 = fminf(roundf(cdiv(og * w_old + obs * ng, w_new)), 255.0f);
    const float r2 = fminf(roundf(cdiv(orr * w_old + obs * nr, w_new)), 255.0f);
    color[vi] = (b2 * 256.0f * 256.0f + g2 * 256.0f) + r2;
  }
  return 1;
}

// Pixel of a point (tsdf.py:351-364: u = int(round_half_even((X·fx)/Z + cx)) in f64, v likewise, in-bounds
// test on the rounded values) computed in f32 where that is certified to give the f64 result, else in f64.
// f32: su = f32(f32(f32(x·fx)·rcp(z)) + cx) with v_rcp_f32 (<= 1 ulp): |su - su64| <= 2^-22·|q|·(1+2^-20) +
// 2^-24·|su| + 2^-52·(|q| + |su|) < 2.6e-7·(|q| + |su|) =: tol. If su lies farther than tol from every
// half-integer, rint(su) = rint(su64) (no half-integer lies between them). z below 1e-30 (subnormal
// reciprocals), values within tol of a tie, and |su| >= 2^22 (then tol > 0.5) take the exact f64 form.
// Precondition z > 0. Returns the pixel index or -1 (outside the image).
__device__ __forceinline__ int pixel_of(const CamD& c, float x, float y, float z) {
  const float r = __builtin_amdgcn_rcpf(z);
  const float qx = (x * c.fxf) * r, qy = (y * c.fyf) * r;
  const float su = qx + c.cxf, sv = qy + c.cyf;
  const float tu = 2.6e-7f * (fabsf(qx) + fabsf(su)), tv = 2.6e-7f * (fabsf(qy) + fabsf(sv));
  const float du = fabsf((su - floorf(su)) - 0.5f), dv = fabsf((sv - floorf(sv)) - 0.5f);
  float u, v;
  if (__builtin_expect(!(z >= 1e-30f) || !(du > tu) || !(dv > tv), 0)) {
    const double Z = z;
    const double uu = rint(((double)x * c.fx) / Z + c.cx), vv = rint(((double)y * c.fy) / Z + c.cy);
    if (!(uu >= 0.0 && uu < (double)c.W && vv >= 0.0 && vv < (double)c.H)) return -1;
    return (int)vv * c.W + (int)uu;
  }
  u = rintf(su);
  v = rintf(sv);
  if (!(u >= 0.f && u < (float)c.W && v >= 0.f && v < (float)c.H)) return -1;
  return (int)v * c.W + (int)u;
}

// TSDF + colour update of one voxel whose pixel, depth d and old values are known (tsdf.py:366-376,
// 442-494; numba f64 promotion). Caller checked d > 0 and d - Z >= -trunc. The SDF quotient uses
// num·(1/w_new) and dd·(1/trunc) with an error bound err (a few f64 ulp); its f32 rounding is taken
// when the whole interval [t - err, t + err] rounds to it (|t - f| + err < |f|·2^-25 <= half the f32
// spacing on either side of f), else the exact quotient runs. Bit-identical to update_voxel.
__device__ __forceinline__ void sdf_color_update(double dd, double trunc, double itrunc, double obs, float w_old,
                                                 float t_old, float nc, float oc, bool with_color, float& w_out,
                                                 float& t_out, float& c_out) {
  const float w_new = (float)((double)w_old + obs);
  const float prod = w_old * t_old;
  const double wn = (double)w_new;
  // 1/w_new; skipped for a wave whose voxels are all first observations (w_new == 1: the source frame)
  double inv = 1.0;
  if (__ballot(w_new != 1.0f)) {
    double w = wn;
    asm volatile("" : "+v"(w));   // opaque: the compiler would otherwise fold the branch away (1/1 == 1)
    inv = 1.0 / w;
  }
  const double dist_a = fmin(1.0, dd * itrunc);
  const double num_a = (double)prod + obs * dist_a;
  const double t_a = num_a * inv;
  const double err = 1e-15 * ((fabs(obs) + fabs(num_a)) * inv + fabs(t_a));
  float t_new = (float)t_a;
  if (__builtin_expect(!(fabs(t_a - (double)t_new) + err < fabs((double)t_new) * 0x1p-25), 0)) {
    const double dist = fmin(1.0, dd / trunc);
    t_new = (float)(((double)prod + obs * dist) / wn);
  }
  w_out = w_new;
  t_out = t_new;
  if (with_color) {
    const float C = 65536.0f;
    float ob = floorf(oc / C);
    float og = floorf((oc - ob * C) / 256.0f);
    float orr = (oc - ob * C) - og * 256.0f;
    float nb = floorf(nc / C);
    float ng = floorf((nc - nb * C) / 256.0f);
    float nr = (nc - nb * C) - ng * 256.0f;
    const float ow = (float)obs;
    // f32(a · f64(1/w_new)) = the correctly rounded f32 a/w_new (see update_voxel)
    float b2 = fminf(255.0f, rintf((float)((double)(w_old * ob + ow * nb) * inv)));
    float g2 = fminf(255.0f, rintf((float)((double)(w_old * og + ow * ng) * inv)));
    float r2 = fminf(255.0f, rintf((float)((double)(w_old * orr + ow * nr) * inv)));
    c_out = (b2 * C + g2 * 256.0f) + r2;
  }
}

// Brick coordinates of brick b (< 2^24) from magic reciprocals: q = (b · M) >> 40 with M = ceil(2^40 / d)
// is floor(b / d) for b < 2^40 / d (d <= 2^16): no 64-bit integer division in the kernel prologue.
struct BrickDiv {
  uint64_t mz, my;
};
static BrickDiv make_div(const BrickGeom& g) {
  BrickDiv d;
  d.mz = ((1ull << 40) + (uint64_t)g.nbz - 1) / (uint64_t)g.nbz;
  d.my = ((1ull << 40) + (uint64_t)g.nby - 1) / (uint64_t)g.nby;
  return d;
}
__device__ __forceinline__ void brick_coords(const BrickGeom& g, const BrickDiv& d, uint32_t b, int& i0, int& j0,
                                             int& k0) {
  const uint32_t r = (uint32_t)(((uint64_t)b * d.mz) >> 40);
  const uint32_t bz = b - r * (uint32_t)g.nbz;
  const uint32_t bx = (uint32_t)(((uint64_t)r * d.my) >> 40);
  const uint32_t by = r - bx * (uint32_t)g.nby;
  i0 = (int)(bx + (uint32_t)g.bx0) * kBrick; j0 = (int)by * kBrick; k0 = (int)bz * kBrick;
}

// per-workgroup (= per-brick) update count, plain store: no contended atomics in the hot kernel
__device__ __forceinline__ void count_updates(int n, uint32_t* counts) {
  if (!counts) return;
  __shared__ int s_w[4];
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = (uint32_t)(s_w[0] + s_w[1] + s_w[2] + s_w[3]);
}

// PAL: node records of the brick's palette staged in LDS once per workgroup; voxel anchors are
// palette ranks (uint8). A brick whose palette overflowed (pal_n > kPal) uses the global anchors.
// amdgpu_waves_per_eu(8): the kernel is memory-latency-bound (60 % of wave time in s_waitcnt), so the
// register budget is capped at 64 VGPRs for full occupancy (87 -> 77 us at 512^3). Prefetching the
// voxels' tsdf/weight/colour ahead of the palette barrier is slower: vmcnt retires in order, so the
// barrier would wait on those HBM loads.
template <bool WARP, bool PAL, bool PYC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_integrate(BrickGeom g, CamD c, const float* __restrict__ depth,
                                                    const float* __restrict__ color_im,
                                                    const float4* __restrict__ nodes, int K,
                                                    const int32_t* __restrict__ list,
                                                    const ushort4* __restrict__ anchors,
                                                    const float4* __restrict__ weights,
                                                    const uint16_t* __restrict__ pal_ids,
                                                    const int32_t* __restrict__ pal_n,
                                                    const uchar4* __restrict__ local, double trunc, double obs,
                                                    float* __restrict__ tsdf, float* __restrict__ weight,
                                                    float* __restrict__ color, uint32_t* counter) {
  __shared__ float4 s_node[PAL ? 4 * kPal : 1];
  const int64_t slot = blockIdx.x;
  const int64_t b = (WARP || list) ? (int64_t)list[slot] : slot;   // source frame: optional brick list (hash shard)
  int64_t bz = b % g.nbz;
  int64_t r = b / g.nbz;
  int64_t by = r % g.nby;
  int64_t bx = r / g.nby + g.bx0;
  const int i0 = (int)bx * kBrick, j0 = (int)by * kBrick, k0 = (int)bz * kBrick;
  bool use_pal = false;
  uchar4 la[2];
  if (PAL) {
    // independent loads first (count, palette ids, the voxels' palette ranks), then the node records
    const int pn = pal_n[slot];
    const int pid = pal_ids[slot * kPal + (threadIdx.x >> 2)];
    la[0] = local[slot * kBrickVox + threadIdx.x];
    la[1] = local[slot * kBrickVox + threadIdx.x + 256];
    use_pal = pn <= kPal;
    if (use_pal && (int)threadIdx.x < 4 * pn) s_node[threadIdx.x] = nodes[4 * (int64_t)pid + (threadIdx.x & 3)];
    __syncthreads();
  }
  int n_upd = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int l = threadIdx.x + h * 256;
    const int i = i0 + (l >> 6), j = j0 + ((l >> 3) & 7), k = k0 + (l & 7);
    if (i >= g.Dx || j >= g.Dy || k >= g.Dz) continue;
    float x = vox2world(g.ox, g.vs, i);
    float y = vox2world(g.oy, g.vs, j);
    float z = vox2world(g.oz, g.vs, k);
    if (WARP) {
      const int64_t si = slot * kBrickVox + l;
      int ids[4];
      if (PAL && use_pal) {
        const uchar4 a = la[h];
        ids[0] = a.x; ids[1] = a.y; ids[2] = a.z; ids[3] = a.w;
        if (ids[K - 1] == kNoLocal) continue;   // skin-invalid voxel: never integrated after the source frame
      } else {
        const ushort4 a = anchors[si];
        ids[0] = a.x; ids[1] = a.y; ids[2] = a.z; ids[3] = a.w;
        if (ids[K - 1] == kNoAnchor) continue;
      }
      float4 ww = weights[si];
      float w[4] = {ww.x, ww.y, ww.z, ww.w};
      if (PAL && use_pal) ed_warp(s_node, ids, w, K, x, y, z);
      else ed_warp(nodes, ids, w, K, x, y, z);
    }
    if (PYC) n_upd += update_voxel_pycuda(c, depth, color_im, (float)trunc, (float)obs, x, y, z, b * kBrickVox + l, tsdf,
                                          weight, color);
    else n_upd += update_voxel(c, depth, color_im, trunc, 1.0 / trunc, obs, x, y, z, b * kBrickVox + l, tsdf, weight, color);
  }
  count_updates(n_upd, counter);
}

// The fused warp + integrate of the skinned bricks for K = 4 anchors and the reference CPU semantics (the
// bench / pipeline case): one 256-thread workgroup per listed brick, voxels l and l + 256 per thread (same
// y and z), three dependent memory trips —
//   1. brick id, palette count / ids, the voxels' palette ranks;
//   2. the palette's node records (into LDS, one barrier) + the skin-valid voxels' weights and old
//      tsdf / weight (branch-free: the other voxels re-read the brick's first voxel);
//   3. depth, colour image and old colour (likewise branch-free);
// then the stores. Warp with the anchors unrolled (no dynamic register indexing), pixel in certified f32
// (pixel_of), SDF rounding certified cheaply (sdf_color_update), per-wave update counts by ballot;
// bit-identical to k_integrate<1,1,0>. The kernel is VALU-bound: every per-wave instruction
// is shared by two voxels.
#ifndef OFX_INT_WPE
#define OFX_INT_WPE 7   // (tuning builds: -DOFX_INT_WPE=n; 7: 72 VGPRs, 12 B of scratch, 90.0 -> 84.9 us against 6;
                        // 8: 64 VGPRs, 56 B of scratch, 146 us: profiles/r05_ab.json)
#endif
template <bool COLOR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OFX_INT_WPE))) void k_integrate_pal4(
    BrickGeom g, BrickDiv bd, CamD c, const float* __restrict__ depth, const float* __restrict__ color_im,
    const float4* __restrict__ nodes, int n_nodes, const int32_t* __restrict__ list,
    const ushort4* __restrict__ anchors, const float4* __restrict__ weights, const uint16_t* __restrict__ pal_ids,
    const int32_t* __restrict__ pal_n, const uchar4* __restrict__ local, double trunc, double itrunc, double obs,
    float* __restrict__ tsdf, float* __restrict__ weight, float* __restrict__ color, uint32_t* counter,
    const uint8_t* __restrict__ active) {
  __shared__ float4 s_node[4 * kPal];
  __shared__ float s_xyz[3 * kBrick];   // vox2world of the brick's 8 x, y and z coordinates
  __shared__ uint32_t s_cnt[4];
  const int tid = threadIdx.x;
  const uint32_t slot = blockIdx.x;
  // ---- trip 1 (unconditional loads: a branch would split the trip)
  const uint32_t b = (uint32_t)list[slot];
  const int pn = pal_n[slot];
  const int pid = pal_ids[slot * kPal + (tid >> 2)];
  uchar4 la[2];
  la[0] = local[slot * kBrickVox + tid];
  la[1] = local[slot * kBrickVox + tid + 256];
  const int live = active ? (int)active[slot] : 1;   // (uniform: a scalar load, with trip 1)
  asm volatile("" ::: "memory");
  if (!live) {   // k_brick_cull proved that no voxel of this brick updates (the whole workgroup leaves)
    if (counter && tid == 0) counter[blockIdx.x] = 0;
    return;
  }
  int i0, j0, k0;
  brick_coords(g, bd, b, i0, j0, k0);
  const bool use_pal = pn <= kPal;
  const int j = j0 + ((tid >> 3) & 7), k = k0 + (tid & 7);
  const bool in_yz = j < g.Dy && k < g.Dz;
  const uint32_t vb = b * (uint32_t)kBrickVox + (uint32_t)tid;   // voxel slot of l = tid (n_slots < 2^31)
  bool act[2];
  ushort4 ga[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    act[h] = in_yz && i0 + (tid >> 6) + 4 * h < g.Dx;
    if (use_pal) {
      act[h] = act[h] && la[h].w != kNoLocal;
    } else {   // palette overflow (> kPal distinct anchors in the brick): global anchors, one more trip
      ga[h] = anchors[slot * kBrickVox + tid + 256 * h];
      act[h] = act[h] && ga[h].w != kNoAnchor;
    }
  }
  // ---- trip 2
  const float4 nrec = nodes[4 * (int64_t)min(pid, n_nodes - 1) + (tid & 3)];
  float4 ww[2];
  float t_old[2], w_old[2];
  // branch-free: a voxel outside the skin loads the brick's first voxel instead (a line the brick reads anyway), so
  // no load sits in a branch and the waits before the barrier / the warp count exactly (masked loads made the
  // compiler wait for each voxel's weights inside its branch and for every load of the trip before the barrier:
  // 94.7 -> 90.9 us isolated, 100.6 -> 94.1 us in the frame loop, profiles/r05_ab.json)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t e = act[h] ? (uint32_t)(tid + 256 * h) : 0u;
    ww[h] = weights[slot * kBrickVox + e];
    t_old[h] = tsdf[b * (uint32_t)kBrickVox + e];
    w_old[h] = weight[b * (uint32_t)kBrickVox + e];
  }
  if (use_pal && tid < 4 * pn) s_node[tid] = nrec;
  if (tid >= 256 - 3 * kBrick) {   // the last 24 lanes (one wave): x, y, z world coordinates of the brick
    const int q = tid - (256 - 3 * kBrick), ax = q >> 3, o = q & 7;
    s_xyz[q] = ax == 0 ? vox2world(g.ox, g.vs, i0 + o) : ax == 1 ? vox2world(g.oy, g.vs, j0 + o)
                                                               : vox2world(g.oz, g.vs, k0 + o);
  }
  __syncthreads();
  const float y0 = s_xyz[kBrick + ((tid >> 3) & 7)], z0 = s_xyz[2 * kBrick + (tid & 7)];
  int pix[2];
  float zw[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    pix[h] = -1;
    zw[h] = 0.f;
    if (!act[h]) continue;
    float px = s_xyz[(tid >> 6) + 4 * h], py = y0, pz = z0;
    const float w[4] = {ww[h].x, ww[h].y, ww[h].z, ww[h].w};
    if (use_pal) {
      const int ids[4] = {la[h].x, la[h].y, la[h].z, la[h].w};
      ed_warp(s_node, ids, w, 4, px, py, pz);
    } else {
      const int ids[4] = {ga[h].x, ga[h].y, ga[h].z, ga[h].w};
      ed_warp(nodes, ids, w, 4, px, py, pz);
    }
    zw[h] = pz;
    if (pz > 0.f) pix[h] = pixel_of(c, px, py, pz);
  }
  // ---- trip 3 (skin-valid voxels; pixel 0 stands in for the unprojected ones)
  float d[2], nc[2], oc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pc = pix[h] >= 0 ? pix[h] : 0;
    d[h] = depth[pc];
    if (COLOR) { nc[h] = color_im[pc]; oc[h] = color[b * (uint32_t)kBrickVox + (act[h] ? (uint32_t)(tid + 256 * h) : 0u)]; }
  }
  // the loaded values pass through an empty asm: both halves' loads are issued before the first use (else the second
  // half's loads sink into its update branch: two more dependent trips)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (COLOR) asm volatile("" : "+v"(d[h]), "+v"(nc[h]), "+v"(oc[h]));
    else asm volatile("" : "+v"(d[h]));
  }
  asm volatile("" ::: "memory");
  uint32_t n_upd = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bool upd = false;
    if (pix[h] >= 0) {
      const double dd = (double)d[h] - (double)zw[h];
      if (d[h] > 0.f && dd >= -trunc) {
        float wn, tn, cn;
        sdf_color_update(dd, trunc, itrunc, obs, w_old[h], t_old[h], COLOR ? nc[h] : 0.f, COLOR ? oc[h] : 0.f,
                         COLOR, wn, tn, cn);
        weight[vb + 256 * h] = wn;
        tsdf[vb + 256 * h] = tn;
        if (COLOR) color[vb + 256 * h] = cn;
        upd = true;
      }
    }
    n_upd += (uint32_t)__popcll(__ballot(upd));   // per-wave count: scalar, no lane shuffles
  }
  if (counter) {
    if ((tid & 63) == 0) s_cnt[tid >> 6] = n_upd;
    __syncthreads();
    if (tid == 0) counter[blockIdx.x] = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
  }
}

// ---- brick cull of the warped integrate (ofx_integrate_palette_cull): which listed bricks can update a voxel at all.
// Per 8x8 pixel tile the largest depth (NaN pixels never update and are skipped; +inf propagates). One thread per tile,
// the tile's 8 rows as 2 x 16-B loads each (lanes = consecutive tiles of a tile row: coalesced); W % 4 == 0 and a 16-B
// aligned image (else the per-pixel loop).
__global__ __launch_bounds__(256) void k_tile_max(const float* __restrict__ depth, int W, int H, int TW, int TH,
                                                  float* __restrict__ tiles) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= TW * TH) return;
  const int tx = t % TW, ty = t / TW;
  float m = 0.f;
  if ((W & 3) == 0 && (reinterpret_cast<uintptr_t>(depth) & 15) == 0 && tx * 8 + 8 <= W && ty * 8 + 8 <= H) {
    float4 v[16];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float4* p = reinterpret_cast<const float4*>(depth + (int64_t)(ty * 8 + r) * W + tx * 8);
      v[2 * r] = p[0];
      v[2 * r + 1] = p[1];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) m = fmaxf(m, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
  } else {
    for (int y = ty * 8; y < min(ty * 8 + 8, H); ++y)
      for (int x = tx * 8; x < min(tx * 8 + 8, W); ++x) m = fmaxf(m, depth[(int64_t)y * W + x]);
  }
  tiles[t] = m;
}

// 16 lanes per listed brick (4 bricks per wave). A voxel p of the brick warps to Σ_k w_k T_k(p) with T_k(p) =
// R_k(p - g_k) + g_k + t_k over its (palette) anchors, weights w_k >= 0 of sum S = Σ/(Σ + 1e-6) (warpfield.py:121) with
// S in [0.999, 1] (every valid anchor lies within 4σ: each w >= exp(-8), Σ >= 1.3e-3). T_k maps the box of the brick's
// voxel centres [c ± h] into [T_k(c) ± |R_k| h] (any matrix R_k); so the warped voxels lie in the box B spanning those
// boxes and their S-scaled copies, grown by a margin far above f32 rounding (1e-4 m). The brick can update a voxel only
// if some point of B has z > 0 projecting into the image (the pixel range of B's corners, ±1 px) onto a pixel of depth
// d > 0 with d - z >= -trunc, i.e. if the largest depth over the tiles of that range is >= z_min(B) - trunc. Bricks
// whose box reaches z < 1e-3, spans more than 64 tiles, or whose palette overflowed are kept (active).
__device__ __forceinline__ float grp16_min(float x) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) x = fminf(x, __shfl_xor(x, off, 16));
  return x;
}
__device__ __forceinline__ float grp16_max(float x) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) x = fmaxf(x, __shfl_xor(x, off, 16));
  return x;
}
__global__ __launch_bounds__(256) void k_brick_cull(BrickGeom g, BrickDiv bd, CamD c, const float4* __restrict__ nodes,
                                                    int n_nodes, const int32_t* __restrict__ list,
                                                    const uint16_t* __restrict__ pal_ids, const int32_t* __restrict__ pal_n,
                                                    int n_list, const float* __restrict__ tiles, int TW, int TH,
                                                    double trunc, uint8_t* __restrict__ active) {
  const int sub = threadIdx.x & 15;
  const int s = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sc = s < n_list ? s : n_list - 1;   // (the last group of the grid may overhang: clamped, not stored)
  const int pn = pal_n[sc];
  const uint32_t b = (uint32_t)list[sc];
  static_assert(kPal == 16 * 4, "k_brick_cull: 16 lanes x 4 palette slots must cover the palette (else not conservative)");
  int pid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) pid[i] = pal_ids[(int64_t)sc * kPal + sub + 16 * i];
  int i0, j0, k0;
  brick_coords(g, bd, b, i0, j0, k0);
  // the voxel centres of the brick (clipped to the volume) span [lo, hi] per axis
  const int ni = min(kBrick, g.Dx - i0), nj = min(kBrick, g.Dy - j0), nk = min(kBrick, g.Dz - k0);
  const float cx0 = vox2world(g.ox, g.vs, i0), cx1 = vox2world(g.ox, g.vs, i0 + ni - 1);
  const float cy0 = vox2world(g.oy, g.vs, j0), cy1 = vox2world(g.oy, g.vs, j0 + nj - 1);
  const float cz0 = vox2world(g.oz, g.vs, k0), cz1 = vox2world(g.oz, g.vs, k0 + nk - 1);
  const float px = 0.5f * (cx0 + cx1), py = 0.5f * (cy0 + cy1), pz = 0.5f * (cz0 + cz1);
  const float hx = 0.5f * (cx1 - cx0), hy = 0.5f * (cy1 - cy0), hz = 0.5f * (cz1 - cz0);
  float lo[3] = {3e38f, 3e38f, 3e38f}, hi[3] = {-3e38f, -3e38f, -3e38f};
  float4 rec[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // (clamped, unconditional: one memory trip)
    const float4* n = nodes + 4 * (int64_t)min(max(pid[i], 0), n_nodes - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) rec[i][q] = n[q];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (sub + 16 * i >= pn || pn > kPal) continue;
    // record [R00 R10 R01 R11 | R02 R12 g0 g1 | t0 t1 R20 R21 | R22 g2 t2 0] (ofx_pack_nodes)
    const float4 a = rec[i][0], bb = rec[i][1], cc = rec[i][2], d = rec[i][3];
    const float dx = px - bb.z, dy = py - bb.w, dz = pz - d.y;
    const float t0 = a.x * dx + a.z * dy + bb.x * dz + bb.z + cc.x;
    const float t1 = a.y * dx + a.w * dy + bb.y * dz + bb.w + cc.y;
    const float t2 = cc.z * dx + cc.w * dy + d.x * dz + d.y + d.z;
    const float e0 = fabsf(a.x) * hx + fabsf(a.z) * hy + fabsf(bb.x) * hz + 1e-4f;
    const float e1 = fabsf(a.y) * hx + fabsf(a.w) * hy + fabsf(bb.y) * hz + 1e-4f;
    const float e2 = fabsf(cc.z) * hx + fabsf(cc.w) * hy + fabsf(d.x) * hz + 1e-4f;
    lo[0] = fminf(lo[0], t0 - e0); hi[0] = fmaxf(hi[0], t0 + e0);
    lo[1] = fminf(lo[1], t1 - e1); hi[1] = fmaxf(hi[1], t1 + e1);
    lo[2] = fminf(lo[2], t2 - e2); hi[2] = fmaxf(hi[2], t2 + e2);
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) { lo[q] = grp16_min(lo[q]); hi[q] = grp16_max(hi[q]); }
  bool keep = pn > kPal || pn <= 0;
  float zmin = 0.f;
  int tx0 = 0, tx1 = -1, ty0 = 0, ty1 = -1;
  if (!keep) {
    constexpr float kS = 0.999f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float l = lo[q], h = hi[q];
      lo[q] = fminf(l, kS * l);
      hi[q] = fmaxf(h, kS * h);
    }
    zmin = lo[2];
    if (hi[2] > 0.f) {
      if (!(lo[2] >= 1e-3f)) {
        keep = true;
      } else {
        float umin = 3e38f, umax = -3e38f, vmin = 3e38f, vmax = -3e38f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float X = (k & 1) ? hi[0] : lo[0], Y = (k & 2) ? hi[1] : lo[1], Z = (k & 4) ? hi[2] : lo[2];
          const float iz = 1.0f / Z;
          const float u = c.fxf * X * iz + c.cxf, v = c.fyf * Y * iz + c.cyf;
          umin = fminf(umin, u); umax = fmaxf(umax, u); vmin = fminf(vmin, v); vmax = fmaxf(vmax, v);
        }
        const float x0 = fmaxf(floorf(umin) - 1.f, 0.f), x1 = fminf(ceilf(umax) + 1.f, (float)(c.W - 1));
        const float y0 = fmaxf(floorf(vmin) - 1.f, 0.f), y1 = fminf(ceilf(vmax) + 1.f, (float)(c.H - 1));
        if (x0 <= x1 && y0 <= y1) {
          tx0 = (int)x0 >> 3; tx1 = (int)x1 >> 3; ty0 = (int)y0 >> 3; ty1 = (int)y1 >> 3;
          if ((tx1 - tx0 + 1) * (ty1 - ty0 + 1) > 64) keep = true;
        }
      }
    }
  }
  // the tiles of the pixel range, 4 per lane
  float dm = 0.f;
  const int ntx = tx1 - tx0 + 1, nt = (tx1 >= tx0 && ty1 >= ty0) ? ntx * (ty1 - ty0 + 1) : 0;
  if (!keep) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = sub + 16 * i;
      if (e < nt) dm = fmaxf(dm, tiles[(int64_t)(ty0 + e / ntx) * TW + tx0 + e % ntx]);
    }
  }
  dm = grp16_max(dm);
  const bool upd = keep || (dm > 0.f && (double)dm - (double)zmin >= -trunc - 1e-4);
  if (sub == 0 && s < n_list) active[s] = upd ? 1 : 0;
}

// Source frame (tsdf.py:395-398: every voxel at its world position, all valid) with per-brick projection
// tables: on the voxel grid u depends only on (i, k) and v only on (j, k), so one workgroup computes the
// brick's 8x8 u-table and 8x8 v-table exactly in f64 (the reference expression, 128 lanes, one each) plus
// the 24 world coordinates, and every voxel then looks its pixel up in LDS. brick_list (may be NULL: all
// bricks of the shard) restricts the pass to the listed bricks (hash-bucket shards). 2 voxels per thread.
template <bool COLOR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_integrate_src(
    BrickGeom g, BrickDiv bd, CamD c, const float* __restrict__ depth, const float* __restrict__ color_im,
    const int32_t* __restrict__ list, double trunc, double itrunc, double obs, float* __restrict__ tsdf,
    float* __restrict__ weight, float* __restrict__ color, uint32_t* counter) {
  __shared__ int s_u[kBrick * kBrick], s_v[kBrick * kBrick];
  __shared__ float s_xyz[3 * kBrick];
  __shared__ uint32_t s_cnt[4];
  const int tid = threadIdx.x;
  const uint32_t b = list ? (uint32_t)list[blockIdx.x] : (uint32_t)blockIdx.x;
  int i0, j0, k0;
  brick_coords(g, bd, b, i0, j0, k0);
  const uint32_t vb = b * (uint32_t)kBrickVox + (uint32_t)tid;
  // old values first (every in-volume voxel: the reference reads them all), then the tables
  const int j = j0 + ((tid >> 3) & 7), k = k0 + (tid & 7);
  bool in[2];
  float t_old[2], w_old[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    in[h] = j < g.Dy && k < g.Dz && i0 + (tid >> 6) + 4 * h < g.Dx;
    if (in[h]) { t_old[h] = tsdf[vb + 256 * h]; w_old[h] = weight[vb + 256 * h]; }
  }
  if (tid < 2 * kBrick * kBrick) {   // u(i, k) for tid < 64, v(j, k) for 64 <= tid < 128 (tsdf.py:351-364)
    const int q = tid & 63, a = q >> 3, kk = q & 7;
    const double Z = (double)vox2world(g.oz, g.vs, k0 + kk);
    int r = -1;
    if (tid < 64) {
      const double X = (double)vox2world(g.ox, g.vs, i0 + a);
      const double u = rint((X * c.fx) / Z + c.cx);
      if (Z > 0.0 && u >= 0.0 && u < (double)c.W) r = (int)u;
      s_u[q] = r;
    } else {
      const double Y = (double)vox2world(g.oy, g.vs, j0 + a);
      const double v = rint((Y * c.fy) / Z + c.cy);
      if (Z > 0.0 && v >= 0.0 && v < (double)c.H) r = (int)v;
      s_v[q] = r;
    }
  } else if (tid >= 256 - kBrick) {
    s_xyz[tid - (256 - kBrick)] = vox2world(g.oz, g.vs, k0 + (tid - (256 - kBrick)));
  }
  __syncthreads();
  const int lz = tid & 7, ly = (tid >> 3) & 7;
  const int vv = s_v[ly * kBrick + lz];
  const float z = s_xyz[lz];
  int pix[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int uu = s_u[((tid >> 6) + 4 * h) * kBrick + lz];
    pix[h] = (in[h] && uu >= 0 && vv >= 0) ? vv * c.W + uu : -1;
  }
  float d[2], nc[2], oc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (pix[h] >= 0) {
      d[h] = depth[pix[h]];
      if (COLOR) { nc[h] = color_im[pix[h]]; oc[h] = color[vb + 256 * h]; }
    }
  }
  asm volatile("" ::: "memory");
  uint32_t n_upd = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bool upd = false;
    if (pix[h] >= 0) {
      const double dd = (double)d[h] - (double)z;
      if (d[h] > 0.f && dd >= -trunc) {
        float wn, tn, cn;
        sdf_color_update(dd, trunc, itrunc, obs, w_old[h], t_old[h], COLOR ? nc[h] : 0.f, COLOR ? oc[h] : 0.f,
                         COLOR, wn, tn, cn);
        weight[vb + 256 * h] = wn;
        tsdf[vb + 256 * h] = tn;
        if (COLOR) color[vb + 256 * h] = cn;
        upd = true;
      }
    }
    n_upd += (uint32_t)__popcll(__ballot(upd));
  }
  if (counter) {
    if ((tid & 63) == 0) s_cnt[tid >> 6] = n_upd;
    __syncthreads();
    if (tid == 0) counter[blockIdx.x] = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
  }
}

// Integrate of explicit points (TSDFVolume.integrate on already deformed points: tsdf.py:442-494 with pts
// from WarpField.deform_tsdf, warpfield.py:369-380): point p updates voxel vox[p] (C-order id), with the
// same arithmetic as the fused kernels (pixel_of / sdf_color_update, or the pycuda form). Points of voxels
// outside this shard are ignored. Voxel ids must be distinct (one writer per voxel).
template <bool PYC>
__global__ __launch_bounds__(256) void k_integrate_points(BrickGeom g, CamD c, const float* __restrict__ depth,
                                                          const float* __restrict__ color_im,
                                                          const float* __restrict__ pts, const int64_t* __restrict__ vox,
                                                          const uint8_t* __restrict__ valid, int64_t n, double trunc,
                                                          double itrunc, double obs, float* __restrict__ tsdf,
                                                          float* __restrict__ weight, float* __restrict__ color,
                                                          uint32_t* n_updated) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int upd = 0;
  if (p < n && (!valid || valid[p])) {
    const int64_t v = vox[p];
    const int64_t DyDz = (int64_t)g.Dy * g.Dz;
    const int i = (int)(v / DyDz), j = (int)((v / g.Dz) % g.Dy), k = (int)(v % g.Dz);
    if (v >= 0 && i < g.Dx && (i >> 3) >= g.bx0 && (i >> 3) < g.bx1) {
      const int64_t b = ((int64_t)((i >> 3) - g.bx0) * g.nby + (j >> 3)) * g.nbz + (k >> 3);
      const int64_t vi = b * kBrickVox + ((i & 7) * 8 + (j & 7)) * 8 + (k & 7);
      const float x = pts[3 * p], y = pts[3 * p + 1], z = pts[3 * p + 2];
      if (PYC) {
        upd = update_voxel_pycuda(c, depth, color_im, (float)trunc, (float)obs, x, y, z, vi, tsdf, weight, color);
      } else if (z > 0.f) {
        const int pix = pixel_of(c, x, y, z);
        if (pix >= 0) {
          const float d = depth[pix];
          const double dd = (double)d - (double)z;
          if (d > 0.f && dd >= -trunc) {
            float wn, tn, cn;
            sdf_color_update(dd, trunc, itrunc, obs, weight[vi], tsdf[vi], color ? color_im[pix] : 0.f,
                             color ? color[vi] : 0.f, color != nullptr, wn, tn, cn);
            weight[vi] = wn;
            tsdf[vi] = tn;
            if (color) color[vi] = cn;
            upd = 1;
          }
        }
      }
    }
  }
  if (n_updated) {
    for (int off = 32; off > 0; off >>= 1) upd += __shfl_xor(upd, off, 64);
    if ((threadIdx.x & 63) == 0 && upd) atomicAdd(n_updated, (uint32_t)upd);
  }
}

__global__ __launch_bounds__(256) void k_deform_points(const float* __restrict__ pts, int64_t n,
                                                        const int32_t* __restrict__ anchors,
                                                        const float* __restrict__ weights,
                                                        const uint8_t* __restrict__ valid, int K,
                                                        const float4* __restrict__ nodes, int normals,
                                                        float* __restrict__ out) {
  int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= n) return;
  float x = pts[3 * p], y = pts[3 * p + 1], z = pts[3 * p + 2];
  bool v = valid ? valid[p] != 0 : true;
  if (v) {
    int ids[4];
    float w[4];
    for (int k = 0; k < K; ++k) { ids[k] = anchors[p * K + k]; w[k] = weights[p * K + k]; }
    if (!normals) {
      ed_warp(nodes, ids, w, K, x, y, z);
    } else {
      // WarpField.deform_normals: deform_lbs with zero translation, weights==0 skipped (warpfield.py:208-231,312-345)
      float ax = 0.f, ay = 0.f, az = 0.f;
      for (int k = 0; k < K; ++k) {
        if (w[k] == 0.f) continue;
        const float4* nd = nodes + 4 * (int64_t)ids[k];
        const float4 a = nd[0], b = nd[1], c = nd[2], d = nd[3];   // record layout: ofx_pack_nodes
        float rx = a.x * x; rx = rx + a.z * y; rx = rx + b.x * z;
        float ry = a.y * x; ry = ry + a.w * y; ry = ry + b.y * z;
        float rz = c.z * x; rz = rz + c.w * y; rz = rz + d.x * z;
        ax = ax + w[k] * rx; ay = ay + w[k] * ry; az = az + w[k] * rz;
      }
      x = ax; y = ay; z = az;
    }
  }
  if (normals) {
    float nrm = (float)sqrt((double)((x * x + y * y) + z * z));
    x = cdiv(x, nrm); y = cdiv(y, nrm); z = cdiv(z, nrm);
  }
  out[3 * p] = x; out[3 * p + 1] = y; out[3 * p + 2] = z;
}

// WarpField.deform_lbs (warpfield.py:208-231, numba; CUDA twin deform_lbs_cuda :234-266 with
// warp_point_with_nodes :607-630): origin-form transforms, y = Σ_k w_k (R_k x + t_k) over the anchors
// with w_k != 0, accumulated from 0 in anchor order, f32; R_k x as ((R0·x + R1·y) + R2·z). Invalid
// points keep x. R f32[N*9] row-major, t f32[N*3] (t = -R g + g + T, warpfield.py:407-408).
__global__ __launch_bounds__(256) void k_deform_lbs(const float* __restrict__ pts, int64_t n,
                                                     const int32_t* __restrict__ anchors,
                                                     const float* __restrict__ weights,
                                                     const uint8_t* __restrict__ valid, int K,
                                                     const float* __restrict__ R, const float* __restrict__ t,
                                                     float* __restrict__ out) {
  int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float x = pts[3 * p], y = pts[3 * p + 1], z = pts[3 * p + 2];
  float ox = x, oy = y, oz = z;
  if (valid ? valid[p] != 0 : true) {
    ox = 0.f; oy = 0.f; oz = 0.f;
    for (int k = 0; k < K; ++k) {
      const float w = weights[p * K + k];
      if (w == 0.f) continue;
      const int64_t a = anchors[p * K + k];
      const float* r = R + 9 * a;
      const float* tt = t + 3 * a;
      const float nx = ((r[0] * x + r[1] * y) + r[2] * z) + tt[0];
      const float ny = ((r[3] * x + r[4] * y) + r[5] * z) + tt[1];
      const float nz = ((r[6] * x + r[7] * y) + r[8] * z) + tt[2];
      ox = ox + w * nx; oy = oy + w * ny; oz = oz + w * nz;
    }
  }
  out[3 * p] = ox; out[3 * p + 1] = oy; out[3 * p + 2] = oz;
}

// F32: the projection of f32 points as numba types cam2pix on an f32 array (tsdf.py:351-364 called from
// get_visible_nodes with the f32 deformed nodes, tsdf.py:614-638): (x·fx)/z + cx in f32 with the f32 intrinsics,
// np.round (half-even) in f32, int(); the depth lookup and the difference stay f64 as get_depth_from_image's
// np.zeros array makes them (tsdf.py:576-612). F32 = false: the f64 form of the integrate path (f64 cam_pts).
__device__ __forceinline__ int64_t project_f32(const CamD& c, float x, float y, float z) {
  const float su = cdiv(x * c.fxf, z) + c.cxf, sv = cdiv(y * c.fyf, z) + c.cyf;
  const float u = rintf(su), v = rintf(sv);
  if (!(u >= 0.0f && u < (float)c.W && v >= 0.0f && v < (float)c.H && z > 0.0f)) return -1;
  return (int64_t)v * c.W + (int64_t)u;
}

template <bool F32>
__global__ void k_visibility(const float* __restrict__ pts, int64_t n, CamD c, const float* __restrict__ depth,
                             double trunc, uint8_t* __restrict__ valid, double* __restrict__ ddiff) {
  int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= n) return;
  double Z;
  int64_t pix;
  if (F32) {
    Z = pts[3 * p + 2];
    pix = project_f32(c, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2]);
  } else {
    pix = project(c, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2], Z);
  }
  double dv = pix >= 0 ? (double)depth[pix] : 0.0;
  double dd = dv - Z;
  valid[p] = (dv > 0.0 && dd >= -trunc) ? 1 : 0;
  if (ddiff) ddiff[p] = dd;
}

static CamD make_cam(const ofx_camera* cam) {
  CamD c;
  c.fx = cam->fx; c.fy = cam->fy; c.cx = cam->cx; c.cy = cam->cy;
  c.fxf = cam->fx; c.fyf = cam->fy; c.cxf = cam->cx; c.cyf = cam->cy;
  c.W = cam->width; c.H = cam->height;
  return c;
}

}  // namespace ofx

using namespace ofx;

namespace {
// profiling hook state (ofx_integrate_timing): hipEvent pairs around the warped integrate kernel launches
std::mutex g_int_mu;
bool g_int_timing = false;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_int_ev;

// events recorded by the dispatch itself (hipExtLaunchKernel: the kernel's own start / end), so host gaps
// before a launch never count
struct IntTimer {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  IntTimer() {
    std::lock_guard<std::mutex> lk(g_int_mu);
    if (!g_int_timing) return;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) e0 = e1 = nullptr;
  }
  ~IntTimer() {
    if (!e0) return;
    std::lock_guard<std::mutex> lk(g_int_mu);
    g_int_ev.emplace_back(e0, e1);
  }
};
#define OFX_TIMED_LAUNCH(T, kernel, grid, block, shm, stream, ...)                                         \
  do {                                                                                                    \
    if ((T).e0)                                                                                           \
      hipExtLaunchKernelGGL(kernel, grid, block, shm, stream, (T).e0, (T).e1, 0, __VA_ARGS__);            \
    else                                                                                                  \
      hipLaunchKernelGGL(kernel, grid, block, shm, stream, __VA_ARGS__);                                  \
  } while (0)
}  // namespace

extern "C" {

int ofx_integrate_timing(int32_t enable, double* kernel_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_int_mu);
  double ms = 0.0;
  for (auto& e : g_int_ev) {
    float t = 0.f;
    OFX_HIP(hipEventSynchronize(e.second));
    OFX_HIP(hipEventElapsedTime(&t, e.first, e.second));
    ms += t;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (kernel_ms) *kernel_ms = ms;
  if (launches) *launches = (int64_t)g_int_ev.size();
  g_int_ev.clear();
  g_int_timing = enable != 0;
  return OFX_OK;
}

int ofx_integrate(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth, const float* color_im,
                  int32_t warp, const float* packed_nodes, int32_t n_nodes, int32_t k, const int32_t* brick_list,
                  int32_t n_list, const uint16_t* anchors, const float* weights, double obs_weight, float* tsdf,
                  float* weight, float* color, uint32_t* n_updated, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(cam && depth && tsdf && weight, "null buffer");
  OFX_CHECK_ARG(cam->width > 0 && cam->height > 0, "bad camera size");
  OFX_CHECK_ARG((color == nullptr) == (color_im == nullptr), "color and color_im must both be set or both NULL");
  CamD c = make_cam(cam);
  hipStream_t hs = as_stream(s);
  OFX_CHECK_ARG(desc->semantics == OFX_SEM_CPU || desc->semantics == OFX_SEM_PYCUDA, "bad semantics %d", desc->semantics);
  const bool pyc = desc->semantics == OFX_SEM_PYCUDA;
  if (!warp && !pyc && g.n_bricks * kBrickVox < (1ll << 31) && !getenv("OFX_INT_GENERIC")) {
    const unsigned nb = brick_list ? (unsigned)n_list : (unsigned)g.n_bricks;
    if (nb == 0) return OFX_OK;
    if (color)
      hipLaunchKernelGGL(k_integrate_src<true>, dim3(nb), dim3(256), 0, hs, g, make_div(g), c, depth, color_im,
                         brick_list, desc->trunc_margin, 1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color,
                         n_updated);
    else
      hipLaunchKernelGGL(k_integrate_src<false>, dim3(nb), dim3(256), 0, hs, g, make_div(g), c, depth, color_im,
                         brick_list, desc->trunc_margin, 1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color,
                         n_updated);
  } else if (!warp) {
    // generic source-frame form: pycuda semantics, shards of >= 2^31 voxels, or the OFX_INT_GENERIC A/B; a brick
    // list (hash shard) is walked as in the warped form
    OFX_CHECK_ARG(brick_list == nullptr || (n_list >= 0 && n_list <= g.n_bricks), "bad n_list");
    const unsigned nb = brick_list ? (unsigned)n_list : (unsigned)g.n_bricks;
    if (nb == 0) return OFX_OK;
    hipLaunchKernelGGL(pyc ? (k_integrate<false, false, true>) : (k_integrate<false, false, false>),
                       dim3(nb), dim3(256), 0, hs, g, c, depth,
                       color_im, (const float4*)nullptr, 1, brick_list, (const ushort4*)nullptr,
                       (const float4*)nullptr, (const uint16_t*)nullptr, (const int32_t*)nullptr,
                       (const uchar4*)nullptr, desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated);
  } else {
    OFX_CHECK_ARG(k >= 1 && k <= 4 && n_nodes >= k, "bad k/n_nodes");
    OFX_CHECK_ARG(n_list >= 0 && n_list <= g.n_bricks, "bad n_list");
    if (n_list == 0) return OFX_OK;
    OFX_CHECK_ARG(packed_nodes && brick_list && anchors && weights, "null warp buffer");
    IntTimer timer;
    OFX_TIMED_LAUNCH(timer, pyc ? (k_integrate<true, false, true>) : (k_integrate<true, false, false>), dim3((unsigned)n_list),
                       dim3(256), 0, hs, g, c, depth, color_im,
                       (const float4*)packed_nodes, k, brick_list, (const ushort4*)anchors, (const float4*)weights,
                       (const uint16_t*)nullptr, (const int32_t*)nullptr, (const uchar4*)nullptr,
                       desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated);
  }
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_integrate_palette(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth,
                          const float* color_im, const float* packed_nodes, int32_t n_nodes, int32_t k,
                          const int32_t* brick_list, int32_t n_list, const uint16_t* anchors, const float* weights,
                          const uint16_t* pal_ids, const int32_t* pal_n, const uint8_t* local_anchors,
                          double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                          ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(cam && depth, "null camera/depth");
  OFX_CHECK_ARG(cam->width > 0 && cam->height > 0, "bad camera size");
  OFX_CHECK_ARG((color == nullptr) == (color_im == nullptr), "color and color_im must both be set or both NULL");
  OFX_CHECK_ARG(k >= 1 && k <= 4 && n_nodes >= k, "bad k/n_nodes");
  OFX_CHECK_ARG(n_list >= 0 && n_list <= g.n_bricks, "bad n_list");
  if (n_list == 0) return OFX_OK;
  OFX_CHECK_ARG(packed_nodes && brick_list && anchors && weights && pal_ids && pal_n && local_anchors,
                "null warp/palette buffer");
  OFX_CHECK_ARG(desc->semantics == OFX_SEM_CPU || desc->semantics == OFX_SEM_PYCUDA, "bad semantics %d", desc->semantics);
  IntTimer timer;
  if (desc->semantics == OFX_SEM_CPU && k == 4 && g.n_bricks * kBrickVox < (1ll << 31) && !getenv("OFX_INT_GENERIC")) {
    if (color)
      OFX_TIMED_LAUNCH(timer, k_integrate_pal4<true>, dim3((unsigned)n_list), dim3(256), 0, as_stream(s), g, make_div(g),
                         make_cam(cam), depth, color_im, (const float4*)packed_nodes, n_nodes, brick_list,
                         (const ushort4*)anchors, (const float4*)weights, pal_ids, pal_n, (const uchar4*)local_anchors,
                         desc->trunc_margin, 1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated,
                         (const uint8_t*)nullptr);
    else
      OFX_TIMED_LAUNCH(timer, k_integrate_pal4<false>, dim3((unsigned)n_list), dim3(256), 0, as_stream(s), g, make_div(g),
                         make_cam(cam), depth, color_im, (const float4*)packed_nodes, n_nodes, brick_list,
                         (const ushort4*)anchors, (const float4*)weights, pal_ids, pal_n, (const uchar4*)local_anchors,
                         desc->trunc_margin, 1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated,
                         (const uint8_t*)nullptr);
    OFX_LAUNCH_CHECK();
    return OFX_OK;
  }
  OFX_TIMED_LAUNCH(timer, desc->semantics == OFX_SEM_PYCUDA ? (k_integrate<true, true, true>) : (k_integrate<true, true, false>),
                     dim3((unsigned)n_list), dim3(256), 0, as_stream(s), g, make_cam(cam),
                     depth, color_im, (const float4*)packed_nodes, k, brick_list, (const ushort4*)anchors,
                     (const float4*)weights, pal_ids, pal_n, (const uchar4*)local_anchors, desc->trunc_margin,
                     obs_weight, tsdf, weight, color, n_updated);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_integrate_palette_cull(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth,
                               const float* color_im, const float* packed_nodes, int32_t n_nodes, int32_t k,
                               const int32_t* brick_list, int32_t n_list, const uint16_t* anchors, const float* weights,
                               const uint16_t* pal_ids, const int32_t* pal_n, const uint8_t* local_anchors,
                               double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                               float* tile_scratch, uint8_t* active, ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(cam && depth, "null camera/depth");
  OFX_CHECK_ARG(cam->width > 0 && cam->height > 0, "bad camera size");
  const bool fast = desc->semantics == OFX_SEM_CPU && k == 4 && g.n_bricks * kBrickVox < (1ll << 31) &&
                    !getenv("OFX_INT_GENERIC");
  if (!fast || !tile_scratch || !active)   // the cull serves the CPU-semantics K = 4 palette kernel only
    return ofx_integrate_palette(desc, cam, depth, color_im, packed_nodes, n_nodes, k, brick_list, n_list, anchors,
                                 weights, pal_ids, pal_n, local_anchors, obs_weight, tsdf, weight, color, n_updated, s);
  OFX_CHECK_ARG((color == nullptr) == (color_im == nullptr), "color and color_im must both be set or both NULL");
  OFX_CHECK_ARG(n_nodes >= k, "bad k/n_nodes");
  OFX_CHECK_ARG(n_list >= 0 && n_list <= g.n_bricks, "bad n_list");
  if (n_list == 0) return OFX_OK;
  OFX_CHECK_ARG(packed_nodes && brick_list && anchors && weights && pal_ids && pal_n && local_anchors,
                "null warp/palette buffer");
  hipStream_t hs = as_stream(s);
  const CamD c = make_cam(cam);
  const BrickDiv bd = make_div(g);
  const int TW = (cam->width + 7) / 8, TH = (cam->height + 7) / 8;
  IntTimer timer;   // one event pair around the three kernels (tile max, cull, integrate)
  if (timer.e0)
    hipExtLaunchKernelGGL(k_tile_max, dim3(grid_for((int64_t)TW * TH, 256)), dim3(256), 0, hs, timer.e0, nullptr, 0,
                          depth, cam->width, cam->height, TW, TH, tile_scratch);
  else
    hipLaunchKernelGGL(k_tile_max, dim3(grid_for((int64_t)TW * TH, 256)), dim3(256), 0, hs, depth, cam->width,
                       cam->height, TW, TH, tile_scratch);
  hipLaunchKernelGGL(k_brick_cull, dim3((unsigned)((n_list + 15) / 16)), dim3(256), 0, hs, g, bd, c,
                     (const float4*)packed_nodes, n_nodes, brick_list, pal_ids, pal_n, n_list,
                     (const float*)tile_scratch, TW, TH, desc->trunc_margin, active);
  auto launch = [&](auto kern) {
    if (timer.e0)
      hipExtLaunchKernelGGL(kern, dim3((unsigned)n_list), dim3(256), 0, hs, nullptr, timer.e1, 0, g, bd, c, depth,
                            color_im, (const float4*)packed_nodes, n_nodes, brick_list, (const ushort4*)anchors,
                            (const float4*)weights, pal_ids, pal_n, (const uchar4*)local_anchors, desc->trunc_margin,
                            1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated,
                            (const uint8_t*)active);
    else
      hipLaunchKernelGGL(kern, dim3((unsigned)n_list), dim3(256), 0, hs, g, bd, c, depth, color_im,
                         (const float4*)packed_nodes, n_nodes, brick_list, (const ushort4*)anchors,
                         (const float4*)weights, pal_ids, pal_n, (const uchar4*)local_anchors, desc->trunc_margin,
                         1.0 / desc->trunc_margin, obs_weight, tsdf, weight, color, n_updated, (const uint8_t*)active);
  };
  if (color) launch(k_integrate_pal4<true>);
  else launch(k_integrate_pal4<false>);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_integrate_points(const ofx_volume_desc* desc, const ofx_camera* cam, const float* depth, const float* color_im,
                         const float* points, const int64_t* voxel_ids, const uint8_t* valid, int64_t n_points,
                         double obs_weight, float* tsdf, float* weight, float* color, uint32_t* n_updated,
                         ofx_stream_t s) {
  BrickGeom g;
  int st = make_geom(desc, &g);
  if (st) return st;
  OFX_CHECK_ARG(cam && depth && tsdf && weight && n_points >= 0, "null buffer / bad size");
  OFX_CHECK_ARG(cam->width > 0 && cam->height > 0, "bad camera size");
  OFX_CHECK_ARG((color == nullptr) == (color_im == nullptr), "color and color_im must both be set or both NULL");
  OFX_CHECK_ARG(desc->semantics == OFX_SEM_CPU || desc->semantics == OFX_SEM_PYCUDA, "bad semantics %d", desc->semantics);
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && voxel_ids, "null points / voxel ids");
  hipLaunchKernelGGL(desc->semantics == OFX_SEM_PYCUDA ? (k_integrate_points<true>) : (k_integrate_points<false>),
                     dim3(grid_for(n_points, 256, 1 << 30)), dim3(256), 0, as_stream(s), g, make_cam(cam), depth,
                     color_im, points, voxel_ids, valid, n_points, desc->trunc_margin, 1.0 / desc->trunc_margin,
                     obs_weight, tsdf, weight, color, n_updated);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_deform_points(const float* points, int64_t n_points, const int32_t* anchors, const float* weights,
                      const uint8_t* valid, int32_t k, const float* packed_nodes, int32_t n_nodes, int32_t normals,
                      float* out, ofx_stream_t s) {
  OFX_CHECK_ARG(n_points >= 0 && k >= 1 && k <= 4 && n_nodes >= k, "bad sizes");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && anchors && weights && packed_nodes && out, "null buffer");
  hipLaunchKernelGGL(k_deform_points, dim3(grid_for(n_points, 256, 1 << 30)), dim3(256), 0, as_stream(s), points,
                     n_points, anchors, weights, valid, k, (const float4*)packed_nodes, normals, out);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_deform_points_lbs(const float* points, int64_t n_points, const int32_t* anchors, const float* weights,
                          const uint8_t* valid, int32_t k, const float* rotations, const float* translations,
                          int32_t n_nodes, float* out, ofx_stream_t s) {
  OFX_CHECK_ARG(n_points >= 0 && k >= 1 && k <= 4 && n_nodes >= 1, "bad sizes");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && anchors && weights && rotations && translations && out, "null buffer");
  hipLaunchKernelGGL(k_deform_lbs, dim3(grid_for(n_points, 256, 1 << 30)), dim3(256), 0, as_stream(s), points,
                     n_points, anchors, weights, valid, k, rotations, translations, out);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_visibility(const float* points, int64_t n_points, const ofx_camera* cam, const float* depth,
                   double trunc_margin, uint8_t* valid, double* depth_diff, ofx_stream_t s) {
  OFX_CHECK_ARG(cam && n_points >= 0, "bad args");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && depth && valid, "null buffer");
  hipLaunchKernelGGL(k_visibility<false>, dim3(grid_for(n_points, 256, 1 << 30)), dim3(256), 0, as_stream(s), points,
                     n_points, make_cam(cam), depth, trunc_margin, valid, depth_diff);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_visibility_f32(const float* points, int64_t n_points, const ofx_camera* cam, const float* depth,
                       double trunc_margin, uint8_t* valid, double* depth_diff, ofx_stream_t s) {
  OFX_CHECK_ARG(cam && n_points >= 0, "bad args");
  if (n_points == 0) return OFX_OK;
  OFX_CHECK_ARG(points && depth && valid, "null buffer");
  hipLaunchKernelGGL(k_visibility<true>, dim3(grid_for(n_points, 256, 1 << 30)), dim3(256), 0, as_stream(s), points,
                     n_points, make_cam(cam), depth, trunc_margin, valid, depth_diff);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

}  // extern "C"
