// Gauss-Newton non-rigid registration solver: block-sparse JᵀJ / Jᵀr assembly + block-Jacobi PCG.
//
// Restates DeformNet.optimize (model/model.py:222-859) for one batch item:
//   unknowns per node i: [ω_i (3) | t_i (3)]  (reference orders all rotations, then all translations;
//                                              the dense oracle maps between the two orders)
//   data rows (3 per match, model.py:416-545): p = Σ_k w_k (R_k(x-g_k)+g_k+t_k)
//       r  = [lf(fx·px/z+cx-tpx) + ld(px-tx), lf(fy·py/z+cy-tpy) + ld(py-ty), ld(pz-tz)]
//       ∂/∂t_k = w_k·[[lf·fx/z+ld, 0, lf·(-fx·px/z²)], [0, lf·fy/z+ld, lf·(-fy·py/z²)], [0,0,ld]]
//       ∂/∂ω_k = S + [[-fx·px/z²·S₂ ], [-fy·py/z²·S₂], [0]] + lf·[[fx/z·S₀],[fy/z·S₁],[0]],  S = -[w_k R_k(x-g_k)]×
//       (the un-weighted -f·p/z² terms reproduce the operator-precedence quirk at model.py:505-510)
//   ARAP rows (3 per directed edge, model.py:554-601): r = la·w(R_i(g_j-g_i)+g_i+t_i-g_j-t_j)
//   motion rows (3 per node, model.py:604-612):       r = lm·c_i(t_i+g_i-target_i)
//   A = JᵀJ + λ_LM·I, b = -Jᵀr, λ_LM halved at gn_i ≡ 2 mod 3 (model.py:418-419, 641-662)
//   x = A⁻¹b (reference: dense LU, model.py:59-86,694-709 -> here: f64 block-Jacobi PCG)
//   early stop on loss increase > stop_diff or unchanged loss (model.py:726-732), then
//   R ← exp([x_ω]) R (kornia 0.7 angle_axis_to_rotation_matrix), t += x_t (model.py:744-748).
//
// MI355X design: JᵀJ is stored as 6x6 f64 blocks in BSR over the node adjacency (diagonal, graph
// edges, co-anchored node pairs) with a dense NxN slot map for O(1) scatter; one thread per
// (match, anchor) builds its 3x6 Jacobian and scatters J_kᵀJ_l blocks with native f64 atomics.
// PCG = 2 kernels per iteration (fused p-update+SpMV+dot, fused axpy+precondition+dots), each ending
// in a last-workgroup reduction of per-workgroup partials in fixed order (deterministic scalars),
// agent-scope release/acquire hand-off per CDNA4 G16.
#include <math.h>
#include <vector>

#include "ofx_common.h"

namespace ofx {

// --------------------------------------------------------------------------------------------
struct Gn {
  int max_nodes = 0, max_matches = 0;
  int N = 0, M = 0, NB = 0;
  ofx_gn_params prm{};
  float fx = 0, fy = 0, cx = 0, cy = 0;
  // problem (f64 device copies)
  double *nodes = nullptr, *tpos = nullptr, *conf = nullptr, *src = nullptr, *wts = nullptr, *tgt = nullptr,
         *tpx = nullptr, *tpy = nullptr, *ew = nullptr;
  int32_t *anc = nullptr, *edges = nullptr;
  // pattern
  int32_t *map = nullptr, *row_ptr = nullptr, *col = nullptr, *row_cnt = nullptr;
  int64_t nnzb = 0, nnzb_cap = 0;
  // state
  double *R = nullptr, *t = nullptr;
  double *A_own = nullptr, *rhs_own = nullptr;
  double *Dinv = nullptr, *x = nullptr, *r = nullptr, *z = nullptr, *p0 = nullptr, *p1 = nullptr, *q = nullptr;
  double* part = nullptr;   // per-WG partials, 4 per WG
  double* scal = nullptr;   // [alpha, beta, rz, bb, rr, pq, loss_prev, ...]
  int32_t* flags = nullptr; // see F_* below
  uint32_t* tickets = nullptr;
  double* loss_log = nullptr;
  int32_t* host_flag = nullptr;  // pinned
  bool setup_done = false;
};

enum { F_DONE = 0, F_STOPPED = 1, F_ILL = 2, F_ACCEPTED = 3, F_PCG_TOTAL = 4, F_APPLY = 5, F_RES_NONFINITE = 6,
       F_PCG_IT = 7, F_COUNT = 8 };
enum { S_ALPHA = 0, S_BETA = 1, S_RZ = 2, S_BB = 3, S_RR = 4, S_PQ = 5, S_LOSS_PREV = 6, S_COUNT = 8 };
constexpr int kPcgBlock = 256;  // threads per WG in node-parallel PCG kernels (4 rows per WG in SpMV)

// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void atomic_add_f64(double* p, double v) { unsafeAtomicAdd(p, v); }

__global__ void k_to_f64(const float* __restrict__ s, double* __restrict__ d, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) d[i] = s ? (double)s[i] : 0.0;
}

__global__ void k_edge_weights(const float* __restrict__ ew, int64_t n, int use, int nb, double* __restrict__ out) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = (use && ew) ? (double)nb * (double)ew[i] : 1.0;
}

__global__ void k_init_state(const float* __restrict__ prev_R, const float* __restrict__ prev_t, int N,
                             double* __restrict__ R, double* __restrict__ t) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  for (int c = 0; c < 9; ++c) R[9 * i + c] = prev_R ? (double)prev_R[9 * i + c] : ((c % 4 == 0) ? 1.0 : 0.0);
  for (int c = 0; c < 3; ++c) t[3 * i + c] = prev_t ? (double)prev_t[3 * i + c] : 0.0;
}

// ---- pattern build ----
__global__ void k_mark(int N, int M, int NB, const int32_t* __restrict__ anc, const int32_t* __restrict__ edges,
                       int32_t* __restrict__ map) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t n_match_pairs = (int64_t)M * 16;
  int64_t n_edge = (int64_t)N * NB;
  if (t < N) map[t * N + t] = 1;
  if (t < n_match_pairs) {
    int64_t m = t / 16;
    int k = (t / 4) % 4, l = t % 4;
    int a = anc[m * 4 + k], b = anc[m * 4 + l];
    map[(int64_t)a * N + b] = 1;
  }
  if (t < n_edge) {
    int i = (int)(t / NB);
    int j = edges[t];
    if (j >= 0) {
      map[(int64_t)i * N + j] = 1;
      map[(int64_t)j * N + i] = 1;
    }
  }
}

// per row: count marks (one WG per row)
__global__ __launch_bounds__(256) void k_row_count(int N, const int32_t* __restrict__ map, int32_t* __restrict__ cnt) {
  __shared__ int s[256];
  int i = blockIdx.x;
  int c = 0;
  for (int j = threadIdx.x; j < N; j += blockDim.x) c += map[(int64_t)i * N + j] != 0;
  s[threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) cnt[i] = s[0];
}

__global__ __launch_bounds__(1024) void k_scan_rows(int N, const int32_t* __restrict__ cnt, int32_t* __restrict__ row_ptr) {
  __shared__ int64_t part[1024];
  int per = (N + blockDim.x - 1) / blockDim.x;
  int s = threadIdx.x * per, e = min(N, s + per);
  int64_t c = 0;
  for (int i = s; i < e; ++i) c += cnt[i];
  part[threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) { int64_t v = part[i]; part[i] = acc; acc += v; }
    row_ptr[N] = (int32_t)acc;
  }
  __syncthreads();
  int64_t o = part[threadIdx.x];
  for (int i = s; i < e; ++i) { row_ptr[i] = (int32_t)o; o += cnt[i]; }
}

// per row: ordered assignment of slots (one WG per row, chunked block prefix)
__global__ __launch_bounds__(256) void k_row_assign(int N, int32_t* __restrict__ map, const int32_t* __restrict__ row_ptr,
                                                    int32_t* __restrict__ col) {
  __shared__ int s[256];
  __shared__ int base;
  int i = blockIdx.x;
  if (threadIdx.x == 0) base = row_ptr[i];
  __syncthreads();
  for (int j0 = 0; j0 < N; j0 += blockDim.x) {
    int j = j0 + threadIdx.x;
    int f = (j < N) ? (map[(int64_t)i * N + j] != 0) : 0;
    s[threadIdx.x] = f;
    __syncthreads();
    // inclusive scan (Hillis-Steele)
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {
      int v = (threadIdx.x >= (unsigned)o) ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += v;
      __syncthreads();
    }
    int incl = s[threadIdx.x];
    int b0 = base;
    if (f) {
      int slot = b0 + incl - 1;
      col[slot] = j;
      map[(int64_t)i * N + j] = slot;
    } else if (j < N) {
      map[(int64_t)i * N + j] = -1;
    }
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) base = b0 + incl;
    __syncthreads();
  }
}

// ---- assembly ----
// add J_aᵀ J_b (J: 3x6 row-major) into block
__device__ __forceinline__ void add_block(double* __restrict__ blk, const double* Ja, const double* Jb) {
#pragma unroll
  for (int c = 0; c < 6; ++c)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double v = Ja[c] * Jb[j] + Ja[6 + c] * Jb[6 + j] + Ja[12 + c] * Jb[12 + j];
      if (v != 0.0) atomic_add_f64(blk + c * 6 + j, v);
    }
}

__device__ __forceinline__ void add_rhs(double* __restrict__ rhs6, const double* Ja, const double r[3]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    double v = Ja[c] * r[0] + Ja[6 + c] * r[1] + Ja[12 + c] * r[2];
    if (v != 0.0) atomic_add_f64(rhs6 + c, -v);
  }
}

struct DataCoef {
  double lf, ld, fx, fy, cx, cy;
};

__device__ void data_jacobian(const Gn& g, const DataCoef& dc, int64_t m, int k, const double p[3], double zinv,
                              double J[18]) {
  int a = g.anc[m * 4 + k];
  double w = g.wts[m * 4 + k];
  const double* R = g.R + 9 * (int64_t)a;
  const double* gn = g.nodes + 3 * (int64_t)a;
  double d0 = g.src[3 * m] - gn[0], d1 = g.src[3 * m + 1] - gn[1], d2 = g.src[3 * m + 2] - gn[2];
  double v0 = w * (R[0] * d0 + R[1] * d1 + R[2] * d2);
  double v1 = w * (R[3] * d0 + R[4] * d1 + R[5] * d2);
  double v2 = w * (R[6] * d0 + R[7] * d1 + R[8] * d2);
  // S = -[v]x
  double S[9] = {0.0, v2, -v1, -v2, 0.0, v0, v1, -v0, 0.0};
  double fxdz = dc.fx * zinv, fydz = dc.fy * zinv;
  double mfx = -(dc.fx * p[0] * zinv) * zinv;
  double mfy = -(dc.fy * p[1] * zinv) * zinv;
  for (int j = 0; j < 3; ++j) {
    J[0 + j] = dc.lf * fxdz * S[0 + j] + mfx * S[6 + j] + dc.ld * S[0 + j];
    J[6 + j] = dc.lf * fydz * S[3 + j] + mfy * S[6 + j] + dc.ld * S[3 + j];
    J[12 + j] = dc.ld * S[6 + j];
  }
  J[3] = dc.lf * w * fxdz + dc.ld * w; J[4] = 0.0; J[5] = dc.lf * w * mfx;
  J[9] = 0.0; J[10] = dc.lf * w * fydz + dc.ld * w; J[11] = dc.lf * w * mfy;
  J[15] = 0.0; J[16] = 0.0; J[17] = dc.ld * w;
}

__device__ void deformed_point(const Gn& g, int64_t m, double p[3]) {
  p[0] = p[1] = p[2] = 0.0;
  for (int k = 0; k < 4; ++k) {
    int a = g.anc[m * 4 + k];
    double w = g.wts[m * 4 + k];
    const double* R = g.R + 9 * (int64_t)a;
    const double* gn = g.nodes + 3 * (int64_t)a;
    const double* tt = g.t + 3 * (int64_t)a;
    double d0 = g.src[3 * m] - gn[0], d1 = g.src[3 * m + 1] - gn[1], d2 = g.src[3 * m + 2] - gn[2];
    p[0] += w * ((R[0] * d0 + R[1] * d1 + R[2] * d2) + gn[0] + tt[0]);
    p[1] += w * ((R[3] * d0 + R[4] * d1 + R[5] * d2) + gn[1] + tt[1]);
    p[2] += w * ((R[6] * d0 + R[7] * d1 + R[8] * d2) + gn[2] + tt[2]);
  }
}

__global__ __launch_bounds__(256) void k_data(Gn g, DataCoef dc, int m0, int m1, double* __restrict__ A,
                                              double* __restrict__ rhs) {
  int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t m = m0 + tid / 4;
  int k = (int)(tid % 4);
  if (m >= m1) return;
  double p[3];
  deformed_point(g, m, p);
  double zinv = 1.0 / (p[2] + 1e-7);
  double r[3];
  double tpx = g.tpx ? g.tpx[m] : 0.0, tpy = g.tpy ? g.tpy[m] : 0.0;
  r[0] = dc.lf * (dc.fx * p[0] * zinv + dc.cx - tpx) + dc.ld * (p[0] - g.tgt[3 * m]);
  r[1] = dc.lf * (dc.fy * p[1] * zinv + dc.cy - tpy) + dc.ld * (p[1] - g.tgt[3 * m + 1]);
  r[2] = dc.ld * (p[2] - g.tgt[3 * m + 2]);
  double Jk[18], Jl[18];
  data_jacobian(g, dc, m, k, p, zinv, Jk);
  int a = g.anc[m * 4 + k];
  for (int l = 0; l < 4; ++l) {
    int b = g.anc[m * 4 + l];
    if (l == k) {
      add_block(A + 36 * (int64_t)g.map[(int64_t)a * g.N + a], Jk, Jk);
    } else {
      data_jacobian(g, dc, m, l, p, zinv, Jl);
      add_block(A + 36 * (int64_t)g.map[(int64_t)a * g.N + b], Jk, Jl);
    }
  }
  add_rhs(rhs + 6 * (int64_t)a, Jk, r);
  if (k == 0) {
    double l2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    double* tail = rhs + 6 * (int64_t)g.N;
    atomic_add_f64(tail + 0, l2);
    if (!isfinite(l2)) atomic_add_f64(tail + 3, 1.0);
  }
}

__global__ __launch_bounds__(256) void k_arap(Gn g, double la, double* __restrict__ A, double* __restrict__ rhs) {
  int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= (int64_t)g.N * g.NB) return;
  int j = g.edges[e];
  if (j < 0) return;
  int i = (int)(e / g.NB);
  double w = g.ew[e];
  const double* R = g.R + 9 * (int64_t)i;
  const double* gi = g.nodes + 3 * (int64_t)i;
  const double* gj = g.nodes + 3 * (int64_t)j;
  const double* ti = g.t + 3 * (int64_t)i;
  const double* tj = g.t + 3 * (int64_t)j;
  double e0 = gj[0] - gi[0], e1 = gj[1] - gi[1], e2 = gj[2] - gi[2];
  double d0 = R[0] * e0 + R[1] * e1 + R[2] * e2;
  double d1 = R[3] * e0 + R[4] * e1 + R[5] * e2;
  double d2 = R[6] * e0 + R[7] * e1 + R[8] * e2;
  double s = la * w;
  double r[3] = {s * (d0 + gi[0] + ti[0] - (gj[0] + tj[0])), s * (d1 + gi[1] + ti[1] - (gj[1] + tj[1])),
                 s * (d2 + gi[2] + ti[2] - (gj[2] + tj[2]))};
  // Srot = -s [d]x
  double Ji[18] = {0.0, s * d2, -s * d1, s, 0, 0,
                   -s * d2, 0.0, s * d0, 0, s, 0,
                   s * d1, -s * d0, 0.0, 0, 0, s};
  double Jj[18] = {0, 0, 0, -s, 0, 0,
                   0, 0, 0, 0, -s, 0,
                   0, 0, 0, 0, 0, -s};
  int64_t N = g.N;
  add_block(A + 36 * (int64_t)g.map[i * N + i], Ji, Ji);
  add_block(A + 36 * (int64_t)g.map[i * N + j], Ji, Jj);
  add_block(A + 36 * (int64_t)g.map[j * N + i], Jj, Ji);
  add_block(A + 36 * (int64_t)g.map[j * N + j], Jj, Jj);
  add_rhs(rhs + 6 * (int64_t)i, Ji, r);
  add_rhs(rhs + 6 * (int64_t)j, Jj, r);
  double l2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
  double* tail = rhs + 6 * N;
  atomic_add_f64(tail + 1, l2);
  if (!isfinite(l2)) atomic_add_f64(tail + 3, 1.0);
}

__global__ __launch_bounds__(256) void k_motion(Gn g, double lm, double* __restrict__ A, double* __restrict__ rhs) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.N) return;
  double c = lm * g.conf[i];
  double r[3];
  for (int q = 0; q < 3; ++q) r[q] = c * (g.t[3 * i + q] + g.nodes[3 * i + q] - g.tpos[3 * i + q]);
  double* blk = A + 36 * (int64_t)g.map[(int64_t)i * g.N + i];
  double cc = c * c;
  if (cc != 0.0)
    for (int q = 0; q < 3; ++q) atomic_add_f64(blk + (3 + q) * 6 + (3 + q), cc);
  for (int q = 0; q < 3; ++q)
    if (c * r[q] != 0.0) atomic_add_f64(rhs + 6 * (int64_t)i + 3 + q, -c * r[q]);
  double l2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
  double* tail = rhs + 6 * (int64_t)g.N;
  atomic_add_f64(tail + 2, l2);
  if (!isfinite(l2)) atomic_add_f64(tail + 3, 1.0);
}

// ---- last-workgroup deterministic reduction (agent-scope release/acquire, CDNA4 G16) ----
// Each WG writes `nv` partials to part[wg*4 + v]; returns true in exactly one WG (the last arriver),
// whose threads may then read every partial.
__device__ __forceinline__ bool last_wg_arrive(uint32_t* ticket, int nwg) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == (uint32_t)(nwg - 1));
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      *ticket = 0;  // reset for the next launch (kernel boundary orders it)
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// sum partial v over nwg workgroups in fixed order (all threads of the last WG get the result)
__device__ double fixed_order_sum(const double* part, int nwg, int v) {
  __shared__ double s[kPcgBlock];
  double acc = 0.0;
  // thread t sums a contiguous slice, then a fixed-shape tree: deterministic
  int per = (nwg + blockDim.x - 1) / blockDim.x;
  int b = threadIdx.x * per, e = min(nwg, b + per);
  for (int w = b; w < e; ++w) acc += part[4 * w + v];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < (unsigned)o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  double r = s[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ double block_sum(double v) {
  __shared__ double s[kPcgBlock];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < (unsigned)o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  double r = s[0];
  __syncthreads();
  return r;
}

// ---- PCG ----
// prepare: LM damping on the diagonal, block-Jacobi inverse, x=0, r=b, z=D⁻¹r, p(old)=0, beta=0,
// partials rz & bb.   thread per node.
__global__ __launch_bounds__(kPcgBlock) void k_pcg_prep(Gn g, double lm, double* __restrict__ A,
                                                         const double* __restrict__ rhs) {
  if (g.flags[F_STOPPED]) return;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  double rz = 0.0, bb = 0.0;
  if (i < g.N) {
    double* blk = A + 36 * (int64_t)g.map[(int64_t)i * g.N + i];
    double a[36], inv[36];
    for (int c = 0; c < 6; ++c) blk[c * 7] += lm;
    for (int c = 0; c < 36; ++c) { a[c] = blk[c]; inv[c] = (c % 7 == 0) ? 1.0 : 0.0; }
    // Gauss-Jordan with partial pivoting
    bool ok = true;
    for (int c = 0; c < 6; ++c) {
      int piv = c;
      double best = fabs(a[c * 6 + c]);
      for (int rr = c + 1; rr < 6; ++rr)
        if (fabs(a[rr * 6 + c]) > best) { best = fabs(a[rr * 6 + c]); piv = rr; }
      if (!(best > 0.0)) { ok = false; break; }
      if (piv != c)
        for (int q = 0; q < 6; ++q) {
          double t0 = a[c * 6 + q]; a[c * 6 + q] = a[piv * 6 + q]; a[piv * 6 + q] = t0;
          double t1 = inv[c * 6 + q]; inv[c * 6 + q] = inv[piv * 6 + q]; inv[piv * 6 + q] = t1;
        }
      double d = 1.0 / a[c * 6 + c];
      for (int q = 0; q < 6; ++q) { a[c * 6 + q] *= d; inv[c * 6 + q] *= d; }
      for (int rr = 0; rr < 6; ++rr)
        if (rr != c) {
          double f = a[rr * 6 + c];
          if (f != 0.0)
            for (int q = 0; q < 6; ++q) { a[rr * 6 + q] -= f * a[c * 6 + q]; inv[rr * 6 + q] -= f * inv[c * 6 + q]; }
        }
    }
    if (!ok)
      for (int c = 0; c < 36; ++c) inv[c] = (c % 7 == 0) ? 1.0 : 0.0;
    double* D = g.Dinv + 36 * (int64_t)i;
    for (int c = 0; c < 36; ++c) D[c] = inv[c];
    double rv[6];
    for (int c = 0; c < 6; ++c) {
      rv[c] = rhs[6 * i + c];
      g.x[6 * i + c] = 0.0;
      g.r[6 * i + c] = rv[c];
      g.p0[6 * i + c] = 0.0;
      g.p1[6 * i + c] = 0.0;
      bb += rv[c] * rv[c];
    }
    for (int c = 0; c < 6; ++c) {
      double zc = 0.0;
      for (int q = 0; q < 6; ++q) zc += inv[c * 6 + q] * rv[q];
      g.z[6 * i + c] = zc;
      rz += rv[c] * zc;
    }
  }
  double s_rz = block_sum(rz);
  double s_bb = block_sum(bb);
  int nwg = gridDim.x;
  if (threadIdx.x == 0) { g.part[4 * blockIdx.x + 0] = s_rz; g.part[4 * blockIdx.x + 1] = s_bb; }
  if (last_wg_arrive(g.tickets + 0, nwg)) {
    double trz = fixed_order_sum(g.part, nwg, 0);
    double tbb = fixed_order_sum(g.part, nwg, 1);
    if (threadIdx.x == 0) {
      g.scal[S_RZ] = trz;
      g.scal[S_BB] = tbb;
      g.scal[S_BETA] = 0.0;
      g.flags[F_DONE] = (tbb == 0.0 || !isfinite(tbb)) ? 1 : 0;
      if (!isfinite(tbb)) g.flags[F_ILL] = 1;
      g.flags[F_PCG_IT] = 0;
    }
  }
}

// K1: p_new = z + beta*p_old (on the fly for every column), q = A p_new, partial p·q; last WG: alpha.
// one wave per block row; lanes stride over the row's blocks.
__global__ __launch_bounds__(kPcgBlock) void k_pcg_spmv(Gn g, const double* __restrict__ A, int parity) {
  if (g.flags[F_DONE] || g.flags[F_STOPPED]) return;
  const double* __restrict__ pold = parity ? g.p0 : g.p1;
  double* __restrict__ pnew = parity ? g.p1 : g.p0;
  const double beta = g.scal[S_BETA];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (kPcgBlock / 64) + (threadIdx.x >> 6);
  double pq = 0.0;
  if (row < g.N) {
    double acc[6] = {0, 0, 0, 0, 0, 0};
    int b0 = g.row_ptr[row], b1 = g.row_ptr[row + 1];
    for (int bi = b0 + lane; bi < b1; bi += 64) {
      int c = g.col[bi];
      double pv[6];
      for (int j = 0; j < 6; ++j) pv[j] = g.z[6 * c + j] + beta * pold[6 * c + j];
      const double* blk = A + 36 * (int64_t)bi;
      for (int rr = 0; rr < 6; ++rr) {
        double s = 0.0;
        for (int j = 0; j < 6; ++j) s += blk[rr * 6 + j] * pv[j];
        acc[rr] += s;
      }
    }
    for (int rr = 0; rr < 6; ++rr)
      for (int off = 32; off > 0; off >>= 1) acc[rr] += __shfl_xor(acc[rr], off, 64);
    if (lane < 6) {
      double mine = acc[0];
      for (int rr = 1; rr < 6; ++rr) if (lane == rr) mine = acc[rr];
      double pn = g.z[6 * row + lane] + beta * pold[6 * row + lane];
      pnew[6 * row + lane] = pn;
      g.q[6 * row + lane] = mine;
      pq = pn * mine;
    }
  }
  double s = block_sum(pq);
  int nwg = gridDim.x;
  if (threadIdx.x == 0) g.part[4 * blockIdx.x + 0] = s;
  if (last_wg_arrive(g.tickets + 1, nwg)) {
    double tpq = fixed_order_sum(g.part, nwg, 0);
    if (threadIdx.x == 0) {
      g.scal[S_PQ] = tpq;
      double rz = g.scal[S_RZ];
      if (!(tpq > 0.0) || !isfinite(tpq)) {
        g.flags[F_DONE] = 1;  // breakdown: keep current x
        g.scal[S_ALPHA] = 0.0;
        if (!isfinite(tpq)) g.flags[F_ILL] = 1;
      } else {
        g.scal[S_ALPHA] = rz / tpq;
      }
    }
  }
}

// K2: x += a p, r -= a q, z = D⁻¹ r, partial r·z, r·r; last WG: beta, convergence.  thread per node.
__global__ __launch_bounds__(kPcgBlock) void k_pcg_update(Gn g, int parity) {
  if (g.flags[F_DONE] || g.flags[F_STOPPED]) return;
  const double* __restrict__ p = parity ? g.p1 : g.p0;
  const double alpha = g.scal[S_ALPHA];
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  double rz = 0.0, rr = 0.0;
  if (i < g.N) {
    double rv[6];
    for (int c = 0; c < 6; ++c) {
      g.x[6 * i + c] += alpha * p[6 * i + c];
      rv[c] = g.r[6 * i + c] - alpha * g.q[6 * i + c];
      g.r[6 * i + c] = rv[c];
      rr += rv[c] * rv[c];
    }
    const double* D = g.Dinv + 36 * (int64_t)i;
    for (int c = 0; c < 6; ++c) {
      double zc = 0.0;
      for (int q = 0; q < 6; ++q) zc += D[c * 6 + q] * rv[q];
      g.z[6 * i + c] = zc;
      rz += rv[c] * zc;
    }
  }
  double s_rz = block_sum(rz);
  double s_rr = block_sum(rr);
  int nwg = gridDim.x;
  if (threadIdx.x == 0) { g.part[4 * blockIdx.x + 0] = s_rz; g.part[4 * blockIdx.x + 1] = s_rr; }
  if (last_wg_arrive(g.tickets + 2, nwg)) {
    double trz = fixed_order_sum(g.part, nwg, 0);
    double trr = fixed_order_sum(g.part, nwg, 1);
    if (threadIdx.x == 0) {
      double old = g.scal[S_RZ];
      g.scal[S_BETA] = (old != 0.0) ? trz / old : 0.0;
      g.scal[S_RZ] = trz;
      g.scal[S_RR] = trr;
      g.flags[F_PCG_IT] += 1;
      g.flags[F_PCG_TOTAL] += 1;
      double tol = g.prm.pcg_tol;
      if (!isfinite(trr)) { g.flags[F_ILL] = 1; g.flags[F_DONE] = 1; }
      else if (trr <= tol * tol * g.scal[S_BB] || trz == 0.0) g.flags[F_DONE] = 1;
    }
  }
}

// After the solve: ill-posed check, loss bookkeeping and early stop (model.py:696-732). Single WG.
__global__ __launch_bounds__(kPcgBlock) void k_step_decide(Gn g, const double* __restrict__ rhs, int n_iter_log) {
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  if (g.flags[F_STOPPED]) return;
  int bad = 0;
  for (int i = threadIdx.x; i < 6 * g.N; i += blockDim.x) bad |= !isfinite(g.x[i]);
  if (bad) atomicOr(&s_bad, 1);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double* tail = rhs + 6 * (int64_t)g.N;
  g.flags[F_RES_NONFINITE] = tail[3] != 0.0 ? 1 : 0;
  g.flags[F_APPLY] = 0;
  if (s_bad || g.flags[F_ILL]) {
    g.flags[F_ILL] = 1;
    g.flags[F_STOPPED] = 1;
    return;
  }
  double loss = sqrt(tail[0] + tail[1] + tail[2]);
  int acc = g.flags[F_ACCEPTED];
  if (acc > 0) {
    double prev = g.scal[S_LOSS_PREV];
    if (loss - prev > g.prm.stop_loss_diff || loss == prev) {
      g.flags[F_STOPPED] = 1;
      return;
    }
  }
  if (acc < n_iter_log) {
    g.loss_log[4 * acc + 0] = loss;
    g.loss_log[4 * acc + 1] = sqrt(tail[0]);
    g.loss_log[4 * acc + 2] = sqrt(tail[1]);
    g.loss_log[4 * acc + 3] = sqrt(tail[2]);
  }
  g.scal[S_LOSS_PREV] = loss;
  g.flags[F_ACCEPTED] = acc + 1;
  g.flags[F_APPLY] = 1;
}

// kornia 0.7.0 angle_axis_to_rotation_matrix + left-multiplicative update (model.py:744-748).
__global__ void k_apply(Gn g) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.N || !g.flags[F_APPLY] || g.flags[F_STOPPED]) return;
  double a0 = g.x[6 * i], a1 = g.x[6 * i + 1], a2 = g.x[6 * i + 2];
  double th2 = a0 * a0 + a1 * a1 + a2 * a2;
  double Ri[9];
  if (th2 > 1e-6) {
    double th = sqrt(th2);
    double wx = a0 / (th + 1e-6), wy = a1 / (th + 1e-6), wz = a2 / (th + 1e-6);
    double c = cos(th), s = sin(th), oc = 1.0 - c;
    Ri[0] = c + wx * wx * oc; Ri[1] = wx * wy * oc - wz * s; Ri[2] = wy * s + wx * wz * oc;
    Ri[3] = wz * s + wx * wy * oc; Ri[4] = c + wy * wy * oc; Ri[5] = -wx * s + wy * wz * oc;
    Ri[6] = -wy * s + wx * wz * oc; Ri[7] = wx * s + wy * wz * oc; Ri[8] = c + wz * wz * oc;
  } else {
    Ri[0] = 1; Ri[1] = -a2; Ri[2] = a1; Ri[3] = a2; Ri[4] = 1; Ri[5] = -a0; Ri[6] = -a1; Ri[7] = a0; Ri[8] = 1;
  }
  double* R = g.R + 9 * (int64_t)i;
  double Rn[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Rn[3 * r + c] = Ri[3 * r] * R[c] + Ri[3 * r + 1] * R[3 + c] + Ri[3 * r + 2] * R[6 + c];
  for (int c = 0; c < 9; ++c) R[c] = Rn[c];
  for (int c = 0; c < 3; ++c) g.t[3 * i + c] += g.x[6 * i + 3 + c];
}

__global__ void k_finish(Gn g, float* __restrict__ rot, float* __restrict__ trans, int32_t* __restrict__ status,
                         double* __restrict__ loss_out, int n_log) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = !g.flags[F_ILL] && !g.flags[F_RES_NONFINITE];
  if (i < g.N) {
    for (int c = 0; c < 9; ++c) rot[9 * i + c] = valid ? (float)g.R[9 * i + c] : ((c % 4 == 0) ? 1.f : 0.f);
    for (int c = 0; c < 3; ++c) trans[3 * i + c] = valid ? (float)g.t[3 * i + c] : 0.f;
  }
  if (i == 0 && status) {
    status[0] = valid ? 1 : 0;
    status[1] = g.flags[F_ACCEPTED];
    status[2] = g.flags[F_PCG_TOTAL];
    status[3] = g.flags[F_ILL];
  }
  if (loss_out && i < 4 * n_log) loss_out[i] = (i / 4 < g.flags[F_ACCEPTED]) ? g.loss_log[i] : 0.0;
}

__global__ void k_reset_flags(Gn g) {
  int i = threadIdx.x;
  if (i < F_COUNT) g.flags[i] = 0;
  if (i < S_COUNT) g.scal[i] = 0.0;
  if (i < 4) g.tickets[i] = 0;
}

// --------------------------------------------------------------------------------------------
static double lm_for_iter(double lm0, int gn_iter) {
  double lm = lm0;
  for (int i = 0; i <= gn_iter; ++i)
    if (i % 3 == 2) lm /= 2;
  return lm;
}

static void free_all(Gn* g) {
  void* ptrs[] = {g->nodes, g->tpos, g->conf, g->src, g->wts, g->tgt, g->tpx, g->tpy, g->ew, g->anc, g->edges,
                  g->map, g->row_ptr, g->col, g->row_cnt, g->R, g->t, g->A_own, g->rhs_own, g->Dinv, g->x, g->r,
                  g->z, g->p0, g->p1, g->q, g->part, g->scal, g->flags, g->tickets, g->loss_log};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (g->host_flag) (void)hipHostFree(g->host_flag);
}

static int gn_pcg(Gn* g, int gn_iter, double* A, double* rhs, hipStream_t hs) {
  const int nwg_node = (g->N + kPcgBlock - 1) / kPcgBlock;
  const int nwg_row = (g->N + (kPcgBlock / 64) - 1) / (kPcgBlock / 64);
  double lm = lm_for_iter(g->prm.lm_factor, gn_iter);
  hipLaunchKernelGGL(k_pcg_prep, dim3(nwg_node), dim3(kPcgBlock), 0, hs, *g, lm, A, rhs);
  OFX_LAUNCH_CHECK();
  const int poll = 8;
  for (int it = 0; it < g->prm.pcg_max_iter; ++it) {
    int parity = it & 1;
    hipLaunchKernelGGL(k_pcg_spmv, dim3(nwg_row), dim3(kPcgBlock), 0, hs, *g, (const double*)A, parity);
    hipLaunchKernelGGL(k_pcg_update, dim3(nwg_node), dim3(kPcgBlock), 0, hs, *g, parity);
    OFX_LAUNCH_CHECK();
    if ((it + 1) % poll == 0 && it + 1 < g->prm.pcg_max_iter) {
      OFX_HIP(hipMemcpyAsync(g->host_flag, g->flags + F_DONE, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
      OFX_HIP(hipStreamSynchronize(hs));
      if (*g->host_flag) break;
    }
  }
  return OFX_OK;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_gn_create(int32_t max_nodes, int32_t max_matches, void** handle) {
  OFX_CHECK_ARG(handle && max_nodes > 0 && max_matches >= 0, "bad gn_create args");
  Gn* g = new Gn();
  g->max_nodes = max_nodes;
  g->max_matches = max_matches;
  int64_t N = max_nodes, M = max_matches > 0 ? max_matches : 1;
  int64_t nwg = (N + 3) / 4 + 8;
#define ALLOC(ptr, n) \
  if (hipMalloc((void**)&(ptr), (size_t)(n) * sizeof(*(ptr))) != hipSuccess) { free_all(g); delete g; set_error("hipMalloc failed"); return OFX_ERR_ALLOC; }
  ALLOC(g->nodes, 3 * N); ALLOC(g->tpos, 3 * N); ALLOC(g->conf, N);
  ALLOC(g->src, 3 * M); ALLOC(g->wts, 4 * M); ALLOC(g->tgt, 3 * M); ALLOC(g->tpx, M); ALLOC(g->tpy, M);
  ALLOC(g->anc, 4 * M);
  ALLOC(g->map, N * N); ALLOC(g->row_ptr, N + 1); ALLOC(g->row_cnt, N);
  ALLOC(g->R, 9 * N); ALLOC(g->t, 3 * N);
  ALLOC(g->Dinv, 36 * N); ALLOC(g->x, 6 * N); ALLOC(g->r, 6 * N); ALLOC(g->z, 6 * N);
  ALLOC(g->p0, 6 * N); ALLOC(g->p1, 6 * N); ALLOC(g->q, 6 * N);
  ALLOC(g->part, 4 * nwg); ALLOC(g->scal, S_COUNT); ALLOC(g->flags, F_COUNT); ALLOC(g->tickets, 4);
  ALLOC(g->loss_log, 4 * 64); ALLOC(g->rhs_own, 6 * N + 4);
#undef ALLOC
  if (hipHostMalloc((void**)&g->host_flag, sizeof(int32_t), 0) != hipSuccess) {
    free_all(g); delete g; set_error("hipHostMalloc failed"); return OFX_ERR_ALLOC;
  }
  (void)hipMemset(g->tickets, 0, 4 * sizeof(uint32_t));
  *handle = g;
  return OFX_OK;
}

int ofx_gn_destroy(void* handle) {
  if (!handle) return OFX_OK;
  Gn* g = (Gn*)handle;
  (void)hipDeviceSynchronize();
  free_all(g);
  delete g;
  return OFX_OK;
}

int ofx_gn_setup(void* handle, const ofx_gn_problem* pb, const ofx_gn_params* prm, int64_t* nnz_blocks,
                 ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && pb && prm, "null handle/problem/params");
  OFX_CHECK_ARG(pb->n_nodes >= 1 && pb->n_nodes <= g->max_nodes, "n_nodes %d outside [1,%d]", pb->n_nodes, g->max_nodes);
  OFX_CHECK_ARG(pb->n_matches >= 0 && pb->n_matches <= g->max_matches, "n_matches %d > max %d", pb->n_matches, g->max_matches);
  OFX_CHECK_ARG(pb->n_neighbors >= 0, "bad n_neighbors");
  OFX_CHECK_ARG(pb->nodes && pb->target_node_pos && pb->node_conf, "null node buffers");
  OFX_CHECK_ARG(pb->n_matches == 0 || (pb->src && pb->anchors && pb->weights && pb->tgt), "null match buffers");
  OFX_CHECK_ARG(prm->num_iter >= 0 && prm->num_iter <= 64, "num_iter must be in [0,64]");
  OFX_CHECK_ARG(prm->pcg_max_iter >= 1, "pcg_max_iter must be >= 1");
  hipStream_t hs = as_stream(s);
  int N = pb->n_nodes, M = pb->n_matches, NB = pb->n_neighbors;
  g->N = N; g->M = M; g->NB = NB; g->prm = *prm;
  g->fx = pb->fx; g->fy = pb->fy; g->cx = pb->cx; g->cy = pb->cy;
  // edges + weights
  if (g->edges) { OFX_HIP(hipFree(g->edges)); g->edges = nullptr; }
  if (g->ew) { OFX_HIP(hipFree(g->ew)); g->ew = nullptr; }
  int64_t ne = (int64_t)N * NB;
  if (ne > 0) {
    OFX_CHECK_ARG(pb->edges, "null edges");
    OFX_HIP(hipMalloc((void**)&g->edges, ne * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->ew, ne * sizeof(double)));
    OFX_HIP(hipMemcpyAsync(g->edges, pb->edges, ne * sizeof(int32_t), hipMemcpyDeviceToDevice, hs));
    hipLaunchKernelGGL(k_edge_weights, dim3(grid_for(ne, 256)), dim3(256), 0, hs, pb->edge_weights, ne,
                       prm->use_edge_weighting, NB, g->ew);
  }
  hipLaunchKernelGGL(k_to_f64, dim3(grid_for(3 * N, 256)), dim3(256), 0, hs, pb->nodes, g->nodes, (int64_t)3 * N);
  hipLaunchKernelGGL(k_to_f64, dim3(grid_for(3 * N, 256)), dim3(256), 0, hs, pb->target_node_pos, g->tpos, (int64_t)3 * N);
  hipLaunchKernelGGL(k_to_f64, dim3(grid_for(N, 256)), dim3(256), 0, hs, pb->node_conf, g->conf, (int64_t)N);
  if (M > 0) {
    hipLaunchKernelGGL(k_to_f64, dim3(grid_for(3 * M, 256)), dim3(256), 0, hs, pb->src, g->src, (int64_t)3 * M);
    hipLaunchKernelGGL(k_to_f64, dim3(grid_for(4 * M, 256)), dim3(256), 0, hs, pb->weights, g->wts, (int64_t)4 * M);
    hipLaunchKernelGGL(k_to_f64, dim3(grid_for(3 * M, 256)), dim3(256), 0, hs, pb->tgt, g->tgt, (int64_t)3 * M);
    hipLaunchKernelGGL(k_to_f64, dim3(grid_for(M, 256)), dim3(256), 0, hs, pb->target_px, g->tpx, (int64_t)M);
    hipLaunchKernelGGL(k_to_f64, dim3(grid_for(M, 256)), dim3(256), 0, hs, pb->target_py, g->tpy, (int64_t)M);
    OFX_HIP(hipMemcpyAsync(g->anc, pb->anchors, (size_t)4 * M * sizeof(int32_t), hipMemcpyDeviceToDevice, hs));
  }
  OFX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_init_state, dim3(grid_for(N, 256)), dim3(256), 0, hs, pb->prev_rot, pb->prev_trans, N, g->R, g->t);
  hipLaunchKernelGGL(k_reset_flags, dim3(1), dim3(64), 0, hs, *g);
  // pattern
  OFX_HIP(hipMemsetAsync(g->map, 0, (size_t)N * N * sizeof(int32_t), hs));
  int64_t nmark = (int64_t)M * 16;
  if (ne > nmark) nmark = ne;
  if (N > nmark) nmark = N;
  hipLaunchKernelGGL(k_mark, dim3(grid_for(nmark, 256, 1 << 30)), dim3(256), 0, hs, N, M, NB, g->anc, g->edges, g->map);
  hipLaunchKernelGGL(k_row_count, dim3(N), dim3(256), 0, hs, N, g->map, g->row_cnt);
  hipLaunchKernelGGL(k_scan_rows, dim3(1), dim3(1024), 0, hs, N, g->row_cnt, g->row_ptr);
  OFX_LAUNCH_CHECK();
  int32_t nnz = 0;
  OFX_HIP(hipMemcpyAsync(&nnz, g->row_ptr + N, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipStreamSynchronize(hs));
  if ((int64_t)nnz > g->nnzb_cap) {
    if (g->col) OFX_HIP(hipFree(g->col));
    if (g->A_own) OFX_HIP(hipFree(g->A_own));
    g->nnzb_cap = (int64_t)nnz + nnz / 4 + 64;
    OFX_HIP(hipMalloc((void**)&g->col, g->nnzb_cap * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->A_own, g->nnzb_cap * 36 * sizeof(double)));
  }
  g->nnzb = nnz;
  hipLaunchKernelGGL(k_row_assign, dim3(N), dim3(256), 0, hs, N, g->map, g->row_ptr, g->col);
  OFX_LAUNCH_CHECK();
  if (nnz_blocks) *nnz_blocks = nnz;
  g->setup_done = true;
  return OFX_OK;
}

int ofx_gn_linearize(void* handle, int32_t gn_iter, int32_t m0, int32_t m1, int32_t add_reg, double* A, double* rhs,
                     ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && g->setup_done, "gn_setup not called");
  OFX_CHECK_ARG(A && rhs, "null A/rhs");
  OFX_CHECK_ARG(m0 >= 0 && m1 <= g->M && m0 <= m1, "bad match range [%d,%d) of %d", m0, m1, g->M);
  (void)gn_iter;
  hipStream_t hs = as_stream(s);
  OFX_HIP(hipMemsetAsync(A, 0, (size_t)g->nnzb * 36 * sizeof(double), hs));
  OFX_HIP(hipMemsetAsync(rhs, 0, (size_t)(6 * g->N + 4) * sizeof(double), hs));
  DataCoef dc;
  dc.lf = sqrt(g->prm.lambda_flow); dc.ld = sqrt(g->prm.lambda_depth);
  dc.fx = g->fx; dc.fy = g->fy; dc.cx = g->cx; dc.cy = g->cy;
  Gn gv = *g;
  if (!(g->tpx && g->M)) { gv.tpx = nullptr; gv.tpy = nullptr; }
  if (m1 > m0)
    hipLaunchKernelGGL(k_data, dim3(grid_for((int64_t)(m1 - m0) * 4, 256, 1 << 30)), dim3(256), 0, hs, gv, dc, m0, m1, A, rhs);
  if (add_reg) {
    int64_t ne = (int64_t)g->N * g->NB;
    if (ne > 0)
      hipLaunchKernelGGL(k_arap, dim3(grid_for(ne, 256, 1 << 30)), dim3(256), 0, hs, gv, sqrt(g->prm.lambda_arap), A, rhs);
    hipLaunchKernelGGL(k_motion, dim3(grid_for(g->N, 256)), dim3(256), 0, hs, gv, sqrt(g->prm.lambda_motion), A, rhs);
  }
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_gn_step(void* handle, int32_t gn_iter, double* A, double* rhs, ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && g->setup_done, "gn_setup not called");
  OFX_CHECK_ARG(A && rhs, "null A/rhs");
  hipStream_t hs = as_stream(s);
  int st = gn_pcg(g, gn_iter, A, rhs, hs);
  if (st) return st;
  hipLaunchKernelGGL(k_step_decide, dim3(1), dim3(kPcgBlock), 0, hs, *g, (const double*)rhs, 64);
  hipLaunchKernelGGL(k_apply, dim3(grid_for(g->N, 256)), dim3(256), 0, hs, *g);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_gn_finish(void* handle, const ofx_gn_result* res, ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && g->setup_done && res && res->rot && res->trans, "bad gn_finish args");
  int n_log = g->prm.num_iter;
  int64_t n = g->N > 4 * n_log ? g->N : 4 * n_log;
  hipLaunchKernelGGL(k_finish, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(s), *g, res->rot, res->trans,
                     res->status, res->loss_log, n_log);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_gn_solve(void* handle, const ofx_gn_problem* pb, const ofx_gn_params* prm, const ofx_gn_result* res,
                 ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  int64_t nnz = 0;
  int st = ofx_gn_setup(handle, pb, prm, &nnz, s);
  if (st) return st;
  for (int it = 0; it < prm->num_iter; ++it) {
    st = ofx_gn_linearize(handle, it, 0, g->M, 1, g->A_own, g->rhs_own, s);
    if (st) return st;
    st = ofx_gn_step(handle, it, g->A_own, g->rhs_own, s);
    if (st) return st;
    // stop host loop early once the device has stopped (costs one sync per GN iteration)
    OFX_HIP(hipMemcpyAsync(g->host_flag, g->flags + F_STOPPED, sizeof(int32_t), hipMemcpyDeviceToHost, as_stream(s)));
    OFX_HIP(hipStreamSynchronize(as_stream(s)));
    if (*g->host_flag) break;
  }
  return ofx_gn_finish(handle, res, s);
}

}  // extern "C"
