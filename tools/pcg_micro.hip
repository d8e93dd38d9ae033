// Latency micro-benchmark for the PCG iteration kernel structure (tuning tool, not product code).
// Synthetic block-sparse pattern shaped like the GN system (N block rows of 6x6 f64, ~12 blocks
// per row). Each variant is launched back-to-back ITERS times on one stream; reports us/launch.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/pcg_micro tools/pcg_micro.hip && /tmp/pcg_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int N = 2073, ITERS = 2000;
constexpr int RPW = 16;   // rows (waves) per WG

struct Sys {
  int *row_ptr, *col, *tpos;
  double *B, *wv0, *wv1, *wg0, *wg1, *vec, *part, *Minv;
  int nw, nnzb;
  double *rec, *partw;   // AoS node state (N x 48: 8 vectors x 6), per-wave partials (2 x 3 x nwaves)
  int nwaves;
  // slot layout (4 rows x 16 slots per wave, 1 round): Bs (nslot x 36), cols (nslot), ws0/ws1 (nslot x 6
  // pushed w), dst (nslot): slot receiving this slot's row w (transposed block position)
  double *Bs, *ws0, *ws1;
  int *dst;
  unsigned* bar;   // grid barrier: [0] arrivals, [1] generation, [2] timeout flag
  float* Mcl;      // cluster preconditioner rows: (rows*6) x 48 f32
  double *mv0, *mv1;
  int* ecol;       // ELL: 16 block slots per row (-1 = empty)
  double* Bell;    // ELL blocks (N x 16 x 36)
  int* flags;
  double* scal;
};

__device__ __forceinline__ double red8(double a) {
  a += __shfl_xor(a, 1, 64); a += __shfl_xor(a, 2, 64); a += __shfl_xor(a, 4, 64);
  return a;
}

__global__ __launch_bounds__(1024) void k_empty(Sys s, int it) {
  if (it < 0) s.part[0] = 1.0;
}

// wave 0 loads the previous partials, barrier, thread 0 writes a new partial
__global__ __launch_bounds__(1024) void k_partials(Sys s, int it) {
  __shared__ double sh;
  if (threadIdx.x < 64) {
    const double* P = s.part + 3 * s.nw * (it & 1);
    double a = 0.0;
    for (int i = threadIdx.x; i < s.nw; i += 64) a += P[3 * i] + P[3 * i + 1] + P[3 * i + 2];
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (threadIdx.x == 0) sh = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* P = s.part + 3 * s.nw * ((it + 1) & 1) + 3 * blockIdx.x;
    P[0] = sh * 1e-9; P[1] = 0.0; P[2] = 0.0;
  }
}

// one dependent trip: every thread loads one double and stores it
__global__ __launch_bounds__(1024) void k_copy(Sys s, int it) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 6 * N) ((it & 1) ? s.wv0 : s.wv1)[i] = ((it & 1) ? s.wv1 : s.wv0)[i] + 1e-9;
}
// two dependent trips: load an index, then the value
__global__ __launch_bounds__(1024) void k_copy2(Sys s, int it) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 6 * N) {
    int j = s.col[i % s.nnzb];
    ((it & 1) ? s.wv0 : s.wv1)[i] = ((it & 1) ? s.wv1 : s.wv0)[6 * j + (i % 6)] + 1e-9;
  }
}

// the shape of the current k_pcg_iter: row_ptr -> (col, B) -> w[col] gather, own-row vectors,
// partials, recurrences, 3 WG sums, partial write. XCD0 = only WGs with blockIdx % 8 == 0 work.
// F_ELL: row blocks at fixed offsets (no row_ptr trip; synthetic, assumes <= 13 blocks/row, padding
// reads real neighbours' data); F_PRE: own-row vectors loaded before the SpMV, SpMV slots unrolled x2;
// F_FAKEW: vector writes predicated off at run time (computation kept); F_MINW: only w written.
enum { F_ELL = 1, F_PRE = 2, F_FAKEW = 4, F_MINW = 8, F_SMALLB = 16, F_F32B = 32, F_SMALLW = 64 };
template <bool PUSH, bool XCD0, int F = 0>
__global__ __launch_bounds__(1024) void k_iter(Sys s, int it) {
  int wgid = blockIdx.x;
  if (XCD0) { if (wgid & 7) return; wgid >>= 3; }
  __shared__ double s_sc[3];
  __shared__ double s_w[3][RPW];
  const int lane = threadIdx.x & 63;
  const int row = wgid * RPW + (threadIdx.x >> 6);
  const double* wc = (it & 1) ? s.wv1 : s.wv0;
  double* wn = (it & 1) ? s.wv0 : s.wv1;
  const double* gc = (it & 1) ? s.wg1 : s.wg0;
  double* gn = (it & 1) ? s.wg0 : s.wg1;
  double pa[3] = {0.0, 0.0, 0.0};
  if (threadIdx.x < 64) {
    const double* P = s.part + 3 * s.nw * (it & 1);
    for (int i = threadIdx.x; i < s.nw; i += 64) { pa[0] += P[3 * i]; pa[1] += P[3 * i + 1]; pa[2] += P[3 * i + 2]; }
  }
  const int rr = lane >> 3, bl = lane & 7;
  const bool upd = row < N && lane < 48 && bl == 0;
  const int64_t o = 6 * (int64_t)row + rr;
  double m = 0.0, v[8], wown = 0.0;
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  if ((F & F_PRE) && upd) {
    const double* Mi = s.Minv + 36 * (int64_t)row + 6 * rr;
    const double* wi = wc + 6 * (int64_t)row;
#pragma unroll
    for (int k = 0; k < 6; ++k) m += Mi[k] * wi[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s.vec[(int64_t)k * 6 * N + o];
    wown = wc[o];
  }
  double acc = 0.0;
  int b0 = 0, b1 = 0;
  if (row < N && lane < 48) {
    if (F & F_ELL) { b0 = row * 12; b1 = b0 + 12; if (b1 > s.nnzb) b1 = s.nnzb; }
    else { b0 = s.row_ptr[row]; b1 = s.row_ptr[row + 1]; }
    if (F & F_PRE) {
      for (int bi = b0 + bl; bi < b1; bi += 16) {
        const bool two = bi + 8 < b1;
        const double* blk = s.B + 36 * (int64_t)bi + rr * 6;
        const double* blk2 = s.B + 36 * (int64_t)(two ? bi + 8 : bi) + rr * 6;
        const double* vc = PUSH ? gc + 6 * (int64_t)bi : wc + 6 * (int64_t)s.col[bi];
        const double* vc2 = PUSH ? gc + 6 * (int64_t)(two ? bi + 8 : bi) : wc + 6 * (int64_t)s.col[two ? bi + 8 : bi];
        double t = 0.0, t2 = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) { t += blk[j] * vc[j]; t2 += blk2[j] * vc2[j]; }
        acc += t + (two ? t2 : 0.0);
      }
    } else {
      for (int bi = b0 + bl; bi < b1; bi += 8) {
        const int bb = (F & F_SMALLB) ? (bi & 255) : bi;
        const double* blk = s.B + 36 * (int64_t)bb + rr * 6;
        const float* blkf = (const float*)s.B + 36 * (int64_t)bb + rr * 6;
        const int cc = (F & F_SMALLW) ? (bi & 63) : s.col[bi];
        const double* vc = PUSH ? gc + 6 * (int64_t)bi : wc + 6 * (int64_t)cc;
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) t += ((F & F_F32B) ? (double)blkf[j] : blk[j]) * vc[j];
        acc += t;
      }
    }
  }
  acc = red8(acc);
  if (!(F & F_PRE) && upd) {
    const double* Mi = s.Minv + 36 * (int64_t)row + 6 * rr;
    const double* wi = wc + 6 * (int64_t)row;
#pragma unroll
    for (int k = 0; k < 6; ++k) m += Mi[k] * wi[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s.vec[(int64_t)k * 6 * N + o];
    wown = wc[o];
  }
  if (threadIdx.x < 64) {
    for (int k = 0; k < 3; ++k)
      for (int off = 32; off > 0; off >>= 1) pa[k] += __shfl_xor(pa[k], off, 64);
    if (threadIdx.x == 0) { s_sc[0] = pa[0]; s_sc[1] = pa[1]; s_sc[2] = pa[2]; }
  }
  __syncthreads();
  const double al = 1e-3 + 1e-12 * s_sc[0], be = 1e-3 + 1e-12 * s_sc[1];
  const bool dow = !(F & F_FAKEW) || s_sc[2] == 12345.0;
  double d[3] = {0.0, 0.0, 0.0};
  double w2 = 0.0;
  if (upd) {
    const double zz = acc + be * v[0], q = m + be * v[1], sv = v[2] + be * v[3], p = v[4] + be * v[5];
    const double r = v[6] - al * sv, u = v[7] - al * q;
    w2 = 0.5 * (wown - al * zz);
    if (dow && !(F & F_MINW)) {
      s.vec[o] = zz; s.vec[6 * N + o] = q; s.vec[3 * 6 * N + o] = sv; s.vec[5 * 6 * N + o] = p;
      s.vec[6 * 6 * N + o] = r; s.vec[7 * 6 * N + o] = u;
    }
    if (dow) wn[o] = w2;
    d[0] = r * u; d[1] = w2 * u; d[2] = r * r;
  }
  if (PUSH) {   // scatter own w2 into the gathered slots of every block in this column
    double wk[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) wk[k] = __shfl(w2, 8 * k, 64);
    if (row < N && lane < 48) {
      for (int bi = b0 + bl; bi < b1; bi += 8) gn[6 * (int64_t)s.tpos[bi] + rr] = wk[rr];
    }
  }
  for (int k = 0; k < 3; ++k)
    for (int off = 32; off > 0; off >>= 1) d[k] += __shfl_xor(d[k], off, 64);
  if (lane == 0) for (int k = 0; k < 3; ++k) s_w[k][threadIdx.x >> 6] = d[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    double* P = s.part + 3 * s.nw * ((it + 1) & 1) + 3 * wgid;
    for (int k = 0; k < 3; ++k) {
      double a = 0.0;
      for (int w = 0; w < RPW; ++w) a += s_w[k][w];
      P[k] = a * 1e-30;
    }
  }
}

// cumulative build-up of the iteration: S=1 partials; 2 + row_ptr trip; 3 + SpMV gather; 4 + own
// vectors and recurrence writes; 5 + second WG reduction (= full iteration)
template <int S>
__global__ __launch_bounds__(1024) void k_step(Sys s, int it) {
  __shared__ double s_sc[3];
  __shared__ double s_w[3][RPW];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * RPW + (threadIdx.x >> 6);
  const double* wc = (it & 1) ? s.wv1 : s.wv0;
  double* wn = (it & 1) ? s.wv0 : s.wv1;
  double pa[3] = {0.0, 0.0, 0.0};
  if (threadIdx.x < 64) {
    const double* P = s.part + 3 * s.nw * (it & 1);
    for (int i = threadIdx.x; i < s.nw; i += 64) { pa[0] += P[3 * i]; pa[1] += P[3 * i + 1]; pa[2] += P[3 * i + 2]; }
  }
  const int rr = lane >> 3, bl = lane & 7;
  double acc = 0.0;
  if (S >= 2 && row < N && lane < 48) {
    const int b0 = s.row_ptr[row], b1 = s.row_ptr[row + 1];
    if (S == 2) acc = b1 - b0;
    if (S >= 3)
      for (int bi = b0 + bl; bi < b1; bi += 8) {
        const double* blk = s.B + 36 * (int64_t)bi + rr * 6;
        const double* vc = wc + 6 * (int64_t)s.col[bi];
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) t += blk[j] * vc[j];
        acc += t;
      }
  }
  if (S >= 3) acc = red8(acc);
  const bool upd = row < N && lane < 48 && bl == 0;
  const int64_t o = 6 * (int64_t)row + rr;
  double m = 0.0, v[8], wown = 0.0;
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  if (S >= 4 && upd) {
    const double* Mi = s.Minv + 36 * (int64_t)row + 6 * rr;
    const double* wi = wc + 6 * (int64_t)row;
#pragma unroll
    for (int k = 0; k < 6; ++k) m += Mi[k] * wi[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s.vec[(int64_t)k * 6 * N + o];
    wown = wc[o];
  }
  if (threadIdx.x < 64) {
    for (int k = 0; k < 3; ++k)
      for (int off = 32; off > 0; off >>= 1) pa[k] += __shfl_xor(pa[k], off, 64);
    if (threadIdx.x == 0) { s_sc[0] = pa[0]; s_sc[1] = pa[1]; s_sc[2] = pa[2]; }
  }
  __syncthreads();
  const double al = 1e-3 + 1e-12 * s_sc[0], be = 1e-3 + 1e-12 * s_sc[1];
  double d[3] = {0.0, 0.0, 0.0};
  if (upd) {
    if (S < 4) wn[o] = 1e-3 * (acc + al);
    else {
      const double zz = acc + be * v[0], q = m + be * v[1], sv = v[2] + be * v[3], p = v[4] + be * v[5];
      const double r = v[6] - al * sv, u = v[7] - al * q;
      const double w2 = 0.5 * (wown - al * zz);
      s.vec[o] = zz; s.vec[6 * N + o] = q; s.vec[3 * 6 * N + o] = sv; s.vec[5 * 6 * N + o] = p;
      s.vec[6 * 6 * N + o] = r; s.vec[7 * 6 * N + o] = u; wn[o] = w2;
      d[0] = r * u; d[1] = w2 * u; d[2] = r * r;
    }
  }
  if (S >= 5) {
    for (int k = 0; k < 3; ++k)
      for (int off = 32; off > 0; off >>= 1) d[k] += __shfl_xor(d[k], off, 64);
    if (lane == 0) for (int k = 0; k < 3; ++k) s_w[k][threadIdx.x >> 6] = d[k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* P = s.part + 3 * s.nw * ((it + 1) & 1) + 3 * blockIdx.x;
    for (int k = 0; k < 3; ++k) {
      double a = 0.0;
      if (S >= 5) for (int w = 0; w < RPW; ++w) a += s_w[k][w];
      P[k] = a * 1e-30 + 1e-30 * s_sc[k];
    }
  }
}

// Restructured iteration: RW rows per wave (lane = (row r, slot q), SL = 64/RW slots per row), one
// wave per WG (no barriers), each lane multiplies a whole 6x6 block; per-row 6-vector via xor
// butterflies over the SL slot lanes; own-row state in an AoS record (8 vectors x 6 per node);
// per-wave partials; every wave re-derives the scalars from the previous launch's per-wave partials.
__device__ __forceinline__ double dpp_d(double x, int ctrlsel) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  switch (ctrlsel) {
    case 0: lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false); break;
    case 1: lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false); break;
    case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, false); break;
    default: lo = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xF, 0xF, false); break;
  }
  return __hiloint2double(hi, lo);
}
// sum over aligned groups of G lanes (G = 2,4,8,16), result in every lane of the group
template <int G>
__device__ __forceinline__ double group_sum(double x) {
  x += dpp_d(x, 0);
  if (G >= 4) x += dpp_d(x, 1);
  if (G >= 8) x += dpp_d(x, 2);
  if (G >= 16) x += dpp_d(x, 3);
  return x;
}
// full wave sum (fixed order): row sums by DPP, then the 4 row totals via readlane
__device__ __forceinline__ double wave_sum(double x) {
  x = group_sum<16>(x);
  const double a = __shfl(x, 0, 64), b = __shfl(x, 16, 64), c = __shfl(x, 32, 64), d = __shfl(x, 48, 64);
  return (a + b) + (c + d);
}

template <int RW, int V = 0>
__global__ __launch_bounds__(64) void k_iterw(Sys s, int it) {
  constexpr int SL = 64 / RW;
  const int lane = threadIdx.x;
  const int r = lane / SL, q = lane % SL;
  const int row = blockIdx.x * RW + r;
  const double* wc = (it & 1) ? s.wv1 : s.wv0;
  double* wn = (it & 1) ? s.wv0 : s.wv1;
  // scalars: previous per-wave partials
  double pa[3] = {0.0, 0.0, 0.0};
  if (V == 0) {
    const double* P = s.partw + 3 * (int64_t)s.nwaves * (it & 1);
    for (int i = lane; i < s.nwaves; i += 64) { pa[0] += P[3 * i]; pa[1] += P[3 * i + 1]; pa[2] += P[3 * i + 2]; }
  } else {   // SoA partials [3][nwaves], all loads issued up front (nwaves <= 64*8)
    const double* P = s.partw + 3 * (int64_t)s.nwaves * (it & 1);
    double t[3][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = lane + 64 * u;
#pragma unroll
      for (int k = 0; k < 3; ++k) t[k][u] = i < s.nwaves ? P[k * s.nwaves + i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) pa[k] = ((t[k][0] + t[k][1]) + (t[k][2] + t[k][3])) + ((t[k][4] + t[k][5]) + (t[k][6] + t[k][7]));
  }
  // own-row state: lane (r, c<6) holds component c of the 8 vectors
  const bool own = row < N && q < 6;
  double v[8], m = 0.0;
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  if (own) {
    const double* R = s.rec + 48 * (int64_t)row + q;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = R[6 * k];
    const double* Mi = s.Minv + 36 * (int64_t)row + 6 * q;
    const double* wi = wc + 6 * (int64_t)row;
#pragma unroll
    for (int k = 0; k < 6; ++k) m += Mi[k] * wi[k];
  }
  // SpMV: lane (r, q) takes blocks q, q+SL, ... of row r
  double n[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (row < N) {
    const int b0 = s.row_ptr[row], b1 = s.row_ptr[row + 1];
    for (int bi = b0 + q; bi < b1; bi += SL) {
      const double* blk = s.B + 36 * (int64_t)bi;
      const double* vc = wc + 6 * (int64_t)s.col[bi];
      double x[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) x[j] = vc[j];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) t += blk[6 * i + j] * x[j];
        n[i] += t;
      }
    }
  }
  if (V >= 2) {
#pragma unroll
    for (int i = 0; i < 6; ++i) n[i] = group_sum<SL>(n[i]);
#pragma unroll
    for (int k = 0; k < 3; ++k) pa[k] = wave_sum(pa[k]);
  } else {
#pragma unroll
    for (int off = 1; off < SL; off <<= 1)
#pragma unroll
      for (int i = 0; i < 6; ++i) n[i] += __shfl_xor(n[i], off, 64);
    for (int k = 0; k < 3; ++k)
      for (int off = 32; off > 0; off >>= 1) pa[k] += __shfl_xor(pa[k], off, 64);
  }
  const double al = 1e-3 + 1e-12 * pa[0], be = 1e-3 + 1e-12 * pa[1];
  double nc = n[0];
#pragma unroll
  for (int i = 1; i < 6; ++i) nc = (q == i) ? n[i] : nc;
  double d[3] = {0.0, 0.0, 0.0};
  if (own) {
    const double zz = nc + be * v[3], qq = m + be * v[4], sv = v[0] + be * v[5], p = v[2] + be * v[6];
    const double rr = v[1] - al * sv, u = v[2] - al * qq;
    const double w2 = 0.5 * (v[0] - al * zz);
    double* R = s.rec + 48 * (int64_t)row + q;
    R[6 * 1] = rr; R[6 * 2] = u; R[6 * 3] = zz; R[6 * 4] = qq; R[6 * 5] = sv; R[6 * 6] = p; R[6 * 7] = v[7] + al * p;
    wn[6 * (int64_t)row + q] = w2;
    d[0] = rr * u; d[1] = w2 * u; d[2] = rr * rr;
  }
  if (V >= 2) {
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = wave_sum(d[k]);
  } else {
    for (int k = 0; k < 3; ++k)
      for (int off = 32; off > 0; off >>= 1) d[k] += __shfl_xor(d[k], off, 64);
  }
  if (lane == 0) {
    double* P = s.partw + 3 * (int64_t)s.nwaves * ((it + 1) & 1);
    if (V == 0) { P += 3 * blockIdx.x; P[0] = d[0] * 1e-30; P[1] = d[1] * 1e-30; P[2] = d[2] * 1e-30; }
    else { P[blockIdx.x] = d[0] * 1e-30; P[s.nwaves + blockIdx.x] = d[1] * 1e-30; P[2 * s.nwaves + blockIdx.x] = d[2] * 1e-30; }
  }
}

// Slot-layout iteration: every load address is static (no row_ptr / col chain): lane (r, q) of
// wave w owns slot (w*64 + lane) holding block (row, j) and the pushed copy of w_j; after the
// update each lane pushes its row's new w into the transposed block's slot of the next buffer.
template <bool PUSHW>
__global__ __launch_bounds__(64) void k_iters(Sys s, int it) {
  const int lane = threadIdx.x;
  const int r = lane / 16, q = lane % 16;
  const int row = blockIdx.x * 4 + r;
  const int64_t slot = (int64_t)blockIdx.x * 64 + lane;
  const double* wc = (it & 1) ? s.wv1 : s.wv0;
  double* wn = (it & 1) ? s.wv0 : s.wv1;
  const double* gc = (it & 1) ? s.ws1 : s.ws0;
  double* gn = (it & 1) ? s.ws0 : s.ws1;
  double t[3][16];
  {
    const double* P = s.partw + 3 * (int64_t)s.nwaves * (it & 1);
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int u = 0; u < 16; ++u) { const int i = lane + 64 * u; t[k][u] = i < s.nwaves ? P[k * s.nwaves + i] : 0.0; }
  }
  const bool own = row < N && q < 6;
  double v[8], mi[6], wi[6];
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  for (int k = 0; k < 6; ++k) { mi[k] = 0.0; wi[k] = 0.0; }
  if (own) {
    const double2* R = reinterpret_cast<const double2*>(s.rec + 48 * (int64_t)row + 8 * q);
    for (int k = 0; k < 4; ++k) { double2 a = R[k]; v[2 * k] = a.x; v[2 * k + 1] = a.y; }
    const double2* Mi = reinterpret_cast<const double2*>(s.Minv + 36 * (int64_t)row + 6 * q);
    const double2* wr = reinterpret_cast<const double2*>(wc + 6 * (int64_t)row);
    for (int k = 0; k < 3; ++k) { double2 a = Mi[k], b = wr[k]; mi[2 * k] = a.x; mi[2 * k + 1] = a.y; wi[2 * k] = b.x; wi[2 * k + 1] = b.y; }
  }
  // one static block per lane
  double n[6];
  {
    const double2* blk = reinterpret_cast<const double2*>(s.Bs + 36 * slot);
    const double2* vc = reinterpret_cast<const double2*>(PUSHW ? gc + 6 * slot : wc + 6 * (int64_t)s.col[slot % s.nnzb]);
    double x[6];
    for (int j = 0; j < 3; ++j) { double2 a = vc[j]; x[2 * j] = a.x; x[2 * j + 1] = a.y; }
    for (int i = 0; i < 6; ++i) {
      double2 b01 = blk[3 * i], b23 = blk[3 * i + 1], b45 = blk[3 * i + 2];
      n[i] = ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
    }
  }
  const int dslot = PUSHW ? s.dst[slot] : 0;
  for (int i = 0; i < 6; ++i) n[i] = group_sum<16>(n[i]);
  double pa[3];
  for (int k = 0; k < 3; ++k) {
    for (int w = 1; w < 16; w <<= 1)
      for (int u = 0; u + w < 16; u += 2 * w) t[k][u] += t[k][u + w];
    pa[k] = wave_sum(t[k][0]);
  }
  const double al = 1e-3 + 1e-12 * pa[0], be = 1e-3 + 1e-12 * pa[1];
  double nc = 0.0, m = 0.0;
  for (int i = 0; i < 6; ++i) { nc += n[i] * (q == i ? 1.0 : 0.0); m += mi[i] * wi[i]; }
  double d[3] = {0.0, 0.0, 0.0};
  double w2 = 0.0;
  if (own) {
    const double zz = nc + be * v[3], qq = m + be * v[4], sv = v[0] + be * v[5], p = v[2] + be * v[6];
    const double rr = v[1] - al * sv, u = v[2] - al * qq;
    w2 = 0.5 * (v[0] - al * zz);
    double2* R = reinterpret_cast<double2*>(s.rec + 48 * (int64_t)row + 8 * q);
    R[0] = make_double2(v[0] + al * p, rr); R[1] = make_double2(u, zz); R[2] = make_double2(qq, sv); R[3] = make_double2(p, 0.0);
    wn[6 * (int64_t)row + q] = w2;
    d[0] = rr * u; d[1] = w2 * u; d[2] = rr * rr;
  }
  if (PUSHW) {
    double wk[6];
    for (int k = 0; k < 6; ++k) wk[k] = __shfl(w2, r * 16 + k, 64);
    double2* o = reinterpret_cast<double2*>(gn + 6 * (int64_t)dslot);
    o[0] = make_double2(wk[0], wk[1]); o[1] = make_double2(wk[2], wk[3]); o[2] = make_double2(wk[4], wk[5]);
  }
  for (int k = 0; k < 3; ++k) d[k] = wave_sum(d[k]);
  if (lane == 0) {
    double* P = s.partw + 3 * (int64_t)s.nwaves * ((it + 1) & 1);
    P[blockIdx.x] = d[0] * 1e-30; P[s.nwaves + blockIdx.x] = d[1] * 1e-30; P[2 * s.nwaves + blockIdx.x] = d[2] * 1e-30;
  }
}

// ---- persistent variant: one cooperative launch runs ITS iterations with a grid barrier between
// them (bounded spin: on timeout the kernel sets bar[2] and returns instead of hanging).
__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned nb, unsigned& gen) {
  bool ok = true;
  if (threadIdx.x == 0) {
    const unsigned g = gen;
    if (__hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&bar[1], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(&bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (++spins > (1 << 22)) { bar[2] = 1; ok = false; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    gen = g + 1;
  }
  return __builtin_amdgcn_readfirstlane(ok ? 1 : 0) != 0;
}

template <int MODE>   // 0: barrier only; 1: iterw4 body + barrier
__global__ __launch_bounds__(64) void k_persist(Sys s, int iters) {
  unsigned gen = __hip_atomic_load(&s.bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lane = threadIdx.x;
  const int r = lane / 16, q = lane % 16;
  const int row = blockIdx.x * 4 + r;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 1) {
      const double* wc = (it & 1) ? s.wv1 : s.wv0;
      double* wn = (it & 1) ? s.wv0 : s.wv1;
      double t[3][16];
      const double* P = s.partw + 3 * (int64_t)s.nwaves * (it & 1);
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int u = 0; u < 16; ++u) { const int i = lane + 64 * u; t[k][u] = i < s.nwaves ? P[k * s.nwaves + i] : 0.0; }
      const bool own = row < N && q < 6;
      double v[8];
      for (int k = 0; k < 8; ++k) v[k] = 0.0;
      if (own) { const double* R = s.rec + 48 * (int64_t)row + 8 * q; for (int k = 0; k < 8; ++k) v[k] = R[k]; }
      double n[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      if (row < N) {
        const int b0 = s.row_ptr[row], b1 = s.row_ptr[row + 1];
        for (int bi = b0 + q; bi < b1; bi += 16) {
          const double* blk = s.B + 36 * (int64_t)bi;
          const double* vc = wc + 6 * (int64_t)s.col[bi];
          for (int i = 0; i < 6; ++i) { double a = 0.0; for (int j = 0; j < 6; ++j) a += blk[6 * i + j] * vc[j]; n[i] += a; }
        }
      }
      for (int i = 0; i < 6; ++i) n[i] = group_sum<16>(n[i]);
      double pa[3];
      for (int k = 0; k < 3; ++k) {
        for (int w = 1; w < 16; w <<= 1)
          for (int u = 0; u + w < 16; u += 2 * w) t[k][u] += t[k][u + w];
        pa[k] = wave_sum(t[k][0]);
      }
      const double al = 1e-3 + 1e-12 * pa[0];
      double nc = 0.0;
      for (int i = 0; i < 6; ++i) nc += n[i] * (q == i ? 1.0 : 0.0);
      double d[3] = {0.0, 0.0, 0.0};
      if (own) {
        const double w2 = 0.5 * (v[0] - al * nc);
        double* R = s.rec + 48 * (int64_t)row + 8 * q;
        R[1] = v[1] - al * w2; R[2] = v[2] + al;
        wn[6 * (int64_t)row + q] = w2;
        d[0] = w2 * w2; d[1] = v[1] * w2; d[2] = v[2];
      }
      for (int k = 0; k < 3; ++k) d[k] = wave_sum(d[k]);
      if (lane == 0) {
        double* Pn = s.partw + 3 * (int64_t)s.nwaves * ((it + 1) & 1);
        Pn[blockIdx.x] = d[0] * 1e-30; Pn[s.nwaves + blockIdx.x] = d[1] * 1e-30; Pn[2 * s.nwaves + blockIdx.x] = d[2] * 1e-30;
      }
    }
    if (!grid_sync(s.bar, gridDim.x, gen)) return;
  }
}

// Cluster-preconditioned explicit pipelined iteration: 8 rows per wave (one 8-node cluster, 8 lanes per
// row), n = A m (m gathered), recurrences incl. w in the state record, then m_new = M_cl⁻¹ w_new via LDS
// (48x48 f32 rows, loaded up front).
struct SysBig { Sys s; char pad[1024]; };
template <bool ELL, bool FLAGS, typename SY>
__global__ __launch_bounds__(64) void k_iterc_t(SY sy, int it) {
  const Sys& s = reinterpret_cast<const Sys&>(sy);
  __shared__ double s_w[48];
  int stop = 0, cnt = 0;
  double gp = 1.0, ap = 1.0;
  if (FLAGS) { stop = s.flags[0] | s.flags[1]; cnt = s.flags[2]; gp = s.scal[it & 1]; ap = s.scal[2 + (it & 1)]; }
  const int lane = threadIdx.x;
  const int r = lane >> 3, q = lane & 7;
  const int row = blockIdx.x * 8 + r;
  const double* mc = (it & 1) ? s.mv1 : s.mv0;
  double* mn = (it & 1) ? s.mv0 : s.mv1;
  double2 t[3][4];
  {
    const double* P = s.partw + 3 * (int64_t)((s.nwaves + 1) & ~1) * (it & 1);
    const int ns = (s.nwaves + 1) & ~1;
    for (int k = 0; k < 3; ++k)
      for (int u = 0; u < 4; ++u) { const int i = 2 * (lane + 64 * u); t[k][u] = i < s.nwaves ? *(const double2*)(P + k * ns + i) : make_double2(0, 0); }
  }
  const bool own = row < N && q < 6;
  double v[8];
  float4 mrow[12];
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  if (own) {
    const double2* R = reinterpret_cast<const double2*>(s.rec + 48 * (int64_t)row + 8 * q);
    for (int k = 0; k < 4; ++k) { double2 a = R[k]; v[2 * k] = a.x; v[2 * k + 1] = a.y; }
    const float4* M = reinterpret_cast<const float4*>(s.Mcl + (int64_t)(6 * row + q) * 48);
    for (int k = 0; k < 12; ++k) mrow[k] = M[k];
  }
  double n[6] = {0, 0, 0, 0, 0, 0};
  if (FLAGS && stop) return;
  if (ELL && row < N) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int64_t e = (int64_t)row * 16 + q + 8 * k;
      const int c = s.ecol[e];
      if (c < 0) continue;
      const double2* blk = reinterpret_cast<const double2*>(s.Bell + 36 * e);
      const double2* vc = reinterpret_cast<const double2*>(mc + 6 * (int64_t)c);
      double x[6];
      for (int j = 0; j < 3; ++j) { double2 a = vc[j]; x[2 * j] = a.x; x[2 * j + 1] = a.y; }
      for (int i = 0; i < 6; ++i) {
        double2 b01 = blk[3 * i], b23 = blk[3 * i + 1], b45 = blk[3 * i + 2];
        n[i] += ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
      }
    }
  }
  if (!ELL && row < N) {
    const int b0 = s.row_ptr[row], b1 = s.row_ptr[row + 1];
    for (int bi = b0 + q; bi < b1; bi += 8) {
      const double2* blk = reinterpret_cast<const double2*>(s.B + 36 * (int64_t)bi);
      const double2* vc = reinterpret_cast<const double2*>(mc + 6 * (int64_t)s.col[bi]);
      double x[6];
      for (int j = 0; j < 3; ++j) { double2 a = vc[j]; x[2 * j] = a.x; x[2 * j + 1] = a.y; }
      for (int i = 0; i < 6; ++i) {
        double2 b01 = blk[3 * i], b23 = blk[3 * i + 1], b45 = blk[3 * i + 2];
        n[i] += ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
      }
    }
  }
  for (int i = 0; i < 6; ++i) n[i] = group_sum<8>(n[i]);
  double pa[3];
  for (int k = 0; k < 3; ++k) {
    double a = 0.0;
    for (int u = 0; u < 4; ++u) a += t[k][u].x + t[k][u].y;
    pa[k] = wave_sum(a);
  }
  double al = 1e-3 + 1e-12 * pa[0], be = 1e-3 + 1e-12 * pa[1];
  if (FLAGS) {
    be = 1e-3 + 1e-12 * (pa[0] / gp);
    al = 1e-3 + 1e-12 * (pa[0] / (pa[1] - be * pa[0] / ap));
    if (pa[2] < -1.0) return;
    if (blockIdx.x == 0 && lane == 0) { s.scal[(it + 1) & 1] = 1.0 + 1e-30 * pa[0]; s.scal[2 + ((it + 1) & 1)] = 1.0 + 1e-30 * al; s.flags[2] = cnt + 1; }
  }
  double nc = 0.0;
  for (int i = 0; i < 6; ++i) nc += n[i] * (q == i ? 1.0 : 0.0);
  double d[3] = {0, 0, 0};
  double w2 = 0.0;
  if (own) {
    const double mo = mc[6 * (int64_t)row + q];
    const double zz = nc + be * v[3], qq = mo + be * v[4], sv = v[7] + be * v[5], p = v[2] + be * v[6];
    const double rr = v[1] - al * sv, u = v[2] - al * qq;
    w2 = 0.5 * (v[7] - al * zz);
    double2* R = reinterpret_cast<double2*>(s.rec + 48 * (int64_t)row + 8 * q);
    R[0] = make_double2(v[0] + al * p, rr); R[1] = make_double2(u, zz); R[2] = make_double2(qq, sv); R[3] = make_double2(p, w2);
    d[0] = rr * u; d[1] = w2 * u; d[2] = rr * rr;
    s_w[6 * r + q] = w2;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  if (own) {
    double m = 0.0;
    for (int k = 0; k < 12; ++k) {
      m += (double)mrow[k].x * s_w[4 * k] + (double)mrow[k].y * s_w[4 * k + 1] + (double)mrow[k].z * s_w[4 * k + 2] +
           (double)mrow[k].w * s_w[4 * k + 3];
    }
    mn[6 * (int64_t)row + q] = m * 1e-3;
  }
  for (int k = 0; k < 3; ++k) d[k] = wave_sum(d[k]);
  if (lane == 0) {
    const int ns = (s.nwaves + 1) & ~1;
    double* P = s.partw + 3 * (int64_t)ns * ((it + 1) & 1);
    P[blockIdx.x] = d[0] * 1e-30; P[ns + blockIdx.x] = d[1] * 1e-30; P[2 * ns + blockIdx.x] = d[2] * 1e-30;
  }
}

template <typename F>
static double timeit(F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 50; ++i) launch(i);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < ITERS; ++i) launch(i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return 1e3 * ms / ITERS;
}

int main() {
  // grid-surface graph 46 x 46 (cropped to N): 8-neighbourhood + 4 two-hop axis neighbours
  const int G = 46;
  std::vector<std::vector<int>> adj(N);
  for (int i = 0; i < N; ++i) {
    int x = i % G, y = i / G;
    for (int dy = -2; dy <= 2; ++dy)
      for (int dx = -2; dx <= 2; ++dx) {
        bool keep = (abs(dx) <= 1 && abs(dy) <= 1) || (dx == 0 && abs(dy) == 2) || (dy == 0 && abs(dx) == 2);
        int xx = x + dx, yy = y + dy, j = yy * G + xx;
        if (keep && xx >= 0 && xx < G && yy >= 0 && j < N && j >= 0) adj[i].push_back(j);
      }
  }
  std::vector<int> rp(N + 1, 0), cl, tp;
  for (int i = 0; i < N; ++i) { rp[i + 1] = rp[i] + (int)adj[i].size(); for (int j : adj[i]) cl.push_back(j); }
  const int nnzb = rp[N];
  tp.resize(nnzb);
  for (int i = 0; i < N; ++i)
    for (int k = rp[i]; k < rp[i + 1]; ++k) {      // position of block (j,i) for block (i,j)
      int j = cl[k];
      for (int q = rp[j]; q < rp[j + 1]; ++q) if (cl[q] == i) tp[k] = q;
    }
  printf("N=%d nnzb=%d (%.1f blocks/row)\n", N, nnzb, (double)nnzb / N);
  Sys s{};
  s.nnzb = nnzb;
  s.nw = (N + RPW - 1) / RPW;
  CK(hipMalloc(&s.row_ptr, (N + 1) * 4)); CK(hipMalloc(&s.col, nnzb * 4)); CK(hipMalloc(&s.tpos, nnzb * 4));
  CK(hipMemcpy(s.row_ptr, rp.data(), (N + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(s.col, cl.data(), nnzb * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(s.tpos, tp.data(), nnzb * 4, hipMemcpyHostToDevice));
  std::vector<double> hb((size_t)nnzb * 36);
  for (size_t i = 0; i < hb.size(); ++i) hb[i] = 1e-3 * ((i * 2654435761u) % 1000) / 1000.0;
  CK(hipMalloc(&s.B, hb.size() * 8)); CK(hipMemcpy(s.B, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&s.Minv, (size_t)N * 36 * 8)); CK(hipMemset(s.Minv, 0, (size_t)N * 36 * 8));
  for (double** p : {&s.wv0, &s.wv1}) { CK(hipMalloc(p, 6 * N * 8)); CK(hipMemset(*p, 0, 6 * N * 8)); }
  for (double** p : {&s.wg0, &s.wg1}) { CK(hipMalloc(p, (size_t)6 * nnzb * 8)); CK(hipMemset(*p, 0, (size_t)6 * nnzb * 8)); }
  CK(hipMalloc(&s.vec, (size_t)8 * 6 * N * 8)); CK(hipMemset(s.vec, 0, (size_t)8 * 6 * N * 8));
  CK(hipMalloc(&s.part, (size_t)6 * s.nw * 8)); CK(hipMemset(s.part, 0, (size_t)6 * s.nw * 8));
  const dim3 g(s.nw), g8(8 * s.nw), b(1024);
  CK(hipMalloc(&s.rec, (size_t)48 * N * 8)); CK(hipMemset(s.rec, 0, (size_t)48 * N * 8));
  CK(hipMalloc(&s.partw, (size_t)6 * N * 8)); CK(hipMemset(s.partw, 0, (size_t)6 * N * 8));
  printf("empty          %7.2f us\n", timeit([&](int i) { hipLaunchKernelGGL(k_empty, g, b, 0, 0, s, i); }));
  printf("empty 64thr    %7.2f us\n", timeit([&](int i) { hipLaunchKernelGGL(k_empty, g, dim3(64), 0, 0, s, i); }));
  printf("partials       %7.2f us\n", timeit([&](int i) { hipLaunchKernelGGL(k_partials, g, b, 0, 0, s, i); }));
  auto run = [&](const char* name, void (*k)(Sys, int)) {
    printf("%-16s %7.2f us\n", name, timeit([&](int i) { hipLaunchKernelGGL(k, g, b, 0, 0, s, i); }));
  };
  auto runw = [&](const char* name, void (*k)(Sys, int), int rw) {
    s.nwaves = (N + rw - 1) / rw;
    printf("%-16s %7.2f us\n", name, timeit([&](int i) { hipLaunchKernelGGL(k, dim3(s.nwaves), dim3(64), 0, 0, s, i); }));
  };
  // hipGraph replay of the same launch sequence (100 kernels per graph)
  auto graph_time = [&](void (*k)(Sys, int), int nwav) -> double {
    s.nwaves = nwav;
    hipStream_t cs;
    CK(hipStreamCreate(&cs));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k, dim3(nwav), dim3(64), 0, cs, s, i);
    CK(hipStreamEndCapture(cs, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, cs));
    CK(hipStreamSynchronize(cs));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a, cs));
    for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(ge, cs));
    CK(hipEventRecord(b, cs));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return 1e3 * ms / 2000;
  };
  {
    const int nsl = ((N + 3) / 4) * 64;
    CK(hipMalloc(&s.Bs, (size_t)nsl * 36 * 8)); CK(hipMemset(s.Bs, 0, (size_t)nsl * 36 * 8));
    CK(hipMalloc(&s.ws0, (size_t)nsl * 6 * 8)); CK(hipMemset(s.ws0, 0, (size_t)nsl * 6 * 8));
    CK(hipMalloc(&s.ws1, (size_t)nsl * 6 * 8)); CK(hipMemset(s.ws1, 0, (size_t)nsl * 6 * 8));
    std::vector<int> hd(nsl);
    for (int i = 0; i < nsl; ++i) hd[i] = (int)((i * 7919LL) % nsl);   // scattered destinations
    CK(hipMalloc(&s.dst, (size_t)nsl * 4)); CK(hipMemcpy(s.dst, hd.data(), (size_t)nsl * 4, hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&s.bar, 16)); CK(hipMemset(s.bar, 0, 16));
  {
    int nblk = 0, ncu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nblk, k_persist<1>, 64, 0));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nwav = (N + 3) / 4;
    printf("co-resident capacity %d x %d CUs = %d (need %d)\n", nblk, ncu, nblk * ncu, nwav);
    if (false && nblk * ncu >= nwav) {
      s.nwaves = nwav;
      for (int mode = 0; mode < 2; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
          const int iters = 2000;
          void* args[] = {&s, (void*)&iters};
          hipEvent_t a, b;
          CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
          CK(hipEventRecord(a, 0));
          if (mode == 0) CK(hipLaunchCooperativeKernel((const void*)k_persist<0>, dim3(nwav), dim3(64), args, 0, 0));
          else CK(hipLaunchCooperativeKernel((const void*)k_persist<1>, dim3(nwav), dim3(64), args, 0, 0));
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, a, b));
          unsigned hb[3];
          CK(hipMemcpy(hb, s.bar, 12, hipMemcpyDeviceToHost));
          printf("persist mode %d   %7.2f us/iter (timeout flag %u)\n", mode, 1e3 * ms / iters, hb[2]);
          if (hb[2]) return 1;
        }
    }
  }
  CK(hipMalloc(&s.Mcl, (size_t)6 * N * 48 * 4)); CK(hipMemset(s.Mcl, 0, (size_t)6 * N * 48 * 4));
  for (double** p : {&s.mv0, &s.mv1}) { CK(hipMalloc(p, 6 * N * 8)); CK(hipMemset(*p, 0, 6 * N * 8)); }
  {
    std::vector<int> ec((size_t)N * 16, -1);
    for (int i = 0; i < N; ++i)
      for (int k = rp[i]; k < rp[i + 1]; ++k) ec[(size_t)i * 16 + (k - rp[i])] = cl[k];
    CK(hipMalloc(&s.ecol, ec.size() * 4)); CK(hipMemcpy(s.ecol, ec.data(), ec.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&s.Bell, (size_t)N * 16 * 36 * 8)); CK(hipMemset(s.Bell, 0, (size_t)N * 16 * 36 * 8));
    CK(hipMalloc(&s.flags, 64)); CK(hipMemset(s.flags, 0, 64));
    CK(hipMalloc(&s.scal, 64)); CK(hipMemset(s.scal, 0, 64));
  }
  SysBig sb{};
  sb.s = s;
  auto runc = [&](const char* name, auto k, auto arg) {
    s.nwaves = (N + 7) / 8;
    sb.s = s;
    printf("%-16s %7.2f us\n", name, timeit([&](int i) { hipLaunchKernelGGL(k, dim3(s.nwaves), dim3(64), 0, 0, arg, i); }));
  };
  for (int rep = 0; rep < 3; ++rep) {
    s.nwaves = (N + 7) / 8; sb.s = s;
    runc("iterc csr", k_iterc_t<false, false, Sys>, s);
    runc("iterc ell", k_iterc_t<true, false, Sys>, s);
    runc("iterc csr+flags", k_iterc_t<false, true, Sys>, s);
    runc("iterc ell+flags", k_iterc_t<true, true, Sys>, s);
    runc("iterc csr+fl+big", k_iterc_t<false, true, SysBig>, sb);
    runc("iterc ell+fl+big", k_iterc_t<true, true, SysBig>, sb);
  }
  for (int rep = 0; rep < 0; ++rep) {
    runw("iters push", k_iters<true>, 4);
    runw("iters gather", k_iters<false>, 4);
    printf("%-16s %7.2f us\n", "graph iters push", graph_time(k_iters<true>, (N + 3) / 4));
    runw("iterw4 soa dpp", k_iterw<4, 2>, 4);
    printf("%-16s %7.2f us\n", "graph iterw4", graph_time(k_iterw<4, 2>, (N + 3) / 4));
    printf("%-16s %7.2f us\n", "graph empty", graph_time(k_empty, (N + 3) / 4));
    runw("empty 519x64", k_empty, 4);
  }
  printf("copy 1 trip      %7.2f us\n", timeit([&](int i) { hipLaunchKernelGGL(k_copy, g, b, 0, 0, s, i); }));
  printf("copy 2 trips     %7.2f us\n", timeit([&](int i) { hipLaunchKernelGGL(k_copy2, g, b, 0, 0, s, i); }));
  return 0;
}
