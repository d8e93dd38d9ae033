// ED-graph construction on the device, bit-exact twins of the reference C++:
//
//   ofx_graph_*            opaque handle: the mesh's vertex adjacency (sorted unique neighbour lists, the
//                          std::set<int> per vertex of graph_proc.cpp:174-186) and scratch
//   ofx_erode_mesh         graph_proc::erode_mesh              csrc/cpu/graph_proc.cpp:17-77
//   ofx_sample_nodes       graph_proc::sample_nodes (no shuffle) csrc/cpu/graph_proc.cpp:79-136
//   ofx_edges_geodesic     graph_proc::compute_edges_geodesic  csrc/cpu/graph_proc.cpp:155-300
//   ofx_edges_euclidean    graph_proc::compute_edges_euclidean csrc/cpu/graph_proc.cpp:302-356
//   ofx_node_edge_cleanup  graph_proc::node_and_edge_clean_up  csrc/cpu/graph_proc.cpp:388-438
//   ofx_compute_clusters   graph_proc::compute_clusters        csrc/cpu/graph_proc.cpp:363-386,440-481
//   (callers: EDGraph.create_graph_from_mesh / update, embedded_deformation_graph.py:153-380,496-609)
//
// How the sequential C++ is reproduced in parallel:
//  * sample_nodes is the lexicographically-first maximal set of the conflict graph (squaredNorm <= c²):
//    rounds over per-vertex lists of lower-id conflicting vertices; a vertex becomes a node when all of them
//    are rejected, and is rejected as soon as one of them is a node (decisions are final, so the rounds
//    converge to the sequential result).
//  * compute_edges_geodesic runs one Dijkstra per thread (nodes in parallel) with libstdc++'s exact binary-heap
//    push/pop (std::priority_queue<..., CustomCompare>), so equal distances pop in the C++ order.
//  * node_and_edge_clean_up removes nodes with <= 1 surviving neighbour until none changes; removal is
//    monotone, so the fixpoint (the least closed removed set) does not depend on the sweep order: parallel
//    Jacobi sweeps give the sequential result.
//  * compute_clusters numbers connected components by their lowest node id (= the C++ traversal order):
//    min-label propagation + a rank of the roots.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ofx_common.h"

namespace ofx {

#define OFX_CHECKS(call)           \
  do {                             \
    const int st_ = (call);        \
    if (st_ != OFX_OK) return st_; \
  } while (0)

__device__ __forceinline__ float eig_sq(float dx, float dy, float dz) {
  const float a = dx * dx, b = dy * dy, c = dz * dz;
  return a + (b + c);   // Eigen 3.3.7 Vector3f redux order
}
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }
__device__ __forceinline__ float fexp(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float fdivr(float a, float b) { return (float)((double)a / (double)b); }

// ------------------------------------------------------------------ adjacency
__global__ __launch_bounds__(256) void k_adj_pairs(const int32_t* __restrict__ faces, int64_t nf, int64_t nv,
                                                   uint64_t* __restrict__ keys, int32_t* __restrict__ bad) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= nf) return;
  const int32_t v[3] = {faces[3 * f], faces[3 * f + 1], faces[3 * f + 2]};
  int o = 0;
  for (int j = 0; j < 3; ++j)
    for (int k = 0; k < 3; ++k) {
      if (j == k) continue;
      uint64_t key = ~0ull;   // sorts last; dropped
      if (v[j] < 0 || v[j] >= nv || v[k] < 0 || v[k] >= nv) atomicOr(bad, 1);
      else if (v[j] != v[k]) key = (uint64_t)v[j] * (uint64_t)nv + (uint64_t)v[k];
      keys[6 * f + o++] = key;
    }
}

__global__ __launch_bounds__(256) void k_adj_unique(const uint64_t* __restrict__ keys, int64_t n, uint8_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  flag[i] = keys[i] != ~0ull && (i == 0 || keys[i] != keys[i - 1]);
}

__global__ __launch_bounds__(256) void k_adj_fill(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ flag,
                                                  const int32_t* __restrict__ pos, int64_t n, int64_t nv,
                                                  int32_t* __restrict__ col, int32_t* __restrict__ rowcnt) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n || !flag[i]) return;
  const int64_t a = (int64_t)(keys[i] / (uint64_t)nv), b = (int64_t)(keys[i] % (uint64_t)nv);
  col[pos[i]] = (int32_t)b;
  atomicAdd(&rowcnt[a], 1);
}

// ------------------------------------------------------------------ erode
__global__ __launch_bounds__(256) void k_erode_count(const int32_t* __restrict__ faces, const uint8_t* __restrict__ alive,
                                                     int64_t nf, int32_t* __restrict__ cnt) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= nf || !alive[f]) return;
  atomicAdd(&cnt[faces[3 * f]], 1);
  atomicAdd(&cnt[faces[3 * f + 1]], 1);
  atomicAdd(&cnt[faces[3 * f + 2]], 1);
}

__global__ __launch_bounds__(256) void k_erode_keep(const int32_t* __restrict__ faces, uint8_t* __restrict__ alive,
                                                    int64_t nf, const int32_t* __restrict__ cnt, int min_nb) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= nf || !alive[f]) return;
  alive[f] = cnt[faces[3 * f]] >= min_nb && cnt[faces[3 * f + 1]] >= min_nb && cnt[faces[3 * f + 2]] >= min_nb;
}

__global__ __launch_bounds__(256) void k_erode_mark(const int32_t* __restrict__ faces, const uint8_t* __restrict__ alive,
                                                    int64_t nf, uint8_t* __restrict__ mask) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= nf || !alive[f]) return;
  mask[faces[3 * f]] = 1;
  mask[faces[3 * f + 1]] = 1;
  mask[faces[3 * f + 2]] = 1;
}

// ------------------------------------------------------------------ sample_nodes
struct Grid {
  float inv_cell;
  uint32_t mask;   // table size - 1 (power of two)
};

__device__ __forceinline__ uint32_t cell_hash(int cx, int cy, int cz, uint32_t mask) {
  return ((uint32_t)cx * 73856093u ^ (uint32_t)cy * 19349663u ^ (uint32_t)cz * 83492791u) & mask;
}
__device__ __forceinline__ void cell_of(const float* p, float inv, int& cx, int& cy, int& cz) {
  cx = (int)floorf(p[0] * inv); cy = (int)floorf(p[1] * inv); cz = (int)floorf(p[2] * inv);
}

// eligible vertices get their cell hash as key; others ~0 (sorted last)
__global__ __launch_bounds__(256) void k_sn_keys(const float* __restrict__ P, const uint8_t* __restrict__ elig, int64_t nv,
                                                 Grid g, uint32_t* __restrict__ key, int32_t* __restrict__ val) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= nv) return;
  uint32_t k = 0xFFFFFFFFu;
  if (elig[v]) {
    int cx, cy, cz;
    cell_of(P + 3 * v, g.inv_cell, cx, cy, cz);
    k = cell_hash(cx, cy, cz, g.mask);
  }
  key[v] = k;
  val[v] = (int32_t)v;
}

__global__ __launch_bounds__(256) void k_sn_bounds(const uint32_t* __restrict__ key, int64_t nv, int32_t* __restrict__ start,
                                                   int32_t* __restrict__ end) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nv || key[i] == 0xFFFFFFFFu) return;
  if (i == 0 || key[i - 1] != key[i]) start[key[i]] = (int32_t)i;
  if (i == nv - 1 || key[i + 1] != key[i]) end[key[i]] = (int32_t)(i + 1);
}

// pass 0: count, pass 1: fill the lower-id conflicting eligible vertices of every eligible vertex (ascending
// id order is not needed: decisions only depend on the set)
template <bool FILL>
__global__ __launch_bounds__(256) void k_sn_conflicts(const float* __restrict__ P, const uint8_t* __restrict__ elig, int64_t nv,
                                                      Grid g, const int32_t* __restrict__ start,
                                                      const int32_t* __restrict__ end, const int32_t* __restrict__ sorted,
                                                      float cov2, int32_t* __restrict__ cnt,
                                                      const int64_t* __restrict__ off, int32_t* __restrict__ list) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= nv || !elig[v]) return;
  const float px = P[3 * v], py = P[3 * v + 1], pz = P[3 * v + 2];
  int cx, cy, cz;
  cell_of(P + 3 * v, g.inv_cell, cx, cy, cz);
  uint32_t seen[27];
  int ns = 0;
  int64_t o = FILL ? off[v] : 0;
  int c = 0;
  for (int dx = -1; dx <= 1; ++dx)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dz = -1; dz <= 1; ++dz) {
        const uint32_t h = cell_hash(cx + dx, cy + dy, cz + dz, g.mask);
        bool dup = false;
        for (int q = 0; q < ns; ++q) dup |= seen[q] == h;   // colliding cells share a bucket: scan it once
        if (dup) continue;
        seen[ns++] = h;
        for (int i = start[h]; i < end[h]; ++i) {
          const int32_t u = sorted[i];
          if (u >= v) continue;
          // (point - node).squaredNorm() <= c² with point = v, node = u (graph_proc.cpp:120); the f32
          // differences only change sign when the roles swap, so the test is symmetric bit for bit
          if (eig_sq(px - P[3 * u], py - P[3 * u + 1], pz - P[3 * u + 2]) <= cov2) {
            if (FILL) list[o + c] = u;
            ++c;
          }
        }
      }
  if (!FILL) cnt[v] = c;
}

enum : int32_t { kUndecided = 0, kNode = 1, kRejected = 2 };

__device__ __forceinline__ int32_t ld_state(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1: L1 bypass, other CUs' stores
}
__device__ __forceinline__ void st_state(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// round form (fallback): one launch per round, every undecided vertex advances its cursor
__global__ __launch_bounds__(256) void k_sn_round(const uint8_t* __restrict__ elig, int64_t nv,
                                                  const int64_t* __restrict__ off, const int32_t* __restrict__ list,
                                                  int64_t* __restrict__ cursor, int32_t* __restrict__ state,
                                                  int32_t* __restrict__ n_undecided) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= nv || !elig[v] || ld_state(state + v) != kUndecided) return;
  int64_t c = cursor[v];
  const int64_t e = off[v + 1];
  int32_t s = kNode;
  for (; c < e; ++c) {
    const int32_t su = ld_state(state + list[c]);   // decisions are final: a stale read only delays
    if (su == kRejected) continue;
    s = su == kNode ? kRejected : kUndecided;
    break;
  }
  cursor[v] = c;
  if (s != kUndecided) st_state(state + v, s);
  else atomicAdd(n_undecided, 1);
}

// persistent form: a fully resident grid (<= 2 workgroups of 256 per CU); thread t owns vertices t, t+T, ...
// in increasing order and advances them as a per-lane state machine inside ONE uniform loop (lanes of a
// wave never wait on each other inside divergent code). The lowest undecided vertex always has all its
// lower neighbours decided and its owner is at it, so the grid makes progress; every spin is bounded
// (timeout -> *err, the host finishes with the round form: decisions already stored are final).
__global__ __launch_bounds__(256) void k_sn_persistent(const uint8_t* __restrict__ elig, int64_t nv,
                                                       const int64_t* __restrict__ off, const int32_t* __restrict__ list,
                                                       int64_t* __restrict__ cursor, int32_t* __restrict__ state,
                                                       int64_t max_iter, int32_t* __restrict__ err) {
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t c = 0, e = 0;
  bool fresh = true;
  for (int64_t it = 0; it < max_iter; ++it) {
    if (__all(v >= nv)) return;
    if (v < nv) {
      if (fresh) {
        if (!elig[v]) { v += T; continue; }
        c = off[v];
        e = off[v + 1];
        fresh = false;
      }
      int32_t decided = kUndecided;
      // advance over decided neighbours (at most 16 per step, so lanes stay in step)
      for (int q = 0; q < 16; ++q) {
        if (c >= e) { decided = kNode; break; }
        const int32_t su = ld_state(state + list[c]);
        if (su == kRejected) { ++c; continue; }
        if (su == kNode) decided = kRejected;
        break;
      }
      if (decided != kUndecided) {
        st_state(state + v, decided);
        v += T;
        fresh = true;
      } else {
        cursor[v] = c;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (v < nv) atomicOr(err, 1);
}

// greedy form (the C++ loop itself, graph_proc.cpp:100-131): ONE workgroup holds the undecided-vertex bitmap
// in LDS (1 bit per vertex, <= 160 KiB). A step takes the 64 lowest undecided vertices: the first is the
// sequential loop's next node (every lower vertex is a node or within c of one); each later one is a node
// iff no node chosen before it in the batch lies within c (a 64x64 conflict mask resolved in order by one
// wave). The workgroup then clears, for every chosen node, the bits of all vertices within c, found in the
// 27 hashed cells around it (positions in cell order, float4 + id). Steps <= nodes; the loop ends when the
// bitmap is empty (<= nv steps, no inter-workgroup waiting).
constexpr int kGreedyThreads = 1024;
constexpr int64_t kGreedyMaxWords = 40 * 1024 - 4096;   // 160 KiB of LDS minus the batch buffers (static LDS)

__global__ __launch_bounds__(256) void k_sn_spos(const float* __restrict__ P, const int32_t* __restrict__ sorted,
                                                 int64_t nv, float4* __restrict__ spos) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const int32_t u = sorted[i];
  spos[i] = make_float4(P[3 * (int64_t)u], P[3 * (int64_t)u + 1], P[3 * (int64_t)u + 2], __int_as_float(u));
}

__global__ __launch_bounds__(kGreedyThreads) void k_sn_greedy(const float* __restrict__ P,
                                                               const uint8_t* __restrict__ elig, int64_t nv, Grid gr,
                                                               const int32_t* __restrict__ bstart,
                                                               const int32_t* __restrict__ bend,
                                                               const float4* __restrict__ spos, float cov2,
                                                               int32_t* __restrict__ state,
                                                               int64_t* __restrict__ n_steps, int64_t* __restrict__ stamps) {
  extern __shared__ uint32_t bits[];
  __shared__ int32_t s_cand[64];
  __shared__ float4 s_sel[64];   // chosen nodes: position + id
  __shared__ int32_t s_nsel;
  __shared__ int64_t s_w;
  __shared__ int32_t s_off[64 * 27], s_rs[64 * 27], s_wsum[kGreedyThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t nw = (nv + 31) >> 5;
  for (int64_t w = tid; w < nw; w += kGreedyThreads) {
    uint32_t x = 0;
    const int64_t v0 = w << 5;
    for (int b = 0; b < 32; ++b)
      if (v0 + b < nv && elig[v0 + b]) x |= 1u << b;
    bits[w] = x;
  }
  __syncthreads();
  int64_t cw = 0;   // every word below cw is empty
  int64_t step = 0;
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0}, t0 = wall_clock64();   // tuning: phase times (stamps != null)
  for (; step < nv; ++step) {
    if (wave == 0) {
      // ---- the (up to) 64 lowest undecided vertices, in order
      int got = 0;
      int64_t first_w = -1;
      for (int64_t w0 = cw; w0 < nw && got < 64 && (got == 0 || w0 < cw + 128); w0 += 64) {   // window: 4096 ids
        const uint32_t x = w0 + lane < nw ? bits[w0 + lane] : 0u;
        const int c = __popc(x);
        int pre = c;   // inclusive prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(pre, o);
          if (lane >= o) pre += y;
        }
        const uint64_t nz = __ballot(x != 0u);
        if (first_w < 0 && nz) first_w = w0 + __builtin_ctzll(nz);
        int slot = got + pre - c;
        for (uint32_t y = x; y && slot < 64; y &= y - 1, ++slot)
          s_cand[slot] = (int32_t)(((w0 + lane) << 5) + __builtin_ctz(y));
        got += __shfl(pre, 63);
      }
      got = min(got, 64);
      if (first_w >= 0) cw = first_w;
      uint64_t ta = stamps ? wall_clock64() : 0;
      // ---- in-batch resolution: lane i holds candidate i
      const bool have = lane < got;
      const int32_t v = have ? s_cand[lane] : 0;
      const float px = have ? P[3 * (int64_t)v] : 0.f, py = have ? P[3 * (int64_t)v + 1] : 0.f,
                  pz = have ? P[3 * (int64_t)v + 2] : 0.f;
      const int ngot = __builtin_amdgcn_readfirstlane(got);   // uniform (SGPR) bound
      uint64_t conf = 0;   // bit j: an earlier candidate j lies within c (point = this, node = j)
#pragma unroll
      for (int j = 0; j < 63; ++j) {   // constant lane indices: v_readlane into scalars
        const float rx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px), j));
        const float ry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py), j));
        const float rz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz), j));
        if (j + 1 < ngot && j < lane && eig_sq(px - rx, py - ry, pz - rz) <= cov2) conf |= 1ull << j;
      }
      uint64_t tb = stamps ? wall_clock64() : 0;
      const uint32_t conf_lo = (uint32_t)conf, conf_hi = (uint32_t)(conf >> 32);
      uint64_t sel = 0;
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const uint64_t row = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)conf_lo, i) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)conf_hi, i) << 32);
        if (i < ngot && !(row & sel)) sel |= 1ull << i;
      }
      if (have && ((sel >> lane) & 1ull)) {
        const int r = __popcll(sel & ((1ull << lane) - 1ull));
        s_sel[r] = make_float4(px, py, pz, __int_as_float(v));
        state[v] = kNode;
      }
      if (stamps) { const uint64_t tc = wall_clock64(); ph[4] += ta - t0; ph[5] += tb - ta; ph[6] += tc - tb; }
      if (lane == 0) { s_nsel = __popcll(sel); s_w = got ? cw : -1; }
    }
    __syncthreads();
    if (stamps) { const uint64_t t = wall_clock64(); ph[0] += t - t0; t0 = t; }
    if (s_w < 0) break;
    cw = s_w;
    // ---- clear everything within c of the chosen nodes. Items = (node, cell): their bucket ranges load in
    // one trip, a workgroup scan flattens them, and every thread tests 8 positions per trip.
    const int nsel = s_nsel, items = nsel * 27;
    int len2[2], rs2[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = 2 * tid + k;
      len2[k] = 0; rs2[k] = 0;
      if (it < items) {
        const float4 q = s_sel[it / 27];
        const int c = it % 27;
        int cx, cy, cz;
        const float qp[3] = {q.x, q.y, q.z};
        cell_of(qp, gr.inv_cell, cx, cy, cz);
        const int dx = c / 9 - 1, dy = (c / 3) % 3 - 1, dz = c % 3 - 1;
        // skip a neighbour cell whose box lies farther than c (0.5 % margin; cells are 1.01·c wide)
        const float cs = 1.f / gr.inv_cell;
        const float gx = dx > 0 ? (cx + 1) * cs - q.x : dx < 0 ? q.x - cx * cs : 0.f;
        const float gy = dy > 0 ? (cy + 1) * cs - q.y : dy < 0 ? q.y - cy * cs : 0.f;
        const float gz = dz > 0 ? (cz + 1) * cs - q.z : dz < 0 ? q.z - cz * cs : 0.f;
        if (fmaxf(gx, 0.f) * fmaxf(gx, 0.f) + fmaxf(gy, 0.f) * fmaxf(gy, 0.f) + fmaxf(gz, 0.f) * fmaxf(gz, 0.f) <=
            cov2 * 1.01f) {
          const uint32_t h = cell_hash(cx + dx, cy + dy, cz + dz, gr.mask);
          rs2[k] = bstart[h];
          len2[k] = bend[h] - rs2[k];
        }
      }
    }
    int x = len2[0] + len2[1];
    const int own = x;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_wsum[wave] = x;
    __syncthreads();
    int base = 0, total = 0;
    for (int q = 0; q < kGreedyThreads / 64; ++q) {
      const int wsum = s_wsum[q];
      base += q < wave ? wsum : 0;
      total += wsum;
    }
    {
      const int ex = base + x - own;
      if (2 * tid < items) { s_off[2 * tid] = ex; s_rs[2 * tid] = rs2[0]; }
      if (2 * tid + 1 < items) { s_off[2 * tid + 1] = ex + len2[0]; s_rs[2 * tid + 1] = rs2[1]; }
    }
    __syncthreads();
    if (stamps) { const uint64_t t = wall_clock64(); ph[1] += t - t0; t0 = t; ph[3] += total; }
    for (int e0 = 8 * tid; e0 < total; e0 += 8 * kGreedyThreads) {   // 8 consecutive positions per thread
      int lo = 0, hi = items - 1;   // last item with s_off <= e0 (one search, then walk)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= e0) lo = mid; else hi = mid - 1;
      }
      float4 u[8];
      int itm[8];
      int it = lo, nxt = it + 1 < items ? s_off[it + 1] : total;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = e0 + k;
        while (e >= nxt && it + 1 < items) { ++it; nxt = it + 1 < items ? s_off[it + 1] : total; }
        itm[k] = e < total ? it : -1;
        u[k] = spos[e < total ? s_rs[it] + (e - s_off[it]) : 0];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (itm[k] < 0) continue;
        const float4 q = s_sel[itm[k] / 27];
        if (eig_sq(u[k].x - q.x, u[k].y - q.y, u[k].z - q.z) <= cov2) {
          const int32_t uid = __float_as_int(u[k].w);
          atomicAnd(&bits[uid >> 5], ~(1u << (uid & 31)));
        }
      }
    }
    __syncthreads();
    if (stamps) { const uint64_t t = wall_clock64(); ph[2] += t - t0; t0 = t; }
  }
  if (tid == 0) {
    *n_steps = step;
    if (stamps) for (int q = 0; q < 7; ++q) stamps[q] = (int64_t)ph[q];
  }
}

__global__ __launch_bounds__(256) void k_sn_flags(const int32_t* __restrict__ state, const uint8_t* __restrict__ elig,
                                                  int64_t nv, uint8_t* __restrict__ is_node) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v < nv) is_node[v] = elig[v] && state[v] == kNode;
}

__global__ __launch_bounds__(256) void k_sn_emit(const float* __restrict__ P, const uint8_t* __restrict__ is_node,
                                                 const int32_t* __restrict__ rank, int64_t nv, float* __restrict__ pos,
                                                 int32_t* __restrict__ idx) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= nv || !is_node[v]) return;
  const int32_t r = rank[v];
  pos[3 * (int64_t)r] = P[3 * v]; pos[3 * (int64_t)r + 1] = P[3 * v + 1]; pos[3 * (int64_t)r + 2] = P[3 * v + 2];
  idx[r] = (int32_t)v;
}

// ------------------------------------------------------------------ graph pyramid down-sampling
// embedded_deformation_graph.py:278-299, sequential by nature (node i's test depends on every kept node
// before it): ONE workgroup keeps the kept nodes' positions in LDS; per node all threads compute the f32
// np.linalg.norm distances ((dx² + dy²) + dz², correctly rounded sqrt) to the kept list in parallel and a
// (distance, index) minimum gives numpy's argmin (first minimum). Two barriers per node.
constexpr int kDsThreads = 1024;
constexpr int kDsMax = 8192;   // kept nodes held in LDS (128 KiB)

__global__ __launch_bounds__(kDsThreads) void k_downsample(const float* __restrict__ P, int n, double cov,
                                                           int32_t* __restrict__ down, int32_t* __restrict__ up,
                                                           int32_t* __restrict__ n_down) {
  __shared__ float4 s_kp[kDsMax];
  __shared__ uint64_t s_best[kDsThreads / 64];
  __shared__ int s_nd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_nd = 0;
  __syncthreads();
  for (int i = 0; i < n; ++i) {
    const float px = P[3 * (int64_t)i], py = P[3 * (int64_t)i + 1], pz = P[3 * (int64_t)i + 2];
    const int nd = s_nd;
    uint64_t best = ~0ull;
    for (int t = tid; t < nd; t += kDsThreads) {
      const float4 q = s_kp[t];
      const float dx = q.x - px, dy = q.y - py, dz = q.z - pz;   // old_nodes[down] - old_nodes[i]
      const float d = sqrt_rn((dx * dx + dy * dy) + dz * dz);
      best = min(best, ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)t);
    }
    for (int o = 32; o >= 1; o >>= 1) best = min(best, (uint64_t)__shfl_xor((unsigned long long)best, o));
    if (lane == 0) s_best[wave] = best;
    __syncthreads();
    if (tid == 0) {
      if (nd == 0) {
        up[i] = i;
        down[0] = i;
        s_kp[0] = make_float4(px, py, pz, 0.f);
        s_nd = 1;
      } else {
        uint64_t b = s_best[0];
        for (int w = 1; w < kDsThreads / 64; ++w) b = min(b, s_best[w]);
        const int j = (int)(uint32_t)b;
        up[i] = j;
        if (!((double)__uint_as_float((uint32_t)(b >> 32)) < cov) && nd < kDsMax) {
          down[nd] = i;
          s_kp[nd] = make_float4(px, py, pz, 0.f);
          s_nd = nd + 1;
        } else if (!((double)__uint_as_float((uint32_t)(b >> 32)) < cov)) {
          s_nd = kDsMax + 1;   // overflow: reported, the host falls back
        }
      }
    }
    __syncthreads();
    if (s_nd > kDsMax) break;
  }
  if (tid == 0) *n_down = s_nd;
}

// ------------------------------------------------------------------ geodesic edges
struct HeapEnt {
  int32_t v;
  float d;
};

// libstdc++ std::__push_heap with comp(a, b) = a.d > b.d
__device__ __forceinline__ void heap_sift_up(HeapEnt* h, int64_t hole, int64_t top, HeapEnt val) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && h[parent].d > val.d) {
    h[hole] = h[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  h[hole] = val;
}

// std::pop_heap on [0, n) followed by pop_back: returns the top, leaves n-1 entries
__device__ __forceinline__ HeapEnt heap_pop(HeapEnt* h, int64_t n) {
  const HeapEnt top = h[0];
  const int64_t len = n - 1;
  if (len > 0) {
    const HeapEnt val = h[len];
    int64_t hole = 0, second = 0;
    while (second < (len - 1) / 2) {
      second = 2 * (second + 1);
      if (h[second].d > h[second - 1].d) second--;
      h[hole] = h[second];
      hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
      second = 2 * (second + 1);
      h[hole] = h[second - 1];
      hole = second - 1;
    }
    heap_sift_up(h, hole, 0, val);
  }
  return top;
}

struct GeoArgs {
  const float* P;
  const uint8_t* valid;      // per vertex (may be null: all valid)
  const int32_t* rowptr;     // adjacency CSR
  const int32_t* col;
  const int32_t* v2n;        // vertex -> node (last node id wins, graph_proc.cpp:190-196) or -1
  const int32_t* node_idx;   // node -> vertex
  int32_t n_nodes, K;
  int64_t nv;
  float cov, max_inf, two_c2;
  int32_t only_valid, enforce;
  int32_t *edges;
  float *wts, *dists, *n2v;  // n2v may be null
  uint32_t* visited;         // bitmap, batch rows of ceil(nv/32) words
  HeapEnt* heap;             // batch rows of cap entries
  int64_t cap;
  int32_t* status;           // per node: 0 ok, 1 heap overflow, 2 invalid vertex reached
};

__global__ __launch_bounds__(64) void k_geodesic(GeoArgs a, const int32_t* __restrict__ todo, int32_t n_todo) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_todo) return;
  const int32_t node = todo[t];
  const int64_t words = (a.nv + 31) / 32;
  uint32_t* vis = a.visited + (int64_t)t * words;
  HeapEnt* h = a.heap + (int64_t)t * a.cap;
  for (int i = 0; i < a.K; ++i) {
    a.edges[(int64_t)node * a.K + i] = -1;
    a.wts[(int64_t)node * a.K + i] = 0.f;
    a.dists[(int64_t)node * a.K + i] = 0.f;
  }
  a.status[node] = 0;
  const int32_t s = a.node_idx[node];
  if (s < 0) return;
  int64_t n = 0;
  h[n++] = HeapEnt{s, 0.f};
  int32_t ids[16];
  float ds[16];
  int cnt = 0;
  while (n > 0) {
    const HeapEnt top = heap_pop(h, n);
    --n;
    const int32_t v = top.v;
    const float d = top.d;
    if (vis[v >> 5] & (1u << (v & 31))) continue;
    if (a.only_valid && a.valid && !a.valid[v]) { a.status[node] = 2; return; }   // the C++ calls exit(0)
    const int32_t m = a.v2n[v];
    if (m >= 0 && m != node) {
      ids[cnt] = m;
      ds[cnt] = d;
      ++cnt;
      if (cnt >= a.K) break;
    }
    if (a.n2v) a.n2v[(int64_t)node * a.nv + v] = d;
    vis[v >> 5] |= 1u << (v & 31);
    const float vx = a.P[3 * (int64_t)v], vy = a.P[3 * (int64_t)v + 1], vz = a.P[3 * (int64_t)v + 2];
    for (int32_t q = a.rowptr[v]; q < a.rowptr[v + 1]; ++q) {
      const int32_t u = a.col[q];
      if (a.only_valid && a.valid && !a.valid[u]) continue;
      const float dist = d + sqrt_rn(eig_sq(vx - a.P[3 * (int64_t)u], vy - a.P[3 * (int64_t)u + 1],
                                            vz - a.P[3 * (int64_t)u + 2]));
      if (a.enforce || dist <= a.max_inf) {
        if (n >= a.cap) { a.status[node] = 1; return; }
        heap_sift_up(h, n, 0, HeapEnt{u, dist});
        ++n;
      }
    }
  }
  // weights (graph_proc.cpp:262-281): exp(-(d*d)/(2c²)) f32, f32 sum, w/sum or w/n
  float w[16];
  float sum = 0.f;
  for (int i = 0; i < cnt; ++i) {
    w[i] = fexp(fdivr(-(ds[i] * ds[i]), a.two_c2));
    sum += w[i];
  }
  for (int i = 0; i < cnt; ++i) {
    const int64_t o = (int64_t)node * a.K + i;
    a.edges[o] = ids[i];
    a.wts[o] = sum > 0.f ? fdivr(w[i], sum) : fdivr(w[i], (float)cnt);
    a.dists[o] = ds[i];
  }
}

// Parallel form: ONE workgroup per node computes the f32 geodesic distances of its neighbourhood by
// label-correcting relaxation in rounds (frontier queues + an open-addressing vertex table in LDS). With
// positive edge lengths fl(d + len) >= d, so the least fixpoint d(v) = min_u fl(d(u) + len(u, v)) is exactly
// the distance the C++ Dijkstra pops each vertex at (its predecessor pops first). Relaxation is bounded by a
// radius R that grows ×1.25 from the coverage (capped at the 2·coverage pruning unless
// enforce_total_num_neighbors) until K candidate nodes lie within R: below R every distance is final, and
// vertices whose edges were cut by R are re-queued when it grows. Pop order then only matters among EQUAL
// distances: ties among the first K+1 candidate nodes, or (with n2v) another vertex at the K-th node's
// distance, send the node to the sequential heap kernel above (status 3); a full table or queue retries with
// the larger table (status 4). Outputs are written only for a settled node.
namespace geo {
constexpr int kThreads = 256;
constexpr int kQueue = 1280;     // frontier slots per queue
constexpr int kCand = 256;       // candidate nodes
constexpr int kMaxRounds = 8192;
enum : int32_t { kOk = 0, kInvalid = 2, kTie = 3, kFull = 4 };
}  // namespace geo

template <int TBL>
__device__ __forceinline__ uint32_t geo_hash(int32_t v) {
  return ((uint32_t)v * 2654435761u) >> (32 - __builtin_ctz(TBL));
}

// TBL vertex slots (keys + f32 distances: 8 B each); 8192 -> ≈ 78 KiB of LDS (2 workgroups per CU),
// 16384 -> ≈ 143 KiB (the retry tier for nodes whose neighbourhood did not fit)
template <int TBL>
__global__ __launch_bounds__(geo::kThreads) void k_geo_relax(GeoArgs a, const int32_t* __restrict__ todo, int32_t n_todo) {
  using namespace geo;
  __shared__ int32_t keys[TBL];
  __shared__ uint32_t dist[TBL];
  __shared__ int32_t queue[2][kQueue];
  __shared__ uint32_t qflag[TBL / 32], bnd[TBL / 32];
  __shared__ float cand_d[kCand];
  __shared__ int32_t cand_m[kCand], cand_v[kCand];
  __shared__ int32_t s_n[2], s_fail, s_nbnd, s_used, s_ncand, s_amb;
  __shared__ float sel_d[17];
  __shared__ int32_t sel_m[17], sel_v[17];
  const int tid = threadIdx.x, lane = tid & 63;
  if ((int)blockIdx.x >= n_todo) return;
  const int32_t node = todo ? todo[blockIdx.x] : (int32_t)blockIdx.x;
  const int32_t s0 = a.node_idx[node];
  if (s0 < 0) {
    if (tid < a.K) {
      a.edges[(int64_t)node * a.K + tid] = -1;
      a.wts[(int64_t)node * a.K + tid] = 0.f;
      a.dists[(int64_t)node * a.K + tid] = 0.f;
    }
    if (tid == 0) a.status[node] = kOk;
    return;
  }
  if (a.only_valid && a.valid && !a.valid[s0]) {   // popped first: the C++ exits
    if (tid == 0) a.status[node] = kInvalid;
    return;
  }
  for (int i = tid; i < TBL; i += kThreads) { keys[i] = -1; dist[i] = 0x7F800000u; }
  for (int i = tid; i < TBL / 32; i += kThreads) { qflag[i] = 0u; bnd[i] = 0u; }
  __syncthreads();
  if (tid == 0) {
    const uint32_t h = geo_hash<TBL>(s0);
    keys[h] = s0; dist[h] = 0u;
    queue[0][0] = (int32_t)h;
    s_n[0] = 1; s_n[1] = 0; s_fail = 0; s_nbnd = 0; s_used = 1; s_amb = 0;
  }
  float R = a.enforce ? a.cov : fminf(a.cov, a.max_inf);
  int cur = 0, rounds = 0;
  for (;;) {
    __syncthreads();
    // ---- relax to the fixpoint under R
    for (;; ++rounds) {
      const int nf = s_n[cur];
      if (nf == 0 || s_fail) break;
      if (rounds >= kMaxRounds) { s_fail = kFull; break; }   // uniform: every thread sees the same counts
      for (int i = tid; i < nf; i += kThreads) {
        const int32_t sl = queue[cur][i];
        atomicAnd(&qflag[sl >> 5], ~(1u << (sl & 31)));
      }
      if (tid == 0) s_n[cur ^ 1] = 0;
      __syncthreads();
      for (int i = tid; i < nf; i += kThreads) {
        const int32_t sl = queue[cur][i];
        const int32_t v = keys[sl];
        const float d = __uint_as_float(dist[sl]);
        const float vx = a.P[3 * (int64_t)v], vy = a.P[3 * (int64_t)v + 1], vz = a.P[3 * (int64_t)v + 2];
        const int32_t q1 = a.rowptr[v + 1];
        bool cut = false;
        for (int32_t q = a.rowptr[v]; q < q1; ++q) {
          const int32_t u = a.col[q];
          if (a.only_valid && a.valid && !a.valid[u]) continue;
          const float nd = d + sqrt_rn(eig_sq(vx - a.P[3 * (int64_t)u], vy - a.P[3 * (int64_t)u + 1],
                                              vz - a.P[3 * (int64_t)u + 2]));
          if (!(nd <= R)) { cut = true; continue; }
          uint32_t h = geo_hash<TBL>(u);
          int32_t probe = 0;
          for (; probe < TBL; ++probe, h = (h + 1) & (TBL - 1)) {
            const int32_t k = keys[h];
            if (k == u) break;
            if (k == -1) {
              const int32_t o = atomicCAS(&keys[h], -1, u);
              if (o == -1) { if (atomicAdd(&s_used, 1) >= TBL * 7 / 8) s_fail = kFull; break; }
              if (o == u) break;
            }
          }
          if (probe == TBL) { s_fail = kFull; break; }
          const uint32_t nb = __float_as_uint(nd);
          if (nb < atomicMin(&dist[h], nb)) {
            if (!(atomicOr(&qflag[h >> 5], 1u << (h & 31)) & (1u << (h & 31)))) {
              const int32_t p = atomicAdd(&s_n[cur ^ 1], 1);
              if (p < kQueue) queue[cur ^ 1][p] = (int32_t)h;
              else s_fail = kFull;
            }
          }
        }
        if (cut && !(atomicOr(&bnd[sl >> 5], 1u << (sl & 31)) & (1u << (sl & 31)))) atomicAdd(&s_nbnd, 1);
      }
      __syncthreads();
      cur ^= 1;
    }
    __syncthreads();
    if (s_fail) break;
    // ---- candidate nodes within R
    if (tid == 0) s_ncand = 0;
    __syncthreads();
    for (int i = tid; i < TBL; i += kThreads) {
      const int32_t v = keys[i];
      if (v < 0) continue;
      const int32_t m = a.v2n[v];
      if (m >= 0 && m != node) {
        const int32_t p = atomicAdd(&s_ncand, 1);
        if (p < kCand) { cand_d[p] = __uint_as_float(dist[i]); cand_m[p] = m; cand_v[p] = v; }
        else s_fail = kFull;
      }
    }
    __syncthreads();
    if (s_fail) break;
    const bool at_cap = !a.enforce && R >= a.max_inf;
    const bool done = s_ncand >= a.K || at_cap || s_nbnd == 0;   // K found, pruning radius reached, or all reached
    __syncthreads();   // every wave has read s_ncand / s_nbnd before thread 0 resets them (else waves diverge)
    if (done) break;
    // ---- grow R; re-queue the vertices whose edges it cut
    R = a.enforce ? R * 1.25f : fminf(R * 1.25f, a.max_inf);
    if (tid == 0) { s_n[cur] = 0; s_nbnd = 0; }
    __syncthreads();
    for (int w = tid; w < TBL / 32; w += kThreads) {
      uint32_t x = bnd[w];
      if (!x) continue;
      bnd[w] = 0u;
      for (; x; x &= x - 1) {
        const int32_t sl = w * 32 + __builtin_ctz(x);
        if (!(atomicOr(&qflag[sl >> 5], 1u << (sl & 31)) & (1u << (sl & 31)))) {
          const int32_t p = atomicAdd(&s_n[cur], 1);
          if (p < kQueue) queue[cur][p] = sl;
          else s_fail = kFull;
        }
      }
    }
  }
  __syncthreads();
  if (s_fail) {
    if (tid == 0) a.status[node] = s_fail;
    return;
  }
  const int nc = s_ncand;
  const int nsel = min(nc, a.K + 1);
  if (tid < 64) {   // wave 0: the nsel smallest candidates in ascending distance
    float ld[kCand / 64];
#pragma unroll
    for (int j = 0; j < kCand / 64; ++j) {
      const int c = lane + 64 * j;
      ld[j] = c < nc ? cand_d[c] : __builtin_inff();
    }
    for (int k = 0; k < nsel; ++k) {
      uint64_t best = ~0ull;
#pragma unroll
      for (int j = 0; j < kCand / 64; ++j) {
        const int c = lane + 64 * j;
        if (c < nc) best = min(best, ((uint64_t)__float_as_uint(ld[j]) << 32) | (uint32_t)c);
      }
      for (int o = 32; o >= 1; o >>= 1) best = min(best, (uint64_t)__shfl_xor((unsigned long long)best, o));
      const int c = (int)(uint32_t)best;
#pragma unroll
      for (int j = 0; j < kCand / 64; ++j)
        if (lane + 64 * j == c) ld[j] = __uint_as_float(0x7F800001u);   // taken (sorts above +inf)
      if (lane == 0) { sel_d[k] = cand_d[c]; sel_m[k] = cand_m[c]; sel_v[k] = cand_v[c]; }
    }
  }
  __syncthreads();
  bool tie = false;
  for (int k = 1; k < nsel; ++k) tie |= sel_d[k] == sel_d[k - 1];
  const int nn = min(nc, a.K);
  const bool brk = nc >= a.K;                       // the C++ breaks at the K-th node
  const float dK = brk ? sel_d[a.K - 1] : __builtin_inff();
  const int32_t vK = brk ? sel_v[a.K - 1] : -1;
  if (!tie && a.n2v && brk) {
    for (int i = tid; i < TBL; i += kThreads)
      if (keys[i] >= 0 && keys[i] != vK && __uint_as_float(dist[i]) == dK) s_amb = 1;
    __syncthreads();
  }
  if (tie || s_amb) {
    if (tid == 0) a.status[node] = kTie;
    return;
  }
  if (a.n2v)
    for (int i = tid; i < TBL; i += kThreads) {
      const int32_t v = keys[i];
      const float d = __uint_as_float(dist[i]);
      if (v >= 0 && (!brk || d < dK)) a.n2v[(int64_t)node * a.nv + v] = d;
    }
  if (tid == 0) {
    float w[16];
    float sum = 0.f;
    for (int i = 0; i < nn; ++i) {
      w[i] = fexp(fdivr(-(sel_d[i] * sel_d[i]), a.two_c2));
      sum += w[i];
    }
    for (int i = 0; i < a.K; ++i) {
      const int64_t o = (int64_t)node * a.K + i;
      a.edges[o] = i < nn ? sel_m[i] : -1;
      a.wts[o] = i < nn ? (sum > 0.f ? fdivr(w[i], sum) : fdivr(w[i], (float)nn)) : 0.f;
      a.dists[o] = i < nn ? sel_d[i] : 0.f;
    }
    a.status[node] = kOk;
  }
}

__global__ __launch_bounds__(256) void k_v2n(const int32_t* __restrict__ node_idx, int32_t n_nodes, int64_t nv,
                                             int32_t* __restrict__ v2n) {
  // the C++ loop assigns in node order, so the LAST node on a vertex wins: max over node ids
  const int32_t n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const int32_t v = node_idx[n];
  if (v >= 0 && v < nv) atomicMax(&v2n[v], n);
}

__global__ __launch_bounds__(256) void k_fill_f32(float* __restrict__ p, int64_t n, float val) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = val;
}

// ------------------------------------------------------------------ euclidean edges
__global__ __launch_bounds__(256) void k_edges_euclid(const float* __restrict__ X, int n_nodes, int K,
                                                      int32_t* __restrict__ edges) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const float px = X[3 * n], py = X[3 * n + 1], pz = X[3 * n + 2];
  float d[16];
  int id[16];
  int cnt = 0;
  for (int j = 0; j < n_nodes; ++j) {
    if (j == n) continue;
    const float d2 = eig_sq(px - X[3 * j], py - X[3 * j + 1], pz - X[3 * j + 2]);
    int pos = cnt;
    for (int s = cnt - 1; s >= 0; --s)
      if (d2 <= d[s]) pos = s;
    if (pos < K) {
      const int last = cnt < K ? cnt : K - 1;
      for (int s = last; s > pos; --s) { d[s] = d[s - 1]; id[s] = id[s - 1]; }
      d[pos] = d2;
      id[pos] = j;
      if (cnt < K) ++cnt;
    }
  }
  for (int s = 0; s < K; ++s) edges[(int64_t)n * K + s] = s < cnt ? id[s] : -1;
}

// ------------------------------------------------------------------ clean-up and clusters
__global__ __launch_bounds__(256) void k_cleanup_sweep(const int32_t* __restrict__ E, int n_nodes, int K,
                                                       const uint8_t* __restrict__ valid_in, uint8_t* __restrict__ removed,
                                                       int32_t* __restrict__ changed) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes || !valid_in[n] || removed[n]) return;
  int c = 0;
  for (int i = 0; i < K; ++i) {
    const int32_t j = E[(int64_t)n * K + i];
    if (j == -1) break;
    if (j >= 0 && j < n_nodes && ((volatile const uint8_t*)removed)[j]) continue;
    ++c;
  }
  if (c <= 1) {
    ((volatile uint8_t*)removed)[n] = 1;
    atomicAdd(changed, 1);
  }
}

__global__ __launch_bounds__(256) void k_cleanup_out(const uint8_t* __restrict__ valid_in, const uint8_t* __restrict__ removed,
                                                     int n_nodes, uint8_t* __restrict__ valid_out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < n_nodes) valid_out[n] = valid_in[n] && !removed[n];
}

__global__ __launch_bounds__(256) void k_cc_init(int32_t* __restrict__ lab, int n_nodes) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < n_nodes) lab[n] = n;
}

// hook: for every edge (n, j) before the row's first -1, both ends take the smaller root label
__global__ __launch_bounds__(256) void k_cc_hook(const int32_t* __restrict__ E, int n_nodes, int K, int32_t* __restrict__ lab,
                                                 int32_t* __restrict__ changed) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  for (int i = 0; i < K; ++i) {
    const int32_t j = E[(int64_t)n * K + i];
    if (j == -1) break;
    if (j < 0 || j >= n_nodes) continue;
    const int32_t a = lab[n], b = lab[j];
    if (a == b) continue;
    const int32_t lo = min(a, b), hi = max(a, b);
    if (atomicMin(&lab[hi], lo) > lo) atomicAdd(changed, 1);
  }
}

__global__ __launch_bounds__(256) void k_cc_jump(int32_t* __restrict__ lab, int n_nodes, int32_t* __restrict__ changed) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const int32_t l = lab[n], ll = lab[l];
  if (ll != l) { lab[n] = ll; atomicAdd(changed, 1); }
}

__global__ __launch_bounds__(256) void k_cc_roots(const int32_t* __restrict__ lab, int n_nodes, uint8_t* __restrict__ root) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < n_nodes) root[n] = lab[n] == n;
}

__global__ __launch_bounds__(256) void k_cc_out(const int32_t* __restrict__ lab, const int32_t* __restrict__ rank, int n_nodes,
                                                int32_t* __restrict__ clusters, int32_t* __restrict__ sizes) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes) return;
  const int32_t c = rank[lab[n]];
  clusters[n] = c;
  if (sizes) atomicAdd(&sizes[c], 1);
}

// ------------------------------------------------------------------ handle
struct Graph {
  int64_t nv = 0, nf = 0;
  int32_t* rowptr = nullptr;   // nv + 1
  int32_t* col = nullptr;
  int64_t ncol = 0;
  const float* P = nullptr;
  const int32_t* faces = nullptr;
  int64_t geo_sequential = 0;   // nodes the last ofx_edges_geodesic ran through the sequential heap kernel
  int64_t sn_steps = 0;         // batches of the last greedy sample_nodes
};

template <typename T>
int dalloc(T** p, int64_t n, hipStream_t s) {
  OFX_HIP(hipMallocAsync((void**)p, (size_t)std::max<int64_t>(n, 1) * sizeof(T), s));
  return OFX_OK;
}
template <typename T>
void dfree(T* p, hipStream_t s) {
  if (p) (void)hipFreeAsync(p, s);
}

inline int exclusive_sum_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t s) {
  size_t tmp = 0;
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)n, s));
  void* t = nullptr;
  OFX_HIP(hipMallocAsync(&t, std::max<size_t>(tmp, 1), s));
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(t, tmp, in, out, (int)n, s));
  OFX_HIP(hipFreeAsync(t, s));
  return OFX_OK;
}
inline int exclusive_sum_u8(const uint8_t* in, int32_t* out, int64_t n, hipStream_t s) {
  size_t tmp = 0;
  hipcub::TransformInputIterator<int32_t, hipcub::CastOp<int32_t>, const uint8_t*> it(in, hipcub::CastOp<int32_t>());
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, out, (int)n, s));
  void* t = nullptr;
  OFX_HIP(hipMallocAsync(&t, std::max<size_t>(tmp, 1), s));
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(t, tmp, it, out, (int)n, s));
  OFX_HIP(hipFreeAsync(t, s));
  return OFX_OK;
}
inline int exclusive_sum_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s) {
  size_t tmp = 0;
  hipcub::TransformInputIterator<int64_t, hipcub::CastOp<int64_t>, const int32_t*> it(in, hipcub::CastOp<int64_t>());
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, out, (int)n, s));
  void* t = nullptr;
  OFX_HIP(hipMallocAsync(&t, std::max<size_t>(tmp, 1), s));
  OFX_HIP(hipcub::DeviceScan::ExclusiveSum(t, tmp, it, out, (int)n, s));
  OFX_HIP(hipFreeAsync(t, s));
  return OFX_OK;
}

template <typename T>
inline int read1(const T* dev, T* host, hipStream_t s) {
  OFX_HIP(hipMemcpyAsync(host, dev, sizeof(T), hipMemcpyDeviceToHost, s));
  OFX_HIP(hipStreamSynchronize(s));
  return OFX_OK;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_graph_create(const float* vertices, int64_t n_vertices, const int32_t* faces, int64_t n_faces, void** handle,
                     ofx_stream_t s) {
  OFX_CHECK_ARG(handle && n_vertices >= 0 && n_faces >= 0, "bad arguments");
  OFX_CHECK_ARG(n_vertices < (1ll << 31) && 6 * n_faces < (1ll << 31), "mesh too large");
  OFX_CHECK_ARG((n_vertices == 0 || vertices) && (n_faces == 0 || faces), "null mesh");
  hipStream_t hs = as_stream(s);
  Graph* g = new Graph();
  g->nv = n_vertices;
  g->nf = n_faces;
  g->P = vertices;
  g->faces = faces;
  *handle = g;
  const int64_t np = 6 * n_faces;
  OFX_CHECKS(dalloc(&g->rowptr, n_vertices + 1, hs));
  OFX_HIP(hipMemsetAsync(g->rowptr, 0, (n_vertices + 1) * sizeof(int32_t), hs));
  if (np == 0) {
    OFX_CHECKS(dalloc(&g->col, 1, hs));
    return OFX_OK;
  }
  uint64_t *keys = nullptr, *keys2 = nullptr;
  uint8_t* flag = nullptr;
  int32_t *pos = nullptr, *cnt = nullptr, *bad = nullptr;
  OFX_CHECKS(dalloc(&keys, np, hs));
  OFX_CHECKS(dalloc(&keys2, np, hs));
  OFX_CHECKS(dalloc(&flag, np, hs));
  OFX_CHECKS(dalloc(&pos, np + 1, hs));
  OFX_CHECKS(dalloc(&cnt, n_vertices + 1, hs));
  OFX_CHECKS(dalloc(&bad, 1, hs));
  OFX_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), hs));
  OFX_HIP(hipMemsetAsync(cnt, 0, (n_vertices + 1) * sizeof(int32_t), hs));
  hipLaunchKernelGGL(k_adj_pairs, dim3(grid_for(n_faces, 256, 1 << 30)), dim3(256), 0, hs, faces, n_faces, n_vertices, keys, bad);
  size_t tmp = 0;
  OFX_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, keys, keys2, (int)np, 0, 64, hs));
  void* t = nullptr;
  OFX_HIP(hipMallocAsync(&t, std::max<size_t>(tmp, 1), hs));
  OFX_HIP(hipcub::DeviceRadixSort::SortKeys(t, tmp, keys, keys2, (int)np, 0, 64, hs));
  OFX_HIP(hipFreeAsync(t, hs));
  hipLaunchKernelGGL(k_adj_unique, dim3(grid_for(np, 256, 1 << 30)), dim3(256), 0, hs, (const uint64_t*)keys2, np, flag);
  OFX_CHECKS(exclusive_sum_u8(flag, pos, np, hs));
  int32_t ncol = 0, hbad = 0;
  // total = pos[np-1] + flag[np-1]
  int32_t last_pos = 0;
  uint8_t last_flag = 0;
  OFX_HIP(hipMemcpyAsync(&last_pos, pos + np - 1, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipMemcpyAsync(&last_flag, flag + np - 1, 1, hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipStreamSynchronize(hs));
  ncol = last_pos + last_flag;
  if (hbad) {
    dfree(keys, hs); dfree(keys2, hs); dfree(flag, hs); dfree(pos, hs); dfree(cnt, hs); dfree(bad, hs);
    set_error("face index out of range [0, %lld)", (long long)n_vertices);
    return OFX_ERR_ARG;
  }
  g->ncol = ncol;
  OFX_CHECKS(dalloc(&g->col, ncol, hs));
  hipLaunchKernelGGL(k_adj_fill, dim3(grid_for(np, 256, 1 << 30)), dim3(256), 0, hs, (const uint64_t*)keys2,
                     (const uint8_t*)flag, (const int32_t*)pos, np, n_vertices, g->col, cnt);
  OFX_CHECKS(exclusive_sum_i32(cnt, g->rowptr, n_vertices + 1, hs));
  OFX_LAUNCH_CHECK();
  dfree(keys, hs); dfree(keys2, hs); dfree(flag, hs); dfree(pos, hs); dfree(cnt, hs); dfree(bad, hs);
  return OFX_OK;
}

int ofx_graph_destroy(void* handle) {
  if (!handle) return OFX_OK;
  Graph* g = (Graph*)handle;
  (void)hipDeviceSynchronize();
  if (g->rowptr) (void)hipFree(g->rowptr);
  if (g->col) (void)hipFree(g->col);
  delete g;
  return OFX_OK;
}

int ofx_graph_geodesic_sequential(void* handle, int64_t* n_nodes) {
  Graph* g = (Graph*)handle;
  OFX_CHECK_ARG(g && n_nodes, "null argument");
  *n_nodes = g->geo_sequential;
  return OFX_OK;
}

/* vertex adjacency (CSR) of the handle's mesh, for inspection: rowptr i32[V+1], col i32[rowptr[V]] */
int ofx_graph_adjacency(void* handle, int32_t* rowptr, int32_t* col, int64_t* n_col, ofx_stream_t s) {
  Graph* g = (Graph*)handle;
  OFX_CHECK_ARG(g && n_col, "null argument");
  *n_col = g->ncol;
  hipStream_t hs = as_stream(s);
  if (rowptr) OFX_HIP(hipMemcpyAsync(rowptr, g->rowptr, (g->nv + 1) * sizeof(int32_t), hipMemcpyDeviceToDevice, hs));
  if (col && g->ncol) OFX_HIP(hipMemcpyAsync(col, g->col, g->ncol * sizeof(int32_t), hipMemcpyDeviceToDevice, hs));
  return OFX_OK;
}

int ofx_erode_mesh(void* handle, int32_t n_iterations, int32_t min_neighbors, uint8_t* non_eroded, ofx_stream_t s) {
  Graph* g = (Graph*)handle;
  OFX_CHECK_ARG(g && non_eroded && n_iterations >= 0, "bad arguments");
  hipStream_t hs = as_stream(s);
  if (g->nv == 0) return OFX_OK;
  OFX_HIP(hipMemsetAsync(non_eroded, 0, g->nv, hs));
  if (g->nf == 0) return OFX_OK;
  uint8_t* alive = nullptr;
  int32_t* cnt = nullptr;
  OFX_CHECKS(dalloc(&alive, g->nf, hs));
  OFX_CHECKS(dalloc(&cnt, g->nv, hs));
  OFX_HIP(hipMemsetAsync(alive, 1, g->nf, hs));
  const dim3 gf(grid_for(g->nf, 256, 1 << 30));
  for (int it = 0; it < n_iterations; ++it) {
    OFX_HIP(hipMemsetAsync(cnt, 0, g->nv * sizeof(int32_t), hs));
    hipLaunchKernelGGL(k_erode_count, gf, dim3(256), 0, hs, g->faces, (const uint8_t*)alive, g->nf, cnt);
    hipLaunchKernelGGL(k_erode_keep, gf, dim3(256), 0, hs, g->faces, alive, g->nf, (const int32_t*)cnt, min_neighbors);
  }
  hipLaunchKernelGGL(k_erode_mark, gf, dim3(256), 0, hs, g->faces, (const uint8_t*)alive, g->nf, non_eroded);
  OFX_LAUNCH_CHECK();
  dfree(alive, hs);
  dfree(cnt, hs);
  return OFX_OK;
}

int ofx_sample_nodes(void* handle, const uint8_t* non_eroded, float node_coverage, int32_t use_only_non_eroded,
                     float* node_positions, int32_t* node_indices, int64_t* n_nodes, int64_t* n_rounds,
                     ofx_stream_t s) {
  Graph* g = (Graph*)handle;
  OFX_CHECK_ARG(g && node_positions && node_indices && n_nodes, "null argument");
  OFX_CHECK_ARG(node_coverage > 0.f, "node_coverage must be > 0");
  OFX_CHECK_ARG(!use_only_non_eroded || non_eroded, "non_eroded mask required");
  hipStream_t hs = as_stream(s);
  const int64_t nv = g->nv;
  *n_nodes = 0;
  if (n_rounds) *n_rounds = 0;
  if (nv == 0) return OFX_OK;
  uint8_t *elig = nullptr, *is_node = nullptr;
  int32_t* state = nullptr;
  uint32_t *key = nullptr, *key2 = nullptr;
  int32_t *val = nullptr, *sorted = nullptr, *bstart = nullptr, *bend = nullptr, *cnt = nullptr, *list = nullptr;
  int32_t *rank = nullptr, *und = nullptr;
  int64_t *off = nullptr, *cursor = nullptr;
  uint32_t tsize = 1;
  while (tsize < 2 * nv) tsize <<= 1;
  OFX_CHECKS(dalloc(&elig, nv, hs));
  if (use_only_non_eroded) OFX_HIP(hipMemcpyAsync(elig, non_eroded, nv, hipMemcpyDeviceToDevice, hs));
  else OFX_HIP(hipMemsetAsync(elig, 1, nv, hs));
  OFX_CHECKS(dalloc(&key, nv, hs));
  OFX_CHECKS(dalloc(&key2, nv, hs));
  OFX_CHECKS(dalloc(&val, nv, hs));
  OFX_CHECKS(dalloc(&sorted, nv, hs));
  OFX_CHECKS(dalloc(&bstart, tsize, hs));
  OFX_CHECKS(dalloc(&bend, tsize, hs));
  OFX_HIP(hipMemsetAsync(bstart, 0, tsize * sizeof(int32_t), hs));
  OFX_HIP(hipMemsetAsync(bend, 0, tsize * sizeof(int32_t), hs));
  // cells a little larger than the coverage so every conflicting pair lies in adjacent cells despite rounding
  Grid gr{1.f / (node_coverage * 1.01f), tsize - 1};
  const float cov2 = node_coverage * node_coverage;
  const dim3 gv(grid_for(nv, 256, 1 << 30));
  hipLaunchKernelGGL(k_sn_keys, gv, dim3(256), 0, hs, g->P, (const uint8_t*)elig, nv, gr, key, val);
  size_t tmp = 0;
  OFX_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, key, key2, val, sorted, (int)nv, 0, 32, hs));
  void* t = nullptr;
  OFX_HIP(hipMallocAsync(&t, std::max<size_t>(tmp, 1), hs));
  OFX_HIP(hipcub::DeviceRadixSort::SortPairs(t, tmp, key, key2, val, sorted, (int)nv, 0, 32, hs));
  OFX_HIP(hipFreeAsync(t, hs));
  hipLaunchKernelGGL(k_sn_bounds, gv, dim3(256), 0, hs, (const uint32_t*)key2, nv, bstart, bend);
  // the greedy form when the bitmap fits one workgroup's LDS (1.28M vertices), else the parallel rounds
  const int64_t nwords = (nv + 31) >> 5;
  const bool greedy = nwords <= kGreedyMaxWords && !getenv("OFX_SN_ROUNDS");
  OFX_CHECKS(dalloc(&state, nv, hs));
  OFX_HIP(hipMemsetAsync(state, 0, nv * sizeof(int32_t), hs));
  constexpr int kChunk = 32;
  int64_t rounds = 0, nr = 0;
  if (greedy) {
    float4* spos = nullptr;
    int64_t* steps = nullptr;
    const bool stamp = getenv("OFX_SN_STAMPS") != nullptr;   // tuning: per-phase times to stderr
    OFX_CHECKS(dalloc(&spos, nv, hs));
    OFX_CHECKS(dalloc(&steps, 8, hs));
    hipLaunchKernelGGL(k_sn_spos, gv, dim3(256), 0, hs, g->P, (const int32_t*)sorted, nv, spos);
    const size_t lds = (size_t)nwords * sizeof(uint32_t);
    OFX_HIP(hipFuncSetAttribute((const void*)k_sn_greedy, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_sn_greedy, dim3(1), dim3(kGreedyThreads), lds, hs, g->P, (const uint8_t*)elig, nv, gr,
                       (const int32_t*)bstart, (const int32_t*)bend, (const float4*)spos, cov2, state, steps,
                       stamp ? steps + 1 : nullptr);
    OFX_LAUNCH_CHECK();
    OFX_CHECKS(read1(steps, &g->sn_steps, hs));
    if (stamp) {
      int64_t st[7];
      OFX_HIP(hipMemcpy(st, steps + 1, sizeof(st), hipMemcpyDeviceToHost));
      fprintf(stderr, "k_sn_greedy: %lld steps; find+resolve %.1f us (find %.1f, positions+conflicts %.1f, "
              "resolve %.1f), ranges+scan %.1f us, clear %.1f us (100 MHz clock); %lld positions tested\n",
              (long long)g->sn_steps, st[0] * 1e-2, st[4] * 1e-2, st[5] * 1e-2, st[6] * 1e-2, st[1] * 1e-2,
              st[2] * 1e-2, (long long)st[3]);
    }
    dfree(spos, hs);
    dfree(steps, hs);
  } else {
  OFX_CHECKS(dalloc(&cnt, nv + 1, hs));
  OFX_HIP(hipMemsetAsync(cnt, 0, (nv + 1) * sizeof(int32_t), hs));
  hipLaunchKernelGGL(k_sn_conflicts<false>, gv, dim3(256), 0, hs, g->P, (const uint8_t*)elig, nv, gr,
                     (const int32_t*)bstart, (const int32_t*)bend, (const int32_t*)sorted, cov2, cnt,
                     (const int64_t*)nullptr, (int32_t*)nullptr);
  OFX_CHECKS(dalloc(&off, nv + 1, hs));
  OFX_CHECKS(exclusive_sum_i32_to_i64(cnt, off, nv + 1, hs));
  int64_t total = 0;
  OFX_CHECKS(read1(off + nv, &total, hs));
  OFX_CHECKS(dalloc(&list, std::max<int64_t>(total, 1), hs));
  hipLaunchKernelGGL(k_sn_conflicts<true>, gv, dim3(256), 0, hs, g->P, (const uint8_t*)elig, nv, gr,
                     (const int32_t*)bstart, (const int32_t*)bend, (const int32_t*)sorted, cov2, cnt,
                     (const int64_t*)off, list);
  OFX_CHECKS(dalloc(&cursor, nv, hs));
  OFX_HIP(hipMemcpyAsync(cursor, off, nv * sizeof(int64_t), hipMemcpyDeviceToDevice, hs));
  OFX_CHECKS(dalloc(&und, kChunk, hs));
  {
    int32_t* err = und;   // reused: zeroed below before the rounds
    OFX_HIP(hipMemsetAsync(err, 0, sizeof(int32_t), hs));
    int dev = 0, ncu = 256;
    OFX_HIP(hipGetDevice(&dev));
    OFX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipLaunchKernelGGL(k_sn_persistent, dim3(2 * ncu), dim3(256), 0, hs, (const uint8_t*)elig, nv, (const int64_t*)off,
                       (const int32_t*)list, cursor, state, (int64_t)1 << 22, err);
    OFX_LAUNCH_CHECK();
    int32_t herr = 0;
    OFX_CHECKS(read1(err, &herr, hs));
    rounds = herr ? -1 : 0;      // -1: the persistent pass timed out; the round form finishes
  }
  for (;;) {
    OFX_HIP(hipMemsetAsync(und, 0, kChunk * sizeof(int32_t), hs));
    for (int r = 0; r < kChunk; ++r)
      hipLaunchKernelGGL(k_sn_round, gv, dim3(256), 0, hs, (const uint8_t*)elig, nv, (const int64_t*)off,
                         (const int32_t*)list, cursor, state, und + r);
    OFX_LAUNCH_CHECK();
    int32_t h[kChunk];
    OFX_HIP(hipMemcpyAsync(h, und, sizeof(h), hipMemcpyDeviceToHost, hs));
    OFX_HIP(hipStreamSynchronize(hs));
    int r = 0;
    while (r < kChunk && h[r] != 0) ++r;
    nr += (r < kChunk) ? r + 1 : kChunk;
    if (r < kChunk) break;
    if (nr > nv + kChunk) { set_error("sample_nodes did not converge"); return OFX_ERR_STATE; }
  }
  }
  OFX_CHECKS(dalloc(&is_node, nv + 1, hs));
  OFX_CHECKS(dalloc(&rank, nv + 1, hs));
  OFX_HIP(hipMemsetAsync(is_node + nv, 0, 1, hs));
  hipLaunchKernelGGL(k_sn_flags, gv, dim3(256), 0, hs, (const int32_t*)state, (const uint8_t*)elig, nv, is_node);
  OFX_CHECKS(exclusive_sum_u8(is_node, rank, nv + 1, hs));
  hipLaunchKernelGGL(k_sn_emit, gv, dim3(256), 0, hs, g->P, (const uint8_t*)is_node, (const int32_t*)rank, nv,
                     node_positions, node_indices);
  OFX_LAUNCH_CHECK();
  int32_t nn = 0;
  OFX_CHECKS(read1(rank + nv, &nn, hs));
  *n_nodes = nn;
  // greedy form: its batches (<= nodes); rounds form: launches of the round kernel after the persistent pass
  // (negative: the persistent pass timed out)
  if (n_rounds) *n_rounds = greedy ? g->sn_steps : (rounds < 0 ? -nr : nr);
  for (void* p : {(void*)elig, (void*)state, (void*)is_node, (void*)key, (void*)key2, (void*)val, (void*)sorted,
                  (void*)bstart, (void*)bend, (void*)cnt, (void*)list, (void*)rank, (void*)und, (void*)off,
                  (void*)cursor})
    dfree(p, hs);
  return OFX_OK;
}

int ofx_edges_geodesic(void* handle, const uint8_t* valid_vertices, const int32_t* node_indices, int32_t n_nodes,
                       int32_t n_max_neighbors, float node_coverage, int32_t allow_only_valid_vertices,
                       int32_t enforce_total_num_neighbors, int32_t* graph_edges, float* graph_edges_weights,
                       float* graph_edges_distances, float* node_to_vertex_distances, ofx_stream_t s) {
  Graph* g = (Graph*)handle;
  OFX_CHECK_ARG(g && n_nodes >= 0, "bad arguments");
  OFX_CHECK_ARG(n_max_neighbors >= 1 && n_max_neighbors <= 16, "n_max_neighbors must be in [1, 16]");
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(node_indices && graph_edges && graph_edges_weights && graph_edges_distances, "null buffer");
  hipStream_t hs = as_stream(s);
  const int64_t nv = g->nv;
  int32_t *v2n = nullptr, *status = nullptr, *todo = nullptr;
  OFX_CHECKS(dalloc(&v2n, nv, hs));
  OFX_HIP(hipMemsetAsync(v2n, 0xFF, std::max<int64_t>(nv, 1) * sizeof(int32_t), hs));
  hipLaunchKernelGGL(k_v2n, dim3(grid_for(n_nodes, 256)), dim3(256), 0, hs, node_indices, n_nodes, nv, v2n);
  if (node_to_vertex_distances)
    hipLaunchKernelGGL(k_fill_f32, dim3(grid_for((int64_t)n_nodes * nv, 256, 65536)), dim3(256), 0, hs,
                       node_to_vertex_distances, (int64_t)n_nodes * nv, -1.f);
  OFX_CHECKS(dalloc(&status, n_nodes, hs));
  OFX_CHECKS(dalloc(&todo, n_nodes, hs));
  std::vector<int32_t> h_todo(n_nodes);
  for (int i = 0; i < n_nodes; ++i) h_todo[i] = i;
  GeoArgs a{};
  a.P = g->P; a.valid = valid_vertices; a.rowptr = g->rowptr; a.col = g->col; a.v2n = v2n; a.node_idx = node_indices;
  a.n_nodes = n_nodes; a.K = n_max_neighbors; a.nv = nv; a.cov = node_coverage;
  a.max_inf = 2.f * node_coverage;
  a.two_c2 = (2.f * node_coverage) * node_coverage;
  a.only_valid = allow_only_valid_vertices; a.enforce = enforce_total_num_neighbors;
  a.edges = graph_edges; a.wts = graph_edges_weights; a.dists = graph_edges_distances; a.n2v = node_to_vertex_distances;
  a.status = status;
  if (!getenv("OFX_GEO_SEQ")) {   // parallel form; ties go sequential, overfull neighbourhoods to the big table
    std::vector<int32_t> rest, big;
    const bool big_only = getenv("OFX_GEO_BIG") != nullptr;   // tuning/test: every node on the 16384-slot form
    if (big_only)
      for (int32_t n = 0; n < n_nodes; ++n) big.push_back(n);
    for (int tier = big_only ? 1 : 0; tier < 2; ++tier) {
      int32_t n_run = tier == 0 ? n_nodes : (int32_t)big.size();
      if (n_run == 0) break;
      if (tier == 0) {
        hipLaunchKernelGGL(k_geo_relax<8192>, dim3((unsigned)n_run), dim3(geo::kThreads), 0, hs, a,
                           (const int32_t*)nullptr, n_run);
      } else {
        OFX_HIP(hipMemcpyAsync(todo, big.data(), big.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
        hipLaunchKernelGGL(k_geo_relax<16384>, dim3((unsigned)n_run), dim3(geo::kThreads), 0, hs, a,
                           (const int32_t*)todo, n_run);
      }
      OFX_LAUNCH_CHECK();
      std::vector<int32_t> st(n_nodes);
      OFX_HIP(hipMemcpyAsync(st.data(), status, n_nodes * sizeof(int32_t), hipMemcpyDeviceToHost, hs));
      OFX_HIP(hipStreamSynchronize(hs));
      std::vector<int32_t> ran;
      if (tier == 0) { ran.resize(n_nodes); for (int32_t n = 0; n < n_nodes; ++n) ran[n] = n; }
      else ran = big;
      big.clear();
      for (int32_t n : ran) {
        if (st[n] == geo::kInvalid) {
          dfree(v2n, hs); dfree(status, hs); dfree(todo, hs);
          set_error("compute_edges_geodesic: node %d reached an invalid vertex (the reference exits)", n);
          return OFX_ERR_STATE;
        }
        if (st[n] == geo::kTie || (st[n] == geo::kFull && tier == 1)) rest.push_back(n);
        else if (st[n] == geo::kFull) big.push_back(n);
      }
    }
    std::sort(rest.begin(), rest.end());
    g->geo_sequential = (int64_t)rest.size();
    h_todo.swap(rest);
  } else {
    g->geo_sequential = n_nodes;
  }
  const int64_t words = (nv + 31) / 32;
  int64_t cap = 8192;
  while (!h_todo.empty()) {
    // batch so that visited bitmaps + heaps stay within ~1 GiB
    const int64_t per = words * 4 + cap * (int64_t)sizeof(HeapEnt);
    const int64_t batch = std::max<int64_t>(1, std::min<int64_t>((int64_t)h_todo.size(), (1ll << 30) / per));
    OFX_HIP(hipMemcpyAsync(todo, h_todo.data(), h_todo.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
    OFX_CHECKS(dalloc(&a.visited, batch * words, hs));
    OFX_CHECKS(dalloc(&a.heap, batch * cap, hs));
    a.cap = cap;
    a.status = status;
    for (int64_t b0 = 0; b0 < (int64_t)h_todo.size(); b0 += batch) {
      const int64_t nb = std::min<int64_t>(batch, (int64_t)h_todo.size() - b0);
      OFX_HIP(hipMemsetAsync(a.visited, 0, nb * words * sizeof(uint32_t), hs));
      hipLaunchKernelGGL(k_geodesic, dim3((unsigned)((nb + 63) / 64)), dim3(64), 0, hs, a, (const int32_t*)(todo + b0),
                         (int32_t)nb);
      OFX_LAUNCH_CHECK();
    }
    std::vector<int32_t> st(n_nodes);
    OFX_HIP(hipMemcpyAsync(st.data(), status, n_nodes * sizeof(int32_t), hipMemcpyDeviceToHost, hs));
    OFX_HIP(hipStreamSynchronize(hs));
    dfree(a.visited, hs);
    dfree(a.heap, hs);
    std::vector<int32_t> again;
    for (int32_t n : h_todo) {
      if (st[n] == 2) {
        dfree(v2n, hs); dfree(status, hs); dfree(todo, hs);
        set_error("compute_edges_geodesic: node %d reached an invalid vertex (the reference exits)", n);
        return OFX_ERR_STATE;
      }
      if (st[n] == 1) again.push_back(n);
    }
    h_todo.swap(again);
    if (!h_todo.empty()) {
      if (cap >= (int64_t)1 << 34) { set_error("geodesic heap capacity exhausted"); return OFX_ERR_RANGE; }
      cap *= 16;
      // a rerun node restarts from scratch: its n2v row may hold partial distances
      if (node_to_vertex_distances)
        for (int32_t n : h_todo)
          hipLaunchKernelGGL(k_fill_f32, dim3(grid_for(nv, 256, 4096)), dim3(256), 0, hs,
                             node_to_vertex_distances + (int64_t)n * nv, nv, -1.f);
    }
  }
  dfree(v2n, hs);
  dfree(status, hs);
  dfree(todo, hs);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_graph_downsample(const float* node_positions, int32_t n_nodes, double node_coverage, int32_t* down_idx,
                         int32_t* up_idx, int32_t* n_down, ofx_stream_t s) {
  OFX_CHECK_ARG(n_nodes >= 0 && n_down, "bad arguments");
  *n_down = 0;
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(node_positions && down_idx && up_idx, "null buffer");
  hipStream_t hs = as_stream(s);
  int32_t* nd = nullptr;
  OFX_CHECKS(dalloc(&nd, 1, hs));
  hipLaunchKernelGGL(k_downsample, dim3(1), dim3(kDsThreads), 0, hs, node_positions, n_nodes, node_coverage, down_idx,
                     up_idx, nd);
  OFX_LAUNCH_CHECK();
  int32_t h = 0;
  OFX_CHECKS(read1(nd, &h, hs));
  dfree(nd, hs);
  if (h > kDsMax) {
    set_error("graph_downsample: more than %d kept nodes", kDsMax);
    return OFX_ERR_RANGE;
  }
  *n_down = h;
  return OFX_OK;
}

int ofx_edges_euclidean(const float* node_positions, int32_t n_nodes, int32_t n_max_neighbors, int32_t* graph_edges,
                        ofx_stream_t s) {
  OFX_CHECK_ARG(n_nodes >= 0 && n_max_neighbors >= 1 && n_max_neighbors <= 16, "bad arguments");
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(node_positions && graph_edges, "null buffer");
  hipLaunchKernelGGL(k_edges_euclid, dim3(grid_for(n_nodes, 256)), dim3(256), 0, as_stream(s), node_positions, n_nodes,
                     n_max_neighbors, graph_edges);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_node_edge_cleanup(const int32_t* graph_edges, int32_t n_nodes, int32_t max_neighbors, const uint8_t* valid_in,
                          uint8_t* valid_out, ofx_stream_t s) {
  OFX_CHECK_ARG(n_nodes >= 0 && max_neighbors >= 0, "bad arguments");
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(graph_edges && valid_in && valid_out, "null buffer");
  hipStream_t hs = as_stream(s);
  uint8_t* removed = nullptr;
  int32_t* changed = nullptr;
  OFX_CHECKS(dalloc(&removed, n_nodes, hs));
  OFX_CHECKS(dalloc(&changed, 1, hs));
  OFX_HIP(hipMemsetAsync(removed, 0, n_nodes, hs));
  const dim3 gn(grid_for(n_nodes, 256));
  for (int it = 0; it <= n_nodes; ++it) {
    OFX_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), hs));
    hipLaunchKernelGGL(k_cleanup_sweep, gn, dim3(256), 0, hs, graph_edges, n_nodes, max_neighbors, valid_in, removed, changed);
    OFX_LAUNCH_CHECK();
    int32_t c = 0;
    OFX_CHECKS(read1(changed, &c, hs));
    if (c == 0) break;
  }
  hipLaunchKernelGGL(k_cleanup_out, gn, dim3(256), 0, hs, valid_in, (const uint8_t*)removed, n_nodes, valid_out);
  OFX_LAUNCH_CHECK();
  dfree(removed, hs);
  dfree(changed, hs);
  return OFX_OK;
}

int ofx_compute_clusters(const int32_t* graph_edges, int32_t n_nodes, int32_t max_neighbors, int32_t* clusters,
                         int32_t* cluster_sizes, int32_t* n_clusters, ofx_stream_t s) {
  OFX_CHECK_ARG(n_nodes >= 0 && max_neighbors >= 0 && n_clusters, "bad arguments");
  *n_clusters = 0;
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(graph_edges && clusters, "null buffer");
  hipStream_t hs = as_stream(s);
  int32_t *lab = nullptr, *changed = nullptr, *rank = nullptr;
  uint8_t* root = nullptr;
  OFX_CHECKS(dalloc(&lab, n_nodes, hs));
  OFX_CHECKS(dalloc(&changed, 1, hs));
  OFX_CHECKS(dalloc(&rank, n_nodes + 1, hs));
  OFX_CHECKS(dalloc(&root, n_nodes + 1, hs));
  const dim3 gn(grid_for(n_nodes, 256));
  hipLaunchKernelGGL(k_cc_init, gn, dim3(256), 0, hs, lab, n_nodes);
  for (int it = 0; it <= 2 * n_nodes + 2; ++it) {
    OFX_HIP(hipMemsetAsync(changed, 0, sizeof(int32_t), hs));
    hipLaunchKernelGGL(k_cc_hook, gn, dim3(256), 0, hs, graph_edges, n_nodes, max_neighbors, lab, changed);
    for (int j = 0; j < 4; ++j) hipLaunchKernelGGL(k_cc_jump, gn, dim3(256), 0, hs, lab, n_nodes, changed);
    OFX_LAUNCH_CHECK();
    int32_t c = 0;
    OFX_CHECKS(read1(changed, &c, hs));
    if (c == 0) break;
  }
  OFX_HIP(hipMemsetAsync(root + n_nodes, 0, 1, hs));
  hipLaunchKernelGGL(k_cc_roots, gn, dim3(256), 0, hs, (const int32_t*)lab, n_nodes, root);
  OFX_CHECKS(exclusive_sum_u8(root, rank, n_nodes + 1, hs));
  if (cluster_sizes) OFX_HIP(hipMemsetAsync(cluster_sizes, 0, n_nodes * sizeof(int32_t), hs));
  hipLaunchKernelGGL(k_cc_out, gn, dim3(256), 0, hs, (const int32_t*)lab, (const int32_t*)rank, n_nodes, clusters,
                     cluster_sizes);
  OFX_LAUNCH_CHECK();
  int32_t nc = 0;
  OFX_CHECKS(read1(rank + n_nodes, &nc, hs));
  *n_clusters = nc;
  dfree(lab, hs); dfree(changed, hs); dfree(rank, hs); dfree(root, hs);
  return OFX_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ get_reduced_graph
namespace ofx {

// numpy's float32 np.sum of a contiguous row of n <= 16 (pairwise_sum: < 8 in order, else 8 partials)
__device__ __forceinline__ float np_sum_f32(const float* a, int n) {
  if (n < 8) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += a[i];
    return s;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i + 8 <= n; i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) s += a[i];
  return s;
}

// one thread per kept node (embedded_deformation_graph.py:382-477)
__global__ __launch_bounds__(256) void k_reduce_graph(const uint8_t* __restrict__ valid, const int32_t* __restrict__ new_id,
                                                      int n_nodes, int K, const float* __restrict__ nodes,
                                                      const int32_t* __restrict__ E, const float* __restrict__ W,
                                                      const float* __restrict__ D, const int32_t* __restrict__ C,
                                                      int any_removed, float* __restrict__ nodes_o, int32_t* __restrict__ E_o,
                                                      float* __restrict__ W_o, float* __restrict__ D_o,
                                                      int32_t* __restrict__ C_o) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_nodes || !valid[n]) return;
  const int r = new_id[n];
  for (int c = 0; c < 3; ++c) nodes_o[3 * (int64_t)r + c] = nodes[3 * (int64_t)n + c];
  if (C_o) C_o[r] = C ? C[n] : -1;
  float w[16];
  int c = 0;
  for (int i = 0; i < K; ++i) { E_o[(int64_t)r * K + i] = -1; w[i] = 0.f; D_o[(int64_t)r * K + i] = 0.f; }
  for (int i = 0; i < K; ++i) {
    const int32_t j = E[(int64_t)n * K + i];
    if (!any_removed) {
      E_o[(int64_t)r * K + i] = j;
      w[i] = W[(int64_t)n * K + i];
      D_o[(int64_t)r * K + i] = D[(int64_t)n * K + i];
      continue;
    }
    if (j >= 0 && j < n_nodes && !valid[j]) continue;          // neighbour on the black list: dropped
    E_o[(int64_t)r * K + c] = (j == -1) ? -1 : new_id[j];
    w[c] = W[(int64_t)n * K + i];
    D_o[(int64_t)r * K + c] = D[(int64_t)n * K + i];
    ++c;
  }
  if (any_removed) {
    const float s = np_sum_f32(w, K);
    // numpy 1.26 (environment.yml:94): f32 scalar + 1e-6 promotes to f64, the in-place f32 division casts back
    if (s > 0.f) {
      const float den = (float)((double)s + 1e-6);
      for (int i = 0; i < K; ++i) w[i] = (float)((double)w[i] / (double)den);
    }
  }
  for (int i = 0; i < K; ++i) W_o[(int64_t)r * K + i] = w[i];
}

}  // namespace ofx

extern "C" int ofx_reduce_graph(const uint8_t* valid_nodes_mask, int32_t n_nodes, int32_t max_neighbors,
                                const float* nodes, const int32_t* edges, const float* edges_weights,
                                const float* edges_distances, const int32_t* clusters, float* nodes_out,
                                int32_t* edges_out, float* weights_out, float* distances_out, int32_t* clusters_out,
                                int32_t* n_kept, ofx_stream_t s) {
  using namespace ofx;
  OFX_CHECK_ARG(n_nodes >= 0 && max_neighbors >= 1 && max_neighbors <= 16 && n_kept, "bad arguments");
  *n_kept = 0;
  if (n_nodes == 0) return OFX_OK;
  OFX_CHECK_ARG(valid_nodes_mask && nodes && edges && edges_weights && edges_distances && nodes_out && edges_out &&
                    weights_out && distances_out, "null buffer");
  hipStream_t hs = as_stream(s);
  int32_t* new_id = nullptr;
  OFX_CHECKS(dalloc(&new_id, n_nodes + 1, hs));
  OFX_CHECKS(exclusive_sum_u8(valid_nodes_mask, new_id, n_nodes, hs));
  int32_t last = 0;
  uint8_t lastv = 0;
  OFX_HIP(hipMemcpyAsync(&last, new_id + n_nodes - 1, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipMemcpyAsync(&lastv, valid_nodes_mask + n_nodes - 1, 1, hipMemcpyDeviceToHost, hs));
  OFX_HIP(hipStreamSynchronize(hs));
  const int32_t kept = last + (lastv ? 1 : 0);
  *n_kept = kept;
  hipLaunchKernelGGL(k_reduce_graph, dim3(grid_for(n_nodes, 256)), dim3(256), 0, hs, valid_nodes_mask,
                     (const int32_t*)new_id, n_nodes, max_neighbors, nodes, edges, edges_weights, edges_distances,
                     clusters, kept < n_nodes ? 1 : 0, nodes_out, edges_out, weights_out, distances_out, clusters_out);
  OFX_LAUNCH_CHECK();
  dfree(new_id, hs);
  return OFX_OK;
}
