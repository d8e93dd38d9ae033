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
// MI355X design.
//  * Every residual row-triple is a "term" (data: 4 anchored nodes, ARAP edge: 2, motion: 1). Once per GN
//    iteration k_terms writes each term's compact record (kRec doubles: the per-anchor vectors and the
//    term's shared scalars, not its four 3x6 Jacobian blocks); the assembly expands a record into the
//    blocks it needs with the same arithmetic, so A and b are the bits the blocks themselves gave.
//  * JᵀJ lives as 6x6 f64 blocks in BSR over the node adjacency (diagonal, edges, co-anchored
//    pairs). Per solve, each block gets a sorted list of the (term, p, q) products that land on it,
//    so assembly is a deterministic gather: one wave per block, lane = block entry (k_blocks); the
//    rhs is the same per node entry (k_rhs). No atomics -> bitwise reproducible A and b.
//  * Node order: setup groups the nodes into clusters of <= kCS graph neighbours (host BFS over the
//    ED graph, first-fit packed into groups of exactly kCS rows, padded with decoupled dummy nodes),
//    and permutes every node-indexed array into that order; k_finish permutes the result back.
//  * PCG: pipelined (Ghysels-Vanroose) with a cluster block-Jacobi preconditioner (explicit inverse
//    of each damped 48x48 cluster diagonal block), ONE kernel per iteration: SpMV + all recurrences
//    + the cluster M⁻¹ (wave-local: one cluster = one wave's rows) + the three dot products. Scalars
//    never leave the device: each launch writes per-wave partial sums and every wave of the NEXT
//    launch re-derives the same scalars from them in a fixed order (kernel boundaries give
//    visibility; no fences, no tickets, no atomics). The host only polls convergence in chunks
//    sized from the previous frame's count for the same GN step.
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <array>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>
#include <utility>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "ofx_common.h"

namespace ofx {

// --------------------------------------------------------------------------------------------
constexpr int kBlk = 256;       // threads per WG
#ifndef OFX_KPROJ   // (tuning builds: -DOFX_KPROJ=<n>)
#define OFX_KPROJ 4
#endif
constexpr int kProj = OFX_KPROJ;   // warm start: Galerkin projection on the last kProj GN-step solutions
constexpr int kProjP = kProj * (kProj + 1) / 2 + kProj;   // projection partial streams (Gram upper triangle + Xᵀb)
constexpr int kCS = 8;        // nodes per preconditioner cluster (= PCG rows per wave)
constexpr int kMaxNodes = 8192;   // dense slot map of (2·max_nodes + kCS)² entries
// Overlapping additive Schwarz (as_on): the ring of a cluster holds its kAsRing A-neighbours with the most coupling terms,
// and a row joins at most kAsX rings, so an output cluster has at most kAsSrc contributing subdomains and kAsRS row
// segments (a kAsD-entry inverse row each); kAsGat >= kAsSrc·kAsDN rounded up to whole passes of the apply's 192
#ifndef OFX_AS_RING   // (tuning builds: -DOFX_AS_RING=<n>; 12 -> 16: 198 -> 158 PCG iterations per bench frame, +10 %)
#define OFX_AS_RING 16
#endif
constexpr int kAsRing = OFX_AS_RING, kAsX = 3, kAsDN = kCS + kAsRing, kAsD = 6 * kAsDN, kAsK = kAsD / 8,
              kAsSrc = 1 + kCS * kAsX, kAsRS = 6 * kCS * (1 + kAsX),
              kAsGat = (kAsSrc * kAsDN + kAsRS - 1) / kAsRS * kAsRS, kAsMeta = 64 + kAsRS;
// One launch per Schwarz PCG iteration (k_as_iter, round 6): per subdomain a table of its rows' blocks (<= kAsDN rows of
// <= kRowMax blocks), the columns they touch (S2, <= kGS nodes) with the <= 1 + kAsX subdomain contributions that sum to m
// there, and the scaled inverse rows in subdomain order (the "tab" buffer, AsTab below)
constexpr int kGB = 512, kGS = 480, kGRow = 96;
constexpr int kAsIterT = 1024;   // k_as_iter's threads: blocks 0..511, S2 nodes from 512, the row waves 13..15
static_assert(kAsSrc * kAsDN <= kAsGat && kAsD % 8 == 0 && kAsD <= 144, "Schwarz tables");

// Everything the kernels read: trivially copyable, passed by value as the kernel argument (host-only
// members live in Gn below, so a launch copies these bytes and nothing else).
struct GnDev {
  int max_nodes = 0, max_matches = 0;
  int N = 0, M = 0, NB = 0;    // N: PCG rows (nodes in cluster order, padded to whole clusters)
  int N_real = 0;              // caller's node count
  int max_pad = 0;             // capacity of the node-indexed arrays (2·max_nodes + kCS)
  int32_t *perm = nullptr;     // row -> caller node (-1: padding), N entries
  int32_t *iperm = nullptr;    // caller node -> row, N_real entries
  int64_t T = 0;        // terms = M + N*NB + N
  ofx_gn_params prm{};
  float fx = 0, fy = 0, cx = 0, cy = 0;
  // problem (f64 device copies)
  double *nodes = nullptr, *tpos = nullptr, *conf = nullptr, *src = nullptr, *wts = nullptr, *tgt = nullptr,
         *tpx = nullptr, *tpy = nullptr, *ew = nullptr;
  int32_t *anc = nullptr, *edges = nullptr;
  // terms
  int32_t* term_node = nullptr;  // T*4, -1 = unused entry
  double* J = nullptr;           // T·kRec term records (k_terms)
  double* res = nullptr;         // T*3
  int64_t T_cap = 0;
  // pattern + contribution lists
  int32_t *map = nullptr, *row_ptr = nullptr, *col = nullptr, *row_cnt = nullptr;   // row_cnt[N]: max row length
  int2* wl = nullptr;            // per PCG wave: its first kWL blocks' columns and packed row bounds (k_wave_list)
  double* Aw = nullptr;          // per PCG wave: its kWL blocks of the operator, [wave][18][kWL] 16-B words (k_pcg_w0)
  int max_deg = 0;               // longest block row of the pattern
  int max_wave = 0;              // most blocks of one PCG wave (kCS rows)
  int32_t* stopw = nullptr;      // per PCG wave and lane: the epoch of the last converged (or stopped) PCG solve
  int32_t ep = 0;                // epoch of the current PCG solve (one per GN step, increasing per handle)
  uint64_t* stamps = nullptr;    // tuning builds (-DOFX_STAMPS): per iteration < 64 and wave, 8 clock stamps
  int32_t* blk_row = nullptr;    // block -> row (clears the slot map's pattern at the next setup)
  float* d_gnodes = nullptr;      // device copy of the graph the row order was built for (optimistic check)
  int32_t* d_gedges = nullptr;
  int32_t* d_gdiff = nullptr;
  int64_t gcap_n = 0, gcap_e = 0;
  int pat_N = 0;                 // N and block count of the pattern currently set in `map`
  int64_t pat_nnzb = 0;
  int64_t ne_cap = 0;            // capacity of edges / ew
  // contribution lists of the UPPER blocks only (col >= row, indexed u = up_of[slot]): the assembly computes each
  // upper block once and also stores its transpose at up_tr[u], so A is exactly symmetric. (A separate gather of the
  // lower block (j, i) would sum the same products in the same order only when no node repeats within a term; with
  // a repeated anchor its last bits could differ from the transpose.)
  int32_t *blk_off = nullptr, *blk_cnt = nullptr, *blk_list = nullptr, *blk_tmp = nullptr;
  int32_t *up_of = nullptr, *up_slot = nullptr, *up_tr = nullptr;   // slot -> u (+ total at [nnzb]), u -> slot, transpose
  int32_t *node_off = nullptr, *node_cnt = nullptr, *node_list = nullptr, *node_tmp = nullptr;
  // the first chunk of every assembly workgroup's list (kCoop codes) and of every node's rhs list (128), at fixed
  // offsets (k_first_codes): k_assemble's first memory trip carries them
  int32_t *blk_first = nullptr, *node_first = nullptr;
  int64_t nnzb = 0, nnzb_cap = 0;
  // state
  double *R = nullptr, *t = nullptr;
  double* racc = nullptr;        // per row: Σ|ω| of the GN steps since its cluster inverse was built (precond_rot_tol)
  int32_t gn_iter_now = 0;       // GN step of the current PCG solve
  double *A_own = nullptr, *rhs_own = nullptr;
  float* Mcl = nullptr;           // cluster inverses, f32, per cluster 48x48 in the lane-interleaved order of mcl_idx
  const double* Aop = nullptr;    // PCG operator (the damped A of the current step)
  double *st = nullptr;          // PCG recurrence state, 6N records of 8 (see the PCG layout note)
  double *m0 = nullptr, *m1 = nullptr;   // double-buffered m = M⁻¹w (gathered by the SpMV)
  double *pcg_alpha = nullptr, *pcg_gamma = nullptr;   // [-, -, 1/x of parity 0, 1] (+ alpha: [4 + par] = thr)
  // pcg_alpha, pcg_gamma, scal, sturm and flags live in ONE allocation at fixed offsets (kSc*), so the PCG iteration
  // reaches all of them through one preloaded pointer argument (no kernel-argument fetch ahead of their loads)
  double* pcs = nullptr;
  double2* sturm = nullptr;       // error-based PCG stop (k_pcg_iter): 64 shifted LDLᵀ pivots + counts
  double *part_p = nullptr, *part_b = nullptr, *part_loss = nullptr;
  int32_t nwg_row = 0, nwg_node = 0, nwg_terms = 0;   // nwg_row: PCG row waves (= workgroups)
  int32_t nw_pad = 0;            // stride of the iteration partial streams: 128·pcg_ku, zero beyond nwg_row
  int32_t pcg_w2 = 1;            // two waves per cluster in k_pcg_iter (OFX_PCG_W1=1: one)
  int32_t pcg_ku = 3;            // partial pairs per lane and stream in k_pcg_iter (pcg_ku_for)
  // overlapping additive Schwarz preconditioner (as_on): subdomain D_c = cluster c's kCS rows + up to kAsRing
  // ring rows; the setup's tables (k_as_choose .. k_as_segments) and the prep's inverses (k_as_invert), applied by
  // k_as_apply between two PCG iteration launches
  int32_t as_on = 0;
  int32_t *as_cand = nullptr, *as_csc = nullptr, *as_acc = nullptr;   // [cluster][kAsRing]: ring candidates, terms, kept
  int32_t* as_dom = nullptr;     // [cluster][kAsDN]: the subdomain's rows (own rows first, -1 = none)
  int32_t* as_meta = nullptr;    // [cluster][kAsMeta]: segment count, source count, row offsets, segment -> source slot
  int32_t* as_gat = nullptr;     // [cluster][kAsGat]: rows gathered into the apply's LDS image (source slot · kAsDN + l)
  int32_t* as_dst = nullptr;     // [cluster][kAsD]: subdomain row -> (output cluster · kAsRS + segment)
  uint16_t* as_slab = nullptr;   // [cluster][kAsK][kAsRS] x 8 fp16: the segments' scaled inverse rows, segment-minor
  int32_t* as_src = nullptr;     // [cluster][kAsSrc]: the apply's source subdomains
  float* as_dsc = nullptr;       // [cluster][kAsD]: the subdomain inverse's scales d = √diag(Z) (k_as_invert)
  float* as_rsc = nullptr;       // [cluster][kAsRS]: the segment rows' scales
  double* as_w = nullptr;        // 6N: the vector the next apply reads (w of the iteration, r0, ...)
  // one launch per iteration (k_as_iter, as_one): the per-subdomain tables, ghost (w, z) of the ring rows, the parity's
  // contributions y_c = Z_c w[D_c] and the subdomain-ordered inverse rows, in ONE buffer (offsets: AsTab)
  int32_t as_one = 0, as_tab_cap = 0;
  char* as_tab = nullptr;
  int32_t *as_mem = nullptr, *as_memn = nullptr;   // per row: its subdomain memberships (c·kAsD + 6·l, <= 1 + kAsX)
  double* scal = nullptr;
  int32_t* flags = nullptr;
  // DeformNet.arap mode with lambda_flow = 0: rows of each multi-node connected graph component
  // (comp_off[c]..comp_off[c+1] in comp_rows), whose common translation is the exact null space
  int32_t *comp_rows = nullptr, *comp_off = nullptr;
  int n_comp = 0, comp_cap = 0;
  double* loss_log = nullptr;
  double* stat = nullptr;         // kMaxLog x [pcg iterations, |b|², loss] of the last solve
  double* step_state = nullptr;   // (kMaxLog+1) x [previous loss, accepted steps] before each GN step
  // Galerkin warm start over the last kProj GN-step solutions of this solve (ring of kProj x 6N each;
  // the previous frame's solutions were measured not to help its first steps):
  // xh = previous solutions, th = A·xh
  double *xh = nullptr, *th = nullptr;
  struct StepArgs* step_args = nullptr;   // device copy (fused GN step in the converging PCG launch)
  bool step_fused = false;                // this step's k_step work was done by the PCG
  int n_prev = 0;                 // valid entries of the ring for the current step
  int warm_now = 0;               // this step starts from the projected x0
  int32_t* host_flags = nullptr;  // pinned, mapped: [H_DONE, H_PCG_IT, H_STOPPED] written by the kernels
  int32_t* hflags = nullptr;      // its device address (system-scope stores: no copy kernel per poll)
  int32_t* setup_stat = nullptr;  // pinned, mapped: the setup's one host read [nnz, max row, max wave, abort, graph diff]
  int32_t* d_setup_stat = nullptr;
  hipEvent_t poll_ev = nullptr;   // recorded after each chunk of PCG launches
  double host_enqueue_us = 0.0;   // tuning build: host time spent enqueuing PCG iterations
  int64_t host_enqueued = 0;
  bool setup_done = false;
  // optional timing of the PCG iteration loop (hipEvents on the caller's stream)
  bool timing = false;
  int64_t n_iter_launches = 0;
};
static_assert(std::is_trivially_copyable<GnDev>::value, "kernel argument");

// The as_tab buffer (k_as_iter), for a capacity of cap clusters: region by region, [cluster][...] each (16-B aligned)
//   blk  [kGB]  int2  the subdomain rows' blocks in row order (CSR order within a row): (A slot, S2 index << 5 | row)
//   con  [kGS]  int4  per S2 node the y indices (c'·kAsD + 6·l') of the subdomains holding it, ascending, -1 after
//   s2n  [kGS]  int   S2 node -> row (the first iteration gathers m from the warm start's m0)
//   row  [kGRow] int  row starts [0, kAsDN], then nd at 25, nb at 26, ns at 27; S2 index of each subdomain row at 32 + l,
//                     its node (row) at 64 + l
//   dsc  [kAsD] f32   the inverse's scales d = √diag Z (k_as_invert)
//   gh   [kAsRing·6] double2  ghost (w, z) of the ring rows (the owners' recurrences, repeated bit for bit)
//   y    [2][cap][kAsD] f64  per parity the contributions y_c = D Ẑ D w[D_c]
//   slab [kAsK][kAsD] uint4  Ẑ's rows (8 fp16 per word), word k of every row contiguous
struct AsTabP {
  int2* blk; int4* con; int32_t* s2n; int32_t* row; float* dsc; double2* gh; double* y; uint4* slab;
};
__host__ __device__ __forceinline__ AsTabP as_tab_at(char* base, int64_t cap) {
  AsTabP p;
  char* q = base;
  p.blk = reinterpret_cast<int2*>(q); q += cap * kGB * 8;
  p.con = reinterpret_cast<int4*>(q); q += cap * kGS * 16;
  p.s2n = reinterpret_cast<int32_t*>(q); q += cap * kGS * 4;
  p.row = reinterpret_cast<int32_t*>(q); q += cap * kGRow * 4;
  p.dsc = reinterpret_cast<float*>(q); q += cap * kAsD * 4;
  p.gh = reinterpret_cast<double2*>(q); q += cap * kAsRing * 6 * 16;
  p.y = reinterpret_cast<double*>(q); q += 2 * cap * kAsD * 8;
  p.slab = reinterpret_cast<uint4*>(q);
  return p;
}
static inline int64_t as_tab_bytes(int64_t cap) {
  return cap * ((int64_t)kGB * 8 + (int64_t)kGS * 16 + (int64_t)kGS * 4 + kGRow * 4 + kAsD * 4 + kAsRing * 6 * 16 +
                2 * kAsD * 8 + (int64_t)kAsK * kAsD * 16);
}

// The solver handle: the kernel-visible state plus host-only members.
struct Gn : GnDev {
  std::vector<float> h_nodes;          // host copy of the graph the current order was built from
  std::vector<int32_t> h_edges, h_perm;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;   // timing events of the PCG loops
  // converged PCG iteration count of the previous solve, per GN step (sizes the first chunk of launches);
  // shared by the solver slots of one frame loop (ofx_gn_share_history)
  struct PcgHist {                  // per GN step the converged counts of the last 4 solves (ring), newest at n % 4
    int c[64][4] = {};
    int n[64] = {};
  };
  std::shared_ptr<PcgHist> last_pcg = std::make_shared<PcgHist>();
  // prefetched setup (ofx_gn_prepare): the next problem's setup runs on a host thread, on the handle's own
  // stream, while the caller's stream still works on the current problem (of another handle)
  std::thread worker;               // persistent (created by the first prefetch): no per-frame thread start
  std::mutex mu;
  std::condition_variable cv;
  bool job = false, quit = false;   // guarded by mu: a prefetch is queued / running; shut down
  // guarded by mu: a queued prefetch waits for its trigger (ofx_gn_prepare_after) — another handle's solve
  // reaching a GN step, that solve returning, or a wait on this handle
  bool gate = false;
  Gn* pf_peer = nullptr;            // (trigger side) the handle whose gated prefetch this handle's next solve opens
  int pf_step = 0;                  // ... at the start of this GN step (or on return)
  Gn* pf_trigger = nullptr;         // (prefetch side) the handle holding this one as pf_peer
  int prep_dev = 0;
  int prep_status = 0;
  bool prepared = false;            // the setup of prep_pb / prep_prm is (being) enqueued on `side`
  ofx_gn_problem prep_pb{};
  ofx_gn_params prep_prm{};
  hipStream_t side = nullptr;
  hipEvent_t ev_in = nullptr, ev_prep = nullptr;   // caller's stream at prepare -> side; side's setup done
  // side-stream work of a prefetch that no caller stream has been ordered after yet: the worker returns before
  // its last kernels (row assignment, contribution lists, ...) have run, and they write this handle's buffers
  bool side_dirty = false;
  hipEvent_t ev_side = nullptr;
  int64_t pf_used = 0, pf_missed = 0;   // solves that used / discarded a prefetched setup
  int32_t ep_next = 1;
  int as_env = -1;                  // OFX_PRECOND override of params.precond (-1: none)
  void (*idle_fn)(void*) = nullptr; // ofx_gn_set_idle_hook: host work run once at the next solve's first PCG wait
  void* idle_arg = nullptr;
  int as_lanes = 2;                 // k_as_apply's lanes per segment (OFX_AS_LANES)
  int as_cap = 0;                   // clusters the Schwarz tables are allocated for
  // the PCG iteration's constant launch arguments (struct PcgIt) in device memory, and the bytes last copied there
  void* d_pcgit = nullptr;
  alignas(16) unsigned char pcgit_last[512] = {};
  bool pcgit_valid = false;
#ifdef OFX_STAMPS   // tuning build: stream idle between a PCG chunk's last launch and the next GN step's first kernel
  std::chrono::steady_clock::time_point t_seen{};   // host saw the step's convergence
  double react_us = 0.0, prologue_us = 0.0;         // -> k_terms enqueued; -> the first PCG chunk launch enqueued
  int64_t react_n = 0;
  hipEvent_t gap_end = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gap_ev;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> entry_ev;   // solve entry -> pose done (the prefetched setup's wait)
  double prep_wait_us = 0.0;
#endif
};

// Order stream hs after everything the prefetch worker enqueued on the handle's side stream (call after
// prep_wait: the worker has finished enqueuing). Every entry point that touches the handle's buffers on a
// caller stream does this first, whether or not the prefetched setup is used.
static int fence_side(Gn* g, hipStream_t hs) {
  if (!g->side || !g->side_dirty) return OFX_OK;
  OFX_HIP(hipEventRecord(g->ev_side, g->side));
  OFX_HIP(hipStreamWaitEvent(hs, g->ev_side, 0));
  g->side_dirty = false;
  return OFX_OK;
}
// the same for host reads of device buffers (synchronous copies do not order after a non-blocking stream)
static int sync_side(Gn* g) {
  if (!g->side || !g->side_dirty) return OFX_OK;
  OFX_HIP(hipStreamSynchronize(g->side));
  g->side_dirty = false;
  return OFX_OK;
}

// F_REFRESH: the GN step whose warm start rebuilds the cluster inverse (set by the previous step's update when a node's
// accumulated rotation passed precond_rot_tol; 0 = none); F_CAPPED: GN steps whose PCG ran into pcg_max_iter
enum { F_DONE = 0, F_STOPPED = 1, F_ILL = 2, F_ACCEPTED = 3, F_PCG_TOTAL = 4, F_APPLY = 5, F_RES_NONFINITE = 6,
       F_PCG_IT = 7, F_PCG_CNT = 8, F_REFRESH = 9, F_CAPPED = 10, F_COUNT = 11 };
// scalars: S_TH_CUR = the current solve's latest θ̂ (error-based stop), S_TH_PREV = the previous GN step's final θ̂
// (k_pcg_w0 moves it per solve; 1e300 = none)
enum { S_LOSS_PREV = 0, S_BB = 1, S_TH_PREV = 2, S_TH_CUR = 3, S_COUNT = 4 };
// host-mapped flags: H_DONE holds the epoch (GnDev::ep) of the last converged PCG solve (from the converging launch's
// lead lane);
// H_STOPPED the epoch of the solve whose GN step stopped the loop (0: running). k_upload clears them per setup.
enum { H_DONE = 0, H_PCG_IT = 1, H_STOPPED = 2, H_COUNT = 3 };
__device__ __forceinline__ void host_flag(const int32_t* hf, int k, int v) {
  __hip_atomic_store(const_cast<int32_t*>(hf) + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int kMaxLog = 64;   // per-GN-step statistics slots
constexpr int32_t kEpochWrap = 1 << 30;   // GnDev::ep restarts at 1 from a setup once it reaches this (a solve adds <= 64)

// the scalar block (GnDev::pcs), in doubles: pcg_alpha [0, 6), pcg_gamma [6, 12), scal [12, 16), sturm (64 double2)
// [16, 144), flags (int32) from 144; written by k_pcg_w0 per solve: the PCG operator's address at 150, the stop tolerances
// (pcg_tol, pcg_err_tol) at 152, 153, the cluster inverses' address at 154, m0 / m1's at 156 / 157. The iteration gets
// the block's address with its parity in bit 3 (the block is 256-B aligned), so it needs no kernel-argument fetch for
// any of them.
constexpr int kPcgStreams = 4;   // k_pcg_iter's per-wave partial streams per parity: γ = r·u, δ = w·u, r·r, p·p
constexpr int kScAlpha = 0, kScGamma = 6, kScScal = 12, kScSturm = 16, kScFlags = 144, kScAop = 150, kScTol = 152,
              kScMcl = 154, kScM = 156, kScSize = 160;

// ---------------------------------------------------------------------------- reductions
template <int CTL>
__device__ __forceinline__ double dpp_mov(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// Sum over each aligned 16-lane row; every lane of the row ends with identical bits.
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp_mov<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_mov<0x141>(x);   // row_half_mirror
  x += dpp_mov<0x140>(x);   // row_mirror
  return x;
}
__device__ __forceinline__ double read_lane(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}
// x from the lanes selected by a broadcast DPP control into the rows of row_mask (0 elsewhere)
template <int CTL, int ROWS>
__device__ __forceinline__ double dpp_bcast(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTL, ROWS, 0xF, false);
  return __hiloint2double(hi, lo);
}
// Full-wave sum, fixed order, uniform result. Call from wave-uniform control flow. After the 16-lane row sums r0..r3,
// row_bcast:15 adds row 0 into row 1 and row 2 into row 3, row_bcast:31 adds row 1 into row 3, whose lane 63 then
// holds (r3 + r2) + (r1 + r0) — bitwise the (r0 + r1) + (r2 + r3) of reading four lanes (f64 addition commutes
// exactly), in 2 DPP adds and one lane read instead of 4 lane reads, 2 moves back to VGPRs and 3 adds.
__device__ __forceinline__ double wave_sum(double x) {
  x = row16_sum(x);
  x += dpp_bcast<0x142, 0xA>(x);   // row_bcast:15 into rows 1, 3
  x += dpp_bcast<0x143, 0x8>(x);   // row_bcast:31 into row 3
  return read_lane(x, 63);
}
// four block sums at once: fixed-order wave sums, then the kBlk/64 wave results combined in wave order
__device__ __forceinline__ void block_sum4(double v[4]) {
  __shared__ double s4[kBlk / 64][4];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = wave_sum(v[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) s4[w][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double a = 0.0;
#pragma unroll
    for (int q = 0; q < kBlk / 64; ++q) a += s4[q][k];
    v[k] = a;
  }
}
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double s[kBlk];
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

// Sum of p[i*stride + off], i < n, in a fixed order; every thread of the WG gets the same bits.
__device__ __forceinline__ double wg_sum_fixed(const double* __restrict__ p, int n, int stride, int off) {
  __shared__ double s_res;
  if (threadIdx.x < 64) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += 64) acc += p[(int64_t)i * stride + off];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (threadIdx.x == 0) s_res = acc;
  }
  __syncthreads();
  double r = s_res;
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------- setup kernels
// graph unchanged since the row order was built? (bitwise compare; any difference sets *diff)
__global__ __launch_bounds__(256) void k_graph_cmp(const float* __restrict__ a, const float* __restrict__ b, int64_t na,
                                                   const int32_t* __restrict__ c, const int32_t* __restrict__ d,
                                                   int64_t nc, int32_t* __restrict__ diff) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool x = false;
  if (i < na) x = __float_as_uint(a[i]) != __float_as_uint(b[i]);
  if (i < nc) x = x || c[i] != d[i];
  if (x) *diff = 1;
}

// Per-solve upload in one launch: f32 problem -> f64 device copies, anchors/edges, edge weights,
// initial R/t, term -> nodes table, flags/stats reset, and the previous pattern's entries of the
// N x N slot map cleared (so the map never needs an N² memset).
struct Upload {
  const float *nodes, *tpos, *conf, *src, *wts, *tgt, *tpx, *tpy, *ew, *prev_R, *prev_t;
  const int32_t *anc, *edges;
  int use_ew;
  int old_N;
  int64_t old_nnzb, n;
};
// caller node -> row (negative ids stay negative)
__device__ __forceinline__ int to_row(const GnDev& g, int a) { return a >= 0 ? g.iperm[a] : a; }
// edge k of row i in row numbering (-1: none, also for padding rows)
__device__ __forceinline__ int edge_row(const GnDev& g, const Upload& u, int i, int k) {
  const int p = g.perm[i];
  return p >= 0 ? to_row(g, u.edges[(int64_t)p * g.NB + k]) : -1;
}
__global__ __launch_bounds__(256) void k_upload(GnDev g, Upload u) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= u.n) return;
  const int N = g.N, M = g.M, NB = g.NB;
  if (i < u.old_nnzb) g.map[(int64_t)g.blk_row[i] * u.old_N + g.col[i]] = 0;
  if (i < 3 * (int64_t)N) {   // padding rows: a node at the origin with confidence 0 and no edges
    const int p = g.perm[i / 3];
    const int64_t s = 3 * (int64_t)p + i % 3;
    g.nodes[i] = p >= 0 ? u.nodes[s] : 0.0;
    g.tpos[i] = p >= 0 ? u.tpos[s] : 0.0;
    g.t[i] = (p >= 0 && u.prev_t) ? (double)u.prev_t[s] : 0.0;
  }
  if (i < 9 * (int64_t)N) {
    const int p = g.perm[i / 9];
    g.R[i] = (p >= 0 && u.prev_R) ? (double)u.prev_R[9 * (int64_t)p + i % 9] : ((i % 9) % 4 == 0 ? 1.0 : 0.0);
  }
  if (i < N) { const int p = g.perm[i]; g.conf[i] = p >= 0 ? u.conf[p] : 0.0; }
  if (i < 3 * (int64_t)M) { g.src[i] = u.src[i]; g.tgt[i] = u.tgt[i]; }
  if (i < 4 * (int64_t)M) { g.wts[i] = u.wts[i]; g.anc[i] = to_row(g, u.anc[i]); }
  if (i < M) { g.tpx[i] = u.tpx ? (double)u.tpx[i] : 0.0; g.tpy[i] = u.tpy ? (double)u.tpy[i] : 0.0; }
  if (i < (int64_t)N * NB) {
    const int r = (int)(i / NB), k = (int)(i % NB);
    const int p = g.perm[r];
    g.edges[i] = edge_row(g, u, r, k);
    g.ew[i] = (p >= 0 && u.use_ew && u.ew) ? (double)NB * (double)u.ew[(int64_t)p * NB + k] : 1.0;
  }
  if (i < g.T) {   // term t -> its (up to 4) rows, straight from the inputs
    int n[4] = {-1, -1, -1, -1};
    if (i < M) {
      for (int k = 0; k < 4; ++k) n[k] = to_row(g, u.anc[i * 4 + k]);
    } else if (i < M + (int64_t)N * NB) {
      const int64_t e = i - M;
      const int j = edge_row(g, u, (int)(e / NB), (int)(e % NB));
      if (j >= 0) { n[0] = (int)(e / NB); n[1] = j; }
    } else {
      n[0] = (int)(i - M - (int64_t)N * NB);
    }
    for (int k = 0; k < 4; ++k) g.term_node[i * 4 + k] = n[k];
  }
  // (cleared here rather than by fill dispatches: every partial stream is read unconditionally up to nw_pad; the wave
  // maximum's slot; the one-launch tables' membership counts, atomically counted again by k_as_members)
  if (i < kProjP * (int64_t)g.nw_pad) g.part_p[i] = 0.0;
  if (i == 0) g.row_cnt[N + 1] = 0;
  if (g.as_memn && i < N) g.as_memn[i] = 0;
  if (i < F_COUNT) g.flags[i] = 0;
  if (i < H_COUNT) host_flag(g.hflags, (int)i, 0);
  if (i < S_COUNT) g.scal[i] = 0.0;
  if (i < 3 * kMaxLog) g.stat[i] = 0.0;
  if (i < 2 * (kMaxLog + 1)) g.step_state[i] = 0.0;
}

// The previous frame's transforms into the state (k_upload's R / t rows) for a setup that was prefetched
// before they existed (ofx_gn_prepare uploads the problem with identity / zero).
__global__ __launch_bounds__(256) void k_pose(GnDev g, const float* __restrict__ prev_R, const float* __restrict__ prev_t) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int N = g.N;
  if (i < 3 * (int64_t)N) {
    const int p = g.perm[i / 3];
    g.t[i] = (p >= 0 && prev_t) ? (double)prev_t[3 * (int64_t)p + i % 3] : 0.0;
  }
  if (i < 9 * (int64_t)N) {
    const int p = g.perm[i / 9];
    g.R[i] = (p >= 0 && prev_R) ? (double)prev_R[9 * (int64_t)p + i % 9] : ((i % 9) % 4 == 0 ? 1.0 : 0.0);
  }
}

// exclusive scan of one int per thread over the workgroup (wave shuffles + one LDS pass); total out
__device__ __forceinline__ int block_exscan(int v, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  if (w == 0) {
    int t = lane < nw ? s_w[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(t, o, 64);
      if (lane >= o) t += y;
    }
    if (lane < nw) s_w[lane] = t;
  }
  __syncthreads();
  const int base = w > 0 ? s_w[w - 1] : 0;
  total = s_w[nw - 1];
  __syncthreads();
  return base + x - v;
}

__global__ void k_mark(GnDev g) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  const int32_t* n = g.term_node + t * 4;
  for (int p = 0; p < 4; ++p) {
    if (n[p] < 0) continue;
    for (int q = 0; q < 4; ++q)
      if (n[q] >= 0) g.map[(int64_t)n[p] * g.N + n[q]] = 1;
  }
}

// cnt[i] = blocks of row i
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

// Per PCG wave (kCS consecutive rows = one contiguous CSR range) its first kWL blocks: the block's column (-1: none)
// and, packed, the wave's first CSR block (19 bits; block k of the wave is that + k), the first block of lane k % 64's
// row relative to it (8 bits) and the row's length (5 bits) — so the iteration reads its gather addresses without the
// row_ptr -> col chain and needs no row_ptr (the packing holds whenever the wave-list forms run: <= kWL blocks per wave,
// <= kRowMax per row, nnzb <= 16·rows < 2^19)
constexpr int kWL = 128;
constexpr int kRowMax = 20;   // longest block row of the wave-list SpMV forms (k_pcg_iter, k_pcg_w0)
static_assert(kRowMax < 32 && kWL <= 255 && 16 * (2 * kMaxNodes + 8) < (1 << 19), "wave-list packing");
__device__ __forceinline__ int wl_base(int2 e) { return e.y & 0x7FFFF; }
__device__ __forceinline__ int wl_rel(int2 e) { return (e.y >> 19) & 0xFF; }
__device__ __forceinline__ int wl_len(int2 e) { return (int)((uint32_t)e.y >> 27); }
__global__ __launch_bounds__(256) void k_wave_max(int nwave, const int32_t* __restrict__ row_ptr, int32_t* __restrict__ out) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w < nwave) atomicMax(out, row_ptr[(w + 1) * kCS] - row_ptr[w * kCS]);
}
__global__ __launch_bounds__(256) void k_wave_list(GnDev g) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= (int64_t)(g.N / kCS) * kWL) return;
  const int w = (int)(e / kWL), k = (int)(e % kWL);
  const int wb = g.row_ptr[w * kCS], b = wb + k;
  const int row = w * kCS + (k % 64) / (64 / kCS);
  // (clamped: a wave or row too long for the wave-list forms is never run through them)
  const uint32_t rel = (uint32_t)min(g.row_ptr[row] - wb, 0xFF), len = (uint32_t)min(g.row_ptr[row + 1] - g.row_ptr[row], 31);
  const uint32_t y = ((uint32_t)wb & 0x7FFFFu) | (rel << 19) | (len << 27);
  g.wl[e] = make_int2(b < g.row_ptr[(w + 1) * kCS] ? g.col[b] : -1, (int)y);
}

// exclusive scan of cnt[0..n) into off[0..n] (off[n] = total), single workgroup: contiguous chunk
// per thread, one block scan of the chunk sums
// (max_out, nullable: max of cnt)
__global__ __launch_bounds__(1024) void k_scan(int64_t n, int32_t* cnt, int32_t* __restrict__ off,
                                               int32_t* __restrict__ max_out, bool clear) {   // clear: cnt = 0 after
  // tiles of 1024 x 32 counts (the setup's lists, up to ~33k entries, in one tile: one memory trip instead of one per
  // 8k entries): thread t scans its 32 contiguous entries (16-B loads and stores), the block scan combines the threads,
  // a carry runs across tiles (fixed order)
  __shared__ int s_w[16];
  __shared__ int s_mx[16];
  constexpr int kPer = 32;
  int carry = 0, mx = 0;
  for (int64_t base = 0; base < n; base += (int64_t)blockDim.x * kPer) {
    const int64_t s0 = base + (int64_t)threadIdx.x * kPer;
    const bool vec = s0 + kPer <= n && ((reinterpret_cast<uintptr_t>(cnt + s0) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(off + s0) & 15) == 0);
    int v[kPer];
    if (vec) {
#pragma unroll
      for (int q = 0; q < kPer / 4; ++q) {
        const int4 a = reinterpret_cast<const int4*>(cnt + s0)[q];
        v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPer; ++k) v[k] = s0 + k < n ? cnt[s0 + k] : 0;
    }
    if (clear) {
      if (vec) {
#pragma unroll
        for (int q = 0; q < kPer / 4; ++q) reinterpret_cast<int4*>(cnt + s0)[q] = make_int4(0, 0, 0, 0);
      } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k)
          if (s0 + k < n) cnt[s0 + k] = 0;
      }
    }
    int c = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) { c += v[k]; mx = max(mx, v[k]); }
    int total;
    int o = block_exscan(c, s_w, total) + carry;
    if (vec) {
#pragma unroll
      for (int q = 0; q < kPer / 4; ++q) {
        int4 r;
        r.x = o; o += v[4 * q];
        r.y = o; o += v[4 * q + 1];
        r.z = o; o += v[4 * q + 2];
        r.w = o; o += v[4 * q + 3];
        reinterpret_cast<int4*>(off + s0)[q] = r;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPer; ++k)
        if (s0 + k < n) { off[s0 + k] = o; o += v[k]; }
    }
    carry += total;
  }
  if (threadIdx.x == 0) off[n] = carry;
  if (clear && threadIdx.x == 0) cnt[n] = 0;
  if (max_out) {
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) mx = max(mx, __shfl_xor(mx, k, 64));
    if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
      int m = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = max(m, s_mx[w]);
      *max_out = m;
    }
  }
}

// ordered slot assignment per block row (one WG per row, one pass): contiguous column chunk per
// thread, block scan of the chunk counts; records col, slot + 1 in the map (0 = not in the
// pattern), and the block's row
__global__ __launch_bounds__(256) void k_row_assign(int N, int32_t* __restrict__ map, const int32_t* __restrict__ row_ptr,
                                                    int32_t* __restrict__ col, int32_t* __restrict__ blk_row) {
  __shared__ int s_w[4];
  const int i = blockIdx.x;
  const int per = (N + 255) / 256;
  const int j0 = threadIdx.x * per, j1 = min(N, j0 + per);
  int32_t* mrow = map + (int64_t)i * N;
  int c = 0;
  for (int j = j0; j < j1; ++j) c += mrow[j] != 0;
  int total;
  int slot = row_ptr[i] + block_exscan(c, s_w, total);
  for (int j = j0; j < j1; ++j)
    if (mrow[j] != 0) {
      col[slot] = j;
      blk_row[slot] = i;
      mrow[j] = slot + 1;
      ++slot;
    }
}

// the setup's host-read scalars into host-mapped memory in one kernel (five small D2H copies through pageable
// memory cost ~15-20 us each on the frame-boundary critical path)
__global__ void k_setup_status(const int32_t* __restrict__ row_ptr, int N, const int32_t* __restrict__ row_cnt,
                               int32_t* __restrict__ gdiff, int32_t* out) {
  if (threadIdx.x != 0) return;
  const int32_t v[4] = {row_ptr[N], row_cnt[N], row_cnt[N + 1], gdiff ? *gdiff : 0};
  if (gdiff) *gdiff = 0;   // (the next optimistic compare starts from zero: no fill dispatch)
#pragma unroll
  for (int k = 0; k < 4; ++k) __hip_atomic_store(out + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Contribution counts / lists of a term's node pairs. Every load of a term is issued before the first atomic and every
// atomic before the first store (unconditional loads at clamped addresses, masked uses): three dependent trips per
// term instead of a chain of map -> up_of -> atomic per pair (33 / 32 us per setup as the pair loop). The atomics' order
// does not matter: counts are sums, and k_seg_rank sorts every list by its unique codes afterwards.
__device__ __forceinline__ void pair_slots(const GnDev& g, int64_t t, int n[4], bool ok[4][4], int u[4][4]) {
  const int4 nn = *reinterpret_cast<const int4*>(g.term_node + t * 4);
  n[0] = nn.x; n[1] = nn.y; n[2] = nn.z; n[3] = nn.w;
  int ms[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ok[p][q] = n[p] >= 0 && n[q] >= n[p];
      ms[p][q] = g.map[ok[p][q] ? (int64_t)n[p] * g.N + n[q] : 0];
    }
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) u[p][q] = g.up_of[ok[p][q] ? ms[p][q] - 1 : 0];
}
__global__ __launch_bounds__(256) void k_pair_count(GnDev g) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  int n[4], u[4][4];
  bool ok[4][4];
  pair_slots(g, t, n, ok, u);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (n[p] >= 0) atomicAdd(&g.node_cnt[n[p]], 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (ok[p][q]) atomicAdd(&g.blk_cnt[u[p][q]], 1);
  }
}

// scatter (order fixed later by k_seg_rank); blk_cnt/node_cnt are reused as cursors (zeroed first)
__global__ __launch_bounds__(256) void k_pair_scatter(GnDev g) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= g.T) return;
  int n[4], u[4][4];
  bool ok[4][4];
  pair_slots(g, t, n, ok, u);
  int no[4], bo[4][4], np[4], bp[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    no[p] = g.node_off[n[p] >= 0 ? n[p] : 0];
#pragma unroll
    for (int q = 0; q < 4; ++q) bo[p][q] = g.blk_off[ok[p][q] ? u[p][q] : 0];
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    np[p] = n[p] >= 0 ? atomicAdd(&g.node_cnt[n[p]], 1) : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) bp[p][q] = ok[p][q] ? atomicAdd(&g.blk_cnt[u[p][q]], 1) : 0;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (n[p] >= 0) g.node_list[no[p] + np[p]] = (int32_t)(t * 4 + p);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (ok[p][q]) g.blk_list[bo[p][q] + bp[p][q]] = (int32_t)(t * 16 + p * 4 + q);
  }
}

// upper-block flags (scanned into up_of) and, after the scan, the upper list with each block's transpose slot
__global__ __launch_bounds__(256) void k_up_flags(GnDev g, int32_t* __restrict__ flag) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s < g.nnzb) flag[s] = g.col[s] >= g.blk_row[s] ? 1 : 0;
  for (int64_t i = s; i < g.nnzb + 32; i += (int64_t)gridDim.x * blockDim.x) g.up_slot[i] = -1;   // -1: no upper block
}
__global__ __launch_bounds__(256) void k_up_list(GnDev g) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  // the contribution counts start from zero (k_pair_count); blk_cnt held the flags the scan before this read
  for (int64_t i = s; i <= g.nnzb || i <= g.N; i += (int64_t)gridDim.x * blockDim.x) {
    if (i <= g.nnzb) g.blk_cnt[i] = 0;
    if (i <= g.N) g.node_cnt[i] = 0;
  }
  if (s >= g.nnzb) return;
  const int r = g.blk_row[s], c = g.col[s];
  if (c < r) return;
  const int u = g.up_of[s];
  g.up_slot[u] = (int32_t)s;
  g.up_tr[u] = g.map[(int64_t)c * g.N + r] - 1;
}

// Deterministic ordering of each segment (values are unique codes): one wave per segment, every
// lane ranks its entries against the whole segment (independent loads, no serial chain), and
// scatters them to their rank in `out`.
__global__ __launch_bounds__(256) void k_seg_rank(const int32_t* __restrict__ off, int64_t nseg,
                                                  const int32_t* __restrict__ in, int32_t* __restrict__ out) {
  const int64_t sgm = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (sgm >= nseg) return;
  const int b = off[sgm], n = off[sgm + 1] - b;
  for (int k = lane; k < n; k += 64) {
    const int v = in[b + k];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += in[b + j] < v;
    out[b + rank] = v;
  }
}

// ---------------------------------------------------------------------------- linearisation
struct DataCoef {
  double lf, ld, la, lm, fx, fy, cx, cy;
};

// Compact term records (kRec doubles per term at J + t·kRec; 160 B against the 576 B of four 3x6 blocks):
//   data  : [v_k w_k] for anchors k = 0..3 (v_k = w_k R_k(x - g_k)) at 4k, then [fx/z fy/z mfx mfy] at 16
//   ARAP  : [d0 d1 d2 s] at 0 (node i: d = R_i(g_j - g_i), s = la·w_e), node j's diagonal -s at 4
//   motion: the three diagonal entries at 0
// term_block() expands (record, slot) into the 3x6 block with the arithmetic the blocks were written with,
// operation for operation, so the assembled A and b are the same bits.
constexpr int kRec = 20;

// slot k of data term m: its anchor's [v w]; slot 0 also the term's shared scalars
__device__ __forceinline__ void data_record(const GnDev& g, const DataCoef& dc, int64_t m, int k, const double p[3],
                                            double zinv, double* __restrict__ rec) {
  int a = g.anc[m * 4 + k];
  double w = g.wts[m * 4 + k];
  const double* R = g.R + 9 * (int64_t)a;
  const double* gn = g.nodes + 3 * (int64_t)a;
  double d0 = g.src[3 * m] - gn[0], d1 = g.src[3 * m + 1] - gn[1], d2 = g.src[3 * m + 2] - gn[2];
  double2* o = reinterpret_cast<double2*>(rec + 4 * k);
  o[0] = make_double2(w * (R[0] * d0 + R[1] * d1 + R[2] * d2), w * (R[3] * d0 + R[4] * d1 + R[5] * d2));
  o[1] = make_double2(w * (R[6] * d0 + R[7] * d1 + R[8] * d2), w);
  if (k == 0) {
    double2* tl = reinterpret_cast<double2*>(rec + 16);
    tl[0] = make_double2(dc.fx * zinv, dc.fy * zinv);
    tl[1] = make_double2(-(dc.fx * p[0] * zinv) * zinv, -(dc.fy * p[1] * zinv) * zinv);
  }
}

enum TermKind { kData = 0, kEdge = 1, kMotion = 2 };
__device__ __forceinline__ int term_kind(const GnDev& g, int64_t t) {
  return t < g.M ? kData : (t < g.M + (int64_t)g.N * g.NB ? kEdge : kMotion);
}

// the 3x6 block of `slot` from the record's words x = rec[4·slot .. +3] and (data) tail = rec[16 .. 19]
__device__ __forceinline__ void term_block(int kind, int slot, const double x[4], const double tail[4],
                                           const DataCoef& dc, double J[18]) {
#pragma unroll
  for (int c = 0; c < 18; ++c) J[c] = 0.0;
  if (kind == kData) {
    const double v0 = x[0], v1 = x[1], v2 = x[2], w = x[3];
    const double fxdz = tail[0], fydz = tail[1], mfx = tail[2], mfy = tail[3];
    // S = -[v]x
    const double S[9] = {0.0, v2, -v1, -v2, 0.0, v0, v1, -v0, 0.0};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      J[0 + j] = dc.lf * fxdz * S[0 + j] + mfx * S[6 + j] + dc.ld * S[0 + j];
      J[6 + j] = dc.lf * fydz * S[3 + j] + mfy * S[6 + j] + dc.ld * S[3 + j];
      J[12 + j] = dc.ld * S[6 + j];
    }
    J[3] = dc.lf * w * fxdz + dc.ld * w; J[5] = dc.lf * w * mfx;
    J[10] = dc.lf * w * fydz + dc.ld * w; J[11] = dc.lf * w * mfy;
    J[17] = dc.ld * w;
  } else if (kind == kEdge && slot == 0) {   // node i: [-s[d]x | s I]
    const double d0 = x[0], d1 = x[1], d2 = x[2], s = x[3];
    J[1] = s * d2; J[2] = -s * d1; J[3] = s;
    J[6] = -s * d2; J[8] = s * d0; J[10] = s;
    J[12] = s * d1; J[13] = -s * d0; J[17] = s;
  } else if (kind == kEdge) {                 // node j: [0 | -s I]
    J[3] = x[0]; J[10] = x[0]; J[17] = x[0];
  } else {
    J[3] = x[0]; J[10] = x[1]; J[17] = x[2];
  }
}

// the record words of (t, slot): two 16-B loads, plus the two of a data term's tail — loaded for every kind (every
// record has them) and zeroed for the others: a load in a kind branch was waited for inside it, one term after another
__device__ __forceinline__ void load_record(const GnDev& g, int64_t t, int slot, int kind, double x[4], double tail[4]) {
  const double2* r = reinterpret_cast<const double2*>(g.J + t * kRec);
  const double2 a = r[2 * slot], b = r[2 * slot + 1];
  const double2 c = r[8], d = r[9];
  x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
  const bool dt = kind == kData;
  tail[0] = dt ? c.x : 0.0; tail[1] = dt ? c.y : 0.0; tail[2] = dt ? d.x : 0.0; tail[3] = dt ? d.y : 0.0;
}

// Anchor k's summand of the deformed point of match m: w_k (R_k (x - g_k) + g_k + t_k) (ED_warp, geometry.py:9-25)
__device__ __forceinline__ void anchor_term(const GnDev& g, int64_t m, int k, double c[3]) {
  int a = g.anc[m * 4 + k];
  double w = g.wts[m * 4 + k];
  const double* R = g.R + 9 * (int64_t)a;
  const double* gn = g.nodes + 3 * (int64_t)a;
  const double* tt = g.t + 3 * (int64_t)a;
  double d0 = g.src[3 * m] - gn[0], d1 = g.src[3 * m + 1] - gn[1], d2 = g.src[3 * m + 2] - gn[2];
  c[0] = w * ((R[0] * d0 + R[1] * d1 + R[2] * d2) + gn[0] + tt[0]);
  c[1] = w * ((R[3] * d0 + R[4] * d1 + R[5] * d2) + gn[1] + tt[1]);
  c[2] = w * ((R[6] * d0 + R[7] * d1 + R[8] * d2) + gn[2] + tt[2]);
}

// Four threads per term (t = id/4, slot k = id%4): slot k writes its node's words of the term record
// (kRec above); slot 0 also writes the residual triple and the loss partials. Terms outside this rank's
// share (data matches outside [m0,m1), regularisers when !add_reg) get all-zero records (exact zero
// blocks) so the fixed contribution lists stay valid.
__global__ __launch_bounds__(kBlk) void k_terms(GnDev g, DataCoef dc, int m0, int m1, int add_reg) {
  // every kernel-argument field in SGPRs up front, in one scalar trip (left to the compiler, each branch loaded its own
  // fields after the branch: four dependent scalar trips ahead of the first vector load)
  asm volatile("" :: "s"(g.J), "s"(g.anc), "s"(g.wts), "s"(g.R), "s"(g.nodes), "s"(g.src), "s"(g.t), "s"(g.tgt),
               "s"(g.tpx), "s"(g.tpy), "s"(g.edges), "s"(g.ew), "s"(g.res), "s"(g.T), "s"(g.M), "s"(g.N), "s"(g.NB),
               "s"(g.conf), "s"(g.tpos), "s"(g.prm.mode), "s"(g.part_loss), "s"(m0), "s"(m1), "s"(add_reg));
  asm volatile("" :: "s"(dc.lf), "s"(dc.ld), "s"(dc.la), "s"(dc.lm), "s"(dc.fx), "s"(dc.fy), "s"(dc.cx), "s"(dc.cy));
  const int64_t id = blockIdx.x * (int64_t)kBlk + threadIdx.x;
  const int64_t t = id >> 2;
  const int k = (int)(id & 3);
  double r[3] = {0.0, 0.0, 0.0};
  double l2[3] = {0.0, 0.0, 0.0};
  double bad = 0.0;
  if (t < g.T) {
    double* rec = g.J + t * kRec;
    if (t < g.M) {
      if (t >= m0 && t < m1) {
        // deformed point: slot k computes its anchor's summand, the four slots (adjacent lanes of one wave, all
        // in this branch together) exchange them and every slot adds them to 0 in the anchor order k = 0..3
        // (the oracle's sequence; each slot used to recompute all four summands itself: 13.2 -> 11.8 us)
        // the residual's target values are loaded by every slot up front (no trip behind the k == 0 branch)
        const double tpx = g.tpx[t], tpy = g.tpy[t];
        const double tg0 = g.tgt[3 * t], tg1 = g.tgt[3 * t + 1], tg2 = g.tgt[3 * t + 2];
        double c[3];
        anchor_term(g, t, k, c);
        const int base = (int)(threadIdx.x & 63) & ~3;
        double p[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int d = 0; d < 3; ++d) p[d] += __shfl(c[d], base + kk, 64);
        double zinv = 1.0 / (p[2] + 1e-7);
        data_record(g, dc, t, k, p, zinv, rec);
        if (k == 0) {
          r[0] = dc.lf * (dc.fx * p[0] * zinv + dc.cx - tpx) + dc.ld * (p[0] - tg0);
          r[1] = dc.lf * (dc.fy * p[1] * zinv + dc.cy - tpy) + dc.ld * (p[1] - tg1);
          r[2] = dc.ld * (p[2] - tg2);
          l2[0] = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        }
      } else {
        double2* o = reinterpret_cast<double2*>(rec + 4 * k);
        o[0] = o[1] = make_double2(0.0, 0.0);
        if (k == 0) reinterpret_cast<double2*>(rec + 16)[0] = reinterpret_cast<double2*>(rec + 16)[1] = make_double2(0.0, 0.0);
      }
    } else if (t < g.M + (int64_t)g.N * g.NB) {
      const int64_t e = t - g.M;
      const int j = g.edges[e];
      // the edge's weight and node i's R, g, t leave with the edge's j (none depends on j; behind the j >= 0 test the
      // weight was a trip of its own, then i's and j's records another)
      const int i = (int)(e / g.NB);
      const double ewv = g.ew[e];
      double Ri[9], gi[3], ti[3];
#pragma unroll
      for (int q = 0; q < 9; ++q) Ri[q] = g.R[9 * (int64_t)i + q];
#pragma unroll
      for (int q = 0; q < 3; ++q) { gi[q] = g.nodes[3 * (int64_t)i + q]; ti[q] = g.t[3 * (int64_t)i + q]; }
      asm volatile("" ::: "memory");
      if (j >= 0 && k < 2) {
        if (add_reg) {
          const double s = dc.la * ewv;
          if (k == 0) {
            const double* gj = g.nodes + 3 * (int64_t)j;
            const double* tj = g.t + 3 * (int64_t)j;
            double e0 = gj[0] - gi[0], e1 = gj[1] - gi[1], e2 = gj[2] - gi[2];
            double d0 = Ri[0] * e0 + Ri[1] * e1 + Ri[2] * e2;
            double d1 = Ri[3] * e0 + Ri[4] * e1 + Ri[5] * e2;
            double d2 = Ri[6] * e0 + Ri[7] * e1 + Ri[8] * e2;
            r[0] = s * (d0 + gi[0] + ti[0] - (gj[0] + tj[0]));
            r[1] = s * (d1 + gi[1] + ti[1] - (gj[1] + tj[1]));
            r[2] = s * (d2 + gi[2] + ti[2] - (gj[2] + tj[2]));
            double2* o = reinterpret_cast<double2*>(rec);   // node i's [d s]
            o[0] = make_double2(d0, d1);
            o[1] = make_double2(d2, s);
            l2[1] = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
          } else {  // node j's diagonal
            rec[4] = -s;
          }
        } else if (k == 0) {
          reinterpret_cast<double2*>(rec)[0] = reinterpret_cast<double2*>(rec)[1] = make_double2(0.0, 0.0);
          rec[4] = 0.0;
        }
      }
    } else if (k == 0) {
      const int i = (int)(t - g.M - (int64_t)g.N * g.NB);
      double J3 = 0.0, J10 = 0.0, J17 = 0.0;
      if (add_reg && g.prm.mode == OFX_GN_ARAP) {
        // DeformNet.arap "flow" rows of the valid nodes (model.py:1766-1784): the Jacobian entry on
        // t_c is the residual itself, as the reference writes it
        const double c = dc.lf * g.conf[i];
        for (int q = 0; q < 3; ++q) r[q] = c * (g.t[3 * i + q] + g.nodes[3 * i + q] - g.tpos[3 * i + q]);
        J3 = r[0]; J10 = r[1]; J17 = r[2];
        l2[0] = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
      } else if (add_reg) {
        double c = dc.lm * g.conf[i];
        for (int q = 0; q < 3; ++q) r[q] = c * (g.t[3 * i + q] + g.nodes[3 * i + q] - g.tpos[3 * i + q]);
        J3 = c; J10 = c; J17 = c;
        l2[2] = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
      }
      rec[0] = J3; rec[1] = J10; rec[2] = J17;
    }
    if (k == 0) {
      g.res[3 * t] = r[0]; g.res[3 * t + 1] = r[1]; g.res[3 * t + 2] = r[2];
      bad = (isfinite(l2[0]) && isfinite(l2[1]) && isfinite(l2[2])) ? 0.0 : 1.0;
    }
  }
  double sv[4] = {l2[0], l2[1], l2[2], bad};
  block_sum4(sv);
  if (threadIdx.x == 0) {
    double* P = g.part_loss + 4 * (int64_t)blockIdx.x;
    P[0] = sv[0]; P[1] = sv[1]; P[2] = sv[2]; P[3] = sv[3];
  }
}

// b = -Jᵀr: one wave per node, entry-parallel (below). WG 0 also reduces the loss partials into the
// rhs tail.
__device__ __forceinline__ void rhs_body(const GnDev& g, const DataCoef& dc, double* __restrict__ rhs, int wg) {
  if (wg == 0 && threadIdx.x < 64) {   // the loss partials of k_terms, 4 streams in one pass, fixed order
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < g.nwg_terms; i += 64) {
      const double4 t = *reinterpret_cast<const double4*>(g.part_loss + 4 * (int64_t)i);
      a[0] += t.x; a[1] += t.y; a[2] += t.z; a[3] += t.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
    if (threadIdx.x == 0) {
      double* tail = rhs + 6 * (int64_t)g.N;
      tail[0] = a[0]; tail[1] = a[1]; tail[2] = a[2]; tail[3] = a[3];
    }
  }
  const int n = wg * (kBlk / 64) + (threadIdx.x >> 6);
  if (n >= g.N) return;
  const int lane = threadIdx.x & 63;
  // one wave per node, one list entry per lane (two per lane per pass: a busy node's ~90 terms in one
  // pass of two dependent trips — code, then J + r — where 10 slots took ~10 serial passes); every load
  // unconditional (clamped index, masked value) so no branch splits a trip; fixed-order wave sums
  const int b = g.node_off[n], e = g.node_off[n + 1];
  int code[2];   // the first pass's codes come with the bounds (node_first), later passes' from the list
#pragma unroll
  for (int j = 0; j < 2; ++j) code[j] = g.node_first[(int64_t)n * 128 + lane + 64 * j];
  asm volatile("" ::: "memory");   // (issued with the bounds, not sunk into the loop behind its entry test)
  double v[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int k0 = b; k0 < e; k0 += 128) {
    bool ok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + lane + 64 * j;
      ok[j] = k < e;
      if (k0 != b) code[j] = g.node_list[ok[j] ? k : e - 1];
    }
    // both entries' records and residuals first (one trip), then the blocks (left in the loop, the second entry's loads
    // issued after the first entry's kind branches: two trips)
    int kind[2];
    double x[2][4], tail[2][4], rv[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t t = code[j] >> 2;
      kind[j] = term_kind(g, t);
      load_record(g, t, code[j] & 3, kind[j], x[j], tail[j]);
      const double* rr = g.res + 3 * t;
      rv[j][0] = rr[0]; rv[j][1] = rr[1]; rv[j][2] = rr[2];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      double P[18];
      term_block(kind[j], code[j] & 3, x[j], tail[j], dc, P);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double t3 = P[c] * rv[j][0] + P[6 + c] * rv[j][1] + P[12 + c] * rv[j][2];
        v[c] += ok[j] ? t3 : 0.0;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) v[c] = wave_sum(v[c]);
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < 6; ++c) rhs[6 * (int64_t)n + c] = -v[c];
}

// JᵀJ blocks, workgroup-cooperative: the workgroup's 16 blocks own one contiguous range of the sorted
// contribution list. Chunks of kCoop entries: one thread per entry loads its two Jacobian blocks (the next
// chunk's codes one chunk ahead) and writes the full 6×6 product to LDS ([output][entry], padded: conflict-
// free writes); then each (block, output) pair — 576 per workgroup, up to 3 per thread — adds its entries of
// the chunk in list order. A block's cost is its share of the workgroup's entries, not its own list length
// (the 16-lane form took ceil(len/16) dependent trips: ~6 for a busy node's diagonal block).
#ifndef OFX_KCOOP
#define OFX_KCOOP 128   // (tuning builds: -DOFX_KCOOP=n, n <= kBlk)
#endif
constexpr int kCoop = OFX_KCOOP;
static_assert(kCoop <= kBlk, "one entry per thread per chunk");
__device__ __forceinline__ void blocks_coop(const GnDev& g, const DataCoef& dc, double* __restrict__ A, int64_t wg,
                                            double lm) {
  __shared__ double s_prod[36 * (kCoop + 1)];
  __shared__ int s_off[17];
  const int tid = threadIdx.x;
  const int64_t sb = wg * (kBlk / 16);   // upper blocks u in [sb, sb + 16); past the upper count up_slot is -1 and
                                         // the lists are empty (blk_off there = the total)
  constexpr int kPairs = (kBlk / 16) * 36;
  constexpr int kU = (kPairs + kBlk - 1) / kBlk;
  // first trip: the 17 list offsets and every pair's output slots (consumed at the end, in flight all along)
  // (every load unconditional, the list offsets first: a load inside the offsets' branch was waited for there, before
  // the other loads issued)
  const int offv = g.blk_off[min<int64_t>(sb + min(tid, kBlk / 16), g.nnzb)];
  int code_next = g.blk_first[wg * kCoop + min(tid, kCoop - 1)];   // the first chunk's codes (k_first_codes)
  int pb[kU], po[kU], os[kU], ot[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int p = tid + kBlk * u;
    pb[u] = p < kPairs ? p / 36 : kBlk / 16 - 1; po[u] = p % 36;
    os[u] = g.up_slot[sb + pb[u]];
    ot[u] = g.up_tr[sb + pb[u]];
  }
  if (tid <= kBlk / 16) s_off[tid] = offv;
  __syncthreads();
  const int E0 = s_off[0], E1 = s_off[kBlk / 16];
  if (E0 == E1) return;   // no upper block here (uniform over the workgroup)
  double acc[kU];
  int lo[kU], hi[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const bool ok = tid + kBlk * u < kPairs;
    lo[u] = ok ? s_off[pb[u]] : 0;
    hi[u] = ok ? s_off[pb[u] + 1] : 0;
    acc[u] = 0.0;
  }
  for (int c0 = E0; c0 < E1; c0 += kCoop) {
    if (tid < kCoop) {
      const int k = c0 + tid;
      const int code = code_next;
      code_next = k + kCoop < E1 ? g.blk_list[k + kCoop] : 0;
      if (k < E1) {
        const int64_t t = code >> 4;
        const int kind = term_kind(g, t), sp = (code >> 2) & 3, sq = code & 3;
        double xp[4], xq[4], tail[4], P[18], Q[18];
        load_record(g, t, sp, kind, xp, tail);
        const double2* r = reinterpret_cast<const double2*>(g.J + t * kRec + 4 * sq);
        const double2 a = r[0], b = r[1];
        xq[0] = a.x; xq[1] = a.y; xq[2] = b.x; xq[3] = b.y;
        term_block(kind, sp, xp, tail, dc, P);
        term_block(kind, sq, xq, tail, dc, Q);
#pragma unroll
        for (int c = 0; c < 6; ++c)
#pragma unroll
          for (int j = 0; j < 6; ++j)
            s_prod[(6 * c + j) * (kCoop + 1) + tid] = P[c] * Q[j] + P[6 + c] * Q[6 + j] + P[12 + c] * Q[12 + j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int a = max(lo[u], c0), b = min(hi[u], c0 + kCoop);
      const double* sp = s_prod + po[u] * (kCoop + 1) - c0;
      double x = acc[u];
      // eight LDS reads in flight, then the eight adds in list order (a one-read-per-add loop waited out the LDS
      // latency per entry: a busy diagonal block's outputs cost ~90 serial round trips per chunk)
      int e = a;
      for (; e + 8 <= b; e += 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = sp[e + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) x += v[k];
      }
      if (e + 4 <= b) {
        double v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = sp[e + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) x += v[k];
        e += 4;
      }
      for (; e < b; ++e) x += sp[e];
      acc[u] = x;
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int p = tid + kBlk * u;
    if (p >= kPairs || os[u] < 0) continue;
    const int64_t s = os[u], st = ot[u];
    double v = acc[u];
    // LM damping of the diagonal blocks (model.py:641-662)
    if (lm != 0.0 && po[u] % 7 == 0 && s == st) v += lm;
    A[36 * s + po[u]] = v;
    if (st != s) A[36 * st + 6 * (po[u] % 6) + po[u] / 6] = v;   // the lower block: the transpose
  }
}

// The first chunk of every assembly workgroup's contribution list and of every node's rhs list at fixed offsets (setup,
// after the lists are sorted): k_assemble loads them with the list bounds instead of one memory trip after them.
__global__ __launch_bounds__(kBlk) void k_first_codes(GnDev g, int nwb) {
  const int b = blockIdx.x, t = threadIdx.x;
  if (b < nwb) {
    const int64_t sb = (int64_t)b * (kBlk / 16);
    const int E0 = g.blk_off[min<int64_t>(sb, g.nnzb)], E1 = g.blk_off[min<int64_t>(sb + kBlk / 16, g.nnzb)];
    if (t < kCoop) g.blk_first[(int64_t)b * kCoop + t] = E0 + t < E1 ? g.blk_list[E0 + t] : 0;
  } else if (t < 128) {
    const int n = b - nwb;
    const int s0 = g.node_off[n], e = g.node_off[n + 1];
    g.node_first[(int64_t)n * 128 + t] = e > s0 ? g.node_list[s0 + t < e ? s0 + t : e - 1] : 0;
  }
}

// JᵀJ blocks and -Jᵀr in one launch: the rhs workgroups first (their per-node loops are the longest
// chains), then nwb workgroups of blocks.
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(4))) void k_assemble(GnDev g, DataCoef dc, double* __restrict__ A, double* __restrict__ rhs,
                                                  int nrw, double lm) {
  // the kernel-argument fields in SGPRs up front (one scalar trip, see k_terms; nrw, the rhs workgroup count, is an
  // argument rather than gridDim.x - nwb: the grid size is one more scalar load)
  asm volatile("" :: "s"(g.N), "s"(g.M), "s"(g.NB), "s"(g.node_list), "s"(g.node_off), "s"(g.nwg_terms),
               "s"(g.part_loss), "s"(g.res), "s"(g.J), "s"(g.blk_list), "s"(g.blk_off), "s"(g.nnzb), "s"(g.up_slot),
               "s"(g.up_tr), "s"(A), "s"(rhs), "s"(nrw), "s"(lm));
  asm volatile("" :: "s"(dc.lf), "s"(dc.ld), "s"(dc.la), "s"(dc.lm), "s"(dc.fx), "s"(dc.fy), "s"(dc.cx), "s"(dc.cy));
  // XCD-aware order: workgroups b and b + 8 share an XCD, so each XCD takes a contiguous run of nodes / upper
  // blocks and the term records they share stay in one L2 (nrw is a multiple of 8, so both halves keep b % 8); a
  // relabelling of which workgroup computes what: A and b are unchanged. Fetch 20.2 -> 7.9 MB per launch, time
  // unchanged (the re-reads were served by the MALL): profiles/r05_ab.json
  const int hw = blockIdx.x, part = hw < nrw ? nrw : (int)gridDim.x - nrw, i = hw < nrw ? hw : hw - nrw;
  const int q = part >> 3, r = part & 7, x = i & 7;
  const int L = x * q + min(x, r) + (i >> 3);
  if (hw < nrw) rhs_body(g, dc, rhs, L);
  else blocks_coop(g, dc, A, L, lm);
}
#ifdef OFX_SPLIT_ASSEMBLE
__global__ __launch_bounds__(kBlk) void k_assemble_blocks(GnDev g, DataCoef dc, double* __restrict__ A, double lm) {
  blocks_coop(g, dc, A, blockIdx.x, lm);
}
__global__ __launch_bounds__(kBlk) void k_assemble_rhs(GnDev g, DataCoef dc, double* __restrict__ rhs) {
  rhs_body(g, dc, rhs, blockIdx.x);
}
#endif

// ---------------------------------------------------------------------------- PCG
// Pipelined preconditioned CG (Ghysels & Vanroose 2014): one global reduction per iteration, ONE
// kernel per iteration. Preconditioner: block Jacobi over clusters of kCS graph-adjacent nodes
// (48x48 blocks of A; setup orders the nodes so that every cluster is the kRW = kCS rows of one
// wave, padding clusters with decoupled dummy nodes). The pipelined recurrences need m = M⁻¹w and
// n = A·m: each launch gathers m (written by the previous launch) for n = A·m, updates its rows,
// and applies its cluster's M⁻¹ to the new w through LDS — wave-local, so still one launch.

// ---- layout. st: per PCG row i and component c an 8-double record [x r u z q s p w] at
// st[(6i+c)*8] (a lane's whole recurrence state in 4 x 16-B accesses); m0/m1 (6N) double-buffer
// the gathered m. Row kernels run one wave per workgroup: lane = (row r of kRW, slot q of kSL);
// slot q multiplies whole 6x6 blocks q, q+kSL, ... of its row, DPP butterflies sum the row's slots;
// lanes q < 6 own component q of the row's vectors. Mcl: per row/component the f32 row of its
// cluster's symmetric inverse (48 entries). Scalars travel as per-wave partials (SoA
// [stream][wave]); every wave of the next launch re-sums them in the same fixed order.
enum { V_X = 0, V_R = 1, V_U = 2, V_Z = 3, V_Q = 4, V_S = 5, V_P = 6, V_W = 7, V_N = 8 };
constexpr int kRW = kCS;        // block rows per wave = cluster size
constexpr int kSL = 64 / kRW;   // lanes (block slots) per row
constexpr int kCD = 6 * kCS;    // cluster dimension
static_assert(kCS * kCS == 64, "k_pcg_prep maps the cluster's kCS x kCS node blocks onto one wave");

// LDS hand-off inside a single-wave workgroup: wait for this wave's LDS operations only. (A
// __syncthreads() is a workgroup-scope release that also drains every outstanding global store —
// a full memory round trip — and one wave needs no s_barrier.) gfx9 s_waitcnt: lgkmcnt(0), others max.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
}

// Sum over each aligned group of kSL (= 8) lanes; every lane of the group ends with identical bits.
__device__ __forceinline__ double slot_sum(double x) {
  x += dpp_mov<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_mov<0x141>(x);   // row_half_mirror
  return x;
}

// Σ_i p[k*nw + i] for K streams, in two phases so the loads can be issued early: load_streams puts
// U entries per lane in registers, reduce_streams adds the tail (nw > 64U) and sums in a fixed
// order; uniform result in every lane.
template <int K, int U>
__device__ __forceinline__ void load_streams(const double* __restrict__ p, int nw, double t[K][U]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = lane + 64 * u;
      t[k][u] = i < nw ? p[(int64_t)k * nw + i] : 0.0;
    }
}
template <int K, int U>
__device__ __forceinline__ void reduce_streams(const double* __restrict__ p, int nw, double t[K][U], double out[K]) {
  const int lane = threadIdx.x & 63;
  double a[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int w = 1; w < U; w <<= 1)
#pragma unroll
      for (int u = 0; u + w < U; u += 2 * w) t[k][u] += t[k][u + w];
    a[k] = t[k][0];
  }
  for (int i = lane + 64 * U; i < nw; i += 64)
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += p[(int64_t)k * nw + i];
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = wave_sum(a[k]);
}
template <int K, int U>
__device__ __forceinline__ void sum_streams(const double* __restrict__ p, int nw, double out[K]) {
  double t[K][U];
  load_streams<K, U>(p, nw, t);
  reduce_streams<K, U>(p, nw, t, out);
}
// Same sums over streams stored with an even stride, read as 16-B pairs (half the load instructions;
// the pad slot of an odd count is kept zero). U pairs per lane cover 128·U entries.
template <int K, int U>
__device__ __forceinline__ void load_streams2(const double* __restrict__ p, int nw, int stride, double2 t[K][U]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = 2 * (lane + 64 * u);
      t[k][u] = i < nw ? *reinterpret_cast<const double2*>(p + (int64_t)k * stride + i) : make_double2(0.0, 0.0);
    }
}
// the same, unconditionally: streams padded to a stride of 128·U entries with zero tails
template <int K, int U>
__device__ __forceinline__ void load_streams2_padded(const double* __restrict__ p, int stride, double2 t[K][U]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int u = 0; u < U; ++u) t[k][u] = *reinterpret_cast<const double2*>(p + (int64_t)k * stride + 2 * (lane + 64 * u));
}
template <int K, int U>
__device__ __forceinline__ void reduce_streams2(const double* __restrict__ p, int nw, int stride, double2 t[K][U],
                                                double out[K]) {
  const int lane = threadIdx.x & 63;
  double a[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = t[k][u].x + t[k][u].y;
#pragma unroll
    for (int w = 1; w < U; w <<= 1)
#pragma unroll
      for (int u = 0; u + w < U; u += 2 * w) v[u] += v[u + w];
    a[k] = v[0];
  }
  for (int i = 2 * (lane + 64 * U); i < nw; i += 128)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double2 x = *reinterpret_cast<const double2*>(p + (int64_t)k * stride + i);
      a[k] += x.x + x.y;
    }
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = wave_sum(a[k]);
}

// a / b by the hardware reciprocal, two Newton steps and one quotient correction (≈ 6 dependent operations against the
// ≈ 11 of IEEE division: div_scale, rcp, four fma, mul, fma, div_fmas, div_fixup); within an ulp of a / b for the finite,
// normal operands the PCG's step scalars are (the PCG is not bit-pinned: it uses fused multiply-adds throughout), and
// non-finite when b is 0 or non-finite, which the breakdown test catches
__device__ __forceinline__ double div_nr(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  const double q = a * r;
  return fma(r, fma(-b, q, a), q);
}

// n[c] without a dynamically indexed array (which the compiler would put in scratch): masked sum,
// exact for finite n (x·1 + 0 terms); a non-finite component poisons the row, as it would anyway.
__device__ __forceinline__ double pick6(const double n[6], int c) {
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) v += n[i] * (c == i ? 1.0 : 0.0);
  return v;
}
// (A v)_row summed over the row's kSL lanes: every lane of the row gets all 6 components.
// [b0, b1) = the row's block range (empty for padding rows).
template <typename G>
__device__ __forceinline__ void row_spmv(const G& g, int b0, int b1, int q, const double* __restrict__ v,
                                         double n[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) n[i] = 0.0;
  for (int bi = b0 + q; bi < b1; bi += kSL) {
    const double2* blk = reinterpret_cast<const double2*>(g.Aop + 36 * (int64_t)bi);
    const double2* vc = reinterpret_cast<const double2*>(v + 6 * (int64_t)g.col[bi]);
    double x[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) { const double2 t = vc[j]; x[2 * j] = t.x; x[2 * j + 1] = t.y; }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double2 b01 = blk[3 * i], b23 = blk[3 * i + 1], b45 = blk[3 * i + 2];
      n[i] += ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) n[i] = slot_sum(n[i]);
}
// row_spmv with the first two slots' blocks and gathers issued together (two dependent trips for rows of
// <= 2·kSL blocks), the same accumulation order
template <class G>
__device__ __forceinline__ void row_spmv_2(const G& g, int b0, int b1, int q, const double* __restrict__ v,
                                           double n[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) n[i] = 0.0;
  const int bi0 = b0 + q, bi1 = bi0 + kSL;
  const bool ok0 = bi0 < b1, ok1 = bi1 < b1;
  const int e[2] = {ok0 ? bi0 : 0, ok1 ? bi1 : 0};
  double x[2][6];
  double2 bb[2][18];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const double2* blk = reinterpret_cast<const double2*>(g.Aop + 36 * (int64_t)e[h]);
    const double2* vc = reinterpret_cast<const double2*>(v + 6 * (int64_t)g.col[e[h]]);
#pragma unroll
    for (int j = 0; j < 3; ++j) { const double2 t = vc[j]; x[h][2 * j] = t.x; x[h][2 * j + 1] = t.y; }
#pragma unroll
    for (int k = 0; k < 18; ++k) bb[h][k] = blk[k];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 0 ? ok0 : ok1) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 b01 = bb[h][3 * i], b23 = bb[h][3 * i + 1], b45 = bb[h][3 * i + 2];
        n[i] += ((b01.x * x[h][0] + b01.y * x[h][1]) + (b23.x * x[h][2] + b23.y * x[h][3])) +
                (b45.x * x[h][4] + b45.y * x[h][5]);
      }
    }
  }
  for (int bi = b0 + q + 2 * kSL; bi < b1; bi += kSL) {
    const double2* blk = reinterpret_cast<const double2*>(g.Aop + 36 * (int64_t)bi);
    const double2* vc = reinterpret_cast<const double2*>(v + 6 * (int64_t)g.col[bi]);
    double xx[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) { const double2 t = vc[j]; xx[2 * j] = t.x; xx[2 * j + 1] = t.y; }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double2 b01 = blk[3 * i], b23 = blk[3 * i + 1], b45 = blk[3 * i + 2];
      n[i] += ((b01.x * xx[0] + b01.y * xx[1]) + (b23.x * xx[2] + b23.y * xx[3])) + (b45.x * xx[4] + b45.y * xx[5]);
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) n[i] = slot_sum(n[i]);
}
__device__ __forceinline__ void load_rec(const double* __restrict__ st, int64_t o, double v[V_N]) {
  const double2* p = reinterpret_cast<const double2*>(st + V_N * o);
#pragma unroll
  for (int k = 0; k < V_N / 2; ++k) { const double2 t = p[k]; v[2 * k] = t.x; v[2 * k + 1] = t.y; }
}
__device__ __forceinline__ void store_rec(double* __restrict__ st, int64_t o, const double v[V_N]) {
  double2* p = reinterpret_cast<double2*>(st + V_N * o);
#pragma unroll
  for (int k = 0; k < V_N / 2; ++k) p[k] = make_double2(v[2 * k], v[2 * k + 1]);
}
// Cluster inverse storage: entry (i, j) of a cluster's 48x48 block at float (j/4 · 48 + i) · 4 + j%4,
// so row i's k-th float4 sits at float4 index k·48 + i: the 48 rows' float4 k are contiguous (LDS
// reads by 48 lanes are bank-conflict free; the block is staged to LDS as one linear image).
__device__ __forceinline__ int64_t mcl_idx(int64_t cluster, int i, int j) {
  return cluster * kCD * kCD + ((j >> 2) * kCD + i) * 4 + (j & 3);
}
// The row's (r, c) f32 row of the cluster inverse, 12 x 16-B loads.
__device__ __forceinline__ void load_mrow(const GnDev& g, int64_t o, float4 mr[kCD / 4]) {
  const float4* p = reinterpret_cast<const float4*>(g.Mcl + mcl_idx(o / kCD, (int)(o % kCD), 0));
#pragma unroll
  for (int k = 0; k < kCD / 4; ++k) mr[k] = p[k * kCD];
}
// (M⁻¹ v)_(r,c) with v the wave's cluster vector staged in LDS (s_v[6 r' + c'], f64)
// (s_v 16-B aligned: the 48 entries come as 24 broadcast reads in two batches of 12 in flight, not 12 dependent rounds)
__device__ __forceinline__ double apply_mrow(const float4 mr[kCD / 4], const double* s_v) {
  double2 vv[kCD / 2];
  const double2* sv2 = reinterpret_cast<const double2*>(s_v);
#pragma unroll
  for (int k = 0; k < kCD / 4; ++k) vv[k] = sv2[k];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = kCD / 4; k < kCD / 2; ++k) vv[k] = sv2[k];
  double a = 0.0;
#pragma unroll
  for (int k = 0; k < kCD / 4; ++k)
    a += (((double)mr[k].x * vv[2 * k].x + (double)mr[k].y * vv[2 * k].y) +
          ((double)mr[k].z * vv[2 * k + 1].x + (double)mr[k].w * vv[2 * k + 1].y));
  return a;
}

// Per cluster (one wave): LM damping of the cluster's diagonal node blocks (written back to A: the
// PCG operator is A + λI) and the explicit inverse of the damped 48x48 cluster matrix by in-place
// Gauss-Jordan (SPD: no pivoting; a non-positive or non-finite pivot falls back to M⁻¹ = I for the
// cluster), stored as symmetrised f32 rows. Lane (ti, tj) = node block (ti, tj) of the cluster, held
// in registers for all 48 (unrolled) steps; step k fetches the old row k / column k entries it needs
// from their owner lanes by cross-lane permutes and the pivot by a lane read — no LDS, no barrier.
// Cold start also: x = 0, r = b, u = M⁻¹ b, z = q = s = p = w = 0, u -> m1.
// The inversion of cluster cl (one wave, lane = node block (ti, tj)): m receives the lane's block of the symmetrised
// f32 inverse, which is also stored to Mcl; the cluster's rows' rotation accumulators restart (precond_rot_tol).
__device__ __forceinline__ void cluster_invert(const GnDev& g, const double* A, int cl, int lane, float m[6][6]) {
  const int base = cl * kCS;
  const int ti = lane / kCS, tj = lane % kCS;
  const int slot = g.map[(int64_t)(base + ti) * g.N + base + tj] - 1;
  double a[6][6];
  {
    const double2* blk = reinterpret_cast<const double2*>(A + 36 * (int64_t)(slot >= 0 ? slot : 0));
#pragma unroll
    for (int e = 0; e < 18; ++e) {
      const double2 v = slot >= 0 ? blk[e] : make_double2(0.0, 0.0);
      a[(2 * e) / 6][(2 * e) % 6] = v.x;
      a[(2 * e + 1) / 6][(2 * e + 1) % 6] = v.y;
    }
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < kCD; ++k) {
    const int K = k / 6, kr = k % 6;
    const double piv = read_lane(a[kr][kr], K * (kCS + 1));
    bad = bad || !(piv > 0.0) || !isfinite(piv);
    const double ip = 1.0 / piv;
    double rk[6], ck[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) rk[c] = __shfl(a[kr][c], K * kCS + tj, 64);
#pragma unroll
    for (int r = 0; r < 6; ++r) ck[r] = __shfl(a[r][kr], ti * kCS + K, 64);
#pragma unroll
    for (int c = 0; c < 6; ++c) rk[c] *= ip;                 // new row k (off the pivot)
    const bool rowk = ti == K, colk = tj == K;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double upd = a[r][c] - ck[r] * rk[c];
        double v = upd;
        if (c == kr) v = colk ? -ck[r] * ip : v;                // column k
        if (r == kr) v = rowk ? ((c == kr && colk) ? ip : rk[c]) : v;   // row k, pivot
        a[r][c] = v;
      }
  }
  // symmetrise with the transposed block (lane (tj, ti)), round to f32, store the cluster rows
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const double t = __shfl(a[c][r], tj * kCS + ti, 64);
      m[r][c] = bad ? ((ti == tj && r == c) ? 1.f : 0.f) : (float)(0.5 * (a[r][c] + t));
    }
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)   // (j, j+1) with j even share a float4
      *reinterpret_cast<float2*>(g.Mcl + mcl_idx(cl, 6 * ti + r, 6 * tj + 2 * c)) =
          make_float2(m[r][2 * c], m[r][2 * c + 1]);
  if (lane < kCS) g.racc[base + lane] = 0.0;
}

__global__ __launch_bounds__(64) void k_pcg_prep(GnDev g, double lm, double* __restrict__ A,
                                                 const double* __restrict__ rhs, int invert) {
  if (g.flags[F_STOPPED]) return;
  const int lane = threadIdx.x;
  const int base = blockIdx.x * kCS;
  const int ti = lane / kCS, tj = lane % kCS;
  (void)lm; (void)invert;   // A arrives damped (k_assemble)
  float m[6][6];
  cluster_invert(g, A, blockIdx.x, lane, m);
  // PCG bookkeeping of this GN step (as k_pcg_proj: after the workgroup's loads)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g.flags[F_DONE] = 0; g.flags[F_PCG_IT] = 0; g.flags[F_PCG_CNT] = 0; g.flags[F_REFRESH] = 0;
  }
  if (g.warm_now) return;
  // cold start: u = M⁻¹ b with the stored (f32) operator; the 8 lanes of a block row sum in fixed order
  double bj[6], u[6];
  const double* bc = rhs + 6 * (int64_t)(base + tj);
#pragma unroll
  for (int c = 0; c < 6; ++c) bj[c] = bc[c];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) acc += (double)m[r][c] * bj[c];
    u[r] = slot_sum(acc);
  }
  if (tj < 6) {
    const int64_t o = 6 * (int64_t)(base + ti) + tj;
    const double uo = pick6(u, tj);
    const double v[V_N] = {0.0, rhs[o], uo, 0.0, 0.0, 0.0, 0.0, 0.0};
    store_rec(g.st, o, v);
    g.m1[o] = uo;
  }
}

// ---------------------------------------------------------------------------- overlapping additive Schwarz
// M⁻¹ = Σ_c R_cᵀ (A_{D_c D_c})⁻¹ R_c over subdomains D_c = cluster c's kCS rows + its ring (on the bench graph
// 2.46x fewer PCG iterations than the cluster blocks, tools/schwarz_study.py). The apply needs w on the neighbours'
// rings, which the iteration has only after a kernel boundary, so each PCG iteration is two launches: k_pcg_iter<.., kAS>
// (SpMV, recurrences, w_new -> as_w) and k_as_apply (m_new = M⁻¹ w_new). Owner computes: the workgroup of output cluster
// c' sums, for its 48 rows, the rows of every subdomain inverse that contains them ("segments", sorted by (row, source)
// so the sum has a fixed order), from a per-cluster slab written by k_as_invert — every slab address is static, so the
// inverse rows leave with the gathered w in one memory trip.
// Setup (per pattern, on the prefetch stream): k_as_choose ranks each cluster's A-neighbours by the number of terms
// coupling them to it (blk_off counts; known before any A exists), k_as_accept lets every row keep the kAsX best of the
// rings that chose it (bounds the tables), k_as_compact writes the subdomains, k_as_segments the apply's tables.

// the candidate ring of cluster c: its distinct A-neighbours outside the cluster, best kAsRing by (terms desc, row asc)
// (a thread per block of the cluster's rows)
__global__ __launch_bounds__(256) void k_as_choose(GnDev g) {
  __shared__ int s_u[256], s_n[256], s_sc[256];
  const int c = blockIdx.x, t = threadIdx.x;
  const int b0 = g.row_ptr[c * kCS], b1 = g.row_ptr[(c + 1) * kCS];
  const int ne = min(b1 - b0, 256);
  int u = -1, n = 0;
  if (t < ne) {
    const int b = b0 + t;
    const int x = g.blk_row[b];
    u = g.col[b];
    if (u / kCS == c) {
      u = -1;
    } else {
      const int lo = min(x, u), hi = max(x, u);
      const int up = g.up_of[g.map[(int64_t)lo * g.N + hi] - 1];
      n = g.blk_off[up + 1] - g.blk_off[up];
    }
  }
  s_u[t] = u;
  s_n[t] = n;
  __syncthreads();
  int sc = -1;   // per distinct candidate (its first entry): the terms coupling it to the cluster
  if (u >= 0) {
    bool first = true;
    int sum = 0;
    for (int f = 0; f < ne; ++f)
      if (s_u[f] == u) { sum += s_n[f]; first = first && f >= t; }
    sc = first ? sum : -1;
  }
  s_sc[t] = sc;
  const int nrep = __syncthreads_count(sc >= 0);
  if (sc >= 0) {
    int rank = 0;
    for (int f = 0; f < ne; ++f) {
      const int s2 = s_sc[f];
      rank += (s2 > sc || (s2 == sc && s_u[f] < u)) ? 1 : 0;
    }
    if (rank < kAsRing) {
      g.as_cand[c * kAsRing + rank] = u;
      g.as_csc[c * kAsRing + rank] = sc;
    }
  }
  if (t >= nrep && t < kAsRing) g.as_cand[c * kAsRing + t] = -1;
}

// row v keeps the kAsX best (terms desc, cluster asc) of the rings that chose it (one wave per row, a lane per block:
// each choosing cluster seen through the first of v's blocks into it — the pattern is symmetric, so a cluster that chose
// v holds a neighbour of v)
__global__ __launch_bounds__(256) void k_as_accept(GnDev g) {
  __shared__ int s_ci[4][64], s_si[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + w;
  if (v >= g.N) return;   // (wave-uniform: no barrier below)
  const int cv = v / kCS;
  const int b0 = g.row_ptr[v], b1 = g.row_ptr[v + 1];
  const int ci = b0 + lane < b1 ? g.col[b0 + lane] / kCS : -1;
  s_ci[w][lane] = ci;
  wave_lds_sync();
  bool ok = ci >= 0 && ci != cv;
  for (int j = 0; j < lane && ok; ++j) ok = s_ci[w][j] != ci;   // first block into the cluster
  int ki = -1, si = -1;
  if (ok) {
    int cand[kAsRing];
#pragma unroll
    for (int k = 0; k < kAsRing; ++k) cand[k] = g.as_cand[ci * kAsRing + k];
#pragma unroll
    for (int k = 0; k < kAsRing; ++k) ki = cand[k] == v ? k : ki;
    if (ki >= 0) si = g.as_csc[ci * kAsRing + ki];
  }
  s_si[w][lane] = si;
  wave_lds_sync();
  if (si < 0) return;
  int rank = 0;
  for (int j = 0; j < b1 - b0 && j < 64; ++j) {
    const int sj = s_si[w][j], cj = s_ci[w][j];
    rank += (sj >= 0 && (sj > si || (sj == si && cj < ci))) ? 1 : 0;
  }
  g.as_acc[ci * kAsRing + ki] = rank < kAsX ? 1 : 0;
}

// subdomain rows of cluster c: its own kCS rows, then the kept ring rows in rank order, -1 after
__global__ __launch_bounds__(64) void k_as_compact(GnDev g) {
  const int c = blockIdx.x, lane = threadIdx.x;
  int u = -1;
  bool keep = false;
  if (lane < kAsRing) {
    u = g.as_cand[c * kAsRing + lane];
    keep = u >= 0 && g.as_acc[c * kAsRing + lane] != 0;
  }
  const uint64_t m = __ballot(keep);
  const int pos = kCS + __popcll(m & ((1ull << lane) - 1));
  const int cnt = kCS + __popcll(m);
  if (keep) g.as_dom[c * kAsDN + pos] = u;
  if (lane < kCS) g.as_dom[c * kAsDN + lane] = c * kCS + lane;
  if (lane >= cnt && lane < kAsDN) g.as_dom[c * kAsDN + lane] = -1;
}

// the apply's tables of output cluster c': its source subdomains (c' and every cluster whose ring holds one of its rows,
// ascending), the gather list, the segments (row r, source s) in (r, s) order with their source slots and row offsets,
// and for each segment its slab position in the source's as_dst (a thread per block of the cluster's rows)
__global__ __launch_bounds__(256) void k_as_segments(GnDev g) {
  __shared__ int s_c[256], s_k[256];
  __shared__ int s_src[kAsSrc];
  __shared__ int s_pos[kAsSrc][kCS];
  const int cp = blockIdx.x, t = threadIdx.x;
  const int b0 = g.row_ptr[cp * kCS], b1 = g.row_ptr[(cp + 1) * kCS];
  const int ne = min(b1 - b0, 255);
  const int c = t < ne ? g.col[b0 + t] / kCS : (t == ne ? cp : -1);
  s_c[t] = c;
  if (t < kAsSrc * kCS) s_pos[t / kCS][t % kCS] = -1;
  __syncthreads();
  bool keep = c >= 0;
  for (int f = 0; f < t && keep; ++f) keep = s_c[f] != c;   // first occurrence
  if (keep && c != cp) {
    int dom[kAsRing];
#pragma unroll
    for (int l = 0; l < kAsRing; ++l) dom[l] = g.as_dom[c * kAsDN + kCS + l];
    bool hit = false;
#pragma unroll
    for (int l = 0; l < kAsRing; ++l) hit = hit || (dom[l] >= 0 && dom[l] / kCS == cp);
    keep = hit;
  }
  s_k[t] = keep ? c : -1;
  const int nsrc = min(__syncthreads_count(keep), kAsSrc);   // (<= 1 + kCS·kAsX by k_as_accept)
  if (keep) {
    int slot = 0;
    for (int f = 0; f < 256; ++f) slot += (s_k[f] >= 0 && s_k[f] < c) ? 1 : 0;
    if (slot < kAsSrc) s_src[slot] = c;
  }
  __syncthreads();
  for (int i = t; i < nsrc * kAsDN; i += 256) {
    const int sl = i / kAsDN, l = i % kAsDN;
    const int u = g.as_dom[s_src[sl] * kAsDN + l];
    if (u >= 0 && u / kCS == cp) s_pos[sl][u % kCS] = l;
  }
  for (int i = t; i < kAsGat; i += 256) {
    const int sl = i / kAsDN, l = i % kAsDN;
    g.as_gat[(int64_t)cp * kAsGat + i] = sl < nsrc ? g.as_dom[s_src[sl] * kAsDN + l] : -1;
  }
  __syncthreads();
  if (t >= 64) return;
  // lane r < 48: output row r's segments (one per source holding its node), offsets by a wave scan
  const int lane = t;
  const int r = lane < 6 * kCS ? lane : 6 * kCS - 1;
  int cnt = 0;
  for (int sl = 0; sl < nsrc; ++sl) cnt += s_pos[sl][r / 6] >= 0 ? 1 : 0;
  if (lane >= 6 * kCS) cnt = 0;
  int off = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(off, o, 64);
    if (lane >= o) off += y;
  }
  const int total = __shfl(off, 63, 64);
  off -= cnt;   // exclusive
  int32_t* mt = g.as_meta + (int64_t)cp * kAsMeta;
  if (lane < 6 * kCS) {
    mt[2 + lane] = off;
    int rs = off;
    for (int sl = 0; sl < nsrc; ++sl) {
      const int l = s_pos[sl][r / 6];
      if (l < 0) continue;
      mt[64 + rs] = sl;
      g.as_dst[(int64_t)s_src[sl] * kAsD + 6 * l + r % 6] = cp * kAsRS + rs;
      ++rs;
    }
  }
  if (lane == 0) { mt[0] = total; mt[1] = nsrc; mt[2 + 6 * kCS] = total; }
  if (lane < kAsSrc) g.as_src[cp * kAsSrc + lane] = lane < nsrc ? s_src[lane] : 0;
}

// ---- tables of the one-launch iteration (k_as_iter; setup, per pattern)
// every row's subdomain memberships as y indices c·kAsD + 6·l (its own subdomain + <= kAsX rings; as_memn zeroed first)
__global__ __launch_bounds__(256) void k_as_members(GnDev g, int ncl) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ncl * kAsDN) return;
  const int c = i / kAsDN, l = i % kAsDN;
  const int u = g.as_dom[i];
  if (u < 0) return;
  const int pos = atomicAdd(g.as_memn + u, 1);
  if (pos < 1 + kAsX) g.as_mem[4 * (int64_t)u + pos] = c * kAsD + 6 * l;
}

// per subdomain c (one workgroup): its rows' blocks in row order, the distinct columns S2 (ascending) with each block's
// S2 index, per S2 node its memberships ascending (the order the apply sums a row's segments in), the row starts and
// every subdomain row's S2 index (its diagonal block's column)
__global__ __launch_bounds__(256) void k_as_tab(GnDev g) {
  __shared__ int s_dom[kAsDN], s_rs[kAsDN + 1];
  __shared__ int s_col[kGB], s_slot[kGB], s_l[kGB], s_first[kGB], s_rank[kGB];
  __shared__ int s_key[kGB], s_scan[kGB], s_len[kAsDN], s_r0[kAsDN];
  const int c = blockIdx.x, t = threadIdx.x;
  const AsTabP tp = as_tab_at(g.as_tab, g.as_tab_cap);
  if (t < kAsDN) {   // every row's length in parallel (one trip; the serial loop below waited for each row's in turn)
    const int d = g.as_dom[c * kAsDN + t];
    s_dom[t] = d;
    const int r0 = g.row_ptr[d >= 0 ? d : 0], r1 = g.row_ptr[d >= 0 ? d + 1 : 0];
    s_r0[t] = r0;
    s_len[t] = d >= 0 ? r1 - r0 : 0;
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0, l = 0;
    for (; l < kAsDN && s_dom[l] >= 0; ++l) {
      s_rs[l] = acc;
      acc += s_len[l];
    }
    for (; l <= kAsDN; ++l) s_rs[l] = acc;
  }
  __syncthreads();
  int nd = 0;
  while (nd < kAsDN && s_dom[nd] >= 0) ++nd;
  const int nb = s_rs[kAsDN];   // (<= kAsDN·kRowMax <= kGB: the Schwarz form needs rows of <= kRowMax blocks)
  for (int i = t; i < kGB; i += 256) {
    if (i < nb) {
      int l = 0;
      while (l + 1 < nd && s_rs[l + 1] <= i) ++l;
      const int b = s_r0[l] + (i - s_rs[l]);
      s_col[i] = g.col[b]; s_slot[i] = b; s_l[i] = l;
      s_key[i] = (g.col[b] << 9) | i;   // (rows < 2^22)
    } else {
      s_col[i] = 0x7FFFFFFF; s_slot[i] = 0; s_l[i] = 0;
      s_key[i] = 0x7FFFFFFF;
    }
  }
  __syncthreads();
  // bitonic sort of (column, block) keys: S2 = the distinct columns in ascending order, each block's rank among them,
  // and "first" = the lowest block index of its column (the key breaks ties by block)
  for (int k = 2; k <= kGB; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < kGB; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const int a = s_key[i], b = s_key[ixj];
          if (((i & k) == 0) == (a > b)) { s_key[i] = b; s_key[ixj] = a; }
        }
      }
      __syncthreads();
    }
  for (int i = t; i < kGB; i += 256)
    s_scan[i] = (i < nb && (i == 0 || (s_key[i] >> 9) != (s_key[i - 1] >> 9))) ? 1 : 0;
  __syncthreads();
  for (int o = 1; o < kGB; o <<= 1) {   // inclusive scan of the first flags
    int v[2];
    for (int q = 0; q < 2; ++q) { const int i = t + 256 * q; v[q] = s_scan[i] + (i >= o ? s_scan[i - o] : 0); }
    __syncthreads();
    for (int q = 0; q < 2; ++q) s_scan[t + 256 * q] = v[q];
    __syncthreads();
  }
  for (int i = t; i < nb; i += 256) {
    const int idx = s_key[i] & (kGB - 1);
    s_rank[idx] = s_scan[i] - 1;
    s_first[idx] = (i == 0 || (s_key[i] >> 9) != (s_key[i - 1] >> 9)) ? 1 : 0;
  }
  __syncthreads();
  const int ns = nb > 0 ? s_scan[nb - 1] : 0;
  // entries past nb / ns repeat the last valid one: k_as_iter's idle lanes load unconditionally, and a common padding
  // address (block 0, y[0]) would be one L2 channel hit by every workgroup
  for (int i = t; i < kGB; i += 256) {
    const int j = i < nb ? i : nb - 1;
    tp.blk[(int64_t)c * kGB + i] = make_int2(s_slot[j], (s_rank[j] << 5) | s_l[j]);
  }
  for (int i = t; i < nb; i += 256) {
    if (!s_first[i]) continue;
    const int u = s_col[i], k = s_rank[i];
    const int n = min(g.as_memn[u], 1 + kAsX);
    int m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = j < n ? g.as_mem[4 * (int64_t)u + j] : 0x7FFFFFFF;
#pragma unroll
    for (int a = 0; a < 4; ++a)   // ascending (the y index grows with the subdomain)
#pragma unroll
      for (int b = 0; b < 3 - a; ++b)
        if (m[b] > m[b + 1]) { const int x = m[b]; m[b] = m[b + 1]; m[b + 1] = x; }
    const int4 e = make_int4(m[0] == 0x7FFFFFFF ? -1 : m[0], m[1] == 0x7FFFFFFF ? -1 : m[1],
                             m[2] == 0x7FFFFFFF ? -1 : m[2], m[3] == 0x7FFFFFFF ? -1 : m[3]);
    tp.con[(int64_t)c * kGS + k] = e;
    tp.s2n[(int64_t)c * kGS + k] = u;
    if (k == ns - 1)   // (the padding past ns: copies of the last node's entries)
      for (int kk = ns; kk < kGS; ++kk) { tp.con[(int64_t)c * kGS + kk] = e; tp.s2n[(int64_t)c * kGS + kk] = u; }
  }
  int32_t* rt = tp.row + (int64_t)c * kGRow;
  if (t <= kAsDN) rt[t] = s_rs[t];
  if (t == 0) { rt[25] = nd; rt[26] = nb; rt[27] = ns; }
  if (t < kAsDN) rt[64 + t] = t < nd ? s_dom[t] : 0;
  for (int i = t; i < nb; i += 256)   // the subdomain row's S2 index: the rank of its diagonal block's column
    if (s_col[i] == s_dom[s_l[i]]) rt[32 + s_l[i]] = s_rank[i];
  if (t >= nd && t < kAsDN) rt[32 + t] = 0;
}

// Per subdomain c (one workgroup of TR x TC threads): the dense damped A_{D_c D_c} (<= kAsD x kAsD, f64, NA x NB entries
// per thread in registers: rows tr + TR·a, columns tc + TC·b), its in-place block Gauss-Jordan inverse (SPD: no pivoting;
// 2x2 pivot blocks through LDS, double-buffered: one barrier per two steps), scaled and rounded to fp16 with a certified
// diagonal margin (below) and written symmetric into the segments' slab rows; a non-positive or non-finite pivot falls
// back to the identity on the cluster's own rows; the cluster's rows' rotation accumulators restart (precond_rot_tol).
// k_as_invert and the refresh inside k_pcg_proj run it on 16 x 16 threads (four waves, 9 x 9 entries each; a 16 x 48
// grid was measured slower, k_as_invert). The arithmetic per entry is the same for any grid. (Every thread of the
// workgroup must call it: it synchronises the workgroup.)
template <int TR, int TC>
__device__ __forceinline__ void as_invert_body(const GnDev& g, const double* __restrict__ A, int c, int t) {
  static_assert(TR == 16 && TC % 16 == 0, "pivot steps: row tile K = k / 16, column tile k / TC");
  constexpr int T = TR * TC, NA = (kAsD + TR - 1) / TR, NB = (kAsD + TC - 1) / TC, kTM = TC / 16;
  constexpr int kSR = TR * NA > TC * NB ? TR * NA : TC * NB;
  __shared__ int s_dom[kAsDN];
  __shared__ int s_sl[kAsDN][kAsDN];
  __shared__ int s_dst[kAsD];
  __shared__ double s_row[2][2][kSR], s_col[2][2][kSR];
  __shared__ __attribute__((aligned(16))) uint16_t s_z[kAsD * kAsD];   // the stored fp16 form, (R, C), both triangles
  const int tr = t / TC, tc = t % TC;
#ifdef OFX_STAMPS   // tuning build: phase stamps of thread 0 in the stamps buffer's iteration-63 slot
#define OFX_AS_STAMP(k) \
  if (t == 0 && g.stamps) g.stamps[((int64_t)63 * g.nwg_row + c) * 8 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define OFX_AS_STAMP(k)
#endif
  OFX_AS_STAMP(0)
  if (t < kAsDN) s_dom[t] = g.as_dom[c * kAsDN + t];
  if (t < kAsD) s_dst[t] = g.as_dst[(int64_t)c * kAsD + t];
  __syncthreads();
  int nd = 0;
  for (int i = 0; i < kAsDN; ++i) nd += s_dom[i] >= 0 ? 1 : 0;
  for (int p = t; p < kAsDN * kAsDN; p += T) {
    const int i = p / kAsDN, j = p % kAsDN;
    s_sl[i][j] = (i < nd && j < nd) ? g.map[(int64_t)s_dom[i] * g.N + s_dom[j]] - 1 : -1;
  }
  __syncthreads();
  const int n = 6 * nd;
  // every load unconditional (clamped addresses, masked values): a load behind a branch gets its own wait
  double M[NA][NB];
  int slv[NA][NB];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int R = tr + TR * a, C = tc + TC * b;
      const int sl = (R < n && C < n) ? s_sl[min(R / 6, kAsDN - 1)][min(C / 6, kAsDN - 1)] : -1;
      slv[a][b] = sl;
      M[a][b] = A[36 * (int64_t)(sl >= 0 ? sl : 0) + 6 * (R % 6) + C % 6];
    }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int R = tr + TR * a, C = tc + TC * b;
      // (beyond n: the identity, never touched by the steps below)
      M[a][b] = (R < n && C < n) ? (slv[a][b] >= 0 ? M[a][b] : 0.0) : (R == C ? 1.0 : 0.0);
    }
  OFX_AS_STAMP(1)
  bool bad = false;
  int buf = 0;
  // Block Gauss-Jordan with 2x2 pivot blocks P = rows / columns {k, k+1} (two elimination steps per barrier: the barrier
  // and LDS latency per step, not the FMAs, set the time with four waves). Step k = 16·K + kk, kk even: the pivot rows are
  // row tile K of threads tr = kk, kk + 1, the pivot columns column tile KB = K / kTM of threads tc = 16·(K % kTM) + kk,
  // + 1 (compile-time tile indices: M[K][.] / M[.][KB] stay in registers).
  auto step2 = [&](auto Kc, int kk) {
    constexpr int K = decltype(Kc)::value;
    if constexpr (K < NA) {   // (discarded for K = 8 with 8-row tiles)
    constexpr int KB = K / kTM, kc0 = 16 * (K % kTM);
    const int k = 16 * K + kk;
    if (tr == kk || tr == kk + 1)
#pragma unroll
      for (int b = 0; b < NB; ++b) s_row[buf][tr - kk][tc + TC * b] = M[K][b];
    if (tc == kc0 + kk || tc == kc0 + kk + 1)
#pragma unroll
      for (int a = 0; a < NA; ++a) s_col[buf][tc - kc0 - kk][tr + TR * a] = M[a][KB];
    __syncthreads();
    const double p00 = s_row[buf][0][k], p01 = s_row[buf][0][k + 1], p10 = s_row[buf][1][k], p11 = s_row[buf][1][k + 1];
    const double det = p00 * p11 - p01 * p10;
    bad = bad || !(p00 > 0.0) || !(det > 0.0) || !isfinite(det);
    const double idet = 1.0 / det;
    const double q00 = p11 * idet, q01 = -p01 * idet, q10 = -p10 * idet, q11 = p00 * idet;   // P⁻¹
    double v0[NB], v1[NB], c0[NA], c1[NA];
#pragma unroll
    for (int b = 0; b < NB; ++b) {   // P⁻¹ A_{K,j}
      const double r0 = s_row[buf][0][tc + TC * b], r1 = s_row[buf][1][tc + TC * b];
      v0[b] = fma(q01, r1, q00 * r0);
      v1[b] = fma(q11, r1, q10 * r0);
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) { c0[a] = s_col[buf][0][tr + TR * a]; c1[a] = s_col[buf][1][tr + TR * a]; }
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) M[a][b] = fma(-c1[a], v1[b], fma(-c0[a], v0[b], M[a][b]));   // (pivot rows / columns below)
    if (tr == kk || tr == kk + 1)
#pragma unroll
      for (int b = 0; b < NB; ++b) M[K][b] = tr == kk ? v0[b] : v1[b];
    if (tc == kc0 + kk || tc == kc0 + kk + 1) {
      const double e0 = tc == kc0 + kk ? q00 : q01, e1 = tc == kc0 + kk ? q10 : q11;
#pragma unroll
      for (int a = 0; a < NA; ++a) M[a][KB] = -fma(c1[a], e1, c0[a] * e0);
      if (tr == kk || tr == kk + 1) M[K][KB] = tr == kk ? e0 : e1;   // the pivot block: P⁻¹
    }
    buf ^= 1;
    }
  };
#define OFX_AS_STEPS(K) \
  for (int kk = 0; kk < 16 && 16 * (K) + kk < n; kk += 2) step2(std::integral_constant<int, (K)>{}, kk);
  OFX_AS_STEPS(0) OFX_AS_STEPS(1) OFX_AS_STEPS(2) OFX_AS_STEPS(3)
  OFX_AS_STEPS(4) OFX_AS_STEPS(5) OFX_AS_STEPS(6) OFX_AS_STEPS(7)
  OFX_AS_STEPS(8)
#undef OFX_AS_STEPS
  bad = __syncthreads_or(bad ? 1 : 0) != 0;
  OFX_AS_STAMP(2)
  // Stored form: Z = D Ẑ D with d = √diag(Z), so Ẑ has a unit diagonal and |Ẑ_ij| <= 1 (Z is SPD), and Ẑ's off-diagonal
  // entries as fp16 (absolute error <= 2^-12). E = the rounding of the off-diagonal entries; the diagonal is stored as
  // 1 + σ with σ = ‖E‖_F + 2^-10 >= ‖E‖₂ + the diagonal's own rounding, so the stored Ẑ̃ >= Ẑ: positive definite whatever
  // Z's conditioning (a plain 16-bit rounding of Z made the moose's subdomains indefinite). A bad domain: the identity on
  // the cluster's own rows.
  __shared__ double s_d[kSR], s_e[T];
  __shared__ double s_sig;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int R = tr + TR * a, C = tc + TC * b;
      if (R == C) s_d[R] = (R < n && !bad) ? sqrt(M[a][b]) : 1.0;
    }
  __syncthreads();
  double dr[NA], dc[NB];
#pragma unroll
  for (int a = 0; a < NA; ++a) dr[a] = s_d[tr + TR * a];
#pragma unroll
  for (int b = 0; b < NB; ++b) dc[b] = s_d[tc + TC * b];
  auto h16 = [](double z) -> _Float16 { return (_Float16)(float)z; };
  double e2 = 0.0;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int R = tr + TR * a, C = tc + TC * b;
      if (R < n && C < n && R < C && !bad) {
        const double z = M[a][b] / (dr[a] * dc[b]);
        const double err = (double)(float)h16(z) - z;
        e2 += 2.0 * err * err;
      }
    }
  s_e[t] = e2;
  __syncthreads();
  if (t < 64) {   // ‖E‖²_F: each lane its strided share of the threads' sums, then the wave (a fixed order)
    double sum = 0.0;
    for (int i = t; i < T; i += 64) sum += s_e[i];
    sum = wave_sum(sum);
    if (t == 0) s_sig = sqrt(sum) + 0x1p-10;
  }
  __syncthreads();
  OFX_AS_STAMP(3)
  const double sig = s_sig;
  // the stored form into LDS (the upper triangle's value to both entries), then the rows to their segments' slab rows
  // as 16-B words (scattered 2-B stores of the entries cost ~80 us per solve)
  auto b16 = [](_Float16 h) { return __builtin_bit_cast(uint16_t, h); };
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int R = tr + TR * a, C = tc + TC * b;
      if (R >= n || C >= kAsD) continue;
      if (C >= n) {
        s_z[R * kAsD + C] = 0;
      } else if (R == C) {
        s_z[R * kAsD + C] = b16(bad ? (_Float16)(R < 6 * kCS ? 1.0f : 0.0f) : h16(1.0 + sig));
      } else if (R < C) {
        const uint16_t h = b16(bad ? (_Float16)0.0f : h16(M[a][b] / (dr[a] * dc[b])));
        s_z[R * kAsD + C] = h;
        s_z[C * kAsD + R] = h;
      }
    }
  if (tc == 0)
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int R = tr + TR * a;
      if (R < kAsD) g.as_dsc[(int64_t)c * kAsD + R] = R < n ? (float)dr[a] : 0.f;
      if (R < kAsD && g.as_one) as_tab_at(g.as_tab, g.as_tab_cap).dsc[(int64_t)c * kAsD + R] = R < n ? (float)dr[a] : 0.f;
      if (R < n) g.as_rsc[s_dst[R]] = (float)dr[a];
    }
  __syncthreads();
  OFX_AS_STAMP(4)
  for (int i = t; i < n * kAsK; i += T) {
    const int R = i / kAsK, k = i % kAsK;
    const int d = s_dst[R], cp = d / kAsRS, rs = d % kAsRS;
    reinterpret_cast<uint4*>(g.as_slab)[((int64_t)cp * kAsK + k) * kAsRS + rs] =
        reinterpret_cast<const uint4*>(s_z + R * kAsD)[k];
  }
  if (g.as_one) {   // k_as_iter's subdomain-ordered copy: word k of row R at slab[(c·kAsK + k)·kAsD + R] (rows fastest)
    uint4* sl = as_tab_at(g.as_tab, g.as_tab_cap).slab + (int64_t)c * kAsK * kAsD;
    for (int i = t; i < n * kAsK; i += T) {
      const int k = i / n, R = i - k * n;
      sl[(int64_t)k * kAsD + R] = reinterpret_cast<const uint4*>(s_z + R * kAsD)[k];
    }
  }
  if (t < kCS) g.racc[c * kCS + t] = 0.0;
  OFX_AS_STAMP(5)
#undef OFX_AS_STAMP
}

// k_as_invert's MFMA form (round 6; OFX_AS_INV_MFMA=1 — as_invert_body stays the default, measured faster below): the same damped
// A_{D_c D_c}, inverted by a blocked Gauss-Jordan on 16 x 16 tiles with f64 MFMA (v_mfma_f64_16x16x4f64) in place of
// 72 two-pivot VALU steps. One workgroup of kNT waves per subdomain: wave w holds tile column w of the padded
// kNP x kNP matrix as MFMA accumulators (tile i, lane l, entry r: row 16·i + (l >> 4) + 4r, column 16·w + (l & 15)).
// Per 16-row panel p: (a) wave p publishes its column — the pivot columns C, with the pivot block as P - I — and P;
// (b) every wave inverts P itself (scalar Gauss-Jordan in its LDS copy, SPD: no pivoting); (c) every wave forms its
// V' = P⁻¹ R_w (R_w: its own tile of the pivot rows) or, in the pivot column, I + P⁻¹; (d) every tile M -= C V' (four
// MFMAs): off the panel the Schur update, on the pivot rows V, on the pivot columns -C P⁻¹, on the pivot block P⁻¹.
// A tile in the C/D layout is already the B operand of its k-steps (register r = k-step), so V' never leaves the
// registers; one barrier per panel (C and P double-buffered). Then the stored form as as_invert_body (scales d, fp16
// Ẑ with the certified margin σ, the slab rows), up to f64 rounding of the inverse.
typedef double as_d4 __attribute__((ext_vector_type(4)));
constexpr int kNT = (kAsD + 15) / 16, kNP = 16 * kNT, kInvT = 64 * kNT;
__device__ __forceinline__ void as_invert_mfma(const GnDev& g, const double* __restrict__ A, int c, int t) {
  constexpr int kPanel = 16 * kNP;                             // doubles of one pivot-column panel
  constexpr int kGJ = (2 * kPanel + 2 * 16 * 17) * 8, kZ = kAsD * kAsD * 2;
  __shared__ __attribute__((aligned(16))) char s_buf[kGJ > kZ ? kGJ : kZ];   // the panels, then the stored form
  __shared__ int s_dom[kAsDN];
  __shared__ int s_sl[kAsDN][kAsDN];
  __shared__ int s_dst[kAsD];
  __shared__ double s_d[kNP], s_e[kInvT];
  __shared__ double s_sig;
  double* s_C = reinterpret_cast<double*>(s_buf);      // [2][kNP][16] the pivot columns (pivot block: P - I)
  double* s_P = s_C + 2 * kPanel;                      // [2][16][17] P⁻¹ (wave p's Gauss-Jordan in place; column 16: scratch)
  uint16_t* s_z = reinterpret_cast<uint16_t*>(s_buf);  // (after the elimination) the stored fp16 form, (R, C)
  const int l = t & 63, lr = l >> 4, lc = l & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
#ifdef OFX_STAMPS
#define OFX_AS_STAMP(k) \
  if (t == 0 && g.stamps) g.stamps[((int64_t)63 * g.nwg_row + c) * 8 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define OFX_AS_STAMP(k)
#endif
  OFX_AS_STAMP(0)
  if (t < kAsDN) s_dom[t] = g.as_dom[c * kAsDN + t];
  if (t < kAsD) s_dst[t] = g.as_dst[(int64_t)c * kAsD + t];
  __syncthreads();
  int nd = 0;
  for (int i = 0; i < kAsDN; ++i) nd += s_dom[i] >= 0 ? 1 : 0;
  for (int q = t; q < kAsDN * kAsDN; q += kInvT) {
    const int i = q / kAsDN, j = q % kAsDN;
    s_sl[i][j] = (i < nd && j < nd) ? g.map[(int64_t)s_dom[i] * g.N + s_dom[j]] - 1 : -1;
  }
  __syncthreads();
  const int n = 6 * nd;
  const int C0 = 16 * w + lc;   // the lane's column
  auto slot = [&](int R, int C) { return (R < n && C < n) ? s_sl[min(R / 6, kAsDN - 1)][min(C / 6, kAsDN - 1)] : -1; };
  as_d4 acc[kNT];
  // every load unconditional (clamped addresses), masked after (the slot looked up again: no registers held)
#pragma unroll
  for (int i = 0; i < kNT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int R = 16 * i + lr + 4 * r;
      const int sl = slot(R, C0);
      acc[i][r] = A[36 * (int64_t)(sl >= 0 ? sl : 0) + 6 * (R % 6) + C0 % 6];
      if (r == 3) __builtin_amdgcn_sched_barrier(0);   // (per tile: the registers)
    }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < kNT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int R = 16 * i + lr + 4 * r;
      // (beyond n: the identity, which the elimination leaves alone)
      acc[i][r] = (R < n && C0 < n) ? (slot(R, C0) >= 0 ? acc[i][r] : 0.0) : (R == C0 ? 1.0 : 0.0);
      if (r == 3) __builtin_amdgcn_sched_barrier(0);
    }
  OFX_AS_STAMP(1)
  bool bad = false;
#ifdef OFX_STAMPS
  uint64_t st_b = 0, st_d = 0;
#endif
  for (int p = 0; p < kNT && 16 * p < n; ++p) {
    // (the lane's row / column offsets from an opaque copy: otherwise every address of the unrolled body is hoisted out
    // of the panel loop and held in registers, which spilled)
    int lo = l;
    asm volatile("" : "+v"(lo));
    const int lr = lo >> 4, lc = lo & 15;
    double* sC = s_C + (p & 1) * kPanel;
    double* sP = s_P + (p & 1) * 16 * 17;
#ifdef OFX_STAMPS
    const uint64_t tb0 = __builtin_amdgcn_s_memtime();
#endif
    // (a) wave p: its column (the pivot columns; the pivot block as P - I) and P⁻¹ (in-place Gauss-Jordan with scalar
    // pivots, SPD: no pivoting; row k and column k of the current block published per step, a wave's LDS operations
    // completing in order); the other waves wait at the barrier
    double e[4];
    if (w == p) {
#pragma unroll
      for (int i = 0; i < kNT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = lr + 4 * r;
          sC[(16 * i + row) * 16 + lc] = acc[i][r] - (i == p && row == lc ? 1.0 : 0.0);
          if (i == p) e[r] = acc[i][r];
        }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (lr == (k & 3)) sP[k * 17 + lc] = e[k >> 2];
        if (lc == k)
#pragma unroll
          for (int r = 0; r < 4; ++r) sP[(lr + 4 * r) * 17 + 16] = e[r];
        wave_lds_sync();   // (other lanes' writes: no load may move above them)
        const double piv = sP[k * 17 + k], rk = sP[k * 17 + lc];
        double ck[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ck[r] = sP[(lr + 4 * r) * 17 + 16];
        bad = bad || !(piv > 0.0) || !isfinite(piv);
        const double ip = 1.0 / piv;
        const double rki = rk * ip;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = lr + 4 * r;
          e[r] = row == k ? (lc == k ? ip : rki) : (lc == k ? -ck[r] * ip : fma(-ck[r], rki, e[r]));
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sP[(lr + 4 * r) * 17 + lc] = e[r];
    }
    __syncthreads();
#ifdef OFX_STAMPS
    const uint64_t tb1 = __builtin_amdgcn_s_memtime();
    st_b += tb1 - tb0;
#endif
    // (c) V' = P⁻¹ R_w (R_w = tile p of the wave's column, in the C/D layout = the B operand by k-step), or I + P⁻¹
    as_d4 v;
    if (w == p) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = e[r] + (lr + 4 * r == lc ? 1.0 : 0.0);
    } else {
      as_d4 rw = acc[0];
#pragma unroll
      for (int i = 1; i < kNT; ++i)
        if (i == p) rw = acc[i];
      v = as_d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        v = __builtin_amdgcn_mfma_f64_16x16x4f64(sP[lc * 17 + 4 * s4 + lr], rw[s4], v, 0, 0, 0);
    }
    // (d) every tile of the column: M -= C V'
#pragma unroll
    for (int i = 0; i < kNT; ++i) {
      const double* ca = sC + (16 * i + lc) * 16 + lr;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(-ca[4 * s4], v[s4], acc[i], 0, 0, 0);
      if (i & 1) __builtin_amdgcn_sched_barrier(0);
    }
#ifdef OFX_STAMPS
    asm volatile("" :: "v"(acc[0]));
    st_d += __builtin_amdgcn_s_memtime() - tb1;
#endif
  }
#ifdef OFX_STAMPS
  if (t == 0 && g.stamps) {
    g.stamps[((int64_t)63 * g.nwg_row + c) * 8 + 6] = st_b;
    g.stamps[((int64_t)63 * g.nwg_row + c) * 8 + 7] = st_d;
  }
#endif
  bad = __syncthreads_or(bad ? 1 : 0) != 0;   // (also: every panel read is done before s_z reuses the buffer)
  OFX_AS_STAMP(2)
  // the stored form (as_invert_body's): d = √diag Z, Ẑ = Z / (d dᵀ) in fp16 with the diagonal 1 + σ
#pragma unroll
  for (int r = 0; r < 4; ++r)   // (the diagonal: tile w of column w)
    if (lr + 4 * r == lc) {
      const int R = 16 * w + lc;
      as_d4 dd = acc[0];
#pragma unroll
      for (int i = 1; i < kNT; ++i)
        if (i == w) dd = acc[i];
      s_d[R] = (R < n && !bad) ? sqrt(dd[r]) : 1.0;
    }
  __syncthreads();
  auto h16 = [](double z) -> _Float16 { return (_Float16)(float)z; };
  auto b16 = [](_Float16 h) { return __builtin_bit_cast(uint16_t, h); };
  // the off-diagonal entries (one division each: rounded, their error summed, both triangles written); the diagonal
  // after σ below
  double e2 = 0.0;
  const double dC = s_d[C0];
#pragma unroll
  for (int i = 0; i < kNT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int R = 16 * i + lr + 4 * r;
      if (R >= n || C0 >= kAsD) continue;
      if (C0 >= n) {
        s_z[R * kAsD + C0] = 0;
      } else if (R < C0) {
        const double z = bad ? 0.0 : acc[i][r] / (s_d[R] * dC);
        const _Float16 h = h16(z);
        const double err = (double)(float)h - z;
        e2 += 2.0 * err * err;
        s_z[R * kAsD + C0] = b16(h);
        s_z[C0 * kAsD + R] = b16(h);
      }
      if (r == 3) __builtin_amdgcn_sched_barrier(0);
    }
  s_e[t] = e2;
  __syncthreads();
  if (t < 64) {   // ‖E‖²_F in a fixed order
    double sum = 0.0;
    for (int i = t; i < kInvT; i += 64) sum += s_e[i];
    sum = wave_sum(sum);
    if (t == 0) s_sig = sqrt(sum) + 0x1p-10;
  }
  __syncthreads();
  OFX_AS_STAMP(3)
  const double sig = s_sig;
  if (t < n) s_z[t * kAsD + t] = b16(bad ? (_Float16)(t < 6 * kCS ? 1.0f : 0.0f) : h16(1.0 + sig));
  if (t < kAsD) {
    const double dr = s_d[t];
    g.as_dsc[(int64_t)c * kAsD + t] = t < n ? (float)dr : 0.f;
    if (g.as_one) as_tab_at(g.as_tab, g.as_tab_cap).dsc[(int64_t)c * kAsD + t] = t < n ? (float)dr : 0.f;
    if (t < n) g.as_rsc[s_dst[t]] = (float)dr;
  }
  __syncthreads();
  OFX_AS_STAMP(4)
  for (int i = t; i < n * kAsK; i += kInvT) {
    const int R = i / kAsK, k = i % kAsK;
    const int d = s_dst[R], cp = d / kAsRS, rs = d % kAsRS;
    reinterpret_cast<uint4*>(g.as_slab)[((int64_t)cp * kAsK + k) * kAsRS + rs] =
        reinterpret_cast<const uint4*>(s_z + R * kAsD)[k];
  }
  if (g.as_one) {   // k_as_iter's subdomain-ordered copy (rows fastest)
    uint4* sl = as_tab_at(g.as_tab, g.as_tab_cap).slab + (int64_t)c * kAsK * kAsD;
    for (int i = t; i < n * kAsK; i += kInvT) {
      const int k = i / n, R = i - k * n;
      sl[(int64_t)k * kAsD + R] = reinterpret_cast<const uint4*>(s_z + R * kAsD)[k];
    }
  }
  if (t < kCS) g.racc[c * kCS + t] = 0.0;
  OFX_AS_STAMP(5)
#undef OFX_AS_STAMP
}

// The subdomain inverses of a solve's first GN step (and precond_every steps); the cold start's records x = 0, r = b and
// the PCG flags too. (A refresh flagged by the previous step runs inside k_pcg_proj<.., true>.)
// k_as_invert's thread grid: 16 x kAsInvTC (16 x 48 = 12 waves measured 119.5 against 110 us per solve with 16 x 16: each
// step's LDS row / column reads grow with the threads — 172 against 82 KB per two-step — and bound it)
constexpr int kAsInvTC = 16;
template <bool kMfma>   // (as_invert_mfma: kInvT threads, OFX_AS_INV_MFMA=1; or as_invert_body, the default: 256)
__global__ __launch_bounds__(kMfma ? kInvT : 16 * kAsInvTC) void k_as_invert(GnDev g, const double* __restrict__ A,
                                                                                   const double* __restrict__ rhs) {
  const int c = blockIdx.x, t = threadIdx.x;
  if (g.flags[F_STOPPED]) return;
  if constexpr (kMfma) as_invert_mfma(g, A, c, t);
  else as_invert_body<16, kAsInvTC>(g, A, c, t);
  if (!g.warm_now && t < 6 * kCS) {   // cold start: x = 0, r = b (u = M⁻¹ b comes from k_as_apply into m1)
    const int64_t o = 6 * (int64_t)c * kCS + t;
    const double v[V_N] = {0.0, rhs[o], 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    store_rec(g.st, o, v);
  }
  if (c == 0 && t == 0) { g.flags[F_DONE] = 0; g.flags[F_PCG_IT] = 0; g.flags[F_PCG_CNT] = 0; g.flags[F_REFRESH] = 0; }
}

// out (48 rows of cluster c) = the Schwarz apply of `in`: the gathered rows of the cluster's source subdomains into an LDS
// image (f64, each row times its source's column scale d; source slot s at s·kAsD), one segment per thread (its kAsD-entry
// fp16 slab row of Ẑ, 16-B word k of every segment contiguous: 1 KB per load instruction), the segments' f64 dot products
// times the row scale into LDS, and each row's segments summed in (row, source) order. 16-bit entries halve the slab
// (~10 MB per launch on the bench graph; with 12-row rings +~10 % frames/s against f32 rows);
// the preconditioner is still one fixed symmetric positive definite linear operator (k_as_invert's stored form).
// Trip 1: the stop word (kTest: the PCG chain's launches after convergence end there), the gather list, the segment's
// source slot and the row offsets; trip 2: the gathered rows and the slab rows together (static addresses; threads past
// the segment count read the last segment's lines, one line per load instruction).
template <bool kTest, int kL>   // kL: lanes per segment (1: 192 threads, 2: 384, 4: 768 — the dot products over more waves)
__global__ __launch_bounds__(kAsRS * kL) void k_as_apply(const int32_t* stopw, const int32_t* meta, const int32_t* gat,
                                                        const uint16_t* slab, const double* in, double* out,
                                                        const int32_t* src, const float* dsc, const float* rsc) {
  constexpr int kT = kAsRS * kL;                 // threads
  constexpr int kG = (kAsGat + kT - 1) / kT;     // gathered rows per thread
  constexpr int kKL = (kAsK + kL - 1) / kL;      // 16-B words of its segment per lane
  __shared__ __attribute__((aligned(16))) double s_w[kAsSrc * kAsD];
  __shared__ double s_seg[kAsRS];
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int sg = t / kL, hl = t % kL;            // the thread's segment and its part
  const int32_t* mt = meta + (int64_t)c * kAsMeta;
  int stop = 0;
  if (kTest) stop = stopw[(int64_t)c * 64 + lane];
  const int nrs = mt[0];
  int gn[kG], sv[kG];   // gathered rows and their source subdomains
#pragma unroll
  for (int j = 0; j < kG; ++j) {
    const int i = min(kT * j + t, kAsGat - 1);
    gn[j] = gat[(int64_t)c * kAsGat + i];
    sv[j] = src[c * kAsSrc + min(i / kAsDN, kAsSrc - 1)];
  }
  const int sl = mt[64 + sg];
  const float rscale = rsc[(int64_t)c * kAsRS + sg];
  const int rr = t < 6 * kCS ? t : 6 * kCS - 1;
  const int o0 = mt[2 + rr], o1 = mt[3 + rr];
  asm volatile("" ::: "memory");
  if (kTest) {
    stop = __builtin_amdgcn_readfirstlane(stop);
    if (stop != 0) return;   // the solve has converged (or stopped): a drained launch
  }
  double2 wg[kG][3];
  float2 dg[kG][3];   // the source subdomains' column scales of the gathered rows
#pragma unroll
  for (int j = 0; j < kG; ++j) {
    const int i = min(kT * j + t, kAsGat - 1);
    const double2* p = reinterpret_cast<const double2*>(in + 6 * (int64_t)(gn[j] >= 0 ? gn[j] : 0));
    const float2* q = reinterpret_cast<const float2*>(dsc + (int64_t)sv[j] * kAsD + 6 * (i % kAsDN));
#pragma unroll
    for (int k = 0; k < 3; ++k) { wg[j][k] = p[k]; dg[j][k] = q[k]; }
  }
  uint4 z[kKL];   // 8 fp16 entries each: words hl·kKL .. of the segment (clamped; the tail word is masked)
  {
    const int rs = sg < nrs ? sg : (nrs > 0 ? nrs - 1 : 0);
    const uint4* zp = reinterpret_cast<const uint4*>(slab) + (int64_t)c * kAsK * kAsRS + rs;
#pragma unroll
    for (int k = 0; k < kKL; ++k) z[k] = zp[min(hl * kKL + k, kAsK - 1) * kAsRS];
  }
#pragma unroll
  for (int j = 0; j < kG; ++j) {
    const int i = kT * j + t;
    if (i < kAsSrc * kAsDN) {
      const bool ok = gn[j] >= 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s_w[6 * i + 2 * k] = ok ? wg[j][k].x * (double)dg[j][k].x : 0.0;
        s_w[6 * i + 2 * k + 1] = ok ? wg[j][k].y * (double)dg[j][k].y : 0.0;
      }
    }
  }
  __syncthreads();
  // the segment's dot product in f64 (fp16 entries exact in f64): the apply is linear to f64 rounding. (An f32 image and
  // f32 products, measured: 3 % faster, but the rounding made the apply nonlinear at 1e-7 — the pipelined recurrences
  // drifted, gn_4k's loss log missed 1e-6 and the ill-conditioned moose ended 0.29 off.)
  double dot = 0.0;
  if (sg < nrs) {
    const double2* w2 = reinterpret_cast<const double2*>(s_w + sl * kAsD);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    auto lo = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xFFFFu)); };
    auto hi = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); };
#pragma unroll
    for (int k = 0; k < kKL; ++k) {
      const int kw = hl * kKL + k;
      if (kw >= kAsK) break;   // (compile-time for kL = 1; the last lane's tail word for kL = 2)
      const double2 p0 = w2[4 * kw], p1 = w2[4 * kw + 1], p2 = w2[4 * kw + 2], p3 = w2[4 * kw + 3];
      a0 = fma(lo(z[k].x), p0.x, a0);
      a1 = fma(hi(z[k].x), p0.y, a1);
      a2 = fma(lo(z[k].y), p1.x, a2);
      a3 = fma(hi(z[k].y), p1.y, a3);
      a0 = fma(lo(z[k].z), p2.x, a0);
      a1 = fma(hi(z[k].z), p2.y, a1);
      a2 = fma(lo(z[k].w), p3.x, a2);
      a3 = fma(hi(z[k].w), p3.y, a3);
    }
    dot = (a0 + a1) + (a2 + a3);
  }
  if (kL >= 2) dot += dpp_mov<0xB1>(dot);   // quad_perm [1, 0, 3, 2]: the pair's two parts (the same sum in both lanes)
  if (kL == 4) dot += dpp_mov<0x4E>(dot);   // quad_perm [2, 3, 0, 1]: the two pairs (fixed order, equal in all four)
  if (sg < nrs && hl == 0) s_seg[sg] = (double)rscale * dot;
  __syncthreads();
  if (t < 6 * kCS) {
    double sv2[kAsX + 1];
#pragma unroll
    for (int j = 0; j <= kAsX; ++j) sv2[j] = s_seg[min(o0 + j, kAsRS - 1)];
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j <= kAsX; ++j) sum += o0 + j < o1 ? sv2[j] : 0.0;
    out[(int64_t)c * 6 * kCS + t] = sum;
  }
}

// Galerkin warm start, pass 1: t_j = A x_j for the n_prev stored solutions (own rows) and per-wave
// partials of the Gram matrix G_ij = x_i·t_j (i <= j, packed) and f_i = x_i·b.
__device__ __forceinline__ constexpr int tri(int i, int j) { return j * (j + 1) / 2 + i; }   // i <= j

// t_j += A_blk x_j (block bk, gathered history rows x) for the stored solutions j < np, in the loop's order
__device__ __forceinline__ void proj_accumulate(const double bk[36], const double x[kProj][6], int np,
                                                double n[kProj][6]) {
#pragma unroll
  for (int j = 0; j < kProj; ++j) {
    if (j < np) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) t += bk[6 * i + k] * x[j][k];
        n[j][i] += t;
      }
    }
  }
}

// kWave: the SpMVs in k_pcg_iter's wave-list form (as k_pcg_w0): the wave's (col, slot) list, row bounds, the own
// rows' b and history values leave in the first trip with the stop flag; the second trip is every block of the wave
// (lane l: blocks l and l + 64) with the kProj history rows it multiplies; the products meet in LDS and each row sums
// its blocks in CSR order. (The row form's first trip is row_ptr, then col, then blocks + gathers.)
// A GN step flagged by the previous step's update (F_REFRESH = this step: some node rotated by more than
// precond_rot_tol since its cluster inverse was built) first rebuilds the cluster inverses here, one wave per
// cluster as k_pcg_prep (k_pcg_proj2 applies them); otherwise the flag costs one scalar load with the stop flag.
// kAS (Schwarz): four waves; wave 0 does the projection (its flags in its first trip), then a refresh flagged by the
// previous step (F_REFRESH = this step) rebuilds the cluster's subdomain inverse (as_invert_body, all four waves: waves
// 1-3 wait for wave 0 at its first barrier; the projection has no workgroup barrier and reads A, not the inverse). (The
// refresh test ahead of the projection cost two dependent scalar trips before its first: 9.2 µs per launch against 7.6
// for the cluster-block form.)
template <bool kWave, bool kAS = false>
__global__ __launch_bounds__(kAS ? 256 : 64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_pcg_proj(GnDev g, const double* rhs,
                                                                                              int gn_iter) {
  // the kernel-argument fields in SGPRs up front (one scalar trip, see k_terms)
  asm volatile("" :: "s"(g.wl), "s"(g.row_ptr), "s"(g.col), "s"(g.xh), "s"(g.th), "s"(g.N), "s"(g.flags), "s"(g.n_prev),
               "s"(g.Aop), "s"(g.part_p), "s"(g.nw_pad), "s"(rhs));
  if constexpr (kWave) {
    __shared__ double s_prod[kProj][(kWL + kRowMax) * 6];
    // the projection (wave 0): returns whether a refresh is flagged for this step (0 when the solve stopped)
    auto project = [&]() -> int {
      const int lane = threadIdx.x;
      const int wv = blockIdx.x;
      const int r = lane / kSL, q = lane % kSL, row = wv * kRW + r;
      const int qc = q < 6 ? q : 5;
      const int64_t oc = 6 * (int64_t)row + qc;
      const int64_t stride = 6 * (int64_t)g.N;
      int2 bl[2];
      bl[0] = g.wl[(int64_t)wv * kWL + lane];
      bl[1] = g.wl[(int64_t)wv * kWL + 64 + lane];
      const int wb0 = g.row_ptr[wv * kRW];
      const int rb0 = g.row_ptr[row], rb1 = g.row_ptr[row + 1];
      const double b = rhs[oc];
      double xo[kProj];
  #pragma unroll
      for (int j = 0; j < kProj; ++j) xo[j] = g.xh[j * stride + oc];
      const int stopped = g.flags[F_STOPPED];
      const int refresh = g.flags[F_REFRESH];
      asm volatile("" ::: "memory");   // the loads above leave with the stop flag (one trip)
      if (stopped) return 0;
      if (!kAS && refresh == gn_iter) {   // (Schwarz: as_invert_body below)
        float mm[6][6];
        cluster_invert(g, g.Aop, wv, lane, mm);
      }
      const int np = g.n_prev;
      double2 ab[2][18], xb[2][kProj][3];
  #pragma unroll
      for (int jj = 0; jj < 2; ++jj) {   // unconditional (padding entries read block 0 / row 0, masked below)
        const int64_t cc = 6 * (int64_t)(bl[jj].x >= 0 ? bl[jj].x : 0);
  #pragma unroll
        for (int h = 0; h < kProj; ++h)
  #pragma unroll
          for (int k = 0; k < 3; ++k) xb[jj][h][k] = reinterpret_cast<const double2*>(g.xh + h * stride + cc)[k];
        const double2* blk = reinterpret_cast<const double2*>(g.Aop + 36 * (int64_t)(bl[jj].x >= 0 ? wl_base(bl[jj]) + 64 * jj + lane : 0));
  #pragma unroll
        for (int k = 0; k < 18; ++k) ab[jj][k] = blk[k];
      }
  #pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const bool ok = bl[jj].x >= 0;
  #pragma unroll
        for (int h = 0; h < kProj; ++h) {
          double x[6];
  #pragma unroll
          for (int k = 0; k < 3; ++k) { x[2 * k] = xb[jj][h][k].x; x[2 * k + 1] = xb[jj][h][k].y; }
  #pragma unroll
          for (int i = 0; i < 6; ++i) {
            const double2 b01 = ab[jj][3 * i], b23 = ab[jj][3 * i + 1], b45 = ab[jj][3 * i + 2];
            const double t = ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
            s_prod[h][(jj * 64 + lane) * 6 + i] = (ok && h < np) ? t : 0.0;
          }
        }
      }
      wave_lds_sync();
      const int len = rb1 - rb0;
      double t[kProj];
  #pragma unroll
      for (int h = 0; h < kProj; ++h) {   // per history vector: its kRowMax reads in flight, then the adds in CSR order
        const double* sp = s_prod[h] + (rb0 - wb0) * 6 + qc;
        double tv[kRowMax];
  #pragma unroll
        for (int k = 0; k < kRowMax; ++k) tv[k] = sp[6 * k];
        __builtin_amdgcn_sched_barrier(0);
        double a = 0.0;
  #pragma unroll
        for (int k = 0; k < kRowMax; ++k) a += k < len ? tv[k] : 0.0;
        t[h] = a;
      }
      double v[kProjP];
  #pragma unroll
      for (int k = 0; k < kProjP; ++k) v[k] = 0.0;
      if (q < 6) {
        double x[kProj];
  #pragma unroll
        for (int j = 0; j < kProj; ++j) {
          x[j] = j < np ? xo[j] : 0.0;
          if (j < np) g.th[j * stride + oc] = t[j];
        }
  #pragma unroll
        for (int j = 0; j < kProj; ++j) {
  #pragma unroll
          for (int i = 0; i <= j; ++i) v[tri(i, j)] = x[i] * t[j];
          v[kProj * (kProj + 1) / 2 + j] = x[j] * b;
        }
      }
  #pragma unroll
      for (int k = 0; k < kProjP; ++k) v[k] = wave_sum(v[k]);
      if (lane == 0)
  #pragma unroll
        for (int k = 0; k < kProjP; ++k) g.part_p[(int64_t)k * g.nw_pad + blockIdx.x] = v[k];
      if (blockIdx.x == 0 && threadIdx.x == 0) { g.flags[F_DONE] = 0; g.flags[F_PCG_IT] = 0; g.flags[F_PCG_CNT] = 0; }
      return refresh == gn_iter ? 1 : 0;
    };
    int ref;
    if (!kAS || threadIdx.x < 64) {
      ref = project();
    } else {
      const int stopped = g.flags[F_STOPPED], refresh = g.flags[F_REFRESH];
      ref = !stopped && refresh == gn_iter ? 1 : 0;
    }
    if constexpr (kAS) {
      if (ref) as_invert_body<16, 16>(g, g.Aop, blockIdx.x, threadIdx.x);
    }
    (void)ref;
    return;
  }
  const int lane = threadIdx.x;
  const int q = lane % kSL, row = blockIdx.x * kRW + lane / kSL;
  const int b0 = g.row_ptr[row], b1 = g.row_ptr[row + 1];   // issued with the stop flag: one trip
  const int refresh = g.flags[F_REFRESH];
  if (g.flags[F_STOPPED]) return;
  if (refresh == gn_iter) {
    float mm[6][6];
    cluster_invert(g, g.Aop, blockIdx.x, lane, mm);
  }
  const int np = g.n_prev;
  const int64_t stride = 6 * (int64_t)g.N;
  double n[kProj][6];
#pragma unroll
  for (int j = 0; j < kProj; ++j)
#pragma unroll
    for (int i = 0; i < 6; ++i) n[j][i] = 0.0;
  {   // the first two slots' blocks, then all their history gathers, issued together (rows of <= 2·kSL blocks:
      // two dependent trips instead of four); unconditional loads (clamped entry, every history row exists)
    const int bi0 = b0 + q, bi1 = bi0 + kSL;
    const bool ok0 = bi0 < b1, ok1 = bi1 < b1;
    const int e0 = ok0 ? bi0 : 0, e1 = ok1 ? bi1 : 0;
    const int64_t cc0 = 6 * (int64_t)g.col[e0], cc1 = 6 * (int64_t)g.col[e1];
    double bk0[36], bk1[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) { bk0[k] = g.Aop[36 * (int64_t)e0 + k]; bk1[k] = g.Aop[36 * (int64_t)e1 + k]; }
    double x0[kProj][6], x1[kProj][6];
#pragma unroll
    for (int j = 0; j < kProj; ++j)
#pragma unroll
      for (int k = 0; k < 6; ++k) { x0[j][k] = g.xh[j * stride + cc0 + k]; x1[j][k] = g.xh[j * stride + cc1 + k]; }
    if (ok0) proj_accumulate(bk0, x0, np, n);
    if (ok1) proj_accumulate(bk1, x1, np, n);
  }
  for (int bi = b0 + q + 2 * kSL; bi < b1; bi += kSL) {
    const double* blk = g.Aop + 36 * (int64_t)bi;
    const int64_t cc = 6 * (int64_t)g.col[bi];
    double bk[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) bk[k] = blk[k];
#pragma unroll
    for (int j = 0; j < kProj; ++j) {
      if (j < np) {
        const double* vc = g.xh + j * stride + cc;
        double x[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) x[k] = vc[k];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double t = 0.0;
#pragma unroll
          for (int k = 0; k < 6; ++k) t += bk[6 * i + k] * x[k];
          n[j][i] += t;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kProj; ++j)
#pragma unroll
    for (int i = 0; i < 6; ++i) n[j][i] = slot_sum(n[j][i]);
  double v[kProjP];
#pragma unroll
  for (int k = 0; k < kProjP; ++k) v[k] = 0.0;
  if (q < 6) {
    const int64_t o = 6 * (int64_t)row + q;
    const double b = rhs[o];
    double x[kProj], t[kProj];
#pragma unroll
    for (int j = 0; j < kProj; ++j) {
      t[j] = pick6(n[j], q);
      x[j] = j < np ? g.xh[j * stride + o] : 0.0;
      if (j < np) g.th[j * stride + o] = t[j];
    }
#pragma unroll
    for (int j = 0; j < kProj; ++j) {
#pragma unroll
      for (int i = 0; i <= j; ++i) v[tri(i, j)] = x[i] * t[j];
      v[kProj * (kProj + 1) / 2 + j] = x[j] * b;
    }
  }
#pragma unroll
  for (int k = 0; k < kProjP; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kProjP; ++k) g.part_p[(int64_t)k * g.nw_pad + blockIdx.x] = v[k];
  // PCG bookkeeping of this GN step (also in k_pcg_prep), stored last: on gfx9 vmcnt counts stores too, so stores
  // ahead of the loads made workgroup 0's first wait a vmcnt(0) that also waited for their acks
  if (blockIdx.x == 0 && threadIdx.x == 0) { g.flags[F_DONE] = 0; g.flags[F_PCG_IT] = 0; g.flags[F_PCG_CNT] = 0; }
}

// The warm start's Galerkin coefficients c (k_pcg_proj2, k_as_proj2; every wave that needs them computes them the same
// way): the Gram partials of k_pcg_proj summed, the <= kProj system G c = X^T b solved by Cholesky on the upper triangle
// (dependent / degenerate directions dropped); false if a coefficient is not finite
template <int KU>
__device__ __forceinline__ bool galerkin_coeffs(const GnDev& g, int np, double2 pt[kProjP][KU], double c[kProj]) {
  double p[kProjP];
  reduce_streams2<kProjP, KU>(g.part_p, g.nw_pad, g.nw_pad, pt, p);
  // G is symmetric in exact arithmetic; use the upper triangle G_ij = x_i·A x_j (i <= j)
  double L[kProj][kProj], y[kProj];
  bool use[kProj];
#pragma unroll
  for (int j = 0; j < kProj; ++j) {
    use[j] = false; y[j] = 0.0; c[j] = 0.0;
#pragma unroll
    for (int i = 0; i < kProj; ++i) L[j][i] = 0.0;
  }
#pragma unroll
  for (int j = 0; j < kProj; ++j) {
    if (j >= np) continue;
    double d = p[tri(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) if (use[k]) d -= L[j][k] * L[j][k];
    if (!(d > 1e-10 * p[tri(j, j)]) || !(p[tri(j, j)] > 0.0)) continue;   // dependent / degenerate
    use[j] = true;
    const double ljj = sqrt(d);
    L[j][j] = ljj;
#pragma unroll
    for (int i = j + 1; i < kProj; ++i) {
      if (i >= np) continue;
      double sd = p[tri(j, i)];
#pragma unroll
      for (int k = 0; k < j; ++k) if (use[k]) sd -= L[i][k] * L[j][k];
      L[i][j] = sd / ljj;
    }
  }
#pragma unroll
  for (int j = 0; j < kProj; ++j) {
    if (!use[j]) continue;
    double sd = p[kProj * (kProj + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) if (use[k]) sd -= L[j][k] * y[k];
    y[j] = sd / L[j][j];
  }
#pragma unroll
  for (int j = kProj - 1; j >= 0; --j) {
    if (!use[j]) continue;
    double sd = y[j];
#pragma unroll
    for (int k = j + 1; k < kProj; ++k) if (use[k]) sd -= L[k][j] * c[k];
    c[j] = sd / L[j][j];
  }
  bool fin = true;
#pragma unroll
  for (int j = 0; j < kProj; ++j) fin = fin && isfinite(c[j]);
  return fin;
}

// Galerkin warm start, pass 2: every wave re-derives G and f from the partials (fixed order,
// identical bits), solves G c = f by pivot-guarded Cholesky (near-dependent history vectors get
// c = 0), and sets x0 = Σ c_j x_j, r0 = b - Σ c_j t_j, u0 = M⁻¹ r0 (cluster, via LDS),
// z = q = s = p = w = 0, u0 -> m1.
// The projection partials are read as KU pairs per lane and stream at the iteration streams' padded stride nw_pad =
// 128·KU (zero beyond the wave count: cleared at setup): unconditional loads, no per-load branches.
template <int KU, bool kAS = false>   // kAS: Schwarz (no cluster inverse; r0 -> as_w for k_as_apply)
__global__ __launch_bounds__(64) void k_pcg_proj2(GnDev g, const double* rhs) {   // (not __restrict__: see k_pcg_w0)
  __shared__ __attribute__((aligned(16))) double s_v[kCD];
  // the kernel-argument fields in SGPRs up front (one scalar trip, see k_terms)
  asm volatile("" :: "s"(g.n_prev), "s"(g.N), "s"(g.Mcl), "s"(g.xh), "s"(g.th), "s"(g.part_p), "s"(g.nw_pad),
               "s"(g.flags), "s"(g.stopw), "s"(g.ep), "s"(g.st), "s"(g.m1), "s"(rhs));
  const int lane = threadIdx.x;
  const int r = lane / kSL, q = lane % kSL, row = blockIdx.x * kRW + r;
  const int np = g.n_prev;
  const bool own = q < 6;
  const int64_t o = 6 * (int64_t)row + q;
  const int64_t oc = 6 * (int64_t)row + (own ? q : 5);   // every lane loads (clamped): one memory trip in all
  const int64_t stride = 6 * (int64_t)g.N;
  float4 mr[kCD / 4];
  if constexpr (!kAS) load_mrow(g, oc, mr);
  const double rb = rhs[oc];
  double xo[kProj], to[kProj];
#pragma unroll
  for (int j = 0; j < kProj; ++j) { xo[j] = g.xh[j * stride + oc]; to[j] = g.th[j * stride + oc]; }
  double2 pt[kProjP][KU];
  load_streams2_padded<kProjP, KU>(g.part_p, g.nw_pad, pt);
  const int stopped = g.flags[F_STOPPED];
  asm volatile("" ::: "memory");   // keep the loads above the exit test (one trip with the flag)
  if (stopped) {   // the solve already stopped: this step's iteration launches end after trip 1
    g.stopw[(int64_t)blockIdx.x * 64 + lane] = g.ep;
    return;
  }
  double c[kProj];
  const bool fin = galerkin_coeffs<KU>(g, np, pt, c);
  double xv = 0.0, rv = 0.0;
  if (own) {
    rv = rb;
#pragma unroll
    for (int j = 0; j < kProj; ++j)
      if (j < np && fin) { xv += c[j] * xo[j]; rv -= c[j] * to[j]; }
    s_v[6 * r + q] = rv;
  }
  __syncthreads();
  if (own) {
    if constexpr (kAS) {   // u0 = M⁻¹ r0 by k_as_apply (as_w -> m1)
      const double v[V_N] = {xv, rv, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      store_rec(g.st, o, v);
      g.as_w[o] = rv;
    } else {
      const double u = apply_mrow(mr, s_v);
      const double v[V_N] = {xv, rv, u, 0.0, 0.0, 0.0, 0.0, 0.0};
      store_rec(g.st, o, v);
      g.m1[o] = u;
    }
  }
}

// The warm start's per-solve scalar-block stores (workgroup 0, lane 0; k_pcg_w0 and k_as_w0): the operator the iteration
// reads (the padded per-wave copy, or A itself for the one-launch Schwarz iteration), the tolerances, the iteration's w_new
// target in the inverse's slot (Schwarz) and the m buffers, the error stop's θ̂ carried over from the previous GN step
__device__ __forceinline__ void w0_lead_stores(const GnDev& g, double th_cur_old, bool wave_copy, bool as) {
  reinterpret_cast<uint64_t*>(g.pcs)[kScAop] = reinterpret_cast<uint64_t>((wave_copy && !g.as_one) ? g.Aw : g.Aop);
  g.pcs[kScTol] = g.prm.pcg_tol;
  // the error stop's τ: one value for both preconditioners (the estimate is Euclidean, k_pcg_iter)
  g.pcs[kScTol + 1] = g.prm.pcg_err_tol;
  reinterpret_cast<uint64_t*>(g.pcs)[kScMcl] = as ? reinterpret_cast<uint64_t>(g.as_w) : reinterpret_cast<uint64_t>(g.Mcl);
  reinterpret_cast<uint64_t*>(g.pcs)[kScM] = reinterpret_cast<uint64_t>(g.m0);
  reinterpret_cast<uint64_t*>(g.pcs)[kScM + 1] = reinterpret_cast<uint64_t>(g.m1);
  // (none for the first GN step of the solve)
  g.pcs[kScScal + S_TH_PREV] = g.gn_iter_now > 0 ? th_cur_old : 1e300;
  g.pcs[kScScal + S_TH_CUR] = 1e300;
}

// w0 = A u0 (u0 gathered from m1), m0 = M⁻¹ w0 (cluster, via LDS); per-wave partials
// (γ0 = r·u, δ0 = w·u, r·r) -> parity 0, b·b -> part_b.
// kWave: the SpMV in k_pcg_iter's wave-list form — the wave's (col, slot) list leaves in the first trip with the state
// and the stop flag, so the blocks and gathers are the second (the row form needs row_ptr -> col -> blocks: three);
// lane l multiplies the wave's blocks l and l + 64, the products meet in LDS, each row sums its blocks in CSR order.
template <bool kWave, bool kAS = false>   // kAS: Schwarz (u0 from m1, w0 -> as_w, no cluster inverse)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_pcg_w0(GnDev g, const double* rhs) {   // (rhs not __restrict__: a restrict load sinks past the exit test)
  __shared__ __attribute__((aligned(16))) double s_v[kCD];
  __shared__ double s_prod[kWave ? (kWL + kRowMax) * 6 : 1];
  // the kernel-argument fields in SGPRs up front (one scalar trip, see k_terms)
  asm volatile("" :: "s"(g.wl), "s"(g.row_ptr), "s"(g.Mcl), "s"(g.st), "s"(g.flags), "s"(g.m0), "s"(g.m1), "s"(g.Aop),
               "s"(g.part_p), "s"(g.part_b), "s"(g.nw_pad), "s"(g.nwg_row), "s"(g.ep), "s"(g.stopw), "s"(g.pcs), "s"(rhs),
               "s"(g.prm.pcg_tol), "s"(g.prm.pcg_err_tol), "s"(g.Mcl), "s"(g.Aw));
  const int lane = threadIdx.x;
  const int wv = blockIdx.x;
  const int r = lane / kSL, q = lane % kSL, row = blockIdx.x * kRW + r;
  const bool own = q < 6;
  const int qc = own ? q : 5;
  const int64_t o = 6 * (int64_t)row + q;
  const int64_t oc = 6 * (int64_t)row + qc;   // every lane loads (clamped)
  // (wave list,) row bounds, own state, M⁻¹ row and b issued with the stop flag: one trip
  int2 bl[2] = {make_int2(-1, 0), make_int2(-1, 0)};
  if (kWave) { bl[0] = g.wl[(int64_t)wv * kWL + lane]; bl[1] = g.wl[(int64_t)wv * kWL + 64 + lane]; }
  // the list and the stop flag leave first (loads retire in issue order): the stop test and trip 2's issue wait for
  // them only, the rest of trip 1 lands under trip 2's flight
  const int stopped = g.flags[F_STOPPED];
  asm volatile("" ::: "memory");
  const int wb0 = g.row_ptr[wv * kRW];
  const int rb0 = g.row_ptr[row], rb1 = g.row_ptr[row + 1];
  const double bo = rhs[oc];
  float4 mr[kCD / 4];
  double v[V_N];
  if constexpr (!kAS) load_mrow(g, oc, mr);
  load_rec(g.st, oc, v);
  const double u_as = g.m1[oc];  // (Schwarz: u0 came from k_as_apply into m1)
  const double w_old = v[V_W];   // unused, but kept live to the end (see the end of the kernel)
  // the previous step's final θ̂ (the lead's bookkeeping below), with trip 1: read inside the lead's branch it was one
  // more trip for workgroup 0 before its SpMV
  const double th_cur_old = g.pcs[kScScal + S_TH_CUR];
  asm volatile("" ::: "memory");
  // this solve's stop words: the epoch if the solve already stopped (its iteration launches end after trip 1), else 0
  // (a converging iteration sets them to the epoch), so the iteration's stop test needs no epoch; and the operator's
  // address into the scalar block, where the iteration finds it through a preloaded pointer. Both are stored last on the
  // main path: vmcnt counts stores too, so stores ahead of trip 2 held its issue until their acks (workgroup 0's eight)
  auto lead_stores = [&]() {
    if (blockIdx.x == 0 && lane == 0) w0_lead_stores(g, th_cur_old, kWave, kAS);
  };
  if (stopped) {
    g.stopw[(int64_t)blockIdx.x * 64 + lane] = g.ep;
    lead_stores();
    return;
  }
  if (kAS) v[V_U] = u_as;
  const double b = own ? bo : 0.0;
  double w;
  double2 ab[2][18];
  if (kWave) {
    double2 xb[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // unconditional loads (padding reads block 0 / m row 0, masked below)
      const double2* blk = reinterpret_cast<const double2*>(g.Aop + 36 * (int64_t)(bl[j].x >= 0 ? wl_base(bl[j]) + 64 * j + lane : 0));
      const double2* vc = reinterpret_cast<const double2*>(g.m1 + 6 * (int64_t)(bl[j].x >= 0 ? bl[j].x : 0));
#pragma unroll
      for (int k = 0; k < 3; ++k) xb[j][k] = vc[k];
#pragma unroll
      for (int k = 0; k < 18; ++k) ab[j][k] = blk[k];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = bl[j].x >= 0;
      double x[6];
#pragma unroll
      for (int k = 0; k < 3; ++k) { x[2 * k] = xb[j][k].x; x[2 * k + 1] = xb[j][k].y; }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 b01 = ab[j][3 * i], b23 = ab[j][3 * i + 1], b45 = ab[j][3 * i + 2];
        const double t = ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
        s_prod[(j * 64 + lane) * 6 + i] = ok ? t : 0.0;
      }
    }
    wave_lds_sync();
    const int len = rb1 - rb0;
    const double* sp = s_prod + (rb0 - wb0) * 6 + qc;
    double tv[kRowMax];
#pragma unroll
    for (int k = 0; k < kRowMax; ++k) tv[k] = sp[6 * k];
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < kRowMax; ++k) a += k < len ? tv[k] : 0.0;
    w = a;
  } else {
    double n[6];
    row_spmv_2(g, rb0, rb1, q, g.m1, n);
    w = pick6(n, q);
  }
  if (own) s_v[6 * r + q] = w;
  __syncthreads();
  double d[4] = {0.0, 0.0, 0.0, 0.0};   // (the stop words hold an older epoch: this solve's launches run)
  if (own) {
    v[V_W] = w;
    store_rec(g.st, o, v);
    if constexpr (kAS) g.as_w[o] = w;        // m0 = M⁻¹ w0 by k_as_apply (as_w -> m0)
    else g.m0[o] = apply_mrow(mr, s_v);
    d[0] = v[V_R] * v[V_U]; d[1] = w * v[V_U]; d[2] = v[V_R] * v[V_R]; d[3] = b * b;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = wave_sum(d[k]);
  const int ns = g.nw_pad;
  if (lane == 0) {
    g.part_p[blockIdx.x] = d[0]; g.part_p[ns + blockIdx.x] = d[1]; g.part_p[2 * ns + blockIdx.x] = d[2];
    g.part_p[3 * ns + blockIdx.x] = 0.0;   // (the direction stream: no direction before the first iteration)
    g.part_b[blockIdx.x] = d[3];
  }
  if (blockIdx.x == 0)   // zero tails of both parities' streams (part_p is also proj scratch) and of part_b
    for (int i = g.nwg_row + lane; i < ns; i += 64) {
#pragma unroll
      for (int k = 0; k < 2 * kPcgStreams; ++k) g.part_p[k * ns + i] = 0.0;
      g.part_b[i] = 0.0;
    }
  // the loaded (dead) w register stays allocated to here: otherwise the compiler reuses it for a temporary of the
  // SpMV's issue and waits for its load first (a vmcnt that held trip 2 behind nearly all of trip 1)
  // the wave's blocks into its padded copy for k_pcg_iter (kWave): last, so no wait here is behind their acks (the
  // one-launch Schwarz iteration reads A itself: no copy)
  if (kWave && !g.as_one) {
    double2* Aw = reinterpret_cast<double2*>(g.Aw) + (int64_t)wv * 18 * kWL;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = bl[j].x >= 0;
#pragma unroll
      for (int k = 0; k < 18; ++k) Aw[k * kWL + 64 * j + lane] = ok ? ab[j][k] : make_double2(0.0, 0.0);
    }
  }
  g.stopw[(int64_t)blockIdx.x * 64 + lane] = 0;
  lead_stores();
  asm volatile("" ::"v"(w_old));
}

// One PCG iteration; par = parity of the iteration (iteration i has par = i & 1), kFirst only for
// iteration 0. Reads partials[par], m[par] and alpha/gamma[par^1]; writes partials[par^1], m[par^1]
// and alpha/gamma[par]. The count of executed iterations lives in flags[F_PCG_CNT] (the lead lane
// increments it).
// Latency structure (one wave per cluster = workgroup): exactly two dependent memory trips, every
// load unconditional (clamped addresses, masked values) so no branch splits a trip. Trip 1: the
// wave's block list, previous partials, own-row state, own m, and the cluster inverse straight to
// LDS (LDS-DMA: no VGPRs held). Trip 2: A blocks and gathered m — lane l multiplies the wave's
// blocks l and l + 64 (balanced over the cluster's rows, whatever their lengths); the products
// meet in LDS and each row sums its blocks in CSR order (fixed order: deterministic).
// Convergence is decided from the partials alone and carried forward through them and a per-lane
// stop word: a converged (or broken-down) launch copies its wave's partials (rr = 0 on breakdown)
// into the next parity and sets the stop words, so later launches of the chunk end after trip 1.
// kWave = false: plain CSR rows (waves of more than kWL blocks or rows longer than kRowMax).
// The iteration kernel's arguments: only what it reads (a ~200-B kernarg instead of the whole Gn:
// the host enqueues ~1000 of these per frame, so per-launch host work is on the critical path).
// What the converging PCG launch needs to also take the GN step (k_step's work, fused): fixed pointers in
// device memory (written once at create), per-step values in the kernel arguments.
struct StepArgs {
  double *R, *t, *xh, *stat, *loss_log, *step_state;
  const double* conf;
  double* racc;
};
struct PcgIt {
  const double* Aop;
  const float* Mcl;
  const int32_t *row_ptr, *col;
  const int2* wl;
  double *m0, *m1, *st, *part_p, *part_b, *pcg_alpha, *pcg_gamma, *scal;
  int32_t *flags, *hflags, *stopw;
  double2* sturm;               // error-based stop: per lead lane s the LDLᵀ pivot of T_k - σ_s I and its negative count
  uint64_t* stamps;
  int32_t nwg_row, nw_pad;
  struct { double pcg_tol, pcg_err_tol; } prm;
  // fused GN step (fuse = 0: k_step runs as its own launch)
  const StepArgs* sa;
  const double* tail;           // rhs + 6N: [loss² total, data, arap, motion, nonfinite]
  double stop_loss_diff;
  double rot_tol;               // precond_rot_tol
  int32_t fuse, gn_iter, N, mode, n_iter_log, warm;
  int32_t ep;                   // this solve's epoch (stop words, H_DONE)
};
static PcgIt pcg_args(const Gn* g) {
  PcgIt a;
  memset(&a, 0, sizeof(a));   // (padding too: the host compares copies bytewise)
  a.Aop = g->Aop; a.Mcl = g->Mcl; a.row_ptr = g->row_ptr; a.col = g->col; a.wl = g->wl;
  a.m0 = g->m0; a.m1 = g->m1; a.st = g->st; a.part_p = g->part_p; a.part_b = g->part_b;
  a.pcg_alpha = g->pcg_alpha; a.pcg_gamma = g->pcg_gamma; a.scal = g->scal;
  a.flags = g->flags; a.hflags = g->hflags; a.stopw = g->stopw; a.stamps = g->stamps;
  a.nwg_row = g->nwg_row; a.nw_pad = g->nw_pad; a.prm.pcg_tol = g->prm.pcg_tol; a.prm.pcg_err_tol = g->prm.pcg_err_tol;
  a.sturm = g->sturm;
  a.sa = g->step_args; a.tail = nullptr; a.stop_loss_diff = g->prm.stop_loss_diff; a.rot_tol = g->prm.precond_rot_tol;
  a.fuse = 0; a.gn_iter = 0; a.N = g->N; a.mode = g->prm.mode; a.n_iter_log = 64; a.warm = g->prm.pcg_warm;
  a.ep = g->ep;
  return a;
}
#ifdef OFX_STAMPS   // tuning build only: phase clock stamps of every wave of the first 64 iterations
#define OFX_STAMP_AT(k)                                                                               \
  if (lane == 0 && g.stamps && cnt < 64) g.stamps[((int64_t)cnt * nw + wv) * 8 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define OFX_STAMP_AT(k)
#endif
#ifdef OFX_STAMPS_SCALARS   // (with OFX_STAMPS) the scalar phase split instead: 1 stop test, 2 trip 2 issued, 3 partials landed,
                            // 4 wave sums, 5 division + leave test, 6 products' start, 7 end
#define OFX_STAMP(k) if ((k) == 1 || (k) == 7) { OFX_STAMP_AT(k) }
#define OFX_STAMPX(k) OFX_STAMP_AT(k)
#else
#define OFX_STAMP(k) OFX_STAMP_AT(k)
#define OFX_STAMPX(k)
#endif
// k_step's work done by the converging PCG launch (every wave for its own rows; wave 0 lane 0 the
// bookkeeping). Every wave derives the same decision from read-only inputs, as k_step's workgroups do.
__device__ __forceinline__ void kornia_exp(const double x[3], double Ri[9]) {
  const double a0 = x[0], a1 = x[1], a2 = x[2];
  const double th2 = a0 * a0 + a1 * a1 + a2 * a2;
  if (th2 > 1e-6) {
    const double th = sqrt(th2);
    const double wx = a0 / (th + 1e-6), wy = a1 / (th + 1e-6), wz = a2 / (th + 1e-6);
    const double c = cos(th), s = sin(th), oc = 1.0 - c;
    Ri[0] = c + wx * wx * oc; Ri[1] = wx * wy * oc - wz * s; Ri[2] = wy * s + wx * wz * oc;
    Ri[3] = wz * s + wx * wy * oc; Ri[4] = c + wy * wy * oc; Ri[5] = -wx * s + wy * wz * oc;
    Ri[6] = -wy * s + wx * wz * oc; Ri[7] = wx * s + wy * wz * oc; Ri[8] = c + wz * wz * oc;
  } else {
    Ri[0] = 1; Ri[1] = -a2; Ri[2] = a1; Ri[3] = a2; Ri[4] = 1; Ri[5] = -a0; Ri[6] = -a1; Ri[7] = a0; Ri[8] = 1;
  }
}
__device__ __forceinline__ void fused_step(const PcgIt& g, int ep, int gn_iter, int wv, int lane, int r, int q, bool own, int64_t o,
                                           int row, double xv, bool ill, int cnt, double bb) {
  const StepArgs& sa = *g.sa;
  const int gi = gn_iter;
  const double* tail = g.tail;
  const double loss = sqrt(tail[0] + tail[1] + tail[2]);
  const double prev = sa.step_state[2 * gi];
  const int acc = (int)sa.step_state[2 * gi + 1];
  const bool stop = ill || (acc > 0 && (loss - prev > g.stop_loss_diff || loss == prev));
  if (wv == 0 && lane == 0) {
    if (gi < kMaxLog) {
      sa.stat[3 * gi + 0] = (double)cnt;
      sa.stat[3 * gi + 1] = bb;
      sa.stat[3 * gi + 2] = loss;
    }
    g.flags[F_RES_NONFINITE] = tail[3] != 0.0 ? 1 : 0;
    if (stop) {
      g.flags[F_STOPPED] = 1;
      host_flag(g.hflags, H_STOPPED, ep);
    } else {
      if (acc < g.n_iter_log) {
        sa.loss_log[4 * acc + 0] = loss;
        sa.loss_log[4 * acc + 1] = sqrt(tail[0]);
        sa.loss_log[4 * acc + 2] = sqrt(tail[1]);
        sa.loss_log[4 * acc + 3] = sqrt(tail[2]);
      }
      sa.step_state[2 * gi + 2] = loss;
      sa.step_state[2 * gi + 3] = (double)(acc + 1);
      g.flags[F_ACCEPTED] = acc + 1;
    }
  }
  if (stop) return;
  if (own && g.warm) sa.xh[(int64_t)(gi % kProj) * 6 * g.N + o] = xv;
  double x[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) x[c] = __shfl(xv, r * kSL + c, 64);   // the row's 6 components (lanes q < 6)
  if (q != 0) return;
  if (g.mode == OFX_GN_ARAP && sa.conf[row] != 0.0) return;   // arap: valid nodes keep R, t (model.py:1940-1943)
  double Ri[9];
  kornia_exp(x, Ri);
  double* R = sa.R + 9 * (int64_t)row;
  double Rc[9], Rn[9];
#pragma unroll
  for (int c = 0; c < 9; ++c) Rc[c] = R[c];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) Rn[3 * a + c] = Ri[3 * a] * Rc[c] + Ri[3 * a + 1] * Rc[3 + c] + Ri[3 * a + 2] * Rc[6 + c];
#pragma unroll
  for (int c = 0; c < 9; ++c) R[c] = Rn[c];
#pragma unroll
  for (int c = 0; c < 3; ++c) sa.t[3 * (int64_t)row + c] += x[3 + c];
  if (g.rot_tol > 0.0) {   // adaptive preconditioner refresh: the next step's warm start rebuilds the cluster inverses
    const double acc = sa.racc[row] + sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    sa.racc[row] = acc;
    if (acc > g.rot_tol) g.flags[F_REFRESH] = gi + 1;
  }
}

// kW2 (with kWave): TWO waves per cluster. Wave h multiplies block slot h·64 + lane (one block per lane, not
// two), stages only its half of the inverse's column groups and applies that half (split-K); the scalar
// work, row sums and recurrences run in both waves (identical bits), wave 0 alone stores. Two LDS barriers
// (products, M⁻¹ halves), no memory release.
// Trip 1 issues the wave list and the stop word first, and waits only for the stop word before the stop test and trip
// 2's issue (the rest of trip 1 lands under trip 2's flight; the scalars and the M⁻¹ apply wait for their own loads,
// which retire in issue order). The lane's row of the cluster inverse (its wave's column half) comes to registers by
// plain loads (the wave's 48 row lanes read 768 contiguous bytes per column group): a pending LDS-DMA would make the
// compiler wait for everything (vmcnt(0)) at the first use of any load. (Round 3's OFX_PCG_EARLY levels 0 / 1 — the
// all-of-trip-1 wait with the inverse by LDS-DMA, the early issue alone — and round 4's level 3 (batched LDS reads) and
// write-through stores lost their A/Bs and are gone: DESIGN §6.)
// No kernel-argument fetch on the main path (late round 4): the first seven arguments are pointers, preloaded
// into SGPRs at wave launch (-amdgpu-kernarg-preload-count, build.py; a struct argument is never preloaded); everything
// else the iteration reads comes through them — the step scalars, tolerances and the operator / inverse / new-m addresses
// from the scalar block sc (GnDev::pcs, k_pcg_w0 writes the addresses and tolerances per solve), whose address carries
// the parity in bit 3; the rows' bounds from the wave list; the other parity's partial streams beside Pc. The stop words
// are reset by k_pcg_w0 per solve, so the stop test needs no epoch. The rest of the launch's arguments (rare paths:
// the converging launch's bookkeeping and fused GN step, the CSR form) live in device memory (gp, one copy per handle,
// rewritten when they change): a 76-B kernel argument instead of ~290 B, which the host enqueues faster. In-process A/B
// against the same kernel with its scalars and addresses through the kernel arguments: -0.27 / -0.28 ms per frame.
// mc / Pc are the parity's m and partial streams.
// kAS (overlapping Schwarz): no cluster inverse — w_new goes to as_w (its address in the scalar block's
// inverse slot) and k_as_apply, the next launch, forms m_new.
template <bool kWave, bool kFirst, int kU, bool kW2 = false, bool kAS = false>   // kU: partial pairs per lane and stream
__global__ __launch_bounds__(kW2 ? 128 : 64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_pcg_iter(
    const int2* wl, const int32_t* stopw, const double* Pc, const double* st, const double* mc, const double* sc,
    const PcgIt* __restrict__ gp, int par, int ep, int gn_iter) {   // (not __restrict__: a restrict load sinks past the exit test)
  const PcgIt& g = *gp;   // (read where used: a copy here made the compiler load it all ahead of trip 1)
  (void)par;              // (the parity comes with sc; par stays in the signature for tools and traces)
  constexpr int kNH = kW2 ? 2 : 1;
  constexpr int kNs = 128 * kU;   // the partial streams' stride (= nw_pad)
  __shared__ __attribute__((aligned(16))) double s_v[kNH][kCD];
  __shared__ double s_prod[kWave ? (kWL + kRowMax) * 6 : 1];
  __shared__ double s_half[kW2 ? 64 : 1];
  const int lane = threadIdx.x & 63;
  const int hw = kW2 ? (int)(threadIdx.x >> 6) : 0;   // wave within the cluster's workgroup
  const int wv = blockIdx.x;
#ifdef OFX_STAMPS
  const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
  // ---- trip 1. The scalar block's addresses first (uniform: scalar loads), then the list and the stop word
  const int par_ = (int)((reinterpret_cast<uintptr_t>(sc) >> 3) & 1);
  const double* scb = sc - par_;
  const uint2 aop_v = reinterpret_cast<const uint2*>(scb)[kScAop];
  const uint2 mcl_v = reinterpret_cast<const uint2*>(scb)[kScMcl];
  const uint2 mn_v = reinterpret_cast<const uint2*>(scb)[kScM + (par_ ^ 1)];   // the new m: the other parity's buffer
  int2 bl0 = make_int2(-1, 0), bl1 = make_int2(-1, 0);
  if (kWave) {
    bl0 = wl[(int64_t)wv * kWL + 64 * hw + lane];
    if (!kW2) bl1 = wl[(int64_t)wv * kWL + 64 + lane];
  }
  int stop_ep = stopw[(int64_t)wv * 64 + lane];   // vector load: retires with trip 1
  asm volatile("" ::: "memory");   // the list and stop word leave first
  // the rest of trip 1 in consumption order (loads retire in issue order): the partials and scalars for the step
  // scalars, then the own state and m for the recurrences, the inverse row last (the M⁻¹ apply)
  const int r = lane / kSL, q = lane % kSL, row = wv * kRW + r;
  const bool own = q < 6;
  const int qc = own ? q : 5;
  const int64_t o = 6 * (int64_t)row + qc;
  double2 tp[kPcgStreams][kU];   // the streams are zero beyond nw up to 128·kU: no masks
#pragma unroll
  for (int k = 0; k < kPcgStreams; ++k)
#pragma unroll
    for (int u = 0; u < kU; ++u) tp[k][u] = *reinterpret_cast<const double2*>(Pc + k * kNs + 2 * (lane + 64 * u));
  double own_p[kPcgStreams];
#pragma unroll
  for (int k = 0; k < kPcgStreams; ++k) own_p[k] = Pc[k * kNs + wv];
  const int cnt = reinterpret_cast<const int32_t*>(scb + kScFlags)[F_PCG_CNT];
  const double2 ra = *reinterpret_cast<const double2*>(scb + kScAlpha + 2);   // 1/α of parities 0, 1
  const double2 rt = *reinterpret_cast<const double2*>(scb + kScAlpha + 4);   // the error-stop bound of parities 0, 1
  const double2 rg = *reinterpret_cast<const double2*>(scb + kScGamma + 2);   // 1/γ of parities 0, 1
  const double2 sd = reinterpret_cast<const double2*>(scb + kScSturm)[lane];   // (every wave loads it: the lead uses it)
  const double bb_stored = scb[kScScal + S_BB];
  const double th_prev = scb[kScScal + S_TH_PREV];
  const double2 tols = *reinterpret_cast<const double2*>(scb + kScTol);       // pcg_tol, pcg_err_tol
  asm volatile("" ::: "memory");
  constexpr int kNB = kWave ? (kW2 ? 1 : 2) : 1;   // blocks per lane
  double2 ab[kNB][18], xb[kNB][3];
  constexpr int kMR = kCD / 4 / kNH;   // the lane's inverse row: float4 column groups of its wave's half
  float4 mreg[kMR];
  double v[V_N];
  load_rec(st, o, v);
  const double m = mc[o];
  asm volatile("" ::: "memory");
  // An address from the scalar block is made scalar and turned back into a global-address-space pointer (a generic
  // pointer would be read with flat loads, which the compiler waits for with vmcnt(0)).
  auto addr = [](uint2 v2) -> uint64_t {
    return ((uint64_t)__builtin_amdgcn_readfirstlane(v2.y) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane(v2.x);
  };
  if constexpr (!kAS) {
    typedef float gf4 __attribute__((ext_vector_type(4)));
    const __attribute__((address_space(1))) gf4* Mw =
        reinterpret_cast<const __attribute__((address_space(1))) gf4*>(addr(mcl_v)) + (int64_t)wv * kCD * kCD / 4;
#pragma unroll
    for (int kk = 0; kk < kMR; ++kk) {
      const gf4 t = Mw[(6 * r + qc) + (kMR * hw + kk) * kCD];
      mreg[kk] = make_float4(t.x, t.y, t.z, t.w);
    }
  }
#ifdef OFX_STAMPS
  const int nw = g.nwg_row;
#endif
  // the rows' bounds: packed in the wave list, or (CSR form) from row_ptr
  int wb0 = 0, b0 = 0, b1 = 0;
  if (kWave) {
    wb0 = wl_base(bl0);
    b0 = wb0 + wl_rel(bl0);
    b1 = b0 + wl_len(bl0);
  } else {
    b0 = g.row_ptr[row];
    b1 = g.row_ptr[row + 1];
  }
  const __attribute__((address_space(1))) double* Aop =
      reinterpret_cast<const __attribute__((address_space(1))) double*>(addr(aop_v));
  // after convergence the rest of the chunk ends here. The empty asm with a memory clobber keeps
  // the trip-1 loads above the exit (otherwise they sink past it and the test would gate them).
  asm volatile("" ::: "memory");
  // the wave's stop words are equal (every lane stores the same value), and so are the scalars below: taken
  // as wave-uniform values the exits are scalar branches, so the main path's waits are not merged with the exit paths'
  // (a divergent exit left a vmcnt(0) at the join in front of the products)
  stop_ep = __builtin_amdgcn_readfirstlane(stop_ep);
  if (stop_ep != 0) return;     // this solve has converged (or stopped): a drained launch (k_pcg_w0 zeroed the words)
#ifdef OFX_STAMPS
  if (lane == 0 && g.stamps && cnt < 64) g.stamps[((int64_t)cnt * nw + wv) * 8] = t_entry;
#endif
  OFX_STAMP(1)
  // ---- trip 2: A blocks and gathered m (issued first; the scalar work below overlaps their flight)
  if (kWave)
#pragma unroll
    for (int j = 0; j < kNB; ++j) {   // unconditional loads (padding reads block 0 / m row 0, masked later)
      const int2 e = j ? bl1 : bl0;
      typedef double gd2 __attribute__((ext_vector_type(2)));   // (a plain vector type: loads through address space 1)
      const int slot = kW2 ? 64 * hw + lane : 64 * j + lane;
      // the wave's padded copy of A (k_pcg_w0), 16-B word k of every slot contiguous (1 KB per load instruction, not 64
      // lines as from the CSR copy: -0.08 / -0.21 ms per frame, profiles/r04_ab.json)
      const __attribute__((address_space(1))) gd2* blw =
          reinterpret_cast<const __attribute__((address_space(1))) gd2*>(Aop) + (int64_t)wv * 18 * kWL + slot;
      const double2* vc = reinterpret_cast<const double2*>(mc + 6 * (int64_t)(e.x >= 0 ? e.x : 0));
      // the gathered m row first: the products of the first block rows start before the block's tail lands
#pragma unroll
      for (int k = 0; k < 3; ++k) xb[j][k] = vc[k];
      asm volatile("" ::: "memory");
      // padding slots read the half's first slot (lines its own lane fetches anyway: no extra bytes; their products
      // are masked) — an exec-masked load would make the compiler's waits at the join conservative
      const __attribute__((address_space(1))) gd2* b = e.x >= 0 ? blw : blw - slot + (kW2 ? 64 * hw : 64 * j);
#pragma unroll
      for (int k = 0; k < 18; ++k) {
        const gd2 t = b[k * kWL];
        ab[j][k] = make_double2(t.x, t.y);
      }
    }
  asm volatile("" ::: "memory");   // keep trip 2 issued here (the compiler would sink it past the exit test)
  __builtin_amdgcn_sched_barrier(0);   // ... and no scalar arithmetic above its issue (it would wait for the partials)
  OFX_STAMPX(2)
#ifdef OFX_STAMPS_SCALARS
  {
    double t_ = tp[2][kU - 1].y;   // (wait for the last partial here)
    asm volatile("" : "+v"(t_) :: "memory");
    tp[2][kU - 1].y = t_;
  }
  OFX_STAMPX(3)
#endif
  const double tol_s = tols.x, etol_s = tols.y;
  // outputs, through the preloaded (const) views or the scalar block: the new m, the other parity's partial streams,
  // the state, the stop words, the lead's scalars
  __attribute__((address_space(1))) double* mn = reinterpret_cast<__attribute__((address_space(1))) double*>(addr(mn_v));
  const int ns = kNs;
  double* Pn = const_cast<double*>(Pc) + (par_ ? -kPcgStreams : kPcgStreams) * (int64_t)kNs;
  double* stw = const_cast<double*>(st);
  int32_t* stopw_w = const_cast<int32_t*>(stopw);
  double* sc_w = const_cast<double*>(scb);
  int32_t* flags_w = reinterpret_cast<int32_t*>(sc_w + kScFlags);
  double tb[kFirst ? 2 * kU : 1];   // the first iteration's |b|² partials (kernel-argument pointer: once per solve)
  if (kFirst) {   // (a pointer read from memory is generic: back to the global address space, or flat loads)
    const __attribute__((address_space(1))) double* pb =
        reinterpret_cast<const __attribute__((address_space(1))) double*>(reinterpret_cast<uint64_t>(g.part_b));
#pragma unroll
    for (int u = 0; u < 2 * kU; ++u) tb[u] = pb[lane + 64 * u];
  }
  const double rgam_prev = kFirst ? 1.0 : ((par_ ^ 1) ? rg.y : rg.x);     // 1/γ, 1/α of the previous iteration
  const double ralpha_prev = kFirst ? 1.0 : ((par_ ^ 1) ? ra.y : ra.x);
  const double thr_prev = kFirst ? 0.0 : ((par_ ^ 1) ? rt.y : rt.x);       // error-based stop: bound on γ (below)
  // ---- scalars from the partials (trip-1 data)
  double pa[kPcgStreams];
#pragma unroll
  for (int k = 0; k < kPcgStreams; ++k) {
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < kU; ++u) t += tp[k][u].x + tp[k][u].y;
    pa[k] = wave_sum(t);
  }
#ifdef OFX_STAMPS_SCALARS
  asm volatile("" : "+v"(pa[0]), "+v"(pa[1]), "+v"(pa[2]) :: "memory");
  OFX_STAMPX(4)
#endif
  double bb = bb_stored;
  if (kFirst) {
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < 2 * kU; ++u) t += tb[u];
    bb = wave_sum(t);
  }
  const double gam = pa[0], del = pa[1], rr = pa[2], pp = pa[3];   // pp = ‖p‖² of the previous iteration's direction
  const double tol = tol_s;
  const bool lead = wv == 0 && lane == 0 && hw == 0;
  const bool w0 = hw == 0;   // the wave that stores (kW2: both compute the same bits)
  double beta = 0.0, alpha;
  if (kFirst) {
    alpha = div_nr(gam, del);
  } else {
    beta = gam * rgam_prev;
    alpha = div_nr(gam, del - beta * gam * ralpha_prev);
  }
  // Stop: the relative residual ‖r‖ <= tol·‖b‖ AND (pcg_err_tol = τ > 0) the estimated Euclidean norm of the solution
  // error ‖e‖₂ ≈ √(γ·μ/θ̂) <= τ, or the relative residual at the f64 floor (1e-12). The estimate (round 6):
  // ‖e‖²_A = rᵀA⁻¹r <= γ/λ_min(M⁻¹A) with γ = rᵀM⁻¹r, θ̂ the previous iteration's estimate of λ_min(M⁻¹A) from below
  // (kept by the lead wave, below); late in a solve the error lies along the slowest modes, which the last search
  // direction p follows, so ‖e‖²₂ ≈ ‖e‖²_A·μ with μ = ‖p‖²/pᵀAp = pp·α/γ of the previous iteration (Hestenes–Stiefel:
  // ‖e_k‖² - ‖e_k+1‖² = (‖p_k‖²/p_kᵀAp_k)(‖e_k‖²_A + ‖e_k+1‖²_A)). Measured in the norm of the 1e-5 bar, it needs no
  // preconditioner-specific factor (round 5 tightened an M-norm rule 4x under Schwarz). thr = τ²·θ̂; the test is
  // γ·pp/γ_prev <= thr/α_prev (the reciprocals are carried). The residual alone cannot see the error of an
  // ill-conditioned system (real data: DESIGN §6).
  const double etol = etol_s;
  const bool conv = (rr <= tol * tol * bb && (etol <= 0.0 || gam * pp * rgam_prev <= thr_prev * ralpha_prev)) ||
                    gam == 0.0 || rr <= 1e-24 * bb;
  int leave = (conv || !isfinite(alpha) || !(alpha > 0.0)) ? 1 : 0;
  leave = __builtin_amdgcn_readfirstlane(leave);
  OFX_STAMPX(5)
  if (leave) {   // converged, or breakdown (A SPD => alpha > 0): keep x
    if (kFirst && lead) sc_w[kScScal + S_BB] = bb;
    if (!w0) return;
    if (lane == 0) {
      Pn[wv] = own_p[0]; Pn[ns + wv] = own_p[1]; Pn[2 * ns + wv] = conv ? own_p[2] : 0.0; Pn[3 * ns + wv] = own_p[3];
    }
    stopw_w[(int64_t)wv * 64 + lane] = ep;
    const bool ill = !conv && !isfinite(alpha);
    if (g.fuse && !g.flags[F_STOPPED]) fused_step(g, ep, gn_iter, wv, lane, r, q, own, o, row, v[V_X], ill, cnt, bb);
    if (lead && !g.flags[F_DONE] && !g.flags[F_STOPPED]) {   // first launch to see it
      g.flags[F_DONE] = 1; g.flags[F_PCG_IT] = cnt; g.flags[F_PCG_TOTAL] += cnt;
      if (ill) g.flags[F_ILL] = 1;
      host_flag(g.hflags, H_PCG_IT, cnt);
      __hip_atomic_store(g.hflags + H_DONE, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);   // after the count
    }
    return;
  }
  // the lead's scalar stores (read by the next launch only) are issued last — on gfx9 vmcnt counts stores too,
  // so stores issued here made the lead wave's first wait on trip 2 a vmcnt(0) that also waited for their acks
  // the Lanczos tridiagonal of the preconditioned operator grows by one row per iteration: T_kk = 1/α_k + β_{k-1}/α_{k-1},
  // T_{k,k-1}² = β_{k-1}/α_{k-1}² (β_{k-1} = γ_k/γ_{k-1}); its smallest eigenvalue (Ritz value) θ_k decreases towards
  // λ_min(M⁻¹A). Lane s of the lead wave keeps the LDLᵀ pivot d_k(σ_s) = T_kk - σ_s - T²_{k,k-1}/d_{k-1}(σ_s) of
  // T_k - σ_s I and the count of negative pivots, which is the number of Ritz values below σ_s (Sylvester's inertia;
  // the bisection count of LAPACK's dstebz): O(1) per iteration. Shifts σ_s = 2^(-e_s/4), e_s = s for s < 40 (quarter
  // octaves down to 2^-9.75), 2s - 40 beyond (half octaves down to 2^-21.5). θ̂ = the largest σ_s with no Ritz value below
  // it (θ_k / 2^(1/4) < θ̂ <= θ_k above 2^-10; 1 if θ_k >= 1; 0 below the last shift). Early in a solve θ_k still
  // over-estimates λ_min, so a GN step after the first also takes the previous step's final θ̂ when that is smaller (the
  // step's operator differs little from the previous one's: on the moose a warm-started step stopped after 64
  // iterations with 3.7e-5 left without it, tools/errstop_study.py). thr = pcg_err_tol²·min(θ̂, θ̂_prev).
  double2 sd_new = sd;
  double thr_new = 0.0, th_cur = 1e300;
  auto shift = [](int s) {   // σ_s
    const int e = s < 40 ? s : 2 * s - 40;
    const int k = e & 3;
    const double c = k == 0 ? 1.0 : k == 1 ? 0.84089641525371454303 : k == 2 ? 0.70710678118654752440
                                                                            : 0.59460355750136053336;
    return ldexp(c, -(e >> 2));
  };
  if (wv == 0 && hw == 0 && etol > 0.0) {   // (workgroup-uniform)
    const double rca = 1.0 / alpha;
    const double diag = kFirst ? rca : rca + beta * ralpha_prev;
    const double e2 = kFirst ? 0.0 : beta * ralpha_prev * ralpha_prev;
    const double sig = shift(lane);
    double d = (diag - sig) - (kFirst ? 0.0 : e2 / sd.x);
    if (fabs(d) < 1e-300) d = -1e-300;        // an exact zero pivot counts as negative (dstebz's pivmin)
    const double c = (kFirst ? 0.0 : sd.y) + (d < 0.0 ? 1.0 : 0.0);
    sd_new = make_double2(d, c);
    const uint64_t free_ = __ballot(c == 0.0);   // the shifts with no Ritz value below them: a suffix of the lanes
    const double th = free_ ? shift(__ffsll((unsigned long long)free_) - 1) : 0.0;
    th_cur = th;
    const double tu = fmin(th, th_prev);
    thr_new = (etol * etol) * tu;
  }
  auto lead_stores = [&]() {
    if (lead) {
      sc_w[kScAlpha + 2 + par_] = 1.0 / alpha; sc_w[kScGamma + 2 + par_] = 1.0 / gam; flags_w[F_PCG_CNT] = cnt + 1;
      sc_w[kScAlpha + 4 + par_] = thr_new;
      if (etol > 0.0) sc_w[kScScal + S_TH_CUR] = th_cur;
    }
    if (wv == 0 && hw == 0 && etol > 0.0) reinterpret_cast<double2*>(sc_w + kScSturm)[lane] = sd_new;
    if (kFirst && lead) sc_w[kScScal + S_BB] = bb;
  };
  OFX_STAMP(2)
  OFX_STAMPX(6)
  // ---- n = A m (own component)
  double nc;
  if (kWave) {
#pragma unroll
    for (int j = 0; j < kNB; ++j) {
      const bool ok = (j ? bl1 : bl0).x >= 0;
      const int slot = kW2 ? 64 * hw + lane : j * 64 + lane;
      double x[6];
#pragma unroll
      for (int k = 0; k < 3; ++k) { x[2 * k] = xb[j][k].x; x[2 * k + 1] = xb[j][k].y; }
#pragma unroll
      for (int i = 0; i < 6; ++i) {   // (the PCG is not bit-pinned: fused multiply-adds)
        const double2 b01 = ab[j][3 * i], b23 = ab[j][3 * i + 1], b45 = ab[j][3 * i + 2];
        const double t = fma(b45.y, x[5], fma(b45.x, x[4], fma(b23.y, x[3], fma(b23.x, x[2], fma(b01.y, x[1], b01.x * x[0])))));
        s_prod[slot * 6 + i] = ok ? t : 0.0;
      }
    }
    OFX_STAMP(3)
    if (kW2) {   // both waves' products: an LDS barrier (no memory release)
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
    } else {
      wave_lds_sync();
    }
    // row sums in CSR order (rows of at most kRowMax blocks; unrolled reads at immediate offsets,
    // masked; s_prod is padded so the reads past the wave's last block stay inside it)
    const int len = b1 - b0;
    const double* sp = s_prod + (b0 - wb0) * 6 + qc;
    // every read in flight before the first add (left to the compiler, each pair of reads was waited for before the
    // next pair issued: ten LDS round trips in a row)
    double tv[kRowMax];
#pragma unroll
    for (int k = 0; k < kRowMax; ++k) tv[k] = sp[6 * k];
    __builtin_amdgcn_sched_barrier(0);
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < kRowMax; ++k) a += k < len ? tv[k] : 0.0;
    nc = a;
  } else {
    double n[6];
    row_spmv(g, b0, b1, q, mc, n);
    nc = pick6(n, qc);
  }
  OFX_STAMP(4)
  double d[kPcgStreams] = {0.0, 0.0, 0.0, 0.0};
  {
    const double zz = fma(beta, v[V_Z], nc);
    const double qq = fma(beta, v[V_Q], m);
    const double sv = fma(beta, v[V_S], v[V_W]);
    const double p = fma(beta, v[V_P], v[V_U]);
    const double rn = fma(-alpha, sv, v[V_R]);
    const double un = fma(-alpha, qq, v[V_U]);
    const double w2 = fma(-alpha, zz, v[V_W]);
    if (own) {
      const double nv[V_N] = {fma(alpha, p, v[V_X]), rn, un, zz, qq, sv, p, w2};
      if (w0) store_rec(stw, o, nv);   // (the same buffer as st, written)
      if (kAS) {
        if (w0) reinterpret_cast<__attribute__((address_space(1))) double*>(addr(mcl_v))[o] = w2;
      } else {
        s_v[hw][6 * r + q] = w2;
      }
      d[0] = rn * un; d[1] = w2 * un; d[2] = rn * rn; d[3] = p * p;
    }
  }
  OFX_STAMP(5)
  if (!kAS) wave_lds_sync();
  if constexpr (kAS) {
    // (m_new: k_as_apply)
  } else if (kW2) {      // split-K: wave h applies column groups [6h, 6h + 6); wave 0 adds the halves (fixed order)
    double hsum = 0.0;
    if (own) {
      // the half's 24 values in flight before the first FMA (left to the compiler: five LDS round trips in a row)
      double2 vv[kCD / 4];
      const double2* sv2 = reinterpret_cast<const double2*>(&s_v[hw][4 * (kCD / 8) * hw]);
#pragma unroll
      for (int i = 0; i < kCD / 4; ++i) vv[i] = sv2[i];
      __builtin_amdgcn_sched_barrier(0);
      double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < kCD / 8; ++kk) {
        const float4 t = mreg[kk];
        a[0] = fma((double)t.x, vv[2 * kk].x, a[0]);
        a[1] = fma((double)t.y, vv[2 * kk].y, a[1]);
        a[2] = fma((double)t.z, vv[2 * kk + 1].x, a[2]);
        a[3] = fma((double)t.w, vv[2 * kk + 1].y, a[3]);
      }
      hsum = (a[0] + a[1]) + (a[2] + a[3]);
    }
    if (hw == 1) s_half[lane] = hsum;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (w0 && own) mn[o] = hsum + s_half[lane];
  } else if (own) {      // m of the next iteration: M⁻¹ w_new, cluster-local (the lane's inverse row in registers)
    double a[4] = {0.0, 0.0, 0.0, 0.0};   // four independent FMA chains
#pragma unroll
    for (int k = 0; k < kCD / 4; ++k) {
      const float4 t = mreg[k];
      a[0] = fma((double)t.x, s_v[0][4 * k], a[0]);
      a[1] = fma((double)t.y, s_v[0][4 * k + 1], a[1]);
      a[2] = fma((double)t.z, s_v[0][4 * k + 2], a[2]);
      a[3] = fma((double)t.w, s_v[0][4 * k + 3], a[3]);
    }
    mn[o] = (a[0] + a[1]) + (a[2] + a[3]);
  }
  OFX_STAMP(6)
  // the four per-wave partials of the next launch: kW2's second wave (idle otherwise here) sums and stores the third and
  // fourth, from the same bits wave 0 holds, so wave 0's tail is two wave sums instead of four
  if (!w0) {
    if (kW2) {
      const double s2 = wave_sum(d[2]), s3 = wave_sum(d[3]);
      if (lane == 0) { Pn[2 * ns + wv] = s2; Pn[3 * ns + wv] = s3; }
    }
    return;
  }
  d[0] = wave_sum(d[0]);
  d[1] = wave_sum(d[1]);
  if (!kW2) { d[2] = wave_sum(d[2]); d[3] = wave_sum(d[3]); }
  if (lane == 0) {
    Pn[wv] = d[0]; Pn[ns + wv] = d[1];
    if (!kW2) { Pn[2 * ns + wv] = d[2]; Pn[3 * ns + wv] = d[3]; }
  }
  lead_stores();
  OFX_STAMP(7)
}

// One launch per Schwarz PCG iteration (round 6; OFX_AS_ONE=0 restores k_pcg_iter<.., kAS> + k_as_apply).
// The two-launch form needs two exchanges per iteration — the SpMV n = A m reads m on the neighbours' rows, the apply
// m = M⁻¹ w reads w on the subdomains' rings — and a kernel boundary for each. Here workgroup c works on its whole
// subdomain D_c (own 8 rows + ring): it keeps ghost copies of the ring rows' recurrence vectors (w, z), forms n = A m on
// all of D_c's rows (3x the SpMV rows) and the ring rows' z, w updates exactly as their owners do (the same blocks, the
// same m bits, the same operations: bit-identical copies), and applies its own subdomain inverse, y_c = D Ẑ D w[D_c]. The
// next launch sums m on the columns it needs from the <= 1 + kAsX contributions per node in ascending subdomain order —
// the order in which k_as_apply sums a row's segments, each contribution being that segment's value — so the iterates are
// bitwise those of the two-launch form. One exchange per iteration: one kernel boundary.
// Roles (1024 threads; the rows first in dispatch order): waves 0-2 the rows: 0 the own rows (k_pcg_iter's wave: scalars,
// stop, recurrences, partials, the converging launch's GN step), 1-2 the ring rows (ghost z, w); waves 3-7 one S2 node each
// (its contributions summed into m; a second pass past 320 nodes) and one inverse row half each (the dot product, as
// k_as_apply's two lanes); waves 8-15 the blocks of D_c's rows (the A rows and the products). Trip 1: the stop word, tables, state,
// partials, inverse rows; trip 2: the A blocks and the contributions. Three barriers (m, products, the w image).
// k_as_iter's workgroup barrier: LDS writes complete (lgkmcnt(0)), then s_barrier — no memory fence: __syncthreads()
// would also wait for every outstanding global load and store of the wave (the A rows, the inverse rows, the state
// stores), which the roles consume or retire later
__device__ __forceinline__ void as_lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}
#ifdef OFX_STAMPS   // tuning build: per (iteration < 64, cluster) 8 clock stamps — 0 entry, 1 trip 1 landed, 2 scalars done,
                    // 3 after barrier 1, 4 after barrier 2, 5 after barrier 3 (own-row wave), 6 end; 7: the row sums done (after 4)
#define OFX_AS_ITER_STAMP(k, cn) \
  if (lane == 0 && g.stamps && (cn) < 64) g.stamps[((int64_t)(cn) * nwg + c) * 8 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define OFX_AS_ITER_STAMP(k, cn)
#endif
template <bool kFirst, int kU, bool kRowSplit>
__global__ __launch_bounds__(kAsIterT) void k_as_iter(const int32_t* stopw, const double* Pc, const double* st,
                                                      const double* sc, const char* tab, int cap, int xcd_per, int nwg,
                                                      int ep, const PcgIt* gp, int gn_iter) {
  const PcgIt& g = *gp;
  constexpr int kNs = 128 * kU;
  constexpr int kS2W = 5 * 64;   // S2 nodes per pass (waves 3-7)
  __shared__ __attribute__((aligned(16))) double s_m[kGS * 6];
  __shared__ __attribute__((aligned(16))) double s_prod[(kGB + kRowMax) * 6];
  __shared__ __attribute__((aligned(16))) double s_w[kAsD];
  __shared__ int s_leave;
  __shared__ double s_ab[2];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);   // (uniform: the roles below are scalar branches)
  // workgroups are dealt to the 8 XCDs round robin: with xcd_per > 0 XCD x runs clusters [x·xcd_per, (x+1)·xcd_per), so
  // its L2 holds one contiguous run of subdomains with their shared ring rows and blocks (the grid is 8·xcd_per)
  const int c = xcd_per > 0 ? (int)(blockIdx.x & 7) * xcd_per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (c >= nwg) return;   // (the padding workgroups of the XCD form, before any barrier)
  const AsTabP tp = as_tab_at(const_cast<char*>(tab), cap);
  const int par_ = (int)((reinterpret_cast<uintptr_t>(sc) >> 3) & 1);
  const double* scb = sc - par_;
  const int32_t* rt = tp.row + (int64_t)c * kGRow;
  const double* yr = tp.y + (int64_t)par_ * cap * kAsD;   // the previous launch's contributions
  // Each role issues trip 1 (the stop word first), tests the stop word (drained launches end there, before any
  // barrier), issues trip 2, and meets the others at three barriers: (1) m on S2 + the stop decision, (2) the block
  // products, (3) the w image. Loads are unconditional (clamped), the roles' data live only inside their branch.
  if (wave >= 8) {  // ---------------- blocks (waves 8-15; tb = block index)
    const int tb = t - kGB;
    int stop_ep = stopw[(int64_t)c * 64 + lane];
    const int nb = rt[26];
    typedef double gd2 __attribute__((ext_vector_type(2)));
    const __attribute__((address_space(1))) gd2* A2 =
        reinterpret_cast<const __attribute__((address_space(1))) gd2*>(reinterpret_cast<const uint64_t*>(scb)[kScAop]);
    if (kRowSplit) {
      // one thread per (block, row): pair p = t + 512 j, block p / 6, row p % 6 — the wave's 64 lanes read ~11 blocks'
      // rows as consecutive 48-B pieces (a thread per whole 288-B block touched 64 lines per load instruction)
      constexpr int kP = (kGB * 6 + kGB - 1) / kGB;   // pairs per thread (6)
      int2 be[kP];
#pragma unroll
      for (int j = 0; j < kP; ++j) be[j] = tp.blk[(int64_t)c * kGB + (tb + kGB * j) / 6];
      asm volatile("" ::: "memory");
      stop_ep = __builtin_amdgcn_readfirstlane(stop_ep);
      if (stop_ep != 0) return;
      double2 ar[kP][3];
#pragma unroll
      for (int j = 0; j < kP; ++j)
        if (tb - lane + kGB * j < 6 * nb)   // (wave-uniform)
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const gd2 x = A2[18 * (int64_t)be[j].x + 3 * ((tb + kGB * j) % 6) + k];
            ar[j][k] = make_double2(x.x, x.y);
          }
      as_lds_barrier();   // (1)
#pragma unroll
      for (int j = 0; j < kP; ++j) {
        const int pp = tb + kGB * j;
        if (pp < 6 * nb) {   // k_pcg_iter's operation order (row i of the block's product)
          const int k = be[j].y >> 5;
          double x[6];
#pragma unroll
          for (int q = 0; q < 6; ++q) x[q] = s_m[6 * k + q];
          const double2 b01 = ar[j][0], b23 = ar[j][1], b45 = ar[j][2];
          s_prod[pp] = fma(b45.y, x[5], fma(b45.x, x[4], fma(b23.y, x[3], fma(b23.x, x[2], fma(b01.y, x[1], b01.x * x[0])))));
        }
      }
      as_lds_barrier();   // (2)
      as_lds_barrier();   // (3)
      return;
    }
    const int2 be = tp.blk[(int64_t)c * kGB + tb];
    asm volatile("" ::: "memory");
    stop_ep = __builtin_amdgcn_readfirstlane(stop_ep);
    if (stop_ep != 0) return;
    const __attribute__((address_space(1))) gd2* b = A2 + 18 * (int64_t)be.x;
    const bool any = tb - lane < nb;   // (wave-uniform: waves past the subdomain's blocks load nothing)
    double2 ab[18];
    if (any)
#pragma unroll
      for (int k = 0; k < 18; ++k) { const gd2 x = b[k]; ab[k] = make_double2(x.x, x.y); }
    as_lds_barrier();   // (1)
    if (any && tb < nb) {   // k_pcg_iter's operation order
      const int k = be.y >> 5;
      double x[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) x[j] = s_m[6 * k + j];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 b01 = ab[3 * i], b23 = ab[3 * i + 1], b45 = ab[3 * i + 2];
        s_prod[tb * 6 + i] =
            fma(b45.y, x[5], fma(b45.x, x[4], fma(b23.y, x[3], fma(b23.x, x[2], fma(b01.y, x[1], b01.x * x[0])))));
      }
    }
    as_lds_barrier();   // (2)
    as_lds_barrier();   // (3)
    return;
  }
  if (wave >= 3) {  // ---------------- S2 nodes (m) and inverse rows (y): waves 3-7
    const int ts = t - 192;
    int stop_ep = stopw[(int64_t)c * 64 + lane];
    const int k2 = ts < kGS ? ts : kGS - 1;
    const int4 cn = tp.con[(int64_t)c * kGS + k2];
    const int nd = rt[25], ns = rt[27];
    const int ry = min(ts >> 1, kAsD - 1), hl = ts & 1;
    asm volatile("" ::: "memory");
    stop_ep = __builtin_amdgcn_readfirstlane(stop_ep);
    if (stop_ep != 0) return;
    // m on S2: 0 + the contributions in ascending subdomain order (k_as_apply's sum of a row's segments, each
    // contribution being that segment's value); the first iteration's (m0 = M⁻¹ w0) k_as_w0 left in y[0]
    auto gather = [&](int4 e4, double mv[6]) {
      double2 cz[4][3];
      {
        const int e[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#ifndef OFX_AS_NOSKIP   // absent contributions (a node is in 3.1 subdomains on average) load nothing: exec-masked lanes
          if (j == 0 || e[j] >= 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) cz[j][k] = reinterpret_cast<const double2*>(yr + e[j])[k];
          } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) cz[j][k] = make_double2(0.0, 0.0);
          }
#else                   // (an absent one re-reads the first: no extra lines)
          const double2* p = reinterpret_cast<const double2*>(yr + (e[j] >= 0 ? e[j] : e[0]));
#pragma unroll
          for (int k = 0; k < 3; ++k) cz[j][k] = p[k];
#endif
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e[4] = {e4.x, e4.y, e4.z, e4.w};
        double mx = 0.0, my = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { mx += e[j] >= 0 ? cz[j][k].x : 0.0; my += e[j] >= 0 ? cz[j][k].y : 0.0; }
        mv[2 * k] = mx; mv[2 * k + 1] = my;
      }
    };
    if (ts - lane < ns) {   // (wave-uniform: waves past the S2 nodes gather nothing)
      double mv[6];
      gather(cn, mv);
      if (ts < ns)
#pragma unroll
        for (int j = 0; j < 6; ++j) s_m[6 * ts + j] = mv[j];
    }
    if (ns > kS2W)   // (rare: more than 320 distinct columns) further passes, one more trip each
      for (int kk = ts + kS2W; kk < ns; kk += kS2W) {
        double mv[6];
        gather(tp.con[(int64_t)c * kGS + kk], mv);
#pragma unroll
        for (int j = 0; j < 6; ++j) s_m[6 * kk + j] = mv[j];
      }
    as_lds_barrier();   // (1)
    // the inverse rows now (only the last phase reads them; issued with the first trip they queued the whole
    // workgroup's small loads behind 46 KB per workgroup)
    uint4 z[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) z[k] = tp.slab[((int64_t)c * kAsK + 9 * hl + k) * kAsD + ry];
    const float dsc_r = tp.dsc[(int64_t)c * kAsD + ry];
    as_lds_barrier();   // (2)
    as_lds_barrier();   // (3)
    if (s_leave) return;   // (converged: no contributions; the row waves took the leave path)
    // y_c = D Ẑ (D w): k_as_apply's segment dot (two lanes, four chains, the pair summed by DPP) times the row scale
    const double2* w2p = reinterpret_cast<const double2*>(s_w);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    auto lo = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xFFFFu)); };
    auto hi = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); };
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int kw = 9 * hl + k;
      const double2 p0 = w2p[4 * kw], p1 = w2p[4 * kw + 1], p2 = w2p[4 * kw + 2], p3 = w2p[4 * kw + 3];
      a0 = fma(lo(z[k].x), p0.x, a0);
      a1 = fma(hi(z[k].x), p0.y, a1);
      a2 = fma(lo(z[k].y), p1.x, a2);
      a3 = fma(hi(z[k].y), p1.y, a3);
      a0 = fma(lo(z[k].z), p2.x, a0);
      a1 = fma(hi(z[k].z), p2.y, a1);
      a2 = fma(lo(z[k].w), p3.x, a2);
      a3 = fma(hi(z[k].w), p3.y, a3);
    }
    double dot = (a0 + a1) + (a2 + a3);
    dot += dpp_mov<0xB1>(dot);   // quad_perm [1, 0, 3, 2]: the row's two halves
    if (hl == 0 && ts < 2 * kAsD && (ts >> 1) < 6 * nd)
      tp.y[(int64_t)(par_ ^ 1) * cap * kAsD + (int64_t)c * kAsD + (ts >> 1)] = (double)dsc_r * dot;
    return;
  }
  // ---------------- rows: wave 0 the own rows (k_pcg_iter's wave), 1-2 the ring rows (ghost z, w)
  const int jr = wave, r = lane >> 3, q = lane & 7;
#ifdef OFX_STAMPS
  const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
  const bool own = q < 6;
  const int qc = own ? q : 5;
  const int l = 8 * jr + r;                       // subdomain row
  const int row = c * kCS + r;                    // (own rows)
  const int64_t o = 6 * (int64_t)row + qc;
  int stop_ep = stopw[(int64_t)c * 64 + lane];
  // wave 0 alone reads the partials and the step scalars (every wave of every workgroup reading the same few KB, written
  // by all workgroups of the previous launch, made them one hot spot) and hands alpha, beta and the decision to 1-2
  double2 tpp[kPcgStreams][kU];
  double own_p[kPcgStreams];
  int cnt = 0;
  double2 ra = make_double2(0.0, 0.0), rtb = ra, rg = ra, sd = ra, tols = ra;
  double bb_stored = 0.0, th_prev = 0.0;
  if (jr == 0) {
#pragma unroll
    for (int k = 0; k < kPcgStreams; ++k)
#pragma unroll
      for (int u = 0; u < kU; ++u) tpp[k][u] = *reinterpret_cast<const double2*>(Pc + k * kNs + 2 * (lane + 64 * u));
#pragma unroll
    for (int k = 0; k < kPcgStreams; ++k) own_p[k] = Pc[k * kNs + c];
    cnt = reinterpret_cast<const int32_t*>(scb + kScFlags)[F_PCG_CNT];
    ra = *reinterpret_cast<const double2*>(scb + kScAlpha + 2);
    rtb = *reinterpret_cast<const double2*>(scb + kScAlpha + 4);
    rg = *reinterpret_cast<const double2*>(scb + kScGamma + 2);
    sd = reinterpret_cast<const double2*>(scb + kScSturm)[lane];
    bb_stored = scb[kScScal + S_BB];
    th_prev = scb[kScScal + S_TH_PREV];
    tols = *reinterpret_cast<const double2*>(scb + kScTol);
  }
  const int nd = rt[25];
  const int rs = rt[l], re = rt[l + 1], rk = rt[32 + l];
  const float dsc_l = tp.dsc[(int64_t)c * kAsD + 6 * l + qc];
  double v[V_N];
  double wg = 0.0, zg = 0.0;
  const int gi = (c * kAsRing + (l >= kCS ? l - kCS : 0)) * 6 + qc;
  if (jr == 0) {
    load_rec(st, o, v);
  } else if (kFirst) {   // the owners' w0 from as_w (k_pcg_w0), z0 = +0 (their records hold +0 there). Not their state
    // records: the owners rewrite those in this very launch, and with more workgroups than CUs a later workgroup would
    // read the new values
    const double* w0v = reinterpret_cast<const double*>(reinterpret_cast<const uint64_t*>(scb)[kScMcl]);
    wg = w0v[6 * (int64_t)rt[64 + l] + qc];
    zg = 0.0;
  } else {
    const double2 gz = tp.gh[gi];
    wg = gz.x;
    zg = gz.y;
  }
  asm volatile("" ::: "memory");
  stop_ep = __builtin_amdgcn_readfirstlane(stop_ep);
  if (stop_ep != 0) return;
#ifdef OFX_STAMPS
  if (jr == 0 && lane == 0 && g.stamps && cnt < 64) g.stamps[((int64_t)cnt * nwg + c) * 8] = t_entry;
#endif
  if (jr == 0) { OFX_AS_ITER_STAMP(1, cnt) }
  double tb[kFirst ? 2 * kU : 1];
  if (kFirst && jr == 0) {   // the first iteration's |b|² partials
    const __attribute__((address_space(1))) double* pb =
        reinterpret_cast<const __attribute__((address_space(1))) double*>(reinterpret_cast<uint64_t>(g.part_b));
#pragma unroll
    for (int u = 0; u < 2 * kU; ++u) tb[u] = pb[lane + 64 * u];
  }
  // ---- scalars and the stop decision (k_pcg_iter's), wave 0, ahead of barrier 1: the S2 waves' contributions (a
  // second dependent trip behind their static table) land after the partials, so the scalars cost no time here
  const double etol = tols.y;
  double alpha = 0.0, beta = 0.0, gam = 0.0, bb = bb_stored, ralpha_prev = 1.0;
  bool conv = false;
  int leave = 0;
  const bool lead = c == 0 && jr == 0 && lane == 0;
  if (jr == 0) {
    const double tol = tols.x;
    const double rgam_prev = kFirst ? 1.0 : ((par_ ^ 1) ? rg.y : rg.x);
    ralpha_prev = kFirst ? 1.0 : ((par_ ^ 1) ? ra.y : ra.x);
    const double thr_prev = kFirst ? 0.0 : ((par_ ^ 1) ? rtb.y : rtb.x);
    double pa[kPcgStreams];
#pragma unroll
    for (int k = 0; k < kPcgStreams; ++k) {
      double tt = 0.0;
#pragma unroll
      for (int u = 0; u < kU; ++u) tt += tpp[k][u].x + tpp[k][u].y;
      pa[k] = wave_sum(tt);
    }
    if (kFirst) {
      double tt = 0.0;
#pragma unroll
      for (int u = 0; u < 2 * kU; ++u) tt += tb[u];
      bb = wave_sum(tt);
    }
    gam = pa[0];
    const double del = pa[1], rr = pa[2], pp = pa[3];
    if (kFirst) {
      alpha = div_nr(gam, del);
    } else {
      beta = gam * rgam_prev;
      alpha = div_nr(gam, del - beta * gam * ralpha_prev);
    }
    conv = (rr <= tol * tol * bb && (etol <= 0.0 || gam * pp * rgam_prev <= thr_prev * ralpha_prev)) || gam == 0.0 ||
           rr <= 1e-24 * bb;
    leave = (conv || !isfinite(alpha) || !(alpha > 0.0)) ? 1 : 0;
    leave = __builtin_amdgcn_readfirstlane(leave);
    if (lane == 0) { s_leave = leave; s_ab[0] = alpha; s_ab[1] = beta; }
    OFX_AS_ITER_STAMP(2, cnt)
  }
  as_lds_barrier();   // (1)
  if (jr == 0) { OFX_AS_ITER_STAMP(3, cnt) }
  as_lds_barrier();   // (2)
  if (jr == 0) { OFX_AS_ITER_STAMP(4, cnt) }
  if (jr != 0) {
    leave = s_leave;
    alpha = s_ab[0];
    beta = s_ab[1];
  }
  if (leave) {       // converged, or breakdown (A SPD => alpha > 0): keep x (k_pcg_iter's leave path)
    if (jr != 0) {
      as_lds_barrier();   // (3)
      return;
    }
    const bool ill = !conv && !isfinite(alpha);
    if (kFirst && lead) const_cast<double*>(scb)[kScScal + S_BB] = bb;
    double* Pn = const_cast<double*>(Pc) + (par_ ? -kPcgStreams : kPcgStreams) * (int64_t)kNs;
    if (lane == 0) {
      Pn[c] = own_p[0]; Pn[kNs + c] = own_p[1]; Pn[2 * kNs + c] = conv ? own_p[2] : 0.0; Pn[3 * kNs + c] = own_p[3];
    }
    const_cast<int32_t*>(stopw)[(int64_t)c * 64 + lane] = ep;
    if (g.fuse && !g.flags[F_STOPPED]) fused_step(g, ep, gn_iter, c, lane, r, q, own, o, row, v[V_X], ill, cnt, bb);
    if (lead && !g.flags[F_DONE] && !g.flags[F_STOPPED]) {
      g.flags[F_DONE] = 1; g.flags[F_PCG_IT] = cnt; g.flags[F_PCG_TOTAL] += cnt;
      if (ill) g.flags[F_ILL] = 1;
      host_flag(g.hflags, H_PCG_IT, cnt);
      __hip_atomic_store(g.hflags + H_DONE, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    as_lds_barrier();   // (3)
    return;
  }
  // n on the subdomain row: its blocks in CSR order (k_pcg_iter's row sum)
  const int rlen = l < nd ? re - rs : 0;
  const double* sp = s_prod + rs * 6 + qc;
  double tv[kRowMax];
#pragma unroll
  for (int k = 0; k < kRowMax; ++k) tv[k] = sp[6 * k];
  __builtin_amdgcn_sched_barrier(0);
  double nc = 0.0;
#pragma unroll
  for (int k = 0; k < kRowMax; ++k) nc += k < rlen ? tv[k] : 0.0;
#ifdef OFX_STAMPS
  if (jr == 0) { asm volatile("" :: "v"(nc)); OFX_AS_ITER_STAMP(7, cnt) }
#endif
  double d[kPcgStreams] = {0.0, 0.0, 0.0, 0.0};
  double w2;
  if (jr == 0) {
    const double m = s_m[6 * rk + qc];
    const double zz = fma(beta, v[V_Z], nc);
    const double qq = fma(beta, v[V_Q], m);
    const double sv = fma(beta, v[V_S], v[V_W]);
    const double p = fma(beta, v[V_P], v[V_U]);
    const double rn = fma(-alpha, sv, v[V_R]);
    const double un = fma(-alpha, qq, v[V_U]);
    w2 = fma(-alpha, zz, v[V_W]);
    if (own) {
      const double nv[V_N] = {fma(alpha, p, v[V_X]), rn, un, zz, qq, sv, p, w2};
      store_rec(const_cast<double*>(st), o, nv);
      d[0] = rn * un; d[1] = w2 * un; d[2] = rn * rn; d[3] = p * p;
    }
  } else {
    const double zz = fma(beta, zg, nc);
    w2 = fma(-alpha, zz, wg);
    if (own && l < nd) tp.gh[gi] = make_double2(w2, zz);
  }
  if (own) s_w[6 * l + q] = l < nd ? w2 * (double)dsc_l : 0.0;
  as_lds_barrier();   // (3)
  if (jr != 0) return;
  OFX_AS_ITER_STAMP(5, cnt)
  // ---- the lead wave's Ritz bracket (k_pcg_iter's Sturm step) and the error-stop threshold τ²·min(θ̂, θ̂_prev)
  double2 sd_new = sd;
  double thr_new = 0.0, th_cur = 1e300;
  auto shift = [](int s) {
    const int e = s < 40 ? s : 2 * s - 40;
    const int k = e & 3;
    const double cc = k == 0 ? 1.0 : k == 1 ? 0.84089641525371454303 : k == 2 ? 0.70710678118654752440
                                                                             : 0.59460355750136053336;
    return ldexp(cc, -(e >> 2));
  };
  if (c == 0 && etol > 0.0) {
    const double rca = 1.0 / alpha;
    const double diag = kFirst ? rca : rca + beta * ralpha_prev;
    const double e2 = kFirst ? 0.0 : beta * ralpha_prev * ralpha_prev;
    const double sig = shift(lane);
    double dd = (diag - sig) - (kFirst ? 0.0 : e2 / sd.x);
    if (fabs(dd) < 1e-300) dd = -1e-300;
    const double cc = (kFirst ? 0.0 : sd.y) + (dd < 0.0 ? 1.0 : 0.0);
    sd_new = make_double2(dd, cc);
    const uint64_t free_ = __ballot(cc == 0.0);
    const double th = free_ ? shift(__ffsll((unsigned long long)free_) - 1) : 0.0;
    th_cur = th;
    const double tu = fmin(th, th_prev);
    thr_new = (etol * etol) * tu;
  }
  // ---- the own rows' partials of the next launch, the lead's scalars
  double* Pn = const_cast<double*>(Pc) + (par_ ? -kPcgStreams : kPcgStreams) * (int64_t)kNs;
#pragma unroll
  for (int k = 0; k < kPcgStreams; ++k) d[k] = wave_sum(d[k]);
  if (lane == 0) { Pn[c] = d[0]; Pn[kNs + c] = d[1]; Pn[2 * kNs + c] = d[2]; Pn[3 * kNs + c] = d[3]; }
  double* sc_w = const_cast<double*>(scb);
  int32_t* flags_w = reinterpret_cast<int32_t*>(sc_w + kScFlags);
  if (lead) {
    sc_w[kScAlpha + 2 + par_] = 1.0 / alpha; sc_w[kScGamma + 2 + par_] = 1.0 / gam; flags_w[F_PCG_CNT] = cnt + 1;
    sc_w[kScAlpha + 4 + par_] = thr_new;
    if (etol > 0.0) sc_w[kScScal + S_TH_CUR] = th_cur;
  }
  if (c == 0 && etol > 0.0) reinterpret_cast<double2*>(sc_w + kScSturm)[lane] = sd_new;
  if (kFirst && lead) sc_w[kScScal + S_BB] = bb;
  OFX_AS_ITER_STAMP(6, cnt)
}

// The Schwarz warm start's w0 launch of the one-launch iteration (as_one; in place of k_pcg_w0<true, true> + the apply of
// w0): per subdomain c (the k_as_iter tables and workgroup mapping), u0 on S2 — kGather: summed from the contributions
// k_as_proj2 left in y[1] (the apply's sums, bit for bit), else the cold start's apply of b in m1 — w0 = A u0
// on every subdomain row with k_pcg_w0's products and CSR-order row sums, the own rows' records, as_w and partials exactly
// as k_pcg_w0, and the contributions y_c = D Ẑ D w0[D_c] into y[0], which the first k_as_iter sums into m0 = M⁻¹ w0 (the
// apply's segment sums, bit for bit). Roles as k_as_iter: waves 0-2 the rows (0 own), 3-7 S2 and the inverse rows, 8-15
// the (block, row) products; barriers (1) u0 on S2, (2) the products, (3) the w image.
template <bool kGather>
__global__ __launch_bounds__(kAsIterT) void k_as_w0(GnDev g, const double* rhs, int xcd_per) {   // (rhs: see k_pcg_w0)
  __shared__ __attribute__((aligned(16))) double s_m[kGS * 6];
  __shared__ __attribute__((aligned(16))) double s_prod[(kGB + kRowMax) * 6];
  __shared__ __attribute__((aligned(16))) double s_w[kAsD];
  asm volatile("" :: "s"(g.as_tab), "s"(g.as_tab_cap), "s"(g.N), "s"(g.flags), "s"(g.m1), "s"(g.Aop), "s"(g.st),
               "s"(g.stopw), "s"(g.ep), "s"(g.pcs), "s"(rhs), "s"(g.part_p), "s"(g.part_b), "s"(g.nw_pad), "s"(g.as_w));
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nwg = g.N / kCS;
  const int c = xcd_per > 0 ? (int)(blockIdx.x & 7) * xcd_per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (c >= nwg) return;
  const AsTabP tp = as_tab_at(g.as_tab, g.as_tab_cap);
  const int32_t* rt = tp.row + (int64_t)c * kGRow;
  const int stopped = g.flags[F_STOPPED];   // (the same for every wave: all leave before the first barrier)
  if (wave >= 8) {  // ---------------- (block, row) products (waves 8-15)
    const int tb = t - kGB;
    constexpr int kP = (kGB * 6 + kGB - 1) / kGB;
    int2 be[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) be[j] = tp.blk[(int64_t)c * kGB + (tb + kGB * j) / 6];
    const int nb = rt[26];
    asm volatile("" ::: "memory");
    if (stopped) return;
    const double2* A2 = reinterpret_cast<const double2*>(g.Aop);
    double2 ar[kP][3];
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if (tb - lane + kGB * j < 6 * nb)   // (wave-uniform)
#pragma unroll
        for (int k = 0; k < 3; ++k) ar[j][k] = A2[18 * (int64_t)be[j].x + 3 * ((tb + kGB * j) % 6) + k];
    as_lds_barrier();   // (1)
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const int pp = tb + kGB * j;
      if (pp < 6 * nb) {   // k_pcg_w0's operation order
        const int k = be[j].y >> 5;
        double x[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) x[q] = s_m[6 * k + q];
        const double2 b01 = ar[j][0], b23 = ar[j][1], b45 = ar[j][2];
        s_prod[pp] = ((b01.x * x[0] + b01.y * x[1]) + (b23.x * x[2] + b23.y * x[3])) + (b45.x * x[4] + b45.y * x[5]);
      }
    }
    as_lds_barrier();   // (2)
    as_lds_barrier();   // (3)
    return;
  }
  if (wave >= 3) {  // ---------------- u0 on S2, then the inverse rows (y): waves 3-7
    constexpr int kS2W = 5 * 64;
    const int ts = t - 192;
    const int k2 = ts < kGS ? ts : kGS - 1;
    int s2u = 0;
    int4 cn = make_int4(-1, -1, -1, -1);
    if (kGather) cn = tp.con[(int64_t)c * kGS + k2];
    else s2u = tp.s2n[(int64_t)c * kGS + k2];
    const int nd = rt[25], ns = rt[27];
    const int ry = min(ts >> 1, kAsD - 1), hl = ts & 1;
    asm volatile("" ::: "memory");
    if (stopped) return;
    const double* yr = tp.y + (int64_t)g.as_tab_cap * kAsD;   // (y[1])
    auto gather = [&](int4 e4, int u, double mv[6]) {
      if (kGather) {   // 0 + the contributions in ascending subdomain order (k_as_iter's sums)
        const int e[4] = {e4.x, e4.y, e4.z, e4.w};
        double2 cz[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j == 0 || e[j] >= 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) cz[j][k] = reinterpret_cast<const double2*>(yr + e[j])[k];
          } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) cz[j][k] = make_double2(0.0, 0.0);
          }
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double mx = 0.0, my = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) { mx += e[j] >= 0 ? cz[j][k].x : 0.0; my += e[j] >= 0 ? cz[j][k].y : 0.0; }
          mv[2 * k] = mx; mv[2 * k + 1] = my;
        }
      } else {
        const double2* p = reinterpret_cast<const double2*>(g.m1 + 6 * (int64_t)u);
#pragma unroll
        for (int k = 0; k < 3; ++k) { const double2 x = p[k]; mv[2 * k] = x.x; mv[2 * k + 1] = x.y; }
      }
    };
    if (ts - lane < ns) {   // (wave-uniform)
      double mv[6];
      gather(cn, s2u, mv);
      if (ts < ns)
#pragma unroll
        for (int k = 0; k < 6; ++k) s_m[6 * ts + k] = mv[k];
    }
    if (ns > kS2W)   // (rare: more than 320 distinct columns)
      for (int kk = ts + kS2W; kk < ns; kk += kS2W) {
        double mv[6];
        gather(kGather ? tp.con[(int64_t)c * kGS + kk] : make_int4(-1, -1, -1, -1),
               kGather ? 0 : tp.s2n[(int64_t)c * kGS + kk], mv);
#pragma unroll
        for (int k = 0; k < 6; ++k) s_m[6 * kk + k] = mv[k];
      }
    as_lds_barrier();   // (1)
    uint4 z[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) z[k] = tp.slab[((int64_t)c * kAsK + 9 * hl + k) * kAsD + ry];
    const float dsc_r = tp.dsc[(int64_t)c * kAsD + ry];
    as_lds_barrier();   // (2)
    as_lds_barrier();   // (3)
    // y_c = D Ẑ (D w0): k_as_iter's (k_as_apply's) segment dot times the row scale
    const double2* w2p = reinterpret_cast<const double2*>(s_w);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    auto lo = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xFFFFu)); };
    auto hi = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); };
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int kw = 9 * hl + k;
      const double2 p0 = w2p[4 * kw], p1 = w2p[4 * kw + 1], p2 = w2p[4 * kw + 2], p3 = w2p[4 * kw + 3];
      a0 = fma(lo(z[k].x), p0.x, a0);
      a1 = fma(hi(z[k].x), p0.y, a1);
      a2 = fma(lo(z[k].y), p1.x, a2);
      a3 = fma(hi(z[k].y), p1.y, a3);
      a0 = fma(lo(z[k].z), p2.x, a0);
      a1 = fma(hi(z[k].z), p2.y, a1);
      a2 = fma(lo(z[k].w), p3.x, a2);
      a3 = fma(hi(z[k].w), p3.y, a3);
    }
    double dot = (a0 + a1) + (a2 + a3);
    dot += dpp_mov<0xB1>(dot);   // the row's two halves
    if (hl == 0 && ts < 2 * kAsD && (ts >> 1) < 6 * nd)
      tp.y[(int64_t)c * kAsD + (ts >> 1)] = (double)dsc_r * dot;   // (parity 0: the first iteration's)
    return;
  }
  // ---------------- rows: wave 0 the own rows (k_pcg_w0's wave), 1-2 the ring rows (w0 for the image only)
  const int jr = wave, r = lane >> 3, q = lane & 7;
  const bool own = q < 6;
  const int qc = own ? q : 5;
  const int l = 8 * jr + r;
  const int row = c * kCS + r;
  const int64_t o = 6 * (int64_t)row + q, oc = 6 * (int64_t)row + qc;
  const int nd = rt[25];
  const int rs = rt[l], re = rt[l + 1];
  const float dsc_l = tp.dsc[(int64_t)c * kAsD + 6 * l + qc];
  const int rk = rt[32 + l];   // (the row's S2 index: its u0 in s_m)
  double v[V_N];
  double u_as = 0.0, bo = 0.0, th_cur_old = 0.0;
  if (jr == 0) {
    load_rec(g.st, oc, v);
    if (!kGather) u_as = g.m1[oc];
    bo = rhs[oc];
    th_cur_old = g.pcs[kScScal + S_TH_CUR];
  }
  asm volatile("" ::: "memory");
  if (stopped) {   // the solve already stopped: this step's iteration launches end after trip 1
    if (jr == 0) {
      g.stopw[(int64_t)c * 64 + lane] = g.ep;
      if (c == 0 && lane == 0) w0_lead_stores(g, th_cur_old, true, true);
    }
    return;
  }
  as_lds_barrier();   // (1)
  if (kGather && jr == 0) u_as = s_m[6 * rk + qc];
  as_lds_barrier();   // (2)
  const int len = l < nd ? re - rs : 0;
  const double* sp = s_prod + rs * 6 + qc;
  double tv[kRowMax];
#pragma unroll
  for (int k = 0; k < kRowMax; ++k) tv[k] = sp[6 * k];
  double w = 0.0;
#pragma unroll
  for (int k = 0; k < kRowMax; ++k) w += k < len ? tv[k] : 0.0;
  double d[4] = {0.0, 0.0, 0.0, 0.0};
  if (jr == 0 && own) {
    v[V_U] = u_as;
    v[V_W] = w;
    store_rec(g.st, o, v);
    g.as_w[o] = w;
    d[0] = v[V_R] * v[V_U]; d[1] = w * v[V_U]; d[2] = v[V_R] * v[V_R]; d[3] = bo * bo;
  }
  if (own) s_w[6 * l + q] = l < nd ? w * (double)dsc_l : 0.0;
  as_lds_barrier();   // (3)
  if (jr != 0) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = wave_sum(d[k]);
  const int ns = g.nw_pad;
  if (lane == 0) {
    g.part_p[c] = d[0]; g.part_p[ns + c] = d[1]; g.part_p[2 * ns + c] = d[2];
    g.part_p[3 * ns + c] = 0.0;   // (the direction stream: no direction before the first iteration)
    g.part_b[c] = d[3];
  }
  if (c == 0)   // zero tails of both parities' streams and of part_b
    for (int i = nwg + lane; i < ns; i += 64) {
#pragma unroll
      for (int k = 0; k < 2 * kPcgStreams; ++k) g.part_p[k * ns + i] = 0.0;
      g.part_b[i] = 0.0;
    }
  g.stopw[(int64_t)c * 64 + lane] = 0;
  if (c == 0 && lane == 0) w0_lead_stores(g, th_cur_old, true, true);
}

// The Schwarz warm start's second projection launch of the one-launch iteration (as_one, warm steps; in place of
// k_pcg_proj2<KU, true> + the apply of r0): per subdomain c, the Galerkin coefficients (wave 0, k_pcg_proj2's), x0 and
// r0 = b - Σ c_j A x_j on the own rows (their records, as k_pcg_proj2) and r0 on the ring rows (the same expression on
// the stored A x_j: no SpMV), and the contributions y_c = D Ẑ D r0[D_c] into y[1], which k_as_w0<true> sums into
// u0 = M⁻¹ r0. Waves 0-2 the rows, 3-7 the inverse rows; barriers (1) the coefficients, (2) the r0 image.
template <int KU>
__global__ __launch_bounds__(512) void k_as_proj2(GnDev g, const double* rhs, int xcd_per) {   // (rhs: see k_pcg_w0)
  __shared__ __attribute__((aligned(16))) double s_w[kAsD];
  __shared__ double s_c[kProj];
  __shared__ int s_fin;
  asm volatile("" :: "s"(g.as_tab), "s"(g.as_tab_cap), "s"(g.N), "s"(g.flags), "s"(g.n_prev), "s"(g.xh), "s"(g.th),
               "s"(g.part_p), "s"(g.nw_pad), "s"(g.stopw), "s"(g.ep), "s"(g.st), "s"(rhs));
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nwg = g.N / kCS;
  const int c = xcd_per > 0 ? (int)(blockIdx.x & 7) * xcd_per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (c >= nwg) return;
  const AsTabP tp = as_tab_at(g.as_tab, g.as_tab_cap);
  const int32_t* rt = tp.row + (int64_t)c * kGRow;
  const int stopped = g.flags[F_STOPPED];   // (the same for every wave: all leave before the first barrier)
  if (wave >= 3) {  // ---------------- the inverse rows (static: issued first), the dot after barrier 2
    const int ts = t - 192;
    const int ry = min(ts >> 1, kAsD - 1), hl = ts & 1;
    const int nd = rt[25];
    uint4 z[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) z[k] = tp.slab[((int64_t)c * kAsK + 9 * hl + k) * kAsD + ry];
    const float dsc_r = tp.dsc[(int64_t)c * kAsD + ry];
    asm volatile("" ::: "memory");
    if (stopped) return;
    as_lds_barrier();   // (1)
    as_lds_barrier();   // (2)
    const double2* w2p = reinterpret_cast<const double2*>(s_w);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    auto lo = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xFFFFu)); };
    auto hi = [](uint32_t u) { return (double)(float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); };
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int kw = 9 * hl + k;
      const double2 p0 = w2p[4 * kw], p1 = w2p[4 * kw + 1], p2 = w2p[4 * kw + 2], p3 = w2p[4 * kw + 3];
      a0 = fma(lo(z[k].x), p0.x, a0);
      a1 = fma(hi(z[k].x), p0.y, a1);
      a2 = fma(lo(z[k].y), p1.x, a2);
      a3 = fma(hi(z[k].y), p1.y, a3);
      a0 = fma(lo(z[k].z), p2.x, a0);
      a1 = fma(hi(z[k].z), p2.y, a1);
      a2 = fma(lo(z[k].w), p3.x, a2);
      a3 = fma(hi(z[k].w), p3.y, a3);
    }
    double dot = (a0 + a1) + (a2 + a3);
    dot += dpp_mov<0xB1>(dot);   // the row's two halves
    if (hl == 0 && ts < 2 * kAsD && (ts >> 1) < 6 * nd)
      tp.y[(int64_t)g.as_tab_cap * kAsD + (int64_t)c * kAsD + (ts >> 1)] = (double)dsc_r * dot;   // (y[1])
    return;
  }
  // ---------------- rows: wave 0 the own rows (k_pcg_proj2's wave), 1-2 the ring rows (r0 for the image only)
  const int jr = wave, r = lane >> 3, q = lane & 7;
  const bool own = q < 6;
  const int qc = own ? q : 5;
  const int l = 8 * jr + r;
  const int row = c * kCS + r;
  const int64_t o = 6 * (int64_t)row + q;
  const int nd = rt[25];
  const int64_t og = jr == 0 ? 6 * (int64_t)row + qc : 6 * (int64_t)rt[64 + l] + qc;   // (ring rows past nd: row 0)
  const float dsc_l = tp.dsc[(int64_t)c * kAsD + 6 * l + qc];
  const int np = g.n_prev;
  const int64_t stride = 6 * (int64_t)g.N;
  const double rb = rhs[og];
  double xo[kProj], to[kProj];
#pragma unroll
  for (int j = 0; j < kProj; ++j) { xo[j] = jr == 0 ? g.xh[j * stride + og] : 0.0; to[j] = g.th[j * stride + og]; }
  double2 pt[kProjP][KU];
  if (jr == 0) load_streams2_padded<kProjP, KU>(g.part_p, g.nw_pad, pt);
  asm volatile("" ::: "memory");
  if (stopped) {   // the solve already stopped: this step's iteration launches end after trip 1
    if (jr == 0) g.stopw[(int64_t)c * 64 + lane] = g.ep;
    return;
  }
  if (jr == 0) {
    double cj[kProj];
    const bool fin = galerkin_coeffs<KU>(g, np, pt, cj);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < kProj; ++j) s_c[j] = cj[j];
      s_fin = fin ? 1 : 0;
    }
  }
  as_lds_barrier();   // (1)
  const bool fin = s_fin != 0;
  double xv = 0.0, rv = rb;
#pragma unroll
  for (int j = 0; j < kProj; ++j)
    if (j < np && fin) { const double cj = s_c[j]; xv += cj * xo[j]; rv -= cj * to[j]; }
  if (jr == 0 && own) {
    const double v[V_N] = {xv, rv, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    store_rec(g.st, o, v);
  }
  if (own) s_w[6 * l + q] = l < nd ? rv * (double)dsc_l : 0.0;
  as_lds_barrier();   // (2)
}

// After the solve of GN step k: ill-posed check, loss bookkeeping, early stop (model.py:696-732) and,
// if accepted, the kornia 0.7.0 angle_axis_to_rotation_matrix + left-multiplicative update
// (model.py:744-748) — one launch. Every workgroup derives the same decision from read-only inputs
// (flags set by the PCG, this step's rhs tail, step_state[k]); workgroup 0 alone writes the
// bookkeeping (flags, loss log, step_state[k+1], statistics). xsave (nullable): ring slot receiving
// this step's solution for the following steps' warm start.
__global__ __launch_bounds__(256) void k_step(GnDev g, const double* __restrict__ rhs, int n_iter_log, int pcg_max,
                                              int gn_iter, double* __restrict__ xsave) {
  if (g.flags[F_STOPPED]) return;
  const double* tail = rhs + 6 * (int64_t)g.N;
  const double loss = sqrt(tail[0] + tail[1] + tail[2]);
  const double prev = g.step_state[2 * gn_iter];
  const int acc = (int)g.step_state[2 * gn_iter + 1];
  const bool ill = g.flags[F_ILL] != 0;
  const bool stop = ill || (acc > 0 && (loss - prev > g.prm.stop_loss_diff || loss == prev));
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    double bbv[1];
    sum_streams<1, 16>(g.part_b, g.nwg_row, bbv);
    if (threadIdx.x == 0) {
      const bool done = g.flags[F_DONE] != 0;
      if (!done) { g.flags[F_PCG_TOTAL] += pcg_max; g.flags[F_CAPPED] += 1; }
      if (gn_iter < kMaxLog) {
        g.stat[3 * gn_iter + 0] = done ? (double)g.flags[F_PCG_IT] : (double)pcg_max;
        g.stat[3 * gn_iter + 1] = bbv[0];
        g.stat[3 * gn_iter + 2] = loss;
      }
      g.flags[F_RES_NONFINITE] = tail[3] != 0.0 ? 1 : 0;
      if (stop) {
        g.flags[F_STOPPED] = 1;
        host_flag(g.hflags, H_STOPPED, g.ep);
      } else {
        if (acc < n_iter_log) {
          g.loss_log[4 * acc + 0] = loss;
          g.loss_log[4 * acc + 1] = sqrt(tail[0]);
          g.loss_log[4 * acc + 2] = sqrt(tail[1]);
          g.loss_log[4 * acc + 3] = sqrt(tail[2]);
        }
        g.step_state[2 * gn_iter + 2] = loss;
        g.step_state[2 * gn_iter + 3] = (double)(acc + 1);
        g.flags[F_ACCEPTED] = acc + 1;
      }
    }
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.N || stop) return;
  double x[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) x[c] = g.st[V_N * (6 * (int64_t)i + c) + V_X];
  if (xsave)
#pragma unroll
    for (int c = 0; c < 6; ++c) xsave[6 * (int64_t)i + c] = x[c];
  if (g.prm.mode == OFX_GN_ARAP && g.conf[i] != 0.0) return;   // arap: valid nodes keep R, t (model.py:1940-1943)
  double a0 = x[0], a1 = x[1], a2 = x[2];
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
  for (int c = 0; c < 3; ++c) g.t[3 * i + c] += x[3 + c];
  if (g.prm.precond_rot_tol > 0.0) {   // as fused_step
    const double acc = g.racc[i] + sqrt(a0 * a0 + a1 * a1 + a2 * a2);
    g.racc[i] = acc;
    if (acc > g.prm.precond_rot_tol) g.flags[F_REFRESH] = gn_iter + 1;
  }
}

// arap mode, lambda_flow = 0: remove each connected component's mean translation from the PCG
// solution (one wave per component, fixed-order sums). A·n = λ_LM·n for that common translation n and
// b ⊥ n, so the dense LU solution has no n component; CG barely resolves the λ_LM eigenvalue.
__global__ __launch_bounds__(64) void k_null_project(GnDev g) {
  const int c = blockIdx.x;
  const int b = g.comp_off[c], e = g.comp_off[c + 1];
  double s[3] = {0.0, 0.0, 0.0};
  for (int k = b + (int)threadIdx.x; k < e; k += 64) {
    const int64_t i = g.comp_rows[k];
#pragma unroll
    for (int q = 0; q < 3; ++q) s[q] += g.st[V_N * (6 * i + 3 + q) + V_X];
  }
  double mean[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) mean[q] = wave_sum(s[q]) / (double)(e - b);
  for (int k = b + (int)threadIdx.x; k < e; k += 64) {
    const int64_t i = g.comp_rows[k];
#pragma unroll
    for (int q = 0; q < 3; ++q) g.st[V_N * (6 * i + 3 + q) + V_X] -= mean[q];
  }
}

__global__ void k_finish(GnDev g, float* __restrict__ rot, float* __restrict__ trans, int32_t* __restrict__ status,
                         double* __restrict__ loss_out, int n_log) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = !g.flags[F_ILL] && !g.flags[F_RES_NONFINITE];
  if (i < g.N_real) {   // caller order
    const int64_t r = g.iperm[i];
    for (int c = 0; c < 9; ++c) rot[9 * i + c] = valid ? (float)g.R[9 * r + c] : ((c % 4 == 0) ? 1.f : 0.f);
    for (int c = 0; c < 3; ++c) trans[3 * i + c] = valid ? (float)g.t[3 * r + c] : 0.f;
  }
  if (i == 0 && status) {
    status[0] = valid ? 1 : 0;
    status[1] = g.flags[F_ACCEPTED];
    status[2] = g.flags[F_PCG_TOTAL];
    status[3] = g.flags[F_ILL];
    status[4] = g.flags[F_CAPPED];
  }
  if (loss_out && i < 4 * n_log) loss_out[i] = (i / 4 < g.flags[F_ACCEPTED]) ? g.loss_log[i] : 0.0;
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
                  g->term_node, g->J, g->res, g->map, g->row_ptr, g->col, g->blk_row, g->row_cnt, g->wl, g->Aw, g->stopw, g->blk_off, g->blk_cnt,
                  g->blk_list, g->blk_tmp, g->node_tmp, g->node_off, g->node_cnt, g->node_list, g->blk_first, g->node_first, g->R, g->t, g->A_own, g->rhs_own, g->Mcl,
                  g->st, g->m0, g->m1, g->pcs, g->racc,
                  g->part_p, g->part_b, g->part_loss,
                  g->loss_log, g->stat, g->step_state, g->xh, g->th, g->step_args, g->d_gnodes, g->d_gedges, g->d_gdiff, g->perm, g->iperm, g->comp_rows, g->comp_off,
                  g->up_of, g->up_slot, g->up_tr, g->as_cand, g->as_csc, g->as_acc, g->as_dom, g->as_meta, g->as_gat,
                  g->as_dst, g->as_slab, g->as_w, g->as_src, g->as_dsc, g->as_rsc, g->as_tab, g->as_mem, g->as_memn};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (g->host_flags) (void)hipHostFree(g->host_flags);
  if (g->setup_stat) (void)hipHostFree(g->setup_stat);
  if (g->poll_ev) (void)hipEventDestroy(g->poll_ev);
  if (g->d_pcgit) (void)hipFree(g->d_pcgit);
}

// Row order for the cluster preconditioner (host, from the ED graph). Clusters: the lowest
// unassigned node seeds a cluster that grows breadth-first over graph edges, candidates of each
// visited node taken nearest-to-seed first, up to kCS members. Groups: clusters first-fit packed by
// decreasing size into groups of kCS rows, unused rows are padding (-1). perm[row] = node.
static void order_rows(int N, int NB, const float* nodes, const int32_t* edges, std::vector<int32_t>& perm) {
  std::vector<int32_t> lab(N, -1), members;
  std::vector<int32_t> c_off{0};
  std::vector<int32_t> front, cand;
  for (int s0 = 0; s0 < N; ++s0) {
    if (lab[s0] >= 0) continue;
    const int c = (int)c_off.size() - 1;
    const size_t first = members.size();
    lab[s0] = c;
    members.push_back(s0);
    front.assign(1, s0);
    const float* ps = nodes + 3 * (int64_t)s0;
    auto d2 = [&](int j) {
      const float* pj = nodes + 3 * (int64_t)j;
      const double a = (double)pj[0] - ps[0], b = (double)pj[1] - ps[1], e = (double)pj[2] - ps[2];
      return a * a + b * b + e * e;
    };
    for (size_t f = 0; f < front.size() && members.size() - first < (size_t)kCS; ++f) {
      const int cur = front[f];
      cand.clear();
      for (int k = 0; k < NB; ++k) {
        const int j = edges[(int64_t)cur * NB + k];
        if (j >= 0 && j < N && lab[j] < 0 && std::find(cand.begin(), cand.end(), j) == cand.end()) cand.push_back(j);
      }
      std::sort(cand.begin(), cand.end(), [&](int a, int b) {
        const double da = d2(a), db = d2(b);
        return da < db || (da == db && a < b);
      });
      for (int j : cand) {
        if (members.size() - first >= (size_t)kCS) break;
        lab[j] = c;
        members.push_back(j);
        front.push_back(j);
      }
    }
    c_off.push_back((int32_t)members.size());
  }
  const int nc = (int)c_off.size() - 1;
  std::vector<int32_t> order(nc);
  for (int c = 0; c < nc; ++c) order[c] = c;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return c_off[a + 1] - c_off[a] > c_off[b + 1] - c_off[b]; });
  std::vector<int32_t> fill;                       // per group
  std::vector<std::vector<int32_t>> grp;
  for (int c : order) {
    const int sz = c_off[c + 1] - c_off[c];
    size_t k = 0;
    while (k < fill.size() && fill[k] + sz > kCS) ++k;
    if (k == fill.size()) { fill.push_back(0); grp.emplace_back(); }
    fill[k] += sz;
    grp[k].push_back(c);
  }
  perm.assign(grp.size() * kCS, -1);
  for (size_t k = 0; k < grp.size(); ++k) {
    int r = (int)k * kCS;
    for (int c : grp[k])
      for (int m = c_off[c]; m < c_off[c + 1]; ++m) perm[r++] = members[m];
  }
}

// Partial pairs per lane and stream of k_pcg_iter for a cluster (wave) count: the streams are 2·64·kU wide, so
// fewer loads and adds per lane for fewer clusters (2: <= 256, 3: <= 384, 4: <= 512, 8: <= 1024, 17: <= 2176
// clusters; kU = 2 for config 3's 250 clusters: -0.031 ms per frame against 3, same frames, profiles/r04_ab.json).
// OFX_PCG_KU=<2|3|4|8|17> forces one (A/B, read per setup; it must still cover the count).
static int pcg_ku_for(int waves) {
  int ku = waves <= 256 ? 2 : waves <= 384 ? 3 : waves <= 512 ? 4 : waves <= 1024 ? 8 : 17;
  if (const char* e = getenv("OFX_PCG_KU")) {
    const int f = atoi(e);
    if ((f == 2 || f == 3 || f == 4 || f == 8 || f == 17) && 128 * f >= waves) ku = f;
  }
  return ku;
}

using PcgKernel = void (*)(const int2*, const int32_t*, const double*, const double*, const double*, const double*,
                          const PcgIt*, int, int, int);
template <int KU>
static void pcg_pick(bool wave, bool w2, bool as, PcgKernel& first, PcgKernel& rest) {
  if (as) {   // (wave-list forms only)
    if constexpr (KU <= 3) {
      if (w2) {
        first = k_pcg_iter<true, true, KU, true, true>;
        rest = k_pcg_iter<true, false, KU, true, true>;
        return;
      }
    }
    first = k_pcg_iter<true, true, KU, false, true>;
    rest = k_pcg_iter<true, false, KU, false, true>;
    return;
  }
  if constexpr (KU <= 3) {
    if (wave && w2) {
      first = k_pcg_iter<true, true, KU, true>;
      rest = k_pcg_iter<true, false, KU, true>;
      return;
    }
  }
  if (wave) {
    first = k_pcg_iter<true, true, KU, false>;
    rest = k_pcg_iter<true, false, KU, false>;
  } else {
    first = k_pcg_iter<false, true, KU, false>;
    rest = k_pcg_iter<false, false, KU, false>;
  }
}

static int gn_pcg(Gn* g, int gn_iter, double* A, double* rhs, hipStream_t hs) {
  double lm = lm_for_iter(g->prm.lm_factor, gn_iter);
  g->ep = g->ep_next++;   // this solve's epoch (read by the launches below through their GnDev / PcgIt copies)
  g->gn_iter_now = gn_iter;
  g->warm_now = 0;
  if (g->prm.pcg_warm && gn_iter > 0) {   // k_step of the previous steps filled the ring
    g->n_prev = gn_iter < kProj ? gn_iter : kProj;
    g->warm_now = 1;
  }
  g->Aop = A;
  // the cluster inverse is rebuilt every precond_every GN steps; steps in between (always warm started,
  // proj2 applies the stored M⁻¹) only damp A's diagonal
  const int every = g->prm.precond_every > 1 ? g->prm.precond_every : 1;
  const int invert = (!g->warm_now || gn_iter % every == 0) ? 1 : 0;
  // wave-list SpMV forms (k_pcg_proj, k_pcg_w0, k_pcg_iter) when every wave's blocks fit the list and every row kRowMax
  const bool wave = g->max_wave <= kWL && g->max_deg <= kRowMax;
  const bool as = g->as_on != 0;   // (the setup enables it only with the wave-list forms)
  const int ncl = g->N / kCS;
  auto as_apply = [&](bool test, const double* in, double* out) {
    auto k = g->as_lanes == 1 ? (test ? k_as_apply<true, 1> : k_as_apply<false, 1>)
           : g->as_lanes == 4 ? (test ? k_as_apply<true, 4> : k_as_apply<false, 4>)
                              : (test ? k_as_apply<true, 2> : k_as_apply<false, 2>);
    hipLaunchKernelGGL(k, dim3(ncl), dim3(g->as_lanes * kAsRS), 0, hs, (const int32_t*)g->stopw, (const int32_t*)g->as_meta,
                       (const int32_t*)g->as_gat, (const uint16_t*)g->as_slab, in, out, (const int32_t*)g->as_src,
                       (const float*)g->as_dsc, (const float*)g->as_rsc);
  };
  if (as) {
    // the subdomain inverses: rebuilt like the cluster inverses (invert); a refresh flagged by the previous step runs
    // inside k_pcg_proj<.., true>
    if (invert) {
      const char* me = getenv("OFX_AS_INV_MFMA");   // (A/B; read per solve): 1 = the MFMA form
      const bool mf = me && atoi(me) == 1;
      hipLaunchKernelGGL(mf ? k_as_invert<true> : k_as_invert<false>, dim3(ncl), dim3(mf ? kInvT : 16 * kAsInvTC), 0,
                         hs, *g, (const double*)A, (const double*)rhs);
    }
    if (!g->warm_now) as_apply(false, rhs, g->m1);   // cold start: u0 = M⁻¹ b
  } else if (invert) {
    hipLaunchKernelGGL(k_pcg_prep, dim3(g->N / kCS), dim3(64), 0, hs, *g, lm, A, (const double*)rhs, invert);
  }
  // the one-launch iteration's workgroups: XCD-contiguous cluster runs (OFX_AS_XCD=0: workgroup = cluster; A/B, read per
  // solve), XCD x running clusters [x·xcd_per, (x+1)·xcd_per)
  const bool one = as && g->as_one;
  int xcd_per = 0, one_grid = ncl;
  if (one) {
    const char* xe = getenv("OFX_AS_XCD");
    xcd_per = (xe && atoi(xe) == 0) ? 0 : (ncl + 7) / 8;
    one_grid = xcd_per > 0 ? 8 * xcd_per : ncl;
  }
  if (g->warm_now) {
    if (as) hipLaunchKernelGGL((k_pcg_proj<true, true>), dim3(g->nwg_row), dim3(256), 0, hs, *g, (const double*)rhs, gn_iter);
    else if (wave) hipLaunchKernelGGL(k_pcg_proj<true>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs, gn_iter);
    else hipLaunchKernelGGL(k_pcg_proj<false>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs, gn_iter);
    if (one) {   // x0, r0 and the contributions of u0 = M⁻¹ r0 in one launch (k_as_proj2)
      switch (g->pcg_ku) {
        case 2: hipLaunchKernelGGL(k_as_proj2<2>, dim3(one_grid), dim3(512), 0, hs, *g, (const double*)rhs, xcd_per); break;
        case 3: hipLaunchKernelGGL(k_as_proj2<3>, dim3(one_grid), dim3(512), 0, hs, *g, (const double*)rhs, xcd_per); break;
        default: hipLaunchKernelGGL(k_as_proj2<4>, dim3(one_grid), dim3(512), 0, hs, *g, (const double*)rhs, xcd_per); break;
      }
    } else switch (g->pcg_ku) {
      case 2: if (as) hipLaunchKernelGGL((k_pcg_proj2<2, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
              else hipLaunchKernelGGL(k_pcg_proj2<2>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs); break;
      case 3: if (as) hipLaunchKernelGGL((k_pcg_proj2<3, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
              else hipLaunchKernelGGL(k_pcg_proj2<3>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs); break;
      case 4: if (as) hipLaunchKernelGGL((k_pcg_proj2<4, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
              else hipLaunchKernelGGL(k_pcg_proj2<4>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs); break;
      case 8: if (as) hipLaunchKernelGGL((k_pcg_proj2<8, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
              else hipLaunchKernelGGL(k_pcg_proj2<8>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs); break;
      default: if (as) hipLaunchKernelGGL((k_pcg_proj2<17, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
               else hipLaunchKernelGGL(k_pcg_proj2<17>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs); break;
    }
    if (as && !one) as_apply(false, g->as_w, g->m1);   // u0 = M⁻¹ r0
  }
  if (one) {   // w0 = A u0 and the contributions of m0 = M⁻¹ w0 in one launch (k_as_w0; u0 from k_as_proj2's contributions)
    if (g->warm_now) hipLaunchKernelGGL(k_as_w0<true>, dim3(one_grid), dim3(kAsIterT), 0, hs, *g, (const double*)rhs, xcd_per);
    else hipLaunchKernelGGL(k_as_w0<false>, dim3(one_grid), dim3(kAsIterT), 0, hs, *g, (const double*)rhs, xcd_per);
  } else {
    if (as) hipLaunchKernelGGL((k_pcg_w0<true, true>), dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
    else if (wave) hipLaunchKernelGGL(k_pcg_w0<true>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
    else hipLaunchKernelGGL(k_pcg_w0<false>, dim3(g->nwg_row), dim3(64), 0, hs, *g, (const double*)rhs);
    if (as) as_apply(false, g->as_w, g->m0);     // m0 = M⁻¹ w0
  }
  OFX_LAUNCH_CHECK();
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g->timing) {
    OFX_HIP(hipEventCreate(&e0));
    OFX_HIP(hipEventCreate(&e1));
    OFX_HIP(hipEventRecord(e0, hs));
  }
  // Chunks of launches, flags polled between chunks. Launch i tests convergence of the state after
  // i iterations, and launches after convergence end after one scalar load, so the first chunk
  // covers the previous frame's count for this GN step plus a small margin. (A hipGraph replay of
  // parity-pair chunks was measured: no gain over plain launches for this kernel.)
  const int max_it = g->prm.pcg_max_iter;
  Gn::PcgHist& ph = *g->last_pcg;
  const int hk = gn_iter & 63;
  const int lp = ph.n[hk] > 0 ? ph.c[hk][(ph.n[hk] - 1) & 3] : 0;   // the previous solve's count for this GN step
  // Chunk rule (round 4, `profiles/r04_ab.json`): an under-estimate (the smallest of the last 3 counts) with top-ups of
  // 3-4 launches and a poll event 3 launches ahead of each chunk's end cut the drained launches from ~100 to ~30-55 per
  // frame but never the frame time (+0.02 ... +0.33 ms): the drains overlap the host's reaction to convergence, while
  // every top-up risks an empty queue. The first chunk stays the previous count + 4, and 8 more when one runs out.
  const dim3 grid(g->nwg_row), block(64);
  // variants: wave-list SpMV (short rows) or CSR rows; partial-sum width kU for the cluster count (pcg_ku_for);
  // two waves per cluster only up to 384 clusters (kU = 3): config 4's 490 clusters ran 5.38 us per launch
  // with one wave and kU = 4, 5.58 with two; kU = 8: 5.66 vs 5.91; kU = 17: 6.35 vs 6.93 (A/B, 1278.9
  // iterations per frame; one wave per cluster and kU = 17 was the round-1 form for > 384 clusters: 95 vs 111
  // frames/s)
  const bool w2 = wave && g->pcg_w2 && g->pcg_ku <= 3;
  PcgKernel iter0 = nullptr, iter = nullptr;
  switch (g->pcg_ku) {
    case 2: pcg_pick<2>(wave, w2, as, iter0, iter); break;
    case 3: pcg_pick<3>(wave, w2, as, iter0, iter); break;
    case 4: pcg_pick<4>(wave, w2, as, iter0, iter); break;
    case 8: pcg_pick<8>(wave, w2, as, iter0, iter); break;
    default: pcg_pick<17>(wave, w2, as, iter0, iter); break;
  }
  const dim3 block_it(w2 ? 128 : 64);
  // one launch per Schwarz iteration (k_as_iter; the setup built its tables)
  // (the arguments up to ep fill the 14 preloaded SGPRs: the workgroup's cluster test and trip 1 wait for no kernarg fetch)
  using AsIterKernel = void (*)(const int32_t*, const double*, const double*, const double*, const char*, int, int, int,
                                int, const PcgIt*, int);
  AsIterKernel one0 = nullptr, one1 = nullptr;
  if (one) {
    // the block loads: a thread per (block, row) (default) or per block (OFX_AS_ROWSPLIT=0; A/B, read per solve)
    const char* rse = getenv("OFX_AS_ROWSPLIT");
    const bool rsp = !(rse && atoi(rse) == 0);
    switch (g->pcg_ku) {
      case 2: if (rsp) { one0 = k_as_iter<true, 2, true>; one1 = k_as_iter<false, 2, true>; }
              else { one0 = k_as_iter<true, 2, false>; one1 = k_as_iter<false, 2, false>; } break;
      case 3: if (rsp) { one0 = k_as_iter<true, 3, true>; one1 = k_as_iter<false, 3, true>; }
              else { one0 = k_as_iter<true, 3, false>; one1 = k_as_iter<false, 3, false>; } break;
      default: if (rsp) { one0 = k_as_iter<true, 4, true>; one1 = k_as_iter<false, 4, true>; }
               else { one0 = k_as_iter<true, 4, false>; one1 = k_as_iter<false, 4, false>; } break;
    }
  }
  // No stream sync: the converging launch stores H_DONE straight into host memory and the host
  // spins on it, so the next GN step is enqueued while the chunk's remaining (no-op) launches drain.
  // The chunk event only tells "all launched iterations ran without converging" -> launch more. (Measured
  // and dropped: a first chunk of exactly the previous count, topped up by 4 from a marker event 3 launches
  // before each chunk's end — 690.5 instead of 694.3 launches per frame, but 5.15 instead of 5.06-5.12 us per
  // launch with the marker in the stream: -0.5 %, A/B x3.)
  volatile int32_t* hf = g->host_flags;
  PcgIt pa = pcg_args(g);
  // the converging launch also takes the GN step (not when arap's null-space projection must run first)
  pa.fuse = g->n_comp == 0 ? 1 : 0;
  pa.tail = rhs + 6 * (int64_t)g->N;
  pa.ep = 0;   // (the epoch and the GN step go by value with each launch)
  // the device copy of the constant arguments: rewritten only when they change (a setup, another A / rhs)
  static_assert(sizeof(PcgIt) <= sizeof(g->pcgit_last), "PcgIt staging");
  if (!g->pcgit_valid || memcmp(&pa, g->pcgit_last, sizeof(PcgIt)) != 0) {
    OFX_HIP(hipMemcpyAsync(g->d_pcgit, &pa, sizeof(PcgIt), hipMemcpyHostToDevice, hs));   // (pageable: staged at the call)
    memcpy(g->pcgit_last, &pa, sizeof(PcgIt));
    g->pcgit_valid = true;
  }
  const PcgIt* gp = static_cast<const PcgIt*>(g->d_pcgit);
  g->step_fused = false;
  int chunk = lp > 0 ? lp + 4 : 64;
  // Later GN steps: the previous frame's count for this step scaled by how this frame's step 0 compared with the
  // previous frame's (the steps' counts move together frame to frame) + a margin (OFX_PCG_RATIO=<margin>, default 2;
  // "off": the previous count + 4; read per solve, A/B). tools/chunk_sim.py on recorded counts: 89 -> 55 drained
  // launches per frame at the same number of top-ups.
  const char* re = getenv("OFX_PCG_RATIO");
  const bool ratio_on = !(re && strcmp(re, "off") == 0);
  const int ratio_margin = (re && ratio_on) ? atoi(re) : 2;
  if (ratio_on && hk > 0 && lp > 0 && ph.n[0] >= 2) {
    const int c0 = ph.c[0][(ph.n[0] - 1) & 3], c0p = ph.c[0][(ph.n[0] - 2) & 3];
    if (c0 > 0 && c0p > 0) {
      const double ratio = std::min(2.0, std::max(0.5, (double)c0 / (double)c0p));
      chunk = std::max(4, (int)std::lround(lp * ratio) + ratio_margin);
    }
  }
  // iterations per top-up after a chunk ran out (OFX_PCG_TOPUP=<n>, A/B; read per solve): 8 for the cluster blocks, 4 for
  // Schwarz (two launches each: 472 -> 458 launches per frame, 360 / 344 -> 378 / 361 frames/s; 2 with a margin of 1:
  // 442 launches but 4.0 us each, slower; profiles/r05_ab.json)
  const char* te = getenv("OFX_PCG_TOPUP");
  const int topup = te && atoi(te) > 0 ? atoi(te) : (as ? 4 : 8);
  int it = 0;
  while (it < max_it) {
    const int n = chunk < max_it - it ? chunk : max_it - it;
#ifdef OFX_STAMPS
    const auto h0 = std::chrono::steady_clock::now();
    if (it == 0 && gn_iter > 0 && g->t_seen.time_since_epoch().count())
      g->prologue_us += std::chrono::duration<double, std::micro>(h0 - g->t_seen).count();
#endif
    if (one) {   // one launch per iteration (k_as_iter)
      for (int k = 0; k < n; ++k, ++it) {
        const int par = it & 1;
        hipLaunchKernelGGL(it == 0 ? one0 : one1, dim3(one_grid), dim3(kAsIterT), 0, hs, (const int32_t*)g->stopw,
                           (const double*)(g->part_p + kPcgStreams * (int64_t)g->nw_pad * par), (const double*)g->st,
                           (const double*)g->pcs + par, (const char*)g->as_tab, g->as_tab_cap, xcd_per, ncl, g->ep, gp,
                           gn_iter);
      }
    } else {
      for (int k = 0; k < n; ++k, ++it) {
        const int par = it & 1;
        hipLaunchKernelGGL(it == 0 ? iter0 : iter, grid, block_it, 0, hs, (const int2*)g->wl, (const int32_t*)g->stopw,
                           (const double*)(g->part_p + kPcgStreams * (int64_t)g->nw_pad * par), (const double*)g->st,
                           (const double*)(par ? g->m1 : g->m0), (const double*)g->pcs + par, gp, par, g->ep,
                           gn_iter);
        if (as) as_apply(true, g->as_w, par ? g->m0 : g->m1);   // m of the next iteration = M⁻¹ w_new
      }
    }
#ifdef OFX_STAMPS
    g->host_enqueue_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
    g->host_enqueued += n;
#endif
    OFX_LAUNCH_CHECK();
    if (g->timing) OFX_HIP(hipEventRecord(e1, hs));
    OFX_HIP(hipEventRecord(g->poll_ev, hs));
    bool ran = false;
    if (g->idle_fn) {   // (ofx_gn_set_idle_hook: the host would only spin here)
      void (*fn)(void*) = g->idle_fn;
      void* arg = g->idle_arg;
      g->idle_fn = nullptr;
      g->idle_arg = nullptr;
      fn(arg);
    }
    // converged: the converging launch's lead lane stored H_DONE (the next step's kernels follow it on the stream);
    // stopped (by an earlier solve: this one's launches end at their stop words; by this solve's converging launch):
    // nothing to wait for
    for (int spin = 0; hf[H_DONE] < g->ep && !hf[H_STOPPED]; ++spin) {
      if ((spin & 63) == 63) {
        const hipError_t q = hipEventQuery(g->poll_ev);
        if (q == hipSuccess) { ran = true; break; }
        if (q != hipErrorNotReady) OFX_HIP(q);
      }
    }
    if (hf[H_STOPPED]) break;
    if (hf[H_DONE] >= g->ep) {
#ifdef OFX_STAMPS
      g->t_seen = std::chrono::steady_clock::now();
#endif
      ph.c[hk][ph.n[hk] & 3] = hf[H_PCG_IT];
      ++ph.n[hk];
      g->step_fused = pa.fuse != 0;
      break;
    }
    (void)ran;   // the chunk ran out without convergence: next chunk
    chunk = topup;
  }
  g->n_iter_launches += (as && !one) ? 2 * it : it;   // (two-launch Schwarz: each iteration is two launches)
  if (g->timing) g->ev.emplace_back(e0, e1);
#ifdef OFX_STAMPS
  if (getenv("OFX_GAP_EVENTS")) {
    OFX_HIP(hipEventCreate(&g->gap_end));
    OFX_HIP(hipEventRecord(g->gap_end, hs));
  }
#endif
  return OFX_OK;
}

static int gn_setup(Gn* g, const ofx_gn_problem* pb, const ofx_gn_params* prm, int64_t* nnz_blocks, ofx_stream_t s);

// the prefetch worker of this handle has finished enqueuing the queued setup (its status is in prep_status)
static void open_gate(Gn* g) {
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->gate) return;
    g->gate = false;
  }
  g->cv.notify_all();
}

static void prep_wait(Gn* g) {
  if (!g->worker.joinable()) return;
  open_gate(g);   // a gated prefetch not triggered yet starts now
  std::unique_lock<std::mutex> lk(g->mu);
  g->cv.wait(lk, [g] { return !g->job; });
}

// Unlink a gated prefetch's trigger pair (either side): at destroy, and when a new prefetch replaces the link.
static void pf_unlink(Gn* g) {
  if (g->pf_peer) {
    g->pf_peer->pf_trigger = nullptr;
    g->pf_peer = nullptr;
  }
  if (g->pf_trigger) {
    g->pf_trigger->pf_peer = nullptr;
    g->pf_trigger = nullptr;
  }
}

// The solve on `g` reached GN step `it` (or returns: it < 0): start the prefetch it gates.
static void pf_fire(Gn* g, int it) {
  Gn* p = g->pf_peer;
  if (!p || (it >= 0 && it < g->pf_step)) return;
  pf_unlink(g);
  open_gate(p);
}

static void prep_worker(Gn* g) {
  std::unique_lock<std::mutex> lk(g->mu);
  for (;;) {
    g->cv.wait(lk, [g] { return (g->job && !g->gate) || g->quit; });
    if (g->quit) return;
    lk.unlock();
    int r = (hipSetDevice(g->prep_dev) == hipSuccess && hipStreamWaitEvent(g->side, g->ev_in, 0) == hipSuccess)
                ? OFX_OK : OFX_ERR_HIP;
    if (r == OFX_OK) r = gn_setup(g, &g->prep_pb, &g->prep_prm, nullptr, (ofx_stream_t)g->side);
    if (r == OFX_OK && hipEventRecord(g->ev_prep, g->side) != hipSuccess) r = OFX_ERR_HIP;
    lk.lock();
    g->prep_status = r;
    g->job = false;
    g->cv.notify_all();
  }
}

static bool same_problem(const ofx_gn_problem& a, const ofx_gn_problem& b) {   // all but the pose
  return a.n_nodes == b.n_nodes && a.n_matches == b.n_matches && a.n_neighbors == b.n_neighbors &&
         a.nodes == b.nodes && a.edges == b.edges && a.edge_weights == b.edge_weights &&
         a.target_node_pos == b.target_node_pos && a.node_conf == b.node_conf && a.src == b.src &&
         a.anchors == b.anchors && a.weights == b.weights && a.tgt == b.tgt && a.target_px == b.target_px &&
         a.target_py == b.target_py && a.fx == b.fx && a.fy == b.fy && a.cx == b.cx && a.cy == b.cy;
}

static bool same_params(const ofx_gn_params& a, const ofx_gn_params& b) {
  return a.num_iter == b.num_iter && a.use_edge_weighting == b.use_edge_weighting &&
         a.pcg_max_iter == b.pcg_max_iter && a.pcg_warm == b.pcg_warm && a.lambda_flow == b.lambda_flow &&
         a.lambda_depth == b.lambda_depth && a.lambda_arap == b.lambda_arap && a.lambda_motion == b.lambda_motion &&
         a.lm_factor == b.lm_factor && a.stop_loss_diff == b.stop_loss_diff && a.pcg_tol == b.pcg_tol &&
         a.mode == b.mode && a.precond_every == b.precond_every && a.pcg_err_tol == b.pcg_err_tol &&
         a.precond_rot_tol == b.precond_rot_tol && a.precond == b.precond;
}

}  // namespace ofx

using namespace ofx;

extern "C" {

int ofx_gn_create(int32_t max_nodes, int32_t max_matches, void** handle) {
  OFX_CHECK_ARG(handle && max_nodes > 0 && max_matches >= 0, "bad gn_create args");
  if (max_nodes > kMaxNodes) {
    set_error("max_nodes %d > %d (dense slot map over the padded rows)", max_nodes, kMaxNodes);
    return OFX_ERR_RANGE;
  }
  Gn* g = new Gn();
  {   // tuning / A-B: OFX_PCG_W1=1 (any value but "0" / empty) selects one wave per cluster
    const char* e = getenv("OFX_PCG_W1");
    g->pcg_w2 = (e && e[0] && strcmp(e, "0") != 0) ? 0 : 1;
    const char* pe = getenv("OFX_PRECOND");   // A/B override of params.precond: "as" = Schwarz, "bj" = cluster blocks
    g->as_env = (pe && strcmp(pe, "as") == 0) ? 1 : (pe && strcmp(pe, "bj") == 0) ? 0 : -1;
    // lanes per Schwarz segment in k_as_apply (OFX_AS_LANES=1|2|4, A/B): 2 (16-row rings: 410 / 432 / 412 against
    // 387 / 390 / 372 frames/s with one, one box; with 12-row rings one and two were within noise)
    const char* le = getenv("OFX_AS_LANES");
    const int lv = le ? atoi(le) : 2;
    g->as_lanes = (lv == 1 || lv == 4) ? lv : 2;
  }
  g->max_nodes = max_nodes;
  g->max_matches = max_matches;
  // rows: clusters of <= kCS first-fit packed into groups of kCS; at most one group is at most half
  // full, so rows <= 2·nodes + kCS
  g->max_pad = 2 * max_nodes + kCS;
  int64_t N = g->max_pad, M = max_matches > 0 ? max_matches : 1;
#define ALLOC(ptr, n) \
  if (hipMalloc((void**)&(ptr), (size_t)(n) * sizeof(*(ptr))) != hipSuccess) { free_all(g); delete g; set_error("hipMalloc failed"); return OFX_ERR_ALLOC; }
  ALLOC(g->nodes, 3 * N); ALLOC(g->tpos, 3 * N); ALLOC(g->conf, N);
  ALLOC(g->src, 3 * M); ALLOC(g->wts, 4 * M); ALLOC(g->tgt, 3 * M); ALLOC(g->tpx, M); ALLOC(g->tpy, M);
  ALLOC(g->anc, 4 * M);
  ALLOC(g->map, N * N); ALLOC(g->row_ptr, N + 1); ALLOC(g->row_cnt, N + 2);
  ALLOC(g->node_off, N + 1); ALLOC(g->node_cnt, N + 1); ALLOC(g->node_first, N * 128);
  ALLOC(g->R, 9 * N); ALLOC(g->t, 3 * N); ALLOC(g->racc, N);
  ALLOC(g->Mcl, 6 * N * kCD); ALLOC(g->st, V_N * 6 * N); ALLOC(g->m0, 6 * N); ALLOC(g->m1, 6 * N);
  ALLOC(g->xh, kProj * 6 * N); ALLOC(g->th, kProj * 6 * N); ALLOC(g->step_args, 1);
  ALLOC(g->perm, N); ALLOC(g->iperm, max_nodes); ALLOC(g->wl, N / kCS * kWL); ALLOC(g->Aw, N / kCS * kWL * 36);
  ALLOC(g->stopw, N / kCS * 64);
  const int64_t max_row_wg = ((N + kRW - 1) / kRW + 1) & ~1;
  const int64_t max_ns = 128 * 17;   // nw_pad bound: 2·64·17 >= max_pad / kCS waves
  static_assert(2 * 64 * 17 * kCS >= 2 * kMaxNodes + kCS, "partial stream width");
  static_assert(kProjP >= 2 * kPcgStreams, "part_p: kProjP projection streams / 2 x 4 iteration streams, stride nw_pad");
  (void)max_row_wg;
  ALLOC(g->part_p, kProjP * max_ns); ALLOC(g->part_b, max_ns);
  static_assert(S_COUNT <= kScSturm - kScScal && 2 * kScFlags + F_COUNT <= 2 * kScAop && kScAop < kScSize,
                "scalar block layout");
  ALLOC(g->pcs, kScSize);
  g->pcg_alpha = g->pcs + kScAlpha; g->pcg_gamma = g->pcs + kScGamma; g->scal = g->pcs + kScScal;
  g->sturm = reinterpret_cast<double2*>(g->pcs + kScSturm); g->flags = reinterpret_cast<int32_t*>(g->pcs + kScFlags);
  ALLOC(g->loss_log, 4 * 64); ALLOC(g->stat, 3 * kMaxLog); ALLOC(g->step_state, 2 * (kMaxLog + 1)); ALLOC(g->rhs_own, 6 * N + 4);
#undef ALLOC
  if (hipMalloc(&g->d_pcgit, sizeof(g->pcgit_last)) != hipSuccess) {
    free_all(g); delete g; set_error("hipMalloc failed"); return OFX_ERR_ALLOC;
  }
  if (hipMemset(g->map, 0, (size_t)N * N * sizeof(int32_t)) != hipSuccess ||   // pattern entries are cleared per setup
      hipMemset(g->stopw, 0, (size_t)(N / kCS) * 64 * sizeof(int32_t)) != hipSuccess) {   // epoch 0: none converged
    free_all(g); delete g; set_error("hipMemset failed"); return OFX_ERR_HIP;
  }
  if (hipHostMalloc((void**)&g->host_flags, H_COUNT * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&g->hflags, g->host_flags, 0) != hipSuccess ||
      hipHostMalloc((void**)&g->setup_stat, 8 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&g->d_setup_stat, g->setup_stat, 0) != hipSuccess ||
      hipEventCreateWithFlags(&g->poll_ev, hipEventDisableTiming) != hipSuccess) {
    free_all(g); delete g; set_error("hipHostMalloc failed"); return OFX_ERR_ALLOC;
  }
  {   // the fused GN step's fixed pointers (fused_step), in device memory
    const StepArgs h{g->R, g->t, g->xh, g->stat, g->loss_log, g->step_state, g->conf, g->racc};
    if (hipMemcpy(g->step_args, &h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) {
      free_all(g); delete g; set_error("hipMemcpy failed"); return OFX_ERR_HIP;
    }
  }

  *handle = g;
  return OFX_OK;
}

int ofx_gn_timing(void* handle, int32_t enable, double* pcg_ms, int64_t* iter_launches, int64_t* n_solves) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g, "null handle");
  double ms = 0.0;
  for (auto& e : g->ev) {
    float t = 0.f;
    OFX_HIP(hipEventSynchronize(e.second));
    OFX_HIP(hipEventElapsedTime(&t, e.first, e.second));
    ms += t;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (pcg_ms) *pcg_ms = ms;
  if (iter_launches) *iter_launches = g->n_iter_launches;
  if (n_solves) *n_solves = (int64_t)g->ev.size();
  g->ev.clear();
  g->n_iter_launches = 0;
  g->timing = enable != 0;
  return OFX_OK;
}

int ofx_gn_info(void* handle, int64_t* info) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && info, "null handle/info");
  info[0] = g->N_real; info[1] = g->M; info[2] = g->nnzb; info[3] = g->T; info[4] = g->N;
  return OFX_OK;
}

int ofx_gn_precond_info(void* handle, int64_t* info) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);
  OFX_CHECK_ARG(g && info, "null handle/info");
  for (int k = 0; k < 8; ++k) info[k] = 0;
  info[0] = g->as_on;
  info[6] = kAsD;
  info[7] = (g->as_on && !g->as_one) ? 2 : 1;
  if (!g->as_on) return OFX_OK;
  const int ncl = g->N / kCS;
  const int sd = sync_side(g);
  if (sd) return sd;
  OFX_HIP(hipDeviceSynchronize());
  std::vector<int32_t> meta((size_t)ncl * kAsMeta), gat((size_t)ncl * kAsGat), dom((size_t)ncl * kAsDN);
  OFX_HIP(hipMemcpy(meta.data(), g->as_meta, meta.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  OFX_HIP(hipMemcpy(gat.data(), g->as_gat, gat.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  OFX_HIP(hipMemcpy(dom.data(), g->as_dom, dom.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  int64_t segs = 0, srcs = 0, rows = 0, drows = 0;
  for (int c = 0; c < ncl; ++c) {
    segs += meta[(size_t)c * kAsMeta];
    srcs += meta[(size_t)c * kAsMeta + 1];
    for (int i = 0; i < kAsGat; ++i) rows += gat[(size_t)c * kAsGat + i] >= 0 ? 1 : 0;
    for (int l = 0; l < kAsDN; ++l) drows += dom[(size_t)c * kAsDN + l] >= 0 ? 1 : 0;
  }
  info[1] = ncl; info[2] = segs; info[3] = srcs; info[4] = rows; info[5] = drows;
  return OFX_OK;
}

int ofx_gn_stopped(void* handle, int32_t* stopped) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && stopped, "null handle/stopped");
  *stopped = ((const volatile int32_t*)g->host_flags)[H_STOPPED] ? 1 : 0;
  return OFX_OK;
}

int ofx_gn_step_fused(void* handle, int32_t* fused) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && fused, "null handle/fused");
  *fused = g->step_fused ? 1 : 0;
  return OFX_OK;
}

int ofx_gn_pcg_waves(void* handle, int32_t* waves) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && waves, "null handle/waves");
  *waves = (g->pcg_w2 && g->pcg_ku <= 3) ? 2 : 1;   // the last setup's form (two only up to 384 clusters)
  return OFX_OK;
}

int ofx_gn_stats(void* handle, double* out, int32_t cap) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && out && cap >= 0, "bad gn_stats args");
  const int ss = sync_side(g);
  if (ss) return ss;
  int n = cap < kMaxLog ? cap : kMaxLog;
  if (n > 0) OFX_HIP(hipMemcpy(out, g->stat, 3 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
  return OFX_OK;
}

int ofx_gn_row_order(void* handle, int32_t* perm, int32_t cap) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && g->setup_done && perm, "gn_setup not called / null perm");
  OFX_CHECK_ARG(cap >= (int)g->h_perm.size(), "cap %d < rows %d", cap, (int)g->h_perm.size());
  memcpy(perm, g->h_perm.data(), g->h_perm.size() * sizeof(int32_t));
  return OFX_OK;
}

#ifdef OFX_STAMPS
// tuning build only (not part of include/ofx.h): arm (n > 0) / read back the PCG phase stamps
int ofx_gn_host_enqueue(void* handle, double* us, int64_t* n) {
  Gn* g = (Gn*)handle;
  *us = g->host_enqueue_us; *n = g->host_enqueued;
  g->host_enqueue_us = 0.0; g->host_enqueued = 0;
  return OFX_OK;
}
int ofx_gn_gaps(void* handle, double* ms, int64_t* n) {   // sum of the recorded step-boundary gaps (then cleared)
  Gn* g = (Gn*)handle;
  double t = 0.0;
  for (auto& e : g->gap_ev) {
    float x = 0.f;
    OFX_HIP(hipEventSynchronize(e.second));
    OFX_HIP(hipEventElapsedTime(&x, e.first, e.second));
    t += x;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  *ms = t;
  *n = (int64_t)g->gap_ev.size();
  g->gap_ev.clear();
  double te = 0.0;
  for (auto& e : g->entry_ev) {
    float x = 0.f;
    OFX_HIP(hipEventSynchronize(e.second));
    OFX_HIP(hipEventElapsedTime(&x, e.first, e.second));
    te += x;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (getenv("OFX_GAP_VERBOSE") && !g->entry_ev.empty())
    fprintf(stderr, "solve entry -> setup waited + pose done: %.1f us per solve (%zu); host prep_wait %.1f us per solve\n",
            1e3 * te / g->entry_ev.size(), g->entry_ev.size(), g->prep_wait_us / g->entry_ev.size());
  g->entry_ev.clear();
  g->prep_wait_us = 0.0;
  if (getenv("OFX_GAP_VERBOSE"))
    fprintf(stderr, "host: convergence seen -> k_terms enqueued %.2f us, -> first chunk launch %.2f us (n %lld)\n",
            g->react_us / (double)(g->react_n ? g->react_n : 1), g->prologue_us / (double)(g->react_n ? g->react_n : 1),
            (long long)g->react_n);
  g->react_us = g->prologue_us = 0.0;
  g->react_n = 0;
  return OFX_OK;
}
int ofx_gn_stamps(void* handle, uint64_t* out, int64_t n) {
  Gn* g = (Gn*)handle;
  const int64_t cap = (int64_t)64 * (g->max_pad / kCS) * 8;
  if (!g->stamps) OFX_HIP(hipMalloc((void**)&g->stamps, cap * sizeof(uint64_t)));
  if (out) OFX_HIP(hipMemcpy(out, g->stamps, (n < cap ? n : cap) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  OFX_HIP(hipMemset(g->stamps, 0, cap * sizeof(uint64_t)));
  return OFX_OK;
}
#endif

int ofx_gn_destroy(void* handle) {
  if (!handle) return OFX_OK;
  Gn* g = (Gn*)handle;
  if (g->pf_peer) pf_fire(g, -1);   // a prefetch this handle would have started: start it now
  pf_unlink(g);
  prep_wait(g);
  if (g->worker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      g->quit = true;
    }
    g->cv.notify_all();
    g->worker.join();
  }
  (void)hipDeviceSynchronize();
  if (g->side) (void)hipStreamDestroy(g->side);
  if (g->ev_in) (void)hipEventDestroy(g->ev_in);
  if (g->ev_prep) (void)hipEventDestroy(g->ev_prep);
  if (g->ev_side) (void)hipEventDestroy(g->ev_side);
  free_all(g);
  delete g;
  return OFX_OK;
}

int ofx_gn_setup(void* handle, const ofx_gn_problem* pb, const ofx_gn_params* prm, int64_t* nnz_blocks,
                 ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g, "null handle");
  prep_wait(g);            // an explicit setup replaces a prefetched one
  g->prepared = false;
  g->prep_status = OFX_OK;
  const int fs = fence_side(g, as_stream(s));   // its side-stream kernels write the buffers this setup reuses
  if (fs) return fs;
  return gn_setup(g, pb, prm, nnz_blocks, s);
}

}  // extern "C"

static int prepare_impl(Gn* g, const ofx_gn_problem* pb, const ofx_gn_params* prm, ofx_stream_t s, Gn* trigger,
                        int step) {
  OFX_CHECK_ARG(g && pb && prm, "null handle/problem/params");
  OFX_CHECK_ARG(trigger != g, "a prefetch cannot be triggered by its own handle");
  prep_wait(g);
  pf_unlink(g);
  g->prepared = false;
  g->prep_status = OFX_OK;
  if (!g->side) {
    OFX_HIP(hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking));
    OFX_HIP(hipEventCreateWithFlags(&g->ev_in, hipEventDisableTiming));
    OFX_HIP(hipEventCreateWithFlags(&g->ev_prep, hipEventDisableTiming));
    OFX_HIP(hipEventCreateWithFlags(&g->ev_side, hipEventDisableTiming));
  }
  OFX_HIP(hipGetDevice(&g->prep_dev));
  // everything enqueued on the caller's stream so far (the problem's producers, this handle's last solve) comes
  // before the prefetched setup
  OFX_HIP(hipEventRecord(g->ev_in, as_stream(s)));
  g->prep_pb = *pb;
  g->prep_pb.prev_rot = nullptr;    // the pose is loaded by the solve (k_pose)
  g->prep_pb.prev_trans = nullptr;
  g->prep_prm = *prm;
  g->prepared = true;
  g->side_dirty = true;
  if (!g->worker.joinable()) g->worker = std::thread(prep_worker, g);
  if (trigger) {   // the trigger's next solve opens the gate (pf_fire); it gates one prefetch at a time
    if (trigger->pf_peer) pf_fire(trigger, -1);
    pf_unlink(trigger);
    trigger->pf_peer = g;
    trigger->pf_step = step;
    g->pf_trigger = trigger;
  }
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->gate = trigger != nullptr;
    g->job = true;
  }
  g->cv.notify_all();
  return OFX_OK;
}

extern "C" {

int ofx_gn_prepare(void* handle, const ofx_gn_problem* pb, const ofx_gn_params* prm, ofx_stream_t s) {
  return prepare_impl((Gn*)handle, pb, prm, s, nullptr, 0);
}

int ofx_gn_prepare_after(void* handle, const ofx_gn_problem* pb, const ofx_gn_params* prm, ofx_stream_t s,
                         void* trigger, int32_t gn_step) {
  OFX_CHECK_ARG(trigger, "null trigger handle");
  return prepare_impl((Gn*)handle, pb, prm, s, (Gn*)trigger, gn_step);
}

int ofx_gn_share_history(void* handle, void* other) {
  Gn* g = (Gn*)handle;
  Gn* o = (Gn*)other;
  OFX_CHECK_ARG(g && o, "null handle");
  g->last_pcg = o->last_pcg;
  return OFX_OK;
}

int ofx_gn_set_idle_hook(void* handle, void (*fn)(void*), void* arg) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g, "null handle");
  g->idle_fn = fn;
  g->idle_arg = fn ? arg : nullptr;
  return OFX_OK;
}

int ofx_gn_prefetch_stats(void* handle, int64_t* used, int64_t* missed) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g && used && missed, "null handle/outputs");
  *used = g->pf_used;
  *missed = g->pf_missed;
  return OFX_OK;
}

int ofx_gn_prepare_wait(void* handle, ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  OFX_CHECK_ARG(g, "null handle");
  prep_wait(g);
  return fence_side(g, as_stream(s));   // all of the prefetch's side-stream work, whatever its status
}

}  // extern "C"

namespace ofx {

static int gn_setup(Gn* g, const ofx_gn_problem* pb, const ofx_gn_params* prm, int64_t* nnz_blocks, ofx_stream_t s) {
  OFX_CHECK_ARG(g && pb && prm, "null handle/problem/params");
  OFX_CHECK_ARG(pb->n_nodes >= 1 && pb->n_nodes <= g->max_nodes, "n_nodes %d outside [1,%d]", pb->n_nodes, g->max_nodes);
  OFX_CHECK_ARG(pb->n_matches >= 0 && pb->n_matches <= g->max_matches, "n_matches %d > max %d", pb->n_matches, g->max_matches);
  OFX_CHECK_ARG(pb->n_neighbors >= 0, "bad n_neighbors");
  OFX_CHECK_ARG(pb->nodes && pb->target_node_pos && pb->node_conf, "null node buffers");
  OFX_CHECK_ARG(pb->n_matches == 0 || (pb->src && pb->anchors && pb->weights && pb->tgt), "null match buffers");
  OFX_CHECK_ARG(prm->num_iter >= 0 && prm->num_iter <= 64, "num_iter must be in [0,64]");
  OFX_CHECK_ARG(prm->pcg_max_iter >= 1, "pcg_max_iter must be >= 1");
  OFX_CHECK_ARG(prm->precond_rot_tol >= 0.0, "precond_rot_tol must be >= 0");
  OFX_CHECK_ARG(prm->precond == OFX_PRECOND_CLUSTER || prm->precond == OFX_PRECOND_SCHWARZ || prm->precond == OFX_PRECOND_AUTO,
                "bad precond %d", prm->precond);
  hipStream_t hs = as_stream(s);
  int N0 = pb->n_nodes, M = pb->n_matches, NB = pb->n_neighbors;
  if ((int64_t)N0 * NB > 0) OFX_CHECK_ARG(pb->edges, "null edges");
  // row order (cluster preconditioner): rebuilt when the graph differs from the previous solve's. If a
  // row order exists for a graph of the same size, assume it still holds and compare on the device; the
  // result is read with the pattern size below (no extra sync) and a changed graph restarts the setup.
  const bool optimistic = !g->h_perm.empty() && g->h_nodes.size() == 3 * (size_t)N0 &&
                          g->h_edges.size() == (size_t)N0 * NB && g->gcap_n >= 3 * (int64_t)N0 &&
                          g->gcap_e >= (int64_t)N0 * NB && g->d_gdiff;
  if (optimistic) {   // (d_gdiff is zero: k_setup_status cleared it after reading)
    const int64_t na = 3 * (int64_t)N0, nc = (int64_t)N0 * NB;
    hipLaunchKernelGGL(k_graph_cmp, dim3(grid_for(na > nc ? na : nc, 256, 1 << 30)), dim3(256), 0, hs, pb->nodes,
                       (const float*)g->d_gnodes, na, pb->edges, (const int32_t*)g->d_gedges, nc, g->d_gdiff);
  } else {
    std::vector<float> hn(3 * (size_t)N0);
    std::vector<int32_t> he((size_t)N0 * NB);
    OFX_HIP(hipMemcpyAsync(hn.data(), pb->nodes, hn.size() * sizeof(float), hipMemcpyDeviceToHost, hs));
    if (!he.empty())
      OFX_HIP(hipMemcpyAsync(he.data(), pb->edges, he.size() * sizeof(int32_t), hipMemcpyDeviceToHost, hs));
    OFX_HIP(hipStreamSynchronize(hs));
    if (hn != g->h_nodes || he != g->h_edges || g->h_perm.empty()) {
      order_rows(N0, NB, hn.data(), he.data(), g->h_perm);
      std::vector<int32_t> ip(N0, -1);
      for (size_t r = 0; r < g->h_perm.size(); ++r)
        if (g->h_perm[r] >= 0) ip[g->h_perm[r]] = (int32_t)r;
      if ((int)g->h_perm.size() > g->max_pad) { set_error("row order overflow"); return OFX_ERR_RANGE; }
      OFX_HIP(hipMemcpyAsync(g->perm, g->h_perm.data(), g->h_perm.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
      OFX_HIP(hipMemcpyAsync(g->iperm, ip.data(), ip.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
      OFX_HIP(hipStreamSynchronize(hs));   // pageable sources
      g->h_nodes.swap(hn);
      g->h_edges.swap(he);
    }
    // device copy of this graph for the next solves' optimistic check
    if (3 * (int64_t)N0 > g->gcap_n) {
      if (g->d_gnodes) OFX_HIP(hipFree(g->d_gnodes));
      g->gcap_n = 3 * (int64_t)N0;
      OFX_HIP(hipMalloc((void**)&g->d_gnodes, g->gcap_n * sizeof(float)));
    }
    if ((int64_t)N0 * NB > g->gcap_e || !g->d_gedges) {
      if (g->d_gedges) OFX_HIP(hipFree(g->d_gedges));
      g->gcap_e = (int64_t)N0 * NB > 1 ? (int64_t)N0 * NB : 1;
      OFX_HIP(hipMalloc((void**)&g->d_gedges, g->gcap_e * sizeof(int32_t)));
    }
    if (!g->d_gdiff) OFX_HIP(hipMalloc((void**)&g->d_gdiff, sizeof(int32_t)));
    OFX_HIP(hipMemsetAsync(g->d_gdiff, 0, sizeof(int32_t), hs));   // (this path reads none: a stale flag must not stay)
    OFX_HIP(hipMemcpyAsync(g->d_gnodes, pb->nodes, 3 * (size_t)N0 * sizeof(float), hipMemcpyDeviceToDevice, hs));
    if ((int64_t)N0 * NB > 0)
      OFX_HIP(hipMemcpyAsync(g->d_gedges, pb->edges, (size_t)N0 * NB * sizeof(int32_t), hipMemcpyDeviceToDevice, hs));
  }
  OFX_CHECK_ARG(prm->mode == OFX_GN_OPTIMIZE || prm->mode == OFX_GN_ARAP, "bad gn mode %d", prm->mode);
  OFX_CHECK_ARG(prm->mode != OFX_GN_ARAP || M == 0, "arap mode takes no match rows");
  const int N = (int)g->h_perm.size();
  g->n_comp = 0;
  if (prm->mode == OFX_GN_ARAP && prm->lambda_flow == 0.0) {
    // connected components of the (undirected) ED graph, rows listed per component
    std::vector<int32_t> lab(N0, -1), rows, off{0}, stack;
    std::vector<std::vector<int32_t>> adj(N0);
    for (int i = 0; i < N0; ++i)
      for (int k = 0; k < NB; ++k) {
        const int j = g->h_edges[(size_t)i * NB + k];
        if (j >= 0 && j < N0 && j != i) { adj[i].push_back(j); adj[j].push_back(i); }
      }
    std::vector<int32_t> ip(N0, -1);
    for (int r = 0; r < N; ++r)
      if (g->h_perm[r] >= 0) ip[g->h_perm[r]] = r;
    for (int s0 = 0; s0 < N0; ++s0) {
      if (lab[s0] >= 0 || adj[s0].empty()) continue;
      const size_t first = rows.size();
      lab[s0] = 1;
      stack.assign(1, s0);
      while (!stack.empty()) {
        const int v = stack.back();
        stack.pop_back();
        rows.push_back(ip[v]);
        for (int j : adj[v])
          if (lab[j] < 0) { lab[j] = 1; stack.push_back(j); }
      }
      std::sort(rows.begin() + first, rows.end());
      off.push_back((int32_t)rows.size());
    }
    g->n_comp = (int)off.size() - 1;
    if (g->n_comp > 0) {
      if ((int)rows.size() + (int)off.size() > g->comp_cap) {
        if (g->comp_rows) OFX_HIP(hipFree(g->comp_rows));
        if (g->comp_off) OFX_HIP(hipFree(g->comp_off));
        g->comp_cap = (int)(rows.size() + off.size());
        OFX_HIP(hipMalloc((void**)&g->comp_rows, g->comp_cap * sizeof(int32_t)));
        OFX_HIP(hipMalloc((void**)&g->comp_off, g->comp_cap * sizeof(int32_t)));
      }
      OFX_HIP(hipMemcpyAsync(g->comp_rows, rows.data(), rows.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
      OFX_HIP(hipMemcpyAsync(g->comp_off, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
      OFX_HIP(hipStreamSynchronize(hs));   // pageable sources
    }
  }
  g->N = N; g->N_real = N0; g->M = M; g->NB = NB; g->prm = *prm;
  g->fx = pb->fx; g->fy = pb->fy; g->cx = pb->cx; g->cy = pb->cy;
  g->T = (int64_t)M + (int64_t)N * NB + N;
  g->nwg_row = N / kRW;
  g->pcg_ku = pcg_ku_for(g->nwg_row);
  g->nw_pad = 128 * g->pcg_ku;
  // every partial stream is read unconditionally up to nw_pad: the tails must be zero (the kernels write only the
  // entries of their own waves; k_pcg_w0 re-zeroes the iteration streams' tails, nothing writes the others'): k_upload
  // clears them
  g->nwg_node = (N + kBlk - 1) / kBlk;
  g->nwg_terms = (int32_t)((4 * g->T + kBlk - 1) / kBlk);
  // per-solve buffers sized by T
  if (g->T > g->T_cap) {
    for (auto pp : {(void**)&g->term_node, (void**)&g->J, (void**)&g->res, (void**)&g->node_list,
                    (void**)&g->blk_list, (void**)&g->node_tmp, (void**)&g->blk_tmp, (void**)&g->part_loss})
      if (*pp) { OFX_HIP(hipFree(*pp)); *pp = nullptr; }
    int64_t c = g->T + g->T / 4 + 64;
    OFX_HIP(hipMalloc((void**)&g->term_node, 4 * c * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->J, kRec * c * sizeof(double)));
    OFX_HIP(hipMalloc((void**)&g->res, 3 * c * sizeof(double)));
    OFX_HIP(hipMalloc((void**)&g->node_list, 4 * c * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->blk_list, 16 * c * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->node_tmp, 4 * c * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->blk_tmp, 16 * c * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->part_loss, 4 * ((4 * c + kBlk - 1) / kBlk) * sizeof(double)));
    g->T_cap = c;
  }
  // edges + weights (capacity kept across solves)
  int64_t ne = (int64_t)N * NB;
  if (ne > g->ne_cap) {
    if (g->edges) { OFX_HIP(hipFree(g->edges)); g->edges = nullptr; }
    if (g->ew) { OFX_HIP(hipFree(g->ew)); g->ew = nullptr; }
    g->ne_cap = ne;
    OFX_HIP(hipMalloc((void**)&g->edges, ne * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->ew, ne * sizeof(double)));
  }
  Upload u;
  u.nodes = pb->nodes; u.tpos = pb->target_node_pos; u.conf = pb->node_conf; u.src = pb->src; u.wts = pb->weights;
  u.tgt = pb->tgt; u.tpx = pb->target_px; u.tpy = pb->target_py; u.ew = pb->edge_weights; u.prev_R = pb->prev_rot;
  u.prev_t = pb->prev_trans; u.anc = pb->anchors; u.edges = pb->edges; u.use_ew = prm->use_edge_weighting;
  u.old_N = g->pat_N; u.old_nnzb = g->pat_N > 0 ? g->pat_nnzb : 0;
  {
    int64_t n = g->T;
    for (int64_t v : {9 * (int64_t)N, 4 * (int64_t)M, ne, u.old_nnzb, (int64_t)3 * kMaxLog, (int64_t)2 * (kMaxLog + 1),
                      (int64_t)F_COUNT, (int64_t)kProjP * g->nw_pad})
      n = v > n ? v : n;
    u.n = n;
  }
  if (g->ep_next >= kEpochWrap) {   // PCG epochs restart before int32 overflow: stop words cleared on this stream (after
                                     // every earlier launch of the handle); k_upload clears the host flags
    OFX_HIP(hipMemsetAsync(g->stopw, 0, (size_t)(g->max_pad / kCS) * 64 * sizeof(int32_t), hs));
    g->ep_next = 1;
  }
  hipLaunchKernelGGL(k_upload, dim3(grid_for(u.n, 256, 1 << 30)), dim3(256), 0, hs, *g, u);
  OFX_LAUNCH_CHECK();
  // terms -> block pattern
  unsigned gT = grid_for(g->T, 256, 1 << 30);
  hipLaunchKernelGGL(k_mark, dim3(gT), dim3(256), 0, hs, *g);
  hipLaunchKernelGGL(k_row_count, dim3(N), dim3(256), 0, hs, N, g->map, g->row_cnt);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, hs, (int64_t)N, g->row_cnt, g->row_ptr, g->row_cnt + N, false);
  hipLaunchKernelGGL(k_wave_max, dim3(grid_for(N / kCS, 256)), dim3(256), 0, hs, N / kCS, g->row_ptr, g->row_cnt + N + 1);
  OFX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_setup_status, dim3(1), dim3(64), 0, hs, (const int32_t*)g->row_ptr, N,
                     (const int32_t*)g->row_cnt,
                     optimistic ? g->d_gdiff : nullptr, g->d_setup_stat);
  OFX_LAUNCH_CHECK();
  OFX_HIP(hipStreamSynchronize(hs));
  const volatile int32_t* ss = g->setup_stat;
  const int32_t nnz = ss[0], lens[2] = {ss[1], ss[2]}, gdiff = ss[3];
  if (gdiff) {   // the graph changed: clear the slot map marked with the stale order and start over
    OFX_HIP(hipMemsetAsync(g->map, 0, (size_t)g->max_pad * g->max_pad * sizeof(int32_t), hs));
    g->pat_N = 0;
    g->pat_nnzb = 0;
    g->h_perm.clear();
    return gn_setup(g, pb, prm, nnz_blocks, s);
  }
  g->max_deg = lens[0];
  g->max_wave = lens[1];
  if ((int64_t)nnz + 1 > g->nnzb_cap) {
    for (auto pp : {(void**)&g->col, (void**)&g->blk_row, (void**)&g->A_own, (void**)&g->blk_off,
                    (void**)&g->blk_cnt, (void**)&g->up_of, (void**)&g->up_slot, (void**)&g->up_tr, (void**)&g->blk_first})
      if (*pp) { OFX_HIP(hipFree(*pp)); *pp = nullptr; }
    g->nnzb_cap = (int64_t)nnz + nnz / 4 + 64;
    OFX_HIP(hipMalloc((void**)&g->col, g->nnzb_cap * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->blk_row, g->nnzb_cap * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->A_own, g->nnzb_cap * 36 * sizeof(double)));
    OFX_HIP(hipMalloc((void**)&g->blk_off, (g->nnzb_cap + 1) * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->blk_cnt, (g->nnzb_cap + 1) * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->up_of, (g->nnzb_cap + 1) * sizeof(int32_t)));
    OFX_HIP(hipMalloc((void**)&g->up_slot, (g->nnzb_cap + 32) * sizeof(int32_t)));   // + a workgroup's overhang
    OFX_HIP(hipMalloc((void**)&g->up_tr, (g->nnzb_cap + 32) * sizeof(int32_t)));
    // k_assemble's block workgroups: (nnzb + N) / 2 + 1 upper blocks at most, 16 per workgroup
    OFX_HIP(hipMalloc((void**)&g->blk_first, ((g->nnzb_cap + g->max_pad) / 2 / 16 + 2) * kCoop * sizeof(int32_t)));
  }
  g->nnzb = nnz;
  hipLaunchKernelGGL(k_row_assign, dim3(N), dim3(256), 0, hs, N, g->map, g->row_ptr, g->col, g->blk_row);
  hipLaunchKernelGGL(k_wave_list, dim3(grid_for((int64_t)(N / kCS) * kWL, 256, 1 << 30)), dim3(256), 0, hs, *g);
  g->pat_N = N;
  g->pat_nnzb = nnz;
  // upper blocks: slot -> u by a scan of the flags (blk_cnt as scratch), u -> slot and transpose
  hipLaunchKernelGGL(k_up_flags, dim3(grid_for(nnz, 256, 1 << 30)), dim3(256), 0, hs, *g, g->blk_cnt);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, hs, (int64_t)nnz, g->blk_cnt, g->up_of, (int32_t*)nullptr, false);
  hipLaunchKernelGGL(k_up_list, dim3(grid_for(nnz, 256, 1 << 30)), dim3(256), 0, hs, *g);
  // contribution lists (sorted -> deterministic assembly order); blocks indexed by u (the entries past the upper
  // count stay empty)
  hipLaunchKernelGGL(k_pair_count, dim3(gT), dim3(256), 0, hs, *g);
  // (the scans clear the counts behind them: k_pair_scatter reuses them as cursors)
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, hs, (int64_t)nnz, g->blk_cnt, g->blk_off, (int32_t*)nullptr, true);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, hs, (int64_t)N, g->node_cnt, g->node_off, (int32_t*)nullptr, true);
  hipLaunchKernelGGL(k_pair_scatter, dim3(gT), dim3(256), 0, hs, *g);
  hipLaunchKernelGGL(k_seg_rank, dim3(grid_for(nnz, 4, 1 << 30)), dim3(256), 0, hs, (const int32_t*)g->blk_off, (int64_t)nnz,
                     (const int32_t*)g->blk_list, g->blk_tmp);
  hipLaunchKernelGGL(k_seg_rank, dim3(grid_for(N, 4, 1 << 30)), dim3(256), 0, hs, (const int32_t*)g->node_off, (int64_t)N,
                     (const int32_t*)g->node_list, g->node_tmp);
  std::swap(g->blk_list, g->blk_tmp);
  std::swap(g->node_list, g->node_tmp);
  {
    const int nwb = nnz > 0 ? (int)grid_for((nnz + N) / 2 + 1, kBlk / 16, 1 << 30) : 0;   // (as the assembly's launch)
    hipLaunchKernelGGL(k_first_codes, dim3(nwb + N), dim3(kBlk), 0, hs, *g, nwb);
  }
  OFX_LAUNCH_CHECK();
  // Schwarz tables (blk_off still holds the per-block term counts' offsets)
  g->as_on = 0;
  constexpr int kAsAutoNodes = 1536;   // OFX_PRECOND_AUTO: Schwarz from this graph size on (ofx.h)
  const bool as_req = g->as_env >= 0 ? g->as_env == 1
                                     : (g->prm.precond == OFX_PRECOND_SCHWARZ ||
                                        (g->prm.precond == OFX_PRECOND_AUTO && g->N_real >= kAsAutoNodes));
  if (as_req && g->max_wave <= kWL && g->max_deg <= kRowMax) {   // (the Schwarz form needs the wave-list PCG)
    const int ncl = N / kCS;
    if (ncl > g->as_cap) {
      for (auto pp : {(void**)&g->as_cand, (void**)&g->as_csc, (void**)&g->as_acc, (void**)&g->as_dom, (void**)&g->as_meta,
                      (void**)&g->as_gat, (void**)&g->as_dst, (void**)&g->as_slab, (void**)&g->as_w, (void**)&g->as_src,
                      (void**)&g->as_dsc, (void**)&g->as_rsc})
        if (*pp) { OFX_HIP(hipFree(*pp)); *pp = nullptr; }
      const int cap = g->max_pad / kCS;
      OFX_HIP(hipMalloc((void**)&g->as_cand, (size_t)cap * kAsRing * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_csc, (size_t)cap * kAsRing * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_acc, (size_t)cap * kAsRing * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_dom, (size_t)cap * kAsDN * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_meta, (size_t)cap * kAsMeta * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_gat, (size_t)cap * kAsGat * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_dst, (size_t)cap * kAsD * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_slab, (size_t)cap * kAsK * kAsRS * 8 * sizeof(uint16_t)));
      OFX_HIP(hipMalloc((void**)&g->as_w, (size_t)g->max_pad * 6 * sizeof(double)));
      OFX_HIP(hipMalloc((void**)&g->as_src, (size_t)cap * kAsSrc * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_dsc, (size_t)cap * kAsD * sizeof(float)));
      OFX_HIP(hipMalloc((void**)&g->as_rsc, (size_t)cap * kAsRS * sizeof(float)));
      OFX_HIP(hipMemsetAsync(g->as_rsc, 0, (size_t)cap * kAsRS * sizeof(float), hs));
      OFX_HIP(hipMemsetAsync(g->as_slab, 0, (size_t)cap * kAsK * kAsRS * 8 * sizeof(uint16_t), hs));
      if (g->as_tab) OFX_HIP(hipFree(g->as_tab));
      if (g->as_mem) OFX_HIP(hipFree(g->as_mem));
      if (g->as_memn) OFX_HIP(hipFree(g->as_memn));
      OFX_HIP(hipMalloc((void**)&g->as_tab, (size_t)as_tab_bytes(cap)));
      OFX_HIP(hipMemsetAsync(g->as_tab, 0, (size_t)as_tab_bytes(cap), hs));
      OFX_HIP(hipMalloc((void**)&g->as_mem, (size_t)g->max_pad * 4 * sizeof(int32_t)));
      OFX_HIP(hipMalloc((void**)&g->as_memn, (size_t)g->max_pad * sizeof(int32_t)));
      OFX_HIP(hipMemsetAsync(g->as_memn, 0, (size_t)g->max_pad * sizeof(int32_t), hs));
      g->as_cap = cap;
      g->as_tab_cap = cap;
    }
    hipLaunchKernelGGL(k_as_choose, dim3(ncl), dim3(256), 0, hs, *g);
    hipLaunchKernelGGL(k_as_accept, dim3(grid_for(N, 4)), dim3(256), 0, hs, *g);
    hipLaunchKernelGGL(k_as_compact, dim3(ncl), dim3(64), 0, hs, *g);
    hipLaunchKernelGGL(k_as_segments, dim3(ncl), dim3(256), 0, hs, *g);
    // one launch per iteration (k_as_iter) when every subdomain's workgroup gets a CU at once: a k_as_iter workgroup
    // holds a whole CU (16 waves at 120 VGPRs), so more subdomains than CUs run in two rounds per launch (config 4's 502
    // on 256 CUs: 12.4 us per iteration, 142.8 frames/s against 165.6 with two launches). OFX_AS_ONE=0 / 1: off / on
    // regardless of the CU count (A/B, tests: k_pcg_iter<.., kAS> + k_as_apply is bitwise the same); never past kU = 4
    // (its partial registers spill)
    const char* one = getenv("OFX_AS_ONE");
    int ncu = 0;
    {
      int dev = 0;
      OFX_HIP(hipGetDevice(&dev));
      OFX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const bool one_on = one ? atoi(one) != 0 : ncl <= ncu;
    g->as_one = (one_on && g->pcg_ku <= 4) ? 1 : 0;
    if (g->as_one) {   // (as_memn: cleared by k_upload, or at allocation)
      hipLaunchKernelGGL(k_as_members, dim3(grid_for((int64_t)ncl * kAsDN, 256)), dim3(256), 0, hs, *g, ncl);
      hipLaunchKernelGGL(k_as_tab, dim3(ncl), dim3(256), 0, hs, *g);
    }
    OFX_LAUNCH_CHECK();
    g->as_on = 1;
  }
  if (nnz_blocks) *nnz_blocks = nnz;
  g->setup_done = true;
  return OFX_OK;
}

}  // namespace ofx

extern "C" {

int ofx_gn_linearize(void* handle, int32_t gn_iter, int32_t m0, int32_t m1, int32_t add_reg, double* A, double* rhs,
                     ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && g->setup_done, "gn_setup not called");
  OFX_CHECK_ARG(A && rhs, "null A/rhs");
  OFX_CHECK_ARG(m0 >= 0 && m1 <= g->M && m0 <= m1, "bad match range [%d,%d) of %d", m0, m1, g->M);
  // A: nnz_blocks x 36 f64, rhs: 6·rows + 4 f64 (rows = ofx_gn_info()[4])
  hipStream_t hs = as_stream(s);
  const int fs = fence_side(g, hs);
  if (fs) return fs;
#ifdef OFX_STAMPS
  if (g->gap_end && gn_iter == 0) {   // the previous solve's last step: a frame boundary, not a GN-step one
    (void)hipEventDestroy(g->gap_end);
    g->gap_end = nullptr;
  }
  if (g->gap_end) {
    hipEvent_t e;
    OFX_HIP(hipEventCreate(&e));
    OFX_HIP(hipEventRecord(e, hs));
    g->gap_ev.emplace_back(g->gap_end, e);
    g->gap_end = nullptr;
  }
#endif
  DataCoef dc;
  dc.lf = sqrt(g->prm.lambda_flow); dc.ld = sqrt(g->prm.lambda_depth);
  dc.la = sqrt(g->prm.lambda_arap); dc.lm = sqrt(g->prm.lambda_motion);
  dc.fx = g->fx; dc.fy = g->fy; dc.cx = g->cx; dc.cy = g->cy;
  hipLaunchKernelGGL(k_terms, dim3(g->nwg_terms), dim3(kBlk), 0, hs, *g, dc, m0, m1, add_reg);
#ifdef OFX_STAMPS
  if (gn_iter > 0 && g->t_seen.time_since_epoch().count()) {
    g->react_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g->t_seen).count();
    ++g->react_n;
  }
#endif
  // the LM damping λ_k I (model.py:418-419,641-662) is added by the rank that adds the regularisers, so a
  // sum over ranks carries it once
  const double lm = add_reg ? lm_for_iter(g->prm.lm_factor, gn_iter) : 0.0;
  // upper blocks: (nnzb + diagonal blocks) / 2 <= (nnzb + rows) / 2 (the pattern is symmetric); workgroups past
  // the device-side count return at once
  const int nwb = g->nnzb > 0 ? (int)grid_for((g->nnzb + g->N) / 2 + 1, kBlk / 16, 1 << 30) : 0;
#ifdef OFX_SPLIT_ASSEMBLE   // tuning build: the two halves as separate kernels (rocprof times each)
  if (nwb) hipLaunchKernelGGL(k_assemble_blocks, dim3(nwb), dim3(kBlk), 0, hs, *g, dc, A, lm);
  hipLaunchKernelGGL(k_assemble_rhs, dim3(grid_for(g->N, kBlk / 64)), dim3(kBlk), 0, hs, *g, dc, rhs);
#else
  const int nrw = ((int)grid_for(g->N, kBlk / 64) + 7) & ~7;   // (a multiple of 8: see k_assemble)
  hipLaunchKernelGGL(k_assemble, dim3(nwb + nrw), dim3(kBlk), 0, hs, *g, dc, A, rhs, nrw, lm);
#endif
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_gn_step(void* handle, int32_t gn_iter, double* A, double* rhs, ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && g->setup_done, "gn_setup not called");
  OFX_CHECK_ARG(A && rhs, "null A/rhs");
  hipStream_t hs = as_stream(s);
  const int fs = fence_side(g, hs);
  if (fs) return fs;
  int st = gn_pcg(g, gn_iter, A, rhs, hs);
  if (st) return st;
  if (g->step_fused) return OFX_OK;   // the converging PCG launch took the step (fused_step)
  if (g->n_comp > 0) hipLaunchKernelGGL(k_null_project, dim3(g->n_comp), dim3(64), 0, hs, *g);
  double* xsave = g->prm.pcg_warm ? g->xh + (int64_t)(gn_iter % kProj) * 6 * g->N : nullptr;
  hipLaunchKernelGGL(k_step, dim3(grid_for(g->N, 256)), dim3(256), 0, hs, *g, (const double*)rhs, 64,
                     g->prm.pcg_max_iter, gn_iter, xsave);
  OFX_LAUNCH_CHECK();
  return OFX_OK;
}

int ofx_gn_finish(void* handle, const ofx_gn_result* res, ofx_stream_t s) {
  Gn* g = (Gn*)handle;
  if (g) prep_wait(g);   // a prefetch thread of this handle has finished
  OFX_CHECK_ARG(g && g->setup_done && res && res->rot && res->trans, "bad gn_finish args");
  const int fs = fence_side(g, as_stream(s));
  if (fs) return fs;
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
  OFX_CHECK_ARG(g && pb && prm && res, "null handle/problem/params/result");
  struct PfReturn {   // a gated prefetch (ofx_gn_prepare_after) not started by a GN step starts on every return
    Gn* g;
    ~PfReturn() { pf_fire(g, -1); }
  } pf_guard{g};
#ifdef OFX_STAMPS
  hipEvent_t ev_entry = nullptr;
  if (getenv("OFX_GAP_EVENTS")) {
    OFX_HIP(hipEventCreate(&ev_entry));
    OFX_HIP(hipEventRecord(ev_entry, as_stream(s)));
  }
  const auto tw0 = std::chrono::steady_clock::now();
#endif
  prep_wait(g);
#ifdef OFX_STAMPS
  g->prep_wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw0).count();
#endif
  // a setup prefetched for exactly this problem (ofx_gn_prepare): wait for it on the caller's stream and load
  // the pose; otherwise (none, another problem, or it failed) set up here
  const bool use = g->prepared && g->prep_status == OFX_OK && same_problem(g->prep_pb, *pb) &&
                   same_params(g->prep_prm, *prm);
  if (g->prepared) ++(use ? g->pf_used : g->pf_missed);
  g->prepared = false;
  g->prep_status = OFX_OK;
  // used or not, the prefetch's side-stream kernels may still be writing this handle's buffers: the caller's
  // stream waits for all of them before anything here reuses the handle (a discarded prefetch included)
  int st = fence_side(g, as_stream(s));
  if (st) return st;
  if (use) {
    hipStream_t hs = as_stream(s);
    if (pb->prev_rot || pb->prev_trans)
      hipLaunchKernelGGL(k_pose, dim3(grid_for(9 * (int64_t)g->N, 256)), dim3(256), 0, hs, *g, pb->prev_rot,
                         pb->prev_trans);
    OFX_LAUNCH_CHECK();
  } else {
    st = gn_setup(g, pb, prm, nullptr, s);
    if (st) return st;
  }
#ifdef OFX_STAMPS
  if (ev_entry) {
    hipEvent_t e;
    OFX_HIP(hipEventCreate(&e));
    OFX_HIP(hipEventRecord(e, as_stream(s)));
    g->entry_ev.emplace_back(ev_entry, e);
  }
#endif
  for (int it = 0; it < prm->num_iter; ++it) {
    st = ofx_gn_linearize(handle, it, 0, g->M, 1, g->A_own, g->rhs_own, s);
    if (st) return st;
    pf_fire(g, it);   // (after this step's first kernels are queued)
    st = ofx_gn_step(handle, it, g->A_own, g->rhs_own, s);
    if (st) return st;
    // host_flags was refreshed by this step's PCG poll, i.e. after the previous step's stop
    // decision: a stop costs at most one extra (no-op) linearisation instead of a sync per step
    if (((const volatile int32_t*)g->host_flags)[H_STOPPED]) break;
  }
  return ofx_gn_finish(handle, res, s);
}

}  // extern "C"
