"""Gauss-Newton non-rigid registration behind the reference's solver APIs, backed by libofx.

* GaussNewtonSolver.optimize — DeformNet.optimize (model/model.py:222-859) for one batch item:
  same inputs (graph nodes/edges, motion-complete node targets + confidence, source points with
  anchors/weights, target points, intrinsics, prev rot/trans), same outputs (node_rotations,
  node_translations, valid_solve, convergence_info).
* Registration.optimize — NonRigidICP/model/registration_fusion.py:98-145 API (returns
  node_rotations, node_translations, deformed_nodes_to_target, warped_verts, convergence_info,
  source/target frame ids) with the GN solver in place of the Adam/lietorch loop.
* GaussNewtonSolver.arap — DeformNet.arap (model/model.py:1639-1986): the graph-update solve that moves
  only the invalid (invisible / new) nodes under ARAP with the valid nodes held at their transforms.
* optimize_distributed — match-sharded multi-GPU solve: every rank assembles JᵀJ/Jᵀr over its own
  matches, one all-reduce (sum) of the block-sparse accumulators per GN iteration, identical solve
  on every rank.
"""
import ctypes
import math
import os

import numpy as np
import torch

from . import _lib, ops  # noqa: F401  (ops registers torch.ops.ofx.*)
from ._lib import call, byref
from .sharding import match_range

GN_DEFAULTS = dict(num_iter=10, lambda_flow=0.0, lambda_depth=1.0, lambda_arap=0.5, lambda_motion=1.0,
                   lm_factor=1e-7, stop_loss_diff=1.0, use_edge_weighting=False, pcg_max_iter=2000, pcg_tol=2e-6,
                   pcg_warm=True, precond_every=10, pcg_err_tol=2e-6, precond_rot_tol=0.3, precond="auto")
# PCG preconditioner (ofx_gn_params.precond): overlapping additive Schwarz, the 8-node cluster blocks, or
# auto (Schwarz for graphs of >= 1536 nodes)
_PRECOND = {"cluster": 0, "schwarz": 1, "auto": 2}
MAX_MATCHES_EVAL = 10000   # settings/custom_settings.py:36


def _t(x, device, dtype):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        if x.dtype == dtype and x.device == device and x.is_contiguous():
            return x   # per-frame fast path (host time: no .to / .contiguous dispatch)
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


def _prefetch_lead(num_iter):
    """OFX_PREFETCH_LEAD (A/B only): an integer clamped to [0, num_iter]; anything else is the default 1."""
    try:
        v = int(os.environ.get("OFX_PREFETCH_LEAD", "1"))
    except ValueError:
        return 1
    return min(max(v, 0), int(num_iter))


_IDLE_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_void_p)   # ofx_gn_set_idle_hook's fn


class GaussNewtonSolver:
    def __init__(self, max_nodes, max_matches=MAX_MATCHES_EVAL, device=None, **params):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.params = dict(GN_DEFAULTS)
        self.params.update(params)
        self.max_nodes, self.max_matches = int(max_nodes), int(max_matches)
        self._keep = []
        # solver slots (handle, ordering token): a second one is made by the first prefetch (optimize(prefetch=)),
        # which sets up the next problem on the slot the current solve does not use
        self._slots = [self._new_slot()]
        self._cur = 0                   # slot of the next optimize()
        self._pending = [None, None]    # a prefetched problem's tensors, alive until its solve
        self._deferred = None           # defer_to_next_solve: (fn, handle) pending
        self._deferred_cb = None        # its ctypes callback, kept alive
        self._deferred_exc = None       # an exception it raised inside a solve, re-raised by the next call
        self._side = None               # torch stream that orders a prefetch before the current solve
        # GN steps of the current solve a prefetch overlaps: its setup starts when the solve begins step
        # num_iter - prefetch_lead (ofx_gn_prepare_after); 0 = when the solve's host loop returns
        self.prefetch_lead = _prefetch_lead(self.params["num_iter"])   # (env: A/B only)
        self._h, self._state = self._slots[0]   # the last solve's slot (info / stats / stopped / arap / distributed)

    def _new_slot(self):
        h = _lib.c_void_p()
        with torch.cuda.device(self.device):
            call("ofx_gn_create", self.max_nodes, self.max_matches, byref(h))
        return h, torch.zeros(1, dtype=torch.int32, device=self.device)   # ofx::gn_* ordering token (ops.py)

    def __del__(self):
        for h, _ in getattr(self, "_slots", []):
            if h is not None and h.value:
                try:
                    _lib.lib.ofx_gn_destroy(h)
                except Exception:
                    pass
        self._slots = []
        self._h = None

    def timing(self, enable=True):
        """(pcg_ms, k_pcg_iter launches, timed PCG solves) recorded since the last call over all slots; then
        (re)arm."""
        tot = [0.0, 0, 0]
        for h, _ in self._slots:
            ms, n, ns = _lib.c_double(), _lib.c_int64(), _lib.c_int64()
            call("ofx_gn_timing", h, 1 if enable else 0, byref(ms), byref(n), byref(ns))
            tot = [tot[0] + ms.value, tot[1] + n.value, tot[2] + ns.value]
        return tuple(tot)

    def prefetch_stats(self):
        """(solves that used a prefetched setup, solves that discarded one) over all slots."""
        used = missed = 0
        for h, _ in self._slots:
            u, m = _lib.c_int64(), _lib.c_int64()
            call("ofx_gn_prefetch_stats", h, byref(u), byref(m))
            used, missed = used + u.value, missed + m.value
        return used, missed

    def defer_to_next_solve(self, fn):
        """Run fn() once inside the next optimize(), while its host loop waits for the first GN step's PCG chunk
        (ofx_gn_set_idle_hook: the host only spins there), or at that optimize's return if it never waited. A frame
        loop enqueues the previous frame's integrate this way without delaying the next solve's first launches.
        flush_deferred() runs a pending fn now."""
        self.flush_deferred()
        h = self._slots[self._cur][0]

        def hook(_arg):
            self._run_deferred()
        self._deferred_cb = _IDLE_HOOK(hook)
        self._deferred = (fn, h)
        call("ofx_gn_set_idle_hook", h, ctypes.cast(self._deferred_cb, ctypes.c_void_p), None)

    def _run_deferred(self):
        d, self._deferred = self._deferred, None
        if d is None:
            return
        try:
            d[0]()
        except BaseException as e:   # (inside the library's host loop: kept, raised by the next Python-level call)
            self._deferred_exc = e

    def flush_deferred(self):
        """Run a pending defer_to_next_solve() fn now (and raise what a deferred fn raised)."""
        if self._deferred is not None:
            call("ofx_gn_set_idle_hook", self._deferred[1], None, None)
            self._run_deferred()
        if self._deferred_exc is not None:
            e, self._deferred_exc = self._deferred_exc, None
            raise e

    def drain(self):
        """Order the current stream after any prefetched setup still in flight (ofx_gn_prepare_wait): a
        synchronisation afterwards covers it."""
        s = _lib.stream_ptr(torch.cuda.current_stream(self.device))
        for h, _ in self._slots:
            call("ofx_gn_prepare_wait", h, s)

    def info(self):
        """[n_nodes, n_matches, JᵀJ block count, residual terms, PCG rows] of the last solve's setup."""
        arr = (ctypes.c_int64 * 5)()
        call("ofx_gn_info", self._h, arr)
        return list(arr)

    def precond_info(self):
        """The last setup's preconditioner: dict(schwarz, clusters, segments, sources, gathered_rows, subdomain_rows,
        row_length, launches_per_iteration)
        (ofx_gn_precond_info; synchronises the device: tools and bench only)."""
        arr = (ctypes.c_int64 * 8)()
        call("ofx_gn_precond_info", self._h, arr)
        return dict(zip(("schwarz", "clusters", "segments", "sources", "gathered_rows", "subdomain_rows", "row_length",
                         "launches_per_iteration"), list(arr)))

    def stopped(self):
        """The solve's stop flag as the host sees it (ofx_gn_stopped: no synchronisation)."""
        f = ctypes.c_int32()
        call("ofx_gn_stopped", self._h, byref(f))
        return bool(f.value)

    def pcg_waves(self):
        """Waves per cluster workgroup of the PCG iteration kernel in the last setup (2 up to 384 clusters, else 1;
        1 under OFX_PCG_W1=1)."""
        w = ctypes.c_int32()
        call("ofx_gn_pcg_waves", self._h, byref(w))
        return w.value

    def step_fused(self):
        """True if the last GN step's update was taken by its converging PCG launch (include/ofx.h
        ofx_gn_step_fused): its stop flag is then already visible to the host."""
        f = ctypes.c_int32()
        call("ofx_gn_step_fused", self._h, byref(f))
        return bool(f.value)

    def row_order(self):
        """PCG row -> node of the last setup (-1: padding row); the order of rhs / the state rows."""
        rows = self.info()[4]
        arr = np.empty(rows, np.int32)
        call("ofx_gn_row_order", self._h, arr.ctypes.data_as(ctypes.c_void_p), rows)
        return arr

    def stats(self):
        """Per GN step of the last solve: (PCG iterations, |b|², loss) rows; steps that did not run are 0."""
        n = int(self.params["num_iter"])
        arr = (ctypes.c_double * (3 * max(1, n)))()
        call("ofx_gn_stats", self._h, arr, n)
        return np.array(arr[:3 * n], dtype=np.float64).reshape(n, 3)

    def _plist(self, mode=0, pcg_tol=None):
        """GN parameters as the ofx::gn_* operators take them (ops._gn_params)."""
        q = self.params
        fp = [float(q["lambda_flow"]), float(q["lambda_depth"]), float(q["lambda_arap"]), float(q["lambda_motion"]),
              float(q["lm_factor"]), float(q["stop_loss_diff"]), float(q["pcg_tol"] if pcg_tol is None else pcg_tol),
              float(q.get("pcg_err_tol", 0.0)), float(q.get("precond_rot_tol", 0.0))]
        ip = [int(q["num_iter"]), int(bool(q["use_edge_weighting"])), int(q["pcg_max_iter"]), int(bool(q["pcg_warm"])),
              int(mode), int(q.get("precond_every", 1)), _PRECOND[q.get("precond", "cluster")]]
        return fp, ip

    def _problem(self, graph_nodes, graph_edges, graph_edges_weights, target_node_position, node_confidence,
                 source_points, anchors, weights, target_points, intrinsics, target_px, target_py, prev_rot,
                 prev_trans, keep=True):
        """Device tensors of one problem in the ofx::gn_* operators' argument order (+ N, M)."""
        d = self.device
        nodes = _t(graph_nodes, d, torch.float32).reshape(-1, 3)
        N = nodes.shape[0]
        src = _t(source_points, d, torch.float32).reshape(-1, 3)
        M = src.shape[0]
        if N > self.max_nodes or M > self.max_matches:
            raise ValueError(f"problem ({N} nodes, {M} matches) exceeds solver capacity "
                             f"({self.max_nodes}, {self.max_matches})")
        args = [nodes, _t(graph_edges, d, torch.int32).reshape(N, -1), _t(graph_edges_weights, d, torch.float32),
                (_t(target_node_position, d, torch.float32).reshape(N, 3) if target_node_position is not None
                 else nodes.clone()),
                (_t(node_confidence, d, torch.float32).reshape(N) if node_confidence is not None
                 else torch.zeros(N, device=d)),
                src, _t(anchors, d, torch.int32).reshape(M, 4), _t(weights, d, torch.float32).reshape(M, 4),
                _t(target_points, d, torch.float32).reshape(M, 3), _t(target_px, d, torch.float32),
                _t(target_py, d, torch.float32), _t(prev_rot, d, torch.float32), _t(prev_trans, d, torch.float32),
                [float(v) for v in np.asarray(intrinsics, np.float64).reshape(-1)[:4]]]
        if keep:
            self._keep = args   # the last problem's inputs (arap reads prev_trans back)
        return args, N, M

    @staticmethod
    def _pack(out, sync):
        rot, trans, status, loss = out
        res = {"node_rotations": rot, "node_translations": trans, "_status": status, "_loss": loss}
        if sync:
            st = status.cpu().numpy()
            loss = loss.cpu().numpy()[:st[1]]
            res["valid_solve"] = int(st[0])
            res["convergence_info"] = {"total": loss[:, 0].tolist(), "data": loss[:, 1].tolist(),
                                       "arap": loss[:, 2].tolist(), "motion": loss[:, 3].tolist(),
                                       "valid": int(st[0]), "gn_iterations": int(st[1]),
                                       "pcg_iterations": int(st[2]), "pcg_capped_steps": int(st[4]),
                                       "errors": ["Solver failed: Ill-posed system!"] if st[3] else []}
        return res

    def optimize(self, graph_nodes, graph_edges, graph_edges_weights, target_node_position, node_confidence,
                 source_points, anchors, weights, target_points, intrinsics, target_px=None, target_py=None,
                 prev_rot=None, prev_trans=None, sync=True, prefetch=None):
        """model.py:222-859 (batch item) through torch.ops.ofx.gn_solve. Returns torch device tensors (+ host
        convergence info if sync).

        prefetch: the NEXT frame's problem as a dict of this method's argument names (graph_nodes ...
        target_points, optional target_px / target_py; intrinsics default to this call's; no pose). Its setup
        (upload, JᵀJ pattern, with the setup's host sync) is started on the other solver slot when this solve's
        host loop returns, ordered before this solve, and runs concurrently with this frame's tail
        (torch.ops.ofx.gn_prepare); the next optimize() with that problem (the same device tensors) then skips
        its setup. The prefetched tensors must not change until
        that call."""
        args, N, M = self._problem(graph_nodes, graph_edges, graph_edges_weights, target_node_position,
                                   node_confidence, source_points, anchors, weights, target_points, intrinsics,
                                   target_px, target_py, prev_rot, prev_trans)
        fp, ip = self._plist()
        cur = self._cur
        h, st = self._slots[cur]
        if prefetch is not None:
            # The prefetch problem's tensors are made first (any conversion / default it needs runs on the current
            # stream), then the prefetch is ordered after the work enqueued so far (those producers, its inputs,
            # the other slot's last solve) but not after this solve: it is started when this solve's host loop
            # returns, so its kernels overlap this frame's tail (the drained PCG launches, the integrate) instead
            # of the PCG chain. Inputs that need conversion are new tensors on every call, so such a prefetch is
            # correct but never matches the next solve (it is set up inline then: prefetch_stats counts a miss).
            q = dict(prefetch)
            pa, _, _ = self._problem(q["graph_nodes"], q["graph_edges"], q["graph_edges_weights"],
                                     q["target_node_position"], q["node_confidence"], q["source_points"],
                                     q["anchors"], q["weights"], q["target_points"], q.get("intrinsics", intrinsics),
                                     q.get("target_px"), q.get("target_py"), None, None, keep=False)
            before = torch.cuda.Event()
            before.record()
            lead = int(self.prefetch_lead)
            if lead > 0:   # queued now, started by this solve at GN step num_iter - lead (or when it returns)
                self._prefetch(pa, before, h, int(self.params["num_iter"]) - lead, fp, ip)
        if self._deferred is not None and self._deferred[1].value != h.value:   # (hooked on another slot)
            self.flush_deferred()
        out = torch.ops.ofx.gn_solve(st, h.value, *args, fp, ip)
        self.flush_deferred()   # (a deferred fn the solve never reached — no PCG wait — runs now; its exception too)
        self._pending[cur] = None
        self._h, self._state = h, st
        if prefetch is not None:
            if lead <= 0:
                self._prefetch(pa, before, None, 0, fp, ip)
            self._cur = 1 - cur
        return self._pack(out, sync)

    def _prefetch(self, pa, before, trigger, step, fp, ip):
        """Queue the next problem's setup on the other slot, ordered after `before` (torch.ops.ofx.gn_prepare)."""
        nxt = 1 - self._cur
        if len(self._slots) < 2:
            self._slots.append(self._new_slot())
            call("ofx_gn_share_history", self._slots[1][0], self._slots[0][0])
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        h1, st1 = self._slots[nxt]
        with torch.cuda.stream(self._side):
            self._side.wait_event(before)
            torch.ops.ofx.gn_prepare(st1, h1.value, *pa[:11], pa[13], fp, ip, trigger.value if trigger else 0,
                                     max(step, 0))
        self._pending[nxt] = pa

    def arap(self, graph_nodes, source_node_position, target_node_position, valid_nodes_mask, original_graph_nodes,
             graph_edges, graph_edges_weights, graph_clusters, R_current, t_current, sync=True, pcg_tol=1e-10):
        """model.py:1639-1986. graph_nodes (N,3) at the source; source/target_node_position (V,3) of the
        V valid nodes (mask order); only invalid nodes are updated. The reference builds its ARAP rows on
        original_graph_nodes and its data rows on graph_nodes; its only caller passes the same array for
        both (run_model.py:604-619), which this solver requires. Returns node_rotations (N,3,3),
        node_translations (N,3), deformed_nodes_to_target (V,3), valid_solve, convergence_info."""
        d = self.device
        nodes = _t(graph_nodes, d, torch.float32).reshape(-1, 3)
        N = nodes.shape[0]
        if original_graph_nodes is not None and not torch.equal(_t(original_graph_nodes, d, torch.float32).reshape(N, 3),
                                                                nodes):
            raise ValueError("arap: original_graph_nodes must equal graph_nodes (run_model.py:604-619)")
        valid = _t(valid_nodes_mask, d, torch.bool).reshape(N)
        vidx = torch.nonzero(valid).reshape(-1)
        conv = {"total": [], "arap": [], "data": [], "condition_numbers": [], "valid": 0, "errors": []}
        if vidx.numel() == 0:                          # model.py:1683-1687
            conv["errors"].append("Solver failed: No valid correspondences after filtering")
            return {"convergence_info": conv}
        src = _t(source_node_position, d, torch.float32).reshape(-1, 3)
        if not torch.equal(src, nodes[vidx]):
            raise ValueError("arap: source_node_position must be graph_nodes[valid_nodes_mask] (tsdf.py:660-661)")
        tpos = torch.zeros((N, 3), device=d)
        tpos[vidx] = _t(target_node_position, d, torch.float32).reshape(-1, 3)
        z3 = np.zeros((0, 3), np.float32)
        args, N, _ = self._problem(nodes, graph_edges, graph_edges_weights, tpos, valid.float(), z3,
                                   np.zeros((0, 4), np.int32), np.zeros((0, 4), np.float32), z3, (1.0, 1.0, 0.0, 0.0),
                                   None, None, R_current, t_current)
        fp, ip = self._plist(mode=1, pcg_tol=pcg_tol)
        out = torch.ops.ofx.gn_solve(self._state, self._h.value, *args, fp, ip)
        res = self._pack(out, sync)
        t_init = self._keep[12]                              # prev_trans as uploaded
        t0 = t_init[vidx] if t_init is not None else torch.zeros_like(src)
        res["deformed_nodes_to_target"] = src + t0          # valid nodes never move (model.py:1719,1961-1962)
        if sync:
            ci = res["convergence_info"]
            res["convergence_info"] = {"total": ci["total"], "arap": ci["arap"], "data": ci["data"],
                                       "condition_numbers": [], "valid": ci["valid"], "errors": ci["errors"],
                                       "gn_iterations": ci["gn_iterations"], "pcg_iterations": ci["pcg_iterations"],
                                       "pcg_capped_steps": ci["pcg_capped_steps"]}
        return res

    def optimize_distributed(self, graph_nodes, graph_edges, graph_edges_weights, target_node_position,
                             node_confidence, source_points, anchors, weights, target_points, intrinsics,
                             target_px=None, target_py=None, prev_rot=None, prev_trans=None, group=None, sync=True,
                             timer=None):
        """Match-sharded solve over torch.distributed: rank r assembles matches [r*M/W, (r+1)*M/W);
        A and rhs are all-reduced (sum) once per GN iteration; rank 0 adds ARAP + motion rows.
        timer: a list that receives (start, end) CUDA events around each GN step's all-reduce."""
        import torch.distributed as dist
        args, N, M = self._problem(graph_nodes, graph_edges, graph_edges_weights, target_node_position,
                                   node_confidence, source_points, anchors, weights, target_points, intrinsics,
                                   target_px, target_py, prev_rot, prev_trans)
        fp, ip = self._plist()
        h = self._h.value
        nnz, rows = (int(v) for v in torch.ops.ofx.gn_setup(self._state, h, *args, fp, ip))
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        m0, m1 = match_range(M, rank, world)
        A = torch.empty(nnz * 36, dtype=torch.float64, device=self.device)
        rhs = torch.empty(6 * rows + 4, dtype=torch.float64, device=self.device)   # include/ofx.h: ofx_gn_linearize
        for it in range(int(self.params["num_iter"])):
            torch.ops.ofx.gn_linearize(self._state, h, it, m0, m1, rank == 0, A, rhs)
            if timer is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            dist.all_reduce(A, group=group)
            dist.all_reduce(rhs, group=group)
            if timer is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                timer.append((e0, e1))
            torch.ops.ofx.gn_step(self._state, h, it, A, rhs)
            # The stop decision of step `it` is identical on every rank (identical all-reduced systems). A step fused
            # into its converging PCG launch stored the stop flag before the convergence flag the host already saw;
            # otherwise (k_step as its own launch, after pcg_max_iter launches) the flag is written asynchronously:
            # read it only after the step has run, so that every rank leaves the loop after the same step and the
            # collectives stay matched.
            if not self.step_fused():
                torch.cuda.current_stream(self.device).synchronize()
            if self.stopped():
                break
        out = torch.ops.ofx.gn_finish(self._state, h, N, int(self.params["num_iter"]))
        return self._pack(out, sync)


def depth_2_pc_device(depth, intrin):
    from .image_proc import depth_2_pc_device as f
    return f(depth, intrin)


class Registration:
    """registration_fusion.py:37-397 API with the Gauss-Newton solver (DeformNet.optimize formulation)."""

    def __init__(self, canonical_vertices, graph, warpfield, K, vis=None, max_matches=MAX_MATCHES_EVAL, seed=0,
                 **gn_params):
        self.graph = graph
        self.warpfield = warpfield
        self.intrinsics = np.asarray(K, np.float64)
        self.vis = vis
        self.device = warpfield.device
        self.max_matches = max_matches
        self.rng = np.random.default_rng(seed)
        self.solver = GaussNewtonSolver(graph.nodes.shape[0], max_matches, self.device, **gn_params)
        self.prev_rot = None
        self.prev_trans = None
        self.update(canonical_vertices)

    def update(self, canonical_vertices):
        """registration_fusion.py:66-85: skin the canonical vertices, keep the valid ones."""
        a, w, v = self.warpfield.skin_device(canonical_vertices)
        self.valid_source_verts = v.cpu().numpy()
        vt = torch.as_tensor(np.ascontiguousarray(canonical_vertices, np.float32), device=self.device)
        self.source_pcd = vt[v]
        self.point_anchors = a[v]
        self.anchor_weight = w[v]

    def _intr4(self):
        K = self.intrinsics
        return (K[0, 0], K[1, 1], K[0, 2], K[1, 2]) if K.shape == (3, 3) else tuple(K.reshape(-1)[:4])

    def optimize(self, optical_flow_data, scene_flow_data, complete_node_motion_data, target_frame_data,
                 landmarks=None):
        im = target_frame_data.get("im") if isinstance(target_frame_data, dict) else None
        if im is not None:   # registration_fusion.py:104-109: target cloud + pixel map (ofx_depth_to_pc)
            depth = torch.as_tensor(np.ascontiguousarray(im[-1], np.float32), device=self.device)
            self.tgt_pcd, self.pix_2_pcd = depth_2_pc_device(depth, self.intrinsics)
        tm = np.asarray(scene_flow_data["target_matches"], np.float32)[self.valid_source_verts]
        vv = np.asarray(scene_flow_data["valid_verts"], bool)
        sel = np.nonzero(vv[: self.source_pcd.shape[0]])[0]
        if sel.size > self.max_matches:           # model.py:319-334 (reference: unseeded randperm)
            sel = np.sort(self.rng.choice(sel, self.max_matches, replace=False))
        idx = torch.as_tensor(sel, device=self.device, dtype=torch.int64)
        tloc, tconf = complete_node_motion_data if complete_node_motion_data is not None else (None, None)
        out = self.solver.optimize(self.graph.nodes, self.graph.edges, self.graph.edges_weights, tloc, tconf,
                                   self.source_pcd[idx], self.point_anchors[idx], self.anchor_weight[idx],
                                   tm[sel], self._intr4(), prev_rot=self.prev_rot, prev_trans=self.prev_trans)
        R, T = out["node_rotations"], out["node_translations"]
        self.prev_rot, self.prev_trans = R.clone(), T.clone()
        nodes_t = torch.as_tensor(self.graph.nodes, device=self.device)
        self.warpfield.set_node_transforms(R, T)
        warped = self.warpfield.deform_device(self.source_pcd, self.point_anchors, self.anchor_weight)
        # dtypes as registration_fusion.py:363-377: rotations numpy f64 (scipy as_matrix), translations a CPU
        # tensor, deformed nodes and warped vertices device tensors
        res = {"warped_verts": warped, "node_rotations": R.cpu().numpy().astype(np.float64), "node_translations": T.cpu(),
               "deformed_nodes_to_target": nodes_t + T, "convergence_info": out["convergence_info"],
               "valid_solve": out["valid_solve"],
               "source_frame_id": optical_flow_data["source_id"], "target_frame_id": optical_flow_data["target_id"]}
        return res


def run_arap(solver, reduced_graph_dict, model_data, graph, log=None):
    """run_model.py:448-627 (Model.run_arap): initialise every invalid node from its highest-weight already-
    updated graph neighbour (queue ordered by the number of valid neighbours, descending), then the device
    DeformNet.arap GN (GaussNewtonSolver.arap) on all nodes. Returns node_rotations (N,3,3), node_translations
    (N,3), deformed_nodes_to_target (N,3), source/target frame ids, convergence_info, valid_solve.
    np.argsort's tie order in the reference is unspecified (quicksort); here it is stable."""
    for k in ("node_rotations", "node_translations", "deformed_nodes_to_target"):
        assert np.asarray(model_data[k]).dtype == np.float32, f"model_data[{k}] not np.float32"
    valid = np.asarray(reduced_graph_dict["valid_nodes_mask"]).reshape(-1).astype(bool)
    N = len(graph.nodes)
    assert len(valid) == N, f"Valid nodes not from current graph. Expected:{N} got:{len(valid)}"
    R = np.tile(np.eye(3, dtype=np.float32)[None], (N, 1, 1))
    T = np.zeros((N, 3), np.float32)
    R[valid] = model_data["node_rotations"]
    T[valid] = model_data["node_translations"]
    invalid = np.where(~valid)[0]
    n_edges = np.sum(graph.edges != -1, axis=1)
    vis = [np.sum(valid[graph.edges[n, :n_edges[n]]]) for n in invalid]
    queue = list(invalid[np.argsort(vis, kind="stable")[::-1]])
    g = np.asarray(reduced_graph_dict["all_nodes_at_source"], np.float32)
    updated = valid.copy()
    while updated.sum() < N:
        L = len(queue)
        for i in range(L):
            ind = queue[i]
            nb = graph.edges[ind, :n_edges[ind]]
            cand = np.where(updated[nb])[0]
            if len(cand) == 0:
                queue.append(ind)
                continue
            c = graph.edges[ind, cand[np.argmax(graph.edges_weights[ind, cand])]]
            R[ind] = R[c]
            T[ind] = R[ind] @ (g[ind] - g[c]) + T[c] + g[c] - g[ind]
            updated[ind] = True
        del queue[:L]
        if len(queue) == 0 or len(queue) == L:
            break
    res = solver.arap(g, reduced_graph_dict["valid_nodes_at_source"], model_data["deformed_nodes_to_target"], valid, g,
                      graph.edges, graph.edges_weights, graph.clusters, R, T)
    out = {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in res.items()}
    out["deformed_nodes_to_target"] = g + out["node_translations"]
    out["source_frame_id"] = model_data.get("source_frame_id")
    out["target_frame_id"] = model_data.get("target_frame_id")
    return out
