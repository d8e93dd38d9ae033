"""FusionPipeline — the per-frame loop of the reference's working driver
(fusion_with_occlusion/fusion_tests/lepard_nicp_test.py:401-540, test4) restricted to the hot path:

    solve (GN, DeformNet.optimize formulation)  ->  warpfield.update_transformations
    ->  tsdf.integrate(target frame)  (skin cache -> ED warp -> project -> TSDF/weight/colour)

Learned front-ends (Lepard scene flow, OcclusionFusion motion completion), marching cubes and graph
updates are outside the hot path; their outputs (matches, node motion targets + confidence) are
inputs here. Everything stays device-resident across frames; no host copies inside step().
"""
from dataclasses import dataclass
from types import SimpleNamespace

import numpy as np
import torch

from .registration import GaussNewtonSolver
from .tsdf import TSDFVolume
from .warpfield import EDGraph, WarpField


@dataclass
class FrameInputs:
    im: torch.Tensor        # (6,H,W) f32 device
    src: torch.Tensor       # (M,3)
    anchors: torch.Tensor   # (M,4) i32
    weights: torch.Tensor   # (M,4) f32
    tgt: torch.Tensor       # (M,3)
    tpos: torch.Tensor      # (N,3)
    conf: torch.Tensor      # (N,)


class FusionPipeline:
    def __init__(self, seq, origin, voxel_size, dims, n_matches=10000, device=None, shard=None, gn_params=None,
                 with_color=True, overlap=False):
        self.seq = seq
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        cam = seq.cam
        self.intr = (cam.fx, cam.fy, cam.cx, cam.cy)
        self.fopt = SimpleNamespace(source_frame=0, skip_rate=1)
        self.vol = TSDFVolume.from_grid(origin, voxel_size, dims, self.intr, self.fopt, device=self.device, shard=shard)
        self.vol.with_color = with_color
        self.graph = EDGraph(seq.nodes, seq.edges, seq.edge_weights, node_coverage=seq.node_coverage)
        self.wf = WarpField(self.graph, self.vol)
        self.nodes_t = torch.from_numpy(seq.nodes).to(self.device)
        self.edges_t = torch.from_numpy(seq.edges).to(self.device)
        self.ew_t = torch.from_numpy(seq.edge_weights).to(self.device)
        self.n_matches = n_matches
        self.solver = GaussNewtonSolver(seq.nodes.shape[0], n_matches, self.device, **(gn_params or {}))
        self.prev_rot = None
        self.prev_trans = None
        self.last = None
        # overlap=True: frame t's integrate runs on a stream of its own, ordered after frame t's solve but not before
        # frame t+1's — the next solve needs frame t's transforms, not its volume (bit for bit the sequential result;
        # a caller reading the volume synchronises the device, not only its own stream)
        self.overlap = overlap
        self.int_stream = None

    def prepare(self, t):
        """Host-side synthetic inputs of frame t -> device (outside any timed region)."""
        d = self.device
        src, tgt, tpos, conf = self.seq.solver_inputs(t, self.n_matches)
        a, w, v = self.wf.skin_device(src)
        keep = v
        return FrameInputs(im=torch.from_numpy(self.seq.frame(t)).to(d), src=torch.from_numpy(src).to(d)[keep],
                           anchors=a[keep], weights=w[keep], tgt=torch.from_numpy(tgt).to(d)[keep],
                           tpos=torch.from_numpy(tpos).to(d), conf=torch.from_numpy(conf).to(d))

    def integrate_source(self, fi):
        self.vol.integrate({"im": fi.im, "id": 0})
        self.wf.skin_tsdf_cache()

    def problem(self, fi):
        """Frame fi's GN problem as GaussNewtonSolver.optimize(prefetch=) takes it."""
        return dict(graph_nodes=self.nodes_t, graph_edges=self.edges_t, graph_edges_weights=self.ew_t,
                    target_node_position=fi.tpos, node_confidence=fi.conf, source_points=fi.src, anchors=fi.anchors,
                    weights=fi.weights, target_points=fi.tgt)

    def solve(self, fi, next_fi=None):
        """GN solve of frame fi; next_fi: the next frame, whose solver setup is prefetched concurrently. Frame fi's
        depth/colour unpacking for its integrate is enqueued first (TSDFVolume.stage), so the host work between the
        solve's return and the integrate launch is only the integrate's own."""
        self.vol.stage(fi.im)
        out = self.solver.optimize(self.nodes_t, self.edges_t, self.ew_t, fi.tpos, fi.conf, fi.src, fi.anchors,
                                   fi.weights, fi.tgt, self.intr, prev_rot=self.prev_rot, prev_trans=self.prev_trans,
                                   sync=False, prefetch=None if next_fi is None else self.problem(next_fi))
        self.prev_rot, self.prev_trans = out["node_rotations"], out["node_translations"]
        return out

    def integrate(self, fi, t, count_updates=False, after=None):
        """Frame t's warp + integrate. overlap=True: on the pipeline's integrate stream, ordered after frame t's solve,
        and enqueued by the host inside the NEXT solve (GaussNewtonSolver.defer_to_next_solve: while that solve's host
        loop waits for its first PCG chunk), so the host work of the enqueue no longer sits between two solves;
        flush() runs a pending one now. after(): more work for that stream, right after the integrate. Returns a list
        that gets the integrate's (start, end) timing events once it is enqueued (overlap) or None."""
        if not (self.overlap and self.device.type == "cuda"):
            self._integrate(fi, t, count_updates)
            if after is not None:
                after()
            return None
        if self.int_stream is None:
            self.int_stream = torch.cuda.Stream(self.device)
        s = self.int_stream
        solved = torch.cuda.Event()
        solved.record()   # (the solve's stream: frame t's transforms are final here)
        staged, self.vol._staged = getattr(self.vol, "_staged", None), None   # (frame t's unpacked depth / colour)
        R, T = self.prev_rot, self.prev_trans
        events = []

        def enqueue():
            s.wait_event(solved)
            for x in (R, T) + (tuple(staged[1:]) if staged is not None else ()):
                if isinstance(x, torch.Tensor) and x.is_cuda:
                    x.record_stream(s)   # (made on the solve's stream: kept from reuse until the integrate has run)
            cur = getattr(self.vol, "_staged", None)
            self.vol._staged = staged
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record()
                self.wf.set_node_transforms(R, T)
                self.wf.frame_id = t
                self.vol.update(fi.im, t)
                self.vol.integrate_device(count_updates=count_updates)
                e1.record()
                if after is not None:
                    after()
            self.vol._staged = cur
            events.extend((e0, e1))

        self.solver.defer_to_next_solve(enqueue)
        return events

    def flush(self):
        """Enqueue a deferred (overlapped) integrate now: before reading the volume or timing the loop's end."""
        self.solver.flush_deferred()

    def _integrate(self, fi, t, count_updates=False):
        self.wf.set_node_transforms(self.prev_rot, self.prev_trans)
        self.wf.frame_id = t
        self.vol.update(fi.im, t)
        self.vol.integrate_device(count_updates=count_updates)

    def step(self, fi, t, count_updates=False, next_fi=None):
        self.last = self.solve(fi, next_fi)
        self.integrate(fi, t, count_updates)
        return self.last
