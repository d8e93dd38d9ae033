"""Synthetic depth sequences and deformation graphs for benches and tests.

Pinhole 640x480, fx=fy=525, cx=319.5, cy=239.5, centre-cropped to 640x448 as the reference frame
loader does (cy -= 16; options.py:13-14, utils/image_proc.py:303-311). Depth in metres (f32),
1 mm Gaussian noise, quantised to 1 mm. Scene: sphere R=0.35 m at (0,0,1.4) in front of a
1.6x1.2 m backing plane at z=1.75 (the survey's 0.6x0.6 m plane is fully hidden by the sphere
silhouette, so it is enlarged). Non-rigid motion: the sphere breathes (radius) and drifts (centre);
the plane is static. Occlusion (BASELINE config 3): a vertical bar (0.14 m wide, z=0.9 m)
enters from the left after frame 0 and sweeps over the sphere and back (up to ~30 % of the sphere's
pixels hidden); matches come only from surface points visible in the target frame, and the motion
term confidence is 1 for visible nodes, 0.3 for occluded ones.

Graphs (config_sequence): the reference's create_graph_from_depth
(embedded_deformation_graph.py:95-256) on the source frame, on the device — backprojected depth ->
compute_mesh_from_depth (max triangle distance 0.05) -> erode_mesh -> sample_nodes (no shuffle) -> 8 geodesic
edges -> node_and_edge_clean_up + reduced graph (EDGraph.from_mesh: csrc-pinned kernels), with the node coverage
tuned per config to its node count (BASELINE_CONFIGS[c]["coverage"]). SyntheticSequence.build's default
(graph="euclidean", kept for the tuning tools) is a greedy coverage sampler of surface points (the rule of csrc
sample_nodes, csrc/cpu/graph_proc.cpp:79-136, with a spatial hash instead of the O(N²) scan) with 8 Euclidean
nearest-node edges (csrc compute_edges_euclidean semantics, graph_proc.cpp:302-356).
"""
import math
from dataclasses import dataclass

import numpy as np


@dataclass
class Intrinsics:
    fx: float
    fy: float
    cx: float
    cy: float
    width: int
    height: int

    def as_vec(self):
        return np.array([self.fx, self.fy, self.cx, self.cy], np.float64)


def bench_camera(scale=1):
    """640x480 -> 640x448 crop; scale=2 gives the 320x240 (-> 320x224) camera of config 1."""
    return Intrinsics(525.0 / scale, 525.0 / scale, 319.5 / scale, (239.5 - 16) / scale, 640 // scale, 448 // scale)


def _axis_angle(axis, theta):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(theta) * K + (1.0 - math.cos(theta)) * (K @ K)


@dataclass
class SphereScene:
    """motion="nonrigid" (BASELINE configs 3-5): the sphere breathes and drifts, the plane is static.
    motion="rigid" (config 2): sphere + plane move as one rigid body about the sphere centre, at most
    1.5° of rotation and 1 cm of translation per frame (≤2°, ≤1 cm)."""
    center: tuple = (0.0, 0.0, 1.4)
    radius: float = 0.35
    plane_z: float = 1.75
    plane_half: tuple = (0.8, 0.6)
    occluder: bool = True
    occ_z: float = 0.9
    occ_half: float = 0.07
    motion: str = "nonrigid"
    phase: float = 0.0          # time offset of the non-rigid motion and the occluder sweep (independent scenes)

    @staticmethod
    def variant(seed):
        """An independent non-rigid scene with the occluder (BASELINE config 5: one scene per GPU): sphere centre,
        radius, occluder depth and motion phase drawn from the seed; the same size class as config 3."""
        rng = np.random.default_rng(seed)
        return SphereScene(center=(float(rng.uniform(-0.08, 0.08)), float(rng.uniform(-0.06, 0.06)),
                                   float(rng.uniform(1.3, 1.5))),
                           radius=float(rng.uniform(0.3, 0.38)), occ_z=float(rng.uniform(0.8, 1.0)),
                           phase=float(rng.uniform(0.0, 30.0)))

    def occluder_x(self, t):
        """x centre of the occluding bar at frame t: out of view at t=0, over the sphere for t≈8..24."""
        return -0.75 + 0.375 * (1.0 - math.cos(0.2 * (t + self.phase)))

    def rigid_pose(self, t):
        """(R_t, T_t): canonical (frame-0) point p -> R_t (p - c0) + c0 + T_t. R_0 = I, T_0 = 0."""
        theta = math.radians(10.0) * math.sin(0.15 * t)          # |dθ/dt| <= 1.5° per frame
        R = _axis_angle((0.3, 1.0, 0.2), theta)

        def tr(s):
            return np.array([0.05 * math.sin(0.12 * s), 0.03 * math.sin(0.15 * s + 0.5), 0.04 * math.sin(0.1 * s)])
        return R, tr(t) - tr(0)                                     # |dT/dt| <= 0.9 cm per frame

    def frame_params(self, t):
        """Sphere centre/radius at frame t (smooth non-rigid drift + breathing; rigid: translated centre)."""
        c = np.array(self.center, np.float64)
        if self.motion == "rigid":
            return c + self.rigid_pose(t)[1], self.radius
        s = t + self.phase
        c = c + np.array([0.01 * math.sin(0.3 * s), 0.008 * math.sin(0.2 * s + 1.0), 0.012 * math.sin(0.25 * s)])
        r = self.radius * (1.0 + 0.03 * math.sin(0.35 * s))
        return c, r

    def deform_points(self, pts, t):
        """Ground-truth motion of canonical (frame-0) surface points to frame t."""
        pts = np.asarray(pts, np.float64)
        if self.motion == "rigid":
            R, T = self.rigid_pose(t)
            c0 = np.array(self.center, np.float64)
            return (pts - c0) @ R.T + c0 + T
        c0, r0 = self.frame_params(0)
        c, r = self.frame_params(t)
        out = pts.copy()
        on_sphere = pts[:, 2] < self.plane_z - 0.02
        out[on_sphere] = c + (r / r0) * (pts[on_sphere] - c0)
        return out

    def render(self, cam, t=0, rng=None, noise=0.001):
        H, W = cam.height, cam.width
        u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
        dx = (u - cam.cx) / cam.fx
        dy = (v - cam.cy) / cam.fy
        if self.motion == "rigid":
            return self._render_rigid(dx, dy, t, rng, noise)
        c, r = self.frame_params(t)
        # sphere: |z*(dx,dy,1) - c|^2 = r^2
        a = dx * dx + dy * dy + 1.0
        b = -2.0 * (dx * c[0] + dy * c[1] + c[2])
        cc = c @ c - r * r
        disc = b * b - 4 * a * cc
        zs = np.where(disc >= 0, (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a), np.inf)
        zp = np.full_like(dx, self.plane_z)
        inplane = (np.abs(dx * self.plane_z) <= self.plane_half[0]) & (np.abs(dy * self.plane_z) <= self.plane_half[1])
        zp = np.where(inplane, zp, np.inf)
        z = np.minimum(zs, zp)
        if self.occluder:
            xo = self.occluder_x(t)
            hit = np.abs(dx * self.occ_z - xo) <= self.occ_half
            z = np.where(hit, np.minimum(z, self.occ_z), z)
        return self._finish(z, rng, noise)

    def _finish(self, z, rng, noise):
        if rng is not None and noise > 0:
            z = z + rng.normal(0.0, noise, z.shape)
        z = np.where(np.isfinite(z), np.round(z * 1000.0) / 1000.0, 0.0)
        return z.astype(np.float32)

    def _render_rigid(self, dx, dy, t, rng, noise):
        """Ray cast of the rigidly moved sphere + plane: rays z·(dx, dy, 1) taken into the canonical frame
        (q = R_tᵀ (p - c0 - T_t) + c0 = z·R_tᵀ d + o) and intersected with the canonical scene."""
        R, T = self.rigid_pose(t)
        c0 = np.array(self.center, np.float64)
        o = c0 - R.T @ (c0 + T)
        d = np.stack([dx, dy, np.ones_like(dx)], -1) @ R          # rows: R_tᵀ d
        oc = o - c0
        a = (d * d).sum(-1)
        b = 2.0 * (d @ oc)
        cc = oc @ oc - self.radius ** 2
        disc = b * b - 4 * a * cc
        zs = np.where(disc >= 0, (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a), np.inf)
        with np.errstate(divide="ignore", invalid="ignore"):
            zp = (self.plane_z - o[2]) / d[..., 2]
        qx, qy = o[0] + zp * d[..., 0], o[1] + zp * d[..., 1]
        inplane = (zp > 0) & (np.abs(qx) <= self.plane_half[0]) & (np.abs(qy) <= self.plane_half[1])
        z = np.minimum(zs, np.where(inplane, zp, np.inf))
        if self.occluder:
            hit = np.abs(dx * self.occ_z - self.occluder_x(t)) <= self.occ_half
            z = np.where(hit, np.minimum(z, self.occ_z), z)
        return self._finish(z, rng, noise)


def backproject(depth, cam):
    """depth_2_pc (NonRigidICP/model/geometry.py:44-59) for valid pixels -> (P,3) f32."""
    H, W = depth.shape
    u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    m = depth > 0
    z = depth[m].astype(np.float64)
    X = (u[m] - cam.cx) * z / cam.fx
    Y = (v[m] - cam.cy) * z / cam.fy
    return np.stack([X, Y, z], 1).astype(np.float32)


def make_image(depth, rgb=None):
    """(6,H,W) f32 image as the reference frame loader builds it: rgb in [0,1], then points (X,Y,Z)."""
    H, W = depth.shape
    if rgb is None:
        yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing='ij')
        rgb = np.stack([xx, yy, 0.5 * (xx + yy)]).astype(np.float32)
    im = np.zeros((6, H, W), np.float32)
    im[:3] = rgb
    im[5] = depth
    return im


def sample_nodes(points, coverage, seed=0):
    """Greedy coverage sampling (csrc sample_nodes rule: a point becomes a node iff no node lies
    within `coverage`), visiting points in a seeded shuffled order, spatial-hash accelerated."""
    pts = np.asarray(points, np.float32)
    order = np.random.default_rng(seed).permutation(pts.shape[0])
    cell = float(coverage)
    c2 = float(coverage) ** 2
    grid = {}
    nodes = []
    keys = np.floor(pts / cell).astype(np.int64)
    for idx in order:
        p = pts[idx]
        k = keys[idx]
        ok = True
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                for dz in (-1, 0, 1):
                    for q in grid.get((k[0] + dx, k[1] + dy, k[2] + dz), ()):
                        d = p - nodes[q]
                        if float(d @ d) <= c2:
                            ok = False
                            break
                    if not ok:
                        break
                if not ok:
                    break
            if not ok:
                break
        if ok:
            grid.setdefault((k[0], k[1], k[2]), []).append(len(nodes))
            nodes.append(p)
    return np.array(nodes, np.float32).reshape(-1, 3)


def euclidean_edges(nodes, k=8):
    """k nearest other nodes (ascending distance), -1 padded; uniform edge weights 1/k."""
    nodes = np.asarray(nodes, np.float32)
    N = nodes.shape[0]
    kk = min(k, N - 1)
    edges = -np.ones((N, k), np.int32)
    for s in range(0, N, 2048):
        d = ((nodes[s:s + 2048, None, :] - nodes[None]) ** 2).sum(-1)
        d[np.arange(d.shape[0]), np.arange(s, s + d.shape[0])] = np.inf
        if kk > 0:
            idx = np.argsort(d, axis=1, kind='stable')[:, :kk]
            edges[s:s + d.shape[0], :kk] = idx
    w = np.where(edges >= 0, 1.0 / k, 0.0).astype(np.float32)
    return edges, w


def depth_graph(depth, cam, coverage, device=None, max_triangle_distance=0.05, n_neighbours=8):
    """SURVEY §8(d) graph of one depth frame on the device: the reference's create_graph_from_depth
    (embedded_deformation_graph.py:95-256) — backproject_depth (csrc/cpu/image_proc.cpp:351-401),
    compute_mesh_from_depth (image_proc.cpp:405-545), then EDGraph.from_mesh (erode_mesh, sample_nodes without
    shuffle, compute_edges_geodesic, node_and_edge_clean_up + get_reduced_graph, compute_clusters;
    graph_proc.cpp:17-481). -> (nodes (N,3) f32, edges (N,K) i32, edge weights (N,K) f32)."""
    import torch
    from .image_proc import backproject_depth_device, compute_mesh_from_depth_device
    from .warpfield import EDGraph
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    d = torch.from_numpy(np.ascontiguousarray(depth, np.float32)).to(dev)
    pimg = backproject_depth_device(d, cam.fx, cam.fy, cam.cx, cam.cy)
    mesh = compute_mesh_from_depth_device(pimg, max_triangle_distance, with_pixels=False)
    g = EDGraph.from_mesh(mesh["vertices"], mesh["faces"],
                          {"node_coverage": float(coverage), "num_neighbours": int(n_neighbours),
                           "max_triangle_distance": float(max_triangle_distance)}, device=dev)
    return (np.ascontiguousarray(g.nodes, np.float32), np.ascontiguousarray(g.edges, np.int32),
            np.ascontiguousarray(g.edges_weights, np.float32))


def coverage_for_nodes(points, target_nodes, seed=0, iters=8):
    """Bisection on node coverage to hit ~target_nodes."""
    lo, hi = 0.002, 0.5
    sub = points[np.random.default_rng(seed).permutation(points.shape[0])[:60000]]
    best = None
    for _ in range(iters):
        mid = math.sqrt(lo * hi)
        n = sample_nodes(sub, mid, seed).shape[0]
        best = mid
        if n > target_nodes:
            lo = mid
        else:
            hi = mid
    return best


def frame_depth(scene, cam, seed, t):
    """Depth of frame t of the seeded sequence (noise stream seed·1000 + t)."""
    return scene.render(cam, t, np.random.default_rng(seed * 1000 + t))


def source_depth(scene, cam, seed):
    """The source frame's depth (frame 0): the canonical surface, and what the depth-mesh graph is built on."""
    return frame_depth(scene, cam, seed, 0)


@dataclass
class SyntheticSequence:
    """A seeded sequence: frames, canonical surface, graph and per-frame solver inputs."""
    cam: Intrinsics
    scene: SphereScene
    nodes: np.ndarray
    edges: np.ndarray
    edge_weights: np.ndarray
    node_coverage: float
    canonical_points: np.ndarray
    seed: int = 0

    @staticmethod
    def build(n_nodes=2000, cam=None, seed=3, coverage=None, scene=None, graph="euclidean", device=None):
        """scene: SphereScene() (non-rigid with the occluder, configs 3-5) unless given, e.g.
        SphereScene(motion="rigid", occluder=False) for config 2.
        graph: "euclidean" — greedy sampling of a 60k-point subset of a noisy frame-0 render (coverage bisected to
        n_nodes) + 8 Euclidean edges; "geodesic" — depth_graph() of the source frame (frame 0, as fused) on
        `device` with the given coverage; or a given (nodes, edges, edge_weights) triple built
        from the source frame the same way (coverage given; e.g. the reference's compiled C++ in the CPU fixture
        generator). The matches are drawn from the canonical points: the backprojected source frame."""
        cam = cam or bench_camera()
        scene = scene or SphereScene()
        if isinstance(graph, str) and graph == "euclidean":
            d0 = scene.render(cam, 0, np.random.default_rng(seed))
            pts = backproject(d0, cam)
            cov = coverage if coverage is not None else coverage_for_nodes(pts, n_nodes, seed)
            sub = pts[np.random.default_rng(seed).permutation(pts.shape[0])[:60000]]
            nodes = sample_nodes(sub, cov, seed)
            edges, ew = euclidean_edges(nodes, 8)
            return SyntheticSequence(cam, scene, nodes, edges, ew, float(cov), pts, seed)
        if coverage is None:
            raise ValueError("a depth-mesh graph needs its node coverage")
        d0 = source_depth(scene, cam, seed)
        if isinstance(graph, str):
            if graph != "geodesic":
                raise ValueError(f"unknown graph kind {graph!r}")
            nodes, edges, ew = depth_graph(d0, cam, coverage, device)
        else:
            nodes, edges, ew = (np.ascontiguousarray(graph[0], np.float32), np.ascontiguousarray(graph[1], np.int32),
                                np.ascontiguousarray(graph[2], np.float32))
        return SyntheticSequence(cam, scene, nodes, edges, ew, float(coverage), backproject(d0, cam), seed)

    def frame(self, t):
        return make_image(frame_depth(self.scene, self.cam, self.seed, t))

    def visible(self, pts_t, t, tol=0.01):
        """Points (already at frame t) seen by the camera in frame t: the noise-free rendered depth at
        their pixel is not in front of them by more than tol."""
        cam = self.cam
        z = pts_t[:, 2]
        u = np.rint(pts_t[:, 0] * cam.fx / z + cam.cx).astype(np.int64)
        v = np.rint(pts_t[:, 1] * cam.fy / z + cam.cy).astype(np.int64)
        inside = (z > 0) & (u >= 0) & (u < cam.width) & (v >= 0) & (v < cam.height)
        d = self.scene.render(cam, t)
        dv = np.zeros_like(z)
        dv[inside] = d[v[inside], u[inside]]
        return inside & (dv > 0) & (dv >= z - tol)

    def solver_inputs(self, t, n_matches=10000, occluded_conf=0.3):
        """Matches (canonical surface point visible in frame t -> its position at frame t + 1 mm noise)
        and node motion targets (ground-truth node motion, confidence 1 visible / occluded_conf for
        nodes that are back-facing or hidden by the occluder)."""
        rng = np.random.default_rng(self.seed * 7919 + t)
        cand = self.canonical_points
        pos_t = self.scene.deform_points(cand, t)
        vis = np.nonzero(self.visible(pos_t, t))[0] if self.scene.occluder else np.arange(cand.shape[0])
        sel = np.sort(rng.choice(vis, size=min(n_matches, vis.shape[0]), replace=False))
        src = cand[sel]
        tgt = pos_t[sel] + rng.normal(0, 0.001, src.shape)
        tpos = self.scene.deform_points(self.nodes, t)
        c, r = self.scene.frame_params(t)
        facing = (self.nodes[:, 2] < c[2]) | (self.nodes[:, 2] > self.scene.plane_z - 0.02)
        if self.scene.occluder:
            facing = facing & self.visible(tpos, t, tol=0.02)
        conf = np.where(facing, 1.0, occluded_conf).astype(np.float32)
        return src.astype(np.float32), tgt.astype(np.float32), tpos.astype(np.float32), conf


# BASELINE.json configs: volume dims / voxel size / origin, graph size, motion, occluder, camera
# scale (2: the 320x240 -> 320x224 camera of config 1), the sequence seed (= config index) and the node coverage of
# the depth-mesh graph that gives the config's node count (measured with the reference's compiled C++ on the
# source frame, tools/graph_coverage.py: 199 / 1020 / 1998 / 4016 nodes, 8 edges each).
BASELINE_CONFIGS = {
    1: dict(dims=128, voxel=0.008, origin=(-0.512, -0.512, 0.9), nodes=200, motion="nonrigid", occluder=False,
            cam_scale=2, seed=1, coverage=0.1),
    2: dict(dims=256, voxel=0.004, origin=(-0.512, -0.512, 0.9), nodes=1000, motion="rigid", occluder=False,
            cam_scale=1, seed=2, coverage=0.043),
    3: dict(dims=512, voxel=0.004, origin=(-1.024, -1.024, 0.5), nodes=2000, motion="nonrigid", occluder=True,
            cam_scale=1, seed=3, coverage=0.03),
    4: dict(dims=1024, voxel=0.002, origin=(-1.024, -1.024, 0.5), nodes=4000, motion="nonrigid", occluder=True,
            cam_scale=1, seed=4, coverage=0.0205),
}
# 8 independent config-3-class scenes, one per GPU: rank 0 is config 3 itself, rank r > 0 its own seeded scene
# (SphereScene.variant(5000 + r)) and noise stream (seed 5000 + r)
BASELINE_CONFIGS[5] = dict(BASELINE_CONFIGS[3])


def config_scene(config, rank=0):
    """(scene, seed) of BASELINE config `config`; config 5: rank r's independent scene."""
    c = BASELINE_CONFIGS[config]
    if config == 5 and rank > 0:
        return SphereScene.variant(5000 + rank), 5000 + rank
    return SphereScene(motion=c["motion"], occluder=c["occluder"]), c["seed"]


def config_coverage(config, n_nodes=None):
    """Node coverage of the config's depth-mesh graph; another node count scales it as 1/sqrt(nodes) (surface
    sampling)."""
    c = BASELINE_CONFIGS[config]
    cov = c["coverage"]
    if n_nodes and int(n_nodes) != c["nodes"]:
        cov = cov * math.sqrt(c["nodes"] / float(n_nodes))
    return cov


def config_sequence(config, n_nodes=None, rank=0, device=None, graph="geodesic"):
    """The seeded synthetic sequence of BASELINE config `config` (1..5; config 5: the scene of `rank`). Its graph
    is the SURVEY §8(d) depth-mesh graph of the source frame built on `device` (graph="geodesic"), a given
    (nodes, edges, edge_weights) triple of that graph (CPU fixture generators), or graph="euclidean"."""
    c = BASELINE_CONFIGS[config]
    scene, seed = config_scene(config, rank)
    cov = config_coverage(config, n_nodes) if not (isinstance(graph, str) and graph == "euclidean") else None
    return SyntheticSequence.build(n_nodes or c["nodes"], cam=bench_camera(c["cam_scale"]), seed=seed, scene=scene,
                                   coverage=cov, graph=graph, device=device)
