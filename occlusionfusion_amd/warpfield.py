"""WarpField + EDGraph — drop-ins for fusion_with_occlusion/warpfield.py and the state part of
embedded_deformation_graph.py, backed by libofx.

Transforms are kept node-relative on device (R_k, T_k with x' = R_k(x-g_k)+g_k+T_k, as
Registration.deform_ED applies them, registration_fusion.py:157-184). The reference's origin-form
`translations` (t = -R g + g + T, warpfield.py:407-408) are exposed as a derived property.
"""
import logging
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, ops  # noqa: F401  (ops registers torch.ops.ofx.*)
from ._lib import call, ptr, stream_ptr, byref

log = logging.getLogger(__name__)


DEFAULT_GRAPH_PARAMETERS = {   # embedded_deformation_graph.py:60-69 (graph_config.json defaults)
    "max_triangle_distance": 0.05, "erosion_num_iterations": 1, "erosion_min_neighbours": 3,
    "node_coverage": 0.05, "min_neighbours": 2, "num_neighbours": 8, "require_mask": True}


class EDGraph:
    """Embedded-deformation graph (embedded_deformation_graph.py:26-741): nodes (N,3) f32, edges (N,K) i32
    (-1 padded), edges_weights / edges_distances (N,K) f32, clusters (N,1) i32, node_indices (N,1) and the
    graph_generation_parameters dict. Built either from given arrays (the hot-path state) or from a mesh /
    a TSDFVolume (EDGraph.from_mesh / from_tsdf) with the device graph-construction kernels (graph_proc)."""

    def __init__(self, nodes, edges, edges_weights=None, clusters=None, node_coverage=0.05, graph_neighbours=8):
        self.log = log
        self.nodes = np.ascontiguousarray(nodes, np.float32)
        self.edges = np.ascontiguousarray(edges, np.int32)
        N = self.nodes.shape[0]
        self.edges_weights = (np.ascontiguousarray(edges_weights, np.float32) if edges_weights is not None
                              else np.where(self.edges >= 0, 1.0 / max(1, self.edges.shape[1]), 0).astype(np.float32))
        self.edges_distances = np.zeros(self.edges.shape, np.float32)
        self.clusters = (np.asarray(clusters, np.int32).reshape(N, 1) if clusters is not None
                         else np.zeros((N, 1), np.int32))
        self.node_indices = -np.ones((N, 1), np.int32)
        self.num_nodes = N
        self.graph_generation_parameters = dict(DEFAULT_GRAPH_PARAMETERS, node_coverage=float(node_coverage),
                                                num_neighbours=int(graph_neighbours), graph_neighbours=int(graph_neighbours),
                                                erosion_num_iterations=10, erosion_min_neighbours=4)

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_mesh(cls, vertices, faces, graph_generation_parameters=None, device=None, with_pyramid=False):
        """create_graph_from_mesh (embedded_deformation_graph.py:174-256) on the device."""
        g = cls.__new__(cls)
        g.log = log
        g.graph_generation_parameters = dict(DEFAULT_GRAPH_PARAMETERS, **(graph_generation_parameters or {}))
        g.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        g.create_graph_from_mesh(vertices, faces, with_pyramid=with_pyramid)
        return g

    @classmethod
    def from_tsdf(cls, tsdf, graph_generation_parameters=None, with_pyramid=False):
        """create_graph_from_tsdf (embedded_deformation_graph.py:80-86): graph of the TSDF's marching-cubes mesh."""
        g = cls.from_mesh(*tsdf.get_mesh()[:2], graph_generation_parameters, tsdf.device, with_pyramid)
        g.tsdf = tsdf
        tsdf.graph = g
        return g

    def erode_mesh(self, vertices, faces, num_iterations=-1):
        """embedded_deformation_graph.py:153-172 — any non-zero num_iterations is replaced by the configured
        erosion_num_iterations (the reference's `if num_iterations:`). -> non-eroded mask (V,1) bool."""
        from .graph_proc import MeshGraph
        if num_iterations:
            num_iterations = self.graph_generation_parameters["erosion_num_iterations"]
        mg = MeshGraph(vertices, faces, getattr(self, "device", None))
        return mg.erode(num_iterations, self.graph_generation_parameters["erosion_min_neighbours"]).cpu().numpy()[:, None]

    def create_graph_from_mesh(self, vertices, faces, with_pyramid=False):
        from .graph_proc import MeshGraph
        p = self.graph_generation_parameters
        cov, K = float(p["node_coverage"]), int(p["num_neighbours"])
        mg = MeshGraph(vertices, faces, getattr(self, "device", None))
        assert mg.nv > 0 and mg.nf > 0
        ne = mg.erode(p["erosion_num_iterations"], p["erosion_min_neighbours"])   # erode_mesh(num_iterations=-1)
        pos, idx = mg.sample_nodes(ne, cov, True)
        E, W, D, _ = mg.edges_geodesic(idx, K, cov, True, True)                      # visible_vertices = all ones
        self._mesh = mg
        self.vertices = mg.vertices.cpu().numpy()
        self.faces = mg.faces.cpu().numpy()
        self.nodes = pos.cpu().numpy()
        self.node_indices = idx.cpu().numpy().reshape(-1, 1)
        self.edges, self.edges_weights, self.edges_distances = E.cpu().numpy(), W.cpu().numpy(), D.cpu().numpy()
        self.clusters = -np.ones((self.edges.shape[0], 1), np.int32)
        self.remove_nodes_with_not_enough_neighbours()
        self.compute_clusters()
        if with_pyramid:
            self.create_graph_pyramid()

    def remove_nodes_with_not_enough_neighbours(self):
        """embedded_deformation_graph.py:330-369 (node_and_edge_clean_up + get_reduced_graph)."""
        from .graph_proc import node_edge_cleanup_device
        dev = self._dev()
        E = torch.from_numpy(self.edges).to(dev)
        valid = node_edge_cleanup_device(E, torch.ones(E.shape[0], dtype=torch.bool, device=dev))
        r = self.get_reduced_graph(valid.cpu().numpy().reshape(-1, 1))
        self.nodes, self.edges = r["valid_nodes_at_source"], r["graph_edges"]
        self.edges_weights, self.edges_distances = r["graph_edges_weights"], r["graph_edges_distances"]
        self.clusters, self.num_nodes = r["graph_clusters"], int(r["num_nodes"])
        self.node_indices = self.node_indices[r["valid_nodes_mask"].reshape(-1)]

    def _dev(self):
        return getattr(self, "device", None) or torch.device("cuda", torch.cuda.current_device())

    def get_reduced_graph(self, valid_nodes_mask):
        """embedded_deformation_graph.py:382-477 on the device (ofx_reduce_graph)."""
        dev = self._dev()
        m = np.asarray(valid_nodes_mask).reshape(-1).astype(bool)
        N, K = self.edges.shape
        kw = dict(device=dev)
        vm = torch.from_numpy(m.astype(np.uint8)).to(dev)
        src = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
               (self.nodes, self.edges, self.edges_weights, self.edges_distances, self.clusters.reshape(-1))]
        out = [torch.empty((N, 3), dtype=torch.float32, **kw), torch.empty((N, K), dtype=torch.int32, **kw),
               torch.empty((N, K), dtype=torch.float32, **kw), torch.empty((N, K), dtype=torch.float32, **kw),
               torch.empty(N, dtype=torch.int32, **kw)]
        n = _lib.c_int32()
        call("ofx_reduce_graph", ptr(vm), N, K, *[ptr(t) for t in src], *[ptr(t) for t in out], byref(n), stream_ptr())
        k = int(n.value)
        if k == 0:
            raise RuntimeError("No nodes! (embedded_deformation_graph.py:399-401)")
        nodes, E, W, D, C = (t[:k].cpu().numpy() for t in out)
        self.log.info(f"Node filtering: initial num nodes: {k} | invalid nodes: {N - k}")
        return {"all_nodes_at_source": self.nodes.copy(), "valid_nodes_at_source": nodes, "graph_edges": E,
                "graph_edges_weights": W, "graph_edges_distances": D, "graph_clusters": C.reshape(-1, 1),
                "num_nodes": np.array(k, dtype=np.int64), "valid_nodes_mask": m.reshape(-1, 1)}

    def compute_clusters(self):
        """embedded_deformation_graph.py:371-380."""
        from .graph_proc import clusters_device
        cl, sizes = clusters_device(torch.from_numpy(self.edges).to(self._dev()))
        self.clusters = cl.cpu().numpy().reshape(-1, 1)
        for i, sz in enumerate(sizes):
            if sz <= 2:
                self.log.error(f"Cluster is too small {sizes}")
                self.log.error(f"It only has nodes:{np.where(self.clusters == i)[0]}")
        return sizes

    def create_graph_pyramid(self):
        """embedded_deformation_graph.py:261-328 (input of the OcclusionFusion motion-completion network):
        greedy down-sampling at doubled coverage per level (ofx_graph_downsample: numpy's f32 norms and argmin
        order), geodesic edges of the kept nodes over the mesh, all on the device."""
        from .graph_proc import MeshGraph, downsample_device
        cov = float(self.graph_generation_parameters["node_coverage"])
        mg = getattr(self, "_mesh", None) or MeshGraph(self.vertices, self.faces, self._dev())
        pyd = {"nn_index_l0": self.edges}
        old_nodes, idx = self.nodes, self.node_indices
        for level, k in zip(range(1, 4), (6, 4, 3)):
            cov *= 2
            down, up = downsample_device(old_nodes, cov, self._dev())   # the reference's greedy loop, on device
            idx = idx[down]
            E, _, _, _ = mg.edges_geodesic(idx.reshape(-1), k, cov, False, True)
            pyd[f"down_sample_idx{level}"] = down
            pyd[f"up_sample_idx{level}"] = up
            pyd[f"nn_index_l{level}"] = E.cpu().numpy()
            old_nodes = old_nodes[down]
        self.pyd = pyd
        return pyd

    def get_graph_pyramid(self):
        return self.pyd

    def update(self, canonical_model_vertices, canonical_model_faces, new_verts_indices, plot_update=False):
        """embedded_deformation_graph.py:496-609: add nodes at uncovered vertices (greedy, coverage apart,
        numpy f32 norms as the reference), re-anchor every node to its nearest canonical vertex, rebuild the
        geodesic edges on the device, clean up, cluster. Returns whether nodes were added."""
        from .graph_proc import MeshGraph, knn_device
        if len(new_verts_indices) == 0:
            return False
        cov = float(self.graph_generation_parameters["node_coverage"])
        V = np.ascontiguousarray(canonical_model_vertices, np.float32)
        new = []
        for x in new_verts_indices:   # float(): numpy 1.26 (environment.yml:94) compares f32 scalar vs float in f64
            if float(np.min(np.linalg.norm(self.nodes - V[x], axis=1))) < cov:
                continue
            if new and float(np.min(np.linalg.norm(V[new] - V[x], axis=1))) < cov:
                continue
            new.append(x)
        if not new:
            return False
        self.nodes = np.concatenate([self.nodes, V[new]], axis=0)
        dev = self._dev()
        # node_indices = argmin over vertices of |node - vertex| (calculate_distance_matrix, :491-501)
        idx, _ = knn_device(torch.from_numpy(self.nodes).to(dev), torch.from_numpy(V).to(dev), 1)
        self.node_indices = idx.cpu().numpy().reshape(-1, 1)
        K = int(self.graph_generation_parameters["num_neighbours"])
        mg = MeshGraph(V, canonical_model_faces, dev)
        E, W, D, _ = mg.edges_geodesic(self.node_indices.reshape(-1), K, cov, True, True)
        self._mesh = mg
        self.vertices, self.faces = V, np.asarray(canonical_model_faces)
        self.edges, self.edges_weights, self.edges_distances = E.cpu().numpy(), W.cpu().numpy(), D.cpu().numpy()
        self.clusters = -np.ones((self.edges.shape[0], 1), np.int32)
        self.remove_nodes_with_not_enough_neighbours()
        self.compute_clusters()
        return True

    # ---------------------------------------------------------------- on-disk formats (utils/utils.py:205-383)
    def save(self, directory, name="graph"):
        """Graph arrays in the reference's .bin formats (utils/utils.py save_graph_*)."""
        from . import formats
        import os
        os.makedirs(directory, exist_ok=True)
        formats.save_graph_nodes(os.path.join(directory, f"{name}_nodes.bin"), self.nodes)
        formats.save_graph_edges(os.path.join(directory, f"{name}_edges.bin"), self.edges)
        formats.save_graph_edges_weights(os.path.join(directory, f"{name}_edges_weights.bin"), self.edges_weights)
        formats.save_graph_clusters(os.path.join(directory, f"{name}_clusters.bin"), self.clusters)

    @classmethod
    def load(cls, directory, name="graph", node_coverage=0.05):
        from . import formats
        import os
        nodes = formats.load_graph_nodes(os.path.join(directory, f"{name}_nodes.bin"))
        edges = formats.load_graph_edges(os.path.join(directory, f"{name}_edges.bin"))
        w = formats.load_graph_edges_weights(os.path.join(directory, f"{name}_edges_weights.bin"))
        cl = formats.load_graph_clusters(os.path.join(directory, f"{name}_clusters.bin"))
        return cls(nodes, edges, w, cl, node_coverage=node_coverage, graph_neighbours=edges.shape[1])


@dataclass
class SkinCache:
    brick_list: torch.Tensor   # int32 [n_list] shard-local brick ids
    n_list: int
    anchors: torch.Tensor      # uint16 as int16 storage [n_list*512*4]
    weights: torch.Tensor      # f32 [n_list*512*4]
    k: int
    pal_ids: torch.Tensor = None   # int16 storage of u16 [n_list*PALETTE] node palette per brick
    pal_n: torch.Tensor = None     # int32 [n_list] distinct anchors per brick (> PALETTE: overflow)
    local: torch.Tensor = None     # uint8 [n_list*512*4] anchors as palette ranks (0xFF invalid)


def _t(x, device, dtype):
    if isinstance(x, torch.Tensor):
        if x.dtype == dtype and x.device == device and x.is_contiguous():
            return x   # per-frame fast path (host time: no .to / .contiguous dispatch)
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


class WarpField:
    """Warp field over an EDGraph and a TSDFVolume (warpfield.py:21-604)."""

    def __init__(self, graph, tsdf, visualizer=None, kdtree_leaf_size=16):
        self.graph = graph
        self.tsdf = tsdf
        self.vis = visualizer
        self.device = tsdf.device
        src = getattr(tsdf.fopt, "source_frame", 0) if not isinstance(tsdf.fopt, dict) else tsdf.fopt.get("source_frame", 0)
        self.frame_id = src
        self.log = log
        self.updating_warpfield = False
        self.use_pytorch = True      # warpfield.py:75: deform() -> deform_ED; False -> origin-form deform_lbs
        self._set_graph(graph)
        tsdf.warpfield = self

    def _set_graph(self, graph):
        N = graph.nodes.shape[0]
        self.num_nodes = N
        self.graph_neighbours = min(N, 4)                                   # warpfield.py:60
        self.node_coverage = float(graph.graph_generation_parameters["node_coverage"])
        self.nodes_t = _t(graph.nodes, self.device, torch.float32)
        self.R_t = torch.eye(3, device=self.device).repeat(N, 1, 1).contiguous()
        self.T_t = torch.zeros((N, 3), device=self.device)
        self.deformed_nodes = graph.nodes.copy()
        self._packed = None
        self._cache = None

    # ------------------------------------------------------------------ transforms
    @property
    def rotations(self):
        return self.R_t.cpu().numpy()

    @property
    def translations(self):
        """Origin form t = -R g + g + T (warpfield.py:407-408)."""
        R, T, g = self.R_t.double(), self.T_t.double(), self.nodes_t.double()
        return (-(R @ g.unsqueeze(-1)).squeeze(-1) + g + T).float().cpu().numpy()

    def set_node_transforms(self, R, T):
        """Node-relative rotations (N,3,3) and translations (N,3), device or host."""
        self.R_t = _t(R, self.device, torch.float32).reshape(self.num_nodes, 3, 3)
        self.T_t = _t(T, self.device, torch.float32).reshape(self.num_nodes, 3)
        self._packed = None

    def packed_nodes(self):
        """(N,16) f32 device rows [R | t | g] of the current transforms (ofx_pack_nodes), repacked into one buffer
        kept across frames (stream-ordered after the previous frame's readers)."""
        if self._packed is None:
            buf = getattr(self, "_packed_buf", None)
            if buf is None or buf.shape[0] != self.num_nodes or buf.device != self.R_t.device:
                buf = torch.empty((self.num_nodes, 16), dtype=torch.float32, device=self.device)
                self._packed_buf = buf
            call("ofx_pack_nodes", ptr(self.R_t), ptr(self.T_t), ptr(self.nodes_t), self.num_nodes, ptr(buf),
                 stream_ptr())
            self._packed = buf
        return self._packed

    def update_transformations(self, nnrt_data):
        """warpfield.py:389-420: adopt the solver's node-relative (R, T); deformed nodes; frame id."""
        assert self.frame_id == self.tsdf.frame_id, \
            f"Warpfield maps to:{self.frame_id}th frame but TSDF maps to:{self.tsdf.frame_id}th frame"
        self.set_node_transforms(nnrt_data["node_rotations"], nnrt_data["node_translations"])
        dn = nnrt_data["deformed_nodes_to_target"]
        self.deformed_nodes = dn.detach().cpu().numpy() if isinstance(dn, torch.Tensor) else np.asarray(dn)
        self.frame_id = nnrt_data["target_frame_id"]

    def get_transformation_wrt_graph_node(self):
        """warpfield.py:422-436 -> (rotations, node-relative translations)."""
        return self.rotations, self.T_t.cpu().numpy()

    def get_transformation_wrt_origin(self, rotations, translations):
        """warpfield.py:438-449: translations + g - R g."""
        N = rotations.shape[0]
        g = self.graph.nodes[:N].astype(np.float64)
        return rotations, translations + g - np.einsum("nij,nj->ni", rotations, g)

    def get_deformed_nodes(self):
        assert self.frame_id == self.tsdf.frame_id
        return self.deformed_nodes

    # ------------------------------------------------------------------ skinning
    def skin_device(self, points, nodes=None):
        """Device skinning -> (anchors int32 (P,K), weights f32 (P,K), valid bool (P,)) tensors."""
        pts = _t(points, self.device, torch.float32).reshape(-1, 3)
        nd = self.nodes_t if nodes is None else _t(nodes, self.device, torch.float32).reshape(-1, 3)
        K = min(nd.shape[0], 4)
        return torch.ops.ofx.skin_points(pts, nd, float(self.node_coverage), K)

    def skin(self, points, nodes=None, ensure_num_neigbours=False):
        """warpfield.py:83-129 (numpy in, numpy out)."""
        a, w, v = self.skin_device(points, nodes)
        return a.cpu().numpy(), w.cpu().numpy(), v.cpu().numpy()

    def skin_image(self, nodes, image_data):
        """warpfield.py:143-199: mesh the (masked) point image (compute_mesh_from_depth), skin its vertices
        against `nodes` and scatter anchors / weights to the vertex pixels -> {"pixel_anchors" (H,W,K) i32,
        "pixel_weights" (H,W,K) f32}; pixels without a vertex hold 0 / 0 as in the reference."""
        from .image_proc import compute_mesh_from_depth_device
        self.source_im = image_data["im"]
        im = _t(image_data["im"], self.device, torch.float32)
        point_image = im[3:]
        if image_data.get("mask") is not None:
            m = _t(image_data["mask"], self.device, torch.float32)
            point_image = point_image * (m > 0).float()[None]
        mesh = compute_mesh_from_depth_device(point_image.contiguous(),
                                              self.graph.graph_generation_parameters["max_triangle_distance"])
        a, w, _ = self.skin_device(mesh["vertices"], nodes=nodes)
        H, W = point_image.shape[1:3]
        K = self.graph_neighbours
        pa = torch.zeros((H, W, K), dtype=torch.int32, device=self.device)
        pw = torch.zeros((H, W, K), dtype=torch.float32, device=self.device)
        px = mesh["vertex_pixels"].long()
        pa[px[:, 1], px[:, 0]] = a
        pw[px[:, 1], px[:, 0]] = w
        self.log.info(f"Skinned Source Image, valid pixels:{int((pa != -1).all(-1).sum())}")
        return {"pixel_anchors": pa.cpu().numpy(), "pixel_weights": pw.cpu().numpy()}

    def find_unreachable_nodes(self, points):
        """warpfield.py:462-485: indices of points farther than 2·node_coverage from every node, sorted by that
        distance descending (1-NN by ofx_knn_points; the reference's pykdtree distance rounding and argsort tie
        order are unpinned)."""
        from .graph_proc import knn_device
        pts = _t(points, self.device, torch.float32).reshape(-1, 3)
        _, d2 = knn_device(pts, self.nodes_t, 1)
        dist = torch.sqrt(d2.reshape(-1).double()).float()
        un = torch.nonzero(dist > np.float32(2 * self.node_coverage)).reshape(-1)
        if un.numel() == 0:
            return []
        order = torch.argsort(dist[un], stable=True).flip(0)
        return un[order].cpu().numpy()

    def update_graph(self, solver=None):
        """warpfield.py:487-582 (the reference's drivers keep this call commented out): add nodes where the eroded
        canonical model leaves the graph's coverage, re-skin the TSDF and estimate the new nodes' transforms by
        ARAP from the existing ones (run_model.py:448-627 -> DeformNet.arap on the device). The vertex subset /
        index quirk of the reference (indices into the non-eroded subset used on the full vertex array) is kept."""
        from .registration import GaussNewtonSolver, run_arap
        self.updating_warpfield = True
        verts, faces = self.tsdf.get_canonical_model()[:2]
        keep = self.graph.erode_mesh(verts, faces, num_iterations=3).reshape(-1)
        new_idx = self.find_unreachable_nodes(verts[keep])
        if len(new_idx) == 0:
            self.updating_warpfield = False
            return False
        old_n = self.graph.nodes.shape[0]
        R_old, T_old = self.R_t.cpu().numpy(), self.T_t.cpu().numpy()
        update = self.graph.update(verts, faces, new_idx)
        if update:
            N = self.graph.nodes.shape[0]
            self._set_graph(self.graph)
            self.skin_tsdf_cache()
            mask = np.zeros(N, bool)
            mask[:old_n] = True
            red = self.graph.get_reduced_graph(mask)
            td = {"source_frame_id": getattr(self.tsdf.fopt, "source_frame", 0), "target_frame_id": self.frame_id,
                  "node_rotations": R_old.astype(np.float32), "node_translations": T_old.astype(np.float32)}
            td["deformed_nodes_to_target"] = (self.graph.nodes[mask] + td["node_translations"]).astype(np.float32)
            solver = solver or GaussNewtonSolver(N, 1, self.device)
            est = run_arap(solver, red, td, self.graph, self.log)
            self.set_node_transforms(est["node_rotations"], est["node_translations"])
            self.deformed_nodes = est["deformed_nodes_to_target"]
        self.frame_id = self.tsdf.frame_id
        self.updating_warpfield = False
        return update

    def skin_tsdf_cache(self):
        """Bricked skin cache of the TSDF voxel grid (warpfield.py:131-141 cache semantics)."""
        if self._cache is None or self.updating_warpfield:
            t = self.tsdf
            K = self.graph_neighbours
            blist = torch.empty(max(1, t.n_bricks), dtype=torch.int32, device=self.device)
            cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
            call("ofx_skin_volume_bricks", byref(t.desc), ptr(self.nodes_t), self.num_nodes, self.node_coverage, K,
                 ptr(blist), ptr(cnt), stream_ptr())
            n_list = int(cnt.item())
            if t.owned_mask is not None:   # hash shard: only this rank's bricks (sharding.hash_owner)
                own = blist[:n_list][t.owned_mask[blist[:n_list].long()]]
                n_list = int(own.shape[0])
                blist = torch.zeros(max(1, t.n_bricks), dtype=torch.int32, device=self.device)
                blist[:n_list] = own
            anchors = torch.empty(max(1, n_list) * 512 * 4, dtype=torch.int16, device=self.device)
            weights = torch.empty(max(1, n_list) * 512 * 4, dtype=torch.float32, device=self.device)
            call("ofx_skin_volume", byref(t.desc), ptr(self.nodes_t), self.num_nodes, self.node_coverage, K, ptr(blist),
                 n_list, ptr(anchors), ptr(weights), stream_ptr())
            P = _lib.PALETTE
            pal_ids = torch.empty(max(1, n_list) * P, dtype=torch.int16, device=self.device)
            pal_n = torch.empty(max(1, n_list), dtype=torch.int32, device=self.device)
            local = torch.empty(max(1, n_list) * 512 * 4, dtype=torch.uint8, device=self.device)
            call("ofx_skin_palette", ptr(anchors), n_list, K, self.num_nodes, ptr(pal_ids), ptr(pal_n), ptr(local),
                 stream_ptr())
            self._cache = SkinCache(blist[:max(1, n_list)], n_list, anchors, weights, K, pal_ids, pal_n, local)
        return self._cache

    def skin_tsdf(self):
        """API parity: dense (V,K) anchors, weights and valid mask of the voxel grid (numpy)."""
        c = self.skin_tsdf_cache()
        t = self.tsdf
        V = (t.x_hi - t.x_lo) * int(t._vol_dim[1]) * int(t._vol_dim[2])
        a = torch.empty((V, c.k), dtype=torch.int32, device=self.device)
        w = torch.empty((V, c.k), dtype=torch.float32, device=self.device)
        v = torch.empty(V, dtype=torch.uint8, device=self.device)
        call("ofx_skin_volume_to_dense", byref(t.desc), ptr(c.brick_list), c.n_list, ptr(c.anchors), ptr(c.weights),
             c.k, ptr(a), ptr(w), ptr(v), stream_ptr())
        return a.cpu().numpy(), w.cpu().numpy(), v.cpu().numpy().astype(bool)

    # ------------------------------------------------------------------ deformation
    def deform_device(self, points, anchors, weights, valid=None, normals=False):
        pts = _t(points, self.device, torch.float32).reshape(-1, 3)
        a = _t(anchors, self.device, torch.int32)
        w = _t(weights, self.device, torch.float32)
        v = None if valid is None else _t(valid, self.device, torch.uint8)
        return torch.ops.ofx.deform_points(pts, a, w, v, self.packed_nodes(), bool(normals))

    def deform_lbs_device(self, node_rotations, node_translations, points, anchors, weights, valid_pts=None):
        """warpfield.py:208-231 deform_lbs (origin-form R x + t, weights == 0 skipped) on device."""
        pts = _t(points, self.device, torch.float32).reshape(-1, 3)
        R = _t(node_rotations, self.device, torch.float32).reshape(-1, 9)
        tt = _t(node_translations, self.device, torch.float32).reshape(-1, 3)
        a = _t(anchors, self.device, torch.int32)
        w = _t(weights, self.device, torch.float32)
        v = None if valid_pts is None else _t(valid_pts, self.device, torch.uint8)
        out = torch.empty_like(pts)
        call("ofx_deform_points_lbs", ptr(pts), pts.shape[0], ptr(a), ptr(w), ptr(v), a.shape[1], ptr(R), ptr(tt),
             R.shape[0], ptr(out), stream_ptr())
        return out

    def deform_lbs(self, node_rotations, node_translations, world_pts, world_anchors, world_weights, valid_pts):
        """warpfield.py:208-231 (numpy in, numpy out)."""
        return self.deform_lbs_device(node_rotations, node_translations, world_pts, world_anchors, world_weights,
                                      valid_pts).cpu().numpy()

    def deform(self, points, anchors, weights, reshape_gpu_vol=None, valid_pts=None):
        """warpfield.py:270-305: use_pytorch=True -> deform_ED semantics; False -> deform_lbs with the
        origin-form (rotations, translations) (its CPU and numba-CUDA branches compute the same formula)."""
        if not self.use_pytorch:
            return self.deform_lbs(self.rotations.astype(np.float32), self.translations.astype(np.float32), points,
                                   anchors, weights, valid_pts)
        return self.deform_device(points, anchors, weights, valid_pts).cpu().numpy()

    def deform_normals(self, normals, anchors, weights, reshape_gpu_vol=None, valid_pts=None):
        """warpfield.py:312-345."""
        return self.deform_device(normals, anchors, weights, valid_pts, normals=True).cpu().numpy()

    def deform_mesh(self, vertices, normals):
        """warpfield.py:347-367."""
        a, w, v = self.skin(vertices)
        dv = self.deform(vertices, a, w, None, v)
        dn = self.deform_normals(normals, a, w, None, v) if normals is not None else None
        return dv, dn, a, w, v

    def deform_tsdf(self):
        """warpfield.py:369-380 -> (deformed world points (V,3), valid (V,)) — materialises the whole grid
        on the host; the integrate path never calls this (it warps on the fly inside ofx_integrate)."""
        assert self.frame_id == self.tsdf.frame_id
        a, w, v = self.skin_tsdf()
        pts = self.tsdf.world_pts
        return self.deform(pts, a, w, None, v), v
