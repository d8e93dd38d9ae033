"""Numerical study (CPU, not product): overlapping additive Schwarz against the product's cluster block Jacobi.

Runs the product's 10-step GN loop in numpy (errstop_study's systems, Galerkin warm start over the last 4 step
solutions, relative-residual stop 1e-6, preconditioner built once per solve from the first step's A as the product
does without a refresh) and counts PCG iterations for
  B      : cluster block Jacobi over the BFS 8-node clusters (the product),
  AS/g   : additive Schwarz, each cluster extended by its graph one-ring (deformation-graph edges),
  AS/a   : the same with the ring taken from A's block pattern (every node coupled to the cluster),
  AS/gK  : the graph ring capped at the K nodes most strongly coupled to the cluster (Frobenius norm of A's blocks),
  AS/cK  : A's pattern ring capped at the K nodes with the most terms (match anchor pairs + edges) coupling them to the
           cluster (a proxy the setup knows before any A exists),
and prints the subdomain inverses' total size (entries of the dense per-subdomain inverses) beside the count.
Usage: python tools/schwarz_study.py [1k|2k|4k|moose ...]
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import scipy.sparse as sp
from errstop_study import load, system, clusters, galerkin
from oracle import fusion_oracle as fo


def node_groups(P):
    return [idx[::6] // 6 for idx in clusters(P["nodes"], P["edges"])]


def rings(P, A, groups, kind, cap=None):
    N = P["nodes"].shape[0]
    if kind == "g":
        adj = [set() for _ in range(N)]
        for i, row in enumerate(P["edges"]):
            for j in row:
                if j >= 0:
                    adj[i].add(int(j)); adj[int(j)].add(i)
    else:
        Ab = A.tocoo()
        adj = [set() for _ in range(N)]
        for r, c in zip(Ab.row // 6, Ab.col // 6):
            adj[r].add(int(c))
    Ad = A.tocsr()
    cnt = None
    if kind == "e":   # graph-only proxy (static per graph): the number of deformation-graph edges to the cluster
        cnt = {}
        ed, _ = fo.gn_edges(P["edges"])
        for x, y in ed:
            for k in ((int(x), int(y)), (int(y), int(x))):
                cnt[k] = cnt.get(k, 0) + 1
        adj = [set() for _ in range(N)]
        for (x, y) in cnt:
            if x != y:
                adj[x].add(y)
    if kind == "c":   # coupling proxy known at setup: the number of terms (matches' anchor pairs, graph edges) per block
        cnt = {}
        for a in np.asarray(P["anc"], np.int64):
            for x in a:
                for y in a:
                    cnt[(int(x), int(y))] = cnt.get((int(x), int(y)), 0) + 1
        ed, _ = fo.gn_edges(P["edges"])
        for x, y in ed:
            for k in ((int(x), int(y)), (int(y), int(x))):
                cnt[k] = cnt.get(k, 0) + 1
        adj = [set() for _ in range(N)]
        for (x, y) in cnt:
            if x != y:
                adj[x].add(y)
    out = []
    for g in groups:
        gs = set(int(v) for v in g)
        ring = sorted(set().union(*(adj[v] for v in gs)) - gs)
        if cap is not None and len(ring) > cap:
            idx = np.concatenate([np.arange(6 * v, 6 * v + 6) for v in g])
            w = []
            for v in ring:
                if cnt is not None:
                    w.append(sum(cnt.get((int(u), v), 0) for u in g) - 1e-9 * v)
                else:
                    blk = Ad[idx][:, 6 * v:6 * v + 6].toarray()
                    w.append(np.linalg.norm(blk))
            ring = [ring[i] for i in np.argsort(w, kind="stable")[::-1][:cap]]
        out.append((np.asarray(g, np.int64), [int(v) for v in ring],
                    [0.0 if cnt is None else float(sum(cnt.get((int(u), v), 0) for u in g)) for v in ring]))
    X = int(os.environ.get("AS_X", "0"))
    if X > 0:   # each node joins at most X rings: the X clusters with the most coupling terms (ties: lower cluster)
        choosers = {}
        for ci, (g, ring, sc) in enumerate(out):
            for v, s_ in zip(ring, sc):
                choosers.setdefault(v, []).append((-s_, ci))
        keep = set()
        for v, lst in choosers.items():
            for _, ci in sorted(lst)[:X]:
                keep.add((ci, v))
        out = [(g, [v for v in ring if (ci, v) in keep], sc) for ci, (g, ring, sc) in enumerate(out)]
    mult = {}
    for g, ring, _ in out:
        for v in ring:
            mult[v] = mult.get(v, 0) + 1
    if mult:
        h = np.bincount(list(mult.values()))
        nsrc = [len({ci for ci, (g2, r2, _) in enumerate(out) if ci == cj or set(r2) & set(int(x) for x in g)})
                for cj, (g, _, _) in enumerate(out)]
        print(f"   ring multiplicity histogram {h.tolist()}  max src domains per cluster {max(nsrc)}", flush=True)
    return [np.concatenate([g, np.asarray(ring, np.int64)]) for g, ring, _ in out]


def as_prec(A, doms):
    rows, cols, vals = [], [], []
    size = 0
    for d in doms:
        idx = np.concatenate([np.arange(6 * v, 6 * v + 6) for v in d])
        inv = np.linalg.inv(A[idx][:, idx].toarray())
        size += inv.size
        rr, cc = np.meshgrid(idx, idx, indexing="ij")
        rows.append(rr.ravel()); cols.append(cc.ravel()); vals.append(inv.ravel())
    M = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=A.shape)
    return M, size


def pcg(A, b, M, x0, tol=1e-6, maxit=8000):
    x = x0.copy()
    r = b - A @ x
    z = M @ r
    p = z.copy()
    gam = r @ z
    bb = b @ b
    for it in range(maxit):
        if r @ r <= tol * tol * bb or gam == 0.0:
            return x, it
        q = A @ p
        a = gam / (p @ q)
        x += a * p
        r -= a * q
        z = M @ r
        g2 = r @ z
        p = z + (g2 / gam) * p
        gam = g2
    return x, maxit


def gn(P, mode, cap=None):
    N = P["nodes"].shape[0]
    R, t = np.tile(np.eye(3), (N, 1, 1)), np.zeros((N, 3))
    groups = node_groups(P)
    lm = 1e-7
    hist, its, losses = [], [], []
    M = None
    size = 0
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if M is None:
            doms = groups if mode == "B" else rings(P, A, groups, mode, cap)
            M, size = as_prec(A, doms)
        x0 = galerkin(A, b, hist[-4:])
        x, it = pcg(A, b, M, x0)
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    err = max(np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max())
    return sum(its), its, size, err


if __name__ == "__main__":
    names = sys.argv[1:] or ["2k"]
    for name in names:
        P = load({"2k": "gn_2k", "1k": "gn_1k", "4k": "gn_4k", "moose": "moose"}.get(name, name))
        base = None
        modes = [(m, None if c == "-" else int(c)) for m, c in (x.split(":") for x in os.environ.get(
            "AS_MODES", "B:-,g:-,g:6,g:12,a:-").split(","))]
        for mode, cap in modes:
            label = "B (product)" if mode == "B" else f"AS/{mode}{'' if cap is None else cap}"
            tot, its, size, err = gn(P, mode, cap)
            base = base or tot
            print(f"{name:5s} {label:12s} pcg {tot:6d} ({base / tot:4.2f}x)  inverse entries {size:9d}  "
                  f"err {err:.1e}  {its}", flush=True)
