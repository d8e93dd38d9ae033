"""Numerical study (CPU, not product): two-level preconditioners for the GN steps' PCG.

The product's PCG uses cluster block Jacobi (BFS clusters of 8 nodes, exact 48x48 inverses). This study adds a coarse
space per aggregate of clusters and counts PCG iterations over the fixture's 10-step GN loop (Galerkin warm start over
the last 4 step solutions, stop at relative residual 1e-6 as the product), for
  B    : cluster block Jacobi alone (the product),
  add  : additive two-level  M⁻¹ = B⁻¹ + P (PᵀAP)⁻¹ Pᵀ,
  def  : deflation-balanced (A-DEF2 / "BNN-lite")  M⁻¹ = (I - P E⁻¹ PᵀA) B⁻¹ (I - A P E⁻¹ Pᵀ) + P E⁻¹ Pᵀ,
with P = per-aggregate piecewise-constant dof blocks ("agg6": 6 columns per aggregate, one per dof type) or rigid modes
("rigid": translation + rotation about the aggregate centroid acting on [ω|t]).
Usage: python tools/coarse_study.py [2k|1k|moose] [agg]   (agg = clusters per aggregate, default 1)
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import scipy.sparse as sp
import scipy.linalg as sl
from errstop_study import load, system, clusters, make_minv, galerkin
from oracle import fusion_oracle as fo


def cluster_labels(nodes, edges, c=8):
    groups = clusters(nodes, edges, c)
    lab = np.empty(nodes.shape[0], np.int64)
    for l, idx in enumerate(groups):
        lab[idx[::6] // 6] = l
    return groups, lab


def merge_aggregates(lab, nodes, agg):
    """greedy: merge `agg` spatially adjacent clusters (by centroid order along a space-filling sort)"""
    if agg == 1:
        return lab
    nc = lab.max() + 1
    cen = np.stack([nodes[lab == l].mean(0) for l in range(nc)])
    # morton-ish: sort by quantised coordinates
    q = np.floor((cen - cen.min(0)) / 0.15).astype(np.int64)
    order = np.lexsort((q[:, 2], q[:, 1], q[:, 0]))
    newl = np.empty(nc, np.int64)
    newl[order] = np.arange(nc) // agg
    return newl[lab]


def prolong(nodes, alab, kind):
    N = nodes.shape[0]
    na = alab.max() + 1
    rows, cols, vals = [], [], []
    if kind == "agg6":
        for d in range(6):
            rows.append(6 * np.arange(N) + d); cols.append(6 * alab + d); vals.append(np.ones(N))
        return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(6 * N, 6 * na))
    # rigid: column (a, d): d<3 translation e_d, d>=3 rotation about axis e_{d-3} through the centroid:
    #   node j: ω = e, t = e x (g_j - c)
    cen = np.stack([nodes[alab == a].mean(0) for a in range(na)])
    rel = nodes - cen[alab]
    for d in range(3):
        rows.append(6 * np.arange(N) + 3 + d); cols.append(6 * alab + d); vals.append(np.ones(N))
    for d in range(3):
        e = np.zeros(3); e[d] = 1
        rows.append(6 * np.arange(N) + d); cols.append(6 * alab + 3 + d); vals.append(np.ones(N))
        tr = np.cross(e, rel)
        for c in range(3):
            rows.append(6 * np.arange(N) + 3 + c); cols.append(6 * alab + 3 + d); vals.append(tr[:, c])
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(6 * N, 6 * na))


def make_prec(A, Bi, P, kind):
    if P is None:
        return lambda r: Bi @ r
    E = (P.T @ (A @ P)).toarray()
    Ec = sl.cho_factor(E)

    def cs(v):
        return P @ sl.cho_solve(Ec, P.T @ v)
    if kind == "add":
        return lambda r: Bi @ r + cs(r)

    def dfl(r):
        y = r - A @ cs(r)
        z = Bi @ y
        return z - cs(A @ z) + cs(r)
    return dfl


def pcg(A, b, M, x0, tol=1e-6, maxit=5000):
    x = x0.copy()
    r = b - A @ x
    z = M(r)
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
        z = M(r)
        g2 = r @ z
        p = z + (g2 / gam) * p
        gam = g2
    return x, maxit


def gn(P, prec, pkind, agg, label):
    N = P["nodes"].shape[0]
    nodes = P["nodes"].astype(np.float64)
    R, t = np.tile(np.eye(3), (N, 1, 1)), np.zeros((N, 3))
    groups, lab = cluster_labels(P["nodes"], P["edges"])
    alab = merge_aggregates(lab, nodes, agg)
    Pm = None if prec == "B" else prolong(nodes, alab, pkind)
    lm = 1e-7
    hist, its, losses = [], [], []
    Bi = None
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Bi is None:
            Bi, _ = make_minv(A, groups)
        M = make_prec(A, Bi, Pm, prec)
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
    dR, dt = np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max()
    nc = 0 if Pm is None else Pm.shape[1]
    print(f"{label:28s} coarse {nc:5d}  dR {dR:.1e} dt {dt:.1e}  pcg {sum(its):5d} {its}", flush=True)


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "2k"
    aggs = [int(a) for a in sys.argv[2:]] or [1]
    P = load({"2k": "gn_2k", "1k": "gn_1k", "4k": "gn_4k", "moose": "moose"}.get(name, name))
    gn(P, "B", None, 1, "B (product)")
    for agg in aggs:
        for pk in ("agg6", "rigid"):
            for pr in ("add", "def"):
                gn(P, pr, pk, agg, f"{pr}/{pk}/agg{agg}")
