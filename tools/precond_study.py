"""Tuning study (CPU, not product): PCG iteration counts of the GN system under block-Jacobi variants.

Builds the first GN step's A = JᵀJ + λI (sparse, node-major 6 DOF per node [rot|trans]) of the bench
workload and counts CG iterations to relative residual 1e-7 for: 6x6 block Jacobi (the product's
preconditioner) and cluster block Jacobi over groups of c spatially close nodes (c = 2, 4, 8).
"""
import math
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.sparse as sp
from occlusionfusion_amd import synthetic as S
from oracle import fusion_oracle as fo


def skew(v):
    z = np.zeros(v.shape[:-1] + (3, 3))
    z[..., 0, 1], z[..., 0, 2] = -v[..., 2], v[..., 1]
    z[..., 1, 0], z[..., 1, 2] = v[..., 2], -v[..., 0]
    z[..., 2, 0], z[..., 2, 1] = -v[..., 1], v[..., 0]
    return z


def build_A(seq, t):
    src, tgt, tpos, conf = seq.solver_inputs(t, 10000)
    anc, w, v = fo.skin(src, seq.nodes, seq.node_coverage)
    src, tgt, anc, w = src[v].astype(np.float64), tgt[v].astype(np.float64), anc[v].astype(np.int64), w[v].astype(np.float64)
    g = seq.nodes.astype(np.float64)
    N, M = g.shape[0], src.shape[0]
    cam = seq.cam
    fx, fy = cam.fx, cam.fy
    rows, cols, vals = [], [], []
    defp = np.zeros((M, 3))
    for k in range(4):
        defp += w[:, k:k + 1] * (src - g[anc[:, k]] + g[anc[:, k]])
    zinv = 1.0 / (defp[:, 2] + 1e-7)
    mfx = -(fx * defp[:, 0] * zinv) * zinv
    mfy = -(fy * defp[:, 1] * zinv) * zinv
    r3 = np.arange(M) * 3
    for k in range(4):
        nk = anc[:, k]
        wk = w[:, k]
        Sk = -skew(wk[:, None] * (src - g[nk]))
        for i in range(3):
            for j in range(3):
                val = Sk[:, i, j].copy()
                if i == 0:
                    val = val + mfx * Sk[:, 2, j]
                if i == 1:
                    val = val + mfy * Sk[:, 2, j]
                rows.append(r3 + i); cols.append(6 * nk + j); vals.append(val)
            rows.append(r3 + i); cols.append(6 * nk + 3 + i); vals.append(wk)
    nrow = 3 * M
    E = [(i, j) for i in range(N) for j in seq.edges[i] if j >= 0]
    E = np.array(E)
    la = math.sqrt(0.5)
    i0, i1 = E[:, 0], E[:, 1]
    d = g[i1] - g[i0]
    Sa = -la * skew(d)
    re = nrow + np.arange(len(E)) * 3
    for i in range(3):
        for j in range(3):
            rows.append(re + i); cols.append(6 * i0 + j); vals.append(Sa[:, i, j])
        rows.append(re + i); cols.append(6 * i0 + 3 + i); vals.append(np.full(len(E), la))
        rows.append(re + i); cols.append(6 * i1 + 3 + i); vals.append(np.full(len(E), -la))
    nrow += 3 * len(E)
    rm = nrow + np.arange(N) * 3
    for i in range(3):
        rows.append(rm + i); cols.append(6 * np.arange(N) + 3 + i); vals.append(conf.astype(np.float64))
    nrow += 3 * N
    J = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(nrow, 6 * N))
    A = (J.T @ J + 1e-7 * sp.eye(6 * N)).tocsr()
    b = np.random.default_rng(0).normal(size=6 * N)
    return A, b


def clusters(nodes, edges, c):
    """greedy: take the lowest unassigned node, grow by BFS over graph edges to c members"""
    N = nodes.shape[0]
    lab = -np.ones(N, np.int64)
    nxt = 0
    for s in range(N):
        if lab[s] >= 0:
            continue
        grp = [s]
        lab[s] = nxt
        front = [s]
        while len(grp) < c and front:
            cur = front.pop(0)
            cand = [j for j in edges[cur] if j >= 0 and lab[j] < 0]
            cand.sort(key=lambda j: float(((nodes[j] - nodes[s]) ** 2).sum()))
            for j in cand:
                if len(grp) >= c:
                    break
                lab[j] = nxt
                grp.append(j)
                front.append(j)
        nxt += 1
    return lab


def block_jacobi(A, lab):
    n = A.shape[0] // 6
    groups = {}
    for i, l in enumerate(lab):
        groups.setdefault(l, []).append(i)
    Minv = sp.lil_matrix(A.shape)
    blocks = []
    for l, mem in groups.items():
        idx = np.concatenate([np.arange(6 * m, 6 * m + 6) for m in mem])
        blk = A[idx][:, idx].toarray()
        blocks.append((idx, np.linalg.inv(blk)))
    rows, cols, vals = [], [], []
    for idx, inv in blocks:
        rr, cc = np.meshgrid(idx, idx, indexing="ij")
        rows.append(rr.ravel()); cols.append(cc.ravel()); vals.append(inv.ravel())
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=A.shape)


def pcg_iters(A, b, Minv, tol=1e-7, maxit=5000):
    x = np.zeros_like(b)
    r = b.copy()
    z = Minv @ r
    p = z.copy()
    rz = r @ z
    bb = math.sqrt(b @ b)
    for it in range(maxit):
        if math.sqrt(r @ r) <= tol * bb:
            return it
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        z = Minv @ r
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return maxit


if __name__ == "__main__":
    seq = S.SyntheticSequence.build(2000, seed=3)
    for t in (4, 14):
        A, b = build_A(seq, t)
        N = seq.nodes.shape[0]
        print(f"frame {t}: N={N}, nnz={A.nnz}")
        for c in (1, 2, 4, 8):
            lab = np.arange(N) if c == 1 else clusters(seq.nodes, seq.edges, c)
            Minv = block_jacobi(A, lab)
            print(f"  cluster {c}: groups={lab.max() + 1}, PCG iterations={pcg_iters(A, b, Minv)}", flush=True)


def order_by_clusters(nodes, edges, c):
    """row order: greedy BFS clusters of c nodes, stragglers kept adjacent; waves take c consecutive rows"""
    lab = clusters(nodes, edges, c)
    order = np.argsort(lab, kind="stable")
    return order


def consecutive_groups(order, c):
    lab = np.empty(len(order), np.int64)
    lab[order] = np.arange(len(order)) // c
    return lab


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "consecutive":
    seq = S.SyntheticSequence.build(2000, seed=3)
    for t in (4, 14):
        A, b = build_A(seq, t)
        N = seq.nodes.shape[0]
        for c in (4, 8):
            order = order_by_clusters(seq.nodes, seq.edges, c)
            lab = consecutive_groups(order, c)
            Minv = block_jacobi(A, lab)
            print(f"frame {t} consecutive-{c}: PCG iterations={pcg_iters(A, b, Minv)}", flush=True)
