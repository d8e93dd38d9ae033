"""Tuning study (CPU, not product): PCG iterations over the 10 GN steps of one frame (sparse numpy
restatement of the GN linearisation) for warm-start strategies:
  cold      x0 = 0
  proj4     Galerkin projection on the last 4 GN-step solutions (the product's warm start)
  krylov    x0 = sum_i p_i (p_i·b)/(p_i·A_old p_i) over the previous step's PCG directions
  both      krylov directions + last 4 solutions, Galerkin with the new A (small dense solve)
  prev1     x0 = the previous step's solution (no projection: no global reduction before the PCG)
  extrap    x0 = 2 x_{k-1} - x_{k-2} (linear extrapolation, likewise reduction-free)
"""
import math
import os
import sys
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


class Problem:
    def __init__(self, seq, t):
        src, tgt, tpos, conf = seq.solver_inputs(t, 10000)
        anc, w, v = fo.skin(src, seq.nodes, seq.node_coverage)
        self.src, self.tgt = src[v].astype(np.float64), tgt[v].astype(np.float64)
        self.anc, self.w = anc[v].astype(np.int64), w[v].astype(np.float64)
        self.tpos, self.conf = tpos.astype(np.float64), conf.astype(np.float64)
        self.g = seq.nodes.astype(np.float64)
        self.cam = seq.cam
        E = [(i, j) for i in range(len(self.g)) for j in seq.edges[i] if j >= 0]
        self.E = np.array(E)

    def linearize(self, R, t, lm):
        g, src, anc, w = self.g, self.src, self.anc, self.w
        N, M = g.shape[0], src.shape[0]
        fx, fy = self.cam.fx, self.cam.fy
        defp = np.zeros((M, 3))
        rot = []
        for k in range(4):
            nk = anc[:, k]
            rk = np.einsum('mij,mj->mi', R[nk], src - g[nk])
            rot.append(rk)
            defp += w[:, k:k + 1] * (rk + g[nk] + t[nk])
        zinv = 1.0 / (defp[:, 2] + 1e-7)
        mfx = -(fx * defp[:, 0] * zinv) * zinv
        mfy = -(fy * defp[:, 1] * zinv) * zinv
        rows, cols, vals = [], [], []
        r3 = np.arange(M) * 3
        for k in range(4):
            nk = anc[:, k]
            wk = w[:, k]
            Sk = -skew(wk[:, None] * rot[k])
            for i in range(3):
                for j in range(3):
                    val = Sk[:, i, j].copy()
                    if i == 0:
                        val = val + mfx * Sk[:, 2, j]
                    if i == 1:
                        val = val + mfy * Sk[:, 2, j]
                    rows.append(r3 + i); cols.append(6 * nk + j); vals.append(val)
                rows.append(r3 + i); cols.append(6 * nk + 3 + i); vals.append(wk)
        res = [(defp - self.tgt).reshape(-1)]
        nrow = 3 * M
        la = math.sqrt(0.5)
        i0, i1 = self.E[:, 0], self.E[:, 1]
        d = np.einsum('eij,ej->ei', R[i0], g[i1] - g[i0])
        res.append((la * (d + g[i0] + t[i0] - (g[i1] + t[i1]))).reshape(-1))
        Sa = -la * skew(d)
        re = nrow + np.arange(len(i0)) * 3
        for i in range(3):
            for j in range(3):
                rows.append(re + i); cols.append(6 * i0 + j); vals.append(Sa[:, i, j])
            rows.append(re + i); cols.append(6 * i0 + 3 + i); vals.append(np.full(len(i0), la))
            rows.append(re + i); cols.append(6 * i1 + 3 + i); vals.append(np.full(len(i0), -la))
        nrow += 3 * len(i0)
        rm = nrow + np.arange(N) * 3
        for i in range(3):
            rows.append(rm + i); cols.append(6 * np.arange(N) + 3 + i); vals.append(self.conf)
        res.append((self.conf[:, None] * (t + g - self.tpos)).reshape(-1))
        nrow += 3 * N
        J = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(nrow, 6 * N))
        r = np.concatenate(res)
        A = (J.T @ J + lm * sp.eye(6 * N)).tocsr()
        b = -(J.T @ r)
        return A, b


def block_inv(A):
    n = A.shape[0] // 6
    D = np.zeros((n, 6, 6))
    A = A.tocsr()
    for i in range(n):
        D[i] = np.linalg.inv(A[6 * i:6 * i + 6, 6 * i:6 * i + 6].toarray())
    return D


def apply_M(D, v):
    return np.einsum('nij,nj->ni', D, v.reshape(-1, 6)).reshape(-1)


def pcg(A, b, D, x0, tol=1e-7, maxit=3000):
    x = x0.copy()
    r = b - A @ x
    u = apply_M(D, r)
    p = u.copy()
    ru = r @ u
    bb = math.sqrt(b @ b)
    P, PAP = [], []
    for it in range(maxit):
        if math.sqrt(r @ r) <= tol * bb:
            return x, it, P, PAP
        q = A @ p
        pq = p @ q
        a = ru / pq
        P.append(p.copy()); PAP.append(pq)
        x += a * p
        r -= a * q
        u = apply_M(D, r)
        ru2 = r @ u
        p = u + (ru2 / ru) * p
        ru = ru2
    return x, maxit, P, PAP


def galerkin(A, b, X):
    """A-norm optimal combination of the columns of X (pivot-guarded Cholesky on XᵀAX)."""
    AX = A @ X
    G = X.T @ AX
    f = X.T @ b
    try:
        c = np.linalg.solve(G + 1e-14 * np.trace(G) / G.shape[0] * np.eye(G.shape[0]), f)
    except np.linalg.LinAlgError:
        return np.zeros(A.shape[0])
    return X @ c


def kry_init(b, P, PAP, maxv):
    x0 = np.zeros_like(b)
    for p, pq in list(zip(P, PAP))[:maxv]:
        x0 += p * ((p @ b) / pq)
    return x0


def run(prob, mode, N):
    R = np.tile(np.eye(3), (N, 1, 1))
    t = np.zeros((N, 3))
    lm = 1e-7
    hist, P, PAP = [], [], []
    its = []
    for k in range(10):
        if k % 3 == 2:
            lm /= 2
        A, b = prob.linearize(R, t, lm)
        D = block_inv(A)
        x0 = np.zeros(6 * N)
        if mode == "proj4" and hist:
            x0 = galerkin(A, b, np.stack(hist[-4:], 1))
        elif mode == "prev1" and hist:
            x0 = hist[-1].copy()
        elif mode == "extrap" and hist:
            x0 = (2 * hist[-1] - hist[-2]) if len(hist) > 1 else hist[-1].copy()
        elif mode == "krylov" and P:
            x0 = kry_init(b, P, PAP, 400)
        elif mode == "both" and hist:
            xk = kry_init(b, P, PAP, 400)
            x0 = galerkin(A, b, np.stack(hist[-4:] + [xk], 1))
        x, it, P, PAP = pcg(A, b, D, x0)
        its.append(it)
        hist.append(x)
        Ri = fo.angle_axis_to_rotation_matrix(x.reshape(N, 6)[:, :3])
        R = Ri @ R
        t = t + x.reshape(N, 6)[:, 3:]
    return its


if __name__ == "__main__":
    seq = S.SyntheticSequence.build(2000, seed=3)
    prob = Problem(seq, int(sys.argv[1]) if len(sys.argv) > 1 else 12)
    N = seq.nodes.shape[0]
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ("cold", "proj4", "krylov", "both")
    for mode in modes:
        its = run(prob, mode, N)
        print(mode, sum(its), its, flush=True)


def cluster_groups(nodes, edges, cs):
    """BFS clusters of <= cs nodes (lowest unassigned seed, grow over graph edges by distance), then
    whole clusters first-fit into consecutive groups of <= cs nodes (one wave each)."""
    N = nodes.shape[0]
    lab = -np.ones(N, np.int64)
    cl = []
    for s in range(N):
        if lab[s] >= 0:
            continue
        grp = [s]
        lab[s] = len(cl)
        front = [s]
        while len(grp) < cs and front:
            cur = front.pop(0)
            cand = [j for j in edges[cur] if j >= 0 and lab[j] < 0]
            cand.sort(key=lambda j: float(((nodes[j] - nodes[s]) ** 2).sum()))
            for j in cand:
                if len(grp) >= cs:
                    break
                lab[j] = len(cl)
                grp.append(j)
                front.append(j)
        cl.append(grp)
    groups, cur = [], []
    for c in cl:
        if len(cur) + len(c) > cs:
            groups.append(cur)
            cur = []
        cur = cur + c
    if cur:
        groups.append(cur)
    return groups


def group_inv(A, groups):
    A = A.tocsr()
    out = []
    for gr in groups:
        idx = np.concatenate([np.arange(6 * m, 6 * m + 6) for m in gr])
        out.append((idx, np.linalg.inv(A[idx][:, idx].toarray())))
    return out


def apply_G(Gi, v):
    o = np.zeros_like(v)
    for idx, inv in Gi:
        o[idx] = inv @ v[idx]
    return o


def pcg_g(A, b, Gi, x0, tol=1e-7, maxit=3000):
    x = x0.copy()
    r = b - A @ x
    u = apply_G(Gi, r)
    p = u.copy()
    ru = r @ u
    bb = math.sqrt(b @ b)
    for it in range(maxit):
        if math.sqrt(r @ r) <= tol * bb:
            return x, it
        q = A @ p
        a = ru / (p @ q)
        x += a * p
        r -= a * q
        u = apply_G(Gi, r)
        ru2 = r @ u
        p = u + (ru2 / ru) * p
        ru = ru2
    return x, maxit


def run_groups(prob, groups, N):
    R = np.tile(np.eye(3), (N, 1, 1))
    t = np.zeros((N, 3))
    lm = 1e-7
    hist, its = [], []
    for k in range(10):
        if k % 3 == 2:
            lm /= 2
        A, b = prob.linearize(R, t, lm)
        Gi = group_inv(A, groups)
        x0 = galerkin(A, b, np.stack(hist[-4:], 1)) if hist else np.zeros(6 * N)
        x, it = pcg_g(A, b, Gi, x0)
        its.append(it)
        hist.append(x)
        R = fo.angle_axis_to_rotation_matrix(x.reshape(N, 6)[:, :3]) @ R
        t = t + x.reshape(N, 6)[:, 3:]
    return its


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "groups":
    for cs in (4, 8, 16):
        groups = cluster_groups(seq.nodes, seq.edges, cs)
        its = run_groups(prob, groups, N)
        print(f"groups cs={cs} n={len(groups)} rows={cs * len(groups)}", sum(its), its, flush=True)
