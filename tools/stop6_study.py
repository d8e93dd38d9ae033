"""Numerical study (CPU, not product): one PCG stop rule for both preconditioners (round 6).

Restates the product's GN loop in numpy/scipy closely enough to rank stop rules by the transforms' max error against
every f64 oracle fixture:
  * rows grouped as the product's setup groups them (gn.hip order_rows: BFS clusters of <= 8 nodes first-fit packed into
    8-row groups), the cluster block Jacobi over those groups, or the overlapping Schwarz subdomains (k_as_choose /
    k_as_accept: each group's ring = its 16 A-neighbours with the most coupling terms, a row kept by at most 3 rings);
  * the preconditioner built at the solve's first step and rebuilt when a node's accumulated rotation passes
    precond_rot_tol (0.3 rad), the Galerkin warm start over the last 4 step solutions, LM 1e-7 halved at steps 2/5/8,
    the loss-based early stop;
  * θ̂ as the device forms it: the largest shift σ_s = 2^(-e_s/4) of the grid with no Ritz value of the CG Lanczos
    tridiagonal below it, taken as min(θ̂, θ̂_prev) after a solve's first step.
Rules (all with the relative residual <= 2e-6, or the 1e-12 floor):
  cur   : round 5's product rule, √γ <= τ_M θ̂ with τ_M = 1e-5 (cluster blocks) / 2.5e-6 (Schwarz)
  gam:τ : √γ <= τ θ̂ for both preconditioners
  z:τ:d : ‖z‖₂ <= τ θ̂ (z = M⁻¹r: the error e = (M⁻¹A)⁻¹ z measured in the Euclidean norm the bar uses, not in the
          preconditioner's norm) holding at d consecutive iterations
Usage: python tools/stop6_study.py [fixture ...] -- [rule ...]
"""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import scipy.sparse as sp
from errstop_study import system, galerkin
from oracle import fusion_oracle as fo

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
KCS, RING, ASX = 8, 16, 3
SHIFTS = []
for s_ in range(64):
    e_ = s_ if s_ < 40 else 2 * s_ - 40
    SHIFTS.append((1.0, 0.84089641525371454303, 0.70710678118654752440, 0.59460355750136053336)[e_ & 3] * 2.0 ** -(e_ >> 2))


def fixture(name, f=0):
    """(problem dict, start R, start t, oracle R, oracle t) of fixture `name` frame f."""
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    N = g["nodes"].shape[0]
    if name == "moose":
        K = g["K"]
        P = dict(nodes=g["nodes"], edges=g["edges"], tpos=g["nodes"], conf=np.zeros(N, np.float32), src=g["src"],
                 anc=g["anchors"], wts=g["weights"], tgt=g["tgt"], intr=(K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
        return P, None, None, g["R"], g["t"]
    p = "" if "frames" not in g.files else f"f{f}_"
    P = dict(nodes=g["nodes"], edges=g["edges"], tpos=g[p + "tpos"], conf=g[p + "conf"], src=g[p + "src"],
             anc=g[p + "anchors"], wts=g[p + "weights"], tgt=g[p + "tgt"], intr=tuple(g["intr"]))
    R0 = g["f0_R"] if f else None
    t0 = g["f0_t"] if f else None
    return P, R0, t0, g[p + "R"], g[p + "t"]


def order_groups(nodes, edges):
    """gn.hip order_rows: node groups of <= 8 (padding dropped)."""
    N, NB = nodes.shape[0], edges.shape[1]
    lab = -np.ones(N, np.int64)
    clusters = []
    nd = nodes.astype(np.float64)
    for s0 in range(N):
        if lab[s0] >= 0:
            continue
        c = len(clusters)
        lab[s0] = c
        mem = [s0]
        front = [s0]
        f = 0
        while f < len(front) and len(mem) < KCS:
            cur = front[f]
            f += 1
            cand = []
            for k in range(NB):
                j = int(edges[cur, k])
                if 0 <= j < N and lab[j] < 0 and j not in cand:
                    cand.append(j)
            d2 = [float(((nd[j] - nd[s0]) ** 2).sum()) for j in cand]
            cand = [j for _, j in sorted(zip(d2, cand))]
            for j in cand:
                if len(mem) >= KCS:
                    break
                lab[j] = c
                mem.append(j)
                front.append(j)
        clusters.append(mem)
    order = sorted(range(len(clusters)), key=lambda c: -len(clusters[c]))
    fill, grp = [], []
    for c in order:
        sz = len(clusters[c])
        k = 0
        while k < len(fill) and fill[k] + sz > KCS:
            k += 1
        if k == len(fill):
            fill.append(0)
            grp.append([])
        fill[k] += sz
        grp[k].extend(clusters[c])
    return [np.asarray(g, np.int64) for g in grp]


def coupling_counts(P):
    """terms per node pair (x != y): match anchor pairs + graph edges (the contribution-list counts)."""
    cnt = {}
    for a in np.asarray(P["anc"], np.int64):
        for x in a:
            for y in a:
                if x >= 0 and y >= 0 and x != y:
                    cnt[(int(x), int(y))] = cnt.get((int(x), int(y)), 0) + 1
    ed, _ = fo.gn_edges(P["edges"])
    for x, y in ed:
        if x != y:
            for k in ((int(x), int(y)), (int(y), int(x))):
                cnt[k] = cnt.get(k, 0) + 1
    return cnt


def schwarz_domains(P, groups):
    cnt = coupling_counts(P)
    N = P["nodes"].shape[0]
    gid = np.empty(N, np.int64)
    for ci, g in enumerate(groups):
        gid[g] = ci
    score = [dict() for _ in groups]
    for (x, y), n in cnt.items():
        cx = gid[x]
        if gid[y] != cx:
            score[cx][y] = score[cx].get(y, 0) + n
    rings = []
    for ci in range(len(groups)):
        items = sorted(score[ci].items(), key=lambda kv: (-kv[1], kv[0]))[:RING]
        rings.append(items)
    choosers = {}
    for ci, items in enumerate(rings):
        for v, s in items:
            choosers.setdefault(v, []).append((-s, ci))
    keep = set()
    for v, lst in choosers.items():
        for _, ci in sorted(lst)[:ASX]:
            keep.add((ci, v))
    return [np.concatenate([g, np.asarray([v for v, _ in rings[ci] if (ci, v) in keep], np.int64)])
            for ci, g in enumerate(groups)]


def fp16_form(Z):
    """k_as_invert's stored form: Z = D Ẑ D, Ẑ's off-diagonal entries in fp16, its diagonal 1 + σ (σ = ‖E‖_F + 2^-10)."""
    d = np.sqrt(np.diag(Z))
    Zh = Z / np.outer(d, d)
    H = Zh.astype(np.float16).astype(np.float64)
    E = np.triu(H - Zh, 1)
    sig = math.sqrt(2.0 * (E * E).sum()) + 2.0 ** -10
    np.fill_diagonal(H, float(np.float16(1.0 + sig)))
    H = np.triu(H) + np.triu(H, 1).T
    return H * np.outer(d, d)


def build_minv(A, doms, f16=False):
    rows, cols, vals = [], [], []
    for d in doms:
        idx = (6 * d[:, None] + np.arange(6)[None, :]).reshape(-1)
        inv = np.linalg.inv(A[idx][:, idx].toarray())
        if f16:
            inv = fp16_form(inv)
        rr, cc = np.meshgrid(idx, idx, indexing="ij")
        rows.append(rr.ravel()); cols.append(cc.ravel()); vals.append(inv.ravel())
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=A.shape)


class Sturm:
    """the lead wave's shifted LDLᵀ pivots of T_k - σ_s I (k_pcg_iter): θ̂ = largest shift with no Ritz value below."""
    def __init__(self):
        self.d = np.zeros(64)
        self.c = np.zeros(64)
        self.k = 0

    def push(self, alpha, beta_prev, alpha_prev):
        sig = np.asarray(SHIFTS)
        if self.k == 0:
            diag, e2 = 1.0 / alpha, 0.0
            d = diag - sig
        else:
            diag = 1.0 / alpha + beta_prev / alpha_prev
            e2 = beta_prev / alpha_prev ** 2
            d = (diag - sig) - e2 / self.d
        d = np.where(np.abs(d) < 1e-300, -1e-300, d)
        self.c = self.c + (d < 0)
        self.d = d
        self.k += 1
        free = np.nonzero(self.c == 0)[0]
        return SHIFTS[free[0]] if free.size else 0.0


def pcg(A, b, Mi, x0, rule, th_prev, tol=2e-6, maxit=2000):
    x = x0.copy()
    r = b - A @ x
    z = Mi @ r
    p = z.copy()
    gam = r @ z
    bb = b @ b
    st = Sturm()
    th = None
    a_prev = b_prev = None
    passes = 0
    mu = None
    for it in range(maxit):
        rr = r @ r
        if gam == 0.0 or rr <= 1e-24 * bb:
            return x, it, th
        if th is not None and rr <= tol * tol * bb:
            thm = min(th, th_prev) if th_prev is not None else th
            ok = rule(gam=gam, zz=z @ z, th=thm, mu=mu)
            passes = passes + 1 if ok else 0
            if passes >= rule.d:
                return x, it, th
        else:
            passes = 0
        q = A @ p
        pq = p @ q
        mu = (p @ p) / pq
        a = gam / pq
        x += a * p
        r -= a * q
        z = Mi @ r
        g2 = r @ z
        beta = g2 / gam
        th = st.push(a, b_prev, a_prev)
        a_prev, b_prev = a, beta
        p = z + beta * p
        gam = g2
    return x, maxit, th


def gn(name, f, precond, rule, rot_tol=0.3):
    P, R0, t0, Rs, ts = fixture(name, f)
    N = P["nodes"].shape[0]
    R = np.tile(np.eye(3), (N, 1, 1)) if R0 is None else R0.astype(np.float64).copy()
    t = np.zeros((N, 3)) if t0 is None else t0.astype(np.float64).copy()
    groups = order_groups(P["nodes"], P["edges"])
    doms = groups if precond == "bj" else schwarz_domains(P, groups)
    lm = 1e-7
    hist, its, losses = [], [], []
    Mi, th_prev = None, None
    racc = np.zeros(N)
    refresh = False
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Mi is None or refresh:
            Mi = build_minv(A, doms, f16=precond == "as")
            racc[:] = 0.0
        x, it, th = pcg(A, b, Mi, galerkin(A, b, hist[-4:]), rule, th_prev if gi else None)
        th_prev = th if th is not None else th_prev
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        racc += np.linalg.norm(xr[:, :3], axis=1)
        refresh = rot_tol > 0 and bool((racc > rot_tol).any())
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    return max(np.abs(R - Rs).max(), np.abs(t - ts).max()), sum(its), its


def make_rule(spec, precond):
    kind, *a = spec.split(":")
    if kind == "cur":
        tau = 1e-5 if precond == "bj" else 2.5e-6
        f = lambda gam, zz, th, mu: gam <= (tau * th) ** 2
        f.d = 1
    elif kind == "gam":
        tau = float(a[0])
        f = lambda gam, zz, th, mu: gam <= (tau * th) ** 2
        f.d = int(a[1]) if len(a) > 1 else 1
    elif kind == "z":
        tau = float(a[0])
        f = lambda gam, zz, th, mu: zz <= (tau * th) ** 2
        f.d = int(a[1]) if len(a) > 1 else 1
    elif kind == "hs":   # ‖e‖₂ ≈ ‖e‖_A·√μ, ‖e‖²_A <= γ/θ̂, μ = ‖p‖²/pᵀAp (the last search direction)
        tau = float(a[0])
        f = lambda gam, zz, th, mu: th > 0 and gam * mu <= tau * tau * th
        f.d = int(a[1]) if len(a) > 1 else 1
    else:
        raise ValueError(spec)
    return f


FIXTURES = {"small": ("gn_small", 0), "1k": ("gn_1k", 0), "2k0": ("gn_2k", 0), "2k1": ("gn_2k", 1),
            "4k": ("gn_4k", 0), "c5r1": ("gn_c5r1", 0), "c5r7": ("gn_c5r7", 0), "moose": ("moose", 0),
            "hole": ("gn_2k_hole", 0)}

if __name__ == "__main__":
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    fx = argv[:cut] or ["small", "1k", "2k0", "2k1", "moose"]
    rules = argv[cut + 1:] or ["cur"]
    pcs = os.environ.get("PCS", "bj,as").split(",")
    for key in fx:
        name, f = FIXTURES[key]
        if not os.path.exists(os.path.join(GOLD, name + ".npz")):
            print(f"{key}: no fixture")
            continue
        for pc in pcs:
            for spec in rules:
                e, n, its = gn(name, f, pc, make_rule(spec, pc))
                print(f"{key:6s} {pc:3s} {spec:14s} err {e:.2e}  pcg {n:5d} {its}", flush=True)


def diag(name, f, precond, spec):
    """per GN step: the true error of the PCG solution against a direct solve of the same system beside the rule's
    estimates at the stop (‖e‖₂ true | √(γμ/θ̂) | √γ/θ̂ | ‖e‖_A true, √(γ/θ̂) its bound)."""
    import scipy.sparse.linalg as spl
    P, R0, t0, Rs, ts = fixture(name, f)
    N = P["nodes"].shape[0]
    R = np.tile(np.eye(3), (N, 1, 1)) if R0 is None else R0.astype(np.float64).copy()
    t = np.zeros((N, 3)) if t0 is None else t0.astype(np.float64).copy()
    groups = order_groups(P["nodes"], P["edges"])
    doms = groups if precond == "bj" else schwarz_domains(P, groups)
    lm, hist, Mi, th_prev, racc, refresh = 1e-7, [], None, None, np.zeros(N), False
    rule = make_rule(spec, precond)
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Mi is None or refresh:
            Mi = build_minv(A, doms, f16=precond == "as")
            racc[:] = 0.0
        seen = {}

        def rec(**kw):
            seen.update(kw)
            return rule(**kw)
        rec.d = rule.d
        x, it, th = pcg(A, b, Mi, galerkin(A, b, hist[-4:]), rec, th_prev if gi else None)
        th_prev = th if th is not None else th_prev
        xs = spl.spsolve(A.tocsc(), b)
        e = x - xs
        g_, mu, thm = seen.get("gam", np.nan), seen.get("mu", np.nan), seen.get("th", np.nan)
        print(f"  step {gi} it {it:4d} |e|inf {np.abs(e).max():.2e} |e|2 {np.linalg.norm(e):.2e} "
              f"hs {math.sqrt(g_ * mu / thm):.2e} M-est {math.sqrt(g_) / thm:.2e} |e|A {math.sqrt(e @ (A @ e)):.2e} "
              f"A-bound {math.sqrt(g_ / thm):.2e} mu {mu:.2e} th {thm:.2e}", flush=True)
        hist.append(x)
        xr = x.reshape(N, 6)
        racc += np.linalg.norm(xr[:, :3], axis=1)
        refresh = bool((racc > 0.3).any())
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    print(f"{name} {precond} {spec}: final err {max(np.abs(R - Rs).max(), np.abs(t - ts).max()):.2e}")
