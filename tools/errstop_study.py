"""Numerical study (CPU, not product): PCG stop rules for the GN steps against the dense f64 oracle fixtures.

For the moose landmark problem (tests/golden/moose.npz) and a bench frame (gn_2k.npz frame 10) runs the product's
10-step GN loop in numpy — cluster block-Jacobi PCG (BFS clusters of 8 nodes), Galerkin warm start over the last 4
step solutions — under several stop rules, and prints the final transforms' max error against the fixture and the
PCG iterations. Per iteration it also records the estimates a device-side rule could use:
  rr = ‖r‖², gam = rᵀM⁻¹r, the Lanczos tridiagonal of the preconditioned operator from (α, β) and its smallest Ritz
  value θ_min, and compares ‖e‖₂ (true, against a direct solve) with √gam/θ_min and ‖r‖/θ_min.
Usage: python tools/errstop_study.py [moose|2k] [trace]
"""
import math
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl
from scipy.linalg import eigvalsh_tridiagonal
from oracle import fusion_oracle as fo

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def load(name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    if name == "moose":
        K = g["K"]
        N = g["nodes"].shape[0]
        return dict(nodes=g["nodes"], edges=g["edges"], tpos=g["nodes"], conf=np.zeros(N, np.float32), src=g["src"],
                    anc=g["anchors"], wts=g["weights"], tgt=g["tgt"], intr=(K[0, 0], K[1, 1], K[0, 2], K[1, 2]),
                    R=g["R"], t=g["t"], loss=g["loss_total"])
    p = "f0_"
    return dict(nodes=g["nodes"], edges=g["edges"], tpos=g[p + "tpos"], conf=g[p + "conf"], src=g[p + "src"],
                anc=g[p + "anchors"], wts=g[p + "weights"], tgt=g[p + "tgt"], intr=tuple(g["intr"]), R=g[p + "R"],
                t=g[p + "t"], loss=g[p + "loss_total"])


def system(P, R, t, lm):
    """A (node-major 6N, csr), b, ‖res‖ of one linearisation (gn_optimize_sparse's rows, lambda_flow = 0)."""
    g = P["nodes"].astype(np.float64)
    N = g.shape[0]
    src, anc, wts, tgt = (P["src"].astype(np.float64), P["anc"].astype(np.int64), P["wts"].astype(np.float64),
                          P["tgt"].astype(np.float64))
    M = src.shape[0]
    fx, fy = float(P["intr"][0]), float(P["intr"][1])
    conf = P["conf"].astype(np.float64)
    tpos = P["tpos"].astype(np.float64)
    rr, cc, vv = [], [], []

    def put(r, c, v):
        rr.append(np.asarray(r, np.int64).reshape(-1))
        cc.append(np.asarray(c, np.int64).reshape(-1))
        vv.append(np.broadcast_to(np.asarray(v, np.float64), np.shape(r)).reshape(-1))
    defp = np.zeros((M, 3))
    for k in range(4):
        nk = anc[:, k]
        defp += wts[:, k:k + 1] * (np.einsum('mij,mj->mi', R[nk], src - g[nk]) + g[nk] + t[nk])
    zinv = 1.0 / (defp[:, 2] + 1e-7)
    mfx, mfy = -(fx * defp[:, 0] * zinv) * zinv, -(fy * defp[:, 1] * zinv) * zinv
    rowsM = np.arange(M) * 3
    for k in range(4):
        nk, wk = anc[:, k], wts[:, k]
        S = -fo.skew(wk[:, None] * np.einsum('mij,mj->mi', R[nk], src - g[nk]))
        for c in range(3):
            put(rowsM + c, 6 * nk + 3 + c, wk)
        for j in range(3):
            put(rowsM, 6 * nk + j, mfx * S[:, 2, j])
            put(rowsM + 1, 6 * nk + j, mfy * S[:, 2, j])
        for i in range(3):
            for j in range(3):
                put(rowsM + i, 6 * nk + j, S[:, i, j])
    res = [(defp - tgt).reshape(-1)]
    edges, _ = fo.gn_edges(P["edges"])
    E = edges.shape[0]
    la = math.sqrt(0.5)
    i0, i1 = edges[:, 0], edges[:, 1]
    delta = np.einsum('eij,ej->ei', R[i0], g[i1] - g[i0])
    res.append((la * (delta + g[i0] + t[i0] - (g[i1] + t[i1]))).reshape(-1))
    rowsE = 3 * M + np.arange(E) * 3
    for c in range(3):
        put(rowsE + c, 6 * i0 + 3 + c, la)
        put(rowsE + c, 6 * i1 + 3 + c, -la)
    Sa = -la * fo.skew(delta)
    for i in range(3):
        for j in range(3):
            put(rowsE + i, 6 * i0 + j, Sa[:, i, j])
    ids = np.arange(N)
    for c in range(3):
        put(3 * M + 3 * E + 3 * ids + c, 6 * ids + 3 + c, conf)
    res.append((conf[:, None] * (t + g - tpos)).reshape(-1))
    res = np.concatenate(res)
    J = sp.csr_matrix((np.concatenate(vv), (np.concatenate(rr), np.concatenate(cc))), shape=(res.size, 6 * N))
    A = (J.T @ J + lm * sp.eye(6 * N)).tocsr()
    return A, -(J.T @ res), float(np.linalg.norm(res))


def clusters(nodes, edges, c=8):
    N = nodes.shape[0]
    lab = -np.ones(N, np.int64)
    nxt = 0
    for s in range(N):
        if lab[s] >= 0:
            continue
        grp, front = [s], [s]
        lab[s] = nxt
        while len(grp) < c and front:
            cur = front.pop(0)
            for j in edges[cur]:
                if j >= 0 and lab[j] < 0 and len(grp) < c:
                    lab[j] = nxt
                    grp.append(j)
                    front.append(j)
        nxt += 1
    return [np.concatenate([np.arange(6 * m, 6 * m + 6) for m in np.nonzero(lab == l)[0]]) for l in range(nxt)]


def make_minv(A, groups):
    rows, cols, vals = [], [], []
    lmin_M = np.inf
    for idx in groups:
        blk = A[idx][:, idx].toarray()
        lmin_M = min(lmin_M, np.linalg.eigvalsh(blk)[0])
        inv = np.linalg.inv(blk)
        rr, cc = np.meshgrid(idx, idx, indexing="ij")
        rows.append(rr.ravel()); cols.append(cc.ravel()); vals.append(inv.ravel())
    Mi = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=A.shape)
    return Mi, lmin_M


def ritz_min(alphas, betas):
    k = len(alphas)
    d = np.empty(k)
    e = np.empty(max(k - 1, 0))
    for j in range(k):
        d[j] = 1.0 / alphas[j] + (betas[j - 1] / alphas[j - 1] if j > 0 else 0.0)
        if j < k - 1:
            e[j] = math.sqrt(betas[j]) / alphas[j]
    return float(eigvalsh_tridiagonal(d, e, select="i", select_range=(0, 0))[0])


def pcg(A, b, Mi, x0, stop, xstar=None, trace=None, maxit=5000):
    """Standard PCG (the pipelined product form is the same recurrence). stop(state) -> bool."""
    x = x0.copy()
    r = b - A @ x
    z = Mi @ r
    p = z.copy()
    gam = r @ z
    bb = b @ b
    alphas, betas = [], []
    for it in range(maxit):
        rr = r @ r
        th = ritz_min(alphas, betas) if alphas else None
        st = dict(it=it, rr=rr, bb=bb, gam=gam, theta=th, zz=z @ z)
        if trace is not None and xstar is not None:
            st["err"] = float(np.abs(x - xstar).max())
            st["err2"] = float(np.linalg.norm(x - xstar))
            trace.append(st)
        if gam == 0.0 or stop(st):
            return x, it
        q = A @ p
        a = gam / (p @ q)
        x += a * p
        r -= a * q
        z = Mi @ r
        g2 = r @ z
        beta = g2 / gam
        alphas.append(a)
        betas.append(beta)
        p = z + beta * p
        gam = g2
    return x, maxit


def galerkin(A, b, X):
    if not X:
        return np.zeros_like(b)
    Xm = np.stack(X, 1)
    G = Xm.T @ (A @ Xm)
    try:
        c = np.linalg.solve(G, Xm.T @ b)
    except np.linalg.LinAlgError:
        return np.zeros_like(b)
    return Xm @ c


def gn(P, stop, label, trace_step=None):
    N = P["nodes"].shape[0]
    R, t = np.tile(np.eye(3), (N, 1, 1)), np.zeros((N, 3))
    groups = clusters(P["nodes"], P["edges"])
    lm = 1e-7
    hist, its, losses = [], [], []
    Mi = None
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Mi is None:
            Mi, lminM = make_minv(A, groups)
        x0 = galerkin(A, b, hist[-4:])
        trace = [] if trace_step == gi else None
        xstar = spl.spsolve(A.tocsc(), b) if trace is not None else None
        x, it = pcg(A, b, Mi, x0, stop, xstar, trace)
        if trace is not None:
            for s in trace[::max(1, len(trace) // 40)] + trace[-1:]:
                th = s["theta"] or float("nan")
                print(f"  it {s['it']:4d} rel {math.sqrt(s['rr'] / s['bb']):.2e} err_inf {s['err']:.2e} err2 {s['err2']:.2e}"
                      f" sqrt(gam)/th {math.sqrt(s['gam']) / th:.2e} |r|/th {math.sqrt(s['rr']) / th:.2e}"
                      f" |z|/th {math.sqrt(s['zz']) / th:.2e} theta {th:.2e}")
            print(f"  lambda_min(A) {spl.eigsh(A, 1, sigma=0, which='LM')[0][0]:.3e}  lambda_min(M) {lminM:.3e}")
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    dR, dt = np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max()
    print(f"{label:40s} dR {dR:.2e} dt {dt:.2e} pcg {sum(its):5d} {its}", flush=True)


def rel(tol):
    return lambda s: s["rr"] <= tol * tol * s["bb"]


def err_rule(tau, kind, floor_rel=1e-12):
    """stop when the error estimate is below tau (absolute), or the residual hits floor_rel."""
    def f(s):
        if s["rr"] <= floor_rel ** 2 * s["bb"]:
            return True
        th = s["theta"]
        if th is None or s["it"] < 3:
            return False
        est = {"gam": math.sqrt(s["gam"]), "r": math.sqrt(s["rr"]), "z": math.sqrt(s["zz"])}[kind] / th
        return est <= tau
    return f


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "moose"
    P = load(name if name == "moose" else "gn_2k")
    if len(sys.argv) > 2 and sys.argv[2] == "trace":
        gn(P, rel(1e-10), "trace step 0 (tol 1e-10)", trace_step=0)
        gn(P, rel(1e-10), "trace step 5 (tol 1e-10)", trace_step=5)
        sys.exit(0)
    for tol in (1e-6, 1e-7, 1e-8, 1e-9):
        gn(P, rel(tol), f"rel {tol:g}")
    for kind in ("gam", "r", "z"):
        for tau in (1e-6, 1e-7):
            gn(P, err_rule(tau, kind), f"err[{kind}] tau {tau:g}")


def gn_prev_theta(P, tau, kind, label, rel_cap=None, step0_rel=1e-6):
    """stop rule with θ_min taken from the PREVIOUS GN step's final tridiagonal (step 0: relative residual
    step0_rel): est = (√gam | ‖r‖) / θ_prev <= tau, optionally also requiring rel <= rel_cap."""
    N = P["nodes"].shape[0]
    R, t = np.tile(np.eye(3), (N, 1, 1)), np.zeros((N, 3))
    groups = clusters(P["nodes"], P["edges"])
    lm = 1e-7
    hist, its, losses, thetas = [], [], [], []
    Mi = None
    th_prev = None
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Mi is None:
            Mi, _ = make_minv(A, groups)
        x0 = galerkin(A, b, hist[-4:])
        last = {}

        def stop(s):
            last.update(s)
            if th_prev is None:
                return s["rr"] <= step0_rel ** 2 * s["bb"]
            if rel_cap is not None and s["rr"] > rel_cap ** 2 * s["bb"]:
                return False
            if s["rr"] <= 1e-24 * s["bb"]:
                return True
            v = math.sqrt(s["gam"] if kind == "gam" else s["rr"])
            return v / th_prev <= tau
        x, it = pcg(A, b, Mi, x0, stop)
        th_prev = last.get("theta") or th_prev
        thetas.append(th_prev)
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    dR, dt = np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max()
    print(f"{label:40s} dR {dR:.2e} dt {dt:.2e} pcg {sum(its):5d} {its} theta {['%.1e' % v for v in thetas]}",
          flush=True)


SHIFTS = [0.5 ** (k / 1.0) * 0.25 for k in range(24)]   # 0.25 ... 3e-8, factor 2


def grid_rule(tau, kind, shifts=SHIFTS, floor_rel=1e-12):
    """the device form: θ̂ = the lower end of the shift bracket holding the smallest Ritz value of the current
    solve's tridiagonal (Sturm counts of T_k - σ_s I, updated O(1) per iteration per shift); stop when
    (√gam | ‖r‖) / θ̂ <= tau, or the relative residual reaches floor_rel."""
    def f(s):
        if s["rr"] <= floor_rel ** 2 * s["bb"]:
            return True
        th = s["theta"]
        if th is None:
            return False
        lo = shifts[-1] * 0.5
        for sg in shifts:          # descending: the first shift at or below θ is the bracket's lower end
            if sg <= th:
                lo = sg
                break
        v = math.sqrt(s["gam"] if kind == "gam" else s["rr"])
        return v <= tau * lo
    return f


def load_chain(name, f):
    """gn_2k / gn_4k frame f (the chained frame 1 starts from frame 0's oracle result), gn_1k, gn_small."""
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    if name in ("gn_1k", "gn_small"):
        return dict(nodes=g["nodes"], edges=g["edges"], tpos=g["tpos"], conf=g["conf"], src=g["src"], anc=g["anchors"],
                    wts=g["weights"], tgt=g["tgt"], intr=tuple(g["intr"]), R=g["R"], t=g["t"], loss=g["loss_total"],
                    R0=None, t0=None)
    p = f"f{f}_"
    return dict(nodes=g["nodes"], edges=g["edges"], tpos=g[p + "tpos"], conf=g[p + "conf"], src=g[p + "src"],
                anc=g[p + "anchors"], wts=g[p + "weights"], tgt=g[p + "tgt"], intr=tuple(g["intr"]), R=g[p + "R"],
                t=g[p + "t"], loss=g[p + "loss_total"], R0=g["f0_R"] if f else None, t0=g["f0_t"] if f else None)


def gn2(P, stop, label):
    """gn() from the fixture's starting pose, also reporting the loss log's max relative error."""
    N = P["nodes"].shape[0]
    R = np.tile(np.eye(3), (N, 1, 1)) if P.get("R0") is None else P["R0"].copy()
    t = np.zeros((N, 3)) if P.get("t0") is None else P["t0"].copy()
    groups = clusters(P["nodes"], P["edges"])
    lm = 1e-7
    hist, its, losses = [], [], []
    Mi = None
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = system(P, R, t, lm)
        if Mi is None:
            Mi, _ = make_minv(A, groups)
        x, it = pcg(A, b, Mi, galerkin(A, b, hist[-4:]), stop)
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    dR, dt = np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max()
    lr = np.abs(np.array(losses) / P["loss"][:len(losses)] - 1).max() if len(losses) == len(P["loss"]) else float("nan")
    print(f"{label:34s} dR {dR:.2e} dt {dt:.2e} loss {lr:.1e} pcg {sum(its):5d} {its}", flush=True)


def both_rule(tau, tol=1e-6, kind="gam"):
    """today's relative residual AND the error estimate (the estimate only tightens)."""
    g = grid_rule(tau, kind)
    return lambda s: (s["rr"] <= tol * tol * s["bb"] and g(s)) or s["rr"] <= 1e-24 * s["bb"]
