"""Numerical study (CPU, not product): the GN steps' cluster preconditioner refresh and the error-based PCG stop, on
every f64 oracle fixture (tests/golden: the moose demo pair, gn_2k frames 0/1, gn_1k, gn_4k, gn_c5r1, gn_small).

numpy restatement of the product's loop (tools/errstop_study.py: BFS clusters of 8, Galerkin warm start over the last 4
step solutions, 10 GN steps) with
  * the refresh policy: "never" (round 4: one cluster inverse per solve), "always", or rebuilt when some node's
    accumulated rotation Σ|ω| since the last rebuild passes a threshold (the product's precond_rot_tol);
  * the stop: relative residual 2e-6 AND √γ/θ̂ <= 1e-5, θ̂ the bracket of the smallest Ritz value on the shift grid
    (ratio √2: round 4; 2^(1/4): round 5), optionally min(θ̂, the previous GN step's final θ̂) ("carry").
Prints PCG iterations per GN step and the transforms' max error against the fixture.

  python tools/refresh_study.py [policy|stop]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import errstop_study as es  # noqa: E402
from oracle import fusion_oracle as fo  # noqa: E402


def shifts(q):
    return [2.0 ** (-k * q) for k in range(64)]


def theta_hat(th, sh):
    if th is None:
        return None
    for s in sh:
        if s <= th:
            return s
    return 0.0


def run(P, tol=2e-6, tau=1e-5, q=0.25, carry=True, refresh=0.1, policy=None, maxit=2000):
    N = P["nodes"].shape[0]
    R = np.tile(np.eye(3), (N, 1, 1)) if P.get("R0") is None else P["R0"].copy()
    t = np.zeros((N, 3)) if P.get("t0") is None else P["t0"].copy()
    groups = es.clusters(P["nodes"], P["edges"], 8)
    sh = shifts(q)
    lm = 1e-7
    hist, its, losses, acc, Mi, prev = [], [], [], np.zeros(N), None, None
    for gi in range(10):
        if gi % 3 == 2:
            lm /= 2
        A, b, loss = es.system(P, R, t, lm)
        fresh = Mi is None or (policy == "always") or (policy is None and refresh > 0 and acc.max() > refresh)
        if fresh:
            Mi, _ = es.make_minv(A, groups)
            acc[:] = 0
        last = {}

        def stop(s):
            last.update(s)
            if s["rr"] <= 1e-24 * s["bb"] or s["gam"] == 0:
                return True
            if s["rr"] > tol * tol * s["bb"]:
                return False
            if tau <= 0:
                return True
            th = theta_hat(s["theta"], sh)
            th = 1.0 if th is None else th
            if carry and prev is not None:
                th = min(th, prev)
            return math.sqrt(s["gam"]) <= tau * th
        x, it = es.pcg(A, b, Mi, es.galerkin(A, b, hist[-4:]), stop, maxit=maxit)
        if last.get("theta") is not None:
            prev = theta_hat(last["theta"], sh)
        if losses and (loss - losses[-1] > 1.0 or loss == losses[-1]):
            break
        losses.append(loss)
        its.append(it)
        hist.append(x)
        xr = x.reshape(N, 6)
        acc += np.linalg.norm(xr[:, :3], axis=1)
        R = fo.angle_axis_to_rotation_matrix(xr[:, :3]) @ R
        t = t + xr[:, 3:]
    return sum(its), max(np.abs(R - P["R"]).max(), np.abs(t - P["t"]).max()), its


def cases():
    yield "moose", es.load("moose")
    for n, f in (("gn_2k", 0), ("gn_2k", 1), ("gn_1k", 0), ("gn_4k", 0), ("gn_c5r1", 0), ("gn_c5r7", 0),
                 ("gn_small", 0)):
        yield f"{n}f{f}", es.load_chain(n, f)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "stop"
    if what == "policy":
        variants = [("never", dict(refresh=0, q=0.5, carry=False)), ("always", dict(policy="always")),
                    ("rot>0.02", dict(refresh=0.02)), ("rot>0.05", dict(refresh=0.05)), ("rot>0.1", dict(refresh=0.1))]
    else:
        variants = [("round 4 (no refresh, sqrt2 grid)", dict(refresh=0, q=0.5, carry=False)),
                    ("refresh", dict(q=0.5, carry=False)),
                    ("refresh + 2^(1/4) grid", dict(carry=False)),
                    ("refresh + grid + carry (product)", dict()),
                    ("... + residual 5e-6", dict(tol=5e-6)),
                    ("... + residual 1e-5, tau 2e-5", dict(tol=1e-5, tau=2e-5))]
    for name, P in cases():
        for lab, kw in variants:
            s, e, its = run(P, **kw)
            print(f"{name:10s} {lab:36s} pcg {s:5d} err {e:.2e} {its}", flush=True)
