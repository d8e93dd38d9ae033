"""Numerical study (CPU, not product): how far the PCG stop of each GN step can be relaxed while the 10-step GN
transforms stay within the 1e-5 bar of the f64 oracle fixtures. Runs errstop_study's numpy restatement of the product
loop (cluster block Jacobi, Galerkin warm start) from each fixture's starting pose under the product's current rule
(relative residual 1e-6 AND error estimate √γ/θ̂ <= 1e-5, θ̂ on the shift grid) and relaxed variants, and prints the
transforms' max error, the loss log's max relative error and the PCG iterations.

    python tools/stoprule_study.py [fixtures...]   (default: gn_2k:0 gn_2k:1 gn_1k moose gn_c5r1:0 gn_c5r7:0)
"""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from errstop_study import load, load_chain, gn2, grid_rule  # noqa: E402

TAU_DEVICE = None


def rule(tol, tau, min_it=0, kind="gam"):
    """relative residual <= tol AND (tau > 0) √γ/θ̂ <= tau, after min_it iterations; or the residual floor 1e-12"""
    g = grid_rule(tau, kind) if tau > 0 else (lambda s: True)

    def f(s):
        if s["rr"] <= 1e-24 * s["bb"]:
            return True
        return s["it"] >= min_it and s["rr"] <= tol * tol * s["bb"] and g(s)
    return f


RULES_ALL = [
    ("product: rel 1e-6 & err 1e-5", rule(1e-6, 1e-5)),
    ("rel 3e-6 & err 1e-5", rule(3e-6, 1e-5)),
    ("rel 1e-5 & err 1e-5", rule(1e-5, 1e-5)),
    ("rel 1e-5 & err 3e-6", rule(1e-5, 3e-6)),
    ("rel 3e-5 & err 3e-6", rule(3e-5, 3e-6)),
    ("err 3e-6 alone, >= 8 it", rule(1.0, 3e-6, 8)),
    ("err 1e-6 alone, >= 8 it", rule(1.0, 1e-6, 8)),
]


RULES2 = [
    ("product: rel 1e-6 & err 1e-5", rule(1e-6, 1e-5)),
    ("rel 2e-6 & err 1e-5", rule(2e-6, 1e-5)),
    ("rel 2e-6 & err 5e-6", rule(2e-6, 5e-6)),
    ("rel 3e-6 & err 5e-6", rule(3e-6, 5e-6)),
]
RULES = RULES2 if os.environ.get("RULES") == "2" else RULES_ALL


def fixture(spec):
    name, _, f = spec.partition(":")
    if name == "moose":
        P = load("moose")
        P["R0"] = P["t0"] = None
        return P
    return load_chain(name, int(f or 0))


if __name__ == "__main__":
    specs = sys.argv[1:] or ["gn_2k:0", "gn_2k:1", "gn_1k", "moose", "gn_c5r1:0", "gn_c5r7:0"]
    for spec in specs:
        P = fixture(spec)
        print(f"== {spec}: {P['nodes'].shape[0]} nodes", flush=True)
        for label, r in RULES:
            gn2(P, r, label)
