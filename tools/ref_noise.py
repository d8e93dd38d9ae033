"""Tuning study (not product): the reference's OWN numerical noise per GN step. DeformNet.optimize forms
A = JᵀJ as a dense f32 matmul and solves with f32 LU (model/model.py:641-709, torch f32). This compares that
f32 solution against the f64 solution of the same system (bench frame, 2073 nodes, 10k matches) on the GPU,
to size the PCG tolerance against the noise the reference itself carries."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import scipy.sparse as sp
import torch

import precond_study as ps
from occlusionfusion_amd import synthetic as S


def build_J(seq, t):
    src_A = ps.build_A   # reuse its row construction by re-running it with a capture of J
    captured = {}
    orig = sp.csr_matrix

    def grab(*a, **k):
        m = orig(*a, **k)
        if "J" not in captured and m.shape[1] % 6 == 0 and m.shape[0] > m.shape[1]:
            captured["J"] = m
        return m
    ps.sp.csr_matrix = grab
    try:
        src_A(seq, t)
    finally:
        ps.sp.csr_matrix = orig
    return captured["J"]


def main():
    dev = torch.device("cuda", 0)
    seq = S.SyntheticSequence.build(2000, seed=3)
    out = []
    for t in (4, 14):
        J = build_J(seq, t)
        n = J.shape[1]
        rng = np.random.default_rng(t)
        r = rng.normal(0, 1e-3, J.shape[0])
        Jd32 = torch.from_numpy(J.toarray().astype(np.float32)).to(dev)
        A32 = Jd32.T @ Jd32 + 1e-7 * torch.eye(n, device=dev)
        b32 = -(Jd32.T @ torch.from_numpy(r.astype(np.float32)).to(dev))
        LU, piv = torch.linalg.lu_factor(A32)
        x32 = torch.linalg.lu_solve(LU, piv, b32[:, None])[:, 0].double()
        del Jd32, LU
        Jd64 = torch.from_numpy(J.toarray()).to(dev)
        A64 = Jd64.T @ Jd64 + 1e-7 * torch.eye(n, device=dev, dtype=torch.float64)
        b64 = -(Jd64.T @ torch.from_numpy(r).to(dev))
        x64 = torch.linalg.solve(A64, b64)
        d = (x32 - x64)
        N = n // 6
        rec = {"frame": t, "n": n, "x_max": x64.abs().max().item(), "err_max": d.abs().max().item(),
               "err_rel": (d.norm() / x64.norm()).item(),
               "err_rot_max": d[:3 * N].abs().max().item(), "err_trans_max": d[3 * N:].abs().max().item()}
        # what a PCG relative-residual tolerance tau means for the same system: the solution error of an
        # f64 solve stopped at ||A x - b|| = tau ||b|| along the worst direction is <= cond * tau; report the
        # residual the f32 solution itself leaves: ||A64 x32 - b64|| / ||b64||
        rec["f32_relres"] = ((A64 @ x32 - b64).norm() / b64.norm()).item()
        out.append(rec)
        print(json.dumps(rec), flush=True)
        del Jd64, A64, A32
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
