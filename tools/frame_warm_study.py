"""Tuning study (CPU, not product): PCG iterations of a frame's FIRST GN step when it starts from the previous
frame's solutions. Within a frame the product warm-starts steps 1-9 by the Galerkin projection on the last 4 step
solutions (tools/recycle_study.py); step 0 starts cold (x0 = 0), because the previous frame's last 4 solutions (its
steps 6-9: drift directions) did not help. Here the frame loop is chained (state carried, as prev_rot / prev_trans
carry it) on config 3's depth-mesh graph (tests/golden/gn_2k.npz) with the 8-node cluster block-Jacobi
preconditioner, tol 1e-6, and step 0 of every frame tries:
  cold     x0 = 0 (the product)
  last4    Galerkin on the previous frame's last 4 step solutions
  s0       Galerkin on the previous frame's step-0 solution
  s0s      Galerkin on [previous step 0, previous frame's total increment (sum of its 10 steps)]
  s0s2     s0s + the step-0 solution of the frame before

  python tools/frame_warm_study.py [first_frame] [n_frames]
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from occlusionfusion_amd import synthetic as S
from oracle import fusion_oracle as fo
import recycle_study as rs


def frame(prob, R, t, groups, x0_step0, tol=1e-6):
    N = R.shape[0]
    lm = 1e-7
    hist, its = [], []
    for k in range(10):
        if k % 3 == 2:
            lm /= 2
        A, b = prob.linearize(R, t, lm)
        Gi = rs.group_inv(A, groups)
        if k == 0:
            x0 = x0_step0(A, b) if x0_step0 else np.zeros(6 * N)
        else:
            x0 = rs.galerkin(A, b, np.stack(hist[-4:], 1))
        x, it = rs.pcg_g(A, b, Gi, x0, tol=tol)
        its.append(it)
        hist.append(x)
        R = fo.angle_axis_to_rotation_matrix(x.reshape(N, 6)[:, :3]) @ R
        t = t + x.reshape(N, 6)[:, 3:]
    return its, hist, R, t


def main():
    f0 = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = np.load(os.path.join(here, "tests/golden/gn_2k.npz"))
    seq = S.config_sequence(3, graph=(g["nodes"], g["edges"], g["edge_weights"]))
    N = seq.nodes.shape[0]
    groups = rs.cluster_groups(seq.nodes, seq.edges, 8)
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ("cold", "last4", "s0", "s0s", "s0s2")
    # one reference chain (cold step 0) supplies the state every frame starts from, so all modes see the same systems
    R = np.tile(np.eye(3), (N, 1, 1))
    t = np.zeros((N, 3))
    prev = []   # per frame: its 10 step solutions
    for q in range(nf):
        prob = rs.Problem(seq, f0 + q)
        row = {}
        for mode in modes:
            basis = None
            if prev:
                h = prev[-1]
                if mode == "last4":
                    basis = h[-4:]
                elif mode == "s0":
                    basis = [h[0]]
                elif mode == "s0s":
                    basis = [h[0], np.sum(h, 0)]
                elif mode == "s0s2":
                    basis = [h[0], np.sum(h, 0)] + ([prev[-2][0]] if len(prev) > 1 else [])
            start = (lambda A, b, X=basis: rs.galerkin(A, b, np.stack(X, 1))) if basis else None
            its, hist, R1, t1 = frame(prob, R, t, groups, start)
            row[mode] = its
            if mode == "cold":
                nxt = (hist, R1, t1)
        hist, R, t = nxt
        prev.append(hist)
        print(f"frame {f0 + q}: " + "  ".join(f"{m} {v[0]:4d} (frame {sum(v)})" for m, v in row.items()), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
