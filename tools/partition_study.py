"""Tuning study (CPU, not product): PCG iterations of one chained frame (10 GN steps, Galerkin warm start, tol 1e-6)
under the 8-node cluster block-Jacobi preconditioner for different node partitions of config 3's depth-mesh graph
(tests/golden/gn_2k.npz):
  bfs      the product's order_rows (gn.hip): BFS clusters from the lowest unassigned node, nearest-to-seed first,
           fragments first-fit packed by decreasing size into groups of 8 rows
  rcb      recursive coordinate bisection of the node positions (longest extent, median split) into parts of <= 8
  rcbN     rcb followed by N passes of pairwise boundary swaps that raise the in-part edge count

  python tools/partition_study.py [frame] [modes]
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from occlusionfusion_amd import synthetic as S
import recycle_study as rs
import frame_warm_study as fw

CS = 8


def bfs_groups(nodes, edges):
    N = nodes.shape[0]
    lab = -np.ones(N, np.int64)
    cl = []
    for s in range(N):
        if lab[s] >= 0:
            continue
        grp = [s]
        lab[s] = len(cl)
        front = [s]
        f = 0
        while f < len(front) and len(grp) < CS:
            cur = front[f]
            f += 1
            cand = []
            for j in edges[cur]:
                if j >= 0 and lab[j] < 0 and j not in cand:
                    cand.append(int(j))
            d = lambda j: float(((nodes[j].astype(np.float64) - nodes[s]) ** 2).sum())
            cand.sort(key=lambda j: (d(j), j))
            for j in cand:
                if len(grp) >= CS:
                    break
                lab[j] = len(cl)
                grp.append(j)
                front.append(j)
        cl.append(grp)
    order = sorted(range(len(cl)), key=lambda c: -len(cl[c]))
    fill, groups = [], []
    for c in order:
        k = 0
        while k < len(fill) and fill[k] + len(cl[c]) > CS:
            k += 1
        if k == len(fill):
            fill.append(0)
            groups.append([])
        fill[k] += len(cl[c])
        groups[k] += cl[c]
    return groups


def rcb_groups(nodes, idx=None):
    if idx is None:
        idx = np.arange(nodes.shape[0])
    if len(idx) <= CS:
        return [list(idx)]
    p = nodes[idx].astype(np.float64)
    ax = int(np.argmax(p.max(0) - p.min(0)))
    # split so that both halves fill whole parts of CS where possible
    nparts = -(-len(idx) // CS)
    left_parts = nparts // 2
    nl = min(len(idx) - 1, max(1, round(len(idx) * left_parts / nparts)))
    o = np.lexsort((idx, p[:, ax]))
    return rcb_groups(nodes, idx[o[:nl]]) + rcb_groups(nodes, idx[o[nl:]])


def refine(groups, edges, passes):
    """Greedy pairwise swaps between parts that raise the number of graph edges inside parts."""
    lab = {}
    for g, mem in enumerate(groups):
        for m in mem:
            lab[m] = g
    adj = {i: set(int(j) for j in edges[i] if j >= 0) for i in lab}
    for i in list(adj):
        for j in list(adj[i]):
            adj.setdefault(j, set()).add(i)

    def gain(i, g):   # edges of i into part g
        return sum(1 for j in adj[i] if lab[j] == g)

    for _ in range(passes):
        moved = 0
        for i in sorted(lab):
            gi = lab[i]
            best = None
            for j in sorted(adj[i]):
                gj = lab[j]
                if gj == gi:
                    continue
                for k in sorted(groups[gj]):
                    # swap i <-> k
                    d = (gain(i, gj) - gain(i, gi)) + (gain(k, gi) - gain(k, gj)) - 2 * (k in adj[i])
                    if d > 0 and (best is None or d > best[0]):
                        best = (d, k, gj)
            if best:
                _, k, gj = best
                groups[gi].remove(i); groups[gj].remove(k)
                groups[gi].append(k); groups[gj].append(i)
                lab[i], lab[k] = gj, gi
                moved += 1
        if not moved:
            break
    return groups


def edge_cut(groups, edges):
    lab = {m: g for g, mem in enumerate(groups) for m in mem}
    inside = sum(1 for i in lab for j in edges[i] if j >= 0 and lab[int(j)] == lab[i])
    total = sum(1 for i in lab for j in edges[i] if j >= 0)
    return inside / total


def main():
    fr = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ("bfs", "rcb", "rcb2")
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = np.load(os.path.join(here, "tests/golden/gn_2k.npz"))
    seq = S.config_sequence(3, graph=(g["nodes"], g["edges"], g["edge_weights"]))
    N = seq.nodes.shape[0]
    # the frame's start state: the chained cold-start solve of the frames before it (as frame_warm_study)
    R = np.tile(np.eye(3), (N, 1, 1))
    t = np.zeros((N, 3))
    base = bfs_groups(seq.nodes, seq.edges)
    for q in range(fr - 2, fr):
        _, _, R, t = fw.frame(rs.Problem(seq, q), R, t, base, None)
    prob = rs.Problem(seq, fr)
    for mode in modes:
        if mode == "bfs":
            groups = bfs_groups(seq.nodes, seq.edges)
        elif mode.startswith("rcb"):
            groups = rcb_groups(seq.nodes)
            if len(mode) > 3:
                groups = refine(groups, seq.edges, int(mode[3:]))
        elif mode.startswith("bfsr"):
            groups = refine(bfs_groups(seq.nodes, seq.edges), seq.edges, int(mode[4:]))
        full = sum(1 for x in groups if len(x) == CS)
        its, _, _, _ = fw.frame(prob, R, t, groups, None)
        print(f"{mode}: {len(groups)} groups ({full} full), in-part edges {edge_cut(groups, seq.edges):.3f}, "
              f"PCG {sum(its)} {its}", flush=True)


if __name__ == "__main__":
    main()
