"""GPU, world_size 2 on one device over gloo: the match-sharded Gauss-Newton path
(GaussNewtonSolver.optimize_distributed: per-rank ofx_gn_linearize of a match range, all_reduce(sum)
of the block-sparse A and rhs, identical ofx_gn_step on every rank) against the single-process
solve and the dense f64 oracle fixture. RCCL needs one device per rank, so the collective here is
gloo on device tensors; the kernels and the exchange pattern are the multi-GPU ones.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(g):
    return (g["nodes"], g["edges"], g["edge_weights"], g["tpos"], g["conf"], g["src"], g["anchors"], g["weights"],
            g["tgt"], g["intr"])


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from occlusionfusion_amd import GaussNewtonSolver
        g = np.load(os.path.join(ROOT, "tests/golden/gn_small.npz"))
        s = GaussNewtonSolver(len(g["nodes"]), 1000)
        out = s.optimize_distributed(*_inputs(g), sync=True)
        q.put((rank, (out["node_rotations"].cpu().numpy(), out["node_translations"].cpu().numpy(),
                      out["valid_solve"])))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def test_gn_match_sharded_two_ranks(cuda, golden_dir):
    from occlusionfusion_amd import GaussNewtonSolver
    g = np.load(os.path.join(golden_dir, "gn_small.npz"))
    ref = GaussNewtonSolver(len(g["nodes"]), 1000).optimize(*_inputs(g))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
    (R0, t0, v0), (R1, t1, v1) = res[0], res[1]
    np.testing.assert_array_equal(R0, R1)      # every rank solves the identical all-reduced system
    np.testing.assert_array_equal(t0, t1)
    assert v0 == v1 == int(g["valid"])
    np.testing.assert_allclose(R0, ref["node_rotations"].cpu().numpy(), atol=1e-6, rtol=0)
    np.testing.assert_allclose(t0, ref["node_translations"].cpu().numpy(), atol=1e-6, rtol=0)
    np.testing.assert_allclose(R0, g["R"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(t0, g["t"], atol=1e-5, rtol=0)
