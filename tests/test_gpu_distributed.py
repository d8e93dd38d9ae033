"""GPU: the match-sharded Gauss-Newton path (GaussNewtonSolver.optimize_distributed: per-rank ofx_gn_linearize of
a match range, all_reduce(sum) of the block-sparse A and rhs, identical ofx_gn_step on every rank) against the
single-process solve and the dense f64 oracle fixture.
* world size 2 on one device over gloo (RCCL needs one device per rank): the kernels and the exchange pattern of
  the multi-GPU path, including an early stop decided on the non-fused step path (every rank leaves after the
  same GN step, so the collectives stay matched);
* world size 1 over RCCL (backend "nccl", initialised as bench.py does, device_id given): the device-tensor
  all_reduce of A and rhs, and the halo exchange's point-to-point pattern (batch_isend_irecv) with itself.
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


def _worker(rank, world, port, q, backend="gloo", params=None, p2p=False):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        if backend == "nccl":     # RCCL, as bench.py initialises it
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        from occlusionfusion_amd import GaussNewtonSolver
        g = np.load(os.path.join(ROOT, "tests/golden/gn_small.npz"))
        s = GaussNewtonSolver(len(g["nodes"]), 1000, **(params or {}))
        out = s.optimize_distributed(*_inputs(g), sync=True)
        res = [out["node_rotations"].cpu().numpy(), out["node_translations"].cpu().numpy(), out["valid_solve"],
               out["convergence_info"]["gn_iterations"]]
        if p2p:                   # the slab halo exchange's RCCL point-to-point pattern, rank 0 with itself
            from occlusionfusion_amd.sharding import _global
            x = torch.arange(1 << 16, dtype=torch.float32, device=dev)
            y = torch.empty_like(x)
            ops = [dist.P2POp(dist.isend, x, _global(0, None)), dist.P2POp(dist.irecv, y, _global(0, None))]
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            torch.cuda.synchronize()
            res.append(bool(torch.equal(x, y)))
        q.put((rank, tuple(res)))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def _run(world, backend="gloo", params=None, p2p=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, backend, params, p2p)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    return res


def test_gn_match_sharded_two_ranks(cuda, golden_dir):
    from occlusionfusion_amd import GaussNewtonSolver
    g = np.load(os.path.join(golden_dir, "gn_small.npz"))
    ref = GaussNewtonSolver(len(g["nodes"]), 1000).optimize(*_inputs(g))
    res = _run(2)
    (R0, t0, v0, _), (R1, t1, v1, _) = res[0], res[1]
    np.testing.assert_array_equal(R0, R1)      # every rank solves the identical all-reduced system
    np.testing.assert_array_equal(t0, t1)
    assert v0 == v1 == int(g["valid"])
    np.testing.assert_allclose(R0, ref["node_rotations"].cpu().numpy(), atol=1e-6, rtol=0)
    np.testing.assert_allclose(t0, ref["node_translations"].cpu().numpy(), atol=1e-6, rtol=0)
    np.testing.assert_allclose(R0, g["R"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(t0, g["t"], atol=1e-5, rtol=0)


def test_gn_distributed_stop_on_the_unfused_step_path(cuda, golden_dir):
    """The early stop (model.py:726-732) fires at GN step 1 (stop_loss_diff < 0) while PCG stops at its iteration cap
    (the step runs as k_step, which writes the host flag asynchronously): both ranks stop after the same step."""
    from occlusionfusion_amd import GaussNewtonSolver
    params = dict(pcg_max_iter=3, stop_loss_diff=-1e9)
    g = np.load(os.path.join(golden_dir, "gn_small.npz"))
    ref = GaussNewtonSolver(len(g["nodes"]), 1000, **params).optimize(*_inputs(g))
    res = _run(2, params=params)
    (R0, t0, v0, n0), (R1, t1, v1, n1) = res[0], res[1]
    assert n0 == n1 == ref["convergence_info"]["gn_iterations"] == 1
    np.testing.assert_array_equal(R0, R1)
    np.testing.assert_array_equal(t0, t1)
    np.testing.assert_allclose(R0, ref["node_rotations"].cpu().numpy(), atol=1e-9, rtol=0)
    np.testing.assert_allclose(t0, ref["node_translations"].cpu().numpy(), atol=1e-9, rtol=0)


def test_rccl_world1_allreduce_and_p2p(cuda, golden_dir):
    from occlusionfusion_amd import GaussNewtonSolver
    g = np.load(os.path.join(golden_dir, "gn_small.npz"))
    ref = GaussNewtonSolver(len(g["nodes"]), 1000).optimize(*_inputs(g))
    R, t, v, n, p2p_ok = _run(1, backend="nccl", p2p=True)[0]
    assert v == 1 and n == ref["convergence_info"]["gn_iterations"] and p2p_ok
    # all_reduce over one rank returns the rank's own system: the local solve's transforms
    np.testing.assert_allclose(R, ref["node_rotations"].cpu().numpy(), atol=1e-9, rtol=0)
    np.testing.assert_allclose(t, ref["node_translations"].cpu().numpy(), atol=1e-9, rtol=0)
    np.testing.assert_allclose(R, g["R"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(t, g["t"], atol=1e-5, rtol=0)
