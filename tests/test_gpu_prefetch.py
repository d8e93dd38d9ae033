"""GPU: the prefetched solver setup (ofx_gn_prepare / GaussNewtonSolver.optimize(prefetch=) — frame t+1's
upload and JᵀJ pattern built on the other solver slot while frame t solves) gives bit for bit the transforms
and the fused volume of the inline setup, over chained frames; a prefetch for a different problem is
discarded and set up inline."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def make_pipe(cuda, config=1):
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    c = S.BASELINE_CONFIGS[config]
    seq = S.config_sequence(config)
    D = c["dims"]
    pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=cuda)
    frames = [pipe.prepare(t) for t in range(7)]
    pipe.integrate_source(frames[0])
    return pipe, frames


def run(cuda, prefetch):
    pipe, frames = make_pipe(cuda)
    out = []
    for t in range(1, 6):
        res = pipe.solve(frames[t], frames[t + 1] if prefetch else None)
        pipe.integrate(frames[t], t)
        out.append((pipe.prev_rot.clone(), pipe.prev_trans.clone(), res["_status"].clone()))
    pipe.solver.drain()
    torch.cuda.synchronize()
    return pipe, out


def test_prefetched_setup_equals_inline(cuda):
    p0, ref = run(cuda, False)
    p1, got = run(cuda, True)
    used, missed = p1.solver.prefetch_stats()
    assert (used, missed) == (4, 0)          # frames 2..5 used the setup prefetched during the previous frame
    assert p0.solver.prefetch_stats() == (0, 0)
    for (R0, T0, s0), (R1, T1, s1) in zip(ref, got):
        assert torch.equal(R0, R1) and torch.equal(T0, T1) and torch.equal(s0, s1)
        assert int(s1[0]) == 1 and int(s1[1]) > 0
    for a, b in ((p0.vol.tsdf_b, p1.vol.tsdf_b), (p0.vol.weight_b, p1.vol.weight_b), (p0.vol.color_b, p1.vol.color_b)):
        assert torch.equal(a, b)


def test_prefetch_for_another_problem_is_discarded(cuda):
    pipe, frames = make_pipe(cuda)
    ref, _ = make_pipe(cuda)
    # prefetch frame 3, then solve frame 2: the prefetch no longer matches and is set up inline
    pipe.solve(frames[1], frames[3])
    ref.solve(frames[1])
    pipe.solve(frames[2])
    ref.solve(frames[2])
    torch.cuda.synchronize()
    assert pipe.solver.prefetch_stats() == (0, 1)
    assert torch.equal(pipe.prev_rot, ref.prev_rot) and torch.equal(pipe.prev_trans, ref.prev_trans)
