"""GPU: the prefetched solver setup (ofx_gn_prepare / GaussNewtonSolver.optimize(prefetch=) — frame t+1's
upload and JᵀJ pattern built on the other solver slot while frame t solves) gives bit for bit the transforms
and the fused volume of the inline setup, over chained frames, whether the setup starts when the previous solve
returns or during its last GN steps (ofx_gn_prepare_after); a prefetch for a different problem is discarded and set
up inline; a gated prefetch whose trigger never solves still runs."""
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


def run(cuda, prefetch, lead=1):
    pipe, frames = make_pipe(cuda)
    pipe.solver.prefetch_lead = lead
    out = []
    for t in range(1, 6):
        res = pipe.solve(frames[t], frames[t + 1] if prefetch else None)
        pipe.integrate(frames[t], t)
        out.append((pipe.prev_rot.clone(), pipe.prev_trans.clone(), res["_status"].clone()))
    pipe.solver.drain()
    torch.cuda.synchronize()
    return pipe, out


@pytest.mark.parametrize("lead", [0, 1, 3, 10])
def test_prefetched_setup_equals_inline(cuda, lead):
    p0, ref = run(cuda, False)
    p1, got = run(cuda, True, lead)
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


def test_discarded_larger_prefetch_is_ordered_before_the_inline_setup(cuda):
    """A prefetch is discarded while its side-stream setup may still run, and that setup reallocates the slot's
    buffers (its problem is larger than any the slot held): the miss solve, issued right away, must wait for all of
    it (ofx_gn_solve fences the side stream whether or not the prefetch is used) and equal the plain solve."""
    from occlusionfusion_amd import GaussNewtonSolver
    from occlusionfusion_amd.pipeline import FusionPipeline, FrameInputs
    from occlusionfusion_amd import synthetic as S
    c = S.BASELINE_CONFIGS[1]
    seq = S.config_sequence(1, device=cuda)
    D = c["dims"]

    def pipeline():
        p = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), n_matches=3000, device=cuda)
        p.solver = GaussNewtonSolver(len(seq.nodes), 10000, cuda)   # room for the larger prefetched problem
        fr = [p.prepare(t) for t in range(6)]
        p.integrate_source(fr[0])
        return p, fr

    pipe, frames = pipeline()
    ref, rframes = pipeline()
    big = FrameInputs(im=frames[3].im, tpos=frames[3].tpos, conf=frames[3].conf,
                      **{k: torch.cat([getattr(frames[t], k) for t in (3, 4, 5)])
                         for k in ("src", "anchors", "weights", "tgt")})
    assert big.src.shape[0] > 2 * frames[1].src.shape[0]
    pipe.solve(frames[1], frames[2])          # slot 1 set up for frame 2
    pipe.solve(frames[2], big)                # frame 2 uses it; slot 0 (sized for frame 1) prefetches 3x the matches
    pipe.solve(frames[3])                     # miss, issued at once: inline setup on slot 0
    for t in (1, 2, 3):
        ref.solve(rframes[t])
    torch.cuda.synchronize()
    assert pipe.solver.prefetch_stats() == (1, 1)
    assert torch.equal(pipe.prev_rot, ref.prev_rot) and torch.equal(pipe.prev_trans, ref.prev_trans)


@pytest.mark.parametrize("destroy_trigger", [False, True])
def test_gated_prefetch_without_its_trigger_solve(cuda, destroy_trigger):
    """ofx_gn_prepare_after with a trigger handle that never solves: the prefetch starts when the solve that uses it
    waits for it, or when the trigger handle is destroyed, and gives the inline result."""
    from occlusionfusion_amd import _lib
    pipe, frames = make_pipe(cuda)
    ref, _ = make_pipe(cuda)
    s = pipe.solver
    pipe.solve(frames[1])
    ref.solve(frames[1])
    trig, _ = s._new_slot()
    q = pipe.problem(frames[2])
    pa, _, _ = s._problem(q["graph_nodes"], q["graph_edges"], q["graph_edges_weights"], q["target_node_position"],
                          q["node_confidence"], q["source_points"], q["anchors"], q["weights"], q["target_points"],
                          pipe.intr, None, None, None, None, keep=False)
    before = torch.cuda.Event()
    before.record()
    s._prefetch(pa, before, trig, 0, *s._plist())
    s._cur = 1 - s._cur
    if destroy_trigger:
        _lib.lib.ofx_gn_destroy(trig)
    pipe.solve(frames[2])
    ref.solve(frames[2])
    torch.cuda.synchronize()
    if not destroy_trigger:
        _lib.lib.ofx_gn_destroy(trig)
    assert s.prefetch_stats() == (1, 0)
    assert torch.equal(pipe.prev_rot, ref.prev_rot) and torch.equal(pipe.prev_trans, ref.prev_trans)


def test_overlapped_integrate_equals_sequential(cuda):
    """FusionPipeline(overlap=True) (bench.py's default): frame t's integrate on a stream of its own, beside frame t+1's
    solve, enqueued by the host inside that solve (GaussNewtonSolver.defer_to_next_solve) — the same transforms and
    bit for bit the same fused volume and per-brick update counts as the sequential loop, with the prefetched setup
    on as well."""
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    res = []
    for overlap in (False, True):
        c = S.BASELINE_CONFIGS[1]
        seq = S.config_sequence(1)
        D = c["dims"]
        pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=cuda, overlap=overlap)
        frames = [pipe.prepare(t) for t in range(8)]
        pipe.integrate_source(frames[0])
        outs = []
        for t in range(1, 7):
            pipe.solve(frames[t], frames[t + 1])
            pipe.integrate(frames[t], t, count_updates=True)
            outs.append((pipe.prev_rot, pipe.prev_trans))
        pipe.flush()
        pipe.solver.drain()
        torch.cuda.synchronize()
        assert (pipe.int_stream is not None) == overlap
        res.append((pipe, outs))
    (p0, o0), (p1, o1) = res
    for (R0, T0), (R1, T1) in zip(o0, o1):
        assert torch.equal(R0, R1) and torch.equal(T0, T1)
    for a, b in ((p0.vol.tsdf_b, p1.vol.tsdf_b), (p0.vol.weight_b, p1.vol.weight_b), (p0.vol.color_b, p1.vol.color_b),
                 (p0.vol.n_updated, p1.vol.n_updated)):
        assert torch.equal(a, b)
