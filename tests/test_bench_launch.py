"""bench.py's multi-rank launcher on the CPU (gloo): `--gpus N` starts N rank processes itself (a
torch.distributed.run child) and reports n_gpus = N with one per-rank record each; a world size that
differs from --gpus is refused. The device work is skipped (--launch-check), the plumbing (process group,
barrier, max-over-ranks timing, per-rank gather) is the bench's own."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = dict(os.environ, OMP_NUM_THREADS="1")
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_gpus2_starts_two_ranks():
    r = _bench("--gpus", "2", "--launch-check", "--backend", "gloo", "--steps", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert [p["rank"] for p in d["per_rank"]] == [0, 1]
    assert len({p["pid"] for p in d["per_rank"]}) == 2          # two processes, not one
    assert d["max_elapsed_s"] == max(p["elapsed_s"] for p in d["per_rank"])


def test_config5_replicas_run_independent_scenes():
    """BASELINE config 5 (the default at --gpus N > 1): one independent scene per rank, rank 0 = config 3."""
    from occlusionfusion_amd import synthetic as S
    r = _bench("--gpus", "2", "--launch-check", "--backend", "gloo", "--steps", "1", "--config", "5")
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    seeds = [p["scene_seed"] for p in d["per_rank"]]
    assert len(set(seeds)) == 2 and seeds[0] == S.BASELINE_CONFIGS[3]["seed"]
    assert d["per_rank"][0]["scene"] != d["per_rank"][1]["scene"]
    r = _bench("--gpus", "2", "--launch-check", "--backend", "gloo", "--steps", "1")   # default config at N > 1
    assert r.returncode == 0 and [p["config"] for p in _line(r.stdout)["per_rank"]] == [5, 5]
    s0, s1 = S.config_scene(5, 0), S.config_scene(5, 1)
    cam = S.bench_camera(4)
    assert s0[0] == S.config_scene(3)[0] and s0[1] == S.config_scene(3)[1]
    assert not np.array_equal(S.frame_depth(s0[0], cam, s0[1], 2), S.frame_depth(s1[0], cam, s1[1], 2))


def test_gpus3_shard_mode():
    r = _bench("--gpus", "3", "--launch-check", "--backend", "gloo", "--steps", "1", "--mode", "shard")
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 3 and d["mode"] == "shard" and len(d["per_rank"]) == 3


def test_world_size_must_match_gpus():
    r = _bench("--gpus", "2", "--launch-check", env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE 1 != --gpus 2" in (r.stderr + r.stdout)
