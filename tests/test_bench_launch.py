"""bench.py's multi-rank launcher on the CPU (gloo): `--gpus N` starts N rank processes itself (a
torch.distributed.run child) and reports n_gpus = N with one per-rank record each; a world size that
differs from --gpus is refused. The device work is skipped (--launch-check), the plumbing (process group,
barrier, max-over-ranks timing, per-rank gather) is the bench's own."""
import json
import os
import subprocess
import sys

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


def test_gpus3_shard_mode():
    r = _bench("--gpus", "3", "--launch-check", "--backend", "gloo", "--steps", "1", "--mode", "shard")
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 3 and d["mode"] == "shard" and len(d["per_rank"]) == 3


def test_world_size_must_match_gpus():
    r = _bench("--gpus", "2", "--launch-check", env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE 1 != --gpus 2" in (r.stderr + r.stdout)
