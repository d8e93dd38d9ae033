"""Fusion frames/sec (warp + integrate + solve), 640x480 (->640x448) synthetic depth -> 512³ TSDF @4 mm,
~2k-node ED graph, 10k matches, on MI355X.

One step = one frame of the reference's fusion loop (lepard_nicp_test.py:test4): GN solve
(DeformNet.optimize formulation, 10 iterations) -> update node transforms -> fused skin-cache warp +
TSDF/weight/colour integrate of the new frame. All inputs are device-resident before timing.

  python bench.py [--gpus N --steps K --warmup W] [--config 1..5] [--mode replicas|shard]
                  [--solve replicated|allreduce] [--dims 512] [--nodes 2000]

--gpus N > 1 without a torch.distributed environment: bench.py starts N ranks itself (a child
    `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...` running this file,
    started before anything touches the GPU) and exits with its status; under torchrun it checks
    WORLD_SIZE == --gpus.
--config (BASELINE.json configs): 3 (default at --gpus 1) 512³ @4 mm, ~2k nodes, non-rigid + occluder; 2 256³
    @4 mm, ~1k nodes, rigid sequence; 1 128³ @8 mm, 200 nodes, 320x240 camera; 4 1024³ @2 mm, ~4k nodes;
    5 (default at --gpus N > 1) = one independent config-3-class scene per GPU in replicas mode: rank 0 runs
    config 3 itself, rank r its own seeded scene (synthetic.config_scene), so N=1 and rank 0 are the same workload.
    Every graph is the SURVEY §8(d) depth-mesh graph of the source frame (sample_nodes + 8 geodesic edges, built on
    the device: synthetic.depth_graph).
--mode replicas (default, BASELINE config 5): one independent scene per GPU, no collective,
    value = frames of all ranks / max-rank time (weak scaling).
--mode shard (BASELINE config 4 style): ONE volume, its bricks dealt to ranks by spatial hash bucket
    (each rank skins and integrates only its bricks); the solve is replicated (--solve replicated: every
    rank assembles all matches, no collective) or match-sharded (--solve allreduce: one RCCL all-reduce
    of the GN JᵀJ/Jᵀr accumulators per GN iteration); value = frames / time (strong scaling).
--launch-check: rank plumbing only (process group, barrier, max-over-ranks timing, per-rank gather) with
    no device work — what tests/test_bench_launch.py runs on the CPU over gloo.
"""
import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM = 8.0e12   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# tools/pmc_traffic.sh + tools/pmc_summary.py: the newest round's summary
PMC_FILE = next((f for f in (os.path.join(ROOT, "profiles", f"r{r:02d}_pmc_traffic.json") for r in range(9, 0, -1))
                 if os.path.exists(f)), os.path.join(ROOT, "profiles", "r05_pmc_traffic.json"))

from occlusionfusion_amd.synthetic import BASELINE_CONFIGS as CONFIGS  # noqa: E402  (configs 1-5)


def pmc_traffic(kernel, workload, extra=()):
    """Per-launch HBM bytes of `kernel` (+ the kernels in `extra` that run once per launch of it, if measured) from the
    committed rocprofv3 PMC summary (separate counter passes cannot run inside the timed bench) — only when that
    summary was measured on this very workload; otherwise None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        if d.get("workload") != workload:
            return None
        return d["kernels"][kernel]["traffic_bytes"] + sum(d["kernels"][k]["traffic_bytes"] for k in extra
                                                           if k in d["kernels"])
    except (OSError, KeyError, ValueError):
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", type=int, choices=sorted(CONFIGS), default=None)
    p.add_argument("--mode", choices=["replicas", "shard"], default="replicas")
    p.add_argument("--solve", choices=["replicated", "allreduce"], default="replicated",
                   help="shard mode: replicated assembly (no collective) or match-sharded + all-reduce")
    p.add_argument("--dims", type=int, default=None)
    p.add_argument("--voxel", type=float, default=None)
    p.add_argument("--nodes", type=int, default=None)
    p.add_argument("--matches", type=int, default=10000)
    p.add_argument("--scene-rank", type=int, default=None,
                   help="config 5: run this rank's independent scene (default: the process's own rank)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--gn", action="append", default=[], metavar="KEY=VALUE", help=argparse.SUPPRESS)   # (A/B: GN params)
    p.add_argument("--no-prefetch", dest="prefetch", action="store_false",
                   help="set up each frame's solve inline instead of prefetching it during the previous frame")
    p.add_argument("--no-overlap", dest="overlap", action="store_false",
                   help="run each frame's integrate on the solve's stream (default: on a stream of its own, beside the "
                        "next frame's solve, which needs only this frame's transforms)")
    p.add_argument("--cpu-sample", type=int, default=1 << 24)
    p.add_argument("--json-out", default=None)
    p.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--moose", action="store_true",
                   help="time the reference's real solver input instead (NonRigidICP moose demo pair, "
                        "tests/golden/moose.npz): ms per GN optimize, PCG iterations, error against the f64 oracle")
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL; gloo for "
                                                   "CPU launch checks and rehearsals with ranks sharing a device)")
    a = p.parse_args()
    if a.config is None:
        a.config = 5 if a.gpus > 1 and a.mode == "replicas" else 3
    cfg = dict(CONFIGS[a.config])
    for k in ("dims", "voxel", "nodes"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    a.cfg = cfg
    if a.backend is None:
        a.backend = "gloo" if a.launch_check else "nccl"
    return a


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a):
    """Start --gpus ranks as fresh processes (torch.distributed.run, one per GPU) before any GPU call and
    return their exit status. The child processes re-enter main() with WORLD_SIZE set."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    return subprocess.run(cmd, env=env).returncode


def launch_check(a, world, rank):
    """Plumbing of the multi-rank bench without device work: the same barrier / max-over-ranks / gather."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(a.backend)
        dist.barrier()
    t0 = time.perf_counter()
    x = torch.ones(1 << 16)
    for _ in range(a.steps):
        x = x * 1.0001
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64)
    from occlusionfusion_amd.synthetic import config_scene
    scene, seed = config_scene(a.config, rank if a.mode == "replicas" else 0)   # the workload this rank would run
    mine = {"rank": rank, "pid": os.getpid(), "elapsed_s": elapsed, "config": a.config, "scene_seed": seed,
            "scene": {"center": list(scene.center), "radius": scene.radius, "phase": scene.phase}}
    per_rank = [mine]
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "steps": a.steps, "mode": a.mode,
                          "backend": a.backend, "max_elapsed_s": float(el.item()), "per_rank": per_rank}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE {world} != --gpus {a.gpus}")
    if a.launch_check:
        return launch_check(a, world, rank)
    if a.moose:
        return moose_bench(a)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())   # rehearsals: several ranks may share one device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline

    cfg = a.cfg
    D = a.dims
    origin = cfg["origin"] if (a.dims, a.voxel) == (cfg["dims"], cfg["voxel"]) else \
        (-D * a.voxel / 2, -D * a.voxel / 2, 0.5)
    scene_rank = (a.scene_rank if a.scene_rank is not None else rank) if a.mode == "replicas" else 0
    seq = S.config_sequence(a.config, a.nodes, rank=scene_rank, device=dev)
    scene_seed = int(seq.seed)
    sharded = a.mode == "shard" and world > 1
    shard = (rank, world, "hash") if sharded else None   # spatial-hash brick buckets (sharding.hash_owner)
    gn_over = {}
    for kv in a.gn:   # (tuning A/B only; the bench line is quoted at the defaults)
        k, v = kv.split("=", 1)
        gn_over[k] = v if k == "precond" else float(v)
    pipe = FusionPipeline(seq, origin, a.voxel, (D, D, D), n_matches=a.matches, device=dev, shard=shard,
                          gn_params=gn_over or None, overlap=a.overlap)
    total = a.warmup + a.steps + 1
    frames = [pipe.prepare(t) for t in range(total + 1)]   # + the frame the last timed step prefetches
    torch.cuda.synchronize()
    pipe.integrate_source(frames[0])
    cache = pipe.wf.skin_tsdf_cache()
    K = cache.k
    n_skin_valid = int((cache.anchors.view(-1, 4)[:, K - 1] != -1).sum().item()) if cache.n_list else 0
    torch.cuda.synchronize()
    allreduce = sharded and a.solve == "allreduce"
    ar_events = []

    prefetch = a.prefetch and not allreduce

    def solve(fi, nxt):
        if allreduce:
            out = pipe.solver.optimize_distributed(pipe.nodes_t, pipe.edges_t, pipe.ew_t, fi.tpos, fi.conf, fi.src,
                                                   fi.anchors, fi.weights, fi.tgt, pipe.intr, prev_rot=pipe.prev_rot,
                                                   prev_trans=pipe.prev_trans, sync=False, timer=ar_events)
            pipe.prev_rot, pipe.prev_trans = out["node_rotations"], out["node_translations"]
            return out
        # software pipelining: frame t+1's solver setup runs on the other solver slot while frame t solves
        return pipe.solve(fi, nxt if prefetch else None)

    ev = lambda: torch.cuda.Event(enable_timing=True)
    # overlapped integrates: the frame loop's solves go on a stream of the greatest priority, so the hardware queues
    # dispatch the latency-bound solve chain's workgroups ahead of the integrate beside it (default priority)
    loop_stream = torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1]) if a.overlap else None
    loop_ctx = torch.cuda.stream(loop_stream) if loop_stream is not None else contextlib.nullcontext()
    loop_ctx.__enter__()
    for t in range(1, 1 + a.warmup):
        solve(frames[t], frames[t + 1])
        pipe.integrate(frames[t], t)
    pipe.flush()   # (the last warmup frame's integrate: not inside the timed region)
    pipe.solver.drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ar_events.clear()
    marks = []
    upd = []
    pipe.solver.timing(True)               # arm hipEvent timing of the PCG loops (same stream)
    pipe.vol.integrate_timing(True)        # library hipEvents around each warped integrate launch (same stream)
    t0 = time.perf_counter()
    for t in range(1 + a.warmup, total):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        out = solve(frames[t], frames[t + 1])
        e1.record()
        # (one device reduce of the update counts per frame, on the integrate's stream right after it; read after timing)
        ie = pipe.integrate(frames[t], t, count_updates=True,
                            after=lambda: upd.append(pipe.vol.n_updated[:cache.n_list].sum(dtype=torch.int32)))
        if ie is None:   # (sequential: the integrate on the solve's stream)
            e2.record()
            marks.append((e0, e1, (e1, e2), out))
        else:            # (overlapped: its events on its own stream, recorded when it is enqueued — in the next solve)
            marks.append((e0, e1, ie, out))
    pipe.flush()          # (the last timed frame's integrate, enqueued now: inside the timed region)
    pipe.solver.drain()   # the last step's prefetched setup (of a frame not timed) counts inside the region
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    loop_ctx.__exit__(None, None, None)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed_max = float(el.item())
    pcg_ms, pcg_launches, _ = pipe.solver.timing(False)
    pf_used, pf_missed = pipe.solver.prefetch_stats()
    N_, M_, nnzb, _T, rows = pipe.solver.info()
    pci = pipe.solver.precond_info()
    t_solve = np.array([m[0].elapsed_time(m[1]) for m in marks]) * 1e-3
    t_int = np.array([m[2][0].elapsed_time(m[2][1]) for m in marks]) * 1e-3
    pcg = [int(m[3]["_status"][2].item()) for m in marks]
    gn_it = [int(m[3]["_status"][1].item()) for m in marks]
    valid = [int(m[3]["_status"][0].item()) for m in marks]
    U = float(np.mean([int(u.item()) for u in upd]))
    kint_ms, kint_n = pipe.vol.integrate_timing(False)
    t_kint_loop = kint_ms * 1e-3 / max(1, kint_n)
    # The same launch in isolation (after the timed region, untimed for `value`): in the frame loop the
    # integrate shares the GPU with the next frame's prefetched solver setup, so its in-loop
    # duration is not the kernel's own. Re-integrating the last frame into a scratch copy of the volume runs
    # the identical work (same listed bricks, skins, depth: the update set does not depend on old values).
    vol = pipe.vol
    keep = (vol.tsdf_b, vol.weight_b, vol.color_b)
    vol.tsdf_b, vol.weight_b, vol.color_b = (x.clone() for x in keep)
    torch.cuda.synchronize()
    vol.integrate_timing(True)
    # on a stream of its own: a launch on the legacy null stream waits for every other blocking stream the frame loop
    # created (solve, integrate, prefetch slots), and those cross-stream waits landed between the three kernels the
    # events bracket (140-150 us per launch instead of the kernels' 80)
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        for _ in range(20):
            vol.integrate_device(count_updates=True)
    torch.cuda.synchronize()
    kiso_ms, kiso_n = vol.integrate_timing(False)
    vol.tsdf_b, vol.weight_b, vol.color_b = keep
    t_kint = kiso_ms * 1e-3 / max(1, kiso_n)
    t_ar = (sum(x.elapsed_time(y) for x, y in ar_events) * 1e-3 / a.steps) if ar_events else 0.0
    mine = {"rank": rank, "device": local, "scene_seed": scene_seed, "nodes": int(seq.nodes.shape[0]),
            "ms_per_frame": 1e3 * elapsed / a.steps,
            "solve_ms": 1e3 * float(np.mean(t_solve)), "allreduce_ms": 1e3 * t_ar,
            "integrate_ms": 1e3 * float(np.mean(t_int)), "integrate_kernel_us": 1e6 * t_kint_loop,
            "listed_bricks": cache.n_list, "updated_voxels": U, "pcg_iters_per_frame": float(np.mean(pcg))}
    per_rank = [mine]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    frames_done = a.steps * (world if a.mode == "replicas" else 1)
    value = frames_done / elapsed_max
    # algorithmic bytes of one integrate launch: palette-rank anchors 4 B per voxel
    # of every listed brick + the brick's palette (64 x u16 + count); weights 16 B + tsdf/weight 8 B read
    # per skin-valid voxel; per updated voxel tsdf/weight write 8 B + colour read+write 8 B. Node records
    # and the depth/colour images are L2-resident and not counted.
    B_listed = cache.n_list * (512 * 4 + 132) + n_skin_valid * 24 + U * 16
    # with the brick cull (ofx_integrate_palette_cull, the default): the bricks it keeps move those bytes, every listed
    # brick its palette count + ids (132 B) and flag (1 B) through the cull, and the depth image is read once for the
    # tile maxima; the timed span covers the three kernels
    act = getattr(vol, "_cull", None) if getattr(vol, "brick_cull", False) else None
    if act is not None and cache.n_list:
        live = act[1][:cache.n_list].to(torch.bool)
        sv_slot = (cache.anchors.view(cache.n_list, 512, 4)[:, :, K - 1] != -1).sum(1)
        n_live, sv_live = int(live.sum().item()), int(sv_slot[live].sum().item())
        H_, W_ = (int(v) for v in vol.depth_t.shape)
        B = n_live * (512 * 4 + 132) + cache.n_list * 133 + H_ * W_ * 4 + sv_live * 24 + U * 16
    else:
        n_live, sv_live, B = cache.n_list, n_skin_valid, B_listed
    achieved = B / t_kint
    # SURVEY §8(d)'s per-unit figure over the voxels this launch processes (every voxel of a listed brick):
    # 32 B skin + 8 B tsdf/weight read per voxel, 8 B tsdf/weight write per updated voxel (colour separately)
    B_survey = cache.n_list * 512 * 40 + U * 8
    # k_pcg_iter algorithmic (unique) bytes per PCG iteration: per JᵀJ block its 6x6 f64 values (288 B) + its
    # (col, slot) wave-list entry (8 B); per PCG row (nodes in cluster order, padded) the cluster-inverse
    # rows (6 x 48 f32 = 1152 B), the 8-vector state read + written (2 x 384 B), m read (48 B; the
    # neighbour gathers re-read these) and the new m written (48 B). DESIGN.md §5. Launches after the
    # converging one (drained: they end after the first memory trip) move no algorithmic bytes, so the
    # per-launch figure is iterations x bytes / launches, over the same launches rocprof averages.
    B_pcg = nnzb * 296 + rows * (1152 + 768 + 48 + 48)
    if pci["schwarz"]:
        # overlapping Schwarz (the default): an iteration is k_pcg_iter without the cluster inverse (the state, own m,
        # w_new written: 768 + 48 + 48 B per row) + k_as_apply: per segment its fp16 inverse row (2 B per entry), row scale and
        # source slot (8 B); per output cluster its segment count / offsets (52 x 4 B), source list (100 B) and stop word
        # (256 B); per gathered row its index (4 B); w (48 B per row) and the subdomains' column scales (24 B per
        # subdomain row) once; m written (48 B per row)
        C_ = pci["clusters"]
        B_apply = (pci["segments"] * (2 * pci["row_length"] + 8) + C_ * (52 * 4 + 100 + 256) + pci["gathered_rows"] * 4 + rows * 48
                   + pci["subdomain_rows"] * 24 + rows * 48)
        B_pcg = nnzb * 296 + rows * (768 + 48 + 48) + B_apply
    one = bool(pci["schwarz"]) and pci.get("launches_per_iteration", 2) == 1
    if one:
        # one launch per iteration (k_as_iter, round 6): the operator's blocks once (288 B; the kernel re-reads each block
        # for up to 1 + kAsX subdomains from L2), each subdomain's fp16 inverse rows (288 B per segment) and their scales
        # (4 B), the own rows' state read + written (768 B per row), the ring rows' ghost (w, z) read + written (32 B per
        # component), the contributions written and read (16 B per segment)
        ring_rows = max(0, pci["subdomain_rows"] - rows)
        B_pcg = nnzb * 288 + pci["segments"] * (288 + 4 + 16) + rows * 768 + ring_rows * 6 * 32
    iters = float(np.sum(pcg))
    launches = max(1, pcg_launches)
    t_pcg = pcg_ms * 1e-3 / launches
    B_launch = B_pcg * iters / launches
    workload = (f"{D}^3 TSDF @{a.voxel * 1e3:g} mm, {seq.nodes.shape[0]} nodes, {a.matches} matches, "
                f"{seq.cam.width}x{seq.cam.height} depth, {cfg['motion']}{' + occluder' if cfg['occluder'] else ''}, "
                f"GN 10 it")
    pcg_traffic = pmc_traffic("k_as_iter" if one else "k_pcg_iter", workload)
    if pci["schwarz"] and not one:   # per launch: the mean of the pair (the chain alternates them)
        t_apply = pmc_traffic("k_as_apply", workload)
        pcg_traffic = None if pcg_traffic is None or t_apply is None else 0.5 * (pcg_traffic + t_apply)
    res = {
        "metric": f"fusion frames/sec (warp+integrate+solve), {640 // cfg['cam_scale']}x{480 // cfg['cam_scale']} depth "
                  f"-> {D}^3 TSDF",
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed_max / a.steps, "higher_is_better": True,
        "scaling": "weak" if a.mode == "replicas" else "strong", "vs_baseline": None, "dtype": "f32/f64",
        "data": f"synthetic (seeded sphere+plane {cfg['motion']} sequence"
                f"{' with a moving occluder hiding up to ~38 % of the object' if cfg['occluder'] else ''}, 1 mm noise, "
                f"matches from visible points; SURVEY §8(d), BASELINE config {a.config})",
        "config": {"workload": workload, "baseline_config": a.config, "mode": a.mode,
                   "solve": (a.solve if sharded else "local"), "dims": D, "voxel_size_m": a.voxel,
                   "nodes": int(seq.nodes.shape[0]), "matches": a.matches,
                   "parallelism": f"{a.mode}{world}" + (f"-{a.solve}" if sharded else ""),
                   "setup_prefetch": prefetch, "integrate_overlap": bool(a.overlap), "scene_seed": scene_seed},
        "breakdown_ms": {"solve": 1e3 * float(np.mean(t_solve)), "integrate": 1e3 * float(np.mean(t_int)),
                         "allreduce": 1e3 * t_ar, "pcg_iters_per_frame": float(np.mean(pcg)),
                         "gn_iters": float(np.mean(gn_it)), "valid_solves": int(np.sum(valid)),
                         "prefetched_setups_used": pf_used, "prefetched_setups_missed": pf_missed},
        "per_rank": per_rank,
        "roofline": {"kernel": ("k_as_iter (one launch per pipelined PCG iteration: the subdomain's block SpMV with ghost "
                                "ring rows, the recurrences and its overlapping Schwarz inverse)") if one else
                               ("k_pcg_iter + k_as_apply (one pipelined PCG iteration = two launches: wave-list block "
                                "SpMV + recurrences, then the overlapping Schwarz apply)") if pci["schwarz"] else
                               ("k_pcg_iter (pipelined PCG iteration: wave-list block SpMV + recurrences + cluster "
                                "block-Jacobi apply)"), "bound": "latency", "preconditioner": pci,
                     "achieved": B_launch / t_pcg / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": B_launch / t_pcg / PEAK_HBM,
                     "traffic": pcg_traffic, "traffic_source": os.path.relpath(PMC_FILE, ROOT),
                     "bytes_per_iteration": B_pcg, "bytes_per_launch": B_launch, "avg_launch_us": 1e6 * t_pcg,
                     "launches_per_frame": launches / a.steps, "iterations_per_frame": iters / a.steps,
                     "us_per_iteration": 1e6 * pcg_ms * 1e-3 / max(1.0, iters), "nnz_blocks": nnzb,
                     "note": "dominant kernel by time; latency-bound: one launch per iteration = the dispatch / "
                             "kernel-boundary floor + two dependent memory trips + the wave's instruction stream "
                             "(DESIGN.md §5); the 11-12 MB working set is L2/MALL-resident across launches. frac = "
                             "bytes_per_launch / avg_launch_us / peak"},
        "roofline_integrate": {"kernel": "k_tile_max + k_brick_cull + k_integrate_pal4 (per-frame brick cull, then the "
                                         "fused warp+integrate with an LDS node palette; VALU-bound: DESIGN.md "
                                         "section 5)", "bound": "hbm",
                               "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                               "frac": achieved / PEAK_HBM, "traffic": pmc_traffic("k_integrate_warp", workload, ("k_brick_cull", "k_tile_max")),
                               "bytes_per_launch": B,
                               "bytes_note": "this layout's minimal bytes for the bricks the per-frame cull keeps "
                                             "(palette ranks, reads for skin-valid voxels only) + the cull's own reads; "
                                             "frac_listed_bytes: the same per-unit bytes over every listed brick (the "
                                             "work the launch covers); SURVEY 8(d)'s per-unit figure below",
                               "cull_kept_bricks": n_live, "cull_kept_skin_valid_voxels": sv_live,
                               "listed_bytes_per_launch": B_listed, "frac_listed_bytes": B_listed / t_kint / PEAK_HBM,
                               "survey_bytes_per_launch": B_survey, "frac_survey_bytes": B_survey / t_kint / PEAK_HBM,
                               "avg_launch_us": 1e6 * t_kint, "timing": "20 launches of the last frame in isolation "
                               "(library hipEvents around each launch)", "in_loop_avg_launch_us": 1e6 * t_kint_loop,
                               "listed_bricks": cache.n_list,
                               "skin_valid_voxels": n_skin_valid, "updated_voxels": U},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:   # the CPU baseline is an N=1 datapoint
        res["cpu_baseline"] = cpu_baseline(pipe, frames[total - 1], total - 1, a)
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def moose_bench(a):
    """The reference's only real solver input (NonRigidICP/main.py:35-48: the moose demo pair's 427 valid Lepard
    landmarks on the 271-node depth-mesh graph, tests/golden/moose.npz): K timed DeformNet.optimize solves after W
    warmup ones, at the default parameters and with the round-4 preconditioner policy (precond_rot_tol = 0: the cluster
    inverse built once per solve) beside it. Reports ms per optimize (events around the K calls), PCG iterations per
    optimize, capped steps, and the transforms' max error against the dense f64 oracle's (the fixture)."""
    from occlusionfusion_amd import GaussNewtonSolver
    g = np.load(os.path.join(ROOT, "tests", "golden", "moose.npz"), allow_pickle=False)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = g["nodes"].shape[0]
    K = g["K"]
    intr = (float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]))
    args = [torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("nodes", "edges", "edge_weights", "nodes")]
    rest = [torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("src", "anchors", "weights", "tgt")]
    conf = torch.zeros(N, device=dev)

    def run(**prm):
        s = GaussNewtonSolver(N, 1000, dev, **prm)
        call = lambda: s.optimize(*args, conf, *rest, intr, sync=False)
        for _ in range(a.warmup):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        outs = [call() for _ in range(a.steps)]
        e1.record()
        torch.cuda.synchronize()
        st = np.stack([o["_status"].cpu().numpy() for o in outs])
        o = outs[-1]
        err = max(float(np.abs(o["node_rotations"].cpu().numpy() - g["R"]).max()),
                  float(np.abs(o["node_translations"].cpu().numpy() - g["t"]).max()))
        return {"ms_per_optimize": e0.elapsed_time(e1) / a.steps, "pcg_iterations": float(st[:, 2].mean()),
                "gn_steps": float(st[:, 1].mean()), "capped_steps": int(st[:, 4].max()), "valid": int(st[:, 0].min()),
                "max_abs_err_vs_f64_oracle": err, "pcg_per_gn_step": [int(v) for v in s.stats()[:, 0]]}

    cur = run()
    old = run(precond_rot_tol=0.0)
    res = {"metric": "moose landmark GN optimize (NonRigidICP demo pair, 271 nodes, 427 landmarks, 10 GN steps)",
           "value": cur["ms_per_optimize"], "unit": "ms/optimize", "higher_is_better": False, "n_gpus": 1,
           "steps": a.steps, "warmup": a.warmup, "dtype": "f64", "data": "real (tests/golden/moose.npz: the reference's "
           "NonRigidICP/demo/moose6OK9_AttackTrotRM pair)", "default": cur, "precond_rot_tol_0": old}
    line = json.dumps(res)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


def cpu_model():
    """`lscpu` model name of the host (from /proc/cpuinfo: the same field lscpu prints)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def dense_gn_terms(rows, N6, threads):
    """The dense GN step's two dominant costs (model.py:641-709: JᵀJ of the rows x N6 Jacobian, LU of N6²),
    measured at the current BLAS thread count on bounded sub-problems and scaled by their flop counts: JᵀJ of a
    (rs x m) slab (m = min(N6, 4096), rs <= rows) -> GFLOP/s -> 2·rows·N6² flops; LU of min(N6, 6000)² scaled by the
    cube. Returns (t_JtJ, t_LU, GEMM GFLOP/s)."""
    from scipy.linalg import lu_factor
    m = min(N6, 4096)
    rs = int(min(rows, max(m, (12e9 * max(1, threads) / 25.0) // (2.0 * m * m))))   # ~0.5 s per thread-equivalent
    J = np.random.default_rng(1).random((rs, m))
    J.T @ J[:, :64]
    t0 = time.perf_counter()
    J.T @ J
    rate = 2.0 * rs * m * m / (time.perf_counter() - t0)
    t_mm = 2.0 * rows * N6 * N6 / rate
    n = min(N6, 6000)
    A = np.random.default_rng(2).random((n, n)) + n * np.eye(n)
    del J
    t0 = time.perf_counter()
    lu_factor(A)
    t_lu = (time.perf_counter() - t0) * (N6 / n) ** 3
    return t_mm, t_lu, rate / 1e9


def cpu_config1_full(dev, threads):
    """configs 1-2 run fully on the CPU. BASELINE config 1 (128³ @8 mm, ~200 nodes, 320x224, 10k
    matches) with the oracle port, unsampled: the source frame fused (untimed) and the volume's skin cached (as
    WarpField.skin_tsdf caches it, untimed); then warped frame 1, the whole frame timed: the
    matches' skin (oracle k-NN), the 10-step dense float64 GN solve (oracle gn_optimize: dense J, JᵀJ, LU) and the
    warp + integrate of all 2.1M voxels (oracle/cpu_ref.c, OpenMP)."""
    from occlusionfusion_amd import synthetic as S
    from oracle import cpu_ref
    from oracle import fusion_oracle as fo
    c = S.BASELINE_CONFIGS[1]
    seq = S.config_sequence(1, device=dev)     # the graph: SURVEY §8(d) depth-mesh graph (pinned to the csrc)
    D = c["dims"]
    dims = (D, D, D)
    origin = np.asarray(c["origin"], np.float32)
    vs = np.float32(c["voxel"])
    world = fo.world_points(origin, np.array(dims), float(vs))
    V = world.shape[0]
    intr = seq.cam.as_vec()
    nodes = seq.nodes
    cpu_ref.set_threads(threads)
    an_v, w_v, ok_v = fo.skin(world, nodes, seq.node_coverage)
    im0 = seq.frame(0)
    tsdf, weight, color = np.ones(V, np.float32), np.zeros(V, np.float32), np.zeros(V, np.float32)
    vox = np.arange(V, dtype=np.int64)
    cpu_ref.integrate(dims, origin, vs, vox, fo.depth_of(im0), fo.pack_color(im0), intr, tsdf, weight, color)
    R = T = None
    per = []
    for t in (1,):
        im = seq.frame(t)
        t0 = time.perf_counter()
        src, tgt, tpos, conf = seq.solver_inputs(t, 10000)
        a_, w_, v_ = fo.skin(src, nodes, seq.node_coverage)
        t1 = time.perf_counter()
        res = fo.gn_optimize(nodes, seq.edges, seq.edge_weights, tpos, conf, src[v_], a_[v_], w_[v_], tgt[v_], intr,
                             prev_rot=R, prev_trans=T)
        R, T = res["node_rotations"], res["node_translations"]
        t2 = time.perf_counter()
        cpu_ref.integrate(dims, origin, vs, vox, fo.depth_of(im), fo.pack_color(im), intr, tsdf, weight, color,
                          warp=True, anchors=an_v, weights=w_v, valid=ok_v.astype(np.uint8), R=R.reshape(-1, 9),
                          T=T, nodes=nodes)
        t3 = time.perf_counter()
        per.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2, len(res["convergence_info"]["total"])))
    sec = float(np.mean([x[0] for x in per]))
    return {"value": 1.0 / sec, "unit": "frames/s", "cores": threads, "kind": "port", "s_per_frame": sec,
            "s_skin_matches": float(np.mean([x[1] for x in per])), "s_gn": float(np.mean([x[2] for x in per])),
            "s_warp_integrate": float(np.mean([x[3] for x in per])), "gn_steps": [x[4] for x in per],
            "sample": f"BASELINE config 1 unsampled: {D}^3 voxels ({V}), {nodes.shape[0]} nodes, 10k matches, warped "
                      f"frame 1 timed whole (match skin + 10-step dense f64 GN + warp/integrate of every voxel)"}


def cpu_baseline(pipe, fi, t, a):
    """The oracle port on the host cores, on a bounded sample of the same frame (kind "port": the reference
    Python cannot run here or travel; oracle/ restates it line for line):
    * warp+integrate: oracle/cpu_ref.c (C/OpenMP restatement of tsdf.py:378-494 + geometry.py:9-25) on a
      uniform random sample of the volume's voxels (skin precomputed, as the reference caches it), scaled
      to the whole volume;
    * solve: ONE Gauss-Newton step of the dense float64 restatement of DeformNet.optimize
      (oracle.fusion_oracle.gn_optimize, num_iter=1: dense J, JᵀJ, LU as model.py:222-859) on this frame's
      inputs and state, scaled x10 (the reference runs 10 GN iterations; the bench sequence never stops early).
    CPU frames/s = 1 / (t_warp+integrate + 10 x t_gn_step), with all host threads (OMP_NUM_THREADS, BLAS
    threads) and, as `single_thread`, with one: the integrate sample at one OpenMP thread and the GN step's
    dominant dense JᵀJ product on 1/64 of J's columns at one BLAS thread (x64), plus the one-thread LU."""
    from oracle import cpu_ref
    from oracle import fusion_oracle as fo
    vol = pipe.vol
    Dx, Dy, Dz = (int(d) for d in vol._vol_dim)
    V = Dx * Dy * Dz
    n = min(a.cpu_sample, V)
    rng = np.random.default_rng(0)
    vox = np.sort(rng.choice(V, n, replace=False))
    i, r = vox // (Dy * Dz), vox % (Dy * Dz)
    j, k = r // Dz, r % Dz
    o = vol._vol_origin.astype(np.float64)
    vs = np.float64(vol._voxel_size)
    pts = np.stack([(o[0] + vs * i.astype(np.float32).astype(np.float64)),
                    (o[1] + vs * j.astype(np.float32).astype(np.float64)),
                    (o[2] + vs * k.astype(np.float32).astype(np.float64))], 1).astype(np.float32)
    an, w, v = pipe.wf.skin_device(pts)
    an, w, v = an.cpu().numpy(), w.cpu().numpy(), v.cpu().numpy().astype(np.uint8)
    tsdf0, color0, weight0 = (x.reshape(-1).copy() for x in vol.get_volume())
    R = pipe.prev_rot.cpu().numpy().reshape(-1, 9)
    T = pipe.prev_trans.cpu().numpy()
    im = fi.im.cpu().numpy()
    depth, cim = fo.depth_of(im), fo.pack_color(im)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))

    def integrate_sample(nv):
        tsdf, weight, color = tsdf0.copy(), weight0.copy(), color0.copy()
        t0 = time.perf_counter()
        cpu_ref.integrate((Dx, Dy, Dz), vol._vol_origin, vol._voxel_size, vox[:nv], depth, cim, pipe.intr, tsdf,
                          weight, color, warp=True, anchors=an[:nv], weights=w[:nv], valid=v[:nv], R=R, T=T,
                          nodes=pipe.graph.nodes)
        return time.perf_counter() - t0

    cpu_ref.set_threads(threads)
    dt_int = integrate_sample(n)
    per_frame_int = dt_int * V / n
    g = pipe
    gn_args = (g.graph.nodes, g.seq.edges, g.seq.edge_weights, fi.tpos.cpu().numpy(), fi.conf.cpu().numpy(),
               fi.src.cpu().numpy(), fi.anchors.cpu().numpy(), fi.weights.cpu().numpy(), fi.tgt.cpu().numpy(),
               pipe.intr)
    N6 = 6 * g.graph.nodes.shape[0]
    rows = 3 * int(fi.src.shape[0]) + 3 * int((np.asarray(g.seq.edges) >= 0).sum()) + 3 * g.graph.nodes.shape[0]
    if N6 <= 12600:     # up to ~2.1k nodes: one real dense GN step of the oracle (≈ 11 s at 2k nodes, 16 threads)
        t0 = time.perf_counter()
        fo.gn_optimize(*gn_args, prev_rot=R.reshape(-1, 3, 3), prev_trans=T, num_iter=1)
        dt_gn = time.perf_counter() - t0
        gn_how = "one dense float64 GN step (oracle gn_optimize, numpy/LAPACK)"
    else:               # larger graphs: the step's dominant terms, each on a bounded slice, scaled
        dt_mm, dt_lu, gf = dense_gn_terms(rows, N6, threads)
        dt_gn = dt_mm + dt_lu
        gn_how = (f"dense GN step estimated from its dominant terms at {threads} BLAS threads: JᵀJ ({rows}x{N6}) "
                  f"at the measured {gf:.0f} GFLOP/s of a 4096-column slab + LU scaled from a 6000² factorisation")
    per_frame = per_frame_int + 10 * dt_gn
    out = {"value": 1.0 / per_frame, "unit": "frames/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
           "sample": f"warp+integrate (oracle/cpu_ref.c, OpenMP) of {n} uniformly sampled voxels of the {Dx}^3 frame "
                     f"(x{V / n:.0f} scaled, skin precomputed, {dt_int:.3f} s) + {gn_how} ({dt_gn:.2f} s) x 10 GN "
                     f"iterations",
           "ms_per_frame_warp_integrate": 1e3 * per_frame_int, "s_per_gn_step": dt_gn}
    # one thread: a 1/16 integrate sample, and the dense GN step's cost terms at one BLAS thread
    try:
        from threadpoolctl import threadpool_limits
        cpu_ref.set_threads(1)
        n1 = max(1, n // 16)
        dt_int1 = integrate_sample(n1)
        cpu_ref.set_threads(threads)
        with threadpool_limits(limits=1):
            dt_mm, dt_lu, gf1 = dense_gn_terms(rows, N6, 1)
        gn1 = dt_mm + dt_lu
        pf1 = dt_int1 * V / n1 + 10 * gn1
        out["single_thread"] = {"value": 1.0 / pf1, "unit": "frames/s", "cores": 1,
                                "ms_per_frame_warp_integrate": 1e3 * dt_int1 * V / n1, "s_per_gn_step": gn1,
                                "sample": f"integrate of {n1} sampled voxels at 1 OpenMP thread ({dt_int1:.3f} s, "
                                          f"x{V / n1:.0f}); GN step = dense JᵀJ ({rows}x{N6}) at the measured "
                                          f"{gf1:.0f} GFLOP/s of a 4096-column slab at 1 BLAS thread ({dt_mm:.1f} s) + "
                                          f"LU of {N6}² ({dt_lu:.1f} s, scaled from at most 6000²)"}
    except Exception as e:  # the reported baseline must not break the bench line
        out["single_thread"] = {"error": repr(e)}
    try:
        out["config1_full"] = cpu_config1_full(pipe.device, threads)
    except Exception as e:
        out["config1_full"] = {"error": repr(e)}
    return out


if __name__ == "__main__":
    main()
