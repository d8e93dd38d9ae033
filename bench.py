"""Fusion frames/sec (warp + integrate + solve), 640x480 (->640x448) synthetic depth -> 512³ TSDF @4 mm,
~2k-node ED graph, 10k matches, on MI355X.

One step = one frame of the reference's fusion loop (lepard_nicp_test.py:test4): GN solve
(DeformNet.optimize formulation, 10 iterations) -> update node transforms -> fused skin-cache warp +
TSDF/weight/colour integrate of the new frame. All inputs are device-resident before timing.

  python bench.py [--gpus N --steps K --warmup W] [--mode replicas|shard] [--dims 512] [--nodes 2000]

--mode replicas (default, BASELINE config 5): one independent 512³ scene per GPU, no collective,
    value = frames of all ranks / max-rank time (weak scaling).
--mode shard (BASELINE config 4 style): ONE volume x-sharded across ranks (bricks), matches sharded,
    one RCCL all-reduce of the GN JᵀJ/Jᵀr accumulators per GN iteration; value = frames / time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM = 8.0e12   # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")   # tools/pmc_traffic.sh + tools/pmc_summary.py


def pmc_traffic(kernel):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC summary (separate counter passes
    cannot run inside the timed bench), or None."""
    try:
        with open(PMC_FILE) as f:
            return json.load(f)["kernels"][kernel]["traffic_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=["replicas", "shard"], default="replicas")
    p.add_argument("--dims", type=int, default=512)
    p.add_argument("--voxel", type=float, default=0.004)
    p.add_argument("--nodes", type=int, default=2000)
    p.add_argument("--matches", type=int, default=10000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=1 << 24)
    p.add_argument("--json-out", default=None)
    p.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsals "
                                                     "with several ranks on one device)")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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

    D = a.dims
    origin = (-D * a.voxel / 2, -D * a.voxel / 2, 0.5)
    seq = S.SyntheticSequence.build(a.nodes, seed=3)
    shard = (rank, world) if (a.mode == "shard" and world > 1) else None
    pipe = FusionPipeline(seq, origin, a.voxel, (D, D, D), n_matches=a.matches, device=dev, shard=shard)
    total = a.warmup + a.steps + 1
    frames = [pipe.prepare(t) for t in range(total)]
    torch.cuda.synchronize()
    pipe.integrate_source(frames[0])
    cache = pipe.wf.skin_tsdf_cache()
    K = cache.k
    n_skin_valid = int((cache.anchors.view(-1, 4)[:, K - 1] != -1).sum().item()) if cache.n_list else 0
    torch.cuda.synchronize()

    def solve(fi):
        if a.mode == "shard" and world > 1:
            g = pipe
            out = pipe.solver.optimize_distributed(g.nodes_t, g.edges_t, g.ew_t, fi.tpos, fi.conf, fi.src, fi.anchors,
                                                   fi.weights, fi.tgt, pipe.intr, prev_rot=pipe.prev_rot,
                                                   prev_trans=pipe.prev_trans, sync=False)
            pipe.prev_rot, pipe.prev_trans = out["node_rotations"], out["node_translations"]
            return out
        return pipe.solve(fi)

    ev = lambda: torch.cuda.Event(enable_timing=True)
    for t in range(1, 1 + a.warmup):
        solve(frames[t])
        pipe.integrate(frames[t], t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    marks = []
    upd = []
    pipe.solver.timing(True)               # arm hipEvent timing of the PCG loops (same stream)
    pipe.vol.kernel_timer = []             # hipEvents around each warped integrate launch
    t0 = time.perf_counter()
    for t in range(1 + a.warmup, total):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        out = solve(frames[t])
        e1.record()
        pipe.integrate(frames[t], t, count_updates=True)
        e2.record()
        upd.append(pipe.vol.n_updated[:cache.n_list].sum())   # device-side sum, read after timing
        marks.append((e0, e1, e2, out))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    pcg_ms, pcg_launches, _ = pipe.solver.timing(False)
    N_, M_, nnzb, _T, rows = pipe.solver.info()
    t_solve = np.array([m[0].elapsed_time(m[1]) for m in marks]) * 1e-3
    t_int = np.array([m[1].elapsed_time(m[2]) for m in marks]) * 1e-3
    pcg = [int(m[3]["_status"][2].item()) for m in marks]
    gn_it = [int(m[3]["_status"][1].item()) for m in marks]
    valid = [int(m[3]["_status"][0].item()) for m in marks]
    U = float(np.mean([int(u.item()) for u in upd]))
    t_kint = float(np.mean([a.elapsed_time(b) for a, b in pipe.vol.kernel_timer])) * 1e-3
    pipe.vol.kernel_timer = None

    frames_done = a.steps * (world if a.mode == "replicas" else 1)
    value = frames_done / elapsed
    # algorithmic bytes of one integrate launch: palette-rank anchors 4 B per voxel
    # of every listed brick + the brick's palette (64 x u16 + count); weights 16 B + tsdf/weight 8 B read
    # per skin-valid voxel; per updated voxel tsdf/weight write 8 B + colour read+write 8 B. Node records
    # and the depth/colour images are L2-resident and not counted.
    B = cache.n_list * (512 * 4 + 132) + n_skin_valid * 24 + U * 16
    t_int_avg = float(np.mean(t_int))
    achieved = B / t_kint
    # k_pcg_iter algorithmic (unique) bytes per launch: per JᵀJ block its 6x6 f64 values (288 B) + its
    # (col, slot) wave-list entry (8 B); per PCG row (nodes in cluster order, padded) the cluster-inverse
    # rows (6 x 48 f32 = 1152 B), the 8-vector state read + written (2 x 384 B), m read (48 B; the
    # neighbour gathers re-read these) and the new m written (48 B). DESIGN.md §5.
    B_pcg = nnzb * 296 + rows * (1152 + 768 + 48 + 48)
    t_pcg = pcg_ms * 1e-3 / max(1, pcg_launches)
    ach_pcg = B_pcg / t_pcg
    res = {
        "metric": "fusion frames/sec (warp+integrate+solve), 640x480 depth -> 512^3 TSDF",
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps, "higher_is_better": True,
        "scaling": "weak" if a.mode == "replicas" else "strong", "vs_baseline": None, "dtype": "f32/f64",
        "data": "synthetic (seeded sphere+plane non-rigid sequence with a moving occluder hiding up to ~38 % of the object, 1 mm noise, matches from visible points; SURVEY §8(d), BASELINE config 3)",
        "config": {"workload": f"{D}^3 TSDF @{a.voxel * 1e3:g} mm, {seq.nodes.shape[0]} nodes, "
                               f"{a.matches} matches, 640x448 depth, GN 10 it",
                   "mode": a.mode, "dims": D, "voxel_size_m": a.voxel, "nodes": int(seq.nodes.shape[0]),
                   "matches": a.matches, "parallelism": f"{a.mode}{world}"},
        "breakdown_ms": {"solve": 1e3 * float(np.mean(t_solve)), "integrate": 1e3 * t_int_avg,
                         "pcg_iters_per_frame": float(np.mean(pcg)), "gn_iters": float(np.mean(gn_it)),
                         "valid_solves": int(np.sum(valid))},
        "roofline": {"kernel": "k_pcg_iter (pipelined PCG iteration: wave-list block SpMV + recurrences + cluster block-Jacobi apply)", "bound": "hbm",
                     "achieved": ach_pcg / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": ach_pcg / PEAK_HBM,
                     "traffic": pmc_traffic("k_pcg_iter"), "traffic_source": os.path.relpath(PMC_FILE, ROOT),
                     "bytes_per_launch": B_pcg, "avg_launch_us": 1e6 * t_pcg,
                     "launches_per_frame": pcg_launches / a.steps, "nnz_blocks": nnzb,
                     "note": "dominant kernel by time; latency-bound (one launch per iteration: launch floor + two dependent memory trips + the wave's instruction stream)"},
        "roofline_integrate": {"kernel": "k_integrate<true,true> (fused warp+integrate, LDS node palette)", "bound": "hbm",
                               "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                               "frac": achieved / PEAK_HBM, "traffic": pmc_traffic("k_integrate_warp"),
                               "bytes_per_launch": B,
                               "avg_launch_us": 1e6 * t_kint, "listed_bricks": cache.n_list,
                               "skin_valid_voxels": n_skin_valid, "updated_voxels": U},
    }
    if rank == 0 and not a.no_cpu_baseline:
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


def cpu_baseline(pipe, fi, t, a):
    """The oracle port on the host cores, on a bounded sample of the same frame:
    * warp+integrate: oracle/cpu_ref.c (C/OpenMP restatement of tsdf.py:378-494 + geometry.py:9-25) on a
      uniform random sample of the volume's voxels (skin precomputed, as the reference caches it), scaled
      to the whole volume;
    * solve: ONE Gauss-Newton step of the dense float64 restatement of DeformNet.optimize
      (oracle.fusion_oracle.gn_optimize, num_iter=1: dense J, JᵀJ, LU as model.py:222-859) on this frame's
      inputs and state, scaled x10 (the reference runs 10 GN iterations; the bench sequence never stops early).
    CPU frames/s = 1 / (t_warp+integrate + 10 x t_gn_step)."""
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
    tsdf, color, weight = (x.reshape(-1).copy() for x in vol.get_volume())
    R = pipe.prev_rot.cpu().numpy().reshape(-1, 9)
    T = pipe.prev_trans.cpu().numpy()
    im = fi.im.cpu().numpy()
    depth, cim = fo.depth_of(im), fo.pack_color(im)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    cpu_ref.integrate((Dx, Dy, Dz), vol._vol_origin, vol._voxel_size, vox, depth, cim, pipe.intr, tsdf, weight, color,
                      warp=True, anchors=an, weights=w, valid=v, R=R, T=T, nodes=pipe.graph.nodes)
    dt_int = time.perf_counter() - t0
    per_frame_int = dt_int * V / n
    g = pipe
    t0 = time.perf_counter()
    fo.gn_optimize(g.graph.nodes, g.seq.edges, g.seq.edge_weights, fi.tpos.cpu().numpy(), fi.conf.cpu().numpy(),
                   fi.src.cpu().numpy(), fi.anchors.cpu().numpy(), fi.weights.cpu().numpy(), fi.tgt.cpu().numpy(),
                   pipe.intr, prev_rot=R.reshape(-1, 3, 3), prev_trans=T, num_iter=1)
    dt_gn = time.perf_counter() - t0
    per_frame = per_frame_int + 10 * dt_gn
    return {"value": 1.0 / per_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"warp+integrate (oracle/cpu_ref.c, OpenMP) of {n} uniformly sampled voxels of the {Dx}^3 frame "
                      f"(x{V / n:.0f} scaled, skin precomputed, {dt_int:.3f} s) + one dense float64 GN step "
                      f"(oracle gn_optimize, numpy/LAPACK, {dt_gn:.2f} s) x 10 GN iterations",
            "ms_per_frame_warp_integrate": 1e3 * per_frame_int, "s_per_gn_step": dt_gn}


if __name__ == "__main__":
    main()
