#!/usr/bin/env python3
"""Benchmark of the MI355X SIFT hot path (BASELINE.json metric: SIFT images/s + features/s at
1080p on 1/2/4/8 MI355X).

A step = one pass of the hot path (Gaussian pyramid -> DoG extrema -> orientation ->
descriptors, HIP kernels behind the C ABI of include/sgpu.h) over one batch of synthetic
1920x1080 u8 images per GPU, already resident in HBM (staged once before timing).  Workload:
the per-GPU shard of BASELINE config C3 (128 images per GPU) with the parameters of config C2
(-fo 0 -no 4 -d 3).  Multi-GPU: one process per GPU, images sharded (weak scaling), RCCL (inside
libsiftgpu, over xGMI) only for the per-image feature-count all-gather; torch.distributed
(gloo, host) is the rendezvous.  Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import sgpu  # noqa: E402  (loads libsiftgpu.so before torch: one HIP runtime, /opt/rocm's)
from sgpu_types import default_options  # noqa: E402
from sift_synth import synth_batch, synth_descriptors, synth_guided_scene, quantize  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters (spec)
I8_MFMA_PEAK_TOPS = 5000.0     # dense i8 MFMA = 2x the ~2.5 PF bf16 rate (same guide)


def geometry_sum(w, h, octaves):
    tot, ww, hh = 0, w & ~3, h
    for _ in range(octaves):
        tot += ((ww + 3) // 4 * 4) * hh
        ww >>= 1
        hh >>= 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--unique", type=int, default=16, help="distinct synthetic images per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-match", action="store_true")
    ap.add_argument("--match-n", type=int, default=50000)
    ap.add_argument("--dist-backend", default="rccl", choices=["rccl", "gloo"],
                    help="rccl: the count all-gather runs on RCCL over xGMI inside libsiftgpu "
                         "(the real run); gloo: host all-gather (rehearsal: ranks may then "
                         "share one GPU)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: WORLD_SIZE={world} differs from --gpus {args.gpus}", file=sys.stderr)
    sgpu.lib()   # libsiftgpu (and /opt/rocm's HIP runtime) before torch: torch never touches
                 # the GPU here -- torch.distributed (gloo, host) is only the rendezvous
    # Initialise /opt/rocm's HIP runtime now, before `import torch` maps torch's own copy of
    # libamdhip64: a context created after the torch import and the gloo rendezvous otherwise
    # finds no device (observed on the box with two ranks).
    n_dev = sgpu.device_count()
    dist = None
    device = local
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        # gloo announces its peers on stdout; keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        if args.dist_backend == "gloo":
            device = local % max(1, n_dev)

    B, W, H = args.batch, args.width, args.height
    opts = default_options(octave_num=args.octaves)
    ctx = sgpu.SiftContext(device, opts)
    rccl = world > 1 and args.dist_backend == "rccl"
    if rccl:
        # RCCL communicator of the per-rank contexts; the id travels over the host rendezvous
        uid = [sgpu.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    # shard of the global batch: images [rank*B, (rank+1)*B), seeds 3000 + global index
    imgs = synth_batch(B, W, H, seed0=3000 + rank * B, unique=args.unique)
    ctx.stage(imgs)

    def step():
        ctx.extract_staged()   # returns after the GPU work of the step has completed
        counts = np.fromiter((ctx.count(i) for i in range(B)), np.int32, B)
        if rccl:
            ctx.allgather_i32(counts, world)   # RCCL over xGMI: global per-image feature counts
        elif dist is not None:
            import torch
            out = [torch.zeros(B, dtype=torch.int32) for _ in range(world)]
            dist.all_gather(out, torch.from_numpy(counts))
        return counts

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    pyr_ms = 0.0
    stage_acc = {}
    feats = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        c = step()
        feats += int(c.sum())
        t = ctx.timing()
        pyr_ms += t["pyramid"]
        for k, v in t.items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local_feats = feats
    if rccl:
        elapsed = float(ctx.allreduce_f64(elapsed, op_max=True)[0])
        feats = int(ctx.allreduce_f64(float(feats), op_max=False)[0])
    elif dist is not None:
        import torch
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        f = torch.tensor([feats], dtype=torch.int64)
        dist.all_reduce(f)
        feats = int(f.item())

    n_gauss = 1 + args.octaves * 5                      # level 0 of octave 0 + 5 levels/octave
    total_images = B * world * args.steps
    sumN = geometry_sum(W, H, args.octaves)
    pyr_bytes = 48.0 * sumN * B * args.steps          # 48 B per pyramid px
    achieved = pyr_bytes / (pyr_ms * 1e-3) / 1e9 if pyr_ms > 0 else 0.0

    traffic, prof_note = profiled_traffic(B, W, H, args.octaves)
    result = {
        "metric": "SIFT images/sec at 1080p (features/sec alongside), 1/2/4/8 MI355X",
        "value": total_images / elapsed,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"C3 per-GPU shard: {B} x {W}x{H} u8 gray per GPU per step, "
                        f"C2 parameters -fo 0 -no {args.octaves} -d 3 (BASELINE.json configs[1-2])",
            "images_per_gpu": B, "width": W, "height": H, "octaves": args.octaves,
            "parallelism": f"dp{world}",
        },
        "features_per_sec": feats / elapsed,
        "features_per_image": local_feats / (B * args.steps),
        "stage_ms_per_step": {k: v / args.steps for k, v in stage_acc.items() if k != "match"},
        "roofline": {
            "kernel": f"k_gauss_pk2 (separable Gaussian level; all {n_gauss} launches of a step, "
                      "HIP events around them on the library's stream)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE + WRITE_SIZE)",
            "traffic_source": prof_note,
            "algorithmic_bytes_per_launch": 48.0 * sumN * B / n_gauss,
            "avg_launch_ms": pyr_ms / args.steps / n_gauss,
        },
    }

    if rank == 0 and world == 1 and not args.no_match:
        result["match"] = bench_match(ctx, args.match_n)
    if world > 1 and not args.no_match:
        sm = bench_match_sharded(ctx, args.match_n, rank, world, None if rccl else dist)
        if rank == 0:
            result["match_sharded"] = sm
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(imgs, opts)
    if rank == 0:
        print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


def profiled_traffic(B, W, H, octaves):
    """HBM bytes per Gaussian launch from the committed rocprofv3 summary of this workload
    (tests/profile_kernels.sh + tests/pmc_summary.py), or None when no summary matches."""
    import glob
    if (B, W, H, octaves) != (128, 1920, 1080, 4):
        return None, "no profile for this workload"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")))
    for path in reversed(files):
        try:
            s = json.load(open(path))
            fams = [f for f in s["launches_per_extract"] if f.startswith("k_gauss")]
            n = sum(s["launches_per_extract"][f] for f in fams)
            b = sum(s["fetch_bytes_per_extract"][f] + s["write_bytes_per_extract"][f] for f in fams)
            return b / n, os.path.relpath(path, ROOT)
        except (KeyError, ValueError, OSError):
            continue
    return None, "no profile summary committed"


def bench_match(ctx, n):
    """Config C5: n x n SiftMatch (u8 dot products on i8 MFMA + fused top-2), mutual best."""
    d1 = synth_descriptors(n, 5000)
    d2 = synth_descriptors(n, 5001, base=d1, n_dup=min(20000, n // 2))
    q1, q2 = quantize(d1), quantize(d2)
    ctx.match(q1, q2)   # warm-up (uploads, distance table)
    reps, ms, m = 5, 0.0, None
    for _ in range(reps):
        m = ctx.match(q1, q2)
        ms += ctx.timing()["match"]
    ms /= reps
    ops = 2.0 * 128 * n * n * 2      # both directions (rows and columns) are computed
    # guided matching (GetGuidedSiftMatch) on a synthetic two-view scene of the same size
    g1, g2, l1, l2, H, F = synth_guided_scene(n, n, 5002)
    ctx.match_guided(g1, g2, l1, l2, H, F)
    gms, gm = 0.0, None
    for _ in range(reps):
        gm = ctx.match_guided(g1, g2, l1, l2, H, F)
        gms += ctx.timing()["match"]
    gms /= reps
    return {"workload": f"C5 {n}x{n} u8 descriptors, mutual best match",
            "ms": ms, "matches": int(len(m)),
            "tops": ops / (ms * 1e-3) / 1e12,
            "mfma_util": ops / (ms * 1e-3) / 1e12 / I8_MFMA_PEAK_TOPS,
            "guided_ms": gms, "guided_matches": int(len(gm))}


def bench_match_sharded(ctx, n, rank, world, host_dist=None):
    """Config C5 with set 1 sharded over the ranks: each rank matches its rows
    against all of set 2, the per-column states travel by one RCCL all-gather, and the rank
    keeps its rows' mutual pairs (sgpu_match_sharded).  Reported: the slowest rank's device
    time and wall time per call, and the total pair count (equal to the 1-GPU count).
    host_dist (gloo rehearsal, ranks sharing a GPU): the same exchange over torch.distributed."""
    from sift_dist import match_sharded_host, shard
    try:
        d1 = synth_descriptors(n, 5000)
        d2 = synth_descriptors(n, 5001, base=d1, n_dup=min(20000, n // 2))
        q1, q2 = quantize(d1), quantize(d2)
        s, e = shard(n, rank, world)
        def one():
            if host_dist is None:
                return ctx.match_sharded(q1[s:e], s, q2)
            rows, cols = ctx.match_shard_begin(q1[s:e], s, q2)
            return match_sharded_host(rows, cols, s, host_dist)

        one()   # warm-up
        reps, dev, wall, m = 5, 0.0, 0.0, None
        for _ in range(reps):
            t0 = time.perf_counter()
            m = one()
            wall += time.perf_counter() - t0
            dev += ctx.timing()["match"]
        v = [dev / reps, wall / reps * 1e3, float(len(m))]
        if host_dist is None:
            v[:2] = ctx.allreduce_f64(v[:2], op_max=True).tolist()
            v[2] = float(ctx.allreduce_f64(v[2], op_max=False)[0])
        else:
            import torch
            t = torch.tensor(v[:2], dtype=torch.float64)
            host_dist.all_reduce(t, op=host_dist.ReduceOp.MAX)
            c = torch.tensor([v[2]], dtype=torch.float64)
            host_dist.all_reduce(c)
            v = t.tolist() + c.tolist()
        return {"workload": f"C5 {n}x{n}, set 1 sharded over {world} ranks, "
                            f"{'RCCL' if host_dist is None else 'gloo'} all-gather of the column "
                            f"states", "device_ms": v[0], "wall_ms": v[1], "matches": int(v[2])}
    except Exception as ex:   # never costs the main measurement
        return {"error": str(ex)}


def cpu_baseline(imgs, opts):
    """The CPU oracle (oracle/, a C++ restatement of the reference) on a bounded sample of the
    same workload: one staged image per OpenMP thread (about 1 s of wall time, 15-20 s of CPU
    work on 16 threads)."""
    import oracle_py
    threads = max(1, min(16, os.cpu_count() or 1, len(imgs)))
    n = threads
    secs, feats = oracle_py.bench_extract(imgs[:n], opts, threads=threads)
    return {"value": n / secs, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} of the staged 1920x1080 images (-fo 0 -no 4 -d 3), one per OpenMP "
                      f"thread, oracle/liboracle.so (g++ -O3, strict IEEE)",
            "features_per_image": feats / n}


if __name__ == "__main__":
    main()
