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
from sift_synth import synth_batch_fast, synth_descriptors, synth_guided_scene, quantize  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters (spec)
I8_MFMA_PEAK_TOPS = 5000.0     # dense i8 MFMA = 2x the ~2.5 PF bf16 rate (same guide)


def geometry_sum(w, h, octaves):
    tot, ww, hh = 0, w & ~3, h
    for _ in range(octaves):
        tot += ((ww + 3) // 4 * 4) * hh
        ww >>= 1
        hh >>= 1
    return tot


def self_launch(n):
    """`--gpus N` without a launcher: start N ranks of this script as child processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would) and return
    the worst exit code.  Runs before anything touches the GPU in this process."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--workload", default="c3", choices=["c3", "c4"],
                    help="c3: 128 x 1920x1080 per GPU (-no 4), the headline; c4: BASELINE "
                         "configs[3], 4096x4096 tiles with 6 octaves, as the headline line")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 sub-measurement")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-in / host-out (PCIe-inclusive) sub-measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c2", action="store_true",
                    help="skip the single-image drop-in API measurement (speed.cpp protocol)")
    ap.add_argument("--no-match", action="store_true")
    ap.add_argument("--match-n", type=int, default=50000)
    ap.add_argument("--verify", action="store_true",
                    help="after the timed steps: every rank all-gathers (feature count, 64-bit "
                         "digest of keys + descriptors) per image, rank 0 recomputes a sample of "
                         "the other ranks' images on its own GPU and compares (SURVEY.md 4 (vi))")
    ap.add_argument("--dist-backend", default="rccl", choices=["rccl", "gloo"],
                    help="rccl: the count all-gather runs on RCCL over xGMI inside libsiftgpu "
                         "(the real run); gloo: host all-gather (rehearsal: ranks may then "
                         "share one GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.workload == "c4":
        args.width = args.height = 4096
        args.octaves = 6
        if args.batch == 128:
            args.batch = 16
    c2 = None
    if rank == 0 and world == 1 and args.workload == "c3" and not args.no_c2:
        # C2 is its own program (speed.cpp's protocol, a child process): it runs before this
        # process initialises the HIP runtime at all, so that the child has the GPU to itself,
        # as speed.cpp does (with this process's runtime up beside it, idle, the child's RunSIFT
        # read 0.313-0.316 ms against 0.289-0.293 alone: profiles/bench_r05n.json,
        # tests/diag/c2_ab.sh)
        c2 = bench_c2(cpu=False)
    sgpu.lib()   # libsiftgpu (and /opt/rocm's HIP runtime) before torch: torch never touches
                 # the GPU here -- torch.distributed (gloo, host) is only the rendezvous
    # Initialise /opt/rocm's HIP runtime now, before `import torch` maps torch's own copy of
    # libamdhip64: a context created after the torch import and the gloo rendezvous otherwise
    # finds no device (observed on the box with two ranks).
    n_dev = sgpu.device_count()
    dist = None
    device = local
    if args.dist_backend == "rccl" and (n_dev < world or local >= n_dev):
        # one GPU per rank (MultiThreadSIFT.cpp:141-155 binds one device per worker): fail here,
        # before any rendezvous, instead of leaving the peers waiting in the RCCL init
        sys.exit(f"bench.py: rank {rank}: {n_dev} GPU(s) visible, {world} ranks need one each "
                 f"(--dist-backend gloo rehearses several ranks on one GPU)")
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
    if c2 is not None and "error" not in c2 and not args.no_cpu_baseline:
        c2["cpu_baseline"] = bench_c2_cpu()
    ctx = sgpu.SiftContext(device, opts)
    rccl = world > 1 and args.dist_backend == "rccl"
    if rccl:
        # RCCL communicator of the per-rank contexts; the id travels over the host rendezvous
        uid = [sgpu.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    # shard of the global batch: images [rank*B, (rank+1)*B), distinct seeds 3000 + global
    # index (4000 + index for C4), SURVEY.md §8(d)
    imgs = synth_batch_fast(B, W, H, (4000 if args.workload == "c4" else 3000) + rank * B)
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

    verify = None
    if args.verify:
        # outside the timed region: the last step's results of every image of every rank, as
        # (count, digest) records, one all-gather (RCCL over xGMI, or gloo in a rehearsal); rank
        # 0 extracts a sample of the other ranks' images itself (a batch of its own: batch
        # composition changes no bit, tests/test_gpu_parity.py) and compares the records
        from sift_dist import image_digest, verify_sample, verify_records, gather_records
        recs = np.array([image_digest(*ctx.features(i)) for i in range(B)], np.int32)
        if rccl:
            allrec = ctx.allgather_i32(recs.reshape(-1), world).reshape(-1, 3)
        elif dist is not None:
            allrec = gather_records(recs, dist)
        else:
            allrec = recs
        if rank == 0:
            sample = verify_sample(world, B, 2)
            seed0 = 4000 if args.workload == "c4" else 3000
            simgs = np.stack([synth_batch_fast(1, W, H, seed0 + g)[0] for g in sample])
            ctx.extract(simgs)
            verify = verify_records(allrec, {g: image_digest(*ctx.features(k))
                                             for k, g in enumerate(sample)})

    # level filters and their kernel launches, as the library ran them (the diagonal schedule
    # shares launches between octaves, the paired-level kernel filters two levels per launch;
    # DESIGN.md 4.3-4.5)
    n_gauss, n_filters = ctx.pyramid_launches()
    total_images = B * world * args.steps
    sumN = geometry_sum(W, H, args.octaves)
    pyr_bytes = 48.0 * sumN * B * args.steps          # 48 B per pyramid px
    achieved = pyr_bytes / (pyr_ms * 1e-3) / 1e9 if pyr_ms > 0 else 0.0

    traffic, prof_note = profiled_traffic(B, W, H, args.octaves)
    if args.workload == "c4":
        workload = (f"C4: {B} x {W}x{H} u8 gray tiles per GPU per step, -fo 0 -no "
                    f"{args.octaves} -d 3 (BASELINE.json configs[3], HBM-bound pyramid stress)")
        metric = "SIFT images/sec on 4096x4096 6-octave tiles (features/sec alongside)"
    else:
        workload = (f"C3 per-GPU shard: {B} x {W}x{H} u8 gray per GPU per step, "
                    f"C2 parameters -fo 0 -no {args.octaves} -d 3 (BASELINE.json configs[1-2])")
        metric = "SIFT images/sec at 1080p (features/sec alongside), 1/2/4/8 MI355X"
    result = {
        "metric": metric,
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
            "workload": workload,
            "images_per_gpu": B, "width": W, "height": H, "octaves": args.octaves,
            "parallelism": f"dp{world}",
        },
        "features_per_sec": feats / elapsed,
        "features_per_image": local_feats / (B * args.steps),
        "stage_ms_per_step": {k: v / args.steps for k, v in stage_acc.items() if k != "match"},
        "roofline": {
            "kernel": f"k_gauss_lean / k_gauss_diag / k_gauss_duo (separable Gaussian levels: "
                      f"the {n_filters} level filters of a step in {n_gauss} launches, back to "
                      "back on the library's stream, HIP events around them)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x the calibrated "
                            "read factor + WRITE_SIZE x the write factor)",
            "traffic_source": prof_note,
            "algorithmic_bytes_per_launch": 48.0 * sumN * B / n_gauss,
            "avg_launch_ms": pyr_ms / args.steps / n_gauss,
        },
    }

    # SURVEY.md §8(d), "full detection (reported separately)": pyramid + extremum stages.  The
    # reference moves 168 B per octave pixel there (pyramid 48 + DoG 60 + gradient writes 24 +
    # extremum reads 36); this build never stores the DoG or gradient images, and its algorithmic
    # bytes are 48 + 24 B (the extremum kernel reads the d + 3 = 6 Gaussian planes once).  `frac`
    # is those algorithmic bytes over the stage time (bytes a kernel re-reads do not count as
    # achievement); the counter bytes of the committed profile of this same tree, when there is
    # one, are reported beside it, and the reference-equivalent rate (168 B over the same time)
    # is not a fraction of any peak.
    det_ms = stage_acc.get("pyramid", 0.0) + stage_acc.get("detect", 0.0)
    if det_ms > 0:
        det_s = det_ms * 1e-3 / args.steps
        alg = (48.0 + 4.0 * (3 + 3)) * sumN * B
        moved, src = detection_traffic(B, W, H, args.octaves)
        result["full_detection"] = {
            "ms_per_step": det_ms / args.steps,
            "algorithmic_bytes_per_step": alg,
            "achieved_GBps": alg / det_s / 1e9,
            "frac": alg / det_s / 1e9 / HBM_PEAK_GBS,
            "measured_bytes_per_step": moved, "measured_source": src,
            "measured_GBps": moved / det_s / 1e9 if moved else None,
            "measured_over_algorithmic": moved / alg if moved else None,
            "reference_equivalent_GBps": 168.0 * sumN * B / det_s / 1e9,
            "note": "pyramid + extremum stages; frac = algorithmic 72 B x sum(N) per image over "
                    "their time; measured = calibrated rocprofv3 counter bytes of the committed "
                    "profile of this source tree (null when none); the reference-equivalent rate "
                    "counts the reference's 168 B x sum(N) per image (SURVEY.md 8d), whose DoG and "
                    "gradient images are never stored here"}
    if rank == 0 and world == 1 and not args.no_match:
        result["match"] = bench_match(ctx, args.match_n, cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and args.workload == "c3" and not args.no_c4:
        result["c4"] = bench_c4(ctx, cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and args.workload == "c3" and not args.no_e2e:
        result["end_to_end"] = bench_end_to_end(ctx, imgs, B, W, H)
    if world > 1 and not args.no_match:
        sm = bench_match_sharded(ctx, args.match_n, rank, world, None if rccl else dist)
        if rank == 0:
            result["match_sharded"] = sm
    if c2 is not None:
        result["c2"] = c2
    if verify is not None:
        result["verify"] = verify
    if rank == 0 and not args.no_cpu_baseline:
        # rank 0 on the host cores beside its GPU work, for every N (the line is self-contained)
        result["cpu_baseline"] = cpu_baseline(imgs, opts)
    if rank == 0:
        print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


def matching_profile(B, W, H, octaves):
    """The newest committed calibrated rocprofv3 summary (tests/profile_kernels.sh +
    tests/pmc_summary.py) of this workload whose source digest (tests/prof_common.py) equals the
    tree being benchmarked, as (summary, note); (None, reason) when there is none -- counters of
    older kernels are never divided by the current kernels' time."""
    import glob
    from prof_common import source_digest
    if (B, W, H, octaves) != (128, 1920, 1080, 4):
        return None, "no profile for this workload"
    here = source_digest()
    newest = None
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")))):
        try:
            s = json.load(open(path))
        except (ValueError, OSError):
            continue
        if not s.get("calibrated_all_kernels") or "hbm_bytes_per_extract" not in s:
            continue
        newest = newest or os.path.relpath(path, ROOT)
        if s.get("source_digest") == here:
            return s, (f"{os.path.relpath(path, ROOT)} (source digest {here}, profiled on box "
                       f"{s.get('box', '?')})")
    return None, (f"no calibrated profile of this source tree (digest {here}) committed; the "
                  f"newest, {newest}, is of another tree" if newest else
                  "no calibrated profile summary committed")


def profiled_traffic(B, W, H, octaves):
    """HBM bytes per Gaussian launch from the committed calibrated summary of this tree and
    workload, or None.  The summary's FETCH_SIZE / WRITE_SIZE are corrected per access width with
    the committed calibration (tests/pmc_calib.sh; MI355X_MICROARCH.md: FETCH_SIZE counts 1/2 of
    a 16-B-per-lane streaming read)."""
    s, note = matching_profile(B, W, H, octaves)
    if s is None:
        return None, note
    try:
        fams = [f for f in s["launches_per_extract"] if f.startswith("k_gauss")]
        n = sum(s["launches_per_extract"][f] for f in fams)
        b = sum(s["hbm_bytes_per_extract"][f] for f in fams)
        return b / n, note
    except (KeyError, ZeroDivisionError):
        return None, "malformed summary: " + note


def detection_traffic(B, W, H, octaves):
    """HBM bytes per extract of the Gaussian and extremum kernels from the committed calibrated
    summary of this tree (see matching_profile), or None."""
    s, note = matching_profile(B, W, H, octaves)
    if s is None:
        return None, note
    h = s["hbm_bytes_per_extract"]
    fams = [f for f in h if f.startswith("k_gauss") or f.startswith("k_extrema")]
    if not any(f.startswith("k_extrema") for f in fams):
        return None, "no extremum kernel in " + note
    return sum(h[f] for f in fams), note


def bench_match(ctx, n, cpu=True):
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
    ops = 2.0 * 128 * n * n          # F = 2 * 128 * N1 * N2 useful ops
    # the same call through the one-GEMM mutual kernel (both decisions from one set of dots)
    ctx.set_debug_flags(ctx.DEBUG_FUSED_MATCH)
    ctx.match(q1, q2)
    fms, fm = 0.0, None
    for _ in range(reps):
        fm = ctx.match(q1, q2)
        fms += ctx.timing()["match"]
    fms /= reps
    ctx.set_debug_flags(0)
    # guided matching (GetGuidedSiftMatch) on a synthetic two-view scene of the same size
    g1, g2, l1, l2, H, F = synth_guided_scene(n, n, 5002)
    ctx.match_guided(g1, g2, l1, l2, H, F)
    gms, gm = 0.0, None
    for _ in range(reps):
        gm = ctx.match_guided(g1, g2, l1, l2, H, F)
        gms += ctx.timing()["match"]
    gms /= reps
    out = {"workload": f"C5 {n}x{n} u8 descriptors, mutual best match",
            "ms": ms, "matches": int(len(m)),
            "path": "i8-MFMA GEMM with a keyless top-2 fold (ratiomax <= 1) for the row side, "
                    "then the sets swapped for the columns some row matched, over the rows of "
                    "set 1 whose largest dot reaches the passing rows' ratio-test bound",
            "ops": ops, "ops_note": "F = 2*128*N1*N2 counted once (SURVEY.md 8d)",
            "tops": ops / (ms * 1e-3) / 1e12,
            "mfma_util": ops / (ms * 1e-3) / 1e12 / I8_MFMA_PEAK_TOPS,
            "fused_ms": fms, "fused_matches": int(len(fm)),
            "fused_mfma_util": ops / (fms * 1e-3) / 1e12 / I8_MFMA_PEAK_TOPS,
            "guided_ms": gms, "guided_matches": int(len(gm))}
    if cpu:
        # the oracle's row side (exact int32 dots + running top-2),
        # row-blocked over OpenMP threads; the mutual match needs both sides, so the full-size
        # time is 2 x the measured row side
        import oracle_py
        threads = max(1, min(16, os.cpu_count() or 1))
        rows = n   # the whole row side (about 1 s on 16 cores); the column side is symmetric
        secs = oracle_py.bench_match_rows(q1, rows, q2, threads)
        full_ms = 2.0 * (n / rows) * secs * 1e3
        out["cpu_baseline"] = {"value": full_ms, "unit": f"ms per {n}x{n} mutual match",
                               "cores": threads, "kind": "port",
                               "sample": f"row side of {rows} of the {n} rows against all {n} "
                                         f"columns (oracle/liboracle.so, g++ -O3), "
                                         f"{secs:.2f} s, extrapolated to both sides",
                               "gpu_speedup": full_ms / ms}
    return out


def bench_c4(ctx, batch=16, steps=10, warmup=3, cpu=True):
    """BASELINE configs[3]: 4096x4096 tiles, -no 6 (the HBM-bound pyramid stress), a batch of
    `batch` distinct tiles (seeds 4000..) staged in HBM, `steps` timed passes after `warmup`
    untimed ones (the headline's defaults: one warm-up and 3 steps read the pyramid ~4 % slower
    than the standalone --workload c4 run).
    Roofline of the pyramid stage as for the headline: 48 B per octave pixel, sum N = 22,364,160
    px per tile (1.0735 GB per tile)."""
    opts = default_options(octave_num=6)
    c4 = sgpu.SiftContext(ctx.device, opts)
    try:
        imgs = synth_batch_fast(batch, 4096, 4096, 4000)
        c4.stage(imgs)
        for _ in range(warmup):
            c4.extract_staged()
        t0 = time.perf_counter()
        pyr, feats, st = 0.0, 0, {}
        for _ in range(steps):
            c4.extract_staged()
            feats += c4.total()
            t = c4.timing()
            pyr += t["pyramid"]
            for k, v in t.items():
                st[k] = st.get(k, 0.0) + v
        el = time.perf_counter() - t0
        sumN = geometry_sum(4096, 4096, 6)
        n_gauss, n_filt = c4.pyramid_launches()   # as the library ran them
        achieved = 48.0 * sumN * batch * steps / (pyr * 1e-3) / 1e9
        out = {"workload": f"C4: {batch} x 4096x4096 u8 tiles per step, -fo 0 -no 6 -d 3, "
                            f"staged in HBM", "value": batch * steps / el, "unit": "images/s",
                "ms_per_step": el / steps * 1e3, "features_per_image": feats / (batch * steps),
                "stage_ms_per_step": {k: v / steps for k, v in st.items() if k != "match"},
                "roofline": {"kernel": f"k_gauss_lean / k_gauss_diag / k_gauss_duo ({n_filt} level "
                                       f"filters in {n_gauss} launches per step)",
                             "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                             "algorithmic_bytes_per_launch": 48.0 * sumN * batch / n_gauss,
                             "avg_launch_ms": pyr / steps / n_gauss}}
        if cpu:
            # the oracle on the same tiles, one per OpenMP thread
            import oracle_py
            threads = max(1, min(8, batch, os.cpu_count() or 1))   # ~10 s of wall time
            secs, cf = oracle_py.bench_extract(imgs[:threads], opts, threads=threads)
            out["cpu_baseline"] = {"value": threads / secs, "unit": "images/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{threads} of the staged 4096x4096 tiles (-no 6), "
                                             f"one per OpenMP thread, oracle/liboracle.so",
                                   "features_per_image": cf / threads}
            s1, _ = oracle_py.bench_extract(imgs[:1], opts, threads=1)
            out["cpu_baseline"]["one_thread"] = {"value": 1.0 / s1, "unit": "images/s",
                                                 "cores": 1, "sample": "tile 0, one thread"}
        return out
    finally:
        c4.close()


def bench_end_to_end(ctx, imgs, B, W, H, nbatches=16):
    """Host-in / host-out throughput (sgpu_extract_stream): batches of B images in page-locked
    host memory go up over PCIe, through the whole path, and every key and descriptor comes
    back to page-locked host memory -- the work of the reference's RunSIFT + GetFeatureVector per
    image (PyramidCU.cpp:949-976 upload, :434 descriptor download).  Uploads of batch k+1 and
    downloads of batch k-1 overlap batch k's kernels.  Two distinct input batches (seeds 3000..,
    the staged one, and 3000 + B..) alternate over `nbatches` batches; one warm-up call."""
    pins = []
    try:
        ins = []
        for k, src in enumerate((imgs, synth_batch_fast(B, W, H, 3000 + B))):
            p = sgpu.PinnedArray(src.shape, np.uint8)
            p.array[...] = src
            pins.append(p)
            ins.append(p.array)
        cap = nbatches * B * 4000
        kb = sgpu.PinnedArray((cap, 4), np.float32)
        db = sgpu.PinnedArray((cap, 128), np.float32)
        pins += [kb, db]
        batches = [ins[k % 2] for k in range(nbatches)]
        ctx.extract_stream(batches[:2], kb.array, db.array)   # warm-up (buffers, capacities)
        t0 = time.perf_counter()
        k, d, c = ctx.extract_stream(batches, kb.array, db.array)
        el = time.perf_counter() - t0
        in_bytes = float(nbatches) * B * W * H
        out_bytes = float(len(k)) * (16 + 512)
        return {"workload": f"{nbatches} batches of {B} x {W}x{H} u8 from page-locked host "
                            "memory, keys + descriptors back to page-locked host memory "
                            "(sgpu_extract_stream)",
                "value": nbatches * B / el, "unit": "images/s",
                "ms_per_batch": el / nbatches * 1e3,
                "features_per_image": float(len(k)) / (nbatches * B),
                "pcie_bytes_per_batch": {"h2d": in_bytes / nbatches, "d2h": out_bytes / nbatches},
                "pcie_GBps": {"h2d": in_bytes / el / 1e9, "d2h": out_bytes / el / 1e9}}
    except Exception as ex:   # never costs the main measurement
        return {"error": str(ex)}
    finally:
        for p in pins:
            p.free()


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
        # every rank reaches here together: sgpu_match_sharded agrees on failure (an all-reduce of
        # a status flag) before its all-gather, and the timing all-reduces above run only after
        # every rank's match returned
        return {"error": str(ex)}


def bench_c2(repeat=30, cpu=True):
    """BASELINE configs[1]: one 1920x1080 image through the drop-in C++ API, TestWin/speed.cpp's
    protocol (speed.cpp:60-155): bin/speed_replica (SiftGPU.h, directly linked) loads the PGM
    once, warms up, then times `repeat` x RunSIFT() -- host image in, keys and descriptors back in
    the object's host buffers, as the reference's RunSIFT -- and `repeat` more for the per-stage
    _timing slots.  The child process shares the GPU with this (idle) one."""
    import subprocess
    import tempfile
    from sift_synth import synth_image
    exe = os.path.join(ROOT, "modify-sift-gpu_amd", "bin", "speed_replica")
    img = synth_image(1920, 1080, 2000)       # C2 seed 2000
    try:
        with tempfile.TemporaryDirectory() as td:
            pgm = os.path.join(td, "c2.pgm")
            with open(pgm, "wb") as f:
                f.write(b"P5\n1920 1080\n255\n" + img.tobytes())
            # three runs of the protocol (each its own process, as speed.cpp), the median kept:
            # one run's 30 calls share the box's state of the moment (one read 0.53 ms with a
            # slow descriptor download, against 0.38-0.41 in the runs around it)
            runs = []
            for _ in range(3):
                r = subprocess.run([exe, str(repeat), "--", "-i", pgm, "-fo", "0", "-no", "4", "-d", "3"],
                                   capture_output=True, text=True, timeout=300)
                if r.returncode != 0:
                    return {"error": f"speed_replica exit {r.returncode}: {r.stderr[-300:]}"}
                runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
        runs.sort(key=lambda x: x["avg_ms"])
        sp = runs[1]
    except Exception as ex:   # never costs the main measurement
        return {"error": str(ex)}
    out = {"workload": "C2: one 1920x1080 u8 PGM, -fo 0 -no 4 -d 3, SiftGPU::RunSIFT() through "
                       "include/SiftGPU.h (TestWin/speed.cpp protocol, bin/speed_replica)",
           "value": 1e3 / sp["avg_ms"], "unit": "images/s", "ms_per_image": sp["avg_ms"],
           "features": sp["features"], "repeat": sp["repeat"], "stable": sp["stable"],
           "runs_ms_per_image": [x["avg_ms"] for x in runs], "run_kept": "median of 3",
           "timing_ms": sp["timing_ms"],
           "note": "host image in, features in the object's host buffers; _timing slots as "
                   "SiftGPU.cpp:368 / speed.cpp:147-153"}
    if cpu:
        out["cpu_baseline"] = bench_c2_cpu()
    return out


def bench_c2_cpu():
    """C2's CPU baseline: the oracle on the same image, one thread and all cores."""
    import oracle_py
    from sift_synth import synth_image
    img = synth_image(1920, 1080, 2000)
    secs, feats = oracle_py.bench_extract(img[None], default_options(octave_num=4), threads=1)
    out = {"value": 1.0 / secs, "unit": "images/s", "cores": 1, "kind": "port",
           "sample": "the same image, one thread, oracle/liboracle.so",
           "ms_per_image": secs * 1e3, "features": int(feats)}
    # all cores (1 thread and all cores): copies of the image, one per thread
    threads = max(1, min(16, os.cpu_count() or 1))
    sa, _ = oracle_py.bench_extract(np.repeat(img[None], threads, 0),
                                    default_options(octave_num=4), threads=threads)
    out["all_cores"] = {"value": threads / sa, "unit": "images/s", "cores": threads,
                        "sample": f"{threads} copies of the image, one per OpenMP thread"}
    return out


def cpu_baseline(imgs, opts):
    """The CPU oracle (oracle/, a C++ restatement of the reference) on a bounded sample of the
    same workload: one staged image per OpenMP thread (about 1 s of wall time, 15-20 s of CPU
    work on 16 threads)."""
    import oracle_py
    threads = max(1, min(16, os.cpu_count() or 1, len(imgs)))
    n = threads
    secs, feats = oracle_py.bench_extract(imgs[:n], opts, threads=threads)
    return {"value": n / secs, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} of the staged {imgs.shape[2]}x{imgs.shape[1]} images (-fo 0 -no "
                      f"{opts.octave_num} -d 3), one per OpenMP thread, oracle/liboracle.so "
                      f"(g++ -O3, strict IEEE)",
            "features_per_image": feats / n}


if __name__ == "__main__":
    main()
