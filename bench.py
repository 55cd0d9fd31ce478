#!/usr/bin/env python3
"""bench.py — MI355X throughput of the ORB-SLAM3 hot path (BASELINE.json configs).

Headline (N=1 default): BASELINE.json configs[1] — synthetic 640x480, 8-level pyramid,
1000 features/frame, ORBextractor only.  One step = one pass of the extractor over a batch
of B synthetic frames already resident in HBM.  value = frames/s of the whole job.

Multi-GPU: one process per GPU (torch.distributed.run); each rank extracts its own batch
(frames are independent: weak scaling, no collective on the data path).  Timing is
barrier + synchronize on both sides of exactly K steps; the max over ranks is reported.

Also reported: the dominant kernel's roofline (HIP events around every stage during the
timed steps), and the CPU baseline (the oracle restatement, rank 0 at N=1 only).

Second leg ("lba", BASELINE.json configs[3]): Optimizer::LocalBundleAdjustment's LM/Schur
solve on synthetic 50 KF x 2000 point x 8 observation windows (2% outliers, 48 free KFs),
a batch of independent windows per GPU per call (windows shard across ranks like frames).
Reported as LM iterations/s (one OptimizationAlgorithmLevenberg::solve incl. its trials),
whole job, plus LBA calls/s, the single-window latency and the oracle's single-core rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def level_sizes(w, h, nlevels=8, scale=1.2):
    """ComputePyramid level sizes (ORBextractor.cc:1157) in the reference's float arithmetic."""
    sizes = []
    s = [1.0]
    for i in range(1, nlevels):
        s.append(float(np.float32(np.float64(np.float32(s[-1])) * np.float64(np.float32(scale)))))
    for l in range(nlevels):
        inv = np.float32(1.0) / np.float32(s[l])
        sizes.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return sizes


def algorithmic_bytes(w, h, kps_per_frame):
    """Per-frame algorithmic HBM bytes of each stage."""
    sz = level_sizes(w, h)
    P = [a * b for a, b in sz]
    out = {
        "k_resize": sum(P[:-1]) + sum(P[1:]),        # read level l-1, write level l
        "k_fast_wave": sum(P),                        # read every level pixel once (+ candidates, small)
        "k_octree": 0,                                # candidate lists only (KB, L2-resident)
        "k_layout": 0,
        "k_orb": kps_per_frame * (4 + 28 + 32),       # kp in, kp + descriptor out (43x43 raw windows: L2)
    }
    pipeline = P[0] + sum(P[1:]) + sum(P) + kps_per_frame * 60  # SURVEY.md §8(d) B_frame
    return out, pipeline


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--unique", type=int, default=256, help="distinct synthetic frames per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=384)
    ap.add_argument("--lba-windows", type=int, default=64, help="LBA windows per GPU per call (0 = skip)")
    ap.add_argument("--lba-calls", type=int, default=3)
    ap.add_argument("--lba-inflight", type=int, default=3, help="LBA solver handles driven concurrently")
    ap.add_argument("--match-pairs", type=int, default=128, help="(keyframe, frame) pairs per GPU per step (0 = skip)")
    ap.add_argument("--pose-frames", type=int, default=512, help="PoseOptimization frames per GPU per call (0 = skip)")
    ap.add_argument("--stereo-pairs", type=int, default=128, help="stereo frames per GPU per step (0 = skip)")
    ap.add_argument("--inflight", type=int, default=3, help="extraction batches in flight (handles / streams)")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth

    W, H, B = args.width, args.height, args.batch
    nuniq = min(args.unique, B)
    base = synth.frames(range(rank * 100000, rank * 100000 + nuniq), W, H)
    frames_np = np.concatenate([base] * ((B + nuniq - 1) // nuniq))[:B]
    d_imgs = torch.from_numpy(frames_np).to(device)
    # `inflight` batches in flight: each slot has its own extractor handle (scratch), output
    # buffers and stream, so consecutive batches overlap the way a serving loop keeps several
    # requests on the GPU; every frame of every step is still processed inside the timed region
    NS = max(1, args.inflight)
    exs = [slamhot.ORBextractor(nfeatures=args.nfeatures, device=local_rank, max_size=(W, H), max_batch=B)
           for _ in range(NS)]
    ex = exs[0]
    cap = ex.cap
    outs = [(torch.zeros((B, cap, 28), dtype=torch.uint8, device=device),
             torch.zeros((B, cap, 32), dtype=torch.uint8, device=device),
             torch.zeros(B, dtype=torch.int32, device=device), torch.zeros(B, dtype=torch.int32, device=device))
            for _ in range(NS)]
    d_kps, d_desc, d_n, d_mono = outs[0]
    stream_objs = [torch.cuda.Stream(device) for _ in range(NS)]
    calls = [0] * NS

    def step(i):
        k_, d_, n_, m_ = outs[i % NS]
        exs[i % NS].extract_batch_device(d_imgs.data_ptr(), B, W, H, k_.data_ptr(), d_.data_ptr(), cap, n_.data_ptr(),
                                         m_.data_ptr(), lap=(0, 0), stream=stream_objs[i % NS].cuda_stream)
        calls[i % NS] += 1

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-stage HIP-event timing in a second, isolated pass: K batches through handle 0 alone
    # (one batch in flight), so each stage's launch duration is the kernel's own, not shared
    # with concurrent batches; `rocprofv3 ... bench.py --inflight 1` reproduces it
    ex.stage_stats(reset=True)
    ex.set_profiling(True)
    calls[0] = 0
    for i in range(args.steps):
        step(0)
    torch.cuda.synchronize(device)
    ex.set_profiling(False)
    stages = ex.stage_stats(reset=True)
    prof_calls = calls[0]

    n_host = d_n.cpu().numpy()
    kps_per_frame = float(n_host.mean())
    dig = sdist.digest(d_desc[:, :64].cpu().numpy())
    elapsed, _ = sdist.reduce_run(dist, device, elapsed, B * args.steps)
    total_kps = sum(c for c, _ in sdist.gather_digests(dist, device, world, int(n_host.sum()), dig))

    frames_total = B * args.steps * world
    value = frames_total / elapsed
    ms_per_step = elapsed / args.steps * 1000.0

    # dominant kernel roofline (HIP events around each stage, on the launch stream)
    alg, pipe_bytes = algorithmic_bytes(W, H, kps_per_frame)
    dom = max(stages, key=lambda k: stages[k][0])
    dom_ms, dom_launches = stages[dom]
    dom_avg_s = dom_ms / 1000.0 / max(dom_launches, 1)
    # the extractor splits a batch into frame ranges on concurrent streams: one launch of a
    # stage covers B * steps / launches frames
    frames_per_launch = B * prof_calls / max(dom_launches, 1)
    dom_bytes = alg.get(dom, 0) * frames_per_launch
    achieved = dom_bytes / dom_avg_s / 1e9 if dom_avg_s > 0 else 0.0
    stage_avg_ms = {k: v[0] / max(prof_calls, 1) for k, v in stages.items()}  # per batch, summed over ranges
    traffic = None
    tf = ROOT / "profiles" / "traffic_latest.json"
    if tf.exists():
        try:
            tj = json.loads(tf.read_text())
            if tj.get("kernel") == dom and tj.get("batch") == B and tj.get("width") == W:
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": "ORB extract+match frames/s and LocalBA iters/s per GPU; ATE vs reference",
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded procedural textures, slamhot/synth.py)",
        "config": {
            "workload": f"ORBextractor-only, synthetic {W}x{H} 8-level pyramid, {args.nfeatures} feat/frame "
                        f"(BASELINE.json configs[1])",
            "frames_per_gpu_per_step": B,
            "nfeatures": args.nfeatures,
            "levels": 8,
            "scale_factor": 1.2,
            "fast_thresholds": [20, 7],
            "parallelism": f"frame-sharded x{world}",
            "batches_in_flight": NS,
            "keypoints_per_frame": round(kps_per_frame, 1),
            "total_keypoints": total_kps,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": int(dom_bytes),
            "frames_per_launch": frames_per_launch,
            "measured": "HIP events, isolated pass after the timed region (1 batch in flight, stages serialized)",
            "avg_launch_ms": round(dom_avg_s * 1000.0, 5),
        },
        "stages_ms_per_step": {k: round(v, 5) for k, v in stage_avg_ms.items()},
        "pipeline_roofline": {
            "bytes_per_frame": int(pipe_bytes),
            "achieved_GBps": round(pipe_bytes * B / (ms_per_step / 1000.0) / 1e9, 2),
        },
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, W, H)

    if args.match_pairs > 0:
        result["match"] = match_leg(args, rank, world, local_rank, dist, device)
    if args.lba_windows > 0:
        result["lba"] = lba_leg(args, rank, world, local_rank, dist, device)
    if args.pose_frames > 0:
        result["pose"] = pose_leg(args, rank, world, local_rank, dist, device)
    if args.stereo_pairs > 0:
        result["stereo"] = stereo_leg(args, rank, world, local_rank, dist, device)

    if rank == 0:
        print(json.dumps(result), flush=True)
    for e in exs:
        e.close()
    if dist:
        dist.destroy_process_group()


def match_leg(args, rank, world, local_rank, dist, device):
    """Extract + ComputeBoW + SearchByBoW(KF, Frame) frames/s (BASELINE.json configs[2] shape on
    synthetic data: no EuRoC images here).  A step extracts 2P frames (P keyframes and P frames
    that are shifted / rotated copies of them), builds every FeatureVector on the device and
    matches the P pairs; everything stays in HBM."""
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    Pn, W, H = args.match_pairs, args.width, args.height
    nuniq = min(16, Pn)
    seeds = sdist.shard(nuniq * world, rank, world)
    kfs = [synth.frame(20000 + s, W, H) for s in seeds]
    rng = np.random.default_rng(rank)
    pairs_img = []
    for i in range(nuniq):
        dx, dy, a = rng.uniform(-8, 8), rng.uniform(-6, 6), rng.uniform(-10, 10)
        pairs_img.append((kfs[i], synth.shifted(kfs[i], dx, dy, a, 40000 + seeds[i])))
    imgs = np.stack([im for i in range(Pn) for im in pairs_img[i % nuniq]])
    F = len(imgs)
    # the vocabulary is built (or, with ORBvoc.txt, loaded) once and replicated from rank 0
    par, leaf, dn, wn = sdist.broadcast_arrays(dist, device, synth.vocab(10, 6, 0) if rank == 0 else None)
    voc = slamhot.Vocabulary(par, leaf, dn, wn, k=10, L=6, device=local_rank)
    m = slamhot.ORBmatcher(0.7, True, device=local_rank)
    ex = slamhot.ORBextractor(nfeatures=args.nfeatures, device=local_rank, max_size=(W, H), max_batch=F)
    cap = ex.cap
    d_img = torch.from_numpy(imgs).to(device)
    d_kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=device)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=device)
    d_n = torch.zeros(F, dtype=torch.int32, device=device)
    d_mono = torch.zeros(F, dtype=torch.int32, device=device)
    pairs = [(2 * i, 2 * i + 1) for i in range(Pn)]
    d_a2b = torch.zeros((Pn, cap), dtype=torch.int32, device=device)
    d_b2a = torch.zeros((Pn, cap), dtype=torch.int32, device=device)
    d_nm = torch.zeros(Pn, dtype=torch.int32, device=device)
    # one real stream orders extraction before matching (NULL would mean each handle's own stream)
    stream_obj = torch.cuda.Stream(device)
    stream = stream_obj.cuda_stream

    def step():
        ex.extract_batch_device(d_img.data_ptr(), F, W, H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                d_n.data_ptr(), d_mono.data_ptr(), stream=stream)
        m.bow_match_batch_device(voc, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), pairs,
                                 d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr(), stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    skipped = m.bow_match_batch_status(stream)
    nm = d_nm.cpu().numpy()
    elapsed, frames_all = sdist.reduce_run(dist, device, elapsed, float(F * args.steps))
    out = {
        "metric": "ORB extract + ComputeBoW + SearchByBoW frames/s",
        "value": round(frames_all / elapsed, 2),
        "unit": "frames/s",
        "dtype": "u8",
        "config": {"workload": f"synthetic {W}x{H}, {args.nfeatures} feat/frame, {Pn} (keyframe, frame) pairs "
                               f"per GPU per step, synthetic k=10 L=6 vocabulary, levelsup 4, nnratio 0.7, "
                               f"checkOri (BASELINE.json configs[2] shape)",
                   "parallelism": f"pair-sharded x{world}"},
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "matches_per_pair": round(float(nm.mean()), 1),
        "skipped_pairs": skipped,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        p = ob.params(nfeatures=args.nfeatures)
        t0 = time.perf_counter()
        done = 0
        while done < min(8, nuniq) and time.perf_counter() - t0 < 10.0:
            sides = []
            for im in pairs_img[done]:
                k, d, _ = ob.extract(im, p)
                _, wt, nid = ob.vocab_transform(par, leaf, dn, wn, 6, d, 4)
                sides.append((d, k["angle"], None) + synth.feature_vector(nid, wt))
            ob.search_by_bow(sides[0], sides[1], 0.7, True, False)
            done += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(2 * done / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{done} pairs ({2 * done} frames) one at a time on one core: oracle "
                                         f"extract + vocabulary transform + FeatureVector + SearchByBoW"}
    ex.close()
    m.close()
    voc.close()
    return out


def pose_leg(args, rank, world, local_rank, dist, device):
    """Optimizer::PoseOptimization frames/s: batches of synthetic frames (1000 keypoints, 80%
    with MapPoints, 10% outliers, EuRoC intrinsics), one workgroup per frame."""
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    nf = args.pose_frames
    pool = [synth.pose_frame(s) for s in sdist.shard(16 * world, rank, world)]
    frames = [pool[i % len(pool)] for i in range(nf)]
    S = slamhot.PoseOptimizer(device=local_rank)
    S.solve(frames[:8])
    if dist:
        dist.barrier()
    calls = 3
    t0 = time.perf_counter()
    for _ in range(calls):
        res = S.solve(frames)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed, total = sdist.reduce_run(dist, device, time.perf_counter() - t0, float(nf * calls))
    out = {
        "metric": "Optimizer::PoseOptimization frames/s",
        "value": round(total / elapsed, 1),
        "unit": "frames/s",
        "dtype": "f64",
        "config": {"workload": "synthetic frames, 1000 keypoints, ~800 MapPoint observations, 10% outliers, "
                               "4 x optimize(10)", "frames_per_gpu_per_call": nf,
                   "parallelism": f"frame-sharded x{world}"},
        "ms_per_call": round(elapsed / calls * 1e3, 3),
        "mean_inliers": round(float(np.mean([r["n_inliers"] for r in res])), 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        t0 = time.perf_counter()
        k = 0
        while k < len(pool) and time.perf_counter() - t0 < 3.0:
            ob.pose_optimization(pool[k])
            k += 1
        out["cpu_baseline"] = {"value": round(k / (time.perf_counter() - t0), 2), "unit": "frames/s", "cores": 1,
                               "kind": "port", "sample": f"{k} frames one at a time on one core; "
                                                         f"oracle/pose_oracle.cpp -O3"}
    S.close()
    return out


def stereo_leg(args, rank, world, local_rank, dist, device):
    """Stereo Frame construction frames/s (EuRoC stereo shape, BASELINE.json configs[3]:
    752x480, 1200 features): a step rectifies P raw left and P raw right images with the
    EuRoC calibration (cv::remap, stereo_euroc.cc:168-169), extracts both and runs
    ComputeStereoMatches on the P pairs, all device-resident.  rectify_ms / stereo_ms isolate
    the remap and matching kernels (torch events on the launch stream)."""
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    P, W, H, NF = args.stereo_pairs, 752, 480, 1200
    from slamhot import euroc
    calib = {k: np.array(v) if isinstance(v, list) else v
             for k, v in json.loads((ROOT / "tests" / "golden" / "euroc_stereo_calib.json").read_text()).items()}
    maps = [euroc.init_undistort_rectify_map(calib[f"{sd}.K"], calib[f"{sd}.D"], calib[f"{sd}.R"], calib[f"{sd}.P"],
                                             (W, H)) for sd in ("LEFT", "RIGHT")]
    # raw camera images: synthetic rectified pairs pushed back through the calibration
    seeds = sdist.shard(8 * world, rank, world)
    prs = []
    for s_ in seeds:
        lr = synth.stereo_pair(int(s_) + 500, W, H)
        prs.append(tuple(synth.unrectify(im, *mp) for im, mp in zip(lr, maps)))
    il = np.stack([prs[i % len(prs)][0] for i in range(P)])
    ir = np.stack([prs[i % len(prs)][1] for i in range(P)])
    mbf = synth.EUROC_STEREO["bf"]
    mb = mbf / synth.EUROC_STEREO["fx"]
    left = slamhot.ORBextractor(nfeatures=NF, device=local_rank, max_size=(W, H), max_batch=P)
    right = slamhot.ORBextractor(nfeatures=NF, device=local_rank, max_size=(W, H), max_batch=P)
    sm = slamhot.StereoMatcher(device=local_rank)
    rect = [euroc.Rectifier(*mp, device=local_rank) for mp in maps]
    cap = left.cap
    d_raw_l, d_raw_r = torch.from_numpy(il).to(device), torch.from_numpy(ir).to(device)
    d_il, d_ir = torch.empty_like(d_raw_l), torch.empty_like(d_raw_r)
    bufs = [(torch.zeros((P, cap, 28), dtype=torch.uint8, device=device),
             torch.zeros((P, cap, 32), dtype=torch.uint8, device=device),
             torch.zeros(P, dtype=torch.int32, device=device), torch.zeros(P, dtype=torch.int32, device=device))
            for _ in range(2)]
    d_ur = torch.empty((P, cap), dtype=torch.float32, device=device)
    d_dep = torch.empty((P, cap), dtype=torch.float32, device=device)
    stream = torch.cuda.Stream(device)  # a real stream: NULL would mean each handle's own stream
    ev = []
    ev_rect = []

    def step(timed=False):
        if timed:
            r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r0.record(stream)
        for rc, raw, out in ((rect[0], d_raw_l, d_il), (rect[1], d_raw_r, d_ir)):
            rc.rectify_batch_device(P, raw.data_ptr(), W, W * H, out.data_ptr(), W, W * H, stream=stream.cuda_stream)
        if timed:
            r1.record(stream)
            ev_rect.append((r0, r1))
        for ex, img, (k, d, n, m) in ((left, d_il, bufs[0]), (right, d_ir, bufs[1])):
            ex.extract_batch_device(img.data_ptr(), P, W, H, k.data_ptr(), d.data_ptr(), cap, n.data_ptr(),
                                    m.data_ptr(), stream=stream.cuda_stream)
        (kl, dl, nl, _), (kr, dr, nr, _) = bufs
        if timed:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        sm.match_batch_device(left, right, P, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(),
                              dr.data_ptr(), nr.data_ptr(), cap, mbf, mb, d_ur.data_ptr(), d_dep.data_ptr(),
                              stream=stream.cuda_stream)
        if timed:
            b.record(stream)
            ev.append((a, b))

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    steps = max(args.steps // 2, 3)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(timed=True)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed, total = sdist.reduce_run(dist, device, time.perf_counter() - t0, float(P * steps))
    stereo_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rect_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_rect]))
    nl_h = bufs[0][2].cpu().numpy()
    ur = d_ur.cpu().numpy()
    matched = float(np.mean([(ur[f, : nl_h[f]] >= 0).sum() for f in range(P)]))
    out = {
        "metric": "stereo Frame (2x remap + 2x ORB extract + ComputeStereoMatches) frames/s",
        "value": round(total / elapsed, 1),
        "unit": "frames/s",
        "dtype": "u8",
        "config": {"workload": f"synthetic raw stereo pairs {W}x{H} (EuRoC calibration), {NF} features, EuRoC bf",
                   "pairs_per_gpu_per_step": P, "parallelism": f"frame-sharded x{world}"},
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "stereo_match_ms_per_step": round(stereo_ms, 4),
        "rectify_ms_per_step": round(rect_ms, 4),
        "rectify_GBps": round(2 * P * W * H * 2 / (rect_ms / 1e3) / 1e9, 1),
        "stereo_match_frames_per_s": round(P / (stereo_ms / 1e3), 1),
        "mean_stereo_matches": round(matched, 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        p = ob.params(nfeatures=NF)
        sc, isc, _, _, _ = ob.levels(p)
        t_ex = t_st = 0.0
        k = 0
        while k < len(prs) and t_ex + t_st < 10.0:
            t1 = time.perf_counter()
            l_img = ob.remap_linear(prs[k][0], rect[0].map_x, rect[0].map_y)
            r_img = ob.remap_linear(prs[k][1], rect[1].map_x, rect[1].map_y)
            kl, dl, _ = ob.extract(l_img, p)
            kr, dr, _ = ob.extract(r_img, p)
            t_ex += time.perf_counter() - t1
            pl, pr = ob.pyramid(l_img, p), ob.pyramid(r_img, p)  # built inside extract too; untimed
            t2 = time.perf_counter()
            ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, mbf, mb)
            t_st += time.perf_counter() - t2
            k += 1
        out["cpu_baseline"] = {"value": round(k / (t_ex + t_st), 2), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{k} stereo frames on one core (oracle remap x2 + extract x2 + "
                                         f"oracle/stereo_oracle.cpp, -O3)",
                               "stereo_match_only_frames_per_s": round(k / t_st, 1)}
    for rc in rect:
        rc.close()
    left.close()
    right.close()
    sm.close()
    return out


def sdist_shard_seeds(rank, world, n):
    from slamhot import dist as sdist
    return sdist.shard(n * world, rank, world)


def lba_leg(args, rank, world, local_rank, dist, device):
    """LM iterations/s of the device LBA solver on config-4 windows (BASELINE.json configs[3])."""
    import torch

    import slamhot
    from slamhot import synth
    nwin = args.lba_windows
    # windows are sharded by rank: rank r solves its own seeds (independent units)
    pool = [synth.lba_window(s) for s in sdist_shard_seeds(rank, world, 8)]
    windows = [pool[i % len(pool)] for i in range(nwin)]
    S = slamhot.LocalBundleAdjustment(device=local_rank)
    S.solve(windows[: min(4, nwin)])  # warm-up
    single = S.solve(pool[0])
    dev1, plan1, _ = S.last_stats()
    # accuracy: ATE of the solved KeyFrame centres against the windows' ground truth
    ate_dev = [window_ate(w, r["kf_Tcw"]) for w, r in zip(pool, S.solve(pool))]
    ate_init = [window_ate(w, w["kf_Tcw"]) for w in pool]
    it1 = single["iterations"][0] + single["iterations"][1]
    # `lba_inflight` solver handles driven from host threads (the C call releases the GIL), each
    # on its own window set: one call's host planning overlaps another's device LM loop.  The
    # windows are flattened to C structs before the timed region, as a C++ caller holds them.
    import threading
    NL = max(1, args.lba_inflight)
    solvers = [S] + [slamhot.LocalBundleAdjustment(device=local_rank) for _ in range(NL - 1)]
    runs = [sv.prepare(windows) for sv in solvers]
    for r_ in runs:
        r_()
    stats = [[0, 0.0, 0.0] for _ in range(NL)]

    def worker(t):
        for _ in range(args.lba_calls):
            stats[t][0] += runs[t]()
            d, pl, _ = solvers[t].last_stats()
            stats[t][1] += d
            stats[t][2] += pl

    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(1, NL)]
    for th in ths:
        th.start()
    worker(0)
    for th in ths:
        th.join()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    iters = sum(x[0] for x in stats)
    dev_ms = sum(x[1] for x in stats) / NL
    plan_ms = sum(x[2] for x in stats) / NL
    from slamhot import dist as sdist
    dev_max, _ = sdist.reduce_run(dist, device, dev_ms, 0.0)
    elapsed, iters_all = sdist.reduce_run(dist, device, elapsed, float(iters))
    out = {
        "metric": "LocalBundleAdjustment LM iterations/s",
        "value": round(iters_all / elapsed, 1),
        "unit": "LM iterations/s",
        "dtype": "f64",
        "config": {"workload": "synthetic LocalBA 50 KF x 2000 pts x 8 obs, 2% outliers, 48 free KFs, "
                               "schedule 5 + 10 (BASELINE.json configs[3])",
                   "windows_per_gpu_per_call": nwin, "calls": args.lba_calls,
                   "parallelism": f"window-sharded x{world}"},
        "lba_calls_per_s": round(nwin * args.lba_calls * NL * world / elapsed, 2),
        "solves_in_flight": NL,
        "ms_per_call": round(elapsed / args.lba_calls * 1e3, 3),  # NL calls run concurrently
        "device_lm_iters_per_s_one_solver": round(iters_all / NL / (dev_max / 1e3), 1) if dev_max > 0 else None,
        "host_plan_ms_per_call": round(plan_ms / args.lba_calls, 3),
        "single_window": {"lm_iterations": it1, "device_ms": round(dev1, 3),
                          "ms_per_lm_iteration": round(dev1 / max(it1, 1), 4)},
        "ate": {"metric": "ATE RMSE of the window's KeyFrame centres vs ground truth after LBA "
                          "(SE3 alignment, slamhot.ate = evaluate_ate_scale.py align)",
                "unit": "m", "windows": len(pool),
                "initial": round(float(np.mean(ate_init)), 7), "device": round(float(np.mean(ate_dev)), 7)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        reps, cpu_iters, ate_cpu = 0, 0, []
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0 and reps < len(pool):
            r = ob.lba_solve(pool[reps])
            cpu_iters += r["iterations"][0] + r["iterations"][1]
            ate_cpu.append(window_ate(pool[reps], r["kf_Tcw"]))
            reps += 1
        dt = time.perf_counter() - t0
        # matched accuracy: the oracle (restated reference solver) on the same windows
        out["ate"]["oracle_same_windows"] = round(float(np.mean(ate_cpu)), 7)
        out["ate"]["device_same_windows"] = round(float(np.mean(ate_dev[:reps])), 7)
        out["cpu_baseline"] = {
            "value": round(cpu_iters / dt, 2), "unit": "LM iterations/s", "cores": 1, "kind": "port",
            "sample": f"{reps} config-4 windows, one at a time on one core; oracle/lba_oracle.cpp "
                      f"(g2o LM/Schur restatement, dense LDL^T) -O3 -march=x86-64-v3",
        }
    for sv in solvers:
        sv.close()
    return out


def window_ate(w, kf_Tcw):
    """RMSE (m) of KeyFrame camera centres C = -R^T t against the window's ground truth after
    the SE3 alignment of evaluate_ate_scale.py (slamhot.ate.align)."""
    from slamhot import ate
    T = np.asarray(kf_Tcw, np.float64).reshape(-1, 4, 4)
    est = -np.einsum("kji,kj->ki", T[:, :3, :3], T[:, :3, 3])
    G = np.asarray(w["gt_T"], np.float64)
    gt = -np.einsum("kji,kj->ki", G[:, :3, :3], G[:, :3, 3])
    _, _, _, _, err, _ = ate.align(est.T, gt.T)
    return float(np.sqrt(np.mean(err * err)))


def cpu_baseline(args, W, H):
    """The oracle (restated reference CPU path, oracle/orb_oracle.cpp) on the host cores:
    one frame per std::thread at a time, as Frame.cc:119-122 runs extraction."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_bind as ob
    from slamhot import synth
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    nuniq = 32
    imgs = synth.frames(range(5000, 5000 + nuniq), W, H)
    imgs = np.concatenate([imgs] * ((args.cpu_frames + nuniq - 1) // nuniq))[: args.cpu_frames]
    p = ob.params(nfeatures=args.nfeatures)
    ob.extract_many(imgs[:cores], p, nthreads=cores)  # warm-up
    t0 = time.perf_counter()
    ob.extract_many(imgs, p, nthreads=cores)
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    single = 16
    ob.extract_many(imgs[:single], p, nthreads=1)
    dt1 = time.perf_counter() - t1
    return {
        "value": round(len(imgs) / dt, 2),
        "unit": "frames/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{len(imgs)} synthetic {W}x{H} frames, {args.nfeatures} feat, {cores} threads "
                  f"(one frame per thread); oracle/orb_oracle.cpp -O3 -march=x86-64-v3",
        "per_core_frames_per_s": round(single / dt1, 2),
    }


if __name__ == "__main__":
    main()
