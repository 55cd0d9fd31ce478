#!/usr/bin/env python3
"""bench.py — MI355X throughput of the ORB-SLAM3 hot path (BASELINE.json configs).

Headline (`value`): BASELINE.json's metric "ORB extract+match frames/s" on the configuration it
names for it, configs[2] — EuRoC-shaped stereo (752x480, 1200 features/frame, EuRoC
calibration): one step takes P raw stereo frames already resident in HBM through
  cv::remap x2 (stereo_euroc.cc:168-169) -> ORBextractor x2 (Frame.cc:119-122) ->
  Frame::ComputeStereoMatches -> Frame::ComputeBoW -> ORBmatcher::SearchByBoW(KF, F) against
  the previous frame of its sequence (Tracking::TrackReferenceKeyFrame, Tracking.cc:2800-2830)
with everything device-resident.  The images are synthetic renders of a textured room along
smooth camera paths (slamhot/synth.py: stereo_sequence), pushed back through the EuRoC
calibration to raw camera images; the vocabulary is a synthetic k=10 L=6 tree (no ORBvoc.txt
in this image).  value = stereo frames/s of the whole job.

Also reported, each with its own roofline / CPU baseline where it has one:
  extract  configs[1]: ORBextractor-only, synthetic 640x480 8-level pyramid, 1000 features,
           plus the drop-in path's host-image -> host-keypoints rate and single-frame latency
  lba      configs[3]: Optimizer::LocalBundleAdjustment LM/Schur on 50 KF x 2000 pt x 8 obs
           windows (LM iterations/s, FP64 FLOP/s vs peak, ATE vs ground truth and vs the oracle)
  pose     Optimizer::PoseOptimization frames/s
  track    configs[4] per GPU: the per-sequence stereo tracking chain (slamhot_tracker_*)

Multi-GPU: one process per GPU (torch.distributed.run), every rank runs its own frames /
windows / sequences (independent units: weak scaling, no collective on the data path).
Timing is barrier + synchronize on both sides of exactly K steps; the max over ranks is
reported.  CPU baselines (the oracle restatement on the host cores, rank 0 at N=1 only) run
after the timed regions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2  # 256 CUs x 4 SIMDs, one wave64 VALU instr / 2 cycles, 2.4 GHz
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector / matrix (spec)
LBA_FLOP_PER_ITER = 31.85e6    # one LM iteration of a config-4 window, one trial
LBA_FLOP_PER_EXTRA_TRIAL = 27.05e6  # Schur 17.59 + Cholesky 8.13 + back-substitution 0.61 + errors 0.72


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
    """Per-frame algorithmic HBM bytes of each extractor stage."""
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


def host_cores():
    """CPU threads for the CPU baselines: this process's affinity, capped at the GPU box's CPU
    share per GPU (16; the box's nproc shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def socket_cores():
    """Physical cores of one socket of the host (/proc/cpuinfo "cpu cores"), or None."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("cpu cores"):
                return int(line.split(":", 1)[1])
    except (OSError, ValueError):
        pass
    return None


def add_full_socket(result):
    """BASELINE.md's full-socket CPU number beside every measured CPU baseline.  The GPU box grants
    16 CPU threads per GPU (bench.py host_cores), so an all-core run is not allowed there: the
    full-socket figure is the measured per-thread rate scaled linearly to the socket's physical
    cores -- an upper bound on what the restated CPU path reaches on the whole socket."""
    sc = socket_cores()
    legs = [result] + [v for v in result.values() if isinstance(v, dict)]
    for leg in legs:
        cb = leg.get("cpu_baseline") if isinstance(leg, dict) else None
        if not isinstance(cb, dict) or not sc or not cb.get("cores"):
            continue
        cb["full_socket"] = {"cores": sc, "value_linear_upper_bound": round(cb["value"] / cb["cores"] * sc, 2),
                             "unit": cb.get("unit"), "measured": False,
                             "why": "the GPU box's CPU share is 16 threads per GPU; scaled from the measured "
                                    f"{cb['cores']}-thread rate to the socket's {sc} physical cores (linear, upper bound)"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


PHASE = {"file": None, "rank": 0, "leg": None}


def phase(what):
    """The leg child's current phase, kept in a file its parent reads when the leg fails or times out:
    a rank stuck in its own work ("compute: ...") is told apart from ranks waiting for it in a
    collective ("collective: ...").  Rank 0 also logs each phase on stderr."""
    if PHASE["file"]:
        try:
            Path(PHASE["file"]).write_text(what)
        except OSError:
            pass
    if PHASE["rank"] == 0 and PHASE["leg"]:
        progress(f"  {PHASE['leg']}: {what}")


def timed_region(dist, device, fn, steps):
    """barrier + synchronize, K calls of fn(i), synchronize + barrier; seconds.  Python's cyclic
    garbage collector is collected before and paused inside the region: a gen-2 pass over the
    objects earlier legs left stalls the host threads that queue the device work (the LBA leg read
    ~10% lower after any other leg), which a C / C++ caller of the library does not have."""
    import gc

    import torch
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda d: None)
    gc.collect()
    sync(device)
    if dist:
        phase("collective: barrier before the timed region")
        dist.barrier()
    sync(device)
    was = gc.isenabled()
    gc.disable()
    try:
        phase(f"compute: timed region ({steps} steps)")
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        sync(device)
        if dist:
            phase("collective: barrier after the timed region")
            dist.barrier()
        el = time.perf_counter() - t0
        phase("compute: after the timed region")
        return el
    finally:
        if was:
            gc.enable()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, timeout_s):
    """`bench.py --gpus N` without WORLD_SIZE in the environment: start N rank processes of this
    script (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free MASTER_PORT; rank r
    drives cuda:r over nccl), relay rank 0's JSON line and return the job's exit status.  This
    process never touches the GPU (no torch import) and never execs: the ranks are children.  A rank
    that fails ends the job (the others are terminated, its status returned); a job still running
    after `timeout_s` is killed (status 124)."""
    import signal
    import subprocess
    import threading
    env = dict(os.environ)
    env.update(WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve())] + argv, env=e,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, stderr=None))
    lines = []

    def relay():  # rank 0's stdout: the JSON line to our stdout, anything else to stderr
        for raw in procs[0].stdout:
            s = raw.decode(errors="replace")
            if s.lstrip().startswith("{"):
                lines.append(s)
            else:
                sys.stderr.write(s)
    t = threading.Thread(target=relay, daemon=True)
    t.start()

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t_end = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    # one waiter per rank records when it exited: a rank that fails takes the others down (their
    # collectives see the connection close), and the job's status is the first failure's
    exits = {}

    def waiter(r, p):
        c = p.wait()
        exits[r] = (time.monotonic(), c)
    for r, p in enumerate(procs):
        threading.Thread(target=waiter, args=(r, p), daemon=True).start()
    deadline = time.monotonic() + timeout_s
    status = 0
    while True:
        done = dict(exits)
        bad = sorted((tc[0], r, tc[1]) for r, tc in done.items() if tc[1] != 0)
        if bad:
            _, r, c = bad[0]
            status = c if c > 0 else 128 - c
            sys.stderr.write(f"bench.py launcher: rank {r} exited with {c}; stopping the job\n")
            stop_all()
            break
        if len(done) == n:
            break
        if time.monotonic() > deadline:
            sys.stderr.write(f"bench.py launcher: job still running after {timeout_s:.0f} s; killing it\n")
            stop_all()
            status = 124
            break
        time.sleep(0.05)
    t.join(timeout=10)
    if status == 0:
        if len(lines) != 1:
            sys.stderr.write(f"bench.py launcher: rank 0 printed {len(lines)} JSON lines, expected 1\n")
            return 1
        sys.stdout.write(lines[0])
        sys.stdout.flush()
    return status


def roofline_from_stages(stages, calls, frames_per_call, W, H, kps_per_frame):
    """Dominant extractor kernel vs the HBM peak (+ its VALU issue rate when a PMC summary of the
    same kernel and shape is committed under profiles/)."""
    alg, _ = algorithmic_bytes(W, H, kps_per_frame)
    dom = max(stages, key=lambda k: stages[k][0])
    dom_ms, launches = stages[dom]
    avg_s = dom_ms / 1000.0 / max(launches, 1)
    frames_per_launch = frames_per_call * calls / max(launches, 1)
    dom_bytes = alg.get(dom, 0) * frames_per_launch
    achieved = dom_bytes / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic, valu = None, None
    tf = ROOT / "profiles" / "traffic_latest.json"
    if tf.exists():
        try:
            tj = json.loads(tf.read_text())
            if tj.get("kernel") == dom and tj.get("batch") == frames_per_launch and tj.get("width") == W:
                traffic = tj.get("bytes_per_launch")
                if tj.get("valu_instr_per_launch"):
                    vi = float(tj["valu_instr_per_launch"])
                    valu = {"achieved": round(vi / avg_s / 1e12, 4), "peak": round(VALU_PEAK_WAVE_INSTR / 1e12, 4),
                            "unit": "T wave64 VALU instr/s", "frac": round(vi / avg_s / VALU_PEAK_WAVE_INSTR, 4),
                            "valu_instr_per_launch": int(vi), "source": "SQ_INSTS_VALU, profiles/traffic_latest.json"}
        except Exception:
            traffic = None
    roof = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": int(dom_bytes),
        "frames_per_launch": frames_per_launch,
        "measured": "HIP events on the launch stream around the kernel's stage of one batch, isolated pass after "
                    "the timed region (1 batch in flight); k_fast_wave's stage is two dispatches (cell classes B then "
                    "A, DESIGN.md §2): rocprof's per-dispatch average is about half of avg_launch_ms",
        "avg_launch_ms": round(avg_s * 1000.0, 5),
    }
    if valu:
        roof["valu_ceiling"] = valu
    return roof


# ------------------------------------------------------------------------------------------
# orchestration: every leg in a child process of its own, with a deadline
# ------------------------------------------------------------------------------------------
LEG_ORDER = ("dry", "dryaux", "headline", "extract", "lba", "pose", "track", "localmap", "projection")
# seconds a leg may take (child start .. exit, CPU baseline included); the round-4 driver run of
# every leg took 21 s in one process, so each cap is several times the leg's normal length.  The
# whole job also has one deadline (--job-deadline) below the driver's 600 s limit: a leg starts
# only with the time that is left.
LEG_CAP_S = {"dry": 90, "dryaux": 90, "headline": 150, "extract": 90, "lba": 120, "pose": 60, "track": 120,
             "localmap": 60, "projection": 60}
T_START = time.monotonic()
T0_WALL = float(os.environ.get("SLAMHOT_BENCH_T0", time.time()))  # the rank's start (leg children inherit it)


def progress(msg, rank=0):
    """One flushed stderr line per orchestration event (leg start / phase / done / failure), so a
    stalled run says where it stopped; seconds since the rank process started."""
    sys.stderr.write(f"bench[r{rank} {time.time() - T0_WALL:7.1f}s] {msg}\n")
    sys.stderr.flush()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--legs", default="headline,extract,lba,pose,track,localmap,projection",
                    help="comma list of legs to run (headline = configs[2] extract+match)")
    # 256 stereo frames per step: the same steady-state rate as 128 (121-124k frames/s at 100 steps), but the
    # pipeline fill and drain of a short timed region weigh half as much (20 steps: 118.7-119.7k against
    # 112.2-116.0k with 128, profiles/r06j_pairs.txt)
    ap.add_argument("--pairs", type=int, default=256, help="headline: stereo frames per GPU per step")
    ap.add_argument("--inflight", type=int, default=4, help="batches in flight (handles / streams) per leg (3 / 4 / 5: headline 103.0k / 105.6k / 95.8k, profiles/r04h_inflight.txt)")
    ap.add_argument("--batch", type=int, default=256, help="extract leg: frames per GPU per step")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--unique", type=int, default=256, help="extract leg: distinct synthetic frames per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=384)
    ap.add_argument("--lba-windows", type=int, default=128, help="LBA windows per GPU per call")
    ap.add_argument("--lba-calls", type=int, default=6)
    # 6 solvers: 138.8-140.6k LM it/s after the extractor legs against 122.7-127.0k with 4 and
    # 129.3-137.1k with 3 (tools/ab/r05_lba_inflight.sh, profiles/r05_lba_plan.txt)
    ap.add_argument("--lba-inflight", type=int, default=6, help="LBA solver handles driven concurrently")
    ap.add_argument("--lba-stagger-ms", type=float, default=6.0,
                    help="LBA: solver t starts t x this many ms late, so the solvers' host planning phases "
                         "(~5 ms per 128-window call) fall between the others' device phases instead of "
                         "all at once (independent LocalMapping clients arrive out of phase)")
    ap.add_argument("--pose-frames", type=int, default=512, help="PoseOptimization frames per GPU per call")
    ap.add_argument("--localmap-frames", type=int, default=256, help="localmap leg: frames per call")
    ap.add_argument("--projection-frames", type=int, default=256,
                    help="projection leg: frames per batched SearchByProjection(F, LastFrame) call")
    ap.add_argument("--track-seqs", type=int, default=64, help="track leg: sequences per GPU (lock-step)")
    ap.add_argument("--track-frames", type=int, default=56, help="track leg: steps (frames per sequence)")
    ap.add_argument("--track-inflight", type=int, default=1,
                    help="track leg: tracker handles the sequences are split over (each its own stream)")
    ap.add_argument("--launch-timeout", type=float, default=570.0,
                    help="--gpus N > 1 started without WORLD_SIZE: seconds before the rank processes are killed "
                         "(below the driver's 600 s, so the launcher reports first)")
    ap.add_argument("--job-deadline", type=float, default=540.0,
                    help="seconds from a rank's start by which every leg must have ended (legs that would "
                         "start later are skipped and recorded as such)")
    ap.add_argument("--leg-timeout-scale", type=float, default=1.0, help="multiplies every leg's own cap (LEG_CAP_S)")
    ap.add_argument("--in-process", action="store_true",
                    help="run every leg in this process, one after another (N = 1 only): for profilers such as "
                         "rocprofv3, whose preloaded library initialises the GPU in this process, which must then "
                         "start no other program")
    ap.add_argument("--leg-child", default=None, help=argparse.SUPPRESS)      # internal: run one leg here
    ap.add_argument("--leg-deadline", type=float, default=0.0, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def leg_list(args):
    want = [x.strip() for x in args.legs.split(",") if x.strip()]
    bad = [x for x in want if x not in LEG_ORDER]
    if bad:
        raise SystemExit(f"bench.py: unknown leg(s) {bad}; known: {list(LEG_ORDER)}")
    skip = {"lba": args.lba_windows <= 0, "pose": args.pose_frames <= 0, "track": args.track_seqs <= 0,
            "localmap": args.localmap_frames <= 0, "projection": args.projection_frames <= 0}
    return [x for x in LEG_ORDER if x in want and not skip.get(x, False)]


def main():
    args = parse_args()
    if args.leg_child:
        sys.exit(child_main(args))
    legs = leg_list(args)
    if args.in_process:
        if args.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) != 1:
            raise SystemExit("bench.py: --in-process runs one rank (--gpus 1)")
        sys.exit(in_process_main(args, legs))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's `python bench.py --gpus N`: one child process per GPU, before any GPU call
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    sys.exit(rank_main(args, legs))


class LegCoord:
    """What the rank processes of a job share about its legs (nothing when world = 1): a gloo group
    on the host (no GPU call in these processes) for the per-leg rendezvous port and deadline, which
    rank 0 chooses, and the statuses gathered after each leg; and its store, where a rank whose leg
    failed says so at once, so the other ranks end their own leg child instead of waiting in a
    collective until the deadline."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank
        self.dist = self.store = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            sys.stdout.flush()
            saved = os.dup(1)  # gloo may print to fd 1, which carries only the JSON line
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist
            self.store = dist.distributed_c10d._get_default_store()

    def plan(self, leg, deadline):
        """(port, deadline) of this leg, the same on every rank (rank 0's)."""
        obj = [_free_port() if self.rank == 0 else 0, deadline]
        if self.dist:
            self.dist.broadcast_object_list(obj, src=0)
        return int(obj[0]), float(obj[1])

    def fail(self, leg, why):
        if self.store is not None:
            self.store.set(f"bench/legfail/{leg}", f"{self.rank}:{why}")

    def peer_failed(self, leg):
        if self.store is None:
            return None
        key = f"bench/legfail/{leg}"
        if self.store.check([key]):
            return self.store.get(key).decode()
        return None

    def gather(self, status):
        if not self.dist:
            return [status]
        out = [None] * self.world
        self.dist.all_gather_object(out, status)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def run_leg_child(args, leg, deadline, port, coord, scratch):
    """Run one leg in a fresh child process (`bench.py --leg-child LEG`); returns (status, payload).
    The child's stderr is ours; its stdout carries rank 0's one JSON line.  A child still running at
    `deadline` seconds is stopped (SIGTERM, then SIGKILL after 10 s) and the leg is a timeout."""
    import signal
    import subprocess
    import threading
    rank, world = coord.rank, coord.world
    env = dict(os.environ)
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the child's group has its own store (rank 0's child)
    env.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SLAMHOT_BENCH_SCRATCH=scratch,
               SLAMHOT_BENCH_T0=repr(T0_WALL))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # a library wait on device progress gives up well before the leg's deadline (SLAM_ETIMEDOUT)
    env.setdefault("SLAMHOT_WAIT_TIMEOUT_S", str(max(5, int(min(60.0, deadline / 3)))))
    argv = [a for a in sys.argv[1:]]
    cmd = [sys.executable, "-u", str(Path(__file__).resolve())] + argv + ["--leg-child", leg,
                                                                           "--leg-deadline", f"{deadline:.1f}"]
    t0 = time.monotonic()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=None)
    lines = []

    def relay():
        for raw in p.stdout:
            s = raw.decode(errors="replace")
            if s.lstrip().startswith("{"):
                lines.append(s)
            else:
                sys.stderr.write(s)
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    status = None
    while True:
        rc = p.poll()
        if rc is not None:
            status = {"status": "ok" if rc == 0 else "failed", "rc": rc}
            break
        if time.monotonic() - t0 > deadline:
            status = {"status": "timeout", "rc": 124}
            break
        peer = coord.peer_failed(leg)
        if peer is not None:
            status = {"status": "peer_failed", "rc": 1, "peer": peer}
            break
        time.sleep(0.1)
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    th.join(timeout=10)
    status.update(rank=rank, after_s=round(time.monotonic() - t0, 1))
    if status["status"] == "failed" and status["after_s"] >= deadline - 6.0:
        status.update(status="timeout", why="stopped itself at its deadline (stack dump on stderr)")
    if status["status"] != "ok":
        try:
            status["phase"] = (Path(scratch) / f"phase.{leg}").read_text()
        except OSError:
            status["phase"] = None
    if status["status"] in ("failed", "timeout"):
        coord.fail(leg, status["status"])
    payload = None
    if status["status"] == "ok" and rank == 0:
        if len(lines) != 1:
            status.update(status="failed", rc=1, why=f"rank 0 printed {len(lines)} JSON lines, expected 1")
        else:
            payload = json.loads(lines[0])["result"]
    return status, payload


def merge_leg(result, leg, payload):
    if leg == "dry":
        result.update(payload)
    elif leg == "headline":
        for k in ("value", "ms_per_step", "config", "roofline", "cpu_baseline"):
            if k in payload:
                result[k] = payload.pop(k)
        result["headline_detail"] = payload
    elif leg == "extract":
        result["extract"] = payload
        if result["value"] is None:  # headline off (profiling runs): the extract leg's line
            result.update(value=payload["value"], ms_per_step=payload["ms_per_step"], config=payload["config"],
                          roofline=payload["roofline"])
    else:
        result[leg] = payload


def rank_main(args, legs):
    """One rank of the job (the only one at N = 1): runs each leg in a child process of its own
    (fresh HIP context, its own deadline), merges the legs into the one JSON line (rank 0) and
    records a leg that failed or timed out as an error entry; the first leg of the list (the
    headline) is the line's value, so its failure fails the job, naming the leg and the rank."""
    import tempfile
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus and rank == 0:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; one rank per GPU, n_gpus = {world}\n")
    if rank == 0:
        progress(f"bench.py: legs {','.join(legs)}, {world} rank(s), steps {args.steps}, warmup {args.warmup}")
    # this process never touches the GPU; importing torch here pages the image in once (1-2 min on
    # a fresh box) outside every leg's deadline
    import torch  # noqa: F401
    coord = LegCoord(world, rank)
    result = {
        "metric": "ORB extract+match frames/s and LocalBA iters/s per GPU; ATE vs reference",
        "value": None, "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (rendered textured-room stereo sequences / procedural frames, slamhot/synth.py)",
    }
    legs_info = {}
    primary_fail = None
    with tempfile.TemporaryDirectory(prefix="slamhot_bench_") as scratch:
        for leg in legs:
            left = args.job_deadline - (time.monotonic() - T_START)
            want = min(LEG_CAP_S[leg] * args.leg_timeout_scale, left - 5.0)
            port, deadline = coord.plan(leg, want)
            if deadline < 5.0:
                if rank == 0:
                    progress(f"leg {leg} skipped: {left:.0f} s left of the job deadline")
                result[leg] = {"error": "skipped", "why": f"job deadline ({args.job_deadline:.0f} s) reached"}
                if leg == legs[0]:
                    primary_fail = (leg, {"status": "skipped", "rank": rank, "rc": 124})
                    break
                continue
            if rank == 0:
                progress(f"leg {leg} start (deadline {deadline:.0f} s)")
            status, payload = run_leg_child(args, leg, deadline, port, coord, scratch)
            sts = coord.gather(status)
            bad = [s_ for s_ in sts if s_["status"] != "ok"]
            legs_info[leg] = {"s": status["after_s"], "status": "ok" if not bad else "error"}
            if not bad:
                if rank == 0:
                    progress(f"leg {leg} done in {status['after_s']:.1f} s")
                    merge_leg(result, leg, payload)
                continue
            # the rank that failed first (a peer that stopped because of it is not the cause)
            # and of the ranks that timed out together, one stuck in its own work, not one waiting for
            # it in a collective
            def waiting(s_):
                return (s_.get("phase") or "").startswith("collective")
            cause = sorted(bad, key=lambda s_: (s_["status"] == "peer_failed", waiting(s_), s_["after_s"]))[0]
            err = {"error": cause["status"], "rank": cause["rank"], "rc": cause["rc"], "after_s": cause["after_s"],
                   "deadline_s": round(deadline, 1), "phase": cause.get("phase"),
                   "ranks": {str(s_["rank"]): f"{s_['status']} ({s_.get('phase')})" for s_ in bad}}
            if "why" in cause:
                err["why"] = cause["why"]
            if rank == 0:
                progress(f"leg {leg} FAILED: {cause['status']} on rank {cause['rank']} (rc {cause['rc']}) after "
                         f"{cause['after_s']:.1f} s, in phase: {cause.get('phase')}")
            if leg == legs[0]:
                primary_fail = (leg, cause)
                break
            result[leg] = err
    coord.close()
    if primary_fail:
        leg, cause = primary_fail
        sys.stderr.write(f"bench.py: leg {leg} {cause['status']} on rank {cause['rank']} (phase: {cause.get('phase')}); "
                         f"no line printed\n")
        rc = int(cause.get("rc") or 1)
        return rc if 0 < rc < 256 else 1
    if rank == 0:
        result["legs"] = {"isolation": "one child process per leg (fresh HIP context), per-leg deadline",
                          "wall_s": legs_info, "job_wall_s": round(time.monotonic() - T_START, 1)}
        add_full_socket(result)
        print(json.dumps(result), flush=True)
    return 0


def in_process_main(args, legs):
    """--in-process: every leg in this process, in order (no child processes, no per-leg deadline),
    merged into the same JSON line as rank_main's."""
    result = {
        "metric": "ORB extract+match frames/s and LocalBA iters/s per GPU; ATE vs reference",
        "value": None, "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (rendered textured-room stereo sequences / procedural frames, slamhot/synth.py)",
    }
    wall = {}
    import tempfile
    with tempfile.TemporaryDirectory(prefix="slamhot_bench_") as scratch:
        os.environ["SLAMHOT_BENCH_SCRATCH"] = scratch
        for leg in legs:
            t0 = time.monotonic()
            progress(f"leg {leg} start (in process)")
            payload = run_leg(args, leg)
            wall[leg] = {"s": round(time.monotonic() - t0, 1), "status": "ok"}
            progress(f"leg {leg} done in {wall[leg]['s']:.1f} s")
            merge_leg(result, leg, payload)
    result["legs"] = {"isolation": "in process (--in-process): every leg in one process, in order", "wall_s": wall,
                      "job_wall_s": round(time.monotonic() - T_START, 1)}
    add_full_socket(result)
    print(json.dumps(result), flush=True)
    return 0


def run_leg(args, leg, world=1, rank=0, local_rank=0):
    """One leg in this process (N = 1): the device, the context, the leg function; its result dict."""
    import torch
    dry = leg in ("dry", "dryaux")
    gpu = local_rank
    if dry:
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", gpu)
        torch.cuda.set_device(device)
    PHASE.update(rank=rank, leg=leg, file=None)
    ctx = dict(args=args, rank=rank, world=world, local_rank=gpu, dist=None, device=device, leg=leg,
               cpu=(rank == 0 and world == 1 and not args.no_cpu_baseline))
    fn = {"dry": dry_leg, "dryaux": dry_leg, "headline": headline_leg, "extract": extract_leg, "lba": lba_leg,
          "pose": pose_leg, "track": track_leg, "localmap": localmap_leg, "projection": projection_leg}[leg]
    return fn(ctx)


def child_main(args):
    """One leg in this process (started by rank_main): the rank's process group on the leg's own
    port, the leg, rank 0 prints {"leg", "result"}.  A Python stack dump of every thread and exit
    just before the parent's deadline, so a stall leaves its place on stderr."""
    import faulthandler
    leg = args.leg_child
    PHASE.update(rank=int(os.environ.get("RANK", "0")), leg=leg,
                 file=os.path.join(os.environ["SLAMHOT_BENCH_SCRATCH"], f"phase.{leg}")
                 if os.environ.get("SLAMHOT_BENCH_SCRATCH") else None)
    phase("compute: starting (import torch, process group)")
    if args.leg_deadline > 0:
        faulthandler.dump_traceback_later(max(1.0, args.leg_deadline - 5.0), exit=True)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # dry legs: the GPU-free rehearsal of the launcher and the collectives (host only, gloo)
    dry = leg in ("dry", "dryaux")
    # one GPU per rank; SLAMHOT_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # cuda:(local_rank mod device_count), collectives on host copies) — the driver's runs use nccl
    backend = "gloo" if dry else os.environ.get("SLAMHOT_BENCH_BACKEND", "nccl")
    ndev = max(torch.cuda.device_count(), 1)
    gpu = local_rank % ndev if backend == "gloo" else local_rank
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dry:
            torch.cuda.set_device(gpu)
        # the process-group libraries may print to fd 1 (gloo's "[Gloo] Rank 0 is connected ...");
        # stdout carries only the JSON line, so fd 1 points at stderr while they initialise
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            else:
                dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if dry:
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", gpu)
        torch.cuda.set_device(device)
    phase("compute: leg setup")
    ctx = dict(args=args, rank=rank, world=world, local_rank=gpu, dist=dist, device=device, leg=leg,
               cpu=(rank == 0 and world == 1 and not args.no_cpu_baseline))
    fn = {"dry": dry_leg, "dryaux": dry_leg, "headline": headline_leg, "extract": extract_leg, "lba": lba_leg,
          "pose": pose_leg, "track": track_leg, "localmap": localmap_leg, "projection": projection_leg}[leg]
    out = fn(ctx)
    phase("compute: leg done")
    if rank == 0:
        print(json.dumps({"leg": leg, "result": out}), flush=True)
    if dist:
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()
    return 0


def dry_leg(ctx):
    """GPU-free rehearsal of the multi-rank plumbing (`--legs dry`, gloo): every rank renders its
    shard of synthetic 320x240 frames (global frame index = rank x frames-per-rank + i) and hashes
    them, K steps inside the same barrier-bracketed timed region, then the same max-time / unit-sum
    reductions and digest gather as the real legs.  Nothing is measured here; it is what
    `tests/test_bench_launch.py` runs through the `--gpus N` launcher."""
    from slamhot import dist as sdist
    from slamhot import synth
    args, dist, device, rank = ctx["args"], ctx["dist"], ctx["device"], ctx["rank"]
    n = max(1, args.pairs // 32)
    idx = [rank * n + i for i in range(n)]
    state = {}
    # the failure paths under test (tests/test_bench_launch.py): SLAMHOT_DRY_FAIL_RANK=r fails rank r
    # of leg "dry"; SLAMHOT_DRY_HANG=leg:r hangs rank r of that leg (a host stall: no progress, no exit)
    if ctx["leg"] == "dry" and os.environ.get("SLAMHOT_DRY_FAIL_RANK") == str(rank):
        sys.stderr.write(f"dry leg: rank {rank} failing on request\n")
        sys.exit(3)
    if os.environ.get("SLAMHOT_DRY_HANG") == f"{ctx['leg']}:{rank}":
        sys.stderr.write(f"{ctx['leg']} leg: rank {rank} hanging on request\n")
        while True:
            time.sleep(1)

    def step(_):
        state["dig"] = sdist.combine(sdist.unit_hash(g, synth.frame(g, 320, 240)) for g in idx)
    step(0)
    elapsed = timed_region(dist, device, step, args.steps)
    el, units = sdist.reduce_run(dist, device, elapsed, float(n * args.steps))
    digs = sdist.gather_digests(dist, device, ctx["world"], n, state["dig"])
    return {"value": round(units / el, 2), "ms_per_step": round(el / args.steps * 1e3, 4), "dtype": "u8",
            "data": "synthetic frames (slamhot/synth.py), host only", "scaling": "weak",
            "config": {"workload": "dry: launcher / collective rehearsal, no GPU work", "frames_per_rank": n,
                       "parallelism": f"frame-sharded x{ctx['world']}"},
            "rank_digests": [d for _, d in digs],
            "digest": {"units_per_rank": n, "job": sdist.combine(d for _, d in digs)}}


# ------------------------------------------------------------------------------------------
# headline: configs[2] stereo extract + match
# ------------------------------------------------------------------------------------------
SEQ_LEN = 8      # consecutive frames per synthetic sequence chunk (frame j's KF is frame j - 1)
SEQ_RENDER = 64  # frames per rendered sequence (one textured room per sequence)


def euroc_maps():
    from slamhot import euroc
    calib = {k: np.array(v) if isinstance(v, list) else v
             for k, v in json.loads((ROOT / "tests" / "golden" / "euroc_stereo_calib.json").read_text()).items()}
    return [euroc.init_undistort_rectify_map(calib[f"{sd}.K"], calib[f"{sd}.D"], calib[f"{sd}.R"], calib[f"{sd}.P"],
                                             (752, 480)) for sd in ("LEFT", "RIGHT")]


def stereo_chunks(rank, maps, nframes):
    """nframes distinct raw stereo frames for this rank (raw L, raw R): rendered sequences of up
    to SEQ_RENDER frames, cut into chunks of SEQ_LEN consecutive frames; rendered and unrectified
    on the host threads before the timed region."""
    from concurrent.futures import ThreadPoolExecutor

    from slamhot import synth
    th = host_cores()
    Ls, Rs = [], []
    nseq = (nframes + SEQ_RENDER - 1) // SEQ_RENDER
    for s in range(nseq):
        n = min(SEQ_RENDER, nframes - s * SEQ_RENDER)
        # sequence seeds follow the global frame order (rank r holds global sequences r * nseq + s), so
        # one process rendering world x nframes frames (a multiple of SEQ_RENDER) sees the same frames
        L, R, _ = synth.stereo_sequence(101 + rank * nseq + s, n, threads=th)
        Ls += list(L)
        Rs += list(R)
    with ThreadPoolExecutor(th) as pool:
        rl = list(pool.map(lambda im: synth.unrectify(im, *maps[0]), Ls))
        rr = list(pool.map(lambda im: synth.unrectify(im, *maps[1]), Rs))
    return np.stack(rl), np.stack(rr)


def load_chunks(ctx, maps, nframes):
    """stereo_chunks(rank, maps, nframes), rendered once per rank: the first leg child that needs them
    renders and leaves them in the rank's scratch directory (SLAMHOT_BENCH_SCRATCH), later ones load
    them."""
    d = os.environ.get("SLAMHOT_BENCH_SCRATCH")
    f = Path(d) / f"chunks_{nframes}.npz" if d else None
    if f is not None and f.exists():
        z = np.load(f)
        return z["l"], z["r"]
    phase(f"compute: rendering {nframes} stereo frames")
    raw_l, raw_r = stereo_chunks(ctx["rank"], maps, nframes)
    if f is not None:
        tmp = f.with_suffix(".tmp.npz")
        np.savez(tmp, l=raw_l, r=raw_r)
        tmp.rename(f)
    return raw_l, raw_r


def kf_of(i):
    """Reference keyframe of batch frame i: the previous frame of its sequence chunk (the chunk's
    first frame takes its last one)."""
    return i - 1 if i % SEQ_LEN else i + SEQ_LEN - 1


def headline_leg(ctx):
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import euroc, synth
    args, device, dist, lr = ctx["args"], ctx["device"], ctx["dist"], ctx["local_rank"]
    W, H, NF = 752, 480, 1200
    P = max(SEQ_LEN, args.pairs // SEQ_LEN * SEQ_LEN)
    maps = euroc_maps()
    raw_l, raw_r = load_chunks(ctx, maps, P)
    nu = len(raw_l)  # every frame of the batch is distinct
    il, ir = raw_l, raw_r
    pairs = [(kf_of(i), i) for i in range(P)]
    mbf = synth.EUROC_STEREO["bf"]
    mb = mbf / synth.EUROC_STEREO["fx"]
    voc_arrays = sdist.broadcast_arrays(dist, device, synth.vocab(10, 6, 0) if ctx["rank"] == 0 else None)
    voc = slamhot.Vocabulary(*voc_arrays, k=10, L=6, device=lr)
    d_raw_l, d_raw_r = torch.from_numpy(il).to(device), torch.from_numpy(ir).to(device)
    NS = max(1, args.inflight)

    class Slot:
        pass

    slots = []
    for _ in range(NS):
        s = Slot()
        s.rect = [euroc.Rectifier(*mp, device=lr) for mp in maps]
        s.exl = slamhot.ORBextractor(nfeatures=NF, device=lr, max_size=(W, H), max_batch=P)
        s.exr = slamhot.ORBextractor(nfeatures=NF, device=lr, max_size=(W, H), max_batch=P)
        s.sm = slamhot.StereoMatcher(device=lr)
        s.m = slamhot.ORBmatcher(0.7, True, device=lr)
        cap = s.exl.cap
        s.img = [torch.empty_like(d_raw_l), torch.empty_like(d_raw_r)]
        s.out = [(torch.zeros((P, cap, 28), dtype=torch.uint8, device=device),
                  torch.zeros((P, cap, 32), dtype=torch.uint8, device=device),
                  torch.zeros(P, dtype=torch.int32, device=device), torch.zeros(P, dtype=torch.int32, device=device))
                 for _ in range(2)]
        s.ur = torch.empty((P, cap), dtype=torch.float32, device=device)
        s.dep = torch.empty((P, cap), dtype=torch.float32, device=device)
        s.a2b = torch.zeros((P, cap), dtype=torch.int32, device=device)
        s.b2a = torch.zeros((P, cap), dtype=torch.int32, device=device)
        s.nm = torch.zeros(P, dtype=torch.int32, device=device)
        s.stream = torch.cuda.Stream(device)
        slots.append(s)
    cap = slots[0].exl.cap
    ev = {"rectify": [], "extract": [], "stereo": [], "bow": []}

    def step(i, timed=False):
        s = slots[i % NS]
        st = s.stream.cuda_stream
        marks = []

        def mark():
            if timed:
                e = torch.cuda.Event(enable_timing=True)
                e.record(s.stream)
                marks.append(e)
        mark()
        for rc, raw, out in ((s.rect[0], d_raw_l, s.img[0]), (s.rect[1], d_raw_r, s.img[1])):
            rc.rectify_batch_device(P, raw.data_ptr(), W, W * H, out.data_ptr(), W, W * H, stream=st)
        mark()
        for ex, img, (k, d, n, m) in ((s.exl, s.img[0], s.out[0]), (s.exr, s.img[1], s.out[1])):
            ex.extract_batch_device(img.data_ptr(), P, W, H, k.data_ptr(), d.data_ptr(), cap, n.data_ptr(),
                                    m.data_ptr(), stream=st)
        mark()
        (kl, dl, nl, _), (kr, dr, nr, _) = s.out
        s.sm.match_batch_device(s.exl, s.exr, P, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(),
                                dr.data_ptr(), nr.data_ptr(), cap, mbf, mb, s.ur.data_ptr(), s.dep.data_ptr(),
                                stream=st)
        mark()
        s.m.bow_match_batch_device(voc, P, kl.data_ptr(), dl.data_ptr(), cap, nl.data_ptr(), pairs, s.a2b.data_ptr(),
                                   s.b2a.data_ptr(), s.nm.data_ptr(), stream=st)
        mark()
        if timed:
            for k_, a, b in zip(("rectify", "extract", "stereo", "bow"), marks[:-1], marks[1:]):
                ev[k_].append((a, b))

    phase("compute: warm-up steps")
    for i in range(max(args.warmup, 1)):
        step(i)
    elapsed = timed_region(dist, device, step, args.steps)
    # isolated pass: one batch in flight, per-stage HIP events (extractor stages on the left
    # handle; `rocprofv3 ... bench.py --legs headline --inflight 1` reproduces the kernel times)
    s0 = slots[0]
    s0.exl.stage_stats(reset=True)
    s0.exl.set_profiling(True)
    nprof = max(10, min(args.steps, 50))
    for _ in range(nprof):
        step(0, timed=True)
    torch.cuda.synchronize(device)
    s0.exl.set_profiling(False)
    stages = s0.exl.stage_stats(reset=True)
    stage_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}

    nl_h = s0.out[0][2].cpu().numpy()
    nm_h = s0.nm.cpu().numpy()
    ur_h = s0.ur.cpu().numpy()
    skipped = s0.m.bow_match_batch_status(s0.stream.cuda_stream)
    kps_per_frame = float(nl_h.mean())
    # parity digest over this rank's frames (all distinct): per frame a hash of its keypoints,
    # descriptors, stereo uR and both match directions, mixed with the frame's global index
    # (rank * nu + i), summed (slamhot.dist.unit_hash / combine)
    kk, dd = s0.out[0][0].cpu().numpy(), s0.out[0][1].cpu().numpy()
    a2b_h, b2a_h = s0.a2b.cpu().numpy(), s0.b2a.cpu().numpy()
    nuniq = min(nu, P)
    dig = sdist.combine(sdist.unit_hash(ctx["rank"] * nu + i, kk[i, :nl_h[i]], dd[i, :nl_h[i]], ur_h[i, :nl_h[i]],
                                        a2b_h[i, :nl_h[kf_of(i)]], b2a_h[i, :nl_h[i]], nm_h[i:i + 1])
                        for i in range(nuniq))
    el, frames_all = sdist.reduce_run(dist, device, elapsed, float(P * args.steps))
    digs = sdist.gather_digests(dist, device, ctx["world"], int(nm_h[:nuniq].sum()), dig)
    out = {
        "value": round(frames_all / el, 2),
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "config": {
            "workload": f"configs[2] shape: stereo {W}x{H} raw pairs (EuRoC calibration) -> remap x2 -> "
                        f"ORBextractor x2 ({NF} feat, 8 levels, 1.2, 20/7) -> ComputeStereoMatches -> ComputeBoW "
                        f"-> SearchByBoW(previous frame as KF, F) (nnratio 0.7, checkOri); synthetic k=10 L=6 "
                        f"vocabulary",
            "stereo_frames_per_gpu_per_step": P, "distinct_frames_per_gpu": nu,
            "parallelism": f"frame-sharded x{ctx['world']}",
            "batches_in_flight": NS, "keypoints_per_frame": round(kps_per_frame, 1),
        },
        "roofline": roofline_from_stages(stages, nprof, P, W, H, kps_per_frame),
        "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
        "extractor_stage_ms_per_launch": {k: round(v[0] / max(v[1], 1), 5) for k, v in stages.items()},
        "matches_per_pair": round(float(nm_h.mean()), 1),
        "stereo_matches_per_frame": round(float(np.mean([(ur_h[f, :nl_h[f]] >= 0).sum() for f in range(P)])), 1),
        "bow_general_pairs": skipped,
        "rank_digests": [d for _, d in digs],
        "digest": {"units_per_rank": nuniq, "job": sdist.combine(d for _, d in digs),
                   "what": "rank_digests: per rank, reproducible run to run; job: their sum, equal to one process's "
                           "digest over world x frames since frame content follows the global frame index; each term "
                           "= sum over frames of BLAKE2b(global frame index, keypoints, descriptors, "
                           "mvuRight, SearchByBoW a2b / b2a, nmatches) mod 2^62"},
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        out["cpu_baseline"] = headline_cpu(raw_l, raw_r, maps, voc_arrays, mbf, mb, NF)
    for s in slots:
        for rc in s.rect:
            rc.close()
        s.exl.close()
        s.exr.close()
        s.sm.close()
        s.m.close()
    voc.close()
    return out


def headline_cpu(raw_l, raw_r, maps, voc_arrays, mbf, mb, NF):
    """The oracle chain (restated reference CPU path) on the host cores: one sequence chunk per
    thread, frames in order (KF = previous frame), each frame remap x2 + extract x2 +
    ComputeStereoMatches + vocabulary transform + FeatureVector + SearchByBoW."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_bind as ob
    from slamhot import synth
    par, leaf, dn, wn = voc_arrays
    p = ob.params(nfeatures=NF)
    sc, isc, _, _, _ = ob.levels(p)

    nch = len(raw_l) // SEQ_LEN

    def chunk(c):
        prev = None
        base = (c % nch) * SEQ_LEN
        for j in range(SEQ_LEN):
            l_img = ob.remap_linear(raw_l[base + j], *maps[0])
            r_img = ob.remap_linear(raw_r[base + j], *maps[1])
            # the stereo matcher reads the pyramids the two extractions built (mvImagePyramid,
            # Frame.cc:801, 891), as the reference does
            kl, dl, _, pl = ob.extract_with_pyramid(l_img, p)
            kr, dr, _, pr = ob.extract_with_pyramid(r_img, p)
            ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, mbf, mb)
            _, wt, nid = ob.vocab_transform(par, leaf, dn, wn, 6, dl, 4)
            side = (dl, kl["angle"], None) + synth.feature_vector(nid, wt)
            if prev is not None:
                ob.search_by_bow(prev, side, 0.7, True, False)
            prev = side
        return SEQ_LEN

    cores = host_cores()
    nchunks = 2 * cores
    chunk(0)  # warm-up
    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as pool:
        frames = sum(pool.map(chunk, range(nchunks)))
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 2), "unit": "frames/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{nchunks} sequence chunks x {SEQ_LEN} stereo frames (the headline's distinct frames), one "
                      f"chunk per thread on {cores} threads: oracle remap x2 + extract x2 (each leaving its "
                      f"mvImagePyramid) + stereo_oracle on those pyramids + vocabulary transform + FeatureVector + "
                      f"SearchByBoW; oracle -O3"}


# ------------------------------------------------------------------------------------------
# extract: configs[1] ORBextractor-only + the drop-in host path
# ------------------------------------------------------------------------------------------
def extract_leg(ctx):
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    args, device, dist, rank = ctx["args"], ctx["device"], ctx["dist"], ctx["rank"]
    W, H, B = args.width, args.height, args.batch
    nuniq = min(args.unique, B)
    base = synth.frames(range(rank * 100000, rank * 100000 + nuniq), W, H)
    frames_np = np.concatenate([base] * ((B + nuniq - 1) // nuniq))[:B]
    d_imgs = torch.from_numpy(frames_np).to(device)
    # `inflight` batches in flight: each slot has its own extractor handle (scratch), output
    # buffers and stream; every frame of every step is still processed inside the timed region
    NS = max(1, args.inflight)
    exs = [slamhot.ORBextractor(nfeatures=args.nfeatures, device=ctx["local_rank"], max_size=(W, H), max_batch=B)
           for _ in range(NS)]
    ex = exs[0]
    cap = ex.cap
    outs = [(torch.zeros((B, cap, 28), dtype=torch.uint8, device=device),
             torch.zeros((B, cap, 32), dtype=torch.uint8, device=device),
             torch.zeros(B, dtype=torch.int32, device=device), torch.zeros(B, dtype=torch.int32, device=device))
            for _ in range(NS)]
    streams = [torch.cuda.Stream(device) for _ in range(NS)]

    def step(i):
        k_, d_, n_, m_ = outs[i % NS]
        exs[i % NS].extract_batch_device(d_imgs.data_ptr(), B, W, H, k_.data_ptr(), d_.data_ptr(), cap, n_.data_ptr(),
                                         m_.data_ptr(), lap=(0, 0), stream=streams[i % NS].cuda_stream)

    for i in range(args.warmup):
        step(i)
    elapsed = timed_region(dist, device, step, args.steps)
    ex.stage_stats(reset=True)
    ex.set_profiling(True)
    for _ in range(args.steps):
        step(0)
    torch.cuda.synchronize(device)
    ex.set_profiling(False)
    stages = ex.stage_stats(reset=True)
    n_host = outs[0][2].cpu().numpy()
    kps_per_frame = float(n_host.mean())
    el, frames_all = sdist.reduce_run(dist, device, elapsed, float(B * args.steps))
    _, pipe_bytes = algorithmic_bytes(W, H, kps_per_frame)
    ms_per_step = el / args.steps * 1000.0

    # the drop-in path as Tracking calls it: host image in, host keypoints / descriptors out
    # (slamhot_extract_batch / slamhot_extract: H2D + extraction + D2H, synchronous)
    hb = 32
    ex.extract_batch(frames_np[:hb])
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        ex.extract_batch(frames_np[:hb])
    host_batch_fps = hb * reps / (time.perf_counter() - t0)
    lat = []
    for i in range(60):
        t1 = time.perf_counter()
        ex(frames_np[i % nuniq])
        lat.append(time.perf_counter() - t1)
    lat = np.array(lat[10:]) * 1e3
    out = {
        "metric": "ORBextractor frames/s",
        "value": round(frames_all / el, 2),
        "unit": "frames/s",
        "ms_per_step": round(ms_per_step, 4),
        "config": {"workload": f"ORBextractor-only, synthetic {W}x{H} 8-level pyramid, {args.nfeatures} feat/frame "
                               f"(BASELINE.json configs[1])",
                   "frames_per_gpu_per_step": B, "nfeatures": args.nfeatures, "levels": 8, "scale_factor": 1.2,
                   "fast_thresholds": [20, 7], "parallelism": f"frame-sharded x{ctx['world']}",
                   "batches_in_flight": NS, "keypoints_per_frame": round(kps_per_frame, 1)},
        "roofline": roofline_from_stages(stages, args.steps, B, W, H, kps_per_frame),
        "stages_ms_per_step": {k: round(v[0] / max(args.steps, 1), 5) for k, v in stages.items()},
        "pipeline_roofline": {"bytes_per_frame": int(pipe_bytes),
                              "achieved_GBps": round(pipe_bytes * B / (ms_per_step / 1000.0) / 1e9, 2)},
        "host_path": {
            "batch_frames_per_s": round(host_batch_fps, 1),
            "batch": hb,
            "single_frame_latency_ms": {"median": round(float(np.median(lat)), 3),
                                        "p90": round(float(np.percentile(lat, 90)), 3)},
            "note": "slamhot_extract_batch / slamhot_extract with host buffers (H2D image + extraction + D2H "
                    "keypoints and descriptors, synchronous) — the call Frame.cc:119-122 makes",
        },
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        out["cpu_baseline"] = extract_cpu(args, W, H)
    for e in exs:
        e.close()
    return out


def extract_cpu(args, W, H):
    """The oracle (restated reference CPU path, oracle/orb_oracle.cpp) on the host cores:
    one frame per std::thread at a time, as Frame.cc:119-122 runs extraction."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_bind as ob
    from slamhot import synth
    cores = host_cores()
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
    return {"value": round(len(imgs) / dt, 2), "unit": "frames/s", "cores": cores, "kind": "port", "cpu": cpu_model(),
            "sample": f"{len(imgs)} synthetic {W}x{H} frames, {args.nfeatures} feat, {cores} threads "
                      f"(one frame per thread); oracle/orb_oracle.cpp -O3",
            "per_core_frames_per_s": round(single / dt1, 2)}


# ------------------------------------------------------------------------------------------
# pose: Optimizer::PoseOptimization
# ------------------------------------------------------------------------------------------
def pose_leg(ctx):
    """Optimizer::PoseOptimization frames/s: batches of synthetic frames (1000 keypoints, 80%
    with MapPoints, 10% outliers, EuRoC intrinsics), one workgroup per frame."""
    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    args, device, dist = ctx["args"], ctx["device"], ctx["dist"]
    nf = args.pose_frames
    pool = [synth.pose_frame(s) for s in sdist.shard(16 * ctx["world"], ctx["rank"], ctx["world"])]
    frames = [pool[i % len(pool)] for i in range(nf)]
    S = slamhot.PoseOptimizer(device=ctx["local_rank"])
    S.solve(frames[:8])
    calls = 10
    # the C call on frames marshalled before the timed region (a C++ Tracking caller holds them
    # as structs already); results converted after it
    run = S.prepare(frames)
    warm_for(run, 0.3)
    elapsed = timed_region(dist, device, lambda i: run(), calls)
    res = [run.results()]
    el, total = sdist.reduce_run(dist, device, elapsed, float(nf * calls))
    out = {
        "metric": "Optimizer::PoseOptimization frames/s",
        "measured": "the C call slamhot_pose_optimization on frames marshalled before the timed region (host "
                    "buffers in and out: staging, PCIe, kernels, read-back)",
        "value": round(total / el, 1),
        "unit": "frames/s",
        "dtype": "f64",
        "config": {"workload": "synthetic frames, 1000 keypoints, ~800 MapPoint observations, 10% outliers, "
                               "4 x optimize(10)", "frames_per_gpu_per_call": nf,
                   "parallelism": f"frame-sharded x{ctx['world']}"},
        "ms_per_call": round(el / calls * 1e3, 3),
        "mean_inliers": round(float(np.mean([r["n_inliers"] for r in res[-1]])), 1),
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        cores = host_cores()
        work = [pool[i % len(pool)] for i in range(64 * cores)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            list(ex.map(ob.pose_optimization, work))
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(work) / dt, 2), "unit": "frames/s", "cores": cores, "kind": "port",
                               "cpu": cpu_model(),
                               "sample": f"{len(work)} frames on {cores} threads (one frame per task); "
                                         f"oracle/pose_oracle.cpp -O3"}
    S.close()
    return out


# ------------------------------------------------------------------------------------------
# localmap: batched Tracking::SearchLocalPoints (isInFrustum + SearchByProjection)
# ------------------------------------------------------------------------------------------
def warm_for(run, seconds):
    """Untimed calls of a secondary leg for at least `seconds` (at least one): each leg starts in a
    fresh process after an idle gap, and a few calls of a few ms would otherwise be timed while
    the GPU and host clocks still ramp up."""
    t0 = time.perf_counter()
    run()
    while time.perf_counter() - t0 < seconds:
        run()


def call_split(m, wall_ms):
    """Where a batched host-buffer matcher call's time goes (last timed call, events on its
    stream): its kernels, its device-side span (first upload .. read-back done), and the share of
    the host wall clock per call that the kernels take."""
    k, span = m.last_batch_stats()
    return {"kernel_ms": round(k, 4), "device_span_ms": round(span, 4), "wall_ms": round(wall_ms, 4),
            "kernel_share": round(k / wall_ms, 4) if wall_ms > 0 else None,
            "what": "kernel_ms: grid + (isInFrustum) + SearchByProjection kernels; device_span_ms: first H2D "
                    "chunk queued .. read-back done (staging runs on host threads and overlaps the chunked uploads)"}


def localmap_leg(ctx):
    """Tracking::SearchLocalPoints frames/s through slamhot_search_local_points_batch: P frames per
    call (1200 features, ~1200 local MapPoints each: back-projected features plus points behind,
    outside, too near / far, at grazing angles, already seen or bad), host buffers in and out —
    the drop-in call, PCIe included."""
    import torch

    import slamhot
    from slamhot import dist as sdist
    sys.path.insert(0, str(ROOT / "tests"))
    import scenes
    args, device, dist = ctx["args"], ctx["device"], ctx["dist"]
    P = args.localmap_frames
    uniq = []
    for seed in sdist.shard(16 * ctx["world"], ctx["rank"], ctx["world"]):
        S = scenes.scene(1000 + seed)
        fv, keep = scenes.frame_view(S)
        geom, desc = scenes.local_map_geom(S)
        uniq.append((fv, keep, geom, desc))
    views = [uniq[i % len(uniq)][0] for i in range(P)]
    geoms = [uniq[i % len(uniq)][2] for i in range(P)]
    descs = [uniq[i % len(uniq)][3] for i in range(P)]
    m = slamhot.ORBmatcher(0.8, device=ctx["local_rank"])
    # arguments marshalled once, as a C++ Tracking thread holds them: the timed call is the C call
    run = m.prepare_batch("local", views, (geoms, descs))
    warm_for(run, 0.3)
    calls = 10
    res = []
    elapsed = timed_region(dist, device, lambda i: (run(), res.append(run.results())), calls)
    el, total = sdist.reduce_run(dist, device, elapsed, float(P * calls))
    out = {
        "metric": "Tracking::SearchLocalPoints frames/s (batched, host buffers)",
        "measured": "the C call slamhot_search_local_points_batch on arguments marshalled before the timed region "
                    "(host buffers in and out: staging, PCIe, kernels, read-back)",
        "value": round(total / el, 1),
        "unit": "frames/s",
        "dtype": "f32 / u8",
        "config": {"workload": f"{P} frames per call, 1200 features and ~{int(np.mean([len(g) for g in geoms]))} local "
                               f"MapPoints each, th 1, nnratio 0.8 (slamhot_search_local_points_batch)",
                   "parallelism": f"frame-sharded x{ctx['world']}"},
        "ms_per_call": round(el / calls * 1e3, 3),
        "mean_matches": round(float(np.mean([r[0] for r in res[-1]])), 1),
        "call_split": call_split(m, el / calls * 1e3),
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        import oracle_bind as ob
        cores = host_cores()

        def one(i):
            fv, _, g, d = uniq[i % len(uniq)]
            _, tr = ob.is_in_frustum(fv, g, 0.5)
            ob.search_by_projection_local(fv, tr, d, 0.8, 1.0, False, 50.0)
            return 1

        work = list(range(64 * cores))
        one(0)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as pool:
            n = sum(pool.map(one, work))
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / dt, 1), "unit": "frames/s", "cores": cores, "kind": "port",
                               "cpu": cpu_model(),
                               "sample": f"{n} frames on {cores} threads: oracle isInFrustum + SearchByProjection"}
    m.close()
    return out


def projection_leg(ctx):
    """TrackWithMotionModel's matcher, SearchByProjection(Frame&, const Frame& LastFrame, th = 7,
    bMono = false) with ORBmatcher(0.9, true) (Tracking.cc:2683-2716, ORBmatcher.cc:2173-2389),
    frames/s through slamhot_search_by_projection_last_batch: P (current frame, last frame) pairs
    per call, 1200 features and ~1000 last-frame MapPoints each, host buffers in and out (the
    drop-in call, PCIe included); plus the KeyFrame variant (Relocalization, th 10, ORBdist 100)."""
    import slamhot
    from slamhot import dist as sdist
    sys.path.insert(0, str(ROOT / "tests"))
    import scenes
    args, device, dist = ctx["args"], ctx["device"], ctx["dist"]
    P = args.projection_frames
    uniq = []
    for seed in sdist.shard(16 * ctx["world"], ctx["rank"], ctx["world"]):
        S = scenes.scene(2000 + seed)
        fv, keep = scenes.frame_view(S)
        lf, lkeep = scenes.last_frame(S, mono=False, motion=0.05)
        kf, kkeep = scenes.kf_points(S)
        uniq.append((fv, lf, kf, (S, keep, lkeep, kkeep)))
    views = [uniq[i % len(uniq)][0] for i in range(P)]
    lfs = [uniq[i % len(uniq)][1] for i in range(P)]
    kfs = [uniq[i % len(uniq)][2] for i in range(P)]
    m = slamhot.ORBmatcher(0.9, True, device=ctx["local_rank"])
    # arguments marshalled once, as a C++ Tracking thread holds them: the timed call is the C call
    run = m.prepare_batch("last", views, lfs, 7.0, False)
    warm_for(run, 0.3)
    calls = 10
    res = []
    elapsed = timed_region(dist, device, lambda i: (run(), res.append(run.results())), calls)
    el, total = sdist.reduce_run(dist, device, elapsed, float(P * calls))
    split = call_split(m, el / calls * 1e3)
    mk = slamhot.ORBmatcher(0.75, True, device=ctx["local_rank"])
    runk = mk.prepare_batch("kf", views, kfs, 10.0, 100)
    warm_for(runk, 0.3)
    resk = []
    elk = timed_region(dist, device, lambda i: (runk(), resk.append(runk.results())), calls)
    elk, totk = sdist.reduce_run(dist, device, elk, float(P * calls))
    out = {
        "metric": "SearchByProjection(F, LastFrame) frames/s (TrackWithMotionModel's matcher, batched, host buffers)",
        "measured": "the C call slamhot_search_by_projection_last_batch on arguments marshalled before the timed region "
                    "(host buffers in and out: staging, PCIe, kernels, read-back)",
        "value": round(total / el, 1),
        "unit": "frames/s",
        "dtype": "f32 / u8",
        "config": {"workload": f"{P} (frame, last frame) pairs per call, 1200 features and "
                               f"~{int(np.mean([v.n for v in lfs]))} last-frame features each, th 7, nnratio 0.9, "
                               f"checkOri (slamhot_search_by_projection_last_batch)",
                   "parallelism": f"frame-sharded x{ctx['world']}"},
        "ms_per_call": round(el / calls * 1e3, 3),
        "mean_matches": round(float(np.mean([r[0] for r in res[-1]])), 1),
        "call_split": split,
        "keyframe_variant": {"metric": "SearchByProjection(F, KF, set, th 10, ORBdist 100) frames/s (batched)",
                             "value": round(totk / elk, 1), "ms_per_call": round(elk / calls * 1e3, 3),
                             "mean_matches": round(float(np.mean([r[0] for r in resk[-1]])), 1),
                             "call_split": call_split(mk, elk / calls * 1e3)},
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        import oracle_bind as ob
        cores = host_cores()

        def one(i):
            fv, lf, _, _ = uniq[i % len(uniq)]
            ob.search_by_projection_last(fv, lf, 0.9, True, 7.0, False)
            return 1

        work = list(range(64 * cores))
        one(0)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as pool:
            n = sum(pool.map(one, work))
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / dt, 1), "unit": "frames/s", "cores": cores, "kind": "port",
                               "cpu": cpu_model(),
                               "sample": f"{n} frames on {cores} threads: oracle SearchByProjection(F, LastFrame)"}
    m.close()
    mk.close()
    return out


# ------------------------------------------------------------------------------------------
# lba: configs[3] Optimizer::LocalBundleAdjustment
# ------------------------------------------------------------------------------------------
def lba_leg(ctx):
    """LM iterations/s of the device LBA solver on config-4 windows (BASELINE.json configs[3])."""
    import threading

    import torch

    import slamhot
    from slamhot import dist as sdist
    from slamhot import synth
    args, device, dist, lr = ctx["args"], ctx["device"], ctx["dist"], ctx["local_rank"]
    nwin = args.lba_windows
    # windows are sharded by rank: rank r solves its own seeds (independent units)
    pool = [synth.lba_window(s) for s in sdist.shard(8 * ctx["world"], ctx["rank"], ctx["world"])]
    windows = [pool[i % len(pool)] for i in range(nwin)]
    S = slamhot.LocalBundleAdjustment(device=lr)
    S.solve(windows[: min(4, nwin)])  # warm-up
    single = S.solve(pool[0])
    dev1, plan1, _ = S.last_stats()
    ate_dev = [window_ate(w, r["kf_Tcw"]) for w, r in zip(pool, S.solve(pool))]
    ate_init = [window_ate(w, w["kf_Tcw"]) for w in pool]
    it1 = single["iterations"][0] + single["iterations"][1]
    phase("compute: LBA drop-in call (tests/cpp/shim_driver lbatime)")
    drop_in = lba_drop_in(pool[0])
    # `lba_inflight` solver handles driven from host threads (the C call releases the GIL), each
    # on its own window set: one call's host planning overlaps another's device LM loop.  The
    # windows are flattened to C structs before the timed region, as a C++ caller holds them.
    NL = max(1, args.lba_inflight)
    solvers = [S] + [slamhot.LocalBundleAdjustment(device=lr) for _ in range(NL - 1)]
    runs = [sv.prepare(windows) for sv in solvers]
    for r_ in runs:
        r_()
    res0 = runs[0].results()
    trials_per_call = sum(r["trials"] for r in res0)
    iters_per_call = sum(r["iterations"][0] + r["iterations"][1] for r in res0)
    stats = [[0, 0.0, 0.0] for _ in range(NL)]

    def worker(t):
        if args.lba_stagger_ms > 0:
            time.sleep(t * args.lba_stagger_ms / 1e3)
        for _ in range(args.lba_calls):
            stats[t][0] += runs[t]()
            d, pl, _ = solvers[t].last_stats()
            stats[t][1] += d
            stats[t][2] += pl

    def run_all(_):
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(1, NL)]
        for th in ths:
            th.start()
        worker(0)
        for th in ths:
            th.join()

    elapsed = timed_region(dist, device, run_all, 1)
    iters = sum(x[0] for x in stats)
    dev_ms = sum(x[1] for x in stats) / NL
    plan_ms = sum(x[2] for x in stats) / NL
    dev_max, _ = sdist.reduce_run(dist, device, dev_ms, 0.0)
    el, iters_all = sdist.reduce_run(dist, device, elapsed, float(iters))
    rate = iters_all / el
    extra = max(trials_per_call - iters_per_call, 0) / max(iters_per_call, 1)
    flop_per_iter = LBA_FLOP_PER_ITER + extra * LBA_FLOP_PER_EXTRA_TRIAL
    tf = rate * flop_per_iter / 1e12
    out = {
        "metric": "LocalBundleAdjustment LM iterations/s",
        "value": round(rate, 1),
        "unit": "LM iterations/s",
        "dtype": "f64",
        "config": {"workload": "synthetic LocalBA 50 KF x 2000 pts x 8 obs, 2% outliers, 48 free KFs, "
                               "schedule 5 + 10 (BASELINE.json configs[3])",
                   "windows_per_gpu_per_call": nwin, "calls": args.lba_calls,
                   "parallelism": f"window-sharded x{ctx['world']}"},
        "roofline": {"bound": "fp64", "achieved": round(tf, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / FP64_PEAK_TFLOPS, 5),
                     "flop_per_lm_iteration": round(flop_per_iter), "trials_per_iteration": round(1 + extra, 3),
                     "note": "algorithmic FLOP (SURVEY.md §8d: 31.85 MFLOP per iteration + 27.05 per extra trial) x "
                             "whole-job LM iterations/s; MFMA-busy cycles per kernel in profiles/"},
        "lba_calls_per_s": round(nwin * args.lba_calls * NL * ctx["world"] / el, 2),
        "solves_in_flight": NL,
        "solver_start_stagger_ms": args.lba_stagger_ms,
        "ms_per_call": round(el / args.lba_calls * 1e3, 3),  # NL calls run concurrently
        "device_lm_iters_per_s_one_solver": round(iters_all / NL / (dev_max / 1e3), 1) if dev_max > 0 else None,
        "host_plan_ms_per_call": round(plan_ms / args.lba_calls, 3),
        "single_window": {"lm_iterations": it1, "device_ms": round(dev1, 3),
                          "ms_per_lm_iteration": round(dev1 / max(it1, 1), 4),
                          "drop_in": drop_in},
        "ate": {"metric": "ATE RMSE of the window's KeyFrame centres vs ground truth after LBA "
                          "(SE3 alignment, slamhot.ate = evaluate_ate_scale.py align)",
                "unit": "m", "windows": len(pool),
                "initial": round(float(np.mean(ate_init)), 7), "device": round(float(np.mean(ate_dev)), 7)},
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind as ob
        cores = host_cores()
        # single core: the drop-in comparison (LocalMapping solves one window at a time)
        reps, cpu_iters, ate_cpu = 0, 0, []
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0 and reps < len(pool):
            r = ob.lba_solve(pool[reps])
            cpu_iters += r["iterations"][0] + r["iterations"][1]
            ate_cpu.append(window_ate(pool[reps], r["kf_Tcw"]))
            reps += 1
        dt1 = time.perf_counter() - t0
        # every host core: independent windows, one per thread
        work = [pool[i % len(pool)] for i in range(2 * cores)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            its = list(ex.map(lambda w: sum(ob.lba_solve(w)["iterations"]), work))
        dtn = time.perf_counter() - t0
        out["ate"]["oracle_same_windows"] = round(float(np.mean(ate_cpu)), 7)
        out["ate"]["device_same_windows"] = round(float(np.mean(ate_dev[:reps])), 7)
        out["cpu_baseline"] = {
            "value": round(sum(its) / dtn, 2), "unit": "LM iterations/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{len(work)} config-4 windows on {cores} threads (one window per task); oracle/lba_oracle.cpp "
                      f"(g2o LM/Schur restatement, dense LDL^T) -O3",
            "one_core": {"value": round(cpu_iters / dt1, 2), "windows": reps,
                         "ms_per_lm_iteration": round(dt1 * 1e3 / max(cpu_iters, 1), 3),
                         "ms_per_call": round(dt1 * 1e3 / max(reps, 1), 3)},
        }
    for sv in solvers:
        sv.close()
    return out


def lba_drop_in(W, reps=25):
    """Wall-clock of the drop-in Optimizer::LocalBundleAdjustment call on one config-4 window: the
    C++ shim (include/slamhot_orbslam3.hpp: window build over the map objects, flattening, plan,
    upload, device solve, download, vToErase, pose / point write-back) run by tests/cpp/shim_driver
    in its own process on a freshly loaded map per call, 24 calls as LocalMapping makes them one after
    another (median and p90); the first call (allocations) is reported apart."""
    import subprocess
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import shim_io
    from slamhot import optimizer as opt
    if not shim_io.DRIVER.exists():
        return None
    pmap, kfs, mps = opt.map_from_window(W)
    with tempfile.TemporaryDirectory() as d:
        mp, op = Path(d) / "map.bin", Path(d) / "out.bin"
        shim_io.write_map(mp, pmap, kfs, mps)
        r = subprocess.run([str(shim_io.DRIVER), "lbatime", str(mp), str(op), str(reps)], capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            return {"error": r.stderr[-300:]}
        b = shim_io.Blob(op.read_bytes())
        counts = [b.i32() for _ in range(4)]
        ms, st = b.vec("<f8"), b.vec("<f8")
    return {"wall_ms_per_call": round(float(np.median(ms[1:])), 3), "calls": int(len(ms) - 1),
            "p90_ms_per_call": round(float(np.percentile(ms[1:], 90)), 3),
            "first_call_ms": round(float(ms[0]), 3), "device_ms": round(float(st[0]), 3),
            "plan_ms": round(float(st[1]), 3), "host_device_round_trips": int(st[2]),
            "num_fixedKF_OptKF_MPs_edges": counts,
            "what": "tests/cpp/shim_driver lbatime: the LocalBundleAdjustment shim end to end (window build from the "
                    "map objects, flatten, plan, H2D, device LM 5 + 10, D2H, vToErase, write-back) per call"}


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


# ------------------------------------------------------------------------------------------
# track: configs[4] — the per-sequence stereo tracking chain
# ------------------------------------------------------------------------------------------
def pingpong(n, steps):
    """Frame index of step k walking 0..n-1..0.. (a continuous path over n rendered frames)."""
    period = 2 * (n - 1)
    return [k % period if k % period < n else period - k % period for k in range(steps)]


def track_leg(ctx):
    """configs[4]: per-sequence stereo tracking (slamhot_tracker_*): S sequences per GPU advance in
    lock-step, one raw stereo frame each per step, through the whole device-resident chain
    (remap x2, extract x2, stereo, BoW + SearchByBoW vs the reference KF, PoseOptimization,
    SearchLocalPoints, PoseOptimization, keyframe insertion).  Sequence s replays rendered chunk
    s % (number of chunks) back and forth (a continuous path).  value = sequence-frames/s of the whole job."""
    import torch

    import slamhot
    from slamhot import ate
    from slamhot import dist as sdist
    from slamhot import synth
    args, device, dist, lr = ctx["args"], ctx["device"], ctx["dist"], ctx["local_rank"]
    S, K = args.track_seqs, args.track_frames
    W, H = 752, 480
    maps = euroc_maps()
    # the headline's frames (its leg child left them in the rank's scratch directory)
    raw_l, raw_r = load_chunks(ctx, maps, max(SEQ_LEN, args.pairs // SEQ_LEN * SEQ_LEN))
    nch = len(raw_l) // SEQ_LEN
    voc_arrays = sdist.broadcast_arrays(dist, device, synth.vocab(10, 6, 0) if ctx["rank"] == 0 else None)
    voc = slamhot.Vocabulary(*voc_arrays, k=10, L=6, device=lr)
    cam = (np.float32(synth.EUROC_STEREO["fx"]), np.float32(synth.EUROC_STEREO["fx"]), np.float32(367.4517211914062),
           np.float32(252.2008514404297), np.float32(synth.EUROC_STEREO["bf"]))
    # device frames: d_l[f] holds frame f of every sequence
    d_l, d_r = [], []
    for f in range(SEQ_LEN):
        idx = [(s % nch) * SEQ_LEN + f for s in range(S)]
        d_l.append(torch.from_numpy(np.ascontiguousarray(raw_l[idx])).to(device))
        d_r.append(torch.from_numpy(np.ascontiguousarray(raw_r[idx])).to(device))
    order = pingpong(SEQ_LEN, K)
    # the S sequences split over G tracker handles (each its own stream; sequences are
    # independent, so the split changes no result), stepped in turn from this thread
    G = max(1, min(args.track_inflight, S))
    sizes = [S // G + (1 if g < S % G else 0) for g in range(G)]
    offs = [sum(sizes[:g]) * W * H for g in range(G)]

    def step_all(Ts, f):
        for g, Tg in enumerate(Ts):
            Tg.step_device(d_l[f].data_ptr() + offs[g], d_r[f].data_ptr() + offs[g])

    warm = [slamhot.Tracker(voc, n, cam, maps=maps, device=lr) for n in sizes]
    for f in order[: min(K, 2 * SEQ_LEN)]:
        step_all(warm, f)
    for w_ in warm:
        w_.records()
        w_.close()
    Ts = [slamhot.Tracker(voc, n, cam, maps=maps, device=lr) for n in sizes]
    recs = []

    def step(k):
        step_all(Ts, order[k])

    elapsed = timed_region(dist, device, step, K)
    # a second pass for the per-step records (same inputs, fresh tracker): lost / keyframe counts,
    # inliers and the trajectory of sequence 0 for the ATE
    T2 = slamhot.Tracker(voc, S, cam, maps=maps, device=lr)
    for k in range(K):
        f = order[k]
        T2.step_device(d_l[f].data_ptr(), d_r[f].data_ptr())
        recs.append(T2.records())
    T2.close()
    for Tg in Ts:
        Tg.close()
    # configs[4] literally: ONE sequence on the GPU (its frame latency bounds a live camera)
    T1 = slamhot.Tracker(voc, 1, cam, maps=maps, device=lr)
    for k in range(min(K, 4)):
        T1.step_device(d_l[order[k]][:1].data_ptr(), d_r[order[k]][:1].data_ptr())
    T1.records()
    T1.close()
    T1 = slamhot.Tracker(voc, 1, cam, maps=maps, device=lr)
    el1 = timed_region(None, device, lambda k: T1.step_device(d_l[order[k]][:1].data_ptr(),
                                                              d_r[order[k]][:1].data_ptr()), K)
    T1.close()
    voc.close()
    el, units = sdist.reduce_run(dist, device, elapsed, float(S * K))
    lost = sum(r["lost"] for rr in recs[1:] for r in rr)
    kfs = sum(r["is_keyframe"] for rr in recs for r in rr)
    inl = float(np.mean([r["n_inl"] for rr in recs[1:] for r in rr]))
    # ATE of sequence 0 (chunk 0): centres of the tracked poses vs ground truth (SE3 + scale
    # alignment of evaluate_ate_scale.py); the tracker starts at the identity, GT at its frame 0
    gt = synth.sequence_poses(101 + 17 * ctx["rank"], SEQ_LEN)
    est_c = np.stack([-(r[0]["Tcw"][:3, :3].T.astype(np.float64) @ r[0]["Tcw"][:3, 3]) for r in recs])
    gt_c = np.stack([-(gt[f][:3, :3].T @ gt[f][:3, 3]) for f in order])
    _, _, _, _, err, _ = ate.align(est_c.T, gt_c.T)
    out = {
        "metric": "stereo tracking sequence-frames/s (configs[4] per GPU)",
        "value": round(units / el, 2),
        "unit": "sequence-frames/s",
        "dtype": "u8 / f64",
        "config": {"workload": f"{S} stereo sequences per GPU in lock-step, {K} raw 752x480 frames each (rendered room, "
                               f"EuRoC calibration): remap x2, ORBextractor x2 (1200), ComputeStereoMatches, ComputeBoW + "
                               f"SearchByBoW vs reference KF, PoseOptimization, SearchLocalPoints, PoseOptimization, "
                               f"NeedNewKeyFrame / CreateNewKeyFrame — all device-resident",
                   "parallelism": f"sequence-sharded x{ctx['world']}", "tracker_handles": G},
        "ms_per_step": round(el / K * 1e3, 3),
        "per_sequence_frames_per_s": round(K / el, 1),
        "single_sequence": {"frames_per_s": round(K / el1, 1), "ms_per_frame": round(el1 / K * 1e3, 3),
                            "note": "one sequence alone on the GPU (nseq = 1), same frames"},
        "lost_frames": int(lost), "keyframes": int(kfs), "mean_inliers": round(inl, 1),
        "ate_seq0_m": round(float(np.sqrt(np.mean(err * err))), 5),
    }
    if ctx["cpu"]:
        phase("compute: CPU baseline (oracle on the host cores)")
        out["cpu_baseline"] = track_cpu(raw_l, raw_r, maps, voc_arrays, order[: 2 * SEQ_LEN])
    return out


def track_cpu(raw_l, raw_r, maps, voc_arrays, order):
    """The oracle chain (tests/track_oracle.py) on the host cores, one sequence per thread."""
    sys.path.insert(0, str(ROOT / "tests"))
    import track_oracle as to
    P = to.params()
    cores = host_cores()

    nch = len(raw_l) // SEQ_LEN

    def run(c):
        st = to.SeqState()
        base = (c % nch) * SEQ_LEN
        for f in order:
            to.step(P, voc_arrays, maps, st, raw_l[base + f], raw_r[base + f])
        return len(order)

    run(0)  # warm-up
    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as pool:
        frames = sum(pool.map(run, range(cores)))
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 2), "unit": "sequence-frames/s", "cores": cores, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{cores} sequences x {len(order)} stereo frames, one sequence per thread: the oracle chain "
                      f"tests/track_oracle.py (oracle remap, extract, stereo, BoW, PoseOptimization, SearchLocalPoints)"}


if __name__ == "__main__":
    main()
