"""bench.py --gpus N as the driver runs it (`python bench.py --gpus N`, no WORLD_SIZE): the script
starts its own N rank processes, relays rank 0's one JSON line and fails when a rank fails or the
job hangs.  Exercised on CPU through the GPU-free `--legs dry` leg (gloo collectives)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=str(ROOT))


def _line(p):
    lines = [s for s in p.stdout.splitlines() if s.strip()]
    assert len(lines) == 1, (p.stdout, p.stderr[-2000:])
    return json.loads(lines[0])


def test_gpus_two_launches_two_ranks():
    p = _run(["--gpus", "2", "--legs", "dry", "--steps", "3", "--warmup", "1", "--pairs", "128"])
    assert p.returncode == 0, p.stderr[-3000:]
    r = _line(p)
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["scaling"] == "weak"
    assert len(r["rank_digests"]) == 2 and r["rank_digests"][0] != r["rank_digests"][1]
    assert r["value"] > 0 and r["config"]["parallelism"] == "frame-sharded x2"
    # frame content follows the global frame index: the job digest of 2 ranks x 4 frames equals one
    # process over 8 frames
    p1 = _run(["--gpus", "1", "--legs", "dry", "--steps", "1", "--warmup", "0", "--pairs", "256"])
    assert p1.returncode == 0, p1.stderr[-3000:]
    r1 = _line(p1)
    assert r1["n_gpus"] == 1 and len(r1["rank_digests"]) == 1
    assert r["digest"]["job"] == r1["digest"]["job"] != 0


def test_gpus_launcher_fails_when_a_rank_fails():
    p = _run(["--gpus", "2", "--legs", "dry", "--steps", "2", "--warmup", "0"], {"SLAMHOT_DRY_FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr[-3000:])
    assert p.stdout.strip() == ""
    # the rank whose leg failed is named (rank 0's leg child was stopped because of it)
    assert "leg dry failed on rank 1" in p.stderr, p.stderr[-3000:]


def test_hung_leg_in_one_rank_is_an_error_record():
    """A leg that hangs in one rank (a host stall: no progress, no exit) ends at its deadline as an
    error entry naming the leg, the rank and where it stopped, and the line (the first leg's value)
    is still printed, well inside the job deadline."""
    p = _run(["--gpus", "2", "--legs", "dry,dryaux", "--steps", "2", "--warmup", "0", "--leg-timeout-scale", "0.2"],
             {"SLAMHOT_DRY_HANG": "dryaux:1"})
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
    r = _line(p)
    assert r["value"] > 0 and r["n_gpus"] == 2
    e = r["dryaux"]
    assert e["error"] == "timeout" and e["rank"] == 1, e
    assert e["phase"].startswith("compute"), e
    assert e["ranks"]["0"].startswith("timeout (collective"), e
    assert r["legs"]["wall_s"]["dryaux"]["status"] == "error"
    assert "leg dryaux FAILED: timeout on rank 1" in p.stderr
    # every Python thread's stack of the stalled child is on stderr
    assert "in dry_leg" in p.stderr


def test_single_rank_hung_leg_keeps_the_line():
    """N = 1, as the driver runs bench.py: the hung second leg is recorded, the first leg's value
    printed, and the job ends near the leg's deadline (not the driver's limit)."""
    p = _run(["--legs", "dry,dryaux", "--steps", "2", "--warmup", "0", "--leg-timeout-scale", "0.15"],
             {"SLAMHOT_DRY_HANG": "dryaux:0"})
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
    r = _line(p)
    assert r["value"] > 0 and r["dryaux"]["error"] == "timeout" and r["dryaux"]["rank"] == 0
    assert r["legs"]["job_wall_s"] < 60


def test_hung_first_leg_fails_the_job_by_name():
    p = _run(["--legs", "dry", "--steps", "2", "--warmup", "0", "--leg-timeout-scale", "0.15"],
             {"SLAMHOT_DRY_HANG": "dry:0"})
    assert p.returncode != 0 and p.stdout.strip() == ""
    assert "leg dry timeout on rank 0" in p.stderr, p.stderr[-2000:]


def test_job_deadline_skips_legs_that_cannot_start():
    """A leg starts only with the time left of the job deadline: none left, nothing runs, and the job
    fails naming the first leg."""
    p = _run(["--legs", "dry,dryaux", "--steps", "2", "--warmup", "0", "--job-deadline", "1"])
    assert p.returncode != 0 and p.stdout.strip() == ""
    assert "leg dry skipped" in p.stderr, p.stderr[-2000:]


def test_torchrun_launch_runs_legs_in_children():
    """The driver's N > 1 form: `python -m torch.distributed.run --nproc-per-node N ... bench.py`.
    Each rank process (torchrun's worker, on the agent's store) runs its legs in child processes with
    a process group of their own, and exactly one JSON line reaches stdout."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2",
                        "--legs", "dry,dryaux", "--steps", "2", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    r = _line(p)
    assert r["n_gpus"] == 2 and len(r["rank_digests"]) == 2
    assert r["dryaux"]["value"] > 0 and r["legs"]["wall_s"]["dryaux"]["status"] == "ok"
