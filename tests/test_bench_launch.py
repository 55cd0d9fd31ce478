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
    # the first rank to fail sets the status (rank 0 then fails too, on the closed connection)
    assert "rank 1 exited with 3" in p.stderr


def test_gpus_launcher_kills_a_hung_job():
    # far more steps than the timeout allows: the launcher kills both ranks and reports 124
    p = _run(["--gpus", "2", "--legs", "dry", "--steps", "100000", "--warmup", "0", "--launch-timeout", "4"])
    assert p.returncode == 124, (p.returncode, p.stderr[-3000:])
    assert p.stdout.strip() == ""
