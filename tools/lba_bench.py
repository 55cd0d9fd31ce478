"""Local-BA throughput probe: config-4 windows (50 KF x 2000 pts x 8 obs), batched.
Prints per batch size: wall ms per solve call, device ms, LM iterations/s, LBA calls/s."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402

import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="1,8,32,64,128")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cpu", action="store_true")
a = ap.parse_args()
batches = [int(b) for b in a.batches.split(",")]
pool = [synth.lba_window(s) for s in range(8)]
S = slamhot.LocalBundleAdjustment()
S.solve(pool[0])
out = []
for B in batches:
    Ws = [pool[i % len(pool)] for i in range(B)]
    best = None
    for _ in range(a.reps):
        t = time.perf_counter()
        res = S.solve(Ws)
        wall = time.perf_counter() - t
        dev, plan, syncs = S.last_stats()
        if best is None or wall < best[0]:
            best = (wall, dev, plan, syncs, res)
    wall, dev, plan, syncs, res = best
    iters = sum(r["iterations"][0] + r["iterations"][1] for r in res)
    trials = sum(r["trials"] for r in res)
    line = dict(batch=B, wall_ms=wall * 1e3, device_ms=dev, plan_ms=plan, syncs=syncs, lm_iters=iters, trials=trials,
                lm_iters_per_s=iters / wall, lm_iters_per_s_device=iters / (dev / 1e3), lba_calls_per_s=B / wall)
    print(json.dumps(line), flush=True)
    out.append(line)
if a.cpu:
    import oracle_bind as ob
    t = time.perf_counter()
    r = ob.lba_solve(pool[0])
    dt = time.perf_counter() - t
    it = r["iterations"][0] + r["iterations"][1]
    print(json.dumps(dict(cpu_oracle_ms=dt * 1e3, lm_iters=it, trials=r["trials"], lm_iters_per_s=it / dt)))
