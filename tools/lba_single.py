"""Experiment helper: one config-4 window solved repeatedly (LocalMapping's per-KeyFrame call), for
a rocprofv3 kernel trace of the single-window latency."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

W = synth.lba_window(0)
S = slamhot.LocalBundleAdjustment(device=0)
for _ in range(3):
    S.solve(W)
t = []
for _ in range(10):
    t0 = time.perf_counter()
    r = S.solve(W)
    t.append(time.perf_counter() - t0)
t.sort()
print("median ms", 1e3 * t[len(t) // 2], "iterations", r["iterations"], "trials", r["trials"], "stats", S.last_stats())
S.close()
