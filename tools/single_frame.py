"""Experiment helper: the per-image host-buffer call (slamhot_extract) repeated on one VGA frame,
for a rocprofv3 kernel trace of the single-frame latency."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

img = synth.frame(3, 640, 480)
ex = slamhot.ORBextractor(nfeatures=1000, device=0, max_size=(640, 480))
for _ in range(20):
    ex(img)
t = []
for _ in range(100):
    t0 = time.perf_counter()
    ex(img)
    t.append(time.perf_counter() - t0)
t.sort()
print("median ms", 1e3 * t[len(t) // 2])
ex.close()
