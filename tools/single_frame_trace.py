"""Experiment helper: a few single-frame calls (slamhot_extract) through a trace build of the
library (SLAMHOT_LIB), to collect its device printf phase marks."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

img = synth.frame(3, 640, 480)
ex = slamhot.ORBextractor(nfeatures=1000, device=0, max_size=(640, 480))
for _ in range(3):
    ex(img)
ex.close()
