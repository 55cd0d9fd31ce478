"""Experiment helper: one extraction of the headline's 128 rectified EuRoC frames with an
instrumented library (SLAMHOT_LIB=lib/ab/libslamhot_ftrace.so, built -DSLAMHOT_FAST_TRACE): the
kernel prints per-pass cycle counts of sampled cells."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

Ls = []
for s in range(8):
    L, _, _ = synth.stereo_sequence(101 + s, 16)
    Ls += list(L)
imgs = np.stack(Ls[:128])
ex = slamhot.ORBextractor(nfeatures=1200, device=0, max_size=(752, 480), max_batch=128)
ex.extract_batch(imgs)
ex.close()
