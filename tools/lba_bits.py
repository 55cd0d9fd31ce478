"""Dump the LBA results of a fixed set of windows (poses, points, outlier flags, iteration / trial counts)
to an .npz, to compare two builds bit for bit:  SLAMHOT_LIB=... python3 tools/lba_bits.py OUT.npz"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

wins = [synth.lba_window(s, stereo_frac=0.3 * (s % 3), body_frac=0.5 if s % 4 == 1 else 0.0) for s in range(12)]
S = slamhot.LocalBundleAdjustment()
res = S.solve(wins)
out = {}
for i, r in enumerate(res):
    for k, v in r.items():
        out[f"{i}_{k}"] = np.asarray(v)
np.savez(sys.argv[1], **out)
print("saved", len(res), "windows")
