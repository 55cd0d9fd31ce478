"""Golden vectors for slamhot/ate.py, produced with the reference's own evaluation functions
(/root/reference/evaluation/{associate.py,evaluate_ate_scale.py}: `associate`, `align`), which
import under Python 3 here.  Only inputs and outputs are saved
(tests/golden/ate.npz); nothing of the reference's code is copied.  Run in the build container
only (the GPU box has no /root/reference)."""
import sys
import warnings
from pathlib import Path

import numpy as np

REF = Path("/root/reference/evaluation")
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REF))
warnings.filterwarnings("ignore")
import associate as ref_assoc  # noqa: E402
import evaluate_ate_scale as ref_ate  # noqa: E402

rng = np.random.default_rng(7)
out = {}
for case in range(4):
    n = 60 + 40 * case
    t = np.cumsum(rng.uniform(0.04e9, 0.06e9, n))          # ns stamps
    gt = np.cumsum(rng.normal(0, 0.05, (n, 3)), 0)
    ang = rng.uniform(0, np.pi)
    R = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
    s_true = rng.uniform(0.5, 2.0)
    est = (gt @ R.T) * s_true + rng.normal(0, 0.01, (n, 3)) + rng.normal(0, 1, 3)
    t_est = t + rng.normal(0, 3e6, n)                       # jittered, some dropped
    keep = rng.random(n) > 0.1
    first = {float(a): [str(x) for x in p] + ["0", "0", "0", "1"] for a, p in zip(t, gt)}
    second = {float(a): [str(x) for x in p] + ["0", "0", "0", "1"] for a, p in zip(t_est[keep], est[keep])}
    matches = ref_assoc.associate(first, second, 0.0, 20000000.0)
    fx = np.matrix([[float(v) for v in first[a][0:3]] for a, b in matches]).transpose()
    sx = np.matrix([[float(v) for v in second[b][0:3]] for a, b in matches]).transpose()
    rot, transGT, errGT, trans, err, s = ref_ate.align(sx, fx)
    out[f"c{case}_t"] = t
    out[f"c{case}_gt"] = gt
    out[f"c{case}_test"] = t_est[keep]
    out[f"c{case}_est"] = est[keep]
    out[f"c{case}_matches"] = np.array(matches)
    out[f"c{case}_rot"] = np.asarray(rot)
    out[f"c{case}_s"] = np.array(s)
    out[f"c{case}_err"] = np.asarray(err)
    out[f"c{case}_errGT"] = np.asarray(errGT)
np.savez_compressed(ROOT / "tests" / "golden" / "ate.npz", **out)
print("wrote", ROOT / "tests" / "golden" / "ate.npz")
