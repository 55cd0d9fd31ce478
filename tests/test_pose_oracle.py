"""CPU checks of the PoseOptimization oracle: convergence toward the true pose, outlier
detection on planted outliers, early return below 3 observations."""
import numpy as np

import oracle_bind as ob
from slamhot import synth


def test_converges_and_flags_planted_outliers():
    f = synth.pose_frame(5, n=800, outlier_frac=0.0)
    r = ob.pose_optimization(f)
    gt = f["gt_Tcw"]
    assert np.abs(r["Tcw"][:3, 3] - gt[:3, 3]).max() < 5e-3
    assert r["n_inliers"] > 0.9 * r["n_initial"]
    f2 = synth.pose_frame(5, n=800, outlier_frac=0.25)
    r2 = ob.pose_optimization(f2)
    assert r2["n_initial"] - r2["n_inliers"] >= 0.2 * r2["n_initial"]


def test_fewer_than_three_observations():
    f = synth.pose_frame(6, n=5, mp_frac=1.0)
    f["has_mp"][:] = [1, 0, 1, 0, 0]
    r = ob.pose_optimization(f)
    assert r["n_initial"] == 2 and r["n_inliers"] == 0
    assert np.array_equal(r["Tcw"], f["Tcw"])
