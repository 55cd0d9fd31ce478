"""GPU parity of Optimizer::PoseOptimization (slamhot_pose_optimization) against the CPU
restatement (oracle/pose_oracle.cpp).  Pose within 1e-5, identical outlier flags and inlier
counts (LM decisions identical; only FP64 summation order differs)."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def popt():
    import slamhot
    s = slamhot.PoseOptimizer()
    yield s
    s.close()


def _check(g, o):
    assert g["n_initial"] == o["n_initial"]
    assert g["n_inliers"] == o["n_inliers"]
    assert np.array_equal(g["outlier"], o["outlier"])
    assert np.abs(g["Tcw"].astype(np.float64) - o["Tcw"]).max() <= 1e-5


@pytest.mark.parametrize("seed,stereo", [(0, 0.0), (1, 0.0), (2, 0.5), (3, 1.0)])
def test_pose_frames(popt, seed, stereo):
    f = synth.pose_frame(seed, stereo_frac=stereo)
    g, o = popt.solve(f), ob.pose_optimization(f)
    _check(g, o)
    gt = f["gt_Tcw"]
    assert np.abs(g["Tcw"][:3, 3] - gt[:3, 3]).max() < np.abs(f["Tcw"][:3, 3] - gt[:3, 3]).max()


def test_pose_batch_and_small_frames(popt):
    frames = [synth.pose_frame(10 + i, n=n, mp_frac=0.9, stereo_frac=0.3 * (i % 2), outlier_frac=0.2)
              for i, n in enumerate([1500, 40, 12, 9, 2, 600])]
    gs = popt.solve(frames)
    for f, g in zip(frames, gs):
        _check(g, ob.pose_optimization(f))
    # fewer than 3 observations: returns 0 and leaves the pose untouched
    tiny = synth.pose_frame(99, n=3, mp_frac=0.5)
    tiny["has_mp"][:] = [1, 1, 0]
    g = popt.solve(tiny)
    assert g["n_inliers"] == 0 and np.array_equal(g["Tcw"], tiny["Tcw"])


@pytest.mark.parametrize("outliers", [0.6, 0.95])
def test_pose_mostly_outliers(popt, outliers):
    """Most observations are gross outliers: the chi2 gates of the four rounds
    (Optimizer.cc PoseOptimization, 5.991 / 7.815) flag nearly every edge, the later rounds run
    on few inliers, and the outcome (flags, inlier count, pose) still equals the oracle's."""
    frames = [synth.pose_frame(40 + i, outlier_frac=outliers, stereo_frac=0.5 * i) for i in range(2)]
    for f, g in zip(frames, popt.solve(frames)):
        _check(g, ob.pose_optimization(f))


def test_pose_large_initial_error(popt):
    f = synth.pose_frame(20, rot_deg=5.0, trans_m=0.3, outlier_frac=0.3)
    _check(popt.solve(f), ob.pose_optimization(f))


def test_pose_prepared_run_repeats(popt):
    """prepare(): the bench's C call on pre-marshalled frames gives solve()'s results, call after call."""
    frames = [synth.pose_frame(30 + i, stereo_frac=0.5 * (i % 2)) for i in range(5)]
    run = popt.prepare(frames)
    for _ in range(2):
        run()
        for f, g, s in zip(frames, run.results(), popt.solve(frames)):
            assert np.array_equal(g["Tcw"], s["Tcw"]) and np.array_equal(g["outlier"], s["outlier"])
            _check(g, ob.pose_optimization(f))
