"""CPU checks of the Frame::UndistortKeyPoints / ComputeImageBounds oracle
(oracle/frame_oracle.cpp) against an independent numpy restatement of OpenCV 4.2.0's
cvUndistortPointsInternal (default TermCriteria(COUNT, 5)), bit for bit — numpy float64 is IEEE
double with the same evaluation order — including the icdist < 0 early exit (regression_14583)
and the dist[0] == 0 identity branch (Frame.cc:732-736).  Parity unpinned otherwise: OpenCV is
not in this image."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

CAM = synth.EUROC_MONO_CAM
K = np.array([CAM["fx"], CAM["fy"], CAM["cx"], CAM["cy"]], np.float32)
D = np.array(CAM["dist"], np.float32)


def numpy_undistort(u, v, K, dist):
    fx, fy, cx, cy = [float(x) for x in np.asarray(K, np.float32)]
    k = np.zeros(14)
    k[:len(dist)] = np.asarray(dist, np.float32).astype(np.float64)
    ifx, ify = 1.0 / fx, 1.0 / fy
    out = []
    for uf, vf in zip(np.asarray(u, np.float32), np.asarray(v, np.float32)):
        u_, v_ = float(uf), float(vf)
        x = (u_ - cx) * ifx
        y = (v_ - cy) * ify
        x0, y0 = x, y
        for _ in range(5):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            if icdist < 0:
                x = (u_ - cx) * ifx
                y = (v_ - cy) * ify
                break
            dX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
            dY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
            x = (x0 - dX) * icdist
            y = (y0 - dY) * icdist
        xx = fx * x + 0.0 * y + cx
        yy = 0.0 * x + fy * y + cy
        ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
        out.append((np.float32(xx * ww), np.float32(yy * ww)))
    return np.array(out, np.float32).reshape(-1, 2)


def _kps(u, v):
    k = np.zeros(len(u), ob.KP_DTYPE)
    k["x"], k["y"] = u, v
    k["octave"] = np.arange(len(u)) % 8
    k["angle"] = np.linspace(0, 359, len(u))
    k["response"] = 1.5
    k["size"] = 31
    return k


@pytest.mark.parametrize("dist", [D, np.append(D, np.float32(0.01)), np.array([0.12, -0.05, 0.001, -0.002], np.float32)])
def test_undistort_matches_numpy(dist):
    rng = np.random.default_rng(0)
    u = rng.uniform(0, 752, 2000).astype(np.float32)
    v = rng.uniform(0, 480, 2000).astype(np.float32)
    kps = _kps(u, v)
    got = ob.undistort_keypoints(kps, K, dist)
    ref = numpy_undistort(u, v, K, dist)
    assert np.array_equal(got["x"], ref[:, 0]) and np.array_equal(got["y"], ref[:, 1])
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(got[f], kps[f])


def test_undistort_icdist_negative_branch():
    """A strong positive-k1-free model whose denominator turns negative during the iteration:
    the point falls back to the undistorted ray start (OpenCV regression_14583)."""
    dist = np.array([-2.5, 0.0, 0.0, 0.0], np.float32)
    u = np.array([0.0, 5.0, 752.0, 700.0, 367.0], np.float32)
    v = np.array([0.0, 470.0, 480.0, 10.0, 248.0], np.float32)
    got = ob.undistort_keypoints(_kps(u, v), K, dist)
    ref = numpy_undistort(u, v, K, dist)
    assert np.array_equal(got["x"], ref[:, 0]) and np.array_equal(got["y"], ref[:, 1])
    # the corner took the early exit: it maps to itself through K
    assert abs(float(got["x"][0]) - 0.0) < 1e-3


def test_identity_when_k1_is_zero():
    kps = _kps(np.array([1.5, 700.25], np.float32), np.array([2.0, 400.0], np.float32))
    got = ob.undistort_keypoints(kps, K, np.array([0.0, 0.1, 0.01, 0.01], np.float32))
    assert np.array_equal(got.view(np.uint8), kps.view(np.uint8))


def test_image_bounds():
    b = ob.image_bounds(K, D, 752, 480)
    c = numpy_undistort(np.array([0, 752, 0, 752], np.float32), np.array([0, 0, 480, 480], np.float32), K, D)
    assert b[0] == min(c[0, 0], c[2, 0]) and b[1] == max(c[1, 0], c[3, 0])
    assert b[2] == min(c[0, 1], c[1, 1]) and b[3] == max(c[2, 1], c[3, 1])
    assert b[0] < 0 and b[1] > 752  # barrel distortion pushes the corners out
    assert np.array_equal(ob.image_bounds(K, np.zeros(4, np.float32), 752, 480), [0, 752, 0, 480])
