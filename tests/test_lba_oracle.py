"""CPU checks of the local-BA oracle (oracle/lba_oracle.cpp): an independent numpy
restatement of the robust chi2 at the initial estimate (Converter::toSE3Quat, Pinhole
projection, stereo float-invz quirk, Huber with float dsqr), convergence on noise-free
windows, the LM schedule bounds and the stop flag."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

f32 = np.float32


def _quat_from_R(R):
    t = R[0, 0] + R[1, 1] + R[2, 2]
    if t > 0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        q = np.array([(R[2, 1] - R[1, 2]) * t, (R[0, 2] - R[2, 0]) * t, (R[1, 0] - R[0, 1]) * t, w])
    else:
        i = 0
        if R[1, 1] > R[0, 0]:
            i = 1
        if R[2, 2] > R[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q = np.zeros(4)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def _rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def numpy_robust_chi2(W):
    fx, fy, cx, cy, bf = [float(c) for c in W["cam"]]
    T = W["kf_Tcw"].reshape(-1, 4, 4).astype(np.float64)
    Rs = np.array([_rot(_quat_from_R(t[:3, :3])) for t in T])
    ts = T[:, :3, 3]
    X = W["pt_pos"].astype(np.float64)[W["edge_pt"]]
    Xc = np.einsum("eij,ej->ei", Rs[W["edge_kf"]], X) + ts[W["edge_kf"]]
    obs = W["edge_obs"].astype(np.float64)
    info = W["edge_inv_sigma2"].astype(np.float64)
    stereo = W["edge_obs"][:, 2] >= 0
    chi = np.zeros(len(X))
    mono = ~stereo
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    chi[mono] = (((obs[:, 0] - u) ** 2 + (obs[:, 1] - v) ** 2) * info)[mono]
    invz = (1.0 / Xc[:, 2]).astype(f32).astype(np.float64)
    us = Xc[:, 0] * invz * fx + cx
    vs = Xc[:, 1] * invz * fy + cy
    urs = us - (f32(bf) * invz.astype(f32)).astype(np.float64)
    chi_s = ((obs[:, 0] - us) ** 2 + (obs[:, 1] - vs) ** 2 + (obs[:, 2] - urs) ** 2) * info
    chi[stereo] = chi_s[stereo]
    dm, ds = float(f32(np.sqrt(5.991))), float(f32(np.sqrt(7.815)))
    delta = np.where(stereo, ds, dm)
    dsqr = np.where(stereo, float(f32(ds * ds)), float(f32(dm * dm)))
    rob = np.where(chi <= dsqr, chi, 2 * np.sqrt(chi) * delta - dsqr)
    return rob.sum()


@pytest.mark.parametrize("stereo", [0.0, 0.4])
def test_initial_chi2_matches_numpy(stereo):
    W = synth.lba_window(40, n_kf=12, n_pt=200, obs_per_pt=5, stereo_frac=stereo)
    r = ob.lba_solve(W, iters_first=1, iters_second=0)
    np.testing.assert_allclose(r["chi2_initial"], numpy_robust_chi2(W), rtol=1e-9)


def test_noise_free_window_converges_to_ground_truth():
    W = synth.lba_window(41, n_kf=15, n_pt=400, obs_per_pt=6, outlier_frac=0.0, noise=0.0)
    r = ob.lba_solve(W)
    assert r["chi2_final"] < 1e-6 * r["chi2_initial"]
    assert r["n_outlier"] == 0
    assert np.abs(r["pt_pos"] - W["gt_pts"]).max() < 1e-3
    T = r["kf_Tcw"].reshape(-1, 4, 4)
    assert np.abs(T[:, :3, 3] - W["gt_T"][:, :3, 3]).max() < 1e-3


def test_schedule_bounds_and_monotone_chi2():
    W = synth.lba_window(42, n_kf=20, n_pt=500, obs_per_pt=6, stereo_frac=0.3)
    r = ob.lba_solve(W)
    assert 1 <= r["iterations"][0] <= 5 and 0 <= r["iterations"][1] <= 10
    assert r["chi2_final"] <= r["chi2_initial"]
    assert r["trials"] >= r["iterations"][0] + r["iterations"][1]
    # the robust cost the solver reports at the end is the one of the returned estimate
    assert r["n_outlier"] >= int(0.5 * 0.02 * len(W["edge_pt"]))


def test_stop_flag_returns_inputs():
    W = synth.lba_window(43, n_kf=8, n_pt=50, obs_per_pt=3)
    r = ob.lba_solve(W, stop=1)
    assert np.array_equal(r["kf_Tcw"], W["kf_Tcw"]) and np.array_equal(r["pt_pos"], W["pt_pos"])
    assert r["iterations"] == (0, 0) and r["n_outlier"] == 0


def test_fixed_camera_poses_pass_through():
    W = synth.lba_window(44, n_kf=10, n_pt=100, obs_per_pt=4)
    r = ob.lba_solve(W)
    T = r["kf_Tcw"].reshape(-1, 16)
    fixed2 = W["kf_fixed"] == 2
    assert np.array_equal(T[fixed2], W["kf_Tcw"][fixed2])
    # the init KF (fixed, written back) only round-trips through SE3Quat
    assert np.abs(T[0] - W["kf_Tcw"][0]).max() < 1e-6


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def test_body_edge_initial_chi2_matches_numpy():
    """EdgeSE3ProjectXYZToBody (OptimizableTypes.h:117-144): obs - project2((mTrl * T_lw).map(X)),
    Huber as mono; checked against numpy on the composed SE3Quat."""
    W = synth.lba_window(45, n_kf=12, n_pt=200, obs_per_pt=5, body_frac=0.6)
    body = W["edge_body"].astype(bool)
    assert body.any()
    T = W["kf_Tcw"].reshape(-1, 4, 4).astype(np.float64)
    Trl = W["kf_Trl"].reshape(-1, 4, 4).astype(np.float64)
    fx2, fy2, cx2, cy2 = [float(c) for c in W["cam2"][:4]]
    chi = []
    for i in np.flatnonzero(body):
        k = W["edge_kf"][i]
        q1, q2 = _quat_from_R(Trl[k, :3, :3]), _quat_from_R(T[k, :3, :3])
        q = _qmul(q1, q2)
        q = (-q if q[3] < 0 else q) / np.linalg.norm(q)
        t = Trl[k, :3, 3] + _rot(q1) @ T[k, :3, 3]
        Xr = _rot(q) @ W["pt_pos"][W["edge_pt"][i]].astype(np.float64) + t
        e = W["edge_obs"][i, :2] - np.array([fx2 * Xr[0] / Xr[2] + cx2, fy2 * Xr[1] / Xr[2] + cy2])
        chi.append(float(e @ e) * float(W["edge_inv_sigma2"][i]))
    chi = np.array(chi)
    dm = float(f32(np.sqrt(5.991)))
    dsqr = float(f32(dm * dm))
    rob_body = np.where(chi <= dsqr, chi, 2 * np.sqrt(chi) * dm - dsqr).sum()
    Wm = {k: v for k, v in W.items() if k not in ("edge_body", "kf_Trl", "cam2")}
    for k in ("edge_pt", "edge_kf", "edge_obs", "edge_inv_sigma2"):
        Wm[k] = W[k][~body]
    r = ob.lba_solve(W, iters_first=1, iters_second=0)
    np.testing.assert_allclose(r["chi2_initial"], numpy_robust_chi2(Wm) + rob_body, rtol=1e-9)


def test_body_edge_identity_rig_equals_duplicate_mono_edge():
    """With mTrl = identity and camera2 = camera, a body edge is the same residual and Jacobian as
    a second mono edge on the left camera: both windows solve to the same estimate."""
    W = synth.lba_window(46, n_kf=10, n_pt=150, obs_per_pt=4, body_frac=0.5)
    Wb = dict(W)
    Wb["kf_Trl"] = np.tile(np.eye(4, dtype=np.float32).reshape(1, 16), (len(W["kf_fixed"]), 1))
    Wb["cam2"] = W["cam"]
    Wm = {k: v for k, v in Wb.items() if k not in ("edge_body", "kf_Trl", "cam2")}
    rb, rm = ob.lba_solve(Wb), ob.lba_solve(Wm)
    assert rb["iterations"] == rm["iterations"] and rb["trials"] == rm["trials"]
    assert np.array_equal(rb["edge_outlier"], rm["edge_outlier"])
    np.testing.assert_allclose(rb["chi2_final"], rm["chi2_final"], rtol=1e-9)
    assert np.abs(rb["kf_Tcw"] - rm["kf_Tcw"]).max() < 1e-6
    assert np.abs(rb["pt_pos"] - rm["pt_pos"]).max() < 1e-6


def test_body_edge_noise_free_window_converges():
    """Residual and Jacobians of the body edge agree with each other: a noise-free rig window
    converges to the ground truth."""
    W = synth.lba_window(47, n_kf=15, n_pt=400, obs_per_pt=6, outlier_frac=0.0, noise=0.0, body_frac=0.7)
    r = ob.lba_solve(W)
    assert r["chi2_final"] < 1e-6 * r["chi2_initial"]
    assert r["n_outlier"] == 0
    assert np.abs(r["pt_pos"] - W["gt_pts"]).max() < 1e-3
