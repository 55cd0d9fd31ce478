"""GPU parity of the local-BA LM/Schur solve (slamhot_lba_solve) against the CPU restatement
of g2o (oracle/lba_oracle.cpp), through the C-ABI.

Tolerance (BASELINE.json north_star): poses and points within 1e-5.  Both sides compute in
FP64 with the same float quirks; they differ only in summation order and in the linear solver
(dense blocked LDL^T on the device, dense natural-order LDL^T in the oracle), so the LM
decisions (accept / reject, iteration counts, outlier sets) are expected to agree exactly."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module")
def solver():
    import slamhot
    s = slamhot.LocalBundleAdjustment()
    yield s
    s.close()


def _check(g, o, chi_rtol=1e-8):
    assert g["iterations"] == o["iterations"]
    assert g["trials"] == o["trials"]
    np.testing.assert_allclose(g["chi2_initial"], o["chi2_initial"], rtol=chi_rtol)
    np.testing.assert_allclose(g["chi2_final"], o["chi2_final"], rtol=chi_rtol)
    np.testing.assert_allclose(g["lambda_final"], o["lambda_final"], rtol=1e-6)
    assert np.array_equal(g["edge_outlier"], o["edge_outlier"])
    assert g["n_outlier"] == o["n_outlier"]
    assert np.abs(g["kf_Tcw"].astype(np.float64) - o["kf_Tcw"]).max() <= TOL
    assert np.abs(g["pt_pos"].astype(np.float64) - o["pt_pos"]).max() <= TOL


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lba_full_window_mono(solver, seed):
    """Config 4: 50 KF x 2000 points x 8 obs, 2% outliers, 48 free KFs."""
    W = synth.lba_window(seed)
    g = solver.solve(W)
    o = ob.lba_solve(W)
    _check(g, o)
    assert g["chi2_final"] < g["chi2_initial"]


@pytest.mark.parametrize("seed", [3, 4])
def test_lba_full_window_stereo(solver, seed):
    """Variant 4b: 30% stereo observations (float invz, float bf*invz quirk)."""
    W = synth.lba_window(seed, stereo_frac=0.3)
    g = solver.solve(W)
    o = ob.lba_solve(W)
    _check(g, o)


@pytest.mark.parametrize("seed,stereo", [(50, 0.0), (51, 0.3)])
def test_lba_full_window_body_edges(solver, seed, stereo):
    """EdgeSE3ProjectXYZToBody (C4): KeyFrames with a second pinhole camera, 40% of the left
    observations followed by a right-camera observation through mTrl."""
    W = synth.lba_window(seed, stereo_frac=stereo, body_frac=0.4)
    assert W["edge_body"].sum() > 1000
    g = solver.solve(W)
    o = ob.lba_solve(W)
    _check(g, o)
    assert g["chi2_final"] < g["chi2_initial"]


def test_lba_batch_mixed_body_and_plain(solver):
    """A batch mixing rig windows (body edges) and single-camera windows."""
    Ws = [synth.lba_window(60 + i, n_kf=10 + 3 * i, n_pt=200 + 50 * i, obs_per_pt=5,
                           body_frac=0.5 if i % 2 == 0 else 0.0, stereo_frac=0.2 * (i % 3)) for i in range(5)]
    for W, g in zip(Ws, solver.solve(Ws)):
        _check(g, ob.lba_solve(W))


def test_lba_small_windows(solver):
    for seed in range(5, 11):
        W = synth.lba_window(seed, n_kf=8 + seed, n_pt=150 + 20 * seed, obs_per_pt=4, stereo_frac=0.2 * (seed % 2))
        _check(solver.solve(W), ob.lba_solve(W))


def test_lba_batch_matches_single(solver):
    """Batched mode: independent windows in one call give the per-window answers."""
    Ws = [synth.lba_window(20 + i, n_kf=10 + 7 * i, n_pt=300 + 100 * i, obs_per_pt=5) for i in range(5)]
    gs = solver.solve(Ws)
    for W, g in zip(Ws, gs):
        _check(g, ob.lba_solve(W))


def test_lba_user_lambda_and_schedule(solver):
    W = synth.lba_window(30, n_kf=20, n_pt=500, obs_per_pt=6)
    for kw in [dict(user_lambda_init=100.0), dict(iters_first=2, iters_second=0), dict(iters_first=0, iters_second=3)]:
        _check(solver.solve(W, **kw), ob.lba_solve(W, **kw))


def test_lba_stop_flag_before_start(solver):
    """*pbStopFlag set before optimize: LocalBundleAdjustment returns without writing back."""
    W = synth.lba_window(31, n_kf=12, n_pt=200, obs_per_pt=4)
    g = solver.solve(W, stop_flag=1)
    assert np.array_equal(g["kf_Tcw"], W["kf_Tcw"])
    assert np.array_equal(g["pt_pos"], W["pt_pos"])
    assert g["n_outlier"] == 0 and g["iterations"] == (0, 0)
    _check(g, ob.lba_solve(W, stop=1))


def test_lba_degenerate_windows(solver):
    """All KFs fixed (points only), a free KF without edges, and an empty edge set."""
    W = synth.lba_window(32, n_kf=10, n_pt=120, obs_per_pt=4)
    Wf = dict(W, kf_fixed=np.where(W["kf_fixed"] == 0, 2, W["kf_fixed"]).astype(np.uint8))
    _check(solver.solve(Wf), ob.lba_solve(Wf))
    # drop every edge of KF 5: it becomes an inactive vertex
    keep = W["edge_kf"] != 5
    We = dict(W, edge_pt=W["edge_pt"][keep], edge_kf=W["edge_kf"][keep], edge_obs=W["edge_obs"][keep],
              edge_inv_sigma2=W["edge_inv_sigma2"][keep])
    _check(solver.solve(We), ob.lba_solve(We))
    W0 = dict(W, edge_pt=W["edge_pt"][:0], edge_kf=W["edge_kf"][:0], edge_obs=W["edge_obs"][:0],
              edge_inv_sigma2=W["edge_inv_sigma2"][:0])
    _check(solver.solve(W0), ob.lba_solve(W0))


def test_lba_rejects_bad_input(solver):
    import slamhot
    W = synth.lba_window(33, n_kf=8, n_pt=60, obs_per_pt=3)
    bad = dict(W, edge_pt=W["edge_pt"][::-1].copy())  # not point-major
    with pytest.raises(slamhot.SlamError):
        solver.solve(bad)
    bad = dict(W, edge_kf=np.full_like(W["edge_kf"], 99))
    with pytest.raises(slamhot.SlamError):
        solver.solve(bad)


def test_lba_deterministic(solver):
    W = synth.lba_window(34)
    a, b = solver.solve(W), solver.solve(W)
    assert np.array_equal(a["kf_Tcw"], b["kf_Tcw"]) and np.array_equal(a["pt_pos"], b["pt_pos"])


def test_lba_stop_flag_bool_before_start(solver):
    """The reference's bool* pbStopFlag passed as is (slam_lba_options.stop_flag_bool)."""
    import ctypes as C
    W = synth.lba_window(33, n_kf=12, n_pt=200, obs_per_pt=4)
    g = solver.solve(W, stop_flag=C.c_bool(True))
    _check(g, ob.lba_solve(W, stop=1))
    _check(solver.solve(W, stop_flag=C.c_bool(False)), ob.lba_solve(W))


def test_lba_per_window_lambda(solver):
    """Batched windows of different maps: each window's pMap->IsInertial() sets its own lambda0."""
    Ws = [dict(synth.lba_window(40 + i, n_kf=10 + 3 * i, n_pt=250, obs_per_pt=5), user_lambda_init=100.0 * (i % 2))
          for i in range(4)]
    for W, g in zip(Ws, solver.solve(Ws)):
        _check(g, ob.lba_solve(W))
    g1 = solver.solve(Ws[1])
    _check(g1, ob.lba_solve(Ws[1], user_lambda_init=100.0))


def test_lba_stop_flag_mid_solve(solver):
    """mbAbortBA set by another thread while the device LM loop runs: the solve stops early (g2o
    checks terminate() per iteration and per trial), every window's trajectory is a prefix of the
    unstopped one, and outputs stay finite.  The flag is the caller's live bool; it is set at a
    sweep of delays across the call so that at least one lands inside the LM loop."""
    import ctypes as C
    import threading
    import time
    Ws = [synth.lba_window(200 + i, n_kf=30, n_pt=1200, obs_per_pt=6) for i in range(96)]
    flag = C.c_bool(False)
    run = solver.prepare(Ws, stop_flag=flag)
    n_full = run()
    full = run.results()
    t0 = time.perf_counter()
    run()
    t_call = time.perf_counter() - t0
    dev_ms, plan_ms, _ = solver.last_stats()
    partial = []
    for frac in np.linspace(0.3, 0.98, 12):
        flag.value = False
        timer = threading.Timer(frac * t_call, lambda: setattr(flag, "value", True))
        timer.start()
        n_part = run()
        timer.join()
        part = run.results()
        assert n_part <= n_full
        for f, p in zip(full, part):
            assert p["iterations"][0] <= f["iterations"][0] and p["iterations"][1] <= f["iterations"][1]
            assert np.isfinite(p["kf_Tcw"]).all() and np.isfinite(p["pt_pos"]).all()
            if p["iterations"] == f["iterations"] and p["trials"] == f["trials"]:
                assert np.array_equal(p["kf_Tcw"], f["kf_Tcw"]) and np.array_equal(p["pt_pos"], f["pt_pos"])
        partial.append(n_part)
    flag.value = False
    assert run() == n_full  # the flag is re-read per call
    assert any(0 < n < n_full for n in partial), (partial, n_full, t_call, dev_ms, plan_ms)


def test_lba_large_window_and_mixed_batch(solver):
    """5000 points: the per-pose point bitmaps span 79 words, so the device-built Schur
    contribution lists (k_ct_fill) take more than one 64-word pass; batched with a config-4
    window and a small one (different word counts per window)."""
    big = synth.lba_window(60, n_pt=5000)
    ws = [synth.lba_window(61, n_kf=12, n_pt=300, obs_per_pt=4), big, synth.lba_window(62)]
    gs = solver.solve(ws)
    for W, g in zip(ws, gs):
        _check(g, ob.lba_solve(W))
