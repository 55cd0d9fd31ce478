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
    assert g["n_outlier"] == 0 and g["iterations"] == (0, 0) and g["ran"] == 0
    _check(g, ob.lba_solve(W, stop=1))
    assert solver.solve(W)["ran"] == 1


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
    # a point seen twice by one free KeyFrame through non-adjacent edges (g2o would add two
    # Hessian blocks for one (pose, point) pair): refused by the host plan's KeyFrame stamps
    ekf = W["edge_kf"].copy()
    ept = W["edge_pt"]
    p0 = np.nonzero(np.bincount(ept) >= 3)[0][0]
    e = np.nonzero(ept == p0)[0]
    free = np.nonzero(W["kf_fixed"] == 0)[0]
    k = ekf[e[0]] if W["kf_fixed"][ekf[e[0]]] == 0 else free[0]
    ekf[e[0]] = ekf[e[2]] = k
    ekf[e[1]] = next(x for x in range(len(W["kf_fixed"])) if x != k)
    bad = dict(W, edge_kf=ekf)
    with pytest.raises(slamhot.SlamError):
        solver.solve(bad)
    # the same three edges with the repeated KeyFrame adjacent (a body edge's follower) pass
    ekf2 = ekf.copy()
    ekf2[e[1]], ekf2[e[2]] = ekf[e[2]], ekf[e[1]]
    solver.solve(dict(W, edge_kf=ekf2))


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
    """mbAbortBA set while the device LM loop runs: the solve stops early (g2o checks terminate()
    per iteration and per trial), every window's trajectory is a prefix of the unstopped one,
    outputs stay finite, and a stop inside optimize(5) skips optimize(10) (Optimizer.cc:
    1933-1935).  The caller's live bool is set by the solver's step hook
    (slam_lba_options.step_hook) once LM step k's counters are in, a known point of the loop
    instead of a wall-clock time; the solver then reads it like any other thread's write, so the
    stop lands within the steps already queued behind k (the host's ring, at most 3 more) — the
    bound is what is asserted, not an exact step."""
    import ctypes as C
    Ws = [synth.lba_window(200 + i, n_kf=20, n_pt=500, obs_per_pt=6, stereo_frac=0.2 * (i % 2)) for i in range(8)]
    flag = C.c_bool(False)
    run = solver.prepare(Ws, stop_flag=flag)
    n_full = run()
    full = run.results()
    steps = run.steps()
    assert steps >= 14 and not flag.value, steps
    for k in (0, 2, steps // 2, steps - 9):
        flag.value = False
        n_part = run(stop_at_step=k)
        part = run.results()
        assert flag.value and 0 < n_part < n_full, (k, n_part, n_full, steps)
        assert run.steps() <= k + 6, (k, run.steps())  # at most the ring of queued steps after the stop
        for f, p in zip(full, part):
            assert p["ran"] == 1
            assert p["iterations"][0] <= f["iterations"][0] and p["iterations"][1] <= f["iterations"][1]
            assert np.isfinite(p["kf_Tcw"]).all() and np.isfinite(p["pt_pos"]).all()
            if k <= 2:
                assert p["iterations"][1] == 0  # stopped inside optimize(5): optimize(10) skipped
            if p["iterations"] == f["iterations"] and p["trials"] == f["trials"]:
                assert np.array_equal(p["kf_Tcw"], f["kf_Tcw"]) and np.array_equal(p["pt_pos"], f["pt_pos"])
    flag.value = False
    assert run() == n_full  # the flag is re-read per call
    assert all(np.array_equal(a["kf_Tcw"], b["kf_Tcw"]) for a, b in zip(run.results(), full))


def test_lba_stop_flag_at_optimize5_boundary_deep_ring(solver):
    """A stop that lands on optimize(5)'s last step with more than 8 windows (the host keeps three
    steps in flight instead of two).  The step that ends optimize(5) starts optimize(10) on the
    device unless it has already seen the stop; the steps queued behind the hook's step before the
    flag was mirrored (at most depth - 1 = 2) run without seeing it.  Guaranteed: at most two
    iterations of optimize(10), every trajectory a prefix of the unstopped one, optimize(5)
    complete; the usual case (the next step's k_trial_control sees the flag) is one at most."""
    import ctypes as C
    base = synth.lba_window(300, n_kf=30, n_pt=800, obs_per_pt=6, stereo_frac=0.3)  # oracle: (5, 10) iterations
    Ws = [base] * 12  # identical windows: the batch moves in lock-step, one boundary step for all
    flag = C.c_bool(False)
    run = solver.prepare(Ws, stop_flag=flag)
    run()
    full = run.results()
    it5 = full[0]["iterations"][0]
    assert it5 == 5 and full[0]["iterations"][1] >= 6
    # the last step of optimize(5): the first stop step after which optimize(5) is complete
    kb = None
    for k in range(0, 40):
        flag.value = False
        run(stop_at_step=k)
        if run.results()[0]["iterations"][0] == it5:
            kb = k
            break
    assert kb is not None and kb >= 1  # optimize(5) completes from a stop a little before its last step (queued steps)
    for k in (kb, kb + 1):
        flag.value = False
        run(stop_at_step=k)
        for f, p in zip(full, run.results()):
            assert p["ran"] == 1 and p["iterations"][0] == it5
            assert p["iterations"][1] <= 2 + (k - kb), (k, kb, p["iterations"])
            assert p["iterations"][1] <= f["iterations"][1]
            assert np.isfinite(p["kf_Tcw"]).all() and np.isfinite(p["pt_pos"]).all()
    flag.value = False
    run(stop_at_step=kb)
    assert run.results()[0]["iterations"][1] <= 2


@pytest.mark.parametrize("kw", [dict(stereo_frac=0.3), dict(body_frac=0.4, stereo_frac=0.2), dict()])
def test_lba_camera_per_keyframe(solver, kw):
    """Every edge uses its own KeyFrame's camera (Optimizer.cc:1840, 1869-1873, 1906): a window
    whose odd KeyFrames carry a second calibration (kf_cam / kf_cam2) vs the oracle."""
    W = synth.lba_window(70, n_kf=24, n_pt=800, obs_per_pt=6, mixed_cams=True, **kw)
    assert len(np.unique(W["kf_cam"][:, 0])) == 2
    g = solver.solve(W)
    _check(g, ob.lba_solve(W))
    assert g["chi2_final"] < g["chi2_initial"]
    # the per-KeyFrame cameras matter: one camera for all would have been a different problem
    wrong = ob.lba_solve({k: v for k, v in W.items() if k not in ("kf_cam", "kf_cam2")})
    assert wrong["n_outlier"] > g["n_outlier"]


def test_lba_batch_of_different_calibrations(solver):
    """One batch holding windows of two different calibrations and a mixed one (configs[4]
    sequences of different cameras batched together; round 2 rejected such batches)."""
    Ws = [synth.lba_window(71, n_kf=14, n_pt=300, obs_per_pt=5),
          synth.lba_window(72, n_kf=14, n_pt=300, obs_per_pt=5, mixed_cams="all", stereo_frac=0.3),
          synth.lba_window(73, n_kf=16, n_pt=400, obs_per_pt=5, mixed_cams=True, body_frac=0.4),
          synth.lba_window(74, n_kf=12, n_pt=250, obs_per_pt=5, mixed_cams="all", body_frac=0.3)]
    assert Ws[1]["cam"][0] != Ws[0]["cam"][0]
    for W, g in zip(Ws, solver.solve(Ws)):
        _check(g, ob.lba_solve(W))


def test_lba_large_window_and_mixed_batch(solver):
    """5000 points: the per-pose point bitmaps span 79 words, so the device-built Schur
    contribution lists (k_ct_fill) take more than one 64-word pass; batched with a config-4
    window and a small one (different word counts per window)."""
    big = synth.lba_window(60, n_pt=5000)
    ws = [synth.lba_window(61, n_kf=12, n_pt=300, obs_per_pt=4), big, synth.lba_window(62)]
    gs = solver.solve(ws)
    for W, g in zip(ws, gs):
        _check(g, ob.lba_solve(W))


@pytest.mark.parametrize("kernel", ["rows", "blocks"])
def test_lba_schur_kernels(solver, monkeypatch, kernel):
    """Both Schur-complement kernels on one batch, forced through SLAMHOT_SCHUR: k_schur_rows
    (a workgroup per block row; the default from 256 free poses up) and k_schur_blocks (the default
    for a few windows).  The batch holds mono, stereo and rig (body-edge) config-4 windows, a
    5000-point window whose poses have ~830 edges each (W formed in three 384-edge chunks,
    recomputed per round), per-KeyFrame cameras and a small window."""
    monkeypatch.setenv("SLAMHOT_SCHUR", kernel)
    Ws = [synth.lba_window(0), synth.lba_window(3, stereo_frac=0.3),
          synth.lba_window(51, stereo_frac=0.3, body_frac=0.4), synth.lba_window(60, n_pt=5000),
          synth.lba_window(70, n_kf=24, n_pt=800, obs_per_pt=6, mixed_cams=True),
          synth.lba_window(61, n_kf=12, n_pt=300, obs_per_pt=4)]
    for W, g in zip(Ws, solver.solve(Ws)):
        _check(g, ob.lba_solve(W))


def test_lba_warmup_then_solve():
    """slamhot_lba_warmup (what slamhot::LocalBundleAdjuster runs at construction) leaves a handle
    whose next solve equals a fresh handle's and the oracle's (no state leaks from the synthetic
    window), and a smaller window after a larger one reuses the sized buffers."""
    import slamhot
    W = synth.lba_window(3, stereo_frac=0.3)
    fresh = slamhot.LocalBundleAdjustment()
    g0 = fresh.solve(W)
    fresh.close()
    warm = slamhot.LocalBundleAdjustment()
    warm.warmup(50, 2000, 8)
    g1 = warm.solve(W)
    small = synth.lba_window(4, n_kf=12, n_pt=300, obs_per_pt=5)
    g2 = warm.solve(small)
    warm.close()
    for k in ("kf_Tcw", "pt_pos", "edge_outlier"):
        assert np.array_equal(g0[k], g1[k]), k
    assert g0["iterations"] == g1["iterations"] and g0["trials"] == g1["trials"]
    _check(g1, ob.lba_solve(W))
    _check(g2, ob.lba_solve(small))
