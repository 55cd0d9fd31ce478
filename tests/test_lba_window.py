"""Window construction of Optimizer::LocalBundleAdjustment (Optimizer.cc:1613-1718) in the host
mirror (slamhot/optimizer.py), its flattening into slam_lba_problem, and (GPU) the full mirror
against a direct slamhot_lba_solve of the same window."""
import numpy as np
import pytest

from slamhot import optimizer as opt
from slamhot import synth


def _window():
    return synth.lba_window(50, n_kf=10, n_pt=120, obs_per_pt=4)


def test_fallback_moves_lowest_local_kf_to_fixed():
    W = _window()
    pmap, kfs, mps = opt.map_from_window(W)
    local, fixed, local_mps, nfix = opt.build_window(kfs[-1], pmap)
    # every KF is covisible with the current one: no fixed cameras, the init KF counts as 1,
    # so the lowest-id other local KF (id 1) is moved to the fixed list (:1676-1711)
    assert nfix == 2
    assert [k.mnId for k in fixed] == [1]
    assert sorted(k.mnId for k in local) == [0] + list(range(2, 10))
    # lLocalMapPoints: first-seen order over the local KFs (current KF first, :1631-1655)
    expect, seen = [], set()
    for k in [kfs[-1]] + kfs[-1].covisible:
        for mp in k.mvpMapPoints:
            if mp is not None and mp.mnId not in seen:
                seen.add(mp.mnId)
                expect.append(mp.mnId)
    assert [mp.mnId for mp in local_mps] == expect
    Wf, kf_order, refs = opt.flatten_window(local, fixed, local_mps, pmap)
    assert np.array_equal(Wf["kf_fixed"], W["kf_fixed"])  # KF 0 init-fixed, KF 1 fixed camera
    assert np.array_equal(Wf["kf_Tcw"], W["kf_Tcw"])
    # same edge set, point-major in first-seen order, KFs ascending inside a point
    ids = np.array([mp.mnId for mp in local_mps])
    got = sorted(zip(ids[Wf["edge_pt"]].tolist(), Wf["edge_kf"].tolist(), Wf["edge_obs"][:, 0].tolist()))
    ref = sorted(zip(W["edge_pt"].tolist(), W["edge_kf"].tolist(), W["edge_obs"][:, 0].tolist()))
    assert got == ref
    assert np.all(np.diff(Wf["edge_pt"]) >= 0)


def test_partial_covisibility_yields_fixed_cameras():
    W = _window()
    pmap, kfs, mps = opt.map_from_window(W, covis_order=[])
    kfs[-1].covisible = [kfs[8], kfs[7]]
    local, fixed, local_mps, nfix = opt.build_window(kfs[-1], pmap)
    assert [k.mnId for k in local] == [9, 8, 7]
    # every other KF observing a local point is a fixed camera, in first-seen order
    assert nfix == len(fixed) >= 2
    assert all(k.mnId not in (7, 8, 9) for k in fixed)
    seen = set()
    order = []
    for mp in local_mps:
        for k in mp.GetObservations():
            if k.mnId not in (7, 8, 9) and k.mnId not in seen:
                seen.add(k.mnId)
                order.append(k.mnId)
    assert [k.mnId for k in fixed] == order


def test_bad_and_foreign_keyframes_are_excluded():
    W = _window()
    pmap, kfs, mps = opt.map_from_window(W)
    kfs[4].bad = True
    kfs[5].map = opt.Map(init_kf_id=99)
    mps[0].bad = True
    local, fixed, local_mps, nfix = opt.build_window(kfs[-1], pmap)
    ids = {k.mnId for k in local} | {k.mnId for k in fixed}
    assert 4 not in ids and 5 not in ids
    assert all(mp.mnId != 0 for mp in local_mps)


def test_lonely_keyframe_aborts():
    pmap = opt.Map(init_kf_id=0)
    keys = np.zeros(1, dtype=[("x", "<f4"), ("y", "<f4"), ("octave", "<i4")])
    kf = opt.KeyFrame(5, np.eye(4), keys, [-1.0], [1.0], (400, 400, 300, 200, 40), pmap)
    mp = opt.MapPoint(0, [0, 0, 2], pmap)
    kf.mvpMapPoints[0] = mp
    mp.AddObservation(kf, 0)
    assert opt.build_window(kf, pmap) is None  # 0 fixed KFs: LBA aborted (:1714-1718)


@pytest.mark.gpu
def test_mirror_equals_direct_solve():
    import slamhot
    W = synth.lba_window(51, n_kf=12, n_pt=300, obs_per_pt=5, stereo_frac=0.3)
    S = slamhot.LocalBundleAdjustment()
    direct = S.solve(W)
    pmap, kfs, mps = opt.map_from_window(W)
    counts = opt.LocalBundleAdjustment(kfs[-1], False, pmap, S)
    assert counts == (2, 11, 300, len(W["edge_pt"]))
    # the mirror feeds points in first-seen order (the synthetic window is id-ordered), so
    # only summation order differs: within the LBA tolerance
    for i, k in enumerate(kfs):
        if W["kf_fixed"][i] != 2:
            assert np.abs(k.GetPose().reshape(-1) - direct["kf_Tcw"][i]).max() <= 1e-5
        else:
            assert np.array_equal(k.GetPose().reshape(-1), W["kf_Tcw"][i])
    for i, mp in enumerate(mps):
        assert np.abs(mp.GetWorldPos() - direct["pt_pos"][i]).max() <= 1e-5
    n_obs = sum(len(mp.observations) for mp in mps)
    assert n_obs == len(W["edge_pt"]) - direct["n_outlier"]
    assert pmap.change_index == 1
    S.close()


def test_fuse_apply_order_and_replace():
    """ORBmatcher::Fuse's update half (ORBmatcher.cc:1789-1816): Replace keeps the MapPoint
    with more observations, a replaced MapPoint later in the list is skipped, a MapPoint that
    entered the KeyFrame earlier in the call is skipped, free slots get AddObservation."""
    import numpy as np

    from slamhot.optimizer import KeyFrame, Map, MapPoint, fuse_apply
    pmap = Map()
    keys = np.zeros(4, dtype=[("x", "<f4"), ("y", "<f4"), ("octave", "<i4")])
    cam = (400.0, 400.0, 320.0, 240.0, 40.0)
    kf = KeyFrame(0, np.eye(4), keys, [-1, 5.0, -1, -1], np.ones(8), cam, pmap)
    other = KeyFrame(1, np.eye(4), keys, [-1, -1, -1, -1], np.ones(8), cam, pmap)
    b = MapPoint(10, [0, 0, 1], pmap)            # in kf slot 0, 1 observation
    kf.mvpMapPoints[0] = b
    b.AddObservation(kf, 0)
    a = MapPoint(11, [0, 0, 1], pmap)            # 2 observations elsewhere -> survives
    a.AddObservation(other, 0)
    a.AddObservation(KeyFrame(2, np.eye(4), keys, [-1] * 4, np.ones(8), cam, pmap), 1)
    other.mvpMapPoints[0] = a
    c = MapPoint(12, [0, 0, 1], pmap)            # free slot 2
    d = MapPoint(13, [0, 0, 1], pmap)            # also matches slot 2 (after c entered)
    e = MapPoint(14, [0, 0, 1], pmap)            # too far
    n = fuse_apply(kf, [a, b, c, d, e, None], [0, 0, 2, 2, 3, -1], [10, 10, 20, 30, 51, 256])
    assert n == 3                                # a (replace), c (add), d (slot 2 now holds c: replace)
    assert b.isBad() and kf.GetMapPoint(0) is a and a.IsInKeyFrame(kf)
    # c has one observation, d none: d.Observations() = 0 < 1 -> c.Replace(d)? no: pMPinKF=c has
    # more (1 > 0), so d.Replace(c): d turns bad, c keeps the slot
    assert d.isBad() and kf.GetMapPoint(2) is c
    assert not e.IsInKeyFrame(kf)
