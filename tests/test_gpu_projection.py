"""GPU parity: SearchByProjection (local map, last frame, keyframe) vs the CPU oracle."""
import numpy as np
import pytest

import oracle_bind as ob
import scenes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("th,far,nnratio", [(1.0, False, 0.8), (3.0, False, 0.8), (5.0, True, 0.9), (1.0, False, 0.6)])
def test_local_map(seed, th, far, nnratio):
    import slamhot
    S = scenes.scene(seed)
    fv, keep = scenes.frame_view(S, with_pose=False)
    mps, desc = scenes.local_map(S)
    m = slamhot.ORBmatcher(nnratio)
    ng, fg = m.SearchByProjection_local(fv, mps, desc, th, far, 20.0)
    no, fo = ob.search_by_projection_local(fv, mps, desc, nnratio, th, far, 20.0)
    m.close()
    assert ng == no and ng > 50
    assert np.array_equal(fg, fo)


@pytest.mark.parametrize("seed", [3, 4])
@pytest.mark.parametrize("th,mono,check_ori", [(7.0, False, True), (15.0, True, True), (7.0, False, False),
                                               (14.0, False, True)])
def test_last_frame(seed, th, mono, check_ori):
    import slamhot
    S = scenes.scene(seed)
    fv, keep = scenes.frame_view(S)
    lf, lkeep = scenes.last_frame(S, mono, motion=0.02 if seed == 3 else 0.2)
    m = slamhot.ORBmatcher(0.9, check_ori)
    ng, fg = m.SearchByProjection_last(fv, lf, th, mono)
    no, fo = ob.search_by_projection_last(fv, lf, 0.9, check_ori, th, mono)
    m.close()
    assert ng == no and no > 20
    assert np.array_equal(fg, fo)


@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("th,orb_dist", [(10.0, 100), (3.0, 64)])
def test_keyframe(seed, th, orb_dist):
    import slamhot
    S = scenes.scene(seed)
    fv, keep = scenes.frame_view(S)
    kf, kkeep = scenes.kf_points(S)
    m = slamhot.ORBmatcher(0.75, True)
    ng, fg = m.SearchByProjection_kf(fv, kf, th, orb_dist)
    no, fo = ob.search_by_projection_kf(fv, kf, 0.75, True, th, orb_dist)
    m.close()
    assert ng == no and no > 20
    assert np.array_equal(fg, fo)


@pytest.mark.parametrize("seed", [7, 8, 9])
@pytest.mark.parametrize("th,far", [(1.0, False), (3.0, True), (15.0, False)])
def test_search_local_points(seed, th, far):
    """Tracking::SearchLocalPoints: device isInFrustum + SearchByProjection vs the oracle's
    isInFrustum followed by its SearchByProjection."""
    import slamhot
    S = scenes.scene(seed)
    fv, keep = scenes.frame_view(S)
    geom, desc = scenes.local_map_geom(S)
    m = slamhot.ORBmatcher(0.8)
    ng, fg, ntg, trg = m.SearchLocalPoints(fv, geom, desc, th, far, 20.0)
    m.close()
    nto, tro = ob.is_in_frustum(fv, geom, 0.5)
    assert ntg == nto and nto > 300
    assert np.array_equal(trg["in_view"], tro["in_view"])
    # mTrackProjX/Y are written as soon as the point is in the image (Frame.cc:521-522)
    assert np.array_equal(trg["proj_x"], tro["proj_x"]) and np.array_equal(trg["proj_y"], tro["proj_y"])
    assert (trg["proj_x"][tro["in_view"] == 0] >= 0).sum() > 0
    v = tro["in_view"] == 1
    for f in ("proj_xr", "depth", "view_cos", "scale_level"):
        assert np.array_equal(trg[f][v], tro[f][v]), f
    no, fo = ob.search_by_projection_local(fv, tro, desc, 0.8, th, far, 20.0)
    assert ng == no and no > 50
    assert np.array_equal(fg, fo)


def test_local_map_above_lds_cap():
    """A local map whose resolution state (4 (2N + 2 nMP) bytes) exceeds the 150 KB LDS budget:
    the state moves to HBM and the matches stay the oracle's (the reference has no such limit)."""
    import slamhot
    S = scenes.scene(10)
    fv, keep = scenes.frame_view(S, with_pose=False)
    mps, desc = scenes.local_map(S, n_extra=20000)
    assert 4 * (2 * fv.n + 2 * len(mps)) > 150 * 1024
    m = slamhot.ORBmatcher(0.8)
    ng, fg = m.SearchByProjection_local(fv, mps, desc, 3.0, False, 20.0)
    no, fo = ob.search_by_projection_local(fv, mps, desc, 0.8, 3.0, False, 20.0)
    m.close()
    assert ng == no and ng > 50
    assert np.array_equal(fg, fo)


def test_search_local_points_batch():
    """slamhot_search_local_points_batch: many (Frame, local map) problems in one upload and two
    launches equal the single calls and the oracle, including a local map above the LDS budget."""
    import slamhot
    views, keeps, geoms, descs = [], [], [], []
    for seed in range(20, 28):
        S = scenes.scene(seed)
        fv, keep = scenes.frame_view(S)
        geom, desc = scenes.local_map_geom(S, n_extra=300 if seed != 25 else 12000)
        views.append(fv)
        keeps.append((S, keep))
        geoms.append(geom)
        descs.append(desc)
    m = slamhot.ORBmatcher(0.8)
    out = m.SearchLocalPoints_batch(views, geoms, descs, 1.0, False, 20.0)
    for i, (nm, fm, nt) in enumerate(out):
        ns, fs, nts, _ = m.SearchLocalPoints(views[i], geoms[i], descs[i], 1.0, False, 20.0)
        assert (nm, nt) == (ns, nts) and np.array_equal(fm, fs), i
        nto, tro = ob.is_in_frustum(views[i], geoms[i], 0.5)
        no, fo = ob.search_by_projection_local(views[i], tro, descs[i], 0.8, 1.0, False, 20.0)
        assert nt == nto and nm == no and np.array_equal(fm, fo), i
    m.close()


def test_search_by_projection_last_batch():
    """slamhot_search_by_projection_last_batch (TrackWithMotionModel's matcher over many frames in
    one launch) equals the single calls and the oracle, at th 7 and its 2th retry, mono and stereo,
    with and without the rotation check."""
    import slamhot
    views, lfs, keeps = [], [], []
    for seed in range(40, 52):
        S = scenes.scene(seed)
        fv, keep = scenes.frame_view(S)
        lf, lkeep = scenes.last_frame(S, mono=False, motion=(0.02, 0.2, 0.6)[seed % 3])
        views.append(fv)
        lfs.append(lf)
        keeps.append((S, keep, lkeep))
    for th, mono, ori in [(7.0, False, True), (14.0, False, True), (15.0, True, False)]:
        m = slamhot.ORBmatcher(0.9, ori)
        out = m.SearchByProjection_last_batch(views, lfs, th, mono)
        assert len(out) == len(views)
        for i, (nm, fm) in enumerate(out):
            ns, fs = m.SearchByProjection_last(views[i], lfs[i], th, mono)
            no, fo = ob.search_by_projection_last(views[i], lfs[i], 0.9, ori, th, mono)
            assert nm == ns == no and np.array_equal(fm, fs) and np.array_equal(fm, fo), (th, mono, ori, i)
        assert sum(nm for nm, _ in out) > 20 * len(out)
        m.close()


def test_search_by_projection_kf_batch():
    """slamhot_search_by_projection_kf_batch (Relocalization's projection matcher, batched) equals
    the single calls and the oracle at both of the reference's (th, ORBdist) settings."""
    import slamhot
    views, kfs, keeps = [], [], []
    for seed in range(60, 70):
        S = scenes.scene(seed)
        fv, keep = scenes.frame_view(S)
        kf, kkeep = scenes.kf_points(S)
        views.append(fv)
        kfs.append(kf)
        keeps.append((S, keep, kkeep))
    m = slamhot.ORBmatcher(0.75, True)
    for th, orb_dist in [(10.0, 100), (3.0, 64)]:  # Tracking.cc:3538, :3563
        out = m.SearchByProjection_kf_batch(views, kfs, th, orb_dist)
        for i, (nm, fm) in enumerate(out):
            ns, fs = m.SearchByProjection_kf(views[i], kfs[i], th, orb_dist)
            no, fo = ob.search_by_projection_kf(views[i], kfs[i], 0.75, True, th, orb_dist)
            assert nm == ns == no and np.array_equal(fm, fs) and np.array_equal(fm, fo), (th, orb_dist, i)
    m.close()


def test_projection_batches_empty_and_degenerate():
    """Empty batch, a frame with no last-frame MapPoints and a KeyFrame with nothing usable."""
    import slamhot
    m = slamhot.ORBmatcher(0.9, True)
    assert m.SearchByProjection_last_batch([], [], 7.0, False) == []
    S = scenes.scene(80)
    fv, keep = scenes.frame_view(S)
    lf, lkeep = scenes.last_frame(S)
    lkeep[3][:] = 0  # has_mp: no MapPoints at all
    kf, kkeep = scenes.kf_points(S)
    kkeep[1][:] = 0  # use
    (n1, f1), = m.SearchByProjection_last_batch([fv], [lf], 7.0, False)
    (n2, f2), = m.SearchByProjection_kf_batch([fv], [kf], 10.0, 100)
    assert n1 == 0 and n2 == 0 and (f1 == -1).all() and (f2 == -1).all()
    m.close()


@pytest.mark.parametrize("kind", ["last", "kf", "local"])
def test_projection_batches_threaded_staging(kind):
    """Batches large enough for the threaded staging (a frame count of at least 16 spreads the
    pinned-image copies over up to 8 host threads: matcher.hip staged_upload), one frame above
    kGridSortMax (4096 features: its grid is built on the host while the others' are built on the
    device): every frame equals the single call and the oracle."""
    import slamhot
    nfr = 64
    views, others, descs = [], [], []
    for i in range(nfr):
        S = scenes.scene(100 + i, n_feat=7000 if i == 37 else 1200)
        fv, keep = scenes.frame_view(S)
        views.append(fv)
        if kind == "last":
            lf, lkeep = scenes.last_frame(S, mono=False, motion=(0.02, 0.2)[i % 2])
            others.append((lf, lkeep, keep))
        elif kind == "kf":
            kf, kkeep = scenes.kf_points(S)
            others.append((kf, kkeep, keep))
        else:
            geom, desc = scenes.local_map_geom(S, n_extra=300)
            others.append((geom, keep))
            descs.append(desc)
    assert views[37].n > 4096
    if kind == "last":
        m = slamhot.ORBmatcher(0.9, True)
        out = m.SearchByProjection_last_batch(views, [o[0] for o in others], 7.0, False)
        for i, (nm, fm) in enumerate(out):
            ns, fs = m.SearchByProjection_last(views[i], others[i][0], 7.0, False)
            no, fo = ob.search_by_projection_last(views[i], others[i][0], 0.9, True, 7.0, False)
            assert nm == ns == no and np.array_equal(fm, fs) and np.array_equal(fm, fo), i
    elif kind == "kf":
        m = slamhot.ORBmatcher(0.75, True)
        out = m.SearchByProjection_kf_batch(views, [o[0] for o in others], 10.0, 100)
        for i, (nm, fm) in enumerate(out):
            ns, fs = m.SearchByProjection_kf(views[i], others[i][0], 10.0, 100)
            no, fo = ob.search_by_projection_kf(views[i], others[i][0], 0.75, True, 10.0, 100)
            assert nm == ns == no and np.array_equal(fm, fs) and np.array_equal(fm, fo), i
    else:
        m = slamhot.ORBmatcher(0.8)
        geoms = [o[0] for o in others]
        out = m.SearchLocalPoints_batch(views, geoms, descs, 1.0, False, 20.0)
        for i, (nm, fm, nt) in enumerate(out):
            ns, fs, nts, _ = m.SearchLocalPoints(views[i], geoms[i], descs[i], 1.0, False, 20.0)
            assert (nm, nt) == (ns, nts) and np.array_equal(fm, fs), i
            nto, tro = ob.is_in_frustum(views[i], geoms[i], 0.5)
            no, fo = ob.search_by_projection_local(views[i], tro, descs[i], 0.8, 1.0, False, 20.0)
            assert nt == nto and nm == no and np.array_equal(fm, fo), i
    m.close()
