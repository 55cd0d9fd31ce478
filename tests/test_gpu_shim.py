"""GPU: the drop-in shim bodies (include/slamhot_orbslam3.hpp) compiled against ORB-SLAM3
stand-ins and run through tests/cpp/shim_driver give the same map updates as the Python mirror
over the same device solver: Optimizer::LocalBundleAdjustment (window, solve, vToErase, pose and
point write-back, UpdateNormalAndDepth, IncreaseChangeIndex) and Optimizer::PoseOptimization."""
import numpy as np
import pytest

import oracle_bind as ob
import shim_io
import slamhot
from slamhot import optimizer as opt
from slamhot import synth

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not shim_io.DRIVER.exists(), reason="shim_driver not built")]


@pytest.mark.parametrize("seed,kw", [(80, dict(n_kf=14, n_pt=400, obs_per_pt=5, stereo_frac=0.3)),
                                     (81, dict(n_kf=12, n_pt=300, obs_per_pt=5, body_frac=0.5))])
def test_shim_local_bundle_adjustment_equals_mirror(seed, kw, tmp_path):
    import slamhot
    W = synth.lba_window(seed, **kw)
    pmap, kfs, mps = opt.map_from_window(W)
    shim_io.write_map(tmp_path / "map.bin", pmap, kfs, mps)
    b = shim_io.run("lba", tmp_path / "map.bin", tmp_path / "out.bin")
    counts = (b.i32(), b.i32(), b.i32(), b.i32())
    change = b.i32()
    T, P, obs, upd = b.vec("<f4"), b.vec("<f4"), b.vec("<i4"), b.vec("<i4")
    S = slamhot.LocalBundleAdjustment()
    mcounts = opt.LocalBundleAdjustment(kfs[-1], False, pmap, S)
    S.close()
    assert counts == mcounts and change == pmap.change_index == 1
    assert np.array_equal(T.reshape(-1, 4, 4), np.stack([k.GetPose() for k in kfs]))
    assert np.array_equal(P.reshape(-1, 3), np.stack([m.GetWorldPos() for m in mps]))
    mobs = sorted((k.mnId, m.mnId) for m in mps for k in m.observations)
    assert sorted(map(tuple, obs.reshape(-1, 2))) == mobs
    assert np.array_equal(upd, [m.normal_updates for m in mps])
    assert len(mobs) < sum(len(m.observations) for m in opt.map_from_window(W)[2])  # outliers erased


def _write_pose_frame(path, f):
    import struct
    n = len(f["kps"])
    b = bytearray(struct.pack("<i", n))
    b += np.asarray(f["Tcw"], np.float32).tobytes() + np.asarray(f["cam"], np.float32).tobytes()
    b += np.asarray(f["inv_sigma2"], np.float32).tobytes()
    for i in range(n):
        kp = f["kps"][i]
        b += struct.pack("<ffifi", kp["x"], kp["y"], int(kp["octave"]), f["uright"][i], int(f["has_mp"][i]))
        b += np.asarray(f["mp_pos"][i], np.float32).tobytes()
    path.write_bytes(bytes(b))


def test_shim_pose_optimization_too_few_correspondences(tmp_path):
    """Below 3 correspondences PoseOptimization returns 0 with the pose untouched, but its edge
    loop has already set mvbOutlier[i] = false for every feature with a MapPoint
    (Optimizer.cc:864-1013); the driver starts from stale `true` flags."""
    f = synth.pose_frame(91, stereo_frac=0.3)
    has = np.zeros(len(f["kps"]), np.uint8)
    has[[5, 17]] = 1
    f["has_mp"] = has
    _write_pose_frame(tmp_path / "f.bin", f)
    r = shim_io.run("pose", tmp_path / "f.bin", tmp_path / "o.bin")
    ninl, T, outl = r.i32(), r.vec("<f4"), r.vec("u1")
    assert ninl == 0
    assert np.array_equal(T.reshape(4, 4), np.asarray(f["Tcw"], np.float32).reshape(4, 4))
    assert not outl[has.astype(bool)].any() and outl[~has.astype(bool)].all()


def test_shim_pose_optimization_equals_device_and_oracle(tmp_path):
    import slamhot
    f = synth.pose_frame(90, stereo_frac=0.3)
    _write_pose_frame(tmp_path / "f.bin", f)
    r = shim_io.run("pose", tmp_path / "f.bin", tmp_path / "o.bin")
    ninl, T, outl = r.i32(), r.vec("<f4"), r.vec("u1")
    S = slamhot.PoseOptimizer()
    g = S.solve(f)
    S.close()
    assert ninl == g["n_inliers"]
    assert np.array_equal(T.reshape(4, 4), np.asarray(g["Tcw"]).reshape(4, 4))
    has = f["has_mp"].astype(bool)
    assert np.array_equal(outl[has], np.asarray(g["outlier"])[has])
    o = ob.pose_optimization(f)
    assert o["n_inliers"] == ninl
    assert np.abs(T.reshape(4, 4) - np.asarray(o["Tcw"]).reshape(4, 4)).max() <= 1e-5


def _bow_side_bytes(kps, desc, valid, fv):
    import struct
    node_id, node_off, node_feat = fv
    b = bytearray(struct.pack("<i", len(desc))) + np.ascontiguousarray(desc, np.uint8).tobytes()
    b += np.asarray(kps["angle"], np.float32).tobytes()
    if valid is not None:
        b += np.asarray(valid, np.uint8).tobytes()
    b += struct.pack("<i", len(node_id)) + np.asarray(node_id, np.uint32).tobytes()
    b += np.asarray(node_off, np.int32).tobytes() + np.asarray(node_feat, np.uint32).tobytes()
    return bytes(b)


def test_shim_search_by_bow_ratio_per_call(tmp_path):
    """The reference constructs ORBmatcher(0.7, true) in TrackReferenceKeyFrame (Tracking.cc:2566)
    and ORBmatcher(0.75, true) in Relocalization (:3475) on the same Tracking thread: the binding of
    INTEGRATION.md must run each SearchByBoW at its own matcher's ratio (the device handle is shared
    per thread, the ratio is not)."""
    import struct
    par, leaf, vd, vw = synth.vocab(10, 4, 3)
    img0 = synth.frame(21, 752, 480)
    img1 = synth.shifted(img0, 3, 2, 4.0, 5)
    k0, d0, _ = ob.extract(img0, ob.params(nfeatures=1200))
    k1, d1, _ = ob.extract(img1, ob.params(nfeatures=1200))
    fv = []
    for d in (d0, d1):
        _, wt, nid = ob.vocab_transform(par, leaf, vd, vw, 4, d, 2)
        fv.append(synth.feature_vector(nid, wt))
    valid = (np.random.default_rng(4).random(len(k0)) < 0.85).astype(np.uint8)
    calls = [(0.7, True), (0.75, True), (0.7, True), (0.9, False)]
    b = struct.pack("<i", len(calls)) + b"".join(struct.pack("<fi", r, int(c)) for r, c in calls)
    b += _bow_side_bytes(k0, d0, valid, fv[0]) + _bow_side_bytes(k1, d1, None, fv[1])
    (tmp_path / "pair.bin").write_bytes(b)
    r = shim_io.run("bow", tmp_path / "pair.bin", tmp_path / "o.bin")
    A = (d0, k0["angle"], valid) + fv[0]
    B = (d1, k1["angle"], None) + fv[1]
    got = []
    for ratio, ori in calls:
        n, idx = r.i32(), r.vec("<i4")
        no, _, b2a = ob.search_by_bow(A, B, ratio, ori, False)
        assert n == no and np.array_equal(idx, b2a), (ratio, ori)
        got.append(n)
    assert got[0] != got[1], "the fixture must separate the two ratios"


# ---------------------------------------------------------------- every other shim body
import scenes  # noqa: E402


def _ids(initial_state, base):
    return np.where(initial_state >= 0, base + np.arange(len(initial_state)), -1)


def _expect_projection(fo, init_ids, mp_ids):
    """CurrentFrame.mvpMapPoints after SearchByProjection: the matched MapPoint (fo >= 0), NULL where
    the rotation check dropped an assignment (fo == -2), else what the entry held before."""
    return np.where(fo >= 0, mp_ids[np.maximum(fo, 0)], np.where(fo == -2, -1, init_ids))


def test_shim_search_by_projection_last_frame(tmp_path):
    """ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:2173-2389)
    through the reference-typed shim: the last frame's mvpMapPoints / mvbOutlier become the
    matcher's input, the matches (and the rotation check's NULLs) land in CurrentFrame.mvpMapPoints.
    TrackWithMotionModel's th 7 / 2th retry, mono th 15, without the rotation check."""
    total_null = 0
    for seed, motion in ((3, 0.02), (4, 0.2)):
        S = scenes.scene(seed)
        fv, keep = scenes.frame_view(S)
        lf, lk = scenes.last_frame(S, mono=False, motion=motion)
        Tl, kl, klu, has, outl, pos, desc, obs = lk
        calls = [(7.0, 0, 0.9, 1), (14.0, 0, 0.9, 1), (15.0, 1, 0.9, 1), (7.0, 0, 0.9, 0)]
        o = shim_io.Out()
        shim_io.write_frame(o, fv, S["k"], S["k"], S["uright"], S["d"], S["state"], np.zeros(len(S["k"])), S["Tcw"])
        o.i32(len(kl)).raw(Tl, np.float32)
        rec = np.zeros(len(kl), np.dtype([("k", "V28"), ("ku", "V28"), ("h", "u1"), ("o", "u1"), ("b", "u1"),
                                          ("p", "<f4", 3), ("d", "u1", 32)]))
        rec["k"], rec["ku"] = kl.view("V28"), klu.view("V28")
        rec["h"], rec["o"], rec["b"], rec["p"], rec["d"] = has, outl, obs, pos, desc
        o.raw(rec).i32(len(calls))
        for th, mono, ratio, ori in calls:
            o.f32(th).i32(mono).f32(ratio).i32(ori)
        r = shim_io.run_any("projlast", o, tmp_path)
        init = _ids(S["state"], 1000000)
        for th, mono, ratio, ori in calls:
            n, ids = r.i32(), r.vec("<i4")
            no, fo = ob.search_by_projection_last(fv, lf, ratio, ori, th, mono)
            assert n == no and no > 20, (seed, th, mono, ori)
            assert np.array_equal(ids, _expect_projection(fo, init, np.arange(len(kl)))), (seed, th, mono, ori)
            total_null += int(((fo == -2) & (S["state"] == 0)).sum())
    assert total_null > 0, "the fixture must exercise a rotation NULL over a pre-existing MapPoint"


def test_shim_search_by_projection_keyframe(tmp_path):
    """ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    (ORBmatcher.cc:2391-2513): the KeyFrame's MapPoints that are NULL, bad or in sAlreadyFound are
    not projected; Relocalization's two settings (Tracking.cc:3538, :3563) and checkOri off."""
    for seed in (5, 6):
        S = scenes.scene(seed)
        fv, keep = scenes.frame_view(S)
        kf, kk = scenes.kf_points(S)
        kps, use, pos, maxd, mind, desc = kk
        rng = np.random.default_rng(100 + seed)
        why = rng.integers(0, 3, len(use))  # where use == 0: no MapPoint / bad / already found
        has = (use == 1) | (why != 0)
        bad = (use == 0) & (why == 1)
        found = (use == 0) & (why == 2)
        o = shim_io.Out()
        shim_io.write_frame(o, fv, S["k"], S["k"], S["uright"], S["d"], S["state"], np.zeros(len(S["k"])), S["Tcw"])
        rec = np.zeros(len(kps), np.dtype([("ku", "V28"), ("h", "u1"), ("b", "u1"), ("f", "u1"), ("p", "<f4", 3),
                                           ("mx", "<f4"), ("mn", "<f4"), ("d", "u1", 32)]))
        rec["ku"] = kps.view("V28")
        rec["h"], rec["b"], rec["f"], rec["p"], rec["mx"], rec["mn"], rec["d"] = has, bad, found, pos, maxd, mind, desc
        o.i32(len(kps)).raw(rec)
        calls = [(10.0, 100, 0.75, 1), (3.0, 64, 0.75, 1), (10.0, 100, 0.75, 0)]
        o.i32(len(calls))
        for th, od, ratio, ori in calls:
            o.f32(th).i32(od).f32(ratio).i32(ori)
        r = shim_io.run_any("projkf", o, tmp_path)
        init = _ids(S["state"], 1000000)
        for th, od, ratio, ori in calls:
            n, ids = r.i32(), r.vec("<i4")
            no, fo = ob.search_by_projection_kf(fv, kf, ratio, ori, th, od)
            assert n == no and no > 20, (seed, th, od)
            assert np.array_equal(ids, _expect_projection(fo, init, 2000000 + np.arange(len(kps)))), (seed, th, od)


def test_shim_search_by_bow_keyframe_keyframe(tmp_path):
    """ORBmatcher::SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.cc:823-963): both sides need a
    MapPoint that is not bad; vpMatches12[i] = the KF2 MapPoint KF1 feature i matched."""
    import struct
    par, leaf, vd, vw = synth.vocab(10, 4, 3)
    img0 = synth.frame(22, 752, 480)
    img1 = synth.shifted(img0, 3, 2, 4.0, 5)
    k0, d0, _ = ob.extract(img0, ob.params(nfeatures=1200))
    k1, d1, _ = ob.extract(img1, ob.params(nfeatures=1200))
    rng = np.random.default_rng(9)
    sides, obs_sides = [], []
    for k, d in ((k0, d0), (k1, d1)):
        _, wt, nid = ob.vocab_transform(par, leaf, vd, vw, 4, d, 2)
        fv = synth.feature_vector(nid, wt)
        has = (rng.random(len(k)) < 0.85).astype(np.uint8)
        bad = (rng.random(len(k)) < 0.05).astype(np.uint8)
        b = struct.pack("<i", len(d)) + np.ascontiguousarray(d, np.uint8).tobytes()
        b += np.asarray(k["angle"], np.float32).tobytes() + has.tobytes() + bad.tobytes()
        b += struct.pack("<i", len(fv[0])) + np.asarray(fv[0], np.uint32).tobytes()
        b += np.asarray(fv[1], np.int32).tobytes() + np.asarray(fv[2], np.uint32).tobytes()
        sides.append(b)
        obs_sides.append((d, k["angle"], (has & (1 - bad)).astype(np.uint8)) + fv)
    calls = [(0.75, True), (0.9, True), (0.6, False)]
    blob = struct.pack("<i", len(calls)) + b"".join(struct.pack("<fi", r, int(c)) for r, c in calls) + b"".join(sides)
    (tmp_path / "kk.bin").write_bytes(blob)
    r = shim_io.run("bowkk", tmp_path / "kk.bin", tmp_path / "kk.out")
    for ratio, ori in calls:
        n, ids = r.i32(), r.vec("<i4")
        no, a2b, _ = ob.search_by_bow(obs_sides[0], obs_sides[1], ratio, ori, True)
        assert n == no and no > 50, (ratio, ori)
        assert np.array_equal(ids, a2b), (ratio, ori)


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (5, 0), (5, 1), (0, 2), (1, 3), (2, 1)])
def test_shim_compute_bow(scoring, weighting, tmp_path):
    """Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:721-728, KeyFrame.cc:105-114) =
    TemplatedVocabulary::transform(desc, mBowVec, mFeatVec, 4) (TemplatedVocabulary.h:1139-1206):
    mBowVec words and values bit for bit (DBoW2's weighting and L1 / L2 / no normalisation,
    stopped words dropped), mFeatVec at level L-4, for ORBvoc's TF_IDF + L1 and every other
    scoring / weighting branch; a second Frame::ComputeBoW keeps the vectors (:723)."""
    k, L = 4, 6
    par, leaf, vd, vw = synth.vocab(k, L, 11, stop_frac=0.05)
    img = synth.frame(23, 752, 480)
    _, d, _ = ob.extract(img, ob.params(nfeatures=1000))
    d = np.concatenate([d, d[:40]])  # repeated descriptors: several features per word
    o = shim_io.Out().i32(1, k, L, scoring, weighting, len(par))
    o.raw(par, np.int32).raw(leaf, np.uint8).raw(vd, np.uint8).raw(vw, np.float64).i32(len(d)).raw(d, np.uint8)
    r = shim_io.run_any("computebow", o, tmp_path)
    w, wt, nid = ob.vocab_transform(par, leaf, vd, vw, L, d, 4)
    ew, ev, en, eo, ef = ob.bow_vectors(w, wt, nid, scoring, weighting)
    assert len(ew) > 30 and len(en) > 5
    for side in ("Frame", "KeyFrame"):
        gw, gv, gn, go, gf = r.vec("<u4"), r.vec("<f8"), r.vec("<u4"), r.vec("<i4"), r.vec("<u4")
        assert np.array_equal(gw, ew) and np.array_equal(gv.view(np.uint64), ev.view(np.uint64)), side
        assert np.array_equal(gn, en) and np.array_equal(go, eo) and np.array_equal(gf, ef), side
    assert (wt <= 0).any(), "the fixture must contain stopped words"


def test_shim_orbextractor_call(tmp_path):
    """ORBextractor::operator() through the shim (ORBextractor.cc:1068-1150): keypoints, descriptors
    and monoIndex bit-exact, and the public mvImagePyramid refreshed per call with the oracle's
    levels (Frame::ComputeStereoMatches reads it, Frame.cc:801, 891); lap (0, 1000) reverses the
    list (mono, Frame.cc:306); an empty image returns -1 and leaves mvImagePyramid alone; one
    extractor grows from EuRoC to HD."""
    p = ob.params(nfeatures=1000)
    imgs = [(synth.frame(31, 752, 480), (0, 0)), (synth.frame(32, 640, 480), (0, 1000)),
            (np.zeros((0, 0), np.uint8), (0, 0)), (synth.frame(33, 1280, 720), (100, 400))]
    o = shim_io.Out().i32(p.nfeatures, p.nlevels, p.ini_th_fast, p.min_th_fast).f32(p.scale_factor).i32(len(imgs))
    for img, lap in imgs:
        h, w = img.shape
        o.i32(w, h, *lap).raw(img, np.uint8)
    r = shim_io.run_any("extract", o, tmp_path)
    last_pyr = None
    for img, lap in imgs:
        mono, kps, desc = r.i32(), r.vec(ob.KP_DTYPE).view(np.uint8), r.vec("u1")
        nl = r.i32()
        pyr = []
        for _ in range(nl):
            rows, cols = r.i32(), r.i32()
            pyr.append(r.vec("u1").reshape(rows, cols))
        if img.size == 0:
            assert mono == -1 and len(kps) == 0
            assert len(pyr) == len(last_pyr) and all(np.array_equal(a, b) for a, b in zip(pyr, last_pyr))
            continue
        ko, do, mo = ob.extract(img, p, lap)
        assert mono == mo and np.array_equal(kps, ko.view(np.uint8).ravel()) and np.array_equal(desc, do.ravel())
        po = ob.pyramid(img, p)
        assert len(pyr) == len(po) and all(np.array_equal(a, b) for a, b in zip(pyr, po))
        last_pyr = pyr


def test_shim_compute_stereo_matches(tmp_path):
    """The stereo Frame constructor's host path (Frame.cc:98-152): the two ORBextractorCall shims,
    then the ComputeStereoMatches shim (Frame.cc:794-964); everything against the oracle's own
    extraction, pyramids and stereo matcher."""
    p = ob.params(nfeatures=1200)
    mbf = synth.EUROC_STEREO["bf"]
    mb = mbf / synth.EUROC_STEREO["fx"]
    il, ir = synth.stereo_pair(7, 752, 480, 4.0, 40.0, 2.0)
    o = shim_io.Out().i32(p.nfeatures, p.nlevels, p.ini_th_fast, p.min_th_fast).f32(p.scale_factor, mbf, mb)
    o.i32(752, 480).raw(il, np.uint8).raw(ir, np.uint8)
    r = shim_io.run_any("stereo", o, tmp_path)
    kl, dl = r.vec(ob.KP_DTYPE).view(np.uint8), r.vec("u1")
    kr, dr = r.vec(ob.KP_DTYPE).view(np.uint8), r.vec("u1")
    ur, dep = r.vec("<f4"), r.vec("<f4")
    klo, dlo, _ = ob.extract(il, p)
    kro, dro, _ = ob.extract(ir, p)
    assert np.array_equal(kl, klo.view(np.uint8).ravel()) and np.array_equal(dl, dlo.ravel())
    assert np.array_equal(kr, kro.view(np.uint8).ravel()) and np.array_equal(dr, dro.ravel())
    sc, isc, _, _, _ = ob.levels(p)
    uro, depo = ob.stereo_matches(klo, dlo, kro, dro, ob.pyramid(il, p), ob.pyramid(ir, p), sc, isc, mbf, mb)
    assert np.array_equal(ur, uro) and np.array_equal(dep, depo)
    assert (ur >= 0).sum() > 300


@pytest.mark.parametrize("seed,th,far", [(7, 1.0, False), (8, 3.0, True), (9, 15.0, False)])
def test_shim_search_local_points(seed, th, far, tmp_path):
    """Tracking::SearchLocalPoints (Tracking.cc:3187-3258) through the shim: the frame's own
    MapPoints are marked seen (bad ones dropped from the frame), every other local MapPoint gets
    isInFrustum's tracking fields (Frame.cc:497-554: mbTrackInView, mTrackProjX/Y also for points
    rejected after the image test, XR / depth / level / viewing cosine when in view) and
    IncreaseVisible, mmProjectPoints gets the in-view ones, and SearchByProjection's matches land
    in F.mvpMapPoints — all against the oracle's isInFrustum + SearchByProjection."""
    S = scenes.scene(seed)
    k, d, ur, state = S["k"], S["d"], S["uright"], S["state"].copy()
    n = len(k)
    rng = np.random.default_rng(200 + seed)
    fbad = ((state >= 0) & (rng.random(n) < 0.2)).astype(np.uint8)
    fv, keep = scenes.frame_view(S)
    geom, desc = scenes.local_map_geom(S)
    m = len(geom)
    # some of the frame's own MapPoints also sit in the local map
    refs = rng.choice(np.flatnonzero(state >= 0), 30, replace=False)
    at = np.sort(rng.choice(m, 30, replace=False))
    ref = np.full(m, -1, np.int32)
    ref[at] = refs
    o = shim_io.Out()
    shim_io.write_frame(o, fv, k, k, ur, d, state, fbad, S["Tcw"], mnId=7)
    rec = np.zeros(m, np.dtype([("ref", "<i4"), ("p", "<f4", 3), ("nrm", "<f4", 3), ("mn", "<f4"), ("mx", "<f4"),
                                ("s", "u1"), ("b", "u1"), ("o", "u1"), ("d", "u1", 32)]))
    rec["ref"], rec["p"], rec["nrm"] = ref, geom["pos"], geom["normal"]
    rec["mn"], rec["mx"] = geom["min_dist"], geom["max_dist"]
    rec["s"], rec["b"], rec["o"], rec["d"] = geom["seen"], geom["is_bad"], geom["has_obs"], desc
    o.i32(m).raw(rec).f32(th).i32(int(far)).f32(20.0)
    r = shim_io.run_any("localpoints", o, tmp_path)
    nto_g, nm_g, fids = r.i32(), r.i32(), r.vec("<i4")
    inview, fl, iv = r.vec("u1"), r.vec("<f4").reshape(-1, 5), r.vec("<i4").reshape(-1, 3)
    own_vis, pid, pxy = r.vec("<i4"), r.vec("<i4"), r.vec("<f4").reshape(-1, 2)
    # the reference's view of the same objects
    state2 = np.where(fbad == 1, -1, state).astype(np.int8)
    g2 = geom.copy()
    isref = ref >= 0
    g2["seen"][isref] = fbad[ref[isref]] == 0
    g2["is_bad"][isref] = fbad[ref[isref]]
    g2["has_obs"][isref] = state[ref[isref]] == 1
    fv2, keep2 = slamhot.make_frame_view(k, d, ur, state2, Tcw=S["Tcw"])
    nto, tro = ob.is_in_frustum(fv2, g2, 0.5)
    no, fo = ob.search_by_projection_local(fv2, tro, desc, 0.8, th, far, 20.0)
    assert nto_g == nto and nm_g == no and no > 50
    local_ids = np.where(isref, 1000000 + ref, 3000000 + np.arange(m))
    init = _ids(state2, 1000000)
    assert np.array_equal(fids, np.where(fo >= 0, local_ids[np.maximum(fo, 0)], init))
    act = (g2["seen"] == 0) & (g2["is_bad"] == 0)
    v = act & (tro["in_view"] == 1)
    assert np.array_equal(inview.astype(bool), v)
    assert np.array_equal(fl[act, 0], tro["proj_x"][act]) and np.array_equal(fl[act, 1], tro["proj_y"][act])
    assert np.array_equal(fl[v, 2], tro["proj_xr"][v]) and np.array_equal(fl[v, 3], tro["depth"][v])
    assert np.array_equal(fl[v, 4], tro["view_cos"][v]) and np.array_equal(iv[v, 0], tro["scale_level"][v])
    assert np.array_equal(iv[~isref, 1], 1 + v[~isref])  # IncreaseVisible once per frustum hit
    assert np.array_equal(own_vis, np.where(state >= 0, 1 + (fbad == 0), 1))
    assert (fl[~act & ~isref, 0] == -1).all() and not inview[~act].any()
    assert np.array_equal(pid, np.sort(local_ids[v]))
    order = np.argsort(local_ids[v])
    assert np.array_equal(pxy, np.stack([tro["proj_x"][v], tro["proj_y"][v]], 1)[order])


def test_shim_fuse(tmp_path):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:1629-1818) through the shim, the update
    half included: the KeyFrame's MapPoints, every MapPoint's bad flag, nObs and observations after
    the call equal the Python mirror applying the same half in list order to the oracle's search
    (Replace in both directions, AddObservation, NULL entries, bad and already-in-KF skips)."""
    from slamhot import optimizer as opt
    S = scenes.scene(12)
    k, d, ur, Tcw = S["k"], S["d"], S["uright"], S["Tcw"]
    n = len(k)
    geom, desc = scenes.fuse_mps(S)
    rng = np.random.default_rng(77)
    m_list = len(geom)
    # extra MapPoints already in the KeyFrame (the Replace targets), not in the list
    occ = rng.choice(n, n // 4, replace=False)
    m = m_list + len(occ)
    pos = np.concatenate([geom["pos"], rng.normal(0, 1, (len(occ), 3))]).astype(np.float32)
    nrm = np.concatenate([geom["normal"], np.tile([0, 0, 1], (len(occ), 1))]).astype(np.float32)
    mind = np.concatenate([geom["min_dist"], np.ones(len(occ))]).astype(np.float32)
    maxd = np.concatenate([geom["max_dist"], np.ones(len(occ))]).astype(np.float32)
    bad = np.concatenate([geom["is_bad"], rng.random(len(occ)) < 0.05]).astype(np.uint8)
    dsc = np.concatenate([desc, rng.integers(0, 256, (len(occ), 32), dtype=np.uint8)])
    kf_idx = np.full(m, -1, np.int32)
    kf_idx[m_list:] = occ
    free = np.setdiff1d(np.arange(n), occ)
    seen = np.flatnonzero(geom["seen"])  # list MapPoints already in the KeyFrame
    kf_idx[seen] = rng.choice(free, len(seen), replace=False)
    ndummy = 6
    others = [np.sort(rng.choice(ndummy, rng.integers(0, 5), replace=False)) for _ in range(m)]
    lst = list(rng.permutation(m_list))
    for pos_null in rng.choice(len(lst), 12, replace=False):
        lst.insert(int(pos_null), -1)
    th = 3.0
    sc, isig, lsf = shim_io.level_tables()
    fv, keep = slamhot.make_frame_view(k, d, ur, None, Tcw=Tcw)
    o = shim_io.Out().i32(n).raw(Tcw, np.float32).f32(fv.fx, fv.fy, fv.cx, fv.cy, fv.bf, fv.b)
    o.i32(0, 0, 752, 480).f32(fv.grid_inv_w, fv.grid_inv_h).i32(8).raw(sc, np.float32).f32(lsf).raw(isig, np.float32)
    rec = np.zeros(n, np.dtype([("ku", "V28"), ("ur", "<f4"), ("d", "u1", 32)]))
    rec["ku"], rec["ur"], rec["d"] = k.view("V28"), ur, d
    o.raw(rec).i32(m, ndummy)
    for j in range(m):
        o.raw(pos[j]).raw(nrm[j]).f32(mind[j], maxd[j]).raw(np.uint8(bad[j])).raw(dsc[j]).i32(kf_idx[j], len(others[j]))
        o.i32(*others[j])
    o.i32(len(lst), *lst).f32(th)
    r = shim_io.run_any("fuse", o, tmp_path)
    nf_g, kfm_g, st_g, obs_g = r.i32(), r.vec("<i4"), r.vec("<i4").reshape(-1, 2), r.vec("<i4")
    # the mirror: same map, oracle search, update half in list order
    pm = opt.Map()
    cam = (fv.fx, fv.fy, fv.cx, fv.cy, fv.bf)
    K = opt.KeyFrame(0, Tcw, k, ur, isig, cam, pm)
    D = [opt.KeyFrame(1 + i, np.eye(4), np.zeros(m, slamhot.KP_DTYPE), -np.ones(m), isig, cam, pm) for i in range(ndummy)]
    mps = [opt.MapPoint(j, pos[j], pm) for j in range(m)]
    for j, mp in enumerate(mps):
        mp.bad = bool(bad[j])
        if kf_idx[j] >= 0:
            mp.AddObservation(K, int(kf_idx[j]))
            K.mvpMapPoints[kf_idx[j]] = mp
        for dd in others[j]:
            mp.AddObservation(D[dd], j)
            D[dd].mvpMapPoints[j] = mp
    objs = [mps[j] if j >= 0 else None for j in lst]
    g = np.zeros(len(objs), slamhot.MP_GEOM_DTYPE)
    gd = np.zeros((len(objs), 32), np.uint8)
    for i, mp in enumerate(objs):
        if mp is None:
            g["is_bad"][i] = 1
            continue
        j = mp.mnId
        g["pos"][i], g["normal"][i], g["min_dist"][i], g["max_dist"][i] = pos[j], nrm[j], mind[j], maxd[j]
        g["is_bad"][i], g["seen"][i], g["has_obs"][i] = mp.isBad(), mp.IsInKeyFrame(K), mp.Observations() > 0
        gd[i] = dsc[j]
    bi, bd = ob.fuse_search(fv, isig, g, gd, th)
    nf = opt.fuse_apply(K, objs, bi, bd)
    assert nf_g == nf and nf > 100
    assert np.array_equal(kfm_g, [mp.mnId if mp is not None else -1 for mp in K.mvpMapPoints])
    assert np.array_equal(st_g[:, 0], [mp.isBad() for mp in mps])
    assert np.array_equal(st_g[:, 1], [mp.Observations() for mp in mps])
    exp = []
    for mp in mps:
        ob_ = sorted((kf.mnId, li) for kf, (li, ri) in mp.observations.items())
        exp += [len(ob_)] + [x for p in ob_ for x in p]
    assert np.array_equal(obs_g, exp)
    assert sum(mp.isBad() for mp in mps) > int(bad.sum()), "the fixture must exercise Replace"
