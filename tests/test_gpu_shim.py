"""GPU: the drop-in shim bodies (include/slamhot_orbslam3.hpp) compiled against ORB-SLAM3
stand-ins and run through tests/cpp/shim_driver give the same map updates as the Python mirror
over the same device solver: Optimizer::LocalBundleAdjustment (window, solve, vToErase, pose and
point write-back, UpdateNormalAndDepth, IncreaseChangeIndex) and Optimizer::PoseOptimization."""
import numpy as np
import pytest

import oracle_bind as ob
import shim_io
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
