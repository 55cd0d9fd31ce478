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


def test_shim_pose_optimization_equals_device_and_oracle(tmp_path):
    import struct

    import slamhot
    f = synth.pose_frame(90, stereo_frac=0.3)
    n = len(f["kps"])
    b = bytearray(struct.pack("<i", n))
    b += np.asarray(f["Tcw"], np.float32).tobytes() + np.asarray(f["cam"], np.float32).tobytes()
    b += np.asarray(f["inv_sigma2"], np.float32).tobytes()
    for i in range(n):
        kp = f["kps"][i]
        b += struct.pack("<ffifi", kp["x"], kp["y"], int(kp["octave"]), f["uright"][i], int(f["has_mp"][i]))
        b += np.asarray(f["mp_pos"][i], np.float32).tobytes()
    (tmp_path / "f.bin").write_bytes(bytes(b))
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
