"""The drop-in LocalBundleAdjustment shim's window construction and flattening
(include/slamhot_orbslam3.hpp: BuildLocalWindow / FlattenLocalWindow, Optimizer.cc:1613-1918),
compiled against ORB-SLAM3 stand-ins (tests/cpp/shim_driver), equals the Python mirror
(slamhot.optimizer.build_window / flatten_window) on the same maps, bit for bit.  Host logic:
no device needed."""
import numpy as np
import pytest

import shim_io
from slamhot import optimizer as opt
from slamhot import synth

pytestmark = pytest.mark.skipif(not shim_io.DRIVER.exists(), reason="tests/cpp/shim_driver not built")


def _mirror_flatten(pmap, kfs):
    win = opt.build_window(kfs[-1], pmap)
    if win is None:
        return None
    local, fixed, local_mps, num_fixed = win
    W, order, refs = opt.flatten_window(local, fixed, local_mps, pmap)
    return dict(num_fixed=num_fixed, num_local=len(local), num_mps=len(local_mps),
                kf_ids=np.array([k.mnId for k in order]), mp_ids=np.array([m.mnId for m in local_mps]), **W)


CASES = {
    "mono": dict(seed=70, kw=dict(n_kf=12, n_pt=300, obs_per_pt=5), covis=None),
    "stereo": dict(seed=71, kw=dict(n_kf=10, n_pt=250, obs_per_pt=4, stereo_frac=0.4), covis=None),
    "rig": dict(seed=72, kw=dict(n_kf=10, n_pt=250, obs_per_pt=4, body_frac=0.5), covis=None),
    # only three covisible KFs: the rest see local points -> lFixedCameras, no fallback
    "partial_covis": dict(seed=73, kw=dict(n_kf=14, n_pt=300, obs_per_pt=5), covis=[12, 11, 5]),
    # no covisible KF but one: fixed-camera fallback (:1676-1712) moves the lowest ids
    "fallback": dict(seed=74, kw=dict(n_kf=6, n_pt=120, obs_per_pt=6), covis=[4, 3, 2, 1]),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_shim_window_equals_mirror(case, tmp_path):
    c = CASES[case]
    W = synth.lba_window(c["seed"], **c["kw"])
    pmap, kfs, mps = opt.map_from_window(W)
    if c["covis"] is not None:
        kfs[-1].covisible = [kfs[i] for i in c["covis"]]
    shim_io.write_map(tmp_path / "map.bin", pmap, kfs, mps)
    got = shim_io.read_flatten(shim_io.run("flatten", tmp_path / "map.bin", tmp_path / "out.bin"))
    # the mirror marks its objects (mnBALocalForKF ...) like the reference: fresh map
    pmap, kfs, mps = opt.map_from_window(W)
    if c["covis"] is not None:
        kfs[-1].covisible = [kfs[i] for i in c["covis"]]
    ref = _mirror_flatten(pmap, kfs)
    assert got["ok"] == 1 and ref is not None
    for k in ("num_fixed", "num_local", "num_mps"):
        assert got[k] == ref[k], k
    for k in ("kf_ids", "mp_ids", "kf_Tcw", "kf_fixed", "pt_pos", "edge_pt", "edge_kf", "edge_obs", "edge_inv_sigma2"):
        assert np.array_equal(got[k].ravel(), np.asarray(ref[k]).ravel()), k
    if "edge_body" in ref:
        assert np.array_equal(got["edge_body"], ref["edge_body"])
        assert np.array_equal(got["kf_Trl"].ravel(), ref["kf_Trl"].ravel())
    else:
        assert len(got["edge_body"]) == 0
