"""slamhot/ate.py against golden vectors made with the reference's own associate / align
(tools/make_ate_golden.py), plus file parsing and known answers."""
from pathlib import Path

import numpy as np
import pytest

from slamhot import ate

G = np.load(Path(__file__).parent / "golden" / "ate.npz")


def _dicts(c):
    first = {float(a): [str(x) for x in p] + ["0", "0", "0", "1"] for a, p in zip(G[f"c{c}_t"], G[f"c{c}_gt"])}
    second = {float(a): [str(x) for x in p] + ["0", "0", "0", "1"] for a, p in zip(G[f"c{c}_test"], G[f"c{c}_est"])}
    return first, second


@pytest.mark.parametrize("c", range(4))
def test_associate_and_align_match_reference(c):
    first, second = _dicts(c)
    m = ate.associate(first, second, 0.0, 20000000.0)
    assert np.array_equal(np.array(m), G[f"c{c}_matches"])
    fx = np.array([[float(v) for v in first[a][0:3]] for a, b in m]).T
    sx = np.array([[float(v) for v in second[b][0:3]] for a, b in m]).T
    rot, transGT, errGT, trans, err, s = ate.align(sx, fx)
    np.testing.assert_allclose(rot, G[f"c{c}_rot"], atol=1e-12)
    np.testing.assert_allclose(s, G[f"c{c}_s"], rtol=1e-12)
    np.testing.assert_allclose(err, G[f"c{c}_err"].ravel(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(errGT, G[f"c{c}_errGT"].ravel(), rtol=1e-10, atol=1e-12)


def test_read_file_list_and_known_answer(tmp_path):
    gt = tmp_path / "gt.txt"
    est = tmp_path / "est.txt"
    rng = np.random.default_rng(1)
    P = np.cumsum(rng.normal(size=(50, 3)), 0)
    with open(gt, "w") as f:
        f.write("# timestamp tx ty tz qx qy qz qw\n")
        for i, p in enumerate(P):
            f.write(f"{1e9 + i * 5e7:.0f},{p[0]},{p[1]},{p[2]},0,0,0,1\n")
    with open(est, "w") as f:
        for i, p in enumerate(P):
            q = 2.5 * p + np.array([1.0, -2.0, 0.5])
            f.write(f"{1e9 + i * 5e7 + 1e6:.0f} {q[0]} {q[1]} {q[2]} 0 0 0 1\n")
    first, second = ate.read_file_list(str(gt)), ate.read_file_list(str(est))
    assert len(first) == len(second) == 50
    rmse, s, rmse_sim3, n = ate.evaluate(first, second)
    assert n == 50
    assert s == pytest.approx(0.4, rel=1e-12)       # aligns est onto gt: 1 / 2.5
    assert rmse_sim3 == pytest.approx(0.0, abs=1e-9)
    assert rmse > 0.1                                 # SE3-only alignment cannot absorb the scale


def test_window_ate_bench_helper():
    """bench.py's LBA accuracy report: camera-centre ATE is ~0 for the ground truth itself
    and the restated reference LBA brings a perturbed config-4 window well below its start."""
    import bench
    import oracle_bind as ob
    from slamhot import synth
    w = synth.lba_window(1)
    assert bench.window_ate(w, w["gt_T"].reshape(-1, 16)) < 1e-12
    a0 = bench.window_ate(w, w["kf_Tcw"])
    a1 = bench.window_ate(w, ob.lba_solve(w)["kf_Tcw"])
    assert 0.01 < a0 < 0.05 and a1 < 0.5 * a0
