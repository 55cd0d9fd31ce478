"""EuRoC I/O around the hot path: image-list loader, OpenCV-YAML settings, rectification maps
and the remap oracle, trajectory writer."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob
from slamhot import ate, euroc, synth

GOLD = Path(__file__).resolve().parent / "golden" / "euroc_stereo_calib.json"


@pytest.fixture(scope="module")
def calib():
    c = json.loads(GOLD.read_text())
    return {k: np.array(v) if isinstance(v, list) else v for k, v in c.items()}


@pytest.fixture(scope="module")
def maps(calib):
    out = {}
    for side in ("LEFT", "RIGHT"):
        out[side] = euroc.init_undistort_rectify_map(calib[f"{side}.K"], calib[f"{side}.D"], calib[f"{side}.R"],
                                                     calib[f"{side}.P"], (calib[f"{side}.width"],
                                                                          calib[f"{side}.height"]))
    return out


def test_load_images(tmp_path):
    (tmp_path / "times.txt").write_text("1403636579763555584\n1403636579813555456\n\n")
    L, R, T = euroc.LoadImages("/d/cam0/data", "/d/cam1/data", str(tmp_path / "times.txt"))
    assert L == ["/d/cam0/data/1403636579763555584.png", "/d/cam0/data/1403636579813555456.png"]
    assert R[1] == "/d/cam1/data/1403636579813555456.png"
    assert T[0] == pytest.approx(1403636579.763555584)


def test_read_settings(tmp_path):
    y = tmp_path / "s.yaml"
    y.write_text('%YAML:1.0\n\nCamera.type: "PinHole"\nCamera.fx: 435.2\nLEFT.height: 480\n'
                 'LEFT.D: !!opencv-matrix\n   rows: 1\n   cols: 5\n   dt: d\n'
                 '   data:[-0.28, 0.07, 0.0001,\n      1.7e-05, 0.0]\n# comment\nViewer.KeyFrameSize: 0.05\n')
    s = euroc.read_settings(str(y))
    assert s["Camera.type"] == "PinHole" and s["Camera.fx"] == 435.2 and s["LEFT.height"] == 480
    assert s["LEFT.D"].shape == (1, 5) and s["LEFT.D"][0, 3] == 1.7e-05
    assert s["Viewer.KeyFrameSize"] == 0.05


def test_rectification_maps(calib, maps):
    """Rectified principal point maps back through R and the distortion model onto the raw
    image; maps are finite and near identity plus distortion (EuRoC radial k1 = -0.28)."""
    for side in ("LEFT", "RIGHT"):
        mx, my = maps[side]
        assert mx.shape == (480, 752) and np.isfinite(mx).all()
        P = calib[f"{side}.P"]
        cx, cy = P[0, 2], P[1, 2]
        j, i = int(round(cx)), int(round(cy))
        K = calib[f"{side}.K"]
        assert abs(mx[i, j] - K[0, 2]) < 12 and abs(my[i, j] - K[1, 2]) < 12
        # barrel distortion pulls corners inwards in the raw image
        assert mx[0, 0] > 0 and mx[0, -1] < 751


def _py_remap(src, mx, my):
    sh, sw = src.shape
    X = np.rint(mx.astype(np.float32) * np.float32(32)).astype(np.int64)   # rint = round half even
    Y = np.rint(my.astype(np.float32) * np.float32(32)).astype(np.int64)
    sx, sy, fx, fy = X >> 5, Y >> 5, X & 31, Y & 31
    pad = np.zeros((sh + 4, sw + 4), np.int64)
    pad[2:-2, 2:-2] = src
    def at(yy, xx):
        ok = (xx >= -2) & (xx < sw + 2) & (yy >= -2) & (yy < sh + 2)
        v = pad[np.clip(yy + 2, 0, sh + 3), np.clip(xx + 2, 0, sw + 3)]
        return np.where(ok, v, 0)
    v = (at(sy, sx) * (32 - fx) * (32 - fy) + at(sy, sx + 1) * fx * (32 - fy) + at(sy + 1, sx) * (32 - fx) * fy +
         at(sy + 1, sx + 1) * fx * fy) * 32
    return np.clip((v + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def test_remap_oracle_vs_numpy(maps):
    src = synth.frame(3, 752, 480)
    mx, my = maps["LEFT"]
    # exercise borders and exact half fractions too
    mx2, my2 = mx.copy(), my.copy()
    mx2[:5] = -1.5 + np.arange(752) / 100.0
    my2[-3:] = 479.25
    mx2[10, :64] = np.arange(64) + 0.015625  # X = 32k + 0.5: round half to even
    for a, b in ((mx, my), (mx2, my2)):
        assert np.array_equal(ob.remap_linear(src, a, b), _py_remap(src, a, b))


def test_trajectory_writer_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    Ts, times = [], []
    for k in range(20):
        a = rng.normal(0, 0.3, 3)
        th = np.linalg.norm(a)
        Kx = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]) / th
        R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = rng.normal(0, 2, 3)
        Ts.append(T.astype(np.float32))
        times.append(1403636579.763555584 + 0.05 * k)
    f = tmp_path / "traj.txt"
    euroc.save_trajectory_euroc(str(f), times, Ts)
    lines = f.read_text().splitlines()
    assert len(lines) == 20 and len(lines[0].split()) == 8
    assert lines[0].split()[0] == f"{1e9 * times[0]:.6f}"
    est = ate.read_file_list(str(f))
    assert len(est) == 20
    for (t, row), T in zip(sorted(est.items()), Ts):
        twc = -T[:3, :3].T.astype(np.float64) @ T[:3, 3]
        assert np.allclose([float(x) for x in row[:3]], twc, atol=1e-5)
        q = np.array([float(x) for x in row[3:7]])
        assert abs(np.linalg.norm(q) - 1) < 1e-6
