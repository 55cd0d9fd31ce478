"""The C++ host layer (include/slamhot.hpp) — ORBextractor, ORBmatcher::SearchByBoW and
Optimizer::LocalBundleAdjustment as a C++ caller of the reference uses them — driven by
tests/cpp/host_driver (built by __graft_entry__.build()) and checked against the CPU oracle:
bit-exact keypoints / descriptors / pyramid / match indices, LBA within 1e-5.

The not-gpu test checks the other half of the contract: without a gfx950 device the C++
layer raises slamhot::Error(SLAM_ENODEV) (exit code 3) instead of computing anything."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

ROOT = Path(__file__).resolve().parents[1]
DRIVER = Path(os.environ.get("SLAMHOT_HOST_DRIVER", str(ROOT / "tests" / "cpp" / "host_driver")))  # sanitizer builds: tools/sanitize.sh


def _run(*args, check=True):
    if not DRIVER.exists():
        pytest.fail(f"{DRIVER} not built (run __graft_entry__.build())")
    r = subprocess.run([str(DRIVER), *map(str, args)], capture_output=True, text=True, timeout=120)
    if check and r.returncode != 0:
        raise AssertionError(f"host_driver {args[0]} rc={r.returncode}: {r.stderr}")
    return r


def _write_side(path, desc, angle, valid, node_id, node_off, node_feat):
    with open(path, "wb") as f:
        f.write(np.int32(len(desc)).tobytes())
        f.write(np.ascontiguousarray(desc, np.uint8).tobytes())
        f.write(np.ascontiguousarray(angle, np.float32).tobytes())
        f.write(np.int32(valid is not None).tobytes())
        if valid is not None:
            f.write(np.ascontiguousarray(valid, np.uint8).tobytes())
        f.write(np.int32(len(node_id)).tobytes())
        f.write(np.ascontiguousarray(node_id, np.uint32).tobytes())
        f.write(np.ascontiguousarray(node_off, np.int32).tobytes())
        f.write(np.ascontiguousarray(node_feat, np.uint32).tobytes())


def _write_window(path, w, inertial=False):
    with open(path, "wb") as f:
        f.write(np.array([len(w["kf_fixed"]), len(w["pt_pos"]), len(w["edge_pt"]), int(inertial)], np.int32).tobytes())
        f.write(np.asarray(w["cam"], np.float32).tobytes())
        f.write(np.ascontiguousarray(w["kf_Tcw"], np.float32).tobytes())
        f.write(np.ascontiguousarray(w["kf_fixed"], np.uint8).tobytes())
        f.write(np.ascontiguousarray(w["pt_pos"], np.float32).tobytes())
        f.write(np.ascontiguousarray(w["edge_pt"], np.int32).tobytes())
        f.write(np.ascontiguousarray(w["edge_kf"], np.int32).tobytes())
        f.write(np.ascontiguousarray(w["edge_obs"], np.float32).tobytes())
        f.write(np.ascontiguousarray(w["edge_inv_sigma2"], np.float32).tobytes())


def test_cpp_layer_fails_loudly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    img = synth.frame(3, 640, 480)
    img.tofile(tmp_path / "img.u8")
    r = _run("extract", 640, 480, 1000, 0, 0, tmp_path / "img.u8", tmp_path / "out", check=False)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "gfx950" in r.stderr
    assert not (tmp_path / "out.kp").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("size,nf,lap", [((640, 480), 1000, (0, 0)), ((752, 480), 1200, (0, 1000)),
                                         ((641, 479), 1000, (100, 400))])
def test_cpp_orbextractor_bitexact(tmp_path, size, nf, lap):
    w, h = size
    img = synth.frame(90 + w % 7, w, h)
    img.tofile(tmp_path / "img.u8")
    _run("extract", w, h, nf, lap[0], lap[1], tmp_path / "img.u8", tmp_path / "out")
    meta = (tmp_path / "out.meta").read_text().split()
    n, mono, empty_ret, nlev = int(meta[0]), int(meta[1]), int(meta[2]), int(meta[3])
    kg = np.fromfile(tmp_path / "out.kp", ob.KP_DTYPE)
    dg = np.fromfile(tmp_path / "out.desc", np.uint8).reshape(-1, 32)
    ko, do, mo = ob.extract(img, ob.params(nfeatures=nf), lap=lap)
    assert n == len(ko) == len(kg) and mono == mo
    assert empty_ret == -1                                   # ORBextractor.cc:1072-1073
    assert np.array_equal(kg.view(np.uint8), ko.view(np.uint8))
    assert np.array_equal(dg, do)
    # getters (ORBextractor.h:61-81) and mvImagePyramid (ORBextractor.h:83)
    scale = np.array(meta[5:5 + nlev], np.float32)
    nfeat = np.array(meta[5 + nlev:5 + 2 * nlev], np.int64)
    s_o, _, _, _, nf_o = ob.levels(ob.params(nfeatures=nf))
    assert nlev == 8 and np.array_equal(scale, s_o) and np.array_equal(nfeat, nf_o)
    pyr = np.fromfile(tmp_path / "out.pyr", np.uint8)
    ref = ob.pyramid(img)
    assert np.array_equal(pyr, np.concatenate([r.ravel() for r in ref]))


@pytest.mark.gpu
@pytest.mark.parametrize("strict", [0, 1])
def test_cpp_orbmatcher_search_by_bow(tmp_path, strict):
    import slamhot
    par, leaf, d, wt = synth.vocab(10, 6, 0)
    voc = slamhot.Vocabulary(par, leaf, d, wt, k=10, L=6)
    img0 = synth.frame(1, 752, 480)
    sides = []
    rng = np.random.default_rng(7)
    for i, img in enumerate((img0, synth.shifted(img0, 3, 2, 2.0, 8))):
        k, desc, _ = ob.extract(img, ob.params(nfeatures=1200))
        _, wtk, nid = voc.transform(desc, 4)
        valid = (rng.random(len(k)) < 0.85).astype(np.uint8) if (i == 0 or strict) else None
        sides.append((desc, k["angle"], valid) + synth.feature_vector(nid, wtk))
    voc.close()
    _write_side(tmp_path / "a.bin", *sides[0])
    _write_side(tmp_path / "b.bin", *sides[1])
    _run("bow", strict, 0.75, tmp_path / "a.bin", tmp_path / "b.bin", tmp_path / "m.bin")
    out = np.fromfile(tmp_path / "m.bin", np.int32)
    n_o, a2b_o, b2a_o = ob.search_by_bow(sides[0], sides[1], 0.75, True, bool(strict))
    ref = a2b_o if strict else b2a_o
    assert out[0] == n_o
    assert np.array_equal(out[1:1 + len(ref)], ref)
    assert out[1 + len(ref)] == ob.descriptor_distance(sides[0][0][0], sides[1][0][0])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3])
def test_cpp_local_bundle_adjustment(tmp_path, seed):
    W = synth.lba_window(seed)
    _write_window(tmp_path / "w.bin", W)
    _run("lba", tmp_path / "w.bin", tmp_path / "r.bin")
    b = (tmp_path / "r.bin").read_bytes()
    head = np.frombuffer(b[:32], np.int32)
    chi2 = np.frombuffer(b[32:48], np.float64)
    nkf, npt, ne = len(W["kf_fixed"]), len(W["pt_pos"]), len(W["edge_pt"])
    off = 48
    kf = np.frombuffer(b[off:off + nkf * 64], np.float32).reshape(nkf, 16)
    off += nkf * 64
    pt = np.frombuffer(b[off:off + npt * 12], np.float32).reshape(npt, 3)
    off += npt * 12
    outl = np.frombuffer(b[off:off + ne], np.uint8)
    fixed = np.asarray(W["kf_fixed"])
    # counters as Optimizer.cc reports them (:1630-1675, :1749, :1656, :1919)
    assert head[0] == int((fixed > 0).sum()) and head[1] == int((fixed != 2).sum())
    assert head[2] == npt and head[3] == ne
    o = ob.lba_solve(W)
    assert list(head[4:6]) == list(o["iterations"]) and head[6] == o["trials"] and head[7] == o["n_outlier"]
    np.testing.assert_allclose(chi2, [o["chi2_initial"], o["chi2_final"]], rtol=1e-8)
    assert np.array_equal(outl, o["edge_outlier"])
    assert np.abs(kf.astype(np.float64) - o["kf_Tcw"].reshape(nkf, 16)).max() <= 1e-5
    assert np.abs(pt.astype(np.float64) - o["pt_pos"].reshape(npt, 3)).max() <= 1e-5
