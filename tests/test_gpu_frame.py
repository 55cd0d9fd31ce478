"""GPU parity of Frame construction after extraction: Frame::UndistortKeyPoints and
Frame::ComputeImageBounds (Frame.cc:730-792) on the device vs the oracle, bit-exact; and
BASELINE.json configs[0] — EuRoC MH01-shaped monocular Frames (752x480 raw distorted images,
the initialisation extractor at 5 x 1000 features for the first frames, then 1000 features,
ExtractORB(0, im, 0, 1000), UndistortKeyPoints) — driven through the C++ host layer
(tests/cpp/host_driver mono) and checked frame by frame against the oracle."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
CAM = synth.EUROC_MONO_CAM
K = np.array([CAM["fx"], CAM["fy"], CAM["cx"], CAM["cy"]], np.float32)
D = np.array(CAM["dist"], np.float32)


@pytest.fixture(scope="module")
def mono_frames():
    imgs, _ = synth.mono_sequence(5, 10)
    return imgs


def test_undistort_device_bitexact(mono_frames):
    import slamhot
    kps, _, _ = ob.extract(mono_frames[0], ob.params(nfeatures=1000))
    rng = np.random.default_rng(1)
    extra = np.zeros(3000, ob.KP_DTYPE)
    extra["x"] = rng.uniform(-5, 760, 3000)
    extra["y"] = rng.uniform(-5, 485, 3000)
    extra["octave"] = rng.integers(0, 8, 3000)
    for k in (kps, extra):
        for dist in (D, np.append(D, np.float32(0.02)), np.array([-2.5, 0, 0, 0], np.float32),
                     np.array([0.0, 0.1, 0, 0], np.float32)):
            g = slamhot.UndistortKeyPoints(k, K, dist)
            o = ob.undistort_keypoints(k, K, dist)
            assert np.array_equal(g.view(np.uint8), o.view(np.uint8))


def test_undistort_batch_device_and_bounds(mono_frames):
    import torch

    import slamhot
    F = 4
    ex = slamhot.ORBextractor(nfeatures=1000, max_size=(752, 480), max_batch=F)
    cap = ex.cap
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(np.ascontiguousarray(mono_frames[:F])).to(dev)
    d_k = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    d_d = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(F, dtype=torch.int32, device=dev)
    d_m = torch.zeros(F, dtype=torch.int32, device=dev)
    d_u = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    ex.extract_batch_device(d_img.data_ptr(), F, 752, 480, d_k.data_ptr(), d_d.data_ptr(), cap, d_n.data_ptr(),
                            d_m.data_ptr(), lap=(0, 1000), stream=s.cuda_stream)
    slamhot.undistort_keypoints_batch_device(K, D, F, d_k.data_ptr(), d_n.data_ptr(), cap, d_u.data_ptr(),
                                             stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    n = d_n.cpu().numpy()
    kk = d_k.cpu().numpy()
    uu = d_u.cpu().numpy()
    for f in range(F):
        k = kk[f, :n[f]].copy().view(ob.KP_DTYPE).ravel()
        u = uu[f, :n[f]].copy().view(ob.KP_DTYPE).ravel()
        assert np.array_equal(u.view(np.uint8), ob.undistort_keypoints(k, K, D).view(np.uint8))
    ex.close()
    assert np.array_equal(slamhot.ComputeImageBounds(K, D, 752, 480), ob.image_bounds(K, D, 752, 480))


def test_config1_monocular_sequence_through_cpp_host(mono_frames, tmp_path):
    """configs[0]: the first 3 frames through the initialisation extractor (5000 features), the
    rest through the 1000-feature tracking extractor, lapping area (0, 1000), mvKeysUn."""
    drv = ROOT / "tests" / "cpp" / "host_driver"
    n, n_init = len(mono_frames), 3
    (tmp_path / "imgs.u8").write_bytes(np.ascontiguousarray(mono_frames).tobytes())
    (tmp_path / "calib.bin").write_bytes(K.tobytes() + struct.pack("<i", len(D)) + D.tobytes())
    r = subprocess.run([str(drv), "mono", "752", "480", str(n), str(n_init), "1000", str(tmp_path / "imgs.u8"),
                        str(tmp_path / "calib.bin"), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    b = (tmp_path / "out.bin").read_bytes()
    bounds = np.frombuffer(b, np.float32, 4, 0)
    assert np.array_equal(bounds, ob.image_bounds(K, D, 752, 480))
    o = 16
    for f in range(n):
        cnt, mono = struct.unpack_from("<ii", b, o)
        o += 8
        kps = np.frombuffer(b, ob.KP_DTYPE, cnt, o)
        o += 28 * cnt
        kun = np.frombuffer(b, ob.KP_DTYPE, cnt, o)
        o += 28 * cnt
        desc = np.frombuffer(b, np.uint8, 32 * cnt, o).reshape(cnt, 32)
        o += 32 * cnt
        nf = 5000 if f < n_init else 1000
        ko, do, mo = ob.extract(mono_frames[f], ob.params(nfeatures=nf), lap=(0, 1000))
        assert cnt == len(ko) and mono == mo, (f, cnt, len(ko), mono, mo)
        assert np.array_equal(kps.view(np.uint8), ko.view(np.uint8)), f
        assert np.array_equal(desc, do), f
        assert np.array_equal(kun.view(np.uint8), ob.undistort_keypoints(ko, K, D).view(np.uint8)), f
        assert cnt > (3000 if f < n_init else 800)
    assert o == len(b)
