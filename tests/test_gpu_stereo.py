"""GPU parity: Frame::ComputeStereoMatches (Frame.cc:794-964) through
slamhot_stereo_match_batch_device vs the CPU oracle (oracle/stereo_oracle.cpp) on the same
keypoints, descriptors and pyramids — mvuRight / mvDepth bit-exact."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu

MBF = synth.EUROC_STEREO["bf"]
MB = MBF / synth.EUROC_STEREO["fx"]


def _pairs(specs, W=752, H=480):
    L, R = [], []
    for seed, dmin, dmax, noise in specs:
        l, r = synth.stereo_pair(seed, W, H, dmin, dmax, noise)
        L.append(l)
        R.append(r)
    return np.stack(L), np.stack(R)


def _check(left, right, out, nfeat, mbf=MBF, mb=MB):
    sc = left.GetScaleFactors()
    isc = left.GetInverseScaleFactors()
    kept = 0
    for f, (kl, dl, kr, dr, ur, dep) in enumerate(out):
        pl = [left.pyramid_level(l, f) for l in range(left.nlevels)]
        pr = [right.pyramid_level(l, f) for l in range(right.nlevels)]
        ur_o, dep_o = ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, mbf, mb)
        assert np.array_equal(ur, ur_o), f"frame {f}: {np.flatnonzero(ur != ur_o)[:10]}"
        assert np.array_equal(dep, dep_o)
        kept += int((ur >= 0).sum())
    return kept


def test_stereo_batch_bitexact():
    import slamhot
    specs = [(1, 4.0, 40.0, 2.0), (2, 2.0, 20.0, 3.0), (3, 10.0, 80.0, 2.0), (4, 0.5, 6.0, 1.0)]
    il, ir = _pairs(specs)
    F, H, W = il.shape
    left = slamhot.ORBextractor(nfeatures=1200, max_size=(W, H), max_batch=F)
    right = slamhot.ORBextractor(nfeatures=1200, max_size=(W, H), max_batch=F)
    out = slamhot.ComputeStereoMatches(left, right, il, ir, MBF, MB)
    # the extraction itself is the reference's (frame 0 against the oracle extractor)
    k0, d0, _ = ob.extract(il[0], ob.params(nfeatures=1200))
    assert np.array_equal(out[0][0].view(np.uint8), k0.view(np.uint8))
    assert np.array_equal(out[0][1], d0)
    kept = _check(left, right, out, 1200)
    assert kept > 4 * 300
    # matched disparities sit on the synthetic field (sanity of the whole pipeline)
    kl, _, _, _, ur, _ = out[0]
    m = ur >= 0
    assert np.median(kl["x"][m] - ur[m]) > 4.0
    left.close()
    right.close()


def test_stereo_small_and_wide_baselines():
    """Tiny mb (huge maxD: every band candidate passes the u window) and a large one."""
    import slamhot
    il, ir = _pairs([(5, 3.0, 30.0, 2.0), (6, 1.0, 12.0, 2.0)], 640, 480)
    F, H, W = il.shape
    left = slamhot.ORBextractor(nfeatures=1000, max_size=(W, H), max_batch=F)
    right = slamhot.ORBextractor(nfeatures=1000, max_size=(W, H), max_batch=F)
    for mbf, mb in ((MBF, 0.01), (MBF, 2.0), (20.0, 0.05)):
        out = slamhot.ComputeStereoMatches(left, right, il, ir, mbf, mb)
        _check(left, right, out, 1000, mbf, mb)
    left.close()
    right.close()


@pytest.mark.parametrize("levels, scale", [(12, 1.1), (16, 1.05), (4, 1.6)])
def test_stereo_non_default_pyramids(levels, scale):
    """Octaves past 7 and wide / narrow row bands (2 * scale[octave]): the band table's packed
    octave and x, and the SAD windows on every level, against the oracle (odd width, 733 x 461)."""
    import slamhot
    il, ir = _pairs([(7, 3.0, 30.0, 2.0), (8, 1.0, 12.0, 2.0)], 733, 461)
    F, H, W = il.shape
    kw = dict(nfeatures=1500, scaleFactor=scale, nlevels=levels, max_size=(W, H), max_batch=F)
    left, right = slamhot.ORBextractor(**kw), slamhot.ORBextractor(**kw)
    out = slamhot.ComputeStereoMatches(left, right, il, ir, MBF, MB)
    assert _check(left, right, out, 1500) > 100
    assert max(int(o[0]["octave"].max()) for o in out) >= min(levels - 1, 8)
    left.close()
    right.close()


def test_stereo_same_image_and_empty_right():
    """Right == left + noise (disparities around 0: the disparity <= 0 branch) and a flat
    right image (no right keypoints: every mvuRight stays -1)."""
    import slamhot
    l = synth.frame(9, 752, 480)
    rng = np.random.default_rng(2)
    r_same = np.clip(l.astype(np.int32) + rng.integers(-3, 4, size=l.shape), 0, 255).astype(np.uint8)
    r_flat = np.full_like(l, 128)
    il = np.stack([l, l])
    ir = np.stack([r_same, r_flat])
    left = slamhot.ORBextractor(nfeatures=1000, max_size=(752, 480), max_batch=2)
    right = slamhot.ORBextractor(nfeatures=1000, max_size=(752, 480), max_batch=2)
    out = slamhot.ComputeStereoMatches(left, right, il, ir, MBF, MB)
    _check(left, right, out, 1000)
    assert len(out[1][2]) == 0
    assert np.all(out[1][4] == -1) and np.all(out[1][5] == -1)
    assert (out[0][4] >= 0).sum() > 100
    left.close()
    right.close()


def test_stereo_geometry_mismatch_rejected():
    import torch

    import slamhot
    left = slamhot.ORBextractor(nfeatures=500, max_size=(752, 480), max_batch=1)
    right = slamhot.ORBextractor(nfeatures=500, max_size=(752, 480), max_batch=1)
    il = synth.frame(3, 752, 480)[None]
    ir = synth.frame(4, 640, 480)[None]
    dev = torch.device("cuda", 0)
    cap = left.cap
    bufs = []
    for ex, im in ((left, il), (right, ir)):
        d_img = torch.from_numpy(im).to(dev)
        d_k = torch.zeros((1, cap, 28), dtype=torch.uint8, device=dev)
        d_d = torch.zeros((1, cap, 32), dtype=torch.uint8, device=dev)
        d_n = torch.zeros(1, dtype=torch.int32, device=dev)
        d_m = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        ex.extract_batch_device(d_img.data_ptr(), 1, im.shape[2], im.shape[1], d_k.data_ptr(), d_d.data_ptr(), cap,
                                d_n.data_ptr(), d_m.data_ptr())
        bufs.append((d_img, d_k, d_d, d_n))
    torch.cuda.synchronize()
    d_ur = torch.empty((1, cap), dtype=torch.float32, device=dev)
    d_dep = torch.empty((1, cap), dtype=torch.float32, device=dev)
    m = slamhot.StereoMatcher()
    (_, kl, dl, nl), (_, kr, dr, nr) = bufs
    with pytest.raises(slamhot.SlamError):
        m.match_batch_device(left, right, 1, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(),
                             dr.data_ptr(), nr.data_ptr(), cap, MBF, MB, d_ur.data_ptr(), d_dep.data_ptr())
    with pytest.raises(slamhot.SlamError):  # two frames requested, one extracted
        m.match_batch_device(left, left, 2, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kl.data_ptr(),
                             dl.data_ptr(), nl.data_ptr(), cap, MBF, MB, d_ur.data_ptr(), d_dep.data_ptr())
    m.close()
    left.close()
    right.close()


def test_stereo_stream_ordered_batch():
    """The bench's shape: both extractions and the matcher queued on one stream with no host
    sync in between, 16 pairs per batch."""
    import torch

    import slamhot
    P, W, H = 16, 752, 480
    prs = [synth.stereo_pair(500 + s, W, H) for s in range(P)]
    il = np.stack([p[0] for p in prs])
    ir = np.stack([p[1] for p in prs])
    dev = torch.device("cuda", 0)
    left = slamhot.ORBextractor(nfeatures=1200, max_size=(W, H), max_batch=P)
    right = slamhot.ORBextractor(nfeatures=1200, max_size=(W, H), max_batch=P)
    sm = slamhot.StereoMatcher()
    cap = left.cap
    d_il, d_ir = torch.from_numpy(il).to(dev), torch.from_numpy(ir).to(dev)
    bufs = [(torch.zeros((P, cap, 28), dtype=torch.uint8, device=dev),
             torch.zeros((P, cap, 32), dtype=torch.uint8, device=dev),
             torch.zeros(P, dtype=torch.int32, device=dev), torch.zeros(P, dtype=torch.int32, device=dev))
            for _ in range(2)]
    d_ur = torch.empty((P, cap), dtype=torch.float32, device=dev)
    d_dep = torch.empty((P, cap), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)  # a real stream: NULL would mean each handle's own stream
    torch.cuda.synchronize()
    for ex, img, (k, d, n, m) in ((left, d_il, bufs[0]), (right, d_ir, bufs[1])):
        ex.extract_batch_device(img.data_ptr(), P, W, H, k.data_ptr(), d.data_ptr(), cap, n.data_ptr(),
                                m.data_ptr(), stream=stream.cuda_stream)
    (kl, dl, nl, _), (kr, dr, nr, _) = bufs
    sm.match_batch_device(left, right, P, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(), dr.data_ptr(),
                          nr.data_ptr(), cap, MBF, MB, d_ur.data_ptr(), d_dep.data_ptr(), stream=stream.cuda_stream)
    torch.cuda.synchronize()
    nl_h, nr_h = nl.cpu().numpy(), nr.cpu().numpy()
    kl_h, kr_h = kl.cpu().numpy().view(ob.KP_DTYPE), kr.cpu().numpy().view(ob.KP_DTYPE)
    dl_h, dr_h = dl.cpu().numpy(), dr.cpu().numpy()
    ur, dep = d_ur.cpu().numpy(), d_dep.cpu().numpy()
    out = [(kl_h[f, :nl_h[f]].ravel(), dl_h[f, :nl_h[f]], kr_h[f, :nr_h[f]].ravel(), dr_h[f, :nr_h[f]],
            ur[f, :nl_h[f]], dep[f, :nl_h[f]]) for f in range(P)]
    kept = _check(left, right, out, 1200)
    assert kept > P * 200
    sm.close()
    left.close()
    right.close()


def test_stereo_host_buffer_form():
    """slamhot_compute_stereo_matches: the Frame constructor's host path (two host extractions,
    then ComputeStereoMatches on host keypoints) equals the oracle."""
    import slamhot
    il, ir = _pairs([(7, 4.0, 40.0, 2.0)])
    left = slamhot.ORBextractor(nfeatures=1200, max_size=(752, 480))
    right = slamhot.ORBextractor(nfeatures=1200, max_size=(752, 480))
    kl, dl, _ = left(il[0])
    kr, dr, _ = right(ir[0])
    sm = slamhot.StereoMatcher()
    ur, dep = sm.compute(left, right, kl, dl, kr, dr, MBF, MB)
    assert _check(left, right, [(kl, dl, kr, dr, ur, dep)], 1200) > 300
    sm.close()
    left.close()
    right.close()
