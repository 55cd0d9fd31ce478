"""GPU parity: libslamhot extractor vs the CPU oracle (ORBextractor.cc restated).

Bit-exact: pyramid pixels, keypoint order/coords/size/angle/response/octave, descriptor bits.
"""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu

SIZES = [(640, 480), (752, 480), (1280, 720)]


def _compare(kg, dg, mg, ko, do, mo):
    assert len(kg) == len(ko), (len(kg), len(ko))
    assert mg == mo
    for f in ("x", "y", "size", "response", "octave", "class_id"):
        bad = np.nonzero(kg[f] != ko[f])[0]
        assert bad.size == 0, (f, bad[:10], kg[bad[:3]], ko[bad[:3]])
    bad = np.nonzero(kg["angle"].view(np.uint32) != ko["angle"].view(np.uint32))[0]
    assert bad.size == 0, ("angle", bad[:10], kg[bad[:3]], ko[bad[:3]])
    bad = np.nonzero((dg != do).any(axis=1))[0]
    assert bad.size == 0, ("desc", bad[:10])


@pytest.mark.parametrize("size", SIZES)
def test_pyramid_bitexact(gpu_extractor_factory, size):
    w, h = size
    ex = gpu_extractor_factory(nfeatures=1000, max_size=size)
    img = synth.frame(7, w, h)
    ex(img)
    ref = ob.pyramid(img)
    for l in range(8):
        got = ex.pyramid_level(l)
        assert got.shape == ref[l].shape
        assert np.array_equal(got, ref[l]), (l, np.argwhere(got != ref[l])[:5])


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_extract_bitexact(gpu_extractor_factory, size, seed):
    w, h = size
    nf = 1200 if size == (752, 480) else 1000
    ex = gpu_extractor_factory(nfeatures=nf, max_size=size)
    img = synth.frame(100 + seed, w, h)
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img, ob.params(nfeatures=nf))
    _compare(kg, dg, mg, ko, do, mo)


@pytest.mark.parametrize("size", [(641, 479), (322, 241), (333, 247)])
def test_odd_sizes_bitexact(gpu_extractor_factory, size):
    """Rows that are not dword multiples (byte staging paths) and small levels where the
    7x7 blur window of a keypoint reflects at the level border (BORDER_REFLECT_101).  Smaller
    images make the reference divide by zero (ORBextractor.cc:783, nRows = 0 at level 7)."""
    w, h = size
    ex = gpu_extractor_factory(nfeatures=1000, max_size=size)
    img = synth.frame(55, w, h)
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img, ob.params(nfeatures=1000))
    _compare(kg, dg, mg, ko, do, mo)


@pytest.mark.parametrize("size", [(4095, 480), (3000, 320), (1920, 1080)])
def test_extreme_sizes_bitexact(gpu_extractor_factory, size):
    """The widest accepted image (4095 columns: level pitch 4096; 9-10 DistributeOctTree roots per
    level), a 3000 x 320 strip (12-15 roots, near the 16-root table), and full HD, 2000 features;
    pyramid and keypoints bit-exact."""
    w, h = size
    ex = gpu_extractor_factory(nfeatures=2000, max_size=size)
    img = synth.frame(77, w, h)
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img, ob.params(nfeatures=2000))
    _compare(kg, dg, mg, ko, do, mo)
    ref = ob.pyramid(img)
    for l in range(8):
        assert np.array_equal(ex.pyramid_level(l), ref[l]), l


def test_root_table_limits_rejected():
    """More than 16 DistributeOctTree roots on a level (an aspect ratio beyond ~16:1, e.g. 4095 x
    250: 19-29 roots) is outside the device's root table: SLAM_EINVAL at create, no launch."""
    import slamhot
    with pytest.raises(slamhot.SlamError) as e:
        slamhot.ORBextractor(nfeatures=1000, max_size=(4095, 250))
    assert e.value.status == slamhot.SLAM_EINVAL


def test_portrait_geometry_rejected():
    """An image more than ~2x taller than wide: DistributeOctTree's root count
    round((maxX - minX) / (maxY - minY)) is 0 on some level and the reference divides by it and
    reads an empty node list (ORBextractor.cc:541-560, undefined behaviour; the restated oracle
    crashes the same way, so it is not run here).  The device extractor refuses the geometry
    when the handle is created: SLAM_EINVAL, no launch."""
    import slamhot
    with pytest.raises(slamhot.SlamError) as e:
        slamhot.ORBextractor(nfeatures=1000, max_size=(256, 2400))
    assert e.value.status == slamhot.SLAM_EINVAL


@pytest.mark.parametrize("lap", [(0, 0), (0, 1000), (100, 400)])
def test_lapping_order(gpu_extractor_factory, lap):
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480))
    img = synth.frame(5)
    kg, dg, mg = ex(img, lap)
    ko, do, mo = ob.extract(img, ob.params(), lap=lap)
    _compare(kg, dg, mg, ko, do, mo)


def test_batch_matches_single(gpu_extractor_factory):
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480), max_batch=8)
    imgs = synth.frames(range(20, 28))
    kps, desc, n, mono = ex.extract_batch(imgs)
    for f in range(8):
        ko, do, mo = ob.extract(imgs[f])
        _compare(kps[f][: n[f]], desc[f][: n[f]], mono[f], ko, do, mo)


@pytest.mark.parametrize("nf", [500, 2000, 5000])
def test_feature_budgets(gpu_extractor_factory, nf):
    ex = gpu_extractor_factory(nfeatures=nf, max_size=(752, 480))
    img = synth.frame(33, 752, 480)
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img, ob.params(nfeatures=nf))
    _compare(kg, dg, mg, ko, do, mo)


def test_flat_and_noise_images(gpu_extractor_factory):
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480))
    rng = np.random.default_rng(3)
    for img in (np.full((480, 640), 128, np.uint8),
                rng.integers(0, 256, (480, 640), dtype=np.uint8)):
        kg, dg, mg = ex(img)
        ko, do, mo = ob.extract(img)
        _compare(kg, dg, mg, ko, do, mo)


def test_low_contrast_minth_retry(gpu_extractor_factory):
    """Low-contrast texture (corners mostly between minThFAST 7 and iniThFAST 20), next to a
    high-contrast half: most cells of the left half are empty at iniTh and take the minTh
    attempt (ORBextractor.cc:825-841), the right half does not."""
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480))
    rng = np.random.default_rng(11)
    img = (128 + rng.integers(-9, 10, (480, 640))).astype(np.uint8)
    img[:, 320:] = synth.frame(12)[:, 320:]
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img)
    assert len(ko) > 500
    _compare(kg, dg, mg, ko, do, mo)


def test_minth_retry_dense_compass(gpu_extractor_factory):
    """A one-pixel checkerboard of amplitude 12 (100 / 112) on the left half: every pixel passes
    the compass pre-test at minThFAST 7 and none at iniThFAST 20, and no 9-arc exists at either
    (12 of the 16 circle pixels have the centre's colour).  Its cells are empty at iniTh, and
    their minTh attempt grows the pass-A list past the compass scores the first attempt kept at
    the end of the list region, so k_fast_wave falls back to deriving them from the ROI again.
    Textured right half."""
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480))
    yy, xx = np.mgrid[0:480, 0:640]
    img = np.where((xx + yy) & 1, 112, 100).astype(np.uint8)
    img[:, 320:] = synth.frame(13)[:, 320:]
    kg, dg, mg = ex(img)
    ko, do, mo = ob.extract(img)
    assert len(ko) > 300
    _compare(kg, dg, mg, ko, do, mo)


def test_kitti_stereo_settings(gpu_extractor_factory):
    """Examples/Stereo/KITTI04-12.yaml:21-54: 1241 x 376, 2000 features, iniThFAST 12, minThFAST 7."""
    ex = gpu_extractor_factory(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=12, minThFAST=7,
                               max_size=(1241, 376))
    for seed in (3, 4):
        img = synth.frame(300 + seed, 1241, 376)
        kg, dg, mg = ex(img)
        ko, do, mo = ob.extract(img, ob.params(nfeatures=2000, ini=12, mn=7))
        _compare(kg, dg, mg, ko, do, mo)
        assert len(kg) > 1800


@pytest.mark.parametrize("scale,levels,nf", [(1.3, 6, 1000), (1.15, 10, 1500), (2.0, 3, 800), (1.2, 1, 500),
                                             (1.05, 16, 1200)])
def test_non_default_pyramid(gpu_extractor_factory, scale, levels, nf):
    """Other ORBextractor.scaleFactor / nLevels: the level geometry, per-level feature split and
    the scale tables follow the parameters (ORBextractor.cc:408-468, 1152-1177).  16 levels is the
    most the plan takes (kMaxLevels): k_orb3's level lookup reads every level's first slot, and the
    last level's keypoints must come out bit-exact too."""
    ex = gpu_extractor_factory(nfeatures=nf, scaleFactor=scale, nlevels=levels, max_size=(752, 480))
    img = synth.frame(410 + levels, 752, 480)
    kg, dg, mg = ex(img)
    p = ob.params(nfeatures=nf, scale=scale, nlevels=levels)
    ko, do, mo = ob.extract(img, p)
    _compare(kg, dg, mg, ko, do, mo)
    assert (kg["octave"] == levels - 1).sum() > 0  # the last level holds keypoints
    sc, isc, s2, is2, nfl = ob.levels(p)
    assert np.array_equal(ex.GetScaleFactors(), sc) and np.array_equal(ex.GetInverseScaleSigmaSquares(), is2)
    assert np.array_equal(ex.GetFeaturesPerLevel(), nfl)
    ref = ob.pyramid(img, p)
    for l in range(levels):
        assert np.array_equal(ex.pyramid_level(l), ref[l]), l


@pytest.mark.parametrize("small,l0", [("1", "1"), ("0", "0")])
def test_octree_wave_forms(gpu_extractor_factory, monkeypatch, small, l0):
    """k_octree<4> (key loops over four waves, node-list scans on wave 0) and k_octree<1> give the
    same keypoints: the per-image call (all levels in one launch) and a 10-frame batch (level 0 in
    its own launch) with each form, bit-exact against the oracle.  Textured VGA frames put ~3.6k
    candidates on level 0 (several key-loop rounds per wave) and reach the careful phase."""
    monkeypatch.setenv("SLAMHOT_OCT_SMALL", small)
    monkeypatch.setenv("SLAMHOT_OCT_L0", l0)
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(640, 480), max_batch=10)
    for seed in (3, 91):
        img = synth.frame(seed)
        _compare(*ex(img), *ob.extract(img))
    imgs = synth.frames(range(70, 80))
    kps, desc, n, mono = ex.extract_batch(imgs)
    for f in range(10):
        ko, do, mo = ob.extract(imgs[f])
        _compare(kps[f][: n[f]], desc[f][: n[f]], mono[f], ko, do, mo)
    ex2 = gpu_extractor_factory(nfeatures=5000, max_size=(752, 480))  # Tracking's 5x init extractor
    img = synth.frame(92, 752, 480)
    _compare(*ex2(img), *ob.extract(img, ob.params(nfeatures=5000)))


@pytest.mark.parametrize("graph", ["1", "0"])
def test_host_call_graph_and_stream_paths(gpu_extractor_factory, monkeypatch, graph):
    """The per-image host-buffer call is captured as a HIP graph per shape (frame size, lapping
    area, batch size, capacity) and replayed; SLAMHOT_EXTRACT_GRAPH=0 keeps plain stream calls.
    One handle alternates shapes (re-capture) and repeats them (replay); a 5-frame batch takes the
    small-batch launches (one FAST dispatch, one octree launch); a 12-frame batch the batch
    pipeline.  Every result bit-exact against the oracle."""
    monkeypatch.setenv("SLAMHOT_EXTRACT_GRAPH", graph)
    ex = gpu_extractor_factory(nfeatures=1000, max_size=(752, 480), max_batch=12)
    calls = [((640, 480), (0, 0), 40), ((752, 480), (0, 1000), 41), ((640, 480), (0, 0), 42),
             ((640, 480), (100, 400), 43), ((752, 480), (0, 1000), 44)]
    for (w, h), lap, seed in calls:
        img = synth.frame(seed, w, h)
        kg, dg, mg = ex(img, lap)
        ko, do, mo = ob.extract(img, ob.params(), lap=lap)
        _compare(kg, dg, mg, ko, do, mo)
    for nb in (5, 12):
        imgs = synth.frames(range(60, 60 + nb))
        kps, desc, n, mono = ex.extract_batch(imgs)
        for f in range(nb):
            ko, do, mo = ob.extract(imgs[f])
            _compare(kps[f][: n[f]], desc[f][: n[f]], mono[f], ko, do, mo)
