"""CPU oracle known-answer tests and independent cross-checks (no GPU).

The oracle restates ORBextractor/ORBmatcher and the OpenCV 4.2.0 primitives they call; no
reference golden vectors exist for this path, so these tests pin the
restatement: known answers, an independent numpy formulation of each primitive, and the
committed fixtures in tests/golden/ (regression)."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

OFF16 = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
         (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


# ------------------------------------------------------------------ scale tables
def test_levels_match_reference_tables():
    scale, inv, s2, inv2, nf = ob.levels(ob.params(nfeatures=1000))
    assert nf.tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    _, _, _, _, nf1200 = ob.levels(ob.params(nfeatures=1200))
    assert nf1200.tolist() == [261, 217, 181, 151, 126, 105, 87, 72]
    assert scale[0] == 1 and abs(scale[1] - 1.2) < 1e-6
    assert np.allclose(s2, scale * scale) and np.allclose(inv * scale, 1)


def test_pyramid_sizes():
    sizes = [p.shape[::-1] for p in ob.pyramid(synth.frame(0))]
    assert sizes == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161),
                     (179, 134)]


# ------------------------------------------------------------------ resize
def np_resize_linear(src, dw, dh):
    """Independent numpy restatement of OpenCV 4.2.0 INTER_LINEAR 8U (fixed point 2^11)."""
    sh, sw = src.shape
    sx_scale, sy_scale = 1.0 / (dw / sw), 1.0 / (dh / sh)
    dx = np.arange(dw)
    fx = ((dx + 0.5) * sx_scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    fx = np.where(sx < 0, np.float32(0), fx)
    sx = np.where(sx < 0, 0, sx)
    clip = sx + 1 >= sw
    xmax = int(np.argmax(clip)) if clip.any() else dw
    fx = np.where(sx >= sw - 1, np.float32(0), fx)
    sx = np.where(sx >= sw - 1, sw - 1, sx)
    a0 = np.rint((np.float32(1) - fx) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(fx * np.float32(2048)).astype(np.int64)
    s = src.astype(np.int64)
    sx1 = np.minimum(sx + 1, sw - 1)
    D = s[:, sx] * a0 + s[:, sx1] * a1
    D[:, xmax:] = s[:, sx[xmax:]] * 2048
    dy = np.arange(dh)
    fy = ((dy + 0.5) * sy_scale - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = np.rint((np.float32(1) - fy) * np.float32(2048)).astype(np.int64)
    b1 = np.rint(fy * np.float32(2048)).astype(np.int64)
    y0 = np.clip(sy, 0, sh - 1)
    y1 = np.clip(sy + 1, 0, sh - 1)
    out = (((b0[:, None] * (D[y0] >> 4)) >> 16) + ((b1[:, None] * (D[y1] >> 4)) >> 16) + 2) >> 2
    return out.astype(np.uint8)


@pytest.mark.parametrize("shape,dst", [((480, 640), (533, 400)), ((400, 533), (444, 333)),
                                       ((137, 91), (76, 114)), ((50, 60), (50, 42))])
def test_resize_matches_numpy_restatement(shape, dst):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, shape, dtype=np.uint8)
    got = ob.resize_linear(src, *dst)
    ref = np_resize_linear(src, *dst)
    assert np.array_equal(got, ref)


def test_resize_constant_and_pyramid_chain():
    src = np.full((480, 640), 77, np.uint8)
    assert (ob.resize_linear(src, 533, 400) == 77).all()
    img = synth.frame(3)
    pyr = ob.pyramid(img)
    for l in range(1, 8):
        assert np.array_equal(pyr[l], np_resize_linear(pyr[l - 1], pyr[l].shape[1], pyr[l].shape[0]))


# ------------------------------------------------------------------ FAST
def np_fast(roi, t):
    """Independent formulation of cv::FAST(roi, t, nonmax): corner = 9 contiguous of 16
    brighter/darker; score = max over 9-windows of min|d| (sign-consistent) - 1; strict 3x3
    NMS with non-corners and untested pixels counting as 0."""
    h, w = roi.shape
    I = roi.astype(np.int32)
    score = np.zeros((h, w), np.int32)
    corner = np.zeros((h, w), bool)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = I[y, x]
            d = np.array([v - I[y + dy, x + dx] for dx, dy in OFF16])
            dd = np.concatenate([d, d[:8]])
            win_min = np.array([dd[s:s + 9].min() for s in range(16)])
            win_max = np.array([dd[s:s + 9].max() for s in range(16)])
            M = max(win_min.max(), -win_max.min())
            if M > t:
                corner[y, x] = True
                score[y, x] = M - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if not corner[y, x]:
                continue
            s = score[y, x]
            nb = score[y - 1:y + 2, x - 1:x + 2].copy()
            nb[1, 1] = -1
            if (s > nb).all():
                out.append((x, y, s))
    return np.array(out, np.int32).reshape(-1, 3)


@pytest.mark.parametrize("t", [7, 20, 0, 60])
def test_fast_matches_independent_formulation(t):
    rng = np.random.default_rng(t)
    for trial in range(3):
        roi = rng.integers(0, 256, (30, 33), dtype=np.uint8)
        if trial == 1:
            roi = (roi // 64 * 64).astype(np.uint8)  # plateaus: ties in scores
        if trial == 2:
            roi = synth.frame(trial)[100:140, 200:245]
        got = ob.fast(roi, t)
        ref = np_fast(roi, t)
        assert np.array_equal(got, ref), (t, trial)


def test_fast_known_answers():
    assert len(ob.fast(np.full((20, 20), 100, np.uint8), 7)) == 0
    img = np.zeros((15, 15), np.uint8)
    img[7, 7] = 255
    kps = ob.fast(img, 20)
    assert kps.tolist() == [[7, 7, 254]]


# ------------------------------------------------------------------ blur
def np_blur(img, k):
    h, w = img.shape
    pad = np.pad(img.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    H = sum(k[i] * pad[:, i:i + w] for i in range(7))
    V = sum(k[j] * H[j:j + h, :] for j in range(7))
    return np.minimum((V + (1 << 15)) >> 16, 255).astype(np.uint8)


def test_blur_known_answers_and_kernel_switch():
    const = np.full((40, 50), 200, np.uint8)
    assert (ob.gaussian_blur7(const, ed=True) == 200).all()       # ED kernel sums to 256
    assert (ob.gaussian_blur7(const, ed=False) == 202).all()      # per-tap kernel sums to 257
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (37, 61), dtype=np.uint8)
    assert np.array_equal(ob.gaussian_blur7(img, True), np_blur(img, [18, 34, 48, 56, 48, 34, 18]))
    assert np.array_equal(ob.gaussian_blur7(img, False), np_blur(img, [18, 34, 49, 55, 49, 34, 18]))


# ------------------------------------------------------------------ angle, sincos
def test_fast_atan2_known_answers():
    assert ob.fast_atan2(0.0, 1.0) == 0.0
    assert abs(ob.fast_atan2(1.0, 1.0) - 45.0) < 0.01
    assert abs(ob.fast_atan2(1.0, 0.0) - 90.0) < 0.01
    assert abs(ob.fast_atan2(0.0, -1.0) - 180.0) < 0.01
    assert abs(ob.fast_atan2(-1.0, 0.0) - 270.0) < 0.01
    rng = np.random.default_rng(0)
    y = rng.normal(0, 1e5, 20000).astype(np.float32)
    x = rng.normal(0, 1e5, 20000).astype(np.float32)
    ref = np.degrees(np.arctan2(y, x)) % 360
    got = np.array([ob.fast_atan2(a, b) for a, b in zip(y[:2000], x[:2000])])
    err = np.abs((got - ref[:2000] + 180) % 360 - 180)
    assert err.max() < 0.02  # OpenCV fastAtan2 accuracy class
    assert ob.check_atan2(y, x) == 0  # device restatement == oracle, bit for bit


def test_sincosf_restatement_exhaustive():
    """device_math_core.hpp's glibc sincosf restatement vs this host's glibc, every float
    in [0, 6.3) (the descriptor's whole angle range)."""
    assert ob.check_sincosf(0.0, 6.3) == 0


# ------------------------------------------------------------------ extractor
def test_extract_lapping_reverses_order():
    img = synth.frame(4)
    k0, d0, m0 = ob.extract(img, lap=(0, 0))
    k1, d1, m1 = ob.extract(img, lap=(0, 1000))
    assert m0 == len(k0) and m1 == 0
    assert np.array_equal(k1[::-1], k0) and np.array_equal(d1[::-1], d0)


def test_extract_invariants():
    img = synth.frame(5, 752, 480)
    k, d, m = ob.extract(img, ob.params(nfeatures=1200))
    _, _, _, _, nf = ob.levels(ob.params(nfeatures=1200))
    counts = np.bincount(k["octave"], minlength=8)
    assert (counts >= nf).all() and (counts <= nf + 3).all()
    assert (np.diff(k["octave"]) >= 0).all()  # level-major order
    assert ((k["angle"] >= 0) & (k["angle"] < 360)).all()
    assert (k["class_id"] == -1).all()
    sizes = np.array([31, 37, 44, 53, 64, 77, 92, 111], np.float32)
    assert np.array_equal(k["size"], sizes[k["octave"]])


def test_extract_flat_image_has_no_keypoints():
    k, d, m = ob.extract(np.full((480, 640), 90, np.uint8))
    assert len(k) == 0 and m == 0


# ------------------------------------------------------------------ matchers
def test_hamming_matches_numpy():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    ref = np.unpackbits(a ^ b, axis=1).sum(1)
    got = np.array([ob.descriptor_distance(x, y) for x, y in zip(a, b)])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("counts,expect", [
    ([0] * 30, (-1, -1, -1)),
    ([5] + [0] * 29, (0, -1, -1)),
    ([10, 2, 1] + [0] * 27, (0, 1, 2)),           # 1 is not < 0.1*10 = 1.0
    ([10, 0, 0, 9, 9] + [0] * 25, (0, 3, 4)),     # ties: strict ">" keeps the first
    ([100, 9, 50] + [0] * 27, (0, 2, -1)),
    ([100, 5, 8] + [0] * 27, (0, -1, -1)),        # max2 < 0.1*max1 drops both
])
def test_three_maxima(counts, expect):
    assert ob.three_maxima(counts) == expect


def py_search_by_bow(A, B, nnratio, check_ori, strict):
    """Plain-Python restatement of ORBmatcher::SearchByBoW for cross-checking the oracle."""
    dA, angA, vA, nidA, offA, featA = A
    dB, angB, vB, nidB, offB, featB = B
    ham = lambda x, y: int(np.unpackbits(x ^ y).sum())
    a2b = {}
    b2a = {}
    bins = {}
    posB = {int(n): i for i, n in enumerate(nidB)}
    for ia, node in enumerate(nidA):
        if int(node) not in posB:
            continue
        ib = posB[int(node)]
        for ka in featA[offA[ia]:offA[ia + 1]]:
            if vA is not None and not vA[ka]:
                continue
            b1, b2, bi = 256, 256, -1
            for kb in featB[offB[ib]:offB[ib + 1]]:
                if kb in b2a or (vB is not None and not vB[kb]):
                    continue
                dist = ham(dA[ka], dB[kb])
                if dist < b1:
                    b2, b1, bi = b1, dist, kb
                elif dist < b2:
                    b2 = dist
            ok = b1 < 50 if strict else b1 <= 50
            if ok and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                a2b[ka] = bi
                b2a[bi] = ka
                rot = np.float32(angA[ka]) - np.float32(angB[bi])
                if rot < 0:
                    rot = np.float32(rot + np.float32(360))
                r = np.float32(rot * np.float32(1.0 / 30))
                bn = int(np.floor(r + np.float32(0.5)))
                bins[ka] = 0 if bn == 30 else bn
    if check_ori:
        counts = np.bincount(np.array(list(bins.values()), int), minlength=30)[:30]
        keep = ob.three_maxima(counts)
        for ka, bn in list(bins.items()):
            if bn not in keep:
                del b2a[a2b.pop(ka)]
    return len(a2b), a2b


def test_search_by_bow_oracle_vs_python():
    par, leaf, dn, wn = synth.vocab(6, 3, 1)
    rng = np.random.default_rng(4)
    base = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    noise = rng.random((300, 256)) < 0.05
    other = np.packbits(np.unpackbits(base, axis=1) ^ noise, axis=1)
    _, wa, na = ob.vocab_transform(par, leaf, dn, wn, 3, base, 1)
    _, wb, nb = ob.vocab_transform(par, leaf, dn, wn, 3, other, 1)
    ang_a = rng.uniform(0, 360, 300).astype(np.float32)
    ang_b = ((ang_a + rng.normal(0, 10, 300)) % 360).astype(np.float32)
    for strict, vA, vB in [(False, (rng.random(300) < .8).astype(np.uint8), None),
                           (True, (rng.random(300) < .8).astype(np.uint8), (rng.random(300) < .8).astype(np.uint8))]:
        A = (base, ang_a, vA) + synth.feature_vector(na, wa)
        B = (other, ang_b, vB) + synth.feature_vector(nb, wb)
        for check_ori in (True, False):
            n, a2b, b2a = ob.search_by_bow(A, B, 0.8, check_ori, strict)
            pn, pa2b = py_search_by_bow(A, B, 0.8, check_ori, strict)
            assert n == pn
            assert {i: int(a2b[i]) for i in np.nonzero(a2b >= 0)[0]} == pa2b
