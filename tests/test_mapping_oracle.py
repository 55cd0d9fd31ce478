"""CPU checks of the LocalMapping-matcher oracle (oracle/mapping_oracle.cpp) against
independent numpy restatements.  Parity unpinned: the reference ships no fixtures for these."""
import ctypes as C

import numpy as np

import oracle_bind as ob
from fpexact import fmaf


def observation_sets(seed, n_mp=300, max_n=40):
    """Per MapPoint a cluster of observed descriptors (a base pattern plus a few bit flips,
    some outliers): many equal medians, so the first-index tie-break matters."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, max_n + 1, n_mp)
    sizes[:5] = [0, 1, 2, 3, 64]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    desc = np.zeros((off[-1], 32), np.uint8)
    for m in range(n_mp):
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        for j in range(sizes[m]):
            bits = np.unpackbits(base)
            flips = rng.integers(0, 4) if rng.random() < 0.85 else rng.integers(20, 120)
            bits[rng.choice(256, size=flips, replace=False)] ^= 1
            desc[off[m] + j] = np.packbits(bits)
    return off, desc


def np_distinctive(off, desc):
    bits = np.unpackbits(desc, axis=1)
    best = []
    for m in range(len(off) - 1):
        D = bits[off[m]:off[m + 1]]
        N = len(D)
        if N == 0:
            best.append(-1)
            continue
        dist = (D[:, None, :] != D[None, :, :]).sum(2)
        med = np.sort(dist, axis=1)[:, int(0.5 * (N - 1))]
        best.append(int(np.argmin(med)))  # first minimum
    return np.array(best, np.int32)


def test_distinctive_descriptors_oracle():
    off, desc = observation_sets(0)
    assert np.array_equal(ob.distinctive_descriptors(off, desc), np_distinctive(off, desc))


def test_fmaf_helper():
    rng = np.random.default_rng(0)
    for a, b, c in rng.normal(size=(2000, 3)).astype(np.float32):
        assert fmaf(a, b, np.float32(0)) == np.float32(a * b)  # one rounding of an exact product
        assert fmaf(a, np.float32(1), c) == np.float32(a + c)
    # a product whose low bits an unfused multiply-add would lose
    x = np.float32(1 + 2 ** -12)
    assert fmaf(x, x, np.float32(-1)) != np.float32(x * x) - np.float32(1)


def _py_triangulation(K1, K2, F, ep, only_stereo, coarse):
    """SearchForTriangulation_ (ORBmatcher.cc:1208-1433) without the rotation check, numpy
    float32 scalars with the compiled reference's contractions (exact fmaf above); F and ep
    from the pair's poses (oracle_fp_tri_geometry, pinned by tests/test_fp_sites.py);
    FeatureVector co-iteration as a dict intersection."""
    f32 = np.float32
    bits1, bits2 = np.unpackbits(K1["desc"], axis=1), np.unpackbits(K2["desc"], axis=1)
    nodes2 = {int(K2["node_id"][j]): K2["node_feat"][K2["node_off"][j]:K2["node_off"][j + 1]]
              for j in range(len(K2["node_id"]))}
    m12 = np.full(len(K1["kps_un"]), -1, np.int32)
    for j in range(len(K1["node_id"])):
        cand = nodes2.get(int(K1["node_id"][j]))
        if cand is None:
            continue
        for idx1 in K1["node_feat"][K1["node_off"][j]:K1["node_off"][j + 1]]:
            if K1["has_mp"][idx1]:
                continue
            s1 = K1["uright"][idx1] >= 0
            if only_stereo and not s1:
                continue
            k1 = K1["kps_un"][idx1]
            best, bi = 50, -1
            for idx2 in cand:
                if K2["has_mp"][idx2]:
                    continue
                s2 = K2["uright"][idx2] >= 0
                if only_stereo and not s2:
                    continue
                dist = int((bits1[idx1] != bits2[idx2]).sum())
                if dist > 50 or dist > best:
                    continue
                k2 = K2["kps_un"][idx2]
                if not s1 and not s2:
                    ex, ey = f32(ep[0] - k2["x"]), f32(ep[1] - k2["y"])
                    if fmaf(ex, ex, f32(ey * ey)) < f32(100 * K2["scale"][k2["octave"]]):
                        continue
                x1, y1 = f32(k1["x"]), f32(k1["y"])
                x2, y2 = f32(k2["x"]), f32(k2["y"])
                a = f32(fmaf(x1, F[0, 0], f32(y1 * F[1, 0])) + F[2, 0])
                b = f32(fmaf(x1, F[0, 1], f32(y1 * F[1, 1])) + F[2, 1])
                c = f32(fmaf(y1, F[1, 2], f32(x1 * F[0, 2])) + F[2, 2])
                num = f32(fmaf(b, y2, f32(a * x2)) + c)
                den = fmaf(a, a, f32(b * b))
                ok = den != 0 and float(f32(f32(num * num) / den)) < 3.84 * float(K2["level_sigma2"][k2["octave"]])
                if ok or coarse:
                    best, bi = dist, idx2
            m12[idx1] = bi
    return m12


def test_triangulation_oracle_vs_python():
    import scenes
    import slamhot
    kfs, poses = scenes.tri_keyframes(5, n_kf=2, n_pts=500)
    t1, k1 = slamhot.make_tri_kf(kfs[0])
    t2, k2 = slamhot.make_tri_kf(kfs[1])
    ep, R12, t12, F12 = (C.c_float * 2)(), (C.c_float * 9)(), (C.c_float * 3)(), (C.c_float * 9)()
    ob.lib().oracle_fp_tri_geometry(t1.Rcw, t1.tcw, t1.Ow, t1.cam, t2.Rcw, t2.tcw, t2.cam, ep, R12, t12, F12)
    F = np.array(F12[:], np.float32).reshape(3, 3)
    ep = np.array(ep[:], np.float32)
    for only_stereo, coarse in ((False, False), (True, False), (False, True)):
        pr = slamhot.make_tri_pair(0, 1, only_stereo, coarse)
        n, m12 = ob.search_for_triangulation(t1, t2, pr, False)
        ref = _py_triangulation(kfs[0], kfs[1], F, ep, only_stereo, coarse)
        assert np.array_equal(m12, ref)
        assert n == (ref >= 0).sum() and n > 20
