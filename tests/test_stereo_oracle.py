"""CPU checks of the ComputeStereoMatches oracle (oracle/stereo_oracle.cpp): an independent
numpy/Python restatement of Frame.cc:794-964 agrees with it bit for bit, disparities land on
the synthetic field, and the reference's edge behaviour (no right keypoints, median cut)
holds.  Parity unpinned: the reference ships no stereo fixtures."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

MBF = synth.EUROC_STEREO["bf"]
MB = MBF / synth.EUROC_STEREO["fx"]


@pytest.fixture(scope="module")
def pair():
    l, r = synth.stereo_pair(1, 752, 480, 4.0, 40.0, 2.0)
    p = ob.params(nfeatures=1200)
    kl, dl, _ = ob.extract(l, p)
    kr, dr, _ = ob.extract(r, p)
    sc, isc, _, _, _ = ob.levels(p)
    return kl, dl, kr, dr, ob.pyramid(l, p), ob.pyramid(r, p), sc, isc


def _cround(x):
    """std::round: half away from zero (np.round rounds half to even)."""
    return np.float32(np.sign(x) * np.floor(np.abs(np.float64(x)) + 0.5))


def _py_stereo(kl, dl, kr, dr, pl, pr, sc, isc, mbf, mb, cut=True):
    """Frame::ComputeStereoMatches restated with numpy float32 scalars (Frame.cc:794-964)."""
    f32 = np.float32
    n = len(kl)
    ur = np.full(n, -1, np.float32)
    dep = np.full(n, -1, np.float32)
    nrows = pl[0].shape[0]
    rows = [[] for _ in range(nrows)]
    for iR in range(len(kr)):
        y = f32(kr["y"][iR])
        r = f32(2.0) * sc[kr["octave"][iR]]
        for yi in range(int(np.floor(f32(y - r))), int(np.ceil(f32(y + r))) + 1):
            if 0 <= yi < nrows:
                rows[yi].append(iR)
    bits = np.unpackbits(dr, axis=1)
    maxD = f32(f32(mbf) / f32(mb))
    kept = []
    for iL in range(n):
        uL, vL, lev = f32(kl["x"][iL]), f32(kl["y"][iL]), int(kl["octave"][iL])
        cands = rows[int(vL)]
        if not cands:
            continue
        minU, maxU = f32(uL - maxD), uL
        if maxU < 0:
            continue
        c = np.array(cands)
        ok = (kr["octave"][c] >= lev - 1) & (kr["octave"][c] <= lev + 1) & (kr["x"][c] >= minU) & (kr["x"][c] <= maxU)
        c = c[ok]
        if len(c) == 0:
            continue
        dist = (np.unpackbits(dl[iL])[None, :] != bits[c]).sum(1)
        j = int(np.argmin(dist))  # first minimum = smallest iR (candidates ascend)
        if dist[j] >= 75:
            continue
        s = isc[lev]
        suL, svL, suR0 = _cround(f32(uL * s)), _cround(f32(vL * s)), _cround(f32(f32(kr["x"][c[j]]) * s))
        if suR0 < 0 or suR0 + 11 >= pl[lev].shape[1]:
            continue
        y0, x0, r0 = int(svL) - 5, int(suL) - 5, int(suR0)
        IL = pl[lev][y0:y0 + 11, x0:x0 + 11].astype(np.int64)
        sads = [int(np.abs(IL - pr[lev][y0:y0 + 11, r0 + k - 5:r0 + k + 6].astype(np.int64)).sum())
                for k in range(-5, 6)]
        b = int(np.argmin(sads))
        if b in (0, 10):
            continue
        d1, d2, d3 = f32(sads[b - 1]), f32(sads[b]), f32(sads[b + 1])
        deltaR = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if deltaR < -1 or deltaR > 1:
            continue
        buR = f32(sc[lev] * f32(f32(suR0 + f32(b - 5)) + deltaR))
        disp = f32(uL - buR)
        if 0 <= disp < maxD:
            if disp <= 0:
                disp = f32(0.01)
                buR = f32(float(uL) - 0.01)
            dep[iL] = f32(f32(mbf) / disp)
            ur[iL] = buR
            kept.append((sads[b], iL))
    if kept and cut:
        kept.sort()
        th = f32(f32(1.5) * f32(1.4)) * f32(kept[len(kept) // 2][0])
        for sad, i in kept:
            if not f32(sad) < th:
                ur[i] = dep[i] = -1
    return ur, dep


def test_oracle_matches_python_restatement(pair):
    kl, dl, kr, dr, pl, pr, sc, isc = pair
    ur, dep = ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, MBF, MB)
    ur_p, dep_p = _py_stereo(kl, dl, kr, dr, pl, pr, sc, isc, MBF, MB)
    assert np.array_equal(ur, ur_p)
    assert np.array_equal(dep, dep_p)
    assert (ur >= 0).sum() > 300


def test_oracle_disparity_on_field(pair):
    kl, dl, kr, dr, pl, pr, sc, isc = pair
    ur, dep = ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, MBF, MB)
    m = ur >= 0
    disp = kl["x"][m] - ur[m]
    assert np.all(disp > 0)
    # depth = bf / disparity exactly as the reference computes it
    assert np.array_equal(dep[m], (np.float32(MBF) / disp.astype(np.float32)).astype(np.float32))
    assert 4.0 < np.median(disp) < 40.0


def test_oracle_no_right_keypoints(pair):
    kl, dl, kr, dr, pl, pr, sc, isc = pair
    ur, dep = ob.stereo_matches(kl, dl, kr[:0], dr[:0], pl, pr, sc, isc, MBF, MB)
    assert np.all(ur == -1) and np.all(dep == -1)


def test_oracle_median_cut(pair):
    """The cut (Frame.cc:950-963) removes exactly the kept matches whose SAD is at least
    1.5f*1.4f times the median SAD, and on this pair it removes some."""
    kl, dl, kr, dr, pl, pr, sc, isc = pair
    ur, _ = ob.stereo_matches(kl, dl, kr, dr, pl, pr, sc, isc, MBF, MB)
    ur_nc, _ = _py_stereo(kl, dl, kr, dr, pl, pr, sc, isc, MBF, MB, cut=False)
    removed = (ur_nc >= 0) & (ur < 0)
    assert removed.sum() > 0
    assert np.all(ur[ur >= 0] == ur_nc[ur >= 0])
    assert not np.any((ur >= 0) & (ur_nc < 0))
