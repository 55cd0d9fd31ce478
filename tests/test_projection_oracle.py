"""CPU: the projection-matcher oracle vs a plain-Python restatement (independent code) on
small seeded scenes; grid semantics known answers."""
import math

import numpy as np
import pytest

import oracle_bind as ob
from fpexact import chain3, norm_d
import scenes

f32 = np.float32


def py_grid(k, inv_w, inv_h):
    cells = {}
    for i in range(len(k)):
        px = int(math.floor(abs(float(f32(k["x"][i]) * inv_w)) + 0.5)) * (1 if k["x"][i] >= 0 else -1)
        py = int(math.floor(abs(float(f32(k["y"][i]) * inv_h)) + 0.5)) * (1 if k["y"][i] >= 0 else -1)
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((px, py), []).append(i)
    return cells


def py_area(k, cells, inv_w, inv_h, x, y, r, minL, maxL):
    x, y, r = f32(x), f32(y), f32(r)
    x0 = max(0, math.floor(f32(f32(x - r) * inv_w)))
    if x0 >= 64:
        return []
    x1 = min(63, math.ceil(f32(f32(x + r) * inv_w)))
    if x1 < 0:
        return []
    y0 = max(0, math.floor(f32(f32(y - r) * inv_h)))
    if y0 >= 48:
        return []
    y1 = min(47, math.ceil(f32(f32(y + r) * inv_h)))
    if y1 < 0:
        return []
    out = []
    chk = minL > 0 or maxL >= 0
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in cells.get((ix, iy), []):
                o = k["octave"][i]
                if chk and (o < minL or (maxL >= 0 and o > maxL)):
                    continue
                if abs(f32(k["x"][i] - x)) < r and abs(f32(k["y"][i] - y)) < r:
                    out.append(i)
    return out


def ham(a, b):
    return int(np.unpackbits(a ^ b).sum())


def py_local(S, mps, desc, nnratio, th):
    k, d, ur = S["k"], S["d"], S["uright"]
    inv_w, inv_h = f32(64) / f32(752), f32(48) / f32(480)
    scale = [f32(1.0)]
    for _ in range(7):
        scale.append(f32(np.float64(scale[-1]) * np.float64(f32(1.2))))
    cells = py_grid(k, inv_w, inv_h)
    state = S["state"].astype(int).copy()
    fm = np.full(len(k), -1)
    nm = 0
    for q, mp in enumerate(mps):
        if not mp["in_view"] or mp["is_bad"]:
            continue
        lvl = int(mp["scale_level"])
        r = f32(2.5) if float(mp["view_cos"]) > 0.998 else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        R = f32(r * scale[lvl])
        best, bl, best2, bl2, bi = 256, -1, 256, -1, -1
        for i in py_area(k, cells, inv_w, inv_h, mp["proj_x"], mp["proj_y"], R, lvl - 1, lvl):
            if state[i] == 1:
                continue
            if ur[i] > 0 and abs(f32(mp["proj_xr"] - ur[i])) > R:
                continue
            dist = ham(desc[q], d[i])
            if dist < best:
                best2, best, bl2, bl, bi = best, dist, bl, int(k["octave"][i]), i
            elif dist < best2:
                bl2, best2 = int(k["octave"][i]), dist
        if best <= 100:
            lim = f32(f32(nnratio) * f32(best2))
            if bl == bl2 and f32(best) > lim:
                continue
            fm[bi] = q
            state[bi] = 1 if mp["has_obs"] else 0
            nm += 1
    return nm, fm


@pytest.mark.parametrize("seed", [10, 11])
def test_local_oracle_vs_python(seed):
    S = scenes.scene(seed, n_feat=300)
    fv, keep = scenes.frame_view(S, with_pose=False)
    mps, desc = scenes.local_map(S, n_extra=100)
    for th, ratio in [(1.0, 0.8), (3.0, 0.6)]:
        no, fo = ob.search_by_projection_local(fv, mps, desc, ratio, th, False, 50.0)
        pn, pf = py_local(S, mps, desc, ratio, th)
        assert no == pn
        assert np.array_equal(fo, pf)


def test_grid_area_known_answers():
    S = scenes.scene(12, n_feat=300)
    k = S["k"]
    inv_w, inv_h = f32(64) / f32(752), f32(48) / f32(480)
    cells = py_grid(k, inv_w, inv_h)
    # every keypoint is found by a tiny window around itself, at its own level
    for i in range(0, len(k), 17):
        idx = py_area(k, cells, inv_w, inv_h, k["x"][i], k["y"][i], 0.5, int(k["octave"][i]), int(k["octave"][i]))
        assert i in idx
    assert py_area(k, cells, inv_w, inv_h, -500.0, 10.0, 3.0, -1, -1) == []


def test_predict_scale_logf_equivalence():
    """MapPoint::PredictScale with glibc logf (the reference) and with the correctly rounded
    logf the device evaluates give the same level for every float ratio in [1e-3, 1e3]."""
    lsf = float(np.float32(np.log(np.float64(np.float32(1.2)))))
    assert ob.check_predict_scale(1e-3, 1e3, lsf) == 0


def _py_in_frustum(fv, T, g, limit=0.5):
    """Frame::isInFrustum restated with numpy float32 scalars (Frame.cc:493-556) and the compiled
    reference's contractions (fpexact: fma chains, cv::norm in double)."""
    f32 = np.float32
    if g["seen"] or g["is_bad"]:
        return None
    R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
    Tr = T.astype(np.float64)
    Ow = (-(Tr[:3, :3].T @ Tr[:3, 3])).astype(np.float32)
    X = g["pos"].astype(np.float32)
    Pc = [f32(chain3(R[r], X) + t[r]) for r in range(3)]
    if Pc[2] < 0:
        return None
    u = f32(f32(f32(fv.fx) * Pc[0]) / Pc[2]) + f32(fv.cx)
    v = f32(f32(f32(fv.fy) * Pc[1]) / Pc[2]) + f32(fv.cy)
    if u < fv.min_x or u > fv.max_x or v < fv.min_y or v > fv.max_y:
        return None
    PO = (X - Ow).astype(np.float32)
    dist = norm_d(PO)
    if dist < f32(0.8) * g["min_dist"] or dist > f32(1.2) * g["max_dist"]:
        return None
    n = g["normal"]
    vc = f32(chain3(PO, n) / dist)
    if vc < limit:
        return None
    ratio = f32(g["max_dist"] / dist)
    lvl = int(np.ceil(f32(f32(np.log(np.float64(ratio))) / f32(fv.log_scale))))
    return u, v, min(max(lvl, 0), fv.nlevels - 1), vc


def test_is_in_frustum_oracle_vs_python():
    S = scenes.scene(11)
    fv, keep = scenes.frame_view(S)
    geom, desc = scenes.local_map_geom(S)
    n, tr = ob.is_in_frustum(fv, geom, 0.5)
    cnt = 0
    for i, g in enumerate(geom):
        r = _py_in_frustum(fv, S["Tcw"], g)
        assert bool(tr["in_view"][i]) == (r is not None), i
        if r is not None:
            cnt += 1
            assert tr["proj_x"][i] == r[0] and tr["proj_y"][i] == r[1]
            assert tr["scale_level"][i] == r[2] and tr["view_cos"][i] == r[3]
    assert cnt == n and n > 300
    # the boundary MapPoints (ratio = 1.2^level) land on both sides of the level edges
    assert len(np.unique(tr["scale_level"][tr["in_view"] == 1])) == 8
