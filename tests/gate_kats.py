"""Known-answer inputs that sit exactly on the gates whose arithmetic the compiled reference
contracts (oracle/fp_sites.hpp): for every case the reference binary's arithmetic
(fma chains, double cv::norm) and the plain float source arithmetic decide the gate differently,
so a kernel or an oracle that drops a contraction flips the answer.

Each builder returns (cases, inputs) where a case records the decision the compiled reference
takes ("fma") and the one unfused float arithmetic would take ("naive"); they always differ.
Shared by tests/test_gate_kats.py (oracle, CPU) and tests/test_gpu_gate_kats.py (kernels).
"""
from __future__ import annotations

import math

import numpy as np

import scenes
import slamhot
from fpexact import chain3, fmaf, norm_d

f32 = np.float32
CAM = (f32(435.2047), f32(435.2047), f32(367.4517), f32(252.2009))
BF = f32(47.9064)
LOG_SCALE = f32(np.log(np.float64(f32(1.2))))


def naive_chain(a, b):
    return f32(f32(f32(f32(0) + f32(a[0] * b[0])) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def naive_norm(v):
    return f32(np.sqrt(naive_chain(v, v)))


def ulps(x, k):
    """x moved k float32 ulps."""
    x = f32(x)
    for _ in range(abs(k)):
        x = np.nextafter(x, f32(np.inf) if k > 0 else f32(-np.inf), dtype=np.float32)
    return x


def level_of(max_d, dist, nlevels=8):
    r = f32(max_d / dist)
    lv = int(math.ceil(float(f32(f32(math.log(float(r))) / LOG_SCALE))))
    return min(max(lv, 0), nlevels - 1)


def _solve_scaled(target, factor, lo=-64, hi=64):
    """A float m with f32(factor * m) == target, searched around target / factor."""
    m0 = f32(target / factor)
    for k in range(lo, hi + 1):
        m = ulps(m0, k)
        if f32(f32(factor) * m) == target:
            return m
    return None


# ------------------------------------------------------------------ Frame::isInFrustum
def frustum_cases(seed=0, want=24):
    """MapPoints for one frame (scenes.scene(seed) pose): each on the minDistance, maxDistance,
    PredictScale or viewCos gate.  Returns (frame S, geom array, limits per MapPoint, cases)."""
    S = scenes.scene(seed, n_feat=50)
    T = S["Tcw"].astype(np.float32)
    R, t = T[:3, :3], T[:3, 3]
    Ow = (-(T[:3, :3].astype(np.float64).T @ T[:3, 3].astype(np.float64))).astype(np.float32)
    rng = np.random.default_rng(1000 + seed)
    geoms, limits, cases = [], [], []
    counts = dict(min=0, max=0, level=0, cos=0)
    tries = 0
    while min(counts.values()) < want // 4 and tries < 200000:
        tries += 1
        u0, v0, z = rng.uniform(40, 700), rng.uniform(40, 440), rng.uniform(0.8, 25)
        Xc = np.array([(u0 - CAM[2]) * z / CAM[0], (v0 - CAM[3]) * z / CAM[1], z])
        X = (R.astype(np.float64).T @ (Xc - t)).astype(np.float32)
        Pc_a = [f32(chain3(R[r], X) + t[r]) for r in range(3)]
        u = f32(f32(CAM[0] * Pc_a[0]) / Pc_a[2]) + CAM[2]
        v = f32(f32(CAM[1] * Pc_a[1]) / Pc_a[2]) + CAM[3]
        if not (0 <= u <= 752 and 0 <= v <= 480) or Pc_a[2] <= 0:
            continue
        PO = (X - Ow).astype(np.float32)
        da, dn = norm_d(PO), naive_norm(PO)
        nrm = (PO / np.linalg.norm(PO.astype(np.float64))).astype(np.float32)
        g = np.zeros(1, slamhot.MP_GEOM_DTYPE)[0]
        g["pos"], g["normal"], g["has_obs"] = X, nrm, 1
        kind = min(counts, key=counts.get)
        if kind in ("min", "max", "level") and da == dn:
            continue
        if kind == "min":
            m = _solve_scaled(max(da, dn), f32(0.8))
            if m is None:
                continue
            g["min_dist"], g["max_dist"] = m, f32(da * 4)
            fma_ok, naive_ok = not (da < f32(0.8) * m), not (dn < f32(0.8) * m)
        elif kind == "max":
            m = _solve_scaled(min(da, dn), f32(1.2))
            if m is None:
                continue
            g["min_dist"], g["max_dist"] = f32(da / 4), m
            fma_ok, naive_ok = not (da > f32(1.2) * m), not (dn > f32(1.2) * m)
        elif kind == "level":
            base = f32(da * f32(1.2) ** int(rng.integers(1, 7)))
            m = next((ulps(base, k) for k in range(-200, 201) if level_of(ulps(base, k), da) !=
                      level_of(ulps(base, k), dn)), None)
            if m is None:
                continue
            g["min_dist"], g["max_dist"] = f32(da / 8), m
            fma_ok, naive_ok = level_of(m, da), level_of(m, dn)
        else:  # viewCos against a limit equal to the larger of the two restatements
            tilt = rng.normal(0, 0.3, 3).astype(np.float32)
            n2 = (nrm + tilt).astype(np.float32)
            n2 = (n2 / np.linalg.norm(n2.astype(np.float64))).astype(np.float32)
            ca, cn = f32(chain3(PO, n2) / da), f32(naive_chain(PO, n2) / dn)
            if ca == cn or min(ca, cn) <= 0.2:
                continue
            g["normal"] = n2
            g["min_dist"], g["max_dist"] = f32(da / 4), f32(da * 4)
            lim = max(ca, cn)
            fma_ok, naive_ok = not (ca < lim), not (cn < lim)
            limits.append(lim)
            geoms.append(g)
            cases.append(dict(kind=kind, fma=fma_ok, naive=naive_ok))
            counts[kind] += 1
            continue
        limits.append(f32(0.5))
        geoms.append(g)
        cases.append(dict(kind=kind, fma=fma_ok, naive=naive_ok))
        counts[kind] += 1
    assert all(c["fma"] != c["naive"] for c in cases)
    return S, np.array(geoms, slamhot.MP_GEOM_DTYPE), np.array(limits, np.float32), cases


# ------------------------------------------------------------------ SearchForTriangulation_
def _tri_kf(kp, Tcw, level_sigma2=1.0, scale=1.0, stereo=False):
    sc = np.full(8, scale, np.float32)
    s2 = np.full(8, level_sigma2, np.float32)
    k = np.zeros(1, slamhot.KP_DTYPE)
    k["x"], k["y"], k["octave"], k["angle"] = kp[0], kp[1], 0, 90.0
    return dict(kps_un=k, desc=np.full((1, 32), 0x5A, np.uint8), uright=np.full(1, 10.0 if stereo else -1, np.float32),
                has_mp=np.zeros(1, np.uint8), node_id=np.array([7], np.int32), node_off=np.array([0, 1], np.int32),
                node_feat=np.array([0], np.int32), scale=sc, level_sigma2=s2, Tcw=Tcw,
                cam=np.array(CAM, np.float32))


def tri_geometry(K1, K2):
    import ctypes as C

    import oracle_bind as ob
    t1, _ = slamhot.make_tri_kf(K1)
    t2, _ = slamhot.make_tri_kf(K2)
    ep, R12, t12, F12 = (C.c_float * 2)(), (C.c_float * 9)(), (C.c_float * 3)(), (C.c_float * 9)()
    ob.lib().oracle_fp_tri_geometry(t1.Rcw, t1.tcw, t1.Ow, t1.cam, t2.Rcw, t2.tcw, t2.cam, ep, R12, t12, F12)
    return np.array(ep[:], np.float32), np.array(F12[:], np.float32).reshape(3, 3)


def _dsqr(F, x1, y1, x2, y2, fused):
    if fused:
        a = f32(fmaf(x1, F[0, 0], f32(y1 * F[1, 0])) + F[2, 0])
        b = f32(fmaf(x1, F[0, 1], f32(y1 * F[1, 1])) + F[2, 1])
        c = f32(fmaf(y1, F[1, 2], f32(x1 * F[0, 2])) + F[2, 2])
        num = f32(fmaf(b, y2, f32(a * x2)) + c)
        den = fmaf(a, a, f32(b * b))
    else:
        a = f32(f32(f32(x1 * F[0, 0]) + f32(y1 * F[1, 0])) + F[2, 0])
        b = f32(f32(f32(x1 * F[0, 1]) + f32(y1 * F[1, 1])) + F[2, 1])
        c = f32(f32(f32(x1 * F[0, 2]) + f32(y1 * F[1, 2])) + F[2, 2])
        num = f32(f32(f32(a * x2) + f32(b * y2)) + c)
        den = f32(f32(a * a) + f32(b * b))
    return f32(f32(num * num) / den)


def triangulation_cases(seed=0, want=16):
    """KeyFrame pairs with one feature each: the epipolar dsqr < 3.84 sigma^2 gate (level_sigma2
    of KF2 chosen between the two restatements' dsqr) and the distance-to-epipole gate (scale of
    KF2 chosen between the two restatements' squared distance; coarse pairs skip the epipolar
    test).  Returns (kfs, pairs [(kf1, kf2, only_stereo, coarse)], cases)."""
    rng = np.random.default_rng(2000 + seed)
    kfs, pairs, cases = [], [], []
    n_epi = n_ep = 0
    while (n_epi < want // 2 or n_ep < want // 2) and len(kfs) < 4 * want + 400:
        T1 = scenes.pose(scenes.rot(*rng.normal(0, 0.05, 3)), rng.normal(0, 0.2, 3)).astype(np.float32)
        T2 = scenes.pose(scenes.rot(*rng.normal(0, 0.05, 3)), np.array([0.3, 0, 0]) + rng.normal(0, 0.05, 3))
        T2 = T2.astype(np.float32)
        x1, y1 = f32(rng.uniform(50, 700)), f32(rng.uniform(50, 430))
        K1 = _tri_kf((x1, y1), T1)
        ep, F = tri_geometry(K1, _tri_kf((0, 0), T2))
        if n_epi <= n_ep:
            # a point near the epipolar line, away from the epipole
            a = float(x1 * F[0, 0] + y1 * F[1, 0] + F[2, 0])
            b = float(x1 * F[0, 1] + y1 * F[1, 1] + F[2, 1])
            c = float(x1 * F[0, 2] + y1 * F[1, 2] + F[2, 2])
            x2 = f32(rng.uniform(50, 700))
            if abs(b) < 1e-9:
                continue
            y2 = f32(-(a * float(x2) + c) / b + rng.normal(0, 2.0))
            if np.hypot(float(ep[0] - x2), float(ep[1] - y2)) < 40:
                continue
            da, dn = _dsqr(F, x1, y1, x2, y2, True), _dsqr(F, x1, y1, x2, y2, False)
            if da == dn or not np.isfinite(da) or not np.isfinite(dn):
                continue
            hi = max(da, dn)
            unc = f32(float(hi) / 3.84)
            # compare in double, as the reference does (NumPy 2 would compare float32 to a
            # Python float in float32)
            unc = next((ulps(unc, k) for k in range(-8, 9)
                        if float(min(da, dn)) < 3.84 * float(ulps(unc, k)) <= float(hi)), None)
            if unc is None:
                continue
            K2 = _tri_kf((x2, y2), T2, level_sigma2=unc)
            fma_ok, naive_ok = float(da) < 3.84 * float(unc), float(dn) < 3.84 * float(unc)
            kind, coarse = "epipolar", False
            n_epi += 1
        else:
            ang = rng.uniform(0, 2 * np.pi)
            rad = rng.uniform(8, 12)
            x2, y2 = f32(ep[0] + rad * np.cos(ang)), f32(ep[1] + rad * np.sin(ang))
            dx, dy = f32(ep[0] - x2), f32(ep[1] - y2)
            qa, qn = fmaf(dx, dx, f32(dy * dy)), f32(f32(dx * dx) + f32(dy * dy))
            if qa == qn:
                continue
            sc = _solve_scaled(max(qa, qn), f32(100.0))
            if sc is None:
                continue
            K2 = _tri_kf((x2, y2), T2, scale=sc)
            fma_ok, naive_ok = not (qa < f32(100) * sc), not (qn < f32(100) * sc)
            kind, coarse = "epipole", True
            n_ep += 1
        kfs += [K1, K2]
        pairs.append((len(kfs) - 2, len(kfs) - 1, False, coarse))
        cases.append(dict(kind=kind, fma=fma_ok, naive=naive_ok))
    assert all(c["fma"] != c["naive"] for c in cases)
    return kfs, pairs, cases


# ------------------------------------------------------------------ stereo reprojection gates
def _one_feature_frame(kx, ky, ur, scale=None):
    k = np.zeros(1, slamhot.KP_DTYPE)
    k["x"], k["y"], k["octave"], k["angle"] = kx, ky, 0, 45.0
    d = np.full((1, 32), 0x33, np.uint8)
    return k, d, np.array([ur], np.float32)


def sbp_last_cases(seed=0, want=12):
    """SearchByProjection(F, LastF): one last-frame MapPoint, one stereo feature; th chosen so
    radius sits between the two restatements' er = |uv.x - mbf*invz - uright|.
    Returns a list of (frame dict, last dict, th, case)."""
    rng = np.random.default_rng(3000 + seed)
    out = []
    T = np.eye(4, dtype=np.float32)
    while len(out) < want:
        u0, v0, z = rng.uniform(60, 690), rng.uniform(60, 420), rng.uniform(1.0, 20.0)
        X = np.array([(u0 - CAM[2]) * z / CAM[0], (v0 - CAM[3]) * z / CAM[1], z], np.float32)
        xc = X.astype(np.float64)  # identity pose: the cv::Mat product is exact
        invz = f32(1.0 / float(f32(xc[2])))
        u = f32(f32(CAM[0] * X[0]) / X[2]) + CAM[2]
        v = f32(f32(CAM[1] * X[1]) / X[2]) + CAM[3]
        ur_true = f32(u - f32(BF / X[2]))
        kpr = f32(ur_true + rng.uniform(-3, 3))
        if not (2 <= u <= 750 and 2 <= v <= 478) or kpr <= 0:
            continue
        ea = abs(f32(fmaf(-BF, invz, u) - kpr))
        en = abs(f32(f32(u - f32(BF * invz)) - kpr))
        if ea == en or max(ea, en) < 0.5:
            continue
        th = _solve_scaled(min(ea, en), f32(1.0))
        if th is None:
            continue
        fma_ok, naive_ok = not (ea > th), not (en > th)
        out.append(dict(u=u, v=v, X=X, kpr=kpr, th=th, T=T, case=dict(kind="sbp_er", fma=fma_ok, naive=naive_ok)))
    assert all(c["case"]["fma"] != c["case"]["naive"] for c in out)
    return out


def fuse_cases(seed=0, want=12):
    """Fuse: one MapPoint, one stereo KeyFrame feature; mvInvLevelSigma2[0] chosen so the chi2
    e2 * invSigma2 > 7.8 gate falls between the two restatements' e2.
    Returns a list of dicts (X, kp, kpr, inv_sigma2, case)."""
    rng = np.random.default_rng(4000 + seed)
    out = []
    while len(out) < want:
        u0, v0, z = rng.uniform(60, 690), rng.uniform(60, 420), rng.uniform(1.0, 20.0)
        X = np.array([(u0 - CAM[2]) * z / CAM[0], (v0 - CAM[3]) * z / CAM[1], z], np.float32)
        invz = f32(f32(1) / X[2])
        u = f32(f32(CAM[0] * X[0]) / X[2]) + CAM[2]
        v = f32(f32(CAM[1] * X[1]) / X[2]) + CAM[3]
        kx, ky = f32(u + rng.normal(0, 1.0)), f32(v + rng.normal(0, 1.0))
        if abs(float(kx - u)) > 2.5 or abs(float(ky - v)) > 2.5:
            continue
        kpr = f32(f32(u - f32(BF * invz)) + rng.normal(0, 1.5))
        ex, ey = f32(u - kx), f32(v - ky)
        ea = fmaf(f32(fmaf(-BF, invz, u) - kpr), f32(fmaf(-BF, invz, u) - kpr), fmaf(ex, ex, f32(ey * ey)))
        ern = f32(f32(u - f32(BF * invz)) - kpr)
        en = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(ern * ern))
        if ea == en or min(ea, en) < 0.05:
            continue
        # isg with (double)f32(lo*isg) <= 7.8 < (double)f32(hi*isg)
        lo, hi = min(ea, en), max(ea, en)
        isg0 = f32(7.8 / float(hi))
        isg = next((ulps(isg0, k) for k in range(-16, 17) if float(f32(lo * ulps(isg0, k))) <= 7.8 <
                    float(f32(hi * ulps(isg0, k)))), None)
        if isg is None:
            continue
        fma_ok, naive_ok = not (float(f32(ea * isg)) > 7.8), not (float(f32(en * isg)) > 7.8)
        out.append(dict(X=X, kx=kx, ky=ky, kpr=kpr, isg=isg, case=dict(kind="fuse_e2", fma=fma_ok, naive=naive_ok)))
    assert all(c["case"]["fma"] != c["case"]["naive"] for c in out)
    return out


def one_mp_geom(X, max_d=None):
    g = np.zeros(1, slamhot.MP_GEOM_DTYPE)
    g["pos"] = X
    d = float(np.linalg.norm(X.astype(np.float64)))
    g["normal"] = (X / d).astype(np.float32)
    g["max_dist"] = f32(d) if max_d is None else max_d
    g["min_dist"] = f32(d / 10)
    g["has_obs"] = 1
    return g
