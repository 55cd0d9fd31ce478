"""Seeded synthetic inputs of the shapes BASELINE.json names (no datasets in this image).

Frames: procedural u8 textures (random rectangles + Gaussian blobs + value noise, clipped to
[0, 255]) as SURVEY.md §8(d) config 2 specifies.  Everything is derived from
``numpy.random.default_rng(seed)`` so a seed fully determines a frame.
"""
from __future__ import annotations

import numpy as np


def _value_noise(rng: np.random.Generator, h: int, w: int, cell: int) -> np.ndarray:
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float64)
    ys = np.arange(h) / cell
    xs = np.arange(w) / cell
    y0 = ys.astype(np.int64)
    x0 = xs.astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)
    fx = fx * fx * (3 - 2 * fx)
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    return (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy


def frame(seed: int, width: int = 640, height: int = 480) -> np.ndarray:
    """One textured grayscale frame (height, width) uint8."""
    rng = np.random.default_rng(seed)
    img = 90.0 + 60.0 * _value_noise(rng, height, width, 48)
    img += 25.0 * _value_noise(rng, height, width, 9)
    for _ in range(60):
        x0, y0 = rng.integers(0, width), rng.integers(0, height)
        rw, rh = rng.integers(8, 120), rng.integers(8, 120)
        img[y0:y0 + rh, x0:x0 + rw] += rng.uniform(-70, 70)
    for _ in range(25):
        cx, cy = rng.uniform(0, width), rng.uniform(0, height)
        s = rng.uniform(3, 25)
        amp = rng.uniform(-80, 80)
        r = int(np.ceil(4 * s))
        x0, x1 = max(0, int(cx) - r), min(width, int(cx) + r + 1)
        y0, y1 = max(0, int(cy) - r), min(height, int(cy) + r + 1)
        if x0 >= x1 or y0 >= y1:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        img[y0:y1, x0:x1] += amp * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
    img += rng.normal(0.0, 4.0, size=img.shape)
    # C order: the broadcasting above leaves a Fortran-ordered array, and device uploads
    # (torch.from_numpy(...).to(dev)) keep strides, so raw data_ptr() users need row-major
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))


def frames(seeds, width: int = 640, height: int = 480) -> np.ndarray:
    """Stack of frames (n, height, width) uint8."""
    return np.ascontiguousarray(np.stack([frame(int(s), width, height) for s in seeds]))


def shifted(img: np.ndarray, dx: float, dy: float, angle_deg: float, seed: int) -> np.ndarray:
    """Rigidly warped copy (nearest neighbour) plus light noise: a 'next frame' for matching."""
    h, w = img.shape
    rng = np.random.default_rng(seed)
    a = np.deg2rad(angle_deg)
    ca, sa = np.cos(a), np.sin(a)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    cx, cy = w / 2, h / 2
    xs = ca * (xx - cx - dx) + sa * (yy - cy - dy) + cx
    ys = -sa * (xx - cx - dx) + ca * (yy - cy - dy) + cy
    xi = np.clip(np.rint(xs), 0, w - 1).astype(np.int64)
    yi = np.clip(np.rint(ys), 0, h - 1).astype(np.int64)
    out = img[yi, xi].astype(np.float64) + rng.normal(0.0, 2.0, size=img.shape)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def vocab(k: int = 10, L: int = 6, seed: int = 0, stop_frac: float = 0.01):
    """Synthetic DBoW2-shaped vocabulary in breadth-first node order (node 0 = root):
    returns (parent int32, is_leaf uint8, desc (n,32) uint8, weight float64).  Node
    descriptors are random; a child is its parent with ~25% of bits flipped, so nearby
    descriptors descend alike.  A fraction of words get weight 0 (stopped words)."""
    rng = np.random.default_rng(seed)
    n = (k ** (L + 1) - 1) // (k - 1)
    parent = np.empty(n, np.int32)
    parent[0] = -1
    idx = np.arange(1, n)
    parent[1:] = (idx - 1) // k
    desc = np.empty((n, 32), np.uint8)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    first = 1
    for lvl in range(1, L + 1):
        cnt = k ** lvl
        par = desc[parent[first:first + cnt]]
        flips = rng.random((cnt, 256)) < 0.25
        bits = np.unpackbits(par, axis=1, bitorder="little") ^ flips.astype(np.uint8)
        desc[first:first + cnt] = np.packbits(bits, axis=1, bitorder="little")
        first += cnt
    is_leaf = np.zeros(n, np.uint8)
    nleaf = k ** L
    is_leaf[n - nleaf:] = 1
    weight = np.zeros(n, np.float64)
    w = rng.uniform(0.5, 3.0, nleaf)
    w[rng.random(nleaf) < stop_frac] = 0.0
    weight[n - nleaf:] = w
    return parent, is_leaf, desc, weight


def feature_vector(node_id: np.ndarray, weight: np.ndarray):
    """DBoW2 FeatureVector as CSR from per-feature (node id, word weight): features whose
    word weight is <= 0 are dropped (TemplatedVocabulary.h:1169), ascending node ids,
    ascending feature indices (FeatureVector::addFeature, FeatureVector.cpp:31-45)."""
    keep = np.nonzero(weight > 0)[0]
    nid = node_id[keep]
    order = np.lexsort((keep, nid))
    nid_s = nid[order]
    feats = keep[order].astype(np.uint32)
    uniq, starts = np.unique(nid_s, return_index=True)
    off = np.append(starts, len(nid_s)).astype(np.int32)
    return uniq.astype(np.uint32), off, feats


# ------------------------------------------------------------------------------------------
# Synthetic local-BA windows
# ------------------------------------------------------------------------------------------
EUROC_CAM = dict(fx=435.2047, fy=435.2047, cx=367.4517, cy=252.2009, bf=47.9064, w=752, h=480)


def _axis_angle(axis, ang):
    axis = axis / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _level_tables(nfeatures=1000, scale_factor=1.2, nlevels=8):
    """Float scale / inverse-sigma^2 tables and per-level feature split as ORBextractor builds
    them (ORBextractor.cc:413-444)."""
    sf = np.float64(np.float32(scale_factor))
    scale = [np.float32(1.0)]
    for _ in range(1, nlevels):
        scale.append(np.float32(np.float64(scale[-1]) * sf))
    scale = np.array(scale, np.float32)
    inv_sigma2 = (np.float32(1.0) / (scale * scale)).astype(np.float32)
    factor = 1.0 / sf
    per = nfeatures * (1 - factor) / (1 - factor ** nlevels)
    nf = []
    for _ in range(nlevels - 1):
        nf.append(round(per))
        per *= factor
    nf.append(max(nfeatures - sum(nf), 0))
    return scale, inv_sigma2, np.array(nf, np.float64)


def lba_window(seed: int, n_kf: int = 50, n_pt: int = 2000, obs_per_pt: int = 8,
               stereo_frac: float = 0.0, outlier_frac: float = 0.02, arc_deg: float = 80.0,
               radius: float = 3.0, noise: float = 1.0, body_frac: float = 0.0, mixed_cams: bool = False):
    """A seeded local-BA window in the layout of slam_lba_problem.

    50 KeyFrames on a ``radius`` arc facing a 4 x 2 x 4 m box of points; every point is seen
    by exactly ``obs_per_pt`` KeyFrames drawn among those where it projects in-image with
    z > 0.3 m; octave drawn with the extractor's per-level feature split; pixel noise
    N(0, 1.2^l); ``outlier_frac`` observations replaced by uniform in-image points;
    KF poses perturbed by 0.5 deg / 2 cm and points by 3 cm.  KF 0 is the map-init KF
    (fixed, written back) and KF 1 is the fallback fixed camera (kf_fixed = 2), so 48 KFs
    are free.  Edges are point-major, KFs in id order.
    ``body_frac`` > 0 gives every KeyFrame a second (pinhole) camera: that fraction of the left
    observations is followed by a right-camera observation, an EdgeSE3ProjectXYZToBody
    (Optimizer.cc:1883-1914), with the rig's mTrl and the second camera's intrinsics.
    ``mixed_cams``: odd KeyFrames carry a second calibration (an Atlas map merged from two
    cameras): the window then has ``kf_cam`` (and ``kf_cam2``), one camera per KeyFrame, as the
    reference binds every edge to its own KeyFrame's camera (Optimizer.cc:1840, 1869-1873, 1906).
    ``mixed_cams="all"``: every KeyFrame uses the second calibration (window-level ``cam``)."""
    rng = np.random.default_rng(seed)
    cam = EUROC_CAM
    cam_b = dict(fx=458.654, fy=457.296, cx=367.215 - 7.5, cy=248.375 + 3.25, bf=52.103, w=752, h=480)
    alt_all = mixed_cams == "all"
    kcam = [cam_b if (alt_all or (mixed_cams and k % 2)) else cam for k in range(n_kf)]
    kfx = np.array([c["fx"] for c in kcam], np.float64)
    kfy = np.array([c["fy"] for c in kcam], np.float64)
    kcx = np.array([c["cx"] for c in kcam], np.float64)
    kcy = np.array([c["cy"] for c in kcam], np.float64)
    scale, inv_sigma2, nf = _level_tables()
    p_level = nf / nf.sum()
    # ground-truth poses Tcw
    Rs, ts = [], []
    for k in range(n_kf):
        a = np.deg2rad(-arc_deg / 2 + arc_deg * k / max(n_kf - 1, 1))
        C = np.array([radius * np.sin(a), 0.3 * np.sin(3 * a), -radius * np.cos(a)])
        z = -C / np.linalg.norm(C)
        x = np.cross(np.array([0.0, -1.0, 0.0]), z)
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R = np.stack([x, y, z])  # rows: camera axes in world
        Rs.append(R)
        ts.append(-R @ C)
    Rs, ts = np.array(Rs), np.array(ts)
    # points: resample until each has enough observing KFs
    pts = np.zeros((n_pt, 3))
    obs_kf = []
    i = 0
    while i < n_pt:
        X = rng.uniform([-2, -1, -2], [2, 1, 2])
        Xc = np.einsum("kij,j->ki", Rs, X) + ts
        z = Xc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = kfx * Xc[:, 0] / z + kcx
            v = kfy * Xc[:, 1] / z + kcy
        ok = (z > 0.3) & (u >= 0) & (u < cam["w"]) & (v >= 0) & (v < cam["h"])
        cand = np.flatnonzero(ok)
        if len(cand) < obs_per_pt:
            continue
        pts[i] = X
        obs_kf.append(np.sort(rng.choice(cand, obs_per_pt, replace=False)))
        i += 1
    edge_pt, edge_kf, obs, isig, body = [], [], [], [], []
    cam2 = dict(fx=431.9, fy=432.4, cx=371.3, cy=249.8)
    cam2_b = dict(fx=455.1, fy=454.7, cx=362.9, cy=251.4)
    kcam2 = [cam2_b if (alt_all or (mixed_cams and k % 2)) else cam2 for k in range(n_kf)]
    R_rl = _axis_angle(np.array([0.2, 1.0, 0.1]), np.deg2rad(0.6))
    t_rl = np.array([-0.110, 0.0012, 0.0021])
    for p in range(n_pt):
        for k in obs_kf[p]:
            Xc = Rs[k] @ pts[p] + ts[k]
            ck = kcam[k]
            lvl = rng.choice(len(p_level), p=p_level)
            s = float(scale[lvl])
            u = ck["fx"] * Xc[0] / Xc[2] + ck["cx"] + noise * rng.normal(0, s)
            v = ck["fy"] * Xc[1] / Xc[2] + ck["cy"] + noise * rng.normal(0, s)
            ur = -1.0
            stereo = rng.random() < stereo_frac
            if stereo:
                ur = u - ck["bf"] / Xc[2] + noise * rng.normal(0, s)
            if rng.random() < outlier_frac:
                u = rng.uniform(0, cam["w"])
                v = rng.uniform(0, cam["h"])
                if stereo:
                    ur = u - rng.uniform(0, 40)
            if stereo and ur < 0:
                ur = 0.0
            edge_pt.append(p)
            edge_kf.append(k)
            obs.append((u, v, ur))
            isig.append(inv_sigma2[lvl])
            body.append(0)
            if body_frac > 0 and rng.random() < body_frac:
                Xr = R_rl @ Xc + t_rl
                if Xr[2] > 0.3:
                    lv2 = rng.choice(len(p_level), p=p_level)
                    s2 = float(scale[lv2])
                    c2 = kcam2[k]
                    u2 = c2["fx"] * Xr[0] / Xr[2] + c2["cx"] + noise * rng.normal(0, s2)
                    v2 = c2["fy"] * Xr[1] / Xr[2] + c2["cy"] + noise * rng.normal(0, s2)
                    if rng.random() < outlier_frac:
                        u2, v2 = rng.uniform(0, cam["w"]), rng.uniform(0, cam["h"])
                    edge_pt.append(p)
                    edge_kf.append(k)
                    obs.append((u2, v2, -1.0))
                    isig.append(inv_sigma2[lv2])
                    body.append(1)
    # perturbed initial estimates
    T0 = np.zeros((n_kf, 16), np.float32)
    for k in range(n_kf):
        R, t = Rs[k], ts[k]
        if k >= 2:
            R = _axis_angle(rng.normal(size=3), np.deg2rad(0.5)) @ R
            d = rng.normal(size=3)
            t = t + 0.02 * d / np.linalg.norm(d)
        M = np.eye(4)
        M[:3, :3] = R
        M[:3, 3] = t
        T0[k] = M.reshape(-1).astype(np.float32)
    d = rng.normal(size=(n_pt, 3))
    P0 = (pts + 0.03 * d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[0] = 1
    if n_kf > 2:
        fixed[1] = 2
    gt_T = np.zeros((n_kf, 4, 4))
    gt_T[:, :3, :3] = Rs
    gt_T[:, :3, 3] = ts
    gt_T[:, 3, 3] = 1
    extra = {}
    if body_frac > 0:
        Trl = np.eye(4)
        Trl[:3, :3] = R_rl
        Trl[:3, 3] = t_rl
        extra = dict(edge_body=np.array(body, np.uint8),
                     kf_Trl=np.tile(Trl.reshape(1, 16), (n_kf, 1)).astype(np.float32),
                     cam2=tuple(np.float32(cam2[k]) for k in ("fx", "fy", "cx", "cy")) + (np.float32(0),))
    if alt_all:
        cam = cam_b
        if body_frac > 0:
            extra["cam2"] = tuple(np.float32(cam2_b[k]) for k in ("fx", "fy", "cx", "cy")) + (np.float32(0),)
    elif mixed_cams:
        extra["kf_cam"] = np.array([[c[k] for k in ("fx", "fy", "cx", "cy", "bf")] for c in kcam], np.float32)
        if body_frac > 0:
            extra["kf_cam2"] = np.array([[c[k] for k in ("fx", "fy", "cx", "cy")] + [0.0] for c in kcam2], np.float32)
    return dict(
        **extra,
        kf_Tcw=T0, kf_fixed=fixed, pt_pos=P0,
        edge_pt=np.array(edge_pt, np.int32), edge_kf=np.array(edge_kf, np.int32),
        edge_obs=np.array(obs, np.float32), edge_inv_sigma2=np.array(isig, np.float32),
        cam=(np.float32(cam["fx"]), np.float32(cam["fy"]), np.float32(cam["cx"]),
             np.float32(cam["cy"]), np.float32(cam["bf"])),
        gt_T=gt_T, gt_pts=pts)


def pose_frame(seed: int, n: int = 1000, mp_frac: float = 0.8, stereo_frac: float = 0.0,
               outlier_frac: float = 0.1, rot_deg: float = 1.0, trans_m: float = 0.05):
    """A seeded Frame for Optimizer::PoseOptimization: `n` undistorted keypoints on EuRoC
    intrinsics, a fraction with MapPoints (world points 1.5-8 m in front of the true camera),
    octave from the extractor's level split, noise N(0, 1.2^l) px, `outlier_frac` of the
    matched observations replaced by uniform in-image points, initial pose perturbed by
    rot_deg / trans_m (as after motion-model prediction)."""
    rng = np.random.default_rng(seed)
    cam = EUROC_CAM
    scale, inv_sigma2, nf = _level_tables()
    p_level = nf / nf.sum()
    Rt = _axis_angle(rng.normal(size=3), np.deg2rad(rng.uniform(0, 30)))
    tt = rng.normal(0, 1, 3)
    kps = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                             ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    ur = np.full(n, -1.0, np.float32)
    has = (rng.random(n) < mp_frac).astype(np.uint8)
    pos = np.zeros((n, 3), np.float32)
    for i in range(n):
        u, v = rng.uniform(5, cam["w"] - 5), rng.uniform(5, cam["h"] - 5)
        z = rng.uniform(1.5, 8.0)
        lvl = rng.choice(len(p_level), p=p_level)
        Xc = np.array([(u - cam["cx"]) * z / cam["fx"], (v - cam["cy"]) * z / cam["fy"], z])
        Xw = Rt.T @ (Xc - tt)
        s = float(scale[lvl])
        uo, vo = u + rng.normal(0, s), v + rng.normal(0, s)
        st = rng.random() < stereo_frac
        if rng.random() < outlier_frac:
            uo, vo = rng.uniform(0, cam["w"]), rng.uniform(0, cam["h"])
        kps["x"][i], kps["y"][i], kps["octave"][i] = uo, vo, lvl
        if st:
            ur[i] = max(0.0, uo - cam["bf"] / z + rng.normal(0, s))
        pos[i] = Xw
    Rp = _axis_angle(rng.normal(size=3), np.deg2rad(rot_deg)) @ Rt
    d = rng.normal(size=3)
    tp = tt + trans_m * d / np.linalg.norm(d)
    T0 = np.eye(4, dtype=np.float32)
    T0[:3, :3] = Rp
    T0[:3, 3] = tp
    gt = np.eye(4)
    gt[:3, :3] = Rt
    gt[:3, 3] = tt
    return dict(Tcw=T0, kps=kps, uright=ur, has_mp=has, mp_pos=pos, inv_sigma2=inv_sigma2,
                cam=(np.float32(cam["fx"]), np.float32(cam["fy"]), np.float32(cam["cx"]),
                     np.float32(cam["cy"]), np.float32(cam["bf"])), gt_Tcw=gt)


EUROC_STEREO = dict(fx=435.2046959714599, bf=47.90639384423901)  # EuRoC.yaml Camera.fx / Camera.bf


def stereo_pair(seed: int, width: int = 752, height: int = 480, d_min: float = 4.0, d_max: float = 40.0,
                noise: float = 2.0):
    """Rectified stereo pair (left, right) uint8: the left frame is `frame(seed)`; the right
    one samples it at x + d(x, y) (linear interpolation, so disparities are sub-pixel) where
    d is a piecewise-planar disparity field in [d_min, d_max] (a slanted background plane
    and a few fronto-parallel boxes), plus Gaussian noise."""
    left = frame(seed, width, height)
    rng = np.random.default_rng(seed + 7919)
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float64)
    d = d_min + (0.35 * (d_max - d_min)) * (xx / width) + 0.1 * (d_max - d_min) * (yy / height)
    for _ in range(4):
        x0, y0 = rng.integers(0, width - 60), rng.integers(0, height - 60)
        bw, bh = rng.integers(60, 240), rng.integers(60, 200)
        d[y0:y0 + bh, x0:x0 + bw] = rng.uniform(0.5 * (d_min + d_max), d_max)
    xs = xx + d
    x0 = np.clip(np.floor(xs).astype(np.int64), 0, width - 1)
    x1 = np.clip(x0 + 1, 0, width - 1)
    fx = np.clip(xs - np.floor(xs), 0.0, 1.0)
    lf = left.astype(np.float64)
    rows = np.arange(height)[:, None]
    right = lf[rows, x0] * (1 - fx) + lf[rows, x1] * fx + rng.normal(0.0, noise, size=left.shape)
    return left, np.ascontiguousarray(np.clip(np.rint(right), 0, 255).astype(np.uint8))


def unrectify(rect: np.ndarray, map_x: np.ndarray, map_y: np.ndarray) -> np.ndarray:
    """A raw (distorted, unrectified) image whose rectification through (map_x, map_y)
    reproduces `rect` up to resampling: rectified pixel r reads the raw image at
    (map_x[r], map_y[r]), so each rectified pixel is splatted there (bilinear weights) and
    the few holes are filled from their neighbours."""
    h, w = rect.shape
    acc = np.zeros((h + 2, w + 2))
    wsum = np.zeros((h + 2, w + 2))
    x0 = np.floor(map_x).astype(np.int64)
    y0 = np.floor(map_y).astype(np.int64)
    fx, fy = map_x - x0, map_y - y0
    val = rect.astype(np.float64)
    for dy, dx, wt in ((0, 0, (1 - fx) * (1 - fy)), (0, 1, fx * (1 - fy)), (1, 0, (1 - fx) * fy), (1, 1, fx * fy)):
        xi, yi = x0 + dx + 1, y0 + dy + 1
        ok = (xi >= 0) & (xi < w + 2) & (yi >= 0) & (yi < h + 2)
        flat = (yi[ok] * (w + 2) + xi[ok]).ravel()
        # bincount accumulates in input order, as np.add.at does (same sums, ~20x faster)
        acc += np.bincount(flat, (val * wt)[ok].ravel(), minlength=acc.size).reshape(acc.shape)
        wsum += np.bincount(flat, wt[ok].ravel(), minlength=acc.size).reshape(acc.shape)
    acc, wsum = acc[1:-1, 1:-1], wsum[1:-1, 1:-1]
    out = np.where(wsum > 1e-6, acc / np.maximum(wsum, 1e-6), np.nan)
    # fill holes from their 4-neighbours, Jacobi passes (each pass reads the previous one); only
    # the hole pixels are visited, the neighbour sum in the order np.nansum over the stacked
    # (up, down, left, right) planes takes
    for _ in range(32):
        ys, xs = np.nonzero(np.isnan(out))
        if len(ys) == 0:
            break
        pad = np.pad(out, 1, constant_values=np.nan)
        acc_n = np.zeros(len(ys))
        cnt = np.zeros(len(ys), np.int64)
        for v in (pad[ys, xs + 1], pad[ys + 2, xs + 1], pad[ys + 1, xs], pad[ys + 1, xs + 2]):
            ok = np.isfinite(v)
            acc_n = acc_n + np.where(ok, v, 0.0)
            cnt += ok
        new = cnt > 0
        if not new.any():  # nothing reachable is left: later passes would change nothing
            break
        out[ys[new], xs[new]] = acc_n[new] / cnt[new]
    out = np.nan_to_num(out, nan=128.0)
    return np.ascontiguousarray(np.clip(np.rint(out), 0, 255).astype(np.uint8))


# --------------------------------------------------------------------------------------------
# Rendered sequences: a textured box room seen by a moving (stereo) pinhole camera, so frame
# poses, stereo disparities and feature tracks are geometrically consistent (tracking chain,
# config-3 / config-5 legs).  Camera convention as the reference: Tcw maps world -> camera,
# x right, y down, z forward; the right camera sits at +b along the left camera's x axis.
# --------------------------------------------------------------------------------------------
ROOM = (-4.0, 4.0, -1.8, 1.8, -3.0, 6.0)  # x0, x1, y0, y1, z0, z1 (m)
_TEX_PER_M = 110.0


def _wall_textures(seed: int):
    """Six wall textures (T x T float) from the procedural frame generator."""
    return [frame(seed * 16 + k, 1024, 1024).astype(np.float64) for k in range(6)]


def _sample(tex, a, b):
    """Bilinear texture lookup at texel coordinates (a, b), wrapped."""
    T = tex.shape[0]
    a0 = np.floor(a)
    b0 = np.floor(b)
    fa, fb = a - a0, b - b0
    a0 = a0.astype(np.int64) % T
    b0 = b0.astype(np.int64) % T
    a1, b1 = (a0 + 1) % T, (b0 + 1) % T
    return ((tex[b0, a0] * (1 - fa) + tex[b0, a1] * fa) * (1 - fb) +
            (tex[b1, a0] * (1 - fa) + tex[b1, a1] * fa) * fb)


EUROC_MONO_CAM = dict(fx=458.654, fy=457.296, cx=367.215, cy=248.375, w=752, h=480,
                      dist=(-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05))  # Monocular/EuRoC.yaml


def _undistort_normalized(xx, yy, cam):
    """Normalised undistorted coordinates of raw pixels (the radial-tangential model inverted by
    fixed-point iteration, as cv::undistortPoints; 20 iterations for rendering)."""
    k1, k2, p1, p2 = cam["dist"][:4]
    k3 = cam["dist"][4] if len(cam["dist"]) > 4 else 0.0
    x0 = (xx - cam["cx"]) / cam["fx"]
    y0 = (yy - cam["cy"]) / cam["fy"]
    x, y = x0.copy(), y0.copy()
    for _ in range(20):
        r2 = x * x + y * y
        icd = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x = (x0 - dx) * icd
        y = (y0 - dy) * icd
    return x, y


def render_view(textures, Tcw, cam=EUROC_CAM, width=None, height=None, noise_seed=None):
    """Ray-cast the textured room from camera pose Tcw (4x4 world -> camera); returns
    (image u8, depth float64 z along the optical axis).  A ``dist`` entry in ``cam`` renders
    the raw (distorted) image of that camera."""
    W = width or cam["w"]
    H = height or cam["h"]
    R, t = Tcw[:3, :3], Tcw[:3, 3]
    C = -R.T @ t
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    if cam.get("dist") is not None:
        nx, ny = _undistort_normalized(xx, yy, cam)
        dc = np.stack([nx, ny, np.ones_like(xx)], -1)
    else:
        dc = np.stack([(xx - cam["cx"]) / cam["fx"], (yy - cam["cy"]) / cam["fy"], np.ones_like(xx)], -1)
    dw = dc @ R  # R^T d per pixel (row vectors)
    best = np.full((H, W), np.inf)
    img = np.zeros((H, W))
    x0, x1, y0, y1, z0, z1 = ROOM
    planes = [(0, x0, (2, 1)), (0, x1, (2, 1)), (1, y0, (0, 2)), (1, y1, (0, 2)), (2, z0, (0, 1)), (2, z1, (0, 1))]
    for k, (ax, val, (ua, va)) in enumerate(planes):
        with np.errstate(divide="ignore", invalid="ignore"):
            s = (val - C[ax]) / dw[..., ax]
        ok = (s > 1e-6) & (s < best)
        if not ok.any():
            continue
        P = C[None, None, :] + s[..., None] * dw
        a = P[..., ua] * _TEX_PER_M
        b = P[..., va] * _TEX_PER_M
        v = _sample(textures[k], a, b)
        img = np.where(ok, v, img)
        best = np.where(ok, s, best)
    depth = best  # dc has z = 1, so the ray parameter is the camera-frame depth
    if noise_seed is not None:
        img = img + np.random.default_rng(noise_seed).normal(0.0, 1.5, size=img.shape)
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8)), depth


def sequence_poses(seed: int, n: int, step_m: float = 0.03, yaw_deg: float = 0.6):
    """Ground-truth Tcw of a smooth walk through the room (looking roughly along +z)."""
    rng = np.random.default_rng(seed)
    c = np.array([rng.uniform(-1.0, 1.0), rng.uniform(-0.3, 0.3), rng.uniform(-1.5, 0.0)])
    yaw, pitch = rng.uniform(-0.3, 0.3), rng.uniform(-0.1, 0.1)
    dyaw = np.deg2rad(yaw_deg) * rng.choice([-1.0, 1.0])
    out = []
    for i in range(n):
        cy_, sy_ = np.cos(yaw), np.sin(yaw)
        cp, sp = np.cos(pitch), np.sin(pitch)
        Ry = np.array([[cy_, 0, sy_], [0, 1, 0], [-sy_, 0, cy_]])
        Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
        Rwc = Ry @ Rx
        T = np.eye(4)
        T[:3, :3] = Rwc.T
        T[:3, 3] = -Rwc.T @ c
        out.append(T)
        fwd = Rwc[:, 2]
        c = c + step_m * (0.7 * fwd + 0.3 * np.array([np.cos(0.1 * i), 0.2 * np.sin(0.07 * i), 0.0]))
        yaw += dyaw * (1.0 + 0.5 * np.sin(0.05 * i))
        pitch = 0.1 * np.sin(0.03 * i + seed)
    return out


def stereo_sequence(seed: int, n: int, cam=EUROC_CAM, step_m: float = 0.03, threads: int = 1):
    """n rectified stereo frames of the room: (lefts (n,H,W) u8, rights, gt Tcw list).
    The right camera is the left one shifted by b = bf / fx along its x axis.  threads > 1
    renders the views concurrently (numpy releases the GIL; same images)."""
    tex = _wall_textures(seed)
    b = cam["bf"] / cam["fx"]
    Ts = sequence_poses(seed, n, step_m)

    def view(j):
        i, right = divmod(j, 2)
        T = Ts[i].copy()
        if right:
            T[0, 3] -= b  # X_right = X_left - (b, 0, 0)
        return render_view(tex, T, cam, noise_seed=seed * 1000 + j)[0]

    if threads > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as pool:
            V = list(pool.map(view, range(2 * n)))
    else:
        V = [view(j) for j in range(2 * n)]
    return np.stack(V[0::2]), np.stack(V[1::2]), Ts


def mono_sequence(seed: int, n: int, cam=EUROC_MONO_CAM, step_m: float = 0.03):
    """n raw monocular frames of the room through a distorting pinhole camera (EuRoC MH01-like,
    Examples/Monocular/EuRoC.yaml): (images (n,H,W) u8, gt Tcw list)."""
    tex = _wall_textures(seed)
    imgs, Ts = [], []
    for i, T in enumerate(sequence_poses(seed, n, step_m)):
        imgs.append(render_view(tex, T, cam, noise_seed=seed * 1000 + i)[0])
        Ts.append(T)
    return np.stack(imgs), Ts
