"""Seeded synthetic tracking scenes for the projection matchers (shared by CPU and GPU tests).
EuRoC stereo intrinsics (Examples/Stereo/EuRoC.yaml:8-31)."""
import numpy as np

import oracle_bind as ob
import slamhot
from slamhot import synth

FX = FY = np.float32(435.2047)
CX, CY = np.float32(367.4517), np.float32(252.2009)
BF = np.float32(47.9064)


def rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay), np.cos(az), np.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def pose(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T.astype(np.float32)


def flip_bits(desc, rng, max_flips):
    bits = np.unpackbits(desc, axis=1)
    for i in range(len(bits)):
        k = rng.integers(0, max_flips + 1)
        bits[i, rng.choice(256, size=k, replace=False)] ^= 1
    return np.packbits(bits, axis=1)


def current_frame(seed, n_feat=1200):
    img = synth.frame(seed, 752, 480)
    k, d, _ = ob.extract(img, ob.params(nfeatures=n_feat))
    return k, d


def scene(seed, n_feat=1200):
    rng = np.random.default_rng(seed)
    k, d = current_frame(seed, n_feat)
    n = len(k)
    uright = np.where(rng.random(n) < 0.6, k["x"] - rng.uniform(5, 40, n), -1).astype(np.float32)
    state = np.full(n, -1, np.int8)
    r = rng.random(n)
    state[r < 0.05] = 0
    state[(r >= 0.05) & (r < 0.10)] = 1
    Tcw = pose(rot(*rng.normal(0, 0.05, 3)), rng.normal(0, 0.3, 3))
    return dict(rng=rng, k=k, d=d, uright=uright, state=state, Tcw=Tcw)


def frame_view(S, with_pose=True):
    return slamhot.make_frame_view(S["k"], S["d"], S["uright"], S["state"], Tcw=S["Tcw"] if with_pose else None)


def local_map(S, n_extra=400):
    rng, k, d = S["rng"], S["k"], S["d"]
    n = len(k)
    sel = rng.permutation(n)[: int(n * 0.8)]
    m = len(sel) + n_extra
    mps = np.zeros(m, slamhot.MP_TRACK_DTYPE)
    desc = np.zeros((m, 32), np.uint8)
    jit = rng.normal(0, 1.2, (len(sel), 2)).astype(np.float32)
    mps["proj_x"][: len(sel)] = k["x"][sel] + jit[:, 0]
    mps["proj_y"][: len(sel)] = k["y"][sel] + jit[:, 1]
    mps["scale_level"][: len(sel)] = np.clip(k["octave"][sel] + rng.integers(-1, 2, len(sel)), 0, 7)
    desc[: len(sel)] = flip_bits(d[sel], rng, 40)
    mps["proj_x"][len(sel):] = rng.uniform(0, 752, n_extra)
    mps["proj_y"][len(sel):] = rng.uniform(0, 480, n_extra)
    mps["scale_level"][len(sel):] = rng.integers(0, 8, n_extra)
    desc[len(sel):] = flip_bits(d[rng.integers(0, n, n_extra)], rng, 90)
    ur = S["uright"]
    base_ur = np.concatenate([np.where(ur[sel] > 0, ur[sel], mps["proj_x"][: len(sel)] - 20), mps["proj_x"][len(sel):] - 15])
    mps["proj_xr"] = (base_ur + rng.normal(0, 3, m)).astype(np.float32)
    mps["depth"] = rng.uniform(0.5, 80, m)
    mps["view_cos"] = rng.uniform(0.99, 1.0, m)
    mps["in_view"] = rng.random(m) < 0.95
    mps["is_bad"] = rng.random(m) < 0.03
    mps["has_obs"] = rng.random(m) < 0.9
    order = rng.permutation(m)
    return mps[order], desc[order]


def backproject(S, x, y, depth):
    Xc = np.stack([(x - CX) / FX * depth, (y - CY) / FY * depth, depth], 1)
    T = S["Tcw"].astype(np.float64)
    R, t = T[:3, :3], T[:3, 3]
    return ((Xc - t) @ R).astype(np.float32)


def last_frame(S, mono=False, motion=0.02):
    rng, k, d = S["rng"], S["k"], S["d"]
    n = len(k)
    depth = rng.uniform(1.0, 20.0, n).astype(np.float32)
    Xw = backproject(S, k["x"] + rng.normal(0, 1.0, n), k["y"] + rng.normal(0, 1.0, n), depth)
    T = S["Tcw"].astype(np.float64)
    Tl = pose(rot(*rng.normal(0, 0.01, 3)) @ T[:3, :3], T[:3, 3] + rng.normal(0, motion, 3))
    kl = k.copy()
    kl["octave"] = np.clip(k["octave"] + rng.integers(-1, 2, n), 0, 7)
    kl_un = kl.copy()
    kl_un["angle"] = np.where(rng.random(n) < 0.8, (k["angle"] + rng.normal(0, 8, n)) % 360,
                              rng.uniform(0, 360, n)).astype(np.float32)
    has_mp = rng.random(n) < 0.85
    outlier = rng.random(n) < 0.05
    has_obs = rng.random(n) < 0.9
    desc = flip_bits(d, rng, 45)
    order = rng.permutation(n)
    return slamhot.make_last_frame(Tl, kl[order], kl_un[order], has_mp[order], outlier[order], Xw[order], desc[order],
                                   has_obs[order])


def kf_points(S):
    rng, k, d = S["rng"], S["k"], S["d"]
    n = len(k)
    depth = rng.uniform(1.0, 20.0, n).astype(np.float32)
    Xw = backproject(S, k["x"] + rng.normal(0, 1.0, n), k["y"] + rng.normal(0, 1.0, n), depth)
    max_d = (depth * rng.uniform(1.0, 3.0, n)).astype(np.float32)
    min_d = (max_d / np.float32(1.2 ** 7)).astype(np.float32)
    kk = k.copy()
    kk["angle"] = np.where(rng.random(n) < 0.8, (k["angle"] + rng.normal(0, 8, n)) % 360,
                           rng.uniform(0, 360, n)).astype(np.float32)
    use = rng.random(n) < 0.9
    desc = flip_bits(d, rng, 45)
    order = rng.permutation(n)
    return slamhot.make_kf_points(kk[order], use[order], Xw[order], max_d[order], min_d[order], desc[order])


def local_map_geom(S, n_extra=300, boundary_frac=0.15):
    """Local MapPoints as Tracking::SearchLocalPoints sees them (slamhot.MP_GEOM_DTYPE):
    most back-projected from current features (so isInFrustum accepts them and the matcher
    finds them), some behind the camera / off-image / out of the distance range / at grazing
    view angles, some already seen or bad, and a fraction whose mfMaxDistance puts the
    predicted level exactly on a scale boundary (ratio = 1.2^l, the MapPoint's creation
    distance)."""
    rng, k, d = S["rng"], S["k"], S["d"]
    n = len(k)
    sel = rng.permutation(n)[: int(n * 0.75)]
    depth = rng.uniform(0.8, 25.0, len(sel)).astype(np.float32)
    X = backproject(S, k["x"][sel] + rng.normal(0, 1.0, len(sel)), k["y"][sel] + rng.normal(0, 1.0, len(sel)), depth)
    Xe = backproject(S, rng.uniform(-200, 952, n_extra), rng.uniform(-150, 630, n_extra),
                     rng.uniform(-5.0, 40.0, n_extra).astype(np.float32))
    pos = np.concatenate([X, Xe]).astype(np.float32)
    m = len(pos)
    T = S["Tcw"].astype(np.float64)
    Ow = -(T[:3, :3].T @ T[:3, 3])
    PO = pos.astype(np.float64) - Ow
    dist = np.linalg.norm(PO, axis=1)
    # normal: mostly towards the camera, some at grazing angles
    nrm = PO / dist[:, None]
    tilt = rng.normal(0, 0.3, (m, 3))
    tilt[rng.random(m) < 0.1] *= 8.0
    nrm = nrm + tilt
    nrm = (nrm / np.linalg.norm(nrm, axis=1)[:, None]).astype(np.float32)
    level = rng.integers(0, 8, m)
    max_d = (dist * np.float32(1.2) ** level * rng.uniform(0.9, 1.6, m)).astype(np.float32)
    b = rng.random(m) < boundary_frac
    # creation distance == current distance: max_d = dist * scaleFactor^level exactly
    sc = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    max_d[b] = (dist[b].astype(np.float32) * sc[level[b]]).astype(np.float32)
    min_d = (max_d / sc[7]).astype(np.float32)
    geom = np.zeros(m, slamhot.MP_GEOM_DTYPE)
    geom["pos"] = pos
    geom["normal"] = nrm
    geom["min_dist"] = min_d
    geom["max_dist"] = max_d
    geom["seen"] = rng.random(m) < 0.05
    geom["is_bad"] = rng.random(m) < 0.03
    geom["has_obs"] = rng.random(m) < 0.9
    desc = np.concatenate([flip_bits(d[sel], rng, 40), flip_bits(d[rng.integers(0, n, n_extra)], rng, 90)])
    order = rng.permutation(m)
    return geom[order], desc[order]


def _Rt(T):
    return T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)


def tri_keyframes(seed, n_kf=4, n_pts=1500, n_nodes=400):
    """KeyFrames around a common point cloud for SearchForTriangulation_: features are noisy
    projections of shared points (descriptor = point pattern + a few flipped bits, FeatureVector
    node = point id hash, so corresponding features share nodes), plus clutter; ~30% already
    have a MapPoint, ~40% are stereo.  Returns (kfs dicts, poses)."""
    rng = np.random.default_rng(seed)
    sc, isig, _ = synth._level_tables()
    sigma2 = (sc * sc).astype(np.float32)
    P = np.stack([rng.uniform(-4, 4, n_pts), rng.uniform(-2.5, 2.5, n_pts), rng.uniform(3, 15, n_pts)], 1)
    base = rng.integers(0, 256, (n_pts, 32), dtype=np.uint8)
    node_of_pt = rng.integers(0, n_nodes, n_pts)
    kfs, poses = [], []
    for k in range(n_kf):
        T = pose(rot(*rng.normal(0, 0.04, 3)), np.array([0.25 * k, rng.normal(0, 0.05), rng.normal(0, 0.1)]))
        R, t = _Rt(T)
        Xc = P @ R.T + t
        u = FX * Xc[:, 0] / Xc[:, 2] + CX
        v = FY * Xc[:, 1] / Xc[:, 2] + CY
        vis = np.flatnonzero((Xc[:, 2] > 0.5) & (u > 5) & (u < 747) & (v > 5) & (v < 475) & (rng.random(n_pts) < 0.8))
        nclut = 200
        n = len(vis) + nclut
        kps = np.zeros(n, slamhot.KP_DTYPE)
        kps["x"][: len(vis)] = u[vis] + rng.normal(0, 0.7, len(vis))
        kps["y"][: len(vis)] = v[vis] + rng.normal(0, 0.7, len(vis))
        kps["x"][len(vis):] = rng.uniform(5, 747, nclut)
        kps["y"][len(vis):] = rng.uniform(5, 475, nclut)
        kps["octave"] = rng.integers(0, 8, n)
        kps["angle"] = np.concatenate([(rng.normal(90, 6, len(vis))) % 360, rng.uniform(0, 360, nclut)])
        desc = np.concatenate([flip_bits(base[vis], rng, 12), rng.integers(0, 256, (nclut, 32), dtype=np.uint8)])
        ur = np.full(n, -1, np.float32)
        st = rng.random(n) < 0.4
        ur[: len(vis)][st[: len(vis)]] = (kps["x"][: len(vis)] - BF / Xc[vis, 2].astype(np.float32))[st[: len(vis)]]
        has_mp = (rng.random(n) < 0.3).astype(np.uint8)
        nid = np.concatenate([node_of_pt[vis], rng.integers(0, n_nodes, nclut)])
        order = rng.permutation(n)
        kps, desc, ur, has_mp, nid = kps[order], desc[order], ur[order], has_mp[order], nid[order]
        uniq, noff, nfeat = synth.feature_vector(nid, np.ones(n))
        kfs.append(dict(kps_un=kps, desc=desc, uright=ur, has_mp=has_mp, node_id=uniq.astype(np.int32),
                        node_off=noff, node_feat=nfeat.astype(np.int32), scale=sc, level_sigma2=sigma2,
                        Tcw=T.astype(np.float32), cam=np.array([FX, FY, CX, CY], np.float32)))
        poses.append(T)
    return kfs, poses


def fuse_mps(S, n_extra=300):
    """MapPoints to fuse into the scene's frame treated as a KeyFrame: most back-projected near
    features (descriptor close to the feature's, mfMaxDistance putting the predicted level on
    the feature's octave, normal along the viewing ray), plus far / behind / off-image / bad /
    already-in-KF ones and some at grazing angles."""
    rng, k, d = S["rng"], S["k"], S["d"]
    n = len(k)
    sel = rng.permutation(n)[: int(n * 0.7)]
    depth = rng.uniform(0.8, 25.0, len(sel)).astype(np.float32)
    X = backproject(S, k["x"][sel] + rng.normal(0, 0.8, len(sel)), k["y"][sel] + rng.normal(0, 0.8, len(sel)), depth)
    Xe = backproject(S, rng.uniform(-200, 952, n_extra), rng.uniform(-150, 630, n_extra),
                     rng.uniform(-5.0, 40.0, n_extra).astype(np.float32))
    pos = np.concatenate([X, Xe]).astype(np.float32)
    m = len(pos)
    T = S["Tcw"].astype(np.float64)
    Ow = -(T[:3, :3].T @ T[:3, 3])
    PO = pos.astype(np.float64) - Ow
    dist = np.linalg.norm(PO, axis=1)
    nrm = PO / dist[:, None] + rng.normal(0, 0.25, PO.shape)
    graze = rng.random(m) < 0.08
    nrm[graze] = rng.normal(0, 1, (graze.sum(), 3))
    nrm = (nrm / np.linalg.norm(nrm, axis=1)[:, None]).astype(np.float32)
    sc = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    oct_ = np.concatenate([k["octave"][sel], rng.integers(0, 8, n_extra)])
    max_d = (dist * sc[oct_] * rng.uniform(1.0, 1.19, m)).astype(np.float32)
    min_d = (max_d / sc[7]).astype(np.float32)
    geom = np.zeros(m, slamhot.MP_GEOM_DTYPE)
    geom["pos"] = pos
    geom["normal"] = nrm
    geom["min_dist"] = min_d
    geom["max_dist"] = max_d
    geom["seen"] = rng.random(m) < 0.05
    geom["is_bad"] = rng.random(m) < 0.03
    geom["has_obs"] = 1
    desc = np.concatenate([flip_bits(d[sel], rng, 45), flip_bits(d[rng.integers(0, n, n_extra)], rng, 90)])
    order = rng.permutation(m)
    return geom[order], desc[order]
