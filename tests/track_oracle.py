"""CPU oracle of the per-sequence stereo tracking chain (BASELINE.json configs[4]; the device
runner is slamhot_tracker_*, csrc/track.hip).  TEST INFRASTRUCTURE: only tests and bench.py's
cpu_baseline use it.

One step of one sequence (Tracking::Track for a rectified stereo camera, Tracking.cc:1256-2350,
with the reference-KeyFrame map of a single tracking thread):
  cv::remap x2 (stereo_euroc.cc:168-169) -> ORBextractor x2 (Frame.cc:119-122) ->
  Frame::ComputeStereoMatches (Frame.cc:794-964) ->
  first frame: Tracking::StereoInitialization (Tracking.cc:2366-2429): N > 500, Tcw = I, a
    KeyFrame whose every feature with depth > 0 gets a MapPoint (Frame::UnprojectStereo);
  later frames with a velocity: Tracking::TrackWithMotionModel (Tracking.cc:2683-2775):
    UpdateLastFrame (mLastFrame.SetPose(Tlr * pRef->GetPose())), SetPose(mVelocity *
    mLastFrame.mTcw), ORBmatcher(0.9, true).SearchByProjection(F, LastFrame, 7) (14 below 20
    matches; < 20: failed), PoseOptimization, outliers dropped (nmatchesMap < 10: failed);
  frames without a velocity, or whose motion model failed: Tracking::TrackReferenceKeyFrame
    (Tracking.cc:2559-2616): ComputeBoW, ORBmatcher(0.7, true).SearchByBoW(refKF, F) (< 15:
    lost), SetPose(mLastFrame.mTcw), Optimizer::PoseOptimization, outliers dropped
    (nmatchesMap < 10: lost);
    Tracking::TrackLocalMap (Tracking.cc:3008-3090): SearchLocalPoints over the reference
    KeyFrame's MapPoints (isInFrustum 0.5, ORBmatcher(0.8).SearchByProjection th = 1),
    PoseOptimization, stereo outliers dropped, mnMatchesInliers;
    the motion model mVelocity = mTcw * LastTwc (Tracking.cc:2058-2068; a lost frame drops it);
    Tracking::NeedNewKeyFrame (Tracking.cc:2944-3040, stereo, LocalMapping idle; thRefRatio 0.4
    while the map holds one KeyFrame) and Tracking::CreateNewKeyFrame (Tracking.cc:3061-3178):
    the frame becomes the reference KeyFrame, keeping its tracked MapPoints and adding new ones
    from stereo depth in depth order until depth > mThDepth and more than 100 points; the frame
    becomes mLastFrame with Tcr = Tcw * Tref^-1 (Tracking.cc:2140-2150).
4x4 float cv::Mat products are restated as double accumulation rounded once (DESIGN.md §1,
deviation 3), identically on the device (csrc/track.hip gemm4).
Map bookkeeping is the minimal one this path needs (documented in DESIGN.md §4g): the local map is
the reference KeyFrame's MapPoints, a MapPoint keeps the descriptor / normal / scale range of its
creation (LocalMapping, which would refine them, is out of scope), Observations() > 0 for all.
"""
from __future__ import annotations

import numpy as np

import oracle_bind as ob

f32 = np.float32

NFEAT = 1200
TH_DEPTH = 35.0          # EuRoC.yaml ThDepth (stereo): mThDepth = mbf * ThDepth / fx (Tracking.cc:609)
CAM = dict(fx=435.2046959714599, fy=435.2046959714599, cx=367.4517211914062, cy=252.2008514404297,
           bf=47.90639384423901)  # EuRoC.yaml Camera.* (rectified)


def params():
    p = ob.params(nfeatures=NFEAT)
    scale, inv_scale, sigma2, inv_sigma2, _ = ob.levels(p)
    c = {k: f32(v) for k, v in CAM.items()}
    return dict(p=p, scale=scale, inv_scale=inv_scale, inv_sigma2=inv_sigma2, fx=c["fx"], fy=c["fy"], cx=c["cx"],
                cy=c["cy"], bf=c["bf"], b=f32(c["bf"] / c["fx"]), th_depth=f32(c["bf"] * f32(TH_DEPTH) / c["fx"]),
                invfx=f32(1.0) / c["fx"], invfy=f32(1.0) / c["fy"])


def camera_center(T):
    """mOw = -mRcw.t() * mtcw as a cv::Mat product (double accumulation, one rounding)."""
    R = T[:3, :3].astype(np.float64)
    t = T[:3, 3].astype(np.float64)
    return np.array([f32(-1.0 * (R[0, i] * t[0] + R[1, i] * t[1] + R[2, i] * t[2])) for i in range(3)], f32)


def unproject(P, T, kp, depth):
    """Frame::UnprojectStereo (Frame.cc:1006-1022): mRwc * x3Dc + mOw, one cv::gemm with beta."""
    z = f32(depth)
    x = (f32(kp["x"]) - P["cx"]) * z * P["invfx"]
    y = (f32(kp["y"]) - P["cy"]) * z * P["invfy"]
    xc = np.array([x, y, z], np.float64)
    R = T[:3, :3].astype(np.float64)
    Ow = camera_center(T)
    return np.array([f32((R[0, i] * xc[0] + R[1, i] * xc[1] + R[2, i] * xc[2]) * 1.0 + float(Ow[i]) * 1.0)
                     for i in range(3)], f32)


def mappoint_geometry(P, pos, Ow, octave):
    """MapPoint::UpdateNormalAndDepth with one observation (MapPoint.cc:486-538)."""
    PC = (pos - Ow).astype(f32)
    nd = np.sqrt(float(PC[0]) * float(PC[0]) + float(PC[1]) * float(PC[1]) + float(PC[2]) * float(PC[2]))
    dist = f32(nd)
    normal = np.array([f32(float(PC[k]) / nd) for k in range(3)], f32)
    maxd = dist * f32(P["scale"][octave])
    mind = maxd / f32(P["scale"][-1])
    return normal, f32(mind), f32(maxd)


class KeyFrame:
    """The reference KeyFrame of a sequence: features + one MapPoint slot per feature."""

    def __init__(self, kps, desc, Tcw):
        n = len(kps)
        self.kps, self.desc, self.Tcw = kps, desc, Tcw
        self.valid = np.zeros(n, np.uint8)
        self.pos = np.zeros((n, 3), f32)
        self.normal = np.zeros((n, 3), f32)
        self.mind = np.zeros(n, f32)
        self.maxd = np.zeros(n, f32)
        self.mdesc = np.zeros((n, 32), np.uint8)


class SeqState:
    def __init__(self):
        self.initialized = False
        self.Tcw = np.eye(4, dtype=f32)
        self.kf: KeyFrame | None = None
        self.n_ref = 0
        self.has_vel = False
        self.V = np.eye(4, dtype=f32)       # mVelocity
        self.Tlr = np.eye(4, dtype=f32)     # mlRelativeFramePoses.back()
        self.Tref = np.eye(4, dtype=f32)    # reference KeyFrame pose
        self.nkf = 0
        self.last_kps = None                # mLastFrame.mvKeysUn
        self.last_mp = None                 # mLastFrame.mvpMapPoints as KeyFrame MapPoint slots


def gemm4(A, B):
    """4x4 float cv::Mat product: double accumulation in k order, one rounding per entry."""
    C = np.zeros((4, 4), f32)
    for i in range(4):
        for j in range(4):
            acc = 0.0
            for k in range(4):
                acc += float(A[i, k]) * float(B[k, j])
            C[i, j] = f32(acc)
    return C


def pose_inverse(T):
    """Twc as Frame::UpdatePoseMatrices / KeyFrame::SetPose form it: Rcw^T | -Rcw^T tcw."""
    W = np.zeros((4, 4), f32)
    W[:3, :3] = T[:3, :3].T
    W[:3, 3] = camera_center(T)
    W[3, 3] = 1
    return W


def set_last_frame(st, kps, f_mp, Tcw, new_kf):
    """mLastFrame = Frame(mCurrentFrame) and Tcr (Tracking.cc:2140-2150); after a new KeyFrame the
    frame holds every MapPoint of it (CreateNewKeyFrame, Tracking.cc:3290-3300)."""
    st.last_kps = kps.copy()
    st.last_mp = (np.where(st.kf.valid != 0, np.arange(len(kps)), -1) if new_kf else f_mp).astype(np.int32)
    st.Tlr = gemm4(Tcw, pose_inverse(st.Tref))


def frame_features(P, maps, raw_l, raw_r):
    l_img = ob.remap_linear(raw_l, *maps[0])
    r_img = ob.remap_linear(raw_r, *maps[1])
    kl, dl, _ = ob.extract(l_img, P["p"])
    kr, dr, _ = ob.extract(r_img, P["p"])
    ur, dep = ob.stereo_matches(kl, dl, kr, dr, ob.pyramid(l_img, P["p"]), ob.pyramid(r_img, P["p"]), P["scale"],
                                P["inv_scale"], P["bf"], P["b"])
    return kl, dl, ur, dep


def _bow_side(voc, desc, angle, valid):
    from slamhot import synth
    par, leaf, dn, wn = voc
    _, wt, nid = ob.vocab_transform(par, leaf, dn, wn, 6, desc, 4)
    return (desc, angle, valid) + synth.feature_vector(nid, wt)


def _pose(P, T, kps, ur, f_mp, kf):
    has = f_mp >= 0
    pos = np.zeros((len(kps), 3), f32)
    pos[has] = kf.pos[f_mp[has]]
    return ob.pose_optimization(dict(Tcw=T, kps=kps, uright=ur, has_mp=has.astype(np.uint8), mp_pos=pos,
                                     inv_sigma2=P["inv_sigma2"], cam=(P["fx"], P["fy"], P["cx"], P["cy"], P["bf"])))


def new_keyframe(P, kps, desc, dep, Tcw, f_mp=None, old=None, initial=False):
    """StereoInitialization (every depth > 0) / CreateNewKeyFrame (depth order, stop past
    mThDepth once more than 100 points)."""
    kf = KeyFrame(kps, desc, Tcw)
    Ow = camera_center(Tcw)
    n = len(kps)
    if f_mp is not None:  # tracked MapPoints move to the new KeyFrame unchanged
        for i in np.flatnonzero(f_mp >= 0):
            j = f_mp[i]
            kf.valid[i] = 1
            kf.pos[i], kf.normal[i], kf.mind[i], kf.maxd[i], kf.mdesc[i] = (old.pos[j], old.normal[j], old.mind[j],
                                                                            old.maxd[j], old.mdesc[j])

    def create(i):
        kf.valid[i] = 1
        kf.pos[i] = unproject(P, Tcw, kps[i], dep[i])
        kf.normal[i], kf.mind[i], kf.maxd[i] = mappoint_geometry(P, kf.pos[i], Ow, int(kps[i]["octave"]))
        kf.mdesc[i] = desc[i]

    if initial:
        for i in range(n):
            if dep[i] > 0:
                create(i)
        return kf
    order = sorted((float(dep[i]), i) for i in range(n) if dep[i] > 0)  # vDepthIdx, std::sort of pairs
    npts = 0
    for d, i in order:
        if not kf.valid[i]:
            create(i)
        npts += 1
        if d > P["th_depth"] and npts > 100:
            break
    return kf


def _last_frame_view(st, Tlast):
    import slamhot
    kf = st.kf
    lm = st.last_mp
    j = np.where(lm >= 0, lm, 0)
    has = (lm >= 0) & (kf.valid[j] != 0)
    pos = np.where(has[:, None], kf.pos[j], 0).astype(f32)
    desc = np.where(has[:, None], kf.mdesc[j], 0).astype(np.uint8)
    n = len(lm)
    return slamhot.make_last_frame(Tlast, st.last_kps, st.last_kps, has.astype(np.uint8), np.zeros(n, np.uint8),
                                   pos, desc, np.ones(n, np.uint8))


def step(P, voc, maps, st: SeqState, raw_l, raw_r):
    """One frame; returns the record the device tracker reports for it, with the per-feature
    arrays (uright, bow_match, motion_match, local_match, mappoints)."""
    import slamhot
    kl, dl, ur, dep = frame_features(P, maps, raw_l, raw_r)
    n = len(kl)
    none = np.full(n, -1, np.int32)
    rec = dict(n=n, nbow=0, ninl1=0, nlocal=0, ninl2=0, is_kf=0, lost=0, stereo=int((dep > 0).sum()), n_motion=0,
               motion=0, uright=ur, bow_match=none.copy(), motion_match=none.copy(), local_match=none.copy(),
               mappoints=none.copy())
    if not st.initialized:
        if n > 500:
            st.kf = new_keyframe(P, kl, dl, dep, np.eye(4, dtype=f32), initial=True)
            st.Tcw = np.eye(4, dtype=f32)
            st.initialized = True
            st.n_ref = int(st.kf.valid.sum())
            st.nkf = 1
            st.has_vel = False
            st.Tref = np.eye(4, dtype=f32)
            set_last_frame(st, kl, None, st.Tcw, True)
            rec["is_kf"] = 1
        rec["Tcw"] = st.Tcw.copy()
        return rec
    kf = st.kf
    cam = (P["fx"], P["fy"], P["cx"], P["cy"])
    f_mp = None
    T1 = None
    Tlast = st.Tcw
    if st.has_vel:  # TrackWithMotionModel
        Tlast = gemm4(st.Tlr, st.Tref)
        Tpred = gemm4(st.V, Tlast)
        lf, lkeep = _last_frame_view(st, Tlast)
        fv, keep = slamhot.make_frame_view(kl, dl, ur, np.full(n, -1, np.int8), cam=cam, bf=P["bf"], Tcw=Tpred)
        nm, fm = ob.search_by_projection_last(fv, lf, 0.9, True, 7.0, False)
        if nm < 20:
            nm, fm = ob.search_by_projection_last(fv, lf, 0.9, True, 14.0, False)
        rec["n_motion"] = int(nm)
        if nm >= 20:
            mm = np.where(fm >= 0, st.last_mp[np.maximum(fm, 0)], -1).astype(np.int32)
            rec["motion_match"] = mm.copy()
            r = _pose(P, Tpred, kl, ur, mm, kf)
            mm[r["outlier"].astype(bool) & (mm >= 0)] = -1
            if int((mm >= 0).sum()) >= 10:
                f_mp, T1 = mm, r["Tcw"].astype(f32)
                rec["motion"] = 1
                rec["ninl1"] = int((mm >= 0).sum())
    if f_mp is None:  # TrackReferenceKeyFrame
        A = _bow_side(voc, kf.desc, kf.kps["angle"], kf.valid)
        B = _bow_side(voc, dl, kl["angle"], None)
        nbow, _, b2a = ob.search_by_bow(A, B, 0.7, True, False)
        rec["nbow"] = nbow
        rec["bow_match"] = b2a.astype(np.int32)
        if nbow < 15:
            st.has_vel = False
            rec.update(lost=1, Tcw=st.Tcw.copy())
            return rec
        f_mp = b2a.astype(np.int32).copy()
        r1 = _pose(P, Tlast, kl, ur, f_mp, kf)
        out1 = r1["outlier"].astype(bool) & (f_mp >= 0)
        f_mp[out1] = -1
        rec["ninl1"] = int((f_mp >= 0).sum())
        T1 = r1["Tcw"].astype(f32)
        if rec["ninl1"] < 10:  # the device reports nmatchesMap only for a tracked frame
            st.has_vel = False
            rec.update(lost=1, ninl1=0, Tcw=st.Tcw.copy(), mappoints=f_mp.copy())
            return rec
    # SearchLocalPoints over the reference KeyFrame's MapPoints
    geom = np.zeros(len(kf.kps), slamhot.MP_GEOM_DTYPE)
    geom["pos"], geom["normal"] = kf.pos, kf.normal
    geom["min_dist"], geom["max_dist"] = kf.mind, kf.maxd
    seen = np.zeros(len(kf.kps), np.uint8)
    seen[f_mp[f_mp >= 0]] = 1
    geom["seen"] = seen
    geom["is_bad"] = 1 - kf.valid
    geom["has_obs"] = 1
    state = np.where(f_mp >= 0, 1, -1).astype(np.int8)
    fv, keep = slamhot.make_frame_view(kl, dl, ur, state, cam=cam, bf=P["bf"], Tcw=T1)
    nto, track = ob.is_in_frustum(fv, geom, 0.5)
    nloc = 0
    if nto > 0:
        nloc, fm = ob.search_by_projection_local(fv, track, kf.mdesc, 0.8, 1.0, False, 50.0)
        rec["local_match"] = fm.astype(np.int32)
        f_mp = np.where(fm >= 0, fm, f_mp).astype(np.int32)
    rec["nlocal"] = int(nloc)
    r2 = _pose(P, T1, kl, ur, f_mp, kf)
    out2 = r2["outlier"].astype(bool) & (f_mp >= 0)
    f_mp[out2] = -1  # stereo: outliers leave the frame (Tracking.cc:3060-3061)
    ninl = int((f_mp >= 0).sum())
    rec["ninl2"] = ninl
    rec["mappoints"] = f_mp.copy()
    T2 = r2["Tcw"].astype(f32)
    st.Tcw = T2
    rec["Tcw"] = T2.copy()
    if ninl < 30:
        st.has_vel = False
        rec["lost"] = 1
        return rec
    st.V = gemm4(T2, pose_inverse(Tlast))  # mVelocity = mCurrentFrame.mTcw * LastTwc
    st.has_vel = True
    # NeedNewKeyFrame (stereo; LocalMapping idle so c1b holds): c2
    close = (dep > 0) & (dep < P["th_depth"])
    n_tracked_close = int((close & (f_mp >= 0)).sum())
    n_non_tracked_close = int((close & (f_mp < 0)).sum())
    need_close = n_tracked_close < 100 and n_non_tracked_close > 70
    th_ref_ratio = f32(0.4) if st.nkf < 2 else f32(0.75)
    new_kf = (f32(ninl) < f32(st.n_ref) * th_ref_ratio or need_close) and ninl > 15
    if new_kf:
        st.kf = new_keyframe(P, kl, dl, dep, T2, f_mp=f_mp, old=kf)
        st.n_ref = int(st.kf.valid.sum())
        st.nkf += 1
        st.Tref = T2.copy()
        rec["is_kf"] = 1
    set_last_frame(st, kl, f_mp, T2, new_kf)
    return rec
