"""Host-side mirror of ``Optimizer::LocalBundleAdjustment`` (Optimizer.h:59,
Optimizer.cc:1611-2078) over a minimal map model, with the LM/Schur solve on the device
(``slamhot_lba_solve``).

The map objects carry exactly the fields LocalBundleAdjustment reads (KeyFrame.h:235-261,
MapPoint.h); window construction, flattening, outlier erasure and write-back follow the
reference line by line (cited below).  This is the logic a C++ shim keeps around the C ABI
(INTEGRATION.md); here it drives the tests and the examples.
"""
from __future__ import annotations

import ctypes as C

import numpy as np


class Map:
    def __init__(self, init_kf_id: int = 0, inertial: bool = False):
        self.init_kf_id = init_kf_id      # Map::GetInitKFid
        self.inertial = inertial          # Map::IsInertial
        self.change_index = 0

    def GetInitKFid(self):
        return self.init_kf_id

    def IsInertial(self):
        return self.inertial

    def IncreaseChangeIndex(self):
        self.change_index += 1


class MapPoint:
    def __init__(self, mnId: int, pos, pmap: Map):
        self.mnId = mnId
        self.pos = np.asarray(pos, np.float32).reshape(3)
        self.map = pmap
        self.bad = False
        # std::map<KeyFrame*, tuple<int,int>>: ordered by key; the mirror orders by KF id
        self.observations: dict = {}
        self.mnBALocalForKF = -1
        self.normal_updates = 0

    def isBad(self):
        return self.bad

    def GetMap(self):
        return self.map

    def GetWorldPos(self):
        return self.pos.copy()

    def SetWorldPos(self, p):
        self.pos = np.asarray(p, np.float32).reshape(3)

    def GetObservations(self):
        return dict(sorted(self.observations.items(), key=lambda kv: kv[0].mnId))

    def AddObservation(self, kf, left_idx, right_idx=-1):
        self.observations[kf] = (left_idx, right_idx)

    def EraseObservation(self, kf):
        self.observations.pop(kf, None)

    def UpdateNormalAndDepth(self):
        self.normal_updates += 1

    # --- what ORBmatcher::Fuse's apply half touches (MapPoint.cc)
    def IsInKeyFrame(self, kf):
        return kf in self.observations

    def Observations(self):
        """nObs: 2 per stereo observation, 1 per monocular one (MapPoint::AddObservation)."""
        n = 0
        for kf, (li, ri) in self.observations.items():
            if li != -1:
                n += 2 if kf.mvuRight[li] >= 0 else 1
            if ri != -1:
                n += 1
        return n

    def Replace(self, other):
        """MapPoint::Replace (MapPoint.cc:238-290): observations move to `other` (or are erased
        where `other` is already seen), this point turns bad."""
        if other.mnId == self.mnId:
            return
        obs = self.GetObservations()
        self.observations = {}
        self.bad = True
        self.replaced = other
        for kf, (li, ri) in obs.items():
            if not other.IsInKeyFrame(kf):
                if li != -1:
                    kf.mvpMapPoints[li] = other
                    other.AddObservation(kf, li)
            else:
                if li != -1:
                    kf.mvpMapPoints[li] = None


class KeyFrame:
    def __init__(self, mnId: int, Tcw, keys_un, uright, inv_level_sigma2, cam, pmap: Map):
        self.mnId = mnId
        self.Tcw = np.asarray(Tcw, np.float32).reshape(4, 4)
        self.mvKeysUn = keys_un              # structured array with x, y, octave
        self.mvuRight = np.asarray(uright, np.float32)
        self.mvInvLevelSigma2 = np.asarray(inv_level_sigma2, np.float32)
        self.fx, self.fy, self.cx, self.cy, self.mbf = [np.float32(c) for c in cam]
        self.map = pmap
        self.bad = False
        self.mvpMapPoints = [None] * len(keys_un)
        self.covisible: list = []            # GetVectorCovisibleKeyFrames order
        self.mnBALocalForKF = -1
        self.mnBAFixedForKF = -1
        # second camera (mpCamera2): right keypoints indexed from NLeft, mTrl, its parameters
        self.mpCamera2 = None
        self.mvKeysRight = None
        self.NLeft = -1
        self.mTrl = None

    def set_rig(self, keys_right, Trl, cam2):
        self.mvKeysRight = keys_right
        self.NLeft = len(self.mvKeysUn)
        self.mTrl = np.asarray(Trl, np.float32).reshape(4, 4)
        self.mpCamera2 = tuple(np.float32(c) for c in cam2[:4])
        self.mvpMapPoints = self.mvpMapPoints + [None] * len(keys_right)

    def isBad(self):
        return self.bad

    def GetMap(self):
        return self.map

    def GetPose(self):
        return self.Tcw.copy()

    def SetPose(self, T):
        self.Tcw = np.asarray(T, np.float32).reshape(4, 4)

    def GetVectorCovisibleKeyFrames(self):
        return list(self.covisible)

    def GetMapPointMatches(self):
        return list(self.mvpMapPoints)

    def GetMapPoint(self, idx):
        return self.mvpMapPoints[idx]

    def AddMapPoint(self, mp, idx):
        self.mvpMapPoints[idx] = mp

    def EraseMapPointMatch(self, mp):
        for i, m in enumerate(self.mvpMapPoints):
            if m is mp:
                self.mvpMapPoints[i] = None


def build_window(pKF: KeyFrame, pMap: Map):
    """Local / fixed KeyFrames and local MapPoints (Optimizer.cc:1613-1718).  Returns
    (local_kfs, fixed_kfs, local_mps, num_fixedKF) or None when the reference aborts for
    lack of a fixed KeyFrame (:1714-1718)."""
    local = [pKF]
    pKF.mnBALocalForKF = pKF.mnId
    cur_map = pKF.GetMap()
    for k in pKF.GetVectorCovisibleKeyFrames():                   # :1619-1626
        k.mnBALocalForKF = pKF.mnId
        if not k.isBad() and k.GetMap() is cur_map:
            local.append(k)
    num_fixed = 0
    local_mps = []
    for k in local:                                               # :1631-1655
        if k.mnId == pMap.GetInitKFid():
            num_fixed = 1
        for mp in k.GetMapPointMatches():
            if mp is not None and not mp.isBad() and mp.GetMap() is cur_map:
                if mp.mnBALocalForKF != pKF.mnId:
                    local_mps.append(mp)
                    mp.mnBALocalForKF = pKF.mnId
    fixed = []
    for mp in local_mps:                                          # :1659-1673
        for k in mp.GetObservations():
            if k.mnBALocalForKF != pKF.mnId and k.mnBAFixedForKF != pKF.mnId:
                k.mnBAFixedForKF = pKF.mnId
                if not k.isBad() and k.GetMap() is cur_map:
                    fixed.append(k)
    num_fixed = len(fixed) + num_fixed
    if num_fixed < 2:                                             # :1676-1712
        lower_id = second_id = pKF.mnId
        lower = second = None
        for k in local:
            if k is pKF or k.mnId == pMap.GetInitKFid():
                continue
            if k.mnId < lower_id:
                lower_id, lower = k.mnId, k
            elif k.mnId < second_id:
                second_id, second = k.mnId, k
        if lower is not None:
            fixed.append(lower)
            local.remove(lower)
            num_fixed += 1
        if num_fixed < 2 and second is not None:
            fixed.append(second)
            local.remove(second)
            num_fixed += 1
    if num_fixed == 0:
        return None
    return local, fixed, local_mps, num_fixed


def flatten_window(local, fixed, local_mps, pMap: Map):
    """slam_lba_problem arrays: KFs in vertex-id order, points in lLocalMapPoints order, edges
    point-major in observation order (Optimizer.cc:1737-1918)."""
    kfs = sorted(local + fixed, key=lambda k: k.mnId)
    kf_index = {id(k): i for i, k in enumerate(kfs)}
    fixed_ids = {id(k) for k in fixed}
    kf_fixed = np.array([2 if id(k) in fixed_ids else (1 if k.mnId == pMap.GetInitKFid() else 0) for k in kfs],
                        np.uint8)
    cur_map = local[0].GetMap() if local else None
    rig = any(k.mpCamera2 is not None for k in kfs)
    edge_pt, edge_kf, obs, isig, edge_refs, body = [], [], [], [], [], []
    for pi, mp in enumerate(local_mps):
        for k, (li, ri) in mp.GetObservations().items():
            if k.isBad() or k.GetMap() is not cur_map or id(k) not in kf_index:
                continue
            if li != -1:                                          # mono / stereo (:1819-1880)
                kp = k.mvKeysUn[li]
                ur = float(k.mvuRight[li])
                edge_pt.append(pi)
                edge_kf.append(kf_index[id(k)])
                obs.append((kp["x"], kp["y"], ur if ur >= 0 else -1.0))
                isig.append(k.mvInvLevelSigma2[kp["octave"]])
                edge_refs.append((k, mp))
                body.append(0)
            if k.mpCamera2 is not None and ri != -1:              # EdgeSE3ProjectXYZToBody (:1883-1914)
                kp = k.mvKeysRight[ri - k.NLeft]
                edge_pt.append(pi)
                edge_kf.append(kf_index[id(k)])
                obs.append((kp["x"], kp["y"], -1.0))
                isig.append(k.mvInvLevelSigma2[kp["octave"]])
                edge_refs.append((k, mp))
                body.append(1)
    k0 = kfs[0]
    W = dict(kf_Tcw=np.stack([k.GetPose().reshape(-1) for k in kfs]).astype(np.float32), kf_fixed=kf_fixed,
             pt_pos=np.stack([mp.GetWorldPos() for mp in local_mps]).astype(np.float32) if local_mps
             else np.zeros((0, 3), np.float32),
             edge_pt=np.array(edge_pt, np.int32), edge_kf=np.array(edge_kf, np.int32),
             edge_obs=np.array(obs, np.float32).reshape(-1, 3), edge_inv_sigma2=np.array(isig, np.float32),
             cam=(k0.fx, k0.fy, k0.cx, k0.cy, k0.mbf))
    if rig:
        eye = np.eye(4, dtype=np.float32)
        W["edge_body"] = np.array(body, np.uint8)
        W["kf_Trl"] = np.stack([(k.mTrl if k.mpCamera2 is not None else eye).reshape(-1) for k in kfs])
        c2 = next(k.mpCamera2 for k in kfs if k.mpCamera2 is not None)
        W["cam2"] = tuple(c2) + (np.float32(0),)
    return W, kfs, edge_refs


def LocalBundleAdjustment(pKF: KeyFrame, stop_flag, pMap: Map, solver):
    """Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap, num_fixedKF, num_OptKF, num_MPs,
    num_edges); returns those four counts (-1 counts when the reference returns early)."""
    win = build_window(pKF, pMap)
    if win is None:
        return None
    local, fixed, local_mps, num_fixed = win
    W, kfs, edge_refs = flatten_window(local, fixed, local_mps, pMap)
    counts = (num_fixed, len(local), len(local_mps), len(edge_refs))
    if stop_flag:                                                  # :1921-1923
        return counts
    live = stop_flag if isinstance(stop_flag, (C.c_bool, C.c_uint8, C.c_int32)) else None  # optimizer.setForceStopFlag
    res = solver.solve(W, user_lambda_init=100.0 if pMap.IsInertial() else 0.0, stop_flag=live)
    for e, bad in enumerate(res["edge_outlier"]):                  # :2043-2052
        if bad:
            k, mp = edge_refs[e]
            k.EraseMapPointMatch(mp)
            mp.EraseObservation(k)
    local_ids = {id(k) for k in local}
    for i, k in enumerate(kfs):                                    # :2056-2063
        if id(k) in local_ids:
            k.SetPose(res["kf_Tcw"][i].reshape(4, 4))
    for i, mp in enumerate(local_mps):                             # :2066-2074
        mp.SetWorldPos(res["pt_pos"][i])
        mp.UpdateNormalAndDepth()
    pMap.IncreaseChangeIndex()
    return counts


def map_from_window(W: dict, covis_order=None):
    """Build the map model of a synthetic window (slamhot.synth.lba_window): every KF observes
    its points, KeyFrame 0 is the map-init KF, the last KF is the current one and sees all the
    others as covisible.  Body edges (a rig window) become right-camera keypoints."""
    pmap = Map(init_kf_id=0)
    nk = len(W["kf_fixed"])
    cam = W["cam"]
    body = W.get("edge_body")
    per_kf = [[] for _ in range(nk)]
    per_kf_r = [[] for _ in range(nk)]
    for e in range(len(W["edge_pt"])):
        (per_kf_r if body is not None and body[e] else per_kf)[W["edge_kf"][e]].append(e)
    from .synth import _level_tables
    _, inv_sigma2, _ = _level_tables()
    kfs = []
    for k in range(nk):
        edges = per_kf[k]
        keys = np.zeros(len(edges), dtype=[("x", "<f4"), ("y", "<f4"), ("octave", "<i4")])
        ur = np.full(len(edges), -1.0, np.float32)
        for j, e in enumerate(edges):
            keys["x"][j], keys["y"][j] = W["edge_obs"][e][:2]
            lvl = int(np.argmin(np.abs(inv_sigma2 - W["edge_inv_sigma2"][e])))
            keys["octave"][j] = lvl
            ur[j] = W["edge_obs"][e][2]
        kf = KeyFrame(k, W["kf_Tcw"][k].reshape(4, 4), keys, ur, inv_sigma2, cam, pmap)
        if body is not None:
            kr = np.zeros(len(per_kf_r[k]), dtype=keys.dtype)
            for j, e in enumerate(per_kf_r[k]):
                kr["x"][j], kr["y"][j] = W["edge_obs"][e][:2]
                kr["octave"][j] = int(np.argmin(np.abs(inv_sigma2 - W["edge_inv_sigma2"][e])))
            kf.set_rig(kr, W["kf_Trl"][k], W["cam2"])
        kfs.append(kf)
    mps = [MapPoint(i, W["pt_pos"][i], pmap) for i in range(len(W["pt_pos"]))]
    for k in range(nk):
        for j, e in enumerate(per_kf[k]):
            mp = mps[W["edge_pt"][e]]
            kfs[k].mvpMapPoints[j] = mp
            mp.AddObservation(kfs[k], j)
        for j, e in enumerate(per_kf_r[k]):
            mp = mps[W["edge_pt"][e]]
            jr = kfs[k].NLeft + j
            kfs[k].mvpMapPoints[jr] = mp
            li, _ = mp.observations.get(kfs[k], (-1, -1))
            mp.AddObservation(kfs[k], li, jr)
    cur = kfs[-1]
    cur.covisible = covis_order if covis_order is not None else [kfs[i] for i in range(nk - 2, -1, -1)]
    return pmap, kfs, mps


def fuse_apply(pKF: KeyFrame, vpMapPoints, best_idx, best_dist, TH_LOW: int = 50) -> int:
    """ORBmatcher::Fuse's update half (ORBmatcher.cc:1789-1816) in list order, on the device
    search results (slamhot_fuse_search).  The skip checks are re-evaluated here because
    earlier updates of this call can make a later MapPoint bad or put it into pKF."""
    nFused = 0
    for i, pMP in enumerate(vpMapPoints):
        if pMP is None or pMP.isBad() or pMP.IsInKeyFrame(pKF):
            continue
        if best_dist[i] <= TH_LOW:
            idx = int(best_idx[i])
            pMPinKF = pKF.GetMapPoint(idx)
            if pMPinKF is not None:
                if not pMPinKF.isBad():
                    if pMPinKF.Observations() > pMP.Observations():
                        pMP.Replace(pMPinKF)
                    else:
                        pMPinKF.Replace(pMP)
            else:
                pMP.AddObservation(pKF, idx)
                pKF.AddMapPoint(pMP, idx)
            nFused += 1
    return nFused
