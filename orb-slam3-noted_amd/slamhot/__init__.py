"""Python host mirror of the ORB-SLAM3 hot path over the libslamhot C-ABI (include/slamhot.h).

The classes mirror the reference's operator interface: ``ORBextractor(nfeatures, scaleFactor,
nlevels, iniThFAST, minThFAST)`` with ``__call__(image, lapping) -> (keypoints, descriptors,
monoIndex)`` and the ``Get*`` accessors (ORBextractor.h:49-83).  Compute always runs in the
HIP library; there is no CPU fallback — a missing library or device raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = PKG_ROOT / "lib" / "libslamhot.so"

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

SLAM_OK, SLAM_EINVAL, SLAM_ENOMEM, SLAM_EHIP, SLAM_ECAP, SLAM_ENODEV, SLAM_EEMPTY, SLAM_ETIMEDOUT = 0, -1, -2, -3, -4, -5, -6, -7


class SlamError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {status_string(status)} ({status})")
        self.status = status


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class BowSide(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("angle", C.c_void_p), ("valid", C.c_void_p),
                ("n_nodes", C.c_int32), ("node_id", C.c_void_p), ("node_off", C.c_void_p),
                ("node_feat", C.c_void_p)]


def make_bow_side(desc, angle, valid, node_id, node_off, node_feat):
    """slam_bow_side over numpy arrays; returns (struct, keepalive list)."""
    arrs = [np.ascontiguousarray(desc, np.uint8), np.ascontiguousarray(angle, np.float32),
            None if valid is None else np.ascontiguousarray(valid, np.uint8),
            np.ascontiguousarray(node_id, np.uint32), np.ascontiguousarray(node_off, np.int32),
            np.ascontiguousarray(node_feat, np.uint32)]
    ptr = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    s = BowSide(len(arrs[0]), ptr(arrs[0]), ptr(arrs[1]), ptr(arrs[2]), len(arrs[3]), ptr(arrs[3]), ptr(arrs[4]),
                ptr(arrs[5]))
    return s, arrs


class FrameView(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps_un", C.c_void_p), ("uright", C.c_void_p), ("desc", C.c_void_p),
                ("mp_state", C.c_void_p), ("min_x", C.c_float), ("min_y", C.c_float), ("max_x", C.c_float),
                ("max_y", C.c_float), ("grid_inv_w", C.c_float), ("grid_inv_h", C.c_float),
                ("nlevels", C.c_int32), ("scale", C.c_void_p), ("log_scale", C.c_float), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float), ("b", C.c_float),
                ("Tcw", C.c_void_p)]


MP_GEOM_DTYPE = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("min_dist", "<f4"), ("max_dist", "<f4"),
                          ("seen", "u1"), ("is_bad", "u1"), ("has_obs", "u1"), ("pad", "u1")])
MP_TRACK_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("depth", "<f4"),
                           ("view_cos", "<f4"), ("scale_level", "<i4"), ("in_view", "u1"), ("is_bad", "u1"),
                           ("has_obs", "u1"), ("pad", "u1")])


class LastFrameView(C.Structure):
    _fields_ = [("n", C.c_int32), ("Tcw", C.c_void_p), ("kps", C.c_void_p), ("kps_un", C.c_void_p),
                ("has_mp", C.c_void_p), ("outlier", C.c_void_p), ("mp_pos", C.c_void_p), ("mp_desc", C.c_void_p),
                ("mp_has_obs", C.c_void_p)]


class KFPointsView(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps_un", C.c_void_p), ("use", C.c_void_p), ("mp_pos", C.c_void_p),
                ("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("mp_desc", C.c_void_p)]


def _keep(a, dt):
    return None if a is None else np.ascontiguousarray(a, dt)


def make_frame_view(kps_un, desc, uright=None, mp_state=None, width=752, height=480, scale=None,
                    scale_factor=1.2, cam=(435.2047, 435.2047, 367.4517, 252.2009), bf=47.9064, Tcw=None):
    """slam_frame_view for an undistorted pinhole frame (bounds 0..width/height,
    Frame::ComputeImageBounds with k1 = 0); returns (struct, keepalive)."""
    kps_un = np.ascontiguousarray(kps_un)
    assert kps_un.dtype == KP_DTYPE
    if scale is None:
        scale = [1.0]
        for _ in range(7):
            scale.append(float(np.float32(np.float64(np.float32(scale[-1])) * np.float64(np.float32(scale_factor)))))
    arrs = dict(kps=kps_un, desc=_keep(desc, np.uint8), uright=_keep(uright, np.float32),
                state=_keep(mp_state, np.int8), scale=np.ascontiguousarray(scale, np.float32),
                T=_keep(Tcw, np.float32))
    ptr = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    f32 = np.float32
    v = FrameView()
    v.n = len(kps_un)
    v.kps_un, v.uright, v.desc, v.mp_state = ptr(arrs["kps"]), ptr(arrs["uright"]), ptr(arrs["desc"]), ptr(arrs["state"])
    v.min_x, v.min_y, v.max_x, v.max_y = 0.0, 0.0, float(width), float(height)
    v.grid_inv_w = float(f32(64) / f32(width))
    v.grid_inv_h = float(f32(48) / f32(height))
    v.nlevels = len(scale)
    v.scale = ptr(arrs["scale"])
    v.log_scale = float(f32(np.log(np.float64(f32(scale_factor)))))  # logf (numpy's float32 log differs by an ulp)
    v.fx, v.fy, v.cx, v.cy = cam
    v.bf = bf
    v.b = float(f32(bf) / f32(cam[0]))
    v.Tcw = ptr(arrs["T"])
    return v, arrs


def make_last_frame(Tcw, kps, kps_un, has_mp, outlier, mp_pos, mp_desc, mp_has_obs):
    arrs = [np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(kps), np.ascontiguousarray(kps_un),
            np.ascontiguousarray(has_mp, np.uint8), np.ascontiguousarray(outlier, np.uint8),
            np.ascontiguousarray(mp_pos, np.float32), np.ascontiguousarray(mp_desc, np.uint8),
            np.ascontiguousarray(mp_has_obs, np.uint8)]
    p = [a.ctypes.data_as(C.c_void_p) for a in arrs]
    return LastFrameView(len(arrs[2]), *p), arrs


def make_kf_points(kps_un, use, mp_pos, max_dist, min_dist, mp_desc):
    arrs = [np.ascontiguousarray(kps_un), np.ascontiguousarray(use, np.uint8), np.ascontiguousarray(mp_pos, np.float32),
            np.ascontiguousarray(max_dist, np.float32), np.ascontiguousarray(min_dist, np.float32),
            np.ascontiguousarray(mp_desc, np.uint8)]
    p = [a.ctypes.data_as(C.c_void_p) for a in arrs]
    return KFPointsView(len(arrs[0]), *p), arrs


_lib = None
P = C.c_void_p
I = C.c_int


def lib() -> C.CDLL:
    """Load libslamhot.so (built in-tree by __graft_entry__.build()); raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("SLAMHOT_LIB", str(LIB_PATH)))  # experiment builds (tools/)
    if not path.exists():
        raise RuntimeError(f"libslamhot.so not built: {path} (run __graft_entry__.build())")
    L = C.CDLL(str(path))
    L.slamhot_version.restype = C.c_char_p
    L.slamhot_status_string.argtypes = [I]
    L.slamhot_status_string.restype = C.c_char_p
    L.slamhot_device_count.argtypes = [C.POINTER(I)]
    L.slamhot_extractor_create.argtypes = [C.POINTER(OrbParams), I, I, I, I, C.POINTER(P)]
    L.slamhot_extractor_destroy.argtypes = [P]
    L.slamhot_extractor_destroy.restype = None
    L.slamhot_extractor_levels.argtypes = [P, C.POINTER(I), P, P, P, P, P]
    L.slamhot_extract.argtypes = [P, P, I, I, C.c_size_t, I, I, P, P, I, C.POINTER(I), C.POINTER(I)]
    L.slamhot_extract_batch.argtypes = [P, I, P, I, I, C.c_size_t, I, I, P, P, I, P, P]
    L.slamhot_extract_batch_device.argtypes = [P, I, P, I, I, I, I, P, P, I, P, P, P]
    L.slamhot_pyramid_level.argtypes = [P, I, I, P, C.c_size_t, C.POINTER(I), C.POINTER(I)]
    L.slamhot_extractor_stream.argtypes = [P]
    L.slamhot_extractor_stream.restype = P
    L.slamhot_extractor_set_profiling.argtypes = [P, I]
    L.slamhot_extractor_num_stages.restype = I
    L.slamhot_extractor_stage_name.argtypes = [I]
    L.slamhot_extractor_stage_name.restype = C.c_char_p
    L.slamhot_extractor_stage_stats.argtypes = [P, P, P, I]
    L.slamhot_vocab_create.argtypes = [I, I, I, I, I, I, P, P, P, P, C.POINTER(P)]
    L.slamhot_vocab_load_text.argtypes = [I, C.c_char_p, C.POINTER(P)]
    L.slamhot_vocab_destroy.argtypes = [P]
    L.slamhot_vocab_destroy.restype = None
    L.slamhot_vocab_info.argtypes = [P, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]
    L.slamhot_vocab_transform.argtypes = [P, I, P, I, P, P, P]
    L.slamhot_vocab_transform_device.argtypes = [P, I, P, I, I, P, P, P, P]
    L.slamhot_matcher_create.argtypes = [I, C.POINTER(P)]
    L.slamhot_matcher_destroy.argtypes = [P]
    L.slamhot_matcher_destroy.restype = None
    L.slamhot_matcher_last_batch_stats.argtypes = [P, P, P]
    L.slamhot_search_by_bow.argtypes = [P, C.POINTER(BowSide), C.POINTER(BowSide), C.c_float, I, I, P, P,
                                        C.POINTER(I)]
    L.slamhot_search_by_projection_local.argtypes = [P, C.POINTER(FrameView), I, P, P, C.c_float, C.c_float, I,
                                                     C.c_float, P, C.POINTER(I)]
    L.slamhot_search_by_projection_last.argtypes = [P, C.POINTER(FrameView), C.POINTER(LastFrameView), C.c_float, I,
                                                    C.c_float, I, P, C.POINTER(I)]
    L.slamhot_search_by_projection_kf.argtypes = [P, C.POINTER(FrameView), C.POINTER(KFPointsView), C.c_float, I,
                                                  C.c_float, I, P, C.POINTER(I)]
    _lib = L
    return L


def status_string(st: int) -> str:
    return lib().slamhot_status_string(st).decode()


def check(st: int, what: str) -> int:
    if st < 0:
        raise SlamError(st, what)
    return st


def device_count() -> int:
    n = I(0)
    check(lib().slamhot_device_count(C.byref(n)), "device_count")
    return n.value


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(P)


class ORBextractor:
    """Mirror of ORB_SLAM3::ORBextractor (ORBextractor.h:44-110) on one gfx950 device."""

    def __init__(self, nfeatures: int = 1000, scaleFactor: float = 1.2, nlevels: int = 8,
                 iniThFAST: int = 20, minThFAST: int = 7, device: int = 0,
                 max_size=(1280, 720), max_batch: int = 1):
        self.params = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self.nlevels = nlevels
        self._h = P()
        check(lib().slamhot_extractor_create(C.byref(self.params), device, max_size[0], max_size[1],
                                             max_batch, C.byref(self._h)), "slamhot_extractor_create")
        self.cap = nfeatures * 2 + 64

    def close(self):
        if self._h:
            lib().slamhot_extractor_destroy(self._h)
            self._h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _levels(self):
        L = self.nlevels
        out = [np.zeros(L, np.float32) for _ in range(4)] + [np.zeros(L, np.int32)]
        n = I(0)
        check(lib().slamhot_extractor_levels(self._h, C.byref(n), *[_ptr(a) for a in out]), "levels")
        return out

    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return float(np.float32(self.params.scale_factor))

    def GetScaleFactors(self):
        return self._levels()[0]

    def GetInverseScaleFactors(self):
        return self._levels()[1]

    def GetScaleSigmaSquares(self):
        return self._levels()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._levels()[3]

    def GetFeaturesPerLevel(self):
        return self._levels()[4]

    def __call__(self, image: np.ndarray, vLappingArea=(0, 0)):
        """operator()(image, mask, keypoints, descriptors, vLappingArea) -> monoIndex.

        Returns (keypoints structured array in cv::KeyPoint layout, descriptors N x 32 u8,
        monoIndex)."""
        kps, desc, n, mono = self.extract_batch(image[None], vLappingArea)
        return kps[0][: n[0]].copy(), desc[0][: n[0]].copy(), int(mono[0])

    def extract_batch(self, images: np.ndarray, vLappingArea=(0, 0)):
        images = np.ascontiguousarray(images, dtype=np.uint8)
        nf, h, w = images.shape
        cap = self.cap
        kps = np.zeros((nf, cap), KP_DTYPE)
        desc = np.zeros((nf, cap, 32), np.uint8)
        n = np.zeros(nf, np.int32)
        mono = np.zeros(nf, np.int32)
        st = lib().slamhot_extract_batch(self._h, nf, _ptr(images), w, h, w, int(vLappingArea[0]),
                                         int(vLappingArea[1]), _ptr(kps), _ptr(desc), cap, _ptr(n), _ptr(mono))
        check(st, "slamhot_extract_batch")
        return kps, desc, n, mono

    def pyramid_level(self, level: int, frame: int = 0) -> np.ndarray:
        w, h = I(0), I(0)
        check(lib().slamhot_pyramid_level(self._h, frame, level, None, 0, C.byref(w), C.byref(h)), "pyramid")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().slamhot_pyramid_level(self._h, frame, level, _ptr(out), out.size, C.byref(w), C.byref(h)),
              "pyramid")
        return out

    @property
    def mvImagePyramid(self):
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def extract_batch_device(self, d_imgs: int, nframes: int, width: int, height: int, d_kps: int, d_desc: int,
                             cap: int, d_n: int, d_mono: int, lap=(0, 0), stream: int | None = None):
        """Device-resident batch: all pointers are device addresses (ints)."""
        st = lib().slamhot_extract_batch_device(self._h, nframes, P(d_imgs), width, height, int(lap[0]), int(lap[1]),
                                                P(d_kps), P(d_desc), cap, P(d_n), P(d_mono),
                                                P(stream) if stream else None)
        check(st, "slamhot_extract_batch_device")

    def stream(self) -> int:
        return lib().slamhot_extractor_stream(self._h) or 0

    def set_profiling(self, enable: bool):
        check(lib().slamhot_extractor_set_profiling(self._h, 1 if enable else 0), "set_profiling")

    def stage_stats(self, reset: bool = False):
        """{stage name: (total ms, launches)} accumulated while profiling was on."""
        L = lib()
        ns = L.slamhot_extractor_num_stages()
        ms = np.zeros(ns, np.float64)
        cnt = np.zeros(ns, np.int64)
        check(L.slamhot_extractor_stage_stats(self._h, _ptr(ms), _ptr(cnt), 1 if reset else 0), "stage_stats")
        return {L.slamhot_extractor_stage_name(i).decode(): (float(ms[i]), int(cnt[i])) for i in range(ns)}


class Vocabulary:
    """ORBVocabulary (DBoW2 TemplatedVocabulary<FORB>) resident on one gfx950 device."""

    def __init__(self, parent=None, is_leaf=None, desc=None, weight=None, k=10, L=6, scoring=0, weighting=0,
                 path: str | None = None, device: int = 0):
        self._h = P()
        if path is not None:
            check(lib().slamhot_vocab_load_text(device, path.encode(), C.byref(self._h)), "vocab_load_text")
        else:
            parent = np.ascontiguousarray(parent, np.int32)
            is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
            desc = np.ascontiguousarray(desc, np.uint8)
            weight = np.ascontiguousarray(weight, np.float64)
            check(lib().slamhot_vocab_create(device, k, L, scoring, weighting, len(parent), _ptr(parent),
                                             _ptr(is_leaf), _ptr(desc), _ptr(weight), C.byref(self._h)),
                  "vocab_create")
        k_, L_, nn, nw = I(0), I(0), I(0), I(0)
        check(lib().slamhot_vocab_info(self._h, C.byref(k_), C.byref(L_), C.byref(nn), C.byref(nw)), "vocab_info")
        self.k, self.L, self.n_nodes, self.n_words = k_.value, L_.value, nn.value, nw.value

    def close(self):
        if self._h:
            lib().slamhot_vocab_destroy(self._h)
            self._h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """Per-feature (word id, word weight, node id at level L-levelsup)."""
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        w = np.zeros(n, np.int32)
        wt = np.zeros(n, np.float64)
        nid = np.zeros(n, np.int32)
        check(lib().slamhot_vocab_transform(self._h, n, _ptr(desc), levelsup, _ptr(w), _ptr(wt), _ptr(nid)),
              "vocab_transform")
        return w, wt, nid


class ORBmatcher:
    """Mirror of ORB_SLAM3::ORBmatcher(nnratio, checkOri) (ORBmatcher.h:39-91), pinhole."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri
        self._h = P()
        check(lib().slamhot_matcher_create(device, C.byref(self._h)), "matcher_create")

    def close(self):
        if self._h:
            lib().slamhot_matcher_destroy(self._h)
            self._h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_batch_stats(self):
        """(kernel_ms, span_ms) of the last batched host-buffer call (slamhot_matcher_last_batch_stats)."""
        k, sp = C.c_float(0), C.c_float(0)
        check(lib().slamhot_matcher_last_batch_stats(self._h, C.byref(k), C.byref(sp)), "matcher_last_batch_stats")
        return k.value, sp.value

    def _bow(self, A, B, strict):
        sa, ka = make_bow_side(*A)
        sb, kb = make_bow_side(*B)
        a2b = np.full(sa.n, -1, np.int32)
        b2a = np.full(sb.n, -1, np.int32)
        nm = I(0)
        check(lib().slamhot_search_by_bow(self._h, C.byref(sa), C.byref(sb), self.mfNNratio,
                                          1 if self.mbCheckOrientation else 0, strict, _ptr(a2b), _ptr(b2a),
                                          C.byref(nm)), "search_by_bow")
        return nm.value, a2b, b2a

    def SearchByBoW_KF_F(self, kf, frame):
        """int SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&): kf / frame are tuples
        (desc, angle, valid, node_id, node_off, node_feat); returns (nmatches, per-frame-feature
        matched KF feature index or -1)."""
        n, a2b, b2a = self._bow(kf, frame, 0)
        return n, b2a

    def SearchByBoW_KF_KF(self, kf1, kf2):
        """int SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&): returns (nmatches,
        per-KF1-feature matched KF2 feature index or -1)."""
        n, a2b, b2a = self._bow(kf1, kf2, 1)
        return n, a2b


def _matcher_methods():
    def SearchByProjection_local(self, frame_view, mps, mp_desc, th=3.0, bFarPoints=False, thFarPoints=50.0):
        """int SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)."""
        mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
        fm = np.full(frame_view.n, -1, np.int32)
        nm = I(0)
        check(lib().slamhot_search_by_projection_local(self._h, C.byref(frame_view), len(mps), _ptr(mps),
                                                       _ptr(mp_desc), self.mfNNratio, th, int(bFarPoints),
                                                       thFarPoints, _ptr(fm), C.byref(nm)), "search_by_projection_local")
        return nm.value, fm

    def SearchLocalPoints(self, frame_view, mps, mp_desc, th=1.0, bFarPoints=False, thFarPoints=50.0,
                          viewingCosLimit=0.5):
        """Tracking::SearchLocalPoints (isInFrustum + SearchByProjection) on the device.
        mps: MP_GEOM_DTYPE array.  Returns (nmatches, f_match, nToMatch, track)."""
        L = lib()
        if not getattr(L, "_slp_ready", False):
            L.slamhot_search_local_points.argtypes = [P, C.POINTER(FrameView), I, P, P, C.c_float, C.c_float,
                                                      C.c_float, I, C.c_float, P, C.POINTER(I), P, C.POINTER(I)]
            L._slp_ready = True
        mps = np.ascontiguousarray(mps, MP_GEOM_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
        fm = np.full(frame_view.n, -1, np.int32)
        tr = np.zeros(len(mps), MP_TRACK_DTYPE)
        nm, nt = I(0), I(0)
        check(L.slamhot_search_local_points(self._h, C.byref(frame_view), len(mps), _ptr(mps), _ptr(mp_desc),
                                            viewingCosLimit, self.mfNNratio, th, int(bFarPoints), thFarPoints,
                                            _ptr(tr), C.byref(nt), _ptr(fm), C.byref(nm)), "search_local_points")
        return nm.value, fm, nt.value, tr

    def SearchLocalPoints_batch(self, frame_views, mps_list, desc_list, th=1.0, bFarPoints=False, thFarPoints=50.0,
                                viewingCosLimit=0.5):
        """Batched Tracking::SearchLocalPoints (slamhot_search_local_points_batch): lists of frame
        views / MP_GEOM arrays / descriptors.  Returns [(nmatches, f_match, nToMatch)] per frame."""
        L = lib()
        if not getattr(L, "_slpb_ready", False):
            L.slamhot_search_local_points_batch.argtypes = [P, I, P, P, P, P, C.c_float, C.c_float, C.c_float, I,
                                                            C.c_float, P, P, P]
            L._slpb_ready = True
        nf = len(frame_views)
        fv = (FrameView * nf)(*frame_views)
        mps = [np.ascontiguousarray(m, MP_GEOM_DTYPE) for m in mps_list]
        dsc = [np.ascontiguousarray(d, np.uint8) for d in desc_list]
        fms = [np.full(v.n, -1, np.int32) for v in frame_views]
        nmp = np.array([len(m) for m in mps], np.int32)
        pm = (P * nf)(*[m.ctypes.data for m in mps])
        pd = (P * nf)(*[d.ctypes.data for d in dsc])
        pf = (P * nf)(*[f.ctypes.data for f in fms])
        nt = np.zeros(nf, np.int32)
        nm = np.zeros(nf, np.int32)
        check(L.slamhot_search_local_points_batch(self._h, nf, fv, _ptr(nmp), pm, pd, viewingCosLimit, self.mfNNratio,
                                                  th, int(bFarPoints), thFarPoints, pf, _ptr(nt), _ptr(nm)),
              "search_local_points_batch")
        return [(int(nm[i]), fms[i], int(nt[i])) for i in range(nf)]

    def SearchByProjection_last(self, frame_view, last_view, th, bMono):
        """int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)."""
        fm = np.full(frame_view.n, -1, np.int32)
        nm = I(0)
        check(lib().slamhot_search_by_projection_last(self._h, C.byref(frame_view), C.byref(last_view),
                                                      self.mfNNratio, int(self.mbCheckOrientation), th, int(bMono),
                                                      _ptr(fm), C.byref(nm)), "search_by_projection_last")
        return nm.value, fm

    def SearchByProjection_kf(self, frame_view, kf_view, th, ORBdist):
        """int SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)."""
        fm = np.full(frame_view.n, -1, np.int32)
        nm = I(0)
        check(lib().slamhot_search_by_projection_kf(self._h, C.byref(frame_view), C.byref(kf_view), self.mfNNratio,
                                                    int(self.mbCheckOrientation), th, int(ORBdist), _ptr(fm),
                                                    C.byref(nm)), "search_by_projection_kf")
        return nm.value, fm

    def _proj_batch(self, fn_name, frame_views, others, other_cls, *args):
        L = lib()
        fn = getattr(L, fn_name)
        if not getattr(fn, "_ready", False):
            fn.argtypes = [P, I, P, P, C.c_float, I, C.c_float, I, P, P]
            fn._ready = True
        nf = len(frame_views)
        fv = (FrameView * nf)(*frame_views)
        ov = (other_cls * nf)(*others)
        fms = [np.full(v.n, -1, np.int32) for v in frame_views]
        pf = (P * nf)(*[f.ctypes.data for f in fms])
        nm = np.zeros(nf, np.int32)
        check(fn(self._h, nf, fv, ov, self.mfNNratio, int(self.mbCheckOrientation), *args, pf, _ptr(nm)), fn_name)
        return [(int(nm[i]), fms[i]) for i in range(nf)]

    def prepare_batch(self, kind, frame_views, others, *args):
        """The batched host-buffer call with its arguments marshalled once (what a C++ caller
        already holds): returns run() -> total matches, which makes only the C call;
        run.results() gives [(nmatches, f_match[, nToMatch])].  kind: "last" (others = last-frame
        views, args = th, bMono), "kf" (KeyFrame views, th, ORBdist) or "local" (others = (MP_GEOM
        arrays, descriptor arrays), args = th, bFarPoints, thFarPoints, viewingCosLimit)."""
        L = lib()
        nf = len(frame_views)
        fv = (FrameView * nf)(*frame_views)
        fms = [np.full(v.n, -1, np.int32) for v in frame_views]
        pf = (P * nf)(*[f.ctypes.data for f in fms])
        nm = np.zeros(nf, np.int32)
        h = self._h
        if kind == "local":
            self.SearchLocalPoints_batch(frame_views[:1], others[0][:1], others[1][:1])  # binds argtypes
            mps = [np.ascontiguousarray(m, MP_GEOM_DTYPE) for m in others[0]]
            dsc = [np.ascontiguousarray(d, np.uint8) for d in others[1]]
            nmp = np.array([len(m) for m in mps], np.int32)
            pm = (P * nf)(*[m.ctypes.data for m in mps])
            pd = (P * nf)(*[d.ctypes.data for d in dsc])
            nt = np.zeros(nf, np.int32)
            th, far, thf, vc = (list(args) + [1.0, False, 50.0, 0.5][len(args):])[:4]
            fn = L.slamhot_search_local_points_batch
            call = lambda: fn(h, nf, fv, _ptr(nmp), pm, pd, vc, self.mfNNratio, th, int(far), thf, pf, _ptr(nt),  # noqa: E731
                              _ptr(nm))
            keep = (mps, dsc, nmp, pm, pd, nt)
            results = lambda: [(int(nm[i]), fms[i], int(nt[i])) for i in range(nf)]  # noqa: E731
        else:
            fn_name, cls = (("slamhot_search_by_projection_last_batch", LastFrameView) if kind == "last" else
                            ("slamhot_search_by_projection_kf_batch", KFPointsView))
            fn = getattr(L, fn_name)
            if not getattr(fn, "_ready", False):
                fn.argtypes = [P, I, P, P, C.c_float, I, C.c_float, I, P, P]
                fn._ready = True
            ov = (cls * nf)(*others)
            a0, a1 = float(args[0]), int(args[1])
            call = lambda: fn(h, nf, fv, ov, self.mfNNratio, int(self.mbCheckOrientation), a0, a1, pf, _ptr(nm))  # noqa: E731
            keep = (ov,)
            results = lambda: [(int(nm[i]), fms[i]) for i in range(nf)]  # noqa: E731

        def run():
            check(call(), "matcher batch")
            return int(nm.sum())

        run.keep = (fv, fms, pf, nm, keep)
        run.results = results
        return run

    def SearchByProjection_last_batch(self, frame_views, last_views, th, bMono):
        """Batched SearchByProjection(Frame&, const Frame& LastFrame, th, bMono)
        (slamhot_search_by_projection_last_batch): [(nmatches, f_match)] per frame."""
        return self._proj_batch("slamhot_search_by_projection_last_batch", frame_views, last_views, LastFrameView,
                                float(th), int(bMono))

    def SearchByProjection_kf_batch(self, frame_views, kf_views, th, ORBdist):
        """Batched SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)
        (slamhot_search_by_projection_kf_batch): [(nmatches, f_match)] per frame."""
        return self._proj_batch("slamhot_search_by_projection_kf_batch", frame_views, kf_views, KFPointsView,
                                float(th), int(ORBdist))

    def bow_match_batch_device(self, vocab, nframes, d_kps, d_desc, cap, d_n, pairs, d_a2b, d_b2a, d_nmatches,
                               d_valid=None, levelsup=4, strict=False, stream=None):
        """Device-resident Frame::ComputeBoW + SearchByBoW over (keyframe, frame) index pairs
        (slamhot_bow_match_batch_device); asynchronous on `stream`."""
        L = lib()
        if not getattr(L, "_bowb_ready", False):
            L.slamhot_bow_match_batch_device.argtypes = [P, P, I, P, P, I, P, P, I, P, C.c_float, I, I, I, P, P, P, P]
            L.slamhot_bow_match_batch_status.argtypes = [P, P, C.POINTER(I)]
            L._bowb_ready = True
        pr = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
        check(L.slamhot_bow_match_batch_device(self._h, vocab._h, nframes, P(d_kps), P(d_desc), cap, P(d_n),
                                               P(d_valid) if d_valid else None, len(pr), _ptr(pr), self.mfNNratio,
                                               int(self.mbCheckOrientation), int(strict), levelsup, P(d_a2b),
                                               P(d_b2a), P(d_nmatches), P(stream) if stream else None),
              "bow_match_batch_device")

    def bow_match_batch_status(self, stream=None) -> int:
        sk = I(0)
        check(lib().slamhot_bow_match_batch_status(self._h, P(stream) if stream else None, C.byref(sk)),
              "bow_match_batch_status")
        return sk.value

    ORBmatcher.bow_match_batch_device = bow_match_batch_device
    ORBmatcher.bow_match_batch_status = bow_match_batch_status
    ORBmatcher.SearchByProjection_local = SearchByProjection_local
    ORBmatcher.SearchLocalPoints = SearchLocalPoints
    ORBmatcher.SearchLocalPoints_batch = SearchLocalPoints_batch
    ORBmatcher.SearchByProjection_last = SearchByProjection_last
    ORBmatcher.prepare_batch = prepare_batch
    ORBmatcher.SearchByProjection_kf = SearchByProjection_kf
    ORBmatcher._proj_batch = _proj_batch
    ORBmatcher.SearchByProjection_last_batch = SearchByProjection_last_batch
    ORBmatcher.SearchByProjection_kf_batch = SearchByProjection_kf_batch


_matcher_methods()


# ------------------------------------------------------------------------------------------
# Local bundle adjustment (Optimizer::LocalBundleAdjustment, Optimizer.cc:1611-2078)
# ------------------------------------------------------------------------------------------
class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float)]


class LbaProblem(C.Structure):
    _fields_ = [("n_kf", C.c_int32), ("kf_Tcw", C.c_void_p), ("kf_fixed", C.c_void_p), ("n_pt", C.c_int32),
                ("pt_pos", C.c_void_p), ("n_edge", C.c_int32), ("edge_pt", C.c_void_p), ("edge_kf", C.c_void_p),
                ("edge_obs", C.c_void_p), ("edge_inv_sigma2", C.c_void_p), ("cam", Camera),
                ("user_lambda_init", C.c_double), ("edge_body", C.c_void_p), ("kf_Trl", C.c_void_p),
                ("cam2", Camera), ("kf_cam", C.c_void_p), ("kf_cam2", C.c_void_p)]


class LbaOptions(C.Structure):
    _fields_ = [("iters_first", C.c_int32), ("iters_second", C.c_int32), ("user_lambda_init", C.c_double),
                ("stop_flag_bool", C.c_void_p), ("step_hook", C.c_void_p), ("step_hook_ctx", C.c_void_p)]


class LbaResult(C.Structure):
    _fields_ = [("kf_Tcw", C.c_void_p), ("pt_pos", C.c_void_p), ("edge_outlier", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("trials", C.c_int32), ("n_outlier", C.c_int32),
                ("chi2_initial", C.c_double), ("chi2_final", C.c_double), ("lambda_final", C.c_double),
                ("ran", C.c_int32)]


_LBA_KEYS = {"kf_Tcw": np.float32, "kf_fixed": np.uint8, "pt_pos": np.float32, "edge_pt": np.int32,
             "edge_kf": np.int32, "edge_obs": np.float32, "edge_inv_sigma2": np.float32}


def make_lba_problem(w: dict):
    """slam_lba_problem over a window dict (see synth.lba_window).  Returns (problem, result,
    outputs) where outputs holds the numpy arrays the result points into."""
    arrs = {k: np.ascontiguousarray(w[k], dt) for k, dt in _LBA_KEYS.items()}
    n_kf, n_pt, n_e = len(arrs["kf_fixed"]), len(arrs["pt_pos"]), len(arrs["edge_pt"])
    p = LbaProblem(n_kf, arrs["kf_Tcw"].ctypes.data, arrs["kf_fixed"].ctypes.data, n_pt,
                   arrs["pt_pos"].ctypes.data, n_e, arrs["edge_pt"].ctypes.data, arrs["edge_kf"].ctypes.data,
                   arrs["edge_obs"].ctypes.data, arrs["edge_inv_sigma2"].ctypes.data, Camera(*w["cam"]),
                   float(w.get("user_lambda_init", 0.0)))
    if w.get("edge_body") is not None:  # EdgeSE3ProjectXYZToBody observations (mpCamera2)
        arrs["edge_body"] = np.ascontiguousarray(w["edge_body"], np.uint8)
        arrs["kf_Trl"] = np.ascontiguousarray(w["kf_Trl"], np.float32)
        p.edge_body = arrs["edge_body"].ctypes.data
        p.kf_Trl = arrs["kf_Trl"].ctypes.data
        p.cam2 = Camera(*w["cam2"])
    for key in ("kf_cam", "kf_cam2"):  # a camera per KeyFrame (n_kf x 5: fx, fy, cx, cy, bf)
        if w.get(key) is not None:
            c = np.zeros((n_kf, 5), np.float32)
            v = np.asarray(w[key], np.float32).reshape(n_kf, -1)
            c[:, :v.shape[1]] = v
            arrs[key] = c
            setattr(p, key, c.ctypes.data)
    p._keep = arrs
    out = dict(kf_Tcw=np.zeros((n_kf, 16), np.float32), pt_pos=np.zeros((n_pt, 3), np.float32),
               edge_outlier=np.zeros(n_e, np.uint8))
    r = LbaResult(out["kf_Tcw"].ctypes.data, out["pt_pos"].ctypes.data, out["edge_outlier"].ctypes.data)
    r._keep = out
    return p, r, out


def lba_result_dict(r: LbaResult, out: dict) -> dict:
    d = dict(out)
    d.update(iterations=tuple(r.iterations), trials=r.trials, n_outlier=r.n_outlier,
             chi2_initial=r.chi2_initial, chi2_final=r.chi2_final, lambda_final=r.lambda_final, ran=r.ran)
    return d


class LocalBundleAdjustment:
    """Device LM/Schur solver behind ``slamhot_lba_solve`` — the numeric core of
    ``Optimizer::LocalBundleAdjustment`` (Optimizer.h:59).  ``solve`` takes one window dict or
    a list of them (batched mode) and returns result dicts."""

    def __init__(self, device: int = 0):
        L = lib()
        _bind_lba(L)
        h = P()
        check(L.slamhot_lba_create(device, C.byref(h)), "lba_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().slamhot_lba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, windows, iters_first=5, iters_second=10, user_lambda_init=0.0, stop_flag=None):
        """``stop_flag``: None, a truthy/falsy value (read once), or a live ``ctypes.c_int32`` /
        ``ctypes.c_bool`` that another thread may set while the call runs (``pbStopFlag``); the
        device LM loop reads it at every iteration start and trial end, as g2o's terminate()."""
        single = isinstance(windows, dict)
        ws = [windows] if single else list(windows)
        probs = (LbaProblem * len(ws))()
        ress = (LbaResult * len(ws))()
        outs = []
        for i, w in enumerate(ws):
            p, r, o = make_lba_problem(w)
            probs[i] = p
            ress[i] = r
            outs.append((p, r, o))
        opt = LbaOptions(iters_first, iters_second, user_lambda_init)
        stop = None
        if isinstance(stop_flag, C.c_int32):      # live flag another thread may set mid-solve
            stop = C.byref(stop_flag)
        elif isinstance(stop_flag, (C.c_bool, C.c_uint8)):  # the reference's bool* pbStopFlag
            opt.stop_flag_bool = C.addressof(stop_flag)
        elif stop_flag is not None:
            stop = C.byref(C.c_int32(int(stop_flag)))
        check(lib().slamhot_lba_solve(self._h, len(ws), probs, C.byref(opt), stop, ress), "lba_solve")
        res = [lba_result_dict(ress[i], outs[i][2]) for i in range(len(ws))]
        return res[0] if single else res

    def prepare(self, windows, iters_first=5, iters_second=10, user_lambda_init=0.0, stop_flag=None):
        """Flatten windows into C structs once (what a C++ caller already holds); returns a
        callable that runs slamhot_lba_solve on them and returns the LM iteration total
        (``run.results()`` gives the result dicts).  ``stop_flag``: a live ``ctypes.c_bool``;
        ``run(stop_at_step=k)`` clears it, then sets it from the solver's step hook once step k's
        counters are in (slam_lba_options.step_hook): another thread's abort at a known point; the
        solve stops within the steps already queued behind k (at most 3)."""
        ws = list(windows)
        probs = (LbaProblem * len(ws))()
        ress = (LbaResult * len(ws))()
        keep = []
        for i, w in enumerate(ws):
            p, r, o = make_lba_problem(w)
            probs[i] = p
            ress[i] = r
            keep.append((p, r, o))
        opt = LbaOptions(iters_first, iters_second, user_lambda_init)
        if stop_flag is not None:
            opt.stop_flag_bool = C.addressof(stop_flag)
        h = self._h
        fn = lib().slamhot_lba_solve

        state = dict(stop_at=-1, steps=0)

        def hook(_ctx, step):
            state["steps"] = step + 1
            if step == state["stop_at"]:
                stop_flag.value = True

        hook_c = _STEP_HOOK(hook)

        def run(stop_at_step=None):
            if stop_at_step is not None and stop_flag is None:
                raise ValueError("run(stop_at_step=...) needs prepare(..., stop_flag=ctypes.c_bool())")
            if stop_flag is not None and stop_at_step is not None:
                stop_flag.value = False  # a flag left set by the last run would stop this one on entry
            state["stop_at"] = -1 if stop_at_step is None else int(stop_at_step)
            opt.step_hook = C.cast(hook_c, C.c_void_p) if stop_at_step is not None or stop_flag is not None else None
            check(fn(h, len(ws), probs, C.byref(opt), None, ress), "lba_solve")
            return sum(ress[i].iterations[0] + ress[i].iterations[1] for i in range(len(ws)))

        run.keep = (probs, ress, keep, opt, stop_flag, hook_c)
        run.steps = lambda: state["steps"]  # LM steps the host saw in the last call
        run.results = lambda: [lba_result_dict(ress[i], keep[i][2]) for i in range(len(ws))]
        return run

    def warmup(self, n_kf=50, n_pt=2000, obs_per_pt=8):
        """slamhot_lba_warmup: one synthetic window of that size (kernels loaded, buffers sized)."""
        check(lib().slamhot_lba_warmup(self._h, n_kf, n_pt, obs_per_pt), "lba_warmup")

    def last_stats(self):
        """(device_ms, plan_ms, syncs) of the last solve."""
        ms, plan, syncs = C.c_double(0), C.c_double(0), I(0)
        check(lib().slamhot_lba_last_stats(self._h, C.byref(ms), C.byref(plan), C.byref(syncs)), "lba_last_stats")
        return ms.value, plan.value, syncs.value


_STEP_HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_int32)


def _bind_lba(L):
    if getattr(L, "_lba_ready", False):
        return
    L.slamhot_lba_create.argtypes = [I, C.POINTER(P)]
    L.slamhot_lba_destroy.argtypes = [P]
    L.slamhot_lba_destroy.restype = None
    L.slamhot_lba_solve.argtypes = [P, I, C.POINTER(LbaProblem), C.POINTER(LbaOptions), P, C.POINTER(LbaResult)]
    L.slamhot_lba_last_stats.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(I)]
    L.slamhot_lba_warmup.argtypes = [P, I, I, I]
    L._lba_ready = True


# ------------------------------------------------------------------------------------------
# Motion-only BA (Optimizer::PoseOptimization, Optimizer.cc:824-1118)
# ------------------------------------------------------------------------------------------
class PoseFrame(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("n", C.c_int32), ("kps_un", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("mp_pos", C.c_void_p), ("inv_sigma2", C.c_void_p), ("nlevels", C.c_int32),
                ("cam", Camera)]


class PoseResult(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("outlier", C.c_void_p), ("n_initial", C.c_int32),
                ("n_inliers", C.c_int32)]


def make_pose_frame(f: dict):
    arrs = dict(kps=np.ascontiguousarray(f["kps"], KP_DTYPE), uright=np.ascontiguousarray(f["uright"], np.float32),
                has_mp=np.ascontiguousarray(f["has_mp"], np.uint8), mp_pos=np.ascontiguousarray(f["mp_pos"], np.float32),
                inv_sigma2=np.ascontiguousarray(f["inv_sigma2"], np.float32))
    T = np.ascontiguousarray(f["Tcw"], np.float32).reshape(-1)
    pf = PoseFrame((C.c_float * 16)(*T.tolist()), len(arrs["kps"]), arrs["kps"].ctypes.data,
                   arrs["uright"].ctypes.data, arrs["has_mp"].ctypes.data, arrs["mp_pos"].ctypes.data,
                   arrs["inv_sigma2"].ctypes.data, len(arrs["inv_sigma2"]), Camera(*f["cam"]))
    pf._keep = arrs
    out = np.zeros(len(arrs["kps"]), np.uint8)
    r = PoseResult((C.c_float * 16)(), out.ctypes.data, 0, 0)
    r._keep = out
    return pf, r, out


def pose_result_dict(r: PoseResult, out) -> dict:
    return dict(Tcw=np.array(r.Tcw[:], np.float32).reshape(4, 4), outlier=out.copy(), n_initial=r.n_initial,
                n_inliers=r.n_inliers)


class PoseOptimizer:
    """Device Optimizer::PoseOptimization (slamhot_pose_optimization); `solve` takes one frame
    dict or a list (batched: one workgroup per frame)."""

    def __init__(self, device: int = 0):
        L = lib()
        if not getattr(L, "_pose_ready", False):
            L.slamhot_pose_opt_create.argtypes = [I, C.POINTER(P)]
            L.slamhot_pose_opt_destroy.argtypes = [P]
            L.slamhot_pose_opt_destroy.restype = None
            L.slamhot_pose_optimization.argtypes = [P, I, C.POINTER(PoseFrame), C.POINTER(PoseResult)]
            L._pose_ready = True
        h = P()
        check(L.slamhot_pose_opt_create(device, C.byref(h)), "pose_opt_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().slamhot_pose_opt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, frames):
        single = isinstance(frames, dict)
        fs = [frames] if single else list(frames)
        pfs = (PoseFrame * len(fs))()
        rs = (PoseResult * len(fs))()
        keep = []
        for i, f in enumerate(fs):
            pf, r, out = make_pose_frame(f)
            pfs[i] = pf
            rs[i] = r
            keep.append((pf, r, out))
        check(lib().slamhot_pose_optimization(self._h, len(fs), pfs, rs), "pose_optimization")
        res = [pose_result_dict(rs[i], keep[i][2]) for i in range(len(fs))]
        return res[0] if single else res

    def prepare(self, frames):
        """Marshal `frames` into the C structs once, as a C++ Tracking caller holds them: returns
        run() doing only the slamhot_pose_optimization call (host buffers in and out), with
        run.results() -> the result dicts of the last run."""
        fs = list(frames)
        pfs = (PoseFrame * len(fs))()
        rs = (PoseResult * len(fs))()
        keep = []
        for i, f in enumerate(fs):
            pf, r, out = make_pose_frame(f)
            pfs[i] = pf
            rs[i] = r
            keep.append((pf, r, out))
        h = self._h

        def run():
            check(lib().slamhot_pose_optimization(h, len(fs), pfs, rs), "pose_optimization")

        run.results = lambda: [pose_result_dict(rs[i], keep[i][2]) for i in range(len(fs))]
        run._keep = (pfs, rs, keep)
        return run


# ------------------------------------------------------------------ stereo matching
class StereoMatcher:
    """Device Frame::ComputeStereoMatches (Frame.cc:794-964) over the last batches of two
    ORBextractor handles (slamhot_stereo_match_batch_device)."""

    def __init__(self, device: int = 0):
        L = lib()
        if not getattr(L, "_stereo_ready", False):
            L.slamhot_stereo_create.argtypes = [I, C.POINTER(P)]
            L.slamhot_stereo_destroy.argtypes = [P]
            L.slamhot_stereo_destroy.restype = None
            L.slamhot_stereo_match_batch_device.argtypes = [P, P, P, I, P, P, P, P, P, P, I, C.c_float, C.c_float,
                                                            P, P, P, P]
            L.slamhot_pyramid_level_device.argtypes = [P, I, I, C.POINTER(P), C.POINTER(I), C.POINTER(I),
                                                       C.POINTER(I)]
            L._stereo_ready = True
        h = P()
        check(L.slamhot_stereo_create(device, C.byref(h)), "stereo_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().slamhot_stereo_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def match_batch_device(self, left: ORBextractor, right: ORBextractor, nframes: int, d_kps_l: int, d_desc_l: int,
                           d_n_l: int, d_kps_r: int, d_desc_r: int, d_n_r: int, cap: int, mbf: float, mb: float,
                           d_uright: int, d_depth: int, d_sad: int | None = None, stream: int | None = None):
        """All pointers are device addresses (ints); outputs mvuRight / mvDepth per left keypoint."""
        st = lib().slamhot_stereo_match_batch_device(self._h, left._h, right._h, nframes, P(d_kps_l), P(d_desc_l),
                                                     P(d_n_l), P(d_kps_r), P(d_desc_r), P(d_n_r), cap, mbf, mb,
                                                     P(d_uright), P(d_depth), P(d_sad) if d_sad else None,
                                                     P(stream) if stream else None)
        check(st, "slamhot_stereo_match_batch_device")

    def compute(self, left: ORBextractor, right: ORBextractor, kps_l, desc_l, kps_r, desc_r, mbf: float, mb: float):
        """Frame::ComputeStereoMatches on host arrays after one host extraction on each handle
        (slamhot_compute_stereo_matches): returns (mvuRight, mvDepth)."""
        L = lib()
        if not getattr(L, "_stereo_host_ready", False):
            L.slamhot_compute_stereo_matches.argtypes = [P, P, P, I, P, P, I, P, P, C.c_float, C.c_float, P, P]
            L._stereo_host_ready = True
        kl = np.ascontiguousarray(kps_l, KP_DTYPE)
        kr = np.ascontiguousarray(kps_r, KP_DTYPE)
        dl = np.ascontiguousarray(desc_l, np.uint8)
        dr = np.ascontiguousarray(desc_r, np.uint8)
        ur = np.full(len(kl), -1.0, np.float32)
        dep = np.full(len(kl), -1.0, np.float32)
        check(L.slamhot_compute_stereo_matches(self._h, left._h, right._h, len(kl), _ptr(kl), _ptr(dl), len(kr),
                                               _ptr(kr), _ptr(dr), mbf, mb, _ptr(ur), _ptr(dep)),
              "slamhot_compute_stereo_matches")
        return ur, dep


def ComputeStereoMatches(left: ORBextractor, right: ORBextractor, images_left, images_right, mbf: float, mb: float,
                         matcher: StereoMatcher | None = None):
    """Stereo Frame construction for a batch of rectified pairs (Frame.cc:80-180 stereo path:
    two ORB extractions, then ComputeStereoMatches), device-resident between the steps; torch
    provides the device buffers.  Returns per frame (kps_left, desc_left, kps_right,
    desc_right, mvuRight, mvDepth)."""
    import torch
    il = np.ascontiguousarray(images_left, np.uint8)
    ir = np.ascontiguousarray(images_right, np.uint8)
    if il.ndim == 2:
        il, ir = il[None], ir[None]
    F, H, W = il.shape
    cap = left.cap
    dev = torch.device("cuda", torch.cuda.current_device())
    bufs = []
    for ex, im in ((left, il), (right, ir)):
        d_img = torch.from_numpy(im).to(dev)
        d_kps = torch.zeros((F, cap, KP_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
        d_n = torch.zeros(F, dtype=torch.int32, device=dev)
        d_mono = torch.zeros(F, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        ex.extract_batch_device(d_img.data_ptr(), F, W, H, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(),
                                d_mono.data_ptr())
        bufs.append((d_img, d_kps, d_desc, d_n))
    torch.cuda.synchronize()
    d_ur = torch.empty((F, cap), dtype=torch.float32, device=dev)
    d_dep = torch.empty((F, cap), dtype=torch.float32, device=dev)
    own = matcher is None
    m = matcher or StereoMatcher(dev.index or 0)
    (_, kl, dl, nl), (_, kr, dr, nr) = bufs
    m.match_batch_device(left, right, F, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(), dr.data_ptr(),
                         nr.data_ptr(), cap, mbf, mb, d_ur.data_ptr(), d_dep.data_ptr())
    torch.cuda.synchronize()
    if own:
        m.close()
    nl_h, nr_h = nl.cpu().numpy(), nr.cpu().numpy()
    kl_h, kr_h = kl.cpu().numpy().view(KP_DTYPE), kr.cpu().numpy().view(KP_DTYPE)
    dl_h, dr_h = dl.cpu().numpy(), dr.cpu().numpy()
    ur, dep = d_ur.cpu().numpy(), d_dep.cpu().numpy()
    out = []
    for f in range(F):
        a, b = int(nl_h[f]), int(nr_h[f])
        out.append((kl_h[f, :a].ravel().copy(), dl_h[f, :a].copy(), kr_h[f, :b].ravel().copy(), dr_h[f, :b].copy(),
                    ur[f, :a].copy(), dep[f, :a].copy()))
    return out


# ------------------------------------------------------------------ LocalMapping matchers
class TriKF(C.Structure):
    _fields_ = [("n", I), ("kps_un", P), ("uright", P), ("desc", P), ("has_mp", P), ("n_nodes", I),
                ("node_id", P), ("node_off", P), ("node_feat", P), ("nlevels", I), ("scale", P),
                ("level_sigma2", P), ("Rcw", C.c_float * 9), ("tcw", C.c_float * 3), ("Ow", C.c_float * 3),
                ("cam", C.c_float * 4)]


class TriPair(C.Structure):
    _fields_ = [("kf1", I), ("kf2", I), ("only_stereo", C.c_uint8), ("coarse", C.c_uint8), ("pad", C.c_uint8 * 2)]


def camera_center(Tcw):
    """KeyFrame::SetPose's Ow = -Rwc * tcw (cv::Mat product: double accumulation, rounded once)."""
    T = np.asarray(Tcw, np.float32).astype(np.float64)
    return (-(T[:3, :3].T @ T[:3, 3])).astype(np.float32)


def make_tri_kf(kf: dict):
    """slam_tri_kf from a dict: kps_un (KP_DTYPE), uright, desc, has_mp, node_id/node_off/node_feat
    (mFeatVec CSR), scale, level_sigma2, Tcw (4x4 float), cam (fx, fy, cx, cy) and optionally Ow
    (default: camera_center(Tcw)).  Returns (struct, keepalive)."""
    keep = dict(kps=np.ascontiguousarray(kf["kps_un"], KP_DTYPE), desc=np.ascontiguousarray(kf["desc"], np.uint8),
                has=np.ascontiguousarray(kf["has_mp"], np.uint8),
                nid=np.ascontiguousarray(kf["node_id"], np.int32), noff=np.ascontiguousarray(kf["node_off"], np.int32),
                nf=np.ascontiguousarray(kf["node_feat"], np.int32), sc=np.ascontiguousarray(kf["scale"], np.float32),
                s2=np.ascontiguousarray(kf["level_sigma2"], np.float32))
    ur = kf.get("uright")
    keep["ur"] = None if ur is None else np.ascontiguousarray(ur, np.float32)
    t = TriKF()
    t.n = len(keep["kps"])
    t.kps_un = keep["kps"].ctypes.data if t.n else None
    t.uright = keep["ur"].ctypes.data if keep["ur"] is not None and t.n else None
    t.desc = keep["desc"].ctypes.data if t.n else None
    t.has_mp = keep["has"].ctypes.data if t.n else None
    t.n_nodes = len(keep["nid"])
    t.node_id = keep["nid"].ctypes.data if t.n_nodes else None
    t.node_off = keep["noff"].ctypes.data if t.n_nodes else None
    t.node_feat = keep["nf"].ctypes.data if len(keep["nf"]) else None
    t.nlevels = len(keep["sc"])
    t.scale = keep["sc"].ctypes.data
    t.level_sigma2 = keep["s2"].ctypes.data
    T = np.asarray(kf["Tcw"], np.float32)
    t.Rcw[:] = [float(v) for v in T[:3, :3].ravel()]
    t.tcw[:] = [float(v) for v in T[:3, 3]]
    t.Ow[:] = [float(v) for v in np.asarray(kf.get("Ow", camera_center(T)), np.float32)]
    t.cam[:] = [float(v) for v in np.asarray(kf["cam"], np.float32)]
    return t, keep


def make_tri_pair(kf1: int, kf2: int, only_stereo=False, coarse=False):
    p = TriPair()
    p.kf1, p.kf2 = kf1, kf2
    p.only_stereo, p.coarse = int(only_stereo), int(coarse)
    return p


class Mapper:
    """Device LocalMapping matchers: MapPoint::ComputeDistinctiveDescriptors (batched over
    MapPoints), ORBmatcher::SearchForTriangulation_ and ORBmatcher::Fuse candidate search."""

    def __init__(self, device: int = 0):
        L = lib()
        if not getattr(L, "_mapper_ready", False):
            L.slamhot_mapper_create.argtypes = [I, C.POINTER(P)]
            L.slamhot_mapper_destroy.argtypes = [P]
            L.slamhot_mapper_destroy.restype = None
            L.slamhot_distinctive_descriptors.argtypes = [P, I, P, P, P]
            L.slamhot_search_for_triangulation.argtypes = [P, I, C.POINTER(TriKF), I, C.POINTER(TriPair), I, I, P, P]
            L.slamhot_fuse_search.argtypes = [P, C.POINTER(FrameView), P, I, P, P, C.c_float, P, P]
            L._mapper_ready = True
        h = P()
        check(L.slamhot_mapper_create(device, C.byref(h)), "mapper_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().slamhot_mapper_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def ComputeDistinctiveDescriptors(self, off, desc):
        """off: int32 (n_mp + 1) CSR offsets into desc (total x 32 u8).  Returns best index
        per MapPoint (relative to its first descriptor), -1 when it has none."""
        off = np.ascontiguousarray(off, np.int32)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        best = np.zeros(len(off) - 1, np.int32)
        check(lib().slamhot_distinctive_descriptors(self._h, len(off) - 1, _ptr(off), _ptr(desc) if len(desc) else None,
                                                    _ptr(best)), "distinctive_descriptors")
        return best

    def SearchForTriangulation(self, kfs, pairs, check_ori=False):
        """kfs: list of KeyFrame dicts (make_tri_kf); pairs: list of (kf1, kf2, only_stereo, coarse).
        Returns [(nmatches, vMatchedPairs as an (m, 2) array)]."""
        built = [make_tri_kf(k) for k in kfs]
        K = (TriKF * max(1, len(built)))(*[b[0] for b in built])
        Ps = (TriPair * max(1, len(pairs)))(*[make_tri_pair(*p) for p in pairs])
        cap = max([b[0].n for b in built] + [1])
        m12 = np.full((len(pairs), cap), -1, np.int32)
        nm = np.zeros(len(pairs), np.int32)
        check(lib().slamhot_search_for_triangulation(self._h, len(built), K, len(pairs), Ps, int(check_ori), cap,
                                                     _ptr(m12), _ptr(nm)), "search_for_triangulation")
        out = []
        for p, (a, *_rest) in enumerate(pairs):
            row = m12[p, : built[a][0].n]
            i1 = np.flatnonzero(row >= 0)
            out.append((int(nm[p]), np.stack([i1, row[i1]], 1).astype(np.int64)))
        return out

    def FuseSearch(self, kf_view, inv_level_sigma2, mps, mp_desc, th=3.0):
        """Search half of ORBmatcher::Fuse(pKF, vpMapPoints, th): (best_idx, best_dist) per MapPoint
        (mps: MP_GEOM_DTYPE, seen = IsInKeyFrame(pKF))."""
        mps = np.ascontiguousarray(mps, MP_GEOM_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
        isig = np.ascontiguousarray(inv_level_sigma2, np.float32)
        bi = np.full(len(mps), -1, np.int32)
        bd = np.full(len(mps), 256, np.int32)
        check(lib().slamhot_fuse_search(self._h, C.byref(kf_view), _ptr(isig), len(mps), _ptr(mps), _ptr(mp_desc), th,
                                        _ptr(bi), _ptr(bd)), "fuse_search")
        return bi, bd


# ------------------------------------------------------------------------------------------
# Frame construction: Frame::UndistortKeyPoints / ComputeImageBounds (Frame.cc:730-792)
# ------------------------------------------------------------------------------------------
def _bind_frame(L):
    if getattr(L, "_frame_ready", False):
        return
    L.slamhot_undistort_keypoints.argtypes = [I, P, P, I, I, P, P]
    L.slamhot_undistort_keypoints_batch_device.argtypes = [P, P, I, I, P, P, I, P, P]
    L.slamhot_image_bounds.argtypes = [P, P, I, I, I, P]
    L._frame_ready = True


def UndistortKeyPoints(kps, K, dist, device: int = 0):
    """mvKeysUn of mvKeys for a Pinhole camera K = (fx, fy, cx, cy) with mDistCoef = dist."""
    L = lib()
    _bind_frame(L)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    Kf = np.ascontiguousarray(K, np.float32)
    D = np.ascontiguousarray(dist, np.float32)
    out = np.zeros_like(kps)
    check(L.slamhot_undistort_keypoints(device, _ptr(Kf), _ptr(D), len(D), len(kps), _ptr(kps), _ptr(out)),
          "undistort_keypoints")
    return out


def undistort_keypoints_batch_device(K, dist, nframes, d_kps, d_n, cap, d_kps_un, stream=None):
    L = lib()
    _bind_frame(L)
    Kf = np.ascontiguousarray(K, np.float32)
    D = np.ascontiguousarray(dist, np.float32)
    check(L.slamhot_undistort_keypoints_batch_device(_ptr(Kf), _ptr(D), len(D), nframes, P(d_kps), P(d_n), cap,
                                                     P(d_kps_un), P(stream) if stream else None),
          "undistort_keypoints_batch_device")


def ComputeImageBounds(K, dist, cols, rows):
    L = lib()
    _bind_frame(L)
    Kf = np.ascontiguousarray(K, np.float32)
    D = np.ascontiguousarray(dist, np.float32)
    b = np.zeros(4, np.float32)
    check(L.slamhot_image_bounds(_ptr(Kf), _ptr(D), len(D), cols, rows, _ptr(b)), "image_bounds")
    return b


# ------------------------------------------------------------------------------------------
# Per-sequence stereo tracking chain (slamhot_tracker_*, csrc/track.hip; BASELINE configs[4])
# ------------------------------------------------------------------------------------------
class TrackerConfig(C.Structure):
    _fields_ = [("nseq", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("orb", OrbParams),
                ("cam", Camera), ("th_depth", C.c_float), ("map_lx", C.c_void_p), ("map_ly", C.c_void_p),
                ("map_rx", C.c_void_p), ("map_ry", C.c_void_p)]


class TrackRecord(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("n", C.c_int32), ("n_stereo", C.c_int32), ("n_bow", C.c_int32),
                ("n_inl_ref", C.c_int32), ("n_local", C.c_int32), ("n_inl", C.c_int32), ("is_keyframe", C.c_int32),
                ("lost", C.c_int32), ("initialized", C.c_int32), ("n_motion", C.c_int32), ("motion", C.c_int32),
                ("status", C.c_int32)]


class TrackState(C.Structure):
    _fields_ = [("V", C.c_float * 16), ("Tlr", C.c_float * 16), ("Tref", C.c_float * 16), ("has_vel", C.c_int32),
                ("nkf", C.c_int32), ("last_n", C.c_int32), ("cap", C.c_int32), ("last_kps", C.c_void_p),
                ("last_mp", C.c_void_p)]


class TrackFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("cap", C.c_int32), ("uright", C.c_void_p), ("bow_match", C.c_void_p),
                ("motion_match", C.c_void_p), ("local_match", C.c_void_p), ("mappoints", C.c_void_p)]


class TrackKeyFrame(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("initialized", C.c_int32), ("n_ref", C.c_int32), ("n", C.c_int32),
                ("cap", C.c_int32), ("kps", C.c_void_p), ("desc", C.c_void_p), ("mp_valid", C.c_void_p),
                ("mp_pos", C.c_void_p), ("mp_normal", C.c_void_p), ("mp_min_dist", C.c_void_p),
                ("mp_max_dist", C.c_void_p), ("mp_desc", C.c_void_p)]


class Tracker:
    """nseq stereo sequences tracked in lock-step on one device (Tracking::Track, stereo)."""

    def __init__(self, vocab: Vocabulary, nseq: int, cam, maps=None, width: int = 752, height: int = 480,
                 nfeatures: int = 1200, th_depth: float = 35.0, device: int = 0):
        L = lib()
        if not getattr(L, "_track_ready", False):
            L.slamhot_tracker_create.argtypes = [I, C.POINTER(TrackerConfig), P, C.POINTER(P)]
            L.slamhot_tracker_destroy.argtypes = [P]
            L.slamhot_tracker_destroy.restype = None
            L.slamhot_tracker_step_device.argtypes = [P, P, I, C.c_int64, P, I, C.c_int64]
            L.slamhot_tracker_records.argtypes = [P, P]
            L.slamhot_tracker_keyframe.argtypes = [P, I, C.POINTER(TrackKeyFrame)]
            L.slamhot_tracker_state.argtypes = [P, I, C.POINTER(TrackState)]
            L.slamhot_tracker_frame.argtypes = [P, I, C.POINTER(TrackFrame)]
            L._track_ready = True
        self.nseq, self.W, self.H, self.cap = nseq, width, height, 2 * nfeatures + 64
        self._maps = None
        cfg = TrackerConfig(nseq, width, height, OrbParams(nfeatures, 1.2, 8, 20, 7), Camera(*cam), th_depth)
        if maps is not None:
            self._maps = [np.ascontiguousarray(m, np.float32) for pair in maps for m in pair]
            cfg.map_lx, cfg.map_ly, cfg.map_rx, cfg.map_ry = [m.ctypes.data for m in self._maps]
        self._voc = vocab
        h = P()
        check(L.slamhot_tracker_create(device, C.byref(cfg), vocab._h, C.byref(h)), "tracker_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().slamhot_tracker_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step_device(self, d_left: int, d_right: int, pitch=None, stride=None):
        pitch = pitch or self.W
        stride = stride or self.W * self.H
        check(lib().slamhot_tracker_step_device(self._h, P(d_left), pitch, stride, P(d_right), pitch, stride),
              "tracker_step")

    def records(self):
        recs = (TrackRecord * self.nseq)()
        check(lib().slamhot_tracker_records(self._h, recs), "tracker_records")
        return [dict(Tcw=np.array(r.Tcw[:], np.float32).reshape(4, 4), n=r.n, n_stereo=r.n_stereo, n_bow=r.n_bow,
                     n_inl_ref=r.n_inl_ref, n_local=r.n_local, n_inl=r.n_inl, is_keyframe=r.is_keyframe,
                     lost=r.lost, initialized=r.initialized, n_motion=r.n_motion, motion=r.motion,
                     status=r.status) for r in recs]

    def records_status(self):
        """(slam_status of slamhot_tracker_records, records) without raising on SLAM_ECAP."""
        recs = (TrackRecord * self.nseq)()
        st = lib().slamhot_tracker_records(self._h, recs)
        return st, [dict(status=r.status, lost=r.lost, is_keyframe=r.is_keyframe,
                         Tcw=np.array(r.Tcw[:], np.float32).reshape(4, 4)) for r in recs]

    def state(self, seq: int):
        """The motion-model state and last frame of sequence seq (slamhot_tracker_state)."""
        cap = self.cap
        kps, mp = np.zeros(cap, KP_DTYPE), np.zeros(cap, np.int32)
        st = TrackState()
        st.cap, st.last_kps, st.last_mp = cap, kps.ctypes.data, mp.ctypes.data
        check(lib().slamhot_tracker_state(self._h, seq, C.byref(st)), "tracker_state")
        n = st.last_n
        return dict(V=np.array(st.V[:], np.float32).reshape(4, 4), Tlr=np.array(st.Tlr[:], np.float32).reshape(4, 4),
                    Tref=np.array(st.Tref[:], np.float32).reshape(4, 4), has_vel=st.has_vel, nkf=st.nkf,
                    last_kps=kps[:n].copy(), last_mp=mp[:n].copy())

    def frame(self, seq: int):
        """The last step's per-feature arrays of sequence seq (slamhot_tracker_frame): uright,
        bow_match, motion_match, local_match, mappoints."""
        cap = self.cap
        out = dict(uright=np.zeros(cap, np.float32), bow_match=np.zeros(cap, np.int32),
                   motion_match=np.zeros(cap, np.int32), local_match=np.zeros(cap, np.int32),
                   mappoints=np.zeros(cap, np.int32))
        fr = TrackFrame()
        fr.cap = cap
        for k, a in out.items():
            setattr(fr, k, a.ctypes.data)
        check(lib().slamhot_tracker_frame(self._h, seq, C.byref(fr)), "tracker_frame")
        return {k: v[:fr.n].copy() for k, v in out.items()}

    def keyframe(self, seq: int):
        cap = self.cap
        out = dict(kps=np.zeros(cap, KP_DTYPE), desc=np.zeros((cap, 32), np.uint8), mp_valid=np.zeros(cap, np.uint8),
                   mp_pos=np.zeros((cap, 3), np.float32), mp_normal=np.zeros((cap, 3), np.float32),
                   mp_min_dist=np.zeros(cap, np.float32), mp_max_dist=np.zeros(cap, np.float32),
                   mp_desc=np.zeros((cap, 32), np.uint8))
        kf = TrackKeyFrame()
        kf.cap = cap
        for k, a in out.items():
            setattr(kf, k, a.ctypes.data)
        check(lib().slamhot_tracker_keyframe(self._h, seq, C.byref(kf)), "tracker_keyframe")
        n = kf.n
        res = {k: v[:n].copy() for k, v in out.items()}
        res.update(Tcw=np.array(kf.Tcw[:], np.float32).reshape(4, 4), initialized=kf.initialized, n_ref=kf.n_ref, n=n)
        return res
