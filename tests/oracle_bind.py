"""ctypes binding of oracle/build/liboracle.so — the CPU checker (test infrastructure)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def _lib_path():
    """The AVX-512 build (-march=x86-64-v4, what -march=native gives on the GPU box's EPYC) where
    the CPU has it, else the x86-64-v3 build; SLAMHOT_ORACLE_LIB overrides."""
    import os
    env = os.environ.get("SLAMHOT_ORACLE_LIB")
    if env:
        return Path(env)
    v4 = ROOT / "oracle" / "build" / "liboracle_v4.so"
    try:
        flags = open("/proc/cpuinfo").read()
        if v4.exists() and " avx512f " in flags and " avx512bw " in flags and " avx512vl " in flags:
            return v4
    except OSError:
        pass
    return ROOT / "oracle" / "build" / "liboracle.so"


LIB_PATH = _lib_path()


class KeyPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(str(LIB_PATH))
        P = C.c_void_p
        L.oracle_extract.argtypes = [C.POINTER(OrbParams), P, C.c_int, C.c_int, C.c_size_t, C.c_int,
                                     C.c_int, P, P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_extract.restype = C.c_int
        L.oracle_levels.argtypes = [C.POINTER(OrbParams), P, P, P, P, P]
        L.oracle_pyramid.argtypes = [C.POINTER(OrbParams), P, C.c_int, C.c_int, C.c_size_t, P,
                                     C.c_size_t, P, P, P]
        L.oracle_pyramid.restype = C.c_int
        L.oracle_resize_linear.argtypes = [P, C.c_int, C.c_int, C.c_size_t, P, C.c_int, C.c_int, C.c_size_t]
        L.oracle_fast.argtypes = [P, C.c_int, C.c_int, C.c_size_t, C.c_int, P, C.c_int]
        L.oracle_fast.restype = C.c_int
        L.oracle_gaussian_blur7.argtypes = [P, C.c_int, C.c_int, C.c_size_t, P, C.c_size_t, C.c_int]
        L.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.oracle_fast_atan2.restype = C.c_float
        L.oracle_sincosf.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_keypoints_octree.argtypes = [C.POINTER(OrbParams), P, C.c_int, C.c_int, C.c_size_t, P,
                                              C.c_int, P]
        L.oracle_keypoints_octree.restype = C.c_int
        L.oracle_descriptor_distance.argtypes = [P, P]
        L.oracle_descriptor_distance.restype = C.c_int
        L.oracle_extract_many.argtypes = [C.POINTER(OrbParams), C.c_int, P, C.c_int, C.c_int, C.c_size_t,
                                          C.c_int, C.c_int, C.c_int]
        L.oracle_extract_many.restype = C.c_long
        _lib = L
    return _lib


def params(nfeatures=1000, scale=1.2, nlevels=8, ini=20, mn=7) -> OrbParams:
    return OrbParams(nfeatures, scale, nlevels, ini, mn)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def extract(img: np.ndarray, p: OrbParams | None = None, lap=(0, 0)):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = p.nfeatures * 2 + 64
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n, mono = C.c_int(0), C.c_int(0)
    st = lib().oracle_extract(C.byref(p), _ptr(img), w, h, w, lap[0], lap[1], _ptr(kps), _ptr(desc), cap,
                              C.byref(n), C.byref(mono))
    if st != 0:
        raise RuntimeError(f"oracle_extract status {st}")
    return kps[:n.value].copy(), desc[:n.value].copy(), mono.value


def extract_with_pyramid(img: np.ndarray, p: OrbParams | None = None, lap=(0, 0)):
    """ORBextractor::operator() and its mvImagePyramid from one run: (kps, desc, mono, levels)."""
    p = p or params()
    L = lib()
    if not hasattr(L, "_xp_ready"):
        P = C.c_void_p
        L.oracle_extract_pyr.argtypes = [C.POINTER(OrbParams), P, C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_int, P,
                                         P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), P, C.c_size_t, P, P, P]
        L.oracle_extract_pyr.restype = C.c_int
        L._xp_ready = True
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = p.nfeatures * 2 + 64
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n, mono = C.c_int(0), C.c_int(0)
    pcap = w * h * 4
    out = np.zeros(pcap, np.uint8)
    lw = np.zeros(p.nlevels, np.int32)
    lh = np.zeros(p.nlevels, np.int32)
    off = np.zeros(p.nlevels, np.uint64)
    st = L.oracle_extract_pyr(C.byref(p), _ptr(img), w, h, w, lap[0], lap[1], _ptr(kps), _ptr(desc), cap, C.byref(n),
                              C.byref(mono), _ptr(out), pcap, _ptr(lw), _ptr(lh), _ptr(off))
    if st != 0:
        raise RuntimeError(f"oracle_extract_pyr status {st}")
    pyr = [out[int(off[l]): int(off[l]) + lw[l] * lh[l]].reshape(lh[l], lw[l]) for l in range(p.nlevels)]
    return kps[:n.value].copy(), desc[:n.value].copy(), mono.value, pyr


def levels(p: OrbParams | None = None):
    p = p or params()
    L = p.nlevels
    arrs = [np.zeros(L, np.float32) for _ in range(4)] + [np.zeros(L, np.int32)]
    lib().oracle_levels(C.byref(p), *[_ptr(a) for a in arrs])
    return arrs


def pyramid(img: np.ndarray, p: OrbParams | None = None):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = w * h * max(4, p.nlevels)  # every level is at most the image (16 levels at 1.05: ~8.6x)
    out = np.zeros(cap, np.uint8)
    lw = np.zeros(p.nlevels, np.int32)
    lh = np.zeros(p.nlevels, np.int32)
    off = np.zeros(p.nlevels, np.uint64)
    st = lib().oracle_pyramid(C.byref(p), _ptr(img), w, h, w, _ptr(out), cap, _ptr(lw), _ptr(lh), _ptr(off))
    assert st == 0
    return [out[int(off[l]): int(off[l]) + lw[l] * lh[l]].reshape(lh[l], lw[l]).copy() for l in range(p.nlevels)]


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize_linear(_ptr(src), sw, sh, sw, _ptr(dst), dw, dh, dw)
    return dst


def fast(roi: np.ndarray, threshold: int) -> np.ndarray:
    roi = np.ascontiguousarray(roi, dtype=np.uint8)
    h, w = roi.shape
    cap = w * h
    out = np.zeros((cap, 3), np.int32)
    n = lib().oracle_fast(_ptr(roi), w, h, w, threshold, _ptr(out), cap)
    assert n >= 0
    return out[:n].copy()


def gaussian_blur7(img: np.ndarray, ed: bool = True) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros_like(img)
    lib().oracle_gaussian_blur7(_ptr(img), w, h, w, _ptr(out), w, 1 if ed else 0)
    return out


def fast_atan2(y: float, x: float) -> float:
    return lib().oracle_fast_atan2(y, x)


def sincosf(x: float):
    s, c = C.c_float(), C.c_float()
    lib().oracle_sincosf(x, C.byref(s), C.byref(c))
    return s.value, c.value


def keypoints_octree(img: np.ndarray, p: OrbParams | None = None):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = p.nfeatures * 2 + 64
    kps = np.zeros(cap, KP_DTYPE)
    counts = np.zeros(p.nlevels, np.int32)
    n = lib().oracle_keypoints_octree(C.byref(p), _ptr(img), w, h, w, _ptr(kps), cap, _ptr(counts))
    assert n >= 0
    return kps[:n].copy(), counts


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return lib().oracle_descriptor_distance(_ptr(a), _ptr(b))


def extract_many(imgs: np.ndarray, p: OrbParams | None = None, lap=(0, 0), nthreads=1) -> int:
    p = p or params()
    imgs = np.ascontiguousarray(imgs, dtype=np.uint8)
    n, h, w = imgs.shape
    return lib().oracle_extract_many(C.byref(p), n, _ptr(imgs), w, h, w, lap[0], lap[1], nthreads)


# ---- matchers / vocabulary (oracle/matcher_oracle.cpp)
def _mlib():
    L = lib()
    if not hasattr(L, "_m_ready"):
        P = C.c_void_p
        L.oracle_hamming.argtypes = [P, P]
        L.oracle_hamming.restype = C.c_int
        L.oracle_three_maxima.argtypes = [P, C.c_int, P]
        L.oracle_vocab_transform.argtypes = [C.c_int, P, P, P, P, P, P, C.c_int, P, C.c_int, P, P, P]
        L.oracle_search_by_bow.argtypes = [P, P, C.c_float, C.c_int, C.c_int, P, P]
        L.oracle_search_by_bow.restype = C.c_int
        L._m_ready = True
    return L


def three_maxima(counts):
    counts = np.ascontiguousarray(counts, np.int32)
    ind = np.zeros(3, np.int32)
    _mlib().oracle_three_maxima(_ptr(counts), len(counts), _ptr(ind))
    return tuple(int(x) for x in ind)


def vocab_children(parent):
    n = len(parent)
    cnt = np.bincount(parent[1:], minlength=n)
    ptr = np.zeros(n + 1, np.int32)
    ptr[1:] = np.cumsum(cnt)
    order = np.argsort(parent[1:], kind="stable") + 1
    return ptr, order.astype(np.int32)


_vocab_tables = {}


def _vocab_prepared(parent, is_leaf):
    """Children CSR, leaf flags and word ids of a node table (built once per table)."""
    key = (id(parent), id(is_leaf), len(parent))
    t = _vocab_tables.get(key)
    if t is None or t[0] is not parent:
        ptr, idx = vocab_children(parent)
        leaf = np.ascontiguousarray(is_leaf, np.uint8).copy()
        leaf[ptr[1:] == ptr[:-1]] = 1
        word = np.full(len(parent), -1, np.int32)
        word[np.nonzero(is_leaf)[0]] = np.arange(int(np.count_nonzero(is_leaf)), dtype=np.int32)
        t = (parent, ptr, idx, leaf, word)
        _vocab_tables[key] = t
    return t[1:]


def vocab_transform(parent, is_leaf, desc_nodes, weight_nodes, L, desc, levelsup=4):
    ptr, idx, leaf, word = _vocab_prepared(parent, is_leaf)
    desc = np.ascontiguousarray(desc, np.uint8)
    n = len(desc)
    w = np.zeros(n, np.int32)
    wt = np.zeros(n, np.float64)
    nid = np.zeros(n, np.int32)
    dn = np.ascontiguousarray(desc_nodes, np.uint8)
    wn = np.ascontiguousarray(weight_nodes, np.float64)
    _mlib().oracle_vocab_transform(L, _ptr(ptr), _ptr(idx), _ptr(dn), _ptr(leaf), _ptr(word), _ptr(wn), n,
                                   _ptr(desc), levelsup, _ptr(w), _ptr(wt), _ptr(nid))
    return w, wt, nid


def bow_vectors(word, weight, node, scoring=0, weighting=0):
    """TemplatedVocabulary::transform's BowVector / FeatureVector from the per-feature descent
    (oracle/matcher_oracle.cpp oracle_bow_vectors): (words, values, nodes, offsets, features)."""
    L = _mlib()
    if not hasattr(L, "_bv_ready"):
        P = C.c_void_p
        L.oracle_bow_vectors.argtypes = [C.c_int, P, P, P, C.c_int, C.c_int, P, P, P, P, P, P, P]
        L.oracle_bow_vectors.restype = None
        L._bv_ready = True
    word = np.ascontiguousarray(word, np.int32)
    weight = np.ascontiguousarray(weight, np.float64)
    node = np.ascontiguousarray(node, np.int32)
    n = len(word)
    nw, nn = C.c_int(0), C.c_int(0)
    bw = np.zeros(max(n, 1), np.uint32)
    bv = np.zeros(max(n, 1), np.float64)
    fn = np.zeros(max(n, 1), np.uint32)
    fo = np.zeros(n + 1, np.int32)
    ff = np.zeros(max(n, 1), np.uint32)
    L.oracle_bow_vectors(n, _ptr(word), _ptr(weight), _ptr(node), scoring, weighting, C.byref(nw), _ptr(bw), _ptr(bv),
                         C.byref(nn), _ptr(fn), _ptr(fo), _ptr(ff))
    return bw[:nw.value], bv[:nw.value], fn[:nn.value], fo[:nn.value + 1], ff[:fo[nn.value]]


def search_by_bow(A, B, nnratio, check_ori, strict):
    import slamhot
    sa, ka = slamhot.make_bow_side(*A)
    sb, kb = slamhot.make_bow_side(*B)
    a2b = np.full(sa.n, -1, np.int32)
    b2a = np.full(sb.n, -1, np.int32)
    n = _mlib().oracle_search_by_bow(C.addressof(sa), C.addressof(sb), nnratio, int(check_ori), int(strict),
                                     _ptr(a2b), _ptr(b2a))
    return n, a2b, b2a


def check_sincosf(lo: float, hi: float) -> int:
    L = lib()
    L.oracle_check_sincosf.argtypes = [C.c_float, C.c_float]
    L.oracle_check_sincosf.restype = C.c_long
    return L.oracle_check_sincosf(lo, hi)


def check_atan2(ys, xs) -> int:
    L = lib()
    L.oracle_check_atan2.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    L.oracle_check_atan2.restype = C.c_long
    ys = np.ascontiguousarray(ys, np.float32)
    xs = np.ascontiguousarray(xs, np.float32)
    return L.oracle_check_atan2(len(ys), _ptr(ys), _ptr(xs))


# ---- projection matchers (oracle/projection_oracle.cpp)
def _plib():
    L = lib()
    if not hasattr(L, "_p_ready"):
        P = C.c_void_p
        L.oracle_search_by_projection_local.argtypes = [P, C.c_int, P, P, C.c_float, C.c_float, C.c_int, C.c_float, P]
        L.oracle_search_by_projection_local.restype = C.c_int
        L.oracle_search_by_projection_last.argtypes = [P, P, C.c_float, C.c_int, C.c_float, C.c_int, P]
        L.oracle_search_by_projection_last.restype = C.c_int
        L.oracle_search_by_projection_kf.argtypes = [P, P, C.c_float, C.c_int, C.c_float, C.c_int, P]
        L.oracle_search_by_projection_kf.restype = C.c_int
        L._p_ready = True
    return L


def search_by_projection_local(fv, mps, mp_desc, nnratio, th, far, th_far):
    import slamhot
    mps = np.ascontiguousarray(mps, slamhot.MP_TRACK_DTYPE)
    mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
    fm = np.full(fv.n, -1, np.int32)
    n = _plib().oracle_search_by_projection_local(C.addressof(fv), len(mps), _ptr(mps), _ptr(mp_desc), nnratio, th,
                                                  int(far), th_far, _ptr(fm))
    return n, fm


def search_by_projection_last(fv, lf, nnratio, check_ori, th, mono):
    fm = np.full(fv.n, -1, np.int32)
    n = _plib().oracle_search_by_projection_last(C.addressof(fv), C.addressof(lf), nnratio, int(check_ori), th, int(mono),
                                                 _ptr(fm))
    return n, fm


def search_by_projection_kf(fv, kf, nnratio, check_ori, th, orb_dist):
    fm = np.full(fv.n, -1, np.int32)
    n = _plib().oracle_search_by_projection_kf(C.addressof(fv), C.addressof(kf), nnratio, int(check_ori), th,
                                               int(orb_dist), _ptr(fm))
    return n, fm


# ---- local bundle adjustment (oracle/lba_oracle.cpp)
def lba_solve(w, iters_first=5, iters_second=10, user_lambda_init=0.0, stop=0):
    import slamhot
    L = lib()
    if not hasattr(L, "_lba_ready"):
        L.oracle_lba_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_lba_solve.restype = C.c_int
        L._lba_ready = True
    p, r, out = slamhot.make_lba_problem(w)
    opt = slamhot.LbaOptions(iters_first, iters_second, user_lambda_init)
    L.oracle_lba_solve(C.addressof(p), C.addressof(opt), int(stop), C.addressof(r))
    return slamhot.lba_result_dict(r, out)


# ---- motion-only BA (oracle/pose_oracle.cpp)
def pose_optimization(f):
    import slamhot
    L = lib()
    if not hasattr(L, "_pose_ready"):
        L.oracle_pose_optimization.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_pose_optimization.restype = C.c_int
        L._pose_ready = True
    pf, r, out = slamhot.make_pose_frame(f)
    L.oracle_pose_optimization(C.addressof(pf), C.addressof(r))
    return slamhot.pose_result_dict(r, out)


# ---- stereo matching (oracle/stereo_oracle.cpp)
def stereo_matches(kl, dl, kr, dr, pyr_left, pyr_right, scale, inv_scale, mbf, mb):
    """Frame::ComputeStereoMatches on host arrays; pyr_* are lists of 2-D u8 levels."""
    L = lib()
    V = C.c_void_p
    if not hasattr(L, "_stereo_ready"):
        L.oracle_stereo_matches.argtypes = [C.c_int, V, V, C.c_int, V, V, C.c_int, V, V, V, V, V, V, V, V,
                                            C.c_float, C.c_float, V, V]
        L.oracle_stereo_matches.restype = None
        L._stereo_ready = True
    nl = len(pyr_left)
    kl = np.ascontiguousarray(kl)
    kr = np.ascontiguousarray(kr)
    dl = np.ascontiguousarray(dl, np.uint8)
    dr = np.ascontiguousarray(dr, np.uint8)
    pl = [np.ascontiguousarray(a, np.uint8) for a in pyr_left]
    pr = [np.ascontiguousarray(a, np.uint8) for a in pyr_right]
    ptr_l = (C.c_void_p * nl)(*[a.ctypes.data for a in pl])
    ptr_r = (C.c_void_p * nl)(*[a.ctypes.data for a in pr])
    pitch_l = np.array([a.shape[1] for a in pl], np.int32)
    pitch_r = np.array([a.shape[1] for a in pr], np.int32)
    lw = pitch_l.copy()
    lh = np.array([a.shape[0] for a in pl], np.int32)
    sc = np.ascontiguousarray(scale, np.float32)
    isc = np.ascontiguousarray(inv_scale, np.float32)
    ur = np.zeros(len(kl), np.float32)
    dep = np.zeros(len(kl), np.float32)
    L.oracle_stereo_matches(len(kl), _ptr(kl), _ptr(dl), len(kr), _ptr(kr), _ptr(dr), nl, C.cast(ptr_l, V),
                            C.cast(ptr_r, V), _ptr(pitch_l), _ptr(pitch_r), _ptr(lw), _ptr(lh), _ptr(sc), _ptr(isc),
                            mbf, mb, _ptr(ur), _ptr(dep))
    return ur, dep


def _frlib():
    L = _plib()
    if not hasattr(L, "_fr_ready"):
        L.oracle_is_in_frustum.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_float, C.c_void_p]
        L.oracle_is_in_frustum.restype = C.c_int
        L.oracle_check_predict_scale.argtypes = [C.c_float, C.c_float, C.c_float]
        L.oracle_check_predict_scale.restype = C.c_long
        L._fr_ready = True
    return L


def is_in_frustum(fv, geom, view_cos_limit=0.5):
    """Frame::isInFrustum over a local map (oracle/projection_oracle.cpp); (nToMatch, track)."""
    import slamhot
    geom = np.ascontiguousarray(geom, slamhot.MP_GEOM_DTYPE)
    tr = np.zeros(len(geom), slamhot.MP_TRACK_DTYPE)
    n = _frlib().oracle_is_in_frustum(C.addressof(fv), len(geom), _ptr(geom), view_cos_limit, _ptr(tr))
    return n, tr


def check_predict_scale(lo, hi, log_scale):
    return int(_frlib().oracle_check_predict_scale(lo, hi, log_scale))


# ---- LocalMapping matchers (oracle/mapping_oracle.cpp)
def distinctive_descriptors(off, desc):
    L = lib()
    if not hasattr(L, "_dd_ready"):
        L.oracle_distinctive_descriptors.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_distinctive_descriptors.restype = None
        L._dd_ready = True
    off = np.ascontiguousarray(off, np.int32)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    best = np.zeros(len(off) - 1, np.int32)
    L.oracle_distinctive_descriptors(len(off) - 1, _ptr(off), _ptr(desc), _ptr(best))
    return best


def search_for_triangulation(kf1, kf2, pair, check_ori=False):
    """(nmatches, match12) for one pair; kf1/kf2 are slamhot.TriKF structs, pair a TriPair."""
    L = lib()
    if not hasattr(L, "_tri_ready"):
        L.oracle_search_for_triangulation.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_search_for_triangulation.restype = C.c_int
        L._tri_ready = True
    m12 = np.full(max(1, kf1.n), -1, np.int32)
    n = L.oracle_search_for_triangulation(C.addressof(kf1), C.addressof(kf2), C.addressof(pair), int(check_ori),
                                          _ptr(m12))
    return n, m12[: kf1.n]


def fuse_search(fv, inv_sigma2, geom, desc, th=3.0):
    import slamhot
    L = lib()
    if not hasattr(L, "_fuse_ready"):
        L.oracle_fuse_search.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
                                         C.c_void_p, C.c_void_p]
        L.oracle_fuse_search.restype = None
        L._fuse_ready = True
    geom = np.ascontiguousarray(geom, slamhot.MP_GEOM_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    isig = np.ascontiguousarray(inv_sigma2, np.float32)
    bi = np.zeros(len(geom), np.int32)
    bd = np.zeros(len(geom), np.int32)
    L.oracle_fuse_search(C.addressof(fv), _ptr(isig), len(geom), _ptr(geom), _ptr(desc), th, _ptr(bi), _ptr(bd))
    return bi, bd


# ---- rectification (oracle/rectify_oracle.cpp)
def remap_linear(src, map_x, map_y):
    L = lib()
    if not hasattr(L, "_remap_ready"):
        L.oracle_remap_linear.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                          C.c_int, C.c_void_p, C.c_int]
        L.oracle_remap_linear.restype = None
        L._remap_ready = True
    src = np.ascontiguousarray(src, np.uint8)
    mx = np.ascontiguousarray(map_x, np.float32)
    my = np.ascontiguousarray(map_y, np.float32)
    sh, sw = src.shape
    dh, dw = mx.shape
    dst = np.zeros((dh, dw), np.uint8)
    L.oracle_remap_linear(_ptr(src), sw, sh, sw, _ptr(mx), _ptr(my), dw, dh, _ptr(dst), dw)
    return dst


# ---- Frame construction (oracle/frame_oracle.cpp)
def undistort_keypoints(kps, K, dist):
    L = lib()
    if not hasattr(L, "_frame_ready"):
        L.oracle_undistort_keypoints.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_undistort_keypoints.restype = None
        L.oracle_image_bounds.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.oracle_image_bounds.restype = None
        L._frame_ready = True
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    Kf = np.ascontiguousarray(K, np.float32)
    D = np.ascontiguousarray(dist, np.float32)
    out = np.zeros_like(kps)
    L.oracle_undistort_keypoints(len(kps), _ptr(kps), _ptr(Kf), _ptr(D), len(D), _ptr(out))
    return out


def image_bounds(K, dist, cols, rows):
    undistort_keypoints(np.zeros(0, KP_DTYPE), K, dist)  # binds
    Kf = np.ascontiguousarray(K, np.float32)
    D = np.ascontiguousarray(dist, np.float32)
    b = np.zeros(4, np.float32)
    lib().oracle_image_bounds(_ptr(Kf), _ptr(D), len(D), cols, rows, _ptr(b))
    return b
