"""The oracle's float arithmetic at the matcher gates vs the reference binary's own data flow.

The reference's objects (/root/reference/evaluation/CMakeFiles/ORB_SLAM3.dir/src/*.o, GCC 9.3
-O3 -march=native) are read as data by tools/disasm/fptrace.py: each site's instruction range
is walked symbolically and emitted as C (every FMA contraction, widening and association as
compiled).  That C is built into oracle/_ref/libfpref.so (git-ignored) and compared bit for bit
with oracle/fp_sites.hpp's restatement on seeded random inputs.  Nothing from the reference is
executed.  The reference exists only in the build container, so this is a CPU test that skips
elsewhere; the device kernels are then held to the oracle by the -m gpu parity tests.
"""
from __future__ import annotations

import ctypes as C
import math
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
OBJ = Path("/root/reference/evaluation/CMakeFiles/ORB_SLAM3.dir/src")
pytestmark = pytest.mark.skipif(not OBJ.exists(), reason="reference objects exist only in the build container")

sys.path.insert(0, str(ROOT / "tools" / "disasm"))

P = lambda base, k: f"{base}+0x{4 * k:x}"  # noqa: E731

# name -> (object, ranges, inputs, outputs); object offsets are the ones DESIGN.md §1 cites
SITES = {
    # Pinhole::epipolarConstrain_ (Pinhole.cpp:159-181)
    "epi": ("CameraModels/Pinhole.cpp.o", ["0x70f0:0x7949"],
            [f"*(arg_rdi+0x10)+0x{4 * k:x}" for k in range(4)] + [f"*(arg_rsi+0x10)+0x{4 * k:x}" for k in range(4)]
            + [f"SkewSymmetricMatrix_#1.out[{k}]" for k in range(9)] + [P("arg_r8", k) for k in range(9)]
            + ["arg_rdx+0x0", "arg_rdx+0x4", "arg_rcx+0x0", "arg_rcx+0x4", "%xmm1"],
            [("cmp#2", 0), ("cmp#3", 1), ("cmp#3", 0)]),
    # SearchForTriangulation_ pinhole preamble (ORBmatcher.cc:1215-1240)
    "tri": ("ORBmatcher.cc.o", ["0x12880:0x12b5b", "0x14880:0x14c40"],
            ["GetCameraCenter_#1.xmm0[0]", "GetCameraCenter_#1.xmm0[1]", "GetCameraCenter_#1.xmm1[0]"]
            + [f"GetRotation_#2.out[{k}]" for k in range(9)]
            + ["GetTranslation_#3.xmm0[0]", "GetTranslation_#3.xmm0[1]", "GetTranslation_#3.xmm1[0]"]
            + [f"GetRotation_#5.out[{k}]" for k in range(9)]
            + ["GetTranslation_#6.xmm0[0]", "GetTranslation_#6.xmm0[1]", "GetTranslation_#6.xmm1[0]"],
            [("store:rsp-0x56c", 0), ("store:rsp-0x568", 0), ("store:rsp-0x564", 0)]
            + [(f"store:rsp-0x{0x310 - 4 * k:x}", 0) for k in range(9)]
            + [("live:%xmm1", 0), ("live:%xmm0", 0), ("live:%xmm2", 0)]),
    # Pinhole::project(cv::Matx31f) (Pinhole.cpp:42-48)
    "proj": ("CameraModels/Pinhole.cpp.o", ["0x5e0:0x66a"],
             [f"*(arg_rsi+0x10)+0x{4 * k:x}" for k in range(4)] + [P("arg_rdx", k) for k in range(3)],
             [("store:arg_rdi+0x0", 0), ("store:arg_rdi+0x4", 0)]),
    # cv::normL2Sqr<float,double> as inlined into Frame.cc.o (cv::norm(Matx31f))
    "norm": ("Frame.cc.o", ["0x0:0x2a"], [P("arg_rdi", k) for k in range(3)], [("ret", 0)]),
    # Frame::isInFrustum (Frame.cc:493-556)
    "frustum": ("Frame.cc.o", ["0x9ee0:0xa250"],
                ["GetWorldPos2#1.xmm0[0]", "GetWorldPos2#1.xmm0[1]", "GetWorldPos2#1.xmm1[0]"]
                + [f"arg_rdi+0x{0x1291c + 4 * k:x}" for k in range(9)]
                + [f"arg_rdi+0x{0x12940 + 4 * k:x}" for k in range(3)]
                + [f"arg_rdi+0x{0x12910 + 4 * k:x}" for k in range(3)]
                + ["arg_rdi+0x1a8", "*0x8#2.out[0]", "GetNormal2#6.xmm0[0]", "GetNormal2#6.xmm0[1]",
                   "GetNormal2#6.xmm1[0]", "normL2Sqr<float double>#5.xmm0d"],
                [("store:rsp+0x54", 0), ("store:rsp+0x58", 0), ("store:rsp+0x5c", 0), ("store:arg_rsi+0x24", 0),
                 ("store:arg_rsi+0x40", 0), ("store:arg_rsi+0x2c", 0), ("store:rsp+0x3c", 0)]),
    # SearchByProjection(Frame&, const Frame&, th, bMono) stereo gate (ORBmatcher.cc:2252-2258)
    "sbp_er": ("ORBmatcher.cc.o", ["0x95ac:0x95e4"],
               ["arg_rbp-0xc78", "arg_rcx+0x1a8", "arg_rbp-0xcf8", "(%rax,%rbx,4)"], [("live:%xmm0", 0)]),
    # computeOrbDescriptor's rotated sample (ORBextractor.cc:110-118): a = cos, b = sin (sincosf)
    "orb_rc": ("ORBextractor.cc.o", ["0x6a63:0x6adf"],
               ["arg_rbp-0x408", "arg_rbp-0x404", "int (%rbx)", "int 0x4(%rbx)"], [("int#2", 0), ("int#3", 0)]),
    # ORBextractor ctor: mvScaleFactor[i] = mvScaleFactor[i-1] * scaleFactor (a double member) and
    # mvLevelSigma2[i] = mvScaleFactor[i]^2 (ORBextractor.cc:417-423)
    "ctor_scale": ("ORBextractor.cc.o", ["0x345e:0x348f"], ["arg_rbx+0x38", "-0x4(%rdx,%rax,4)"],
                   [("store:(%rdx,%rax,4)", 0), ("live:%xmm0", 0)]),
    # ctor feature split: factor = 1/scaleFactor, nDesiredFeaturesPerScale (ORBextractor.cc:433-435)
    "ctor_nfeat": ("ORBextractor.cc.o", ["0x315a:0x31b7"],
                   ["arg_rbx+0x38", "int 0x30(%rbx)", "arg_rbp-0x34", "pow#1.xmm0d"],
                   [("store:arg_rbp-0x3c", 0), ("live:%xmm0", 0)]),
    # ctor umax[0..vmax] = cvRound(sqrt(hp2 - v*v)), folded to constants by the compiler (:452-457)
    "umax": ("ORBextractor.cc.o", ["0x3279:0x3303"], [], [("int#%d" % k, 0) for k in range(12)]),
    # ComputePyramid level size cvRound((float)rows|cols * mvInvScaleFactor[level]) (:1157)
    "pyr_size": ("ORBextractor.cc.o", ["0x4d0:0x515"], ["int 0x8(%r14)", "int 0xc(%r14)", "(%rax,%r12,4)"],
                 [("int#0", 0), ("int#1", 0)]),
    # operator(): keypoint->pt *= scale (:1131-1133)
    "kp_scale": ("ORBextractor.cc.o", ["0x6ec0:0x6ee0"], ["arg_rbx+0x0", "arg_rbx+0x4", "arg_rbp-0x470"],
                 [("store:arg_rbx+0x0", 0), ("store:arg_rbx+0x4", 0)]),
    # Frame::PosInGrid: round((pt - mnMin) * mfGridElement*Inv) (Frame.cc:708-718)
    "pos_in_grid": ("Frame.cc.o", ["0x6d30:0x6d8a"],
                    ["arg_rsi+0x0", "arg_rsi+0x4", "got:ORB_SLAM3::Frame::mnMinX-0x4+0x0",
                     "got:ORB_SLAM3::Frame::mfGridElementWidthInv-0x4+0x0", "got:ORB_SLAM3::Frame::mnMinY-0x4+0x0",
                     "got:ORB_SLAM3::Frame::mfGridElementHeightInv-0x4+0x0"],
                    [("int#0", 0), ("int#1", 0)]),
    # Frame::GetFeaturesInArea's cell range: floor / ceil of (x - mnMinX -+ r) * inv (Frame.cc:645-659)
    "area_cells": ("Frame.cc.o", ["0x67c0:0x6899"],
                   ["*(rsp+0x8)+0x0", "*(rsp+0x20)+0x0", "arg_r8+0x0", "got:ORB_SLAM3::Frame::mnMinX-0x4+0x0",
                    "got:ORB_SLAM3::Frame::mnMinY-0x4+0x0", "got:ORB_SLAM3::Frame::mfGridElementWidthInv-0x4+0x0",
                    "got:ORB_SLAM3::Frame::mfGridElementHeightInv-0x4+0x0"],
                   [("int#%d" % k, 0) for k in range(4)]),
    # SearchByBoW(KF, F) rotation bin: roundf(rot * (1/30)), rot < 0 path (+360) and rot >= 0 path
    # (ORBmatcher.cc:391-396)
    "rot_neg": ("ORBmatcher.cc.o", ["0x36e4:0x3711"], ["arg_rdx+0xc", "arg_rax+0xc"], [("int#0", 0)]),
    "rot_pos": ("ORBmatcher.cc.o", ["0x36e4:0x36f8", "0x3700:0x3711"], ["arg_rdx+0xc", "arg_rax+0xc"],
                [("int#0", 0)]),
    # SearchByProjection(F, LastF) window: radius = th * mvScaleFactors[nLastOctave] (ORBmatcher.cc:2225)
    "sbp_radius": ("ORBmatcher.cc.o", ["0x8cc3:0x8cc9"], ["(%rdx,%rax,4)", "%xmm7"], [("live:%xmm0", 0)]),
    # Fuse stereo reprojection chi2 (ORBmatcher.cc:1697, 1735-1745)
    "fuse_e2": ("ORBmatcher.cc.o", ["0x1bc8:0x1c25", "0x1c60:0x1cca"],
                ["rsp+0xa0", "rsp+0xbc", "arg_rdx+0x0", "arg_rdx+0x4", "(%rdi,%rax,4)", "rsp+0x8c", "rsp+0xa8",
                 "(%rdx,%rcx,4)", "rsp+0xb8"],
                [("cmp#1", 0)]),
}


@pytest.fixture(scope="module")
def ref_lib():
    import fptrace
    out = ROOT / "oracle" / "_ref"
    out.mkdir(parents=True, exist_ok=True)
    src = ["#include <math.h>"]
    for name, (obj, ranges, ins, outs) in SITES.items():
        tr = fptrace.trace(str(OBJ / obj), ranges)
        src.append(fptrace.emit_c(tr, f"site_{name}", ins, outs))
    (out / "fp_sites_ref.c").write_text("\n\n".join(src) + "\n")
    so = out / "libfpref.so"
    subprocess.run(["gcc", "-O1", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so), str(out / "fp_sites_ref.c"),
                    "-lm"], check=True)
    L = C.CDLL(str(so))
    for name in SITES:
        getattr(L, f"site_{name}").argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double)]
    return L


@pytest.fixture(scope="module")
def orc():
    import oracle_bind as ob
    return ob.lib()


def call_site(L, name, ins, nout):
    a = (C.c_double * len(ins))(*[float(v) for v in ins])
    o = (C.c_double * nout)()
    getattr(L, f"site_{name}")(a, o)
    return np.array(o[:], np.float64)


def fp(*v):
    return (C.c_float * len(v))(*[float(x) for x in v])


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b)


def rand_rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    return R.astype(np.float32)


def rand_cam(rng):
    return np.array([rng.uniform(300, 800), rng.uniform(300, 800), rng.uniform(200, 500), rng.uniform(150, 350)],
                    np.float32)


N = 4000


def test_epipolar_constrain(ref_lib, orc):
    rng = np.random.default_rng(1)
    out = (C.c_double * 3)()
    for _ in range(N):
        c1, c2 = rand_cam(rng), rand_cam(rng)
        R12 = rand_rot(rng)
        t12 = rng.normal(size=3).astype(np.float32)
        x1, y1, x2, y2 = rng.uniform(0, 752, 4).astype(np.float32)
        unc = np.float32(1.44 ** rng.integers(0, 8))
        S = [0.0, -t12[2], t12[1], t12[2], 0.0, -t12[0], -t12[1], t12[0], 0.0]
        r = call_site(ref_lib, "epi", list(c1) + list(c2) + S + list(R12.ravel()) + [x1, y1, x2, y2, unc], 3)
        orc.oracle_fp_epipolar_vals(fp(*c1), fp(*c2), fp(*R12.ravel()), fp(*t12), C.c_float(x1), C.c_float(y1),
                                    C.c_float(x2), C.c_float(y2), C.c_float(unc), out)
        assert same(r, out[:3]), (r, out[:3])


def test_triangulation_preamble(ref_lib, orc):
    rng = np.random.default_rng(2)
    ep, R12, t12, F12 = (C.c_float * 2)(), (C.c_float * 9)(), (C.c_float * 3)(), (C.c_float * 9)()
    for _ in range(N):
        R1, R2 = rand_rot(rng), rand_rot(rng)
        t1, t2 = rng.normal(size=3).astype(np.float32), rng.normal(size=3).astype(np.float32)
        Cw1 = (-R1.T.astype(np.float64) @ t1).astype(np.float32)
        cam = rand_cam(rng)
        r = call_site(ref_lib, "tri", list(Cw1) + list(R2.ravel()) + list(t2) + list(R1.ravel()) + list(t1), 15)
        orc.oracle_fp_tri_geometry(fp(*R1.ravel()), fp(*t1), fp(*Cw1), fp(*cam), fp(*R2.ravel()), fp(*t2), fp(*cam),
                                   ep, R12, t12, F12)
        C2 = r[:3]
        uv = (C.c_float * 2)()
        orc.oracle_fp_project(fp(*cam), fp(*C2), uv)
        pr = call_site(ref_lib, "proj", list(cam) + list(C2), 2)
        assert same(pr, [uv[0], uv[1]])
        assert same([ep[0], ep[1]], [uv[0], uv[1]])
        assert same(r[3:12], R12[:]), (r[3:12], R12[:])
        assert same(r[12:15], t12[:]), (r[12:15], t12[:])


def test_norm_and_frustum(ref_lib, orc):
    rng = np.random.default_rng(3)
    orc.oracle_fp_norm2.restype = C.c_double
    out = (C.c_double * 7)()
    for _ in range(N):
        v = rng.normal(size=3).astype(np.float32) * np.float32(rng.uniform(0.1, 30))
        assert same([call_site(ref_lib, "norm", list(v), 1)[0]], [orc.oracle_fp_norm2(fp(*v))])
        R = rand_rot(rng)
        t = rng.normal(size=3).astype(np.float32)
        T = np.concatenate([R, t[:, None]], 1).astype(np.float32)
        Ow = (-R.T.astype(np.float64) @ t).astype(np.float32)
        X = (rng.normal(size=3) * 3).astype(np.float32)
        nrm = rng.normal(size=3).astype(np.float32)
        cam = rand_cam(rng)
        bf = np.float32(rng.uniform(20, 60))
        orc.oracle_fp_frustum_vals(fp(*T.ravel()), fp(*Ow), fp(*cam), C.c_float(bf), fp(*X), fp(*nrm), out)
        Pc = np.array(out[:3], np.float32)
        u = call_site(ref_lib, "proj", list(cam) + list(Pc), 2)[0]
        PO = (X - Ow).astype(np.float32)
        d2 = orc.oracle_fp_norm2(fp(*PO))
        r = call_site(ref_lib, "frustum", list(X) + list(R.ravel()) + list(t) + list(Ow) + [bf, u] + list(nrm) + [d2], 7)
        # order: Pc0..2, Pc_dist, viewCos, ur, dist
        assert same(r[:4], out[:4]), (r[:4], out[:4])
        assert same([r[6]], [out[4]]) and same([r[4]], [out[5]]) and same([r[5]], [out[6]]), (r, out[:])


def test_projection_stereo_gates(ref_lib, orc):
    rng = np.random.default_rng(4)
    orc.oracle_fp_sbp_er.restype = C.c_float
    orc.oracle_fp_sbp_er.argtypes = [C.c_float] * 4
    orc.oracle_fp_fuse_e2.restype = C.c_double
    orc.oracle_fp_fuse_e2.argtypes = [C.c_float] * 8
    for _ in range(N):
        u, v, kpx, kpy, kpr = rng.uniform(0, 752, 5).astype(np.float32)
        bf = np.float32(rng.uniform(20, 60))
        invz = np.float32(1.0) / np.float32(rng.uniform(0.3, 30))
        isg = np.float32(1 / 1.44 ** rng.integers(0, 8))
        r = call_site(ref_lib, "sbp_er", [u, bf, invz, kpr], 1)
        assert same(r, [orc.oracle_fp_sbp_er(u, bf, invz, kpr)])
        r = call_site(ref_lib, "fuse_e2", [u, v, kpx, kpy, kpr, bf, invz, isg, u], 1)
        assert same(r, [orc.oracle_fp_fuse_e2(u, v, kpx, kpy, kpr, bf, invz, isg)])


def test_orb_descriptor_rotation(ref_lib, orc):
    rng = np.random.default_rng(5)
    r, c = C.c_int(), C.c_int()
    orc.oracle_orb_sample_rc.argtypes = [C.c_float] * 4 + [C.POINTER(C.c_int)] * 2
    for _ in range(N * 4):
        th = np.float32(rng.uniform(0, 360)) * np.float32(np.pi / 180)
        a, b = np.float32(np.cos(th)), np.float32(np.sin(th))
        x, y = (int(v) for v in rng.integers(-15, 16, 2))
        ref = call_site(ref_lib, "orb_rc", [a, b, x, y], 2)
        orc.oracle_orb_sample_rc(float(x), float(y), float(a), float(b), C.byref(r), C.byref(c))
        assert list(ref) == [r.value, c.value], (ref, r.value, c.value)


# ---- round 4: the remaining float sites of the path (second part)

def test_ctor_scale_tables(ref_lib):
    """ORBextractor ctor tables (ORBextractor.cc:408-468): mvScaleFactor / mvLevelSigma2 through the
    object's own step (float -> double product -> float), their inverses, and the per-level
    feature split (factor = (float)(1 / (double)scaleFactor), pow in double, cvRound per level)."""
    import oracle_bind as ob
    rng = np.random.default_rng(11)
    for _ in range(400):
        sf = np.float32(rng.uniform(1.05, 2.2))
        L = int(rng.integers(1, 13))
        nf = int(rng.integers(100, 6000))
        sc_, inv_, sig_, isig_, nfeat_ = ob.levels(ob.params(nfeatures=nf, scale=float(sf), nlevels=L))
        t = dict(scale=sc_, inv_scale=inv_, sigma2=sig_, inv_sigma2=isig_, nfeat=nfeat_)
        scale, sig = [np.float32(1)], [np.float32(1)]
        for i in range(1, L):
            r = call_site(ref_lib, "ctor_scale", [float(sf), float(scale[-1])], 2)
            scale.append(np.float32(r[0]))
            sig.append(np.float32(r[1]))
        assert same(t["scale"], scale) and same(t["sigma2"], sig), (sf, L)
        assert same(t["inv_scale"], np.float32(1) / np.array(scale, np.float32))
        assert same(t["inv_sigma2"], np.float32(1) / np.array(sig, np.float32))
        factor = np.float32(call_site(ref_lib, "ctor_nfeat", [float(sf), nf, 1.0, 0.0], 2)[0])
        per = np.float32(call_site(ref_lib, "ctor_nfeat", [float(sf), nf, 1.0, math.pow(float(factor), L)], 2)[1])
        want, total = [], 0
        for _l in range(L - 1):  # :436-441: vcvtss2si (round half even), then per *= factor
            want.append(int(np.rint(per)))
            total += want[-1]
            per = np.float32(per * factor)
        want.append(max(nf - total, 0))
        assert list(t["nfeat"]) == want, (sf, L, nf)


def test_umax_constants(ref_lib, orc):
    """umax[0..11] are constants the compiler folded (cvRound of sqrt(225 - v^2)); the rest follow
    the reference's symmetric integer loop (ORBextractor.cc:452-467)."""
    ref = [int(v) for v in call_site(ref_lib, "umax", [], 12)]
    out = (C.c_int * 16)()
    orc.oracle_fp_umax(out)
    assert list(out[:12]) == ref, (list(out), ref)
    um = ref + [0] * 4
    v0 = 0
    for v in range(15, 10, -1):  # vmin = cvCeil(15 * sqrt(2) / 2) = 11
        while um[v0] == um[v0 + 1]:
            v0 += 1
        um[v] = v0
        v0 += 1
    assert list(out) == um


def test_pyramid_level_sizes(ref_lib, orc):
    import oracle_bind as ob
    out = (C.c_int * 2)()
    rng = np.random.default_rng(12)
    for _ in range(N):
        w, h = int(rng.integers(16, 4096)), int(rng.integers(16, 4096))
        inv = np.float32(1) / np.float32(np.float32(rng.uniform(1.05, 2.2)) ** int(rng.integers(0, 12)))
        r = call_site(ref_lib, "pyr_size", [h, w, inv], 2)  # cv::Mat rows at +0x8, cols at +0xc
        orc.oracle_fp_level_size(w, h, C.c_float(inv), out)
        assert [out[1], out[0]] == [int(r[0]), int(r[1])], (w, h, inv, list(out), r)
    for sf in (1.2, 1.5, 2.0):  # the standard geometries through the whole table
        inv_scales = ob.levels(ob.params(scale=sf))[1]
        for w, h in ((752, 480), (640, 480), (1241, 376), (1280, 720)):
            for inv in inv_scales:
                r = call_site(ref_lib, "pyr_size", [h, w, float(inv)], 2)
                orc.oracle_fp_level_size(w, h, C.c_float(inv), out)
                assert [out[1], out[0]] == [int(r[0]), int(r[1])]


def test_keypoint_scaling(ref_lib, orc):
    rng = np.random.default_rng(13)
    out = (C.c_float * 2)()
    for _ in range(N):
        x, y = rng.uniform(0, 800, 2).astype(np.float32)
        s = np.float32(np.float32(1.2) ** int(rng.integers(1, 8)))
        r = call_site(ref_lib, "kp_scale", [x, y, s], 2)
        orc.oracle_fp_kp_scale(C.c_float(x), C.c_float(y), C.c_float(s), out)
        assert same(r, out[:2])


def test_pos_in_grid_and_area_cells(ref_lib, orc):
    """Frame::PosInGrid (roundf, then truncation) and GetFeaturesInArea's cell range (floorf /
    ceilf of the scaled box), incl. values on the .5 rounding boundaries."""
    rng = np.random.default_rng(14)
    pg, ac = (C.c_int * 2)(), (C.c_int * 4)()
    for i in range(N * 2):
        minx, miny = np.float32(rng.uniform(-5, 5, 2).astype(np.float32))
        maxx, maxy = np.float32(minx + rng.uniform(600, 1300)), np.float32(miny + rng.uniform(400, 800))
        iw = np.float32(np.float32(64) / np.float32(maxx - minx))
        ih = np.float32(np.float32(48) / np.float32(maxy - miny))
        if i % 4 == 0:  # exactly on a half cell
            x = np.float32(minx + (np.float32(rng.integers(0, 64)) + np.float32(0.5)) / iw)
            y = np.float32(miny + (np.float32(rng.integers(0, 48)) + np.float32(0.5)) / ih)
        else:
            x = np.float32(rng.uniform(minx - 20, maxx + 20))
            y = np.float32(rng.uniform(miny - 20, maxy + 20))
        r = call_site(ref_lib, "pos_in_grid", [x, y, minx, iw, miny, ih], 2)
        orc.oracle_fp_pos_in_grid(*(C.c_float(v) for v in (x, y, minx, miny, iw, ih)), pg)
        assert list(pg) == [int(v) for v in r], (x, y, list(pg), r)
        rad = np.float32(rng.uniform(1, 100))
        r = call_site(ref_lib, "area_cells", [x, y, rad, minx, miny, iw, ih], 4)
        orc.oracle_fp_area_cells(*(C.c_float(v) for v in (x, y, rad, minx, miny, iw, ih)), ac)
        assert list(ac) == [int(v) for v in r], (x, y, rad, list(ac), r)


def test_rotation_bins(ref_lib, orc):
    """rotHist bin of a match: roundf((a - b [+360]) * (1/30)), 30 -> 0 (ORBmatcher.cc:391-396), for
    both oracle copies (SearchByBoW's and the projection matchers'), incl. angles that land on
    bin edges."""
    orc.oracle_fp_rot_bin_bow.argtypes = [C.c_float] * 2
    orc.oracle_fp_rot_bin_proj.argtypes = [C.c_float] * 2
    rng = np.random.default_rng(15)
    for i in range(N * 4):
        a = np.float32(rng.uniform(0, 360))
        b = np.float32(a - np.float32(15 * rng.integers(-24, 24) + (0 if i % 3 else rng.uniform(-1e-3, 1e-3))))
        if i % 2:
            b = np.float32(rng.uniform(0, 360))
        rot = np.float32(a - b)
        r = int(call_site(ref_lib, "rot_neg" if rot < 0 else "rot_pos", [a, b], 1)[0])
        r = 0 if r == 30 else r
        assert orc.oracle_fp_rot_bin_bow(a, b) == r and orc.oracle_fp_rot_bin_proj(a, b) == r, (a, b, r)


def test_search_radius(ref_lib, orc):
    orc.oracle_fp_search_radius.restype = C.c_float
    orc.oracle_fp_search_radius.argtypes = [C.c_float] * 2
    rng = np.random.default_rng(16)
    for _ in range(N):
        th = np.float32(rng.choice([7, 14, 15, 3, 1, 10, rng.uniform(0.5, 30)]))
        s = np.float32(np.float32(rng.uniform(1.05, 2.2)) ** int(rng.integers(0, 8)))
        r = call_site(ref_lib, "sbp_radius", [s, th], 1)
        assert same(r, [orc.oracle_fp_search_radius(th, s)])


def test_lba_robust_constants(orc):
    """LocalBundleAdjustment's Huber deltas as setDelta receives them (float sqrt widened to double:
    Optimizer.cc.o .LC116 at 0x1b005 / 0x1b799 mono, .LC101 at 0x1b580 stereo) and the outlier
    thresholds it compares chi2 with (.LC105 5.991 at 0x1b2ca, .LC106 7.815 at 0x1ba6c)."""
    import struct
    import fptrace
    obj = str(OBJ / "Optimizer.cc.o")
    tr = fptrace.Tracer(obj, {})
    rel = {a: r for a, _i, _o, r in fptrace.read_range(obj, None, "0x1a270", "0x1d800")}
    val = lambda addr: struct.unpack("<d", tr.const_bytes(rel[addr], 8))[0]  # noqa: E731
    ref = [val(0x1b005), val(0x1b580), val(0x1b2ca), val(0x1ba6c)]
    assert val(0x1b799) == ref[0]
    out = (C.c_double * 4)()
    orc.oracle_fp_lba_consts(out)
    assert list(out) == ref, (list(out), ref)
