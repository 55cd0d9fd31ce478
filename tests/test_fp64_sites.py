"""The oracle's FP64 optimizer arithmetic vs the reference binary's own data flow (round 5).

LocalBundleAdjustment's and PoseOptimization's decisions -- the outlier gates `e->chi2() > 5.991 /
7.815` (Optimizer.cc:1992-2038, 1026-1090), LM's rho (the robust chi2 sum) and the steps -- rest on
the edges' computeError / linearizeOplus, Pinhole::project / projectJac, BaseEdge::chi2 and the
Huber kernel as GCC 9.3 compiled them (-O3 -march=native: FMA contractions inside Eigen's
expressions).  tools/disasm/fptrace.py (packed mode) reads the reference's ORB_SLAM3 and g2o
objects as DATA and emits each site as C; that C is built into oracle/_ref/libfp64ref.so
(git-ignored; nothing from the reference is executed or linked) and compared bit for bit with the
oracle's restatement (oracle/g2o_sites.hpp, the functions lba_oracle.cpp / pose_oracle.cpp call)
on seeded inputs.  Sites whose value flows through an out-of-line call (the edges call
_transformVector, Pinhole::project / projectJac, cam_project) are traced separately and composed
here exactly as the call passes the values.  A CPU test that needs /root/reference (build
container only); the kernels are held to the oracle by the -m gpu LBA / pose tests.
"""
from __future__ import annotations

import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
O = REF / "evaluation/CMakeFiles/ORB_SLAM3.dir/src"
G = REF / "Thirdparty/g2o/build/CMakeFiles/g2o.dir/g2o"
pytestmark = pytest.mark.skipif(not O.exists(), reason="reference objects exist only in the build container")

sys.path.insert(0, str(ROOT / "tools" / "disasm"))

TV_SEC = "@.text._ZNK5Eigen14QuaternionBaseINS_10QuaternionIdLi0EEEE16_transformVectorERKNS_6MatrixIdLi3ELi1ELi0ELi3ELi1EEE"
V1 = "*(*(arg_rdi+0x8)+0x8)"   # _vertices[1] (the pose of a binary edge)
V0 = "*(*(arg_rdi+0x8)+0x0)"   # _vertices[0] (the pose of a unary OnlyPose edge)
Q = lambda v: [f"{v}+0x{o:x}" for o in (0xc0, 0xc8, 0xd0, 0xd8)]   # noqa: E731 SE3Quat rotation x, y, z, w
TV = [f"_transformVector#1.out[{k}]" for k in (0, 2, 4)]
F32 = [f"*(arg_rsi+0x10)+0x{o:x}" for o in (0x0, 0x4, 0x8, 0xc)]  # Pinhole mvParameters fx, fy, cx, cy
XD = ["arg_rdx+0x0", "arg_rdx+0x8", "arg_rdx+0x10"]
ST = lambda base, offs: [(f"store:{base}+0x{o:x}", 0) for o in offs]  # noqa: E731
# Eigen column-major offsets of a 2x3 / 2x6 / 3x3 / 3x6 matrix, read back row-major
CM = lambda R, Cn: [8 * (r + R * c) for r in range(R) for c in range(Cn)]  # noqa: E731
PJ = [f"*0x50#2.out[{k}]" for k in (0, 4, 8, 2, 6, 10)]  # projectJac 2x3 (sret, column-major) row-major

# name -> (object, ranges, inputs, outputs[, f64 entry registers])
SITES = {
    # Eigen::QuaternionBase::_transformVector, the out-of-line COMDAT of both objects
    "tv": (O / "OptimizableTypes.cpp.o", ["0x0:0xb9" + TV_SEC], [f"arg_rsi+0x{8 * k:x}" for k in range(4)] + XD,
           ST("arg_rdi", (0, 8, 0x10))),
    "tv_g2o": (G / "types/types_six_dof_expmap.cpp.o", ["0x0:0xb9" + TV_SEC],
               [f"arg_rsi+0x{8 * k:x}" for k in range(4)] + XD, ST("arg_rdi", (0, 8, 0x10))),
    # Pinhole::project(const Eigen::Vector3d&), Pinhole::projectJac(const Eigen::Vector3d&)
    "proj": (O / "CameraModels/Pinhole.cpp.o", ["0x40:0x87"], F32 + XD, ST("arg_rdi", (0, 8))),
    "projjac": (O / "CameraModels/Pinhole.cpp.o", ["0xe0:0x165"], F32 + XD, ST("arg_rdi", (0x0, 0x20, 0x18, 0x28))),
    # ORB_SLAM3::EdgeSE3ProjectXYZ::computeError around its two calls: Xc = t + tv, err = obs - proj
    "err_mono": (O / "OptimizableTypes.cpp.o", ["0x0:0xae@.text._ZN9ORB_SLAM317EdgeSE3ProjectXYZ12computeErrorEv"],
                 [f"{V1}+0xe0", f"{V1}+0xe8", f"{V1}+0xf0"] + TV + ["arg_rdi+0xa0", "arg_rdi+0xa8",
                                                                 "*%r14#2.out[0]", "*%r14#2.out[2]"],
                 ST("rsp", (0x10, 0x18, 0x20)) + ST("arg_rdi", (0xe0, 0xe8))),
    "err_pose_mono": (O / "OptimizableTypes.cpp.o",
                      ["0x0:0xaa@.text._ZN9ORB_SLAM325EdgeSE3ProjectXYZOnlyPose12computeErrorEv"],
                      [f"{V0}+0xe0", f"{V0}+0xe8", f"{V0}+0xf0"] + TV + ["arg_rdi+0xa0", "arg_rdi+0xa8",
                                                                      "*%r14#2.out[0]", "*%r14#2.out[2]"],
                      ST("rsp", (0x10, 0x18, 0x20)) + ST("arg_rdi", (0xe0, 0xe8))),
    # g2o::EdgeStereoSE3ProjectXYZ::computeError + cam_project (LocalBundleAdjustment's stereo edges)
    "err_stereo": (G / "types/types_six_dof_expmap.cpp.o", ["0x0:0xf1@.text._ZN3g2o23EdgeStereoSE3ProjectXYZ12computeErrorEv"],
                   [f"{V1}+0xe0", f"{V1}+0xe8", f"{V1}+0xf0"] + TV + ["arg_rdi+0xa0", "arg_rdi+0xa8", "arg_rdi+0xb0",
                                                                   "arg_rdi+0x180"]
                   + [f"cam_project#2.out[{k}]" for k in (0, 2, 4)],
                   ST("rsp", (0x30, 0x38, 0x40)) + [("store:rsp+0x2c", 0)] + ST("arg_rdi", (0x100, 0x108, 0x110))),
    "cam_stereo": (G / "types/types_six_dof_expmap.cpp.o", ["0xb90:0xbf9"],
                   XD + [f"arg_rsi+0x{o:x}" for o in (0x160, 0x168, 0x170, 0x178)] + ["arg_rcx+0x0"],
                   ST("arg_rdi", (0, 8, 0x10))),
    # g2o::EdgeStereoSE3ProjectXYZOnlyPose::computeError (its _transformVector inlined) + cam_project
    "err_pose_stereo": (G / "types/types_six_dof_expmap.cpp.o",
                        ["0x0:0x161@.text._ZN3g2o31EdgeStereoSE3ProjectXYZOnlyPose12computeErrorEv"],
                        Q(V0) + [f"{V0}+0xe0", f"{V0}+0xe8", f"{V0}+0xf0", "arg_rdi+0x128", "arg_rdi+0x130",
                                 "arg_rdi+0x138", "arg_rdi+0xa0", "arg_rdi+0xa8", "arg_rdi+0xb0"]
                        + [f"cam_project#1.out[{k}]" for k in (0, 2, 4)],
                        [(f"laststore:rsp+0x{o:x}", 0) for o in (0x20, 0x28, 0x30)] + ST("arg_rdi", (0x100, 0x108, 0x110))),
    "cam_pose_stereo": (G / "types/types_six_dof_expmap.cpp.o", ["0xc90:0xcef"],
                        XD + [f"arg_rsi+0x{o:x}" for o in (0x140, 0x148, 0x150, 0x158, 0x160)],
                        ST("arg_rdi", (0, 8, 0x10))),
    # g2o::BaseEdge<2> / <3>::chi2 (the copies LocalBundleAdjustment and PoseOptimization call)
    "chi2_2": (O / "Optimizer.cc.o", ["0x0:0x36@.text._ZNK3g2o8BaseEdgeILi2EN5Eigen6MatrixIdLi2ELi1ELi0ELi2ELi1EEEE4chi2Ev"],
               [f"arg_rdi+0x{o:x}" for o in (0xc0, 0xc8, 0xd0, 0xd8, 0xe0, 0xe8)], [("ret", 0)]),
    "chi2_3": (O / "Optimizer.cc.o", ["0x0:0x76@.text._ZNK3g2o8BaseEdgeILi3EN5Eigen6MatrixIdLi3ELi1ELi0ELi3ELi1EEEE4chi2Ev"],
               [f"arg_rdi+0x{0xb8 + 8 * k:x}" for k in range(9)] + ["arg_rdi+0x100", "arg_rdi+0x108", "arg_rdi+0x110"],
               [("ret", 0)]),
    # LocalBundleAdjustment's final stereo outlier scan: the chi2 inlined at @0x1b9ff (speculative
    # devirtualisation), compared with 7.815
    "chi2_3_scan": (O / "Optimizer.cc.o", ["0x1b9ff:0x1ba74"],
                    [f"arg_rbx+0x{0xb8 + 8 * k:x}" for k in range(9)] + ["arg_rbx+0x100", "arg_rbx+0x108",
                                                                      "arg_rbx+0x110"],
                    [("cmp#0", 0)]),
    # g2o::RobustKernelHuber::robustify, the e > dsqr branch
    "huber": (G / "core/robust_kernel_impl.cpp.o", ["0x350:0x365", "0x380:0x3c3"],
              ["%xmm0", "arg_rdi+0x8", "arg_rdi+0x10"], ST("arg_rsi", (0, 8)), ["xmm0"]),
    # linearizeOplus bodies
    "lin_mono": (O / "OptimizableTypes.cpp.o", ["0x1840:0x1b7c"],
                 Q(V1) + [f"{V1}+0xe0", f"{V1}+0xe8", "rsp+0xd0"] + TV + PJ,
                 [(f"store:*(arg_rdi+0x118)+0x{o:x}", 0) for o in CM(2, 3)]
                 + [(f"store:*(arg_rdi+0x128)+0x{o:x}", 0) for o in CM(2, 6)]),
    "lin_pose_mono": (O / "OptimizableTypes.cpp.o", ["0x1630:0x1835"],
                      [f"{V0}+0xe0", f"{V0}+0xe8", f"{V0}+0xf0"] + TV + PJ,
                      [(f"store:*(arg_rdi+0xf0)+0x{o:x}", 0) for o in CM(2, 6)]),
    "lin_stereo": (G / "types/types_six_dof_expmap.cpp.o", ["0xcf0:0x1105"],
                   Q(V1) + [f"{V1}+0xe0", f"{V1}+0xe8", "rsp+0x70"] + TV
                   + ["arg_rdi+0x160", "arg_rdi+0x168", "arg_rdi+0x180"],
                   [(f"store:*(arg_rdi+0x140)+0x{o:x}", 0) for o in CM(3, 3)]
                   + [(f"store:*(arg_rdi+0x150)+0x{o:x}", 0) for o in CM(3, 6) if o not in (0x60, 0x50, 0x70)]),
    "lin_pose_stereo": (G / "types/types_six_dof_expmap.cpp.o", ["0x1280:0x1430"],
                        [f"{V0}+0xe0", f"{V0}+0xe8", f"{V0}+0xf0"] + TV
                        + ["arg_rdi+0x140", "arg_rdi+0x148", "arg_rdi+0x160"],
                        [(f"store:*(arg_rdi+0x118)+0x{o:x}", 0) for o in CM(3, 6) if o not in (0x60, 0x50, 0x70)]),
}

# round 6: SE3Quat products (the body edge, oplusImpl), SE3Quat::exp, EdgeSE3ProjectXYZToBody
BODY_ERR = "@.text._ZN9ORB_SLAM323EdgeSE3ProjectXYZToBody12computeErrorEv"
OPLUS = "@.text._ZN3g2o15VertexSE3Expmap9oplusImplEPKd"
EXP = "@.text._ZN3g2o7SE3Quat3expERKN5Eigen6MatrixIdLi6ELi1ELi0ELi6ELi1EEE"
TRL_Q = [f"arg_rdi+0x{o:x}" for o in (0x140, 0x148, 0x150, 0x158)]   # mTrl rotation x, y, z, w
PJC = lambda k: [f"*0x50#{k}.out[{j}]" for j in (0, 4, 8, 2, 6, 10)]  # noqa: E731 projectJac row-major
_PQ = [f"arg_r12+0x{o:x}" for o in (0xc0, 0xc8, 0xd0, 0xd8)]
_OPLUS_IN = ([f"rsp+0x{o:x}" for o in (0x80, 0x88, 0x90, 0x98)] + _PQ + ["rsp+0xa0", "rsp+0xa8", "rsp+0xb0"]
             + [f"_transformVector#1.out[{k}]" for k in (0, 2, 4)])
_OPLUS_OUT = ST("arg_r12", (0xc0, 0xc8, 0xd0, 0xd8, 0xe0, 0xe8, 0xf0))
_EXP_OUT = [(f"laststore:arg_rdi+0x{o:x}", 0) for o in (0, 8, 0x10, 0x18)] + ST("arg_rdi", (0x20, 0x28)) \
    + [("store:rsp-0x190", 0)]
SITES.update({
    # VertexSE3Expmap::oplusImpl after its SE3Quat::exp call: exp(update) * estimate, w >= 0 (the
    # branch skipped) and w < 0 (the negation taken: the range runs straight through it)
    "oplus_mul": (O / "OptimizableTypes.cpp.o", ["0x62:0x152" + OPLUS, "0x15a:0x1b0" + OPLUS], _OPLUS_IN, _OPLUS_OUT),
    "oplus_mul_neg": (O / "OptimizableTypes.cpp.o", ["0x62:0x1b0" + OPLUS], _OPLUS_IN, _OPLUS_OUT),
    # SE3Quat::exp: theta >= 1e-5 (sincos / pow) and the small-angle branch, positive-trace quaternion
    "exp_large": (O / "OptimizableTypes.cpp.o",
                  [a + EXP for a in ("0x0:0xe6", "0x4b8:0x8f6", "0x264:0x2b4", "0x948:0x955", "0x95b:0x9b8",
                                     "0x406:0x442", "0x448:0x469", "0x46b:0x482")],
                  [f"arg_rsi+0x{8 * k:x}" for k in range(6)], _EXP_OUT),
    "exp_small": (O / "OptimizableTypes.cpp.o",
                  [a + EXP for a in ("0x0:0xe6", "0xec:0x2b4", "0x948:0x955", "0x95b:0x9b8", "0x406:0x442",
                                     "0x448:0x469", "0x46b:0x482")],
                  [f"arg_rsi+0x{8 * k:x}" for k in range(6)], _EXP_OUT),
    # ORB_SLAM3::EdgeSE3ProjectXYZToBody::computeError: (mTrl * T).map(X), project, obs - proj
    "err_body": (O / "OptimizableTypes.cpp.o", ["0x0:0x166" + BODY_ERR, "0x174:0x20f" + BODY_ERR],
                 TRL_Q + ["arg_rdi+0x160", "arg_rdi+0x168", "rsp+0x90"] + Q(V1)
                 + [f"_transformVector#1.out[{k}]" for k in (0, 2, 4)]
                 + [f"_transformVector#2.out[{k}]" for k in (0, 2, 4)]
                 + ["arg_rdi+0xa0", "arg_rdi+0xa8", "*%r14#3.out[0]", "*%r14#3.out[2]"],
                 [(f"laststore:rsp+0x{o:x}", 0) for o in (0x60, 0x68, 0x70, 0x78)] + ST("rsp", (0x80, 0x88, 0x90))
                 + ST("rsp", (0x20, 0x28, 0x30)) + ST("arg_rdi", (0xe0, 0xe8))),
    # ORB_SLAM3::EdgeSE3ProjectXYZToBody::linearizeOplus (@0xf30), the product's w >= 0 branch
    "lin_body": (O / "OptimizableTypes.cpp.o", ["0xf30:0x1076", "0x1087:0x1605"],
                 TRL_Q + ["arg_rdi+0x160", "arg_rdi+0x168", "arg_rdi+0x170"] + Q(V1)
                 + [f"{V1}+0xe0", f"{V1}+0xe8", "rsp+0x130"]
                 + [f"_transformVector#{c}.out[{k}]" for c in (2, 3, 4) for k in (0, 2, 4)] + PJC(5) + PJC(6),
                 [(f"store:*(arg_rdi+0x118)+0x{o:x}", 0) for o in CM(2, 3)]
                 + [(f"store:*(arg_rdi+0x128)+0x{o:x}", 0) for o in CM(2, 6)]),
})
NOUT = {k: len(v[3]) for k, v in SITES.items()}


@pytest.fixture(scope="module")
def ref():
    import fptrace
    out = ROOT / "oracle" / "_ref"
    out.mkdir(parents=True, exist_ok=True)
    src = ["#include <math.h>"]
    for name, site in SITES.items():
        obj, ranges, ins, outs = site[:4]
        tr = fptrace.trace(str(obj), ranges, packed=True, f64_regs=site[4] if len(site) > 4 else ())
        src.append(fptrace.emit_c(tr, f"site_{name}", ins, outs))
    (out / "fp64_sites_ref.c").write_text("\n\n".join(src) + "\n")
    so = out / "libfp64ref.so"
    subprocess.run(["gcc", "-O1", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so),
                    str(out / "fp64_sites_ref.c"), "-lm"], check=True)
    L = C.CDLL(str(so))
    for name in SITES:
        getattr(L, f"site_{name}").argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double)]
    return L


@pytest.fixture(scope="module")
def orc():
    import oracle_bind as ob
    L = ob.lib()
    D, Fp = C.POINTER(C.c_double), C.POINTER(C.c_float)
    for n, a in {"tv": [D, D, D], "map": [D, D, D, D], "project": [D, D, D], "neg_project_jac": [Fp, D, D],
                 "rot": [D, D], "lin_mono": [D, D, D, Fp, D, D], "lin_pose_mono": [D, D, D, Fp, D],
                 "lin_stereo": [D, D, D, C.c_double, C.c_double, C.c_double, D, D],
                 "lin_pose_stereo": [D, D, D, C.c_double, C.c_double, C.c_double, D],
                 "cam_stereo": [D] + [C.c_double] * 4 + [C.c_float, D],
                 "cam_pose_stereo": [D] + [C.c_double] * 5 + [D],
                 "chi2_2": [D, C.c_double], "chi2_3": [D, C.c_double],
                 "huber": [C.c_double, C.c_double, C.c_float, D],
                 "se3_mul": [D, D, D, D, D], "se3_exp": [D, D], "body_error": [D, D, D, D, D, D, D, D],
                 "lin_body": [D, D, D, D, D, Fp, D, D]}.items():
        f = getattr(L, f"oracle_fp64_{n}")
        f.argtypes = a
        f.restype = C.c_double if n.startswith("chi2") else None
    return L


def site(L, name, ins):
    a = (C.c_double * max(1, len(ins)))(*[float(v) for v in ins])
    o = (C.c_double * NOUT[name])()
    getattr(L, f"site_{name}")(a, o)
    return np.array(o[:], np.float64)


def dv(*v):
    return (C.c_double * len(v))(*[float(x) for x in v])


def out(n):
    return (C.c_double * n)()


def same(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b)


N = 3000


def rand_pose(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    if q[3] < 0:
        q = -q
    return q, rng.normal(size=3) * rng.uniform(0.1, 5)


def rand_point(rng, q, t):
    """A world point in front of the camera (Xc.z in [0.2, 40])."""
    from scipy.spatial.transform import Rotation
    R = Rotation.from_quat(q).as_matrix()
    Xc = np.array([rng.uniform(-8, 8), rng.uniform(-6, 6), rng.uniform(0.2, 40)])
    return R.T @ (Xc - t)


def rand_cam(rng):
    return np.array([rng.uniform(300, 800), rng.uniform(300, 800), rng.uniform(200, 500), rng.uniform(150, 350)],
                    np.float32)


def test_transform_vector(ref, orc):
    rng = np.random.default_rng(51)
    o = out(3)
    for _ in range(N):
        q, _t = rand_pose(rng)
        v = rng.normal(size=3) * rng.uniform(0.01, 50)
        r = site(ref, "tv", list(q) + list(v))
        assert same(r, site(ref, "tv_g2o", list(q) + list(v)))  # the g2o object's copy is the same code
        orc.oracle_fp64_tv(dv(*q), dv(*v), o)
        assert same(r, o[:]), (r, o[:])


def test_project_and_jacobian(ref, orc):
    rng = np.random.default_rng(52)
    uv, n = out(2), out(6)
    for _ in range(N):
        K = rand_cam(rng)
        X = np.array([rng.normal() * 5, rng.normal() * 5, rng.uniform(0.1, 50)])
        r = site(ref, "proj", list(K) + list(X))
        orc.oracle_fp64_project(dv(*K.astype(np.float64)), dv(*X), uv)
        assert same(r, uv[:])
        j = site(ref, "projjac", list(K) + list(X))  # J00, J02, J11, J12
        orc.oracle_fp64_neg_project_jac((C.c_float * 2)(*K[:2]), dv(*X), n)
        assert same(-j, [n[0], n[2], n[4], n[5]]) and n[1] == 0 and n[3] == 0


def _mono_error(ref, name, t, tv, obs, K):
    """computeError of a mono edge composed from its sites: Xc from the edge body, project(Xc) from
    Pinhole.cpp.o, then err = obs - proj from the edge body."""
    Xc = site(ref, name, list(t) + list(tv) + list(obs) + [0, 0])[:3]
    p = site(ref, "proj", list(K) + list(Xc))
    r = site(ref, name, list(t) + list(tv) + list(obs) + list(p))
    assert same(r[:3], Xc)
    return Xc, r[3:]


def test_edge_errors_mono(ref, orc):
    """EdgeSE3ProjectXYZ (LBA) and EdgeSE3ProjectXYZOnlyPose (PoseOptimization) computeError."""
    rng = np.random.default_rng(53)
    xo, uv = out(3), out(2)
    for _ in range(N):
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        K = rand_cam(rng)
        obs = rng.uniform(0, 752, 2)
        tv = site(ref, "tv", list(q) + list(X))
        for name in ("err_mono", "err_pose_mono"):
            Xc, err = _mono_error(ref, name, t, tv, obs, K)
            orc.oracle_fp64_map(dv(*q), dv(*t), dv(*X), xo)
            assert same(Xc, xo[:]), (name, Xc, xo[:])
            orc.oracle_fp64_project(dv(*K.astype(np.float64)), xo, uv)
            assert same(err, obs - np.array(uv[:])), name


def test_edge_errors_stereo(ref, orc):
    """g2o::EdgeStereoSE3ProjectXYZ (LBA) and EdgeStereoSE3ProjectXYZOnlyPose (PoseOptimization)."""
    rng = np.random.default_rng(54)
    xo, p = out(3), out(3)
    for _ in range(N):
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        K = rand_cam(rng).astype(np.float64)
        bf = float(np.float32(rng.uniform(20, 60)))
        obs = list(rng.uniform(0, 752, 2)) + [rng.uniform(0, 752)]
        tv = site(ref, "tv", list(q) + list(X))
        r0 = site(ref, "err_stereo", list(t) + list(tv) + obs + [bf, 0, 0, 0])
        Xc, bff = r0[:3], r0[3]
        pr = site(ref, "cam_stereo", list(Xc) + list(K) + [bff])
        r = site(ref, "err_stereo", list(t) + list(tv) + obs + [bf] + list(pr))
        orc.oracle_fp64_map(dv(*q), dv(*t), dv(*X), xo)
        assert same(Xc, xo[:])
        orc.oracle_fp64_cam_stereo(xo, *K, C.c_float(np.float32(bf)), p)
        assert same(pr, p[:]) and same(r[4:], np.array(obs) - np.array(p[:]))
        # OnlyPose: the world point is the edge's Xw
        r0 = site(ref, "err_pose_stereo", list(q) + list(t) + list(X) + obs + [0, 0, 0])
        Xc = r0[:3]
        pr = site(ref, "cam_pose_stereo", list(Xc) + list(K) + [bf])
        r = site(ref, "err_pose_stereo", list(q) + list(t) + list(X) + obs + list(pr))
        assert same(Xc, xo[:])
        orc.oracle_fp64_cam_pose_stereo(xo, *K, bf, p)
        assert same(pr, p[:]) and same(r[3:], np.array(obs) - np.array(p[:]))


def test_chi2(ref, orc):
    rng = np.random.default_rng(55)
    for _ in range(N * 2):
        info = float(np.float32(1.0 / 1.44 ** rng.integers(0, 8)))
        e = rng.normal(size=3) * rng.uniform(0.01, 10)
        I2 = [info, 0.0, 0.0, info]  # Information = I * invSigma2, column-major
        assert same([site(ref, "chi2_2", I2 + list(e[:2]))[0]], [orc.oracle_fp64_chi2_2(dv(*e[:2]), info)])
        I3 = [info, 0, 0, 0, info, 0, 0, 0, info]
        c3 = orc.oracle_fp64_chi2_3(dv(*e), info)
        assert same([site(ref, "chi2_3", I3 + list(e))[0]], [c3])
        assert same([site(ref, "chi2_3_scan", I3 + list(e))[0]], [c3])


def test_chi2_gate_kats(ref, orc):
    """Errors on the stereo gate (7.815) where the contracted chi2 and the plain sum decide
    differently: the oracle must decide like the object."""
    rng = np.random.default_rng(56)
    found = 0
    for _ in range(200000):
        info = float(np.float32(1.0 / 1.44 ** rng.integers(0, 8)))
        d = rng.normal(size=3)
        e = d / np.sqrt((d * d).sum() * info) * np.sqrt(7.815)  # chi2 ~= 7.815
        naive = e[0] * (info * e[0]) + e[1] * (info * e[1]) + e[2] * (info * e[2])
        c3 = orc.oracle_fp64_chi2_3(dv(*e), info)
        if (naive > 7.815) == (c3 > 7.815):
            continue
        I3 = [info, 0, 0, 0, info, 0, 0, 0, info]
        r = site(ref, "chi2_3_scan", I3 + list(e))[0]
        assert same([r], [c3]) and (r > 7.815) == (c3 > 7.815)
        found += 1
        if found >= 20:
            break
    assert found >= 20


def test_huber(ref, orc):
    rng = np.random.default_rng(57)
    rho = out(2)
    for _ in range(N):
        delta = float(np.float32(np.sqrt(rng.choice([5.991, 7.815]))))
        dsqr = np.float32(delta * delta)
        e = float(dsqr) * rng.uniform(1.0001, 50)
        r = site(ref, "huber", [e, delta, dsqr])
        orc.oracle_fp64_huber(e, delta, C.c_float(dsqr), rho)
        assert same(r, rho[:]), (r, rho[:])


def _pj(ref, K, Xc):
    j = site(ref, "projjac", list(K) + list(Xc))  # J00, J02, J11, J12 -> sret column-major slots
    return [j[0], 0.0, j[1], 0.0, j[2], j[3]]       # J00, J01, J02, J10, J11, J12 (row-major)


def test_linearize_mono(ref, orc):
    rng = np.random.default_rng(58)
    A, B, xo = out(6), out(12), out(3)
    for _ in range(N):
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        K = rand_cam(rng)
        tv = site(ref, "tv", list(q) + list(X))
        orc.oracle_fp64_map(dv(*q), dv(*t), dv(*X), xo)
        pj = _pj(ref, K, xo[:])
        r = site(ref, "lin_mono", list(q) + list(t) + list(tv) + pj)
        orc.oracle_fp64_lin_mono(dv(*q), dv(*t), dv(*X), (C.c_float * 2)(*K[:2]), A, B)
        assert same(r[:6], A[:]) and same(r[6:], B[:]), (r, A[:], B[:])
        r = site(ref, "lin_pose_mono", list(t) + list(tv) + pj)
        orc.oracle_fp64_lin_pose_mono(dv(*q), dv(*t), dv(*X), (C.c_float * 2)(*K[:2]), B)
        assert same(r, B[:])


def test_linearize_stereo(ref, orc):
    rng = np.random.default_rng(59)
    A, B = out(9), out(18)
    for _ in range(N):
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        fx, fy = (float(np.float32(rng.uniform(300, 800))) for _ in range(2))
        bf = float(np.float32(rng.uniform(20, 60)))
        tv = site(ref, "tv", list(q) + list(X))
        r = site(ref, "lin_stereo", list(q) + list(t) + list(tv) + [fx, fy, bf])
        orc.oracle_fp64_lin_stereo(dv(*q), dv(*t), dv(*X), fx, fy, bf, A, B)
        keep = [i for i in range(18) if i not in (4, 9, 16)]  # the constant zeros are not in the traced range
        assert same(r[:9], A[:]) and same(r[9:], np.array(B[:])[keep]), (r, A[:], B[:])
        r = site(ref, "lin_pose_stereo", list(t) + list(tv) + [fx, fy, bf])
        orc.oracle_fp64_lin_pose_stereo(dv(*q), dv(*t), dv(*X), fx, fy, bf, B)
        assert same(r, np.array(B[:])[keep]) and B[4] == 0 and B[9] == 0 and B[16] == 0


# ---- round 6 -------------------------------------------------------------------------------------

def rand_q(rng, wsign=None):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    if wsign is not None and np.sign(q[3]) != wsign:
        q[3] = -q[3]
    return q


def test_se3_product_oplus(ref, orc):
    """VertexSE3Expmap::oplusImpl's product exp(update) * estimate (quaternion product, normalizeRotation
    with both signs of w, t = a.t + a.r * b.t): the oracle's se3_mul_cc against the object."""
    rng = np.random.default_rng(61)
    o = out(7)
    n_neg = 0
    for _ in range(N):
        a, b = rand_q(rng), rand_q(rng)
        ta, tb = rng.normal(size=3) * 3, rng.normal(size=3) * 3
        tv = site(ref, "tv", list(a) + list(tb))
        orc.oracle_fp64_se3_mul(dv(*a), dv(*ta), dv(*b), dv(*tb), o)
        # the sign of the product's w picks the object's branch: the oracle's own w before normalising
        w = np.fma(-a[2], b[2], np.fma(-b[1], a[1], np.fma(b[3], a[3], -(b[0] * a[0])))) if hasattr(np, "fma") else None
        neg = o[3] < 0 or (w is not None and w < 0)
        r = site(ref, "oplus_mul_neg" if neg else "oplus_mul", list(a) + list(b) + list(ta) + list(tv))
        if not same(r, o[:]):  # w exactly representable near 0: try the other branch before failing
            r = site(ref, "oplus_mul" if neg else "oplus_mul_neg", list(a) + list(b) + list(ta) + list(tv))
            neg = not neg
        n_neg += neg
        assert same(r, o[:]), (r, o[:])
    assert 0 < n_neg < N  # both branches exercised


def test_se3_exp(ref, orc):
    """SE3Quat::exp on LM-sized updates: |omega| from 1e-9 to 0.5 (both sides of the 1e-5 branch)."""
    rng = np.random.default_rng(62)
    o = out(7)
    for k in range(N):
        mag = 10 ** rng.uniform(-9, np.log10(0.5))
        u = list(rng.normal(size=3) / np.sqrt(3) * mag) + list(rng.normal(size=3) * 10 ** rng.uniform(-6, 0))
        theta = np.sqrt(u[0] ** 2 + u[1] ** 2 + u[2] ** 2)
        r = site(ref, "exp_small" if theta < 1e-5 else "exp_large", u)
        orc.oracle_fp64_se3_exp(dv(*u), o)
        assert same(r, o[:]), (k, u, r, o[:])


def test_body_edge_error(ref, orc):
    """EdgeSE3ProjectXYZToBody::computeError: obs - project((mTrl * T).map(X)), composed across its
    _transformVector / Pinhole::project calls."""
    rng = np.random.default_rng(63)
    err = out(2)
    for _ in range(N):
        qrl, trl = rand_q(rng, 1.0), np.array([-0.11, 0.0, 0.0]) + rng.normal(size=3) * 0.01
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        K = rand_cam(rng).astype(np.float64)
        obs = rng.uniform(0, 752, 2)
        tv1 = site(ref, "tv", list(qrl) + list(t))
        base = list(qrl) + list(trl) + list(q) + list(tv1)
        r = site(ref, "err_body", base + [0, 0, 0] + list(obs) + [0, 0])
        qrw, trw = r[:4], r[4:7]
        if qrw[3] < 0:  # the object's negation branch is not in the traced range
            continue
        tv2 = site(ref, "tv", list(qrw) + list(X))
        r = site(ref, "err_body", base + list(tv2) + list(obs) + [0, 0])
        Xr = r[7:10]
        p = site(ref, "proj", list(K) + list(Xr))
        r = site(ref, "err_body", base + list(tv2) + list(obs) + list(p))
        orc.oracle_fp64_body_error(dv(*qrl), dv(*trl), dv(*q), dv(*t), dv(*X), dv(*K), dv(*obs), err)
        assert same(r[10:], err[:]), (r[10:], err[:])
        o = out(7)
        orc.oracle_fp64_se3_mul(dv(*qrl), dv(*trl), dv(*q), dv(*t), o)
        assert same(r[:7], o[:])


def test_linearize_body(ref, orc):
    """EdgeSE3ProjectXYZToBody::linearizeOplus (Xi 2x3, Xj 2x6) composed across its four
    _transformVector calls and two projectJac calls."""
    rng = np.random.default_rng(64)
    A, B = out(6), out(12)
    for _ in range(N):
        qrl, trl = rand_q(rng, 1.0), np.array([-0.11, 0.0, 0.0]) + rng.normal(size=3) * 0.01
        q, t = rand_pose(rng)
        X = rand_point(rng, q, t)
        K = rand_cam(rng)
        o = out(7)
        orc.oracle_fp64_se3_mul(dv(*qrl), dv(*trl), dv(*q), dv(*t), o)
        if o[3] < 0 and abs(o[3]) > 0:  # only the traced (w >= 0) branch
            continue
        tv2 = site(ref, "tv", list(q) + list(X))
        Xl = np.array([t[0] + tv2[0], t[1] + tv2[1], tv2[2] + t[2]])
        tv4 = site(ref, "tv", list(qrl) + list(Xl))
        Xr = np.array([trl[0] + tv4[0], trl[1] + tv4[1], tv4[2] + trl[2]])
        pj = _pj(ref, K, Xr)
        # _pj gives the projectJac entries row-major; the site inputs are those of the sret slots
        r = site(ref, "lin_body", list(qrl) + list(trl) + list(q) + [t[0], t[1], t[2]] + list(tv2) + list(tv2)
                 + list(tv4) + pj + pj)
        orc.oracle_fp64_lin_body(dv(*qrl), dv(*trl), dv(*q), dv(*t), dv(*X), (C.c_float * 2)(*K[:2]), A, B)
        assert same(r[:6], A[:]) and same(r[6:], B[:]), (r, A[:], B[:])
