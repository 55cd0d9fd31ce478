/*
 * g2o_sites.hpp — the FP64 arithmetic of the optimizer edges AS THE REFERENCE COMPILED IT
 * (round 5).  TEST INFRASTRUCTURE ONLY (see oracle.h); used by lba_oracle.cpp and
 * pose_oracle.cpp, exported for tests/test_fp64_sites.py through oracle_fp64_* in fp_sites.cpp.
 *
 * The reference's ORB_SLAM3 and g2o objects were built by GCC 9.3 with -O3 -march=native
 * (evaluation/CMakeFiles/ORB_SLAM3.dir/flags.make:5, Thirdparty/g2o/build/CMakeFiles/g2o.dir/
 * flags.make:6), which contracts a*b + c into FMA wherever Eigen's expression templates leave a
 * product next to a sum.  tools/disasm/fptrace.py (packed mode) reads those objects as data; every
 * function below restates one traced site, in the object's operation order, with each
 * contraction written as std::fma (the oracle is built with -ffp-contract=off).  DESIGN.md §1
 * lists the sites with their offsets; tests/test_fp64_sites.py checks each against C emitted
 * from the objects, bit for bit.
 */
#pragma once
#include <cmath>

#include "g2o_math.hpp"

namespace g2o_oracle {

// Eigen::QuaternionBase<Quaterniond>::_transformVector (Quaternion.h: uv = q.vec() x v; uv += uv;
// v + q.w() * uv + q.vec() x uv), the out-of-line COMDAT in OptimizableTypes.cpp.o (same code in
// g2o's types_six_dof_expmap.cpp.o, inlined alike in EdgeStereoSE3ProjectXYZOnlyPose::
// computeError): each cross-product component is fma(first product, -(second product)), the
// w * uv term is fused with v.
inline void tv_cc(const Quat& q, const double* v, double* o) {
    const double uv0 = std::fma(v[2], q.y, -(v[1] * q.z));
    const double uv1 = std::fma(v[0], q.z, -(q.x * v[2]));
    const double uv2 = std::fma(q.x, v[1], -(q.y * v[0]));
    const double u0 = uv0 + uv0, u1 = uv1 + uv1, u2 = uv2 + uv2;
    const double c0 = std::fma(q.y, u2, -(q.z * u1));
    const double c1 = std::fma(q.z, u0, -(u2 * q.x));
    const double c2 = std::fma(q.x, u1, -(q.y * u0));
    o[0] = std::fma(q.w, u0, v[0]) + c0;
    o[1] = std::fma(q.w, u1, v[1]) + c1;
    o[2] = c2 + std::fma(q.w, u2, v[2]);
}

// SE3Quat::map (se3quat.h:217-220) inside the edges: _transformVector, then + t
// (EdgeSE3ProjectXYZ::computeError @COMDAT+0x65-0x92 in OptimizableTypes.cpp.o)
inline void map_cc(const SE3& T, const double* X, double* o) {
    tv_cc(T.r, X, o);
    o[0] = T.t[0] + o[0];
    o[1] = T.t[1] + o[1];
    o[2] = o[2] + T.t[2];
}

// Quaternion::toRotationMatrix as inlined into the linearizeOplus bodies (OptimizableTypes.cpp.o
// @0x1946-0x1acb, types_six_dof_expmap.cpp.o @0xd1f-0xe97): tyy, tzz, txy, txz, tyz rounded, the
// w terms and txx fused into their sums.  Row-major R.
inline void rot_cc(const Quat& q, double* R) {
    const double tx = q.x + q.x, ty = q.y + q.y, tz = q.z + q.z;
    const double tyy = q.y * ty, tzz = q.z * tz, txy = q.x * ty, txz = q.x * tz, tyz = q.y * tz;
    R[0] = 1.0 - (tyy + tzz);
    R[1] = std::fma(-tz, q.w, txy);
    R[2] = std::fma(ty, q.w, txz);
    R[3] = std::fma(tz, q.w, txy);
    R[4] = 1.0 - std::fma(q.x, tx, tzz);
    R[5] = std::fma(-tx, q.w, tyz);
    R[6] = std::fma(-ty, q.w, txz);
    R[7] = std::fma(tx, q.w, tyz);
    R[8] = 1.0 - std::fma(q.x, tx, tyy);
}

// Pinhole::project(const Eigen::Vector3d&) (Pinhole.cpp:42-48, Pinhole.cpp.o @0x40): float
// parameters widened, (fx * x) / z + cx, no contraction.
inline void project_cc(const double* K, const double* X, double* uv) {
    uv[0] = K[0] * X[0] / X[2] + K[2];
    uv[1] = K[1] * X[1] / X[2] + K[3];
}

// Pinhole::projectJac(const Eigen::Vector3d&) (Pinhole.cpp:88-97, Pinhole.cpp.o @0xe0), negated
// as the edges use it (-pCamera->projectJac(...)): n = {-fx/z, -0, -((-fx)x/z^2); -0, -fy/z,
// -((-fy)y/z^2)} with -fx negated in float before widening.
inline void neg_project_jac_cc(const float* Kf, const double* X, double* n) {
    const double z2 = X[2] * X[2];
    n[0] = -((double)Kf[0] / X[2]);
    n[1] = -0.0;
    n[2] = -((double)(-Kf[0]) * X[0] / z2);
    n[3] = -0.0;
    n[4] = -((double)Kf[1] / X[2]);
    n[5] = -((double)(-Kf[1]) * X[1] / z2);
}

// Eigen's lazy (2x3) * (3xC) product as compiled: out(r, c) = fma(P(r,2), M(2,c), fma(P(r,1),
// M(1,c), P(r,0) * M(0,c))).  P row-major 2x3, M row-major 3xC, out row-major 2xC.
inline void mul23_cc(const double* P, const double* M, int C, double* out) {
    for (int r = 0; r < 2; r++)
        for (int c = 0; c < C; c++)
            out[C * r + c] = std::fma(P[3 * r + 2], M[2 * C + c], std::fma(P[3 * r + 1], M[C + c], P[3 * r] * M[c]));
}

// SE3deriv of the linearizeOplus bodies (OptimizableTypes.cpp:152-155), row-major 3x6
inline void se3_deriv(const double* X, double* S) {
    const double x = X[0], y = X[1], z = X[2];
    const double v[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
    for (int k = 0; k < 18; k++) S[k] = v[k];
}

// ORB_SLAM3::EdgeSE3ProjectXYZ::linearizeOplus (OptimizableTypes.cpp:139-160, @0x1840):
// Xi = -projectJac(Xc) * R (2x3), Xj = -projectJac(Xc) * SE3deriv(Xc) (2x6).  Kf = float fx, fy.
inline void lin_mono_cc(const SE3& T, const double* X, const float* Kf, double* A, double* B) {
    double Xc[3], n[6], R[9], S[18];
    map_cc(T, X, Xc);
    neg_project_jac_cc(Kf, Xc, n);
    rot_cc(T.r, R);
    mul23_cc(n, R, 3, A);
    se3_deriv(Xc, S);
    mul23_cc(n, S, 6, B);
}

// ORB_SLAM3::EdgeSE3ProjectXYZOnlyPose::linearizeOplus (OptimizableTypes.cpp:49-63, @0x1630):
// Xi = -projectJac(Xc) * SE3deriv(Xc)
inline void lin_pose_mono_cc(const SE3& T, const double* Xw, const float* Kf, double* B) {
    double Xc[3], n[6], S[18];
    map_cc(T, Xw, Xc);
    neg_project_jac_cc(Kf, Xc, n);
    se3_deriv(Xc, S);
    mul23_cc(n, S, 6, B);
}

// g2o::EdgeStereoSE3ProjectXYZ::cam_project (types_six_dof_expmap.cpp:190-197, @0xb90): invz in
// float, u = fma(invz x, fx, cx), v alike, ur = u - (float)(invz * bf) with bf a float argument.
inline void cam_project_stereo_cc(const double* X, double fx, double fy, double cx, double cy, float bf,
                                  double* o) {
    const float invz = (float)(1.0 / X[2]);
    const double iz = (double)invz;
    o[0] = std::fma(iz * X[0], fx, cx);
    o[1] = std::fma(iz * X[1], fy, cy);
    o[2] = o[0] - (double)(invz * bf);
}

// g2o::EdgeStereoSE3ProjectXYZOnlyPose::cam_project (types_six_dof_expmap.cpp:377-386, @0xc90):
// as above with bf a double member, ur = fma(-invz, bf, u).
inline void cam_project_pose_stereo_cc(const double* X, double fx, double fy, double cx, double cy, double bf,
                                       double* o) {
    const double iz = (double)(float)(1.0 / X[2]);
    o[0] = std::fma(iz * X[0], fx, cx);
    o[1] = std::fma(iz * X[1], fy, cy);
    o[2] = std::fma(-iz, bf, o[0]);
}

// g2o::BaseEdge<2>::chi2 (base_edge.h:58-61, Optimizer.cc.o COMDAT) with Information = I / s^2:
// (Ie)_k = fma(I(k,1), e1, I(k,0) e0) = info e_k exactly (the off-diagonal terms are +-0), so
// chi2 = e0 (info e0) + e1 (info e1).
inline double chi2_2_cc(const double* e, double info) { return e[0] * (info * e[0]) + e[1] * (info * e[1]); }

// g2o::BaseEdge<3>::chi2 (Optimizer.cc.o COMDAT, inlined alike into LocalBundleAdjustment's
// outlier scan @0x1b9ff): the third term is fused, chi2 = fma(info e2, e2, e0 (info e0) + e1 (info e1)).
inline double chi2_3_cc(const double* e, double info) {
    return std::fma(info * e[2], e[2], e[0] * (info * e[0]) + e[1] * (info * e[1]));
}

// g2o::RobustKernelHuber::robustify (robust_kernel_impl.cpp:79-91, @0x350): dsqr is a float
// member; above it rho0 = fma(2 sqrt(e), delta, -dsqr), rho1 = delta / sqrt(e).
inline void huber_cc(double e, double delta, float dsqr, double* rho) {
    if (e <= (double)dsqr) {
        rho[0] = e;
        rho[1] = 1.0;
    } else {
        const double s = std::sqrt(e);
        rho[0] = std::fma(s + s, delta, -(double)dsqr);
        rho[1] = delta / s;
    }
}

// g2o::EdgeStereoSE3ProjectXYZOnlyPose::linearizeOplus (types_six_dof_expmap.cpp:375-404,
// @0x1280): 3x6 row-major; the "1 + a invz^2" and the stereo-row corrections are fused.
inline void lin_pose_stereo_cc(const SE3& T, const double* Xw, double fx, double fy, double bf, double* A) {
    double Xc[3];
    map_cc(T, Xw, Xc);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double invz = 1.0 / z, invz_2 = invz * invz;
    A[0] = y * x * invz_2 * fx;
    A[1] = -std::fma(x * x, invz_2, 1.0) * fx;
    A[2] = y * invz * fx;
    A[3] = -invz * fx;
    A[4] = 0;
    A[5] = invz_2 * x * fx;
    A[6] = std::fma(y * y, invz_2, 1.0) * fy;
    A[7] = -x * y * invz_2 * fy;
    A[8] = -x * invz * fy;
    A[9] = 0;
    A[10] = -invz * fy;
    A[11] = y * invz_2 * fy;
    A[12] = std::fma(-(y * bf), invz_2, A[0]);
    A[13] = std::fma(x * bf, invz_2, A[1]);
    A[14] = A[2];
    A[15] = A[3];
    A[16] = 0;
    A[17] = std::fma(-invz_2, bf, A[5]);
}

// g2o::EdgeStereoSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:228-275, @0xcf0): Eigen's R
// and the mapping as compiled (rot_cc, map_cc), every Jacobian entry in source order (the divisions
// keep them uncontracted).  A row-major 3x3, B row-major 3x6.
inline void lin_stereo_cc(const SE3& T, const double* X, double fx, double fy, double bf, double* A, double* B) {
    double R[9], Xc[3];
    map_cc(T, X, Xc);
    rot_cc(T.r, R);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double z_2 = z * z;
    A[0] = -fx * R[0] / z + fx * x * R[6] / z_2;
    A[1] = -fx * R[1] / z + fx * x * R[7] / z_2;
    A[2] = -fx * R[2] / z + fx * x * R[8] / z_2;
    A[3] = -fy * R[3] / z + fy * y * R[6] / z_2;
    A[4] = -fy * R[4] / z + fy * y * R[7] / z_2;
    A[5] = -fy * R[5] / z + fy * y * R[8] / z_2;
    A[6] = A[0] - bf * R[6] / z_2;
    A[7] = A[1] - bf * R[7] / z_2;
    A[8] = A[2] - bf * R[8] / z_2;
    B[0] = x * y / z_2 * fx;
    B[1] = -(1 + (x * x / z_2)) * fx;
    B[2] = y / z * fx;
    B[3] = -1. / z * fx;
    B[4] = 0;
    B[5] = x / z_2 * fx;
    B[6] = (1 + y * y / z_2) * fy;
    B[7] = -x * y / z_2 * fy;
    B[8] = -x / z * fy;
    B[9] = 0;
    B[10] = -1. / z * fy;
    B[11] = y / z_2 * fy;
    B[12] = B[0] - bf * y / z_2;
    B[13] = B[1] + bf * x / z_2;
    B[14] = B[2];
    B[15] = B[3];
    B[16] = 0;
    B[17] = B[5] - bf / z_2;
}

// ---- round 6: SE3Quat products, SE3Quat::exp and the body edge --------------------------------

// Eigen's quaternion product a * b as compiled (packed vpermpd / fmadd code; EdgeSE3ProjectXYZToBody::
// computeError COMDAT @0xb1-0x15e and linearizeOplus @0xfeb-0x1074 in OptimizableTypes.cpp.o, and
// VertexSE3Expmap::oplusImpl COMDAT @0xb7-0x150, all the same form): each component is one product
// and three fused terms, in this order.
inline Quat quat_mul_cc(const Quat& a, const Quat& b) {
    Quat r;
    r.w = std::fma(-a.z, b.z, std::fma(-b.y, a.y, std::fma(b.w, a.w, -(b.x * a.x))));
    r.x = std::fma(-a.z, b.y, std::fma(b.z, a.y, std::fma(a.w, b.x, b.w * a.x)));
    r.y = std::fma(-a.x, b.z, std::fma(b.x, a.z, std::fma(a.w, b.y, b.w * a.y)));
    r.z = std::fma(-a.y, b.x, std::fma(b.y, a.x, std::fma(a.w, b.z, b.w * a.z)));
    return r;
}

// SE3Quat::normalizeRotation (se3quat.h:280-285) as compiled: w >= 0, then Eigen's normalize()
// with its packed squared norm (z^2 + x^2) + (w^2 + y^2), dividing only when it is > 0.
inline void normalize_cc(Quat& q) {
    if (q.w < 0) {
        q.x = -q.x;
        q.y = -q.y;
        q.z = -q.z;
        q.w = -q.w;
    }
    const double n2 = (q.z * q.z + q.x * q.x) + (q.w * q.w + q.y * q.y);
    if (n2 > 0.0) {
        const double n = std::sqrt(n2);
        q.x /= n;
        q.y /= n;
        q.z /= n;
        q.w /= n;
    }
}

// SE3Quat::operator* (se3quat.h:104-110) as compiled: t = a.t + a.r._transformVector(b.t),
// r = normalize(a.r * b.r).
inline SE3 se3_mul_cc(const SE3& a, const SE3& b) {
    SE3 r;
    double rt[3];
    tv_cc(a.r, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a.t[i] + rt[i];
    r.r = quat_mul_cc(a.r, b.r);
    normalize_cc(r.r);
    return r;
}

// g2o::SE3Quat::exp (se3quat.h:223-257) as compiled (OptimizableTypes.cpp.o COMDAT, the copy
// VertexSE3Expmap::oplusImpl calls; same code in types_six_dof_expmap.cpp.o).  theta =
// sqrt(fma(w2, w2, w0^2 + w1^2)); Omega^2 by Eigen's lazy 3x3 product, every entry a product and two
// fused terms in the order the object uses, zero operands kept; R = fma(b, S, fma(a, W, I)),
// V = fma(c, S, fma(b, W, I)) with a = sin/theta, b = (1 - cos)/theta^2, c = (theta - sin)/pow(theta, 3)
// (glibc sincos / pow, as the object calls them); below 1e-5 R = S + (I + W) and V = R.  t = V
// upsilon (rows 0 and 1 from column 0, row 2 from column 1), the quaternion from R on the positive
// trace branch (trace summed (R22 + R11) + R00), then normalizeRotation.  The trace <= 0 branch of
// Eigen's conversion (rotations of 120 degrees or more in one update) is not reached by LM steps and
// keeps g2o_math.hpp's unpinned form.
inline SE3 se3_exp_cc(const double* u) {
    const double w0 = u[0], w1 = u[1], w2 = u[2], v0 = u[3], v1 = u[4], v2 = u[5];
    const double theta = std::sqrt(std::fma(w2, w2, w0 * w0 + w1 * w1));
    const double nw0 = -w0, nw1 = -w1, nw2 = -w2;
    // Omega^2 (S[3 * i + j])
    double S[9];
    S[0] = std::fma(nw1, w1, std::fma(w2, nw2, 0.0 * 0.0));
    S[1] = std::fma(w1, w0, std::fma(nw2, 0.0, nw2 * 0.0));
    S[2] = std::fma(w1, 0.0, std::fma(nw0, nw2, 0.0 * w1));
    S[3] = std::fma(nw1, nw0, std::fma(w2, 0.0, w2 * 0.0));
    S[4] = std::fma(nw0, w0, std::fma(0.0, 0.0, nw2 * w2));
    S[5] = std::fma(nw0, 0.0, std::fma(nw0, 0.0, w2 * w1));
    S[6] = std::fma(nw1, 0.0, std::fma(nw1, 0.0, w0 * w2));
    S[7] = std::fma(w1, w2, std::fma(0.0, w0, w0 * 0.0));
    S[8] = std::fma(nw1, w1, std::fma(nw0, w0, 0.0));
    const double W[9] = {0.0, nw2, w1, w2, 0.0, nw0, nw1, w0, 0.0};
    double R[9], V[9];
    if (theta < 0.00001) {
        // (I + Omega) entry by entry as the object forms it: 1.0 on the diagonal, w + 0.0 above / 0.0 - w
        const double IW[9] = {1.0, 0.0 - w2, w1 + 0.0, w2 + 0.0, 1.0, 0.0 - w0, 0.0 - w1, w0 + 0.0, 1.0};
        for (int k = 0; k < 9; k++) R[k] = S[k] + IW[k];
        for (int k = 0; k < 9; k++) V[k] = R[k];
    } else {
        const double a = std::sin(theta) / theta;
        const double b = (1.0 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3.0);
        for (int k = 0; k < 9; k++) {
            const double I = (k % 4 == 0) ? 1.0 : 0.0;
            R[k] = std::fma(b, S[k], std::fma(a, W[k], I));
            V[k] = std::fma(c, S[k], std::fma(b, W[k], I));
        }
    }
    SE3 T;
    T.t[0] = std::fma(V[2], v2, std::fma(v1, V[1], v0 * V[0]));
    T.t[1] = std::fma(V[5], v2, std::fma(v1, V[4], v0 * V[3]));
    T.t[2] = std::fma(v0, V[6], std::fma(v2, V[8], v1 * V[7]));
    const double tr = (R[8] + R[4]) + R[0];
    if (tr > 0.0) {
        const double st = std::sqrt(tr + 1.0);
        const double s = 0.5 / st;
        T.r.w = st * 0.5;
        T.r.x = (R[7] - R[5]) * s;
        T.r.y = (R[2] - R[6]) * s;
        T.r.z = (R[3] - R[1]) * s;
    } else {
        T.r = quat_from_R(R);
    }
    normalize_cc(T.r);
    return T;
}

// VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:71-74): estimate <- exp(update) * estimate
inline SE3 oplus_cc(const double* upd, const SE3& est) { return se3_mul_cc(se3_exp_cc(upd), est); }

// ORB_SLAM3::EdgeSE3ProjectXYZToBody::computeError (OptimizableTypes.h:127-132, COMDAT in
// OptimizableTypes.cpp.o): obs - pCamera->project((mTrl * T_lw).map(X_w)), the product and the
// mapping as compiled (se3_mul_cc, map_cc), K = mpCamera2's fx, fy, cx, cy widened.
inline void body_error_cc(const SE3& Trl, const SE3& T, const double* Xw, const double* K, const double* obs,
                          double* err) {
    double Xr[3], uv[2];
    map_cc(se3_mul_cc(Trl, T), Xw, Xr);
    project_cc(K, Xr, uv);
    err[0] = obs[0] - uv[0];
    err[1] = obs[1] - uv[1];
}

// ORB_SLAM3::EdgeSE3ProjectXYZToBody::linearizeOplus (OptimizableTypes.cpp:192-215, @0xf30) as
// compiled: X_l = T.map(X_w), X_r = mTrl.map(X_l) (map_cc); Xi = -projectJac(X_r) * R(mTrl * T)
// with the product's rotation (quat_mul_cc + normalize_cc, its translation unused); Xj =
// (-projectJac(X_r) * R(mTrl)) * SE3deriv(X_l), both products mul23_cc with every SE3deriv entry
// (zeros and ones kept).  A 2x3, B 2x6 row-major; Kf = mpCamera2's float fx, fy.
inline void lin_body_cc(const SE3& Trl, const SE3& T, const double* Xw, const float* Kf, double* A, double* B) {
    double Xl[3], Xr[3], n[6], Rrw[9], Rrl[9], M[6], S[18];
    Quat q = quat_mul_cc(Trl.r, T.r);
    normalize_cc(q);
    map_cc(T, Xw, Xl);
    map_cc(Trl, Xl, Xr);
    neg_project_jac_cc(Kf, Xr, n);
    rot_cc(q, Rrw);
    mul23_cc(n, Rrw, 3, A);
    rot_cc(Trl.r, Rrl);
    mul23_cc(n, Rrl, 3, M);
    se3_deriv(Xl, S);
    mul23_cc(M, S, 6, B);
}

}  // namespace g2o_oracle
