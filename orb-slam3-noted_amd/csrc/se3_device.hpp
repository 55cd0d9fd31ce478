// se3_device.hpp — device restatement of g2o's SE3Quat / Eigen quaternion arithmetic used by the
// optimizers (se3quat.h:41-296; Eigen Quaternion.h conversions; Eigen 3x3 cofactor inverse).
// A pose record is 8 doubles: qx qy qz qw tx ty tz pad.
#pragma once

#include <hip/hip_runtime.h>

namespace slamhot {
namespace lba {

struct Quat {
    double x, y, z, w;
};

// Eigen's Quaternion(Matrix3) off the positive-trace branch, with the largest diagonal index I as
// a template argument: constant indices keep R and c in registers (a runtime i put a 3x3 array in
// scratch, giving every kernel that converts a rotation a private segment)
template <int I>
__host__ __device__ inline Quat quat_from_R_diag(const double* R) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    Quat q;
    double c[3];
    double t = sqrt(R[4 * I] - R[4 * J] - R[4 * K] + 1.0);
    c[I] = 0.5 * t;
    t = 0.5 / t;
    q.w = (R[3 * K + J] - R[3 * J + K]) * t;
    c[J] = (R[3 * J + I] + R[3 * I + J]) * t;
    c[K] = (R[3 * K + I] + R[3 * I + K]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
    return q;
}

__host__ __device__ inline Quat quat_from_R(const double* R) {
    Quat q;
    double t = R[0] + R[4] + R[8];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (R[7] - R[5]) * t;
        q.y = (R[2] - R[6]) * t;
        q.z = (R[3] - R[1]) * t;
        return q;
    }
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[4 * i]) i = 2;
    return i == 0 ? quat_from_R_diag<0>(R) : i == 1 ? quat_from_R_diag<1>(R) : quat_from_R_diag<2>(R);
}

__host__ __device__ inline void normalize_rotation(Quat& q) {
    if (q.w < 0) {
        q.x = -q.x;
        q.y = -q.y;
        q.z = -q.z;
        q.w = -q.w;
    }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n;
    q.y /= n;
    q.z /= n;
    q.w /= n;
}

__host__ __device__ inline void rot_matrix(const Quat& q, double* R) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz);
    R[1] = txy - twz;
    R[2] = txz + twy;
    R[3] = txy + twz;
    R[4] = 1.0 - (txx + tzz);
    R[5] = tyz - twx;
    R[6] = txz - twy;
    R[7] = tyz + twx;
    R[8] = 1.0 - (txx + tyy);
}

__host__ __device__ inline void quat_rotate(const Quat& q, const double* p, double* out) {
    double uv[3] = {q.y * p[2] - q.z * p[1], q.z * p[0] - q.x * p[2], q.x * p[1] - q.y * p[0]};
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    const double c0 = q.y * uv[2] - q.z * uv[1], c1 = q.z * uv[0] - q.x * uv[2],
                 c2 = q.x * uv[1] - q.y * uv[0];
    out[0] = p[0] + q.w * uv[0] + c0;
    out[1] = p[1] + q.w * uv[1] + c1;
    out[2] = p[2] + q.w * uv[2] + c2;
}

// pose record: qx qy qz qw tx ty tz pad
__device__ inline Quat load_q(const double* P) { return Quat{P[0], P[1], P[2], P[3]}; }

__device__ inline void se3_map(const double* P, const double* X, double* out) {
    quat_rotate(load_q(P), X, out);
    out[0] += P[4];
    out[1] += P[5];
    out[2] += P[6];
}

// ---- the optimizer edges' FP64 sites as the reference's objects compute them (round 5; DESIGN.md
// §1, pinned by tests/test_fp64_sites.py through the oracle's oracle/g2o_sites.hpp).  The edge
// bodies call Eigen's _transformVector out of line (OptimizableTypes.cpp.o COMDAT): each cross
// product component is fma(first product, -(second)), w * uv is fused with v.
__device__ inline void tv_cc(const Quat& q, const double* v, double* o) {
    const double uv0 = __builtin_fma(v[2], q.y, -(v[1] * q.z));
    const double uv1 = __builtin_fma(v[0], q.z, -(q.x * v[2]));
    const double uv2 = __builtin_fma(q.x, v[1], -(q.y * v[0]));
    const double u0 = uv0 + uv0, u1 = uv1 + uv1, u2 = uv2 + uv2;
    const double c0 = __builtin_fma(q.y, u2, -(q.z * u1));
    const double c1 = __builtin_fma(q.z, u0, -(u2 * q.x));
    const double c2 = __builtin_fma(q.x, u1, -(q.y * u0));
    o[0] = __builtin_fma(q.w, u0, v[0]) + c0;
    o[1] = __builtin_fma(q.w, u1, v[1]) + c1;
    o[2] = c2 + __builtin_fma(q.w, u2, v[2]);
}

// SE3Quat::map inside computeError / linearizeOplus / isDepthPositive: _transformVector, then + t
__device__ inline void map_cc(const double* P, const double* X, double* o) {
    tv_cc(load_q(P), X, o);
    o[0] = P[4] + o[0];
    o[1] = P[5] + o[1];
    o[2] = o[2] + P[6];
}

// Quaternion::toRotationMatrix as inlined into the linearizeOplus bodies (row-major)
__device__ inline void rot_cc(const Quat& q, double* R) {
    const double tx = q.x + q.x, ty = q.y + q.y, tz = q.z + q.z;
    const double tyy = q.y * ty, tzz = q.z * tz, txy = q.x * ty, txz = q.x * tz, tyz = q.y * tz;
    R[0] = 1.0 - (tyy + tzz);
    R[1] = __builtin_fma(-tz, q.w, txy);
    R[2] = __builtin_fma(ty, q.w, txz);
    R[3] = __builtin_fma(tz, q.w, txy);
    R[4] = 1.0 - __builtin_fma(q.x, tx, tzz);
    R[5] = __builtin_fma(-tx, q.w, tyz);
    R[6] = __builtin_fma(-ty, q.w, txz);
    R[7] = __builtin_fma(tx, q.w, tyz);
    R[8] = 1.0 - __builtin_fma(q.x, tx, tyy);
}

// Eigen's lazy (2x3) * (3xC) product as compiled: fma(P(r,2), M(2,c), fma(P(r,1), M(1,c), P(r,0) M(0,c)))
template <int C>
__device__ inline void mul23_cc(const double* P, const double* M, double* out) {
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int c = 0; c < C; c++)
            out[C * r + c] = __builtin_fma(P[3 * r + 2], M[2 * C + c], __builtin_fma(P[3 * r + 1], M[C + c], P[3 * r] * M[c]));
}

// BaseEdge<3>::chi2 with Information = I / s^2 as compiled: the third term fused
__device__ inline double chi2_3_cc(const double* e, double info) {
    return __builtin_fma(info * e[2], e[2], e[0] * (info * e[0]) + e[1] * (info * e[1]));
}

// RobustKernelHuber::robustify as compiled (robust_kernel_impl.cpp.o @0x350)
__device__ inline void huber_cc(double c, double delta, float dsqr, double& rho0, double& rho1) {
    if (c <= (double)dsqr) {
        rho0 = c;
        rho1 = 1.;
    } else {
        const double s = sqrt(c);
        rho0 = __builtin_fma(s + s, delta, -(double)dsqr);
        rho1 = delta / s;
    }
}

// ---- round 6: the SE3Quat product, SE3Quat::exp and oplusImpl as the reference's objects compute
// them (oracle/g2o_sites.hpp quat_mul_cc / normalize_cc / se3_exp_cc, pinned by
// tests/test_fp64_sites.py against OptimizableTypes.cpp.o's EdgeSE3ProjectXYZToBody, oplusImpl and
// SE3Quat::exp; sin / cos / pow are the device's, glibc's in the reference).
// Eigen's quaternion product a * b as compiled: one product and three fused terms per component.
__device__ inline Quat quat_mul_cc(const Quat& a, const Quat& b) {
    Quat r;
    r.w = __builtin_fma(-a.z, b.z, __builtin_fma(-b.y, a.y, __builtin_fma(b.w, a.w, -(b.x * a.x))));
    r.x = __builtin_fma(-a.z, b.y, __builtin_fma(b.z, a.y, __builtin_fma(a.w, b.x, b.w * a.x)));
    r.y = __builtin_fma(-a.x, b.z, __builtin_fma(b.x, a.z, __builtin_fma(a.w, b.y, b.w * a.y)));
    r.z = __builtin_fma(-a.y, b.x, __builtin_fma(b.y, a.x, __builtin_fma(a.w, b.z, b.w * a.z)));
    return r;
}

// normalizeRotation as compiled: w >= 0, squared norm (z^2 + x^2) + (w^2 + y^2), divide when > 0
__device__ inline void normalize_cc(Quat& q) {
    if (q.w < 0) {
        q.x = -q.x;
        q.y = -q.y;
        q.z = -q.z;
        q.w = -q.w;
    }
    const double n2 = (q.z * q.z + q.x * q.x) + (q.w * q.w + q.y * q.y);
    if (n2 > 0.0) {
        const double n = sqrt(n2);
        q.x /= n;
        q.y /= n;
        q.z /= n;
        q.w /= n;
    }
}

// SE3Quat::operator* as compiled on pose records: Q = A * B (t = A.t + A.r._transformVector(B.t))
__device__ inline void se3_mul_cc(const double* A, const double* B, double* Qo) {
    double rt[3];
    tv_cc(load_q(A), B + 4, rt);
    Quat r = quat_mul_cc(load_q(A), load_q(B));
    normalize_cc(r);
    Qo[0] = r.x;
    Qo[1] = r.y;
    Qo[2] = r.z;
    Qo[3] = r.w;
    Qo[4] = A[4] + rt[0];
    Qo[5] = A[5] + rt[1];
    Qo[6] = A[6] + rt[2];
    Qo[7] = 0.0;
}

// VertexSE3Expmap::oplusImpl: T <- exp(upd) * T (types_six_dof_expmap.h:71-74), SE3Quat::exp
// (se3quat.h:223-257) with its small-angle branch, both as compiled (g2o_sites.hpp se3_exp_cc).
__device__ inline void se3_exp_mul(const double* upd, const double* cur, double* nxt) {
    const double w0 = upd[0], w1 = upd[1], w2 = upd[2], v0 = upd[3], v1 = upd[4], v2 = upd[5];
    const double theta = sqrt(__builtin_fma(w2, w2, w0 * w0 + w1 * w1));
    const double nw0 = -w0, nw1 = -w1, nw2 = -w2;
    double S[9];
    S[0] = __builtin_fma(nw1, w1, __builtin_fma(w2, nw2, 0.0 * 0.0));
    S[1] = __builtin_fma(w1, w0, __builtin_fma(nw2, 0.0, nw2 * 0.0));
    S[2] = __builtin_fma(w1, 0.0, __builtin_fma(nw0, nw2, 0.0 * w1));
    S[3] = __builtin_fma(nw1, nw0, __builtin_fma(w2, 0.0, w2 * 0.0));
    S[4] = __builtin_fma(nw0, w0, __builtin_fma(0.0, 0.0, nw2 * w2));
    S[5] = __builtin_fma(nw0, 0.0, __builtin_fma(nw0, 0.0, w2 * w1));
    S[6] = __builtin_fma(nw1, 0.0, __builtin_fma(nw1, 0.0, w0 * w2));
    S[7] = __builtin_fma(w1, w2, __builtin_fma(0.0, w0, w0 * 0.0));
    S[8] = __builtin_fma(nw1, w1, __builtin_fma(nw0, w0, 0.0));
    const double Wm[9] = {0.0, nw2, w1, w2, 0.0, nw0, nw1, w0, 0.0};
    double R[9], V[9];
    if (theta < 0.00001) {
        const double IW[9] = {1.0, 0.0 - w2, w1 + 0.0, w2 + 0.0, 1.0, 0.0 - w0, 0.0 - w1, w0 + 0.0, 1.0};
#pragma unroll
        for (int i = 0; i < 9; i++) {
            R[i] = S[i] + IW[i];
            V[i] = R[i];
        }
    } else {
        const double st = sin(theta), ct = cos(theta);
        const double a = st / theta;
        const double b = (1.0 - ct) / (theta * theta);
        const double c = (theta - st) / pow(theta, 3.0);
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            R[i] = __builtin_fma(b, S[i], __builtin_fma(a, Wm[i], I));
            V[i] = __builtin_fma(c, S[i], __builtin_fma(b, Wm[i], I));
        }
    }
    double E[8];
    E[4] = __builtin_fma(V[2], v2, __builtin_fma(v1, V[1], v0 * V[0]));
    E[5] = __builtin_fma(V[5], v2, __builtin_fma(v1, V[4], v0 * V[3]));
    E[6] = __builtin_fma(v0, V[6], __builtin_fma(v2, V[8], v1 * V[7]));
    const double tr = (R[8] + R[4]) + R[0];
    Quat qe;
    if (tr > 0.0) {
        const double sq = sqrt(tr + 1.0);
        const double s = 0.5 / sq;
        qe.w = sq * 0.5;
        qe.x = (R[7] - R[5]) * s;
        qe.y = (R[2] - R[6]) * s;
        qe.z = (R[3] - R[1]) * s;
    } else {
        qe = quat_from_R(R);  // not reached by LM steps (rotations of 120 degrees or more)
    }
    normalize_cc(qe);
    E[0] = qe.x;
    E[1] = qe.y;
    E[2] = qe.z;
    E[3] = qe.w;
    se3_mul_cc(E, cur, nxt);  // exp * T
}

// Eigen 3x3 inverse by cofactors (Eigen/src/LU/InverseImpl.h)
__device__ inline void inverse3(const double* m, double* out) {
#define M_(i, j) m[3 * (i) + (j)]
#define COF(i, j) (M_(((i) + 1) % 3, ((j) + 1) % 3) * M_(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M_(((i) + 1) % 3, ((j) + 2) % 3) * M_(((i) + 2) % 3, ((j) + 1) % 3))
    const double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    const double det = c00 * M_(0, 0) + c10 * M_(1, 0) + c20 * M_(2, 0);
    const double invdet = 1.0 / det;
    out[0] = c00 * invdet;
    out[1] = c10 * invdet;
    out[2] = c20 * invdet;
    out[3] = COF(0, 1) * invdet;
    out[4] = COF(1, 1) * invdet;
    out[5] = COF(2, 1) * invdet;
    out[6] = COF(0, 2) * invdet;
    out[7] = COF(1, 2) * invdet;
    out[8] = COF(2, 2) * invdet;
#undef COF
#undef M_
}

}  // namespace lba
}  // namespace slamhot
