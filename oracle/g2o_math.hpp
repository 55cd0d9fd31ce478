/*
 * g2o_math.hpp — CPU restatement of the g2o / Eigen geometry the optimizers use (SE3Quat,
 * Eigen quaternion conversions, 3x3 cofactor inverse).  TEST INFRASTRUCTURE ONLY (see
 * oracle.h); shared by lba_oracle.cpp and pose_oracle.cpp.
 */
#pragma once
#include <cmath>

namespace g2o_oracle {

struct Quat {
    double x, y, z, w;  // Eigen coeffs() order
};

struct SE3 {
    Quat r;
    double t[3];
};

// Eigen::Quaternion from a rotation matrix (Eigen/src/Geometry/Quaternion.h,
// quaternion_assign_impl<Other,3,3>).  R row-major.
inline Quat quat_from_R(const double* R) {
    auto m = [&](int i, int j) { return R[3 * i + j]; };
    Quat q;
    double c[3];
    double t = m(0, 0) + m(1, 1) + m(2, 2);
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m(2, 1) - m(1, 2)) * t;
        q.y = (m(0, 2) - m(2, 0)) * t;
        q.z = (m(1, 0) - m(0, 1)) * t;
        return q;
    }
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m(k, j) - m(j, k)) * t;
    c[j] = (m(j, i) + m(i, j)) * t;
    c[k] = (m(k, i) + m(i, k)) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
    return q;
}

// SE3Quat::normalizeRotation (se3quat.h:280-285): w >= 0, then Quaternion::normalize.
inline void normalize_rotation(Quat& q) {
    if (q.w < 0) {
        q.x = -q.x;
        q.y = -q.y;
        q.z = -q.z;
        q.w = -q.w;
    }
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n;
    q.y /= n;
    q.z /= n;
    q.w /= n;
}

// Quaternion::toRotationMatrix (Eigen Quaternion.h).
inline void rot_matrix(const Quat& q, double* R) {
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

// Quaternion * Vector3 (Eigen _transformVector): uv = v x p; uv += uv; p + w uv + v x uv.
inline void quat_rotate(const Quat& q, const double* p, double* out) {
    double uv[3] = {q.y * p[2] - q.z * p[1], q.z * p[0] - q.x * p[2], q.x * p[1] - q.y * p[0]};
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2],
                         q.x * uv[1] - q.y * uv[0]};
    out[0] = p[0] + q.w * uv[0] + c[0];
    out[1] = p[1] + q.w * uv[1] + c[1];
    out[2] = p[2] + q.w * uv[2] + c[2];
}

// Quaternion product (Eigen quat_product).
inline Quat quat_mul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

// SE3Quat::map (se3quat.h:217-220)
inline void se3_map(const SE3& T, const double* X, double* out) {
    quat_rotate(T.r, X, out);
    out[0] += T.t[0];
    out[1] += T.t[1];
    out[2] += T.t[2];
}

// SE3Quat::exp (se3quat.h:223-257), including the small-angle branch R = I + W + W^2.
inline SE3 se3_exp(const double* upd) {
    const double om[3] = {upd[0], upd[1], upd[2]};
    const double up[3] = {upd[3], upd[4], upd[5]};
    const double theta = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    double W[9] = {0, -om[2], om[1], om[2], 0, -om[0], -om[1], om[0], 0};  // skew (se3_ops.hpp:27)
    double W2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            W2[3 * i + j] = W[3 * i + 0] * W[0 + j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int k = 0; k < 9; k++) R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + W[k] + W2[k];
        for (int k = 0; k < 9; k++) V[k] = R[k];
    } else {
        const double a = std::sin(theta) / theta;
        const double b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int k = 0; k < 9; k++) {
            const double I = (k % 4 == 0) ? 1.0 : 0.0;
            R[k] = I + a * W[k] + b * W2[k];
            V[k] = I + b * W[k] + c * W2[k];
        }
    }
    SE3 T;
    T.r = quat_from_R(R);
    for (int i = 0; i < 3; i++) T.t[i] = V[3 * i + 0] * up[0] + V[3 * i + 1] * up[1] + V[3 * i + 2] * up[2];
    normalize_rotation(T.r);  // SE3Quat(const Quaterniond&, const Vector3d&)
    return T;
}

// SE3Quat::operator* (se3quat.h:104-110)
inline SE3 se3_mul(const SE3& a, const SE3& b) {
    SE3 r;
    double rt[3];
    quat_rotate(a.r, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a.t[i] + rt[i];
    r.r = quat_mul(a.r, b.r);
    normalize_rotation(r.r);
    return r;
}

// Converter::toSE3Quat (Converter.cc:34-44) -> SE3Quat(R, t) (se3quat.h:56-58)
inline SE3 se3_from_cv(const float* T) {
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[3 * i + j] = T[4 * i + j];
    SE3 s;
    s.r = quat_from_R(R);
    for (int i = 0; i < 3; i++) s.t[i] = T[4 * i + 3];
    normalize_rotation(s.r);
    return s;
}

// Converter::toCvMat(SE3Quat) (Converter.cc:46-68): to_homogeneous_matrix -> float
inline void se3_to_cv(const SE3& s, float* T) {
    double R[9];
    rot_matrix(s.r, R);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[3 * i + j];
        T[4 * i + 3] = (float)s.t[i];
    }
    T[12] = 0.f;
    T[13] = 0.f;
    T[14] = 0.f;
    T[15] = 1.f;
}

// Eigen 3x3 inverse (Eigen/src/LU/InverseImpl.h, compute_inverse<.., 3>): cofactors.
inline void inverse3(const double* m, double* out) {
    auto M = [&](int i, int j) { return m[3 * i + j]; };
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
    const double det = c0[0] * M(0, 0) + c0[1] * M(1, 0) + c0[2] * M(2, 0);
    const double invdet = 1.0 / det;
    out[0] = c0[0] * invdet;
    out[1] = c0[1] * invdet;
    out[2] = c0[2] * invdet;
    out[3] = cof(0, 1) * invdet;
    out[4] = cof(1, 1) * invdet;
    out[5] = cof(2, 1) * invdet;
    out[6] = cof(0, 2) * invdet;
    out[7] = cof(1, 2) * invdet;
    out[8] = cof(2, 2) * invdet;
}


}  // namespace g2o_oracle
