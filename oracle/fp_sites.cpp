/*
 * fp_sites.cpp — C exports of oracle/fp_sites.hpp for tests/test_fp_sites.py, which checks them
 * against C emitted from the reference objects' traced data flow.  TEST INFRASTRUCTURE ONLY.
 */
#include <cmath>

#include "fp_sites.hpp"

extern "C" {

int oracle_fp_inv33(const float* a, float* b) { return oracle_fp::inv33(a, b) ? 1 : 0; }

/* SearchForTriangulation_ preamble + the F12 of epipolarConstrain_ (see fp_sites.hpp) */
void oracle_fp_tri_geometry(const float* R1, const float* t1, const float* Cw1, const float* cam1, const float* R2,
                            const float* t2, const float* cam2, float* ep, float* R12, float* t12, float* F12) {
    oracle_fp::tri_geometry(R1, t1, Cw1, cam1, R2, t2, cam2, ep, R12, t12, F12);
}

/* Pinhole::epipolarConstrain_ for (K1, K2, R12, t12, kp1, kp2, unc): out = {den, dsqr, 3.84 unc};
 * returns the gate. */
int oracle_fp_epipolar_vals(const float* cam1, const float* cam2, const float* R12, const float* t12, float x1,
                            float y1, float x2, float y2, float unc, double* out) {
    const float K1t[9] = {cam1[0], 0.0f, 0.0f, 0.0f, cam1[1], 0.0f, cam1[2], cam1[3], 1.0f};
    const float K2[9] = {cam2[0], 0.0f, cam2[2], 0.0f, cam2[1], cam2[3], 0.0f, 0.0f, 1.0f};
    const float S[9] = {0.0f, -t12[2], t12[1], t12[2], 0.0f, -t12[0], -t12[1], t12[0], 0.0f};
    float K1ti[9], K2i[9], F[9];
    oracle_fp::inv33(K1t, K1ti);
    oracle_fp::inv33(K2, K2i);
    oracle_fp::mul33(K1ti, S, F);
    oracle_fp::mul33(F, R12, F);
    oracle_fp::mul33(F, K2i, F);
    const float a = std::fma(x1, F[0], y1 * F[3]) + F[6];
    const float b = std::fma(x1, F[1], y1 * F[4]) + F[7];
    const float c = std::fma(y1, F[5], x1 * F[2]) + F[8];
    const float num = std::fma(b, y2, a * x2) + c;
    const float den = std::fma(a, a, b * b);
    out[0] = den;
    out[1] = den == 0.0f ? 0.0 : (double)(num * num / den);
    out[2] = 3.84 * (double)unc;
    return oracle_fp::epipolar(F, x1, y1, x2, y2, unc) ? 1 : 0;
}

/* Frame::isInFrustum's float pieces for one point: out = {Pc0, Pc1, Pc2, Pc_dist, dist, viewCos,
 * ur} given Rcw|tcw (row-major 3x4), Ow, camera, bf, X, normal. */
void oracle_fp_frustum_vals(const float* T, const float* Ow, const float* cam, float bf, const float* X,
                            const float* normal, double* out) {
    float Pc[3];
    for (int r = 0; r < 3; r++) Pc[r] = oracle_fp::dot3_chain(T + 4 * r, X) + T[4 * r + 3];
    float uv[2];
    oracle_fp::project(cam, Pc, uv);
    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
    const float dist = (float)std::sqrt(oracle_fp::norm2_d(PO));
    out[0] = Pc[0];
    out[1] = Pc[1];
    out[2] = Pc[2];
    out[3] = (float)std::sqrt(oracle_fp::norm2_d(Pc));
    out[4] = dist;
    out[5] = oracle_fp::dot3_chain(PO, normal) / dist;
    out[6] = oracle_fp::ur_of(uv[0], bf, 1.0f / Pc[2]);
}

}  // extern "C"

extern "C" {

void oracle_fp_project(const float* cam, const float* X, float* uv) { oracle_fp::project(cam, X, uv); }

double oracle_fp_norm2(const float* v) { return oracle_fp::norm2_d(v); }

/* SearchByProjection(F, LastF) stereo gate (ORBmatcher.cc:2252-2258): er = |ur - uright| */
float oracle_fp_sbp_er(float u, float bf, float invz, float kpr) {
    return std::fabs(oracle_fp::ur_of(u, bf, invz) - kpr);
}

/* Fuse stereo chi2 (ORBmatcher.cc:1735-1745): (double)(e2 * invSigma2) */
double oracle_fp_fuse_e2(float u, float v, float kpx, float kpy, float kpr, float bf, float invz, float inv_sigma2) {
    const float ur = oracle_fp::ur_of(u, bf, invz);
    const float ex = u - kpx, ey = v - kpy, er = ur - kpr;
    const float e2 = std::fma(er, er, std::fma(ex, ex, ey * ey));
    return (double)(e2 * inv_sigma2);
}

}  // extern "C"

/* Round 5: the FP64 edge / chi2 / Huber sites of LocalBundleAdjustment and PoseOptimization as
 * the oracle computes them (g2o_sites.hpp), for tests/test_fp64_sites.py.  q = (x, y, z, w),
 * t = translation; matrices row-major. */
#include "g2o_sites.hpp"

namespace {
g2o_oracle::SE3 se3_of(const double* q, const double* t) {
    g2o_oracle::SE3 T;
    T.r = {q[0], q[1], q[2], q[3]};
    for (int i = 0; i < 3; i++) T.t[i] = t[i];
    return T;
}
}  // namespace

extern "C" {

void oracle_fp64_tv(const double* q, const double* v, double* out) {
    g2o_oracle::tv_cc({q[0], q[1], q[2], q[3]}, v, out);
}
void oracle_fp64_map(const double* q, const double* t, const double* X, double* out) {
    g2o_oracle::map_cc(se3_of(q, t), X, out);
}
void oracle_fp64_project(const double* K, const double* X, double* uv) { g2o_oracle::project_cc(K, X, uv); }
void oracle_fp64_neg_project_jac(const float* Kf, const double* X, double* n) { g2o_oracle::neg_project_jac_cc(Kf, X, n); }
void oracle_fp64_rot(const double* q, double* R) { g2o_oracle::rot_cc({q[0], q[1], q[2], q[3]}, R); }
void oracle_fp64_lin_mono(const double* q, const double* t, const double* X, const float* Kf, double* A, double* B) {
    g2o_oracle::lin_mono_cc(se3_of(q, t), X, Kf, A, B);
}
void oracle_fp64_lin_pose_mono(const double* q, const double* t, const double* X, const float* Kf, double* B) {
    g2o_oracle::lin_pose_mono_cc(se3_of(q, t), X, Kf, B);
}
void oracle_fp64_lin_stereo(const double* q, const double* t, const double* X, double fx, double fy, double bf,
                            double* A, double* B) {
    g2o_oracle::lin_stereo_cc(se3_of(q, t), X, fx, fy, bf, A, B);
}
void oracle_fp64_lin_pose_stereo(const double* q, const double* t, const double* X, double fx, double fy, double bf,
                                 double* A) {
    g2o_oracle::lin_pose_stereo_cc(se3_of(q, t), X, fx, fy, bf, A);
}
void oracle_fp64_cam_stereo(const double* X, double fx, double fy, double cx, double cy, float bf, double* out) {
    g2o_oracle::cam_project_stereo_cc(X, fx, fy, cx, cy, bf, out);
}
void oracle_fp64_cam_pose_stereo(const double* X, double fx, double fy, double cx, double cy, double bf, double* out) {
    g2o_oracle::cam_project_pose_stereo_cc(X, fx, fy, cx, cy, bf, out);
}
double oracle_fp64_chi2_2(const double* e, double info) { return g2o_oracle::chi2_2_cc(e, info); }
double oracle_fp64_chi2_3(const double* e, double info) { return g2o_oracle::chi2_3_cc(e, info); }
void oracle_fp64_huber(double e, double delta, float dsqr, double* rho) { g2o_oracle::huber_cc(e, delta, dsqr, rho); }
// round 6: the SE3Quat product, SE3Quat::exp, oplusImpl and the body edge (q as x y z w, t as x y z;
// outputs q then t)
void oracle_fp64_se3_mul(const double* qa, const double* ta, const double* qb, const double* tb, double* out) {
    const g2o_oracle::SE3 r = g2o_oracle::se3_mul_cc(se3_of(qa, ta), se3_of(qb, tb));
    out[0] = r.r.x;
    out[1] = r.r.y;
    out[2] = r.r.z;
    out[3] = r.r.w;
    for (int i = 0; i < 3; i++) out[4 + i] = r.t[i];
}
void oracle_fp64_se3_exp(const double* u, double* out) {
    const g2o_oracle::SE3 r = g2o_oracle::se3_exp_cc(u);
    out[0] = r.r.x;
    out[1] = r.r.y;
    out[2] = r.r.z;
    out[3] = r.r.w;
    for (int i = 0; i < 3; i++) out[4 + i] = r.t[i];
}
void oracle_fp64_body_error(const double* qrl, const double* trl, const double* q, const double* t, const double* X,
                            const double* K, const double* obs, double* err) {
    g2o_oracle::body_error_cc(se3_of(qrl, trl), se3_of(q, t), X, K, obs, err);
}
void oracle_fp64_lin_body(const double* qrl, const double* trl, const double* q, const double* t, const double* X,
                          const float* Kf, double* A, double* B) {
    g2o_oracle::lin_body_cc(se3_of(qrl, trl), se3_of(q, t), X, Kf, A, B);
}

}  // extern "C"
