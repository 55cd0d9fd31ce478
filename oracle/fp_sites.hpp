/*
 * fp_sites.hpp — the reference binary's float arithmetic at the matcher gates, restated with
 * explicit contractions.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The reference is compiled by GCC 9.3 with -O3 -march=native (evaluation/CMakeFiles/
 * ORB_SLAM3.dir/flags.make:5), which contracts a*b+c into FMA wherever the expression allows.
 * The sites below were read off the reference's objects as data (tools/disasm/fptrace.py; object
 * offsets in DESIGN.md §1) and are written here with fmaf / fma so that this oracle computes
 * what that binary computes, whatever compiler builds the oracle (-ffp-contract=off).
 * tests/test_fp_sites.py checks each function against C emitted from the same object trace.
 *
 * Conventions: cv::Matx products (Matx_MatMulOp: s = 0; s += a*b) are fma chains from +0 in
 * k order; cv::norm(Matx31f) is normL2Sqr<float,double> (squares summed in double);
 * Matx33f::inv() is Matx_FastInvOp<float,3> (cofactors, det by the first row).
 */
#ifndef SLAMHOT_ORACLE_FP_SITES_HPP
#define SLAMHOT_ORACLE_FP_SITES_HPP

#include <cmath>

namespace oracle_fp {

// cv::Matx<float,3,3> * cv::Matx<float,3,3> (C = A B), row-major
inline void mul33(const float* A, const float* B, float* C) {
    float T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            float s = std::fma(A[3 * i], B[j], 0.0f);
            s = std::fma(A[3 * i + 1], B[3 + j], s);
            T[3 * i + j] = std::fma(A[3 * i + 2], B[6 + j], s);
        }
    for (int k = 0; k < 9; k++) C[k] = T[k];
}

// cv::Matx33f * cv::Matx31f: fma chain from +0 (Frame.cc.o isInFrustum @0x9f4a..0x9fb2)
inline float dot3_chain(const float* r, const float* x) {
    return std::fma(r[2], x[2], std::fma(r[1], x[1], std::fma(r[0], x[0], 0.0f)));
}

// cv::norm(Matx31f) = sqrt(normL2Sqr<float,double>) (Frame.cc.o @0x0, @0x9fc5..0x9ff7)
inline double norm2_d(const float* v) {
    const double a = v[0], b = v[1], c = v[2];
    return std::fma(c, c, std::fma(b, b, std::fma(a, a, 0.0)));
}

// Matx_FastInvOp<float,3> as compiled (Pinhole.cpp.o @0x7278..0x73f5 and @0x73f5..0x7578).
// Returns false (and zeros) when det == 0, like Matx::inv.
inline bool inv33(const float* A, float* B) {
#define a(i, j) A[3 * (i) + (j)]
    const float m22_10 = a(2, 2) * a(1, 0), m12_20 = a(1, 2) * a(2, 0);
    const float c00 = std::fma(a(1, 1), a(2, 2), -(a(2, 1) * a(1, 2)));
    const float c10 = m22_10 - m12_20;  // a10 a22 - a20 a12, not contracted
    const float c20 = std::fma(a(2, 1), a(1, 0), -(a(1, 1) * a(2, 0)));
    const float det = std::fma(a(0, 2), c20, std::fma(a(0, 0), c00, -(c10 * a(0, 1))));
    if (det == 0.0f) {
        for (int k = 0; k < 9; k++) B[k] = 0.0f;
        return false;
    }
    const float d = 1.0f / det;
    float T[9];
    T[0] = d * c00;
    T[1] = d * std::fma(a(2, 1), a(0, 2), -(a(2, 2) * a(0, 1)));
    T[2] = d * std::fma(a(1, 2), a(0, 1), -(a(1, 1) * a(0, 2)));
    T[3] = (m12_20 - m22_10) * d;
    T[4] = d * std::fma(a(2, 2), a(0, 0), -(a(2, 0) * a(0, 2)));
    T[5] = d * std::fma(a(0, 2), a(1, 0), -(a(0, 0) * a(1, 2)));
    T[6] = d * c20;
    T[7] = d * std::fma(a(2, 0), a(0, 1), -(a(0, 0) * a(2, 1)));
    T[8] = d * std::fma(a(0, 0), a(1, 1), -(a(0, 1) * a(1, 0)));
#undef a
    for (int k = 0; k < 9; k++) B[k] = T[k];
    return true;
}

// Pinhole::project(cv::Matx31f) (Pinhole.cpp.o @0x5e0): (f * x) / z + c, no contraction
inline void project(const float* cam, const float* X, float* uv) {
    uv[0] = cam[0] * X[0] / X[2] + cam[2];
    uv[1] = cam[1] * X[1] / X[2] + cam[3];
}

// SearchForTriangulation_ pinhole preamble (ORBmatcher.cc:1215-1240; ORBmatcher.cc.o
// @0x12880..0x12b5b, @0x14880..0x14c40) and the F12 that Pinhole::epipolarConstrain_
// recomputes on every call (Pinhole.cpp:159-164; Pinhole.cpp.o @0x70f0..0x7949).
// R1,t1 / R2,t2: KeyFrame::GetRotation_ / GetTranslation_ (Tcw); Cw1 = pKF1->GetCameraCenter_();
// cam = {fx, fy, cx, cy}.
inline void tri_geometry(const float* R1, const float* t1, const float* Cw1, const float* cam1,
                         const float* R2, const float* t2, const float* cam2, float* ep, float* R12,
                         float* t12, float* F12) {
    float C2[3];
    for (int r = 0; r < 3; r++) C2[r] = dot3_chain(R2 + 3 * r, Cw1) + t2[r];
    project(cam2, C2, ep);
    // R12 = R1w * R2w.t()
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R12[3 * i + j] = dot3_chain(R1 + 3 * i, R2 + 3 * j);
    // t12 = -R1w * R2w.t() * t2w + t1w: (-R1w) R2w^T is -R12 exactly, then a chain with t2w
    for (int r = 0; r < 3; r++) {
        const float m[3] = {-R12[3 * r], -R12[3 * r + 1], -R12[3 * r + 2]};
        t12[r] = dot3_chain(m, t2) + t1[r];
    }
    // F12 = K1.t().inv() * t12x * R12 * K2.inv()
    const float K1t[9] = {cam1[0], 0.0f, 0.0f, 0.0f, cam1[1], 0.0f, cam1[2], cam1[3], 1.0f};
    const float K2[9] = {cam2[0], 0.0f, cam2[2], 0.0f, cam2[1], cam2[3], 0.0f, 0.0f, 1.0f};
    const float S[9] = {0.0f, -t12[2], t12[1], t12[2], 0.0f, -t12[0], -t12[1], t12[0], 0.0f};
    float K1ti[9], K2i[9], P[9];
    inv33(K1t, K1ti);
    inv33(K2, K2i);
    mul33(K1ti, S, P);
    mul33(P, R12, P);
    mul33(P, K2i, F12);
}

// Pinhole::epipolarConstrain_ per-candidate part (Pinhole.cpp:166-180; Pinhole.cpp.o
// @0x7874..0x791d): dsqr = num^2 / den in float, compared in double with 3.84 * unc.
inline bool epipolar(const float* F, float x1, float y1, float x2, float y2, float unc) {
    const float a = std::fma(x1, F[0], y1 * F[3]) + F[6];
    const float b = std::fma(x1, F[1], y1 * F[4]) + F[7];
    const float c = std::fma(y1, F[5], x1 * F[2]) + F[8];
    const float num = std::fma(b, y2, a * x2) + c;
    const float den = std::fma(a, a, b * b);
    if (den == 0.0f) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)unc;
}

// ORBmatcher.cc:1331-1336 (ORBmatcher.cc.o @0x14539..0x1454f): distex^2 + distey^2 contracted
inline bool near_epipole(const float* ep, float x2, float y2, float scale) {
    const float dx = ep[0] - x2, dy = ep[1] - y2;
    return std::fma(dx, dx, dy * dy) < 100.0f * scale;
}

// uv.x - mbf * invz (Frame.cc.o @0xa1f5, ORBmatcher.cc.o SearchByProjection(F,LastF) @0x95c7,
// Fuse @0x1be1)
inline float ur_of(float u, float bf, float invz) { return std::fma(-bf, invz, u); }

}  // namespace oracle_fp

#endif
