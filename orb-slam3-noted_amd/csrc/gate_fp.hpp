// gate_fp.hpp — the reference binary's float arithmetic at the matcher gates, for the device
// (and the library's host code).  GCC 9.3 -O3 -march=native built the reference
// (evaluation/CMakeFiles/ORB_SLAM3.dir/flags.make:5) and contracted a*b+c into FMA wherever the
// source allows; these functions spell each contraction out with fmaf / fma (the library is
// compiled with -ffp-contract=off), so gates such as dist < minDistance, viewCos, the epipolar
// dsqr < 3.84 sigma^2 and the stereo er > radius decide exactly as the compiled reference does.
// The contraction pattern of every site was read from the reference objects (DESIGN.md §1 lists
// the object offsets); tests/test_fp_sites.py pins the oracle to those objects and the -m gpu
// tests pin these kernels to the oracle.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace slamhot {
namespace gate {

// cv::Matx product row . column: s = 0; s += a*b, contracted -> fma chain from +0 (k = 0, 1, 2)
__host__ __device__ __forceinline__ float chain3(float a0, float b0, float a1, float b1, float a2, float b2) {
    return fmaf(a2, b2, fmaf(a1, b1, fmaf(a0, b0, 0.0f)));
}

// cv::norm(cv::Matx31f)^2 = normL2Sqr<float, double> (squares summed in double)
__host__ __device__ __forceinline__ double norm2(float x, float y, float z) {
    const double a = x, b = y, c = z;
    return fma(c, c, fma(b, b, fma(a, a, 0.0)));
}

// uv.x - mbf * invz
__host__ __device__ __forceinline__ float right_u(float u, float bf, float invz) { return fmaf(-bf, invz, u); }

// C = A * B, cv::Matx33f (row-major); C may alias A or B
__host__ __device__ __forceinline__ void mul33(const float* A, const float* B, float* C) {
    float T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            T[3 * i + j] = chain3(A[3 * i], B[j], A[3 * i + 1], B[3 + j], A[3 * i + 2], B[6 + j]);
    for (int k = 0; k < 9; k++) C[k] = T[k];
}

// cv::Matx33f::inv() = Matx_FastInvOp<float, 3> as compiled: cofactors (some contracted, one
// not), det along the first row, 1/det multiplied in.  Zeros and false when det == 0.
__host__ __device__ __forceinline__ bool inv33(const float* A, float* B) {
    const float p = A[8] * A[3], q = A[5] * A[6];
    const float c00 = fmaf(A[4], A[8], -(A[7] * A[5]));
    const float c20 = fmaf(A[7], A[3], -(A[4] * A[6]));
    const float det = fmaf(A[2], c20, fmaf(A[0], c00, -((p - q) * A[1])));
    if (det == 0.0f) {
        for (int k = 0; k < 9; k++) B[k] = 0.0f;
        return false;
    }
    const float d = 1.0f / det;
    float T[9];
    T[0] = d * c00;
    T[1] = d * fmaf(A[7], A[2], -(A[8] * A[1]));
    T[2] = d * fmaf(A[5], A[1], -(A[4] * A[2]));
    T[3] = (q - p) * d;
    T[4] = d * fmaf(A[8], A[0], -(A[6] * A[2]));
    T[5] = d * fmaf(A[2], A[3], -(A[0] * A[5]));
    T[6] = d * c20;
    T[7] = d * fmaf(A[6], A[1], -(A[0] * A[7]));
    T[8] = d * fmaf(A[0], A[4], -(A[1] * A[3]));
    for (int k = 0; k < 9; k++) B[k] = T[k];
    return true;
}

// SearchForTriangulation_'s per-pair geometry (ORBmatcher.cc:1215-1240) and the F12 that
// Pinhole::epipolarConstrain_ rebuilds from R12, t12 on every call (Pinhole.cpp:161-164).
struct TriGeom {
    float ep[2];
    float F[9];
};

__host__ __device__ inline TriGeom tri_geometry(const float* R1, const float* t1, const float* Cw1, const float* cam1,
                                                const float* R2, const float* t2, const float* cam2) {
    TriGeom g;
    float C2[3];
    for (int r = 0; r < 3; r++)
        C2[r] = chain3(R2[3 * r], Cw1[0], R2[3 * r + 1], Cw1[1], R2[3 * r + 2], Cw1[2]) + t2[r];
    g.ep[0] = cam2[0] * C2[0] / C2[2] + cam2[2];  // Pinhole::project
    g.ep[1] = cam2[1] * C2[1] / C2[2] + cam2[3];
    float R12[9], t12[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R12[3 * i + j] = chain3(R1[3 * i], R2[3 * j], R1[3 * i + 1], R2[3 * j + 1], R1[3 * i + 2], R2[3 * j + 2]);
    for (int r = 0; r < 3; r++)  // -R1w R2w^T t2w + t1w; (-R1w) R2w^T is -R12 bit for bit
        t12[r] = chain3(-R12[3 * r], t2[0], -R12[3 * r + 1], t2[1], -R12[3 * r + 2], t2[2]) + t1[r];
    const float K1t[9] = {cam1[0], 0.0f, 0.0f, 0.0f, cam1[1], 0.0f, cam1[2], cam1[3], 1.0f};
    const float K2[9] = {cam2[0], 0.0f, cam2[2], 0.0f, cam2[1], cam2[3], 0.0f, 0.0f, 1.0f};
    const float S[9] = {0.0f, -t12[2], t12[1], t12[2], 0.0f, -t12[0], -t12[1], t12[0], 0.0f};
    float A[9], B[9];
    inv33(K1t, A);
    mul33(A, S, A);
    mul33(A, R12, A);
    inv33(K2, B);
    mul33(A, B, g.F);
    return g;
}

// Pinhole::epipolarConstrain_ per candidate (Pinhole.cpp:166-180)
__host__ __device__ __forceinline__ bool epipolar_ok(const float* F, float x1, float y1, float x2, float y2,
                                                     float unc) {
    const float a = fmaf(x1, F[0], y1 * F[3]) + F[6];
    const float b = fmaf(x1, F[1], y1 * F[4]) + F[7];
    const float c = fmaf(y1, F[5], x1 * F[2]) + F[8];
    const float num = fmaf(b, y2, a * x2) + c;
    const float den = fmaf(a, a, b * b);
    if (den == 0.0f) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)unc;
}

// distex*distex + distey*distey < 100*scale (ORBmatcher.cc:1331-1336)
__host__ __device__ __forceinline__ bool near_epipole(const float* ep, float x2, float y2, float scale) {
    const float dx = ep[0] - x2, dy = ep[1] - y2;
    return fmaf(dx, dx, dy * dy) < 100.0f * scale;
}

}  // namespace gate
}  // namespace slamhot
