// device_math.hpp — bit-exact device restatements of the libm / OpenCV scalar functions
// the reference ORB path calls.  Compiled with -ffp-contract=off: every rounding step is
// written out, nothing is fused unless fmaf()/fma() is spelled.
#pragma once

#include <stdint.h>

namespace slamhot {

// glibc >= 2.28 sincosf (sysdeps/ieee754/flt-32/s_sincosf.c + sincosf.h + sincosf_data.c),
// the routine the reference's `(float)cos(angle), (float)sin(angle)` pair compiles to
// (ORBextractor.cc:111; `sincosf` in the nm of ORBextractor.cc.o).  Only the |x| < 120
// branches are reachable: the argument is angle*pi/180 with angle in [0, 360).
// Checked bit-exact against this image's glibc over every float in [0, 6.3)
// (tests/test_oracle.py::test_sincosf_restatement_exhaustive keeps that check).
struct SincosTable {
    double c0, c1, c2, c3, c4;
};

__host__ __device__ inline uint32_t sc_abstop12(float x) {
    union { float f; uint32_t u; } v;
    v.f = x;
    return (v.u >> 20) & 0x7ff;
}

__host__ __device__ inline void sc_poly(double x, double x2, bool neg, int n, float* sinp,
                                        float* cosp) {
    const double S1 = -0x1.555545995a603p-3, S2 = 0x1.1107605230bc4p-7,
                 S3 = -0x1.994eb3774cf24p-13;
    const double sg = neg ? -1.0 : 1.0;
    const double C0 = sg * 0x1p0, C1 = sg * -0x1.ffffffd0c621cp-2, C2 = sg * 0x1.55553e1068f19p-5,
                 C3 = sg * -0x1.6c087e89a359dp-10, C4 = sg * 0x1.99343027bf8c3p-16;
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double c2 = C3 + x2 * C4;
    const double s1 = S2 + x2 * S3;
    float* tmp = (n & 1) ? cosp : sinp;
    cosp = (n & 1) ? sinp : cosp;
    sinp = tmp;
    const double c1 = C0 + x2 * C1;
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = x + x3 * S1;
    const double c = c1 + x4 * C2;
    *sinp = (float)(s + x5 * s1);
    *cosp = (float)(c + x6 * c2);
}

__host__ __device__ inline void glibc_sincosf(float y, float* sinp, float* cosp) {
    double x = y;
    if (sc_abstop12(y) < sc_abstop12(0x1.921fb6p-1f)) {  // |y| < pi/4
        const double x2 = x * x;
        if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        sc_poly(x, x2, false, 0, sinp, cosp);
    } else {  // |y| < 120: fast reduction by pi/2
        const double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
        const double r = x * hpi_inv;
        const int32_t n = ((int32_t)r + 0x800000) >> 24;
        x = x - n * hpi;
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
        sc_poly(x * s, x * x, (n & 2) != 0, n, sinp, cosp);
    }
}

// cv::fastAtan2 (OpenCV 4.2.0 core/src/mathfuncs_core.simd.hpp atan_f32, scalar path of
// the SSE-baseline build: no contraction), degrees in [0, 360).
__host__ __device__ inline float cv_fast_atan2(float y, float x) {
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k;
    const float p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k;
    const float p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313080847e-16;  // (float)DBL_EPSILON
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// cvRound(float): round half to even (vcvtss2si with the default MXCSR).
__host__ __device__ inline int cv_round(float v) { return (int)rintf(v); }

}  // namespace slamhot
