/*
 * frame_oracle.cpp — CPU restatement of Frame::UndistortKeyPoints (Frame.cc:730-763) and
 * Frame::ComputeImageBounds (Frame.cc:765-792): cv::undistortPoints(mat, mat, K, mDistCoef,
 * cv::Mat(), mK) [OpenCV 4.2.0, calib3d/src/undistort.dispatch.cpp cvUndistortPointsInternal]
 * with its default TermCriteria(COUNT, 5, 0.01): K, the distortion coefficients and P = mK are
 * converted to double; per point x = (u - cx) / fx (as (u - cx) * (1. / fx)), five fixed-point
 * iterations
 *     r2 = x*x + y*y
 *     icdist = (1 + ((k7 r2 + k6) r2 + k5) r2) / (1 + ((k4 r2 + k1) r2 + k0) r2)
 *     (icdist < 0: x, y back to the undistorted-ray start and stop — regression_14583)
 *     deltaX = 2 k2 x y + k3 (r2 + 2 x x) + k8 r2 + k9 r2 r2
 *     deltaY = k2 (r2 + 2 y y) + 2 k3 x y + k10 r2 + k11 r2 r2
 *     x = (x0 - deltaX) icdist,  y = (y0 - deltaY) icdist
 * (the tilt matrices are the identity for <= 5 coefficients and leave x, y untouched), then
 * P * (x, y, 1): x = (RR00 x + RR01 y + RR02) * ww with RR = P (R = I), ww = 1 / (0 x + 0 y + 1),
 * stored as float.  All double, no contraction (OpenCV's x86-64 baseline build has no FMA).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity unpinned: OpenCV is not in this image and the
 * reference holds no fixtures; numpy restatement in tests/test_frame_oracle.py.
 */
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../include/slamhot.h"

namespace {

struct Undistorter {
    double fx, fy, cx, cy, ifx, ify, k[14];
    double RR[3][3];
    Undistorter(const float* K, const float* dist, int nd, const float* P) {
        fx = K[0];
        fy = K[1];
        cx = K[2];
        cy = K[3];
        ifx = 1. / fx;
        ify = 1. / fy;
        for (int i = 0; i < 14; i++) k[i] = i < nd ? (double)dist[i] : 0.0;
        const double PP[3][3] = {{P[0], 0.0, P[2]}, {0.0, P[1], P[3]}, {0.0, 0.0, 1.0}};
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) RR[i][j] = PP[i][j];  // PP * I (cvMatMul): exact
    }
    void point(float uf, float vf, float& xo, float& yo) const {
        const double u = uf, v = vf;
        double x = (u - cx) * ifx, y = (v - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist =
                (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            if (icdist < 0) {
                x = (u - cx) * ifx;
                y = (v - cy) * ify;
                break;
            }
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        const double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        const double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        const double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        xo = (float)(xx * ww);
        yo = (float)(yy * ww);
    }
};

}  // namespace

extern "C" {

/* Frame::UndistortKeyPoints: K = (fx, fy, cx, cy) of toK() and of mK (the same camera). */
void oracle_undistort_keypoints(int n, const slam_keypoint* kps, const float* K, const float* dist, int ndist,
                                slam_keypoint* out) {
    if (ndist <= 0 || dist[0] == 0.0f) {  // Frame.cc:732-736
        std::memcpy(out, kps, sizeof(slam_keypoint) * n);
        return;
    }
    const Undistorter U(K, dist, ndist, K);
    for (int i = 0; i < n; i++) {
        out[i] = kps[i];
        U.point(kps[i].x, kps[i].y, out[i].x, out[i].y);
    }
}

/* Frame::ComputeImageBounds: bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY). */
void oracle_image_bounds(const float* K, const float* dist, int ndist, int cols, int rows, float* bounds) {
    if (ndist <= 0 || dist[0] == 0.0f) {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
        return;
    }
    const Undistorter U(K, dist, ndist, K);
    const float cx[4] = {0.0f, (float)cols, 0.0f, (float)cols}, cy[4] = {0.0f, 0.0f, (float)rows, (float)rows};
    float x[4], y[4];
    for (int i = 0; i < 4; i++) U.point(cx[i], cy[i], x[i], y[i]);
    bounds[0] = x[2] < x[0] ? x[2] : x[0];  // std::min(mat(0,0), mat(2,0)) = (b < a) ? b : a
    bounds[1] = x[1] < x[3] ? x[3] : x[1];  // std::max(mat(1,0), mat(3,0)) = (a < b) ? b : a
    bounds[2] = y[1] < y[0] ? y[1] : y[0];
    bounds[3] = y[2] < y[3] ? y[3] : y[2];
}

}  // extern "C"
