// frame.hip — Frame construction after extraction: Frame::UndistortKeyPoints (Frame.cc:730-763)
// and Frame::ComputeImageBounds (Frame.cc:765-792), i.e. cv::undistortPoints(pts, pts, K,
// mDistCoef, cv::Mat(), mK) with OpenCV 4.2.0's default 5 fixed-point iterations, on gfx950.
//
// Thread per keypoint, keypoints read where the extractor left them (cap stride per frame):
// 28 B in, 28 B out, ~60 FP64 operations — HBM / latency bound and fused into nothing else
// because monocular Tracking needs mvKeysUn on the host right after extraction anyway.  The
// arithmetic is the oracle's (oracle/frame_oracle.cpp) operation for operation: double, no
// contraction (built with -ffp-contract=off), IEEE division.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>

#include "common.hpp"

namespace slamhot {
namespace {

struct Undist {
    double fx, fy, cx, cy, ifx, ify;
    double k[12];
    double RR[9];
    int identity;  // mDistCoef.at<float>(0) == 0: mvKeysUn = mvKeys (Frame.cc:732-736)
};

Undist make_undist(const float* K, const float* dist, int nd) {
    Undist U{};
    U.fx = K[0];
    U.fy = K[1];
    U.cx = K[2];
    U.cy = K[3];
    U.ifx = 1. / U.fx;
    U.ify = 1. / U.fy;
    for (int i = 0; i < 12; i++) U.k[i] = i < nd ? (double)dist[i] : 0.0;
    const double PP[9] = {K[0], 0.0, K[2], 0.0, K[1], K[3], 0.0, 0.0, 1.0};  // mK as double; RR = PP * I
    for (int i = 0; i < 9; i++) U.RR[i] = PP[i];
    U.identity = (nd <= 0 || dist[0] == 0.0f) ? 1 : 0;
    return U;
}

// cvUndistortPointsInternal's per-point body (undistort.dispatch.cpp), tilt = identity
__host__ __device__ inline void undistort_point(const Undist& U, float uf, float vf, float& xo, float& yo) {
    const double u = uf, v = vf;
    const double* k = U.k;
    double x = (u - U.cx) * U.ifx, y = (v - U.cy) * U.ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((0.0 * r2 + 0.0) * r2 + 0.0) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {  // regression_14583
            x = (u - U.cx) * U.ifx;
            y = (v - U.cy) * U.ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = U.RR[0] * x + U.RR[1] * y + U.RR[2];
    const double yy = U.RR[3] * x + U.RR[4] * y + U.RR[5];
    const double ww = 1. / (U.RR[6] * x + U.RR[7] * y + U.RR[8]);
    xo = (float)(xx * ww);
    yo = (float)(yy * ww);
}

__global__ void __launch_bounds__(256) k_undistort(Undist U, int cap, const slam_keypoint* __restrict__ kps,
                                                   const int32_t* __restrict__ n, slam_keypoint* __restrict__ out) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n[f]) return;
    const size_t o = (size_t)f * cap + i;
    slam_keypoint kp = kps[o];
    if (!U.identity) undistort_point(U, kp.x, kp.y, kp.x, kp.y);
    out[o] = kp;
}

// host-buffer form: per-device scratch + stream, one caller at a time per device
struct Scratch {
    void* d = nullptr;
    size_t cap = 0;
    hipStream_t s = nullptr;
};
std::mutex g_mu;
std::map<int, Scratch> g_scratch;

}  // namespace
}  // namespace slamhot

using namespace slamhot;

extern "C" {

slam_status slamhot_undistort_keypoints_batch_device(const float* K, const float* dist, int ndist, int nframes,
                                                     const void* d_kps, const void* d_n, int cap, void* d_kps_un,
                                                     void* hip_stream) {
    if (!K || ndist < 0 || ndist > 12 || (ndist && !dist) || nframes < 0 || cap <= 0 || !d_kps || !d_n || !d_kps_un)
        return SLAM_EINVAL;
    if (ndist > 5) return SLAM_EINVAL;  // rational / thin-prism / tilt models: not in ORB-SLAM3's settings
    if (nframes == 0) return SLAM_OK;
    const Undist U = make_undist(K, dist, ndist);
    hipLaunchKernelGGL(k_undistort, dim3((cap + 255) / 256, nframes), dim3(256), 0, (hipStream_t)hip_stream, U, cap,
                       (const slam_keypoint*)d_kps, (const int32_t*)d_n, (slam_keypoint*)d_kps_un);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

slam_status slamhot_undistort_keypoints(int device, const float* K, const float* dist, int ndist, int n,
                                        const slam_keypoint* kps, slam_keypoint* kps_un) {
    if (!K || n < 0 || (n && (!kps || !kps_un)) || ndist < 0 || ndist > 5 || (ndist && !dist)) return SLAM_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= ndev) return SLAM_EINVAL;
    if (n == 0) return SLAM_OK;
    std::lock_guard<std::mutex> g(g_mu);
    SLAM_HIP_TRY(hipSetDevice(device));
    Scratch& S = g_scratch[device];
    if (!S.s) SLAM_HIP_TRY(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
    const size_t bytes = 256 + 2 * (size_t)n * sizeof(slam_keypoint);
    if (bytes > S.cap) {
        if (S.d) (void)hipFree(S.d);
        S.d = nullptr;
        S.cap = 0;
        SLAM_HIP_TRY(hipMalloc(&S.d, bytes * 2));
        S.cap = bytes * 2;
    }
    uint8_t* b = (uint8_t*)S.d;
    SLAM_HIP_TRY(hipMemcpyAsync(b, &n, 4, hipMemcpyHostToDevice, S.s));
    SLAM_HIP_TRY(hipMemcpyAsync(b + 256, kps, (size_t)n * sizeof(slam_keypoint), hipMemcpyHostToDevice, S.s));
    slam_keypoint* dout = (slam_keypoint*)(b + 256 + (size_t)n * sizeof(slam_keypoint));
    const slam_status st =
        slamhot_undistort_keypoints_batch_device(K, dist, ndist, 1, b + 256, b, n, dout, (void*)S.s);
    if (st != SLAM_OK) return st;
    SLAM_HIP_TRY(hipMemcpyAsync(kps_un, dout, (size_t)n * sizeof(slam_keypoint), hipMemcpyDeviceToHost, S.s));
    SLAM_HIP_TRY(hipStreamSynchronize(S.s));
    return SLAM_OK;
}

slam_status slamhot_image_bounds(const float* K, const float* dist, int ndist, int cols, int rows, float* bounds) {
    if (!K || !bounds || ndist < 0 || ndist > 5 || (ndist && !dist) || cols <= 0 || rows <= 0) return SLAM_EINVAL;
    const Undist U = make_undist(K, dist, ndist);
    if (U.identity) {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
        return SLAM_OK;
    }
    // four corners, once per camera (Frame::mbInitialComputations): host arithmetic identical
    // to the kernel's (the same __host__ __device__ function)
    const float cx[4] = {0.0f, (float)cols, 0.0f, (float)cols}, cy[4] = {0.0f, 0.0f, (float)rows, (float)rows};
    float x[4], y[4];
    for (int i = 0; i < 4; i++) undistort_point(U, cx[i], cy[i], x[i], y[i]);
    bounds[0] = x[2] < x[0] ? x[2] : x[0];
    bounds[1] = x[1] < x[3] ? x[3] : x[1];
    bounds[2] = y[1] < y[0] ? y[1] : y[0];
    bounds[3] = y[2] < y[3] ? y[3] : y[2];
    return SLAM_OK;
}

}  // extern "C"
