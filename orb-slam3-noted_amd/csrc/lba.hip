// lba.hip — the LM / Schur inner loop of Optimizer::LocalBundleAdjustment on gfx950.
//
// Reference: Optimizer.cc:1611-2078 drives g2o's SparseOptimizer + OptimizationAlgorithmLevenberg
// + BlockSolver<6,3> + LinearSolverEigen (SimplicialLDLT).  Here one call solves a batch of
// independent windows; every window's state (poses, points, Hessian blocks, the dense Schur
// complement, the LM scalars) lives in HBM for the whole solve, and each LM decision is taken
// on the device by a per-window control kernel.  The host queues LM steps (every kernel below
// skips the windows a step does not concern) and polls a step counter the last control block
// publishes into mapped memory, mirroring the caller's stop flag meanwhile.
//
// Once per solve: k_bm_set / k_bm_scan / k_bm_list (per-pose point bitmaps and point-ordered
// edge lists) and k_ct_count / k_ct_scan / k_ct_fill (each Schur block's contribution list).
// Per LM step (all windows of the batch in one launch each):
//   k_linearize      wave / free pose (Hpp, b_p) + thread / point (errors, Huber rho, Hpl, Hll, b_l)
//   k_iter_begin     block / window : chi2 = sum rho, lambda init (iteration 0), stop flag
//   k_point_prep     thread / point : Dinv = (Hll + lambda I)^-1, db = Dinv b_l
//   k_schur_blocks   lanes / 6x6 block of the Schur complement (B Dinv Hpl^T per contribution,
//                    rhs row), written into the tile-major LDL^T scratch
//   k_ldlt_t16       block / window : tile LDL^T on v_mfma_f64_16x16x4f64 (k_ldlt above 288)
//   k_update         thread / KF (exp(x_p) * pose) + thread / point (x_l = Dinv (b_l - Hpl^T x_p))
//   k_trial_error    thread / edge  : error + rho at the trial state
//   k_trial_control  block / window : rho, accept (swap state) or reject, lambda, stop rules
// FP64 throughout, with the reference's float quirks (see oracle/lba_oracle.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include <immintrin.h>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "se3_device.hpp"

namespace slamhot {
namespace lba {

constexpr int kNB = 32;           // LDL^T panel width
constexpr int kMaxN = 480;        // 80 free KeyFrames per window
constexpr int kHplStride = 18;    // doubles per edge: pose-landmark block Hpl = B^T W A (6 x 3)
constexpr int kCtlThreads = 1024;
// k_ldlt_t16 geometry
constexpr int kT16Max = 18;                                  // tile rows (n <= 288)
constexpr int kT16Waves = 16;
constexpr int kT16Tiles = kT16Max * (kT16Max + 1) / 2;
constexpr int kPStride = 17;                                 // panel row stride (doubles): odd, no bank conflicts

typedef double double4_t __attribute__((ext_vector_type(4)));

// dense Schur system geometry: pose dimension padded to a multiple of kNB, rhs in row npad
__host__ __device__ constexpr int ldlt_npad(int n) { return (n + kNB - 1) / kNB * kNB; }
__host__ __device__ constexpr int ldlt_ld(int n) { return ldlt_npad(n) + 8; }
// k_ldlt LDS: PLT kNB x NP (NP = npad rounded to 16 + 16 for the rhs row), T 32x33, rowbuf, d, 1/d, WL
__host__ __device__ constexpr int ldlt_np(int n) { return ldlt_npad(n) + 16; }
__host__ __device__ constexpr size_t ldlt_lds_bytes(int n) {
    return ((size_t)kNB * ldlt_np(n) + kNB * (kNB + 1) + 3 * kNB + kNB * kNB) * sizeof(double);
}

// 6x6 symmetric upper-triangle packing, row-major (r <= c)
__host__ __device__ constexpr int sym6(int r, int c) { return r * 6 - (r * (r - 1)) / 2 + (c - r); }
__host__ __device__ constexpr int sym3(int r, int c) { return r * 3 - (r * (r - 1)) / 2 + (c - r); }

struct EdgeS {
    int pt, kf, hp, win;   // global point, global KF, global free-pose index (-1 fixed), window
    float obs[3];          // u, v, ur (ur = -1 -> mono, kBodyTag -> EdgeSE3ProjectXYZToBody)
    float info;            // invSigma2
};
// obs[2] of a right-camera (EdgeSE3ProjectXYZToBody) observation; the host writes mono edges'
// negative mvuRight as -1, so the tag never collides
constexpr float kBodyTag = -2.0f;
__device__ __forceinline__ bool is_body(const EdgeS& e) { return e.obs[2] == kBodyTag; }

struct WinDesc {
    int kf0, nk, pt0, npt, e0, ne, pose0, np;
    int n, ld, blk0, nblk;
    long long hs_off;      // doubles
    int spe0, nwd;         // first free-pose edge (spe) of the window; 64-point words per pose bitmap
    long long bm0;         // first word of the window's pose bitmaps (np x nwd)
    long long ct0;         // first Schur contribution of the window
};

struct WinCtl {
    double lambda, ni, cur_chi, ini_chi, chi2_initial, chi2_final, user_lambda, tmp_chi;
    int sel, active, need_trial, ok2, need_lin;
    int qmax, nbad, it, iters;
    int trials, opt, result, n_outlier;
    int iters_run[2];
    int iters2;  // iterations of the second optimize() (0: none); k_trial_control moves on to it
};

struct Counters {
    int need_trial, active, seq, pad;
};

struct Cam {
    double fx, fy, cx, cy, bf;
    // mbf as the float the reference multiplies with, held as a double: a float field here was
    // merged with the per-KeyFrame kbf[kf] load into a load through a selected pointer, which put
    // this by-value kernel argument in scratch (a private segment in every kernel taking a Cam)
    double bff;
    double fx2, fy2, cx2, cy2;  // mpCamera2 (body edges)
    const double* trl;          // per global KF: mTrl as a pose record (NULL without body edges)
    // per global KF: its own camera as 8 floats {fx, fy, cx, cy, fx2, fy2, cx2, cy2} and its bf
    // (Optimizer.cc:1840, 1869-1873, 1906); NULL when the whole batch shares the scalars above
    const float4* kcam;
    const float* kbf;
};

// the edge's camera (float parameters promoted, as the reference's edges hold them)
struct Intr {
    double fx, fy, cx, cy, bf;
    float bff;
};
__device__ __forceinline__ Intr left_cam(const Cam& c, int kf) {
    if (!c.kcam) return Intr{c.fx, c.fy, c.cx, c.cy, c.bf, (float)c.bff};
    const float4 a = c.kcam[2 * (long long)kf];
    const float bf = c.kbf[kf];
    return Intr{a.x, a.y, a.z, a.w, bf, bf};
}
__device__ __forceinline__ Intr right_cam(const Cam& c, int kf) {
    if (!c.kcam) return Intr{c.fx2, c.fy2, c.cx2, c.cy2, 0.0, 0.f};
    const float4 a = c.kcam[2 * (long long)kf + 1];
    return Intr{a.x, a.y, a.z, a.w, 0.0, 0.f};
}

// (mTrl * T_lw) as a pose record: SE3Quat::operator* (se3quat.h:104-110) as compiled (round 6)
__device__ inline void body_pose(const double* Trl, const double* P, double* Q) { se3_mul_cc(Trl, P, Q); }

// ---------------------------------------------------------------- edge math
__device__ inline void edge_error(const EdgeS& e, const Cam& cam, const double* P, const double* X,
                                  double* err) {
    double Xc[3];
    if (is_body(e)) {
        // EdgeSE3ProjectXYZToBody::computeError (OptimizableTypes.h:127-132)
        double Q[8];
        const Intr K2 = right_cam(cam, e.kf);
        body_pose(cam.trl + 8 * (long long)e.kf, P, Q);
        map_cc(Q, X, Xc);  // as compiled (OptimizableTypes.cpp.o COMDAT; oracle body_error_cc)
        err[0] = (double)e.obs[0] - (K2.fx * Xc[0] / Xc[2] + K2.cx);
        err[1] = (double)e.obs[1] - (K2.fy * Xc[1] / Xc[2] + K2.cy);
        err[2] = 0.0;
        return;
    }
    const Intr K = left_cam(cam, e.kf);
    map_cc(P, X, Xc);  // the compiled reference's arithmetic from here on (se3_device.hpp, round 5)
    if (e.obs[2] < 0.f) {
        const double u = K.fx * Xc[0] / Xc[2] + K.cx;  // Pinhole::project(Vector3d): no contraction
        const double v = K.fy * Xc[1] / Xc[2] + K.cy;
        err[0] = (double)e.obs[0] - u;
        err[1] = (double)e.obs[1] - v;
        err[2] = 0.0;
    } else {
        // g2o::EdgeStereoSE3ProjectXYZ::cam_project as compiled (types_six_dof_expmap.cpp.o @0xb90)
        const float invz = (float)(1.0 / Xc[2]);
        const double iz = (double)invz;
        const double u = __builtin_fma(iz * Xc[0], K.fx, K.cx);
        const double v = __builtin_fma(iz * Xc[1], K.fy, K.cy);
        const double ur = u - (double)(K.bff * invz);
        err[0] = (double)e.obs[0] - u;
        err[1] = (double)e.obs[1] - v;
        err[2] = (double)e.obs[2] - ur;
    }
}

// BaseEdge::chi2 as compiled (Optimizer.cc.o COMDATs): the 2-D form is the plain sum, the 3-D
// form fuses its third term
__device__ inline double edge_chi2(const EdgeS& e, const double* err) {
    const double info = e.info;
    if (e.obs[2] >= 0.f) return chi2_3_cc(err, info);
    return err[0] * (info * err[0]) + err[1] * (info * err[1]);
}

struct Huber {
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;
};

__device__ inline void robustify(const Huber& hk, bool stereo, double c, double& rho0, double& rho1) {
    huber_cc(c, stereo ? hk.delta_stereo : hk.delta_mono, stereo ? hk.dsqr_stereo : hk.dsqr_mono, rho0, rho1);
}

// ---------------------------------------------------------------- iteration kernels
// Jacobians of one edge at estimate (P, X): A = d e / d X (D x 3), B = d e / d pose (D x 6),
// OptimizableTypes.cpp:139-160 (mono) and types_six_dof_expmap.cpp:228-275 (stereo).
// EdgeSE3ProjectXYZToBody::linearizeOplus (OptimizableTypes.cpp:192-215): with X_l = T.map(X),
// X_r = mTrl.map(X_l): A = -J(X_r) R(mTrl*T), B = (-J(X_r) R(mTrl)) SE3deriv(X_l), left to right.
__device__ inline void body_jacobians(const EdgeS& e, const Cam& cam, const double* P, const double* X, double* A,
                                      double* B) {
    // as compiled (OptimizableTypes.cpp.o @0xf30; oracle lin_body_cc): the product's rotation
    // (quat_mul_cc + normalize_cc), both mappings map_cc, -projectJac(X_r) with float fx, fy, the
    // three products mul23_cc (every SE3deriv entry kept)
    const double* Trl = cam.trl + 8 * (long long)e.kf;
    const Intr K2 = right_cam(cam, e.kf);
    double Xl[3], Xr[3], Rrw[9], Rrl[9], n[6], M[6];
    Quat q = quat_mul_cc(load_q(Trl), load_q(P));
    normalize_cc(q);
    map_cc(P, X, Xl);
    map_cc(Trl, Xl, Xr);
    const double z2 = Xr[2] * Xr[2];
    const float fxf = (float)K2.fx, fyf = (float)K2.fy;
    n[0] = -((double)fxf / Xr[2]);
    n[1] = -0.0;
    n[2] = -((double)(-fxf) * Xr[0] / z2);
    n[3] = -0.0;
    n[4] = -((double)fyf / Xr[2]);
    n[5] = -((double)(-fyf) * Xr[1] / z2);
    rot_cc(q, Rrw);
    mul23_cc<3>(n, Rrw, A);
    rot_cc(load_q(Trl), Rrl);
    mul23_cc<3>(n, Rrl, M);
    const double xl = Xl[0], yl = Xl[1], zl = Xl[2];
    const double S[18] = {0.0, zl, -yl, 1.0, 0.0, 0.0, -zl, 0.0, xl, 0.0, 1.0, 0.0, yl, -xl, 0.0, 0.0, 0.0, 1.0};
    mul23_cc<6>(M, S, B);
    A[6] = A[7] = A[8] = 0;
#pragma unroll
    for (int cc = 0; cc < 6; cc++) B[12 + cc] = 0;
}

__device__ inline void edge_jacobians(bool stereo, const Intr& cam, const double* P, const double* X, double* A,
                                      double* B) {
    // mapping, R and the mono products as the reference's objects compute them (OptimizableTypes.cpp.o
    // @0x1840, types_six_dof_expmap.cpp.o @0xcf0; se3_device.hpp)
    double R[9], Xc[3];
    map_cc(P, X, Xc);
    rot_cc(load_q(P), R);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    if (!stereo) {
        // -projectJac with fx, fy the camera's floats (the edge's doubles are their exact values)
        const double n[6] = {-(cam.fx / z), -0.0, -((double)(-(float)cam.fx) * x / (z * z)),
                             -0.0, -(cam.fy / z), -((double)(-(float)cam.fy) * y / (z * z))};
        mul23_cc<3>(n, R, A);
        const double S[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
        mul23_cc<6>(n, S, B);
        A[6] = A[7] = A[8] = 0;
#pragma unroll
        for (int cc = 0; cc < 6; cc++) B[12 + cc] = 0;
    } else {
        const double fx = cam.fx, fy = cam.fy, bf = cam.bf;
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
}

// Point side of BlockSolver::buildSystem (block_solver.hpp:501-560): thread per MapPoint,
// its edges in insertion order.  Per edge: computeError (error, robust rho) and the
// pose-landmark block Hpl = B^T W A (constructQuadraticForm's transposed-block write,
// base_binary_edge.hpp:88-112); per point: Hll = sum A^T W A and b_l = sum A^T (-rho' Omega e).
__device__ __forceinline__ void lin_points_body(int p, int npt_total, const int* __restrict__ pt_off, const int* __restrict__ pt_win,
                             const EdgeS* __restrict__ E, const WinCtl* __restrict__ ctl,
                             const double* __restrict__ poses, const double* __restrict__ pts,
                             long long pose_stride, long long pt_stride, Cam cam, Huber hk,
                             double* __restrict__ err_out, double* __restrict__ rho_out,
                             double* __restrict__ Hpl_out, double* __restrict__ Hll, double* __restrict__ bl) {
    if (p >= npt_total) return;
    const WinCtl& C = ctl[pt_win[p]];
    if (!C.need_lin) return;
    const double* Xw = pts + C.sel * pt_stride + 4 * (long long)p;
    const double X[3] = {Xw[0], Xw[1], Xw[2]};
    double h[6] = {0, 0, 0, 0, 0, 0}, bb[3] = {0, 0, 0};
    // an edge right after one on the same KeyFrame (its body edge) shares that edge's Hpl block:
    // its product is added to the block in edge order, as g2o's shared Hessian block
    int lead = -1, lead_kf = -1;
    for (int ei = pt_off[p]; ei < pt_off[p + 1]; ei++) {
        const EdgeS e = E[ei];
        const double* P = poses + C.sel * pose_stride + 8 * (long long)e.kf;
        double err[3];
        edge_error(e, cam, P, X, err);
        *(double4_t*)(err_out + 4 * (long long)ei) = double4_t{err[0], err[1], err[2], 0.0};
        const bool stereo = e.obs[2] >= 0.f;
        double rho0, rho1;
        robustify(hk, stereo, edge_chi2(e, err), rho0, rho1);
        rho_out[ei] = rho0;
        double A[9], B[18];
        if (is_body(e))
            body_jacobians(e, cam, P, X, A, B);
        else
            edge_jacobians(stereo, left_cam(cam, e.kf), P, X, A, B);
        const double info = e.info;
        const double w = rho1 * info;
        double om_r[3];
#pragma unroll
        for (int k = 0; k < 3; k++) om_r[k] = (-(info * err[k])) * rho1;
        // 2-D edges (mono, body): row 2 of A and B is zero, and a sum that starts at +0 is
        // unchanged by those +-0 products, so they are skipped (bit-identical: each sum keeps
        // the ((0 + p0) + p1) + p2 order of the full form)
        double sb3[3], sh6[6], hpl[18];
#pragma unroll
        for (int cc = 0; cc < 3; cc++) sb3[cc] = (0.0 + A[cc] * om_r[0]) + A[3 + cc] * om_r[1];
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int cc = r; cc < 3; cc++)
                sh6[sym3(r, cc)] = (0.0 + (A[r] * w) * A[cc]) + (A[3 + r] * w) * A[3 + cc];
        if (stereo) {
#pragma unroll
            for (int cc = 0; cc < 3; cc++) sb3[cc] += A[6 + cc] * om_r[2];
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int cc = r; cc < 3; cc++) sh6[sym3(r, cc)] += (A[6 + r] * w) * A[6 + cc];
        }
#pragma unroll
        for (int k = 0; k < 3; k++) bb[k] += sb3[k];
#pragma unroll
        for (int k = 0; k < 6; k++) h[k] += sh6[k];
        if (e.hp < 0) continue;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int cc = 0; cc < 3; cc++) hpl[3 * r + cc] = (0.0 + (B[r] * w) * A[cc]) + (B[6 + r] * w) * A[3 + cc];
        if (stereo) {
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int cc = 0; cc < 3; cc++) hpl[3 * r + cc] += (B[12 + r] * w) * A[6 + cc];
        }
        if (e.kf == lead_kf) {
            double* out = Hpl_out + (long long)kHplStride * lead;
#pragma unroll
            for (int k = 0; k < 18; k += 2) {
                const double2 o = *(double2*)(out + k);
                *(double2*)(out + k) = double2{o.x + hpl[k], o.y + hpl[k + 1]};
            }
            continue;
        }
        lead = ei;
        lead_kf = e.kf;
        double* out = Hpl_out + (long long)kHplStride * ei;
#pragma unroll
        for (int k = 0; k < 18; k += 2) *(double2*)(out + k) = double2{hpl[k], hpl[k + 1]};
    }
    double* ho = Hll + 8 * (long long)p;
    *(double4_t*)ho = double4_t{h[0], h[1], h[2], h[3]};
    *(double2*)(ho + 4) = double2{h[4], h[5]};
    *(double4_t*)(bl + 4 * (long long)p) = double4_t{bb[0], bb[1], bb[2], 0.0};
}

// wave-wide sum in a fixed order, every lane ends with the same total (every lane of the wave
// must be active).  DPP form: row sums by row_ror 8 / 4 / 2 / 1, rows combined by row_bcast:15 /
// row_bcast:31 into lane 63 ((r2 + r3) + (r0 + r1)), read back uniform: VALU instead of six
// ds_bpermute round trips per double (k_linearize's 27 pose sums per KeyFrame, the chi2 sums).
// SLAMHOT_LBA_SHFL keeps the xor butterfly.
#ifndef SLAMHOT_LBA_SHFL
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ inline double wave_sum(double v) {
    v += dpp_d<0x128, 0xf>(v);  // row_ror:8
    v += dpp_d<0x124, 0xf>(v);  // row_ror:4
    v += dpp_d<0x122, 0xf>(v);  // row_ror:2
    v += dpp_d<0x121, 0xf>(v);  // row_ror:1
    v += dpp_d<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp_d<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
#else
__device__ inline double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
#endif

// per-pose free-pose edge lists built on the device (k_setup_d); pls null: use pe
struct PoseLists {
    const int* pls;
    const int* pbase;
    const int* pcnt;
    const WinDesc* wins;
};

// Pose side of buildSystem: one wave per free KeyFrame, lanes stride over its edges and
// recompute error, robust weight and the pose Jacobian B; Hpp = sum B^T W B,
// b_p = sum B^T (-rho' Omega e), then a butterfly reduction of the 27 sums.
// The pose's edges in edge order: pe[pe_off[pose] ..] when the batch has followers (body edges: a
// follower adds its own Hpp), else its free-pose edge list pls (k_setup_d: the leader edges in point order
// = edge order), which is the same sequence and needs no host-built list.
__device__ __forceinline__ void lin_poses_body(int pose, int lane, int npose_total, const int* __restrict__ pe_off,
                                                   const int* __restrict__ pe, const PoseLists pl, const int* __restrict__ pose_win,
                                                   const EdgeS* __restrict__ E, const WinCtl* __restrict__ ctl,
                                                   const double* __restrict__ poses, const double* __restrict__ pts,
                                                   long long pose_stride, long long pt_stride, Cam cam, Huber hk,
                                                   double* __restrict__ Hpp, double* __restrict__ bp) {
    if (pose >= npose_total) return;
    const int win = pose_win[pose];
    const WinCtl& C = ctl[win];
    if (!C.need_lin) return;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    const int* list = pl.pls ? pl.pls : pe;
    const int i0 = pl.pls ? pl.wins[win].spe0 + pl.pbase[pose] : pe_off[pose];
    const int i1 = pl.pls ? i0 + pl.pcnt[pose] : pe_off[pose + 1];
    for (int i = i0 + lane; i < i1; i += 64) {
        const EdgeS e = E[list[i]];
        const double* P = poses + C.sel * pose_stride + 8 * (long long)e.kf;
        const double* Xw = pts + C.sel * pt_stride + 4 * (long long)e.pt;
        const double X[3] = {Xw[0], Xw[1], Xw[2]};
        double err[3];
        edge_error(e, cam, P, X, err);
        const bool stereo = e.obs[2] >= 0.f;
        double rho0, rho1;
        robustify(hk, stereo, edge_chi2(e, err), rho0, rho1);
        double A[9], B[18];
        if (is_body(e))
            body_jacobians(e, cam, P, X, A, B);
        else
            edge_jacobians(stereo, left_cam(cam, e.kf), P, X, A, B);
        const double info = e.info;
        const double w = rho1 * info;
        double om_r[3];
#pragma unroll
        for (int k = 0; k < 3; k++) om_r[k] = (-(info * err[k])) * rho1;
        // 2-D edges: zero row 2 skipped (bit-identical, as on the point side)
        double s27[27];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int cc = r; cc < 6; cc++) s27[sym6(r, cc)] = (0.0 + (B[r] * w) * B[cc]) + (B[6 + r] * w) * B[6 + cc];
#pragma unroll
        for (int cc = 0; cc < 6; cc++) s27[21 + cc] = (0.0 + B[cc] * om_r[0]) + B[6 + cc] * om_r[1];
        if (stereo) {
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int cc = r; cc < 6; cc++) s27[sym6(r, cc)] += (B[12 + r] * w) * B[12 + cc];
#pragma unroll
            for (int cc = 0; cc < 6; cc++) s27[21 + cc] += B[12 + cc] * om_r[2];
        }
#pragma unroll
        for (int k = 0; k < 27; k++) acc[k] += s27[k];
    }
    double mine = 0.0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
        const double t = wave_sum(acc[k]);
        if (lane == k) mine = t;
    }
    if (lane < 21)
        Hpp[24 * (long long)pose + lane] = mine;
    else if (lane < 27)
        bp[8 * (long long)pose + (lane - 21)] = mine;
}

// buildSystem in one launch: the first nb_pose blocks take the pose side (a wave per free KF,
// two per block; the long per-KF edge loops start first), the rest the point side.
constexpr int kLinThreads = 128;
__global__ void __launch_bounds__(kLinThreads) k_linearize(int nb_pose, int npose_total, const int* __restrict__ pe_off,
                                                           const int* __restrict__ pe, PoseLists pl, const int* __restrict__ pose_win,
                                                           int npt_total, const int* __restrict__ pt_off,
                                                           const int* __restrict__ pt_win, const EdgeS* __restrict__ E,
                                                           const WinCtl* __restrict__ ctl, const double* __restrict__ poses,
                                                           const double* __restrict__ pts, long long pose_stride,
                                                           long long pt_stride, Cam cam, Huber hk,
                                                           double* __restrict__ err_out, double* __restrict__ rho_out,
                                                           double* __restrict__ Hpl_out, double* __restrict__ Hll,
                                                           double* __restrict__ bl, double* __restrict__ Hpp,
                                                           double* __restrict__ bp) {
    const int b = blockIdx.x;
    if (b < nb_pose)
        lin_poses_body(b * (kLinThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x & 63,
                       npose_total, pe_off, pe, pl,
                       pose_win, E, ctl, poses, pts, pose_stride, pt_stride, cam, hk, Hpp, bp);
    else
        lin_points_body((b - nb_pose) * kLinThreads + threadIdx.x, npt_total, pt_off, pt_win, E, ctl, poses, pts,
                        pose_stride, pt_stride, cam, hk, err_out, rho_out, Hpl_out, Hll, bl);
}

// deterministic block sum / max: wave butterflies, then the wave partials in wave order
__device__ inline double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ inline double block_sum(double v, double* sh) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) r += sh[w];
    __syncthreads();
    return r;
}

__device__ inline double block_max(double v, double* sh) {
    v = wave_max(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) r = fmax(r, sh[w]);
    __syncthreads();
    return r;
}

// strided per-thread partial sum with four independent accumulators (loads in flight)
__device__ inline double strided_sum(const double* __restrict__ p, int n) {
    const int T = blockDim.x;
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int i = threadIdx.x;
    for (; i + 3 * T < n; i += 4 * T) {
        a0 += p[i];
        a1 += p[i + T];
        a2 += p[i + 2 * T];
        a3 += p[i + 3 * T];
    }
    for (; i < n; i += T) a0 += p[i];
    return (a0 + a1) + (a2 + a3);
}

// OptimizationAlgorithmLevenberg::solve prologue (optimization_algorithm_levenberg.cpp:61-104)
__global__ void __launch_bounds__(kCtlThreads) k_iter_begin(const WinDesc* __restrict__ wins,
                                                            WinCtl* __restrict__ ctl,
                                                            const double* __restrict__ rho,
                                                            const double* __restrict__ Hpp,
                                                            const double* __restrict__ Hll,
                                                            const volatile int* __restrict__ stop_dev, int seq) {
    __shared__ double sh[kCtlThreads / 64];
    const WinDesc W = wins[blockIdx.x];
    WinCtl& C = ctl[blockIdx.x];
    if (!C.need_lin) return;
    // thread 0: the control block and the stop sample load while the sums run
    WinCtl c;
    int stop = 0;
    if (threadIdx.x == 0) {
        c = C;
        // SparseOptimizer::optimize: no iteration once terminate() (sparse_optimizer.cpp:376);
        // stop_dev[seq & 1]: this step's sample of the host word (k_trial_control of the previous
        // step wrote it; the same value this step's k_trial_control decides on)
        stop = stop_dev[seq & 1];
    }
    const double chi = block_sum(strided_sum(rho + W.e0, W.ne), sh);
    double m = 0;
    if (C.it == 0) {
        for (int i = threadIdx.x; i < W.np; i += kCtlThreads)
            for (int j = 0; j < 6; j++) m = fmax(m, fabs(Hpp[24 * (long long)(W.pose0 + i) + sym6(j, j)]));
        for (int i = threadIdx.x; i < W.npt; i += kCtlThreads)
            for (int j = 0; j < 3; j++) m = fmax(m, fabs(Hll[8 * (long long)(W.pt0 + i) + sym3(j, j)]));
        m = block_max(m, sh);
    }
    if (threadIdx.x == 0) {
        c.need_lin = 0;
        if (stop) {
            c.active = 0;
        } else {
            c.cur_chi = chi;
            c.ini_chi = chi;
            if (c.opt == 0 && c.it == 0) c.chi2_initial = chi;
            if (c.it == 0) {
                c.lambda = c.user_lambda > 0 ? c.user_lambda : 1e-5 * m;
                c.ni = 2;
                c.nbad = 0;
            }
            c.qmax = 0;
            c.need_trial = 1;
        }
        C = c;
    }
}

// ---------------------------------------------------------------- trial kernels

__device__ inline void point_dinv(const double* __restrict__ Hll, long long p, double lam, double* Di) {
    const double* h = Hll + 8 * p;
    const double D[9] = {h[0] + lam, h[1], h[2], h[1], h[3] + lam, h[4], h[2], h[4], h[5] + lam};
    inverse3(D, Di);
}

// Schur per landmark (block_solver.hpp:381-432), the per-point half: Dinv = (Hll + lambda I)^-1
// (Eigen cofactor inverse) and db = Dinv b_l, one thread per point, kPdStride doubles each.  The
// per-edge products B Dinv and B db are formed where they are used (k_schur_blocks), so no
// per-edge record goes through HBM.
constexpr int kPdStride = 12;  // Dinv upper triangle (D00 D01 D02 D11 D12 D22), db (3), pad
// Eigen's cofactor inverse of a symmetric 3x3 is symmetric bit for bit (every cofactor pairs
// the same two products in the same order), so the upper triangle holds all of Dinv.
__device__ __forceinline__ void pd_load(const double* __restrict__ o, double* Di, double* db) {
    const double d00 = o[0], d01 = o[1], d02 = o[2], d11 = o[3], d12 = o[4], d22 = o[5];
    Di[0] = d00; Di[1] = d01; Di[2] = d02;
    Di[3] = d01; Di[4] = d11; Di[5] = d12;
    Di[6] = d02; Di[7] = d12; Di[8] = d22;
    db[0] = o[6]; db[1] = o[7]; db[2] = o[8];
}
__global__ void k_point_prep(int npt_total, const int* __restrict__ pt_win, const WinCtl* __restrict__ ctl,
                             const double* __restrict__ Hll, const double* __restrict__ bl, double* __restrict__ pd) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npt_total) return;
    const WinCtl& C = ctl[pt_win[p]];
    if (!C.need_trial) return;
    double Di[9];
    point_dinv(Hll, p, C.lambda, Di);
    const double* b = bl + 4 * (long long)p;
    double* o = pd + (long long)kPdStride * p;
    o[0] = Di[0]; o[1] = Di[1]; o[2] = Di[2]; o[3] = Di[4]; o[4] = Di[5]; o[5] = Di[8];
#pragma unroll
    for (int r = 0; r < 3; r++) o[6 + r] = Di[3 * r] * b[0] + Di[3 * r + 1] * b[1] + Di[3 * r + 2] * b[2];
    o[9] = o[10] = o[11] = 0.0;
}

// 64-bit value of the partner lane (lane ^ 1): DPP quad_perm [1,0,3,2] on both halves
__device__ __forceinline__ double swap_pair(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// value of lane j (compile-time) within each 32-lane half: ds_swizzle bit mode, and_mask 0,
// or_mask j (no LDS memory traffic, no SGPR round trip)
template <int J>
__device__ inline double bcast32_t(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)b, J << 5), hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), J << 5);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// kSchurLanes (16) lanes per 6x6 block (i1 <= i2) of the Schur complement, four blocks per wave:
// lanes stride over the block's contributions (one per point observed by both poses), each
// accumulating the full 6x6 B_a Dinv Hpl_b^T, then a butterfly inside the lane group (a
// config-4 off-diagonal block has ~50 contributions: ~3 per lane; 8 or 4 lanes measured slower).  The reference
// block (i1, i2) (upper) is written transposed into the lower triangle of the dense row-major
// matrix; diagonal blocks also produce the rhs row b_s = b_p - sum B db (augmented row n).
// Blocks are visited through an order list: every window's diagonal blocks first (one wave
// each: a diagonal block sums a contribution per observation of its pose, ~330 at config 4),
// then the off-diagonal ones (16 lanes each, ~50 contributions).
constexpr int kSchurLanes = 16, kSchurDiagLanes = 64;

template <int W16>
__device__ inline double group_sum(double v) {
#pragma unroll
    for (int o = W16 / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W16);
    return v;
}

// XCD-aware workgroup order (cdna_hip_programming.md T1, bijective form): hardware
// round-robins consecutive workgroups over the 8 XCDs; remapped, each XCD takes a contiguous
// run of the window-major block list, so a window's edge data (B Dinv, Hpl: ~5 MB at config
// 4) is gathered through one XCD's L2 instead of all eight.  Speed only: any placement is
// correct.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// tile-major scratch of k_ldlt_t16 (see there): window w's tiles start at w * kT16Tiles * 256
// doubles, column-major over tile columns; element (R, C), R >= C, of the lower triangle goes to
// tile (R >> 4, C >> 4) in the transposed accumulator layout (lane (R & 15) + 16 (C & 3),
// register (C & 15) >> 2), and for a diagonal tile also to its mirror (C, R).
__device__ __forceinline__ long long blockIdx_win_tiles(int win) { return (long long)win * kT16Tiles * 256; }
__device__ __forceinline__ void t16_put(double* Tw, int n, int R, int Cc, double v) {
    const int T = (n + 15) >> 4, I = R >> 4, J = Cc >> 4;
    const int t = J * T - J * (J - 1) / 2 + (I - J);
    const int r = R & 15, c = Cc & 15;
    Tw[256LL * t + 4 * (r + 16 * (c & 3)) + (c >> 2)] = v;
    if (I == J && r != c) Tw[256LL * t + 4 * (c + 16 * (r & 3)) + (r >> 2)] = v;
}

// ---------------------------------------------------------------- Schur contribution lists
// The Schur contributions of block (i1, i2) are the MapPoints observed by both poses (one
// free-pose edge each: block_solver.hpp:403-430 walks them per landmark), in point order.  They
// are built once per solve on the device instead of on the host (8 B per pair: ~74 MB per 128
// config-4 windows through PCIe, and most of the host plan time): every pose gets a bitmap over
// its window's points and the list of its edges in point order; a block's list is the AND of the
// two bitmaps with each common point ranked inside both pose lists.
//   bm  [W.bm0 + i * nwd + wd]   bit q <-> local point 64 wd + q observed by local pose i
//   bmp [same index]             set bits of pose i before word wd
//   pls [W.spe0 + pbase[i] + r]  r-th free-pose edge (edge id) of pose i in point order
__device__ __forceinline__ void bm_set_body(int s, int nspe_total, const int* __restrict__ spe,
                                            const EdgeS* __restrict__ E, const WinDesc* __restrict__ wins,
                                            unsigned long long* __restrict__ bm, int* __restrict__ spe_hp) {
    if (s >= nspe_total) return;
    const EdgeS e = E[spe[s]];
    spe_hp[s] = e.hp;  // free-pose index per spe entry (the back-substitution's xp row)
    const WinDesc& W = wins[e.win];
    const int lp = e.pt - W.pt0, i = e.hp - W.pose0;
    atomicOr(bm + W.bm0 + (long long)i * W.nwd + (lp >> 6), 1ull << (lp & 63));
}

// one thread per pose of the window: word prefix counts, then the pose list bases in pose order
__device__ __forceinline__ void bm_scan_body(int w, const WinDesc* __restrict__ wins,
                                             const unsigned long long* __restrict__ bm, int* __restrict__ bmp,
                                             int* __restrict__ pbase, int* __restrict__ pcnt) {
    __shared__ int cnt[kMaxN / 6 + 1];
    const WinDesc W = wins[w];
    for (int i = threadIdx.x; i < W.np; i += blockDim.x) {
        const long long o = W.bm0 + (long long)i * W.nwd;
        int run = 0;
        for (int wd = 0; wd < W.nwd; wd++) {
            bmp[o + wd] = run;
            run += __popcll(bm[o + wd]);
        }
        cnt[i] = run;
        pcnt[W.pose0 + i] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int i = 0; i < W.np; i++) {
            pbase[W.pose0 + i] = run;
            run += cnt[i];
        }
    }
}

__device__ __forceinline__ void bm_list_body(int s, int nspe_total, const int* __restrict__ spe,
                                             const EdgeS* __restrict__ E, const WinDesc* __restrict__ wins,
                                             const unsigned long long* __restrict__ bm, const int* __restrict__ bmp,
                                             const int* __restrict__ pbase, int* __restrict__ pls,
                                             int* __restrict__ ppt) {
    if (s >= nspe_total) return;
    const EdgeS e = E[spe[s]];
    const WinDesc& W = wins[e.win];
    const int lp = e.pt - W.pt0, i = e.hp - W.pose0;
    const long long o = W.bm0 + (long long)i * W.nwd + (lp >> 6);
    const int r = bmp[o] + __popcll(bm[o] & ((1ull << (lp & 63)) - 1));
    pls[W.spe0 + pbase[e.hp] + r] = spe[s];
    ppt[W.spe0 + pbase[e.hp] + r] = e.pt;  // its point (k_schur_rows' Dinv)
}

__device__ __forceinline__ int ct_words(const WinDesc& W, const unsigned long long* __restrict__ bm, int i1, int i2,
                                        int wd, unsigned long long* w1, unsigned long long* w2) {
    *w1 = bm[W.bm0 + (long long)i1 * W.nwd + wd];
    *w2 = bm[W.bm0 + (long long)i2 * W.nwd + wd];
    return __popcll(*w1 & *w2);
}

// thread per block: its number of contributions
__device__ __forceinline__ void ct_count_body(int b, int nblk_total, const int2* __restrict__ blk_pose,
                                              const int* __restrict__ blk_win, const WinDesc* __restrict__ wins,
                                              const unsigned long long* __restrict__ bm, int* __restrict__ cnt) {
    if (b >= nblk_total) return;
    const WinDesc& W = wins[blk_win[b]];
    const int2 ij = blk_pose[b];
    int c = 0;
    unsigned long long w1, w2;
    for (int wd = 0; wd < W.nwd; wd++) c += ct_words(W, bm, ij.x, ij.y, wd, &w1, &w2);
    cnt[b] = c;
}

// workgroup per window: ct_off over the window's blocks (exclusive scan from W.ct0)
constexpr int kCtScanThreads = 1024;
__device__ __forceinline__ void ct_scan_body(int w, const WinDesc* __restrict__ wins, const int* __restrict__ cnt,
                                             int* __restrict__ ct_off) {
    __shared__ int part[kCtScanThreads];
    const WinDesc W = wins[w];
    const int per = (W.nblk + kCtScanThreads - 1) / kCtScanThreads;
    const int b0 = min(W.nblk, (int)threadIdx.x * per), b1 = min(W.nblk, b0 + per);
    int sum = 0;
    for (int b = b0; b < b1; b++) sum += cnt[W.blk0 + b];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < kCtScanThreads; o <<= 1) {  // Hillis-Steele inclusive scan
        const int v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    long long run = W.ct0 + part[threadIdx.x] - sum;
    for (int b = b0; b < b1; b++) {
        ct_off[W.blk0 + b] = (int)run;
        run += cnt[W.blk0 + b];
    }
    if (threadIdx.x == kCtScanThreads - 1) ct_off[W.blk0 + W.nblk] = (int)(W.ct0 + part[threadIdx.x]);
}

// wave per block: lane = 64-point word (word-prefix by wave scan), each lane writes the pairs of
// its word's common points in point order
__global__ void __launch_bounds__(256) k_ct_fill(int nblk_total, const int2* __restrict__ blk_pose,
                                                 const int* __restrict__ blk_win, const WinDesc* __restrict__ wins,
                                                 const unsigned long long* __restrict__ bm,
                                                 const int* __restrict__ bmp, const int* __restrict__ pbase,
                                                 const int* __restrict__ pls, const int* __restrict__ ct_off,
                                                 int4* __restrict__ ct) {
    // wave index via v_readfirstlane: wave-uniform, so the block's records load into SGPRs
    const int b = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= nblk_total) return;
    const WinDesc& W = wins[blk_win[b]];
    const int2 ij = blk_pose[b];
    const int* l1 = pls + W.spe0 + pbase[W.pose0 + ij.x];
    const int* l2 = pls + W.spe0 + pbase[W.pose0 + ij.y];
    int pos = ct_off[b];
    for (int wd0 = 0; wd0 < W.nwd; wd0 += 64) {
        const int wd = wd0 + lane;
        unsigned long long w1 = 0, w2 = 0;
        const int c = wd < W.nwd ? ct_words(W, bm, ij.x, ij.y, wd, &w1, &w2) : 0;
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        int k = pos + incl - c;
        if (c) {
            const long long o1 = W.bm0 + (long long)ij.x * W.nwd + wd, o2 = W.bm0 + (long long)ij.y * W.nwd + wd;
            const int r1 = bmp[o1], r2 = bmp[o2];
            unsigned long long m = w1 & w2;
            while (m) {
                const int q = __builtin_ctzll(m);
                const unsigned long long below = (1ull << q) - 1ull;
                m &= m - 1ull;
                // record {edge a, point, edge b, rank of edge a in pose i1's list = k_schur_rows' W row}
                const int ra = r1 + __popcll(w1 & below);
                ct[k++] = int4{l1[ra], W.pt0 + 64 * wd + q, l2[r2 + __popcll(w2 & below)], ra};
            }
        }
        pos += __shfl(incl, 63, 64);
    }
}

template <int NL>
__device__ __forceinline__ void schur_block_body(int wg, int nlist, const int* __restrict__ order,
                                                     const int2* __restrict__ blk_pose,
                                                     const int* __restrict__ blk_win, const int* __restrict__ ct_off,
                                                     const int4* __restrict__ ct, const WinDesc* __restrict__ wins,
                                                     const WinCtl* __restrict__ ctl, const double* __restrict__ Hpp,
                                                     const double* __restrict__ bp, const double* __restrict__ lin,
                                                     const double* __restrict__ pd, double* __restrict__ Hs,
                                                     double* __restrict__ Ts) {
    const int idx = wg * (256 / NL) + threadIdx.x / NL, lane = threadIdx.x % NL;
    const bool live = idx < nlist;
    const int b = order[live ? idx : 0];
    const int win = blk_win[b];
    const WinCtl& C = ctl[win];
    const bool act = live && C.need_trial;
    const WinDesc W = wins[win];
    const int2 ij = blk_pose[b];  // local free-pose indices i1 <= i2
    const int i1 = ij.x, i2 = ij.y;
    // lane = (row half h, contribution stream j): rows 3h..3h+2 of the 6x6 over every
    // kStreams-th contribution; 18 accumulators keep the kernel at 4 waves per SIMD.  Per
    // contribution (edges a of pose i1 and b of pose i2 on point p) the lane forms its rows of
    // B_a Dinv_p (the products k_schur_edges used to store per edge, same expression) and
    // multiplies by Hpl_b^T; a diagonal block also sums its rows of B_a db_p (the rhs).
    const int h = lane & 1, j = lane >> 1;
    constexpr int kStreams = NL / 2;
    double acc[18];
#pragma unroll
    for (int k = 0; k < 18; k++) acc[k] = 0.0;
    double sb[3] = {0, 0, 0};
    // The two lanes of a contribution load one half of Hpl_b each and trade halves by DPP; the
    // next contribution's record is fetched while this one is computed.
    if (act) {
        int k = ct_off[b] + j;
        const int kend = ct_off[b + 1];
        int4 nxt = k < kend ? ct[k] : int4{0, 0, 0, 0};
        while (k < kend) {
            const int4 ab = nxt;
            k += kStreams;
            if (k < kend) nxt = ct[k];
            const double* Ba = lin + (long long)kHplStride * ab.x + 9 * h;
            const double* Bo = lin + (long long)kHplStride * ab.z + 9 * h;
            double ba[9], bo[9], di[9], db[3], bd[9], bj[18];
#pragma unroll
            for (int t = 0; t < 9; t++) ba[t] = Ba[t];
#pragma unroll
            for (int t = 0; t < 9; t++) bo[t] = Bo[t];
            pd_load(pd + (long long)kPdStride * ab.y, di, db);
            // columns in lane order: this lane's rows of Hpl_b first (c' = (c + 3h) mod 6)
#pragma unroll
            for (int t = 0; t < 9; t++) {
                bj[t] = bo[t];
                bj[9 + t] = swap_pair(bo[t]);
            }
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 3; c++)
                    bd[3 * r + c] = ba[3 * r] * di[c] + ba[3 * r + 1] * di[3 + c] + ba[3 * r + 2] * di[6 + c];
            if (i1 == i2) {
#pragma unroll
                for (int r = 0; r < 3; r++) sb[r] += ba[3 * r] * db[0] + ba[3 * r + 1] * db[1] + ba[3 * r + 2] * db[2];
            }
            // acc += B_a Dinv Hpl_b^T with fused multiply-adds: g2o's own build (-O3 -march=native)
            // contracts these Eigen products too; the rounding differs from the oracle's unfused
            // sums well inside the 1e-5 bar (tests/test_gpu_lba.py)
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 6; c++)
                    acc[6 * r + c] = __builtin_fma(bd[3 * r + 2], bj[3 * c + 2],
                                                   __builtin_fma(bd[3 * r + 1], bj[3 * c + 1],
                                                                 __builtin_fma(bd[3 * r], bj[3 * c], acc[6 * r + c])));
        }
    }
    // butterfly over the streams of the same half (lane bits 1..)
#pragma unroll
    for (int k = 0; k < 18; k++) {
#pragma unroll
        for (int o = 2; o < NL; o <<= 1) acc[k] += __shfl_xor(acc[k], o, NL);
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int o = 2; o < NL; o <<= 1) sb[r] += __shfl_xor(sb[r], o, NL);
    }
    const int gp = W.pose0 + i1;
    if (!act) return;
    double* H = Hs + W.hs_off;
    // every lane of a half holds that half's sums: stream j writes its elements j, j+8, j+16
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const int e = j + kStreams * q;  // element of this half (rows 3h.., 6 columns)
        if (e >= 18) break;
        const int r = 3 * h + e / 6, c = e % 6;
        double v = 0.0;
        if (i1 == i2) {
            const int rr = r <= c ? r : c, cc = r <= c ? c : r;
            v = Hpp[24 * (long long)gp + sym6(rr, cc)];
            if (r == c) v += C.lambda;
        }
        double m = 0.0;
        const int ek = 6 * (e / 6) + (c + 3 * h) % 6;  // accumulator columns are in lane order
#pragma unroll
        for (int k = 0; k < 18; k++)
            if (k == ek) m = acc[k];
        v -= m;
        // upper (i1, i2)[r][c] -> lower element (6 i2 + c, 6 i1 + r)
        if (i1 != i2 || r <= c) {
            if (Ts) t16_put(Ts + (long long)blockIdx_win_tiles(win), W.n, 6 * i2 + c, 6 * i1 + r, v);
            else H[(long long)(6 * i2 + c) * W.ld + 6 * i1 + r] = v;
        }
    }
    if (i1 == i2 && j == 0) {  // lanes 0 / 1: rhs rows 0..2 / 3..5
#pragma unroll
        for (int r = 0; r < 3; r++)
            H[(long long)ldlt_npad(W.n) * W.ld + 6 * i1 + 3 * h + r] = bp[8 * (long long)gp + 3 * h + r] - sb[r];
    }
}

// Both Schur block lists in one launch: blocks [0, nb_diag) take the npose diagonal blocks
// (kSchurDiagLanes lanes each), the rest the off-diagonal ones; nb_diag is a multiple of 8 so
// each part keeps its XCD-contiguous mapping.
__global__ void __launch_bounds__(256) k_schur_blocks(int nb_diag, int nblk, int npose, const int* __restrict__ order,
                                                      const int2* __restrict__ blk_pose,
                                                      const int* __restrict__ blk_win, const int* __restrict__ ct_off,
                                                      const int4* __restrict__ ct, const WinDesc* __restrict__ wins,
                                                      const WinCtl* __restrict__ ctl, const double* __restrict__ Hpp,
                                                      const double* __restrict__ bp, const double* __restrict__ lin,
                                                      const double* __restrict__ pd, double* __restrict__ Hs,
                                                      double* __restrict__ Ts) {
    const int b = blockIdx.x;
    if (b < nb_diag) {
        const int wg = xcd_swizzle(b, nb_diag);
        if (wg * (256 / kSchurDiagLanes) >= npose) return;  // padding blocks (whole block)
        schur_block_body<kSchurDiagLanes>(wg, npose, order, blk_pose, blk_win, ct_off, ct, wins, ctl, Hpp, bp, lin,
                                          pd, Hs, Ts);
    } else {
        schur_block_body<kSchurLanes>(xcd_swizzle(b - nb_diag, (int)gridDim.x - nb_diag), nblk - npose,
                                      order + npose, blk_pose, blk_win, ct_off, ct, wins, ctl, Hpp, bp, lin, pd, Hs,
                                      Ts);
    }
}

// ---------------------------------------------------------------- Schur by block row (round 3)
// k_schur_rows: one workgroup per free pose i1 = one block row (i1, i1..np-1) of the Schur
// complement.  The row's W_a = Hpl_a Dinv_p (6x3, one per edge a of pose i1, in point order) is
// formed once into LDS, so a contribution of a block (i1, i2) loads only the other side's Hpl_b
// and its list record and does no B Dinv product (k_schur_blocks, kept as SLAMHOT_SCHUR=blocks,
// re-formed B_a Dinv for every block and read Hpl_a and Dinv each time).
//   W pass: lane pair (rows 3h..3h+2) per edge a: W_a into LDS, its edge id, and the rhs sums
//     Hpl_a db_p;
//   diagonal block: lane quad per edge a, sum W_a Hpl_a^T, reduced over the workgroup in a fixed
//     order (wave butterflies, then the waves in order);
//   off-diagonal rounds: 32 lanes (8 contribution streams x a quad) per block (i1, i2); the
//     record {edge b, rank of edge a} gives Hpl_b and the W row in LDS; per-block butterfly.
// A lane quad (h, v) takes the 3x3 sub-block rows 3h.., columns 3v.. of a 6x6 product: W rows
// from LDS (equal h: one broadcast address), Hpl_b rows 3v.. (equal v: the same bytes in one
// load instruction), nine accumulators.
// Rows with more than kSrChunk edges take W chunk by chunk (recomputed per round): the records of
// a block are in point order, so each stream's chunk boundary is where its ranks pass the chunk.
// Same per-contribution expressions as k_schur_blocks (B Dinv, then an FMA chain per element);
// only the order in which contributions are summed differs.
// 512 threads and a 384-edge W chunk (55 KB): two workgroups per CU at <= 128 VGPRs.  Measured
// and rejected: 768 / 1024 threads at 80 / 64 VGPRs (spills: 366 / 570 us vs 310 us per 128
// config-4 windows).
template <int R>
__device__ __forceinline__ double row_ror(double v) {  // DPP row_ror:R on both halves of a double
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x120 + R, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x120 + R, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Sum over the lanes l, l^4, l^8, l^12 of a 16-lane DPP row (every lane): two row rotations
// (VALU) instead of two ds_bpermute round trips per double (the sums of k_schur_rows' eight
// contribution streams / lane quads; SLAMHOT_SR_SHFL keeps the __shfl_xor butterflies).
__device__ __forceinline__ double sum_quads16(double v) {
    v += row_ror<4>(v);
    v += row_ror<8>(v);
    return v;
}
constexpr int kSrThreads = 512, kSrGroups = kSrThreads / 32, kSrChunk = 384;

// W rows [r0, r1) of pose i1's list into LDS (lane pair per edge, rows 3h..3h+2), and with kSb
// the rhs sums Hpl_a db_p.  A pair takes at most kSrWIt edges of a chunk; all their loads are
// issued before the first product.
constexpr int kSrWIt = (kSrChunk + kSrThreads / 2 - 1) / (kSrThreads / 2);
template <bool kSb>
__device__ __forceinline__ void sr_w(int r0, int r1, const int* __restrict__ lst, const int* __restrict__ lpt,
                                     const double* __restrict__ lin, const double* __restrict__ pd, double* Wl,
                                     int* We, double (&sb)[3]) {
    const int q = threadIdx.x >> 1, h = threadIdx.x & 1;
    int e[kSrWIt], pt[kSrWIt];
#pragma unroll
    for (int m = 0; m < kSrWIt; m++) {
        const int r = r0 + q + m * (kSrThreads / 2);
        e[m] = r < r1 ? lst[r] : -1;
        pt[m] = r < r1 ? lpt[r] : 0;
    }
    double ba[kSrWIt][9], di[kSrWIt][9], db[kSrWIt][3];
#pragma unroll
    for (int m = 0; m < kSrWIt; m++) {
        if (e[m] < 0) continue;
        const double* Ba = lin + (long long)kHplStride * e[m] + 9 * h;
#pragma unroll
        for (int t = 0; t < 9; t++) ba[m][t] = Ba[t];
        pd_load(pd + (long long)kPdStride * pt[m], di[m], db[m]);
    }
#pragma unroll
    for (int m = 0; m < kSrWIt; m++) {
        if (e[m] < 0) continue;
        double* o = Wl + 18 * (q + m * (kSrThreads / 2)) + 9 * h;
        if (h == 0) We[q + m * (kSrThreads / 2)] = e[m];
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
#pragma unroll
            for (int c = 0; c < 3; c++)
                o[3 * rr + c] = ba[m][3 * rr] * di[m][c] + ba[m][3 * rr + 1] * di[m][3 + c] + ba[m][3 * rr + 2] * di[m][6 + c];
        if constexpr (kSb) {
#pragma unroll
            for (int rr = 0; rr < 3; rr++)
                sb[rr] += ba[m][3 * rr] * db[m][0] + ba[m][3 * rr + 1] * db[m][1] + ba[m][3 * rr + 2] * db[m][2];
        }
    }
}

// Products: a contribution W_a Hpl_b^T (6x6) is taken by a lane quad, lane (h, v) the 3x3
// sub-block rows 3h.., columns 3v..: its W rows from LDS (lanes of equal h read the same
// address: a broadcast) and Hpl_b rows 3v.. (lanes of equal v load the same bytes in one
// instruction), nine accumulators, no cross-lane traffic until the final reduction.
__device__ __forceinline__ void sr_fma(const double* Wa, const double* __restrict__ Bo, double (&acc)[9]) {
    double bo[9];
#pragma unroll
    for (int t = 0; t < 9; t++) bo[t] = Bo[t];
#pragma unroll
    for (int rr = 0; rr < 3; rr++) {
        const double w0 = Wa[3 * rr], w1 = Wa[3 * rr + 1], w2 = Wa[3 * rr + 2];
#pragma unroll
        for (int cc = 0; cc < 3; cc++)
            acc[3 * rr + cc] = __builtin_fma(w2, bo[3 * cc + 2], __builtin_fma(w1, bo[3 * cc + 1],
                                                                            __builtin_fma(w0, bo[3 * cc], acc[3 * rr + cc])));
    }
}

// two contributions, loads first; the second one only when `two`
__device__ __forceinline__ void sr_fma2(const double* Wa, const double* __restrict__ Bo, const double* Wa2,
                                        const double* __restrict__ Bo2, bool two, double (&acc)[9]) {
    double w[9], bo[9], w2[9], bo2[9];
#pragma unroll
    for (int t = 0; t < 9; t++) bo[t] = Bo[t];
#pragma unroll
    for (int t = 0; t < 9; t++) bo2[t] = Bo2[t];
#pragma unroll
    for (int t = 0; t < 9; t++) w[t] = Wa[t];
#pragma unroll
    for (int t = 0; t < 9; t++) w2[t] = Wa2[t];
#pragma unroll
    for (int rr = 0; rr < 3; rr++)
#pragma unroll
        for (int cc = 0; cc < 3; cc++)
            acc[3 * rr + cc] = __builtin_fma(w[3 * rr + 2], bo[3 * cc + 2],
                                             __builtin_fma(w[3 * rr + 1], bo[3 * cc + 1],
                                                           __builtin_fma(w[3 * rr], bo[3 * cc], acc[3 * rr + cc])));
    if (two) {
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
#pragma unroll
            for (int cc = 0; cc < 3; cc++)
                acc[3 * rr + cc] = __builtin_fma(w2[3 * rr + 2], bo2[3 * cc + 2],
                                                 __builtin_fma(w2[3 * rr + 1], bo2[3 * cc + 1],
                                                               __builtin_fma(w2[3 * rr], bo2[3 * cc], acc[3 * rr + cc])));
    }
}

__global__ void __launch_bounds__(kSrThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) k_schur_rows(int npose, const int* __restrict__ pose_win,
                                                           const WinDesc* __restrict__ wins,
                                                           const WinCtl* __restrict__ ctl, const int* __restrict__ pls,
                                                           const int* __restrict__ ppt, const int* __restrict__ pbase,
                                                           const int* __restrict__ pcnt,
                                                           const EdgeS* __restrict__ E, const int* __restrict__ ct_off,
                                                           const int4* __restrict__ ct, const double* __restrict__ Hpp,
                                                           const double* __restrict__ bp, const double* __restrict__ lin,
                                                           const double* __restrict__ pd, double* __restrict__ Hs,
                                                           double* __restrict__ Ts) {
    __shared__ double Wl[kSrChunk * 18];
    __shared__ int We[kSrChunk];  // edge id of each W row
    __shared__ double red[kSrThreads / 64][4][9];
    __shared__ double red_sb[kSrThreads / 64][2][3];
    const int gp = xcd_swizzle(blockIdx.x, gridDim.x);  // a window's rows run on one XCD
    if (gp >= npose) return;
    const int win = pose_win[gp];
    const WinCtl& C = ctl[win];
    if (!C.need_trial) return;
    const WinDesc W = wins[win];
    const int i1 = gp - W.pose0;
    const int* lst = pls + W.spe0 + pbase[gp];
    const int* lpt = ppt + W.spe0 + pbase[gp];
    const int cnt = pcnt[gp];
    const int nch = max(1, (cnt + kSrChunk - 1) / kSrChunk);
    double* H = Hs + W.hs_off;
    double* Tw = Ts ? Ts + blockIdx_win_tiles(win) : nullptr;
    auto put = [&](int R, int Cc, double v) {  // lower element (R, Cc) of the Schur system
        if (Tw) t16_put(Tw, W.n, R, Cc, v);
        else H[(long long)R * W.ld + Cc] = v;
    };
    const int quad = threadIdx.x & 3, h = quad & 1, v = quad >> 1;  // sub-block rows 3h.., columns 3v..

    // ---- diagonal block (i1, i1) = sum_a W_a Hpl_a^T (lane quad per edge a) and the rhs rows
    {
        double acc[9], sb[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 9; k++) acc[k] = 0.0;
        const int e4 = threadIdx.x >> 2;  // lane quad per edge
        for (int c = 0; c < nch; c++) {
            const int r0 = c * kSrChunk, r1 = min(cnt, r0 + kSrChunk);
            if (c) __syncthreads();
            sr_w<true>(r0, r1, lst, lpt, lin, pd, Wl, We, sb);
            __syncthreads();
            // edge ids from LDS (the W pass left them there)
            for (int r = r0 + e4; r < r1; r += kSrThreads / 4)
                sr_fma(Wl + 18 * (r - r0) + 9 * h, lin + (long long)kHplStride * We[r - r0] + 9 * v, acc);
        }
        // butterflies over the wave (quads: lane bits 2..5; sb pairs: bits 1..5), then the waves
#ifdef SLAMHOT_SR_SHFL
#pragma unroll
        for (int k = 0; k < 9; k++)
#pragma unroll
            for (int o = 4; o < 64; o <<= 1) acc[k] += __shfl_xor(acc[k], o, 64);
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int o = 2; o < 64; o <<= 1) sb[k] += __shfl_xor(sb[k], o, 64);
#else
#pragma unroll
        for (int k = 0; k < 9; k++) {
            acc[k] = sum_quads16(acc[k]);
            acc[k] += __shfl_xor(acc[k], 16, 64);
            acc[k] += __shfl_xor(acc[k], 32, 64);
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            sb[k] += row_ror<2>(sb[k]);  // pairs: lanes l, l^2 (same h) ...
            sb[k] = sum_quads16(sb[k]);
            sb[k] += __shfl_xor(sb[k], 16, 64);
            sb[k] += __shfl_xor(sb[k], 32, 64);
        }
#endif
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        if (ln < 4) {
#pragma unroll
            for (int k = 0; k < 9; k++) red[wv][ln][k] = acc[k];
        }
        if (ln < 2) {
#pragma unroll
            for (int k = 0; k < 3; k++) red_sb[wv][ln][k] = sb[k];
        }
        __syncthreads();
        const int t = threadIdx.x;
        if (t < 36) {  // element (r, c), r <= c, of the upper block -> lower (6 i1 + c, 6 i1 + r)
            const int r = t / 6, c = t % 6;
            if (r <= c) {
                const int qd = r / 3 + 2 * (c / 3), el = 3 * (r % 3) + c % 3;
                double m = 0.0;
                for (int w = 0; w < kSrThreads / 64; w++) m += red[w][qd][el];
                double val = Hpp[24 * (long long)gp + sym6(r, c)];
                if (r == c) val += C.lambda;
                put(6 * i1 + c, 6 * i1 + r, val - m);
            }
        } else if (t < 42) {
            const int r = t - 36;
            double m = 0.0;
            for (int w = 0; w < kSrThreads / 64; w++) m += red_sb[w][r / 3][r % 3];
            H[(long long)ldlt_npad(W.n) * W.ld + 6 * i1 + r] = bp[8 * (long long)gp + r] - m;
        }
    }

    // ---- off-diagonal blocks (i1, i2 > i1): 32 lanes (8 contribution streams x a quad) per block
    const int g = threadIdx.x >> 5, j = (threadIdx.x & 31) >> 2;
    const int nboff = W.np - 1 - i1;
    for (int rd = 0; rd * kSrGroups < nboff; rd++) {
        const int i2 = i1 + 1 + g + kSrGroups * rd;
        const bool live = i2 < W.np;
        const int b = W.blk0 + (live ? i2 * (i2 + 1) / 2 + i1 : 0);
        int k = live ? ct_off[b] + j : 0;
        const int kend = live ? ct_off[b + 1] : 0;
        double acc[9];
#pragma unroll
        for (int t = 0; t < 9; t++) acc[t] = 0.0;
        for (int c = 0; c < nch; c++) {
            if (nch > 1) {  // this chunk's W (a single chunk's W stays from the diagonal pass)
                __syncthreads();
                double s_[3];
                sr_w<false>(c * kSrChunk, min(cnt, (c + 1) * kSrChunk), lst, lpt, lin, pd, Wl, We, s_);
                __syncthreads();
            }
            const int rbase = c * kSrChunk, rend = rbase + kSrChunk;
            // record = {edge b, rank of edge a}; the next one is fetched while this one is computed
            auto rec_at = [&](int kk) {
                return kk < kend ? *reinterpret_cast<const int2*>(reinterpret_cast<const int*>(ct + kk) + 2)
                                 : int2{0, 1 << 30};
            };
            // ranks grow along a block's list, so an entry past the chunk ends the stream's chunk
            // two of the stream's entries per step (their Hpl_b loads issued together), in order
            int2 ra = rec_at(k), rb = rec_at(k + 8);
            while (ra.y < rend) {
                const int2 na = rec_at(k + 16), nb = rec_at(k + 24);
                const bool two = rb.y < rend;
                sr_fma2(Wl + 18 * (ra.y - rbase) + 9 * h, lin + (long long)kHplStride * ra.x + 9 * v,
                        Wl + 18 * ((two ? rb.y : ra.y) - rbase) + 9 * h,
                        lin + (long long)kHplStride * (two ? rb.x : ra.x) + 9 * v, two, acc);
                if (!two) {
                    k += 8;
                    break;
                }
                k += 16;
                ra = na;
                rb = nb;
            }
        }
#ifdef SLAMHOT_SR_SHFL
#pragma unroll
        for (int t = 0; t < 9; t++)
#pragma unroll
            for (int o = 4; o < 32; o <<= 1) acc[t] += __shfl_xor(acc[t], o, 32);
#else
#pragma unroll
        for (int t = 0; t < 9; t++) {
            acc[t] = sum_quads16(acc[t]);
            acc[t] += __shfl_xor(acc[t], 16, 32);
        }
#endif
        if (live) {
            // every stream of a quad lane holds the sums: stream j writes element j (and 0 also 8)
#pragma unroll
            for (int qq = 0; qq < 2; qq++) {
                const int e = j + 8 * qq;
                if (e >= 9) break;
                double m = 0.0;
#pragma unroll
                for (int kk = 0; kk < 9; kk++)
                    if (kk == e) m = acc[kk];
                put(6 * i2 + 3 * v + e % 3, 6 * i1 + 3 * h + e / 3, 0.0 - m);
            }
        }
    }
}

// Dense LDL^T of the augmented lower-triangular system [[Hs, .], [b_s^T, .]] in place
// (row-major, leading dimension ld).  The pose dimension n is padded to npad (a multiple of
// kNB) with an identity block, which the factorization leaves invariant; the rhs is row npad
// and becomes z = D^-1 L^-1 b_s, then L^T x = z.  Fails like Eigen's
// SimplicialLDLT::factorize only on an exactly zero pivot.
// One 512-thread block per window; per panel of kNB columns:
//   (1) diagonal block: wave 0, lane = row, pivot rows broadcast through LDS,
//   (2) rows below: one thread per row (right-looking inside the row),
//   (3) trailing update C -= (L D) L^T on 16x16 tiles with v_mfma_f64_16x16x4_f64, the panel
//       held column-major in LDS; the rhs row is a GEMV on the side.
#ifdef LBA_PHASE_TIMING
__device__ unsigned long long g_ldlt_phase[8];
#define PHASE_MARK(i)                                                        \
    do {                                                                     \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                           \
            const unsigned long long now = wall_clock64();                   \
            if ((i) > 0) g_ldlt_phase[(i)] += now - g_ldlt_phase[0];         \
            g_ldlt_phase[0] = now;                                           \
        }                                                                    \
    } while (0)
#else
#define PHASE_MARK(i) \
    do {              \
    } while (0)
#endif



// One pivot step of the diagonal-block LDL^T (lane = row, full symmetric rows in registers):
// pivot row J broadcast by ds_swizzle, rows below eliminate with it.
template <int J>
__device__ __forceinline__ void diag_step(double (&row)[kNB], int lane, bool& bad, double* dsh, double* dinv) {
    double rb[kNB];
#pragma unroll
    for (int c = J; c < kNB; c++) rb[c] = bcast32_t<J>(row[c]);
    const double dj = rb[J];
    if (dj == 0.0) bad = true;
    const int rl = lane & (kNB - 1);
    if (rl > J) {
        const double lj = row[J] / dj;
#pragma unroll
        for (int c = J + 1; c < kNB; c++) row[c] = __builtin_fma(-lj, rb[c], row[c]);
        row[J] = lj;
    }
    if (lane == J) {
        dsh[J] = dj;
        dinv[J] = 1.0 / dj;
    }
    if constexpr (J + 1 < kNB) diag_step<J + 1>(row, lane, bad, dsh, dinv);
}

__global__ void __launch_bounds__(512) k_ldlt(const WinDesc* __restrict__ wins, WinCtl* __restrict__ ctl,
                                               double* __restrict__ Hs, double* __restrict__ xp_out) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const WinDesc W = wins[blockIdx.x];
    WinCtl& C = ctl[blockIdx.x];
    if (!C.need_trial) return;
    const int n = W.n, npad = ldlt_npad(n), ld = W.ld, NP = ldlt_np(n);
    double* A = Hs + W.hs_off;
    double* PLT = smem;                          // kNB x NP: panel column q, rows from R0
    double* T = PLT + (size_t)kNB * NP;          // 32 x 33 diagonal block
    double* rowbuf = T + kNB * (kNB + 1);        // pivot-row broadcast
    double* dsh = rowbuf + kNB;                  // pivots
    double* dinv = dsh + kNB;                    // 1 / pivots
    double* WL = dinv + kNB;                     // kNB x kNB: WL[q][j] = d_j L[q][j]
    __shared__ int fail;
    if (threadIdx.x == 0) fail = 0;
    __syncthreads();
    PHASE_MARK(0);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int kb = 0; kb < npad; kb += kNB) {
        const int R0 = kb + kNB;
        // (1) diagonal block
        for (int e = tid; e < kNB * kNB; e += blockDim.x) {
            const int r = e / kNB, c = e % kNB;
            if (c <= r) T[r * (kNB + 1) + c] = A[(long long)(kb + r) * ld + kb + c];
        }
        __syncthreads();
        PHASE_MARK(5);
        if (wid == 0) {
            double row[kNB];
            const int rl = lane & (kNB - 1);
#pragma unroll
            for (int c = 0; c < kNB; c++) row[c] = c <= rl ? T[rl * (kNB + 1) + c] : T[c * (kNB + 1) + rl];
            bool bad = false;
            diag_step<0>(row, lane, bad, dsh, dinv);
            PHASE_MARK(6);
            if (bad && lane == 0) fail = 1;
            if (lane < kNB) {
#pragma unroll
                for (int c = 0; c < kNB; c++)
                    if (c < lane) A[(long long)(kb + lane) * ld + kb + c] = row[c];
                A[(long long)(kb + lane) * ld + kb + lane] = dsh[lane];
#pragma unroll
                for (int j = 0; j < kNB; j++) WL[lane * kNB + j] = j < lane ? dsh[j] * row[j] : 0.0;
            }
        }
        __syncthreads();
        if (fail) break;
        PHASE_MARK(1);
        // (2) rows below (R0 .. npad, the last one is the rhs row)
        for (int r = R0 + tid; r <= npad; r += blockDim.x) {
            double a[kNB];
            double* Ar = A + (long long)r * ld + kb;
#pragma unroll
            for (int j = 0; j < kNB; j += 2) {
                const double2 v = *(const double2*)(Ar + j);
                a[j] = v.x;
                a[j + 1] = v.y;
            }
#pragma unroll
            for (int j = 0; j < kNB; j++) {
                a[j] = a[j] * dinv[j];
#pragma unroll
                for (int q = j + 1; q < kNB; q++) a[q] = __builtin_fma(-a[j], WL[q * kNB + j], a[q]);
            }
#pragma unroll
            for (int j = 0; j < kNB; j += 2) *(double2*)(Ar + j) = double2{a[j], a[j + 1]};
#pragma unroll
            for (int j = 0; j < kNB; j++) PLT[(size_t)j * NP + (r - R0)] = a[j];
        }
        __syncthreads();
        PHASE_MARK(2);
        // (3) trailing update of rows/cols [R0, npad) and of the rhs row npad
        const int mt = (npad - R0) / 16;  // 16-row tiles
        const int ntiles = mt * (mt + 1) / 2;
        const int nwv = (int)(blockDim.x >> 6);
        const int li = lane & 15, lk = lane >> 4;
        auto tile_of = [&](int t, int& ti, int& tj) {
            ti = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
            while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
            while (ti * (ti + 1) / 2 > t) ti--;
            tj = t - ti * (ti + 1) / 2;
        };
        double cn[4] = {0.0, 0.0, 0.0, 0.0};
        int ti = 0, tj = 0;
        if (wid < ntiles) {
            tile_of(wid, ti, tj);
            const double* Cp = A + (long long)(R0 + 16 * ti + lk) * ld + R0 + 16 * tj + li;
#pragma unroll
            for (int v = 0; v < 4; v++) cn[v] = Cp[(long long)(4 * v) * ld];
        }
        for (int t = wid; t < ntiles; t += nwv) {
            const double cc0 = cn[0], cc1 = cn[1], cc2 = cn[2], cc3 = cn[3];
            const int ci = ti, cj = tj;
            double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < kNB; s4 += 4) {
                const int q = s4 + lk;
                const double av = PLT[(size_t)q * NP + 16 * ci + li] * dsh[q];
                const double bv = PLT[(size_t)q * NP + 16 * cj + li];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
            if (t + nwv < ntiles) {  // prefetch the next tile of this wave
                tile_of(t + nwv, ti, tj);
                const double* Cp = A + (long long)(R0 + 16 * ti + lk) * ld + R0 + 16 * tj + li;
#pragma unroll
                for (int v = 0; v < 4; v++) cn[v] = Cp[(long long)(4 * v) * ld];
            }
            double* Ct = A + (long long)(R0 + 16 * ci + lk) * ld + R0 + 16 * cj + li;
            Ct[0] = cc0 - acc[0];
            Ct[(long long)4 * ld] = cc1 - acc[1];
            Ct[(long long)8 * ld] = cc2 - acc[2];
            Ct[(long long)12 * ld] = cc3 - acc[3];
        }
        if (wid == (int)(blockDim.x >> 6) - 1 || ntiles == 0) {
            // rhs row: z[c] -= sum_q (L[npad][q] d_q) L[c][q], c in [R0, npad)
            const double* zl = PLT + (npad - R0);
            double* z = A + (long long)npad * ld;
            for (int c = R0 + lane; c < npad; c += 64) {
                double s = 0.0;
#pragma unroll
                for (int q = 0; q < kNB; q++) s += (zl[(size_t)q * NP] * dsh[q]) * PLT[(size_t)q * NP + (c - R0)];
                z[c] -= s;
            }
        }
        __syncthreads();
        PHASE_MARK(3);
    }
    if (fail) {
        if (tid == 0) C.ok2 = 0;
        return;
    }
    // backward solve L^T x = z (z in row npad), block by block from the last one
    double* z = A + (long long)npad * ld;
    for (int kb = npad - kNB; kb >= 0; kb -= kNB) {
        for (int e = tid; e < kNB * kNB; e += blockDim.x) {
            const int r = e / kNB, c = e % kNB;
            if (c < r) T[r * (kNB + 1) + c] = A[(long long)(kb + r) * ld + kb + c];
        }
        __syncthreads();
        if (wid == 0) {
            const int cl = lane & (kNB - 1);
            double lc[kNB];  // column `lane` of the block: L[k][lane], k > lane
#pragma unroll
            for (int k = 0; k < kNB; k++) lc[k] = k > cl ? T[k * (kNB + 1) + cl] : 0.0;
            double zi = lane < kNB ? z[kb + lane] : 0.0;
#pragma unroll
            for (int k = kNB - 1; k >= 0; k--) {
                const double xk = readlane_d(zi, k);
                if (lane < k) zi = __builtin_fma(-lc[k], xk, zi);
            }
            if (lane < kNB) z[kb + lane] = zi;
        }
        __syncthreads();
        for (int i = tid; i < kb; i += blockDim.x) {
            double sacc = z[i];
#pragma unroll 8
            for (int k = 0; k < kNB; k++) sacc = __builtin_fma(-A[(long long)(kb + k) * ld + i], z[kb + k], sacc);
            z[i] = sacc;
        }
        __syncthreads();
        PHASE_MARK(4);
    }
    for (int i = tid; i < n; i += blockDim.x) xp_out[6 * (long long)W.pose0 + i] = z[i];
    if (tid == 0) C.ok2 = 1;
}

// Tile LDL^T for windows with n <= 288 (48 free KeyFrames): one 1024-thread workgroup per
// window, the lower triangle of the Schur system as 16x16 FP64 tiles in a tile-major scratch
// (2 KB per tile, 32 contiguous bytes per lane: every tile load / store is fully coalesced and
// stays in the XCD's L2 — 342 KB per window at n = 288), the panel and the rhs in LDS.  A tile
// (i, j) is held TRANSPOSED in the v_mfma_f64_16x16x4_f64 accumulator layout (lane l, register
// u = A_ij[l & 15][(l >> 4) + 4u]); in that form register u is directly the operand of k-step u
// of both products below, so no tile is transposed through LDS.
// Per 16-column panel k (round 5: no barrier per panel; the panel TRSM fused into the trailing
// update of the previous panel):
//   (4) tiles (i, j), i >= j > k: A_ij^T -= W_jk D^-1 W_ik^T (4 MFMAs, both operands from the
//       panel buffer P[k & 1]) by the tile's owner (worker wave 1 + t mod 15, fixed for the whole
//       factorization), its column-(k+1) tiles first and kept in registers, the others with the
//       next tile's load in flight; meanwhile wave 0 updates the next diagonal tile (handed over
//       through the LDS by its owner) and factors it (look-ahead, t16_diag: Gauss elimination of
//       [A_kk | I], DPP row broadcasts, giving D, M_{k+1} = L^-T and z_{k+1} = D^-1 L^-1 y);
//   (3) as soon as wave 0 publishes M_{k+1} (polled between trailing tiles) each owner applies
//       the panel TRSM to its column-(k+1) tiles: W^T = M_{k+1}^T A^T (4 MFMAs) into
//       P[(k + 1) & 1], L = W D^-1 back to the scratch, y_i -= L D (M^T y_{k+1}).
// Hand-offs are LDS words with release / acquire (see the panel loop).  Round-4 form: two
// barriers per panel, every wave waiting for the slowest: 113 -> 109 us at n = 288 (mb_ldlt).
// Then L^T x = z right-looking: x_k = M_k z_k by wave 0, tile (k, j) owners subtract L_kj^T x_k
// from z_j (DPP 16-lane sums), synchronised by LDS progress words instead of a barrier per
// step (wave 0 waits only for the one wave that owns column k - 1).  A zero pivot fails the
// solve, like Eigen's SimplicialLDLT.  Results are bit-identical to the round-4 form: every tile,
// y and x sees the same operations in the same order.  (tools/microbench/mb_ldlt, mb_diag)
struct T16Lds {
    double D[256];                         // diagonal tile of the current panel (row-major)
    double M[kT16Max][16 * kPStride];      // M_k = L_kk^-T per panel (row-major, stride 17: the
                                           // back-solve's row-per-lane reads hit distinct banks)
    double dinv[kT16Max][16];              // 1 / d per panel
    double P[2][kT16Max][16 * kPStride];   // W_ik of panels k (read) and k + 1 (written), stride 17
    double Dn[2][256];                     // diagonal tile (k + 2, k + 2) as panel k leaves it
                                           // (lane-major): wave 0 reads it at panel k + 1
    double y[kT16Max * 16];                // b_s, then z, then the back-substitution right-hand side
    double wb[2][16];                      // M_k^T y_k, by panel parity (TRSMs of panel k read it
                                           // while wave 0 may already form panel k + 1's)
    double xs[kT16Max * 16];               // x_k of the back-solve, every k (no reuse: waves lag freely)
    unsigned short tij[kT16Tiles];         // tile list, column-major: (i << 8) | j
    unsigned short col0[kT16Max + 1];      // first tile of column j
    int fail;
    int diag_ready;                        // last panel whose M / dinv / wb / z wave 0 has published
    int tr_first;                          // last column c whose TRSM of tile (c + 1, c) is done
    int dn_ready;                          // last panel k whose Dn[k & 1] (tile (k+2, k+2)) is in
    int trsm_cnt[kT16Max];                 // TRSMs done per column (complete at T - c - 1)
    int done_cnt[kT16Max];                 // worker waves done with panel k (15 = all)
    int x_low;                             // lowest k whose x_k wave 0 has published
    int prog[kT16Waves];                   // back-solve: last step whose updates wave w has applied
    int hang;                              // a hand-off wait ran past kT16SpinCap (bounded waits)
};
// Polls of one LDS hand-off word before the wait gives up (each poll sleeps ~64 cycles, so about a
// quarter of a second; a wait in a healthy factorization lasts well under a microsecond).  A wait
// that gives up raises L.hang, which ends every other wait at once: the kernel finishes, the trial
// fails (ok2 = 0) and the launch's error word tells the host (SLAM_ETIMEDOUT), instead of a
// workgroup spinning forever on a flag that never comes.
constexpr unsigned kT16SpinCap = 1u << 22;
__host__ __device__ constexpr long long t16_tiles_bytes() { return (long long)kT16Tiles * 256 * sizeof(double); }

__device__ __forceinline__ double t16_sum16(double v) {  // sum over the 16 lanes of a DPP row (every lane)
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    v += row_ror<2>(v);
    v += row_ror<1>(v);
    return v;
}

#ifdef LBA_PHASE_TIMING
__device__ unsigned long long g_t16_phase[8];
#define T16_MARK(i)                                                          \
    do {                                                                     \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                           \
            const unsigned long long now = wall_clock64();                   \
            if ((i) > 0) g_t16_phase[(i)] += now - g_t16_phase[0];           \
            g_t16_phase[0] = now;                                            \
        }                                                                    \
    } while (0)
#else
#define T16_MARK(i) \
    do {            \
    } while (0)
#endif

__device__ __forceinline__ double4_t t16_load(const double* tile, int lane) {
    return *(const double4_t*)(tile + 4 * lane);
}
__device__ __forceinline__ void t16_store(double* tile, int lane, double4_t v) { *(double4_t*)(tile + 4 * lane) = v; }

// lane J of every 16-lane DPP row, to the whole row (v_mov_b64 DPP row_newbcast, gfx90a+)
template <int J>
__device__ __forceinline__ double row_bcast(double v) {  // DPP row_newbcast (64-bit DPP, gfx90a+)
    // bound_ctrl with full masks: every lane reads a valid source, the old value is never used
    return __longlong_as_double(__builtin_amdgcn_update_dpp(0LL, __double_as_longlong(v), 0x150 + J, 0xf, 0xf, true));
}
// 1/d: v_rcp_f64 and two Newton steps (the pivot reciprocal is on the serial chain; within
// the LBA tolerance it equals the divided value)
__device__ __forceinline__ double rcp_nr(double d) {
    double x = __builtin_amdgcn_rcp(d);
    x = __builtin_fma(x, __builtin_fma(-d, x, 1.0), x);
    x = __builtin_fma(x, __builtin_fma(-d, x, 1.0), x);
    return x;
}

// one pivot step J of t16_diag (compile-time J: DPP row_newbcast takes an immediate lane).
// Lane (r = lane & 15, g = lane >> 4) holds 8 values of row r: g = 0 / 1 columns 0-7 / 8-15 of
// A, g = 2 / 3 the same of I.  Every group updates all its columns with the pivot row of its own
// group (A columns <= J hold leftovers that are never read again; I columns > J of the pivot row
// are zero), so only rows r <= J need masking, through a zero multiplier.  Measured 2.3 us per
// tile (tools/microbench/mb_diag).
template <int J>
__device__ __forceinline__ void t16_pivot(double (&row)[8], int r, int g, int lane, bool& bad, double dj, double arj) {
    // dj = pivot J (row J's column J), arj = A[r][J] of this lane's row: both read by the previous
    // step right after it updated column J
    if (dj == 0.0) bad = true;
    // the pivot row's broadcasts do not depend on the multiplier: issued while the reciprocal
    // and the bpermute are in flight
    double pr[8];
#pragma unroll
    for (int c = 0; c < 8; c++) pr[c] = row_bcast<J>(row[c]);
    const double inv = rcp_nr(dj);
    const double m = r > J ? arj * inv : 0.0;
    if constexpr (J + 1 < 16) {
        // column J + 1 first, then the next pivot and A[r][J + 1] leave at once (readlane; one
        // ds_bpermute from group gs to the row's four groups: all lanes active, 2.3 us per tile
        // measured against 3.4 us for v_permlane16/32_swap chains); the scheduling barrier keeps
        // them ahead of the other seven columns' updates
        constexpr int en = (J + 1) & 7, gn = (J + 1) >> 3;
        row[en] = __builtin_fma(-m, pr[en], row[en]);
        const double dn = readlane_d(row[en], 16 * gn + J + 1);
        const double an = __shfl(row[en], 16 * gn + r);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (c != en) row[c] = __builtin_fma(-m, pr[c], row[c]);
        t16_pivot<J + 1>(row, r, g, lane, bad, dn, an);
    } else {
#pragma unroll
        for (int c = 0; c < 8; c++) row[c] = __builtin_fma(-m, pr[c], row[c]);
    }
}

// The diagonal tile of panel k (held by wave 0 in the transposed accumulator layout, which for
// a symmetric tile is the tile itself): Gauss elimination of [A_kk | I] without pivoting, the
// four 16-lane groups of wave 0 holding A columns 0-7, 8-15 and I columns 0-7, 8-15 of row
// lane & 15.  The A half ends as D L^T (pivots d_j), the I half as L^-1 = M_k^T.  Then
// z_k = D^-1 M_k^T y_k.
template <class Lds>
__device__ __forceinline__ void t16_diag(Lds& L, int k, double4_t dt, int lane) {
    const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int u = 0; u < 4; u++) L.D[lr * 16 + lq + 4 * u] = dt[u];
    wave_sync();
    const int r = lane & 15, g = lane >> 4;
    double row[8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const int col = 8 * (g & 1) + c;
        row[c] = g < 2 ? L.D[r * 16 + col] : (col == r ? 1.0 : 0.0);
    }
    bool bad = false;
    t16_pivot<0>(row, r, g, lane, bad, readlane_d(row[0], 0), __shfl(row[0], r));
    if (bad && lane == 0) L.fail = 1;
    // 1 / d_r off the chain: pivot r's row is final once it has been eliminated, so the diagonal
    // of the A half is d_r, and rcp_nr gives the same value the chain used
    if (g == (r >> 3)) {
        double dr = row[0];
#pragma unroll
        for (int c = 1; c < 8; c++) dr = (r & 7) == c ? row[c] : dr;
        L.dinv[k][r] = rcp_nr(dr);
    }
    if (g >= 2) {
#pragma unroll
        for (int c = 0; c < 8; c++) L.M[k][(8 * (g & 1) + c) * kPStride + r] = row[c];  // M_k[col][r] = L^-1[r][col]
    }
    wave_sync();
    if (lane < 16) {
        const int c = lane;
        double wb = 0.0;
#pragma unroll
        for (int rr = 0; rr < 16; rr++) wb = __builtin_fma(L.M[k][rr * kPStride + c], L.y[16 * k + rr], wb);
        L.wb[k & 1][c] = wb;
        L.y[16 * k + c] = wb * L.dinv[k][c];
    }
}

// Global hand-off words of the helper-assisted factorization (per window, zero between launches):
// pub[c] counts the published TRSM tiles of column c (W and L written through to L2), rdy[j] the
// tiles of column j the helpers have brought through panel j - 3.
struct T16Sync {
    int pub[kT16Max];
    int rdy[kT16Max];
};

// loads / stores that bypass the CU's L1 (global sc1): the helper hand-offs
__device__ __forceinline__ double4_t t16_load_sc1(const double* tile, int lane) {
    double4_t v;
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __hip_atomic_load(tile + 4 * lane + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
}
__device__ __forceinline__ void t16_store_sc1(double* tile, int lane, const double4_t& v) {
#pragma unroll
    for (int u = 0; u < 4; u++) __hip_atomic_store(tile + 4 * lane + u, v[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every store of this wave has left for L2 (the hand-off counters are added after it)
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// A global counter reaches v (sc1 polls), bounded like the LDS waits: false when it gave up.
__device__ __forceinline__ bool t16_wait_global(const int* w, int v) {
    for (unsigned spin = 0; __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v; spin++) {
        if (spin >= kT16SpinCap) return false;
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// Look-ahead of the helper-assisted form: the main workgroup applies the last kT16LA panels of
// every column itself, the helpers the ones before (panels 0 .. j - kT16LA - 1 of column j), so a
// helper's hand-off has kT16LA - 1 main iterations of slack.
#ifndef SLAMHOT_T16_LA
#define SLAMHOT_T16_LA 4
#endif
constexpr int kT16LA = SLAMHOT_T16_LA;

// kHelp: the main workgroup of the helper-assisted form (k_ldlt_t16x): columns j > kT16LA receive
// their trailing updates of panels 0 .. j - kT16LA - 1 from helper workgroups (ldlt_t16_helper);
// this workgroup applies the last kT16LA (iteration k updates columns k + 1 .. k + kT16LA) and
// everything else as in k_ldlt_t16, and publishes each TRSM tile's W and L for the helpers.  The
// sequence of operations on every tile is the same, so x is bit-identical to the one-workgroup form.
template <bool kHelp>
__device__ __forceinline__ void ldlt_t16_body(T16Lds& L, int win, const WinDesc* __restrict__ wins,
                                              WinCtl* __restrict__ ctl, const double* __restrict__ Hs,
                                              double* __restrict__ Ts, double* __restrict__ Wg, T16Sync* __restrict__ sync,
                                              double* __restrict__ xp_out, int* __restrict__ err_word) {
    const WinDesc W = wins[win];
    WinCtl& C = ctl[win];
    if (!C.need_trial) return;
    const int n = W.n, ld = W.ld, T = (n + 15) >> 4, rhs = ldlt_npad(n);
    if (T == 0) {  // no free pose: an empty system solves trivially
        if (threadIdx.x == 0) C.ok2 = 1;
        return;
    }
    const int ntiles = T * (T + 1) / 2;
    const double* A = Hs + W.hs_off;
    double* Tw = Ts + blockIdx_win_tiles(win);
    double* Gw = kHelp ? Wg + blockIdx_win_tiles(win) : nullptr;  // W tiles for the helpers
    T16Sync* Sy = kHelp ? sync + win : nullptr;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lq = lane >> 4;  // register u of a tile holds [lr][lq + 4u]
    if (tid == 0) {
        int t = 0;
        for (int j = 0; j < T; j++) {
            L.col0[j] = (unsigned short)t;
            for (int i = j; i < T; i++) L.tij[t++] = (unsigned short)((i << 8) | j);
        }
        L.col0[T] = (unsigned short)t;
        L.fail = 0;
        L.hang = 0;
    }
    for (int c = tid; c < 16 * T; c += blockDim.x) L.y[c] = A[(long long)rhs * ld + c];
    if (tid == 0) {
        L.diag_ready = 0;
        L.tr_first = -1;
        L.dn_ready = -1;
        L.x_low = T;
    }
    if (tid < kT16Waves) L.prog[tid] = T;
    if (tid < kT16Max) L.trsm_cnt[tid] = L.done_cnt[tid] = 0;
    __syncthreads();
    T16_MARK(0);
    // (3) of one panel tile (i, kk) held in registers (transposed accumulator layout): W^T =
    // M_kk^T A^T into panel buffer Pb, L = W D^-1 back to the scratch tile t, y_i -= L (M^T y_kk)
    auto trsm = [&](int kk, int i, int t, const double4_t& a, double* Pb) {
        const double* Mk = L.M[kk];
        const double* dkk = L.dinv[kk];
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int u = 0; u < 4; u++)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Mk[(4 * u + lq) * kPStride + lr], a[u], acc, 0, 0, 0);
        double part = 0.0;  // sum_q L_ik[lr][q] (M_k^T y_k)[q] over this lane's q
        double4_t l;
        double* Pi = Pb + i * (16 * kPStride);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = lq + 4 * u;
            Pi[lr * kPStride + q] = acc[u];
            l[u] = acc[u] * dkk[q];
            part = __builtin_fma(l[u], L.wb[kk & 1][q], part);
        }
        const bool pub = kHelp && kk + kT16LA + 1 < T;  // a panel some helper tile still needs
        if (pub) {
            t16_store_sc1(Tw + 256 * t, lane, l);
            t16_store_sc1(Gw + 256 * t, lane, acc);
        } else {
            t16_store(Tw + 256 * t, lane, l);
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        if (lq == 0) L.y[16 * i + lr] -= part;
        // publish: P / y writes ordered before the counters (release)
        if (lane == 0) {
            if (i == kk + 1) __hip_atomic_store(&L.tr_first, kk, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&L.trsm_cnt[kk], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (pub) {  // to the helpers: the tile's W and L are in L2 before the count says so
            drain_stores();
            if (lane == 0) __hip_atomic_fetch_add(&Sy->pub[kk], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // bounded: gives up after kT16SpinCap polls, or at once when another wave gave up (L.hang)
    auto give_up = [&](unsigned spin) {
        if (spin < kT16SpinCap && !__hip_atomic_load(&L.hang, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        __hip_atomic_store(&L.hang, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
    };
    auto wait_at_least = [&](int* w, int v) {
        for (unsigned spin = 0; __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v; spin++) {
            if (give_up(spin)) return;
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // the tiles were written by k_schur_block (t16_put); padding by k_t16_pad
    double4_t diag1 = {0.0, 0.0, 0.0, 0.0};  // wave 0: tile (1, 1), untouched before panel 0
    if (wid == 0) {
        t16_diag(L, 0, t16_load(Tw, lane), lane);
        if (T >= 2) diag1 = t16_load(Tw + 256 * L.col0[1], lane);
    }
    __syncthreads();
    for (int t = L.col0[0] + 1 + wid; t < L.col0[1]; t += kT16Waves) trsm(0, L.tij[t] >> 8, t, t16_load(Tw + 256 * t, lane), L.P[0][0]);
    __syncthreads();
    T16_MARK(1);
    // Panels without a barrier: tile t belongs to worker wave 1 + t mod 15 for the whole
    // factorization (every update of a tile, and its TRSM, in program order on one wave); the
    // hand-offs between waves are LDS words (release / acquire):
    //   trsm_cnt[c]  all TRSMs of column c done -> panel c's trailing updates may read P[c & 1]
    //   diag_ready   M_{k+1}, dinv, wb, z_{k+1} published by wave 0 -> column k+1's TRSMs
    //   tr_first     TRSM (k+1, k) done -> wave 0 may update tile (k+1, k+1) at panel k
    //   dn_ready     tile (k+2, k+2) as panel k leaves it, in Dn[k & 1] -> wave 0 at panel k+1
    //   done_cnt[k]  every worker finished panel k -> P[k & 1] may be rewritten (column k+2)
    // Wave 0 never stops early (a zero pivot only sets L.fail), so no wave waits for a flag that
    // is never raised; the chain of waits only points at earlier panels.
    constexpr int kNw = kT16Waves - 1;
    for (int k = 0; k + 1 < T; k++) {
        const double* dk = L.dinv[k];
        const double* Pk = L.P[k & 1][0];
        double* Pn = L.P[(k + 1) & 1][0];
        // (4) A_ij^T -= W_jk D^-1 W_ik^T for tile t = (i, j)
        auto update = [&](int t, const double4_t& cur) -> double4_t {
            const int i = L.tij[t] >> 8, j = L.tij[t] & 255;
            double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int q = 4 * u + lq;
                const double a = Pk[j * (16 * kPStride) + lr * kPStride + q] * dk[q];
                const double b = Pk[i * (16 * kPStride) + lr * kPStride + q];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
            }
            return cur - acc;
        };
        const int t0 = L.col0[k + 1];  // the next diagonal tile (k + 1, k + 1)
        const int c1 = L.col0[k + 2];  // end of column k + 1
        if (wid == 0) {
            T16_MARK(0);
            // tile (k + 1, k + 1) as panel k - 1 left it (in the LDS, from its owner), W_{k+1,k}
            if (k > 0) wait_at_least(&L.dn_ready, k - 1);
            wait_at_least(&L.tr_first, k);
            const double4_t diag_next = k == 0 ? diag1 : t16_load(L.Dn[(k - 1) & 1], lane);
            T16_MARK(3);
            __builtin_amdgcn_s_setprio(3);  // the critical path: ahead of the trailing MFMA waves
            const double4_t dn = update(t0, diag_next);
            T16_MARK(6);
            t16_diag(L, k + 1, dn, lane);
            __builtin_amdgcn_s_setprio(0);
            if (lane == 0) __hip_atomic_store(&L.diag_ready, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            T16_MARK(7);
        } else {
            const int widx = wid - 1;
            // this wave's first tile at or after t: the next t' >= t with t' mod 15 == widx
            auto first_at = [&](int t) { return t + ((widx - t % kNw) % kNw + kNw) % kNw; };
            int ta = first_at(t0 + 1);  // column k + 1 tiles (at most two: 16 tiles, 15 waves)
            const int tb = ta + kNw;
            double4_t va = {0.0, 0.0, 0.0, 0.0}, vb = {0.0, 0.0, 0.0, 0.0};
            if (ta < c1) va = t16_load(Tw + 256 * ta, lane);
            if (tb < c1) vb = t16_load(Tw + 256 * tb, lane);
            wait_at_least(&L.trsm_cnt[k], T - k - 1);  // W_{., k} complete in P[k & 1]
            // column k + 1 first (held in registers): its TRSMs are on the critical path, so they
            // run as soon as M_{k+1} is published (polled between trailing tiles) and no wave still
            // reads P[(k + 1) & 1] for panel k - 1
            bool pending = ta < c1;
            if (pending) {
                va = update(ta, va);
                if (tb < c1) vb = update(tb, vb);
            }
            auto ready = [&]() {
                return __hip_atomic_load(&L.diag_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= k + 1 &&
                       (k == 0 || __hip_atomic_load(&L.done_cnt[k - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= kNw);
            };
            auto flush = [&]() {
                trsm(k + 1, L.tij[ta] >> 8, ta, va, Pn);
                if (tb < c1) trsm(k + 1, L.tij[tb] >> 8, tb, vb, Pn);
                pending = false;
            };
            // then columns > k + 1, one tile ahead in flight (deeper prefetch measured slower,
            // profiles/r04e_t16_prefetch.txt).  kHelp: columns k + 2 .. k + kT16LA only (the helpers
            // bring the later ones through panel k); column k + kT16LA arrives from the helpers now
            // (its tiles read from L2 once they are published), the others this workgroup updated
            const int tend = kHelp ? L.col0[min(k + kT16LA + 1, T)] : ntiles;
            const int jh = k + kT16LA;  // the column that comes from the helpers in this iteration
            // a helper tile is waited for only with this wave's critical work done: its tiles come
            // last in the range (column-major), the tile before it is updated (and the Dn tile
            // handed to wave 0) first, and the wave's column-(k + 1) TRSMs are flushed first
            auto from_help = [&](int tt) { return kHelp && jh > kT16LA && (L.tij[tt] & 255) == jh; };
            bool waited = false;
            auto ld_help = [&](int tt) {
                if (pending) {
                    wait_at_least(&L.diag_ready, k + 1);
                    if (k > 0) wait_at_least(&L.done_cnt[k - 1], kNw);
                    flush();
                }
                if (!waited && !t16_wait_global(&Sy->rdy[jh], T - jh)) give_up(kT16SpinCap);
                waited = true;
                return t16_load_sc1(Tw + 256 * tt, lane);
            };
            int t = first_at(c1);
            double4_t cur = t >= tend ? double4_t{0.0, 0.0, 0.0, 0.0} : from_help(t) ? ld_help(t) : t16_load(Tw + 256 * t, lane);
            while (t < tend) {
                const int tn = t + kNw;
                const bool nh = tn < tend && from_help(tn);  // loaded after this tile, not ahead
                const double4_t nxt = tn < tend && !nh ? t16_load(Tw + 256 * tn, lane) : double4_t{0.0, 0.0, 0.0, 0.0};
                const double4_t v = update(t, cur);
                if (t == c1) {  // the next panel's diagonal tile: to wave 0 through the LDS
                    t16_store(L.Dn[k & 1], lane, v);
                    if (lane == 0) __hip_atomic_store(&L.dn_ready, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    t16_store(Tw + 256 * t, lane, v);
                }
                if (pending && ready()) flush();
                cur = nh ? ld_help(tn) : nxt;
                t = tn;
            }
            if (pending) {
                wait_at_least(&L.diag_ready, k + 1);
                if (k > 0) wait_at_least(&L.done_cnt[k - 1], kNw);
                flush();
            }
            if (lane == 0) __hip_atomic_fetch_add(&L.done_cnt[k], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    T16_MARK(4);
    if (L.fail || L.hang) {
        if (tid == 0) {
            C.ok2 = 0;
            if (L.hang) atomicAdd(err_word, 1);
        }
        return;
    }
    // L^T x = z, right-looking from the last tile column.  Wave 0 owns the tiles (k, k-1) next to
    // the diagonal: at step k it applies x_k to y_{k-1} and forms x_{k-1} = M_{k-1} y_{k-1}, once
    // the owner of column k-1 (wave 1 + (k-1) mod 15) has applied every earlier x to it; waves w >= 1
    // apply x_k to their columns j < k-1 as soon as x_k is published.  No barrier per step, and each
    // wave's tiles come three steps ahead through a ring of four registers sets, so the L2 latency
    // of a tile load no longer sits in every step (round 4 loaded one step ahead and waited).
    {
        auto put_x = [&](int k) {  // wave 0: x_k from the final y_k
            if (lane < 16) {
                const double* Mk = L.M[k];
                double x = 0.0;
#pragma unroll
                for (int r = 0; r < 16; r++) x = __builtin_fma(Mk[lane * kPStride + r], L.y[16 * k + r], x);
                L.xs[16 * k + lane] = x;
                if (16 * k + lane < n) xp_out[6 * (long long)W.pose0 + 16 * k + lane] = x;
            }
        };
        auto apply = [&](const double4_t& l, int k, int j) {  // y_j -= L_kj^T x_k
            const double xr = L.xs[16 * k + lr];
            double sum[4];
#pragma unroll
            for (int u = 0; u < 4; u++) sum[u] = t16_sum16(l[u] * xr);
            if (lr == 0) {
#pragma unroll
                for (int u = 0; u < 4; u++) L.y[16 * j + lq + 4 * u] -= sum[u];
            }
        };
        auto tile = [&](int k, int j) { return t16_load(Tw + 256 * (L.col0[j] + k - j), lane); };
        auto wait_ge = [&](int* w, int v) {  // LDS word reaches v (counting down: <=); bounded
            for (unsigned spin = 0; __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > v; spin++) {
                if (give_up(spin)) return;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        const int nw1 = kT16Waves - 1;
        const double4_t zero = {0.0, 0.0, 0.0, 0.0};
        double4_t b0 = zero, b1 = zero, b2 = zero, b3 = zero;
        if (wid == 0) {
            put_x(T - 1);
            if (lane == 0) __hip_atomic_store(&L.x_low, T - 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            // step k uses tile (k, k-1) and loads tile (k-3, k-4) into the set step k+1 used
            auto step0 = [&](int k, const double4_t& cur, double4_t& ahead) {
                if (k - 3 >= 1) ahead = tile(k - 3, k - 4);
                // y_{k-1} final but for tile (k, k-1): its owner has applied steps > k
                if (k + 1 <= T - 1) wait_ge(&L.prog[1 + (k - 1) % nw1], k + 1);
                apply(cur, k, k - 1);
                wave_sync();
                put_x(k - 1);
                if (lane == 0) __hip_atomic_store(&L.x_low, k - 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            if (T - 1 >= 1) b0 = tile(T - 1, T - 2);
            if (T - 2 >= 1) b1 = tile(T - 2, T - 3);
            if (T - 3 >= 1) b2 = tile(T - 3, T - 4);
            for (int k = T - 1; k >= 1; k -= 4) {
                step0(k, b0, b3);
                if (k - 1 >= 1) step0(k - 1, b1, b0);
                if (k - 2 >= 1) step0(k - 2, b2, b1);
                if (k - 3 >= 1) step0(k - 3, b3, b2);
            }
        } else {
            // steps k = T-1 .. 2: columns j = wid-1, wid-1+15, ... below k-1 (the first one three
            // steps ahead, a second one (wave 1 at n > 240) loaded on the spot)
            const int j0 = wid - 1;
            auto stepw = [&](int k, const double4_t& cur, double4_t& ahead) {
                if (j0 < k - 4) ahead = tile(k - 3, j0);
                wait_ge(&L.x_low, k);  // x_k published
                apply(cur, k, j0);
                for (int j = j0 + nw1; j < k - 1; j += nw1) apply(tile(k, j), k, j);
                wave_sync();
                if (lane == 0) __hip_atomic_store(&L.prog[wid], k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            if (j0 < T - 2) b0 = tile(T - 1, j0);
            if (j0 < T - 3) b1 = tile(T - 2, j0);
            if (j0 < T - 4) b2 = tile(T - 3, j0);
            for (int k = T - 1; k >= 2 && j0 < k - 1; k -= 4) {
                stepw(k, b0, b3);
                if (k - 1 >= 2 && j0 < k - 2) stepw(k - 1, b1, b0);
                if (k - 2 >= 2 && j0 < k - 3) stepw(k - 2, b2, b1);
                if (k - 3 >= 2 && j0 < k - 4) stepw(k - 3, b3, b2);
            }
        }
    }
    __syncthreads();
    T16_MARK(5);
    if (tid == 0) {
        C.ok2 = L.hang ? 0 : 1;
        if (L.hang) atomicAdd(err_word, 1);
    }
    if (kHelp && tid < kT16Max) {  // every helper has published its last column: reset for the next launch
        Sy->pub[tid] = 0;
        Sy->rdy[tid] = 0;
    }
}

__global__ void __launch_bounds__(kT16Waves * 64) k_ldlt_t16(const WinDesc* __restrict__ wins, WinCtl* __restrict__ ctl,
                                                             const double* __restrict__ Hs, double* __restrict__ Ts,
                                                             double* __restrict__ xp_out, int* __restrict__ err_word) {
    __shared__ T16Lds L;
    ldlt_t16_body<false>(L, blockIdx.x, wins, ctl, Hs, Ts, nullptr, nullptr, xp_out, err_word);
}

// A helper workgroup of window w (one of kT16Helpers): its 16 waves own the tiles (i, j), j > kT16LA,
// round robin in column-major order, keep them in registers, and apply panels p = 0 .. j - kT16LA - 1
// as the main workgroup publishes them (pub[p] = T - p - 1: W_ip from the W copy, L_jp from the tile
// scratch, both sc1 loads), the same MFMA sequence as the main workgroup's update; after its last
// panel a tile goes back to the scratch (sc1) and rdy[j] counts it.
#ifndef SLAMHOT_T16_HELPERS
#define SLAMHOT_T16_HELPERS 2
#endif
constexpr int kT16Helpers = SLAMHOT_T16_HELPERS;
constexpr int kT16HelperOwn = (kT16Max - kT16LA - 1) * (kT16Max - kT16LA) / 2 / (16 * kT16Helpers) + 1;  // tiles per wave
__device__ __forceinline__ void ldlt_t16_helper(int win, int h, const WinDesc* __restrict__ wins,
                                                const WinCtl* __restrict__ ctl, double* __restrict__ Ts,
                                                const double* __restrict__ Wg, T16Sync* __restrict__ sync,
                                                int* __restrict__ err_word) {
    const WinDesc W = wins[win];
    if (!ctl[win].need_trial) return;
    const int T = (W.n + 15) >> 4;
    if (T < kT16LA + 2) return;  // no column has a helper panel
    double* Tw = Ts + blockIdx_win_tiles(win);
    const double* Gw = Wg + blockIdx_win_tiles(win);
    T16Sync* Sy = sync + win;
    const int lane = threadIdx.x & 63, hw = h * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NW = 16 * kT16Helpers;
    auto col0 = [&](int j) { return j * T - j * (j - 1) / 2; };
    // this wave's tiles: the m-th helper tile in column-major order (columns kT16LA + 1 .. T-1),
    // m = hw + NW o (decoded per o, so the arrays stay in registers)
    constexpr int J0 = kT16LA + 1;
    int ti[kT16HelperOwn], tj[kT16HelperOwn];
    double4_t cur[kT16HelperOwn];
    const int nhelp = (T - J0) * (T - J0 + 1) / 2;
    int nown = 0, jmax = -1;
#pragma unroll
    for (int o = 0; o < kT16HelperOwn; o++) {
        const int m = hw + NW * o;
        int i = 0, j = 0;
        if (m < nhelp) {
            int c = 0;
            for (j = J0; j < T; j++) {
                if (m < c + T - j) break;
                c += T - j;
            }
            i = j + (m - c);
            nown = o + 1;
            jmax = j;
        }
        ti[o] = i;
        tj[o] = j;
    }
#pragma unroll
    for (int o = 0; o < kT16HelperOwn; o++)
        if (o < nown) cur[o] = t16_load(Tw + 256 * (col0(tj[o]) + ti[o] - tj[o]), lane);  // k_schur's tiles
    for (int p = 0; p + J0 <= jmax; p++) {
        if (!t16_wait_global(&Sy->pub[p], T - p - 1)) {
            if (lane == 0) atomicAdd(err_word, 1);
            return;
        }
#pragma unroll
        for (int o = 0; o < kT16HelperOwn; o++) {
            if (o >= nown || p > tj[o] - J0) continue;
            const double4_t a = t16_load_sc1(Tw + 256 * (col0(p) + tj[o] - p), lane);  // L_jp
            const double4_t bw = t16_load_sc1(Gw + 256 * (col0(p) + ti[o] - p), lane);  // W_ip
            double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], bw[u], acc, 0, 0, 0);
            cur[o] = cur[o] - acc;
            if (p == tj[o] - J0) {
                t16_store_sc1(Tw + 256 * (col0(tj[o]) + ti[o] - tj[o]), lane, cur[o]);
                drain_stores();
                if (lane == 0) __hip_atomic_fetch_add(&Sy->rdy[tj[o]], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// The helper-assisted factorization for a few windows (LocalMapping's one-window call): block b
// is window b % 8's main workgroup (b < 8) or its helper b / 8 - 1 -- blocks of equal b % 8 share
// an XCD under the round-robin dispatch (speed only: the hand-offs are agent-scope).  The grid
// is 8 x (1 + kT16Helpers) blocks; windows >= nw exit.
__global__ void __launch_bounds__(kT16Waves * 64) k_ldlt_t16x(int nw, const WinDesc* __restrict__ wins, WinCtl* __restrict__ ctl,
                                                              const double* __restrict__ Hs, double* __restrict__ Ts,
                                                              double* __restrict__ Wg, T16Sync* __restrict__ sync,
                                                              double* __restrict__ xp_out, int* __restrict__ err_word) {
    __shared__ T16Lds L;
    const int w = blockIdx.x & 7, slot = blockIdx.x >> 3;
    if (w >= nw) return;
    if (slot == 0)
        ldlt_t16_body<true>(L, w, wins, ctl, Hs, Ts, Wg, sync, xp_out, err_word);
    else
        ldlt_t16_helper(w, slot - 1, wins, ctl, Ts, Wg, sync, err_word);
}


// Identity padding of the dense systems (rows/cols n..npad-1) and a zero rhs tail; the
// factorization keeps it invariant, so it is written once per solve.
__device__ __forceinline__ void ldlt_pad_body(int w, const WinDesc* __restrict__ wins, double* __restrict__ Hs) {
    const WinDesc W = wins[w];
    const int n = W.n, npad = ldlt_npad(n), ld = W.ld;
    double* A = Hs + W.hs_off;
    for (int i = n + threadIdx.x; i < npad; i += blockDim.x) {
        for (int j = 0; j <= i; j++) A[(long long)i * ld + j] = (i == j) ? 1.0 : 0.0;
        A[(long long)npad * ld + i] = 0.0;
    }
}

// Identity padding of the tile scratch (rows / columns n .. 16T-1 of the last tile row): the
// scratch is zeroed once per solve and k_schur_block rewrites every real element each trial;
// the factorization leaves the padding invariant (its W rows are zero).
__device__ __forceinline__ void t16_pad_body(int w, const WinDesc* __restrict__ wins, double* __restrict__ Ts) {
    const WinDesc W = wins[w];
    const int T = (W.n + 15) >> 4;
    for (int R = W.n + (int)threadIdx.x; R < 16 * T; R += blockDim.x) t16_put(Ts + blockIdx_win_tiles(w), W.n, R, R, 1.0);
}

// x_l = Dinv (b_l - Hpl^T x_p) (block_solver.hpp:456-481) and the trial point estimate.
__device__ __forceinline__ void backsub_body(int p, int npt_total, const int* __restrict__ spe_off, const int* __restrict__ spe,
                          const int* __restrict__ spe_hp, const int* __restrict__ pt_win,
                          const WinCtl* __restrict__ ctl, const double* __restrict__ bl,
                          const double* __restrict__ pd, const double* __restrict__ lin,
                          const double* __restrict__ xp, double* __restrict__ xl, double* __restrict__ pts,
                          long long pt_stride) {
    if (p >= npt_total) return;
    const WinCtl& C = ctl[pt_win[p]];
    if (!C.need_trial) return;
    double* x = xl + 4 * (long long)p;
    if (C.ok2) {  // a failed factorization leaves x untouched (block_solver.hpp:451-452)
        double cl[3] = {bl[4 * (long long)p], bl[4 * (long long)p + 1], bl[4 * (long long)p + 2]};
        // two edges per step: both edges' Hpl and x_p rows are in flight together (same
        // accumulation order as one edge at a time)
        const int i1 = spe_off[p + 1];
        for (int i = spe_off[p]; i < i1; i += 2) {
            const bool two = i + 1 < i1;
            const double* H0 = lin + (long long)kHplStride * spe[i];
            const double* x0 = xp + 6 * (long long)spe_hp[i];
            const double* H1 = lin + (long long)kHplStride * spe[two ? i + 1 : i];
            const double* x1 = xp + 6 * (long long)spe_hp[two ? i + 1 : i];
            double h0[18], v0[6], h1[18], v1[6];
#pragma unroll
            for (int k = 0; k < 18; k++) h0[k] = H0[k];
#pragma unroll
            for (int k = 0; k < 6; k++) v0[k] = x0[k];
#pragma unroll
            for (int k = 0; k < 18; k++) h1[k] = H1[k];
#pragma unroll
            for (int k = 0; k < 6; k++) v1[k] = x1[k];
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int r = 0; r < 6; r++) cl[c] += h0[3 * r + c] * (-v0[r]);
            if (two) {
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int r = 0; r < 6; r++) cl[c] += h1[3 * r + c] * (-v1[r]);
            }
        }
        double Di[9], db[3];
        pd_load(pd + (long long)kPdStride * p, Di, db);  // k_point_prep's Dinv of this trial
#pragma unroll
        for (int r = 0; r < 3; r++) x[r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
    }
    const double* cur = pts + C.sel * pt_stride + 4 * (long long)p;
    double* nxt = pts + (1 - C.sel) * pt_stride + 4 * (long long)p;
#pragma unroll
    for (int k = 0; k < 3; k++) nxt[k] = cur[k] + x[k];
}

// VertexSE3Expmap::oplusImpl: T <- exp(x) * T  (types_six_dof_expmap.h:71-74, se3quat.h:223-257)
__device__ __forceinline__ void pose_update_body(int k, int nkf_total, const int* __restrict__ kf_hp, const int* __restrict__ kf_win,
                              const WinCtl* __restrict__ ctl, const double* __restrict__ xp,
                              double* __restrict__ poses, long long pose_stride) {
    if (k >= nkf_total) return;
    const WinCtl& C = ctl[kf_win[k]];
    if (!C.need_trial) return;
    const double* cur = poses + C.sel * pose_stride + 8 * (long long)k;
    double* nxt = poses + (1 - C.sel) * pose_stride + 8 * (long long)k;
    const int h = kf_hp[k];
    if (h < 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = cur[i];
        return;
    }
    se3_exp_mul(xp + 6 * (long long)h, cur, nxt);
}

// the update half of a trial in one launch: blocks [0, nb_kf) apply oplus to the KeyFrames,
// the rest back-substitute and move the MapPoints (block_solver.hpp:434-466)
__global__ void __launch_bounds__(256) k_update(int nb_kf, int nkf_total, const int* __restrict__ kf_hp,
                                                const int* __restrict__ kf_win, int npt_total,
                                                const int* __restrict__ spe_off, const int* __restrict__ spe,
                                                const int* __restrict__ spe_hp, const int* __restrict__ pt_win,
                                                const WinCtl* __restrict__ ctl, const double* __restrict__ bl,
                                                const double* __restrict__ pd, const double* __restrict__ lin,
                                                const double* __restrict__ xp, double* __restrict__ xl,
                                                double* __restrict__ poses, long long pose_stride,
                                                double* __restrict__ pts, long long pt_stride) {
    const int b = blockIdx.x;
    if (b < nb_kf)
        pose_update_body(b * 256 + threadIdx.x, nkf_total, kf_hp, kf_win, ctl, xp, poses, pose_stride);
    else
        backsub_body((b - nb_kf) * 256 + threadIdx.x, npt_total, spe_off, spe, spe_hp, pt_win, ctl, bl, pd, lin, xp, xl,
                     pts, pt_stride);
}

__global__ void k_trial_error(int ne_total, const EdgeS* __restrict__ E, const WinCtl* __restrict__ ctl,
                              const double* __restrict__ poses, const double* __restrict__ pts,
                              long long pose_stride, long long pt_stride, Cam cam, Huber hk,
                              double* __restrict__ err_out, double* __restrict__ rho_out) {
    const int ei = blockIdx.x * blockDim.x + threadIdx.x;
    if (ei >= ne_total) return;
    const EdgeS e = E[ei];
    const WinCtl& C = ctl[e.win];
    if (!C.need_trial) return;
    const double* P = poses + (1 - C.sel) * pose_stride + 8 * (long long)e.kf;
    const double* Xw = pts + (1 - C.sel) * pt_stride + 4 * (long long)e.pt;
    const double X[3] = {Xw[0], Xw[1], Xw[2]};
    double err[3];
    edge_error(e, cam, P, X, err);
    err_out[4 * (long long)ei + 0] = err[0];
    err_out[4 * (long long)ei + 1] = err[1];
    err_out[4 * (long long)ei + 2] = err[2];
    double rho0, rho1;
    robustify(hk, e.obs[2] >= 0.f, edge_chi2(e, err), rho0, rho1);
    rho_out[ei] = rho0;
}

// Per-step counters for the host: every control block adds its window's (need_trial, active)
// and takes a ticket; the last block publishes the totals straight into the pinned host slot
// the host polls (no copy, no counting kernel) and rearms the tally for the next step.
// The three counts share one 64-bit word (need bits 0-20, active 21-41, tickets 42-62), so a
// block's contribution and its ticket are one returning atomic; the last block rearms the word
// with a plain store (the next step's kernels start after this one ends).
constexpr int kTallyBits = 21;
__device__ __forceinline__ void tally_publish(int* __restrict__ tally, int need, int act, int nblocks,
                                              Counters* __restrict__ host_slot, int seq) {
    constexpr unsigned long long field = (1ull << kTallyBits) - 1;
    unsigned long long* word = reinterpret_cast<unsigned long long*>(tally);
    const unsigned long long mine =
        (unsigned long long)need | ((unsigned long long)act << kTallyBits) | (1ull << (2 * kTallyBits));
    const unsigned long long old = atomicAdd(word, mine);
    if ((long long)(old >> (2 * kTallyBits)) == nblocks - 1) {
        const unsigned long long tot = old + mine;
        *word = 0ull;
        // need_trial and active in one store, then the sequence number the host spins on
        *reinterpret_cast<volatile unsigned long long*>(host_slot) =
            (tot & field) | (((tot >> kTallyBits) & field) << 32);
        // device-side hand-offs that gave up this solve (k_ldlt_t16's bounded waits): the host
        // ends the call with SLAM_ETIMEDOUT
        reinterpret_cast<volatile Counters*>(host_slot)->pad = ((volatile int*)tally)[6];
        __threadfence_system();
        reinterpret_cast<volatile Counters*>(host_slot)->seq = seq;
    }
}

// The trial-loop body after the error pass (optimization_algorithm_levenberg.cpp:117-166).
__global__ void __launch_bounds__(kCtlThreads) k_trial_control(const WinDesc* __restrict__ wins,
                                                               WinCtl* __restrict__ ctl,
                                                               const double* __restrict__ rho,
                                                               const double* __restrict__ xp,
                                                               const double* __restrict__ xl,
                                                               const double* __restrict__ bp,
                                                               const double* __restrict__ bl,
                                                               const volatile int* __restrict__ stop_host,
                                                               int* __restrict__ tally,
                                                               Counters* __restrict__ host_slot, int seq) {
    __shared__ double sh[kCtlThreads / 64];
    const WinDesc W = wins[blockIdx.x];
    WinCtl& C = ctl[blockIdx.x];
    // terminate(): block 0 samples the pinned host word (one PCIe read per step, issued early so
    // it overlaps the reductions) into the sample slot of the NEXT step, tally[4 + ((seq + 1) & 1)];
    // every block of this step decides on tally[4 + (seq & 1)], written during the previous step
    // and not touched during this one, so all windows of a step see one value -- a stop the host
    // saw a step later, which is all the reference guarantees between threads anyway
    int stop_fresh = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) stop_fresh = *stop_host;
    int* const stop_next = &tally[4 + ((seq + 1) & 1)];
    if (!C.need_trial) {  // idle window: active == 0 here (k_iter_begin put every active one in a trial)
        if (threadIdx.x == 0) {
            if (blockIdx.x == 0) atomicExch(stop_next, stop_fresh);
            tally_publish(tally, 0, 0, gridDim.x, host_slot, seq);
        }
        return;
    }
    // thread 0 takes the control block and this step's stop sample into registers now: their
    // loads overlap the sums instead of following them on the step's critical path
    WinCtl c;
    int stop = 0;
    if (threadIdx.x == 0) {
        c = C;
        stop = ((volatile int*)tally)[4 + (seq & 1)];  // terminate() at the end of the trial
    }
    double tmpChi = block_sum(strided_sum(rho + W.e0, W.ne), sh);
    const double lam = C.lambda;
    double sc = 0;
    for (int i = threadIdx.x; i < 6 * W.np; i += kCtlThreads) {
        const double xv = xp[6 * (long long)W.pose0 + i];
        sc += xv * (lam * xv + bp[8 * (long long)(W.pose0 + i / 6) + i % 6]);
    }
    for (int i = threadIdx.x; i < 3 * W.npt; i += kCtlThreads) {
        const long long p = W.pt0 + i / 3;
        const double xv = xl[4 * p + i % 3];
        sc += xv * (lam * xv + bl[4 * p + i % 3]);
    }
    double scale = block_sum(sc, sh);
    if (threadIdx.x != 0) return;
    if (blockIdx.x == 0) atomicExch(stop_next, stop_fresh);
    if (!c.ok2) tmpChi = __DBL_MAX__;
    double rho_ = c.cur_chi - tmpChi;
    scale += 1e-3;
    rho_ /= scale;
    c.tmp_chi = tmpChi;
    if (rho_ > 0 && isfinite(tmpChi)) {
        double alpha = 1. - pow((2 * rho_ - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        const double f = fmax(1. / 3., alpha);
        c.lambda = lam * f;
        c.ni = 2;
        c.cur_chi = tmpChi;
        c.sel = 1 - c.sel;  // discardTop: the trial state becomes the estimate
    } else {
        c.lambda = lam * c.ni;
        c.ni *= 2;           // pop: keep the previous estimate
    }
    c.qmax++;
    c.trials++;
    const bool again = rho_ < 0 && c.qmax < 10 && !stop;
    if (again) {
        c.need_trial = 1;
        C = c;
        tally_publish(tally, 1, c.active, gridDim.x, host_slot, seq);
        return;
    }
    c.need_trial = 0;
    int result = 0;  // OK
    if (c.qmax == 10 || rho_ == 0) {
        result = 1;  // Terminate
    } else {
        if ((c.ini_chi - c.cur_chi) * 1e3 < c.ini_chi)
            c.nbad++;
        else
            c.nbad = 0;
        if (c.nbad >= 3) result = 1;
    }
    c.iters_run[c.opt]++;
    c.it++;
    c.chi2_final = c.cur_chi;
    c.active = (result == 0) && c.it < c.iters && !stop;
    if (!c.active && c.opt == 0 && c.iters2 > 0 && !stop) {
        // optimize(5) is over and no stop was seen: bDoMore, initializeOptimization(0) on the same
        // graph and optimize(10) (Optimizer.cc:1931-1986), started here so the next queued step runs
        // its first iteration (a stop set meanwhile is caught by that step's k_iter_begin, so no
        // iteration of optimize(10) runs, as when the reference skips it)
        c.opt = 1;
        c.it = 0;
        c.iters = c.iters2;
        c.active = 1;
    }
    c.need_lin = c.active;  // the next step linearizes again
    C = c;
    tally_publish(tally, 0, c.active, gridDim.x, host_slot, seq);
}

// start of SparseOptimizer::optimize(iters) for every window
__device__ __forceinline__ void opt_begin_body(int w, int nwin, const WinDesc* __restrict__ wins,
                                               WinCtl* __restrict__ ctl, int opt, int iters, int iters2) {
    if (w >= nwin) return;
    WinCtl& C = ctl[w];
    C.opt = opt;
    C.it = 0;
    C.iters = iters;
    C.iters2 = iters2;
    C.active = iters > 0 && wins[w].ne > 0;  // no edges: initializeOptimization fails
    C.need_trial = 0;
    C.need_lin = C.active;
}

// final outlier classification (Optimizer.cc:1995-2038) and float write-back (:2041-2077)
__device__ __forceinline__ void finalize_edge_body(int ei, int ne_total, const EdgeS* __restrict__ E,
                                                   const WinCtl* __restrict__ ctl, const double* __restrict__ poses,
                                                   const double* __restrict__ pts, long long pose_stride,
                                                   long long pt_stride, const double* __restrict__ err,
                                                   const double* __restrict__ trl, uint8_t* __restrict__ outlier) {
    if (ei >= ne_total) return;
    const EdgeS e = E[ei];
    const WinCtl& C = ctl[e.win];
    const double* P = poses + C.sel * pose_stride + 8 * (long long)e.kf;
    const double* Xw = pts + C.sel * pt_stride + 4 * (long long)e.pt;
    const double X[3] = {Xw[0], Xw[1], Xw[2]};
    double Xc[3];
    if (is_body(e)) {  // isDepthPositive in the right camera (OptimizableTypes.h:134-138)
        double Q[8];
        body_pose(trl + 8 * (long long)e.kf, P, Q);
        map_cc(Q, X, Xc);
    } else {
        map_cc(P, X, Xc);  // isDepthPositive: _transformVector + t (Optimizer.cc.o final scan)
    }
    const double ev[3] = {err[4 * (long long)ei], err[4 * (long long)ei + 1], err[4 * (long long)ei + 2]};
    const bool stereo = e.obs[2] >= 0.f;
    const double c = edge_chi2(e, ev);
    outlier[ei] = (c > (stereo ? 7.815 : 5.991) || !(Xc[2] > 0.0)) ? 1 : 0;
}

__device__ __forceinline__ void finalize_state_body(int t, int nkf_total, int npt_total, const int* __restrict__ kf_win,
                                                    const int* __restrict__ pt_win, const WinCtl* __restrict__ ctl,
                                                    const double* __restrict__ poses, const double* __restrict__ pts,
                                                    long long pose_stride, long long pt_stride,
                                                    float* __restrict__ kf_out, float* __restrict__ pt_out) {
    if (t < nkf_total) {
        const double* P = poses + ctl[kf_win[t]].sel * pose_stride + 8 * (long long)t;
        double R[9];
        rot_matrix(load_q(P), R);
        float* T = kf_out + 16 * (long long)t;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[3 * i + j];
            T[4 * i + 3] = (float)P[4 + i];
        }
        T[12] = T[13] = T[14] = 0.f;
        T[15] = 1.f;
    } else if (t < nkf_total + npt_total) {
        const int p = t - nkf_total;
        const double* X = pts + ctl[pt_win[p]].sel * pt_stride + 4 * (long long)p;
        for (int k = 0; k < 3; k++) pt_out[3 * (long long)p + k] = (float)X[k];
    }
}

// one launch after the LM loop: outlier flags per edge | float estimates | the control blocks
// into the read-back region (was two kernels and a device copy)
struct FinalArgs {
    int ne, nkf, npt, nw, nb_edges, nb_state;
    const EdgeS* E;
    const WinCtl* ctl;
    const double* poses;
    const double* pts;
    long long pose_stride, pt_stride;
    const double* err;
    const double* trl;
    const int* kf_win;
    const int* pt_win;
    uint8_t* outlier;
    float* kf_out;
    float* pt_out;
    int* ctl_out;
};
__global__ void __launch_bounds__(256) k_finalize(FinalArgs a) {
    int b = blockIdx.x;
    if (b < a.nb_edges)
        return finalize_edge_body(b * 256 + threadIdx.x, a.ne, a.E, a.ctl, a.poses, a.pts, a.pose_stride, a.pt_stride,
                                  a.err, a.trl, a.outlier);
    b -= a.nb_edges;
    if (b < a.nb_state)
        return finalize_state_body(b * 256 + threadIdx.x, a.nkf, a.npt, a.kf_win, a.pt_win, a.ctl, a.poses, a.pts,
                                   a.pose_stride, a.pt_stride, a.kf_out, a.pt_out);
    const int words = (int)(sizeof(WinCtl) / sizeof(int)) * a.nw;
    for (int i = threadIdx.x; i < words; i += blockDim.x) a.ctl_out[i] = ((const int*)a.ctl)[i];
}

// The per-solve clears (pose bitmaps, increments, errors, tile scratch, the control tally) in one
// launch instead of one fill per buffer
struct ClearRange {
    unsigned long long* p;
    long long n;             // 8-byte words
    unsigned long long v;    // fill value
};
constexpr int kClearMax = 12;
struct ClearList {
    ClearRange r[kClearMax];
    int n;
};
__device__ __forceinline__ void clear_body(const ClearList& L, int b, int nb) {
    const long long stride = (long long)nb * blockDim.x;
    for (int i = 0; i < L.n; i++) {
        unsigned long long* p = L.r[i].p;
        const unsigned long long v = L.r[i].v;
        for (long long e = b * (long long)blockDim.x + threadIdx.x; e < L.r[i].n; e += stride) p[e] = v;
    }
}

// Converter::toSE3Quat on the device for the initial estimates
__device__ __forceinline__ void init_state_body(int t, int nkf_total, int npt_total, const float* __restrict__ kf_in,
                                                const float* __restrict__ pt_in, double* __restrict__ poses,
                                                double* __restrict__ pts) {
    if (t < nkf_total) {
        const float* T = kf_in + 16 * (long long)t;
        double R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = T[4 * i + j];
        Quat q = quat_from_R(R);
        normalize_rotation(q);
        double* P = poses + 8 * (long long)t;
        P[0] = q.x;
        P[1] = q.y;
        P[2] = q.z;
        P[3] = q.w;
        P[4] = T[3];
        P[5] = T[7];
        P[6] = T[11];
        P[7] = 0.0;
    } else if (t < nkf_total + npt_total) {
        const int p = t - nkf_total;
        double* X = pts + 4 * (long long)p;
        for (int k = 0; k < 3; k++) X[k] = pt_in[3 * (long long)p + k];
        X[3] = 0.0;
    }
}

// The per-solve setup in four launches, each the union of independent steps (a block range
// apiece, so every branch is block-uniform).  A lone window pays one dispatch per launch (~5 us
// each in profiles/r04d_dropin_kernels.txt), and eleven launches became four plus k_ct_fill.
struct SetupArgs {
    ClearList clear;
    int nb_clear, nb_init, nb_spe, nb_blk, nb_list, nw_scan, nb_pts;
    const int* pt_off;   // point CSR (edge ranges) and spe offsets, from the host plan
    const int* spe_off;
    int* spe_out;        // per-point free-pose edges sorted by pose, written by spe_build_body
    int nw, nkf, npt, nspe, nblk;
    const WinDesc* wins;
    WinCtl* ctl;
    int opt, iters, iters2;
    const float* kf_in;
    const float* pt_in;
    double* poses;
    double* pts;
    double* Hs;
    double* Ts;  // tile scratch (k_ldlt_t16) or null
    const int* spe;
    const EdgeS* E;
    unsigned long long* bm;
    int* spe_hp;
    int* bmp;
    int* pbase;
    int* pcnt;
    int* pls;
    int* ppt;
    const int2* blk_pose;
    const int* blk_win;
    int* ct_cnt;
    int* ct_off;
};
// thread per point: its free-pose leader edges (hp >= 0, not a body edge's follower: the edge right
// after one of the same point on the same KeyFrame shares its Hpl block) in pose order, stably
// (HplCCS column order: block_solver.hpp:381-481), and their free-pose indices
__device__ __forceinline__ void spe_build_body(int p, int npt_total, const int* __restrict__ pt_off,
                                               const int* __restrict__ spe_off, const EdgeS* __restrict__ E,
                                               int* __restrict__ spe, int* __restrict__ spe_hp) {
    if (p >= npt_total) return;
    const int e0 = pt_off[p], e1 = pt_off[p + 1], s0 = spe_off[p];
    int n = 0, prev_kf = -1;
    for (int i = e0; i < e1; i++) {
        const int kf = E[i].kf, hp = E[i].hp;
        const bool follows = i > e0 && kf == prev_kf;
        prev_kf = kf;
        if (hp < 0 || follows) continue;
        int j = n++;
        for (; j > 0 && spe_hp[s0 + j - 1] > hp; j--) {
            spe[s0 + j] = spe[s0 + j - 1];
            spe_hp[s0 + j] = spe_hp[s0 + j - 1];
        }
        spe[s0 + j] = i;
        spe_hp[s0 + j] = hp;
    }
}

// clears | per-point pose-sorted edge lists | initial estimates | dense padding | optimize() start
__global__ void __launch_bounds__(256) k_setup_a(SetupArgs a) {
    int b = blockIdx.x;
    if (b < a.nb_clear) return clear_body(a.clear, b, a.nb_clear);
    b -= a.nb_clear;
    if (b < a.nb_pts) return spe_build_body(b * 256 + threadIdx.x, a.npt, a.pt_off, a.spe_off, a.E, a.spe_out, a.spe_hp);
    b -= a.nb_pts;
    if (b < a.nb_init) return init_state_body(b * 256 + threadIdx.x, a.nkf, a.npt, a.kf_in, a.pt_in, a.poses, a.pts);
    b -= a.nb_init;
    if (b < a.nw) return ldlt_pad_body(b, a.wins, a.Hs);
    b -= a.nw;
    opt_begin_body(b * 256 + threadIdx.x, a.nw, a.wins, a.ctl, a.opt, a.iters, a.iters2);
}
// pose bitmaps | tile padding (both after the clears)
__global__ void __launch_bounds__(256) k_setup_b(SetupArgs a) {
    int b = blockIdx.x;
    if (b < a.nb_spe) return bm_set_body(b * 256 + threadIdx.x, a.nspe, a.spe, a.E, a.wins, a.bm, a.spe_hp);
    b -= a.nb_spe;
    t16_pad_body(b, a.wins, a.Ts);
}
// bitmap word prefixes and pose list bases | contribution counts per block
__global__ void __launch_bounds__(256) k_setup_c(SetupArgs a) {
    int b = blockIdx.x;
    if (b < a.nw) return bm_scan_body(b, a.wins, a.bm, a.bmp, a.pbase, a.pcnt);
    b -= a.nw;
    ct_count_body(b * 256 + threadIdx.x, a.nblk, a.blk_pose, a.blk_win, a.wins, a.bm, a.ct_cnt);
}
// contribution offsets | pose edge lists
__global__ void __launch_bounds__(kCtScanThreads) k_setup_d(SetupArgs a) {
    int b = blockIdx.x;
    if (b < a.nw_scan) return ct_scan_body(b, a.wins, a.ct_cnt, a.ct_off);
    b -= a.nw_scan;
    bm_list_body(b * kCtScanThreads + threadIdx.x, a.nspe, a.spe, a.E, a.wins, a.bm, a.bmp, a.pbase, a.pls, a.ppt);
}

}  // namespace lba
}  // namespace slamhot

// ==================================================================== host side
using namespace slamhot;
using namespace slamhot::lba;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 256));
        if (e == hipSuccess) cap = std::max<size_t>(bytes, 256);
        return e;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

template <class T>
T* as(DevBuf& b) {
    return (T*)b.p;
}

}  // namespace

// Every per-call input structure lives in one arena: built in place in pinned host memory and
// shipped with a single copy (the reference builds the same graph in g2o: buildStructure).
struct Plan {
    EdgeS* edges;
    WinDesc* wins;
    WinCtl* ctl;
    int *pt_off, *pt_win, *spe_off, *spe, *pe_off, *pe, *pose_win, *kf_hp, *kf_win, *blk_win, *blk_order;
    int2* blk_pose;
    float *kf_in, *pt_in;
    double* kf_trl;  // per KF: mTrl as a pose record (body edges)
    float4* kcam;    // per KF: {fx, fy, cx, cy}, {fx2, fy2, cx2, cy2} (batches of mixed calibrations)
    float* kbf;      // per KF: mbf
};

constexpr int kRing = 4;  // LM steps whose counters are in flight (host-side ring)

// The planning threads of one handle, kept between calls (spawning and joining them twice per
// call cost ~0.1-0.3 ms): run(n, f) calls f(0) on the caller and f(1..n-1) on the workers.
// A worker is created knowing the generation current at its creation (read under the lock), so it
// waits for the next run() and never acts on an older one (a worker created with 0 after gen had
// advanced woke on that stale generation and decremented busy below zero).  run() always waits for
// every worker before it returns, also when a job throws (the job and its captures live on the
// caller's stack); the first exception of a call is returned, never let across the C ABI.
struct PlanPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done;
    unsigned long long gen = 0;
    int busy = 0, n = 0;
    bool stop = false, failed = false;
    const std::function<void(int)>* job = nullptr;

    // the number of threads run() can use (workers + the caller); fewer than asked when thread
    // creation fails, and the caller then runs the rest
    int ensure(int want) {
        std::lock_guard<std::mutex> lk(m);
        while ((int)th.size() < want - 1) {
            const int t = (int)th.size() + 1;
            const unsigned long long g = gen;
            try {
                th.emplace_back([this, t, g] { worker(t, g); });
            } catch (...) {
                break;
            }
        }
        return (int)th.size() + 1;
    }
    // false: a job threw (on the caller or on a worker); every worker has finished either way
    bool run(int nt, const std::function<void(int)>& f) {
        {
            std::lock_guard<std::mutex> lk(m);
            job = &f;
            n = nt;
            busy = (int)th.size();
            failed = false;
            gen++;
        }
        cv.notify_all();
        bool ok = true;
        try {
            f(0);
        } catch (...) {
            ok = false;
        }
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return busy == 0; });
        job = nullptr;
        return ok && !failed;
    }
    void worker(int t, unsigned long long seen) {
        std::unique_lock<std::mutex> lk(m);
        for (;;) {
            cv.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            const std::function<void(int)>* f = job;
            const int nt = n;
            lk.unlock();
            bool ok = true;
            if (t < nt && f) {
                try {
                    (*f)(t);
                } catch (...) {
                    ok = false;
                }
            }
            lk.lock();
            if (!ok) failed = true;
            if (--busy == 0) done.notify_all();
        }
    }
    ~PlanPool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& x : th) x.join();
    }
};

struct slam_lba {
    PlanPool plan_pool;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    Counters* h_cnt = nullptr;  // pinned, mapped: kRing slots, one per step in flight
    Counters* d_hcnt = nullptr; // device view of h_cnt (written by k_trial_control's last block)
    int* h_stop = nullptr;      // pinned, device-visible: the mirrored stop flag
    int* d_stop = nullptr;      // its device address
    unsigned step_seq = 0;      // sequence number of the last LM step queued (never reused)
    double last_ms = 0, last_plan_ms = 0;
    int last_syncs = 0;
    unsigned char* harena = nullptr;  // pinned
    size_t harena_cap = 0;
    DevBuf arena, cnt;
    DevBuf poses, pts, err, rho, lin, Hll, bl, Hpp, bp, pd, xp, xl, Hs, Ts;
    DevBuf Wg, tsync;            // helper-assisted LDL^T (k_ldlt_t16x): W tiles, hand-off words
    DevBuf bm, bmp, pbase, pls;  // pose bitmaps, their word prefixes, pose list bases, pose edge lists
    DevBuf ppt;                  // the point of every pose-list entry
    DevBuf pcnt;                 // free-pose edges per pose (pose list lengths)
    DevBuf spe_hp;               // free-pose index of every spe entry
    DevBuf ct, ct_off, ct_cnt;   // Schur contribution lists (built on the device)
    DevBuf outb;                 // one region for everything read back: KF poses, points, control
                                 // records, outlier flags (one D2H into hout)
    unsigned char* hout = nullptr;  // pinned
    size_t hout_cap = 0;
};

namespace {

struct WinStart {
    int kf0, pt0, e0, pose0, blk0, spe0, pe0;
    long long bm0, ct0, hs0;
    size_t h0;
};

struct PlanSizes {
    std::vector<WinStart> starts;
    int nkf = 0, npt = 0, ne = 0, npose = 0, nblk = 0, nspe = 0, npe = 0, nw = 0;
    long long nbm = 0, nct = 0, hs_total = 0;
    int max_n = 0;
    bool any_body = false;
    bool any_follow = false;           // some free-pose edge follows one of its point on its KeyFrame
    bool per_kf_cam = false;           // the KeyFrames of the batch do not share one calibration
    slam_camera cam{}, cam2{};         // the shared calibration otherwise
};

struct Layout {
    size_t edges, wins, ctl, pt_off, pt_win, spe_off, spe, pe_off, pe, pose_win, kf_hp, kf_win, blk_win,
        blk_order, blk_pose, kf_in, pt_in, kf_trl, kcam, kbf, total;
    size_t host_bytes;  // the host-written prefix (the device-built spe lists come last)
};

Layout make_layout(const PlanSizes& z) {
    Layout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    L.edges = take(sizeof(EdgeS) * z.ne);
    L.wins = take(sizeof(WinDesc) * z.nw);
    L.ctl = take(sizeof(WinCtl) * z.nw);
    L.pt_off = take(sizeof(int) * (z.npt + 1));
    L.pt_win = take(sizeof(int) * z.npt);
    L.spe_off = take(sizeof(int) * (z.npt + 1));
    L.pe_off = take(sizeof(int) * (z.npose + 1));
    L.pe = take(sizeof(int) * z.npe);
    L.pose_win = take(sizeof(int) * z.npose);
    L.kf_hp = take(sizeof(int) * z.nkf);
    L.kf_win = take(sizeof(int) * z.nkf);
    L.blk_win = take(sizeof(int) * z.nblk);
    L.blk_order = take(sizeof(int) * z.nblk);
    L.blk_pose = take(sizeof(int2) * z.nblk);
    L.kf_in = take(sizeof(float) * 16 * z.nkf);
    L.pt_in = take(sizeof(float) * 3 * z.npt);
    L.kf_trl = take(z.any_body ? sizeof(double) * 8 * z.nkf : 0);
    L.kcam = take(z.per_kf_cam ? sizeof(float4) * 2 * z.nkf : 0);
    L.kbf = take(z.per_kf_cam ? sizeof(float) * z.nkf : 0);
    L.host_bytes = off;
    L.spe = take(sizeof(int) * z.nspe);
    L.total = off;
    return L;
}

Plan bind(unsigned char* base, const Layout& L) {
    Plan P;
    P.edges = (EdgeS*)(base + L.edges);
    P.wins = (WinDesc*)(base + L.wins);
    P.ctl = (WinCtl*)(base + L.ctl);
    P.pt_off = (int*)(base + L.pt_off);
    P.pt_win = (int*)(base + L.pt_win);
    P.spe_off = (int*)(base + L.spe_off);
    P.spe = (int*)(base + L.spe);
    P.pe_off = (int*)(base + L.pe_off);
    P.pe = (int*)(base + L.pe);
    P.pose_win = (int*)(base + L.pose_win);
    P.kf_hp = (int*)(base + L.kf_hp);
    P.kf_win = (int*)(base + L.kf_win);
    P.blk_win = (int*)(base + L.blk_win);
    P.blk_order = (int*)(base + L.blk_order);
    P.blk_pose = (int2*)(base + L.blk_pose);
    P.kf_in = (float*)(base + L.kf_in);
    P.pt_in = (float*)(base + L.pt_in);
    P.kf_trl = (double*)(base + L.kf_trl);
    P.kcam = (float4*)(base + L.kcam);
    P.kbf = (float*)(base + L.kbf);
    return P;
}

// host threads of one call's planning (the handle's PlanPool): callers run several solvers at once
// (the bench's LBA leg: 4), and 16 planning threads per call oversubscribed the GPU box's 16-thread
// CPU share, delaying the solver threads that launch the next LM step; with the threads kept
// between calls, 8 measured best (plan 4.0-4.5 -> 2.6-2.8 ms per 128-window call, LBA leg
// 131-134k -> 139-145k LM it/s, profiles/r05_lba_plan.txt).  SLAMHOT_LBA_PLAN_THREADS overrides.
// Seconds a host wait on device progress may last (SLAMHOT_WAIT_TIMEOUT_S, default 60): one LM
// step of a 128-window batch takes about a millisecond.
double wait_timeout_s() {
    static const double v = [] {
        const char* e = std::getenv("SLAMHOT_WAIT_TIMEOUT_S");
        const double x = e ? std::atof(e) : 0.0;
        return x > 0.0 ? x : 60.0;
    }();
    return v;
}

int plan_threads(int n_prob) {
    static const int cap_env = std::getenv("SLAMHOT_LBA_PLAN_THREADS") ? std::atoi(std::getenv("SLAMHOT_LBA_PLAN_THREADS")) : 0;
    const int cap = cap_env > 0 ? cap_env : 8;
    const int hw = (int)std::max(1u, std::min((unsigned)cap, std::thread::hardware_concurrency()));
    return std::max(1, std::min(hw, n_prob));
}

// run fn(w, scratch) for every window on nth threads (window w on thread w % nth)
template <class S, class F>
slam_status for_windows(int n_prob, int nth, F fn, PlanPool* pool) {
    std::vector<slam_status> rs(nth, SLAM_OK);
    auto run = [&](int t) {
        S scratch;
        for (int w = t; w < n_prob; w += nth) {
            const slam_status r = fn(w, scratch);
            if (r != SLAM_OK) rs[t] = r;
        }
    };
    // a scratch allocation that throws (bad_alloc) ends that thread's windows with SLAM_ENOMEM
    auto run_safe = [&](int t) {
        try {
            run(t);
        } catch (...) {
            rs[t] = SLAM_ENOMEM;
        }
    };
    if (nth <= 1) {
        run_safe(0);
    } else if (pool) {
        const int have = pool->ensure(nth);
        const std::function<void(int)> f = [&](int t) {
            for (int u = t; u < nth; u += have) run_safe(u);  // threads the pool could not start: here
        };
        if (!pool->run(std::min(have, nth), f)) return SLAM_ENOMEM;
    } else {
        std::vector<std::thread> th;
        try {
            for (int t = 1; t < nth; t++) th.emplace_back(run_safe, t);
        } catch (...) {  // thread creation failed: the rest run here
            for (int t = (int)th.size() + 1; t < nth; t++) run_safe(t);
        }
        run_safe(0);
        for (auto& x : th) x.join();
    }
    for (slam_status r : rs)
        if (r != SLAM_OK) return r;
    return SLAM_OK;
}

// Pass 1: validation and sizes, per window on the planning threads, then the windows' start
// offsets (prefix sums).  hidx: free-pose index of every KF of every window.
slam_status plan_sizes(int n_prob, const slam_lba_problem* probs, PlanSizes& z, std::vector<int>& hidx_all,
                       std::vector<int>& np_of, PlanPool* pool) {
    z.nw = n_prob;
    np_of.assign(n_prob, 0);
    z.starts.resize(n_prob);
    size_t nkf_all = 0;
    for (int w = 0; w < n_prob; w++) {
        if (probs[w].n_kf < 0 || probs[w].n_pt < 0 || probs[w].n_edge < 0) return SLAM_EINVAL;
        z.starts[w].h0 = nkf_all;
        nkf_all += probs[w].n_kf;
    }
    hidx_all.assign(nkf_all, -1);
    struct WinSz {
        int npe = 0, nspe = 0;
        long long nct = 0;
        bool body = false;
    };
    std::vector<WinSz> sz(n_prob);
    struct SizeScratch {
        std::vector<int> cnt, stamp;
    };
    slam_status st = for_windows<SizeScratch>(n_prob, plan_threads(n_prob), [&](int w, SizeScratch& sc) {
        std::vector<int>& cnt = sc.cnt;
        const slam_lba_problem& P = probs[w];
        if ((P.n_kf && (!P.kf_Tcw || !P.kf_fixed)) || (P.n_pt && !P.pt_pos) ||
            (P.n_edge && (!P.edge_pt || !P.edge_kf || !P.edge_obs || !P.edge_inv_sigma2)))
            return SLAM_EINVAL;
        WinSz& S = sz[w];
        if (P.edge_body && P.n_edge) {
            bool has = false;
            for (int i = 0; i < P.n_edge && !has; i++) has = P.edge_body[i] != 0;
            if (has && !P.kf_Trl) return SLAM_EINVAL;  // body edges need each KeyFrame's mTrl
            S.body = has;
        }
        // One pass over the edges: validation, edges per KeyFrame, and the free-pose edge counts.
        // An edge's KeyFrame has an edge (this one), so it is a free pose iff it is not fixed.
        // Free-pose edges: an edge right after one of the same point on the same KeyFrame (body
        // edge) shares its Hpl block and has no Schur entry of its own; a point with k such edges
        // adds k (k + 1) / 2 Schur contributions.  Two such edges of one point on one KeyFrame
        // that are not adjacent are refused (a KeyFrame stamp per point).
        cnt.assign(P.n_kf, 0);
        std::vector<int>& stamp = sc.stamp;
        stamp.assign(P.n_kf, 0);
        int run = 0, pprev = -1, kprev = -1;
        for (int i = 0; i < P.n_edge; i++) {
            const int p = P.edge_pt[i], k = P.edge_kf[i];
            if (p < 0 || p >= P.n_pt || k < 0 || k >= P.n_kf) return SLAM_EINVAL;
            if (p < pprev) return SLAM_EINVAL;  // point-major insertion order
            cnt[k]++;
            if (p != pprev) {
                S.nct += (long long)run * (run + 1) / 2;
                run = 0;
            }
            const bool follows = p == pprev && k == kprev;
            pprev = p;
            kprev = k;
            if (P.kf_fixed[k] != 0) continue;
            S.npe++;
            if (!follows) {
                if (stamp[k] == p + 1) return SLAM_EINVAL;  // non-adjacent edges of 1 point in 1 KF
                stamp[k] = p + 1;
                S.nspe++;
                run++;
            }
        }
        S.nct += (long long)run * (run + 1) / 2;
        // a KeyFrame without edges is not an active vertex (sparse_optimizer.cpp:262-300): it
        // stays out of the Hessian and keeps its estimate
        int* hidx = &hidx_all[z.starts[w].h0];
        int np = 0;
        for (int k = 0; k < P.n_kf; k++) hidx[k] = P.kf_fixed[k] == 0 && cnt[k] > 0 ? np++ : -1;
        np_of[w] = np;
        if (6 * np > kMaxN) return SLAM_ECAP;
        return SLAM_OK;
    }, pool);
    if (st != SLAM_OK) return st;
    for (int w = 0; w < n_prob; w++) {
        z.any_body = z.any_body || sz[w].body;
        z.any_follow = z.any_follow || sz[w].npe != sz[w].nspe;
    }
    for (int w = 0; w < n_prob; w++) {
        const slam_lba_problem& P = probs[w];
        const int np = np_of[w];
        z.starts[w] = WinStart{z.nkf, z.npt, z.ne, z.npose, z.nblk, z.nspe, z.npe, z.nbm, z.nct, z.hs_total, z.starts[w].h0};
        z.nct += sz[w].nct;
        if (z.any_follow) z.npe += sz[w].npe;  // pe is built only for batches with followers
        z.nspe += sz[w].nspe;
        z.nbm += (long long)np * ((P.n_pt + 63) / 64);
        z.nkf += P.n_kf;
        z.npt += P.n_pt;
        z.ne += P.n_edge;
        z.npose += np;
        z.nblk += np * (np + 1) / 2;
        z.hs_total += (long long)(ldlt_npad(6 * np) + 1) * ldlt_ld(6 * np);
        z.max_n = std::max(z.max_n, 6 * np);
    }
    // one calibration for the whole batch (the usual case: the scalars go in the kernel
    // arguments), else a camera record per KeyFrame (Optimizer.cc:1840, 1869-1873, 1906)
    bool have = false, have2 = false;
    for (int w = 0; w < n_prob && !z.per_kf_cam; w++) {
        const slam_lba_problem& P = probs[w];
        const bool body = sz[w].body;
        for (int k = 0; k < P.n_kf && !z.per_kf_cam; k++) {
            const slam_camera& c = P.kf_cam ? P.kf_cam[k] : P.cam;
            if (!have) z.cam = c, have = true;
            else if (std::memcmp(&c, &z.cam, sizeof(slam_camera)) != 0) z.per_kf_cam = true;
            if (!body) continue;
            const slam_camera& c2 = P.kf_cam2 ? P.kf_cam2[k] : P.cam2;  // bf unused
            if (!have2) z.cam2 = c2, have2 = true;
            else if (std::memcmp(&c2, &z.cam2, 4 * sizeof(float)) != 0) z.per_kf_cam = true;
        }
    }
    return SLAM_OK;
}

// Pass 2: fill the arena in place.
slam_status plan_fill(int n_prob, const slam_lba_problem* probs, const std::vector<int>& hidx_all,
                      const std::vector<int>& np_of, const slam_lba_options* opt, const PlanSizes& Z,
                      const Plan& P, PlanPool* pool) {
    // windows are independent given their start offsets: fill them on host threads
#ifdef SLAMHOT_PLAN_BENCH
    // section cycle counts of plan_fill (rdtsc, summed over windows and threads)
    static std::atomic<long long> pb_sec[5];
    for (auto& x : pb_sec) x = 0;
#define PB_MARK(k) do { const long long t_ = (long long)__rdtsc(); if (k) pb_sec[(k) - 1] += t_ - pb_t; pb_t = t_; } while (0)
#else
#define PB_MARK(k) do {} while (0)
#endif
    auto fill_one = [&](int w, std::vector<int>& pcnt) -> slam_status {
#ifdef SLAMHOT_PLAN_BENCH
        long long pb_t = (long long)__rdtsc();
#endif
        const WinStart& ws = Z.starts[w];
        int nkf = ws.kf0, npt = ws.pt0, ne = ws.e0, npose = ws.pose0, nblk = ws.blk0, nspe = ws.spe0;
        long long hs = ws.hs0;
        const slam_lba_problem& Q = probs[w];
        const int* hidx = &hidx_all[ws.h0];
        const int np = np_of[w];
        WinDesc D{};
        D.kf0 = nkf;
        D.nk = Q.n_kf;
        D.pt0 = npt;
        D.npt = Q.n_pt;
        D.e0 = ne;
        D.ne = Q.n_edge;
        D.pose0 = npose;
        D.np = np;
        D.n = 6 * np;
        D.ld = ldlt_ld(D.n);
        D.blk0 = nblk;
        D.nblk = np * (np + 1) / 2;
        D.hs_off = hs;
        D.spe0 = ws.spe0;
        D.nwd = (Q.n_pt + 63) / 64;
        D.bm0 = ws.bm0;
        D.ct0 = ws.ct0;
        hs += (long long)(ldlt_npad(D.n) + 1) * D.ld;
        P.wins[w] = D;
        WinCtl c{};
        c.user_lambda = Q.user_lambda_init > 0 ? Q.user_lambda_init : opt->user_lambda_init;
        c.lambda = -1;
        c.ni = 2;
        P.ctl[w] = c;
        for (int k = 0; k < Q.n_kf; k++) {
            P.kf_hp[nkf + k] = hidx[k] >= 0 ? npose + hidx[k] : -1;
            P.kf_win[nkf + k] = w;
        }
        std::memcpy(P.kf_in + 16 * (size_t)nkf, Q.kf_Tcw, sizeof(float) * 16 * Q.n_kf);
        if (Z.per_kf_cam)
            for (int k = 0; k < Q.n_kf; k++) {
                const slam_camera& c = Q.kf_cam ? Q.kf_cam[k] : Q.cam;
                const slam_camera& c2 = Q.kf_cam2 ? Q.kf_cam2[k] : Q.cam2;
                P.kcam[2 * (size_t)(nkf + k)] = float4{c.fx, c.fy, c.cx, c.cy};
                P.kcam[2 * (size_t)(nkf + k) + 1] = float4{c2.fx, c2.fy, c2.cx, c2.cy};
                P.kbf[nkf + k] = c.bf;
            }
        if (Z.any_body) {  // Converter::toSE3Quat(pKFi->mTrl) -> SE3Quat(R, t) (se3quat.h:56-58)
            for (int k = 0; k < Q.n_kf; k++) {
                double* rec = P.kf_trl + 8 * (size_t)(nkf + k);
                if (!Q.edge_body || !Q.kf_Trl) {
                    const double id[8] = {0, 0, 0, 1, 0, 0, 0, 0};
                    std::memcpy(rec, id, sizeof(id));
                    continue;
                }
                const float* T = Q.kf_Trl + 16 * (size_t)k;
                double R[9];
                for (int a = 0; a < 3; a++)
                    for (int b = 0; b < 3; b++) R[3 * a + b] = T[4 * a + b];
                Quat q = quat_from_R(R);
                normalize_rotation(q);
                rec[0] = q.x;
                rec[1] = q.y;
                rec[2] = q.z;
                rec[3] = q.w;
                rec[4] = T[3];
                rec[5] = T[7];
                rec[6] = T[11];
                rec[7] = 0.0;
            }
        }
        PB_MARK(0);
        std::memcpy(P.pt_in + 3 * (size_t)npt, Q.pt_pos, sizeof(float) * 3 * Q.n_pt);
        // edge records, and in the same pass the point CSR and the offsets of the per-point
        // free-pose edge lists (the lists themselves, sorted by pose, are built on the device:
        // spe_build_body); a point's entries are written at its first edge (points without
        // edges: at the next point's, or after the last edge)
        int p_next = 0;
        for (int i = 0; i < Q.n_edge; i++) {
            EdgeS& e = P.edges[ne + i];
            const int k = Q.edge_kf[i], p = Q.edge_pt[i];
            for (; p_next <= p; p_next++) {
                P.pt_off[npt + p_next] = ne + i;
                P.pt_win[npt + p_next] = w;
                P.spe_off[npt + p_next] = nspe;
            }
            // the edge right after one on the same KeyFrame (body edge) shares its Hpl block
            const bool follows = i > 0 && Q.edge_pt[i - 1] == p && Q.edge_kf[i - 1] == k;
            nspe += hidx[k] >= 0 && !follows;
            e.pt = npt + p;
            e.kf = nkf + k;
            e.hp = hidx[k] >= 0 ? npose + hidx[k] : -1;
            e.win = w;
            e.obs[0] = Q.edge_obs[3 * i];
            e.obs[1] = Q.edge_obs[3 * i + 1];
            const bool body = Q.edge_body && Q.edge_body[i];
            const float ur = Q.edge_obs[3 * i + 2];
            e.obs[2] = body ? kBodyTag : (ur < 0.f ? -1.0f : ur);
            e.info = Q.edge_inv_sigma2[i];
        }
        for (; p_next < Q.n_pt; p_next++) {
            P.pt_off[npt + p_next] = ne + Q.n_edge;
            P.pt_win[npt + p_next] = w;
            P.spe_off[npt + p_next] = nspe;
        }
        PB_MARK(1);
        const int pe_start = ws.pe0;
        PB_MARK(2);
        // Schur blocks (i1 <= i2: blk = i2 (i2 + 1) / 2 + i1); their contributions come from the
        // pose bitmaps built on the device (k_bm_*)
        for (int i2 = 0, b = 0; i2 < np; i2++)
            for (int i1 = 0; i1 <= i2; i1++, b++) {
                P.blk_pose[nblk + b] = int2{i1, i2};
                P.blk_win[nblk + b] = w;
                // diagonal blocks of all windows first, then the off-diagonal ones
                if (i1 == i2) P.blk_order[npose + i2] = nblk + b;
                else P.blk_order[Z.npose + (nblk - npose) + (b - i2)] = nblk + b;
            }
        PB_MARK(3);
        for (int k = 0; k < np; k++) P.pose_win[npose + k] = w;
        // with followers (body edges): the edges of every free pose (followers included: each adds
        // its own Hpp), insertion order; otherwise the pose side reads the device-built pose lists
        if (Z.any_follow) {
            pcnt.assign(np + 1, 0);
            for (int e = 0; e < Q.n_edge; e++) {
                const int h = hidx[Q.edge_kf[e]];
                if (h >= 0) pcnt[h + 1]++;
            }
            for (int k = 0; k < np; k++) pcnt[k + 1] += pcnt[k];
            for (int k = 0; k < np; k++) P.pe_off[npose + k] = pe_start + pcnt[k];
            for (int e = 0; e < Q.n_edge; e++) {
                const int h = hidx[Q.edge_kf[e]];
                if (h >= 0) P.pe[pe_start + pcnt[h]++] = ne + e;
            }
        }
        PB_MARK(4);
        (void)nkf;
        return SLAM_OK;
    };
    struct FillScratch {
        std::vector<int> pcnt;
    };
    const slam_status st = for_windows<FillScratch>(n_prob, plan_threads(n_prob), [&](int w, FillScratch& sc) {
        return fill_one(w, sc.pcnt);
    }, pool);
    if (st != SLAM_OK) return st;
#ifdef SLAMHOT_PLAN_BENCH
    std::fprintf(stderr, "fill sections (Mcycles): header+edges %.1f, csr %.1f, blocks %.1f, pose lists %.1f\n",
                 pb_sec[0] / 1e6, pb_sec[1] / 1e6, pb_sec[2] / 1e6, pb_sec[3] / 1e6);
#endif
#undef PB_MARK
    P.pt_off[Z.npt] = Z.ne;
    P.spe_off[Z.npt] = Z.nspe;
    if (Z.any_follow) P.pe_off[Z.npose] = Z.npe;
    return SLAM_OK;
}

inline unsigned blocks(long long n, int t) { return (unsigned)std::max<long long>(1, (n + t - 1) / t); }

}  // namespace

extern "C" {

slam_status slamhot_lba_create(int device, slam_lba** out) {
    if (!out) return SLAM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= n) return SLAM_EINVAL;
    slam_lba* s = new (std::nothrow) slam_lba();
    if (!s) return SLAM_ENOMEM;
    s->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess ||
        hipHostMalloc((void**)&s->h_cnt, sizeof(Counters) * kRing, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->d_hcnt, s->h_cnt, 0) != hipSuccess ||
        hipHostMalloc((void**)&s->h_stop, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->d_stop, s->h_stop, 0) != hipSuccess) {
        slamhot_lba_destroy(s);
        return SLAM_EHIP;
    }
    std::memset(s->h_cnt, 0, sizeof(Counters) * kRing);
    if (hipFuncSetAttribute((const void*)k_ldlt, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)ldlt_lds_bytes(kMaxN)) != hipSuccess) {
        slamhot_lba_destroy(s);
        return SLAM_EHIP;
    }
    *out = s;
    return SLAM_OK;
}

void slamhot_lba_destroy(slam_lba* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->h_cnt) (void)hipHostFree(s->h_cnt);
    if (s->h_stop) (void)hipHostFree(s->h_stop);
    if (s->harena) (void)hipHostFree(s->harena);
    if (s->hout) (void)hipHostFree(s->hout);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

// A synthetic window of the given size solved once: loads every kernel of the single-window path
// and sizes the device buffers and the pinned arena, so the caller's first real solve pays none of
// that.  KeyFrames along a line looking down +z (the first two fixed), points in front of them,
// each seen by obs_per_pt consecutive KeyFrames (noise-free projections, every fourth stereo).
slam_status slamhot_lba_warmup(slam_lba* s, int n_kf, int n_pt, int obs_per_pt) {
    if (!s || n_kf < 3 || n_pt < 1 || obs_per_pt < 2 || obs_per_pt > n_kf) return SLAM_EINVAL;
    const slam_camera cam{435.2f, 435.2f, 367.45f, 252.2f, 47.9f};
    std::vector<float> Tcw(16 * (size_t)n_kf, 0.f), pts(3 * (size_t)n_pt), obs, isig;
    std::vector<uint8_t> fixed(n_kf, 0);
    std::vector<int32_t> ept, ekf;
    fixed[0] = 1;
    fixed[1] = 2;
    for (int k = 0; k < n_kf; k++) {
        float* T = &Tcw[16 * (size_t)k];
        T[0] = T[5] = T[10] = T[15] = 1.f;
        T[3] = -(0.05f * (float)k - 0.025f * (float)n_kf);  // t = -C, C = (x_k, 0, 0)
    }
    uint32_t lcg = 12345u;
    auto uni = [&]() {
        lcg = lcg * 1664525u + 1013904223u;
        return (float)(lcg >> 8) * (1.0f / 16777216.0f);
    };
    for (int p = 0; p < n_pt; p++) {
        float* X = &pts[3 * (size_t)p];
        X[0] = 3.f * uni() - 1.5f;
        X[1] = 2.f * uni() - 1.f;
        X[2] = 3.f + 5.f * uni();
        const int k0 = p % (n_kf - obs_per_pt + 1);
        for (int j = 0; j < obs_per_pt; j++) {
            const int k = k0 + j;
            const float xc = X[0] + Tcw[16 * (size_t)k + 3], z = X[2];
            const float u = cam.fx * xc / z + cam.cx + 0.3f * (uni() - 0.5f);
            const float v = cam.fy * X[1] / z + cam.cy + 0.3f * (uni() - 0.5f);
            ept.push_back(p);
            ekf.push_back(k);
            obs.push_back(u);
            obs.push_back(v);
            obs.push_back((ept.size() & 3) == 0 ? u - cam.bf / z : -1.f);
            isig.push_back(1.f);
        }
    }
    slam_lba_problem P{};
    P.n_kf = n_kf;
    P.kf_Tcw = Tcw.data();
    P.kf_fixed = fixed.data();
    P.n_pt = n_pt;
    P.pt_pos = pts.data();
    P.n_edge = (int32_t)ept.size();
    P.edge_pt = ept.data();
    P.edge_kf = ekf.data();
    P.edge_obs = obs.data();
    P.edge_inv_sigma2 = isig.data();
    P.cam = cam;
    std::vector<float> kf_out(Tcw.size()), pt_out(pts.size());
    std::vector<uint8_t> outl(ept.size());
    slam_lba_result R{};
    R.kf_Tcw = kf_out.data();
    R.pt_pos = pt_out.data();
    R.edge_outlier = outl.data();
    slam_lba_options opt{};
    opt.iters_first = 5;
    opt.iters_second = 10;
    return slamhot_lba_solve(s, 1, &P, &opt, nullptr, &R);
}

slam_status slamhot_lba_last_stats(const slam_lba* s, double* device_ms, double* plan_ms, int* syncs) {
    if (!s) return SLAM_EINVAL;
    if (device_ms) *device_ms = s->last_ms;
    if (plan_ms) *plan_ms = s->last_plan_ms;
    if (syncs) *syncs = s->last_syncs;
    return SLAM_OK;
}

slam_status slamhot_lba_solve(slam_lba* s, int n_prob, const slam_lba_problem* probs,
                              const slam_lba_options* opt, const volatile int32_t* stop_flag,
                              slam_lba_result* results) {
    if (!s || n_prob < 0 || (n_prob && (!probs || !results)) || !opt) return SLAM_EINVAL;
    if (opt->iters_first < 0 || opt->iters_second < 0) return SLAM_EINVAL;
    for (int w = 0; w < n_prob; w++)
        if ((probs[w].n_kf && !results[w].kf_Tcw) || (probs[w].n_pt && !results[w].pt_pos) ||
            (probs[w].n_edge && !results[w].edge_outlier))
            return SLAM_EINVAL;
    if (n_prob == 0) return SLAM_OK;
    const volatile uint8_t* stop_b = opt->stop_flag_bool;
    auto user_stop = [&]() -> bool { return (stop_flag && *stop_flag) || (stop_b && *stop_b); };
    const auto t_plan0 = std::chrono::steady_clock::now();
    // SLAMHOT_LBA_TRACE: host timestamps of the call's phases to stderr (latency study)
    const bool trace = std::getenv("SLAMHOT_LBA_TRACE") != nullptr;
    std::chrono::steady_clock::time_point tp[8];
    int ntp = 0;
    auto mark = [&]() {
        if (trace && ntp < 8) tp[ntp++] = std::chrono::steady_clock::now();
    };
    PlanSizes Z;
    std::vector<int> hidx_all, np_of;
    slam_status st = plan_sizes(n_prob, probs, Z, hidx_all, np_of, &s->plan_pool);
    if (st != SLAM_OK) return st;
    const bool stop0 = user_stop();
    for (int w = 0; w < n_prob; w++) {
        slam_lba_result& R = results[w];
        R.iterations[0] = R.iterations[1] = 0;
        R.trials = 0;
        R.n_outlier = 0;
        R.chi2_initial = R.chi2_final = R.lambda_final = 0;
        R.ran = stop0 ? 0 : 1;
    }
    if (stop0) {  // Optimizer.cc:1921-1923: nothing optimized, nothing written back
        for (int w = 0; w < n_prob; w++) {
            const slam_lba_problem& P = probs[w];
            std::memcpy(results[w].kf_Tcw, P.kf_Tcw, sizeof(float) * 16 * P.n_kf);
            std::memcpy(results[w].pt_pos, P.pt_pos, sizeof(float) * 3 * P.n_pt);
            std::memset(results[w].edge_outlier, 0, P.n_edge);
        }
        s->last_ms = 0;
        s->last_plan_ms = 0;
        s->last_syncs = 0;
        return SLAM_OK;
    }
    SLAM_HIP_TRY(hipSetDevice(s->device));
    hipStream_t S = s->stream;
    const int nw = n_prob;
    if (nw >= (1 << kTallyBits)) return SLAM_EINVAL;  // the step tally's 21-bit fields
    const Layout LY = make_layout(Z);
    if (LY.total > s->harena_cap) {
        SLAM_HIP_TRY(hipStreamSynchronize(S));
        if (s->harena) (void)hipHostFree(s->harena);
        s->harena = nullptr;
        s->harena_cap = 0;
        SLAM_HIP_TRY(hipHostMalloc((void**)&s->harena, LY.total, hipHostMallocDefault));
        s->harena_cap = LY.total;
    }
    const Plan HP = bind(s->harena, LY);
    const auto t_fill0 = std::chrono::steady_clock::now();
    st = plan_fill(n_prob, probs, hidx_all, np_of, opt, Z, HP, &s->plan_pool);
    if (st != SLAM_OK) return st;
    if (std::getenv("SLAMHOT_LBA_PLAN_TIMING")) {
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "lba plan: sizes+alloc %.3f ms, fill %.3f ms, arena %.1f MB\n",
                     std::chrono::duration<double, std::milli>(t_fill0 - t_plan0).count(),
                     std::chrono::duration<double, std::milli>(t1 - t_fill0).count(), LY.total / 1e6);
    }
    SLAM_HIP_TRY(s->arena.ensure(LY.total));
    SLAM_HIP_TRY(hipMemcpyAsync(s->arena.p, s->harena, LY.host_bytes, hipMemcpyHostToDevice, S));
    const Plan DP = bind((unsigned char*)s->arena.p, LY);
    struct {
        int nkf, npt, ne, npose, nblk;
    } H{Z.nkf, Z.npt, Z.ne, Z.npose, Z.nblk};
    const long long pose_stride = 8LL * std::max(H.nkf, 1), pt_stride = 4LL * std::max(H.npt, 1);
    SLAM_HIP_TRY(s->cnt.ensure(sizeof(int) * 8));  // k_trial_control's tally (need, active, ticket, -, stop x 2)
    const size_t ne = std::max(H.ne, 1), npt = std::max(H.npt, 1), nps = std::max(H.npose, 1);
    SLAM_HIP_TRY(s->poses.ensure(sizeof(double) * 2 * pose_stride));
    SLAM_HIP_TRY(s->pts.ensure(sizeof(double) * 2 * pt_stride));
    SLAM_HIP_TRY(s->err.ensure(sizeof(double) * 4 * ne));
    SLAM_HIP_TRY(s->rho.ensure(sizeof(double) * ne));
    SLAM_HIP_TRY(s->lin.ensure(sizeof(double) * kHplStride * ne));
    SLAM_HIP_TRY(s->pd.ensure(sizeof(double) * kPdStride * npt));
    SLAM_HIP_TRY(s->Hll.ensure(sizeof(double) * 8 * npt));
    SLAM_HIP_TRY(s->bl.ensure(sizeof(double) * 4 * npt));
    SLAM_HIP_TRY(s->xl.ensure(sizeof(double) * 4 * npt));
    SLAM_HIP_TRY(s->Hpp.ensure(sizeof(double) * 24 * nps));
    SLAM_HIP_TRY(s->bp.ensure(sizeof(double) * 8 * nps));
    SLAM_HIP_TRY(s->xp.ensure(sizeof(double) * 6 * nps));
    SLAM_HIP_TRY(s->bm.ensure(sizeof(unsigned long long) * std::max<long long>(Z.nbm, 1)));
    SLAM_HIP_TRY(s->bmp.ensure(sizeof(int) * std::max<long long>(Z.nbm, 1)));
    SLAM_HIP_TRY(s->pbase.ensure(sizeof(int) * nps));
    SLAM_HIP_TRY(s->pcnt.ensure(sizeof(int) * nps));
    SLAM_HIP_TRY(s->pls.ensure(sizeof(int) * std::max(Z.nspe, 1)));
    SLAM_HIP_TRY(s->ppt.ensure(sizeof(int) * std::max(Z.nspe, 1)));
    SLAM_HIP_TRY(s->spe_hp.ensure(sizeof(int) * std::max(Z.nspe, 1)));
    if (Z.nct >= (1LL << 31)) return SLAM_ECAP;  // int contribution offsets
    SLAM_HIP_TRY(s->ct.ensure(sizeof(int4) * std::max<long long>(Z.nct, 1)));
    SLAM_HIP_TRY(s->ct_off.ensure(sizeof(int) * (Z.nblk + 1)));
    SLAM_HIP_TRY(s->ct_cnt.ensure(sizeof(int) * std::max(Z.nblk, 1)));
    // tile LDL^T (k_ldlt_t16) when every window fits 18 tile rows (SLAMHOT_LDLT=panel: old kernel)
    const char* ldlt_env = std::getenv("SLAMHOT_LDLT");
    const bool use_t16 = Z.max_n <= 16 * kT16Max && !(ldlt_env && !std::strcmp(ldlt_env, "panel"));
    SLAM_HIP_TRY(s->Hs.ensure(sizeof(double) * std::max<long long>(Z.hs_total, 1)));
    if (use_t16) SLAM_HIP_TRY(s->Ts.ensure((size_t)t16_tiles_bytes() * nw));
    // SLAMHOT_LDLT_HELP=1: up to 8 windows factor with helper workgroups on other CUs (k_ldlt_t16x).
    // Measured slower than the one-workgroup kernel at n = 288 (115-128 vs 107 us, x bit-identical,
    // profiles/r06_ldlt_helpers.txt), so it is not the default.
    const char* help_env = std::getenv("SLAMHOT_LDLT_HELP");
    const bool use_help = use_t16 && nw <= 8 && help_env && std::atoi(help_env) != 0;
    if (use_help) {
        SLAM_HIP_TRY(s->Wg.ensure((size_t)t16_tiles_bytes() * 8));
        if (s->tsync.cap < sizeof(T16Sync) * 8) {  // zero once; every launch leaves the words at zero
            SLAM_HIP_TRY(s->tsync.ensure(sizeof(T16Sync) * 8));
            SLAM_HIP_TRY(hipMemsetAsync(s->tsync.p, 0, sizeof(T16Sync) * 8, S));
        }
    }
    // read-back region: [KF poses | points | control records | outlier flags], 256-byte sections
    auto up256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_pt = up256(sizeof(float) * 16 * std::max(H.nkf, 1));
    const size_t o_ctl = o_pt + up256(sizeof(float) * 3 * npt);
    const size_t o_outl = o_ctl + up256(sizeof(WinCtl) * nw);
    const size_t out_bytes = o_outl + up256(ne);
    SLAM_HIP_TRY(s->outb.ensure(out_bytes));
    if (out_bytes > s->hout_cap) {
        SLAM_HIP_TRY(hipStreamSynchronize(S));
        if (s->hout) (void)hipHostFree(s->hout);
        s->hout = nullptr;
        s->hout_cap = 0;
        SLAM_HIP_TRY(hipHostMalloc((void**)&s->hout, out_bytes, hipHostMallocDefault));
        s->hout_cap = out_bytes;
    }
    unsigned char* dout = (unsigned char*)s->outb.p;
    s->last_plan_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_plan0).count();
    mark();  // 0: planned, arena copy queued, buffers sized

    Cam cam;  // the batch's one calibration, or per-KeyFrame records (PlanSizes::per_kf_cam)
    cam.fx = Z.cam.fx;
    cam.fy = Z.cam.fy;
    cam.cx = Z.cam.cx;
    cam.cy = Z.cam.cy;
    cam.bf = Z.cam.bf;
    cam.bff = (double)(float)Z.cam.bf;
    cam.trl = Z.any_body ? DP.kf_trl : nullptr;
    cam.fx2 = Z.cam2.fx;
    cam.fy2 = Z.cam2.fy;
    cam.cx2 = Z.cam2.cx;
    cam.cy2 = Z.cam2.cy;
    cam.kcam = Z.per_kf_cam ? DP.kcam : nullptr;
    cam.kbf = Z.per_kf_cam ? DP.kbf : nullptr;
    Huber hk;
    const float thMono = std::sqrt(5.991), thStereo = std::sqrt(7.815);  // Optimizer.cc:1794-1795
    hk.delta_mono = thMono;
    hk.delta_stereo = thStereo;
    hk.dsqr_mono = (float)(hk.delta_mono * hk.delta_mono);
    hk.dsqr_stereo = (float)(hk.delta_stereo * hk.delta_stereo);

    EdgeS* dE = DP.edges;
    WinDesc* dW = DP.wins;
    WinCtl* dC = DP.ctl;
    int* dTally = as<int>(s->cnt);
    double* poses = as<double>(s->poses);
    double* pts = as<double>(s->pts);
    const int T = 256;
    // the caller's stop flag as the device sees it at the start (k_trial_control's samples, tally
    // words 4 and 5)
    *s->h_stop = user_stop() ? 1 : 0;
    SLAM_HIP_TRY(hipEventRecord(s->ev0, S));
    SetupArgs SA{};
    {
        ClearList CL{};
        long long most = 0;
        auto add = [&](void* p, long long words, unsigned long long v) {
            if (CL.n >= kClearMax) return;  // sized for the ranges below (static_assert-like guard)
            CL.r[CL.n++] = ClearRange{(unsigned long long*)p, words, v};
            most = std::max(most, words);
        };
        add(s->bm.p, std::max<long long>(Z.nbm, 1), 0ull);
        add(s->xp.p, 6 * (long long)nps, 0ull);
        add(s->xl.p, 4 * (long long)npt, 0ull);
        add(s->err.p, 4 * (long long)ne, 0ull);
        const unsigned long long st2 = (unsigned long long)(unsigned)*s->h_stop;
        add(dTally, 1, 0ull);                                         // need, active
        add(dTally + 2, 1, 0ull);                                     // ticket, -
        add(dTally + 4, 1, st2 | (st2 << 32));                        // stop samples x 2
        add(dTally + 6, 1, 0ull);                                     // device error word, -
        if (use_t16) add(s->Ts.p, t16_tiles_bytes() * nw / 8, 0ull);  // tile scratch (padding by k_t16_pad)
        if (CL.n != (use_t16 ? 9 : 8)) return SLAM_EINVAL;  // every range above made it into the list
        SA.clear = CL;
        SA.nb_clear = (int)std::min<long long>(1024, (most + 255) / 256);
    }
    double* tiles = use_t16 ? as<double>(s->Ts) : nullptr;
    // optimize(5) and optimize(10) as one stream of steps: each window's control block moves on to
    // its second optimize() when the first ends without a stop (k_trial_control), so the host
    // neither waits at the boundary nor drains queued steps there
    const int iters_of[2] = {opt->iters_first, opt->iters_second};
    const int o0 = iters_of[0] > 0 ? 0 : 1;
    {
        auto cdiv = [](long long n, int t) { return (int)((n + t - 1) / t); };
        SA.nb_init = cdiv(H.nkf + H.npt, 256);
        SA.nb_pts = cdiv(H.npt, 256);
        SA.pt_off = DP.pt_off;
        SA.spe_off = DP.spe_off;
        SA.spe_out = DP.spe;
        SA.nb_spe = cdiv(Z.nspe, 256);
        SA.nb_blk = cdiv(H.nblk, 256);
        SA.nb_list = cdiv(Z.nspe, kCtScanThreads);
        SA.nw_scan = H.nblk ? nw : 0;
        SA.nw = nw;
        SA.nkf = H.nkf;
        SA.npt = H.npt;
        SA.nspe = Z.nspe;
        SA.nblk = H.nblk;
        SA.wins = dW;
        SA.ctl = dC;
        SA.opt = o0;
        SA.iters = iters_of[o0];
        SA.iters2 = o0 == 0 ? iters_of[1] : 0;
        SA.kf_in = DP.kf_in;
        SA.pt_in = DP.pt_in;
        SA.poses = poses;
        SA.pts = pts;
        SA.Hs = as<double>(s->Hs);
        SA.Ts = tiles;
        SA.spe = DP.spe;
        SA.E = DP.edges;
        SA.bm = as<unsigned long long>(s->bm);
        SA.spe_hp = as<int>(s->spe_hp);
        SA.bmp = as<int>(s->bmp);
        SA.pbase = as<int>(s->pbase);
        SA.pcnt = as<int>(s->pcnt);
        SA.pls = as<int>(s->pls);
        SA.ppt = as<int>(s->ppt);
        SA.blk_pose = DP.blk_pose;
        SA.blk_win = DP.blk_win;
        SA.ct_cnt = as<int>(s->ct_cnt);
        SA.ct_off = as<int>(s->ct_off);
        // (a) clears, initial estimates, dense padding, optimize() start; (b) pose bitmaps and tile
        // padding; (c) bitmap prefixes / pose list bases (pose list lengths even without edges) and
        // contribution counts; (d) contribution offsets and pose edge lists; then the lists
        k_setup_a<<<SA.nb_clear + SA.nb_pts + SA.nb_init + nw + cdiv(nw, 256), 256, 0, S>>>(SA);
        const int nb_b = SA.nb_spe + (use_t16 ? nw : 0);
        if (nb_b) k_setup_b<<<nb_b, 256, 0, S>>>(SA);
        k_setup_c<<<nw + SA.nb_blk, 256, 0, S>>>(SA);
        const int nb_d = SA.nw_scan + SA.nb_list;
        if (nb_d) k_setup_d<<<nb_d, kCtScanThreads, 0, S>>>(SA);
        if (H.nblk)
            k_ct_fill<<<blocks(H.nblk, 4), 256, 0, S>>>(H.nblk, DP.blk_pose, DP.blk_win, DP.wins,
                                                         as<unsigned long long>(s->bm), as<int>(s->bmp),
                                                         as<int>(s->pbase), as<int>(s->pls), as<int>(s->ct_off),
                                                         as<int4>(s->ct));
    }
    const size_t lds_bytes = ldlt_lds_bytes(Z.max_n);
    // Schur complement by block row (k_schur_rows: a workgroup per free pose) for batches with
    // enough rows to fill the chip; a few windows (LocalMapping's one-window call) keep the
    // per-block kernel, whose smaller work items finish a lone window sooner (0.214 vs 0.220 ms
    // per LM iteration).  SLAMHOT_SCHUR=rows / blocks forces one.
    const char* schur_env = std::getenv("SLAMHOT_SCHUR");
    const bool schur_rows = schur_env ? std::strcmp(schur_env, "blocks") != 0 : H.npose >= 256;
    // LM as device-driven steps: a step linearizes the windows that start an iteration
    // (need_lin) and runs one trial for those in the trial loop (need_trial); every kernel skips
    // the other windows, so the host queues steps without waiting for any decision and reads
    // the per-step counters asynchronously (a ring of kRing steps in flight).  While it waits it
    // mirrors the caller's stop flag into pinned memory the control kernels read.
    int syncs = 0, step_no = 0;
    // Wait for a step's counters: the last k_trial_control block stores the step's sequence
    // number into the mapped slot after the counts.  The host spins on that word (mirroring the
    // caller's stop flag meanwhile) and asks the stream for errors now and then, so a faulted
    // kernel ends the wait instead of hanging it.
    // The wait is bounded in wall-clock time (wait_timeout_s(), SLAMHOT_WAIT_TIMEOUT_S): a step
    // whose counters do not arrive by then ends the call with SLAM_ETIMEDOUT, naming the slot, the
    // sequence numbers and the stream state on stderr.  After every 1024 polls the thread also
    // yields its core: several solver threads wait at once beside the planning threads, and a
    // waiter must not hold a core another thread needs to queue the work it waits for.
    const auto wait_deadline = std::chrono::duration<double>(wait_timeout_s());
    auto wait_step = [&](int slot, int seq) -> slam_status {
        volatile Counters* c = s->h_cnt + slot;
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned spin = 1;; spin++) {
            if (c->seq == seq) {
                if (c->pad != 0) {
                    std::fprintf(stderr, "slamhot lba: %d device hand-off wait(s) gave up in k_ldlt_t16 (step seq %d)\n",
                                 (int)c->pad, seq);
                    return SLAM_ETIMEDOUT;
                }
                return SLAM_OK;
            }
            if (!*s->h_stop && user_stop()) *s->h_stop = 1;
            if ((spin & 1023) == 0) {
                const hipError_t e = hipStreamQuery(S);
                if (e == hipSuccess && c->seq != seq) {  // drained without publishing
                    std::fprintf(stderr, "slamhot lba: stream drained without step seq %d (slot %d holds %d)\n", seq, slot,
                                 (int)c->seq);
                    return SLAM_EHIP;
                }
                if (e != hipSuccess && e != hipErrorNotReady) {
                    std::fprintf(stderr, "slamhot lba: stream error %s waiting for step seq %d\n", hipGetErrorName(e), seq);
                    return SLAM_EHIP;
                }
                if (std::chrono::steady_clock::now() - t0 > wait_deadline) {
                    std::fprintf(stderr,
                                 "slamhot lba: no counters for step seq %d after %.0f s (slot %d holds seq %d, stream %s, "
                                 "%d windows); SLAM_ETIMEDOUT\n",
                                 seq, wait_deadline.count(), slot, (int)c->seq,
                                 e == hipErrorNotReady ? "busy" : "idle", nw);
                    return SLAM_ETIMEDOUT;
                }
                std::this_thread::yield();
            }
            _mm_pause();
        }
    };
    // grid partitions of the fused launches
    const int nb_lin_pose = (H.npose + kLinThreads / 64 - 1) / (kLinThreads / 64);
    const int nb_lin = nb_lin_pose + (H.npt + kLinThreads - 1) / kLinThreads;
    const int nb_sdiag = ((H.npose + 256 / kSchurDiagLanes - 1) / (256 / kSchurDiagLanes) + 7) & ~7;
    const int nb_schur = nb_sdiag + (H.nblk - H.npose + 256 / kSchurLanes - 1) / (256 / kSchurLanes);
    const int nb_kf = (H.nkf + 255) / 256;
    const int nb_upd = nb_kf + (H.npt + 255) / 256;
    // the pose side's edge lists: the device-built pls unless the batch has followers (pe)
    const PoseLists pose_lists = Z.any_follow ? PoseLists{nullptr, nullptr, nullptr, nullptr}
                                            : PoseLists{as<int>(s->pls), as<int>(s->pbase), as<int>(s->pcnt), dW};
    auto launch_step = [&](int slot, int seq) -> hipError_t {
        if (nb_lin)
            k_linearize<<<nb_lin, kLinThreads, 0, S>>>(nb_lin_pose, H.npose, DP.pe_off, DP.pe, pose_lists, DP.pose_win, H.npt,
                                                       DP.pt_off, DP.pt_win, dE, dC, poses, pts, pose_stride,
                                                       pt_stride, cam, hk, as<double>(s->err), as<double>(s->rho),
                                                       as<double>(s->lin), as<double>(s->Hll), as<double>(s->bl),
                                                       as<double>(s->Hpp), as<double>(s->bp));
        k_iter_begin<<<nw, kCtlThreads, 0, S>>>(dW, dC, as<double>(s->rho), as<double>(s->Hpp),
                                                as<double>(s->Hll), dTally + 4, seq);
        if (H.npt)
            k_point_prep<<<blocks(H.npt, T), T, 0, S>>>(H.npt, DP.pt_win, dC, as<double>(s->Hll), as<double>(s->bl),
                                                         as<double>(s->pd));
        if (H.nblk && schur_rows)
            k_schur_rows<<<H.npose, kSrThreads, 0, S>>>(H.npose, DP.pose_win, dW, dC, as<int>(s->pls), as<int>(s->ppt),
                                                        as<int>(s->pbase),
                                                        as<int>(s->pcnt), dE, as<int>(s->ct_off), as<int4>(s->ct),
                                                        as<double>(s->Hpp), as<double>(s->bp), as<double>(s->lin),
                                                        as<double>(s->pd), as<double>(s->Hs), tiles);
        else if (H.nblk)
            k_schur_blocks<<<nb_schur, 256, 0, S>>>(nb_sdiag, H.nblk, H.npose, DP.blk_order, DP.blk_pose, DP.blk_win,
                                                    as<int>(s->ct_off), as<int4>(s->ct), dW, dC, as<double>(s->Hpp),
                                                    as<double>(s->bp), as<double>(s->lin), as<double>(s->pd),
                                                    as<double>(s->Hs), tiles);
        if (use_help)
            k_ldlt_t16x<<<8 * (1 + kT16Helpers), kT16Waves * 64, 0, S>>>(nw, dW, dC, as<double>(s->Hs), as<double>(s->Ts),
                                                                         as<double>(s->Wg), as<T16Sync>(s->tsync),
                                                                         as<double>(s->xp), dTally + 6);
        else if (use_t16)
            k_ldlt_t16<<<nw, kT16Waves * 64, 0, S>>>(dW, dC, as<double>(s->Hs), as<double>(s->Ts), as<double>(s->xp),
                                                     dTally + 6);
        else
            k_ldlt<<<nw, 512, lds_bytes, S>>>(dW, dC, as<double>(s->Hs), as<double>(s->xp));
        if (nb_upd)
            k_update<<<nb_upd, 256, 0, S>>>(nb_kf, H.nkf, DP.kf_hp, DP.kf_win, H.npt, DP.spe_off, DP.spe, as<int>(s->spe_hp),
                                            DP.pt_win, dC, as<double>(s->bl), as<double>(s->pd), as<double>(s->lin),
                                            as<double>(s->xp), as<double>(s->xl), poses, pose_stride, pts, pt_stride);
        if (H.ne)
            k_trial_error<<<blocks(H.ne, T), T, 0, S>>>(H.ne, dE, dC, poses, pts, pose_stride, pt_stride, cam, hk,
                                                         as<double>(s->err), as<double>(s->rho));
        k_trial_control<<<nw, kCtlThreads, 0, S>>>(dW, dC, as<double>(s->rho), as<double>(s->xp),
                                                   as<double>(s->xl), as<double>(s->bp), as<double>(s->bl),
                                                   s->d_stop, dTally, s->d_hcnt + slot, seq);
        return hipGetLastError();
    };
    mark();  // 1: setup kernels launched
    // steps queued ahead of the one the host waits on: a few windows (a step of ~0.17 ms against
    // ~30 us to queue the next) need one, which leaves one no-op step after the last instead of
    // two; big batches keep more in flight.  SLAMHOT_LBA_DEPTH overrides (A/B)
    const char* depth_env = std::getenv("SLAMHOT_LBA_DEPTH");
    const int depth = depth_env ? std::max(2, std::min(kRing - 1, std::atoi(depth_env))) : (nw <= 8 ? 2 : kRing - 1);
    {
        long long launched = 0, checked = 0;
        int seqs[kRing] = {0, 0, 0, 0};
        bool done = iters_of[o0] <= 0;
        while (!done) {
            if (launched - checked < depth) {  // keep the device fed
                const int slot = (int)(launched % kRing);
                seqs[slot] = (int)(++s->step_seq & 0x7fffffff);
                SLAM_HIP_TRY(launch_step(slot, seqs[slot]));
                launched++;
                if (launched - checked < 2) continue;  // two steps queued before the first wait
            }
            const int slot = (int)(checked % kRing);
            {
                // an error ends the call here; steps still queued stay ordered on the handle's
                // stream ahead of anything a later call queues
                const slam_status ws = wait_step(slot, seqs[slot]);
                if (ws != SLAM_OK) return ws;
            }
            if (syncs == 0) mark();  // 2: the first step's counters are in
            syncs++;
            checked++;
            if (opt->step_hook) {  // diagnostic hook (slam_lba_options): may set the caller's flag
                opt->step_hook(opt->step_hook_ctx, step_no);
                if (!*s->h_stop && user_stop()) *s->h_stop = 1;
            }
            step_no++;
            const Counters c = s->h_cnt[slot];
            done = c.active == 0 && c.need_trial == 0;
        }
        // the steps still queued are no-ops; the finalize kernels follow them in stream order
    }
    mark();  // 3: LM loop done
    {
        static_assert(sizeof(WinCtl) % sizeof(int) == 0, "k_finalize copies the control blocks as ints");
        FinalArgs FA{};
        FA.ne = H.ne;
        FA.nkf = H.nkf;
        FA.npt = H.npt;
        FA.nw = nw;
        FA.nb_edges = (H.ne + T - 1) / T;
        FA.nb_state = (H.nkf + H.npt + T - 1) / T;
        FA.E = dE;
        FA.ctl = dC;
        FA.poses = poses;
        FA.pts = pts;
        FA.pose_stride = pose_stride;
        FA.pt_stride = pt_stride;
        FA.err = as<double>(s->err);
        FA.trl = cam.trl;
        FA.kf_win = DP.kf_win;
        FA.pt_win = DP.pt_win;
        FA.outlier = dout + o_outl;
        FA.kf_out = (float*)dout;
        FA.pt_out = (float*)(dout + o_pt);
        FA.ctl_out = (int*)(dout + o_ctl);
        k_finalize<<<FA.nb_edges + FA.nb_state + 1, T, 0, S>>>(FA);
    }
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipEventRecord(s->ev1, S));
    // one pinned read-back (pageable copies are synchronous, ~40 us each)
    SLAM_HIP_TRY(hipMemcpyAsync(s->hout, dout, out_bytes, hipMemcpyDeviceToHost, S));
    mark();  // 4: finalize + copies queued
    SLAM_HIP_TRY(hipStreamSynchronize(S));
    mark();  // 5: results on the host
    const float* kf_out = (const float*)s->hout;
    const float* pt_out = (const float*)(s->hout + o_pt);
    const WinCtl* ctl1 = (const WinCtl*)(s->hout + o_ctl);
    const uint8_t* outl = s->hout + o_outl;
    float ms = 0;
    SLAM_HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_syncs = syncs + 1;
    for (int w = 0; w < nw; w++) {
        const slam_lba_problem& P = probs[w];
        const WinDesc& D = HP.wins[w];
        slam_lba_result& R = results[w];
        for (int k = 0; k < P.n_kf; k++) {
            const float* src = P.kf_fixed[k] == 2 ? P.kf_Tcw + 16 * k : &kf_out[16 * (size_t)(D.kf0 + k)];
            std::memcpy(R.kf_Tcw + 16 * k, src, sizeof(float) * 16);
        }
        std::memcpy(R.pt_pos, &pt_out[3 * (size_t)D.pt0], sizeof(float) * 3 * P.n_pt);
        int no = 0;
        for (int i = 0; i < P.n_edge; i++) {
            R.edge_outlier[i] = outl[D.e0 + i];
            no += outl[D.e0 + i];
        }
        R.n_outlier = no;
        const WinCtl& C = ctl1[w];
        R.iterations[0] = C.iters_run[0];
        R.iterations[1] = C.iters_run[1];
        R.trials = C.trials;
        R.chi2_initial = C.chi2_initial;
        R.chi2_final = C.chi2_final;
        R.lambda_final = C.lambda;
    }
    mark();  // 6: results copied out
    if (trace) {
        auto ms_of = [&](int i) { return std::chrono::duration<double, std::milli>(tp[i] - t_plan0).count(); };
        std::fprintf(stderr, "lba trace ms: plan %.3f setup %.3f first_step %.3f loop %.3f queued %.3f synced %.3f out %.3f device %.3f steps %d\n",
                     ms_of(0), ms_of(1), ms_of(2), ms_of(3), ms_of(4), ms_of(5), ms_of(6), s->last_ms, syncs);
    }
    return SLAM_OK;
}

#ifdef SLAMHOT_PLAN_BENCH
// Experiment builds only (tools/microbench/lba_plan_bench.py): the host plan of a call, no device
// work, into ordinary memory; reps repetitions, the last one's phase times returned.
slam_status slamhot_lba_plan_bench(int n_prob, const slam_lba_problem* probs, const slam_lba_options* opt, int reps,
                                   double* sizes_ms, double* fill_ms, double* arena_mb) {
    std::vector<unsigned char> arena;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        PlanSizes Z;
        std::vector<int> hidx_all, np_of;
        static PlanPool bench_pool;
        slam_status st = plan_sizes(n_prob, probs, Z, hidx_all, np_of, &bench_pool);
        if (st != SLAM_OK) return st;
        const Layout LY = make_layout(Z);
        if (arena.size() < LY.total) arena.resize(LY.total);
        const auto t1 = std::chrono::steady_clock::now();
        st = plan_fill(n_prob, probs, hidx_all, np_of, opt, Z, bind(arena.data(), LY), &bench_pool);
        if (st != SLAM_OK) return st;
        const auto t2 = std::chrono::steady_clock::now();
        *sizes_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        *fill_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
        *arena_mb = LY.total / 1e6;
    }
    return SLAM_OK;
}

// Sanitizer builds (tests/cpp/plan_stress.cpp under TSan / ASan, `make sanitize-plan`): nthreads
// host threads, each with a PlanPool and an arena of its own (one per solver handle, as slam_lba
// holds them), plan rounds x ncounts calls of the first counts[c] windows each, so every pool gains
// workers between calls (4 -> 8 -> 128 windows) while the other threads plan too.  Every thread's
// host plan of a call must equal the others' byte for byte (SLAM_EINVAL otherwise).
slam_status slamhot_lba_plan_stress(int nthreads, int rounds, const int* counts, int ncounts, int n_prob,
                                    const slam_lba_problem* probs, const slam_lba_options* opt) {
    if (nthreads < 1 || rounds < 1 || ncounts < 1 || !counts || !probs || !opt) return SLAM_EINVAL;
    const int ncalls = rounds * ncounts;
    std::vector<std::vector<unsigned long long>> hashes(nthreads, std::vector<unsigned long long>(ncalls, 0));
    std::vector<slam_status> st(nthreads, SLAM_OK);
    auto body = [&](int t) {
        PlanPool pool;
        std::vector<unsigned char> arena;
        for (int r = 0; r < rounds; r++)
            for (int c = 0; c < ncounts; c++) {
                const int n = std::min(counts[c], n_prob);
                PlanSizes Z;
                std::vector<int> hidx_all, np_of;
                slam_status s = plan_sizes(n, probs, Z, hidx_all, np_of, &pool);
                if (s != SLAM_OK) { st[t] = s; return; }
                const Layout LY = make_layout(Z);
                arena.assign(LY.total, 0);
                s = plan_fill(n, probs, hidx_all, np_of, opt, Z, bind(arena.data(), LY), &pool);
                if (s != SLAM_OK) { st[t] = s; return; }
                unsigned long long h = 1469598103934665603ull;
                for (size_t i = 0; i < LY.host_bytes; i++) h = (h ^ arena[i]) * 1099511628211ull;
                hashes[t][r * ncounts + c] = h;
            }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(body, t);
    body(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < nthreads; t++)
        if (st[t] != SLAM_OK) return st[t];
    for (int t = 1; t < nthreads; t++)
        if (hashes[t] != hashes[0]) return SLAM_EINVAL;
    return SLAM_OK;
}
#endif

}  // extern "C"
