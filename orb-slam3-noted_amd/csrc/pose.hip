// pose.hip — Optimizer::PoseOptimization (Optimizer.cc:824-1118) on gfx950: motion-only BA,
// one 256-thread workgroup per frame, the whole schedule (4 rounds x optimize(10), g2o LM with
// its trial loop, chi2 re-classification, Huber dropped after round 3) inside one launch.
//
// Per frame: the pose (SE3Quat, FP64) and the LM scalars live in LDS; the observations
// (compacted on the host: MapPoint present) and their last errors live in HBM.  Each LM
// iteration is one pass over the active edges (error, robust weight, Jacobian, 6x6 normal
// equations reduced by wave butterflies in a fixed order) plus one error pass per trial;
// the 6x6 system is solved by one lane (LDL^T).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "se3_device.hpp"
#include "pose_types.hpp"

namespace slamhot {
namespace pose {

using lba::Quat;

constexpr int kThreads = 256;

__host__ __device__ constexpr int sym6(int r, int c) { return r * 6 - (r * (r - 1)) / 2 + (c - r); }

__device__ inline bool is_stereo(const PEdge& e) { return e.idx < 0; }

struct Hub {
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;
};

// computeError of EdgeSE3ProjectXYZOnlyPose (OptimizableTypes.h:41-45) /
// EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.h:218-222, .cpp:339-346: float invz,
// bf a double member), chi2, the Huber kernel and linearizeOplus as the reference's objects compute
// them (round 5: lba::map_cc / chi2_3_cc / huber_cc / mul23_cc, se3_device.hpp)
__device__ inline void perr(const PEdge& e, const double* P, const PFrame& F, double* err) {
    const double X[3] = {e.Xw[0], e.Xw[1], e.Xw[2]};
    double Xc[3];
    lba::map_cc(P, X, Xc);
    const double fx = F.fx, fy = F.fy, cx = F.cx, cy = F.cy;
    if (!is_stereo(e)) {
        err[0] = (double)e.obs[0] - (fx * Xc[0] / Xc[2] + cx);
        err[1] = (double)e.obs[1] - (fy * Xc[1] / Xc[2] + cy);
        err[2] = 0.0;
    } else {
        // cam_project as compiled (types_six_dof_expmap.cpp.o @0xc90)
        const double iz = (double)(float)(1.0 / Xc[2]);
        const double u = __builtin_fma(iz * Xc[0], fx, cx);
        const double v = __builtin_fma(iz * Xc[1], fy, cy);
        err[0] = (double)e.obs[0] - u;
        err[1] = (double)e.obs[1] - v;
        err[2] = (double)e.obs[2] - __builtin_fma(-iz, (double)F.bf, u);
    }
}

__device__ inline double pchi2(const PEdge& e, const double* err) {
    const double info = e.info;
    if (is_stereo(e)) return lba::chi2_3_cc(err, info);
    return err[0] * (info * err[0]) + err[1] * (info * err[1]);
}

__device__ inline void prob(const Hub& h, bool stereo, double c, double& r0, double& r1) {
    lba::huber_cc(c, stereo ? h.delta_stereo : h.delta_mono, stereo ? h.dsqr_stereo : h.dsqr_mono, r0, r1);
}

// linearizeOplus (OptimizableTypes.cpp:49-63 @0x1630; types_six_dof_expmap.cpp:375-404 @0x1280)
__device__ inline void pjac(const PEdge& e, const double* P, const PFrame& F, double* A) {
    const double X[3] = {e.Xw[0], e.Xw[1], e.Xw[2]};
    double Xc[3];
    lba::map_cc(P, X, Xc);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double fx = F.fx, fy = F.fy, bf = F.bf;
    if (!is_stereo(e)) {
        const double n[6] = {-(fx / z), -0.0, -((double)(-(float)fx) * x / (z * z)),
                             -0.0, -(fy / z), -((double)(-(float)fy) * y / (z * z))};
        const double S[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
        lba::mul23_cc<6>(n, S, A);
#pragma unroll
        for (int c = 0; c < 6; c++) A[12 + c] = 0;
    } else {
        const double invz = 1.0 / z, invz_2 = invz * invz;
        A[0] = y * x * invz_2 * fx;
        A[1] = -__builtin_fma(x * x, invz_2, 1.0) * fx;
        A[2] = y * invz * fx;
        A[3] = -invz * fx;
        A[4] = 0;
        A[5] = invz_2 * x * fx;
        A[6] = __builtin_fma(y * y, invz_2, 1.0) * fy;
        A[7] = -x * y * invz_2 * fy;
        A[8] = -x * invz * fy;
        A[9] = 0;
        A[10] = -invz * fy;
        A[11] = y * invz_2 * fy;
        A[12] = __builtin_fma(-(y * bf), invz_2, A[0]);
        A[13] = __builtin_fma(x * bf, invz_2, A[1]);
        A[14] = A[2];
        A[15] = A[3];
        A[16] = 0;
        A[17] = __builtin_fma(-invz_2, bf, A[5]);
    }
}

#ifndef SLAMHOT_POSE_SHFL
// wave sum by DPP (VALU; every lane of the wave active): row sums by row_ror 8 / 4 / 2 / 1, the
// rows combined by row_bcast:15 and row_bcast:31 into lane 63, read back as a uniform value.
// Fixed order ((r2 + r3) + (r0 + r1)); replaces six ds_bpermute round trips per double (the
// 28-value reduction of every LM step).  SLAMHOT_POSE_SHFL keeps the xor butterfly.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ inline double wsum(double v) {
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
__device__ inline double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
#endif

// unpivoted LDL^T of a 6x6 SPD matrix; fails on a negative pivot (Eigen LDLT::isPositive)
__device__ inline bool solve6(const double* M, const double* rhs, double* out) {
    double L[36], d[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double dj = M[6 * j + j];
#pragma unroll
        for (int k = 0; k < j; k++) dj -= L[6 * j + k] * L[6 * j + k] * d[k];
        if (dj < 0.0) return false;
        d[j] = dj;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double sacc = M[6 * i + j];
#pragma unroll
            for (int k = 0; k < j; k++) sacc -= L[6 * i + k] * L[6 * j + k] * d[k];
            L[6 * i + j] = sacc / dj;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        y[i] = rhs[i];
#pragma unroll
        for (int k = 0; k < i; k++) y[i] -= L[6 * i + k] * y[k];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] /= d[i];
#pragma unroll
    for (int i = 5; i >= 0; i--)
#pragma unroll
        for (int k = i + 1; k < 6; k++) y[i] -= L[6 * k + i] * y[k];
#pragma unroll
    for (int i = 0; i < 6; i++) out[i] = y[i];
    return true;
}

struct Shared {
    double est[8], trial[8], pose0[8];
    double H[36], b[6], x[6];
    double red[kThreads / 64][28];
    double lambda, ni, cur_chi, ini_chi;
    int nbad_lm, flag_continue, flag_ok2, nbad_obs, any_active;
};

// sum over the block of up to 28 per-thread values; result in sh.red[0][k] for k < nv
template <int NV>
__device__ inline void block_reduce(double (&v)[NV], Shared& sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        const double t = wsum(v[k]);
        if (lane == 0) sh.red[wid][k] = t;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double t = 0;
        for (int w = 0; w < kThreads / 64; w++) t += sh.red[w][threadIdx.x];
        sh.red[0][threadIdx.x] = t;  // each thread reads and writes only its own column
    }
    __syncthreads();
}

__global__ void __launch_bounds__(kThreads) k_pose_opt(const PFrame* __restrict__ frames,
                                                       const PEdge* __restrict__ edges, double* __restrict__ errs,
                                                       uint8_t* __restrict__ level, uint8_t* __restrict__ outlier,
                                                       POut* __restrict__ out, Hub hub) {
    __shared__ Shared sh;
    const PFrame& F = frames[blockIdx.x];  // by reference: F.Tcw[tid] below would put a copy in scratch
    const int tid = threadIdx.x;
    const int e0 = F.e0, ne = F.ne;
    if (tid == 0) {
        double R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = F.Tcw[4 * i + j];
        Quat q = lba::quat_from_R(R);  // Converter::toSE3Quat
        lba::normalize_rotation(q);
        sh.pose0[0] = q.x;
        sh.pose0[1] = q.y;
        sh.pose0[2] = q.z;
        sh.pose0[3] = q.w;
        sh.pose0[4] = F.Tcw[3];
        sh.pose0[5] = F.Tcw[7];
        sh.pose0[6] = F.Tcw[11];
        sh.pose0[7] = 0;
        for (int k = 0; k < 8; k++) sh.est[k] = sh.pose0[k];
    }
    for (int i = tid; i < ne; i += kThreads) {
        level[e0 + i] = 0;  // all inliers, robust kernel on (bit 1 = kernel removed)
        outlier[e0 + i] = 0;
    }
    __syncthreads();
    if (ne < 3) {  // nInitialCorrespondences < 3: return 0, pose untouched (Optimizer.cc:1012-1013)
        if (tid < 16) out[blockIdx.x].Tcw[tid] = F.Tcw[tid];
        if (tid == 0) out[blockIdx.x].n_inliers = 0;
        return;
    }
    int nbad_obs = 0;
    for (int round = 0; round < 4; round++) {
        if (tid == 0)
            for (int k = 0; k < 8; k++) sh.est[k] = sh.pose0[k];
        // initializeOptimization(0): active = level-0 edges; none -> optimize() does nothing
        {
            double v[1] = {0.0};
            for (int i = tid; i < ne; i += kThreads) v[0] += (level[e0 + i] & 1) ? 0.0 : 1.0;
            block_reduce<1>(v, sh);
        }
        const bool any = sh.red[0][0] > 0.0;
        __syncthreads();
        for (int it = 0; any && it < 10; it++) {
            // computeActiveErrors + activeRobustChi2 + buildSystem at the current estimate
            double acc[28];
#pragma unroll
            for (int k = 0; k < 28; k++) acc[k] = 0.0;
            for (int i = tid; i < ne; i += kThreads) {
                const uint8_t lv = level[e0 + i];
                if (lv & 1) continue;
                const PEdge e = edges[e0 + i];
                double err[3];
                perr(e, sh.est, F, err);
                double* ep = errs + 4 * (size_t)(e0 + i);
                ep[0] = err[0];
                ep[1] = err[1];
                ep[2] = err[2];
                const double c = pchi2(e, err);
                double r0 = c, r1 = 1.0;
                if (!(lv & 2)) prob(hub, is_stereo(e), c, r0, r1);
                acc[27] += r0;
                double A[18];
                pjac(e, sh.est, F, A);
                const double info = e.info, w = r1 * info;
#pragma unroll
                for (int cc = 0; cc < 6; cc++) {
                    double sacc = 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) sacc += A[6 * k + cc] * (info * err[k]);
                    acc[21 + cc] -= r1 * sacc;
                }
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int cc = r; cc < 6; cc++) {
                        double sacc = 0;
#pragma unroll
                        for (int k = 0; k < 3; k++) sacc += (A[6 * k + r] * w) * A[6 * k + cc];
                        acc[sym6(r, cc)] += sacc;
                    }
            }
            block_reduce<28>(acc, sh);
            if (tid == 0) {
                for (int r = 0; r < 6; r++)
                    for (int cc = r; cc < 6; cc++) sh.H[6 * r + cc] = sh.H[6 * cc + r] = sh.red[0][sym6(r, cc)];
                for (int cc = 0; cc < 6; cc++) sh.b[cc] = sh.red[0][21 + cc];
                sh.cur_chi = sh.red[0][27];
                sh.ini_chi = sh.cur_chi;
                if (it == 0) {  // computeLambdaInit (tau = 1e-5)
                    double m = 0;
                    for (int j = 0; j < 6; j++) m = fmax(fabs(sh.H[7 * j]), m);
                    sh.lambda = 1e-5 * m;
                    sh.ni = 2;
                    sh.nbad_lm = 0;
                }
            }
            __syncthreads();
            // trial loop (optimization_algorithm_levenberg.cpp:106-148)
            double rho = 0;
            int qmax = 0;
            for (;;) {
                if (tid == 0) {
                    double Hl[36];
                    for (int k = 0; k < 36; k++) Hl[k] = sh.H[k];
                    for (int j = 0; j < 6; j++) Hl[7 * j] += sh.lambda;
                    sh.flag_ok2 = solve6(Hl, sh.b, sh.x) ? 1 : 0;
                    lba::se3_exp_mul(sh.x, sh.est, sh.trial);
                }
                __syncthreads();
                double v[1] = {0.0};
                for (int i = tid; i < ne; i += kThreads) {
                    const uint8_t lv = level[e0 + i];
                    if (lv & 1) continue;
                    const PEdge e = edges[e0 + i];
                    double err[3];
                    perr(e, sh.trial, F, err);
                    double* ep = errs + 4 * (size_t)(e0 + i);
                    ep[0] = err[0];
                    ep[1] = err[1];
                    ep[2] = err[2];
                    const double c = pchi2(e, err);
                    double r0 = c, r1 = 1.0;
                    if (!(lv & 2)) prob(hub, is_stereo(e), c, r0, r1);
                    v[0] += r0;
                }
                block_reduce<1>(v, sh);
                if (tid == 0) {
                    double tempChi = sh.red[0][0];
                    if (!sh.flag_ok2) tempChi = __DBL_MAX__;
                    double r = sh.cur_chi - tempChi;
                    double scale = 0;
                    for (int j = 0; j < 6; j++) scale += sh.x[j] * (sh.lambda * sh.x[j] + sh.b[j]);
                    scale += 1e-3;
                    r /= scale;
                    if (r > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * r - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        sh.lambda *= fmax(1. / 3., alpha);
                        sh.ni = 2;
                        sh.cur_chi = tempChi;
                        for (int k = 0; k < 8; k++) sh.est[k] = sh.trial[k];
                    } else {
                        sh.lambda *= sh.ni;
                        sh.ni *= 2;
                    }
                    sh.red[0][1] = r;
                }
                __syncthreads();
                rho = sh.red[0][1];
                qmax++;
                __syncthreads();
                if (!(rho < 0 && qmax < 10)) break;
            }
            int stop = 0;
            if (qmax == 10 || rho == 0) {
                stop = 1;
            } else {
                if (tid == 0) {
                    if ((sh.ini_chi - sh.cur_chi) * 1e3 < sh.ini_chi)
                        sh.nbad_lm++;
                    else
                        sh.nbad_lm = 0;
                }
                __syncthreads();
                if (sh.nbad_lm >= 3) stop = 1;
            }
            __syncthreads();
            if (stop) break;
        }
        // classification (Optimizer.cc:1030-1101): chi2 as float against the float thresholds
        double v[1] = {0.0};
        for (int i = tid; i < ne; i += kThreads) {
            const PEdge e = edges[e0 + i];
            double* ep = errs + 4 * (size_t)(e0 + i);
            double err[3];
            if (outlier[e0 + i]) {
                perr(e, sh.est, F, err);
                ep[0] = err[0];
                ep[1] = err[1];
                ep[2] = err[2];
            } else {
                err[0] = ep[0];
                err[1] = ep[1];
                err[2] = ep[2];
            }
            const float chi2 = (float)pchi2(e, err);
            uint8_t lv = level[e0 + i];
            if (chi2 > (is_stereo(e) ? 7.815f : 5.991f)) {
                outlier[e0 + i] = 1;
                lv |= 1;
                v[0] += 1.0;
            } else {
                outlier[e0 + i] = 0;
                lv &= ~1;
            }
            if (round == 2) lv |= 2;  // setRobustKernel(0)
            level[e0 + i] = lv;
        }
        block_reduce<1>(v, sh);
        nbad_obs = (int)sh.red[0][0];
        __syncthreads();
        if (ne < 10) break;  // optimizer.edges().size() < 10
    }
    if (tid == 0) {
        double R[9];
        lba::rot_matrix(lba::load_q(sh.est), R);
        POut& o = out[blockIdx.x];
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) o.Tcw[4 * i + j] = (float)R[3 * i + j];
            o.Tcw[4 * i + 3] = (float)sh.est[4 + i];
        }
        o.Tcw[12] = o.Tcw[13] = o.Tcw[14] = 0.f;
        o.Tcw[15] = 1.f;
        o.n_inliers = ne - nbad_obs;
    }
}

Hub pose_hub() {
    Hub hub;
    const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);  // Optimizer.cc:852-853
    hub.delta_mono = deltaMono;
    hub.delta_stereo = deltaStereo;
    hub.dsqr_mono = (float)(hub.delta_mono * hub.delta_mono);
    hub.dsqr_stereo = (float)(hub.delta_stereo * hub.delta_stereo);
    return hub;
}

hipError_t launch_pose_opt(const PFrame* frames, const PEdge* edges, double* errs, uint8_t* level, uint8_t* outlier,
                           POut* out, int nframes, hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    k_pose_opt<<<nframes, kThreads, 0, s>>>(frames, edges, errs, level, outlier, out, pose_hub());
    return hipGetLastError();
}

}  // namespace pose
}  // namespace slamhot

using namespace slamhot;
using namespace slamhot::pose;

struct slam_pose_opt {
    int device = 0;
    hipStream_t stream = nullptr;
    void *d_frames = nullptr, *d_edges = nullptr, *d_errs = nullptr, *d_level = nullptr, *d_outl = nullptr,
         *d_out = nullptr;
    size_t cap_f = 0, cap_e = 0;
};

namespace {
void free_bufs(slam_pose_opt* h) {
    for (void** p : {&h->d_frames, &h->d_edges, &h->d_errs, &h->d_level, &h->d_outl, &h->d_out}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    h->cap_f = h->cap_e = 0;
}
}  // namespace

extern "C" {

slam_status slamhot_pose_opt_create(int device, slam_pose_opt** out) {
    if (!out) return SLAM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= n) return SLAM_EINVAL;
    slam_pose_opt* h = new (std::nothrow) slam_pose_opt();
    if (!h) return SLAM_ENOMEM;
    h->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return SLAM_EHIP;
    }
    *out = h;
    return SLAM_OK;
}

void slamhot_pose_opt_destroy(slam_pose_opt* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_bufs(h);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

slam_status slamhot_pose_optimization(slam_pose_opt* h, int nframes, const slam_pose_frame* frames,
                                      slam_pose_result* results) {
    if (!h || nframes < 0 || (nframes && (!frames || !results))) return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    std::vector<PFrame> pf(nframes);
    std::vector<PEdge> pe;
    for (int f = 0; f < nframes; f++) {
        const slam_pose_frame& F = frames[f];
        if (F.n < 0 || (F.n && (!F.kps_un || !F.uright || !F.has_mp || !F.mp_pos || !F.inv_sigma2)) ||
            (F.n && !results[f].outlier))
            return SLAM_EINVAL;
        PFrame& P = pf[f];
        std::memcpy(P.Tcw, F.Tcw, sizeof(P.Tcw));
        P.fx = F.cam.fx;
        P.fy = F.cam.fy;
        P.cx = F.cam.cx;
        P.cy = F.cam.cy;
        P.bf = F.cam.bf;
        P.e0 = (int)pe.size();
        for (int i = 0; i < F.n; i++) {
            if (!F.has_mp[i]) continue;
            const int oct = F.kps_un[i].octave;
            if (oct < 0 || oct >= F.nlevels) return SLAM_EINVAL;
            PEdge e;
            const bool stereo = !(F.uright[i] < 0);
            e.obs[0] = F.kps_un[i].x;
            e.obs[1] = F.kps_un[i].y;
            e.obs[2] = stereo ? F.uright[i] : 0.f;
            e.info = F.inv_sigma2[oct];
            e.Xw[0] = F.mp_pos[3 * i];
            e.Xw[1] = F.mp_pos[3 * i + 1];
            e.Xw[2] = F.mp_pos[3 * i + 2];
            e.idx = stereo ? (int)(i | 0x80000000u) : i;
            pe.push_back(e);
        }
        P.ne = (int)pe.size() - P.e0;
    }
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const size_t ne = std::max<size_t>(pe.size(), 1);
    if ((size_t)nframes > h->cap_f || ne > h->cap_e) {
        SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
        free_bufs(h);
        const size_t cf = std::max<size_t>(nframes, 64), ce = std::max<size_t>(ne, 4096);
        SLAM_HIP_TRY(hipMalloc(&h->d_frames, cf * sizeof(PFrame)));
        SLAM_HIP_TRY(hipMalloc(&h->d_out, cf * sizeof(POut)));
        SLAM_HIP_TRY(hipMalloc(&h->d_edges, ce * sizeof(PEdge)));
        SLAM_HIP_TRY(hipMalloc(&h->d_errs, ce * 4 * sizeof(double)));
        SLAM_HIP_TRY(hipMalloc(&h->d_level, ce));
        SLAM_HIP_TRY(hipMalloc(&h->d_outl, ce));
        h->cap_f = cf;
        h->cap_e = ce;
    }
    hipStream_t S = h->stream;
    SLAM_HIP_TRY(hipMemcpyAsync(h->d_frames, pf.data(), nframes * sizeof(PFrame), hipMemcpyHostToDevice, S));
    if (!pe.empty())
        SLAM_HIP_TRY(hipMemcpyAsync(h->d_edges, pe.data(), pe.size() * sizeof(PEdge), hipMemcpyHostToDevice, S));
    SLAM_HIP_TRY(launch_pose_opt((const PFrame*)h->d_frames, (const PEdge*)h->d_edges, (double*)h->d_errs,
                                 (uint8_t*)h->d_level, (uint8_t*)h->d_outl, (POut*)h->d_out, nframes, S));
    std::vector<POut> po(nframes);
    std::vector<uint8_t> outl(pe.size());
    SLAM_HIP_TRY(hipMemcpyAsync(po.data(), h->d_out, nframes * sizeof(POut), hipMemcpyDeviceToHost, S));
    if (!pe.empty())
        SLAM_HIP_TRY(hipMemcpyAsync(outl.data(), h->d_outl, pe.size(), hipMemcpyDeviceToHost, S));
    SLAM_HIP_TRY(hipStreamSynchronize(S));
    for (int f = 0; f < nframes; f++) {
        const slam_pose_frame& F = frames[f];
        slam_pose_result& R = results[f];
        std::memcpy(R.Tcw, po[f].Tcw, sizeof(R.Tcw));
        R.n_initial = pf[f].ne;
        R.n_inliers = po[f].n_inliers;
        int k = pf[f].e0;
        for (int i = 0; i < F.n; i++)
            if (F.has_mp[i]) R.outlier[i] = outl[k++];
    }
    return SLAM_OK;
}

}  // extern "C"
