// track.hip — the per-sequence stereo tracking chain, device-resident (BASELINE.json configs[4]:
// one sequence per GPU; here S sequences advance in lock-step on one GPU so the batched case
// fills the chip).  One step = one stereo frame per sequence:
//
//   cv::remap x2 -> ORBextractor x2 -> Frame::ComputeStereoMatches ->
//   TrackWithMotionModel when a velocity exists (UpdateLastFrame, SearchByProjection(F,
//   LastFrame, 7), retry at 14 below 20 matches, PoseOptimization, >= 10 inliers), else or on
//   its failure TrackReferenceKeyFrame (ComputeBoW + SearchByBoW(reference KF, F),
//   PoseOptimization) -> SearchLocalPoints (isInFrustum + SearchByProjection over the reference
//   KeyFrame's MapPoints) -> PoseOptimization -> motion model update -> NeedNewKeyFrame /
//   CreateNewKeyFrame   (Tracking.cc:1256-3330; tests/track_oracle.py)
//
// Every decision (initialisation, lost, keyframe insertion) is taken on the device: the host
// only enqueues the same launches every step and never waits, so a sequence advances at the
// rate of its kernels.  The reused stages are the library's own kernels (extractor, stereo,
// batched BoW matcher, k_pose_opt, k_is_in_frustum, k_search_by_projection); the glue here is
// one workgroup per sequence: edge packing for PoseOptimization (order-preserving block
// compaction), outlier removal, the Frame grid (Frame::AssignFeaturesToGrid as a sort of
// (cell, index) keys in LDS), the SearchLocalPoints records, and KeyFrame creation (a bitonic
// sort of (depth, index) keys in LDS for CreateNewKeyFrame's depth order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "pose_types.hpp"
#include "projection.hpp"

namespace slamhot {
namespace track {

constexpr int kMaxCap = 4096;   // LDS sorts below hold one key per feature slot
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kT = 1024;        // glue workgroup size

struct Params {
    float fx, fy, cx, cy, bf, b, th_depth, invfx, invfy, log_scale;
    float min_x, max_x, min_y, max_y, grid_inv_w, grid_inv_h;
    float scale[16], inv_sigma2[16];
    int nlevels, cap, S;
};

struct Seq {  // per-sequence state, device resident
    float Tcw[16];      // mLastFrame.mTcw (the last tracked frame's pose)
    float T1[16];       // pose after TrackWithMotionModel / TrackReferenceKeyFrame
    float V[16];        // mVelocity (valid when has_vel)
    float Tlr[16];      // mlRelativeFramePoses.back(): the last frame relative to its reference KF
    float Tref[16];     // the reference KeyFrame's pose (KeyFrame::GetPose)
    float Tlast[16];    // mLastFrame.mTcw as this step uses it (UpdateLastFrame: Tlr * Tref)
    float Tpred[16];    // mVelocity * mLastFrame.mTcw
    int initialized, cur, n_ref, active;
    int has_vel, nkf, mode, last_n;  // mode 1: this step's first pose came from the motion model
    int motion_try, motion_n, fail, pad;
};

struct Rec {  // what one step reports per sequence (slam_track_record)
    float Tcw[16];
    int n, n_stereo, n_bow, n_inl_ref, n_local, n_inl, is_kf, lost, initialized, n_motion, motion, status;
};

struct MapPts {  // the reference KeyFrame's MapPoint slots, one per KF feature (x2: double buffer)
    float4* pos;     // xyz, valid in w (1 / 0)
    float4* normal;
    float2* dist;    // mfMinDistance, mfMaxDistance
    uint8_t* desc;   // 32 B
};

struct Bufs {
    Params P;
    Seq* seq;
    Rec* rec;
    slam_keypoint* kps;   // 2S x cap: [0, S) frames, [S, 2S) reference KeyFrames
    uint8_t* desc;        // 2S x cap x 32
    int32_t* n;           // 2S
    uint8_t* valid;       // 2S x cap (KF MapPoint present; the BoW matcher's d_valid)
    const float* ur;      // S x cap (mvuRight)
    const float* depth;   // S x cap (mvDepth)
    const int32_t* b2a;   // S x cap: F feature -> KF feature (SearchByBoW)
    const int32_t* nbow;  // S
    int32_t* fmp;         // S x cap: F feature -> KF MapPoint slot (-1 none)
    MapPts mp[2];
    pose::PFrame* pf;
    pose::PEdge* pe;      // S x cap
    const pose::POut* po;
    const uint8_t* outl;  // S x cap (per edge)
    slam_mp_geom* geom;   // S x cap
    slam_mp_track* track; // S x cap
    int32_t* n_in_view;   // S
    int8_t* fstate;       // S x cap
    int32_t* cell_start;  // S x (kGridCells + 1)
    int32_t* cell_feat;   // S x cap
    FrustumCall* fcalls;
    DevProjCall* pcalls;
    ProjQuery* queries;   // S x cap
    int32_t* cand_off;    // S x (cap + 1)
    uint32_t* cand;       // S x cand_cap
    int cand_cap;
    int32_t* fmatch;      // S x cap
    int32_t* pout;        // S x 4
    // TrackWithMotionModel: the last frame, its SearchByProjection query arrays, two attempts
    slam_keypoint* lf_kps;  // S x cap: mLastFrame.mvKeysUn
    int32_t* lf_fmp;        // S x cap: mLastFrame.mvpMapPoints as MapPoint slots of the current map
    uint8_t* lf_has;        // S x cap
    uint8_t* lf_zero;       // S x cap, 0: mvbOutlier (outliers left the frame, Tracking.cc:2105-2109)
    uint8_t* lf_one;        // S x cap, 1: Observations() > 0
    float* lf_pos;          // S x cap x 3
    uint8_t* lf_desc;       // S x cap x 32
    const int8_t* fclear;   // S x cap, -1: mvpMapPoints cleared before the search (Tracking.cc:2704)
    DevProjCall* mcalls;    // 2S: th = 7, then 2 th for the sequences below 20 matches
    int32_t* mmatch;        // 2 x S x cap
    int32_t* mout;          // 2 x S x 4
    int32_t* motm;          // S x cap: the motion model's matches (MapPoint slot per feature)
};

__device__ inline size_t slot(const Params& P, int s) { return (size_t)s * P.cap; }

// mOw = -mRcw.t() * mtcw: cv::Mat product, double accumulation rounded once (as the matchers)
__device__ inline void camera_center(const float* T, float* Ow) {
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[i] * (double)T[3] + (double)T[4 + i] * (double)T[7] + (double)T[8 + i] * (double)T[11];
        Ow[i] = (float)(-1.0 * acc);
    }
}

// 4x4 float cv::Mat product (cv::gemm on CV_32F accumulates in double, one rounding per entry,
// DESIGN.md §1 deviation 3): C = A * B, row-major
__device__ inline void gemm4(const float* A, const float* B, float* C) {
    float o[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double acc = 0.0;
            for (int k = 0; k < 4; k++) acc += (double)A[4 * i + k] * (double)B[4 * k + j];
            o[4 * i + j] = (float)acc;
        }
    for (int k = 0; k < 16; k++) C[k] = o[k];
}

// the inverse pose Twc as Frame::UpdatePoseMatrices / KeyFrame::SetPose form it: Rwc = Rcw^T,
// Ow = -Rcw^T tcw, last row (0, 0, 0, 1)
__device__ inline void pose_inverse(const float* T, float* Twc) {
    float Ow[3];
    camera_center(T, Ow);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Twc[4 * r + c] = T[4 * c + r];
        Twc[4 * r + 3] = Ow[r];
    }
    Twc[12] = Twc[13] = Twc[14] = 0.f;
    Twc[15] = 1.f;
}

// order-preserving compaction helper: exclusive prefix of `flag` over the block (chunked)
__device__ inline int block_excl(int flag, int* scratch, int* total) {
    const int incl = block_scan_incl(flag, scratch, total);
    return incl - flag;
}

// PoseOptimization input of sequence s: one edge per frame feature with a MapPoint, in feature
// order (Optimizer.cc:881-978 adds them in that order); Tcw = the pose the optimization starts from.
__device__ void pack_edges(const Bufs& B, int s, const float* Tcw, bool active, int* scratch) {
    const Params& P = B.P;
    const int n = B.n[s], cur = B.seq[s].cur;
    const MapPts& M = B.mp[cur];
    const size_t o = slot(P, s);
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += kT) {
        const int i = c0 + threadIdx.x;
        const int j = (active && i < n) ? B.fmp[o + i] : -1;
        int tot;
        const int pos = block_excl(j >= 0 ? 1 : 0, scratch, &tot);
        if (j >= 0) {
            const slam_keypoint kp = B.kps[o + i];
            const float ur = B.ur[o + i];
            const bool stereo = !(ur < 0);
            pose::PEdge e;
            e.obs[0] = kp.x;
            e.obs[1] = kp.y;
            e.obs[2] = stereo ? ur : 0.f;
            e.info = P.inv_sigma2[min(max(kp.octave, 0), P.nlevels - 1)];
            const float4 X = M.pos[slot(P, s) + j];
            e.Xw[0] = X.x;
            e.Xw[1] = X.y;
            e.Xw[2] = X.z;
            e.idx = stereo ? (int)((unsigned)i | 0x80000000u) : i;
            B.pe[o + base + pos] = e;
        }
        base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pose::PFrame F;
        for (int k = 0; k < 16; k++) F.Tcw[k] = Tcw[k];
        F.fx = P.fx;
        F.fy = P.fy;
        F.cx = P.cx;
        F.cy = P.cy;
        F.bf = P.bf;
        F.e0 = (int)o;
        F.ne = base;
        B.pf[s] = F;
    }
}

// drop the optimization's outliers from the frame (mvpMapPoints[i] = NULL); returns the count kept
__device__ int drop_outliers(const Bufs& B, int s, int* scratch) {
    const Params& P = B.P;
    const size_t o = slot(P, s);
    const int ne = B.pf[s].ne;
    for (int k = threadIdx.x; k < ne; k += kT)
        if (B.outl[o + k]) B.fmp[o + (B.pe[o + k].idx & 0x7fffffff)] = -1;
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < B.n[s]; i += kT) cnt += B.fmp[o + i] >= 0;
    return block_reduce_sum(cnt, scratch);
}

// Frame::AssignFeaturesToGrid (Frame.cc:380-411) as CSR over cells [ix][iy]: (cell, index) keys
// sorted in LDS (keys are unique, so the order inside a cell is the insertion order)
__device__ void build_grid(const Bufs& B, int s, uint32_t* keys) {
    const Params& P = B.P;
    const size_t o = slot(P, s);
    const int n = B.n[s];
    int npad = 1;
    while (npad < n) npad <<= 1;
    for (int i = threadIdx.x; i < npad; i += kT) {
        uint32_t k = 0xFFFFFFFFu;
        if (i < n) {
            const slam_keypoint kp = B.kps[o + i];
            const int px = (int)roundf((kp.x - P.min_x) * P.grid_inv_w);
            const int py = (int)roundf((kp.y - P.min_y) * P.grid_inv_h);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows)
                k = ((uint32_t)(px * kGridRows + py) << 16) | (uint32_t)i;
        }
        keys[i] = k;
    }
    __syncthreads();
    for (int kk = 2; kk <= npad; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < npad; i += kT) {
                const int l = i ^ j;
                if (l > i) {
                    const uint32_t a = keys[i], b = keys[l];
                    const bool up = (i & kk) == 0;
                    if ((a > b) == up) {
                        keys[i] = b;
                        keys[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    int32_t* cs = B.cell_start + (size_t)s * (kGridCells + 1);
    for (int c = threadIdx.x; c <= kGridCells; c += kT) {  // lower_bound(c << 16)
        int lo = 0, hi = npad;
        const uint32_t key = (uint32_t)c << 16;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (keys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        cs[c] = lo;
    }
    for (int i = threadIdx.x; i < n; i += kT)
        if (keys[i] != 0xFFFFFFFFu) B.cell_feat[o + i] = (int32_t)(keys[i] & 0xFFFFu);
    __syncthreads();
}

// ---------------------------------------------------------------- step kernels
// TrackWithMotionModel setup (Tracking.cc:2683-2718), after extraction + stereo + BoW: the frame
// grid, UpdateLastFrame (mLastFrame.SetPose(Tlr * pRef->GetPose()), :2619-2627), the predicted
// pose mVelocity * mLastFrame.mTcw, the last frame's MapPoints as SearchByProjection queries and
// the call records of both attempts (th = 7 stereo, ORBmatcher(0.9, true)).
__global__ void __launch_bounds__(kT) k_motion_setup(Bufs B) {
    __shared__ uint32_t keys[kMaxCap];
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    if (Q.initialized) build_grid(B, s, keys);  // Frame::AssignFeaturesToGrid of the current frame
    const bool try_m = Q.initialized && Q.has_vel;
    const int nq = try_m ? Q.last_n : 0;
    const MapPts& M = B.mp[Q.cur];
    for (int i = threadIdx.x; i < nq; i += kT) {
        const int j = B.lf_fmp[o + i];
        const float4 X = j >= 0 ? M.pos[o + j] : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool has = j >= 0 && X.w != 0.f;
        B.lf_has[o + i] = has;
        B.lf_pos[3 * (o + i)] = X.x;
        B.lf_pos[3 * (o + i) + 1] = X.y;
        B.lf_pos[3 * (o + i) + 2] = X.z;
        uint4* d = reinterpret_cast<uint4*>(B.lf_desc + (o + i) * 32);
        if (has) {
            const uint4* ms = reinterpret_cast<const uint4*>(M.desc + (o + j) * 32);
            d[0] = ms[0];
            d[1] = ms[1];
        }
    }
    if (threadIdx.x != 0) return;
    if (try_m) {
        gemm4(Q.Tlr, Q.Tref, Q.Tlast);   // UpdateLastFrame
        gemm4(Q.V, Q.Tlast, Q.Tpred);    // mCurrentFrame.SetPose(mVelocity * mLastFrame.mTcw)
    } else {
        for (int k = 0; k < 16; k++) Q.Tlast[k] = Q.Tcw[k];
    }
    Q.motion_try = try_m;
    Q.motion_n = 0;
    Q.mode = 0;
    Q.fail = 0;
    for (int a = 0; a < 2; a++) {
        DevProjCall C{};
        DevProjFrame& F = C.F;
        F.n = B.n[s];
        F.kps = B.kps + o;
        F.uright = B.ur + o;
        F.desc = B.desc + o * 32;
        F.state = B.fclear + o;
        F.cell_start = B.cell_start + (size_t)s * (kGridCells + 1);
        F.cell_feat = B.cell_feat + o;
        F.min_x = P.min_x;
        F.min_y = P.min_y;
        F.max_x = P.max_x;
        F.max_y = P.max_y;
        F.inv_w = P.grid_inv_w;
        F.inv_h = P.grid_inv_h;
        F.fx = P.fx;
        F.fy = P.fy;
        F.cx = P.cx;
        F.cy = P.cy;
        F.bf = P.bf;
        F.b = P.b;
        for (int k = 0; k < 16; k++) {
            F.T[k] = Q.Tpred[k];
            C.LT[k] = Q.Tlast[k];
            F.scale[k] = k < P.nlevels ? P.scale[k] : 1.f;
        }
        F.nlevels = P.nlevels;
        C.mode = kProjLast;
        C.nq = a == 0 ? nq : 0;  // the retry's count is set by k_motion_retry
        C.th = a == 0 ? 7.0f : 14.0f;  // Tracking.cc:2710-2714, 2722
        C.mono = 0;
        C.nnratio = 0.9f;
        C.th_dist = 100;  // TH_HIGH
        C.check_ori = 1;
        C.lf_kps = B.lf_kps + o;
        C.lf_kps_un = B.lf_kps + o;  // rectified stereo: mvKeysUn == mvKeys
        C.lf_has_mp = B.lf_has + o;
        C.lf_outlier = B.lf_zero + o;
        C.lf_pos = B.lf_pos + 3 * o;
        C.lf_has_obs = B.lf_one + o;
        C.queries = B.queries + o;
        C.qdesc = B.lf_desc + o * 32;
        C.cand_off = B.cand_off + (size_t)s * (P.cap + 1);
        C.cand = B.cand + (size_t)s * B.cand_cap;
        C.cand_cap = B.cand_cap;
        C.f_match = B.mmatch + (size_t)a * P.S * P.cap + o;
        C.out = B.mout + 4 * ((size_t)a * P.S + s);
        C.gstate = nullptr;
        for (int k = 0; k < 4; k++) C.out[k] = 0;
        B.mcalls[(size_t)a * P.S + s] = C;
    }
}

// "If few matches, uses a wider window search" (Tracking.cc:2718-2724): the second attempt runs
// for the sequences whose first one found fewer than 20 matches
__global__ void k_motion_retry(Bufs B) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B.P.S) return;
    const Seq& Q = B.seq[s];
    const int32_t* out = B.mout + 4 * s;
    B.mcalls[B.P.S + s].nq = (Q.motion_try && out[1] == 0 && out[0] < 20) ? Q.last_n : 0;
}

// the motion model's matches join the frame (MapPoint of the matched last-frame feature) and the
// PoseOptimization input from the predicted pose (Tracking.cc:2726-2735)
__global__ void __launch_bounds__(kT) k_motion_edges(Bufs B) {
    __shared__ int scratch[20];
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    const int32_t* o0 = B.mout + 4 * s;
    const int32_t* o1 = B.mout + 4 * ((size_t)P.S + s);
    const bool retry = Q.motion_try && o0[1] == 0 && o0[0] < 20;
    const bool overflow = Q.motion_try && (o0[1] == 1 || (retry && o1[1] == 1));
    const int nm = !Q.motion_try ? 0 : retry ? o1[0] : o0[0];
    const bool use = Q.motion_try && !overflow && nm >= 20;
    const int32_t* fm = B.mmatch + (retry ? (size_t)P.S * P.cap : 0) + o;
    for (int i = threadIdx.x; i < B.n[s]; i += kT) {
        const int q = use ? fm[i] : -1;
        const int j = q >= 0 ? B.lf_fmp[o + q] : -1;
        B.fmp[o + i] = j;
        B.motm[o + i] = Q.motion_try ? j : -1;
    }
    __syncthreads();
    pack_edges(B, s, Q.Tpred, use, scratch);
    if (threadIdx.x == 0) {
        Q.motion_n = nm;
        if (overflow) Q.fail = 1;
    }
}

// TrackWithMotionModel's end (outliers out, nmatchesMap >= 10, Tracking.cc:2736-2775); where it
// was not tried or failed, TrackReferenceKeyFrame (Tracking.cc:2559-2616): SearchByBoW's matches
// (< 15: lost) -> PoseOptimization input from mLastFrame.mTcw
__global__ void __launch_bounds__(kT) k_ref_edges(Bufs B) {
    __shared__ int scratch[20];
    __shared__ int s_ok;
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    const bool tried = Q.motion_try && Q.motion_n >= 20 && !Q.fail;
    int kept = 0;
    if (tried) kept = drop_outliers(B, s, scratch);  // the motion model's PoseOptimization
    if (threadIdx.x == 0) {
        s_ok = tried && kept >= 10;
        if (s_ok)
            for (int k = 0; k < 16; k++) Q.T1[k] = B.po[s].Tcw[k];
    }
    __syncthreads();
    const bool motion_ok = s_ok;
    const bool active = motion_ok || (Q.initialized && B.nbow[s] >= 15);  // Tracking.cc:2571-2575
    if (!motion_ok)
        for (int i = threadIdx.x; i < B.n[s]; i += kT) B.fmp[o + i] = active ? B.b2a[o + i] : -1;
    __syncthreads();
    pack_edges(B, s, Q.Tlast, active && !motion_ok, scratch);  // mCurrentFrame.SetPose(mLastFrame.mTcw)
    if (threadIdx.x == 0) {
        Q.active = active;
        Q.mode = motion_ok;
        Rec& R = B.rec[s];
        R.n = B.n[s];
        R.n_bow = Q.initialized && !motion_ok ? B.nbow[s] : 0;
        R.n_motion = Q.motion_n;
        R.motion = motion_ok;
        R.n_inl_ref = motion_ok ? kept : 0;
        R.n_local = R.n_inl = 0;
        R.is_kf = 0;
        R.lost = Q.initialized && !active;
        R.initialized = Q.initialized;
        R.status = 0;
    }
}

// after the first PoseOptimization: outliers out (TrackReferenceKeyFrame, :2586-2616); the
// SearchLocalPoints inputs (Tracking.cc:3179-3258): MapPoint records, grid, call records
__global__ void __launch_bounds__(kT) k_local_setup(Bufs B) {
    __shared__ int scratch[20];
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    bool active = Q.active;
    const bool motion = Q.mode == 1;  // the motion model's pose and inliers stand (k_ref_edges)
    const int kept = drop_outliers(B, s, scratch);  // TrackReferenceKeyFrame's PoseOptimization
    if (active && !motion && kept < 10) active = false;  // nmatchesMap >= 10 (:2616)
    const pose::POut& po = B.po[s];
    if (threadIdx.x < 16 && !motion) Q.T1[threadIdx.x] = active ? po.Tcw[threadIdx.x] : Q.Tcw[threadIdx.x];
    const int kfn = active ? B.n[P.S + s] : 0;
    const MapPts& M = B.mp[Q.cur];
    // local MapPoint records: the reference KeyFrame's slots; "seen" = already in the frame
    for (int j = threadIdx.x; j < kfn; j += kT) {
        slam_mp_geom g;
        const float4 X = M.pos[o + j], N = M.normal[o + j];
        const float2 d = M.dist[o + j];
        g.pos[0] = X.x;
        g.pos[1] = X.y;
        g.pos[2] = X.z;
        g.normal[0] = N.x;
        g.normal[1] = N.y;
        g.normal[2] = N.z;
        g.min_dist = d.x;
        g.max_dist = d.y;
        g.seen = 0;
        g.is_bad = X.w == 0.f;
        g.has_obs = 1;
        g.pad = 0;
        B.geom[o + j] = g;
    }
    __syncthreads();
    const int n = active ? B.n[s] : 0;
    for (int i = threadIdx.x; i < B.n[s]; i += kT) {
        const int j = B.fmp[o + i];
        B.fstate[o + i] = j >= 0 ? 1 : -1;
        if (j >= 0) B.geom[o + j].seen = 1;
        if (!active) B.fmatch[o + i] = -1;  // no SearchLocalPoints this step (the launch covers F.n = 0)
    }
    if (threadIdx.x == 0) {
        Q.active = active;
        B.rec[s].n_inl_ref = active ? kept : 0;
        if (Q.initialized && !active) B.rec[s].lost = 1;
        B.n_in_view[s] = 0;
        B.pout[4 * s] = B.pout[4 * s + 1] = B.pout[4 * s + 2] = B.pout[4 * s + 3] = 0;
        const float* T = Q.T1;
        FrustumCall Fc{};
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) Fc.R[3 * r + c] = T[4 * r + c];
            Fc.t[r] = T[4 * r + 3];
        }
        camera_center(T, Fc.Ow);
        Fc.min_x = P.min_x;
        Fc.max_x = P.max_x;
        Fc.min_y = P.min_y;
        Fc.max_y = P.max_y;
        Fc.fx = P.fx;
        Fc.fy = P.fy;
        Fc.cx = P.cx;
        Fc.cy = P.cy;
        Fc.bf = P.bf;
        Fc.log_scale = P.log_scale;
        Fc.view_cos_limit = 0.5f;  // Tracking.cc:3222
        Fc.nlevels = P.nlevels;
        Fc.n = kfn;
        Fc.mps = B.geom + o;
        Fc.track = B.track + o;
        Fc.n_in_view = B.n_in_view + s;
        B.fcalls[s] = Fc;
        DevProjCall C{};
        DevProjFrame& F = C.F;
        F.n = n;
        F.kps = B.kps + o;
        F.uright = B.ur + o;
        F.desc = B.desc + o * 32;
        F.state = B.fstate + o;
        F.cell_start = B.cell_start + (size_t)s * (kGridCells + 1);
        F.cell_feat = B.cell_feat + o;
        F.min_x = P.min_x;
        F.min_y = P.min_y;
        F.max_x = P.max_x;
        F.max_y = P.max_y;
        F.inv_w = P.grid_inv_w;
        F.inv_h = P.grid_inv_h;
        F.fx = P.fx;
        F.fy = P.fy;
        F.cx = P.cx;
        F.cy = P.cy;
        F.bf = P.bf;
        F.b = P.b;
        for (int k = 0; k < 16; k++) {
            F.T[k] = T[k];
            F.scale[k] = k < P.nlevels ? P.scale[k] : 1.f;
        }
        F.nlevels = P.nlevels;
        C.mode = kProjLocal;
        C.nq = kfn;
        C.mps = B.track + o;
        C.th = 1.0f;  // Tracking.cc:3237 (stereo)
        C.th_far = 50.0f;
        C.far_points = 0;
        C.nnratio = 0.8f;
        C.th_dist = 100;
        C.check_ori = 0;
        C.queries = B.queries + o;
        C.qdesc = M.desc + o * 32;
        C.cand_off = B.cand_off + (size_t)s * (P.cap + 1);
        C.cand = B.cand + (size_t)s * B.cand_cap;
        C.cand_cap = B.cand_cap;
        C.f_match = B.fmatch + o;
        C.out = B.pout + 4 * s;
        C.gstate = nullptr;
        B.pcalls[s] = C;
    }
}

// after SearchLocalPoints: its matches join the frame; the second PoseOptimization input
__global__ void __launch_bounds__(kT) k_local_edges(Bufs B) {
    __shared__ int scratch[20];
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    const bool active = Q.active;
    if (active)
        for (int i = threadIdx.x; i < B.n[s]; i += kT) {
            const int m = B.fmatch[o + i];
            if (m >= 0) B.fmp[o + i] = m;
        }
    __syncthreads();
    pack_edges(B, s, Q.T1, active, scratch);
    if (threadIdx.x == 0) {
        B.rec[s].n_local = active ? B.pout[4 * s] : 0;
        if (active && B.pout[4 * s + 1] == 1) Q.fail = 1;  // candidate overflow: matches incomplete
    }
}

// Frame::UnprojectStereo (Frame.cc:1006-1022): mRwc * x3Dc + mOw as one cv::gemm with beta
__device__ inline float4 unproject(const Params& P, const float* T, const float* Ow, slam_keypoint kp, float z) {
    const float x = (kp.x - P.cx) * z * P.invfx;
    const float y = (kp.y - P.cy) * z * P.invfy;
    float out[3];
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[i] * (double)x + (double)T[4 + i] * (double)y + (double)T[8 + i] * (double)z;
        out[i] = (float)(acc * 1.0 + (double)Ow[i] * 1.0);
    }
    return make_float4(out[0], out[1], out[2], 1.f);
}

// a new MapPoint's normal and scale range: MapPoint::UpdateNormalAndDepth with one observation
__device__ inline void mp_geometry(const Params& P, float4 X, const float* Ow, int octave, float4& normal,
                                   float2& dist) {
    const float pc[3] = {X.x - Ow[0], X.y - Ow[1], X.z - Ow[2]};
    const double nd = sqrt((double)pc[0] * (double)pc[0] + (double)pc[1] * (double)pc[1] + (double)pc[2] * (double)pc[2]);
    const float d = (float)nd;
    normal = make_float4((float)((double)pc[0] / nd), (float)((double)pc[1] / nd), (float)((double)pc[2] / nd), 0.f);
    const float maxd = d * P.scale[min(max(octave, 0), P.nlevels - 1)];
    dist = make_float2(maxd / P.scale[P.nlevels - 1], maxd);
}

// the frame becomes the reference KeyFrame: features copied to the KF slot, tracked MapPoints
// kept, new ones from stereo depth — all (StereoInitialization) or in (depth, index) order until
// depth > mThDepth with more than 100 points (CreateNewKeyFrame, Tracking.cc:3268-3318)
__device__ void make_keyframe(const Bufs& B, int s, const float* T, bool initial, uint64_t* keys, int* scratch) {
    const Params& P = B.P;
    const size_t o = slot(P, s), okf = slot(P, P.S + s);
    Seq& Q = B.seq[s];
    const int n = B.n[s];
    const MapPts& Mo = B.mp[Q.cur];
    const MapPts& Mn = B.mp[1 - Q.cur];
    float Ow[3];
    camera_center(T, Ow);
    for (int i = threadIdx.x; i < n; i += kT) {
        B.kps[okf + i] = B.kps[o + i];
        const uint4* sd = reinterpret_cast<const uint4*>(B.desc + (o + i) * 32);
        uint4* dd = reinterpret_cast<uint4*>(B.desc + (okf + i) * 32);
        dd[0] = sd[0];
        dd[1] = sd[1];
        const int j = initial ? -1 : B.fmp[o + i];
        if (j >= 0) {
            Mn.pos[o + i] = Mo.pos[o + j];
            Mn.normal[o + i] = Mo.normal[o + j];
            Mn.dist[o + i] = Mo.dist[o + j];
            const uint4* ms = reinterpret_cast<const uint4*>(Mo.desc + (o + j) * 32);
            uint4* md = reinterpret_cast<uint4*>(Mn.desc + (o + i) * 32);
            md[0] = ms[0];
            md[1] = ms[1];
        } else {
            Mn.pos[o + i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    // depth order: (depth bits, index) keys, depth > 0 only (positive floats order as integers)
    int npad = 1;
    while (npad < n) npad <<= 1;
    for (int i = threadIdx.x; i < npad; i += kT) {
        uint64_t k = ~0ull;
        if (i < n) {
            const float z = B.depth[o + i];
            if (z > 0) k = ((uint64_t)__float_as_uint(z) << 32) | (uint32_t)i;
        }
        keys[i] = k;
    }
    __syncthreads();
    if (!initial) {
        for (int kk = 2; kk <= npad; kk <<= 1)
            for (int j = kk >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < npad; i += kT) {
                    const int l = i ^ j;
                    if (l > i) {
                        const uint64_t a = keys[i], b = keys[l];
                        const bool up = (i & kk) == 0;
                        if ((a > b) == up) {
                            keys[i] = b;
                            keys[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
    }
    // CreateNewKeyFrame's loop stops after the first position p >= 100 with depth > mThDepth
    __shared__ int s_stop;
    if (threadIdx.x == 0) s_stop = 0x7fffffff;
    __syncthreads();
    if (!initial)
        for (int p = threadIdx.x; p < npad; p += kT)
            if (keys[p] != ~0ull && p >= 100 && __uint_as_float((uint32_t)(keys[p] >> 32)) > P.th_depth)
                atomicMin(&s_stop, p);
    __syncthreads();
    const int stop = s_stop;
    for (int p = threadIdx.x; p < npad; p += kT) {
        if (keys[p] == ~0ull || p > stop) continue;
        const int i = (int)(keys[p] & 0xFFFFFFFFu);
        if (Mn.pos[o + i].w != 0.f) continue;  // tracked MapPoint
        const slam_keypoint kp = B.kps[o + i];
        const float4 X = unproject(P, T, Ow, kp, B.depth[o + i]);
        float4 N;
        float2 D;
        mp_geometry(P, X, Ow, kp.octave, N, D);
        Mn.pos[o + i] = X;
        Mn.normal[o + i] = N;
        Mn.dist[o + i] = D;
        const uint4* sd = reinterpret_cast<const uint4*>(B.desc + (o + i) * 32);
        uint4* md = reinterpret_cast<uint4*>(Mn.desc + (o + i) * 32);
        md[0] = sd[0];
        md[1] = sd[1];
    }
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += kT) {
        const bool v = Mn.pos[o + i].w != 0.f;
        B.valid[okf + i] = v;
        cnt += v;
    }
    const int nv = block_reduce_sum(cnt, scratch);
    if (threadIdx.x == 0) {
        B.n[P.S + s] = n;
        Q.cur = 1 - Q.cur;
        Q.n_ref = nv;
    }
}

// after the second PoseOptimization: TrackLocalMap's inliers (stereo outliers leave the frame),
// the pose, NeedNewKeyFrame / CreateNewKeyFrame; uninitialised sequences try StereoInitialization
// the current frame becomes mLastFrame (Tracking.cc:2140): its keypoints and MapPoints (after a
// new KeyFrame, every valid slot of it: CreateNewKeyFrame gives the frame its new MapPoints,
// Tracking.cc:3290-3300) and mlRelativeFramePoses' Tcr = Tcw * Tref^-1 (:2149)
__device__ void set_last_frame(const Bufs& B, int s, bool new_kf) {
    const Params& P = B.P;
    const size_t o = slot(P, s), okf = slot(P, P.S + s);
    Seq& Q = B.seq[s];
    const int n = B.n[s];
    for (int i = threadIdx.x; i < n; i += kT) {
        B.lf_kps[o + i] = B.kps[o + i];
        B.lf_fmp[o + i] = new_kf ? (B.valid[okf + i] ? i : -1) : B.fmp[o + i];
    }
    if (threadIdx.x == 0) {
        float Twr[16];
        pose_inverse(Q.Tref, Twr);  // KeyFrame::GetPoseInverse
        gemm4(Q.Tcw, Twr, Q.Tlr);
        Q.last_n = n;
    }
}

// after the second PoseOptimization: TrackLocalMap's inliers (stereo outliers leave the frame),
// the pose, the motion model, NeedNewKeyFrame / CreateNewKeyFrame, the last frame;
// uninitialised sequences try StereoInitialization
__global__ void __launch_bounds__(kT) k_finish(Bufs B) {
    __shared__ int scratch[20];
    __shared__ uint64_t keys[kMaxCap];
    __shared__ int s_need;
    const int s = blockIdx.x;
    const Params& P = B.P;
    const size_t o = slot(P, s);
    Seq& Q = B.seq[s];
    Rec& R = B.rec[s];
    const int n = B.n[s];
    // stereo points of this frame (diagnostic)
    int ns = 0;
    for (int i = threadIdx.x; i < n; i += kT) ns += B.depth[o + i] > 0;
    ns = block_reduce_sum(ns, scratch);
    if (Q.fail) {  // a SearchByProjection candidate overflow left this step's matches incomplete:
        // the step is void (status 1, reported lost) and the sequence keeps its previous state
        if (threadIdx.x == 0) {
            for (int k = 0; k < 16; k++) R.Tcw[k] = Q.Tcw[k];
            R.status = 1;
            R.lost = 1;
            R.is_kf = 0;
            R.n_stereo = ns;
        }
        return;
    }
    if (!Q.initialized) {  // Tracking::StereoInitialization (Tracking.cc:2366-2429)
        const bool init = n > 500;
        const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        if (init) make_keyframe(B, s, I, true, keys, scratch);
        if (threadIdx.x == 0) {
            for (int k = 0; k < 16; k++) Q.Tcw[k] = Q.Tref[k] = I[k];
            Q.initialized = init;
            Q.nkf = init;
            Q.has_vel = 0;  // mLastFrame has no pose yet: mVelocity stays empty
            for (int k = 0; k < 16; k++) R.Tcw[k] = Q.Tcw[k];
            R.is_kf = init;
            R.initialized = init;
            R.n_stereo = ns;
        }
        __syncthreads();
        if (init) set_last_frame(B, s, true);
        return;
    }
    const bool active = Q.active;
    int ninl = 0;
    if (active) ninl = drop_outliers(B, s, scratch);
    const pose::POut& po = B.po[s];
    // the frame's pose: TrackLocalMap's result; a sequence lost this frame keeps the last pose
    __syncthreads();
    if (threadIdx.x < 16 && active) Q.Tcw[threadIdx.x] = po.Tcw[threadIdx.x];
    __syncthreads();
    bool ok = active && ninl >= 30;  // TrackLocalMap: mnMatchesInliers < 30 -> false
    // NeedNewKeyFrame (Tracking.cc:2944-3040, stereo, LocalMapping idle: c1b holds -> c2 decides)
    int tc = 0, ntc = 0;
    for (int i = threadIdx.x; i < n; i += kT) {
        const float z = B.depth[o + i];
        if (z > 0 && z < P.th_depth) {
            if (B.fmp[o + i] >= 0) tc++;
            else ntc++;
        }
    }
    tc = block_reduce_sum(tc, scratch);
    ntc = block_reduce_sum(ntc, scratch);
    if (threadIdx.x == 0) {
        const bool close = tc < 100 && ntc > 70;
        const float thRefRatio = Q.nkf < 2 ? 0.4f : 0.75f;  // KeyFramesInMap() < 2 (:2990-2992)
        s_need = ok && (((float)ninl < (float)Q.n_ref * thRefRatio || close) && ninl > 15);
        for (int k = 0; k < 16; k++) R.Tcw[k] = Q.Tcw[k];
        R.n_inl = active ? ninl : 0;
        R.lost = !ok;
        R.n_stereo = ns;
        // motion model (Tracking.cc:2058-2068): mVelocity = mTcw * LastTwc, LastTwc from
        // mLastFrame's GetRotationInverse / GetCameraCenter; a lost frame drops it
        if (ok) {
            float Twl[16];
            pose_inverse(Q.Tlast, Twl);
            gemm4(Q.Tcw, Twl, Q.V);
        }
        Q.has_vel = ok;
    }
    __syncthreads();
    const bool need = s_need;
    if (need) {
        make_keyframe(B, s, Q.Tcw, false, keys, scratch);
        if (threadIdx.x == 0) {
            R.is_kf = 1;
            Q.nkf++;
            for (int k = 0; k < 16; k++) Q.Tref[k] = Q.Tcw[k];  // mpReferenceKF = pKF (:3075)
        }
    }
    __syncthreads();
    if (ok) set_last_frame(B, s, need);
}

}  // namespace track
}  // namespace slamhot

using namespace slamhot;
using namespace slamhot::track;

struct slam_tracker {
    int device = 0, S = 0, W = 0, H = 0, cap = 0, cand_cap = 0;
    hipStream_t stream = nullptr;
    slam_extractor *exl = nullptr, *exr = nullptr;
    slam_rectifier *rl = nullptr, *rr = nullptr;
    slam_stereo* st = nullptr;
    slam_matcher* m = nullptr;
    slam_vocab* voc = nullptr;  // borrowed
    Params P{};
    std::vector<int32_t> pairs;
    std::vector<void*> allocs;
    Bufs B{};
    uint8_t *d_rect_l = nullptr, *d_rect_r = nullptr;
    slam_keypoint* d_kps_r = nullptr;
    uint8_t* d_desc_r = nullptr;
    int32_t *d_n_r = nullptr, *d_mono = nullptr, *d_a2b = nullptr, *d_b2a = nullptr, *d_nbow = nullptr;
    int8_t* d_fclear = nullptr;
    float *d_ur = nullptr, *d_depth = nullptr;
    double* d_errs = nullptr;
    uint8_t *d_level = nullptr, *d_outl = nullptr;
    pose::POut* d_po = nullptr;
    int steps = 0;
};

namespace {

template <class T>
slam_status alloc(slam_tracker* t, T** p, size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(count * sizeof(T), 256)) != hipSuccess) return SLAM_ENOMEM;
    if (hipMemset(q, 0, std::max<size_t>(count * sizeof(T), 256)) != hipSuccess) return SLAM_EHIP;
    t->allocs.push_back(q);
    *p = (T*)q;
    return SLAM_OK;
}

void release(slam_tracker* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    for (void* p : t->allocs) (void)hipFree(p);
    if (t->exl) slamhot_extractor_destroy(t->exl);
    if (t->exr) slamhot_extractor_destroy(t->exr);
    if (t->rl) slamhot_rectifier_destroy(t->rl);
    if (t->rr) slamhot_rectifier_destroy(t->rr);
    if (t->st) slamhot_stereo_destroy(t->st);
    if (t->m) slamhot_matcher_destroy(t->m);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

}  // namespace

extern "C" {

slam_status slamhot_tracker_create(int device, const slam_tracker_config* cfg, slam_vocab* voc, slam_tracker** out) {
    if (!out || !cfg || !voc) return SLAM_EINVAL;
    *out = nullptr;
    const int S = cfg->nseq, W = cfg->width, H = cfg->height;
    if (S <= 0 || W <= 0 || H <= 0 || cfg->orb.nlevels < 1 || cfg->orb.nlevels > 16) return SLAM_EINVAL;
    const int cap = 2 * cfg->orb.nfeatures + 64;
    if (cap > kMaxCap) return SLAM_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= ndev) return SLAM_EINVAL;
    slam_tracker* t = new (std::nothrow) slam_tracker();
    if (!t) return SLAM_ENOMEM;
    t->device = device;
    t->S = S;
    t->W = W;
    t->H = H;
    t->cap = cap;
    t->voc = voc;
    slam_status st;
    auto fail = [&](slam_status e) {
        release(t);
        return e;
    };
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(SLAM_EHIP);
    if ((st = slamhot_extractor_create(&cfg->orb, device, W, H, S, &t->exl)) ||
        (st = slamhot_extractor_create(&cfg->orb, device, W, H, S, &t->exr)) || (st = slamhot_stereo_create(device, &t->st)) ||
        (st = slamhot_matcher_create(device, &t->m)))
        return fail(st);
    if (cfg->map_lx) {
        if (!cfg->map_ly || !cfg->map_rx || !cfg->map_ry) return fail(SLAM_EINVAL);
        if ((st = slamhot_rectifier_create(device, W, H, W, H, cfg->map_lx, cfg->map_ly, &t->rl)) ||
            (st = slamhot_rectifier_create(device, W, H, W, H, cfg->map_rx, cfg->map_ry, &t->rr)))
            return fail(st);
    }
    // camera / frame constants, in the reference's float arithmetic
    Params& P = t->P;
    P.fx = cfg->cam.fx;
    P.fy = cfg->cam.fy;
    P.cx = cfg->cam.cx;
    P.cy = cfg->cam.cy;
    P.bf = cfg->cam.bf;
    P.b = P.bf / P.fx;                                   // mb = mbf / fx (Tracking.cc:606)
    P.th_depth = P.bf * cfg->th_depth / P.fx;            // mThDepth (Tracking.cc:609)
    P.invfx = 1.0f / P.fx;
    P.invfy = 1.0f / P.fy;
    P.min_x = 0.f;                                       // rectified: no distortion (Frame.cc:785-790)
    P.max_x = (float)W;
    P.min_y = 0.f;
    P.max_y = (float)H;
    P.grid_inv_w = (float)kGridCols / (P.max_x - P.min_x);
    P.grid_inv_h = (float)kGridRows / (P.max_y - P.min_y);
    P.log_scale = (float)std::log((double)cfg->orb.scale_factor);
    int nl = 0;
    float sc[16], isig[16];
    if ((st = slamhot_extractor_levels(t->exl, &nl, sc, nullptr, nullptr, isig, nullptr))) return fail(st);
    P.nlevels = nl;
    for (int l = 0; l < 16; l++) {
        P.scale[l] = l < nl ? sc[l] : 1.f;
        P.inv_sigma2[l] = l < nl ? isig[l] : 1.f;
    }
    P.cap = cap;
    P.S = S;
    t->cand_cap = cap * 96;
    if (const char* e = std::getenv("SLAMHOT_TRACK_CAND_CAP")) t->cand_cap = std::max(16, std::atoi(e));  // tests: force overflow
    Bufs& B = t->B;
    B.P = P;
    B.cand_cap = t->cand_cap;
    const size_t SC = (size_t)S * cap;
    if ((st = alloc(t, &B.seq, S)) || (st = alloc(t, &B.rec, S)) || (st = alloc(t, &B.kps, 2 * SC)) ||
        (st = alloc(t, &B.desc, 2 * SC * 32)) || (st = alloc(t, &B.n, 2 * S)) || (st = alloc(t, &B.valid, 2 * SC)) ||
        (st = alloc(t, &t->d_ur, SC)) || (st = alloc(t, &t->d_depth, SC)) || (st = alloc(t, &t->d_a2b, SC)) ||
        (st = alloc(t, &t->d_b2a, SC)) || (st = alloc(t, &t->d_nbow, S)) || (st = alloc(t, &B.fmp, SC)) ||
        (st = alloc(t, &B.pf, S)) || (st = alloc(t, &B.pe, SC)) || (st = alloc(t, &t->d_po, S)) ||
        (st = alloc(t, &t->d_outl, SC)) || (st = alloc(t, &t->d_level, SC)) || (st = alloc(t, &t->d_errs, SC * 4)) ||
        (st = alloc(t, &B.geom, SC)) || (st = alloc(t, &B.track, SC)) || (st = alloc(t, &B.n_in_view, S)) ||
        (st = alloc(t, &B.fstate, SC)) || (st = alloc(t, &B.cell_start, (size_t)S * (kGridCells + 1))) ||
        (st = alloc(t, &B.cell_feat, SC)) || (st = alloc(t, &B.fcalls, S)) || (st = alloc(t, &B.pcalls, S)) ||
        (st = alloc(t, &B.queries, SC)) || (st = alloc(t, &B.cand_off, (size_t)S * (cap + 1))) ||
        (st = alloc(t, &B.cand, (size_t)S * t->cand_cap)) || (st = alloc(t, &B.fmatch, SC)) ||
        (st = alloc(t, &B.pout, (size_t)S * 4)) || (st = alloc(t, &t->d_kps_r, SC)) ||
        (st = alloc(t, &t->d_desc_r, SC * 32)) || (st = alloc(t, &t->d_n_r, S)) || (st = alloc(t, &t->d_mono, S)) ||
        (st = alloc(t, &t->d_rect_l, (size_t)S * W * H)) || (st = alloc(t, &t->d_rect_r, (size_t)S * W * H)) ||
        (st = alloc(t, &B.lf_kps, SC)) || (st = alloc(t, &B.lf_fmp, SC)) || (st = alloc(t, &B.lf_has, SC)) ||
        (st = alloc(t, &B.lf_zero, SC)) || (st = alloc(t, &B.lf_one, SC)) || (st = alloc(t, &B.lf_pos, SC * 3)) ||
        (st = alloc(t, &B.lf_desc, SC * 32)) || (st = alloc(t, &t->d_fclear, SC)) || (st = alloc(t, &B.mcalls, 2 * (size_t)S)) ||
        (st = alloc(t, &B.mmatch, 2 * SC)) || (st = alloc(t, &B.mout, 8 * (size_t)S)) || (st = alloc(t, &B.motm, SC)))
        return fail(st);
    if (hipMemset(B.lf_one, 1, SC) != hipSuccess || hipMemset(t->d_fclear, 0xFF, SC) != hipSuccess) return fail(SLAM_EHIP);
    B.fclear = t->d_fclear;
    for (int k = 0; k < 2; k++)
        if ((st = alloc(t, &B.mp[k].pos, SC)) || (st = alloc(t, &B.mp[k].normal, SC)) ||
            (st = alloc(t, &B.mp[k].dist, SC)) || (st = alloc(t, &B.mp[k].desc, SC * 32)))
            return fail(st);
    B.ur = t->d_ur;
    B.depth = t->d_depth;
    B.b2a = t->d_b2a;
    B.nbow = t->d_nbow;
    B.po = t->d_po;
    B.outl = t->d_outl;
    t->pairs.resize(2 * (size_t)S);
    for (int s = 0; s < S; s++) {
        t->pairs[2 * s] = S + s;  // (reference KeyFrame, frame)
        t->pairs[2 * s + 1] = s;
    }
    *out = t;
    return SLAM_OK;
}

void slamhot_tracker_destroy(slam_tracker* t) { release(t); }

slam_status slamhot_tracker_step_device(slam_tracker* t, const void* d_left, int left_pitch, int64_t left_stride,
                                        const void* d_right, int right_pitch, int64_t right_stride) {
    if (!t || !d_left || !d_right) return SLAM_EINVAL;
    SLAM_HIP_TRY(hipSetDevice(t->device));
    const int S = t->S, W = t->W, H = t->H, cap = t->cap;
    hipStream_t s = t->stream;
    Bufs& B = t->B;
    slam_status st;
    const uint8_t* il = (const uint8_t*)d_left;
    const uint8_t* ir = (const uint8_t*)d_right;
    int pl = left_pitch, pr = right_pitch;
    if (t->rl) {  // cv::remap of the raw pair (stereo_euroc.cc:168-169)
        if ((st = slamhot_rectify_batch_device(t->rl, S, d_left, left_pitch, left_stride, t->d_rect_l, W, (int64_t)W * H,
                                               s)) ||
            (st = slamhot_rectify_batch_device(t->rr, S, d_right, right_pitch, right_stride, t->d_rect_r, W,
                                               (int64_t)W * H, s)))
            return st;
        il = t->d_rect_l;
        ir = t->d_rect_r;
        pl = pr = W;
    } else if (left_pitch != W || right_pitch != W || left_stride != (int64_t)W * H || right_stride != (int64_t)W * H) {
        return SLAM_EINVAL;  // the extractor reads tight frames
    }
    (void)pl;
    (void)pr;
    if ((st = slamhot_extract_batch_device(t->exl, S, il, W, H, 0, 0, B.kps, B.desc, cap, B.n, t->d_mono, s)) ||
        (st = slamhot_extract_batch_device(t->exr, S, ir, W, H, 0, 0, t->d_kps_r, t->d_desc_r, cap, t->d_n_r, t->d_mono,
                                           s)) ||
        (st = slamhot_stereo_match_batch_device(t->st, t->exl, t->exr, S, B.kps, B.desc, B.n, t->d_kps_r, t->d_desc_r,
                                                t->d_n_r, cap, t->P.bf, t->P.b, t->d_ur, t->d_depth, nullptr, s)) ||
        (st = slamhot_bow_match_batch_device(t->m, t->voc, 2 * S, B.kps, B.desc, cap, B.n, B.valid, S, t->pairs.data(),
                                             0.7f, 1, 0, 4, t->d_a2b, t->d_b2a, t->d_nbow, s)))
        return st;
    // TrackWithMotionModel (sequences with a velocity), then TrackReferenceKeyFrame where it was
    // not tried or failed; both run as launches over all sequences, the device picks per sequence
    const size_t plds = projection_lds_bytes(cap, cap);
    hipLaunchKernelGGL(k_motion_setup, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(launch_search_by_projection(B.mcalls, S, plds, s));
    hipLaunchKernelGGL(k_motion_retry, dim3((S + 63) / 64), dim3(64), 0, s, B);
    SLAM_HIP_TRY(launch_search_by_projection(B.mcalls + S, S, plds, s));
    hipLaunchKernelGGL(k_motion_edges, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(pose::launch_pose_opt(B.pf, B.pe, t->d_errs, t->d_level, t->d_outl, t->d_po, S, s));
    hipLaunchKernelGGL(k_ref_edges, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(pose::launch_pose_opt(B.pf, B.pe, t->d_errs, t->d_level, t->d_outl, t->d_po, S, s));
    hipLaunchKernelGGL(k_local_setup, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(launch_is_in_frustum(B.fcalls, S, cap, s));
    SLAM_HIP_TRY(launch_search_by_projection(B.pcalls, S, plds, s));
    hipLaunchKernelGGL(k_local_edges, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(pose::launch_pose_opt(B.pf, B.pe, t->d_errs, t->d_level, t->d_outl, t->d_po, S, s));
    hipLaunchKernelGGL(k_finish, dim3(S), dim3(kT), 0, s, B);
    SLAM_HIP_TRY(hipGetLastError());
    t->steps++;
    return SLAM_OK;
}

slam_status slamhot_tracker_records(slam_tracker* t, slam_track_record* out) {
    if (!t || !out) return SLAM_EINVAL;
    static_assert(sizeof(Rec) == sizeof(slam_track_record), "record layout");
    SLAM_HIP_TRY(hipSetDevice(t->device));
    SLAM_HIP_TRY(hipMemcpyAsync(out, t->B.rec, sizeof(Rec) * t->S, hipMemcpyDeviceToHost, t->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(t->stream));
    // a SearchByProjection candidate overflow voided a sequence's step on the device (status 1:
    // its state was kept as before the step); report it
    for (int s = 0; s < t->S; s++)
        if (out[s].status == 1) return SLAM_ECAP;
    return SLAM_OK;
}

slam_status slamhot_tracker_keyframe(slam_tracker* t, int seq, slam_track_keyframe* kf) {
    if (!t || !kf || seq < 0 || seq >= t->S) return SLAM_EINVAL;
    SLAM_HIP_TRY(hipSetDevice(t->device));
    SLAM_HIP_TRY(hipStreamSynchronize(t->stream));
    Seq q;
    int32_t n = 0;
    SLAM_HIP_TRY(hipMemcpy(&q, t->B.seq + seq, sizeof(Seq), hipMemcpyDeviceToHost));
    SLAM_HIP_TRY(hipMemcpy(&n, t->B.n + t->S + seq, 4, hipMemcpyDeviceToHost));
    std::memcpy(kf->Tcw, q.Tcw, sizeof(kf->Tcw));
    kf->initialized = q.initialized;
    kf->n_ref = q.n_ref;
    kf->n = q.initialized ? n : 0;
    if (kf->cap < kf->n) return SLAM_ECAP;
    const size_t o = (size_t)(t->S + seq) * t->cap, om = (size_t)seq * t->cap;
    const MapPts& M = t->B.mp[q.cur];
    std::vector<float4> pos(kf->n), nrm(kf->n);
    std::vector<float2> d(kf->n);
    if (kf->n) {
        SLAM_HIP_TRY(hipMemcpy(kf->kps, t->B.kps + o, sizeof(slam_keypoint) * kf->n, hipMemcpyDeviceToHost));
        SLAM_HIP_TRY(hipMemcpy(kf->desc, t->B.desc + o * 32, 32 * (size_t)kf->n, hipMemcpyDeviceToHost));
        SLAM_HIP_TRY(hipMemcpy(pos.data(), M.pos + om, sizeof(float4) * kf->n, hipMemcpyDeviceToHost));
        SLAM_HIP_TRY(hipMemcpy(nrm.data(), M.normal + om, sizeof(float4) * kf->n, hipMemcpyDeviceToHost));
        SLAM_HIP_TRY(hipMemcpy(d.data(), M.dist + om, sizeof(float2) * kf->n, hipMemcpyDeviceToHost));
        SLAM_HIP_TRY(hipMemcpy(kf->mp_desc, M.desc + om * 32, 32 * (size_t)kf->n, hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < kf->n; i++) {
        kf->mp_valid[i] = pos[i].w != 0.f;
        kf->mp_pos[3 * i] = pos[i].x;
        kf->mp_pos[3 * i + 1] = pos[i].y;
        kf->mp_pos[3 * i + 2] = pos[i].z;
        kf->mp_normal[3 * i] = nrm[i].x;
        kf->mp_normal[3 * i + 1] = nrm[i].y;
        kf->mp_normal[3 * i + 2] = nrm[i].z;
        kf->mp_min_dist[i] = d[i].x;
        kf->mp_max_dist[i] = d[i].y;
    }
    return SLAM_OK;
}

slam_status slamhot_tracker_state(slam_tracker* t, int seq, slam_track_state* st) {
    if (!t || !st || seq < 0 || seq >= t->S) return SLAM_EINVAL;
    SLAM_HIP_TRY(hipSetDevice(t->device));
    SLAM_HIP_TRY(hipStreamSynchronize(t->stream));
    Seq q;
    SLAM_HIP_TRY(hipMemcpy(&q, t->B.seq + seq, sizeof(Seq), hipMemcpyDeviceToHost));
    std::memcpy(st->V, q.V, sizeof(st->V));
    std::memcpy(st->Tlr, q.Tlr, sizeof(st->Tlr));
    std::memcpy(st->Tref, q.Tref, sizeof(st->Tref));
    st->has_vel = q.initialized && q.has_vel;
    st->nkf = q.nkf;
    st->last_n = q.initialized ? q.last_n : 0;
    if (st->cap < st->last_n) return SLAM_ECAP;
    const size_t o = (size_t)seq * t->cap;
    if (st->last_n && st->last_kps)
        SLAM_HIP_TRY(hipMemcpy(st->last_kps, t->B.lf_kps + o, sizeof(slam_keypoint) * st->last_n, hipMemcpyDeviceToHost));
    if (st->last_n && st->last_mp)
        SLAM_HIP_TRY(hipMemcpy(st->last_mp, t->B.lf_fmp + o, 4 * (size_t)st->last_n, hipMemcpyDeviceToHost));
    return SLAM_OK;
}

slam_status slamhot_tracker_frame(slam_tracker* t, int seq, slam_track_frame* fr) {
    if (!t || !fr || seq < 0 || seq >= t->S) return SLAM_EINVAL;
    SLAM_HIP_TRY(hipSetDevice(t->device));
    SLAM_HIP_TRY(hipStreamSynchronize(t->stream));
    int32_t n = 0;
    SLAM_HIP_TRY(hipMemcpy(&n, t->B.n + seq, 4, hipMemcpyDeviceToHost));
    fr->n = n;
    if (fr->cap < n) return SLAM_ECAP;
    const size_t o = (size_t)seq * t->cap;
    auto get = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        return dst && bytes ? hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) : hipSuccess;
    };
    SLAM_HIP_TRY(get(fr->uright, t->d_ur + o, 4 * (size_t)n));
    SLAM_HIP_TRY(get(fr->bow_match, t->d_b2a + o, 4 * (size_t)n));
    SLAM_HIP_TRY(get(fr->motion_match, t->B.motm + o, 4 * (size_t)n));
    SLAM_HIP_TRY(get(fr->local_match, t->B.fmatch + o, 4 * (size_t)n));
    SLAM_HIP_TRY(get(fr->mappoints, t->B.fmp + o, 4 * (size_t)n));
    return SLAM_OK;
}

}  // extern "C"
