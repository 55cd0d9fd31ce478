// projection.hpp — the call records of the SearchByProjection / isInFrustum kernels
// (matcher.hip), shared with the device-resident tracker (track.hip), which fills them on the
// device.  One record per frame: a launch takes an array of them (workgroup / grid row per call).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slamhot.h"

namespace slamhot {

constexpr int kGridCols = 64, kGridRows = 48;  // Frame.h:37-38

struct DevProjFrame {
    int n;
    const slam_keypoint* kps;
    const float* uright;
    const uint8_t* desc;
    const int8_t* state;          // entry mvpMapPoints state
    const int32_t* cell_start;    // kGridCols*kGridRows + 1
    const int32_t* cell_feat;
    float min_x, min_y, max_x, max_y, inv_w, inv_h;
    float fx, fy, cx, cy, bf, b;
    float T[16];
    float scale[16];
    int nlevels;
};

struct ProjQuery {
    float u, v, r;      // window centre and half size
    float ur, er;       // stereo gate: skip candidates with uright > 0 && |ur - uright| > er (er < 0: off)
    int16_t min_level, max_level;
    int32_t valid;
    float angle;        // for the rotation histogram
    int32_t blocking;   // a match by this query occupies the feature for later queries
};

enum { kProjLocal = 0, kProjLast = 1, kProjKF = 2 };

struct DevProjCall {
    DevProjFrame F;
    int mode, nq;
    // local-map inputs
    const slam_mp_track* mps;
    float th, th_far, nnratio;
    int far_points;
    // last-frame inputs
    const slam_keypoint* lf_kps;
    const slam_keypoint* lf_kps_un;
    const uint8_t* lf_has_mp;
    const uint8_t* lf_outlier;
    const float* lf_pos;
    const uint8_t* lf_has_obs;
    float LT[16];
    int mono;
    // prepared queries (KF variant) or scratch for computed ones
    ProjQuery* queries;
    const uint8_t* qdesc;   // nq x 32 query descriptors
    int th_dist;            // acceptance threshold (TH_HIGH or ORBdist)
    int check_ori;
    // scratch / outputs
    int32_t* cand_off;      // nq + 1
    uint32_t* cand;         // (feature << 12) | dist   (capacity cand_cap)
    int cand_cap;
    int32_t* f_match;       // F.n
    int32_t* out;           // [0] nmatches, [1] status (1 = candidate overflow), [2] iterations
    int32_t* gstate;        // resolution state in global memory when it exceeds the LDS (else null)
    int grid_on_device;     // batched calls: F.cell_start / cell_feat are built by k_frame_grid
};

struct FrustumCall {
    float R[9], t[3], Ow[3];
    float min_x, max_x, min_y, max_y, fx, fy, cx, cy, bf;
    float log_scale, view_cos_limit;
    int nlevels, n;
    const slam_mp_geom* mps;
    slam_mp_track* track;
    int32_t* n_in_view;
};


// launchers (matcher.hip): `calls` in device memory; lds = dynamic LDS bytes of the largest call
hipError_t launch_search_by_projection(const DevProjCall* calls, int ncalls, size_t lds, hipStream_t s);
hipError_t launch_is_in_frustum(const FrustumCall* calls, int ncalls, int max_n, hipStream_t s);
size_t projection_lds_bytes(int n_features, int n_queries);  // 0: the call needs gstate (HBM)

}  // namespace slamhot
