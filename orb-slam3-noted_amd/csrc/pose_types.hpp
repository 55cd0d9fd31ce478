// pose_types.hpp — the motion-only BA kernel's frame / edge records (pose.hip), shared with the
// device-resident tracker (track.hip), which builds them on the device.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace slamhot {
namespace pose {

struct PEdge {
    float obs[3];     // u, v, ur
    float info;       // invSigma2
    float Xw[3];
    int idx;          // feature index; bit 31 = stereo
};

struct PFrame {
    float Tcw[16];
    float fx, fy, cx, cy, bf;
    int e0, ne;       // edge range
};

struct POut {
    float Tcw[16];
    int n_inliers;
    int pad[3];
};


// launcher (pose.hip): nframes workgroups; frames / edges / outputs in device memory
hipError_t launch_pose_opt(const PFrame* frames, const PEdge* edges, double* errs, uint8_t* level, uint8_t* outlier,
                           POut* out, int nframes, hipStream_t s);

}  // namespace pose
}  // namespace slamhot
