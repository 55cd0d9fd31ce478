// common.hpp — shared host/device helpers for libslamhot (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

#include "../../include/slamhot.h"

namespace slamhot {

#define SLAM_HIP_TRY(expr)                                                                 \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            std::fprintf(stderr, "slamhot: HIP error %s at %s:%d: %s\n", hipGetErrorName(_e), \
                         __FILE__, __LINE__, #expr);                                       \
            return SLAM_EHIP;                                                              \
        }                                                                                  \
    } while (0)

#define SLAM_TRY_ST(expr)                         \
    do {                                          \
        const slam_status _st = (expr);           \
        if (_st != SLAM_OK) return _st;           \
    } while (0)

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Inclusive block-wide scan of one int per thread (blockDim.x multiple of 64, <= 1024).
// `scratch` needs blockDim.x/64 + 1 ints of LDS.  Returns the inclusive prefix; *total
// receives the block sum.
// Inclusive scan of one int per lane over a full wave by DPP (row_shr 1/2/4/8 Kogge-Stone inside
// each 16-lane row, then row_bcast:15 / row_bcast:31 across rows): VALU, no ds_bpermute.
__device__ __forceinline__ int wave_scan_incl_dpp(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ int block_scan_incl(int v, int* scratch, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int x = wave_scan_incl_dpp(v);
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    if (wid == 0) {
        const int s = wave_scan_incl_dpp(lane < nw ? scratch[lane] : 0);
        if (lane < nw) scratch[lane] = s;
    }
    __syncthreads();
    const int base = wid ? scratch[wid - 1] : 0;
    if (total) *total = scratch[nw - 1];
    __syncthreads();
    return x + base;
}

__device__ __forceinline__ int block_reduce_sum(int v, int* scratch) {
    int total;
    block_scan_incl(v, scratch, &total);
    return total;
}

}  // namespace slamhot
