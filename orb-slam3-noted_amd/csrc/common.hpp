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
__device__ __forceinline__ int block_scan_incl(int v, int* scratch, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    if (wid == 0) {
        int s = lane < nw ? scratch[lane] : 0;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            int y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
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
