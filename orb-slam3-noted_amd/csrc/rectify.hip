// rectify.hip — MI355X (gfx950) cv::remap(INTER_LINEAR, BORDER_CONSTANT 0) with float maps,
// the stereo rectification stereo_euroc.cc:168-169 runs on every EuRoC frame pair.
//
//   k_remap_prep   once per map: X = rne(map_x * 32), Y = rne(map_y * 32) (OpenCV's
//                  saturate_cast<int>), stored as (sx, sy, fx | fy << 5) = integer source
//                  position and 5-bit fractions.
//   k_remap        thread per 4 destination pixels of one row; the prepared map entries stay
//                  in registers while the thread walks kFramesPerBlock frames, so the map is
//                  read once per frame group and every frame costs its source gathers (L2)
//                  plus one 32-bit store per thread.  Weights (32-fx)(32-fy)*32 ... sum to
//                  2^15; result (sum + 2^14) >> 15 (FixedPtCast<int, uchar, 15>).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <new>

#include "common.hpp"

namespace slamhot {
namespace {

constexpr int kRemapThreads = 256;
// 16 frames per workgroup: the map entries are read once per 16 frames (at 8 the map traffic
// equalled the image traffic); rectify stage 0.122 -> 0.115 ms per 128 pairs, headline +1%
// (interleaved A/B); 32 was slower (0.133 ms, too few workgroups).
#ifndef SLAMHOT_REMAP_FPB
#define SLAMHOT_REMAP_FPB 16
#endif
constexpr int kFramesPerBlock = SLAMHOT_REMAP_FPB;  // experiment builds: -DSLAMHOT_REMAP_FPB=<n>
#ifndef SLAMHOT_REMAP_XCD
#define SLAMHOT_REMAP_XCD 1
#endif

struct MapEntry {
    int16_t sx, sy;
    int32_t frac;  // fx | fy << 5
};

__global__ void __launch_bounds__(256) k_remap_prep(int n, const float* mx, const float* my, MapEntry* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float fxs = mx[i] * 32.0f, fys = my[i] * 32.0f;
    // saturate_cast<int>(float): round to nearest even, saturate
    const float lim = 2147483520.0f;  // largest float below 2^31
    const int X = fxs >= 2147483648.0f ? 2147483647 : fxs <= -2147483648.0f ? (int)0x80000000 : __float2int_rn(fminf(fmaxf(fxs, -lim), lim));
    const int Y = fys >= 2147483648.0f ? 2147483647 : fys <= -2147483648.0f ? (int)0x80000000 : __float2int_rn(fminf(fmaxf(fys, -lim), lim));
    MapEntry e;
    e.sx = (int16_t)min(max(X >> 5, -32768), 32767);
    e.sy = (int16_t)min(max(Y >> 5, -32768), 32767);
    e.frac = (X & 31) | ((Y & 31) << 5);
    out[i] = e;
}

__device__ __forceinline__ int remap_px(const uint8_t* src, int sw, int sh, int sp, const MapEntry e) {
    const int sx = e.sx, sy = e.sy;
    const int fx = e.frac & 31, fy = e.frac >> 5;
    const int w00 = (32 - fx) * (32 - fy), w01 = fx * (32 - fy), w10 = (32 - fx) * fy, w11 = fx * fy;
    if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
        const uint8_t* S = src + (size_t)sy * sp + sx;
        const int v = (S[0] * w00 + S[1] * w01 + S[sp] * w10 + S[sp + 1] * w11) * 32;
        return (v + (1 << 14)) >> 15;
    }
    if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) return 0;
    auto at = [&](int yy, int xx) -> int {
        return (xx >= 0 && xx < sw && yy >= 0 && yy < sh) ? src[(size_t)yy * sp + xx] : 0;
    };
    const int v = (at(sy, sx) * w00 + at(sy, sx + 1) * w01 + at(sy + 1, sx) * w10 + at(sy + 1, sx + 1) * w11) * 32;
    return min(max((v + (1 << 14)) >> 15, 0), 255);
}

__global__ void __launch_bounds__(kRemapThreads) k_remap(const MapEntry* map, int dw, int dh, int sw, int sh,
                                                         int nframes, const uint8_t* src, int sp, int64_t sstride,
                                                         uint8_t* dst, int dp, int64_t dstride) {
    const int qw = (dw + 3) >> 2;
    const int t = blockIdx.x * kRemapThreads + threadIdx.x;
    if (t >= qw * dh) return;
    const int y = t / qw, x0 = (t - y * qw) * 4;
    const int nx = min(4, dw - x0);
    MapEntry e[4];
#pragma unroll
    for (int k = 0; k < 4; k++) e[k] = map[(size_t)y * dw + min(x0 + k, dw - 1)];
    const int f0 = blockIdx.y * kFramesPerBlock, f1 = min(nframes, f0 + kFramesPerBlock);
    const bool aligned = nx == 4 && ((dp | (int)(dstride & 3)) & 3) == 0;
    for (int f = f0; f < f1; f++) {
        const uint8_t* S = src + f * sstride;
        uint8_t* D = dst + f * dstride + (size_t)y * dp + x0;
        int v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = remap_px(S, sw, sh, sp, e[k]);
        if (aligned) {
            *reinterpret_cast<uint32_t*>(D) = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                                              ((uint32_t)v[3] << 24);
        } else {
            for (int k = 0; k < nx; k++) D[k] = (uint8_t)v[k];
        }
    }
}

// ---- LDS-tiled form: a workgroup owns a 64 x 16 destination tile.  A rectification map is
// near-identity, so the tile reads a small source box (its bounding box over the tile's map
// entries, +1 for the bilinear taps): the box is staged into LDS with row-contiguous loads
// (out-of-image cells as the border value 0 — exactly remap_px's `at`), then each thread makes
// 4 pixels from LDS.  Boxes are computed once per map (k_tile_boxes); a tile whose box exceeds
// kBoxMax bytes keeps the per-pixel gather path.
constexpr int kTileW = 64, kTileH = 16, kBoxMax = 12 * 1024;

__global__ void __launch_bounds__(256) k_tile_boxes(const MapEntry* map, int dw, int dh, int tiles_x, int4* boxes) {
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    int x0 = 1 << 30, y0 = 1 << 30, x1 = -(1 << 30), y1 = -(1 << 30);
    for (int i = threadIdx.x; i < kTileW * kTileH; i += blockDim.x) {
        const int x = tx * kTileW + (i % kTileW), y = ty * kTileH + i / kTileW;
        if (x >= dw || y >= dh) continue;
        const MapEntry e = map[(size_t)y * dw + x];
        x0 = min(x0, (int)e.sx);
        y0 = min(y0, (int)e.sy);
        x1 = max(x1, (int)e.sx + 1);
        y1 = max(y1, (int)e.sy + 1);
    }
    __shared__ int red[4][256];
    red[0][threadIdx.x] = x0;
    red[1][threadIdx.x] = y0;
    red[2][threadIdx.x] = -x1;
    red[3][threadIdx.x] = -y1;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o)
            for (int k = 0; k < 4; k++) red[k][threadIdx.x] = min(red[k][threadIdx.x], red[k][threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int bx0 = red[0][0], by0 = red[1][0], bx1 = -red[2][0], by1 = -red[3][0];
        const long long bw = (long long)bx1 - bx0 + 1, bh = (long long)by1 - by0 + 1;
        const bool ok = bw > 0 && bh > 0 && (bw + 6) * bh <= kBoxMax && bw + 6 <= 4 * 256;
        boxes[blockIdx.x] = ok ? make_int4(bx0, by0, (int)bw, (int)bh) : make_int4(0, 0, 0, 0);  // w = 0: gather
    }
}

__global__ void __launch_bounds__(256) k_remap_tiled(const MapEntry* map, const int4* boxes, int tiles_x, int dw,
                                                     int dh, int sw, int sh, int nframes, const uint8_t* src, int sp,
                                                     int64_t sstride, uint8_t* dst, int dp, int64_t dstride) {
    __shared__ __attribute__((aligned(16))) uint8_t box[kBoxMax];
    constexpr int kPer = 4;  // box dwords per thread (register double buffer across frames)
#if SLAMHOT_REMAP_XCD
    // XCD-aware order (cdna_hip_programming.md T1): the dispatcher deals consecutive workgroups
    // round-robin over the 8 XCDs; remapped, each XCD takes a contiguous run of (tile, frame group)
    // in tile-fastest order, so the source rows two neighbouring tiles' boxes share are fetched into
    // one L2 instead of two.  Speed only: any placement is correct.
    const int nwg = (int)(gridDim.x * gridDim.y), orig = (int)(blockIdx.x + gridDim.x * blockIdx.y);
    const int xq = nwg >> 3, xr = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int tile = wg % (int)gridDim.x, fgrp = wg / (int)gridDim.x;
#else
    const int tile = blockIdx.x, fgrp = blockIdx.y;
#endif
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int4 B = boxes[tile];
    const int lx = (threadIdx.x & 15) * 4, ly = threadIdx.x >> 4;  // 16 threads x 4 px per row, 16 rows
    const int x0 = tx * kTileW + lx, y = ty * kTileH + ly;
    const bool live = x0 < dw && y < dh;
    const int nx = live ? min(4, dw - x0) : 0;
    MapEntry e[4];
#pragma unroll
    for (int k = 0; k < 4; k++) e[k] = live ? map[(size_t)y * dw + min(x0 + k, dw - 1)] : MapEntry{0, 0, 0};
    const int f0 = fgrp * kFramesPerBlock, f1 = min(nframes, f0 + kFramesPerBlock);
    const bool aligned = nx == 4 && ((dp | (int)(dstride & 3)) & 3) == 0;
    const bool aligned_src = ((sp | (int)(sstride & 3) | (int)((uintptr_t)src & 3)) & 3) == 0;
    // box rows start at the 4-byte-aligned column ax <= B.x; thread (qr, qc) owns dword qc of rows
    // qr, qr + rpp, ... (at most kPer of them, else the tile takes the gather path)
    const int ax = B.x & ~3, q = B.z > 0 ? (B.x - ax + B.z + 3) >> 2 : 1, bw = q * 4;
    const int qr = (int)threadIdx.x / q, qc = (int)threadIdx.x - qr * q, rpp = (int)blockDim.x / q;
    const bool tiled = B.z > 0 && (B.w + rpp - 1) / rpp <= kPer;
    uint32_t nxt[kPer];
    auto load = [&](const uint8_t* S) {
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const int r = qr + j * rpp;
            uint32_t w = 0;
            if (qr < rpp && r < B.w) {
                const int sy = B.y + r, sx = ax + 4 * qc;
                if ((unsigned)sy < (unsigned)sh) {
                    const uint8_t* row = S + (size_t)sy * sp;
                    if (sx >= 0 && sx + 3 < sw && aligned_src) {
                        w = *reinterpret_cast<const uint32_t*>(row + sx);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if ((unsigned)(sx + k) < (unsigned)sw) w |= (uint32_t)row[sx + k] << (8 * k);
                    }
                }
            }
            nxt[j] = w;
        }
    };
    if (tiled && f0 < f1) load(src + f0 * sstride);
    uint32_t* box32 = reinterpret_cast<uint32_t*>(box);
    for (int f = f0; f < f1; f++) {
        const uint8_t* S = src + f * sstride;
        int v[4];
        if (tiled) {
            __syncthreads();  // the previous frame's box reads are done
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const int r = qr + j * rpp;
                if (qr < rpp && r < B.w) box32[r * q + qc] = nxt[j];
            }
            __syncthreads();
            if (f + 1 < f1) load(S + sstride);  // next frame's box in flight during this one's math
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int fx = e[k].frac & 31, fy = e[k].frac >> 5;
                const int w00 = (32 - fx) * (32 - fy), w01 = fx * (32 - fy), w10 = (32 - fx) * fy, w11 = fx * fy;
                const uint8_t* qq = box + (e[k].sy - B.y) * bw + (e[k].sx - ax);
                const int s = (qq[0] * w00 + qq[1] * w01 + qq[bw] * w10 + qq[bw + 1] * w11) * 32;
                v[k] = min(max((s + (1 << 14)) >> 15, 0), 255);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = live ? remap_px(S, sw, sh, sp, e[k]) : 0;
        }
        if (!live) continue;
        uint8_t* D = dst + f * dstride + (size_t)y * dp + x0;
        if (aligned) {
            *reinterpret_cast<uint32_t*>(D) = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                                              ((uint32_t)v[3] << 24);
        } else {
            for (int k = 0; k < nx; k++) D[k] = (uint8_t)v[k];
        }
    }
}

}  // namespace
}  // namespace slamhot

using namespace slamhot;

struct slam_rectifier {
    int device = 0;
    hipStream_t stream = nullptr;
    int sw = 0, sh = 0, dw = 0, dh = 0, tiles_x = 0, ntiles = 0;
    MapEntry* d_map = nullptr;
    int4* d_boxes = nullptr;
};

extern "C" {

slam_status slamhot_rectifier_create(int device, int src_w, int src_h, int dst_w, int dst_h, const float* map_x,
                                     const float* map_y, slam_rectifier** out) {
    if (!out || !map_x || !map_y || src_w <= 0 || src_h <= 0 || dst_w <= 0 || dst_h <= 0 || src_w > 32767 ||
        src_h > 32767)
        return SLAM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= n) return SLAM_EINVAL;
    slam_rectifier* r = new (std::nothrow) slam_rectifier();
    if (!r) return SLAM_ENOMEM;
    r->device = device;
    r->sw = src_w;
    r->sh = src_h;
    r->dw = dst_w;
    r->dh = dst_h;
    const size_t np = (size_t)dst_w * dst_h;
    float* d_f = nullptr;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&r->d_map, np * sizeof(MapEntry)) != hipSuccess || hipMalloc(&d_f, np * 8) != hipSuccess) {
        if (d_f) (void)hipFree(d_f);
        slamhot_rectifier_destroy(r);
        return SLAM_EHIP;
    }
    hipError_t e = hipMemcpy(d_f, map_x, np * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_f + np, map_y, np * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_remap_prep, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, r->stream, (int)np, d_f,
                           d_f + np, r->d_map);
        e = hipGetLastError();
    }
    r->tiles_x = (dst_w + kTileW - 1) / kTileW;
    r->ntiles = r->tiles_x * ((dst_h + kTileH - 1) / kTileH);
    if (e == hipSuccess) e = hipMalloc(&r->d_boxes, sizeof(int4) * r->ntiles);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_tile_boxes, dim3(r->ntiles), dim3(256), 0, r->stream, r->d_map, dst_w, dst_h, r->tiles_x,
                           r->d_boxes);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
    (void)hipFree(d_f);
    if (e != hipSuccess) {
        slamhot_rectifier_destroy(r);
        return SLAM_EHIP;
    }
    *out = r;
    return SLAM_OK;
}

void slamhot_rectifier_destroy(slam_rectifier* r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    if (r->d_map) (void)hipFree(r->d_map);
    if (r->d_boxes) (void)hipFree(r->d_boxes);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

slam_status slamhot_rectify_batch_device(slam_rectifier* r, int nframes, const void* d_src, int src_pitch,
                                         int64_t src_stride, void* d_dst, int dst_pitch, int64_t dst_stride,
                                         void* hip_stream) {
    if (!r || nframes < 0 || (nframes && (!d_src || !d_dst)) || src_pitch < r->sw || dst_pitch < r->dw ||
        (nframes > 1 && (src_stride < (int64_t)src_pitch * r->sh || dst_stride < (int64_t)dst_pitch * r->dh)))
        return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    SLAM_HIP_TRY(hipSetDevice(r->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : r->stream;
    const char* env = std::getenv("SLAMHOT_REMAP");  // "gather": the per-pixel kernel (A/B runs)
    if (env && env[0] == 'g') {
        const int qw = (r->dw + 3) >> 2;
        const dim3 grid((unsigned)((qw * r->dh + kRemapThreads - 1) / kRemapThreads),
                        (unsigned)((nframes + kFramesPerBlock - 1) / kFramesPerBlock));
        hipLaunchKernelGGL(k_remap, grid, dim3(kRemapThreads), 0, s, r->d_map, r->dw, r->dh, r->sw, r->sh, nframes,
                           (const uint8_t*)d_src, src_pitch, src_stride, (uint8_t*)d_dst, dst_pitch, dst_stride);
    } else {
        const dim3 grid((unsigned)r->ntiles, (unsigned)((nframes + kFramesPerBlock - 1) / kFramesPerBlock));
        hipLaunchKernelGGL(k_remap_tiled, grid, dim3(256), 0, s, r->d_map, r->d_boxes, r->tiles_x, r->dw, r->dh, r->sw,
                           r->sh, nframes, (const uint8_t*)d_src, src_pitch, src_stride, (uint8_t*)d_dst, dst_pitch,
                           dst_stride);
    }
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

}  // extern "C"
