// stereo.hip — MI355X (gfx950) Frame::ComputeStereoMatches (Frame.cc:794-964).
//
//   k_stereo_rows    one workgroup per frame: the reference's vRowIndices (:808-824) as a CSR
//                    table — LDS row counters (atomics), block scan, scatter of right keypoint
//                    indices.  Entry order inside a row is arbitrary; the match step breaks
//                    ties by the smallest right index, which is the order the reference's
//                    push_back loop produces, so the result does not depend on it.
//   k_stereo_match   one thread per left keypoint (grid: keypoint chunks x frames): band
//                    candidates filtered by octave and u range, Hamming best < 100 (:849-871),
//                    threshold 75, then the 11x11 SAD search over +-5 columns on the level's
//                    pyramid (:874-915) — eleven running sums updated row by row from one
//                    11-byte left slice and one 21-byte right slice — parabola fit and the
//                    disparity gate (:917-946).  Integer SADs are exact, the float arithmetic
//                    is the reference's operation for operation (no contraction).
//   k_stereo_median  one workgroup per frame: radix select of the median kept SAD in LDS,
//                    cut at 1.5f*1.4f*median (:950-963).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <new>

#include "common.hpp"

namespace slamhot {
namespace {

constexpr int kStMaxLevels = 16;
constexpr int kStMaxRows = 4096;      // level-0 image height limit (extractor limit 4095)
constexpr int kStMaxSort = 8192;      // keypoints per frame for the median sort (LDS)
constexpr int kRowsThreads = 1024;
// one wave per workgroup (keypoints' band searches finish at different times): stereo stage
// 0.125 -> 0.120 ms per 128 pairs, headline +0.6% against 128 threads (interleaved A/B)
constexpr int kMatchThreads = 64;
constexpr int kMedianThreads = 1024;
#ifndef SLAMHOT_ST_CAND
#define SLAMHOT_ST_CAND 4
#endif
constexpr int kStCand = SLAMHOT_ST_CAND;  // band candidates per step of k_stereo_match
#ifndef SLAMHOT_ST_SADROWS
#define SLAMHOT_ST_SADROWS 2
#endif
constexpr int kSadRows = SLAMHOT_ST_SADROWS;
#ifndef SLAMHOT_ST_XCD
#define SLAMHOT_ST_XCD 1
#endif  // SAD window rows whose loads are issued together

// one band-table entry: the right keypoint's index with the two fields the candidate filter reads
// (octave, x), so a candidate costs one 8-byte load instead of an index and a 28-byte keypoint
struct StEnt {
    uint16_t idx;
    int16_t octave;
    float x;
};
static_assert(sizeof(StEnt) == 8, "one 8-byte load per candidate");

struct StereoGeom {
    const uint8_t* base[2][kStMaxLevels];  // level l of frame 0 (left, right)
    int64_t fstride[2][kStMaxLevels];      // bytes between frames at level l
    int pitch[2][kStMaxLevels];
    int lw[kStMaxLevels], lh[kStMaxLevels];
    float scale[kStMaxLevels], inv_scale[kStMaxLevels];
    int nlevels, nrows, cap, ent_cap;
    float mbf, mb;
};

__global__ void __launch_bounds__(kRowsThreads) k_stereo_rows(StereoGeom G, const slam_keypoint* kps_r,
                                                             const int32_t* n_r, int32_t* row_off,
                                                             StEnt* ent) {
    __shared__ int cnt[kStMaxRows];
    __shared__ int scan_tmp[kRowsThreads / 64 + 1];
    const int f = blockIdx.x, t = threadIdx.x;
    const int nrows = G.nrows;
    const int nr = n_r[f];
    const slam_keypoint* K = kps_r + (size_t)f * G.cap;
    for (int r = t; r < nrows; r += kRowsThreads) cnt[r] = 0;
    __syncthreads();
    for (int i = t; i < nr; i += kRowsThreads) {
        const float y = K[i].y;
        const float r = 2.0f * G.scale[K[i].octave];
        const int maxr = (int)ceilf(y + r), minr = (int)floorf(y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, nrows - 1); yi++) atomicAdd(&cnt[yi], 1);
    }
    __syncthreads();
    // exclusive offsets: each thread owns a contiguous chunk of rows
    const int per = (nrows + kRowsThreads - 1) / kRowsThreads;
    const int r0 = t * per, r1 = min(r0 + per, nrows);
    int local = 0;
    for (int r = r0; r < r1; r++) local += cnt[r];
    const int incl = block_scan_incl(local, scan_tmp, nullptr);
    int run = incl - local;
    int32_t* off = row_off + (size_t)f * (nrows + 1);
    for (int r = r0; r < r1; r++) {
        const int c = cnt[r];
        off[r] = run;
        cnt[r] = run;  // becomes the scatter cursor
        run += c;
    }
    if (t == kRowsThreads - 1) off[nrows] = incl;
    __syncthreads();
    StEnt* E = ent + (size_t)f * G.ent_cap;
    for (int i = t; i < nr; i += kRowsThreads) {
        const float y = K[i].y, x = K[i].x;
        const int oct = K[i].octave;
        const float r = 2.0f * G.scale[oct];
        const int maxr = (int)ceilf(y + r), minr = (int)floorf(y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, nrows - 1); yi++)
            E[atomicAdd(&cnt[yi], 1)] = StEnt{(uint16_t)i, (int16_t)oct, x};
    }
}

__device__ __forceinline__ int ham32(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ void __launch_bounds__(kMatchThreads) k_stereo_match(StereoGeom G, const slam_keypoint* kps_l,
                                                               const uint8_t* desc_l, const int32_t* n_l,
                                                               const slam_keypoint* kps_r, const uint8_t* desc_r,
                                                               const int32_t* row_off, const StEnt* ent,
                                                               float* uright, float* depth, int32_t* sad) {
#if SLAMHOT_ST_XCD
    // XCD-aware order (cdna_hip_programming.md T1): consecutive workgroups go round-robin to the 8
    // XCDs; remapped, each XCD takes a contiguous run of (keypoint chunk, frame), so one frame's
    // chunks -- which all read that frame's band table, right descriptors and pyramid windows --
    // share one L2.  Speed only: any placement is correct.
    const int nwg = (int)(gridDim.x * gridDim.y), orig = (int)(blockIdx.x + gridDim.x * blockIdx.y);
    const int xq = nwg >> 3, xr = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int f = wg / (int)gridDim.x;
    const int iL = (wg - f * (int)gridDim.x) * kMatchThreads + threadIdx.x;
#else
    const int f = blockIdx.y;
    const int iL = blockIdx.x * kMatchThreads + threadIdx.x;
#endif
    if (iL >= G.cap) return;
    const size_t o = (size_t)f * G.cap + iL;
    float ur_out = -1.0f, dep_out = -1.0f;
    int sad_out = -1;
    const int nl = n_l[f];
    if (iL < nl) {
        const slam_keypoint kl = kps_l[o];
        const int levelL = kl.octave;
        const float vL = kl.y, uL = kl.x;
        const int row = (int)vL;
        const int32_t* off = row_off + (size_t)f * (G.nrows + 1);
        const float minZ = G.mb, minD = 0.0f;
        const float maxD = G.mbf / minZ;
        const float minU = uL - maxD, maxU = uL - minD;
        int bestDist = 100, bestIdxR = 0;  // ORBmatcher::TH_HIGH
        if (row >= 0 && row < G.nrows && !(maxU < 0)) {
            const uint4* dl = reinterpret_cast<const uint4*>(desc_l + o * 32);
            const uint4 a0 = dl[0], a1 = dl[1];
            const uint8_t* DR = desc_r + (size_t)f * G.cap * 32;
            const StEnt* E = ent + (size_t)f * G.ent_cap;
            const int c0 = off[row], c1 = off[row + 1];
            // candidates kStCand at a time: their band entries (index, octave, x), then the
            // descriptors of those that pass the octave / u filter, loaded together (two dependent
            // rounds per kStCand candidates)
            for (int c = c0; c < c1; c += kStCand) {
                int iR[kStCand];
                bool ok[kStCand];
#pragma unroll
                for (int q = 0; q < kStCand; q++) {
                    ok[q] = false;
                    iR[q] = -1;
                    if (c + q < c1) {
                        const StEnt en = E[c + q];
                        iR[q] = en.idx;
                        ok[q] = !(en.octave < levelL - 1 || en.octave > levelL + 1) && en.x >= minU && en.x <= maxU;
                    }
                }
                uint4 d0[kStCand], d1[kStCand];
#pragma unroll
                for (int q = 0; q < kStCand; q++)
                    if (ok[q]) {
                        const uint4* dr = reinterpret_cast<const uint4*>(DR + (size_t)iR[q] * 32);
                        d0[q] = dr[0];
                        d1[q] = dr[1];
                    }
#pragma unroll
                for (int q = 0; q < kStCand; q++)
                    if (ok[q]) {
                        const int d = ham32(a0, a1, d0[q], d1[q]);
                        if (d < bestDist || (d == bestDist && d < 100 && iR[q] < bestIdxR)) {
                            bestDist = d;
                            bestIdxR = iR[q];
                        }
                    }
            }
        }
        if (bestDist < 75) {  // thOrbDist = (TH_HIGH + TH_LOW) / 2
            const float uR0 = kps_r[(size_t)f * G.cap + bestIdxR].x;
            const float scaleFactor = G.inv_scale[levelL];
            const float scaleduL = roundf(uL * scaleFactor);
            const float scaledvL = roundf(vL * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const int w = 5, L = 5;
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            const int lw = G.lw[levelL], lh = G.lh[levelL];
            const int vy0 = (int)scaledvL - w, ux0 = (int)scaleduL - w, ur0 = (int)scaleduR0;
            const bool inside = !(iniu < 0 || endu >= lw) && vy0 >= 0 && vy0 + 2 * w + 1 <= lh && ux0 >= 0 &&
                                ux0 + 2 * w + 1 <= lw && ur0 - L - w >= 0 && ur0 + L + w + 1 <= lw;
            if (inside) {
                const int pl = G.pitch[0][levelL], pr = G.pitch[1][levelL];
                const uint8_t* PL = G.base[0][levelL] + f * G.fstride[0][levelL] + (size_t)vy0 * pl + ux0;
                const uint8_t* PR = G.base[1][levelL] + f * G.fstride[1][levelL] + (size_t)vy0 * pr + (ur0 - L - w);
                int acc[2 * L + 1];
#pragma unroll
                for (int k = 0; k < 2 * L + 1; k++) acc[k] = 0;
                // packed form: each row's 11 left and 21 right bytes as aligned dword loads, the
                // eleven window offsets by v_alignbyte, the 11-byte row sums by three v_sad_u8
                // (the 12th byte zeroed on both sides); used when the dword reads stay inside
                // the rows (3 bytes of slack before the pitch), else the byte form
                const bool packed = ux0 + 2 * w + 4 <= pl && ur0 + L + w + 4 <= pr;
                if (packed) {
                    // kSadRows rows' dword loads issued together, then their sums
                    for (int y0 = 0; y0 < 2 * w + 1; y0 += kSadRows) {
                        uint32_t wa[kSadRows][4], wb[kSadRows][7];
                        int sa[kSadRows], sb[kSadRows];
#pragma unroll
                        for (int rr = 0; rr < kSadRows; rr++) {
                            const int yy = min(y0 + rr, 2 * w);
                            const uint8_t* ra = PL + (size_t)yy * pl;
                            const uint8_t* rb = PR + (size_t)yy * pr;
                            const uint32_t* da = reinterpret_cast<const uint32_t*>((uintptr_t)ra & ~(uintptr_t)3);
                            const uint32_t* db = reinterpret_cast<const uint32_t*>((uintptr_t)rb & ~(uintptr_t)3);
                            sa[rr] = (int)((uintptr_t)ra & 3);
                            sb[rr] = (int)((uintptr_t)rb & 3);
#pragma unroll
                            for (int q = 0; q < 4; q++) wa[rr][q] = q * 4 < sa[rr] + 2 * w + 1 ? da[q] : 0u;
#pragma unroll
                            for (int q = 0; q < 7; q++) wb[rr][q] = q * 4 < sb[rr] + 2 * w + 2 * L + 1 ? db[q] : 0u;
                        }
#pragma unroll
                        for (int rr = 0; rr < kSadRows; rr++) {
                            if (y0 + rr > 2 * w) break;
                            const uint32_t A0 = __builtin_amdgcn_alignbyte(wa[rr][1], wa[rr][0], sa[rr]);
                            const uint32_t A1 = __builtin_amdgcn_alignbyte(wa[rr][2], wa[rr][1], sa[rr]);
                            const uint32_t A2 = __builtin_amdgcn_alignbyte(wa[rr][3], wa[rr][2], sa[rr]) & 0x00FFFFFFu;
                            uint32_t Bn[6];  // right bytes 0..23 of the row, dword aligned
#pragma unroll
                            for (int q = 0; q < 6; q++) Bn[q] = __builtin_amdgcn_alignbyte(wb[rr][q + 1], wb[rr][q], sb[rr]);
#pragma unroll
                            for (int k = 0; k < 2 * L + 1; k++) {
                                const int qd = k >> 2, sh = k & 3;
                                const uint32_t B0 = __builtin_amdgcn_alignbyte(Bn[qd + 1], Bn[qd], sh);
                                const uint32_t B1 = __builtin_amdgcn_alignbyte(Bn[qd + 2], Bn[qd + 1], sh);
                                const uint32_t B2 = __builtin_amdgcn_alignbyte(Bn[qd + 3], Bn[qd + 2], sh) & 0x00FFFFFFu;
                                acc[k] = (int)__builtin_amdgcn_sad_u8(A2, B2,
                                                                     __builtin_amdgcn_sad_u8(A1, B1,
                                                                                             __builtin_amdgcn_sad_u8(A0, B0, (uint32_t)acc[k])));
                            }
                        }
                    }
                } else {
                    for (int yy = 0; yy < 2 * w + 1; yy++) {
                        uint8_t a[2 * w + 1], b[2 * w + 2 * L + 1];
#pragma unroll
                        for (int x = 0; x < 2 * w + 1; x++) a[x] = PL[(size_t)yy * pl + x];
#pragma unroll
                        for (int x = 0; x < 2 * w + 2 * L + 1; x++) b[x] = PR[(size_t)yy * pr + x];
#pragma unroll
                        for (int k = 0; k < 2 * L + 1; k++)
#pragma unroll
                            for (int x = 0; x < 2 * w + 1; x++) acc[k] += abs((int)a[x] - (int)b[k + x]);
                    }
                }
                int bestDist2 = INT_MAX, bestk = 0;
                float vd[2 * L + 1];
#pragma unroll
                for (int k = 0; k < 2 * L + 1; k++) {
                    const float dist = (float)acc[k];
                    if (dist < (float)bestDist2) {
                        bestDist2 = (int)dist;
                        bestk = k;
                    }
                    vd[k] = dist;
                }
                const int bestincR = bestk - L;
                if (bestincR != -L && bestincR != L) {
                    float dist1 = 0, dist2 = 0, dist3 = 0;
#pragma unroll
                    for (int k = 1; k < 2 * L; k++)
                        if (k == bestk) {
                            dist1 = vd[k - 1];
                            dist2 = vd[k];
                            dist3 = vd[k + 1];
                        }
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = G.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {
                            if (disparity <= 0) {
                                disparity = (float)0.01;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            dep_out = G.mbf / disparity;
                            ur_out = bestuR;
                            sad_out = bestDist2;
                        }
                    }
                }
            }
        }
    }
    uright[o] = ur_out;
    depth[o] = dep_out;
    sad[o] = sad_out;
}

#ifndef SLAMHOT_ST_SELECT
#define SLAMHOT_ST_SELECT 1
#endif

// The (m/2)-th smallest of keys[0..m) — the element std::sort would put at m/2
// (Frame.cc:950-951) — by MSD radix select: 8 bits per pass from the highest non-zero byte
// of the maximum (SADs of an 11 x 11 window fit 15 bits: two passes), a 256-bin LDS
// histogram per pass, one wave scans it.  Replaces a full bitonic sort (55 barriers at 1024).
__device__ __forceinline__ uint32_t radix_select_mid(const uint32_t* keys, int m, uint32_t vmax, uint32_t* hist,
                                                     uint32_t* s_sel, int t) {
    const uint32_t kth = (uint32_t)(m / 2);
    if (vmax == 0) return 0;
    const int top = 31 - __builtin_clz(vmax);
    uint32_t prefix = 0, mask = 0, k = kth;
    for (int shift = (top / 8) * 8; shift >= 0; shift -= 8) {
        if (t < 256) hist[t] = 0;
        __syncthreads();
        for (int i = t; i < m; i += kMedianThreads) {
            const uint32_t v = keys[i];
            if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (t < 64) {
            const uint32_t h0 = hist[4 * t], h1 = hist[4 * t + 1], h2 = hist[4 * t + 2], h3 = hist[4 * t + 3];
            const uint32_t own = h0 + h1 + h2 + h3;
            uint32_t inc = own;  // inclusive scan over the wave
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (t >= o) inc += y;
            }
            uint32_t before = inc - own;
            if (k >= before && k < inc) {  // exactly one lane holds the k-th
                uint32_t b = 4 * t, c = before;
                if (k >= c + h0) { c += h0; b++;
                    if (k >= c + h1) { c += h1; b++;
                        if (k >= c + h2) { c += h2; b++; } } }
                s_sel[0] = b;
                s_sel[1] = k - c;
            }
        }
        __syncthreads();
        prefix |= s_sel[0] << shift;
        mask |= 255u << shift;
        k = s_sel[1];
        __syncthreads();  // s_sel and hist are rewritten by the next pass
    }
    return prefix;
}

__global__ void __launch_bounds__(kMedianThreads) k_stereo_median(int cap, const int32_t* n_l, const int32_t* sad,
                                                                 float* uright, float* depth) {
    __shared__ uint32_t keys[kStMaxSort];
    __shared__ uint32_t hist[256], s_sel[2];
    __shared__ int count;
    __shared__ uint32_t s_max;
    const int f = blockIdx.x, t = threadIdx.x;
    const int n = n_l[f];
    const int32_t* S = sad + (size_t)f * cap;
    if (t == 0) {
        count = 0;
        s_max = 0;
    }
    __syncthreads();
    uint32_t vmax = 0;
    for (int i = t; i < n; i += kMedianThreads) {
        const int v = S[i];
        if (v >= 0) {
            keys[atomicAdd(&count, 1)] = (uint32_t)v;
            vmax = max(vmax, (uint32_t)v);
        }
    }
    if (SLAMHOT_ST_SELECT) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
        if ((t & 63) == 0) atomicMax(&s_max, vmax);
    }
    __syncthreads();
    const int m = count;
    if (m == 0) return;  // the reference reads vDistIdx[0] of an empty vector here
    uint32_t mid;
    if (SLAMHOT_ST_SELECT) {
        mid = radix_select_mid(keys, m, s_max, hist, s_sel, t);
    } else {
        int np = 1;
        while (np < m) np <<= 1;
        for (int i = m + t; i < np; i += kMedianThreads) keys[i] = 0xFFFFFFFFu;
        __syncthreads();
        for (int k = 2; k <= np; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = t; i < np; i += kMedianThreads) {
                    const int p = i ^ j;
                    if (p > i) {
                        const uint32_t x = keys[i], y = keys[p];
                        const bool up = (i & k) == 0;
                        if ((x > y) == up) {
                            keys[i] = y;
                            keys[p] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        mid = keys[m / 2];
    }
    const float median = (float)(int)mid;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = t; i < n; i += kMedianThreads) {
        const int v = S[i];
        if (v >= 0 && !((float)v < thDist)) {
            uright[(size_t)f * cap + i] = -1.0f;
            depth[(size_t)f * cap + i] = -1.0f;
        }
    }
}

}  // namespace
}  // namespace slamhot

using namespace slamhot;

struct slam_stereo {
    int device = 0;
    hipStream_t stream = nullptr;
    void *d_rowoff = nullptr, *d_ent = nullptr, *d_sad = nullptr, *d_io = nullptr;
    size_t cap_rowoff = 0, cap_ent = 0, cap_sad = 0, cap_io = 0;
};

namespace {
slam_status grow(void** p, size_t* cap, size_t need) {
    if (need <= *cap) return SLAM_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, need) != hipSuccess) return SLAM_ENOMEM;
    *cap = need;
    return SLAM_OK;
}
}  // namespace

extern "C" {

slam_status slamhot_stereo_create(int device, slam_stereo** out) {
    if (!out) return SLAM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= n) return SLAM_EINVAL;
    slam_stereo* st = new (std::nothrow) slam_stereo();
    if (!st) return SLAM_ENOMEM;
    st->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess) {
        delete st;
        return SLAM_EHIP;
    }
    *out = st;
    return SLAM_OK;
}

void slamhot_stereo_destroy(slam_stereo* st) {
    if (!st) return;
    (void)hipSetDevice(st->device);
    if (st->stream) (void)hipStreamSynchronize(st->stream);
    for (void* p : {st->d_rowoff, st->d_ent, st->d_sad, st->d_io})
        if (p) (void)hipFree(p);
    if (st->stream) (void)hipStreamDestroy(st->stream);
    delete st;
}

slam_status slamhot_stereo_match_batch_device(slam_stereo* st, slam_extractor* left, slam_extractor* right,
                                              int nframes, const void* d_kps_left, const void* d_desc_left,
                                              const void* d_n_left, const void* d_kps_right,
                                              const void* d_desc_right, const void* d_n_right, int cap,
                                              float mbf, float mb, void* d_uright, void* d_depth, void* d_sad,
                                              void* hip_stream) {
    if (!st || !left || !right || nframes < 0 || cap <= 0 || cap > 65535 || !d_kps_left || !d_desc_left ||
        !d_n_left || !d_kps_right || !d_desc_right || !d_n_right || !d_uright || !d_depth)
        return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    if (cap > kStMaxSort) return SLAM_EINVAL;
    StereoGeom G{};
    float sc[kStMaxLevels], isc[kStMaxLevels];
    int nl = 0;
    if (slamhot_extractor_levels(left, &nl, sc, isc, nullptr, nullptr, nullptr) != SLAM_OK || nl < 1 ||
        nl > kStMaxLevels)
        return SLAM_EINVAL;
    G.nlevels = nl;
    for (int side = 0; side < 2; side++) {
        slam_extractor* ex = side ? right : left;
        for (int l = 0; l < nl; l++) {
            const void* p0 = nullptr;
            const void* p1 = nullptr;
            int pitch = 0, w = 0, h = 0, pitch1 = 0, w1 = 0, h1 = 0;
            if (slamhot_pyramid_level_device(ex, 0, l, &p0, &pitch, &w, &h) != SLAM_OK) return SLAM_EINVAL;
            if (nframes > 1) {
                if (slamhot_pyramid_level_device(ex, nframes - 1, l, &p1, &pitch1, &w1, &h1) != SLAM_OK)
                    return SLAM_EINVAL;  // fewer frames extracted than requested
                // frames of one batch are evenly spaced
                G.fstride[side][l] = ((const uint8_t*)p1 - (const uint8_t*)p0) / (nframes - 1);
            }
            G.base[side][l] = (const uint8_t*)p0;
            G.pitch[side][l] = pitch;
            if (side == 0) {
                G.lw[l] = w;
                G.lh[l] = h;
            } else if (w != G.lw[l] || h != G.lh[l]) {
                return SLAM_EINVAL;  // left and right images must share a geometry
            }
        }
    }
    for (int l = 0; l < nl; l++) {
        G.scale[l] = sc[l];
        G.inv_scale[l] = isc[l];
    }
    G.nrows = G.lh[0];
    if (G.nrows > kStMaxRows) return SLAM_EINVAL;
    // rows one right keypoint can cover: ceil(y + r) - floor(y - r) + 1 <= 4 * scale_max + 3
    G.ent_cap = cap * ((int)std::ceil(4.0f * sc[nl - 1]) + 3);
    G.cap = cap;
    G.mbf = mbf;
    G.mb = mb;
    (void)hipSetDevice(st->device);
    slam_status s;
    if ((s = grow(&st->d_rowoff, &st->cap_rowoff, (size_t)nframes * (G.nrows + 1) * sizeof(int32_t))) ||
        (s = grow(&st->d_ent, &st->cap_ent, (size_t)nframes * G.ent_cap * sizeof(StEnt))))
        return s;
    int32_t* sad = (int32_t*)d_sad;
    if (!sad) {
        if ((s = grow(&st->d_sad, &st->cap_sad, (size_t)nframes * cap * sizeof(int32_t)))) return s;
        sad = (int32_t*)st->d_sad;
    }
    hipStream_t strm = hip_stream ? (hipStream_t)hip_stream : st->stream;
    hipLaunchKernelGGL(k_stereo_rows, dim3(nframes), dim3(kRowsThreads), 0, strm, G,
                       (const slam_keypoint*)d_kps_right, (const int32_t*)d_n_right, (int32_t*)st->d_rowoff,
                       (StEnt*)st->d_ent);
    hipLaunchKernelGGL(k_stereo_match, dim3((cap + kMatchThreads - 1) / kMatchThreads, nframes), dim3(kMatchThreads),
                       0, strm, G, (const slam_keypoint*)d_kps_left, (const uint8_t*)d_desc_left,
                       (const int32_t*)d_n_left, (const slam_keypoint*)d_kps_right, (const uint8_t*)d_desc_right,
                       (const int32_t*)st->d_rowoff, (const StEnt*)st->d_ent, (float*)d_uright, (float*)d_depth,
                       sad);
    hipLaunchKernelGGL(k_stereo_median, dim3(nframes), dim3(kMedianThreads), 0, strm, cap,
                       (const int32_t*)d_n_left, (const int32_t*)sad, (float*)d_uright, (float*)d_depth);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

slam_status slamhot_compute_stereo_matches(slam_stereo* st, slam_extractor* left, slam_extractor* right, int n_left,
                                           const slam_keypoint* kps_left, const uint8_t* desc_left, int n_right,
                                           const slam_keypoint* kps_right, const uint8_t* desc_right, float mbf,
                                           float mb, float* uright, float* depth) {
    if (!st || !left || !right || n_left < 0 || n_right < 0 || (n_left && (!kps_left || !desc_left || !uright ||
                                                                             !depth)) ||
        (n_right && (!kps_right || !desc_right)))
        return SLAM_EINVAL;
    if (n_left == 0) return SLAM_OK;
    const int cap = std::max(std::max(n_left, n_right), 1);
    if (cap > kStMaxSort) return SLAM_EINVAL;
    // one upload: [n_l, n_r | kps L | kps R | desc L | desc R | uright | depth], cap rows each
    const size_t kb = (size_t)cap * sizeof(slam_keypoint), db = (size_t)cap * 32, fb = (size_t)cap * 4;
    const size_t o_kl = 256, o_kr = o_kl + kb, o_dl = o_kr + kb, o_dr = o_dl + db, o_ur = o_dr + db, o_dp = o_ur + fb;
    (void)hipSetDevice(st->device);
    slam_status s;
    if ((s = grow(&st->d_io, &st->cap_io, o_dp + fb))) return s;
    uint8_t* b = (uint8_t*)st->d_io;
    const int32_t ns[2] = {n_left, n_right};
    hipStream_t S = st->stream;
    SLAM_HIP_TRY(hipMemcpyAsync(b, ns, sizeof(ns), hipMemcpyHostToDevice, S));
    SLAM_HIP_TRY(hipMemcpyAsync(b + o_kl, kps_left, (size_t)n_left * sizeof(slam_keypoint), hipMemcpyHostToDevice, S));
    SLAM_HIP_TRY(hipMemcpyAsync(b + o_dl, desc_left, (size_t)n_left * 32, hipMemcpyHostToDevice, S));
    if (n_right) {
        SLAM_HIP_TRY(hipMemcpyAsync(b + o_kr, kps_right, (size_t)n_right * sizeof(slam_keypoint), hipMemcpyHostToDevice,
                                    S));
        SLAM_HIP_TRY(hipMemcpyAsync(b + o_dr, desc_right, (size_t)n_right * 32, hipMemcpyHostToDevice, S));
    }
    s = slamhot_stereo_match_batch_device(st, left, right, 1, b + o_kl, b + o_dl, b, b + o_kr, b + o_dr, b + 4, cap,
                                          mbf, mb, b + o_ur, b + o_dp, nullptr, S);
    if (s != SLAM_OK) return s;
    SLAM_HIP_TRY(hipMemcpyAsync(uright, b + o_ur, (size_t)n_left * 4, hipMemcpyDeviceToHost, S));
    SLAM_HIP_TRY(hipMemcpyAsync(depth, b + o_dp, (size_t)n_left * 4, hipMemcpyDeviceToHost, S));
    SLAM_HIP_TRY(hipStreamSynchronize(S));
    return SLAM_OK;
}

}  // extern "C"
