// extractor.hip — MI355X (gfx950) ORB extractor: the device side of
// ORBextractor::operator() (ORBextractor.cc:1068-1150), batched over frames.
//
// Pipeline per batch (one stream):
//   k_resize4     x (L-1)  chained INTER_LINEAR pyramid            ComputePyramid :1152
//   k_fast_wave   x 1      FAST-9 score + per-cell 3x3 NMS, 1 wave/cell ComputeKeyPointsOctTree :787-853
//   k_fast_cells  x 1      the same for cells wider than one wave (1 WG/cell)
//   k_octree      x 2      quadtree distribution, 1 wave/(frame,lvl) DistributeOctTree :537-761
//   k_layout      x 1      lapping-area output order, 1 WG/frame   operator() :1100-1146
//   k_orb3        x 1      IC angle + 7x7 blur window + rBRIEF,    IC_Angle :75, GaussianBlur :1115,
//                          one wave per kp                         computeOrbDescriptor :106
//
// Data layout in HBM (per handle, batch-major): input frames (level 0, tight rows); pyramid
// levels 1.. per frame, rows padded to 64 B (no blurred copy: k_orb3 blurs windows); per-cell candidate
// slots; per-(frame,level) octree keypoints; per-frame output index map.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "device_math.hpp"
#include "extractor_plan.hpp"

namespace slamhot {

constexpr int kPattern[256 * 4] = {
#include "orb_pattern.inc"
};
// the pattern's point pairs (x0, y0, x1, y1) of bit i packed as four int8 in one dword (every
// coordinate is in [-13, 12]): one load per bit instead of four
struct Pattern8 {
    uint32_t v[256];
};
constexpr Pattern8 make_pattern8() {
    Pattern8 p{};
    for (int i = 0; i < 256; i++)
        p.v[i] = (uint32_t)(uint8_t)kPattern[4 * i] | ((uint32_t)(uint8_t)kPattern[4 * i + 1] << 8) |
                 ((uint32_t)(uint8_t)kPattern[4 * i + 2] << 16) | ((uint32_t)(uint8_t)kPattern[4 * i + 3] << 24);
    return p;
}
__constant__ Pattern8 c_pattern8 = make_pattern8();
// the pattern's point pairs as floats (x0, y0, x1, y1) of bit i: k_orb3 loads one float4 per
// bit and rotates with packed f32 math, no int8 unpacking per sample
struct PatternF {
    float4 v[256];
};
constexpr PatternF make_patternf() {
    PatternF p{};
    for (int i = 0; i < 256; i++)
        p.v[i] = float4{(float)kPattern[4 * i], (float)kPattern[4 * i + 1], (float)kPattern[4 * i + 2],
                        (float)kPattern[4 * i + 3]};
    return p;
}
__constant__ PatternF c_patternf = make_patternf();

// Device copy of the plan (uploaded once per geometry).
struct DevLevel {
    int w, h, pitch;
    int64_t pyr_off, blur_off;
    int minBX, minBY, maxBX, maxBY;
    int cell_begin, cell_end;
    int nfeat, kbase, kcap, key_base, key_cap;
    float scale, size;
    int nIni;
    int root_x0[kMaxRoots], root_x1[kMaxRoots], root_first_x[kMaxRoots];
    int xtab_off, ytab_off, xmax;
};

// k_orb3's per-level fields, 48 bytes: lane k of a wave reads level k's in three 16-byte loads
struct OrbLv {
    int kbase, w, h, pitch;  // first keypoint slot (INT_MAX past the last level), level geometry
    int64_t off, fstride;    // level bytes: base (Bufs img for level 0, else pyr) + f * fstride + off
    float scale, size;
    int pad[2];
};
static_assert(sizeof(OrbLv) == 48, "three 16-byte loads");

struct DevPlan {
    int nlevels, W, H;
    int ncells, slot_cap, kslots, key_slots, max_nodes;
    int ini_th, min_th;
    int64_t pyr_frame, blur_frame;
    int umax[kHalfPatch + 1];
    DevLevel lv[kMaxLevels];
    OrbLv orb_lv[kMaxLevels];
    // k_orb3's IC_Angle weights (see there), per (staging shift sh, |v| (16: no row), half):
    // [0, 5) the disc-byte masks (1 per byte inside |u| <= umax[|v|]) of the lane's five
    // staged dwords, [5, 10) the same bytes weighted by their byte offset, [10, 12) zero
    uint32_t ic_w[4][kHalfPatch + 2][2][12];
};

// Buffers of one batch launch (device pointers).
struct Bufs {
    const uint8_t* img;     // level 0 frames, tight rows (W bytes)
    uint8_t* pyr;           // levels >= 1, per frame pyr_frame bytes
    uint32_t* cell_keys;    // per frame ncells*slot_cap packed candidates
    int32_t* cell_cnt;      // per frame ncells
    uint32_t* keys_g;       // per frame key_slots (octree overflow scratch: keys)
    uint16_t* knode_g;      // per frame key_slots (octree overflow scratch: node ids)
    uint32_t* okp;          // per frame kslots packed octree keypoints (level coords)
    int32_t* ocnt;          // per frame nlevels octree counts
    int32_t* oidx;          // per frame kslots final output index
    int32_t* err;           // per frame error flags
    slam_keypoint* out_kps; // per frame cap
    uint8_t* out_desc;      // per frame cap*32
    int32_t* out_n;         // per frame
    int32_t* out_mono;      // per frame
    const ResizeX* xtab;
    const ResizeY* ytab;
    const CellDesc* cells;
    const DevPlan* plan;
    int kslots, nlevels;       // = plan->kslots / nlevels, at hand in the kernel arguments
    int nframes, cap, lap0, lap1;
};

__device__ __forceinline__ const uint8_t* level_ptr(const Bufs& b, const DevPlan& P, int f, int l) {
    if (l == 0) return b.img + (size_t)f * P.H * P.W;
    return b.pyr + (size_t)f * P.pyr_frame + P.lv[l].pyr_off;
}
__device__ __forceinline__ int level_pitch(const DevPlan& P, int l) {
    return l == 0 ? P.W : P.lv[l].pitch;
}

// packed u16 pairs (v_pk_*_u16) for the SWAR FAST pre-test
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
// XCD-aware workgroup order (MI355X_MICROARCH.md, Workgroup dispatch / XCD placement; guide T1):
// the dispatcher deals workgroups round-robin over the 8 XCDs, each with its own L2, so
// consecutive workgroups -- neighbouring cells / keypoints of one frame, whose windows overlap --
// land on 8 different L2s and each fetches the shared rows from HBM.  This bijective remap of the
// (x, y) grid gives every XCD one contiguous run of it (a few whole frames), so the overlapping
// windows of a frame are fetched once into one L2.  Speed only: any placement is correct.
#ifndef SLAMHOT_NO_XCD_REMAP
__device__ __forceinline__ int2 xcd_block() {
    const int gx = gridDim.x, nwg = gridDim.x * gridDim.y;
    const int orig = blockIdx.x + gx * blockIdx.y;
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    return int2{wg % gx, wg / gx};
}
#else
__device__ __forceinline__ int2 xcd_block() { return int2{(int)blockIdx.x, (int)blockIdx.y}; }
#endif

__device__ __forceinline__ us2 as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }
__device__ __forceinline__ uint32_t as_u32(us2 x) { return __builtin_bit_cast(uint32_t, x); }

// Sum over the wave, result in every lane: DPP within rows of 16 (quad_perm xor 1 / 2,
// half-row and row mirrors: VALU-speed, no LDS crossbar), then the four row sums by
// v_readlane (a __shfl_xor butterfly is six dependent ds_bpermute round trips).
__device__ __forceinline__ int wave_sum_dpp(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);  // row_mirror
    return __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) + __builtin_amdgcn_readlane(x, 32) +
           __builtin_amdgcn_readlane(x, 48);
}

// acc + number of set bits of m below this lane (v_mbcnt_lo/hi)
__device__ __forceinline__ int mbcnt64(uint64_t m, int acc) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)acc));
}

// packed candidate / keypoint: x (12 b) | y (12 b) | score (8 b)
__device__ __forceinline__ uint32_t pack_kp(int x, int y, int s) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
__device__ __forceinline__ int kp_x(uint32_t k) { return (int)(k & 0xFFF); }
__device__ __forceinline__ int kp_y(uint32_t k) { return (int)((k >> 12) & 0xFFF); }
__device__ __forceinline__ int kp_s(uint32_t k) { return (int)(k >> 24); }

// Stage nrows x ndw dwords (row pitch spitch bytes, 4-aligned) into LDS (row stride dstride
// dwords): K independent loads per thread are in flight before their LDS stores.
__device__ __forceinline__ void split_rc(int i, int ndw, float inv, int& r, int& c) {
    r = (int)(((float)i + 0.5f) * inv);
    c = i - r * ndw;
    if (c < 0) { r--; c += ndw; } else if (c >= ndw) { r++; c -= ndw; }
}

template <int K>
__device__ __forceinline__ void stage_u32(uint32_t* dst, int dstride, const uint8_t* src, size_t spitch,
                                          int nrows, int ndw) {
    const int total = nrows * ndw;
    const float inv = 1.0f / (float)ndw;
    for (int base = 0; base < total; base += blockDim.x * K) {
        uint32_t v[K];
        int d[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int i = base + k * blockDim.x + threadIdx.x;
            d[k] = -1;
            if (i < total) {
                int r, c;
                split_rc(i, ndw, inv, r, c);
                v[k] = *reinterpret_cast<const uint32_t*>(src + (size_t)r * spitch + 4 * c);
                d[k] = r * dstride + c;
            }
        }
#pragma unroll
        for (int k = 0; k < K; k++)
            if (d[k] >= 0) dst[d[k]] = v[k];
    }
}




// ---------------------------------------------------------------------------------------
// k_resize4: cv::resize INTER_LINEAR (OpenCV 4.2.0 fixed point 2^11) from the host plan's
// coefficient tables (extractor_plan.hpp build_resize_tables, the reference's own arithmetic).
// Thread = 4 output columns x kRzRows output rows: its four columns are two 16-byte table loads
// and each row one (per-level tables padded to a multiple of 4).  An early version gathered the
// entries one by one per pixel and was bound by it (microbench 199 -> 74 us at L1 when the
// coefficients were recomputed per thread in FP64 instead); the quad loads replace that
// per-thread FP64 math (round 5: stage 0.131 -> 0.126 ms per batch).  A source row loaded for
// output row y is reused for row y+1 when its vertical pair starts there (scale 1.2: most rows).
// ---------------------------------------------------------------------------------------
#ifndef SLAMHOT_RZ_ROWS
#define SLAMHOT_RZ_ROWS 4
#endif
constexpr int kRzRows = SLAMHOT_RZ_ROWS;  // output rows per thread (the y table is padded to 8)
static_assert(8 % kRzRows == 0, "the plan pads each level's y table to a multiple of 8 rows");

__global__ void __launch_bounds__(256) k_resize4(Bufs b, int l) {
    const DevPlan& P = *b.plan;
    const DevLevel& L = P.lv[l];
    const DevLevel& S = P.lv[l - 1];
    const int qw = (L.w + 3) >> 2;
    const int nrb = (L.h + kRzRows - 1) / kRzRows;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * nrb) return;
    const int rb = i / qw, q = i - rb * qw;
    const uint8_t* src = level_ptr(b, P, f, l - 1);
    const int spitch = level_pitch(P, l - 1);
    // the four columns' (sx, a0, a1) from the level's coefficient table (the host plan's
    // OpenCV arithmetic, padded per level so a quad is two 16-byte loads; columns past the edge
    // repeat the last one, as the clamped dx did): no per-thread FP64 coefficient math
    int sxs[4], a0s[4], a1s[4];
    {
        const uint4* xq = reinterpret_cast<const uint4*>(b.xtab + L.xtab_off + 4 * q);
        const uint4 x01 = xq[0], x23 = xq[1];
        const uint32_t sx4[4] = {x01.x, x01.z, x23.x, x23.z}, aa4[4] = {x01.y, x01.w, x23.y, x23.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            sxs[k] = (int)sx4[k];
            a0s[k] = (int)(aa4[k] & 0xFFFF);
            a1s[k] = (int)(aa4[k] >> 16);
        }
    }
    // the thread's rows: (y0, y1, b0 | b1 << 16) per output row, one 16-byte load each
    const uint4* yq = reinterpret_cast<const uint4*>(b.ytab + L.ytab_off) + rb * kRzRows;
    // horizontal pass of one source row (HResizeLinear): D[k] = S[sx]*a0 + S[sx+1]*a1.
    // Dword form: the thread's eight source bytes sx_k, sx_k + 1 lie in the 12 bytes from
    // xb = sx_0 & ~3 when sx_3 + 1 - xb <= 11 (scale factors up to ~2.5): three dword buffer loads
    // per row instead of eight byte loads (the byte loads bound the kernel's memory pipeline), each
    // pair (S[sx], S[sx+1]) gathered by one v_perm into a u16 pair for one v_dot2 with (a0, a1).
    // The resource spans the source level of this frame, so the few bytes read past its last row
    // (weight 0 or unused) come back as zero.  Otherwise (pitch not a multiple of 4, wider
    // spans) the byte loads.
    const int xb = sxs[0] & ~3;
    const bool dw = ((spitch & 3) == 0) && (sxs[3] + 1 - xb <= 11);
    uint32_t selp[4], hiw[4];
    us2 coef[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int o = sxs[k] - xb;              // 0 .. 10
        const int w = o >= 4 ? 1 : 0;           // window {w[w+1], w[w]} holds bytes o, o + 1 (o - 4w <= 6)
        const int ob = o - 4 * w;
        selp[k] = 0x0c000c00u | (uint32_t)ob | ((uint32_t)(ob + 1) << 16);  // [S[sx], 0, S[sx+1], 0]
        hiw[k] = (uint32_t)w;
        coef[k] = us2{(unsigned short)a0s[k], (unsigned short)a1s[k]};
    }
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)src, (short)0, __builtin_amdgcn_readfirstlane(S.h * spitch), 0x00020000);
    auto hrow = [&](int y, int* d) {
        const int yc = min(max(y, 0), S.h - 1);
        if (dw) {
            const int off = yc * spitch + xb;
            const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
            const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, 0);
            const uint32_t w2 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 8, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t lo = hiw[k] ? w1 : w0, hi = hiw[k] ? w2 : w1;
                d[k] = (int)__builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(hi, lo, selp[k])), coef[k], 0u, false);
            }
        } else {
            const uint8_t* r = src + (size_t)yc * spitch;
            int p0[4], p1[4];
#pragma unroll
            for (int k = 0; k < 4; k++) { p0[k] = r[sxs[k]]; p1[k] = r[sxs[k] + 1]; }
#pragma unroll
            for (int k = 0; k < 4; k++) d[k] = __mul24(p0[k], a0s[k]) + __mul24(p1[k], a1s[k]);
        }
    };
    uint8_t* dbase = b.pyr + (size_t)f * P.pyr_frame + L.pyr_off + 4 * q;
    if (dw) {
        // Every source row of the thread's output rows first: both rows of each output row, 24
        // independent dword loads in flight (the level tables are padded to whole row blocks, so
        // rows past the level's last read copies of it), then the products and the stores.  The
        // store of one output row no longer sits between the loads of the next (the source and the
        // destination levels share the pyramid allocation, so the compiler could not hoist them).
        uint4 yt[kRzRows];
#pragma unroll
        for (int rr = 0; rr < kRzRows; rr++) yt[rr] = yq[rr];
        uint32_t w[kRzRows][2][3];
#pragma unroll
        for (int rr = 0; rr < kRzRows; rr++)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int off = (int)(s ? yt[rr].y : yt[rr].x) * spitch + xb;  // rows clamped by the plan
#pragma unroll
                for (int t = 0; t < 3; t++) w[rr][s][t] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4 * t, 0, 0);
            }
        const int nr = min(kRzRows, L.h - rb * kRzRows);
#pragma unroll
        for (int rr = 0; rr < kRzRows; rr++) {
            const int b0 = (int)(yt[rr].z & 0xFFFF), b1 = (int)(yt[rr].z >> 16);
            uint32_t word = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t lo0 = hiw[k] ? w[rr][0][1] : w[rr][0][0], hi0 = hiw[k] ? w[rr][0][2] : w[rr][0][1];
                const uint32_t lo1 = hiw[k] ? w[rr][1][1] : w[rr][1][0], hi1 = hiw[k] ? w[rr][1][2] : w[rr][1][1];
                const int d0 = (int)__builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(hi0, lo0, selp[k])), coef[k], 0u, false);
                const int d1 = (int)__builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(hi1, lo1, selp[k])), coef[k], 0u, false);
                const int v = ((__mul24(b0, d0 >> 4) >> 16) + (__mul24(b1, d1 >> 4) >> 16) + 2) >> 2;
                word |= (uint32_t)(v & 0xFF) << (8 * k);
            }
            if (rr < nr) *reinterpret_cast<uint32_t*>(dbase + (size_t)(rb * kRzRows + rr) * L.pitch) = word;
        }
        return;
    }
    int D0[4], D1[4];
    int have = INT_MIN;  // source row currently held in D1 (INT_MIN: none)
#pragma unroll
    for (int rr = 0; rr < kRzRows; rr++) {
        const int dy = rb * kRzRows + rr;
        if (dy >= L.h) break;
        // rows are clamped (VResizeLinear reads clip(sy+k, 0, h-1)); reuse by clamped index
        const uint4 yt = yq[rr];
        const int y0 = (int)yt.x, y1 = (int)yt.y;
        const int b0 = (int)(yt.z & 0xFFFF), b1 = (int)(yt.z >> 16);
        if (have == y0) {
#pragma unroll
            for (int k = 0; k < 4; k++) D0[k] = D1[k];
        } else {
            hrow(y0, D0);
        }
        hrow(y1, D1);
        have = y1;
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int v = ((__mul24(b0, D0[k] >> 4) >> 16) + (__mul24(b1, D1[k] >> 4) >> 16) + 2) >> 2;
            word |= (uint32_t)(v & 0xFF) << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(dbase + (size_t)dy * L.pitch) = word;
    }
}

// ---------------------------------------------------------------------------------------
// FAST-9/16 corner measure (OpenCV 4.2.0 FAST_t<16> + cornerScore<16>, closed form).
// For centre v and circle p[0..15], d_k = v - p_k.  With window minima/maxima over the 16
// circular windows of 9:  Mdark = max_s min(d[s..s+8]),  Mbright = -min_s max(d[s..s+8]),
// M = max(Mdark, Mbright).  The pixel is a FAST corner at threshold t iff M > t, and then
// cornerScore<16>(t) = M - 1 (independent of t; the early-outs of the reference loop only
// prune).  M <= 0 is stored as 0 (not a corner at any t >= 0).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int fast_measure(const uint8_t* c, int stride, int tlow) {
    const int v = c[0];
    int p[16];
    p[0] = c[3 * stride];
    p[1] = c[3 * stride + 1];
    p[2] = c[2 * stride + 2];
    p[3] = c[stride + 3];
    p[4] = c[3];
    p[5] = c[-stride + 3];
    p[6] = c[-2 * stride + 2];
    p[7] = c[-3 * stride + 1];
    p[8] = c[-3 * stride];
    p[9] = c[-3 * stride - 1];
    p[10] = c[-2 * stride - 2];
    p[11] = c[-stride - 3];
    p[12] = c[-3];
    p[13] = c[stride - 3];
    p[14] = c[2 * stride - 2];
    p[15] = c[3 * stride - 1];
    // corner test at the lowest threshold: 9 contiguous darker or brighter
    uint32_t dk = 0, br = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        dk |= (uint32_t)(p[k] < v - tlow) << k;
        br |= (uint32_t)(p[k] > v + tlow) << k;
    }
    uint32_t a = dk | (dk << 16), bb = br | (br << 16);
    uint32_t ra = a, rb = bb;
#pragma unroll
    for (int s = 1; s < 9; s++) {
        ra &= a >> s;
        rb &= bb >> s;
    }
    if (((ra | rb) & 0xFFFFu) == 0) return 0;
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = v - p[k];
    int m2[16], x2[16];
#pragma unroll
    for (int s = 0; s < 16; s++) {
        m2[s] = min(d[s], d[(s + 1) & 15]);
        x2[s] = max(d[s], d[(s + 1) & 15]);
    }
    int m4[16], x4[16];
#pragma unroll
    for (int s = 0; s < 16; s++) {
        m4[s] = min(m2[s], m2[(s + 2) & 15]);
        x4[s] = max(x2[s], x2[(s + 2) & 15]);
    }
    int mdark = -1000, mbr = 1000;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const int mn9 = min(min(m4[s], m4[(s + 4) & 15]), d[(s + 8) & 15]);
        const int mx9 = max(max(x4[s], x4[(s + 4) & 15]), d[(s + 8) & 15]);
        mdark = max(mdark, mn9);
        mbr = min(mbr, mx9);
    }
    const int M = max(mdark, -mbr);
    return M > 0 ? M : 0;
}

// ---------------------------------------------------------------------------------------
// k_fast_cells: one workgroup per (cell, frame).  The cell ROI [iniY,maxY)x[iniX,maxX) is
// exactly what the reference hands cv::FAST (ORBextractor.cc:808); its tested pixels are
// rows/cols 3..size-4, and NMS compares against 0 outside them (cell-local NMS).  The
// second threshold is used only when the first yields no keypoint after NMS (:825-841).
// Output: candidates in row-major order, packed with LEVEL coordinates.
// ---------------------------------------------------------------------------------------
constexpr int kCellMaxW = 80, kCellMaxH = 80;

__global__ void __launch_bounds__(256) k_fast_cells(Bufs b, const int32_t* list) {
    __shared__ uint8_t roi[kCellMaxH * kCellMaxW];
    __shared__ uint8_t meas[kCellMaxH * kCellMaxW];
    __shared__ int scratch[20];
    const DevPlan& P = *b.plan;
    const int f = blockIdx.y;
    const CellDesc cd = b.cells[list[blockIdx.x]];
    const int l = cd.level;
    const uint8_t* img = level_ptr(b, P, f, l);
    const int pitch = level_pitch(P, l);
    const int cw = cd.cw, ch = cd.ch;
    // stage the ROI (row stride cw in LDS)
    for (int i = threadIdx.x; i < cw * ch; i += blockDim.x) {
        const int r = i / cw, c = i - r * cw;
        roi[i] = img[(size_t)(cd.iniY + r) * pitch + cd.iniX + c];
    }
    __syncthreads();
    const int tw = cw - 6, th = ch - 6;
    const int npx = (tw > 0 && th > 0) ? tw * th : 0;
    const int ti = min(max(P.ini_th, 0), 255), tm = min(max(P.min_th, 0), 255);
    const int tlow = min(ti, tm);
    const int per = (npx + blockDim.x - 1) / blockDim.x;
    const int p0 = threadIdx.x * per, p1 = min(npx, p0 + per);
    for (int i = p0; i < p1; i++) {
        const int r = i / tw, c = i - r * tw;
        meas[i] = (uint8_t)fast_measure(&roi[(r + 3) * cw + c + 3], cw, tlow);
    }
    __syncthreads();
    // NMS at threshold t: corner iff M > t, score M-1; neighbours that are not corners at t
    // (or lie outside the tested region) count as 0.
    auto keep = [&](int i, int t) -> bool {
        const int M = meas[i];
        if (M <= t) return false;
        const int s = M - 1;
        const int r = i / tw, c = i - r * tw;
#pragma unroll
        for (int dr = -1; dr <= 1; dr++) {
#pragma unroll
            for (int dc = -1; dc <= 1; dc++) {
                if (!dr && !dc) continue;
                const int rr = r + dr, cc = c + dc;
                if (rr < 0 || rr >= th || cc < 0 || cc >= tw) continue;
                const int Mn = meas[rr * tw + cc];
                const int sn = Mn > t ? Mn - 1 : 0;
                if (!(s > sn)) return false;
            }
        }
        return true;
    };
    int cnt = 0;
    for (int i = p0; i < p1; i++) cnt += keep(i, ti);
    int total = block_reduce_sum(cnt, scratch);
    int t = ti;
    if (total == 0) {
        t = tm;
        cnt = 0;
        for (int i = p0; i < p1; i++) cnt += keep(i, tm);
    }
    int tot2;
    const int incl = block_scan_incl(cnt, scratch, &tot2);
    int w = incl - cnt;
    uint32_t* slot = b.cell_keys + ((size_t)f * P.ncells + cd.slot) * P.slot_cap;
    for (int i = p0; i < p1; i++) {
        if (keep(i, t)) {
            const int r = i / tw, c = i - r * tw;
            slot[w++] = pack_kp(cd.iniX + 3 + c, cd.iniY + 3 + r, meas[i] - 1);
        }
    }
    if (threadIdx.x == 0) b.cell_cnt[(size_t)f * P.ncells + cd.slot] = tot2;
}

// ---------------------------------------------------------------------------------------
// Exact FAST measure without a threshold: M = max(max_s min d[s..s+8], -min_s max d[s..s+8])
// with d_k = v - p_k over the 16-pixel Bresenham circle (windows by min3/max3 doubling).
// ---------------------------------------------------------------------------------------
// M from the centre v and the circle p[0..15] (p_k in FAST_t<16>'s pixel order)
__device__ __forceinline__ int fast_M_of(int v, const int (&p)[16]) {
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = v - p[k];
    int mn3[16], mx3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        mn3[k] = min(min(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
        mx3[k] = max(max(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    }
    int mdark = -1024, mbr = 1024;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int mn9 = min(min(mn3[k], mn3[(k + 3) & 15]), mn3[(k + 6) & 15]);
        const int mx9 = max(max(mx3[k], mx3[(k + 3) & 15]), mx3[(k + 6) & 15]);
        mdark = max(mdark, mn9);
        mbr = min(mbr, mx9);
    }
    const int M = max(mdark, -mbr);
    return M > 0 ? M : 0;
}

__device__ __forceinline__ int fast_M(const uint8_t* c, int stride) {
    const int p[16] = {c[3 * stride],      c[3 * stride + 1],  c[2 * stride + 2],  c[stride + 3],
                       c[3],               c[-stride + 3],     c[-2 * stride + 2], c[-3 * stride + 1],
                       c[-3 * stride],     c[-3 * stride - 1], c[-2 * stride - 2], c[-stride - 3],
                       c[-3],              c[stride - 3],      c[2 * stride - 2],  c[3 * stride - 1]};
    return fast_M_of(c[0], p);
}

// Necessary condition for a 9-arc at threshold t: every 9-run of the 16-pixel circle holds
// one pixel of each opposite pair (k, k+8), so a bright corner needs min(p_k, p_k+8) < v - t
// and a dark one max(p_k, p_k+8) > v + t for all eight pairs.  Passes ~7% of the pixels of
// textured frames at t = 7 (the compass pre-test of pass A, two pairs, passes ~24%).
__device__ __forceinline__ bool fast_pairs8(const uint8_t* c, int stride, int t) {
    const int v = c[0];
    const int p[16] = {c[3 * stride],      c[3 * stride + 1],  c[2 * stride + 2],  c[stride + 3],
                       c[3],               c[-stride + 3],     c[-2 * stride + 2], c[-3 * stride + 1],
                       c[-3 * stride],     c[-3 * stride - 1], c[-2 * stride - 2], c[-stride - 3],
                       c[-3],              c[stride - 3],      c[2 * stride - 2],  c[3 * stride - 1]};
    int lo = min(p[0], p[8]), hi = max(p[0], p[8]);
#pragma unroll
    for (int k = 1; k < 8; k++) {
        lo = max(lo, min(p[k], p[k + 8]));
        hi = min(hi, max(p[k], p[k + 8]));
    }
    return (lo < v - t) || (hi > v + t);
}

// The eight-pair pre-test and, when it passes, the exact measure from the same 17 reads (the
// single-chunk form of passes B1 + B): 0 when the pre-test fails (then M <= t as well).
__device__ __forceinline__ int fast_pairs8_M(const uint8_t* c, int stride, int t) {
    const int v = c[0];
    const int p[16] = {c[3 * stride],      c[3 * stride + 1],  c[2 * stride + 2],  c[stride + 3],
                       c[3],               c[-stride + 3],     c[-2 * stride + 2], c[-3 * stride + 1],
                       c[-3 * stride],     c[-3 * stride - 1], c[-2 * stride - 2], c[-stride - 3],
                       c[-3],              c[stride - 3],      c[2 * stride - 2],  c[3 * stride - 1]};
    int lo = min(p[0], p[8]), hi = max(p[0], p[8]);
#pragma unroll
    for (int k = 1; k < 8; k++) {
        lo = max(lo, min(p[k], p[k + 8]));
        hi = min(hi, max(p[k], p[k + 8]));
    }
    if (!((lo < v - t) || (hi > v + t))) return 0;
    return fast_M_of(v, p);
}

// ---------------------------------------------------------------------------------------
// k_fast_wave: one WAVE per cell whose tested region is <= 64 columns wide (all cells of
// the standard geometries).  Three order-preserving, wave-compacted passes over the cell:
//   A  compass pre-test on every tested pixel (necessary for a 9-arc at threshold t: it
//      covers one of each opposite pair 0/8 and 4/12)  -> list of survivors
//   B1 the eight-pair test, B exact measure M (fast_M) on the survivors; M > t goes to a
//      zero-padded M map and stays in the (in-place) list.  When A leaves at most 64 pixels
//      (one chunk), B1 and B run as one pass on one set of circle reads (fast_pairs8_M)
//   C  cell-local 3x3 NMS at t on the remaining corners
// t = iniThFAST, then minThFAST only for cells left empty (ORBextractor.cc:808-841).  Lists
// keep row-major order, so the survivors are emitted in cv::FAST's order.
// LDS per wave (host-sized to the widest cell, VGA: 6.5 KB -> 6 workgroups per CU, with
// <= 80 VGPRs): ROI ch x rs | M map (th+2) x ms | list.
// ---------------------------------------------------------------------------------------
constexpr int kRoiStride = 80, kRoiRows = 80;  // widest / tallest cell the wave kernel stages

struct FastWaveLds {
    int roi, map, lst, total;  // byte offsets inside one wave's region, total size
    int rs, ms;                       // ROI / M-map row strides (bytes), sized to the geometry
};

#ifndef SLAMHOT_FAST_WPG
#define SLAMHOT_FAST_WPG 4
#endif
constexpr int kFastWpg = SLAMHOT_FAST_WPG;  // waves (cells) per workgroup

// One wave cell with everything its wave derives from the geometry precomputed on the host
// (ensure_plan): one scalar load instead of cell index -> CellDesc -> level plan, and no
// per-wave integer divisions (lane / d = (lane * m_d) >> 16 with m_d = ceil(2^16 / d), exact for
// lane < 64, d <= 20).
// All fields are dwords: scalar loads, no byte extraction (which the compiler does in VALU).
struct FastWaveCell {
    int64_t roi_off;        // byte offset of the staged ROI's first dword in the frame's level
    int64_t fstride;        // frame stride of that level's base (Bufs img for level 0, else pyr)
    int32_t slot, pitch;    // cell slot; level row pitch
    int32_t level, iniX, iniY, cw, ch;
    int32_t sh, wd, rp, ng; // staging shift (bytes), staged dwords per row, rows per staging pass,
                            // pass-A dword groups
    int32_t g0, rpi, dw;    // first pass-A group, pass-A rows per iteration, dword staging
    int32_t m_wd, m_ng;
};
static_assert(sizeof(FastWaveCell) == 80, "five 16-byte rows");

// One cell after its ROI is in LDS (roi = the ROI origin, `sh` bytes into each staged row): the
// M map zeroed, passes A / B1 / B / C at iniThFAST, again at minThFAST for an empty cell, the
// kept corners emitted to the cell's slot in row-major order.
__device__ __forceinline__ void fast_cell(const Bufs& b, const DevPlan& P, const FastWaveCell& cd, int f, int sh,
                                          const uint8_t* roi, const uint32_t* roi32, uint8_t* map, uint16_t* lst,
                                          const FastWaveLds& lay, int lane) {
    const int cw = cd.cw, ch = cd.ch;
    const int th = ch - 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int ti = min(max(P.ini_th, 0), 255), tm = min(max(P.min_th, 0), 255);
#ifdef SLAMHOT_FAST_TRACE
    // per-pass s_memtime cycles and list sizes of sampled cells (tools/ab/r05_fasttrace.sh)
    long long ftr[12];
    int nftr = 0, fcnt[8], nfc = 0;
    const bool ftrace = f == 5 && (cd.slot % 7) == 3 && lane == 0;
#define FAST_MARK() do { if (ftrace && nftr < 12) ftr[nftr++] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
#define FAST_CNT(x) do { if (ftrace && nfc < 8) fcnt[nfc++] = (x); } while (0)
#else
#define FAST_MARK() do {} while (0)
#define FAST_CNT(x) do {} while (0)
#endif
    FAST_MARK();
    {
        // 16-byte stores, rounded up into the list region (r16-aligned, written before it is read)
        uint4* m128 = reinterpret_cast<uint4*>(map);
        const int nq = ((th + 2) * lay.ms + 15) >> 4;
        for (int i = lane; i < nq; i += 64) m128[i] = uint4{0u, 0u, 0u, 0u};
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

    // The cell keeps the iniThFAST result unless it is empty, then FAST runs again at
    // minThFAST (ORBextractor.cc:808-841).  Passes A / B1 / B run at the threshold of the
    // current attempt (far fewer survivors at iniTh = 20 than at minTh = 7); only empty cells
    // pay for the second attempt.  M is exact, so the map entries of the first attempt stay
    // valid for the second (NMS reads neighbours as M > t ? M - 1 : 0).
    // pass A's lane = (row ar, dword group gd) over the ng dwords that cover the tested columns
    // (ng <= 17, rpi = 64 / ng rows per iteration; host-computed), and the byte mask of its
    // tested columns
    const int ng = cd.ng, rpi = cd.rpi;
    const int ar = (lane * cd.m_ng) >> 16, gd = cd.g0 + (lane - ar * ng);
    uint32_t cmask = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = 4 * gd + k - sh;  // ROI column of byte k
        if (x >= 3 && x <= cw - 4) cmask |= 0xFFu << (8 * k);
    }
    if (ar >= rpi) cmask = 0;
    const int code0 = (4 * gd - sh - 3) + ar * 64;  // code of byte 0 in row 0
    auto keep_at = [&](int e, int t) -> bool {
        const int code = lst[e];
        const int r = code >> 6, c = code & 63;
        const int MS = lay.ms;
        const uint8_t* q = map + (r + 1) * MS + c + 1;
        const int M = q[0];
        auto sc = [&](int x) { return x > t ? x - 1 : 0; };
        int mx = max(max(sc(q[-MS - 1]), sc(q[-MS])), max(sc(q[-MS + 1]), sc(q[-1])));
        mx = max(mx, max(max(sc(q[1]), sc(q[MS - 1])), max(sc(q[MS]), sc(q[MS + 1]))));
        return (M > t) & (M - 1 > mx);
    };
    // Compass-score cache for the second attempt: attempt 1 keeps each lane's per-pixel compass
    // scores s = max(v - L, H - v) (the largest t the pixel passes at, one byte each, one dword per
    // lane and pass-A iteration) at the END of the list region, while its list grows from the start;
    // attempt 2 (minThFAST, about half the cells) reads them back instead of re-deriving them from
    // the ROI.  Valid when attempt 1's list stayed below them (2 * na <= s_off, checked before every
    // store, so a store never lands on the list); attempt 2 checks before each iteration's list
    // writes that the list stays below the scores it has not read yet, and otherwise runs pass A
    // again from the ROI.  All the conditions are wave-uniform.
    const int nit = (th + rpi - 1) / rpi;
    const int s_off = (lay.total - lay.lst) - nit * 256;  // bytes from lst (multiple of 16), < 0: no room
    uint32_t* const scache = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(lst) + s_off) + lane;
    // pass A, four pixels per lane in packed u16 pairs (even / odd bytes of an LDS dword).
    // Lane = (row, dword group) over the dwords covering the tested columns; the compass
    // test per pixel is  min(p0,p8), min(p4,p12) < v - t  (dark) or  max(..) > v + t
    // (bright), i.e. s = max(v - max of the mins, min of the maxes - v) > t (saturating u16).
    // Four ballots (one per byte) + mbcnt give row-major compaction.  Returns the list length,
    // or -1 when a cached pass would overwrite scores it has not read yet.
    auto pass_a = [&](auto from_cache_c, auto keep_s_c, int t) -> int {
        constexpr bool from_cache = decltype(from_cache_c)::value, keep_s = decltype(keep_s_c)::value;
        const us2 T = {(unsigned short)t, (unsigned short)t};
        // the lane's row walks down by rpi rows per iteration; rows past the tested region
        // (m = 0) read the last tested row instead
        const int RS = lay.rs >> 2;
        const uint32_t* row_it = roi32 + (ar + 3) * RS + gd;
        const uint32_t* row_last = roi32 + (th + 2) * RS + gd;
        uint32_t* sp = scache;
        int s_next = s_off + 256;  // where the scores of the iterations after this one start
        int na = 0;
        for (int rt = 0; rt < th; rt += rpi, row_it += rpi * RS, sp += 64, s_next += 256) {
            const bool in = ar < th - rt;
            const uint32_t m = in ? cmask : 0u;
            us2 se, so;  // compass scores of the even / odd bytes
            if constexpr (from_cache) {
                const uint32_t S = *sp;  // byte k = pixel k
                se = as_us2(__builtin_amdgcn_perm(0u, S, 0x0c020c00u));
                so = as_us2(__builtin_amdgcn_perm(0u, S, 0x0c030c01u));
            } else {
                const uint32_t* row = in ? row_it : row_last;
                const uint32_t W0 = row[-1], W1 = row[0], W2 = row[1], U = row[-3 * RS], D = row[3 * RS];
                auto score = [&](uint32_t v, uint32_t p0, uint32_t p8, uint32_t p4, uint32_t p12) -> us2 {
                    const us2 V = as_us2(v), a = as_us2(p0), bq = as_us2(p8), c = as_us2(p4), d = as_us2(p12);
                    const us2 L = __builtin_elementwise_max(__builtin_elementwise_min(a, bq), __builtin_elementwise_min(c, d));
                    const us2 H = __builtin_elementwise_min(__builtin_elementwise_max(a, bq), __builtin_elementwise_max(c, d));
                    return __builtin_elementwise_max(__builtin_elementwise_sub_sat(V, L), __builtin_elementwise_sub_sat(H, V));
                };
                se = score(__builtin_amdgcn_perm(0u, W1, 0x0c020c00u), __builtin_amdgcn_perm(0u, D, 0x0c020c00u),
                           __builtin_amdgcn_perm(0u, U, 0x0c020c00u), __builtin_amdgcn_perm(W2, W1, 0x0c050c03u),
                           __builtin_amdgcn_perm(W1, W0, 0x0c030c01u));
                so = score(__builtin_amdgcn_perm(0u, W1, 0x0c030c01u), __builtin_amdgcn_perm(0u, D, 0x0c030c01u),
                           __builtin_amdgcn_perm(0u, U, 0x0c030c01u), __builtin_amdgcn_perm(W2, W1, 0x0c060c04u),
                           __builtin_amdgcn_perm(W1, W0, 0x0c040c02u));
            }
            const us2 fe = __builtin_elementwise_sub_sat(se, T), fo = __builtin_elementwise_sub_sat(so, T);
            const uint32_t F = (as_u32(fe) | (as_u32(fo) << 8)) & m;  // byte k != 0 <=> pixel k survives
            const bool f0 = (F & 0xFFu) != 0, f1 = (F & 0xFF00u) != 0, f2 = (F & 0xFF0000u) != 0, f3 = (F >> 24) != 0;
            const uint64_t b0 = __ballot(f0), b1 = __ballot(f1), b2 = __ballot(f2), b3 = __ballot(f3);
            const int na_next = na + __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
            if constexpr (from_cache)
                if (2 * na_next > s_next) return -1;
            int pos = mbcnt64(b3, mbcnt64(b2, mbcnt64(b1, mbcnt64(b0, na))));
            const int code = code0 + rt * 64;
            if (f0) lst[pos++] = (uint16_t)code;
            if (f1) lst[pos++] = (uint16_t)(code + 1);
            if (f2) lst[pos++] = (uint16_t)(code + 2);
            if (f3) lst[pos] = (uint16_t)(code + 3);
            na = na_next;
            if constexpr (keep_s)
                if (2 * na <= s_off) *sp = as_u32(se) | (as_u32(so) << 8);
        }
        return na;
    };
    using yes = std::integral_constant<bool, true>;
    using no = std::integral_constant<bool, false>;
    bool cached = false;
    for (int attempt = 0; attempt < 2; attempt++) {
        const int t = attempt == 0 ? ti : tm;
        FAST_MARK();
        int na;
        if (attempt == 0) {
            na = s_off >= 0 ? pass_a(no{}, yes{}, t) : pass_a(no{}, no{}, t);
        } else {
            na = cached ? pass_a(yes{}, no{}, t) : -1;
            if (na < 0) na = pass_a(no{}, no{}, t);
        }
        if (attempt == 0) cached = s_off >= 0 && 2 * na <= s_off;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        FAST_MARK();
        FAST_CNT(na);

        int nb = 0;
        if (na <= 64) {
            // one chunk of compass survivors: B1 and B together, one set of circle reads per pixel
            const bool valid = lane < na;
            const int code = valid ? lst[lane] : 0;
            const int r = code >> 6, c = code & 63;
            int M = 0;
            if (valid) M = fast_pairs8_M(roi + (r + 3) * lay.rs + c + 3, lay.rs, t);
            const bool corner = M > t;
            if (corner) map[(r + 1) * lay.ms + c + 1] = (uint8_t)M;
            const uint64_t m = __ballot(corner);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (corner) lst[__popcll(m & lt)] = (uint16_t)code;
            nb = __popcll(m);
            FAST_MARK();
            FAST_CNT(-1);
        } else {
            // pass B1: the eight-pair pre-test on the compass survivors (in-place compaction)
            {
                int n1 = 0;
                for (int j = 0; j < na; j += 64) {
                    const int e = j + lane;
                    const bool valid = e < na;
                    const int code = valid ? lst[e] : 0;
                    const int r = code >> 6, c = code & 63;
                    const bool keep = valid && fast_pairs8(roi + (r + 3) * lay.rs + c + 3, lay.rs, t);
                    const uint64_t m = __ballot(keep);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    if (keep) lst[n1 + __popcll(m & lt)] = (uint16_t)code;
                    n1 += __popcll(m);
                }
                na = n1;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            FAST_MARK();
            FAST_CNT(na);

            // pass B (compacts the list in place: writes never pass the chunk being read)
            for (int j = 0; j < na; j += 64) {
                const int e = j + lane;
                const bool valid = e < na;
                const int code = valid ? lst[e] : 0;
                const int r = code >> 6, c = code & 63;
                int M = 0;
                if (valid) M = fast_M(roi + (r + 3) * lay.rs + c + 3, lay.rs);
                const bool corner = M > t;
                if (corner) map[(r + 1) * lay.ms + c + 1] = (uint8_t)M;
                const uint64_t m = __ballot(corner);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (corner) lst[nb + __popcll(m & lt)] = (uint16_t)code;
                nb += __popcll(m);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        FAST_MARK();
        FAST_CNT(nb);
        // pass C: cell-local 3x3 NMS at t; count, then emit in list (row-major) order
        int cnt = 0;
        for (int j = 0; j < nb; j += 64) cnt += __popcll(__ballot(j + lane < nb && keep_at(j + lane, t)));
        if (cnt == 0 && attempt == 0 && tm != ti) continue;
        uint32_t* slot = b.cell_keys + ((size_t)f * P.ncells + cd.slot) * P.slot_cap;
        int base = 0;
        for (int j = 0; j < nb; j += 64) {
            const bool k = j + lane < nb && keep_at(j + lane, t);
            const uint64_t m = __ballot(k);
            if (k) {
                const int code = lst[j + lane];
                const int r = code >> 6, c = code & 63;
                const int M = map[(r + 1) * lay.ms + c + 1];
                slot[base + __popcll(m & lt)] = pack_kp(cd.iniX + 3 + c, cd.iniY + 3 + r, M - 1);
            }
            base += __popcll(m);
        }
        if (lane == 0) b.cell_cnt[(size_t)f * P.ncells + cd.slot] = base;
#ifdef SLAMHOT_FAST_TRACE
        FAST_MARK();
        if (ftrace) {
            // marks: 0 start, per attempt: begin, A, B1, B; then the end (after C and the emit)
            const int a = attempt;
            const long long zero = ftr[1] - ftr[0];
            long long A = 0, B1 = 0, B = 0;
            for (int k = 0; k <= a; k++) {
                A += ftr[2 + 4 * k] - ftr[1 + 4 * k];
                B1 += ftr[3 + 4 * k] - ftr[2 + 4 * k];
                B += ftr[4 + 4 * k] - ftr[3 + 4 * k];
            }
            const long long C = ftr[nftr - 1] - ftr[nftr - 2];
            printf("FAST lvl=%d cw=%d ch=%d att=%d nA=%d nB1=%d nB=%d kept=%d zero %lld A %lld B1 %lld B %lld C %lld\n",
                   cd.level, cw, ch, a + 1, fcnt[3 * a], fcnt[3 * a + 1], fcnt[3 * a + 2], base, zero, A, B1, B, C);
        }
#endif
        return;
    }
}

// Stage a cell's ROI rows with independent 32-bit buffer loads (row start aligned down to 4
// bytes, so the ROI origin inside LDS is `sh` bytes into each row).  Lane = (row offset lr,
// dword column lc), fixed for the wave: rows lr, lr + rp, ...; eight rows per lane in flight, each
// load's row offset an SGPR (soffset), the resource bounded at the ROI's last byte so the rows
// past it read zero without touching memory.
__device__ __forceinline__ void stage_roi(const FastWaveCell& c, const uint8_t* src, uint8_t* roi, int rs, int lane) {
    uint32_t* roi32 = reinterpret_cast<uint32_t*>(roi);
    if (c.dw) {
        const int lr = (lane * c.m_wd) >> 16, lc = lane - lr * c.wd;
        if (lr < c.rp) {
            const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)src, (short)0, __builtin_amdgcn_readfirstlane((c.ch - 1) * c.pitch + 4 * c.wd), 0x00020000);
            const int voff = lr * c.pitch + 4 * lc;
            uint32_t* dst = roi32 + lr * (rs >> 2) + lc;
            const int rp = c.rp, step = rp * (rs >> 2);
            if (c.dw == 2) {
                // rows past the ROI land in this wave's own map / list regions (host-checked:
                // (ch + 8 rp - 1) rows of rs bytes fit its layout), which are written before they
                // are read, and read zero (the resource ends at the ROI): no per-row guard
                for (int r0 = 0, q0 = 0; r0 < c.ch; r0 += 8 * rp, q0 += 8) {
                    uint32_t v[8];
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        v[k] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, (r0 + k * rp) * c.pitch, 0);
#pragma unroll
                    for (int k = 0; k < 8; k++) dst[(q0 + k) * step] = v[k];
                }
            } else {
                for (int r0 = 0, q0 = 0; r0 < c.ch; r0 += 8 * rp, q0 += 8) {
                    uint32_t v[8];
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        v[k] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, (r0 + k * rp) * c.pitch, 0);
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        if (lr + r0 + k * rp < c.ch) dst[(q0 + k) * step] = v[k];
                }
            }
        }
    } else {
        for (int r = 0; r < c.ch; r++)
            for (int x = lane; x < c.cw; x += 64) roi[r * rs + x] = src[(size_t)r * c.pitch + x];
    }
}

// ---------------------------------------------------------------------------------------
// k_fast_wave: one WAVE per cell whose tested region is <= 64 columns wide (all cells of
// the standard geometries); see fast_cell for the passes.
// LDS per wave (host-sized to the widest cell of the class): ROI ch x rs | M map (th+2) x ms |
// list.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64 * kFastWpg) __attribute__((amdgpu_waves_per_eu(6, 8))) k_fast_wave(Bufs b, const FastWaveCell* list, int nlist,
                                                   FastWaveLds lay) {
    extern __shared__ __attribute__((aligned(16))) uint8_t fw_smem[];
    // the wave index through v_readfirstlane: known wave-uniform, so the cell record and all the
    // geometry derived from it live in SGPRs (scalar loads, buffer-load soffsets)
    const int wave = kFastWpg == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int2 blk = xcd_block();
    const int idx = blk.x * kFastWpg + wave;
    if (idx >= nlist) return;
    const DevPlan& P = *b.plan;
    const int f = blk.y;
    const FastWaveCell cd = list[idx];
    uint8_t* base_ptr = fw_smem + wave * lay.total;
    const uint8_t* src = (cd.level ? (const uint8_t*)b.pyr : b.img) + (size_t)f * cd.fstride + cd.roi_off;
    stage_roi(cd, src, base_ptr + lay.roi, lay.rs, lane);
    fast_cell(b, P, cd, f, cd.sh, base_ptr + lay.roi + cd.sh, reinterpret_cast<const uint32_t*>(base_ptr + lay.roi),
              base_ptr + lay.map, reinterpret_cast<uint16_t*>(base_ptr + lay.lst), lay, lane);
}

// ---------------------------------------------------------------------------------------
// k_octree: DistributeOctTree (ORBextractor.cc:537-761), one WAVE per (frame, level).
//
// The reference's std::list<ExtractorNode> is represented by the array of alive nodes in
// list order.  A pass that splits the nodes of a set S in push order pi (children n1..n4
// of each, empty ones dropped, pushed to the FRONT; parent erased) yields
//     [children in reverse push order] ++ [unsplit nodes in their previous order],
// i.e. two prefix sums.  Phase A (:592-671) splits every node holding >1 key in list
// order; the careful phase (:671-736) splits candidates ordered by (size desc, sequence
// desc) and stops at the first split that reaches N.  Children receive creation sequence
// numbers in push order; sequence replaces the reference's heap-pointer tie-break (:682,
// nondeterministic in the reference) — documented deviation, identical in the oracle.
// Keys keep their original (cell-major) order; each node keeps its max-response key, the
// first in original order on ties (:742-758).
//
// A level's list never exceeds max(N+3, 4*nIni) nodes (a few hundred) and ~4 passes split
// it, so the work is a chain of small prefix sums: one wave runs them with ballot/mbcnt
// and DPP scans and no workgroup barriers (a 256-thread version spent ~10k cycles per pass
// in s_barrier round trips).  Node arrays and keys live in this wave's LDS (keys spill to
// the per-frame global scratch past key_cap); levels are launched in groups whose LDS size
// fits their key counts (level 0 alone, then the rest).
// ---------------------------------------------------------------------------------------
struct NodeArr {
    uint32_t* xb;  // x0 | x1 << 16
    uint32_t* yb;  // y0 | y1 << 16
    int32_t *cnt, *seq;
};

__device__ __forceinline__ int quadrant_of(uint32_t key, uint32_t xb, uint32_t yb) {
    const int x0 = (int)(xb & 0xFFFF), x1 = (int)(xb >> 16), y0 = (int)(yb & 0xFFFF), y1 = (int)(yb >> 16);
    const int xm = x0 + ((x1 - x0 + 1) >> 1);  // ceil((x1-x0)/2), :481
    const int ym = y0 + ((y1 - y0 + 1) >> 1);
    return (kp_x(key) < xm ? 0 : 1) + (kp_y(key) < ym ? 0 : 2);  // n1, n2, n3, n4 (:513-523)
}

// LDS and global accesses of one wave are ordered for that wave by this fence
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// exclusive prefix sum over the wave's 64 lanes (all active); total in *tot.  DPP
// Kogge-Stone inside rows of 16 (row_shr 1/2/4/8, zero-filled), then row_bcast15 / 31
// carry the row totals into the following rows: VALU-speed steps instead of six dependent
// ds_bpermute round trips.
__device__ __forceinline__ int wave_scan_excl(int v, int* tot) {
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    *tot = __builtin_amdgcn_readlane(x, 63);
    return x - v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

enum { kErrOctreeIters = 1, kErrOctreeNodes = 2, kErrCap = 4 };

__host__ __device__ inline size_t octree_lds_bytes(int maxn, int keycap, int maxcells) {
    size_t s = 0;
    auto add = [&](size_t bytes) { s += (bytes + 15) & ~(size_t)15; };
    for (int i = 0; i < 2; i++) { add(4 * (size_t)maxn); add(4 * (size_t)maxn); add(4 * (size_t)maxn); add(4 * (size_t)maxn); }
    add(16 * (size_t)maxn);                       // cc
    add(8 * (size_t)maxn);                        // cmap
    add(2 * (size_t)maxn); add(2 * (size_t)maxn); add(4 * (size_t)maxn);  // ord, rnk, oarr
    add(4 * (size_t)maxn);                        // best
    add(4 * ((size_t)maxcells + 1));              // coff
    add(4 * (size_t)keycap); add(2 * (size_t)keycap);
    return s;
}

constexpr int kKU = 8;  // keys per lane in flight in the octree key loops

#ifndef SLAMHOT_OCT_WAVES
#define SLAMHOT_OCT_WAVES 4
#endif
constexpr int kOctWaves = SLAMHOT_OCT_WAVES;  // waves per (frame, level) of the multi-wave form

// W waves per (frame, level): the key loops (gather, root / quadrant counts, key remap, best
// key) are spread over all W waves; the node-list steps (prefix sums over at most a few hundred
// nodes) stay on wave 0, whose results the others read from LDS after a barrier.  W = 1 is the
// wave-only form (no workgroup barriers).
template <int W>
__global__ void __launch_bounds__(64 * W) k_octree(Bufs b, int level0, int key_lds_cap, int max_cells) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int bc[8];  // scalars wave 0 hands to the other waves (W > 1)
    constexpr int NT = 64 * W;
    const DevPlan& P = *b.plan;
    const int l = level0 + blockIdx.x, f = blockIdx.y;
    const DevLevel& L = P.lv[l];
    const int MAXN = P.max_nodes;
    const int tid = threadIdx.x, lane = tid & 63, wave = W == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 6);
    auto sync = [&]() {
        if constexpr (W == 1) wave_fence();
        else __syncthreads();
    };
#ifdef SLAMHOT_OCTREE_TRACE
    // experiment builds only: phase timestamps of a few waves
    long long tr[24];
    int ntr = 0;
    const bool trace = (f == 0 || f == 100 || f == 101) && tid == 0;
#define OCT_MARK() do { if (trace && ntr < 24) tr[ntr++] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define OCT_MARK() do {} while (0)
#endif
    OCT_MARK();

    uint8_t* p = smem;
    auto carve = [&](size_t bytes) {
        uint8_t* r = p;
        p += (bytes + 15) & ~(size_t)15;
        return r;
    };
    NodeArr A, B;
    A.xb = (uint32_t*)carve(4 * MAXN); A.yb = (uint32_t*)carve(4 * MAXN);
    A.cnt = (int32_t*)carve(4 * MAXN); A.seq = (int32_t*)carve(4 * MAXN);
    B.xb = (uint32_t*)carve(4 * MAXN); B.yb = (uint32_t*)carve(4 * MAXN);
    B.cnt = (int32_t*)carve(4 * MAXN); B.seq = (int32_t*)carve(4 * MAXN);
    uint4* cc = (uint4*)carve(16 * MAXN);       // child key counts per node (n1..n4)
    uint16_t* cmap = (uint16_t*)carve(8 * MAXN);  // new position of child [node][4]
    uint16_t* ord = (uint16_t*)carve(2 * MAXN);   // split nodes in push order
    int16_t* rnk = (int16_t*)carve(2 * MAXN);     // push index of a node, -1 = not split
    int32_t* oarr = (int32_t*)carve(4 * MAXN);    // child offset of a split node (by push idx)
    uint32_t* best = (uint32_t*)carve(4 * MAXN);
    int32_t* coff = (int32_t*)carve(4 * ((size_t)max_cells + 1));
    uint32_t* keys_l = (uint32_t*)carve(4 * (size_t)key_lds_cap);
    uint16_t* knode_l = (uint16_t*)carve(2 * (size_t)key_lds_cap);
    uint32_t* ccu = reinterpret_cast<uint32_t*>(cc);

    // ---- gather the level's candidates in cell order, relative to (minBX, minBY): cell
    // offsets by one scan, then every key independently (its cell by binary search over the
    // offsets); eight keys per lane advance together so their LDS and HBM loads overlap
    const int cb = L.cell_begin, ncl = L.cell_end - L.cell_begin;
    const int32_t* ccount = b.cell_cnt + (size_t)f * P.ncells;
    int nk = 0;
    if (wave == 0) {
        for (int base = 0; base < ncl; base += 64) {
            const int i = base + lane;
            const int v = i < ncl ? ccount[cb + i] : 0;
            int tot;
            const int ex = wave_scan_excl(v, &tot);
            if (i < ncl) coff[i] = nk + ex;
            nk += tot;
        }
        if constexpr (W > 1) {
            if (lane == 0) bc[0] = nk;
        }
    }
    sync();
    if constexpr (W > 1) nk = bc[0];
    const bool in_lds = nk <= key_lds_cap;
    uint32_t* keys = in_lds ? keys_l : b.keys_g + (size_t)f * P.key_slots + L.key_base;
    uint16_t* knode = in_lds ? knode_l : b.knode_g + (size_t)f * P.key_slots + L.key_base;
    {
        const uint32_t* src = b.cell_keys + ((size_t)f * P.ncells + cb) * P.slot_cap;
        const int steps = ncl > 1 ? 32 - __clz(ncl - 1) : 0;  // ceil(log2(ncl))
        constexpr int U = 8;
        for (int k0 = tid; k0 < nk; k0 += U * NT) {
            // largest c with coff[c] <= k (a non-empty cell); extra steps keep lo == hi
            int lo[U], hi[U];
#pragma unroll
            for (int u = 0; u < U; u++) { lo[u] = 0; hi[u] = ncl - 1; }
            for (int st = 0; st < steps; st++) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int k = min(k0 + u * NT, nk - 1);
                    const int mid = (lo[u] + hi[u] + 1) >> 1;
                    if (coff[mid] <= k) lo[u] = mid; else hi[u] = mid - 1;
                }
            }
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int k = min(k0 + u * NT, nk - 1);
                v[u] = src[(size_t)lo[u] * P.slot_cap + (k - coff[lo[u]])];
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int k = k0 + u * NT;
                if (k < nk) keys[k] = pack_kp(kp_x(v[u]) - L.minBX, kp_y(v[u]) - L.minBY, kp_s(v[u]));
            }
        }
    }
    OCT_MARK();
    const int N = L.nfeat;
    int32_t* out_cnt = b.ocnt + (size_t)f * P.nlevels + l;
    uint32_t* okp = b.okp + (size_t)f * P.kslots + L.kbase;
    if (nk == 0) {
        if (tid == 0) *out_cnt = 0;
        return;
    }

    // ---- roots (:541-583): key -> root (int)(x / hX); empty roots erased
    if (tid < L.nIni) best[tid] = 0;
    sync();
    for (int k0 = tid; k0 < nk; k0 += kKU * NT) {
        uint32_t key[kKU];
#pragma unroll
        for (int u = 0; u < kKU; u++) key[u] = keys[min(k0 + NT * u, nk - 1)];
#pragma unroll
        for (int u = 0; u < kKU; u++) {
            const int k = k0 + NT * u;
            const int x = kp_x(key[u]);
            int r = 0;
            for (int i = 1; i < L.nIni; i++) r += x >= L.root_first_x[i];
            if (k < nk) {
                knode[k] = (uint16_t)r;
                atomicAdd(&best[r], 1u);
            }
        }
    }
    sync();
    int n = 0;
    if (wave == 0) {
        const bool ne = lane < L.nIni && best[lane] > 0;
        const uint64_t m = __ballot(ne);
        if (ne) {
            const int pos = mbcnt64(m, 0);
            A.xb[pos] = (uint32_t)L.root_x0[lane] | ((uint32_t)L.root_x1[lane] << 16);
            A.yb[pos] = (uint32_t)(L.maxBY - L.minBY) << 16;
            A.cnt[pos] = (int)best[lane];
            A.seq[pos] = lane;
            cmap[lane] = (uint16_t)pos;
        }
        n = __popcll(m);
    }
    sync();
    if constexpr (W > 1) n = __popcll(__ballot(lane < L.nIni && best[lane] > 0));  // every wave: the same count
    for (int k0 = tid; k0 < nk; k0 += kKU * NT) {
        int nd[kKU];
#pragma unroll
        for (int u = 0; u < kKU; u++) nd[u] = knode[min(k0 + NT * u, nk - 1)];
        uint16_t cm[kKU];
#pragma unroll
        for (int u = 0; u < kKU; u++) cm[u] = cmap[nd[u]];
#pragma unroll
        for (int u = 0; u < kKU; u++)
            if (k0 + NT * u < nk) knode[k0 + NT * u] = cm[u];
    }
    sync();
    OCT_MARK();
    int seq_next = L.nIni;
    int tprev = 0;  // children region [0, tprev) of the last pass
    bool careful = false;
    bool finish = false;
    int err = 0;

    for (int iter = 0; !finish; iter++) {
        if (iter >= 512) { err |= kErrOctreeIters; break; }
        const int prev = n;
        // -- candidate set and quadrant counts
        for (int i = tid; i < n; i += NT) {
            cc[i] = make_uint4(0, 0, 0, 0);
            rnk[i] = -1;
        }
        sync();
        // kKU keys per lane per step: their node loads overlap, then the atomics
        for (int k0 = tid; k0 < nk; k0 += kKU * NT) {
            int nd[kKU];
            uint32_t key[kKU];
#pragma unroll
            for (int u = 0; u < kKU; u++) {
                const int k = min(k0 + NT * u, nk - 1);
                nd[u] = knode[k];
                key[u] = keys[k];
            }
            int c[kKU];
            uint32_t xb[kKU], yb[kKU];
#pragma unroll
            for (int u = 0; u < kKU; u++) { c[u] = A.cnt[nd[u]]; xb[u] = A.xb[nd[u]]; yb[u] = A.yb[nd[u]]; }
#pragma unroll
            for (int u = 0; u < kKU; u++)
                if (k0 + NT * u < nk && c[u] > 1 && (!careful || nd[u] < tprev))
                    atomicAdd(&ccu[nd[u] * 4 + quadrant_of(key[u], xb[u], yb[u])], 1u);
        }
        sync();
        auto nonempty = [&](int nd) -> int {
            const uint4 q = cc[nd];
            return (q.x > 0) + (q.y > 0) + (q.z > 0) + (q.w > 0);
        };
        // -- node-list steps on wave 0: split set, children offsets, the new list in B
        int T = 0, U = 0, n_to_expand = 0;
        bool overflow = false;
        if (wave == 0) {
            int nsplit = 0;
            if (!careful) {
                // phase A: split every node with >1 key, push order = list order
                for (int base = 0; base < n; base += 64) {
                    const int i = base + lane;
                    const bool c = i < n && A.cnt[i] > 1;
                    const uint64_t m = __ballot(c);
                    if (c) {
                        const int ex = nsplit + mbcnt64(m, 0);
                        rnk[i] = (int16_t)ex;
                        ord[ex] = (uint16_t)i;
                    }
                    nsplit += __popcll(m);
                }
            } else {
                // careful phase: E = children of the last pass with >1 key, ordered by
                // (size desc, sequence desc) = (cnt desc, position asc) inside [0, tprev).
                // rank(i) = #{j : c_j > c_i} + #{j < i : c_j == c_i}: a counting sort when the
                // counts are below MAXN -- histogram H (in `best`, free until the end) turned into
                // suffix sums, E (in `oarr`, free until the children offsets) the count of each
                // value in earlier blocks, and inside a block one ballot per distinct value --
                // instead of comparing every pair (tprev^2 / 64 readlane steps, most of this
                // phase's ~50k cycles at the fine levels)
                int ne = 0;
                int maxc = 0;
                for (int ib = 0; ib < tprev; ib += 64) {
                    const int i = ib + lane;
                    const int ci = i < tprev ? A.cnt[i] : 0;
                    maxc = max(maxc, ci);
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) maxc = max(maxc, __shfl_xor(maxc, o, 64));
                const bool counting = maxc < MAXN;
                if (counting) {
                    int* H = reinterpret_cast<int*>(best);
                    int* Ecnt = reinterpret_cast<int*>(oarr);
                    for (int v = lane; v <= maxc; v += 64) { H[v] = 0; Ecnt[v] = 0; }
                    wave_fence();
                    for (int ib = 0; ib < tprev; ib += 64) {
                        const int i = ib + lane;
                        const int ci = i < tprev ? A.cnt[i] : 0;
                        if (ci > 1) atomicAdd(&H[ci], 1);
                    }
                    wave_fence();
                    // H[v] <- #{candidates with count > v}: lane order = descending v
                    int carry = 0;
                    for (int base = 0; base <= maxc; base += 64) {
                        const int v = maxc - (base + lane);
                        const int h = v >= 0 ? H[v] : 0;
                        int tot;
                        const int ex = wave_scan_excl(h, &tot);
                        wave_fence();
                        if (v >= 0) H[v] = carry + ex;
                        carry += tot;
                    }
                    wave_fence();
                    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                    for (int ib = 0; ib < tprev; ib += 64) {
                        const int i = ib + lane;
                        const int ci = i < tprev ? A.cnt[i] : 0;
                        uint64_t rem = __ballot(ci > 1);
                        ne += __popcll(rem);
                        // larger counts + equal counts of earlier blocks, then equal counts of
                        // lower lanes (one ballot per distinct value in the block, no LDS)
                        int r = ci > 1 ? H[ci] + Ecnt[ci] : 0;
                        while (rem) {
                            const int v = __builtin_amdgcn_readlane(ci, __ffsll((long long)rem) - 1);
                            const uint64_t m = __ballot(ci == v);
                            if ((m >> lane) & 1) r += __popcll(m & lt);
                            rem &= ~m;
                        }
                        if (ci > 1) ord[r] = (uint16_t)i;
                        wave_fence();
                        if (ci > 1) atomicAdd(&Ecnt[ci], 1);
                        wave_fence();
                    }
                }
                for (int ib = 0; ib < tprev && !counting; ib += 64) {
                    const int i = ib + lane;
                    const int ci = i < tprev ? A.cnt[i] : 0;
                    const uint64_t mi = __ballot(ci > 1);
                    ne += __popcll(mi);
                    int r = 0;
                    for (int jb = 0; jb < tprev; jb += 64) {
                        const int cj = jb + lane < tprev ? A.cnt[jb + lane] : 0;
                        const int jn = min(64, tprev - jb);
                        for (int t = 0; t < jn; t++) {
                            const int c = __builtin_amdgcn_readlane(cj, t);
                            r += (c > 1) & ((c > ci) | ((c == ci) & (jb + t < i)));
                        }
                    }
                    if (ci > 1) ord[r] = (uint16_t)i;
                }
                wave_fence();
                // cut: first rank r with n + sum_{r'<=r}(nonempty-1) >= N (:728-729)
                int firstcut = ne - 1, carry = 0;
                for (int base = 0; base < ne; base += 64) {
                    const int r = base + lane;
                    const int v = r < ne ? nonempty(ord[r]) - 1 : 0;
                    int tot;
                    const int incl = carry + wave_scan_excl(v, &tot) + v;
                    const uint64_t m = __ballot(r < ne && n + incl >= N);
                    if (m) { firstcut = base + __ffsll((long long)m) - 1; break; }
                    carry += tot;
                }
                nsplit = firstcut + 1;
                for (int r = lane; r < nsplit; r += 64) rnk[ord[r]] = (int16_t)r;
            }
            wave_fence();
            // -- children offsets in push order
            for (int base = 0; base < nsplit; base += 64) {
                const int r = base + lane;
                const int v = r < nsplit ? nonempty(ord[r]) : 0;
                int tot;
                const int ex = wave_scan_excl(v, &tot);
                if (r < nsplit) oarr[r] = T + ex;
                T += tot;
            }
            overflow = T + (n - nsplit) > MAXN;
            if (!overflow) {
                wave_fence();
                // -- write the new list into B
                int nexp_local = 0;
                for (int base = 0; base < n; base += 64) {
                    const int i = base + lane;
                    const bool valid = i < n;
                    const int r = valid ? rnk[i] : 0;
                    const bool uns = valid && r < 0;
                    const uint64_t m = __ballot(uns);
                    if (uns) {
                        const int pos = T + U + mbcnt64(m, 0);
                        B.xb[pos] = A.xb[i]; B.yb[pos] = A.yb[i];
                        B.cnt[pos] = A.cnt[i]; B.seq[pos] = A.seq[i];
                        cmap[i * 4] = (uint16_t)pos;
                    } else if (valid) {
                        const int o = oarr[r];
                        const uint32_t xb = A.xb[i], yb = A.yb[i];
                        const int x0 = (int)(xb & 0xFFFF), x1 = (int)(xb >> 16), y0 = (int)(yb & 0xFFFF), y1 = (int)(yb >> 16);
                        const int xm = x0 + ((x1 - x0 + 1) >> 1), ym = y0 + ((y1 - y0 + 1) >> 1);
                        const uint4 q4 = cc[i];
                        const uint32_t cq[4] = {q4.x, q4.y, q4.z, q4.w};
                        int kk = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int c = (int)cq[q];
                            if (c > 0) {
                                const int pos = T - 1 - (o + kk);
                                const int nx0 = (q & 1) ? xm : x0, nx1 = (q & 1) ? x1 : xm;
                                const int ny0 = (q & 2) ? ym : y0, ny1 = (q & 2) ? y1 : ym;
                                B.xb[pos] = (uint32_t)nx0 | ((uint32_t)nx1 << 16);
                                B.yb[pos] = (uint32_t)ny0 | ((uint32_t)ny1 << 16);
                                B.cnt[pos] = c;
                                B.seq[pos] = seq_next + o + kk;
                                cmap[i * 4 + q] = (uint16_t)pos;
                                nexp_local += c > 1;
                                kk++;
                            }
                        }
                    }
                    U += __popcll(m);
                }
                n_to_expand = wave_sum(nexp_local);
            }
            if constexpr (W > 1) {
                if (lane == 0) {
                    bc[1] = T;
                    bc[2] = U;
                    bc[3] = n_to_expand;
                    bc[4] = overflow;
                }
            }
        }
        sync();
        if constexpr (W > 1) {
            T = bc[1];
            U = bc[2];
            n_to_expand = bc[3];
            overflow = bc[4] != 0;
        }
        if (overflow) { err |= kErrOctreeNodes; break; }
        // -- remap keys
        for (int k0 = tid; k0 < nk; k0 += kKU * NT) {
            int nd[kKU];
            uint32_t key[kKU];
#pragma unroll
            for (int u = 0; u < kKU; u++) {
                const int k = min(k0 + NT * u, nk - 1);
                nd[u] = knode[k];
                key[u] = keys[k];
            }
            int r[kKU];
            uint32_t xb[kKU], yb[kKU];
#pragma unroll
            for (int u = 0; u < kKU; u++) { r[u] = rnk[nd[u]]; xb[u] = A.xb[nd[u]]; yb[u] = A.yb[nd[u]]; }
            uint16_t cm[kKU];
#pragma unroll
            for (int u = 0; u < kKU; u++) cm[u] = cmap[nd[u] * 4 + (r[u] >= 0 ? quadrant_of(key[u], xb[u], yb[u]) : 0)];
#pragma unroll
            for (int u = 0; u < kKU; u++)
                if (k0 + NT * u < nk) knode[k0 + NT * u] = cm[u];
        }
        sync();
        { NodeArr t = A; A = B; B = t; }
        n = T + U;
        seq_next += T;
        tprev = T;
        OCT_MARK();
        if (!careful) {
            if (n >= N || n == prev) finish = true;               // :667-670
            else if (n + n_to_expand * 3 > N) careful = true;      // :671
        } else {
            if (n >= N || n == prev) finish = true;               // :732-733
        }
    }

    // ---- retain the best key of each node (:740-758)
    for (int i = tid; i < n; i += NT) best[i] = 0;
    sync();
    for (int k0 = tid; k0 < nk; k0 += kKU * NT) {
        uint32_t key[kKU];
        int nd[kKU];
#pragma unroll
        for (int u = 0; u < kKU; u++) {
            const int k = min(k0 + NT * u, nk - 1);
            key[u] = keys[k];
            nd[u] = knode[k];
        }
#pragma unroll
        for (int u = 0; u < kKU; u++) {
            const int k = k0 + NT * u;
            if (k < nk) atomicMax(&best[nd[u]], ((uint32_t)kp_s(key[u]) << 24) | (uint32_t)(0xFFFFFF - k));
        }
    }
    sync();
    const int nout = min(n, L.kcap);
    for (int i = tid; i < nout; i += NT) {
        const int k = 0xFFFFFF - (int)(best[i] & 0xFFFFFF);
        const uint32_t key = keys[k];
        okp[i] = pack_kp(kp_x(key) + L.minBX, kp_y(key) + L.minBY, kp_s(key));
    }
    if (n > L.kcap) err |= kErrOctreeNodes;
    if (tid == 0) {
        *out_cnt = nout;
        if (err) atomicOr(&b.err[f], err);
    }
#ifdef SLAMHOT_OCTREE_TRACE
    OCT_MARK();
    if (trace) {
        long long d[10] = {};
        for (int i = 1; i < ntr && i <= 10; i++) d[i - 1] = tr[i] - tr[i - 1];
        printf("OCT W=%d f=%d l=%d nk=%d n=%d marks=%d: %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld tot=%lld\n", W, f, l,
               nk, n, ntr, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], tr[ntr - 1] - tr[0]);
    }
#endif
}

// ---------------------------------------------------------------------------------------
// k_layout: output order of operator() (ORBextractor.cc:1100-1146), one workgroup per
// frame.  Keypoints are visited level-major in octree order; those whose scaled x lies in
// [lap0, lap1] are written from the back, the rest from the front; returns monoIndex.
// The level-major order is the order of the keypoint slots (level l at kbase_l, its first
// ocnt_l slots used), so each thread takes a run of consecutive slots and one block scan of
// its (lapping, front) counts, packed in one int, places all of them.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_layout(Bufs b) {
    __shared__ int scratch[20];
    const DevPlan& P = *b.plan;
    const int f = blockIdx.x, tid = threadIdx.x, NT = blockDim.x;
    const int32_t* ocnt = b.ocnt + (size_t)f * P.nlevels;
    const int K = P.kslots, per = (K + NT - 1) / NT, s0 = min(tid * per, K), s1 = min(s0 + per, K);
    const float lap0 = (float)b.lap0, lap1 = (float)b.lap1;
    const uint32_t* okp = b.okp + (size_t)f * P.kslots;
    int32_t* oidx = b.oidx + (size_t)f * P.kslots;
    int total = 0, l = 0;
    for (int i = 0; i < P.nlevels; i++) {
        total += ocnt[i];
        if (i > 0 && P.lv[i].kbase <= s0) l = i;  // level of this thread's first slot
    }
    // slot s: 0 unused, 1 front, 2 lapping
    auto kind = [&](int s, int& lv) -> int {
        while (lv + 1 < P.nlevels && s >= P.lv[lv + 1].kbase) lv++;
        const DevLevel& L = P.lv[lv];
        if (s - L.kbase >= ocnt[lv]) return 0;
        float x = (float)kp_x(okp[s]);
        if (lv != 0) x = x * L.scale;  // keypoint->pt *= scale (:1131-1133)
        return x >= lap0 && x <= lap1 ? 2 : 1;
    };
    int nlap = 0, nfront = 0;
    {
        int lv = l;
        for (int s = s0; s < s1; s++) {
            const int k = kind(s, lv);
            nlap += k == 2;
            nfront += k == 1;
        }
    }
    int tot;
    const int packed = (nlap << 16) | nfront;  // both counts < 2^16 (slots per frame)
    const int excl = block_scan_incl(packed, scratch, &tot) - packed;
    int ls = excl >> 16, lm = excl & 0xFFFF;  // lapping / front keypoints before this run
    {
        int lv = l;
        for (int s = s0; s < s1; s++) {
            const int k = kind(s, lv);
            if (k == 2) oidx[s] = total - 1 - ls++;
            else if (k == 1) oidx[s] = lm++;
        }
    }
    if (tid == 0) {
        b.out_n[f] = total;
        b.out_mono[f] = tot & 0xFFFF;
        if (total > b.cap) atomicOr(&b.err[f], kErrCap);
    }
}

// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) (OpenCV 4.2.0 fixed-point 8U path: Q8 taps
// [18,34,48,56,48,34,18], exact u16 row sums, Q16 column sums rounded >> 16) helpers.
__device__ __forceinline__ int refl101(int i, int n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
    return i;
}



// ---------------------------------------------------------------------------------------
// k_orb3: IC angle + GaussianBlur + rBRIEF fused, one wave per keypoint (one per workgroup).
// The reference blurs a clone of every level (ORBextractor.cc:1113-1115) only to sample it
// at the 512 pattern points of each keypoint; here each wave blurs just the 37x37 window the
// rotated pattern can reach (radius 18.38 -> rounded offsets within +-18), from one 43x43
// raw window that also serves IC_Angle (its 31x31 disc is the window's centre).  Same
// integer arithmetic as the OpenCV 8U fixed-point path (Q8 taps, exact row sums, rounded
// (acc + 2^15) >> 16, BORDER_REFLECT_101 at the level bounds), so the bits are those of the
// whole-level blur; the blurred level is never written to HBM.
//   raw: 43 rows x 12 dwords (staged byte j <-> level column xs + j, xs = (kx-21) & ~3)
//   hp : 22 row pairs x 40 dwords of exact horizontal sums, rows 2p | 2p+1 << 16 (column
//        c <-> kx - 18 + c)
// The vertical pass runs only at the sampled pixels (the descriptor stage reads hp directly).
// One 3,520-byte region per wave holds both: hp from byte 0, raw from byte kO3RawOff
// (checked below: each of the horizontal pass's three wave passes writes hp rows that lie
// below every raw byte the later passes read).
// ---------------------------------------------------------------------------------------
constexpr int kO3R = 43, kO3Pairs = 22, kO3RawS = 12, kO3HS = 40;

// Horizontal-pass items (row pair p, 4-column group q) that a sampled pixel can depend on.  A
// pattern point of radius r lands, rotated and rounded to the pixel grid, within r + sqrt(2)/2
// of the keypoint; the largest r is 13 sqrt(2) = 18.385, so every sampled offset (dy, dx) has
// dy^2 + dx^2 <= 364 (19.092^2 = 364.5).  Blurred pixel (y, x) reads row sums y .. y+6 of column x.
// 189 of the 22 x 10 items qualify; the corner items' row sums stay unwritten and only feed
// blurred corner pixels no sample reads.
struct HItems {
    uint8_t v[kO3Pairs * 10];
    int n;
};
constexpr HItems make_hitems() {
    bool need[kO3Pairs][10] = {};
    for (int dy = -18; dy <= 18; dy++)
        for (int dx = -18; dx <= 18; dx++) {
            if (dy * dy + dx * dx > 364) continue;
            for (int hr = dy + 18; hr <= dy + 24; hr++) need[hr / 2][(dx + 18) / 4] = true;
        }
    HItems h{};
    for (int p = 0; p < kO3Pairs; p++)
        for (int q = 0; q < 10; q++)
            if (need[p][q]) h.v[h.n++] = (uint8_t)(p * 10 + q);  // item index of the full 22 x 10 grid
    return h;
}
constexpr HItems kHItemsTable = make_hitems();
constexpr int kHItems = kHItemsTable.n;
static_assert(kHItems <= 192, "horizontal pass items must fit three wave passes");
__constant__ HItems c_hitems = kHItemsTable;

// Smallest 16-byte aligned raw offset such that the hp bytes written by wave pass k (items
// 64k .. 64k+63, 16 B at p*160 + q*16) all lie below the lowest raw byte any later pass reads
// (rows 2p and 2p+1 from dword q: 96p + 4q onwards).
constexpr int hp_raw_offset() {
    for (int x = 0;; x += 16) {
        bool ok = true;
        for (int k = 0; 64 * (k + 1) < kHItems; k++) {
            int we = 0, rs = 1 << 30;
            for (int it = 64 * k; it < 64 * (k + 1); it++) {
                const int p = kHItemsTable.v[it] / 10, q = kHItemsTable.v[it] % 10;
                we = we > p * 160 + q * 16 + 16 ? we : p * 160 + q * 16 + 16;
            }
            for (int it = 64 * (k + 1); it < kHItems; it++) {
                const int p = kHItemsTable.v[it] / 10, q = kHItemsTable.v[it] % 10;
                rs = rs < x + 96 * p + 4 * q ? rs : x + 96 * p + 4 * q;
            }
            if (we > rs) ok = false;
        }
        if (ok) return x;
    }
}
constexpr int kO3RawOff = hp_raw_offset();
// bytes per wave: hp (22 x 160) or raw incl. the discarded 44th row read (16 B past dword 9)
constexpr int kO3WaveBytes = (kO3Pairs * kO3HS * 4 > kO3RawOff + (kO3R + 1) * kO3RawS * 4 + 4)
                                 ? kO3Pairs * kO3HS * 4
                                 : ((kO3RawOff + (kO3R + 1) * kO3RawS * 4 + 4 + 15) & ~15);
static_assert(kO3RawOff % 16 == 0 && kO3WaveBytes % 16 == 0, "16-byte aligned staging");

// One wave (keypoint) per workgroup: each wave frees its LDS and slot the moment it is done
// (keypoint waves finish at different times, and slots past a level's count exit at once).
// 4 per workgroup measured 0.190 ms per 128 EuRoC frames, 1 per workgroup 0.165 ms (headline
// 95.9k -> 101.0k stereo frames/s, interleaved A/B); 2 per workgroup 0.188 ms.
#ifndef SLAMHOT_ORB_WPG
#define SLAMHOT_ORB_WPG 1
#endif
constexpr int kOrbWpg = SLAMHOT_ORB_WPG;  // waves (keypoints) per workgroup

// The 7-tap Gaussian (sigma 2, CV_8U fixed point: taps sum to 256) as byte weights against the
// staged dwords: hblur_w(o, m) = the taps of an output whose window starts at byte o, over
// staged dword m (bytes 4m .. 4m+3); zero where the window misses the dword.
constexpr int kHTap[7] = {18, 34, 48, 56, 48, 34, 18};
constexpr uint32_t hblur_w(int o, int m) {
    uint32_t w = 0;
    for (int j = 0; j < 4; j++) {
        const int t = 4 * m + j - o;
        if (t >= 0 && t <= 6) w |= (uint32_t)kHTap[t] << (8 * j);
    }
    return w;
}
template <int O, int M>
__device__ __forceinline__ uint32_t hdot(const uint32_t (&D)[4], uint32_t acc) {
    if constexpr (hblur_w(O, M) != 0) return __builtin_amdgcn_udot4(D[M], hblur_w(O, M), acc, false);
    else return acc;
}
// one staged row, 4 output columns of shift SH: h[c] sums bytes SH+c .. SH+c+6
template <int SH>
__device__ __forceinline__ void hrow_sh(const uint32_t* row, uint32_t* h) {
    const uint32_t D[4] = {row[0], row[1], row[2], SH == 3 ? row[3] : 0u};
    h[0] = hdot<SH, 2>(D, hdot<SH, 1>(D, hdot<SH, 0>(D, 0u)));
    h[1] = hdot<SH + 1, 3>(D, hdot<SH + 1, 2>(D, hdot<SH + 1, 1>(D, hdot<SH + 1, 0>(D, 0u))));
    h[2] = hdot<SH + 2, 3>(D, hdot<SH + 2, 2>(D, hdot<SH + 2, 1>(D, hdot<SH + 2, 0>(D, 0u))));
    h[3] = hdot<SH + 3, 3>(D, hdot<SH + 3, 2>(D, hdot<SH + 3, 1>(D, hdot<SH + 3, 0>(D, 0u))));
}
static_assert(hblur_w(0, 2) == 0 && hblur_w(2, 3) == 0 && hblur_w(5, 3) == 0 && hblur_w(6, 3) == 18,
              "dword 3 only for windows starting at byte 6; dword 2 not at byte 0");

__global__ void __launch_bounds__(64 * kOrbWpg) k_orb3(Bufs b) {
    // hp and raw share one region per wave (3,520 B per wave)
    __shared__ __attribute__((aligned(16))) uint32_t buf_all[kOrbWpg][kO3WaveBytes / 4];
    const DevPlan& P = *b.plan;
    const int2 blk = xcd_block();
    const int f = blk.y;
    const int wave = kOrbWpg == 1 ? 0 : threadIdx.x >> 6;
    const int slot = blk.x * kOrbWpg + wave;
    const int lane = threadIdx.x & 63;
#ifdef SLAMHOT_ORB_TRACE
    long long otr[8];
    int notr = 0;
    const bool otrace = f == 100 && (slot % 97) == 5 && lane == 0;
#define ORB_MARK() do { if (otrace) otr[notr++] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define ORB_MARK() do {} while (0)
#endif
    ORB_MARK();
    // The prologue is a chain of dependent loads every wave waits through, kept to three steps:
    // (1) the kernel arguments; (2) the keypoint, its output index and the levels' first slots
    // (lane k: level k, one vector load) together, the level = the ballot of the slot against
    // those; (3) the level's fields (scalar loads) and its keypoint count.
    const int nlev = b.nlevels, kslots = b.kslots;
    if (slot >= kslots) return;
    const int oi = b.oidx[(size_t)f * kslots + slot];
    const uint32_t key = b.okp[(size_t)f * kslots + slot];
    // INT_MAX past the last level: lanes >= kMaxLevels must not repeat level kMaxLevels-1's kbase
    // (with nlevels == kMaxLevels that would push the ballot count past the table)
    const int kb = lane < kMaxLevels ? P.orb_lv[lane].kbase : INT_MAX;
    const int l = __builtin_amdgcn_readfirstlane(__popcll(__ballot(slot >= kb)) - 1);  // kbase[0] = 0
    const OrbLv& O = P.orb_lv[l];
    if ((slot - O.kbase >= b.ocnt[(size_t)f * nlev + l]) | (oi >= b.cap)) return;  // one branch
    const int lw = O.w, lh = O.h, pitch = O.pitch;
    const uint8_t* img = (l ? (const uint8_t*)b.pyr : b.img) + (size_t)f * O.fstride + O.off;
    const int kx = kp_x(key), ky = kp_y(key);
    uint32_t* hp = buf_all[wave];
    uint32_t* raw = buf_all[wave] + kO3RawOff / 4;
    const int xs = (kx - 21) & ~3, sh = (kx - 21) - xs;
    // the orientation's weights (DevPlan::ic_w) for this lane's disc row, loaded with the window
    const uint4* icw;
    {
        const int row = lane >> 1;
        const int av = row < 2 * kHalfPatch + 1 ? abs(row - kHalfPatch) : kHalfPatch + 1;
        icw = reinterpret_cast<const uint4*>(P.ic_w[sh][av][lane & 1]);
    }
    const uint4 icw0 = icw[0], icw1 = icw[1], icw2 = icw[2];
    ORB_MARK();
    // ---- stage the raw window    ORB_MARK();
    // ---- stage the raw window (rows ky-21..ky+21 reflected, 12 dwords per row) as three
    // 16-byte pieces per row: 129 pieces, <= 3 per lane, loaded together; pieces that leave
    // the level go byte by byte through BORDER_REFLECT_101 afterwards, one at a time
    {
        const int wfull = (pitch & 3) ? 0 : (lw & ~3);
        uint4 v[3];
        uint32_t slow = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int e = lane + 64 * k;
            v[k] = make_uint4(0, 0, 0, 0);
            if (e < kO3R * 3) {
                const int r = e / 3, part = e - 3 * r;
                const int x = xs + 16 * part;
                if (x >= 0 && x + 16 <= wfull)
                    v[k] = *reinterpret_cast<const uint4*>(img + (size_t)refl101(ky - 21 + r, lh) * pitch + x);
                else
                    slow |= 1u << k;
            }
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int e = lane + 64 * k;
            if (e < kO3R * 3) {
                const int r = e / 3, part = e - 3 * r;
                if (!(slow >> k & 1)) *reinterpret_cast<uint4*>(raw + r * kO3RawS + 4 * part) = v[k];  // 16-byte aligned
            }
        }
        for (int k = 0; k < 3; k++) {
            if (!(slow >> k & 1)) continue;
            const int e = lane + 64 * k;
            const int r = e / 3, part = e - 3 * r;
            const uint8_t* rowp = img + (size_t)refl101(ky - 21 + r, lh) * pitch;
            const int x = xs + 16 * part;
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 16; q++) w[q >> 2] |= (uint32_t)rowp[refl101(min(x + q, lw + 3), lw)] << (8 * (q & 3));
            *reinterpret_cast<uint4*>(raw + r * kO3RawS + 4 * part) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    ORB_MARK();

    // ---- orientation (IC_Angle, ORBextractor.cc:75-102) on the raw centre 31x31
    // Lane = (disc row v, half): the row's bytes as staged dwords (row 21 + v, dwords 1..5 for
    // half 0, 6..10 for half 1: bytes 4..43 hold every column kx-15..kx+15 for any sh) against two
    // weight dwords each (DevPlan::ic_w, by sh, |v| and half): the disc's bytes |u| <= umax[|v|]
    // as 1 (row sum) and as their byte offset b (moment), so sum u I = moment - (sh + 21) sum.
    // Exact integers, like the reference's loops; row 31 (lanes 62, 63) has zero weights.
    int m01, m10;
    {
        const int v = (lane >> 1) - kHalfPatch;
        const uint32_t* rp = raw + (21 + v) * kO3RawS + ((lane & 1) ? 6 : 1);
        const uint32_t w0[5] = {icw0.x, icw0.y, icw0.z, icw0.w, icw1.x};
        const uint32_t w1[5] = {icw1.y, icw1.z, icw1.w, icw2.x, icw2.y};
        uint32_t s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const uint32_t x = rp[i];
            s0 = __builtin_amdgcn_udot4(x, w0[i], s0, false);
            s1 = __builtin_amdgcn_udot4(x, w1[i], s1, false);
        }
        m10 = (int)s1 - (sh + 21) * (int)s0;
        m01 = v * (int)s0;
    }
    m10 = wave_sum_dpp(m10);
    m01 = wave_sum_dpp(m01);
    const float angle = cv_fast_atan2((float)m01, (float)m10);
    ORB_MARK();

    // ---- horizontal pass: 22 row pairs x 10 groups of 4 output columns; output column c
    // needs staged bytes sh+c .. sh+c+6.  sh is wave-uniform: one specialisation per sh, with the
    // seven taps placed at each output's byte offset against the staged dwords (hblur_w), two or
    // three v_dot4 per output and no data realignment.  Rows 2p and 2p+1 go to the low / high
    // half of one dword (hp), so the vertical pass takes two taps per v_dot2_u32_u16.  Row 43 is
    // never staged: its sums only reach blurred rows >= 37, which are not kept.
    int hit[3];
#pragma unroll
    for (int k = 0; k < 3; k++) hit[k] = c_hitems.v[min(lane + 64 * k, kHItems - 1)];
    auto hpass = [&](auto shc) {
        constexpr int SH = decltype(shc)::value;
#pragma unroll
        for (int k = 0; k < 3; k++) {  // 3 passes of the wave instead of 4
            if (lane + 64 * k >= kHItems) break;
            const int pq = hit[k], p = pq / 10, q = pq - p * 10;
            uint32_t h0[4], h1[4];
            hrow_sh<SH>(raw + (2 * p) * kO3RawS + q, h0);
            hrow_sh<SH>(raw + (2 * p + 1) * kO3RawS + q, h1);
            *reinterpret_cast<uint4*>(&hp[p * kO3HS + 4 * q]) =
                make_uint4(h0[0] | (h1[0] << 16), h0[1] | (h1[1] << 16), h0[2] | (h1[2] << 16), h0[3] | (h1[3] << 16));
        }
    };
    switch (sh) {
        case 0: hpass(std::integral_constant<int, 0>{}); break;
        case 1: hpass(std::integral_constant<int, 1>{}); break;
        case 2: hpass(std::integral_constant<int, 2>{}); break;
        default: hpass(std::integral_constant<int, 3>{}); break;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    ORB_MARK();
    // ---- descriptor (computeOrbDescriptor, ORBextractor.cc:106-145), with the vertical pass
    // of the blur evaluated only at the 512 sampled pixels of the 37x37 window.
    const float factor_pi = (float)(3.14159265358979323846 / 180.f);
    float sn, cs;
    glibc_sincosf(angle * factor_pi, &sn, &cs);
    const float a = cs, bb = sn;
    ORB_MARK();
    // Per pattern point: (r, c) = the rotated offset as a packed pair, rounded to nearest-even
    // by adding 1.5 * 2^23 + 18 (cv_round's rint, shifted by the window centre 18, exact for
    // |v| < 2^22): the sum's low bits are r + 18 and c + 18 on top of 0x4B400000.  Blurred pixel
    // (y, x) sums hs rows y .. y+6 of column x: the row pairs y >> 1 .. (y >> 1) + 3, realigned
    // by v_alignbit to start at row y (16 bits for odd y), then fixed taps (k0,k1)(k2,k3)(k4,k5)
    // (k6,-).  acc starts at 2^15 (the rounding term); taps sum to 256, so acc >> 16 <= 255:
    // the whole-level blur's byte, and (acc0 >> 16) < (acc1 >> 16) <=> acc0 < (acc1 & ~0xFFFF).
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 rot_a = {a, -bb}, rot_b = {bb, a};
    constexpr float kRound = 12582930.0f;  // 1.5 * 2^23 + 18
    auto sample = [&](float x, float y) -> uint32_t {
        // r = fma(x, b, y a), c = fma(x, a, -(y b)) (computeOrbDescriptor's GET_VALUE), y (-b) = -(y b)
        const f2 yy = f2{y, y} * rot_a;
        const f2 rc = __builtin_elementwise_fma(f2{x, x}, rot_b, yy);  // {r, c} unrounded
        const f2 rcr = rc + f2{kRound, kRound};
        const uint32_t rb = __float_as_uint(rcr.x), cb = __float_as_uint(rcr.y);
        // (y >> 1) * kO3HS + x from the biased bits: v_mad_u32_u24 reads the low 24 bits of rb >> 1
        // (0xA00000 + (y >> 1)); the constant bias is taken back out of the index
        const uint32_t idx = __umul24(rb >> 1, kO3HS) + cb - (0xA00000u * kO3HS + 0x4B400000u);
        const uint32_t* q = hp + idx;
        const uint32_t q0 = q[0], q1 = q[kO3HS], q2 = q[2 * kO3HS], q3 = q[3 * kO3HS];
        const uint32_t sft = rb << 4;  // v_alignbit reads bits [4:0]: 16 for odd y
        uint32_t acc = 1u << 15;
        acc = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_alignbit(q1, q0, sft)), us2{18, 34}, acc, false);
        acc = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_alignbit(q2, q1, sft)), us2{48, 56}, acc, false);
        acc = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_alignbit(q3, q2, sft)), us2{48, 34}, acc, false);
        acc = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_alignbit(q3, q3, sft)), us2{18, 0}, acc, false);
        return acc;
    };
    uint64_t m[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const float4 pt = c_patternf.v[w * 64 + lane];
        const uint32_t acc0 = sample(pt.x, pt.y), acc1 = sample(pt.z, pt.w);
        m[w] = __ballot(acc0 < (acc1 & 0xFFFF0000u));
    }
    uint8_t* desc = b.out_desc + ((size_t)f * b.cap + oi) * 32;
    if (lane < 4) reinterpret_cast<uint64_t*>(desc)[lane] = lane == 0 ? m[0] : lane == 1 ? m[1] : lane == 2 ? m[2] : m[3];
    if (lane == 4) {
        slam_keypoint kp;
        kp.x = l ? (float)kx * O.scale : (float)kx;
        kp.y = l ? (float)ky * O.scale : (float)ky;
        kp.size = O.size;
        kp.angle = angle;
        kp.response = (float)kp_s(key);
        kp.octave = l;
        kp.class_id = -1;
        b.out_kps[(size_t)f * b.cap + oi] = kp;
    }
#ifdef SLAMHOT_ORB_TRACE
    ORB_MARK();
    if (otrace)
        printf("ORB slot=%d l=%d pro %lld stage %lld ic %lld horiz %lld sincos %lld desc %lld\n", slot, l, otr[1] - otr[0],
               otr[2] - otr[1], otr[3] - otr[2], otr[4] - otr[3], otr[5] - otr[4], otr[6] - otr[5]);
#endif
}

}  // namespace slamhot

// =======================================================================================
// Host side: the slam_extractor handle and the C-ABI (include/slamhot.h).
// =======================================================================================
namespace slamhot {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    slam_status ensure(size_t need) {
        if (need <= bytes) return SLAM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (need == 0) return SLAM_OK;
        if (hipMalloc(&p, need) != hipSuccess) return SLAM_ENOMEM;
        bytes = need;
        return SLAM_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

enum Stage { kStResize = 0, kStFast, kStOctree, kStLayout, kStOrb, kNumStages };
static const char* kStageNames[kNumStages] = {"k_resize", "k_fast_wave", "k_octree",
                                              "k_layout", "k_orb"};

}  // namespace slamhot

using namespace slamhot;

constexpr int kSmallBatch = 8;  // batches up to this size: the small-batch octree launch

struct slam_extractor {
    slam_orb_params prm{};
    int device = 0;
    int max_w = 0, max_h = 0, max_batch = 0;
    hipStream_t stream = nullptr;
    // sub-batch concurrency: a batch is split into nsub frame ranges, each running the whole
    // pipeline on its own stream; latency-bound stages of one
    // range (octree, orb) overlap the VALU-bound FAST of another
    static constexpr int kMaxSub = 4;
    int nsub = 1;
    bool chain_fast = false;
    hipStream_t sub[kMaxSub] = {};
    hipEvent_t sub_fork = nullptr, sub_join[kMaxSub] = {}, sub_fast[kMaxSub] = {};
    bool serial = false;
    std::mutex mu;
    // geometry
    bool have_plan = false;
    Plan plan;
    DevBuf d_plan, d_xtab, d_ytab, d_cells, d_wave_cells, d_wide_cells;
    int n_wave_cells = 0, n_wide_cells = 0;
    FastWaveLds fw_lay{}, fw_lay_b{};  // layouts of the two wave-cell classes (see below)
    FastWaveLds fw_lay_all{};          // one layout for every wave cell (small batches: one dispatch)
    int n_wave_a = 0;                  // d_wave_cells: class A cells first, then class B
    // per-batch buffers
    DevBuf d_img, d_pyr, d_cell_keys, d_cell_cnt, d_keys_g, d_knode_g, d_okp, d_ocnt,
        d_oidx, d_err, d_kps, d_desc, d_n, d_mono;
    int last_frames = 0;
    const uint8_t* last_img = nullptr;  // level-0 pointer of the last run (for pyramid_level)
    // host-buffer path (slamhot_extract / _batch, the call Frame.cc:119-122 makes per image):
    // pinned staging in and out, one device output block, and the whole call (H2D, pipeline,
    // D2H) captured once per shape as a HIP graph and replayed (host_graph below)
    void* h_in = nullptr;
    size_t h_in_bytes = 0;
    void* h_out = nullptr;
    size_t h_out_bytes = 0;
    DevBuf d_out;
    hipGraphExec_t hg_exec = nullptr;
    std::vector<uintptr_t> hg_key;
    bool hg_off = false;  // a capture failed, or SLAMHOT_EXTRACT_GRAPH=0: plain stream calls
    // k_octree launch groups: {first level, levels, keys held in LDS, dynamic LDS bytes}
    struct OctGroup { int l0, nl, keycap; size_t lds; };
    OctGroup oct[2] = {};
    int n_oct = 0;
    // small batches (the per-image call): every level in one launch with its keys in LDS; the
    // two-group split above is for the concurrent batch pipeline, where the octree's LDS is
    // taken from other batches' FAST / orb and level 0 keeps its keys in L2 (one VGA frame:
    // level 0 115 us + levels 1-7 49 us as two launches)
    OctGroup oct_small{};
    OctGroup oct_all{};  // every level in one launch at the levels-1.. budget (SLAMHOT_OCT_MERGE=1, A/B)
    int octree_max_cells = 1;
    // per-stage HIP-event timing (slamhot_extractor_set_profiling)
    bool profiling = false;
    struct Mark { int stage; hipEvent_t a, b; };
    std::vector<Mark> marks;
    std::vector<hipEvent_t> pool;
    double stage_ms[kNumStages] = {};
    long stage_launches[kNumStages] = {};
    hipEvent_t ev() {
        if (pool.empty()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
};

static slam_status ensure_plan(slam_extractor* ex, int W, int H) {
    if (ex->have_plan && ex->plan.W == W && ex->plan.H == H) return SLAM_OK;
    Plan P;
    if (!build_plan(ex->prm, W, H, P)) return SLAM_EINVAL;
    DevPlan dp{};
    dp.nlevels = P.nlevels;
    dp.W = W;
    dp.H = H;
    dp.ncells = P.ncells;
    dp.slot_cap = P.slot_cap;
    dp.kslots = P.kslots;
    dp.key_slots = P.key_slots;
    dp.max_nodes = P.max_nodes;
    dp.ini_th = ex->prm.ini_th_fast;
    dp.min_th = ex->prm.min_th_fast;
    dp.pyr_frame = P.pyr_frame;
    dp.blur_frame = P.blur_frame;
    {
        // umax (ORBextractor.cc:452-467)
        int umax[kHalfPatch + 1];
        const int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
        const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
        const double hp2 = kHalfPatch * kHalfPatch;
        for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
        for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
        for (int v = 0; v <= kHalfPatch; v++) dp.umax[v] = umax[v];
        // k_orb3's IC_Angle weights: lane (row v, half) holds staged dwords k0 .. k0+4 (k0 = 1 or
        // 6) of window row 21 + v, whose byte b is column b - (sh + 21) from the keypoint
        for (int sh = 0; sh < 4; sh++)
            for (int av = 0; av <= kHalfPatch + 1; av++)
                for (int half = 0; half < 2; half++) {
                    uint32_t* w = dp.ic_w[sh][av][half];
                    const int c0 = sh + 21, d = av <= kHalfPatch ? umax[av] : -1;  // -1: no bytes
                    for (int i = 0; i < 12; i++) w[i] = 0;
                    for (int i = 0; i < 5; i++)
                        for (int j = 0; j < 4; j++) {
                            const int bo = 4 * ((half ? 6 : 1) + i) + j;
                            if (d >= 0 && bo >= c0 - d && bo <= c0 + d) {
                                w[i] |= 1u << (8 * j);
                                w[5 + i] |= (uint32_t)bo << (8 * j);
                            }
                        }
                }
    }
    for (int l = 0; l < P.nlevels; l++) {
        const LevelPlan& L = P.lv[l];
        DevLevel& D = dp.lv[l];
        D.w = L.w; D.h = L.h; D.pitch = L.pitch;
        D.pyr_off = L.pyr_off; D.blur_off = L.blur_off;
        D.minBX = L.minBX; D.minBY = L.minBY; D.maxBX = L.maxBX; D.maxBY = L.maxBY;
        D.cell_begin = L.cell_begin; D.cell_end = L.cell_end;
        D.nfeat = L.nfeat; D.kbase = L.kbase; D.kcap = L.kcap;
        D.key_base = L.key_base; D.key_cap = L.key_cap;
        D.scale = L.scale; D.size = L.size; D.nIni = L.nIni;
        for (int i = 0; i < kMaxRoots; i++) {
            D.root_x0[i] = L.root_x0[i]; D.root_x1[i] = L.root_x1[i]; D.root_first_x[i] = L.root_first_x[i];
        }
        D.xtab_off = L.xtab_off; D.ytab_off = L.ytab_off; D.xmax = L.xmax;
        OrbLv& O = dp.orb_lv[l];
        O.kbase = L.kbase; O.w = L.w; O.h = L.h; O.pitch = l ? L.pitch : W;
        O.off = l ? L.pyr_off : 0;
        O.fstride = l ? P.pyr_frame : (int64_t)W * H;
        O.scale = L.scale; O.size = L.size;
    }
    for (int l = P.nlevels; l < kMaxLevels; l++) dp.orb_lv[l].kbase = 0x7FFFFFFF;
    slam_status st;
    if ((st = ex->d_plan.ensure(sizeof(DevPlan))) ||
        (st = ex->d_xtab.ensure(std::max<size_t>(16, P.xtab.size() * sizeof(ResizeX)))) ||
        (st = ex->d_ytab.ensure(std::max<size_t>(16, P.ytab.size() * sizeof(ResizeY)))) ||
        (st = ex->d_cells.ensure(P.cells.size() * sizeof(CellDesc))))
        return st;
    SLAM_HIP_TRY(hipMemcpy(ex->d_plan.p, &dp, sizeof(DevPlan), hipMemcpyHostToDevice));
    if (!P.xtab.empty())
        SLAM_HIP_TRY(hipMemcpy(ex->d_xtab.p, P.xtab.data(), P.xtab.size() * sizeof(ResizeX), hipMemcpyHostToDevice));
    if (!P.ytab.empty())
        SLAM_HIP_TRY(hipMemcpy(ex->d_ytab.p, P.ytab.data(), P.ytab.size() * sizeof(ResizeY), hipMemcpyHostToDevice));
    SLAM_HIP_TRY(hipMemcpy(ex->d_cells.p, P.cells.data(), P.cells.size() * sizeof(CellDesc), hipMemcpyHostToDevice));
    {
        // cells whose tested region fits one wave (<= 64 columns, <= kRoiRows rows) take the
        // wave-per-cell kernel; the rest (tiny levels of small images) the workgroup kernel
        std::vector<int32_t> wave, wide;
        std::vector<const CellDesc*> wc;
        for (const CellDesc& c : P.cells) {
            if (c.cw - 6 <= 64 && c.ch <= kRoiRows && c.cw + 3 <= kRoiStride) wc.push_back(&c);
            else wide.push_back(c.slot);
        }
        // Two classes, each with an LDS layout sized to its own largest cell: class A = the
        // cells that fit the most common cell's box (the full cells of the fine levels), class
        // B = the rest (clipped or coarse-level cells up to ~46 x 57).  One layout for all
        // would size every wave for the largest cell (EuRoC: 9.4 KB, 4 workgroups per CU); class
        // A needs 6.5 KB (6 per CU) and holds ~3/4 of the cells.
        int box_w = 0, box_h = 0;
        {
            std::vector<std::pair<int, int>> dims;
            for (const CellDesc* c : wc) dims.emplace_back(c->cw, c->ch);
            std::sort(dims.begin(), dims.end());
            int best = 0;
            for (size_t i = 0; i < dims.size();) {
                size_t j = i;
                while (j < dims.size() && dims[j] == dims[i]) j++;
                if ((int)(j - i) > best) {
                    best = (int)(j - i);
                    box_w = dims[i].first;
                    box_h = dims[i].second;
                }
                i = j;
            }
        }
        if (std::getenv("SLAMHOT_FAST_ONE_CLASS")) box_w = box_h = 1 << 20;
        std::vector<int32_t> wave_b;
        for (const CellDesc* c : wc) (c->cw <= box_w && c->ch <= box_h ? wave : wave_b).push_back(c->slot);
        auto r16 = [](int v) { return (v + 15) & ~15; };
        auto layout_of = [&](const std::vector<int32_t>& list) {
            int ch_max = 0, th_max = 0, tw_max = 0, cw_max = 0;
            for (int32_t sl : list) {
                const CellDesc& c = P.cells[sl];
                ch_max = std::max(ch_max, (int)c.ch);
                th_max = std::max(th_max, c.ch - 6);
                tw_max = std::max(tw_max, c.cw - 6);
                cw_max = std::max(cw_max, (int)c.cw);
            }
            FastWaveLds lay;
            // ROI rows: staged dwords reach byte sh + cw + 3 and pass A reads one dword past its
            // last group, so cw + 8 bytes (rounded to dwords) cover every access
            lay.rs = std::min(kRoiStride, (cw_max + 8 + 3) & ~3);
            // SLAMHOT_FAST_RS_PAD=<dwords>: extra ROI row stride (LDS bank-spread probe)
            if (const char* e = std::getenv("SLAMHOT_FAST_RS_PAD")) lay.rs += 4 * std::max(0, std::atoi(e));
            lay.ms = tw_max + 2;
            lay.roi = 0;
            lay.map = r16(ch_max * lay.rs);
            lay.lst = lay.map + r16((th_max + 2) * lay.ms);
            lay.total = lay.lst + r16(std::max(1, tw_max * th_max) * 2);
            return lay;
        };
        FastWaveLds lay = layout_of(wave);
        ex->fw_lay_b = layout_of(wave_b);
        ex->n_wave_a = (int)wave.size();
        wave.insert(wave.end(), wave_b.begin(), wave_b.end());
        ex->fw_lay = lay;
        ex->fw_lay_all = layout_of(wave);  // wave now holds both classes
        if (4 * lay.total > 160 * 1024 || 4 * ex->fw_lay_b.total > 160 * 1024) return SLAM_EINVAL;
        SLAM_HIP_TRY(hipFuncSetAttribute((const void*)k_fast_wave, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024));
        // the wave cells' records (FastWaveCell): staging geometry and pass-A lane map per cell
        std::vector<FastWaveCell> wcells;
        wcells.reserve(wave.size());
        auto magic = [](int d) { return (65536 + d - 1) / d; };
        for (int d = 1; d <= 20; d++)  // the lane / d identity k_fast_wave relies on
            for (int x = 0; x < 64; x++)
                if (((x * magic(d)) >> 16) != x / d) return SLAM_EINVAL;
        for (int32_t sl : wave) {
            const CellDesc& c = P.cells[sl];
            const LevelPlan& L = P.lv[c.level];
            FastWaveCell w{};
            w.pitch = c.level ? L.pitch : W;
            w.dw = (w.pitch & 3) == 0;
            w.sh = w.dw ? (c.iniX & 3) : 0;
            w.fstride = c.level ? P.pyr_frame : (int64_t)W * H;
            w.roi_off = (c.level ? L.pyr_off : 0) + (int64_t)c.iniY * w.pitch + (c.iniX - w.sh);
            w.slot = c.slot;
            w.level = c.level;
            w.iniX = c.iniX;
            w.iniY = c.iniY;
            w.cw = c.cw;
            w.ch = c.ch;
            const int wd = (w.sh + c.cw + 3) >> 2, g0 = (w.sh + 3) >> 2, g1 = (w.sh + c.cw - 4) >> 2;
            const int ng = std::max(1, g1 - g0 + 1);  // < 1: no tested column (cw < 7), cmask stays 0
            if (wd < 1 || wd > 20 || ng > 17) return SLAM_EINVAL;
            w.wd = wd;
            w.rp = 64 / wd;
            w.m_wd = magic(wd);
            w.g0 = g0;
            w.ng = ng;
            w.rpi = 64 / ng;
            w.m_ng = magic(ng);
            // unguarded dword staging when the rows it writes past the ROI stay inside the wave's
            // region in every layout the cell can run under (its class's and the one-dispatch one)
            if (w.dw) {
                const FastWaveLds& lc = (int)wcells.size() < ex->n_wave_a ? ex->fw_lay : ex->fw_lay_b;
                const int rows = c.ch + 8 * w.rp - 1;
                if (rows * lc.rs <= lc.total && rows * ex->fw_lay_all.rs <= ex->fw_lay_all.total) w.dw = 2;
            }
            wcells.push_back(w);
        }
        if ((st = ex->d_wave_cells.ensure(std::max<size_t>(sizeof(FastWaveCell), wcells.size() * sizeof(FastWaveCell)))) ||
            (st = ex->d_wide_cells.ensure(std::max<size_t>(4, wide.size() * 4))))
            return st;
        if (!wcells.empty())
            SLAM_HIP_TRY(hipMemcpy(ex->d_wave_cells.p, wcells.data(), wcells.size() * sizeof(FastWaveCell), hipMemcpyHostToDevice));
        if (!wide.empty())
            SLAM_HIP_TRY(hipMemcpy(ex->d_wide_cells.p, wide.data(), wide.size() * 4, hipMemcpyHostToDevice));
        ex->n_wave_cells = (int)wave.size();
        ex->n_wide_cells = (int)wide.size();
    }
    ex->plan = P;
    ex->have_plan = true;
    // k_octree keeps a level's keys in LDS behind its node arrays when they fit (else in
    // the per-frame global scratch, L2-resident).  The octree is latency-bound and runs
    // beside other batches' FAST / orb, so its LDS is what it takes from them: level 0 (one
    // wave per frame, ~4k candidates at VGA) keeps only its nodes in LDS and its keys in L2
    // (slower alone, +7% for the pipeline); the other levels share a launch at 20 KB / wave.
    const size_t lds_max = 160 * 1024;
    int max_cells = 1;
    for (int l = 0; l < P.nlevels; l++) max_cells = std::max(max_cells, P.lv[l].cell_end - P.lv[l].cell_begin);
    ex->octree_max_cells = max_cells;
    const size_t node_bytes = octree_lds_bytes(P.max_nodes, 0, max_cells);
    if (node_bytes + 6 * 256 + 64 > lds_max) return SLAM_EINVAL;
    auto keycap_for = [&](size_t budget) {
        budget = std::min(lds_max, std::max(budget, node_bytes + 6 * 256 + 64));
        return (int)std::min<size_t>(16384, (budget - node_bytes - 64) / 6);
    };
    size_t lds_attr = 0;
    ex->n_oct = 0;
    for (int g = 0; g < 2; g++) {
        const int l0 = g == 0 ? 0 : 1, nl = g == 0 ? 1 : P.nlevels - 1;
        if (nl <= 0) continue;
        slam_extractor::OctGroup& G = ex->oct[ex->n_oct++];
        G.l0 = l0;
        G.nl = nl;
        G.keycap = keycap_for(g == 0 ? 0 : 20 * 1024);
        G.lds = octree_lds_bytes(P.max_nodes, G.keycap, max_cells);
        lds_attr = std::max(lds_attr, G.lds);
    }
    ex->oct_all.l0 = 0;
    ex->oct_all.nl = P.nlevels;
    {
        const char* e = std::getenv("SLAMHOT_OCT_MERGE_KB");  // A/B: the merged launch's LDS budget per wave
        ex->oct_all.keycap = keycap_for((size_t)(e ? std::max(1, std::atoi(e)) : 20) * 1024);
    }
    ex->oct_all.lds = octree_lds_bytes(P.max_nodes, ex->oct_all.keycap, max_cells);
    lds_attr = std::max(lds_attr, ex->oct_all.lds);
    ex->oct_small.l0 = 0;
    ex->oct_small.nl = P.nlevels;
    ex->oct_small.keycap = keycap_for(96 * 1024);
    ex->oct_small.lds = octree_lds_bytes(P.max_nodes, ex->oct_small.keycap, max_cells);
    lds_attr = std::max(lds_attr, ex->oct_small.lds);
    SLAM_HIP_TRY(hipFuncSetAttribute((const void*)k_octree<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds_attr));
    SLAM_HIP_TRY(hipFuncSetAttribute((const void*)k_octree<kOctWaves>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds_attr));
    return SLAM_OK;
}

static slam_status ensure_batch(slam_extractor* ex, int nframes, int cap) {
    const Plan& P = ex->plan;
    const size_t F = (size_t)nframes;
    slam_status st;
    if ((st = ex->d_pyr.ensure(F * P.pyr_frame)) ||
        (st = ex->d_cell_keys.ensure(F * P.ncells * P.slot_cap * 4)) ||
        (st = ex->d_cell_cnt.ensure(F * P.ncells * 4)) ||
        (st = ex->d_keys_g.ensure(F * P.key_slots * 4)) ||
        (st = ex->d_knode_g.ensure(F * P.key_slots * 2)) ||
        (st = ex->d_okp.ensure(F * P.kslots * 4)) || (st = ex->d_ocnt.ensure(F * P.nlevels * 4)) ||
        (st = ex->d_oidx.ensure(F * P.kslots * 4)) || (st = ex->d_err.ensure(F * 4)))
        return st;
    (void)cap;
    return SLAM_OK;
}

// "1" / "0" from the environment (A/B switches), else the default
static bool env_flag(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    return e ? std::strcmp(e, "0") != 0 : dflt;
}

// One frame range [f0, f0 + nframes) of a batch: every per-frame buffer is frame-major, so
// the range is the whole pipeline on pointers advanced by f0 frames.  s = main stream,
static slam_status launch_range(slam_extractor* ex, int f0, int nframes, const uint8_t* d_img, int lap0,
                                int lap1, slam_keypoint* d_kps, uint8_t* d_desc, int cap, int32_t* d_n,
                                int32_t* d_mono, hipStream_t s, hipEvent_t fast_after = nullptr,
                                hipEvent_t fast_done = nullptr) {
    const Plan& P = ex->plan;
    const size_t F = (size_t)f0;
    Bufs b{};
    b.img = d_img + F * P.W * P.H;
    b.pyr = ex->d_pyr.as<uint8_t>() + F * P.pyr_frame;
    b.cell_keys = ex->d_cell_keys.as<uint32_t>() + F * P.ncells * P.slot_cap;
    b.cell_cnt = ex->d_cell_cnt.as<int32_t>() + F * P.ncells;
    b.keys_g = ex->d_keys_g.as<uint32_t>() + F * P.key_slots;
    b.knode_g = ex->d_knode_g.as<uint16_t>() + F * P.key_slots;
    b.okp = ex->d_okp.as<uint32_t>() + F * P.kslots;
    b.ocnt = ex->d_ocnt.as<int32_t>() + F * P.nlevels;
    b.oidx = ex->d_oidx.as<int32_t>() + F * P.kslots;
    b.err = ex->d_err.as<int32_t>() + F;
    b.out_kps = d_kps + F * cap;
    b.out_desc = d_desc + F * cap * 32;
    b.out_n = d_n + F;
    b.out_mono = d_mono + F;
    b.xtab = ex->d_xtab.as<ResizeX>();
    b.ytab = ex->d_ytab.as<ResizeY>();
    b.cells = ex->d_cells.as<CellDesc>();
    b.plan = ex->d_plan.as<DevPlan>();
    b.kslots = P.kslots;
    b.nlevels = P.nlevels;
    b.nframes = nframes;
    b.cap = cap;
    b.lap0 = lap0;
    b.lap1 = lap1;
    SLAM_HIP_TRY(hipMemsetAsync(b.err, 0, (size_t)nframes * 4, s));
    // A/B switches: SLAMHOT_OCT_SMALL / SLAMHOT_OCT_L0 = 1 | 0 (multi-wave octree on / off),
    // read per call (a handle's captured graphs keep the setting they were captured with)
    const bool oct_multi_small = env_flag("SLAMHOT_OCT_SMALL", true);
    const bool oct_multi_l0 = env_flag("SLAMHOT_OCT_L0", false);
    const bool oct_multi_rest = env_flag("SLAMHOT_OCT_REST", false);  // levels 1-7 group multi-wave (A/B)
    const bool oct_merge = env_flag("SLAMHOT_OCT_MERGE", false);      // one launch for every level (A/B)
    hipEvent_t e0 = nullptr;
    auto begin = [&](int, hipStream_t st_ = nullptr) {
        if (ex->profiling) { e0 = ex->ev(); (void)hipEventRecord(e0, st_ ? st_ : s); }
    };
    auto end = [&](int st, hipStream_t st_ = nullptr) {
        if (ex->profiling) {
            hipEvent_t e1 = ex->ev();
            (void)hipEventRecord(e1, st_ ? st_ : s);
            ex->marks.push_back({st, e0, e1});
        }
    };
#ifdef SLAMHOT_EXPERIMENT
    // experiment builds only: SLAMHOT_SKIP=<stage bitmask> leaves stages out (their inputs
    // stay those of the previous batch) to price each stage inside the concurrent pipeline
    static const int skip = std::getenv("SLAMHOT_SKIP") ? std::atoi(std::getenv("SLAMHOT_SKIP")) : 0;
#define SKIP(st) (skip & (1 << (st)))
    // SLAMHOT_FAST_LDS_PAD=<bytes>: extra dynamic LDS per FAST workgroup (occupancy probe)
    static const int fast_pad = std::getenv("SLAMHOT_FAST_LDS_PAD") ? std::atoi(std::getenv("SLAMHOT_FAST_LDS_PAD")) : 0;
#else
#define SKIP(st) 0
    constexpr int fast_pad = 0;
#endif
    begin(kStResize);
    for (int l = 1; l < P.nlevels && !SKIP(kStResize); l++) {
        const int qw = (P.lv[l].w + 3) / 4;
        const int nrb = (P.lv[l].h + kRzRows - 1) / kRzRows;
        hipLaunchKernelGGL(k_resize4, dim3((qw * nrb + 255) / 256, nframes), dim3(256), 0, s, b, l);
    }
    end(kStResize);
    // ranges run FAST one after another (each fills the chip); a range's octree / layout /
    // orb then overlap the next range's FAST
    if (fast_after) SLAM_HIP_TRY(hipStreamWaitEvent(s, fast_after, 0));
    begin(kStFast);
    if (!SKIP(kStFast)) {  // class B cells (larger LDS layout, fewer), then class A
        const int na = ex->n_wave_a, nb = ex->n_wave_cells - ex->n_wave_a;
        constexpr int G = kFastWpg;
        if (nframes <= kSmallBatch && na && nb && kFastWpg * ex->fw_lay_all.total <= 160 * 1024) {
            // a small batch fills a fraction of the chip: one dispatch over both classes at the
            // union layout saves the second launch on the per-image critical path
            hipLaunchKernelGGL(k_fast_wave, dim3((na + nb + G - 1) / G, nframes), dim3(64 * G),
                               G * ex->fw_lay_all.total + fast_pad, s, b, ex->d_wave_cells.as<FastWaveCell>(), na + nb,
                               ex->fw_lay_all);
        } else {
        if (nb)
            hipLaunchKernelGGL(k_fast_wave, dim3((nb + G - 1) / G, nframes), dim3(64 * G),
                               G * ex->fw_lay_b.total + fast_pad, s, b, ex->d_wave_cells.as<FastWaveCell>() + na, nb,
                               ex->fw_lay_b);
        if (na)
            hipLaunchKernelGGL(k_fast_wave, dim3((na + G - 1) / G, nframes), dim3(64 * G),
                               G * ex->fw_lay.total + fast_pad, s, b, ex->d_wave_cells.as<FastWaveCell>(), na, ex->fw_lay);
        }
    }
    if (ex->n_wide_cells)
        hipLaunchKernelGGL(k_fast_cells, dim3(ex->n_wide_cells, nframes), dim3(256), 0, s, b,
                           ex->d_wide_cells.as<int32_t>());
    end(kStFast);
    if (fast_done) SLAM_HIP_TRY(hipEventRecord(fast_done, s));
    begin(kStOctree);
    const bool small = nframes <= kSmallBatch;
    for (int g = 0; g < (small || oct_merge ? 1 : ex->n_oct) && !SKIP(kStOctree); g++) {
        const slam_extractor::OctGroup& G = small ? ex->oct_small : oct_merge ? ex->oct_all : ex->oct[g];
        // the per-image call (small batches) and, for large batches, level 0 run the multi-wave
        // form; levels 1-7 of large batches one wave per (frame, level)
        if (small ? oct_multi_small : (G.l0 == 0 ? oct_multi_l0 : oct_multi_rest))
            hipLaunchKernelGGL(k_octree<kOctWaves>, dim3(G.nl, nframes), dim3(64 * kOctWaves), G.lds, s, b, G.l0,
                               G.keycap, ex->octree_max_cells);
        else
            hipLaunchKernelGGL(k_octree<1>, dim3(G.nl, nframes), dim3(64), G.lds, s, b, G.l0, G.keycap,
                               ex->octree_max_cells);
    }
    end(kStOctree);
    begin(kStLayout);
    hipLaunchKernelGGL(k_layout, dim3(nframes), dim3(256), 0, s, b);
    end(kStLayout);
    begin(kStOrb);
    if (!SKIP(kStOrb)) hipLaunchKernelGGL(k_orb3, dim3((P.kslots + kOrbWpg - 1) / kOrbWpg, nframes), dim3(64 * kOrbWpg), 0, s, b);
    end(kStOrb);
    SLAM_HIP_TRY(hipGetLastError());
#undef SKIP
    return SLAM_OK;
}

// Whole batch on the caller's stream s: one range on s (small batches, SLAMHOT_SERIAL=1), or
// nsub ranges forked from s onto the handle's sub-streams and joined back into s.
static slam_status launch_pipeline(slam_extractor* ex, int nframes, const uint8_t* d_img, int lap0,
                                   int lap1, slam_keypoint* d_kps, uint8_t* d_desc, int cap,
                                   int32_t* d_n, int32_t* d_mono, hipStream_t s) {
    // profiling (per-stage HIP events) serializes the stages on s, so each bracket times one
    // kernel alone (its own launch duration, comparable with rocprofv3's kernel trace)
    const bool serial = ex->serial || ex->profiling;
    int nsub = serial ? 1 : std::min(ex->nsub, nframes / 8);
    if (nsub <= 1) {
        SLAM_TRY_ST(launch_range(ex, 0, nframes, d_img, lap0, lap1, d_kps, d_desc, cap, d_n, d_mono, s));
    } else {
        // range 0 runs on the caller's stream, ranges 1.. on the handle's sub-streams (nsub
        // hardware queues; GPU_MAX_HW_QUEUES is 4 by default)
        SLAM_HIP_TRY(hipEventRecord(ex->sub_fork, s));
        int f0 = 0;
        for (int k = 0; k < nsub; k++) {
            const int nf = nframes / nsub + (k < nframes % nsub ? 1 : 0);
            hipStream_t sk = k ? ex->sub[k] : s;
            if (k) SLAM_HIP_TRY(hipStreamWaitEvent(sk, ex->sub_fork, 0));
            SLAM_TRY_ST(launch_range(ex, f0, nf, d_img, lap0, lap1, d_kps, d_desc, cap, d_n, d_mono, sk,
                                     ex->chain_fast && k ? ex->sub_fast[k - 1] : nullptr,
                                     ex->chain_fast ? ex->sub_fast[k] : nullptr));
            if (k) SLAM_HIP_TRY(hipEventRecord(ex->sub_join[k], sk));
            f0 += nf;
        }
        for (int k = 1; k < nsub; k++) SLAM_HIP_TRY(hipStreamWaitEvent(s, ex->sub_join[k], 0));
    }
    ex->last_frames = nframes;
    ex->last_img = d_img;
    return SLAM_OK;
}

// ---- host-buffer path as a HIP graph.  A per-image call is ~16 kernel launches, a memset and
// six small copies: launch and copy latency, not the GPU, set its time (0.37 ms for a VGA frame).
// The call is captured once per shape (frames, size, lapping area, capacity, buffer addresses) and
// replayed: the image goes through pinned memory (one host memcpy, one DMA), the outputs come
// back as one block (counts, error flags, keypoints, descriptors) into pinned memory.
constexpr int kHostGraphFrames = kSmallBatch;  // larger batches keep the sub-stream pipeline
constexpr slam_status SLAM_ENOTSUP = (slam_status)-100;  // internal: fall back to stream calls

static bool pinned_ensure(void*& p, size_t& have, size_t need) {
    if (need <= have) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    have = 0;
    if (hipHostMalloc(&p, need, hipHostMallocDefault) != hipSuccess) return false;
    have = need;
    return true;
}

static slam_status host_graph_extract(slam_extractor* ex, int nframes, const uint8_t* imgs, int width, int height,
                                      size_t stride, int lap0, int lap1, slam_keypoint* kps, uint8_t* desc, int cap,
                                      int* n, int* mono_index) {
    const size_t F = (size_t)nframes, fb = (size_t)width * height, dcap = (size_t)std::max(cap, 1);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_n = 0, o_mono = 4 * F, o_err = 8 * F, o_kps = al(12 * F);
    const size_t o_desc = al(o_kps + F * dcap * sizeof(slam_keypoint)), out_bytes = o_desc + F * dcap * 32;
    slam_status st;
    if ((st = ex->d_img.ensure(F * fb)) || (st = ex->d_out.ensure(out_bytes))) return st;
    if (!pinned_ensure(ex->h_in, ex->h_in_bytes, F * fb) || !pinned_ensure(ex->h_out, ex->h_out_bytes, out_bytes))
        return SLAM_ENOMEM;
    hipStream_t s = ex->stream;
    uint8_t* dout = ex->d_out.as<uint8_t>();
    const std::vector<uintptr_t> key = {
        (uintptr_t)nframes, (uintptr_t)width, (uintptr_t)height, (uintptr_t)(intptr_t)lap0, (uintptr_t)(intptr_t)lap1,
        (uintptr_t)cap, (uintptr_t)ex->h_in, (uintptr_t)ex->h_out, (uintptr_t)ex->d_img.p, (uintptr_t)ex->d_out.p,
        (uintptr_t)ex->d_plan.p, (uintptr_t)ex->d_xtab.p, (uintptr_t)ex->d_ytab.p, (uintptr_t)ex->d_cells.p,
        (uintptr_t)ex->d_wave_cells.p, (uintptr_t)ex->d_wide_cells.p, (uintptr_t)ex->d_pyr.p,
        (uintptr_t)ex->d_cell_keys.p, (uintptr_t)ex->d_cell_cnt.p, (uintptr_t)ex->d_keys_g.p,
        (uintptr_t)ex->d_knode_g.p, (uintptr_t)ex->d_okp.p, (uintptr_t)ex->d_ocnt.p, (uintptr_t)ex->d_oidx.p,
        (uintptr_t)ex->d_err.p};
    if (!ex->hg_exec || key != ex->hg_key) {
        if (ex->hg_exec) (void)hipGraphExecDestroy(ex->hg_exec);
        ex->hg_exec = nullptr;
        ex->hg_key.clear();
        if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            ex->hg_off = true;
            return SLAM_ENOTSUP;
        }
        bool ok = hipMemcpyAsync(ex->d_img.p, ex->h_in, F * fb, hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && launch_pipeline(ex, nframes, ex->d_img.as<uint8_t>(), lap0, lap1,
                                   reinterpret_cast<slam_keypoint*>(dout + o_kps), dout + o_desc, cap,
                                   reinterpret_cast<int32_t*>(dout + o_n), reinterpret_cast<int32_t*>(dout + o_mono),
                                   s) == SLAM_OK;
        ok = ok && hipMemcpyAsync(dout + o_err, ex->d_err.p, 4 * F, hipMemcpyDeviceToDevice, s) == hipSuccess;
        ok = ok && hipMemcpyAsync(ex->h_out, dout, out_bytes, hipMemcpyDeviceToHost, s) == hipSuccess;
        hipGraph_t graph = nullptr;
        const bool ended = hipStreamEndCapture(s, &graph) == hipSuccess && graph;
        ok = ok && ended && hipGraphInstantiate(&ex->hg_exec, graph, nullptr, nullptr, 0) == hipSuccess;
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
        if (!ok) {
            if (ex->hg_exec) (void)hipGraphExecDestroy(ex->hg_exec);
            ex->hg_exec = nullptr;
            ex->hg_off = true;
            return SLAM_ENOTSUP;
        }
        ex->hg_key = key;
    }
    uint8_t* hin = static_cast<uint8_t*>(ex->h_in);
    for (int f = 0; f < nframes; f++) {
        if (stride == (size_t)width) {
            std::memcpy(hin + f * fb, imgs + f * fb, fb);
        } else {
            for (int y = 0; y < height; y++)
                std::memcpy(hin + f * fb + (size_t)y * width, imgs + ((size_t)f * height + y) * stride, width);
        }
    }
    SLAM_HIP_TRY(hipGraphLaunch(ex->hg_exec, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    ex->last_frames = nframes;
    ex->last_img = ex->d_img.as<uint8_t>();
    const uint8_t* hout = static_cast<const uint8_t*>(ex->h_out);
    std::memcpy(n, hout + o_n, 4 * F);
    std::memcpy(mono_index, hout + o_mono, 4 * F);
    const int32_t* err = reinterpret_cast<const int32_t*>(hout + o_err);
    if (cap > 0) {
        std::memcpy(kps, hout + o_kps, F * cap * sizeof(slam_keypoint));
        std::memcpy(desc, hout + o_desc, F * cap * 32);
    }
    slam_status res = SLAM_OK;
    for (int f = 0; f < nframes; f++) {
        if (err[f] & ~kErrCap) {
            std::fprintf(stderr, "slamhot: extractor internal error flags 0x%x on frame %d\n", err[f], f);
            return SLAM_EINVAL;
        }
        if (n[f] > cap) res = SLAM_ECAP;
    }
    return res;
}

extern "C" {

const char* slamhot_version(void) { return "slamhot 0.1 (gfx950)"; }

const char* slamhot_status_string(slam_status s) {
    switch (s) {
        case SLAM_OK: return "ok";
        case SLAM_EINVAL: return "invalid argument";
        case SLAM_ENOMEM: return "out of memory";
        case SLAM_EHIP: return "HIP runtime error";
        case SLAM_ECAP: return "output capacity too small";
        case SLAM_ENODEV: return "no gfx950 device";
        case SLAM_EEMPTY: return "empty image";
        case SLAM_ETIMEDOUT: return "wait timed out";
        default: return "unknown status";
    }
}

slam_status slamhot_device_count(int* n) {
    if (!n) return SLAM_EINVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return SLAM_OK;
}

slam_status slamhot_extractor_create(const slam_orb_params* params, int device, int max_width,
                                     int max_height, int max_batch, slam_extractor** out) {
    if (!params || !out || max_width <= 0 || max_height <= 0 || max_batch <= 0) return SLAM_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return SLAM_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SLAM_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SLAM_ENODEV;
    Plan probe;
    if (!build_plan(*params, max_width, max_height, probe)) return SLAM_EINVAL;
    slam_extractor* ex = new slam_extractor();
    {
        const char* e = std::getenv("SLAMHOT_SERIAL");
        ex->serial = e && e[0] == '1';
    }
    ex->prm = *params;
    ex->device = device;
    ex->max_w = max_width;
    ex->max_h = max_height;
    ex->max_batch = max_batch;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking) != hipSuccess ||

        hipEventCreateWithFlags(&ex->sub_fork, hipEventDisableTiming) != hipSuccess) {
        slamhot_extractor_destroy(ex);
        return SLAM_EHIP;
    }
    {
        const char* e = std::getenv("SLAMHOT_SUBSTREAMS");
        if (e) ex->nsub = std::max(1, std::min(slam_extractor::kMaxSub, std::atoi(e)));
        const char* c = std::getenv("SLAMHOT_CHAIN_FAST");
        ex->chain_fast = c && c[0] == '1';
        const char* g = std::getenv("SLAMHOT_EXTRACT_GRAPH");
        ex->hg_off = g && g[0] == '0';
    }
    for (int k = 0; k < slam_extractor::kMaxSub; k++)
        if (hipStreamCreateWithFlags(&ex->sub[k], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ex->sub_join[k], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ex->sub_fast[k], hipEventDisableTiming) != hipSuccess) {
            slamhot_extractor_destroy(ex);
            return SLAM_EHIP;
        }
    *out = ex;
    return SLAM_OK;
}

void slamhot_extractor_destroy(slam_extractor* ex) {
    if (!ex) return;
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    DevBuf* bufs[] = {&ex->d_plan, &ex->d_xtab, &ex->d_ytab, &ex->d_cells, &ex->d_wave_cells,
                      &ex->d_wide_cells, &ex->d_img, &ex->d_pyr,
                      &ex->d_cell_keys, &ex->d_cell_cnt, &ex->d_keys_g, &ex->d_knode_g,
                      &ex->d_okp, &ex->d_ocnt, &ex->d_oidx, &ex->d_err, &ex->d_kps, &ex->d_desc,
                      &ex->d_n, &ex->d_mono};
    for (DevBuf* b : bufs) b->release();
    ex->d_out.release();
    if (ex->hg_exec) (void)hipGraphExecDestroy(ex->hg_exec);
    if (ex->h_in) (void)hipHostFree(ex->h_in);
    if (ex->h_out) (void)hipHostFree(ex->h_out);
    for (auto& m : ex->marks) { ex->pool.push_back(m.a); ex->pool.push_back(m.b); }
    for (hipEvent_t e : ex->pool) (void)hipEventDestroy(e);
    for (int k = 0; k < slam_extractor::kMaxSub; k++) {
        if (ex->sub[k]) (void)hipStreamSynchronize(ex->sub[k]);
        for (hipEvent_t e : {ex->sub_join[k], ex->sub_fast[k]})
            if (e) (void)hipEventDestroy(e);
        if (ex->sub[k]) (void)hipStreamDestroy(ex->sub[k]);
    }
    if (ex->sub_fork) (void)hipEventDestroy(ex->sub_fork);

    if (ex->stream) (void)hipStreamDestroy(ex->stream);
    delete ex;
}

slam_status slamhot_extractor_levels(const slam_extractor* ex, int* nlevels, float* scale,
                                     float* inv_scale, float* sigma2, float* inv_sigma2,
                                     int32_t* nfeatures_per_level) {
    if (!ex) return SLAM_EINVAL;
    Plan P;
    build_scale_tables(ex->prm, P);
    const int L = ex->prm.nlevels;
    if (nlevels) *nlevels = L;
    for (int l = 0; l < L; l++) {
        if (scale) scale[l] = P.scale[l];
        if (inv_scale) inv_scale[l] = P.inv_scale[l];
        if (sigma2) sigma2[l] = P.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = P.inv_sigma2[l];
        if (nfeatures_per_level) nfeatures_per_level[l] = P.nfeat[l];
    }
    return SLAM_OK;
}

slam_status slamhot_extract_batch_device(slam_extractor* ex, int nframes, const void* d_imgs,
                                         int width, int height, int lap0, int lap1, void* d_kps,
                                         void* d_desc, int cap, void* d_n, void* d_mono_index,
                                         void* hip_stream) {
    if (!ex || nframes <= 0 || !d_imgs || !d_kps || !d_desc || !d_n || !d_mono_index || cap < 0)
        return SLAM_EINVAL;
    if (width > ex->max_w || height > ex->max_h || nframes > ex->max_batch) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(ex->mu);
    SLAM_HIP_TRY(hipSetDevice(ex->device));
    slam_status st;
    if ((st = ensure_plan(ex, width, height)) || (st = ensure_batch(ex, nframes, cap))) return st;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : ex->stream;
    return launch_pipeline(ex, nframes, (const uint8_t*)d_imgs, lap0, lap1, (slam_keypoint*)d_kps,
                           (uint8_t*)d_desc, cap, (int32_t*)d_n, (int32_t*)d_mono_index, s);
}

slam_status slamhot_extract_batch(slam_extractor* ex, int nframes, const uint8_t* imgs, int width,
                                  int height, size_t stride, int lap0, int lap1,
                                  slam_keypoint* kps, uint8_t* desc, int cap, int* n,
                                  int* mono_index) {
    if (!ex || nframes <= 0 || !n || !mono_index || cap < 0 || (cap > 0 && (!kps || !desc)))
        return SLAM_EINVAL;
    if (!imgs || width <= 0 || height <= 0) return SLAM_EEMPTY;
    if (stride < (size_t)width || width > ex->max_w || height > ex->max_h || nframes > ex->max_batch)
        return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(ex->mu);
    SLAM_HIP_TRY(hipSetDevice(ex->device));
    slam_status st;
    if ((st = ensure_plan(ex, width, height)) || (st = ensure_batch(ex, nframes, cap))) return st;
    if (nframes <= kHostGraphFrames && !ex->profiling && !ex->hg_off) {
        st = host_graph_extract(ex, nframes, imgs, width, height, stride, lap0, lap1, kps, desc, cap, n, mono_index);
        if (st != SLAM_ENOTSUP) return st;  // else: the capture failed, plain stream calls below
    }
    const size_t F = (size_t)nframes, fb = (size_t)width * height;
    const int dcap = std::max(cap, 1);
    if ((st = ex->d_img.ensure(F * fb)) || (st = ex->d_kps.ensure(F * dcap * sizeof(slam_keypoint))) ||
        (st = ex->d_desc.ensure(F * dcap * 32)) || (st = ex->d_n.ensure(F * 4)) ||
        (st = ex->d_mono.ensure(F * 4)))
        return st;
    hipStream_t s = ex->stream;
    for (int f = 0; f < nframes; f++)
        SLAM_HIP_TRY(hipMemcpy2DAsync(ex->d_img.as<uint8_t>() + f * fb, width, imgs + f * height * stride,
                                      stride, width, height, hipMemcpyHostToDevice, s));
    if ((st = launch_pipeline(ex, nframes, ex->d_img.as<uint8_t>(), lap0, lap1, ex->d_kps.as<slam_keypoint>(),
                              ex->d_desc.as<uint8_t>(), cap, ex->d_n.as<int32_t>(), ex->d_mono.as<int32_t>(), s)))
        return st;
    std::vector<int32_t> err(nframes);
    SLAM_HIP_TRY(hipMemcpyAsync(n, ex->d_n.p, F * 4, hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipMemcpyAsync(mono_index, ex->d_mono.p, F * 4, hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipMemcpyAsync(err.data(), ex->d_err.p, F * 4, hipMemcpyDeviceToHost, s));
    if (cap > 0) {
        SLAM_HIP_TRY(hipMemcpyAsync(kps, ex->d_kps.p, F * cap * sizeof(slam_keypoint), hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipMemcpyAsync(desc, ex->d_desc.p, F * cap * 32, hipMemcpyDeviceToHost, s));
    }
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    slam_status res = SLAM_OK;
    for (int f = 0; f < nframes; f++) {
        if (err[f] & ~kErrCap) {
            std::fprintf(stderr, "slamhot: extractor internal error flags 0x%x on frame %d\n", err[f], f);
            return SLAM_EINVAL;
        }
        if (n[f] > cap) res = SLAM_ECAP;
    }
    return res;
}

slam_status slamhot_extract(slam_extractor* ex, const uint8_t* img, int width, int height,
                            size_t stride, int lap0, int lap1, slam_keypoint* kps, uint8_t* desc,
                            int cap, int* n, int* mono_index) {
    return slamhot_extract_batch(ex, 1, img, width, height, stride, lap0, lap1, kps, desc, cap, n,
                                 mono_index);
}

slam_status slamhot_pyramid_level_device(slam_extractor* ex, int frame, int level, const void** d_ptr, int* pitch,
                                         int* width, int* height) {
    if (!ex || !ex->have_plan || frame < 0 || frame >= ex->last_frames || level < 0 ||
        level >= ex->plan.nlevels || !d_ptr || !pitch || !width || !height)
        return SLAM_EINVAL;
    const Plan& P = ex->plan;
    const LevelPlan& L = P.lv[level];
    *width = L.w;
    *height = L.h;
    if (level == 0) {
        *d_ptr = ex->last_img + (size_t)frame * P.W * P.H;
        *pitch = P.W;
    } else {
        *d_ptr = ex->d_pyr.as<uint8_t>() + (size_t)frame * P.pyr_frame + L.pyr_off;
        *pitch = L.pitch;
    }
    return SLAM_OK;
}

slam_status slamhot_pyramid_level(slam_extractor* ex, int frame, int level, uint8_t* dst,
                                  size_t dst_cap, int* width, int* height) {
    if (!ex || !ex->have_plan || frame < 0 || frame >= ex->last_frames || level < 0 ||
        level >= ex->plan.nlevels || !width || !height)
        return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(ex->mu);
    SLAM_HIP_TRY(hipSetDevice(ex->device));
    const Plan& P = ex->plan;
    const LevelPlan& L = P.lv[level];
    *width = L.w;
    *height = L.h;
    if (!dst) return SLAM_OK;
    if (dst_cap < (size_t)L.w * L.h) return SLAM_ECAP;
    const uint8_t* src;
    size_t spitch;
    if (level == 0) {
        src = ex->last_img + (size_t)frame * P.W * P.H;
        spitch = P.W;
    } else {
        src = ex->d_pyr.as<uint8_t>() + (size_t)frame * P.pyr_frame + L.pyr_off;
        spitch = L.pitch;
    }
    SLAM_HIP_TRY(hipMemcpy2DAsync(dst, L.w, src, spitch, L.w, L.h, hipMemcpyDeviceToHost, ex->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(ex->stream));
    return SLAM_OK;
}

void* slamhot_extractor_stream(slam_extractor* ex) { return ex ? (void*)ex->stream : nullptr; }

slam_status slamhot_extractor_set_profiling(slam_extractor* ex, int enable) {
    if (!ex) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(ex->mu);
    ex->profiling = enable != 0;
    return SLAM_OK;
}

int slamhot_extractor_num_stages(void) { return kNumStages; }

const char* slamhot_extractor_stage_name(int stage) {
    return (stage >= 0 && stage < kNumStages) ? kStageNames[stage] : "";
}

slam_status slamhot_extractor_stage_stats(slam_extractor* ex, double* total_ms, long* launches,
                                          int reset) {
    if (!ex) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(ex->mu);
    SLAM_HIP_TRY(hipSetDevice(ex->device));
    for (auto& m : ex->marks) {
        SLAM_HIP_TRY(hipEventSynchronize(m.b));
        float ms = 0.f;
        SLAM_HIP_TRY(hipEventElapsedTime(&ms, m.a, m.b));
        ex->stage_ms[m.stage] += ms;
        ex->stage_launches[m.stage] += 1;
        ex->pool.push_back(m.a);
        ex->pool.push_back(m.b);
    }
    ex->marks.clear();
    for (int i = 0; i < kNumStages; i++) {
        if (total_ms) total_ms[i] = ex->stage_ms[i];
        if (launches) launches[i] = ex->stage_launches[i];
        if (reset) { ex->stage_ms[i] = 0; ex->stage_launches[i] = 0; }
    }
    return SLAM_OK;
}

}  // extern "C"
