// matcher.hip — MI355X (gfx950) DBoW2 vocabulary descent and ORBmatcher::SearchByBoW.
//
//   k_vocab_transform  TemplatedVocabulary::transform (TemplatedVocabulary.h:1229-1271):
//                      kVocG lanes per descriptor; at each level lane j scores child slots
//                      j, j + kVocG, .. (two 16-byte loads + 8 popcounts each) together with
//                      the child's next-level record, (distance, child position) group-min.
//   k_bow_match        SearchByBoW (ORBmatcher.cc:269-471 and 823-963): one workgroup per
//                      (A, B) pair.  Common FeatureVector nodes are independent (every
//                      feature lives in exactly one node), so waves take nodes round-robin;
//                      inside a node the reference's greedy order over A features is kept
//                      (sequential), each step a wave-wide (min, second-min) over the node's
//                      B candidates held in registers.  Rotation histogram +
//                      ComputeThreeMaxima (:2515-2556) close the pair in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <thread>
#include <vector>

#include "common.hpp"
#include "gate_fp.hpp"

#include "projection.hpp"  // DevProjFrame / ProjQuery / DevProjCall / FrustumCall

namespace slamhot {

// ----------------------------------------------------------------------------- vocab
struct DevVocab {
    const uint8_t* desc;        // n_nodes x 32
    const int32_t* child_ptr;   // n_nodes + 1
    const int32_t* child_idx;
    const uint8_t* is_leaf;
    const int32_t* word;        // word id per node (-1 for inner nodes)
    const double* weight;
    const uint8_t* child_desc;  // n_nodes - 1 child slots x 32: desc of child_idx[c]
    const int4* child_next;     // per child slot: {its child range begin, end, node id | leaf << 31, 0}
    int root_c0, root_c1;       // the root's child range
    int L;
};

__device__ __forceinline__ int hamming32(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// min over a DPP row of 16 lanes (quad_perm xor 1 / 2, half-row and row mirrors), in every
// lane of the row; VALU-speed, unlike a __shfl_xor butterfly (dependent ds_bpermute trips)
__device__ __forceinline__ uint32_t row16_min_u32(uint32_t x) {
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));
    return x;
}

// min over the whole (fully active) wave: row minima, then the four rows by v_readlane
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = row16_min_u32(x);
    return min(min((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16)),
               min((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48)));
}

// Lanes per descriptor: lane j scores children j, j + kVocG, ... of the current node (the first
// 16 child slots from registers, further ones -- vocabularies with k > 16 -- in a second loop).
#ifndef SLAMHOT_VOC_G
#define SLAMHOT_VOC_G 8
#endif
constexpr int kVocG = SLAMHOT_VOC_G;
constexpr int kVocS = 16 / kVocG;  // child slots per lane held in registers
static_assert(kVocG == 4 || kVocG == 8 || kVocG == 16, "lanes per descriptor");

// min over the kVocG-lane group (DPP inside rows of 16), in every lane of the group
__device__ __forceinline__ uint32_t group_min_u32(uint32_t x) {
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    if constexpr (kVocG >= 8) x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false));
    if constexpr (kVocG >= 16) x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));
    return x;
}

// n_per_frame (optional): the descriptors are frames of `cap` slots and only the first
// n_per_frame[f] slots of frame f hold features; the empty slots' groups exit at once.
// One global round trip per level: the children's descriptors are stored contiguously per
// parent (child_desc[c] for child slot c) next to each child's own child range, node id and
// leaf flag (child_next[c]), both loaded together; the winner's record then comes from its
// lane by ds_bpermute instead of three dependent loads (child_idx, child_ptr, is_leaf).
constexpr int kVocThreads = 256;  // 64 measured 0.9% slower in the headline
__global__ void __launch_bounds__(kVocThreads) k_vocab_transform(DevVocab V, int n, const uint8_t* desc,
                                                         int desc_stride, int levelsup,
                                                         int32_t* word_id, double* weight,
                                                         int32_t* node_id, const int32_t* __restrict__ n_per_frame,
                                                         int cap) {
    const int g = (blockIdx.x * blockDim.x + threadIdx.x) / kVocG;  // feature
    const int lane = threadIdx.x & 63, j = lane & (kVocG - 1);        // child slot
    if (n_per_frame && g < n && (g % cap) >= n_per_frame[g / cap]) return;  // whole lane group
    const bool live = g < n;
    const int gi = live ? g : 0;
    const uint4* f = reinterpret_cast<const uint4*>(desc + (size_t)gi * desc_stride);
    const uint4 f0 = f[0], f1 = f[1];
    const int nid_level = V.L - levelsup;
    int final_id = 0, level = 0, nid = 0;
    int c0 = V.root_c0, c1 = V.root_c1;
    // every lane of a group follows the same path; bounded by the tree depth
    for (int it = 0; it < 64; it++) {
        ++level;
        uint32_t bestkey = 0xFFFFFFFFu;
        int4 inf[kVocS];
#pragma unroll
        for (int sl = 0; sl < kVocS; sl++) {
            const int c = c0 + j + sl * kVocG;
            inf[sl] = make_int4(0, 0, 0, 0);
            if (c < c1) {
                const uint4* d = reinterpret_cast<const uint4*>(V.child_desc + (size_t)c * 32);
                inf[sl] = V.child_next[c];
                bestkey = min(bestkey, ((uint32_t)hamming32(f0, f1, d[0], d[1]) << 20) | (uint32_t)(c - c0));
            }
        }
        for (int cb = c0 + 16; cb < c1; cb += kVocG) {  // k > 16
            const int c = cb + j;
            if (c < c1) {
                const uint4* d = reinterpret_cast<const uint4*>(V.child_desc + (size_t)c * 32);
                bestkey = min(bestkey, ((uint32_t)hamming32(f0, f1, d[0], d[1]) << 20) | (uint32_t)(c - c0));
            }
        }
        bestkey = group_min_u32(bestkey);
        if (bestkey == 0xFFFFFFFFu) break;  // malformed tree (inner node without children)
        const int pos = (int)(bestkey & 0xFFFFF);
        int4 nx;
        if (pos < 16) {
            const int slot = pos / kVocG, src = (lane & ~(kVocG - 1)) | (pos & (kVocG - 1));
            int4 sel = inf[0];
#pragma unroll
            for (int sl = 1; sl < kVocS; sl++)
                if (slot == sl) sel = inf[sl];
            nx.x = __shfl(sel.x, src, 64);
            nx.y = __shfl(sel.y, src, 64);
            nx.z = __shfl(sel.z, src, 64);
        } else {
            nx = V.child_next[c0 + pos];
        }
        final_id = nx.z & 0x7FFFFFFF;
        if (level == nid_level) nid = final_id;
        if (nx.z < 0) break;  // leaf
        c0 = nx.x;
        c1 = nx.y;
    }
    if (live && j == 0) {
        word_id[g] = V.word[final_id];
        weight[g] = V.weight[final_id];
        node_id[g] = nid;
    }
}

// ----------------------------------------------------------------------------- BoW match
struct DevBowSide {
    const uint8_t* desc;      // n x 32 (row stride 32)
    const float* angle;       // angle of feature i at angle[i * angle_stride]
    int angle_stride;
    const uint8_t* valid;     // n or nullptr
    int n, n_nodes;
    const uint32_t* node_id;
    const int32_t* node_off;
    const uint32_t* node_feat;
};

struct DevBowPair {
    DevBowSide A, B;
    int32_t* a2b;
    int32_t* b2a;
    int32_t* nmatches;
    int general;       // outside k_bow_match's tiles: k_bow_match_any handles the pair
    int8_t* bins;      // k_bow_match_any scratch: rotation bin per A feature (A.n)
    uint8_t* taken;    // k_bow_match_any scratch: B feature already matched (B.n)
};

constexpr int kBowCap = 8192;        // features per side held in LDS
#ifndef SLAMHOT_BOW_THREADS
#define SLAMHOT_BOW_THREADS 1024
#endif
constexpr int kBowThreads = SLAMHOT_BOW_THREADS;  // 16 waves per pair: a wave per common node in turn
constexpr int kBowNodeChunks = 4;    // B candidates per node held in registers: 4 x 64
#ifndef SLAMHOT_BOW_ROWS
#define SLAMHOT_BOW_ROWS 1
#endif
constexpr bool kBowRows = SLAMHOT_BOW_ROWS != 0;  // nodes of <= 16 / 32 B candidates: four / two per wave
#ifndef SLAMHOT_BOW_G32
#define SLAMHOT_BOW_G32 1
#endif
constexpr bool kBowG32 = SLAMHOT_BOW_G32 != 0;  // the 32-lane groups (else 17..32 stay on the wave loop)
#ifndef SLAMHOT_BOW_G64
#define SLAMHOT_BOW_G64 1
#endif
constexpr bool kBowG64 = SLAMHOT_BOW_G64 != 0;  // 33..64 candidates: one node per wave in the group form
#ifndef SLAMHOT_BOW_XCD
#define SLAMHOT_BOW_XCD 1
#endif

__device__ __forceinline__ int rot_bin(float a, float b) {
    // ORBmatcher.cc:391-396: float difference, +360 if negative, std::round(rot * (1/30))
    float rot = a - b;
    if (rot < 0.0f) rot += 360.0f;
    const float factor = 1.0f / 30;
    int bin = (int)roundf(rot * factor);
    if (bin == 30) bin = 0;
    return bin;
}

// ComputeThreeMaxima (ORBmatcher.cc:2515-2556) over the 30 rotation bins
__device__ inline void three_maxima(const int* hist, int* keep) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < 30; i++) {
        const int s = hist[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
    keep[0] = ind1;
    keep[1] = ind2;
    keep[2] = ind3;
}

// The greedy SearchByBoW loop (ORBmatcher.cc:292-425, 853-930) for nodes of at most G B candidates,
// 64 / G nodes per wave (work item g): lane group r (lanes G r .. G r + G - 1) runs the node
// common[first + k] for k = (64 / G) g + r -- lane = B candidate, the group's A feature t broadcast to the group by
// ds_bpermute, best and second best by group minima (DPP inside rows of 16, then swizzles across
// rows for G = 32 / 64).  The same (distance << 16 | position) keys, TH_LOW / nnratio test and
// taken flags as the wave loop, per node in A order: the same matches.
template <int G>
__device__ __forceinline__ uint32_t group_min(uint32_t x) {
    x = row16_min_u32(x);
    if constexpr (G >= 32) x = min(x, (uint32_t)__shfl_xor((int)x, 16, 64));
    if constexpr (G == 64) x = min(x, (uint32_t)__shfl_xor((int)x, 32, 64));
    return x;
}

template <int G>
__device__ __forceinline__ void bow_group(const DevBowSide& A, const DevBowSide& B, const int16_t* common, int first,
                                          int n, int g, int lane, float nnratio, int strict, int16_t* matchA) {
    constexpr int NG = 64 / G;
    const int grp = lane / G, lg = lane & (G - 1);
    {
        const int c = NG * g + grp;
        const bool live = c < n;
        const int e = live ? first + c : 0;
        const int ia = live ? common[2 * e] : 0, ib = live ? common[2 * e + 1] : 0;
        const int a0 = live ? A.node_off[ia] : 0, a1 = live ? A.node_off[ia + 1] : 0;
        const int b0 = live ? B.node_off[ib] : 0, nbn = live ? B.node_off[ib + 1] - b0 : 0;
        // this lane's B candidate
        bool bok = false;
        int bidx = -1;
        uint4 bd0 = make_uint4(0, 0, 0, 0), bd1 = bd0;
        if (lg < nbn) {
            bidx = (int)B.node_feat[b0 + lg];
            bok = !B.valid || B.valid[bidx];
            const uint4* d = reinterpret_cast<const uint4*>(B.desc + (size_t)bidx * 32);
            bd0 = d[0];
            bd1 = d[1];
        }
        // A features in chunks of G per group, lane lg holding feature t0 + lg of its group's node
        int na = a1 - a0;
#pragma unroll
        for (int o = G; o < 64; o <<= 1) na = max(na, __shfl_xor(na, o, 64));
        for (int t0 = 0; t0 < na; t0 += G) {
            int my_idx = -1;
            uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
            if (a0 + t0 + lg < a1) {
                const int ix = (int)A.node_feat[a0 + t0 + lg];
                if (!A.valid || A.valid[ix]) {
                    my_idx = ix;
                    const uint4* dm = reinterpret_cast<const uint4*>(A.desc + (size_t)ix * 32);
                    m0 = dm[0];
                    m1 = dm[1];
                }
            }
            const int tn = min(G, na - t0);
            for (int t = 0; t < tn; t++) {
                const int src = (lane & ~(G - 1)) | t;
                const int idxA = __shfl(my_idx, src, 64);  // -1: past the group's node, or not valid
                const uint4 q0 = make_uint4(__shfl((int)m0.x, src, 64), __shfl((int)m0.y, src, 64),
                                            __shfl((int)m0.z, src, 64), __shfl((int)m0.w, src, 64));
                const uint4 q1 = make_uint4(__shfl((int)m1.x, src, 64), __shfl((int)m1.y, src, 64),
                                            __shfl((int)m1.z, src, 64), __shfl((int)m1.w, src, 64));
                const bool cand = bok && idxA >= 0;
                const int dist = cand ? hamming32(q0, q1, bd0, bd1) : 1024;
                const uint32_t bestkey = group_min<G>(cand ? (((uint32_t)dist << 16) | (uint32_t)lg) : 0xFFFFFFFFu);
                const int best1 = bestkey == 0xFFFFFFFFu ? 256 : (int)(bestkey >> 16);
                const int bpos = (int)(bestkey & 0xFFFF);
                const int sec = (int)group_min<G>((cand && lg != bpos) ? (uint32_t)dist : 256u);
                const bool pass = (strict ? best1 < 50 : best1 <= 50) && ((float)best1 < nnratio * (float)sec);
                if (pass && lg == bpos) {  // the owner lane takes its candidate
                    bok = false;
                    matchA[idxA] = (int16_t)bidx;
                }
            }
        }
    }
}

__global__ void __launch_bounds__(kBowThreads) k_bow_match(const DevBowPair* pairs, float nnratio,
                                                   int check_ori, int strict) {
    __shared__ int16_t matchA[kBowCap];   // B index matched by A feature, -1 none
    __shared__ int8_t binA[kBowCap];
    __shared__ int16_t common[2 * 4096];  // (ia, ib) of common nodes
    __shared__ int hist[32];
    __shared__ int s_ncommon, s_n32, s_n64, s_nsmall, s_next, s_keep[3], s_count;
#if SLAMHOT_BOW_XCD
    // XCD-aware order (cdna_hip_programming.md T1): a run of consecutive pairs per XCD, so the
    // frames that neighbouring pairs share (a sequence's frame is the next pair's KeyFrame) are
    // read into one L2.  Speed only: any placement is correct.
    const int nwg = (int)gridDim.x, orig = (int)blockIdx.x, xq = nwg >> 3, xr = nwg & 7, xcd = orig & 7;
    const DevBowPair pr = pairs[(xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3)];
#else
    const DevBowPair pr = pairs[blockIdx.x];
#endif
    if (pr.general) return;  // k_bow_match_any's pair
#ifdef SLAMHOT_BOW_TRACE
    // phase clocks of one workgroup (experiment builds): start, init, merge-join, per-wave node loop end
    const bool btr = blockIdx.x == 37;
    const long long bt0 = (long long)__builtin_amdgcn_s_memtime();
    long long bt1 = 0, bt2 = 0;
    int bnodes = 0, bfeat = 0;
#endif
    const DevBowSide& A = pr.A;
    const DevBowSide& B = pr.B;
    // a wave's work item comes back from the LDS counter through v_readfirstlane: wave-uniform, so
    // the per-node records load into SGPRs
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < A.n; i += blockDim.x) {
        matchA[i] = -1;
        binA[i] = -1;
    }
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) s_ncommon = s_n32 = s_n64 = s_nsmall = s_next = 0;
    __syncthreads();
#ifdef SLAMHOT_BOW_TRACE
    bt1 = (long long)__builtin_amdgcn_s_memtime();
#endif
    // common node ids (merge-join of two ascending lists), by B candidate count: more than 64 (the
    // wave loop) from the front of `common`, then 17..32, then 33..64, at most 16 from the back; a thread's
    // finds (<= kBowPer, A.n_nodes <= 4096 by the tile condition) wait in registers for the counts
    constexpr int kBowPer = (4096 + kBowThreads - 1) / kBowThreads;
    int fia[kBowPer], flo[kBowPer], fcl[kBowPer];
    int nf = 0;
    for (int ia = tid; ia < A.n_nodes; ia += blockDim.x) {
        const uint32_t id = A.node_id[ia];
        int lo = 0, hi = B.n_nodes;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.node_id[mid] < id) lo = mid + 1; else hi = mid;
        }
        if (lo < B.n_nodes && B.node_id[lo] == id && nf < kBowPer) {
            const int nb = B.node_off[lo + 1] - B.node_off[lo];
            const int cl = !kBowRows ? 0 : nb <= 16 ? 2 : (kBowG32 && nb <= 32) ? 1 : (kBowG64 && nb <= 64) ? 3 : 0;
            atomicAdd(cl == 0 ? &s_ncommon : cl == 1 ? &s_n32 : cl == 2 ? &s_nsmall : &s_n64, 1);
            fia[nf] = ia;
            flo[nf] = lo;
            fcl[nf] = cl;
            nf++;
        }
    }
    __syncthreads();
    const int ncommon = s_ncommon, n32 = s_n32, n16 = s_nsmall, n64 = s_n64;
    if (tid == 0) s_ncommon = s_n32 = s_nsmall = s_n64 = 0;  // placement cursors
    __syncthreads();
    for (int k = 0; k < nf; k++) {
        const int cl = fcl[k];
        const int pos = cl == 0   ? atomicAdd(&s_ncommon, 1)
                        : cl == 1 ? ncommon + atomicAdd(&s_n32, 1)
                        : cl == 3 ? ncommon + n32 + atomicAdd(&s_n64, 1)
                                  : 4095 - atomicAdd(&s_nsmall, 1);
        common[2 * pos] = (int16_t)fia[k];
        common[2 * pos + 1] = (int16_t)flo[k];
    }
    __syncthreads();
#ifdef SLAMHOT_BOW_TRACE
    bt2 = (long long)__builtin_amdgcn_s_memtime();
#endif
    // work items, largest first, taken by the waves from an LDS counter (the node sizes differ ~10x,
    // so a static round-robin left one wave with the big nodes after its share of the small ones):
    // wave-loop nodes (> 64 B candidates), then the 64-, 32- and 16-lane group items
    const int i64 = n64, i32 = (n32 + 1) >> 1, i16 = (n16 + 3) >> 2;
    const int nitems = ncommon + i64 + i32 + i16;
    for (;;) {
        int it = 0;
        if (lane == 0) it = atomicAdd(&s_next, 1);
        it = __builtin_amdgcn_readfirstlane(it);
        if (it >= nitems) break;
        if (it >= ncommon) {
            it -= ncommon;
            if (it < i64) bow_group<64>(A, B, common, ncommon + n32, n64, it, lane, nnratio, strict, matchA);
            else if ((it -= i64) < i32) bow_group<32>(A, B, common, ncommon, n32, it, lane, nnratio, strict, matchA);
            else bow_group<16>(A, B, common, 4096 - n16, n16, it - i32, lane, nnratio, strict, matchA);
            continue;
        }
        const int c = it;
        const int ia = common[2 * c], ib = common[2 * c + 1];
        const int a0 = A.node_off[ia], a1 = A.node_off[ia + 1];
#ifdef SLAMHOT_BOW_TRACE
        bnodes++;
        bfeat += a1 - a0;
#endif
        const int b0 = B.node_off[ib], b1 = B.node_off[ib + 1];
        const int nbn = min(b1 - b0, 64 * kBowNodeChunks);
        // chunks holding candidates (wave-uniform): most vocabulary nodes hold a few features, so
        // the distance sweeps below skip the empty chunks instead of evaluating all four
        const int nch = __builtin_amdgcn_readfirstlane((nbn + 63) >> 6);
        // this lane's B candidates: descriptor, index, validity, taken flag
        uint4 bd0[kBowNodeChunks], bd1[kBowNodeChunks];
        int bidx[kBowNodeChunks];
        bool bok[kBowNodeChunks];
#pragma unroll
        for (int k = 0; k < kBowNodeChunks; k++) {
            const int p = 64 * k + lane;
            bok[k] = false;
            bidx[k] = -1;
            if (p < nbn) {
                const int idx = (int)B.node_feat[b0 + p];
                bidx[k] = idx;
                bok[k] = !B.valid || B.valid[idx];
                const uint4* d = reinterpret_cast<const uint4*>(B.desc + (size_t)idx * 32);
                bd0[k] = d[0];
                bd1[k] = d[1];
            }
        }
        // the node's A features, 64 at a time, loaded lane-distributed (index, validity and
        // descriptor in parallel) and taken in node order by v_readlane: the sequential greedy
        // loop then waits on no memory
        for (int pc = a0; pc < a1; pc += 64) {
          const int cnt = min(64, a1 - pc);
          int my_idx = 0, my_ok = 0;
          uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
          if (lane < cnt) {
              my_idx = (int)A.node_feat[pc + lane];
              my_ok = !A.valid || A.valid[my_idx];
              const uint4* dm = reinterpret_cast<const uint4*>(A.desc + (size_t)my_idx * 32);
              m0 = dm[0];
              m1 = dm[1];
          }
          for (int t = 0; t < cnt; t++) {
            if (!__builtin_amdgcn_readlane(my_ok, t)) continue;
            const int idxA = __builtin_amdgcn_readlane(my_idx, t);
            const uint4 q0 = make_uint4(__builtin_amdgcn_readlane(m0.x, t), __builtin_amdgcn_readlane(m0.y, t),
                                        __builtin_amdgcn_readlane(m0.z, t), __builtin_amdgcn_readlane(m0.w, t));
            const uint4 q1 = make_uint4(__builtin_amdgcn_readlane(m1.x, t), __builtin_amdgcn_readlane(m1.y, t),
                                        __builtin_amdgcn_readlane(m1.z, t), __builtin_amdgcn_readlane(m1.w, t));
            int dist[kBowNodeChunks];
            uint32_t bestkey = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < kBowNodeChunks; k++) {
                dist[k] = 1024;
                if (k >= nch) continue;
                dist[k] = bok[k] ? hamming32(q0, q1, bd0[k], bd1[k]) : 1024;
                const uint32_t key = bok[k] ? (((uint32_t)dist[k] << 16) | (uint32_t)(64 * k + lane)) : 0xFFFFFFFFu;
                bestkey = min(bestkey, key);
            }
            bestkey = wave_min_u32(bestkey);
            const int best1 = bestkey == 0xFFFFFFFFu ? 256 : (int)(bestkey >> 16);
            const int bpos = (int)(bestkey & 0xFFFF);
            int sec = 256;
#pragma unroll
            for (int k = 0; k < kBowNodeChunks; k++)
                if (k < nch && bok[k] && (64 * k + lane) != bpos) sec = min(sec, dist[k]);
            sec = (int)wave_min_u32((uint32_t)sec);
            const bool pass = (strict ? best1 < 50 : best1 <= 50) && ((float)best1 < nnratio * (float)sec);
            if (pass) {
                // the owner lane marks its candidate taken and records the match
#pragma unroll
                for (int k = 0; k < kBowNodeChunks; k++) {
                    if (64 * k + lane == bpos) {
                        bok[k] = false;
                        matchA[idxA] = (int16_t)bidx[k];  // its rotation bin after the node loop
                    }
                }
            }
          }
        }
    }
#ifdef SLAMHOT_BOW_TRACE
    if (btr && lane == 0)
        printf("BOWTRACE wave %d nodes %d feat %d init %lld join %lld loop %lld (ncommon %d nA %d nB %d)\n", tid >> 6, bnodes,
               bfeat, bt1 - bt0, bt2 - bt1, (long long)__builtin_amdgcn_s_memtime() - bt2, ncommon, A.n, B.n);
#endif
    __syncthreads();
    if (check_ori) {
        // the rotation bins of the tentative matches (ORBmatcher.cc:389-398), in parallel: their
        // two angle loads per match no longer sit on a wave's sequential greedy chain
        for (int i = tid; i < A.n; i += blockDim.x) {
            const int m = matchA[i];
            if (m >= 0) {
                const int bn = rot_bin(A.angle[(size_t)i * A.angle_stride], B.angle[(size_t)m * B.angle_stride]);
                binA[i] = (int8_t)bn;
                atomicAdd(&hist[bn], 1);
            }
        }
        __syncthreads();
        if (tid == 0) three_maxima(hist, s_keep);
        __syncthreads();
    }
    if (tid == 0) s_count = 0;
    for (int i = tid; i < B.n; i += blockDim.x) pr.b2a[i] = -1;
    __syncthreads();
    int cnt = 0;
    for (int i = tid; i < A.n; i += blockDim.x) {
        int m = matchA[i];
        if (m >= 0 && check_ori) {
            const int bn = binA[i];
            if (bn != s_keep[0] && bn != s_keep[1] && bn != s_keep[2]) m = -1;
        }
        pr.a2b[i] = m;
        if (m >= 0) {
            pr.b2a[m] = i;
            cnt++;
        }
    }
    atomicAdd(&s_count, cnt);
    __syncthreads();
    if (tid == 0) *pr.nmatches = s_count;
}

// SearchByBoW for pairs outside k_bow_match's tiles (a side over kBowCap features, over 4096
// nodes, or a node of B over 4 x 64 candidates): the same algorithm with its state in global
// memory.  A wave per common node (nodes are independent: a B feature lives in one node),
// the A features of the node in order, the node's B candidates swept in chunks of 64 twice
// (best, then the second best over the other positions), the taken flag per B feature in
// pr.taken, the tentative match in pr.a2b and its rotation bin in pr.bins.
__global__ void __launch_bounds__(512) k_bow_match_any(const DevBowPair* pairs, float nnratio,
                                                       int check_ori, int strict) {
    __shared__ int hist[32];
    __shared__ int s_keep[3], s_count;
    if (!pairs[blockIdx.x].general) return;  // one flag read before the whole record
    const DevBowPair pr = pairs[blockIdx.x];
    const DevBowSide& A = pr.A;
    const DevBowSide& B = pr.B;
    // wave index via v_readfirstlane: wave-uniform, so the per-node records load into SGPRs
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nwaves = blockDim.x >> 6;
    for (int i = tid; i < A.n; i += blockDim.x) {
        pr.a2b[i] = -1;
        pr.bins[i] = -1;
    }
    for (int i = tid; i < B.n; i += blockDim.x) pr.taken[i] = 0;
    if (tid < 32) hist[tid] = 0;
    __syncthreads();
    for (int ia = wave; ia < A.n_nodes; ia += nwaves) {
        const uint32_t id = A.node_id[ia];
        int lo = 0, hi = B.n_nodes;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.node_id[mid] < id) lo = mid + 1; else hi = mid;
        }
        if (lo >= B.n_nodes || B.node_id[lo] != id) continue;  // wave-uniform
        const int a0 = A.node_off[ia], a1 = A.node_off[ia + 1];
        const int b0 = B.node_off[lo], nbn = B.node_off[lo + 1] - b0;
        for (int pa = a0; pa < a1; pa++) {
            const int idxA = (int)A.node_feat[pa];
            if (A.valid && !A.valid[idxA]) continue;
            const uint4* da = reinterpret_cast<const uint4*>(A.desc + (size_t)idxA * 32);
            const uint4 q0 = da[0], q1 = da[1];
            auto dist_at = [&](int p, int& bidx) -> int {  // 1024: not a candidate
                bidx = (int)B.node_feat[b0 + p];
                if ((B.valid && !B.valid[bidx]) || pr.taken[bidx]) return 1024;
                const uint4* d = reinterpret_cast<const uint4*>(B.desc + (size_t)bidx * 32);
                return hamming32(q0, q1, d[0], d[1]);
            };
            uint64_t best = ~0ull;
            for (int c = 0; c < nbn; c += 64) {
                const int p = c + lane;
                int bidx;
                const int d = p < nbn ? dist_at(p, bidx) : 1024;
                if (d < 1024) best = min(best, ((uint64_t)d << 32) | (uint64_t)p);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t x = __shfl_xor(best, o, 64);
                best = min(best, x);
            }
            if (best == ~0ull) continue;
            const int best1 = (int)(best >> 32), bpos = (int)(best & 0xffffffffu);
            int sec = 256;
            for (int c = 0; c < nbn; c += 64) {
                const int p = c + lane;
                int bidx;
                const int d = (p < nbn && p != bpos) ? dist_at(p, bidx) : 1024;
                if (d < 1024) sec = min(sec, d);
            }
            sec = (int)wave_min_u32((uint32_t)sec);
            const bool pass = (strict ? best1 < 50 : best1 <= 50) && ((float)best1 < nnratio * (float)sec);
            if (pass && lane == 0) {
                const int bidx = (int)B.node_feat[b0 + bpos];
                pr.taken[bidx] = 1;
                pr.a2b[idxA] = bidx;  // its rotation bin after the node loop
            }
            __threadfence_block();  // the taken flag is read by the whole wave next
        }
    }
    __syncthreads();
    if (check_ori) {
        for (int i = tid; i < A.n; i += blockDim.x) {
            const int m = pr.a2b[i];
            if (m >= 0) {
                const int bn = rot_bin(A.angle[(size_t)i * A.angle_stride], B.angle[(size_t)m * B.angle_stride]);
                pr.bins[i] = (int8_t)bn;
                atomicAdd(&hist[bn], 1);
            }
        }
        __syncthreads();
        if (tid == 0) three_maxima(hist, s_keep);
        __syncthreads();
    }
    if (tid == 0) s_count = 0;
    for (int i = tid; i < B.n; i += blockDim.x) pr.b2a[i] = -1;
    __syncthreads();
    int cnt = 0;
    for (int i = tid; i < A.n; i += blockDim.x) {
        int m = pr.a2b[i];
        if (m >= 0 && check_ori) {
            const int bn = pr.bins[i];
            if (bn != s_keep[0] && bn != s_keep[1] && bn != s_keep[2]) m = -1;
        }
        pr.a2b[i] = m;
        if (m >= 0) {
            pr.b2a[m] = i;
            cnt++;
        }
    }
    atomicAdd(&s_count, cnt);
    __syncthreads();
    if (tid == 0) *pr.nmatches = s_count;
}

}  // namespace slamhot

// =======================================================================================
// Host side
// =======================================================================================
using namespace slamhot;

namespace {

// ---------------------------------------------------------------------------------------
// Batched device path: Frame::ComputeBoW's FeatureVector per frame, then SearchByBoW per
// (KeyFrame, Frame) pair, without leaving HBM.
// k_featvec: one 1024-thread workgroup per frame.  FeatureVector::addFeature
// (FeatureVector.cpp:31-45) appends feature i to the entry of its level-(L-levelsup) node,
// features whose word weight is <= 0 are skipped (TemplatedVocabulary.h:1169), std::map
// keeps nodes ascending: a bitonic sort of (node << 16 | i) gives exactly that CSR.
// ---------------------------------------------------------------------------------------
constexpr int kFvMax = 8192;  // features per frame (LDS sort keys: 64 KB)
#ifndef SLAMHOT_FV_REG
#define SLAMHOT_FV_REG 1
#endif

// Bitonic sort of P <= 2 * 1024 keys with thread t holding elements 2t and 2t+1 in registers:
// partner distance 1 is inside the thread, 2..64 inside the wave (lane xor j/2), and only
// j >= 128 goes through LDS (10 of the 66 stages at P = 2048, 20 barriers instead of 66).
__device__ __forceinline__ void bitonic_reg2(uint64_t* keys, int P, int tid) {
    const int e = 2 * tid;
    const bool live = e < P;
    uint64_t v0 = live ? keys[e] : ~0ull, v1 = live ? keys[e + 1] : ~0ull;
    for (int k = 2; k <= P; k <<= 1) {
        const bool up = (e & k) == 0;
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j == 1) {
                if ((v0 > v1) == up) {
                    const uint64_t t = v0;
                    v0 = v1;
                    v1 = t;
                }
                continue;
            }
            uint64_t p0, p1;
            if (j <= 64) {
                p0 = __shfl_xor(v0, j >> 1, 64);
                p1 = __shfl_xor(v1, j >> 1, 64);
            } else {
                __syncthreads();  // the previous LDS stage's reads are done
                if (live) {
                    keys[e] = v0;
                    keys[e + 1] = v1;
                }
                __syncthreads();
                p0 = live ? keys[e ^ j] : ~0ull;
                p1 = live ? keys[(e + 1) ^ j] : ~0ull;
            }
            const bool takemin = ((e & j) == 0) == up;
            v0 = takemin ? min(v0, p0) : max(v0, p0);
            v1 = takemin ? min(v1, p1) : max(v1, p1);
        }
    }
    __syncthreads();
    if (live) {
        keys[e] = v0;
        keys[e + 1] = v1;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(1024) k_featvec(int cap, const int32_t* __restrict__ n_per_frame,
                                                  const int32_t* __restrict__ node, const double* __restrict__ weight,
                                                  uint32_t* __restrict__ fv_id, int32_t* __restrict__ fv_off,
                                                  uint32_t* __restrict__ fv_feat, int32_t* __restrict__ fv_n) {
    __shared__ uint64_t keys[kFvMax];
    __shared__ int wsum[16], vsum[16];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(n_per_frame[f], min(cap, kFvMax));
    int P = 1;
    while (P < n) P <<= 1;
    const size_t base = (size_t)f * cap;
    for (int i = tid; i < P; i += blockDim.x)
        keys[i] = (i < n && weight[base + i] > 0) ? (((uint64_t)(uint32_t)node[base + i] << 16) | (uint64_t)i)
                                                   : ~0ull;
    __syncthreads();
    if (SLAMHOT_FV_REG && P <= 2 * (int)blockDim.x) {
        bitonic_reg2(keys, P, tid);
    } else {
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < P; i += blockDim.x) {
                    const int x = i ^ j;
                    if (x > i) {
                        const uint64_t a = keys[i], b = keys[x];
                        const bool up = (i & k) == 0;
                        if ((a > b) == up) {
                            keys[i] = b;
                            keys[x] = a;
                        }
                    }
                }
                __syncthreads();
            }
    }
    // node boundaries -> CSR (chunks of blockDim.x, block-wide scan of the head flags)
    int carry = 0, nvalid = 0;
    for (int c0 = 0; c0 < P; c0 += blockDim.x) {
        const int i = c0 + tid;
        const uint64_t k = i < P ? keys[i] : ~0ull;
        const bool valid = k != ~0ull;
        const bool head = valid && (i == 0 || (keys[i - 1] >> 16) != (k >> 16));
        const uint64_t bal = __ballot(head);
        const int lane = tid & 63, wid = tid >> 6;
        const int before = __popcll(bal & (lane ? (~0ull >> (64 - lane)) : 0ull));
        const uint64_t vbal = __ballot(valid);
        if (lane == 0) {
            wsum[wid] = __popcll(bal);
            vsum[wid] = __popcll(vbal);
        }
        __syncthreads();
        int woff = 0, tot = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
            if (w < wid) woff += wsum[w];
            tot += wsum[w];
            nvalid += vsum[w];
        }
        if (valid) fv_feat[base + i] = (uint32_t)(k & 0xffff);
        if (head) {
            const int idx = carry + woff + before;
            fv_id[base + idx] = (uint32_t)(k >> 16);
            fv_off[(size_t)f * (cap + 1) + idx] = i;
        }
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) {
        fv_n[f] = carry;
        fv_off[(size_t)f * (cap + 1) + carry] = nvalid;
    }
}

// Pair table for k_bow_match from per-frame counts (device side), a wave per pair (lanes scan
// the Frame's nodes for the largest).  Pairs its tiles cannot hold (side > kBowCap features,
// > 4096 nodes, or a Frame node over 4 x 64 candidates) go to k_bow_match_any instead and are
// counted in *status.
__global__ void __launch_bounds__(64) k_make_pairs(int npairs, const int2* __restrict__ pairs, int cap,
                                                   const uint8_t* __restrict__ kps, const uint8_t* __restrict__ desc,
                                                   const int32_t* __restrict__ n_per_frame,
                                                   const uint8_t* __restrict__ valid, const uint32_t* __restrict__ fv_id,
                                                   const int32_t* __restrict__ fv_off,
                                                   const uint32_t* __restrict__ fv_feat, const int32_t* __restrict__ fv_n,
                                                   int32_t* __restrict__ a2b, int32_t* __restrict__ b2a,
                                                   int32_t* __restrict__ nmatch, DevBowPair* __restrict__ out,
                                                   int* __restrict__ status, uint8_t* __restrict__ scratch) {
    const int p = blockIdx.x, lane = threadIdx.x;
    if (p >= npairs) return;
    const int2 ab = pairs[p];
    auto side = [&](int f, bool use_valid) {
        DevBowSide S;
        S.desc = desc + (size_t)f * cap * 32;
        S.angle = reinterpret_cast<const float*>(kps + (size_t)f * cap * sizeof(slam_keypoint)) + 3;
        S.angle_stride = (int)(sizeof(slam_keypoint) / 4);
        S.valid = (use_valid && valid) ? valid + (size_t)f * cap : nullptr;
        S.n = min(n_per_frame[f], cap);
        S.n_nodes = fv_n[f];
        S.node_id = fv_id + (size_t)f * cap;
        S.node_off = fv_off + (size_t)f * (cap + 1);
        S.node_feat = fv_feat + (size_t)f * cap;
        return S;
    };
    DevBowPair pr;
    pr.A = side(ab.x, true);
    pr.B = side(ab.y, false);
    int big = 0;
    for (int i = lane; i < pr.B.n_nodes; i += 64) big |= pr.B.node_off[i + 1] - pr.B.node_off[i] > 64 * kBowNodeChunks;
    big = __any(big);
    if (lane != 0) return;
    pr.a2b = a2b + (size_t)p * cap;
    pr.b2a = b2a + (size_t)p * cap;
    pr.nmatches = nmatch + p;
    pr.bins = reinterpret_cast<int8_t*>(scratch + (size_t)p * 2 * cap);
    pr.taken = scratch + (size_t)p * 2 * cap + cap;
    const bool ok = pr.A.n <= kBowCap && pr.B.n <= kBowCap && pr.A.n_nodes <= 4096 && pr.B.n_nodes <= 4096 && !big;
    pr.general = !ok;
    if (!ok) atomicAdd(status, 1);
    out[p] = pr;
}

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    slam_status ensure(size_t need) {
        if (need <= bytes) return SLAM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, std::max<size_t>(need, 256)) != hipSuccess) return SLAM_ENOMEM;
        bytes = std::max<size_t>(need, 256);
        return SLAM_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

bool gfx950_device(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return false;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace

struct slam_vocab {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    hipStream_t stream = nullptr;
    Buf d_desc, d_child_ptr, d_child_idx, d_leaf, d_word, d_weight, d_child_desc, d_child_next;
    int root_c0 = 0, root_c1 = 0;
    Buf d_in, d_word_out, d_weight_out, d_node_out;
    std::mutex mu;
    DevVocab dev() const {
        DevVocab V;
        V.desc = d_desc.as<uint8_t>();
        V.child_ptr = d_child_ptr.as<int32_t>();
        V.child_idx = d_child_idx.as<int32_t>();
        V.is_leaf = d_leaf.as<uint8_t>();
        V.word = d_word.as<int32_t>();
        V.weight = d_weight.as<double>();
        V.child_desc = d_child_desc.as<uint8_t>();
        V.child_next = d_child_next.as<int4>();
        V.root_c0 = root_c0;
        V.root_c1 = root_c1;
        V.L = L;
        return V;
    }
};

struct slam_matcher {
    int device = 0;
    hipStream_t stream = nullptr;
    Buf d_pair, d_a, d_b, d_out;
    // batched device path (slamhot_bow_match_batch_device)
    Buf b_word, b_weight, b_node, b_fv_id, b_fv_off, b_fv_feat, b_fv_n, b_pairs, b_devpairs, b_status, b_scratch;
    uint8_t* h_stage = nullptr;  // pinned staging of the batched host-buffer calls
    size_t h_cap = 0;
    std::mutex mu;
    // the last batched host-buffer call on the stream: [0] before the first upload, [1] before the
    // first kernel, [2] after the last kernel, [3] after the read-back (slamhot_matcher_last_batch_stats)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float last_kernel_ms = 0, last_span_ms = 0;
    void batch_stats() {
        if (!ev[0] || hipEventElapsedTime(&last_kernel_ms, ev[1], ev[2]) != hipSuccess ||
            hipEventElapsedTime(&last_span_ms, ev[0], ev[3]) != hipSuccess)
            last_kernel_ms = last_span_ms = 0;
    }
    slam_status stage(size_t bytes) {
        if (bytes <= h_cap) return SLAM_OK;
        if (h_stage) (void)hipHostFree(h_stage);
        h_stage = nullptr;
        h_cap = 0;
        if (hipHostMalloc((void**)&h_stage, bytes, hipHostMallocDefault) != hipSuccess) return SLAM_ENOMEM;
        h_cap = bytes;
        return SLAM_OK;
    }
};

extern "C" {

slam_status slamhot_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                                 const int32_t* parent, const uint8_t* is_leaf,
                                 const uint8_t* desc, const double* weight, slam_vocab** out) {
    if (!out || !parent || !is_leaf || !desc || !weight || n_nodes < 1 || L < 1) return SLAM_EINVAL;
    *out = nullptr;
    if (!gfx950_device(device)) return SLAM_ENODEV;
    // children lists in node-table order (DBoW2 appends children as nodes are read)
    std::vector<int32_t> cnt(n_nodes + 1, 0), ptr(n_nodes + 1, 0), idx(std::max(1, n_nodes - 1));
    for (int i = 1; i < n_nodes; i++) {
        if (parent[i] < 0 || parent[i] >= n_nodes) return SLAM_EINVAL;
        cnt[parent[i]]++;
    }
    for (int i = 0; i < n_nodes; i++) ptr[i + 1] = ptr[i] + cnt[i];
    std::vector<int32_t> fill(ptr.begin(), ptr.end() - 1);
    for (int i = 1; i < n_nodes; i++) idx[fill[parent[i]]++] = i;
    std::vector<int32_t> word(n_nodes, -1);
    int nw = 0;
    for (int i = 0; i < n_nodes; i++)
        if (is_leaf[i]) word[i] = nw++;
    std::vector<uint8_t> leaf(is_leaf, is_leaf + n_nodes);
    for (int i = 0; i < n_nodes; i++)
        if (cnt[i] == 0) leaf[i] = 1;  // a childless node ends the descent
    // per child slot: the child's descriptor and {its child range, node id | leaf << 31}
    const size_t nslots = idx.size();
    std::vector<uint8_t> cdesc(nslots * 32, 0);
    std::vector<int32_t> cnext(nslots * 4, 0);
    for (int c = 0; c < ptr[n_nodes]; c++) {
        const int id = idx[c];
        std::memcpy(&cdesc[(size_t)c * 32], desc + (size_t)id * 32, 32);
        cnext[4 * (size_t)c] = ptr[id];
        cnext[4 * (size_t)c + 1] = ptr[id + 1];
        cnext[4 * (size_t)c + 2] = id | (leaf[id] ? (int32_t)0x80000000u : 0);
    }
    slam_vocab* v = new slam_vocab();
    v->device = device;
    v->root_c0 = ptr[0];
    v->root_c1 = ptr[1];
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->n_nodes = n_nodes;
    v->n_words = nw;
    auto fail = [&](slam_status st) { delete v; return st; };
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(SLAM_EHIP);
    slam_status st;
    if ((st = v->d_desc.ensure((size_t)n_nodes * 32)) || (st = v->d_child_ptr.ensure(ptr.size() * 4)) ||
        (st = v->d_child_idx.ensure(idx.size() * 4)) || (st = v->d_leaf.ensure(n_nodes)) ||
        (st = v->d_word.ensure((size_t)n_nodes * 4)) || (st = v->d_weight.ensure((size_t)n_nodes * 8)) ||
        (st = v->d_child_desc.ensure(cdesc.size())) || (st = v->d_child_next.ensure(cnext.size() * 4)))
        return fail(st);
    if (hipMemcpy(v->d_desc.p, desc, (size_t)n_nodes * 32, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_ptr.p, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_idx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_leaf.p, leaf.data(), n_nodes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_word.p, word.data(), (size_t)n_nodes * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_weight.p, weight, (size_t)n_nodes * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_desc.p, cdesc.data(), cdesc.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_next.p, cnext.data(), cnext.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(SLAM_EHIP);
    *out = v;
    return SLAM_OK;
}

// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1350-1436).  Documented
// deviation: blank lines are skipped (the reference turns the trailing empty line of
// ORBvoc.txt into a phantom child of the root with an indeterminate descriptor).
slam_status slamhot_vocab_load_text(int device, const char* path, slam_vocab** out) {
    if (!path || !out) return SLAM_EINVAL;
    std::ifstream f(path);
    if (!f) return SLAM_EINVAL;
    std::string s;
    std::getline(f, s);
    std::stringstream ss(s);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    ss >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return SLAM_EINVAL;
    std::vector<int32_t> parent(1, -1);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    while (std::getline(f, s)) {
        if (s.find_first_not_of(" \t\r\n") == std::string::npos) continue;
        std::stringstream sn(s);
        int pid = 0, isleaf = 0;
        sn >> pid >> isleaf;
        uint8_t d[32] = {0};
        for (int i = 0; i < 32; i++) {
            int n = 0;
            sn >> n;
            d[i] = (uint8_t)n;
        }
        double w = 0;
        sn >> w;
        parent.push_back(pid);
        leaf.push_back(isleaf > 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    return slamhot_vocab_create(device, k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(),
                                desc.data(), weight.data(), out);
}

void slamhot_vocab_destroy(slam_vocab* v) {
    if (!v) return;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    Buf* bufs[] = {&v->d_desc, &v->d_child_ptr, &v->d_child_idx, &v->d_leaf, &v->d_word, &v->d_weight,
                   &v->d_child_desc, &v->d_child_next, &v->d_in, &v->d_word_out, &v->d_weight_out, &v->d_node_out};
    for (Buf* b : bufs) b->release();
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
}

slam_status slamhot_vocab_info(const slam_vocab* v, int* k, int* L, int* n_nodes, int* n_words) {
    if (!v) return SLAM_EINVAL;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return SLAM_OK;
}

slam_status slamhot_vocab_transform_device(slam_vocab* v, int n, const void* d_desc, int desc_stride,
                                           int levelsup, void* d_word_id, void* d_weight, void* d_node_id,
                                           void* hip_stream) {
    if (!v || n < 0 || (n > 0 && (!d_desc || !d_word_id || !d_weight || !d_node_id)) || desc_stride < 32 ||
        (desc_stride & 15))
        return SLAM_EINVAL;
    if (n == 0) return SLAM_OK;
    SLAM_HIP_TRY(hipSetDevice(v->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : v->stream;
    const int blocks = (int)(((size_t)n * kVocG + kVocThreads - 1) / kVocThreads);
    hipLaunchKernelGGL(k_vocab_transform, dim3(blocks), dim3(kVocThreads), 0, s, v->dev(), n, (const uint8_t*)d_desc,
                       desc_stride, levelsup, (int32_t*)d_word_id, (double*)d_weight, (int32_t*)d_node_id,
                       (const int32_t*)nullptr, 1);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

namespace {
// the batched path's transform: nframes x cap slots, only each frame's first n slots
slam_status vocab_transform_frames(slam_vocab* v, int nframes, int cap, const void* d_desc, const int32_t* d_n,
                                   int levelsup, void* d_word_id, void* d_weight, void* d_node_id, hipStream_t s) {
    const size_t n = (size_t)nframes * cap;
    const int blocks = (int)((n * kVocG + kVocThreads - 1) / kVocThreads);
    hipLaunchKernelGGL(k_vocab_transform, dim3(blocks), dim3(kVocThreads), 0, s, v->dev(), (int)n, (const uint8_t*)d_desc, 32,
                       levelsup, (int32_t*)d_word_id, (double*)d_weight, (int32_t*)d_node_id, d_n, cap);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}
}  // namespace

slam_status slamhot_vocab_transform(slam_vocab* v, int n, const uint8_t* desc, int levelsup,
                                    int32_t* word_id, double* weight, int32_t* node_id) {
    if (!v || n < 0 || (n > 0 && (!desc || !word_id || !weight || !node_id))) return SLAM_EINVAL;
    if (n == 0) return SLAM_OK;
    std::lock_guard<std::mutex> g(v->mu);
    SLAM_HIP_TRY(hipSetDevice(v->device));
    slam_status st;
    if ((st = v->d_in.ensure((size_t)n * 32)) || (st = v->d_word_out.ensure((size_t)n * 4)) ||
        (st = v->d_weight_out.ensure((size_t)n * 8)) || (st = v->d_node_out.ensure((size_t)n * 4)))
        return st;
    SLAM_HIP_TRY(hipMemcpyAsync(v->d_in.p, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
    if ((st = slamhot_vocab_transform_device(v, n, v->d_in.p, 32, levelsup, v->d_word_out.p, v->d_weight_out.p,
                                             v->d_node_out.p, v->stream)))
        return st;
    SLAM_HIP_TRY(hipMemcpyAsync(word_id, v->d_word_out.p, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(weight, v->d_weight_out.p, (size_t)n * 8, hipMemcpyDeviceToHost, v->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(node_id, v->d_node_out.p, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(v->stream));
    return SLAM_OK;
}

// TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
// (TemplatedVocabulary.h:1139-1206): the descent on the device (slamhot_vocab_transform), the two
// maps on the host in DBoW2's own order of operations (DBoW2 enums: weighting TF_IDF 0, TF 1, IDF 2,
// BINARY 3; scoring L1_NORM 0, L2_NORM 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4, DOT_PRODUCT 5).
slam_status slamhot_compute_bow(slam_vocab* v, int n, const uint8_t* desc, int levelsup, int* n_words,
                                uint32_t* bow_word, double* bow_value, int* n_nodes, uint32_t* fv_node,
                                int32_t* fv_off, uint32_t* fv_feat) {
    if (!v || n < 0 || !n_words || !n_nodes || (n > 0 && (!desc || !bow_word || !bow_value || !fv_node || !fv_feat)) ||
        !fv_off)
        return SLAM_EINVAL;
    *n_words = 0;
    *n_nodes = 0;
    fv_off[0] = 0;
    if (n == 0) return SLAM_OK;
    std::vector<int32_t> word(n), node(n);
    std::vector<double> weight(n);
    slam_status st = slamhot_vocab_transform(v, n, desc, levelsup, word.data(), weight.data(), node.data());
    if (st) return st;
    // features not stopped (w > 0, :1169), in feature order
    std::vector<uint32_t> kept;
    kept.reserve(n);
    for (int i = 0; i < n; i++)
        if (weight[i] > 0) kept.push_back((uint32_t)i);
    // BowVector: stable sort by word keeps feature order inside a word = addWeight's summation order
    std::vector<uint32_t> by_word(kept);
    std::stable_sort(by_word.begin(), by_word.end(),
                     [&](uint32_t a, uint32_t b) { return (uint32_t)word[a] < (uint32_t)word[b]; });
    const bool sum_weights = v->weighting == 0 || v->weighting == 1;  // TF_IDF, TF: addWeight; else addIfNotExist
    int nw = 0;
    for (size_t j = 0; j < by_word.size();) {
        const uint32_t w = (uint32_t)word[by_word[j]];
        double val = weight[by_word[j]];
        size_t k = j + 1;
        for (; k < by_word.size() && (uint32_t)word[by_word[k]] == w; k++)
            if (sum_weights) val += weight[by_word[k]];
        bow_word[nw] = w;
        bow_value[nw] = val;
        nw++;
        j = k;
    }
    const bool must = v->scoring != 5;  // every ScoringObject but DotProductScoring normalises (ScoringObject.h:74-89)
    if (sum_weights && nw > 0 && !must) {
        const double nd = (double)nw;  // :1174-1180
        for (int j = 0; j < nw; j++) bow_value[j] /= nd;
    }
    if (must) {  // BowVector::normalize (BowVector.cpp:62-84): L2 for L2_NORM, L1 otherwise
        double norm = 0.0;
        if (v->scoring == 1) {
            for (int j = 0; j < nw; j++) norm += bow_value[j] * bow_value[j];
            norm = std::sqrt(norm);
        } else {
            for (int j = 0; j < nw; j++) norm += std::fabs(bow_value[j]);
        }
        if (norm > 0.0)
            for (int j = 0; j < nw; j++) bow_value[j] /= norm;
    }
    *n_words = nw;
    // FeatureVector: node ascending, features ascending inside a node (addFeature appends in order)
    std::vector<uint32_t> by_node(kept);
    std::stable_sort(by_node.begin(), by_node.end(),
                     [&](uint32_t a, uint32_t b) { return (uint32_t)node[a] < (uint32_t)node[b]; });
    int nn = 0;
    for (size_t j = 0; j < by_node.size(); j++) {
        const uint32_t id = (uint32_t)node[by_node[j]];
        if (nn == 0 || fv_node[nn - 1] != id) {
            fv_node[nn] = id;
            fv_off[nn] = (int32_t)j;
            nn++;
        }
        fv_feat[j] = by_node[j];
    }
    fv_off[nn] = (int32_t)by_node.size();
    *n_nodes = nn;
    return SLAM_OK;
}

slam_status slamhot_matcher_create(int device, slam_matcher** out) {
    if (!out) return SLAM_EINVAL;
    *out = nullptr;
    if (!gfx950_device(device)) return SLAM_ENODEV;
    slam_matcher* m = new slam_matcher();
    m->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
        delete m;
        return SLAM_EHIP;
    }
    for (hipEvent_t& e : m->ev)
        if (hipEventCreate(&e) != hipSuccess) {
            slamhot_matcher_destroy(m);
            return SLAM_EHIP;
        }
    *out = m;
    return SLAM_OK;
}

slam_status slamhot_matcher_last_batch_stats(const slam_matcher* m, float* kernel_ms, float* span_ms) {
    if (!m) return SLAM_EINVAL;
    if (kernel_ms) *kernel_ms = m->last_kernel_ms;
    if (span_ms) *span_ms = m->last_span_ms;
    return SLAM_OK;
}

void slamhot_matcher_destroy(slam_matcher* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    m->d_pair.release();
    m->d_a.release();
    m->d_b.release();
    m->d_out.release();
    for (Buf* b : {&m->b_word, &m->b_weight, &m->b_node, &m->b_fv_id, &m->b_fv_off, &m->b_fv_feat, &m->b_fv_n,
                   &m->b_pairs, &m->b_devpairs, &m->b_status, &m->b_scratch})
        b->release();
    if (m->h_stage) (void)hipHostFree(m->h_stage);
    for (hipEvent_t e : m->ev)
        if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

}  // extern "C"

namespace {

// Pack one host slam_bow_side into a device blob; fills the DevBowSide pointers.
size_t bow_side_bytes(const slam_bow_side* S) {
    auto r = [](size_t v) { return (v + 255) & ~(size_t)255; };
    return r((size_t)S->n * 32) + r((size_t)S->n * 4) + r((size_t)S->n) + r((size_t)S->n_nodes * 4) +
           r((size_t)(S->n_nodes + 1) * 4) + r((size_t)std::max(0, S->node_off[S->n_nodes]) * 4);
}

slam_status upload_bow_side(const slam_bow_side* S, uint8_t* base, DevBowSide& D, hipStream_t s) {
    auto r = [](size_t v) { return (v + 255) & ~(size_t)255; };
    uint8_t* p = base;
    D.n = S->n;
    D.n_nodes = S->n_nodes;
    D.desc = p;
    SLAM_HIP_TRY(hipMemcpyAsync(p, S->desc, (size_t)S->n * 32, hipMemcpyHostToDevice, s));
    p += r((size_t)S->n * 32);
    D.angle = reinterpret_cast<const float*>(p);
    D.angle_stride = 1;
    SLAM_HIP_TRY(hipMemcpyAsync(p, S->angle, (size_t)S->n * 4, hipMemcpyHostToDevice, s));
    p += r((size_t)S->n * 4);
    D.valid = nullptr;
    if (S->valid) {
        D.valid = p;
        SLAM_HIP_TRY(hipMemcpyAsync(p, S->valid, (size_t)S->n, hipMemcpyHostToDevice, s));
    }
    p += r((size_t)S->n);
    D.node_id = reinterpret_cast<const uint32_t*>(p);
    SLAM_HIP_TRY(hipMemcpyAsync(p, S->node_id, (size_t)S->n_nodes * 4, hipMemcpyHostToDevice, s));
    p += r((size_t)S->n_nodes * 4);
    D.node_off = reinterpret_cast<const int32_t*>(p);
    SLAM_HIP_TRY(hipMemcpyAsync(p, S->node_off, (size_t)(S->n_nodes + 1) * 4, hipMemcpyHostToDevice, s));
    p += r((size_t)(S->n_nodes + 1) * 4);
    D.node_feat = reinterpret_cast<const uint32_t*>(p);
    const size_t nf = (size_t)std::max(0, S->node_off[S->n_nodes]);
    if (nf) SLAM_HIP_TRY(hipMemcpyAsync(p, S->node_feat, nf * 4, hipMemcpyHostToDevice, s));
    return SLAM_OK;
}

bool bow_side_ok(const slam_bow_side* S) {
    if (!S || S->n < 0 || S->n >= (1 << 24) || S->n_nodes < 0) return false;
    if (S->n > 0 && (!S->desc || !S->angle)) return false;
    if (!S->node_off || (S->n_nodes > 0 && (!S->node_id || !S->node_feat))) return false;
    if (S->node_off[0] != 0) return false;
    for (int i = 0; i < S->n_nodes; i++) {
        if (S->node_off[i + 1] < S->node_off[i]) return false;
        if (i && S->node_id[i] <= S->node_id[i - 1]) return false;
        for (int p = S->node_off[i]; p < S->node_off[i + 1]; p++)
            if (S->node_feat[p] >= (uint32_t)S->n) return false;
    }
    return true;
}

}  // namespace

extern "C" slam_status slamhot_search_by_bow(slam_matcher* m, const slam_bow_side* A, const slam_bow_side* B,
                                             float nnratio, int check_ori, int strict, int32_t* a2b,
                                             int32_t* b2a, int* nmatches) {
    if (!m || !bow_side_ok(A) || !bow_side_ok(B) || !a2b || !b2a || !nmatches) return SLAM_EINVAL;
    // k_bow_match's LDS / register tiles, else the unbounded k_bow_match_any
    bool fits = A->n <= kBowCap && B->n <= kBowCap && A->n_nodes <= 4096 && B->n_nodes <= 4096;
    for (int i = 0; fits && i < B->n_nodes; i++)
        if (B->node_off[i + 1] - B->node_off[i] > 64 * kBowNodeChunks) fits = false;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    slam_status st;
    const size_t ba = bow_side_bytes(A), bb = bow_side_bytes(B);
    const size_t nout = ((size_t)A->n + B->n + 1) * 4;
    if ((st = m->d_a.ensure(ba)) || (st = m->d_b.ensure(bb)) || (st = m->d_out.ensure(nout)) ||
        (st = m->d_pair.ensure(sizeof(DevBowPair))) || (!fits && (st = m->b_scratch.ensure((size_t)A->n + B->n + 8))))
        return st;
    DevBowPair pr{};
    if ((st = upload_bow_side(A, m->d_a.as<uint8_t>(), pr.A, m->stream)) ||
        (st = upload_bow_side(B, m->d_b.as<uint8_t>(), pr.B, m->stream)))
        return st;
    pr.a2b = m->d_out.as<int32_t>();
    pr.b2a = pr.a2b + A->n;
    pr.nmatches = pr.b2a + B->n;
    pr.general = !fits;
    if (!fits) {
        pr.bins = m->b_scratch.as<int8_t>();
        pr.taken = m->b_scratch.as<uint8_t>() + A->n;
    }
    SLAM_HIP_TRY(hipMemcpyAsync(m->d_pair.p, &pr, sizeof(pr), hipMemcpyHostToDevice, m->stream));
    if (fits)
        hipLaunchKernelGGL(k_bow_match, dim3(1), dim3(kBowThreads), 0, m->stream, m->d_pair.as<DevBowPair>(), nnratio,
                           check_ori, strict);
    else
        hipLaunchKernelGGL(k_bow_match_any, dim3(1), dim3(512), 0, m->stream, m->d_pair.as<DevBowPair>(), nnratio,
                           check_ori, strict);
    SLAM_HIP_TRY(hipGetLastError());
    std::vector<int32_t> out((size_t)A->n + B->n + 1);
    SLAM_HIP_TRY(hipMemcpyAsync(out.data(), m->d_out.p, nout, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(m->stream));
    std::copy(out.begin(), out.begin() + A->n, a2b);
    std::copy(out.begin() + A->n, out.begin() + A->n + B->n, b2a);
    *nmatches = out[(size_t)A->n + B->n];
    return SLAM_OK;
}

extern "C" slam_status slamhot_bow_match_batch_device(slam_matcher* m, slam_vocab* v, int nframes, const void* d_kps,
                                                      const void* d_desc, int cap, const void* d_n,
                                                      const void* d_valid, int npairs, const int32_t* pairs,
                                                      float nnratio, int check_ori, int strict, int levelsup,
                                                      void* d_a2b, void* d_b2a, void* d_nmatches, void* hip_stream) {
    if (!m || !v || nframes < 0 || npairs < 0 || cap <= 0 || cap > kFvMax || (nframes && (!d_kps || !d_desc || !d_n)) ||
        (npairs && (!pairs || !d_a2b || !d_b2a || !d_nmatches)) || m->device != v->device)
        return SLAM_EINVAL;
    for (int i = 0; i < 2 * npairs; i++)
        if (pairs[i] < 0 || pairs[i] >= nframes) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
    const size_t nf = (size_t)nframes * cap;
    slam_status st;
    if ((st = m->b_word.ensure(nf * 4)) || (st = m->b_weight.ensure(nf * 8)) || (st = m->b_node.ensure(nf * 4)) ||
        (st = m->b_fv_id.ensure(nf * 4)) || (st = m->b_fv_off.ensure((size_t)nframes * (cap + 1) * 4)) ||
        (st = m->b_fv_feat.ensure(nf * 4)) || (st = m->b_fv_n.ensure((size_t)nframes * 4 + 4)) ||
        (st = m->b_pairs.ensure((size_t)npairs * 8 + 8)) || (st = m->b_devpairs.ensure((size_t)npairs * sizeof(DevBowPair) + 8)) ||
        (st = m->b_status.ensure(4)) || (st = m->b_scratch.ensure((size_t)npairs * 2 * cap + 8)))
        return st;
    if (nframes == 0) return SLAM_OK;
    // Frame::ComputeBoW (Frame.cc:721-728): transform every descriptor slot of every frame
    if ((st = vocab_transform_frames(v, nframes, cap, d_desc, (const int32_t*)d_n, levelsup, m->b_word.p,
                                     m->b_weight.p, m->b_node.p, s)))
        return st;
    hipLaunchKernelGGL(k_featvec, dim3(nframes), dim3(1024), 0, s, cap, (const int32_t*)d_n,
                       m->b_node.as<int32_t>(), m->b_weight.as<double>(), m->b_fv_id.as<uint32_t>(),
                       m->b_fv_off.as<int32_t>(), m->b_fv_feat.as<uint32_t>(), m->b_fv_n.as<int32_t>());
    SLAM_HIP_TRY(hipGetLastError());
    if (npairs == 0) return SLAM_OK;
    SLAM_HIP_TRY(hipMemcpyAsync(m->b_pairs.p, pairs, (size_t)npairs * 8, hipMemcpyHostToDevice, s));
    SLAM_HIP_TRY(hipMemsetAsync(m->b_status.p, 0, 4, s));
    hipLaunchKernelGGL(k_make_pairs, dim3(npairs), dim3(64), 0, s, npairs, m->b_pairs.as<int2>(), cap,
                       (const uint8_t*)d_kps, (const uint8_t*)d_desc, (const int32_t*)d_n, (const uint8_t*)d_valid,
                       m->b_fv_id.as<uint32_t>(), m->b_fv_off.as<int32_t>(), m->b_fv_feat.as<uint32_t>(),
                       m->b_fv_n.as<int32_t>(), (int32_t*)d_a2b, (int32_t*)d_b2a, (int32_t*)d_nmatches,
                       m->b_devpairs.as<DevBowPair>(), m->b_status.as<int>(), m->b_scratch.as<uint8_t>());
    hipLaunchKernelGGL(k_bow_match, dim3(npairs), dim3(kBowThreads), 0, s, m->b_devpairs.as<DevBowPair>(), nnratio,
                       check_ori, strict);
    hipLaunchKernelGGL(k_bow_match_any, dim3(npairs), dim3(512), 0, s, m->b_devpairs.as<DevBowPair>(), nnratio,
                       check_ori, strict);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

extern "C" slam_status slamhot_bow_match_batch_status(slam_matcher* m, void* hip_stream, int* skipped_pairs) {
    if (!m || !skipped_pairs) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
    int v = 0;
    if (m->b_status.p) {
        SLAM_HIP_TRY(hipMemcpyAsync(&v, m->b_status.p, 4, hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
    }
    *skipped_pairs = v;
    return SLAM_OK;
}

// =======================================================================================
// SearchByProjection (ORBmatcher.cc:44-214, 2173-2389, 2391-2513), pinhole.
//
// One workgroup per frame (1024 threads), one launch:
//   1. per query (MapPoint): its search window — from Frame::isInFrustum's fields (local
//      map), from projecting the last frame's MapPoints on the device (last frame; cv::Mat
//      float products restated as double-accumulated gemm), or host-prepared (KeyFrame
//      variant, whose PredictScale needs glibc logf);
//   2. per query: Frame::GetFeaturesInArea over the 64x48 grid in the reference's
//      candidate order (cell column, cell row, insertion order), static filters (levels,
//      box, stereo gate, entry occupancy) and Hamming distances -> candidate lists;
//   3. the reference processes queries sequentially and a match occupies the feature for
//      the later queries.  Jacobi iteration of  choice(q) = f(candidates of q minus features
//      owned by an earlier blocking query)  converges to exactly the sequential result
//      (induction on q) — iterate until no choice changes;
//   4. last assignment per feature wins; rotation histogram + ComputeThreeMaxima.
// =======================================================================================
namespace slamhot {

__device__ __forceinline__ void gemm_rx_t(const float* T, const float* X, float* o) {
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[4 * i] * (double)X[0] + (double)T[4 * i + 1] * (double)X[1] +
                           (double)T[4 * i + 2] * (double)X[2];
        o[i] = (float)(acc * 1.0 + (double)T[4 * i + 3] * 1.0);
    }
}
__device__ __forceinline__ void neg_rtt(const float* T, float* o) {
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[i] * (double)T[3] + (double)T[4 + i] * (double)T[7] +
                           (double)T[8 + i] * (double)T[11];
        o[i] = (float)(-1.0 * acc);
    }
}

__device__ __forceinline__ int hamming_bytes(const uint8_t* a, const uint8_t* b) {
    const uint4* pa = reinterpret_cast<const uint4*>(a);
    const uint4* pb = reinterpret_cast<const uint4*>(b);
    return hamming32(pa[0], pa[1], pb[0], pb[1]);
}

// Frame::GetFeaturesInArea window (Frame.cc:646-673); returns false when empty
__device__ __forceinline__ bool grid_window(const DevProjFrame& F, float x, float y, float r, int& x0,
                                            int& x1, int& y0, int& y1) {
    x0 = max(0, (int)floorf((x - F.min_x - r) * F.inv_w));
    if (x0 >= kGridCols) return false;
    x1 = min(kGridCols - 1, (int)ceilf((x - F.min_x + r) * F.inv_w));
    if (x1 < 0) return false;
    y0 = max(0, (int)floorf((y - F.min_y - r) * F.inv_h));
    if (y0 >= kGridRows) return false;
    y1 = min(kGridRows - 1, (int)ceilf((y - F.min_y + r) * F.inv_h));
    if (y1 < 0) return false;
    return true;
}

// visit the candidates of query q in reference order; fn(feature)
template <class Fn>
__device__ __forceinline__ void for_candidates(const DevProjFrame& F, const ProjQuery& Q, Fn fn) {
    int x0, x1, y0, y1;
    if (!grid_window(F, Q.u, Q.v, Q.r, x0, x1, y0, y1)) return;
    const bool check = (Q.min_level > 0) || (Q.max_level >= 0);
    for (int ix = x0; ix <= x1; ix++) {
        const int c0 = F.cell_start[ix * kGridRows + y0], c1 = F.cell_start[ix * kGridRows + y1 + 1];
        for (int c = c0; c < c1; c++) {
            const int idx = F.cell_feat[c];
            const slam_keypoint kp = F.kps[idx];
            if (check) {
                if (kp.octave < Q.min_level) continue;
                if (Q.max_level >= 0 && kp.octave > Q.max_level) continue;
            }
            const float dx = kp.x - Q.u, dy = kp.y - Q.v;
            if (fabsf(dx) < Q.r && fabsf(dy) < Q.r) fn(idx, kp);
        }
    }
}

__global__ void __launch_bounds__(1024) k_search_by_projection(const DevProjCall* __restrict__ calls) {
    const DevProjCall& C = calls[blockIdx.x];
    __shared__ int scratch[20];
    __shared__ int s_flag, s_hist[32], s_keep[3], s_count;
    const DevProjFrame& F = C.F;
    const int tid = threadIdx.x, NT = blockDim.x;
    const int nq = C.nq;
    // ---- 1. queries
    if (C.mode == kProjLocal) {
        const bool bFactor = C.th != 1.0f;
        for (int q = tid; q < nq; q += NT) {
            const slam_mp_track mp = C.mps[q];
            ProjQuery Q;
            Q.valid = mp.in_view && !(C.far_points && mp.depth > C.th_far) && !mp.is_bad;
            const int level = min(max(mp.scale_level, 0), F.nlevels - 1);
            float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
            if (bFactor) r *= C.th;
            Q.u = mp.proj_x;
            Q.v = mp.proj_y;
            Q.r = r * F.scale[level];
            Q.ur = mp.proj_xr;
            Q.er = r * F.scale[level];
            Q.min_level = (int16_t)(mp.scale_level - 1);
            Q.max_level = (int16_t)mp.scale_level;
            Q.angle = 0.f;
            Q.blocking = mp.has_obs;
            C.queries[q] = Q;
        }
    } else if (C.mode == kProjLast) {
        float twc[3], tlc[3];
        neg_rtt(F.T, twc);
        gemm_rx_t(C.LT, twc, tlc);
        const bool fwd = tlc[2] > F.b && !C.mono;
        const bool bwd = -tlc[2] > F.b && !C.mono;
        for (int q = tid; q < nq; q += NT) {
            ProjQuery Q;
            Q.valid = 0;
            Q.blocking = C.lf_has_obs[q];
            Q.angle = C.lf_kps_un[q].angle;
            Q.er = -1.f;
            if (C.lf_has_mp[q] && !C.lf_outlier[q]) {
                float xc[3];
                gemm_rx_t(F.T, C.lf_pos + 3 * (size_t)q, xc);
                const float invzc = (float)(1.0 / (double)xc[2]);
                if (invzc >= 0) {
                    const float u = F.fx * xc[0] / xc[2] + F.cx;
                    const float v = F.fy * xc[1] / xc[2] + F.cy;
                    if (!(u < F.min_x || u > F.max_x) && !(v < F.min_y || v > F.max_y)) {
                        const int oct = C.lf_kps[q].octave;
                        Q.valid = 1;
                        Q.u = u;
                        Q.v = v;
                        Q.r = C.th * F.scale[min(max(oct, 0), F.nlevels - 1)];
                        Q.ur = gate::right_u(u, F.bf, invzc);  // ORBmatcher.cc.o @0x95c7
                        Q.er = Q.r;
                        if (fwd) { Q.min_level = (int16_t)oct; Q.max_level = -1; }
                        else if (bwd) { Q.min_level = 0; Q.max_level = (int16_t)oct; }
                        else { Q.min_level = (int16_t)(oct - 1); Q.max_level = (int16_t)(oct + 1); }
                    }
                }
            }
            C.queries[q] = Q;
        }
    }
    __syncthreads();
    // ---- 2. candidate lists: count, scan, fill (static filters + distances)
    const bool any_blocks = C.mode == kProjKF;  // KF variant: any MapPoint occupies
    auto pre_blocked = [&](int idx) -> bool {
        const int st = F.state ? F.state[idx] : -1;
        return any_blocks ? st >= 0 : st == 1;
    };
    auto stereo_ok = [&](const ProjQuery& Q, int idx) -> bool {
        if (Q.er < 0.f || !F.uright) return true;
        const float urr = F.uright[idx];
        if (!(urr > 0)) return true;
        return !(fabsf(Q.ur - urr) > Q.er);
    };
    int carry = 0;
    for (int base = 0; base < nq; base += NT) {
        const int q = base + tid;
        int cnt = 0;
        if (q < nq) {
            const ProjQuery Q = C.queries[q];
            if (Q.valid)
                for_candidates(F, Q, [&](int idx, const slam_keypoint&) {
                    if (!pre_blocked(idx) && stereo_ok(Q, idx)) cnt++;
                });
        }
        int tot;
        const int incl = block_scan_incl(cnt, scratch, &tot);
        if (q < nq) C.cand_off[q] = carry + incl - cnt;
        carry += tot;
    }
    if (tid == 0) C.cand_off[nq] = carry;
    if (carry > C.cand_cap) {
        if (tid == 0) C.out[1] = 1;
        return;
    }
    __syncthreads();
    for (int q = tid; q < nq; q += NT) {
        const ProjQuery Q = C.queries[q];
        if (!Q.valid) continue;
        int w = C.cand_off[q];
        const uint8_t* qd = C.qdesc + (size_t)q * 32;
        for_candidates(F, Q, [&](int idx, const slam_keypoint&) {
            if (!pre_blocked(idx) && stereo_ok(Q, idx))
                C.cand[w++] = ((uint32_t)idx << 12) | (uint32_t)hamming_bytes(qd, F.desc + (size_t)idx * 32);
        });
    }
    // ---- 3. Jacobi resolution of the sequential greedy (state in LDS: owner per
    //         feature, two assignment buffers per query, final match per feature)
    extern __shared__ __attribute__((aligned(16))) int32_t proj_smem[];
    int32_t* owner = C.gstate ? C.gstate : proj_smem;  // one workgroup either way
    int32_t* fm = owner + F.n;
    int32_t* cur = fm + F.n;
    int32_t* nxt = cur + nq;
    for (int q = tid; q < nq; q += NT) cur[q] = -2;  // "not computed yet"
    __syncthreads();
    auto choose = [&](int q) -> int {
        const int c0 = C.cand_off[q], c1 = C.cand_off[q + 1];
        if (C.mode == kProjLocal) {
            int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
            for (int c = c0; c < c1; c++) {
                const int idx = (int)(C.cand[c] >> 12), dist = (int)(C.cand[c] & 0xFFF);
                if (owner[idx] < q) continue;
                if (dist < bestDist) {
                    bestDist2 = bestDist;
                    bestDist = dist;
                    bestLevel2 = bestLevel;
                    bestLevel = F.kps[idx].octave;
                    bestIdx = idx;
                } else if (dist < bestDist2) {
                    bestLevel2 = F.kps[idx].octave;
                    bestDist2 = dist;
                }
            }
            if (bestDist <= 100) {
                if (bestLevel == bestLevel2 && (float)bestDist > C.nnratio * (float)bestDist2) return -1;
                if (bestLevel != bestLevel2 || (float)bestDist <= C.nnratio * (float)bestDist2) return bestIdx;
            }
            return -1;
        }
        int bestDist = 256, bestIdx = -1;
        for (int c = c0; c < c1; c++) {
            const int idx = (int)(C.cand[c] >> 12), dist = (int)(C.cand[c] & 0xFFF);
            if (owner[idx] < q) continue;
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        return bestDist <= C.th_dist ? bestIdx : -1;
    };
    int iters = 0;
    for (; iters < nq + 2; iters++) {
        for (int i = tid; i < F.n; i += NT) owner[i] = 0x7fffffff;
        if (tid == 0) s_flag = 0;
        __syncthreads();
        for (int q = tid; q < nq; q += NT) {
            const int a = cur[q];
            if (a >= 0 && (any_blocks || C.queries[q].blocking)) atomicMin(&owner[a], q);
        }
        __syncthreads();
        int changed = 0;
        for (int q = tid; q < nq; q += NT) {
            const int a = C.queries[q].valid ? choose(q) : -1;
            nxt[q] = a;
            changed |= a != cur[q];
        }
        if (changed) s_flag = 1;
        __syncthreads();
        int32_t* t = cur;
        cur = nxt;
        nxt = t;
        const int fl = s_flag;
        __syncthreads();
        if (!fl) break;
    }
    // ---- 4. finalize: last assignment per feature wins; rotation consistency
    for (int i = tid; i < F.n; i += NT) fm[i] = -1;
    if (tid < 32) s_hist[tid] = 0;
    if (tid == 0) s_count = 0;
    __syncthreads();
    int cnt = 0;
    for (int q = tid; q < nq; q += NT) {
        const int a = cur[q];
        if (a >= 0) {
            atomicMax(&fm[a], q);
            cnt++;
            if (C.check_ori) atomicAdd(&s_hist[rot_bin(C.queries[q].angle, F.kps[a].angle)], 1);
        }
    }
    atomicAdd(&s_count, cnt);
    __syncthreads();
    if (C.check_ori) {
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < 30; i++) {
                const int sv = s_hist[i];
                if (sv > max1) { max3 = max2; max2 = max1; max1 = sv; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (sv > max2) { max3 = max2; max2 = sv; ind3 = ind2; ind2 = i; }
                else if (sv > max3) { max3 = sv; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            s_keep[0] = ind1; s_keep[1] = ind2; s_keep[2] = ind3;
        }
        __syncthreads();
        int drop = 0;
        for (int q = tid; q < nq; q += NT) {
            const int a = cur[q];
            if (a >= 0) {
                const int bin = rot_bin(C.queries[q].angle, F.kps[a].angle);
                if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2]) {
                    fm[a] = -2;  // set to NULL after all assignments (ORBmatcher.cc:2371-2386, 2491-2510)
                    drop++;
                }
            }
        }
        atomicSub(&s_count, drop);
        __syncthreads();
    }
    for (int i = tid; i < F.n; i += NT) C.f_match[i] = fm[i];
    if (tid == 0) {
        C.out[0] = s_count;
        C.out[2] = iters + 1;
    }
}

// Frame::isInFrustum (Frame.cc:493-556) for a Frame with Nleft == -1, one thread per local
// MapPoint, in the compiled reference's float arithmetic (gate_fp.hpp): cv::Matx33f x Matx31f
// and Matx::dot as fma chains, cv::norm summed in double, Pinhole::project as (f * x) / z + c.
// MapPoint::PredictScale's ceil(logf(ratio) / mfLogScaleFactor) uses the correctly rounded
// logf ((float)log((double)r)); its ceil equals glibc logf's for every ratio in [1e-3, 1e3]
// (exhaustive check, tests/test_projection_oracle.py).
__global__ void __launch_bounds__(256) k_is_in_frustum(const FrustumCall* __restrict__ calls) {
    const FrustumCall& C = calls[blockIdx.y];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const slam_mp_geom g = C.mps[i];
    slam_mp_track tr{};
    tr.proj_x = -1.0f;
    tr.proj_y = -1.0f;
    tr.scale_level = -1;
    tr.is_bad = g.is_bad;
    tr.has_obs = g.has_obs;
    tr.in_view = 0;
    bool ok = !g.seen && !g.is_bad;
    // Frame::isInFrustum as compiled (Frame.cc.o @0x9ee0; gate_fp.hpp): Matx products as fma
    // chains, cv::norm in double, mTrackProjX/Y written once the point is in the image
    float Pc[3];
#pragma unroll
    for (int r = 0; r < 3; r++)
        Pc[r] = gate::chain3(C.R[3 * r], g.pos[0], C.R[3 * r + 1], g.pos[1], C.R[3 * r + 2], g.pos[2]) + C.t[r];
    const float Pc_dist = (float)sqrt(gate::norm2(Pc[0], Pc[1], Pc[2]));
    const float PcZ = Pc[2];
    const float invz = 1.0f / PcZ;
    if (PcZ < 0.0f) ok = false;
    const float u = C.fx * Pc[0] / PcZ + C.cx;
    const float v = C.fy * Pc[1] / PcZ + C.cy;
    if (u < C.min_x || u > C.max_x || v < C.min_y || v > C.max_y) ok = false;
    if (ok) {
        tr.proj_x = u;
        tr.proj_y = v;
    }
    const float maxDistance = 1.2f * g.max_dist;
    const float minDistance = 0.8f * g.min_dist;
    const float PO[3] = {g.pos[0] - C.Ow[0], g.pos[1] - C.Ow[1], g.pos[2] - C.Ow[2]};
    const float dist = (float)sqrt(gate::norm2(PO[0], PO[1], PO[2]));
    if (dist < minDistance || dist > maxDistance) ok = false;
    const float viewCos = gate::chain3(PO[0], g.normal[0], PO[1], g.normal[1], PO[2], g.normal[2]) / dist;
    if (viewCos < C.view_cos_limit) ok = false;
    if (ok) {
        const float ratio = g.max_dist / dist;
        const float lr = (float)log((double)ratio);
        int nScale = (int)ceilf(lr / C.log_scale);
        if (nScale < 0) nScale = 0;
        else if (nScale >= C.nlevels) nScale = C.nlevels - 1;
        tr.in_view = 1;
        tr.proj_x = u;
        tr.proj_xr = gate::right_u(u, C.bf, invz);
        tr.depth = Pc_dist;
        tr.proj_y = v;
        tr.scale_level = nScale;
        tr.view_cos = viewCos;
        atomicAdd(C.n_in_view, 1);
    }
    C.track[i] = tr;
}


constexpr size_t kProjLdsMax = 150 * 1024;

size_t projection_lds_bytes(int n_features, int n_queries) {
    const size_t lds = (size_t)4 * (2 * (size_t)n_features + 2 * (size_t)n_queries);
    return lds > kProjLdsMax ? 0 : lds;
}

hipError_t launch_search_by_projection(const DevProjCall* calls, int ncalls, size_t lds, hipStream_t s) {
    if (ncalls <= 0) return hipSuccess;
    hipError_t e = hipFuncSetAttribute((const void*)k_search_by_projection, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds + 16);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_search_by_projection, dim3(ncalls), dim3(1024), lds, s, calls);
    return hipGetLastError();
}

hipError_t launch_is_in_frustum(const FrustumCall* calls, int ncalls, int max_n, hipStream_t s) {
    if (ncalls <= 0 || max_n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_is_in_frustum, dim3((max_n + 255) / 256, ncalls), dim3(256), 0, s, calls);
    return hipGetLastError();
}

}  // namespace slamhot

namespace {

// Frame::AssignFeaturesToGrid (Frame.cc:380-411) as CSR, cells ordered [ix][iy]
void build_grid_csr(const slam_frame_view* F, std::vector<int32_t>& start, std::vector<int32_t>& feat) {
    const int ncell = kGridCols * kGridRows;
    std::vector<int32_t> cell(F->n, -1), cnt(ncell, 0);
    for (int i = 0; i < F->n; i++) {
        const slam_keypoint& kp = F->kps_un[i];
        const int px = (int)std::round((kp.x - F->min_x) * F->grid_inv_w);
        const int py = (int)std::round((kp.y - F->min_y) * F->grid_inv_h);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        cell[i] = px * kGridRows + py;
        cnt[cell[i]]++;
    }
    start.assign(ncell + 1, 0);
    for (int c = 0; c < ncell; c++) start[c + 1] = start[c] + cnt[c];
    feat.assign(std::max(1, start[ncell]), 0);
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    for (int i = 0; i < F->n; i++)
        if (cell[i] >= 0) feat[fill[cell[i]]++] = i;
}

struct Blob {  // bump allocator over one device buffer, uploads from host
    uint8_t* base;
    size_t off = 0;
    hipStream_t s;
    template <class T>
    const T* put(const T* host, size_t count) {
        if (!host || !count) return nullptr;
        uint8_t* p = base + off;
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        (void)hipMemcpyAsync(p, host, count * sizeof(T), hipMemcpyHostToDevice, s);
        return reinterpret_cast<const T*>(p);
    }
    template <class T>
    T* take(size_t count) {
        uint8_t* p = base + off;
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        return reinterpret_cast<T*>(p);
    }
};

bool frame_ok(const slam_frame_view* F) {
    return F && F->n >= 0 && F->n < (1 << 20) && (F->n == 0 || (F->kps_un && F->desc)) && F->nlevels >= 1 &&
           F->nlevels <= 16 && F->scale;
}

bool last_ok(const slam_last_frame* LF) {
    return LF && LF->Tcw && LF->n >= 0 &&
           (LF->n == 0 || (LF->kps && LF->kps_un && LF->has_mp && LF->outlier && LF->mp_pos && LF->mp_desc &&
                           LF->mp_has_obs));
}

bool kf_ok(const slam_kf_points* KF) {
    return KF && KF->n >= 0 &&
           (KF->n == 0 || (KF->kps_un && KF->use && KF->mp_pos && KF->max_dist && KF->min_dist && KF->mp_desc));
}

slam_status run_projection(slam_matcher* m, const slam_frame_view* F, DevProjCall& Cc, int nq,
                           const std::vector<ProjQuery>* host_queries, const uint8_t* qdesc,
                           int32_t* f_match, int* nmatches,
                           const std::function<void(Blob&, DevProjCall&)>& put_inputs) {
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    std::vector<int32_t> start, feat;
    build_grid_csr(F, start, feat);
    int cap = std::max(4096, nq * 64);
    for (int attempt = 0; attempt < 2; attempt++) {
        const size_t need = (size_t)F->n * (sizeof(slam_keypoint) + 4 + 32 + 1 + 4 * 2) + start.size() * 4 +
                            feat.size() * 4 + (size_t)nq * (sizeof(ProjQuery) + 32 + 4 * 3 + 2 * sizeof(slam_mp_track) + sizeof(slam_mp_geom) + 64) +
                            (size_t)cap * 4 + 64 * 1024 + (size_t)4 * (2 * (size_t)F->n + 2 * (size_t)nq) + 512;
        slam_status st;
        if ((st = m->d_a.ensure(need * 2))) return st;
        Blob B{m->d_a.as<uint8_t>(), 0, m->stream};
        DevProjCall C = Cc;
        C.F.n = F->n;
        C.F.kps = B.put(F->kps_un, F->n);
        C.F.uright = B.put(F->uright, F->n);
        C.F.desc = B.put(F->desc, (size_t)F->n * 32);
        C.F.state = B.put(F->mp_state, F->n);
        C.F.cell_start = B.put(start.data(), start.size());
        C.F.cell_feat = B.put(feat.data(), feat.size());
        put_inputs(B, C);
        C.nq = nq;
        if (host_queries) C.queries = const_cast<ProjQuery*>(B.put(host_queries->data(), host_queries->size()));
        else C.queries = B.take<ProjQuery>(std::max(1, nq));
        C.qdesc = B.put(qdesc, (size_t)nq * 32);
        C.cand_off = B.take<int32_t>(nq + 1);
        C.cand = B.take<uint32_t>(cap);
        C.cand_cap = cap;
        C.f_match = B.take<int32_t>(std::max(1, F->n));
        C.out = B.take<int32_t>(4);
        SLAM_HIP_TRY(hipMemsetAsync(C.out, 0, 16, m->stream));
        const size_t lds = projection_lds_bytes(F->n, nq);
        C.gstate = nullptr;
        if (!lds)  // large local map: the owner / match / assignment arrays in HBM
            C.gstate = B.take<int32_t>(2 * (size_t)F->n + 2 * (size_t)nq);
        const DevProjCall* dC = B.put(&C, 1);
        SLAM_HIP_TRY(launch_search_by_projection(dC, 1, lds, m->stream));
        int32_t out[4];
        SLAM_HIP_TRY(hipMemcpyAsync(out, C.out, 16, hipMemcpyDeviceToHost, m->stream));
        if (F->n) SLAM_HIP_TRY(hipMemcpyAsync(f_match, C.f_match, (size_t)F->n * 4, hipMemcpyDeviceToHost, m->stream));
        SLAM_HIP_TRY(hipStreamSynchronize(m->stream));
        if (out[1] == 1) {  // candidate overflow: exact size is cand_off[nq]
            int32_t total = 0;
            SLAM_HIP_TRY(hipMemcpy(&total, C.cand_off + nq, 4, hipMemcpyDeviceToHost));
            cap = total + 1024;
            continue;
        }
        *nmatches = out[0];
        return SLAM_OK;
    }
    return SLAM_EINVAL;
}

void fill_frame(DevProjCall& C, const slam_frame_view* F) {
    C.F.min_x = F->min_x;
    C.F.min_y = F->min_y;
    C.F.max_x = F->max_x;
    C.F.max_y = F->max_y;
    C.F.inv_w = F->grid_inv_w;
    C.F.inv_h = F->grid_inv_h;
    C.F.fx = F->fx;
    C.F.fy = F->fy;
    C.F.cx = F->cx;
    C.F.cy = F->cy;
    C.F.bf = F->bf;
    C.F.b = F->b;
    C.F.nlevels = F->nlevels;
    for (int i = 0; i < 16; i++) {
        C.F.T[i] = F->Tcw ? F->Tcw[i] : 0.f;
        C.F.scale[i] = i < F->nlevels ? F->scale[i] : 1.f;
    }
}

}  // namespace

extern "C" slam_status slamhot_search_by_projection_local(slam_matcher* m, const slam_frame_view* F, int n_mp,
                                                          const slam_mp_track* mps, const uint8_t* mp_desc,
                                                          float nnratio, float th, int far_points, float th_far,
                                                          int32_t* f_match, int* nmatches) {
    if (!m || !frame_ok(F) || n_mp < 0 || (n_mp && (!mps || !mp_desc)) || !f_match || !nmatches) return SLAM_EINVAL;
    DevProjCall C{};
    fill_frame(C, F);
    C.mode = kProjLocal;
    C.th = th;
    C.th_far = th_far;
    C.far_points = far_points;
    C.nnratio = nnratio;
    C.th_dist = 100;
    C.check_ori = 0;
    return run_projection(m, F, C, n_mp, nullptr, mp_desc, f_match, nmatches,
                          [&](Blob& B, DevProjCall& c) { c.mps = B.put(mps, n_mp); });
}

extern "C" slam_status slamhot_search_local_points(slam_matcher* m, const slam_frame_view* F, int n_mp,
                                                   const slam_mp_geom* mps, const uint8_t* mp_desc,
                                                   float view_cos_limit, float nnratio, float th, int far_points,
                                                   float th_far, slam_mp_track* track, int* n_to_match,
                                                   int32_t* f_match, int* nmatches) {
    if (!m || !frame_ok(F) || !F->Tcw || n_mp < 0 || (n_mp && (!mps || !mp_desc)) || !n_to_match || !f_match ||
        !nmatches)
        return SLAM_EINVAL;
    DevProjCall C{};
    fill_frame(C, F);
    C.mode = kProjLocal;
    C.th = th;
    C.th_far = th_far;
    C.far_points = far_points;
    C.nnratio = nnratio;
    C.th_dist = 100;
    C.check_ori = 0;
    FrustumCall Fc{};
    const float* T = F->Tcw;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Fc.R[3 * r + c] = T[4 * r + c];
        Fc.t[r] = T[4 * r + 3];
        // mOw = -mRcw.t() * mtcw as a cv::Mat product (double accumulation, one rounding)
        const double acc = (double)T[r] * T[3] + (double)T[4 + r] * T[7] + (double)T[8 + r] * T[11];
        Fc.Ow[r] = (float)(-1.0 * acc);
    }
    Fc.min_x = F->min_x;
    Fc.max_x = F->max_x;
    Fc.min_y = F->min_y;
    Fc.max_y = F->max_y;
    Fc.fx = F->fx;
    Fc.fy = F->fy;
    Fc.cx = F->cx;
    Fc.cy = F->cy;
    Fc.bf = F->bf;
    Fc.log_scale = F->log_scale;
    Fc.view_cos_limit = view_cos_limit;
    Fc.nlevels = F->nlevels;
    Fc.n = n_mp;
    slam_status st = run_projection(m, F, C, n_mp, nullptr, mp_desc, f_match, nmatches,
                                    [&](Blob& B, DevProjCall& c) {
                                        Fc.mps = B.put(mps, n_mp);
                                        Fc.track = B.take<slam_mp_track>(std::max(1, n_mp));
                                        Fc.n_in_view = B.take<int32_t>(1);
                                        (void)hipMemsetAsync(Fc.n_in_view, 0, 4, B.s);
                                        (void)launch_is_in_frustum(B.put(&Fc, 1), 1, n_mp, B.s);
                                        c.mps = Fc.track;
                                    });
    if (st != SLAM_OK) return st;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipMemcpy(n_to_match, Fc.n_in_view, 4, hipMemcpyDeviceToHost));
    if (track && n_mp) SLAM_HIP_TRY(hipMemcpy(track, Fc.track, sizeof(slam_mp_track) * n_mp, hipMemcpyDeviceToHost));
    return SLAM_OK;
}

namespace {
constexpr int kGridSortMax = 4096;  // frames above this many features keep the host-built grid
__global__ void k_frame_grid(const DevProjCall* __restrict__ calls);
slam_status staged_upload(int nframes, const std::vector<size_t>& off, uint8_t* host, uint8_t* dev, hipStream_t st,
                          int threads, const std::function<void(int)>& stage);
}  // namespace

// Batched Tracking::SearchLocalPoints: nframes independent (Frame, local map) problems.  Every
// frame's inputs are staged into one pinned host image on several host threads and uploaded in
// chunks as they complete; the Frame grids are built on the device (k_frame_grid); one
// isInFrustum launch (grid row per frame) and one SearchByProjection launch (workgroup per
// frame); every frame's results back with one copy.
extern "C" slam_status slamhot_search_local_points_batch(slam_matcher* m, int nframes, const slam_frame_view* frames,
                                                         const int32_t* n_mp, const slam_mp_geom* const* mps,
                                                         const uint8_t* const* mp_desc, float view_cos_limit,
                                                         float nnratio, float th, int far_points, float th_far,
                                                         int32_t* const* f_match, int32_t* n_to_match,
                                                         int32_t* nmatches) {
    if (!m || nframes < 0 || (nframes && (!frames || !n_mp || !mps || !mp_desc || !f_match || !n_to_match || !nmatches)))
        return SLAM_EINVAL;
    for (int f = 0; f < nframes; f++)
        if (!frame_ok(&frames[f]) || !frames[f].Tcw || n_mp[f] < 0 || (n_mp[f] && (!mps[f] || !mp_desc[f])) ||
            (frames[f].n && !f_match[f]))
            return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    constexpr int kStageThreads = 8;
    const int ncell = kGridCols * kGridRows;
    // host image: per frame kps | uright | desc | state | (host grid) | mps | mp_desc, the call
    // records; then device-only scratch (device grid, track, queries, cand_off, cand, gstate) and
    // the results (f_match, out, n_in_view)
    struct Off {
        size_t kps, ur, desc, st, cs, cf, mps, md, tr, q, co, cand, fm, out, niv, gs;
        int cand_cap;
        bool gstate, dgrid;
    };
    std::vector<Off> O(nframes);
    std::vector<std::vector<int32_t>> starts(nframes), feats(nframes);
    std::vector<size_t> frame_off(nframes + 1);
    size_t off = 0, lds = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    for (int f = 0; f < nframes; f++) {
        const slam_frame_view& F = frames[f];
        const int nq = n_mp[f];
        Off& o = O[f];
        o.dgrid = F.n <= kGridSortMax;
        if (!o.dgrid) build_grid_csr(&F, starts[f], feats[f]);
        frame_off[f] = off;
        o.kps = take(sizeof(slam_keypoint) * F.n);
        o.ur = take(F.uright ? 4 * (size_t)F.n : 0);
        o.desc = take(32 * (size_t)F.n);
        o.st = take(F.mp_state ? (size_t)F.n : 0);
        o.cs = o.dgrid ? 0 : take(4 * starts[f].size());
        o.cf = o.dgrid ? 0 : take(4 * feats[f].size());
        o.mps = take(sizeof(slam_mp_geom) * nq);
        o.md = take(32 * (size_t)nq);
    }
    const size_t calls_off = take(sizeof(DevProjCall) * nframes), fc_off = take(sizeof(FrustumCall) * nframes);
    frame_off[nframes] = calls_off;
    const size_t in_bytes = off;  // the host image: inputs and call records
    for (int f = 0; f < nframes; f++) {  // device-only scratch
        const int nq = n_mp[f];
        Off& o = O[f];
        if (o.dgrid) {
            o.cs = take(4 * (size_t)(ncell + 1));
            o.cf = take(4 * (size_t)std::max(1, frames[f].n));
        }
        o.tr = take(sizeof(slam_mp_track) * std::max(1, nq));
        o.q = take(sizeof(ProjQuery) * std::max(1, nq));
        o.co = take(4 * (size_t)(nq + 1));
        o.cand_cap = std::max(4096, nq * 64);
        o.cand = take(4 * (size_t)o.cand_cap);
        const size_t need = projection_lds_bytes(frames[f].n, nq);
        o.gstate = need == 0;
        o.gs = take(o.gstate ? 4 * (2 * (size_t)frames[f].n + 2 * (size_t)nq) : 0);
        if (!o.gstate) lds = std::max(lds, need);
    }
    // the outputs of every frame in one contiguous tail: one copy back
    const size_t res_off = off;
    for (int f = 0; f < nframes; f++) {
        O[f].fm = take(4 * (size_t)std::max(1, frames[f].n));
        O[f].out = take(16);
        O[f].niv = take(4);
    }
    const size_t total = off;
    std::unique_lock<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    slam_status st;
    if ((st = m->d_a.ensure(total))) return st;
    uint8_t* D = m->d_a.as<uint8_t>();
    // inputs and results through one pinned staging buffer: [inputs | results]
    if ((st = m->stage(in_bytes + (total - res_off)))) return st;
    uint8_t* H = m->h_stage;
    uint8_t* R = m->h_stage + in_bytes;
    hipStream_t S = m->stream;
    auto stage_frame = [&](int f) {
        const slam_frame_view& F = frames[f];
        const Off& o = O[f];
        const int nq = n_mp[f];
        auto put = [&](size_t at, const void* src, size_t bytes) {
            if (src && bytes) std::memcpy(H + at, src, bytes);
        };
        put(o.kps, F.kps_un, sizeof(slam_keypoint) * F.n);
        put(o.ur, F.uright, F.uright ? 4 * (size_t)F.n : 0);
        put(o.desc, F.desc, 32 * (size_t)F.n);
        put(o.st, F.mp_state, F.mp_state ? (size_t)F.n : 0);
        if (!o.dgrid) {
            put(o.cs, starts[f].data(), 4 * starts[f].size());
            put(o.cf, feats[f].data(), 4 * feats[f].size());
        }
        put(o.mps, mps[f], sizeof(slam_mp_geom) * nq);
        put(o.md, mp_desc[f], 32 * (size_t)nq);
        DevProjCall C{};
        fill_frame(C, &F);
        C.F.n = F.n;
        C.F.kps = (const slam_keypoint*)(D + o.kps);
        C.F.uright = F.uright ? (const float*)(D + o.ur) : nullptr;
        C.F.desc = D + o.desc;
        C.F.state = F.mp_state ? (const int8_t*)(D + o.st) : nullptr;
        C.F.cell_start = (const int32_t*)(D + o.cs);
        C.F.cell_feat = (const int32_t*)(D + o.cf);
        C.grid_on_device = o.dgrid;
        C.mode = kProjLocal;
        C.nq = nq;
        C.mps = (const slam_mp_track*)(D + o.tr);
        C.th = th;
        C.th_far = th_far;
        C.far_points = far_points;
        C.nnratio = nnratio;
        C.th_dist = 100;
        C.check_ori = 0;
        C.queries = (ProjQuery*)(D + o.q);
        C.qdesc = D + o.md;
        C.cand_off = (int32_t*)(D + o.co);
        C.cand = (uint32_t*)(D + o.cand);
        C.cand_cap = o.cand_cap;
        C.f_match = (int32_t*)(D + o.fm);
        C.out = (int32_t*)(D + o.out);
        C.gstate = o.gstate ? (int32_t*)(D + o.gs) : nullptr;
        std::memcpy(H + calls_off + sizeof(DevProjCall) * f, &C, sizeof(C));
        FrustumCall Fc{};
        const float* T = F.Tcw;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) Fc.R[3 * r + c] = T[4 * r + c];
            Fc.t[r] = T[4 * r + 3];
            const double acc = (double)T[r] * T[3] + (double)T[4 + r] * T[7] + (double)T[8 + r] * T[11];
            Fc.Ow[r] = (float)(-1.0 * acc);
        }
        Fc.min_x = F.min_x;
        Fc.max_x = F.max_x;
        Fc.min_y = F.min_y;
        Fc.max_y = F.max_y;
        Fc.fx = F.fx;
        Fc.fy = F.fy;
        Fc.cx = F.cx;
        Fc.cy = F.cy;
        Fc.bf = F.bf;
        Fc.log_scale = F.log_scale;
        Fc.view_cos_limit = view_cos_limit;
        Fc.nlevels = F.nlevels;
        Fc.n = nq;
        Fc.mps = (const slam_mp_geom*)(D + o.mps);
        Fc.track = (slam_mp_track*)(D + o.tr);
        Fc.n_in_view = (int32_t*)(D + o.niv);
        std::memcpy(H + fc_off + sizeof(FrustumCall) * f, &Fc, sizeof(Fc));
    };
    SLAM_HIP_TRY(hipEventRecord(m->ev[0], S));
    if ((st = staged_upload(nframes, frame_off, H, D, S, kStageThreads, stage_frame))) return st;
    int max_nq = 1;
    for (int f = 0; f < nframes; f++) max_nq = std::max(max_nq, n_mp[f]);
    SLAM_HIP_TRY(hipMemcpyAsync(D + calls_off, H + calls_off, in_bytes - calls_off, hipMemcpyHostToDevice, S));
    SLAM_HIP_TRY(hipMemsetAsync(D + res_off, 0, total - res_off, S));  // out[] and n_in_view start at 0
    SLAM_HIP_TRY(hipEventRecord(m->ev[1], S));
    hipLaunchKernelGGL(k_frame_grid, dim3(nframes), dim3(1024), 0, S, (const DevProjCall*)(D + calls_off));
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(launch_is_in_frustum((const FrustumCall*)(D + fc_off), nframes, max_nq, S));
    SLAM_HIP_TRY(launch_search_by_projection((const DevProjCall*)(D + calls_off), nframes, lds, S));
    SLAM_HIP_TRY(hipEventRecord(m->ev[2], S));
    // results: per frame f_match, out[4], n_in_view (one copy of the whole tail back)
    SLAM_HIP_TRY(hipMemcpyAsync(R, D + res_off, total - res_off, hipMemcpyDeviceToHost, S));
    SLAM_HIP_TRY(hipEventRecord(m->ev[3], S));
    SLAM_HIP_TRY(hipStreamSynchronize(S));
    m->batch_stats();
    std::vector<int> redo;
    for (int f = 0; f < nframes; f++) {
        const Off& o = O[f];
        const int32_t* out = (const int32_t*)(R + (o.out - res_off));
        if (out[1] == 1) {  // candidate overflow: this frame again through the single-call path
            redo.push_back(f);
            continue;
        }
        nmatches[f] = out[0];
        n_to_match[f] = *(const int32_t*)(R + (o.niv - res_off));
        if (frames[f].n) std::memcpy(f_match[f], R + (o.fm - res_off), 4 * (size_t)frames[f].n);
    }
    g.unlock();  // the single-call path takes the handle's lock itself
    slam_status rs = SLAM_OK;
    for (int f : redo) {
        int n = 0, ntm = 0;
        rs = slamhot_search_local_points(m, &frames[f], n_mp[f], mps[f], mp_desc[f], view_cos_limit, nnratio, th,
                                         far_points, th_far, nullptr, &ntm, f_match[f], &n);
        if (rs != SLAM_OK) break;
        nmatches[f] = n;
        n_to_match[f] = ntm;
    }
    return rs;
}

extern "C" slam_status slamhot_search_by_projection_last(slam_matcher* m, const slam_frame_view* F,
                                                         const slam_last_frame* LF, float nnratio, int check_ori,
                                                         float th, int mono, int32_t* f_match, int* nmatches) {
    if (!m || !frame_ok(F) || !F->Tcw || !last_ok(LF) || !f_match || !nmatches) return SLAM_EINVAL;
    DevProjCall C{};
    fill_frame(C, F);
    C.mode = kProjLast;
    C.th = th;
    C.mono = mono;
    C.nnratio = nnratio;
    C.th_dist = 100;
    C.check_ori = check_ori;
    for (int i = 0; i < 16; i++) C.LT[i] = LF->Tcw[i];
    return run_projection(m, F, C, LF->n, nullptr, LF->mp_desc, f_match, nmatches, [&](Blob& B, DevProjCall& c) {
        c.lf_kps = B.put(LF->kps, LF->n);
        c.lf_kps_un = B.put(LF->kps_un, LF->n);
        c.lf_has_mp = B.put(LF->has_mp, LF->n);
        c.lf_outlier = B.put(LF->outlier, LF->n);
        c.lf_pos = B.put(LF->mp_pos, (size_t)LF->n * 3);
        c.lf_has_obs = B.put(LF->mp_has_obs, LF->n);
    });
}

// The KeyFrame variant's per-MapPoint geometry (projection, distance gate and
// MapPoint::PredictScale with glibc logf, MapPoint.cc:551-566) runs here on the host, in
// the reference's arithmetic; candidate search and resolution run on the device.
namespace {
void kf_queries(const slam_frame_view* F, const slam_kf_points* KF, float th, ProjQuery* qs) {
    const float* T = F->Tcw;
    float Ow[3];
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[i] * T[3] + (double)T[4 + i] * T[7] + (double)T[8 + i] * T[11];
        Ow[i] = (float)(-1.0 * acc);
    }
    for (int i = 0; i < KF->n; i++) qs[i] = ProjQuery{};
    for (int i = 0; i < KF->n; i++) {
        ProjQuery& Q = qs[i];
        Q.valid = 0;
        Q.blocking = 1;
        Q.er = -1.f;
        Q.angle = KF->kps_un[i].angle;
        if (!KF->use[i]) continue;
        const float* X = KF->mp_pos + 3 * (size_t)i;
        float xc[3];
        for (int r = 0; r < 3; r++) {
            const double acc = (double)T[4 * r] * X[0] + (double)T[4 * r + 1] * X[1] + (double)T[4 * r + 2] * X[2];
            xc[r] = (float)(acc * 1.0 + (double)T[4 * r + 3] * 1.0);
        }
        const float u = F->fx * xc[0] / xc[2] + F->cx;
        const float v = F->fy * xc[1] / xc[2] + F->cy;
        if (u < F->min_x || u > F->max_x || v < F->min_y || v > F->max_y) continue;
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        const float dist3D = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist3D < 0.8f * KF->min_dist[i] || dist3D > 1.2f * KF->max_dist[i]) continue;
        const float ratio = KF->max_dist[i] / dist3D;
        int level = (int)std::ceil(std::log(ratio) / F->log_scale);
        if (level < 0) level = 0;
        else if (level >= F->nlevels) level = F->nlevels - 1;
        Q.valid = 1;
        Q.u = u;
        Q.v = v;
        Q.r = th * F->scale[level];
        Q.min_level = (int16_t)(level - 1);
        Q.max_level = (int16_t)(level + 1);
    }
}

// Bump layout over one pinned host image and its device copy: a sizing pass (host == nullptr)
// fixes every offset, the filling pass repeats the same puts with the buffers in place.
struct Stager {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t off = 0;
    template <class T>
    const T* put(const T* src, size_t count) {
        if (!src || !count) return nullptr;
        const size_t o = off;
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        if (host) std::memcpy(host + o, src, count * sizeof(T));
        return reinterpret_cast<const T*>(dev + o);
    }
    // a region the caller fills in place on the host (nullptr in the sizing pass); device address
    template <class T>
    T* fill(size_t count, T** host_at) {
        const size_t o = off;
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        *host_at = host && count ? reinterpret_cast<T*>(host + o) : nullptr;
        return count ? reinterpret_cast<T*>(dev + o) : nullptr;
    }
    template <class T>
    T* take(size_t count) {
        const size_t o = off;
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        return reinterpret_cast<T*>(dev + o);
    }
};

// Frame::AssignFeaturesToGrid (Frame.cc:380-411) + PosInGrid (:708-718) for the batched calls,
// workgroup per frame: (cell << 16 | index) keys sorted in LDS (the keys are unique, so the order
// inside a cell is the insertion order), cell starts by binary search.  Frames above
// kGridSortMax features keep the host-built grid.
__global__ void __launch_bounds__(1024) k_frame_grid(const DevProjCall* __restrict__ calls) {
    __shared__ uint32_t keys[kGridSortMax];
    const DevProjCall& C = calls[blockIdx.x];
    const int n = C.F.n;
    if (n > kGridSortMax || !C.grid_on_device) return;
    const float min_x = C.F.min_x, min_y = C.F.min_y, inv_w = C.F.inv_w, inv_h = C.F.inv_h;
    int npad = 1;
    while (npad < n) npad <<= 1;
    for (int i = threadIdx.x; i < npad; i += blockDim.x) {
        uint32_t k = 0xFFFFFFFFu;
        if (i < n) {
            const slam_keypoint kp = C.F.kps[i];
            const int px = (int)roundf((kp.x - min_x) * inv_w);
            const int py = (int)roundf((kp.y - min_y) * inv_h);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows)
                k = ((uint32_t)(px * kGridRows + py) << 16) | (uint32_t)i;
        }
        keys[i] = k;
    }
    __syncthreads();
    for (int kk = 2; kk <= npad; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < npad; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const uint32_t a = keys[i], b = keys[l];
                    if ((a > b) == ((i & kk) == 0)) {
                        keys[i] = b;
                        keys[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    int32_t* cs = const_cast<int32_t*>(C.F.cell_start);
    int32_t* cf = const_cast<int32_t*>(C.F.cell_feat);
    for (int c = threadIdx.x; c <= kGridCols * kGridRows; c += blockDim.x) {  // lower_bound(c << 16)
        int lo = 0, hi = npad;
        const uint32_t key = (uint32_t)c << 16;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (keys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        cs[c] = lo;
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (keys[i] != 0xFFFFFFFFu) cf[i] = (int32_t)(keys[i] & 0xFFFFu);
}


// Stage nframes frames into the pinned host image and upload them in chunks: host threads copy
// the frames in index order (frame f's bytes at [off[f], off[f + 1])), and the calling thread
// sends each chunk of frames to the device as soon as all its frames are in, while the threads
// fill the next one -- the staging copies and the PCIe transfer overlap instead of following one
// another.  Stream operations are issued from the calling thread only.
slam_status staged_upload(int nframes, const std::vector<size_t>& off, uint8_t* host, uint8_t* dev, hipStream_t st,
                          int threads, const std::function<void(int)>& stage) {
    if (nframes <= 0) return SLAM_OK;
    const int nchunk = std::max(1, std::min(nframes, 8));
    auto lo = [&](int c) { return (int)((long long)nframes * c / nchunk); };
    std::vector<int> chunk_of(nframes);
    for (int c = 0; c < nchunk; c++)
        for (int f = lo(c); f < lo(c + 1); f++) chunk_of[f] = c;
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[nchunk]);
    for (int c = 0; c < nchunk; c++) done[c].store(0);
    std::atomic<int> next{0};
    auto one = [&](int f) {
        stage(f);
        done[chunk_of[f]].fetch_add(1, std::memory_order_release);
    };
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nth = std::max(1, std::min({threads, hw, nframes / 8}));
    std::vector<std::thread> th;
    // helper threads take frames from the shared counter, so the calling thread finishes whatever
    // they do not: a thread that cannot be created only costs speed (the ones created are joined)
    try {
        th.reserve(nth);
        for (int t = 1; t < nth; t++)
            th.emplace_back([&] {
                for (int f; (f = next.fetch_add(1)) < nframes;) one(f);
            });
    } catch (...) {
    }
    int c = 0;
    hipError_t err = hipSuccess;
    auto flush = [&] {
        while (c < nchunk && done[c].load(std::memory_order_acquire) == lo(c + 1) - lo(c)) {
            const size_t a = off[lo(c)], b = off[lo(c + 1)];
            if (b > a && err == hipSuccess) err = hipMemcpyAsync(dev + a, host + a, b - a, hipMemcpyHostToDevice, st);
            c++;
        }
    };
    for (int f; (f = next.fetch_add(1)) < nframes;) {
        one(f);
        flush();
    }
    while (c < nchunk) {
        flush();
        if (c < nchunk) std::this_thread::yield();
    }
    for (auto& x : th) x.join();
    if (err != hipSuccess) {
        // copies queued before the failure may still read the pinned image: let them finish
        // before the caller (or its next call on this handle) reuses it
        (void)hipStreamSynchronize(st);
        return SLAM_EHIP;
    }
    return SLAM_OK;
}

// Batched SearchByProjection over nframes independent problems of one mode (last frame /
// KeyFrame): every frame's inputs and call record staged into one pinned host image (a sizing
// pass fixes every frame's offset, then the frames are copied in on several host threads) and
// uploaded with one copy; the Frame grids built on the device (k_frame_grid); one
// k_search_by_projection launch (a workgroup per frame); every frame's f_match / counters back
// with one copy.  `inputs(f, S, C)` puts the mode's per-frame inputs and returns the query count;
// a frame whose candidates overflow the preset capacity goes again through `single(f)`.
slam_status run_projection_batch(slam_matcher* m, int nframes, const slam_frame_view* frames, const DevProjCall& proto,
                                 const std::function<int(int, Stager&, DevProjCall&)>& inputs,
                                 int32_t* const* f_match, int32_t* nmatches,
                                 const std::function<slam_status(int, int*)>& single) {
    constexpr int kStageThreads = 8;
    const int ncell = kGridCols * kGridRows;
    std::vector<std::vector<int32_t>> starts(nframes), feats(nframes);
    for (int f = 0; f < nframes; f++)
        if (frames[f].n > kGridSortMax) build_grid_csr(&frames[f], starts[f], feats[f]);
    std::vector<DevProjCall> calls(nframes);
    std::vector<size_t> frame_off(nframes), fm_off(nframes), out_off(nframes);
    size_t in_bytes = 0, res_off = 0, total = 0, lds = 0, calls_off = 0;
    auto stage_frame = [&](int f, Stager& S) {
        const slam_frame_view& F = frames[f];
        DevProjCall C = proto;
        fill_frame(C, &F);
        C.F.n = F.n;
        C.F.kps = S.put(F.kps_un, F.n);
        C.F.uright = S.put(F.uright, F.n);
        C.F.desc = S.put(F.desc, (size_t)F.n * 32);
        C.F.state = S.put(F.mp_state, F.n);
        C.grid_on_device = F.n <= kGridSortMax;
        if (!C.grid_on_device) {
            C.F.cell_start = S.put(starts[f].data(), starts[f].size());
            C.F.cell_feat = S.put(feats[f].data(), feats[f].size());
        }
        C.nq = inputs(f, S, C);
        calls[f] = C;
    };
    auto scratch = [&](Stager& S) {  // device-only: grids, queries, candidates, results
        for (int f = 0; f < nframes; f++) {
            DevProjCall& C = calls[f];
            const int nq = C.nq;
            if (C.grid_on_device) {
                C.F.cell_start = S.take<int32_t>(ncell + 1);
                C.F.cell_feat = S.take<int32_t>(std::max(1, frames[f].n));
            }
            if (!C.queries) C.queries = S.take<ProjQuery>(std::max(1, nq));
            C.cand_off = S.take<int32_t>(nq + 1);
            C.cand_cap = std::max(4096, nq * 64);
            C.cand = S.take<uint32_t>(C.cand_cap);
            const size_t need = projection_lds_bytes(frames[f].n, nq);
            C.gstate = need ? nullptr : S.take<int32_t>(2 * (size_t)frames[f].n + 2 * (size_t)nq);
            if (need) lds = std::max(lds, need);
        }
        res_off = S.off;  // results of every frame in one tail: one copy back
        for (int f = 0; f < nframes; f++) {
            fm_off[f] = S.off;
            calls[f].f_match = S.take<int32_t>(std::max(1, frames[f].n));
            out_off[f] = S.off;
            calls[f].out = S.take<int32_t>(4);
        }
        total = S.off;
    };
    // sizing pass: offsets only
    {
        Stager S;
        for (int f = 0; f < nframes; f++) {
            frame_off[f] = S.off;
            stage_frame(f, S);
        }
        calls_off = S.off;
        S.off += (sizeof(DevProjCall) * nframes + 255) & ~(size_t)255;
        in_bytes = S.off;
        scratch(S);
    }
    std::unique_lock<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    {
        slam_status st;
        if ((st = m->d_a.ensure(total)) || (st = m->stage(in_bytes + (total - res_off)))) return st;
    }
    uint8_t* D = m->d_a.as<uint8_t>();
    hipStream_t st = m->stream;
    // filling pass: frames copied into the pinned image on several threads, uploaded in chunks
    // as they complete
    {
        std::vector<size_t> offs(frame_off);
        offs.push_back(calls_off);
        SLAM_HIP_TRY(hipEventRecord(m->ev[0], st));
        slam_status ss = staged_upload(nframes, offs, m->h_stage, D, st, kStageThreads, [&](int f) {
            Stager S;
            S.host = m->h_stage;
            S.dev = D;
            S.off = frame_off[f];
            stage_frame(f, S);
        });
        if (ss != SLAM_OK) return ss;
    }
    {
        Stager S;
        S.dev = D;
        S.off = in_bytes;
        scratch(S);
        std::memcpy(m->h_stage + calls_off, calls.data(), sizeof(DevProjCall) * nframes);
    }
    uint8_t* R = m->h_stage + in_bytes;
    SLAM_HIP_TRY(hipMemcpyAsync(D + calls_off, m->h_stage + calls_off, in_bytes - calls_off, hipMemcpyHostToDevice, st));
    SLAM_HIP_TRY(hipMemsetAsync(D + res_off, 0, total - res_off, st));
    SLAM_HIP_TRY(hipEventRecord(m->ev[1], st));
    hipLaunchKernelGGL(k_frame_grid, dim3(nframes), dim3(1024), 0, st, (const DevProjCall*)(D + calls_off));
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(launch_search_by_projection((const DevProjCall*)(D + calls_off), nframes, lds, st));
    SLAM_HIP_TRY(hipEventRecord(m->ev[2], st));
    SLAM_HIP_TRY(hipMemcpyAsync(R, D + res_off, total - res_off, hipMemcpyDeviceToHost, st));
    SLAM_HIP_TRY(hipEventRecord(m->ev[3], st));
    SLAM_HIP_TRY(hipStreamSynchronize(st));
    m->batch_stats();
    std::vector<int> redo;
    for (int f = 0; f < nframes; f++) {
        const int32_t* out = (const int32_t*)(R + (out_off[f] - res_off));
        if (out[1] == 1) {
            redo.push_back(f);
            continue;
        }
        nmatches[f] = out[0];
        if (frames[f].n) std::memcpy(f_match[f], R + (fm_off[f] - res_off), 4 * (size_t)frames[f].n);
    }
    g.unlock();  // the single-call path takes the handle's lock itself
    slam_status rs = SLAM_OK;
    for (int f : redo) {
        int n = 0;
        if ((rs = single(f, &n)) != SLAM_OK) break;
        nmatches[f] = n;
    }
    return rs;
}
}  // namespace

extern "C" slam_status slamhot_search_by_projection_kf(slam_matcher* m, const slam_frame_view* F,
                                                       const slam_kf_points* KF, float nnratio, int check_ori,
                                                       float th, int orb_dist, int32_t* f_match, int* nmatches) {
    if (!m || !frame_ok(F) || !F->Tcw || !kf_ok(KF) || !f_match || !nmatches) return SLAM_EINVAL;
    (void)nnratio;
    std::vector<ProjQuery> qs(KF->n);
    kf_queries(F, KF, th, qs.data());
    DevProjCall C{};
    fill_frame(C, F);
    C.mode = kProjKF;
    C.th_dist = orb_dist;
    C.check_ori = check_ori;
    return run_projection(m, F, C, KF->n, &qs, KF->mp_desc, f_match, nmatches, [](Blob&, DevProjCall&) {});
}

extern "C" slam_status slamhot_search_by_projection_last_batch(slam_matcher* m, int nframes,
                                                               const slam_frame_view* frames,
                                                               const slam_last_frame* last, float nnratio,
                                                               int check_ori, float th, int mono,
                                                               int32_t* const* f_match, int32_t* nmatches) {
    if (!m || nframes < 0 || (nframes && (!frames || !last || !f_match || !nmatches))) return SLAM_EINVAL;
    for (int f = 0; f < nframes; f++)
        if (!frame_ok(&frames[f]) || !frames[f].Tcw || !last_ok(&last[f]) || (frames[f].n && !f_match[f]))
            return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    DevProjCall proto{};
    proto.mode = kProjLast;
    proto.th = th;
    proto.mono = mono;
    proto.nnratio = nnratio;
    proto.th_dist = 100;
    proto.check_ori = check_ori;
    return run_projection_batch(
        m, nframes, frames, proto,
        [&](int f, Stager& S, DevProjCall& c) {
            const slam_last_frame& LF = last[f];
            for (int i = 0; i < 16; i++) c.LT[i] = LF.Tcw[i];
            c.lf_kps = S.put(LF.kps, LF.n);
            c.lf_kps_un = S.put(LF.kps_un, LF.n);
            c.lf_has_mp = S.put(LF.has_mp, LF.n);
            c.lf_outlier = S.put(LF.outlier, LF.n);
            c.lf_pos = S.put(LF.mp_pos, (size_t)LF.n * 3);
            c.lf_has_obs = S.put(LF.mp_has_obs, LF.n);
            c.qdesc = S.put(LF.mp_desc, (size_t)LF.n * 32);
            c.queries = nullptr;
            return LF.n;
        },
        f_match, nmatches,
        [&](int f, int* n) {
            return slamhot_search_by_projection_last(m, &frames[f], &last[f], nnratio, check_ori, th, mono, f_match[f], n);
        });
}

extern "C" slam_status slamhot_search_by_projection_kf_batch(slam_matcher* m, int nframes, const slam_frame_view* frames,
                                                             const slam_kf_points* kfs, float nnratio, int check_ori,
                                                             float th, int orb_dist, int32_t* const* f_match,
                                                             int32_t* nmatches) {
    if (!m || nframes < 0 || (nframes && (!frames || !kfs || !f_match || !nmatches))) return SLAM_EINVAL;
    for (int f = 0; f < nframes; f++)
        if (!frame_ok(&frames[f]) || !frames[f].Tcw || !kf_ok(&kfs[f]) || (frames[f].n && !f_match[f]))
            return SLAM_EINVAL;
    if (nframes == 0) return SLAM_OK;
    DevProjCall proto{};
    proto.mode = kProjKF;
    proto.th_dist = orb_dist;
    proto.check_ori = check_ori;
    // the per-MapPoint queries (the reference's host arithmetic) are computed straight into the
    // pinned image by the staging threads, overlapping the uploads of earlier frames
    return run_projection_batch(
        m, nframes, frames, proto,
        [&](int f, Stager& S, DevProjCall& c) {
            ProjQuery* hq = nullptr;
            c.queries = S.fill<ProjQuery>(kfs[f].n, &hq);
            if (hq) kf_queries(&frames[f], &kfs[f], th, hq);
            c.qdesc = S.put(kfs[f].mp_desc, (size_t)kfs[f].n * 32);
            return kfs[f].n;
        },
        f_match, nmatches,
        [&](int f, int* n) {
            return slamhot_search_by_projection_kf(m, &frames[f], &kfs[f], nnratio, check_ori, th, orb_dist, f_match[f], n);
        });
}
