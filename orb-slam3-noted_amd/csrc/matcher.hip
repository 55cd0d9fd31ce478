// matcher.hip — MI355X (gfx950) DBoW2 vocabulary descent and ORBmatcher::SearchByBoW.
//
//   k_vocab_transform  TemplatedVocabulary::transform (TemplatedVocabulary.h:1229-1271):
//                      16 lanes per descriptor; at each level lane j scores child j (two
//                      16-byte loads + 8 popcounts), (distance, child position) wave-min.
//   k_bow_match        SearchByBoW (ORBmatcher.cc:269-471 and 823-963): one workgroup per
//                      (A, B) pair.  Common FeatureVector nodes are independent (every
//                      feature lives in exactly one node), so waves take nodes round-robin;
//                      inside a node the reference's greedy order over A features is kept
//                      (sequential), each step a wave-wide (min, second-min) over the node's
//                      B candidates held in registers.  Rotation histogram +
//                      ComputeThreeMaxima (:2515-2556) close the pair in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "common.hpp"

namespace slamhot {

// ----------------------------------------------------------------------------- vocab
struct DevVocab {
    const uint8_t* desc;        // n_nodes x 32
    const int32_t* child_ptr;   // n_nodes + 1
    const int32_t* child_idx;
    const uint8_t* is_leaf;
    const int32_t* word;        // word id per node (-1 for inner nodes)
    const double* weight;
    int L;
};

__device__ __forceinline__ int hamming32(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ void __launch_bounds__(256) k_vocab_transform(DevVocab V, int n, const uint8_t* desc,
                                                         int desc_stride, int levelsup,
                                                         int32_t* word_id, double* weight,
                                                         int32_t* node_id) {
    const int g = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;  // feature
    const int j = threadIdx.x & 15;                                // child slot
    const bool live = g < n;
    const int gi = live ? g : 0;
    const uint4* f = reinterpret_cast<const uint4*>(desc + (size_t)gi * desc_stride);
    const uint4 f0 = f[0], f1 = f[1];
    const int nid_level = V.L - levelsup;
    int final_id = 0, level = 0, nid = 0;
    bool leaf = false;
    // every lane of a 16-lane group follows the same path; bounded by the tree depth
    for (int it = 0; it < 64 && !leaf; it++) {
        ++level;
        const int c0 = V.child_ptr[final_id], c1 = V.child_ptr[final_id + 1];
        uint32_t bestkey = 0xFFFFFFFFu;
        for (int cb = c0; cb < c1; cb += 16) {
            const int c = cb + j;
            uint32_t key = 0xFFFFFFFFu;
            if (c < c1) {
                const int id = V.child_idx[c];
                const uint4* d = reinterpret_cast<const uint4*>(V.desc + (size_t)id * 32);
                key = ((uint32_t)hamming32(f0, f1, d[0], d[1]) << 20) | (uint32_t)(c - c0);
            }
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, o, 16));
            bestkey = min(bestkey, key);
        }
        if (bestkey == 0xFFFFFFFFu) break;  // malformed tree (inner node without children)
        final_id = V.child_idx[c0 + (int)(bestkey & 0xFFFFF)];
        if (level == nid_level) nid = final_id;
        leaf = V.is_leaf[final_id] != 0;
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
};

constexpr int kBowCap = 8192;        // features per side held in LDS
constexpr int kBowNodeChunks = 4;    // B candidates per node held in registers: 4 x 64

__device__ __forceinline__ int rot_bin(float a, float b) {
    // ORBmatcher.cc:391-396: float difference, +360 if negative, std::round(rot * (1/30))
    float rot = a - b;
    if (rot < 0.0f) rot += 360.0f;
    const float factor = 1.0f / 30;
    int bin = (int)roundf(rot * factor);
    if (bin == 30) bin = 0;
    return bin;
}

__global__ void __launch_bounds__(256) k_bow_match(const DevBowPair* pairs, float nnratio,
                                                   int check_ori, int strict) {
    __shared__ int16_t matchA[kBowCap];   // B index matched by A feature, -1 none
    __shared__ int8_t binA[kBowCap];
    __shared__ int16_t common[2 * 4096];  // (ia, ib) of common nodes
    __shared__ int hist[32];
    __shared__ int s_ncommon, s_keep[3], s_count;
    const DevBowPair pr = pairs[blockIdx.x];
    const DevBowSide& A = pr.A;
    const DevBowSide& B = pr.B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    for (int i = tid; i < A.n; i += blockDim.x) {
        matchA[i] = -1;
        binA[i] = -1;
    }
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) s_ncommon = 0;
    __syncthreads();
    // common node ids (merge-join of two ascending lists)
    for (int ia = tid; ia < A.n_nodes; ia += blockDim.x) {
        const uint32_t id = A.node_id[ia];
        int lo = 0, hi = B.n_nodes;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.node_id[mid] < id) lo = mid + 1; else hi = mid;
        }
        if (lo < B.n_nodes && B.node_id[lo] == id) {
            const int k = atomicAdd(&s_ncommon, 1);
            if (k < 4096) {
                common[2 * k] = (int16_t)ia;
                common[2 * k + 1] = (int16_t)lo;
            }
        }
    }
    __syncthreads();
    const int ncommon = min(s_ncommon, 4096);
    for (int c = wave; c < ncommon; c += nwaves) {
        const int ia = common[2 * c], ib = common[2 * c + 1];
        const int a0 = A.node_off[ia], a1 = A.node_off[ia + 1];
        const int b0 = B.node_off[ib], b1 = B.node_off[ib + 1];
        const int nbn = min(b1 - b0, 64 * kBowNodeChunks);
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
        for (int pa = a0; pa < a1; pa++) {
            const int idxA = (int)A.node_feat[pa];
            if (A.valid && !A.valid[idxA]) continue;
            const uint4* da = reinterpret_cast<const uint4*>(A.desc + (size_t)idxA * 32);
            const uint4 q0 = da[0], q1 = da[1];
            int dist[kBowNodeChunks];
            uint32_t bestkey = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < kBowNodeChunks; k++) {
                dist[k] = bok[k] ? hamming32(q0, q1, bd0[k], bd1[k]) : 1024;
                const uint32_t key = bok[k] ? (((uint32_t)dist[k] << 16) | (uint32_t)(64 * k + lane)) : 0xFFFFFFFFu;
                bestkey = min(bestkey, key);
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) bestkey = min(bestkey, (uint32_t)__shfl_xor((int)bestkey, o, 64));
            const int best1 = bestkey == 0xFFFFFFFFu ? 256 : (int)(bestkey >> 16);
            const int bpos = (int)(bestkey & 0xFFFF);
            int sec = 256;
#pragma unroll
            for (int k = 0; k < kBowNodeChunks; k++)
                if (bok[k] && (64 * k + lane) != bpos) sec = min(sec, dist[k]);
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) sec = min(sec, __shfl_xor(sec, o, 64));
            const bool pass = (strict ? best1 < 50 : best1 <= 50) && ((float)best1 < nnratio * (float)sec);
            if (pass) {
                // the owner lane marks its candidate taken and records the match
#pragma unroll
                for (int k = 0; k < kBowNodeChunks; k++) {
                    if (64 * k + lane == bpos) {
                        bok[k] = false;
                        matchA[idxA] = (int16_t)bidx[k];
                        if (check_ori)
                            binA[idxA] = (int8_t)rot_bin(A.angle[(size_t)idxA * A.angle_stride],
                                                         B.angle[(size_t)bidx[k] * B.angle_stride]);
                    }
                }
            }
        }
    }
    __syncthreads();
    if (check_ori) {
        for (int i = tid; i < A.n; i += blockDim.x)
            if (matchA[i] >= 0) atomicAdd(&hist[binA[i]], 1);
        __syncthreads();
        if (tid == 0) {
            // ComputeThreeMaxima (ORBmatcher.cc:2515-2556)
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
            s_keep[0] = ind1;
            s_keep[1] = ind2;
            s_keep[2] = ind3;
        }
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

}  // namespace slamhot

// =======================================================================================
// Host side
// =======================================================================================
using namespace slamhot;

namespace {

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
    Buf d_desc, d_child_ptr, d_child_idx, d_leaf, d_word, d_weight;
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
        V.L = L;
        return V;
    }
};

struct slam_matcher {
    int device = 0;
    hipStream_t stream = nullptr;
    Buf d_pair, d_a, d_b, d_out;
    std::mutex mu;
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
    slam_vocab* v = new slam_vocab();
    v->device = device;
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
        (st = v->d_word.ensure((size_t)n_nodes * 4)) || (st = v->d_weight.ensure((size_t)n_nodes * 8)))
        return fail(st);
    if (hipMemcpy(v->d_desc.p, desc, (size_t)n_nodes * 32, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_ptr.p, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_child_idx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_leaf.p, leaf.data(), n_nodes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_word.p, word.data(), (size_t)n_nodes * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(v->d_weight.p, weight, (size_t)n_nodes * 8, hipMemcpyHostToDevice) != hipSuccess)
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
                   &v->d_in, &v->d_word_out, &v->d_weight_out, &v->d_node_out};
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
    const int blocks = (int)(((size_t)n * 16 + 255) / 256);
    hipLaunchKernelGGL(k_vocab_transform, dim3(blocks), dim3(256), 0, s, v->dev(), n, (const uint8_t*)d_desc,
                       desc_stride, levelsup, (int32_t*)d_word_id, (double*)d_weight, (int32_t*)d_node_id);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

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
    *out = m;
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
    if (!S || S->n < 0 || S->n > kBowCap || S->n_nodes < 0 || S->n_nodes > 4096) return false;
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
    // every node of B must be representable in the register tile of k_bow_match
    for (int i = 0; i < B->n_nodes; i++)
        if (B->node_off[i + 1] - B->node_off[i] > 64 * kBowNodeChunks) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    slam_status st;
    const size_t ba = bow_side_bytes(A), bb = bow_side_bytes(B);
    const size_t nout = ((size_t)A->n + B->n + 1) * 4;
    if ((st = m->d_a.ensure(ba)) || (st = m->d_b.ensure(bb)) || (st = m->d_out.ensure(nout)) ||
        (st = m->d_pair.ensure(sizeof(DevBowPair))))
        return st;
    DevBowPair pr{};
    if ((st = upload_bow_side(A, m->d_a.as<uint8_t>(), pr.A, m->stream)) ||
        (st = upload_bow_side(B, m->d_b.as<uint8_t>(), pr.B, m->stream)))
        return st;
    pr.a2b = m->d_out.as<int32_t>();
    pr.b2a = pr.a2b + A->n;
    pr.nmatches = pr.b2a + B->n;
    SLAM_HIP_TRY(hipMemcpyAsync(m->d_pair.p, &pr, sizeof(pr), hipMemcpyHostToDevice, m->stream));
    hipLaunchKernelGGL(k_bow_match, dim3(1), dim3(256), 0, m->stream, m->d_pair.as<DevBowPair>(), nnratio,
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
