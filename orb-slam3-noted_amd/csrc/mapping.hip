// mapping.hip — MI355X (gfx950) LocalMapping matchers.
//
//   k_distinctive   MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:349-423): one wave
//                   per MapPoint.  Lane i owns descriptor i (rows i, i+64, ...); its median
//                   distance vDists[(N-1)/2] is found by a 9-step binary search over the
//                   distance range [0, 256] (count of d(i, j) <= v), so no N x N table is
//                   stored; (median, i) wave-min picks the first least median.
//   k_triangulation ORBmatcher::SearchForTriangulation_ (ORBmatcher.cc:1208-1433): one
//                   workgroup per KeyFrame pair, one thread per KF1 feature of its
//                   FeatureVector.  This fork never sets vbMatched2, so every KF1 feature's
//                   search is independent: scan its node's KF2 list in order keeping the LAST
//                   epipolar-consistent candidate of least distance (<= TH_LOW, `dist >
//                   bestDist` rejects only larger ones), then the rotation histogram.
//   k_fuse_search   ORBmatcher::Fuse (ORBmatcher.cc:1629-1818) search half, one thread per
//                   MapPoint: cv::Mat products as double accumulation rounded once (as the
//                   projection matchers), PredictScale with the correctly rounded logf, the
//                   KeyFrame grid walked in the reference's order (ix outer, iy inner, cell
//                   insertion order), chi2 gates 7.8 / 5.99, first least Hamming distance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "common.hpp"
#include "gate_fp.hpp"

namespace slamhot {
namespace {

constexpr int kDistThreads = 256;

__device__ __forceinline__ int ham(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ void __launch_bounds__(kDistThreads) k_distinctive(int n_mp, const int32_t* off, const uint8_t* desc,
                                                              int32_t* best) {
    const int mpi = blockIdx.x * (kDistThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int lane = threadIdx.x & 63;
    if (mpi >= n_mp) return;
    const int o = off[mpi];
    const int N = off[mpi + 1] - o;
    if (N <= 0) {
        if (lane == 0) best[mpi] = -1;
        return;
    }
    const uint4* D = reinterpret_cast<const uint4*>(desc + (size_t)o * 32);
    const int k = (N - 1) / 2;  // vDists[0.5*(N-1)]: the double index truncates
    uint32_t key = 0xFFFFFFFFu;
    for (int i = lane; i < N; i += 64) {
        const uint4 a0 = D[2 * i], a1 = D[2 * i + 1];
        // smallest v with #{j : d(i, j) <= v} > k  (d(i, i) = 0 counts, as Distances[i][i])
        int lo = 0, hi = 256;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int c = 0;
            for (int j = 0; j < N; j++) c += ham(a0, a1, D[2 * j], D[2 * j + 1]) <= mid;
            if (c > k) hi = mid;
            else lo = mid + 1;
        }
        key = min(key, ((uint32_t)lo << 16) | (uint32_t)i);
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, s, 64));
    if (lane == 0) best[mpi] = (int32_t)(key & 0xFFFFu);
}

struct TriKF {
    int n, n_nodes, nlevels;
    const slam_keypoint* kps;
    const float* uright;
    const uint8_t* desc;
    const uint8_t* has_mp;
    const int32_t* node_id;
    const int32_t* node_off;
    const int32_t* node_feat;
    float scale[16], sigma2[16];
    float R[9], t[3], Ow[3], cam[4];
};

constexpr int kTriThreads = 256;
constexpr int kHisto = 30;

__device__ __forceinline__ int rot_bin(float a, float b) {  // ORBmatcher.cc:1390-1396
    float rot = a - b;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

__global__ void __launch_bounds__(kTriThreads) k_triangulation(const TriKF* kfs, const slam_tri_pair* pairs,
                                                              int check_ori, int cap, int32_t* match12,
                                                              int32_t* nmatches) {
    __shared__ int hist[kHisto];
    __shared__ int nm;
    __shared__ int keep[3];
    __shared__ gate::TriGeom G;
    const slam_tri_pair P = pairs[blockIdx.x];
    const TriKF& A = kfs[P.kf1];
    const TriKF& B = kfs[P.kf2];
    int32_t* M = match12 + (size_t)blockIdx.x * cap;
    const int t = threadIdx.x;
    if (t < kHisto) hist[t] = 0;
    if (t == 0) {
        nm = 0;
        // epipole, R12, t12 and epipolarConstrain_'s F12 as compiled (ORBmatcher.cc.o @0x12880,
        // @0x14880; Pinhole.cpp.o @0x70f0)
        G = gate::tri_geometry(A.R, A.t, A.Ow, A.cam, B.R, B.t, B.cam);
    }
    for (int i = t; i < cap; i += kTriThreads) M[i] = -1;
    __syncthreads();
    const int total = A.n_nodes ? A.node_off[A.n_nodes] : 0;
    for (int f = t; f < total; f += kTriThreads) {
        // node of this entry (largest j with node_off[j] <= f)
        int lo = 0, hi = A.n_nodes - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (A.node_off[mid] <= f) lo = mid;
            else hi = mid - 1;
        }
        const int nid = A.node_id[lo];
        int l2 = 0, h2 = B.n_nodes - 1, j2 = -1;
        while (l2 <= h2) {
            const int mid = (l2 + h2) >> 1;
            const int v = B.node_id[mid];
            if (v == nid) {
                j2 = mid;
                break;
            }
            if (v < nid) l2 = mid + 1;
            else h2 = mid - 1;
        }
        if (j2 < 0) continue;
        const int idx1 = A.node_feat[f];
        if (A.has_mp[idx1]) continue;
        const bool bStereo1 = A.uright && A.uright[idx1] >= 0;
        if (P.only_stereo && !bStereo1) continue;
        const slam_keypoint kp1 = A.kps[idx1];
        const uint4* d1 = reinterpret_cast<const uint4*>(A.desc + (size_t)idx1 * 32);
        const uint4 a0 = d1[0], a1 = d1[1];
        int bestDist = 50, bestIdx2 = -1;  // TH_LOW
        for (int c = B.node_off[j2]; c < B.node_off[j2 + 1]; c++) {
            const int idx2 = B.node_feat[c];
            if (B.has_mp[idx2]) continue;  // vbMatched2 is never set in this fork
            const bool bStereo2 = B.uright && B.uright[idx2] >= 0;
            if (P.only_stereo && !bStereo2) continue;
            const uint4* d2 = reinterpret_cast<const uint4*>(B.desc + (size_t)idx2 * 32);
            const int dist = ham(a0, a1, d2[0], d2[1]);
            if (dist > 50 || dist > bestDist) continue;
            const slam_keypoint kp2 = B.kps[idx2];
            if (!bStereo1 && !bStereo2 && gate::near_epipole(G.ep, kp2.x, kp2.y, B.scale[kp2.octave])) continue;
            if (gate::epipolar_ok(G.F, kp1.x, kp1.y, kp2.x, kp2.y, B.sigma2[kp2.octave]) || P.coarse) {
                bestIdx2 = idx2;
                bestDist = dist;
            }
        }
        if (bestIdx2 >= 0) {
            M[idx1] = bestIdx2;
            atomicAdd(&nm, 1);
            if (check_ori) atomicAdd(&hist[rot_bin(kp1.angle, B.kps[bestIdx2].angle)], 1);
        }
    }
    __syncthreads();
    if (check_ori) {
        if (t == 0) {  // ComputeThreeMaxima (ORBmatcher.cc:2515-2556)
            int max1 = 0, max2 = 0, max3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int i = 0; i < kHisto; i++) {
                const int s = hist[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    i3 = i2; i2 = i1; i1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    i3 = i2; i2 = i;
                } else if (s > max3) {
                    max3 = s;
                    i3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                i2 = -1;
                i3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                i3 = -1;
            }
            keep[0] = i1;
            keep[1] = i2;
            keep[2] = i3;
        }
        __syncthreads();
        for (int i = t; i < A.n; i += kTriThreads) {
            const int j = M[i];
            if (j < 0) continue;
            const int bin = rot_bin(A.kps[i].angle, B.kps[j].angle);
            if (bin != keep[0] && bin != keep[1] && bin != keep[2]) {
                M[i] = -1;
                atomicSub(&nm, 1);
            }
        }
        __syncthreads();
    }
    if (t == 0) nmatches[blockIdx.x] = nm;
}

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:42-43)
constexpr int kFuseThreads = 128;

struct FuseKF {
    float T[12];  // Rcw | tcw row-major
    float Ow[3];
    float fx, fy, cx, cy, bf;
    float min_x, min_y, max_x, max_y, inv_w, inv_h;
    float log_scale;
    int nlevels, n;
    float scale[16], inv_sigma2[16];
    const slam_keypoint* kps;
    const float* uright;
    const uint8_t* desc;
    const int32_t* cell_start;  // kGridCols * kGridRows + 1, cells [ix][iy]
    const int32_t* cell_feat;
};

__global__ void __launch_bounds__(kFuseThreads) k_fuse_search(FuseKF K, int n_mp, const slam_mp_geom* mps,
                                                              const uint8_t* mp_desc, float th, int32_t* best_idx,
                                                              int32_t* best_dist) {
    const int i = blockIdx.x * kFuseThreads + threadIdx.x;
    if (i >= n_mp) return;
    const slam_mp_geom g = mps[i];
    int bestDist = 256, bestIdx = -1;
    do {
        if (g.is_bad || g.seen) break;  // isBad(), IsInKeyFrame(pKF)
        float p3Dc[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double acc = (double)K.T[4 * r] * (double)g.pos[0] + (double)K.T[4 * r + 1] * (double)g.pos[1] +
                               (double)K.T[4 * r + 2] * (double)g.pos[2];
            p3Dc[r] = (float)(acc * 1.0 + (double)K.T[4 * r + 3] * 1.0);
        }
        if (p3Dc[2] < 0.0f) break;
        const float invz = 1 / p3Dc[2];
        const float u = K.fx * p3Dc[0] / p3Dc[2] + K.cx;  // Pinhole::project
        const float v = K.fy * p3Dc[1] / p3Dc[2] + K.cy;
        if (!(u >= K.min_x && u < K.max_x && v >= K.min_y && v < K.max_y)) break;  // KeyFrame::IsInImage
        const float ur = gate::right_u(u, K.bf, invz);  // ORBmatcher.cc.o Fuse @0x1be1
        const float maxDistance = 1.2f * g.max_dist;
        const float minDistance = 0.8f * g.min_dist;
        const float PO[3] = {g.pos[0] - K.Ow[0], g.pos[1] - K.Ow[1], g.pos[2] - K.Ow[2]};
        const float dist3D = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist3D < minDistance || dist3D > maxDistance) break;
        const double dot = (double)PO[0] * g.normal[0] + (double)PO[1] * g.normal[1] + (double)PO[2] * g.normal[2];
        if (dot < 0.5 * dist3D) break;
        const float ratio = g.max_dist / dist3D;
        int level = (int)ceilf((float)log((double)ratio) / K.log_scale);
        if (level < 0) level = 0;
        else if (level >= K.nlevels) level = K.nlevels - 1;
        const float radius = th * K.scale[level];
        // KeyFrame::GetFeaturesInArea (KeyFrame.cc:737-781)
        const int nMinCellX = max(0, (int)floorf((u - K.min_x - radius) * K.inv_w));
        if (nMinCellX >= kGridCols) break;
        const int nMaxCellX = min(kGridCols - 1, (int)ceilf((u - K.min_x + radius) * K.inv_w));
        if (nMaxCellX < 0) break;
        const int nMinCellY = max(0, (int)floorf((v - K.min_y - radius) * K.inv_h));
        if (nMinCellY >= kGridRows) break;
        const int nMaxCellY = min(kGridRows - 1, (int)ceilf((v - K.min_y + radius) * K.inv_h));
        if (nMaxCellY < 0) break;
        const uint4* dm = reinterpret_cast<const uint4*>(mp_desc + (size_t)i * 32);
        const uint4 a0 = dm[0], a1 = dm[1];
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const int c = ix * kGridRows + iy;
                for (int e = K.cell_start[c]; e < K.cell_start[c + 1]; e++) {
                    const int idx = K.cell_feat[e];
                    const slam_keypoint kp = K.kps[idx];
                    if (!(fabsf(kp.x - u) < radius && fabsf(kp.y - v) < radius)) continue;
                    const int kpLevel = kp.octave;
                    if (kpLevel < level - 1 || kpLevel > level) continue;
                    const float kpr = K.uright ? K.uright[idx] : -1.0f;
                    if (kpr >= 0) {
                        const float ex = u - kp.x, ey = v - kp.y, er = ur - kpr;
                        const float e2 = fmaf(er, er, fmaf(ex, ex, ey * ey));  // Fuse @0x1c98, @0x1cb5
                        if ((double)(e2 * K.inv_sigma2[kpLevel]) > 7.8) continue;
                    } else {
                        const float ex = u - kp.x, ey = v - kp.y;
                        const float e2 = fmaf(ex, ex, ey * ey);
                        if ((double)(e2 * K.inv_sigma2[kpLevel]) > 5.99) continue;
                    }
                    const uint4* dk = reinterpret_cast<const uint4*>(K.desc + (size_t)idx * 32);
                    const int dist = ham(a0, a1, dk[0], dk[1]);
                    if (dist < bestDist) {
                        bestDist = dist;
                        bestIdx = idx;
                    }
                }
            }
    } while (false);
    best_idx[i] = bestIdx;
    best_dist[i] = bestDist;
}

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    slam_status ensure(size_t n) {
        if (n <= cap) return SLAM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, std::max<size_t>(n, 256)) != hipSuccess) return SLAM_ENOMEM;
        cap = std::max<size_t>(n, 256);
        return SLAM_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

}  // namespace
}  // namespace slamhot

using namespace slamhot;

struct slam_mapper {
    int device = 0;
    hipStream_t stream = nullptr;
    DBuf d_in, d_out;
    std::mutex mu;
};

extern "C" {

slam_status slamhot_mapper_create(int device, slam_mapper** out) {
    if (!out) return SLAM_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SLAM_ENODEV;
    if (device < 0 || device >= n) return SLAM_EINVAL;
    slam_mapper* m = new (std::nothrow) slam_mapper();
    if (!m) return SLAM_ENOMEM;
    m->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
        delete m;
        return SLAM_EHIP;
    }
    *out = m;
    return SLAM_OK;
}

void slamhot_mapper_destroy(slam_mapper* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    m->d_in.release();
    m->d_out.release();
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

slam_status slamhot_distinctive_descriptors(slam_mapper* m, int n_mp, const int32_t* off, const uint8_t* desc,
                                            int32_t* best) {
    if (!m || n_mp < 0 || (n_mp && (!off || !best))) return SLAM_EINVAL;
    if (n_mp == 0) return SLAM_OK;
    const int total = off[n_mp];
    if (off[0] != 0 || total < 0 || (total && !desc)) return SLAM_EINVAL;
    for (int i = 0; i < n_mp; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > 65535) return SLAM_EINVAL;
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    const size_t off_b = ((size_t)(n_mp + 1) * 4 + 255) & ~(size_t)255;
    slam_status st;
    if ((st = m->d_in.ensure(off_b + (size_t)total * 32)) || (st = m->d_out.ensure((size_t)n_mp * 4))) return st;
    uint8_t* din = m->d_in.as<uint8_t>();
    SLAM_HIP_TRY(hipMemcpyAsync(din, off, (size_t)(n_mp + 1) * 4, hipMemcpyHostToDevice, m->stream));
    if (total) SLAM_HIP_TRY(hipMemcpyAsync(din + off_b, desc, (size_t)total * 32, hipMemcpyHostToDevice, m->stream));
    const int per = kDistThreads / 64;
    hipLaunchKernelGGL(k_distinctive, dim3((n_mp + per - 1) / per), dim3(kDistThreads), 0, m->stream, n_mp,
                       (const int32_t*)din, (const uint8_t*)(din + off_b), m->d_out.as<int32_t>());
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(best, m->d_out.p, (size_t)n_mp * 4, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(m->stream));
    return SLAM_OK;
}


slam_status slamhot_search_for_triangulation(slam_mapper* m, int n_kfs, const slam_tri_kf* kfs, int n_pairs,
                                             const slam_tri_pair* pairs, int check_ori, int cap,
                                             int32_t* match12, int32_t* nmatches) {
    if (!m || n_kfs < 0 || n_pairs < 0 || (n_pairs && (!kfs || !pairs || !match12 || !nmatches)) || cap < 0)
        return SLAM_EINVAL;
    if (n_pairs == 0) return SLAM_OK;
    for (int k = 0; k < n_kfs; k++) {
        const slam_tri_kf& K = kfs[k];
        if (K.n < 0 || K.n_nodes < 0 || K.nlevels < 1 || K.nlevels > 16 || !K.scale || !K.level_sigma2) return SLAM_EINVAL;
        if (K.n && (!K.kps_un || !K.desc || !K.has_mp)) return SLAM_EINVAL;
        if (K.n_nodes && (!K.node_id || !K.node_off || !K.node_feat)) return SLAM_EINVAL;
        if (K.n_nodes && (K.node_off[0] != 0 || K.node_off[K.n_nodes] < 0)) return SLAM_EINVAL;
        for (int j = 0; j < K.n_nodes; j++)
            if (K.node_off[j + 1] < K.node_off[j] || (j && K.node_id[j] <= K.node_id[j - 1])) return SLAM_EINVAL;
        for (int f = 0; f < (K.n_nodes ? K.node_off[K.n_nodes] : 0); f++)
            if (K.node_feat[f] < 0 || K.node_feat[f] >= K.n) return SLAM_EINVAL;
        for (int i = 0; i < K.n; i++)
            if (K.kps_un[i].octave < 0 || K.kps_un[i].octave >= K.nlevels) return SLAM_EINVAL;
    }
    for (int p = 0; p < n_pairs; p++) {
        if (pairs[p].kf1 < 0 || pairs[p].kf1 >= n_kfs || pairs[p].kf2 < 0 || pairs[p].kf2 >= n_kfs) return SLAM_EINVAL;
        if (kfs[pairs[p].kf1].n > cap) return SLAM_ECAP;
    }
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    // one staging blob: KF arrays, KF records, pairs
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    size_t need = al(sizeof(TriKF) * n_kfs) + al(sizeof(slam_tri_pair) * n_pairs);
    for (int k = 0; k < n_kfs; k++) {
        const slam_tri_kf& K = kfs[k];
        const int nf = K.n_nodes ? K.node_off[K.n_nodes] : 0;
        need += al(sizeof(slam_keypoint) * K.n) + al(4 * (size_t)K.n) + al(32 * (size_t)K.n) + al(K.n) +
                al(4 * (size_t)K.n_nodes) + al(4 * (size_t)(K.n_nodes + 1)) + al(4 * (size_t)nf);
    }
    slam_status st;
    if ((st = m->d_in.ensure(need)) || (st = m->d_out.ensure((size_t)n_pairs * cap * 4 + 4 * (size_t)n_pairs + 256)))
        return st;
    std::vector<uint8_t> host(need);
    size_t off = 0;
    uint8_t* dbase = m->d_in.as<uint8_t>();
    auto put = [&](const void* src, size_t bytes) -> const void* {
        if (!src || !bytes) return nullptr;
        std::memcpy(host.data() + off, src, bytes);
        const void* d = dbase + off;
        off += al(bytes);
        return d;
    };
    std::vector<TriKF> recs(n_kfs);
    std::vector<float> ur_default;
    for (int k = 0; k < n_kfs; k++) {
        const slam_tri_kf& K = kfs[k];
        TriKF& R = recs[k];
        R.n = K.n;
        R.n_nodes = K.n_nodes;
        R.nlevels = K.nlevels;
        R.kps = (const slam_keypoint*)put(K.kps_un, sizeof(slam_keypoint) * K.n);
        R.uright = (const float*)put(K.uright, 4 * (size_t)K.n);
        R.desc = (const uint8_t*)put(K.desc, 32 * (size_t)K.n);
        R.has_mp = (const uint8_t*)put(K.has_mp, K.n);
        R.node_id = (const int32_t*)put(K.node_id, 4 * (size_t)K.n_nodes);
        R.node_off = (const int32_t*)put(K.node_off, K.n_nodes ? 4 * (size_t)(K.n_nodes + 1) : 0);
        R.node_feat = (const int32_t*)put(K.node_feat, K.n_nodes ? 4 * (size_t)K.node_off[K.n_nodes] : 0);
        for (int l = 0; l < 16; l++) {
            R.scale[l] = l < K.nlevels ? K.scale[l] : 1.0f;
            R.sigma2[l] = l < K.nlevels ? K.level_sigma2[l] : 1.0f;
        }
        std::memcpy(R.R, K.Rcw, sizeof(R.R));
        std::memcpy(R.t, K.tcw, sizeof(R.t));
        std::memcpy(R.Ow, K.Ow, sizeof(R.Ow));
        std::memcpy(R.cam, K.cam, sizeof(R.cam));
    }
    const TriKF* d_recs = (const TriKF*)put(recs.data(), sizeof(TriKF) * n_kfs);
    const slam_tri_pair* d_pairs = (const slam_tri_pair*)put(pairs, sizeof(slam_tri_pair) * n_pairs);
    SLAM_HIP_TRY(hipMemcpyAsync(dbase, host.data(), off, hipMemcpyHostToDevice, m->stream));
    int32_t* d_m12 = m->d_out.as<int32_t>();
    int32_t* d_nm = d_m12 + (size_t)n_pairs * cap;
    hipLaunchKernelGGL(k_triangulation, dim3(n_pairs), dim3(kTriThreads), 0, m->stream, d_recs, d_pairs, check_ori,
                       cap, d_m12, d_nm);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(match12, d_m12, (size_t)n_pairs * cap * 4, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(nmatches, d_nm, (size_t)n_pairs * 4, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(m->stream));
    return SLAM_OK;
}


slam_status slamhot_fuse_search(slam_mapper* m, const slam_frame_view* F, const float* inv_level_sigma2, int n_mp,
                                const slam_mp_geom* mps, const uint8_t* mp_desc, float th, int32_t* best_idx,
                                int32_t* best_dist) {
    if (!m || !F || !F->Tcw || !inv_level_sigma2 || F->n < 0 || F->nlevels < 1 || F->nlevels > 16 || !F->scale ||
        (F->n && (!F->kps_un || !F->desc)) || n_mp < 0 || (n_mp && (!mps || !mp_desc || !best_idx || !best_dist)))
        return SLAM_EINVAL;
    if (n_mp == 0) return SLAM_OK;
    for (int i = 0; i < F->n; i++)
        if (F->kps_un[i].octave < 0 || F->kps_un[i].octave >= F->nlevels) return SLAM_EINVAL;
    // KeyFrame grid (Frame::AssignFeaturesToGrid, copied into the KeyFrame) as CSR
    const int ncell = kGridCols * kGridRows;
    std::vector<int32_t> cell(F->n, -1), start(ncell + 1, 0), feat(std::max(1, F->n));
    for (int i = 0; i < F->n; i++) {
        const int px = (int)std::round((F->kps_un[i].x - F->min_x) * F->grid_inv_w);
        const int py = (int)std::round((F->kps_un[i].y - F->min_y) * F->grid_inv_h);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        cell[i] = px * kGridRows + py;
        start[cell[i] + 1]++;
    }
    for (int c = 0; c < ncell; c++) start[c + 1] += start[c];
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    for (int i = 0; i < F->n; i++)
        if (cell[i] >= 0) feat[fill[cell[i]]++] = i;
    FuseKF K{};
    const float* T = F->Tcw;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 4; c++) K.T[4 * r + c] = T[4 * r + c];
        const double acc = (double)T[r] * T[3] + (double)T[4 + r] * T[7] + (double)T[8 + r] * T[11];
        K.Ow[r] = (float)(-1.0 * acc);  // KeyFrame::GetCameraCenter: -Rcw^T tcw as a cv::Mat product
    }
    K.fx = F->fx;
    K.fy = F->fy;
    K.cx = F->cx;
    K.cy = F->cy;
    K.bf = F->bf;
    K.min_x = F->min_x;
    K.min_y = F->min_y;
    K.max_x = F->max_x;
    K.max_y = F->max_y;
    K.inv_w = F->grid_inv_w;
    K.inv_h = F->grid_inv_h;
    K.log_scale = F->log_scale;
    K.nlevels = F->nlevels;
    K.n = F->n;
    for (int l = 0; l < 16; l++) {
        K.scale[l] = l < F->nlevels ? F->scale[l] : 1.0f;
        K.inv_sigma2[l] = l < F->nlevels ? inv_level_sigma2[l] : 1.0f;
    }
    std::lock_guard<std::mutex> g(m->mu);
    SLAM_HIP_TRY(hipSetDevice(m->device));
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t need = al(sizeof(slam_keypoint) * F->n) + al(4 * (size_t)F->n) + al(32 * (size_t)F->n) +
                        al(4 * start.size()) + al(4 * feat.size()) + al(sizeof(slam_mp_geom) * n_mp) + al(32 * (size_t)n_mp);
    slam_status st;
    if ((st = m->d_in.ensure(need)) || (st = m->d_out.ensure(8 * (size_t)n_mp))) return st;
    std::vector<uint8_t> host(need);
    size_t off = 0;
    uint8_t* dbase = m->d_in.as<uint8_t>();
    auto put = [&](const void* src, size_t bytes) -> const void* {
        if (!src || !bytes) return nullptr;
        std::memcpy(host.data() + off, src, bytes);
        const void* d = dbase + off;
        off += al(bytes);
        return d;
    };
    K.kps = (const slam_keypoint*)put(F->kps_un, sizeof(slam_keypoint) * F->n);
    K.uright = (const float*)put(F->uright, 4 * (size_t)F->n);
    K.desc = (const uint8_t*)put(F->desc, 32 * (size_t)F->n);
    K.cell_start = (const int32_t*)put(start.data(), 4 * start.size());
    K.cell_feat = (const int32_t*)put(feat.data(), 4 * feat.size());
    const slam_mp_geom* d_mps = (const slam_mp_geom*)put(mps, sizeof(slam_mp_geom) * n_mp);
    const uint8_t* d_desc = (const uint8_t*)put(mp_desc, 32 * (size_t)n_mp);
    SLAM_HIP_TRY(hipMemcpyAsync(dbase, host.data(), off, hipMemcpyHostToDevice, m->stream));
    int32_t* d_bi = m->d_out.as<int32_t>();
    int32_t* d_bd = d_bi + n_mp;
    hipLaunchKernelGGL(k_fuse_search, dim3((n_mp + kFuseThreads - 1) / kFuseThreads), dim3(kFuseThreads), 0,
                       m->stream, K, n_mp, d_mps, d_desc, th, d_bi, d_bd);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(best_idx, d_bi, 4 * (size_t)n_mp, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(best_dist, d_bd, 4 * (size_t)n_mp, hipMemcpyDeviceToHost, m->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(m->stream));
    return SLAM_OK;
}

}  // extern "C"
