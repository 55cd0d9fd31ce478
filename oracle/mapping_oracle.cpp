/*
 * mapping_oracle.cpp — CPU restatement of the LocalMapping matchers:
 * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:349-423), ORBmatcher::SearchForTriangulation_
 * (ORBmatcher.cc:1208-1433, pinhole KeyFrames), the search half of ORBmatcher::Fuse
 * (ORBmatcher.cc:1629-1788).  TEST INFRASTRUCTURE ONLY
 * (see oracle.h).  Parity unpinned (no reference fixtures for these functions).
 */
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../include/slamhot.h"
#include "fp_sites.hpp"

namespace {

int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
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
}

}  // namespace

extern "C" {

/* One SearchForTriangulation_ call; match12 (K1.n) = idx2 or -1.  Returns nmatches. */
int oracle_search_for_triangulation(const slam_tri_kf* K1, const slam_tri_kf* K2, const slam_tri_pair* P,
                                    int check_ori, int32_t* match12) {
    const int HISTO_LENGTH = 30, TH_LOW = 50;
    // epipole, R12, t12 (ORBmatcher.cc:1215-1240) and the F12 Pinhole::epipolarConstrain_
    // recomputes from them on every call (Pinhole.cpp:161-164); the F12 argument is unused
    float ep[2], R12[9], t12[3], F12[9];
    oracle_fp::tri_geometry(K1->Rcw, K1->tcw, K1->Ow, K1->cam, K2->Rcw, K2->tcw, K2->cam, ep, R12, t12, F12);
    int nmatches = 0;
    std::vector<bool> vbMatched2(K2->n, false);  // never set below, as in the reference
    for (int i = 0; i < K1->n; i++) match12[i] = -1;
    std::vector<int> rotHist[30];
    const float factor = 1.0f / HISTO_LENGTH;
    int f1 = 0, f2 = 0;
    while (f1 < K1->n_nodes && f2 < K2->n_nodes) {
        if (K1->node_id[f1] == K2->node_id[f2]) {
            for (int i1 = K1->node_off[f1]; i1 < K1->node_off[f1 + 1]; i1++) {
                const int idx1 = K1->node_feat[i1];
                if (K1->has_mp[idx1]) continue;
                const bool bStereo1 = K1->uright && K1->uright[idx1] >= 0;
                if (P->only_stereo && !bStereo1) continue;
                const slam_keypoint& kp1 = K1->kps_un[idx1];
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = K2->node_off[f2]; i2 < K2->node_off[f2 + 1]; i2++) {
                    const int idx2 = K2->node_feat[i2];
                    if (vbMatched2[idx2] || K2->has_mp[idx2]) continue;
                    const bool bStereo2 = K2->uright && K2->uright[idx2] >= 0;
                    if (P->only_stereo && !bStereo2) continue;
                    const int dist = hamming32(K1->desc + 32 * (size_t)idx1, K2->desc + 32 * (size_t)idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const slam_keypoint& kp2 = K2->kps_un[idx2];
                    if (!bStereo1 && !bStereo2 && oracle_fp::near_epipole(ep, kp2.x, kp2.y, K2->scale[kp2.octave]))
                        continue;
                    if (oracle_fp::epipolar(F12, kp1.x, kp1.y, kp2.x, kp2.y, K2->level_sigma2[kp2.octave]) ||
                        P->coarse) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    const slam_keypoint& kp2 = K2->kps_un[bestIdx2];
                    match12[idx1] = bestIdx2;
                    nmatches++;
                    if (check_ori) {
                        float rot = kp1.angle - kp2.angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        rotHist[bin].push_back(idx1);
                    }
                }
            }
            f1++;
            f2++;
        } else if (K1->node_id[f1] < K2->node_id[f2]) {
            f1 = (int)(std::lower_bound(K1->node_id, K1->node_id + K1->n_nodes, K2->node_id[f2]) - K1->node_id);
        } else {
            f2 = (int)(std::lower_bound(K2->node_id, K2->node_id + K2->n_nodes, K1->node_id[f1]) - K2->node_id);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx : rotHist[i]) {
                match12[idx] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}


void oracle_distinctive_descriptors(int n_mp, const int32_t* off, const uint8_t* desc, int32_t* best) {
    for (int m = 0; m < n_mp; m++) {
        const size_t N = (size_t)(off[m + 1] - off[m]);
        const uint8_t* D = desc + (size_t)off[m] * 32;
        if (N == 0) {
            best[m] = -1;
            continue;
        }
        std::vector<float> Distances(N * N);
        for (size_t i = 0; i < N; i++) {
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int distij = hamming32(D + 32 * i, D + 32 * j);
                Distances[i * N + j] = distij;
                Distances[j * N + i] = distij;
            }
        }
        int BestMedian = INT_MAX;
        int BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances.begin() + i * N, Distances.begin() + (i + 1) * N);
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[(size_t)(0.5 * (N - 1))];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best[m] = BestIdx;
    }
}

/* ORBmatcher::Fuse (ORBmatcher.cc:1629-1788), search half, one MapPoint at a time in list order
 * (bRight = false, NLeft == -1): best_idx / best_dist per MapPoint. */
void oracle_fuse_search(const slam_frame_view* F, const float* inv_level_sigma2, int n_mp, const slam_mp_geom* mps,
                        const uint8_t* mp_desc, float th, int32_t* best_idx, int32_t* best_dist) {
    const int GRID_COLS = 64, GRID_ROWS = 48;
    std::vector<std::vector<int>> grid(GRID_COLS * GRID_ROWS);  // KeyFrame::mGrid
    for (int i = 0; i < F->n; i++) {
        const int px = (int)std::round((F->kps_un[i].x - F->min_x) * F->grid_inv_w);
        const int py = (int)std::round((F->kps_un[i].y - F->min_y) * F->grid_inv_h);
        if (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) continue;
        grid[px * GRID_ROWS + py].push_back(i);
    }
    const float* T = F->Tcw;
    float Ow[3];
    for (int r = 0; r < 3; r++) {
        const double acc = (double)T[r] * T[3] + (double)T[4 + r] * T[7] + (double)T[8 + r] * T[11];
        Ow[r] = (float)(-1.0 * acc);
    }
    for (int i = 0; i < n_mp; i++) {
        const slam_mp_geom& g = mps[i];
        best_idx[i] = -1;
        best_dist[i] = 256;
        if (g.is_bad || g.seen) continue;
        float p3Dc[3];  // Rcw * p3Dw + tcw (cv::Mat gemm: double accumulation)
        for (int r = 0; r < 3; r++) {
            const double acc = (double)T[4 * r] * g.pos[0] + (double)T[4 * r + 1] * g.pos[1] + (double)T[4 * r + 2] * g.pos[2];
            p3Dc[r] = (float)(acc * 1.0 + (double)T[4 * r + 3] * 1.0);
        }
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0], y = p3Dc[1], z = p3Dc[2];
        const float u = F->fx * x / z + F->cx, v = F->fy * y / z + F->cy;
        if (!(u >= F->min_x && u < F->max_x && v >= F->min_y && v < F->max_y)) continue;
        const float ur = oracle_fp::ur_of(u, F->bf, invz);  // ORBmatcher.cc.o Fuse @0x1be1
        const float maxDistance = 1.2f * g.max_dist;
        const float minDistance = 0.8f * g.min_dist;
        const float PO[3] = {g.pos[0] - Ow[0], g.pos[1] - Ow[1], g.pos[2] - Ow[2]};
        const float dist3D = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const double dot = (double)PO[0] * g.normal[0] + (double)PO[1] * g.normal[1] + (double)PO[2] * g.normal[2];
        if (dot < 0.5 * dist3D) continue;
        const float ratio = g.max_dist / dist3D;
        int nPredictedLevel = (int)std::ceil(std::log(ratio) / F->log_scale);  // logf
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= F->nlevels) nPredictedLevel = F->nlevels - 1;
        const float radius = th * F->scale[nPredictedLevel];
        std::vector<int> vIndices;  // KeyFrame::GetFeaturesInArea (KeyFrame.cc:737-781)
        const int nMinCellX = std::max(0, (int)std::floor((u - F->min_x - radius) * F->grid_inv_w));
        const int nMaxCellX = std::min(GRID_COLS - 1, (int)std::ceil((u - F->min_x + radius) * F->grid_inv_w));
        const int nMinCellY = std::max(0, (int)std::floor((v - F->min_y - radius) * F->grid_inv_h));
        const int nMaxCellY = std::min(GRID_ROWS - 1, (int)std::ceil((v - F->min_y + radius) * F->grid_inv_h));
        if (nMinCellX < GRID_COLS && nMaxCellX >= 0 && nMinCellY < GRID_ROWS && nMaxCellY >= 0)
            for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
                for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
                    for (int idx : grid[ix * GRID_ROWS + iy]) {
                        const float distx = F->kps_un[idx].x - u, disty = F->kps_un[idx].y - v;
                        if (std::fabs(distx) < radius && std::fabs(disty) < radius) vIndices.push_back(idx);
                    }
        int bestDist = 256, bestIdx = -1;
        for (int idx : vIndices) {
            const slam_keypoint& kp = F->kps_un[idx];
            const int kpLevel = kp.octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            if (F->uright && F->uright[idx] >= 0) {
                const float ex = u - kp.x, ey = v - kp.y, er = ur - F->uright[idx];
                const float e2 = std::fma(er, er, std::fma(ex, ex, ey * ey));  // Fuse @0x1c98, @0x1cb5
                if (e2 * inv_level_sigma2[kpLevel] > 7.8) continue;
            } else {
                const float ex = u - kp.x, ey = v - kp.y;
                const float e2 = std::fma(ex, ex, ey * ey);
                if (e2 * inv_level_sigma2[kpLevel] > 5.99) continue;
            }
            const int dist = hamming32(mp_desc + 32 * (size_t)i, F->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        best_idx[i] = bestIdx;
        best_dist[i] = bestDist;
    }
}

}  // extern "C"
