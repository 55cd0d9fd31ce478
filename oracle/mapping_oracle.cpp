/*
 * mapping_oracle.cpp — CPU restatement of the LocalMapping matchers:
 * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:349-423), ORBmatcher::SearchForTriangulation_
 * (ORBmatcher.cc:1208-1433, pinhole KeyFrames).  TEST INFRASTRUCTURE ONLY
 * (see oracle.h).  Parity unpinned (no reference fixtures for these functions).
 */
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../include/slamhot.h"

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

// Pinhole::epipolarConstrain_ (Pinhole.cpp:159-181)
bool epipolar(const float* F, const slam_keypoint& kp1, const slam_keypoint& kp2, float unc) {
    const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
    const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
    const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * unc;
}

}  // namespace

extern "C" {

/* One SearchForTriangulation_ call; match12 (K1.n) = idx2 or -1.  Returns nmatches. */
int oracle_search_for_triangulation(const slam_tri_kf* K1, const slam_tri_kf* K2, const slam_tri_pair* P,
                                    int check_ori, int32_t* match12) {
    const int HISTO_LENGTH = 30, TH_LOW = 50;
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
                    if (!bStereo1 && !bStereo2) {
                        const float distex = P->ep[0] - kp2.x;
                        const float distey = P->ep[1] - kp2.y;
                        if (distex * distex + distey * distey < 100 * K2->scale[kp2.octave]) continue;
                    }
                    if (epipolar(P->F12, kp1, kp2, K2->level_sigma2[kp2.octave]) || P->coarse) {
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

}  // extern "C"
