/*
 * stereo_oracle.cpp — CPU restatement of Frame::ComputeStereoMatches (Frame.cc:794-964):
 * row-band candidate table, ORB Hamming best match (< (TH_HIGH + TH_LOW) / 2), 11x11 SAD
 * window search over +-5 columns on the matching pyramid level, parabola sub-pixel fit,
 * disparity gate, median-based outlier rejection.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Parity unpinned (no reference fixtures; OpenCV's cv::norm(L1) restated as an integer sum).
 */
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "../include/slamhot.h"

namespace {

int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

}  // namespace

extern "C" {

/* Left/right keypoints and descriptors of one stereo frame; pyr_left/right[l] point at
 * level l (row stride pitch_*[l]), level sizes lw/lh; scale[l] = mvScaleFactors[l],
 * inv_scale[l] = mvInvScaleFactors[l].  Outputs: uright[n_left], depth[n_left]. */
void oracle_stereo_matches(int n_left, const slam_keypoint* kl, const uint8_t* dl, int n_right,
                           const slam_keypoint* kr, const uint8_t* dr, int nlevels, const uint8_t* const* pyr_left,
                           const uint8_t* const* pyr_right, const int* pitch_left, const int* pitch_right,
                           const int* lw, const int* lh, const float* scale, const float* inv_scale, float mbf,
                           float mb, float* uright, float* depth) {
    for (int i = 0; i < n_left; i++) {
        uright[i] = -1.0f;
        depth[i] = -1.0f;
    }
    const int TH_HIGH = 100, TH_LOW = 50;
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = lh[0];
    std::vector<std::vector<size_t>> vRowIndices(nRows);
    for (int iR = 0; iR < n_right; iR++) {
        const float kpY = kr[iR].y;
        const float r = 2.0f * scale[kr[iR].octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) vRowIndices[yi].push_back(iR);  // reference: unchecked
    }
    const float minZ = mb;
    const float minD = 0;
    const float maxD = mbf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    for (int iL = 0; iL < n_left; iL++) {
        const int levelL = kl[iL].octave;
        const float vL = kl[iL].y, uL = kl[iL].x;
        const long row = (long)vL;  // vector index from a float
        if (row < 0 || row >= nRows) continue;
        const std::vector<size_t>& vCandidates = vRowIndices[row];
        if (vCandidates.empty()) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        for (size_t iC = 0; iC < vCandidates.size(); iC++) {
            const size_t iR = vCandidates[iC];
            if (kr[iR].octave < levelL - 1 || kr[iR].octave > levelL + 1) continue;
            const float uR = kr[iR].x;
            if (uR >= minU && uR <= maxU) {
                const int dist = hamming32(dl + 32 * (size_t)iL, dr + 32 * iR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist >= thOrbDist) continue;
        const float uR0 = kr[bestIdxR].x;
        const float scaleFactor = inv_scale[levelL];
        const float scaleduL = std::round(uL * scaleFactor);
        const float scaledvL = std::round(vL * scaleFactor);
        const float scaleduR0 = std::round(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= lw[levelL]) continue;
        const int vy0 = (int)scaledvL - w, ux0 = (int)scaleduL - w, ur0 = (int)scaleduR0;
        // windows the reference slices must lie inside the level (it asserts otherwise)
        if (vy0 < 0 || vy0 + 2 * w + 1 > lh[levelL] || ux0 < 0 || ux0 + 2 * w + 1 > lw[levelL] || ur0 - L - w < 0 ||
            ur0 + L + w + 1 > lw[levelL])
            continue;
        int bestDist2 = INT_MAX;
        int bestincR = 0;
        float vDists[2 * L + 1];
        const uint8_t* PL = pyr_left[levelL];
        const uint8_t* PR = pyr_right[levelL];
        const int pl = pitch_left[levelL], pr = pitch_right[levelL];
        for (int incR = -L; incR <= L; incR++) {
            long s = 0;
            for (int yy = 0; yy < 2 * w + 1; yy++)
                for (int xx = 0; xx < 2 * w + 1; xx++)
                    s += std::abs((int)PL[(size_t)(vy0 + yy) * pl + ux0 + xx] -
                                  (int)PR[(size_t)(vy0 + yy) * pr + ur0 + incR - w + xx]);
            const float dist = (float)(double)s;  // cv::norm returns double
            if (dist < bestDist2) {
                bestDist2 = (int)dist;
                bestincR = incR;
            }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = mbf / disparity;
            uright[iL] = bestuR;
            vDistIdx.push_back(std::pair<int, int>(bestDist2, iL));
        }
    }
    if (vDistIdx.empty()) return;  // reference reads vDistIdx[0] (undefined) here
    std::sort(vDistIdx.begin(), vDistIdx.end());
    const float median = vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist) break;
        uright[vDistIdx[i].second] = -1;
        depth[vDistIdx[i].second] = -1;
    }
}

}  // extern "C"
