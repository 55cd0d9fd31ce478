/*
 * projection_oracle.cpp — CPU restatement of ORBmatcher::SearchByProjection (three
 * variants) and the Frame grid (Frame::AssignFeaturesToGrid / PosInGrid /
 * GetFeaturesInArea).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Parity status: unpinned against the real reference (no golden vectors, no OpenCV here).
 * The float cv::Mat products of the reference (Rcw*x+tcw, -Rcw.t()*tcw) are restated as
 * OpenCV's gemm with double accumulation rounded once to float; cv::norm of a 3-vector as
 * a double sum of squares; log/ceil through this host's glibc.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/slamhot.h"
#include "fp_sites.hpp"

namespace {

const int GRID_COLS = 64, GRID_ROWS = 48;  // Frame.h:37-38
const int TH_HIGH = 100, HISTO_LENGTH = 30;

int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

int rot_bin(float a, float b) {
    float rot = a - b;
    if (rot < 0.0) rot += 360.0f;
    const float factor = 1.0f / HISTO_LENGTH;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// Frame::PosInGrid (Frame.cc:708-718): round((x - mnMinX) * mfGridElementWidthInv)
inline void pos_in_grid(float x, float y, float min_x, float min_y, float inv_w, float inv_h, int& px, int& py) {
    px = (int)std::round((x - min_x) * inv_w);
    py = (int)std::round((y - min_y) * inv_h);
}

// Frame::GetFeaturesInArea's cell range (Frame.cc:645-659): floor / ceil of the scaled box
inline void area_cells(float x, float y, float r, float min_x, float min_y, float inv_w, float inv_h, int* c) {
    c[0] = (int)std::floor((x - min_x - r) * inv_w);
    c[1] = (int)std::ceil((x - min_x + r) * inv_w);
    c[2] = (int)std::floor((y - min_y - r) * inv_h);
    c[3] = (int)std::ceil((y - min_y + r) * inv_h);
}

struct Grid {
    std::vector<std::vector<int>> cells;  // [ix * GRID_ROWS + iy]
};

// Frame::AssignFeaturesToGrid + PosInGrid (Frame.cc:380-411, 708-718)
Grid build_grid(const slam_frame_view* F) {
    Grid g;
    g.cells.assign(GRID_COLS * GRID_ROWS, {});
    for (int i = 0; i < F->n; i++) {
        const slam_keypoint& kp = F->kps_un[i];
        int px, py;
        pos_in_grid(kp.x, kp.y, F->min_x, F->min_y, F->grid_inv_w, F->grid_inv_h, px, py);
        if (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) continue;
        g.cells[px * GRID_ROWS + py].push_back(i);
    }
    return g;
}

// Frame::GetFeaturesInArea (Frame.cc:640-706)
std::vector<int> features_in_area(const slam_frame_view* F, const Grid& g, float x, float y, float r,
                                  int minLevel, int maxLevel) {
    std::vector<int> out;
    int cb[4];
    area_cells(x, y, r, F->min_x, F->min_y, F->grid_inv_w, F->grid_inv_h, cb);
    const int nMinCellX = std::max(0, cb[0]);
    if (nMinCellX >= GRID_COLS) return out;
    const int nMaxCellX = std::min(GRID_COLS - 1, cb[1]);
    if (nMaxCellX < 0) return out;
    const int nMinCellY = std::max(0, cb[2]);
    if (nMinCellY >= GRID_ROWS) return out;
    const int nMaxCellY = std::min(GRID_ROWS - 1, cb[3]);
    if (nMaxCellY < 0) return out;
    const bool check = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
            for (int idx : g.cells[ix * GRID_ROWS + iy]) {
                const slam_keypoint& kp = F->kps_un[idx];
                if (check) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float dx = kp.x - x, dy = kp.y - y;
                if (std::fabs(dx) < r && std::fabs(dy) < r) out.push_back(idx);
            }
    return out;
}

// cv::Mat float products (gemm, double accumulation)
void mat_mul_add(const float* T, const float* X, float* out) {  // R * X + t, T 4x4 row-major
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[4 * i] * X[0] + (double)T[4 * i + 1] * X[1] + (double)T[4 * i + 2] * X[2];
        out[i] = (float)(acc * 1.0 + (double)T[4 * i + 3] * 1.0);
    }
}
void neg_rt_t(const float* T, float* out) {  // -R^T * t
    for (int i = 0; i < 3; i++) {
        const double acc = (double)T[i] * T[3] + (double)T[4 + i] * T[7] + (double)T[8 + i] * T[11];
        out[i] = (float)(-1.0 * acc);
    }
}

// SearchByProjection(F, LastF)'s window (ORBmatcher.cc:2221): th * mvScaleFactors[nLastOctave]
inline float search_radius(float th, float scale) { return th * scale; }

float radius_by_viewing_cos(float c) { return c > 0.998 ? 2.5f : 4.0f; }  // ORBmatcher.cc:216-222

struct Assign {
    std::vector<int32_t> f_mp;      // current mvpMapPoints (query index) after this call
    std::vector<uint8_t> blocking;  // current entry blocks (obs > 0)
};

}  // namespace

extern "C" {

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
int oracle_search_by_projection_local(const slam_frame_view* F, int n_mp, const slam_mp_track* mps,
                                      const uint8_t* mp_desc, float nnratio, float th, int far_points,
                                      float th_far, int32_t* f_match) {
    const Grid g = build_grid(F);
    std::vector<int8_t> state(F->n);
    for (int i = 0; i < F->n; i++) {
        state[i] = F->mp_state ? F->mp_state[i] : -1;
        f_match[i] = -1;
    }
    int nmatches = 0;
    const bool bFactor = th != 1.0;
    for (int q = 0; q < n_mp; q++) {
        const slam_mp_track& mp = mps[q];
        if (!mp.in_view) continue;
        if (far_points && mp.depth > th_far) continue;
        if (mp.is_bad) continue;
        const int level = mp.scale_level;
        float r = radius_by_viewing_cos(mp.view_cos);
        if (bFactor) r *= th;
        const std::vector<int> idxs =
            features_in_area(F, g, mp.proj_x, mp.proj_y, r * F->scale[level], level - 1, level);
        if (idxs.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int idx : idxs) {
            if (state[idx] == 1) continue;  // holds a MapPoint with observations
            if (F->uright && F->uright[idx] > 0) {
                const float er = std::fabs(mp.proj_xr - F->uright[idx]);
                if (er > r * F->scale[level]) continue;
            }
            const int dist = hamming(mp_desc + (size_t)q * 32, F->desc + (size_t)idx * 32);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F->kps_un[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F->kps_un[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                f_match[bestIdx] = q;
                state[bestIdx] = mp.has_obs ? 1 : 0;
                nmatches++;
            }
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
int oracle_search_by_projection_last(const slam_frame_view* F, const slam_last_frame* LF, float nnratio,
                                     int check_ori, float th, int mono, int32_t* f_match) {
    (void)nnratio;
    const Grid g = build_grid(F);
    std::vector<int8_t> state(F->n);
    for (int i = 0; i < F->n; i++) {
        state[i] = F->mp_state ? F->mp_state[i] : -1;
        f_match[i] = -1;
    }
    std::vector<int> rotHist[HISTO_LENGTH];
    float twc[3], tlc[3];
    neg_rt_t(F->Tcw, twc);
    mat_mul_add(LF->Tcw, twc, tlc);
    const bool bForward = tlc[2] > F->b && !mono;
    const bool bBackward = -tlc[2] > F->b && !mono;
    int nmatches = 0;
    for (int i = 0; i < LF->n; i++) {
        if (!LF->has_mp[i] || LF->outlier[i]) continue;
        float xc[3];
        mat_mul_add(F->Tcw, LF->mp_pos + 3 * (size_t)i, xc);
        const float invzc = (float)(1.0 / xc[2]);
        if (invzc < 0) continue;
        const float u = F->fx * xc[0] / xc[2] + F->cx;
        const float v = F->fy * xc[1] / xc[2] + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const int nLastOctave = LF->kps[i].octave;
        const float radius = search_radius(th, F->scale[nLastOctave]);
        std::vector<int> idxs;
        if (bForward) idxs = features_in_area(F, g, u, v, radius, nLastOctave, -1);
        else if (bBackward) idxs = features_in_area(F, g, u, v, radius, 0, nLastOctave);
        else idxs = features_in_area(F, g, u, v, radius, nLastOctave - 1, nLastOctave + 1);
        if (idxs.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : idxs) {
            if (state[i2] == 1) continue;
            if (F->uright && F->uright[i2] > 0) {
                const float ur = oracle_fp::ur_of(u, F->bf, invzc);  // ORBmatcher.cc.o @0x95c7
                const float er = std::fabs(ur - F->uright[i2]);
                if (er > radius) continue;
            }
            const int dist = hamming(LF->mp_desc + (size_t)i * 32, F->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            f_match[bestIdx2] = i;
            state[bestIdx2] = LF->mp_has_obs[i] ? 1 : 0;
            nmatches++;
            if (check_ori) rotHist[rot_bin(LF->kps_un[i].angle, F->kps_un[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (check_ori) {
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int idx : rotHist[b]) {
                f_match[idx] = -2;  // CurrentFrame.mvpMapPoints[idx] = NULL
                nmatches--;
            }
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
int oracle_search_by_projection_kf(const slam_frame_view* F, const slam_kf_points* KF, float nnratio,
                                   int check_ori, float th, int orb_dist, int32_t* f_match) {
    (void)nnratio;
    const Grid g = build_grid(F);
    std::vector<int8_t> state(F->n);
    for (int i = 0; i < F->n; i++) {
        state[i] = F->mp_state ? F->mp_state[i] : -1;
        f_match[i] = -1;
    }
    std::vector<int> rotHist[HISTO_LENGTH];
    float Ow[3];
    neg_rt_t(F->Tcw, Ow);
    int nmatches = 0;
    for (int i = 0; i < KF->n; i++) {
        if (!KF->use[i]) continue;
        const float* X = KF->mp_pos + 3 * (size_t)i;
        float xc[3];
        mat_mul_add(F->Tcw, X, xc);
        const float u = F->fx * xc[0] / xc[2] + F->cx;
        const float v = F->fy * xc[1] / xc[2] + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        const float dist3D = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        const float maxDistance = 1.2f * KF->max_dist[i];
        const float minDistance = 0.8f * KF->min_dist[i];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float ratio = KF->max_dist[i] / dist3D;
        int level = (int)std::ceil(std::log(ratio) / F->log_scale);
        if (level < 0) level = 0;
        else if (level >= F->nlevels) level = F->nlevels - 1;
        const float radius = th * F->scale[level];
        const std::vector<int> idxs = features_in_area(F, g, u, v, radius, level - 1, level + 1);
        if (idxs.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : idxs) {
            if (state[i2] >= 0) continue;  // any MapPoint
            const int dist = hamming(KF->mp_desc + (size_t)i * 32, F->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= orb_dist) {
            f_match[bestIdx2] = i;
            state[bestIdx2] = 1;
            nmatches++;
            if (check_ori) rotHist[rot_bin(KF->kps_un[i].angle, F->kps_un[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (check_ori) {
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int idx : rotHist[b]) {
                f_match[idx] = -2;  // CurrentFrame.mvpMapPoints[idx] = NULL
                nmatches--;
            }
        }
    }
    return nmatches;
}

/* Frame::isInFrustum (Frame.cc:493-556, Nleft == -1) over a local map as
 * Tracking::SearchLocalPoints calls it (Tracking.cc:3213-3226), with the contractions of the
 * reference binary (Frame.cc.o @0x9ee0, oracle/fp_sites.hpp): Matx products as fma chains,
 * cv::norm in double, PO.dot(Pn) as an fma chain, mTrackProjXR = fma(-mbf, invz, u);
 * PredictScale (MapPoint.cc:551-566) with glibc logf.  Returns nToMatch. */
int oracle_is_in_frustum(const slam_frame_view* F, int n_mp, const slam_mp_geom* mps, float view_cos_limit,
                         slam_mp_track* track) {
    float Ow[3];
    neg_rt_t(F->Tcw, Ow);
    const float* T = F->Tcw;
    int n_in = 0;
    for (int i = 0; i < n_mp; i++) {
        const slam_mp_geom& g = mps[i];
        slam_mp_track& tr = track[i];
        std::memset(&tr, 0, sizeof(tr));
        tr.proj_x = -1.0f;
        tr.proj_y = -1.0f;
        tr.scale_level = -1;
        tr.is_bad = g.is_bad;
        tr.has_obs = g.has_obs;
        if (g.seen || g.is_bad) continue;  // Tracking.cc:3217-3220
        float Pc[3];
        for (int r = 0; r < 3; r++) Pc[r] = oracle_fp::dot3_chain(T + 4 * r, g.pos) + T[4 * r + 3];
        const float Pc_dist = (float)std::sqrt(oracle_fp::norm2_d(Pc));
        const float PcZ = Pc[2];
        const float invz = 1.0f / PcZ;
        if (PcZ < 0.0f) continue;
        float uv[2];
        const float cam[4] = {F->fx, F->fy, F->cx, F->cy};
        oracle_fp::project(cam, Pc, uv);
        const float u = uv[0], v = uv[1];
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        tr.proj_x = u;  // written as soon as the point lands in the image (Frame.cc:521-522)
        tr.proj_y = v;
        const float maxDistance = 1.2f * g.max_dist;
        const float minDistance = 0.8f * g.min_dist;
        float PO[3];
        for (int k = 0; k < 3; k++) PO[k] = g.pos[k] - Ow[k];
        const float dist = (float)std::sqrt(oracle_fp::norm2_d(PO));
        if (dist < minDistance || dist > maxDistance) continue;
        const float viewCos = oracle_fp::dot3_chain(PO, g.normal) / dist;
        if (viewCos < view_cos_limit) continue;
        const float ratio = g.max_dist / dist;
        int nScale = (int)std::ceil(std::log(ratio) / F->log_scale);  // std::log(float) = logf
        if (nScale < 0) nScale = 0;
        else if (nScale >= F->nlevels) nScale = F->nlevels - 1;
        tr.in_view = 1;
        tr.proj_xr = oracle_fp::ur_of(u, F->bf, invz);
        tr.depth = Pc_dist;
        tr.scale_level = nScale;
        tr.view_cos = viewCos;
        n_in++;
    }
    return n_in;
}

/* MapPoint::PredictScale with glibc logf vs with the correctly rounded logf the device uses
 * ((float)log((double)r)): number of float ratios in [lo, hi] (every bit pattern) whose
 * predicted level (before clamping) differs. */
long oracle_check_predict_scale(float lo, float hi, float log_scale) {
    uint32_t a, b;
    std::memcpy(&a, &lo, 4);
    std::memcpy(&b, &hi, 4);
    long bad = 0;
    for (uint32_t u = a; u <= b; u++) {
        float r;
        std::memcpy(&r, &u, 4);
        const int g = (int)std::ceil(std::log(r) / log_scale);
        const int c = (int)std::ceil((float)std::log((double)r) / log_scale);
        bad += g != c;
    }
    return bad;
}

/* single float sites for tests/test_fp_sites.py (vs the reference objects) */
int oracle_fp_rot_bin_proj(float a, float b) { return rot_bin(a, b); }
void oracle_fp_pos_in_grid(float x, float y, float min_x, float min_y, float inv_w, float inv_h, int* out) {
    pos_in_grid(x, y, min_x, min_y, inv_w, inv_h, out[0], out[1]);
}
void oracle_fp_area_cells(float x, float y, float r, float min_x, float min_y, float inv_w, float inv_h, int* out) {
    area_cells(x, y, r, min_x, min_y, inv_w, inv_h, out);
}
float oracle_fp_search_radius(float th, float scale) { return search_radius(th, scale); }

}  // extern "C"
