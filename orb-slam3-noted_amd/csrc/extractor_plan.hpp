// extractor_plan.hpp — host-side geometry of one ORB extraction (sizes, cell grid, resize
// coefficient tables, octree roots), computed exactly as the reference computes it so the
// device kernels only do integer work.  Plain C++ (no HIP), shared by the HIP library.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/slamhot.h"

namespace slamhot {

constexpr int kMaxLevels = 16;
constexpr int kMaxRoots = 16;
constexpr int kEdgeThreshold = 19;  // ORBextractor.cc:72
constexpr int kPatchSize = 31;      // ORBextractor.cc:70
constexpr int kHalfPatch = 15;      // ORBextractor.cc:71

inline int host_round(float v) { return (int)std::lrintf(v); }  // cvRound

struct LevelPlan {
    int w, h, pitch;         // level image; pitch is a multiple of 64 bytes
    int64_t pyr_off;         // byte offset of level (l >= 1) inside a frame's pyramid block
    int64_t blur_off;        // byte offset inside a frame's blurred block
    int minBX, minBY, maxBX, maxBY;  // ComputeKeyPointsOctTree borders (ORBextractor.cc:771-774)
    int cell_begin, cell_end;        // range in the cell table
    int nfeat;               // mnFeaturesPerLevel[level]
    int kbase, kcap;         // octree output slots of this level inside a frame
    int key_base, key_cap;   // candidate (FAST keypoint) slots of this level inside a frame
    float scale;             // mvScaleFactor[level]
    float size;              // (float)(int)(PATCH_SIZE * scale)  (ORBextractor.cc:862)
    int nIni;                // DistributeOctTree root count (ORBextractor.cc:541)
    int root_x0[kMaxRoots], root_x1[kMaxRoots];
    int root_first_x[kMaxRoots];  // smallest relative x with (int)(x / hX) >= i
    int xtab_off, ytab_off;  // resize coefficient tables (levels >= 1)
    int xmax;                // resize: first dx whose source column clips
};

struct CellDesc {
    int16_t level, iniX, iniY, cw, ch, pad;
    int32_t slot;  // slot index (0..ncells) inside a frame
};

struct ResizeX {
    int32_t sx;
    int16_t a0, a1;
};
struct ResizeY {
    int32_t y0, y1;
    int16_t b0, b1;
    int32_t pad;
};

struct Plan {
    slam_orb_params prm{};
    int nlevels = 0, W = 0, H = 0;
    LevelPlan lv[kMaxLevels]{};
    int ncells = 0, slot_cap = 0;  // per-frame cell slots, each slot_cap candidates
    int kslots = 0;                // per-frame octree output slots (sum of kcap)
    int key_slots = 0;             // per-frame candidate slots (sum of key_cap)
    int max_nodes = 0;             // octree alive-node bound (LDS sizing)
    int64_t pyr_frame = 0, blur_frame = 0;
    std::vector<CellDesc> cells;
    std::vector<ResizeX> xtab;
    std::vector<ResizeY> ytab;
    // reference scale tables (ORBextractor.cc:413-444)
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat;
};

inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

// ORBextractor::ORBextractor, ORBextractor.cc:408-444 (`scaleFactor` is a double member).
inline void build_scale_tables(const slam_orb_params& p, Plan& P) {
    const int L = p.nlevels;
    const double sf = (double)p.scale_factor;
    P.scale.assign(L, 1.f);
    P.sigma2.assign(L, 1.f);
    for (int i = 1; i < L; i++) {
        P.scale[i] = (float)((double)P.scale[i - 1] * sf);
        P.sigma2[i] = P.scale[i] * P.scale[i];
    }
    P.inv_scale.resize(L);
    P.inv_sigma2.resize(L);
    for (int i = 0; i < L; i++) {
        P.inv_scale[i] = 1.0f / P.scale[i];
        P.inv_sigma2[i] = 1.0f / P.sigma2[i];
    }
    P.nfeat.assign(L, 0);
    const float factor = (float)(1.0f / sf);
    float per = p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        P.nfeat[l] = host_round(per);
        sum += P.nfeat[l];
        per *= factor;
    }
    P.nfeat[L - 1] = std::max(p.nfeatures - sum, 0);
}

// cv::resize INTER_LINEAR coefficient tables (OpenCV 4.2.0 hal::resize, fixed point 2^11).
inline int clamp_short(int v) { return std::max(-32768, std::min(32767, v)); }

inline void build_resize_tables(int sw, int sh, int dw, int dh, Plan& P, LevelPlan& L) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    L.xtab_off = (int)P.xtab.size();
    L.ytab_off = (int)P.ytab.size();
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
        }
        ResizeX e;
        e.sx = sx;
        e.a0 = (int16_t)clamp_short(host_round((1.f - fx) * 2048));
        e.a1 = (int16_t)clamp_short(host_round(fx * 2048));
        P.xtab.push_back(e);
    }
    L.xmax = xmax;
    // columns at/after xmax use D = S[sx] * 2048 (HResizeLinear's tail loop): encode them as
    // (a0, a1) = (2048, 0) so the device formula S[sx]*a0 + S[sx+1]*a1 is branch-free
    for (int dx = xmax; dx < dw; dx++) {
        P.xtab[L.xtab_off + dx].a0 = 2048;
        P.xtab[L.xtab_off + dx].a1 = 0;
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        ResizeY e;
        e.y0 = std::min(std::max(sy, 0), sh - 1);
        e.y1 = std::min(std::max(sy + 1, 0), sh - 1);
        e.b0 = (int16_t)clamp_short(host_round((1.f - fy) * 2048));
        e.b1 = (int16_t)clamp_short(host_round(fy * 2048));
        e.pad = 0;
        P.ytab.push_back(e);
    }
    // k_resize4 reads a thread's 4 columns as two 16-byte vectors and its rows (up to 8) one entry
    // each: each level's tables padded (x to a multiple of 4, y of 8) with copies of the last entry
    // (the clamped column / row the kernel would compute), so the next level's tables stay aligned
    while (P.xtab.size() % 4) P.xtab.push_back(P.xtab.back());
    while (P.ytab.size() % 8) P.ytab.push_back(P.ytab.back());
}

// Everything a W x H extraction needs.  Returns false for unsupported geometry.
inline bool build_plan(const slam_orb_params& p, int W, int H, Plan& P) {
    if (p.nlevels < 1 || p.nlevels > kMaxLevels || W <= 0 || H <= 0 || W > 4095 || H > 4095 ||
        p.nfeatures < 0 || !(p.scale_factor > 1.0f))
        return false;
    P = Plan();
    P.prm = p;
    P.nlevels = p.nlevels;
    P.W = W;
    P.H = H;
    build_scale_tables(p, P);
    int64_t pyr = 0, blur = 0;
    int kslots = 0, key_slots = 0;
    int max_nodes = 0;
    int slot_cap = 0;
    for (int l = 0; l < P.nlevels; l++) {
        LevelPlan& L = P.lv[l];
        // ComputePyramid sizes, ORBextractor.cc:1157
        L.w = host_round((float)W * P.inv_scale[l]);
        L.h = host_round((float)H * P.inv_scale[l]);
        if (L.w < 2 * kEdgeThreshold || L.h < 2 * kEdgeThreshold) return false;
        L.pitch = round_up(L.w, 64);
        L.pyr_off = l == 0 ? 0 : pyr;
        if (l > 0) pyr += (int64_t)L.pitch * L.h;
        L.blur_off = blur;
        blur += (int64_t)L.pitch * L.h;
        if (l > 0) build_resize_tables(P.lv[l - 1].w, P.lv[l - 1].h, L.w, L.h, P, L);
        // ComputeKeyPointsOctTree cell grid, ORBextractor.cc:767-806
        L.minBX = kEdgeThreshold - 3;
        L.minBY = L.minBX;
        L.maxBX = L.w - kEdgeThreshold + 3;
        L.maxBY = L.h - kEdgeThreshold + 3;
        const float Wc = 35;
        const float width = (float)(L.maxBX - L.minBX), height = (float)(L.maxBY - L.minBY);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        if (nCols <= 0 || nRows <= 0) return false;
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        L.cell_begin = (int)P.cells.size();
        int key_cap = 0;
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(L.minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= L.maxBY - 3) continue;
            if (maxY > L.maxBY) maxY = (float)L.maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(L.minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= L.maxBX - 6) continue;
                if (maxX > L.maxBX) maxX = (float)L.maxBX;
                CellDesc c;
                c.level = (int16_t)l;
                c.iniX = (int16_t)iniX;
                c.iniY = (int16_t)iniY;
                c.cw = (int16_t)((int)maxX - (int)iniX);
                c.ch = (int16_t)((int)maxY - (int)iniY);
                c.pad = 0;
                c.slot = (int)P.cells.size();
                P.cells.push_back(c);
                // strict 3x3 NMS keeps at most one corner per 2x2 block of tested pixels
                const int tw = std::max(0, c.cw - 6), th = std::max(0, c.ch - 6);
                const int cap = ((tw + 1) / 2) * ((th + 1) / 2);
                slot_cap = std::max(slot_cap, cap);
                key_cap += cap;
            }
        }
        L.cell_end = (int)P.cells.size();
        L.key_base = key_slots;
        L.key_cap = key_cap;
        key_slots += key_cap;
        L.nfeat = P.nfeat[l];
        L.scale = P.scale[l];
        L.size = (float)(int)(kPatchSize * P.scale[l]);
        // DistributeOctTree roots, ORBextractor.cc:541-561
        const int dX = L.maxBX - L.minBX, dY = L.maxBY - L.minBY;
        const int nIni = (int)std::round((float)dX / dY);
        if (nIni < 1 || nIni > kMaxRoots) return false;
        L.nIni = nIni;
        const float hX = (float)dX / nIni;
        for (int i = 0; i < nIni; i++) {
            L.root_x0[i] = (int)(hX * (float)i);
            L.root_x1[i] = (int)(hX * (float)(i + 1));
            L.root_first_x[i] = 0;
        }
        for (int i = 1; i < nIni; i++) {
            int x = 0;
            while ((int)((float)x / hX) < i) x++;
            L.root_first_x[i] = x;
        }
        // alive nodes never exceed max(N + 3, 4 * nIni) (octree)
        const int nodes = std::max(L.nfeat + 3, 4 * nIni);
        max_nodes = std::max(max_nodes, nodes);
        L.kbase = kslots;
        L.kcap = nodes;
        kslots += nodes;
    }
    P.ncells = (int)P.cells.size();
    P.slot_cap = slot_cap;
    P.kslots = kslots;
    P.key_slots = key_slots;
    P.max_nodes = round_up(max_nodes, 64);
    P.pyr_frame = round_up((int)pyr, 256);
    P.blur_frame = round_up((int)blur, 256);
    return true;
}

}  // namespace slamhot
