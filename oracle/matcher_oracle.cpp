/*
 * matcher_oracle.cpp — CPU restatement of the ORB-SLAM3 Hamming matchers and the DBoW2
 * vocabulary descent.  TEST INFRASTRUCTURE ONLY (see oracle.h): checker + CPU baseline.
 *
 * Parity status: restated from the reference sources cited per function; no reference
 * golden vectors exist for this path -> "parity unpinned" against the
 * real reference, pinned by the known-answer tests in tests/test_matcher_oracle.py.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "matcher_oracle.h"

namespace {

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:2561-2577) == FORB::distance (FORB.cpp:81-101)
int hamming(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t wa, wb;
        std::memcpy(&wa, a + 4 * i, 4);
        std::memcpy(&wb, b + 4 * i, 4);
        uint32_t v = wa ^ wb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24;
    }
    return dist;
}

const int TH_HIGH = 100;  // ORBmatcher.cc:36
const int TH_LOW = 50;    // ORBmatcher.cc:37
const int HISTO_LENGTH = 30;

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:2515-2556)
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

// rotation bin of a match (ORBmatcher.cc:391-396): float difference, +360 if negative,
// std::round (half away from zero) of rot * (1.0f/30)
int rot_bin(float a, float b) {
    float rot = a - b;
    if (rot < 0.0) rot += 360.0f;
    const float factor = 1.0f / HISTO_LENGTH;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

}  // namespace

extern "C" {

int oracle_hamming(const uint8_t* a, const uint8_t* b) { return hamming(a, b); }

void oracle_three_maxima(const int32_t* counts, int L, int32_t* ind) {
    std::vector<std::vector<int>> h(L);
    for (int i = 0; i < L; i++) h[i].resize(counts[i]);
    int i1 = -1, i2 = -1, i3 = -1;
    three_maxima(h.data(), L, i1, i2, i3);
    ind[0] = i1;
    ind[1] = i2;
    ind[2] = i3;
}

// TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
// (TemplatedVocabulary.h:1229-1271): descend from the root, at every level take the child
// with the smallest Hamming distance (first child wins ties); record the node reached at
// level L - levelsup.
void oracle_vocab_transform(int L, const int32_t* child_ptr, const int32_t* child_idx,
                            const uint8_t* node_desc, const uint8_t* is_leaf,
                            const int32_t* word_of_node, const double* weight_of_node, int n,
                            const uint8_t* desc, int levelsup, int32_t* word_id, double* weight,
                            int32_t* node_id) {
    const int nid_level = L - levelsup;
    for (int i = 0; i < n; i++) {
        const uint8_t* f = desc + (size_t)i * 32;
        int final_id = 0, level = 0, nid = 0;
        if (nid_level <= 0) nid = 0;
        do {
            ++level;
            const int c0 = child_ptr[final_id], c1 = child_ptr[final_id + 1];
            int best = child_idx[c0];
            int best_d = hamming(f, node_desc + (size_t)best * 32);
            for (int c = c0 + 1; c < c1; c++) {
                const int id = child_idx[c];
                const int d = hamming(f, node_desc + (size_t)id * 32);
                if (d < best_d) {
                    best_d = d;
                    best = id;
                }
            }
            final_id = best;
            if (level == nid_level) nid = final_id;
        } while (!is_leaf[final_id]);
        word_id[i] = word_of_node[final_id];
        weight[i] = weight_of_node[final_id];
        node_id[i] = nid;
    }
}

// TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)'s map building
// (TemplatedVocabulary.h:1139-1206) over the per-feature descent results of oracle_vocab_transform,
// with DBoW2's containers: BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84),
// FeatureVector::addFeature (FeatureVector.cpp:31-45).  weighting: TF_IDF 0, TF 1, IDF 2, BINARY 3;
// scoring: L1_NORM 0, L2_NORM 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4, DOT_PRODUCT 5
// (ScoringObject.h:74-89: all but DOT_PRODUCT normalise, L2 only for L2_NORM).
void oracle_bow_vectors(int n, const int32_t* word_id, const double* weight, const int32_t* node_id,
                        int scoring, int weighting, int* n_words, uint32_t* bow_word, double* bow_value,
                        int* n_nodes, uint32_t* fv_node, int32_t* fv_off, uint32_t* fv_feat) {
    std::map<unsigned int, double> v;
    std::map<unsigned int, std::vector<unsigned int>> fv;
    const bool must = scoring != 5;
    for (int i = 0; i < n; i++) {
        const double w = weight[i];
        if (!(w > 0)) continue;
        const unsigned int id = (unsigned int)word_id[i];
        auto vit = v.lower_bound(id);
        if (weighting == 0 || weighting == 1) {
            if (vit != v.end() && !(id < vit->first)) vit->second += w;
            else v.insert(vit, std::make_pair(id, w));
        } else if (vit == v.end() || id < vit->first) {
            v.insert(vit, std::make_pair(id, w));
        }
        fv[(unsigned int)node_id[i]].push_back((unsigned int)i);
    }
    if ((weighting == 0 || weighting == 1) && !v.empty() && !must) {
        const double nd = v.size();
        for (auto& kv : v) kv.second /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (scoring == 1) {
            for (auto& kv : v) norm += kv.second * kv.second;
            norm = std::sqrt(norm);
        } else {
            for (auto& kv : v) norm += std::fabs(kv.second);
        }
        if (norm > 0.0)
            for (auto& kv : v) kv.second /= norm;
    }
    int j = 0;
    for (auto& kv : v) {
        bow_word[j] = kv.first;
        bow_value[j++] = kv.second;
    }
    *n_words = j;
    int k = 0, f = 0;
    fv_off[0] = 0;
    for (auto& kv : fv) {
        fv_node[k] = kv.first;
        for (unsigned int i : kv.second) fv_feat[f++] = i;
        fv_off[++k] = f;
    }
    *n_nodes = k;
}

// SearchByBoW, both variants (ORBmatcher.cc:269-471 KF-Frame, 823-963 KF-KF), pinhole
// (Nleft == -1, no second camera).  Side A is iterated (the KF / KF1), side B holds the
// candidates (the Frame / KF2).  valid_a / valid_b: MapPoint present and not bad
// (valid_b NULL = every candidate allowed, the Frame case).  strict=0: accept
// bestDist <= TH_LOW (KF-Frame, :373); strict=1: bestDist < TH_LOW (KF-KF, :907).
// Outputs a2b / b2a (-1 = no match); returns the match count.
int oracle_search_by_bow(const slam_bow_side* A, const slam_bow_side* B, float nnratio,
                         int check_ori, int strict, int32_t* a2b, int32_t* b2a) {
    for (int i = 0; i < A->n; i++) a2b[i] = -1;
    for (int i = 0; i < B->n; i++) b2a[i] = -1;
    std::vector<int> rot_hist[HISTO_LENGTH];
    std::vector<int> match_a;  // A index of each accepted match, by histogram slot
    int nmatches = 0;
    int ia = 0, ib = 0;
    while (ia < A->n_nodes && ib < B->n_nodes) {
        if (A->node_id[ia] == B->node_id[ib]) {
            for (int pa = A->node_off[ia]; pa < A->node_off[ia + 1]; pa++) {
                const int idxA = (int)A->node_feat[pa];
                if (A->valid && !A->valid[idxA]) continue;
                const uint8_t* dA = A->desc + (size_t)idxA * 32;
                int best1 = 256, best2 = 256, bestIdx = -1;
                for (int pb = B->node_off[ib]; pb < B->node_off[ib + 1]; pb++) {
                    const int idxB = (int)B->node_feat[pb];
                    if (b2a[idxB] >= 0) continue;  // vpMapPointMatches[idxB] / vbMatched2
                    if (B->valid && !B->valid[idxB]) continue;
                    const int dist = hamming(dA, B->desc + (size_t)idxB * 32);
                    if (dist < best1) {
                        best2 = best1;
                        best1 = dist;
                        bestIdx = idxB;
                    } else if (dist < best2) {
                        best2 = dist;
                    }
                }
                const bool pass = strict ? best1 < TH_LOW : best1 <= TH_LOW;
                if (pass && (float)best1 < nnratio * (float)best2) {
                    a2b[idxA] = bestIdx;
                    b2a[bestIdx] = idxA;
                    if (check_ori) rot_hist[rot_bin(A->angle[idxA], B->angle[bestIdx])].push_back(idxA);
                    nmatches++;
                }
            }
            ia++;
            ib++;
        } else if (A->node_id[ia] < B->node_id[ib]) {
            while (ia < A->n_nodes && A->node_id[ia] < B->node_id[ib]) ia++;  // lower_bound
        } else {
            while (ib < B->n_nodes && B->node_id[ib] < A->node_id[ia]) ib++;
        }
    }
    if (check_ori) {
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima(rot_hist, HISTO_LENGTH, i1, i2, i3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idxA : rot_hist[i]) {
                b2a[a2b[idxA]] = -1;
                a2b[idxA] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}

/* SearchByBoW's rotation bin (ORBmatcher.cc:391-396) for tests/test_fp_sites.py */
int oracle_fp_rot_bin_bow(float a, float b) { return rot_bin(a, b); }

}  // extern "C"
