/* matcher_oracle.h — CPU restatement of the matchers / vocabulary descent.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity unpinned (no reference golden vectors). */
#ifndef SLAMHOT_MATCHER_ORACLE_H
#define SLAMHOT_MATCHER_ORACLE_H
#include <stdint.h>

#include "../include/slamhot.h"

#ifdef __cplusplus
extern "C" {
#endif
int oracle_hamming(const uint8_t* a, const uint8_t* b);
void oracle_three_maxima(const int32_t* counts, int L, int32_t* ind);
void oracle_vocab_transform(int L, const int32_t* child_ptr, const int32_t* child_idx,
                            const uint8_t* node_desc, const uint8_t* is_leaf,
                            const int32_t* word_of_node, const double* weight_of_node, int n,
                            const uint8_t* desc, int levelsup, int32_t* word_id, double* weight,
                            int32_t* node_id);
void oracle_bow_vectors(int n, const int32_t* word_id, const double* weight, const int32_t* node_id,
                        int scoring, int weighting, int* n_words, uint32_t* bow_word, double* bow_value,
                        int* n_nodes, uint32_t* fv_node, int32_t* fv_off, uint32_t* fv_feat);
int oracle_search_by_bow(const slam_bow_side* A, const slam_bow_side* B, float nnratio,
                         int check_ori, int strict, int32_t* a2b, int32_t* b2a);
#ifdef __cplusplus
}
#endif
#endif
