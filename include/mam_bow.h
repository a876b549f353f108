/*
 * mam_bow.h — C-ABI drop-in boundary for DBoW2's vocabulary-tree transform on gfx950 (MI355X).
 *
 * Replaces (ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>, include/ORBVocabulary.h:29-30):
 *   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
 *                                          reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1216-1259
 *   the per-feature loop of transform(features, BowVector, FeatureVector, levelsup)   :1125-1192
 *   as called by KeyFrame::ComputeBoW / Frame::ComputeBoW (src/KeyFrame.cc:98-107, src/Frame.cc:738-745, levelsup 4).
 *
 * The tree is given as the reference's text vocabulary lists it (loadFromTextFile, :1338-1420): node 0 is the
 * root, nodes 1..n-1 in file order with their parent, leaf flag, 32-byte descriptor and weight; a node's
 * children are in file order; word ids are assigned to leaves in file order.
 *
 * The device computes, per feature, the leaf reached by the descent (first minimum Hamming distance among the
 * children at every level), its word id and weight, and the node at level L - levelsup. Building the BowVector
 * (weights summed per word in feature order, then the scoring's normalisation) and the FeatureVector (features per
 * node, in feature order) is the caller's (MAM3SLAM::ORBVocabulary, mam3slam_amd/bow.py): both are std::map
 * insertions the reference does on the host as well.
 */
#ifndef MAM_BOW_H
#define MAM_BOW_H

#include <stddef.h>
#include <stdint.h>

#include "mam_orb.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mam_bow_vocab mam_bow_vocab;

/* n_nodes includes the root (index 0; parent[0], is_leaf[0], desc row 0 and weight[0] are ignored). parent[i] < i
 * for i >= 1 (the text format's order). k / L / weighting / scoring are the header values (kept for the caller). */
int mam_bow_create(int device, int k, int L, int weighting, int scoring, int n_nodes, const int32_t* parent,
                   const uint8_t* is_leaf, const uint8_t* desc, const double* weight, mam_bow_vocab** out);
void mam_bow_destroy(mam_bow_vocab* voc);
int mam_bow_words(mam_bow_vocab* voc);   /* number of words (leaves) */

/* Per feature i of n (descriptors n x 32, host pointers): out_word[i], out_weight[i] (0 = stopped word: the reference
 * skips the feature), out_nid[i] = the node at level L - levelsup (0 = root when L - levelsup <= 0; the leaf itself if
 * the leaf is shallower, where the reference leaves the value unset). Synchronous. */
int mam_bow_transform(mam_bow_vocab* voc, int n, const uint8_t* desc, int levelsup, uint32_t* out_word,
                      double* out_weight, uint32_t* out_nid);

/* Batched over frames on the device: frame f's descriptors at desc + f*desc_stride*32, count counts[2f] (the
 * extractor's batched layout); outputs at out_* + f*desc_stride. Asynchronous on `stream` (NULL = the vocabulary's). */
int mam_bow_transform_batch_device(mam_bow_vocab* voc, int nframes, const uint8_t* desc, int desc_stride,
                                   const int32_t* counts, int levelsup, uint32_t* out_word, double* out_weight,
                                   uint32_t* out_nid, void* stream);

int mam_bow_set_profiling(mam_bow_vocab* voc, int enable);
int mam_bow_stage_times(mam_bow_vocab* voc, double* ms_out, int64_t* launches_out);   /* [0] transform */

#ifdef __cplusplus
}
#endif
#endif /* MAM_BOW_H */
