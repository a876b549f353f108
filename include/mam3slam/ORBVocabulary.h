/*
 * MAM3SLAM::ORBVocabulary — DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (include/ORBVocabulary.h:29-30 of
 * the reference) for the calls the hot path makes: loadFromTextFile and transform(features, BowVector,
 * FeatureVector, levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1192, 1338-1420). The tree descent of
 * every feature runs on gfx950 (include/mam_bow.h); the maps are built on the host exactly as DBoW2 builds them.
 */
#ifndef MAM3SLAM_ORBVOCABULARY_H
#define MAM3SLAM_ORBVOCABULARY_H

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../mam_bow.h"
#include "Types.h"

namespace MAM3SLAM {

/* DBoW2::BowVector (word id -> value) and DBoW2::FeatureVector (node id -> feature indices), std::map order. */
typedef std::map<unsigned int, double> BowVector;
typedef std::map<unsigned int, std::vector<unsigned int>> FeatureVector;

class ORBVocabulary {
public:
    explicit ORBVocabulary(int device = 0) : mDevice(device) {}
    ~ORBVocabulary();
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;

    /* TemplatedVocabulary.h:1338-1420 (empty lines skipped). false on a malformed file. */
    bool loadFromTextFile(const std::string& filename);
    /* The same tree from arrays (node 0 = root; nodes 1.. in text-file order). */
    void create(int k, int L, int scoring, int weighting, const std::vector<int32_t>& parent,
                const std::vector<uint8_t>& isLeaf, const std::vector<uint8_t>& desc, const std::vector<double>& weight);

    /* transform(features, v, fv, levelsup) for the rows of an N x 32 descriptor matrix. */
    void transform(const Mat8U& features, BowVector& v, FeatureVector& fv, int levelsup) const;

    bool empty() const { return mVoc == nullptr; }
    unsigned int size() const;   /* number of words */
    int getBranchingFactor() const { return mK; }
    int getDepthLevels() const { return mL; }

private:
    int mDevice;
    int mK = 0, mL = 0, mScoring = 0, mWeighting = 0;
    mam_bow_vocab* mVoc = nullptr;
};

}  // namespace MAM3SLAM
#endif
