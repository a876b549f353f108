// MAM3SLAM::ORBVocabulary over include/mam_bow.h (see include/mam3slam/ORBVocabulary.h).
#include <cmath>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "mam3slam/ORBVocabulary.h"

namespace MAM3SLAM {

ORBVocabulary::~ORBVocabulary() {
    if (mVoc) mam_bow_destroy(mVoc);
}

void ORBVocabulary::create(int k, int L, int scoring, int weighting, const std::vector<int32_t>& parent,
                           const std::vector<uint8_t>& isLeaf, const std::vector<uint8_t>& desc,
                           const std::vector<double>& weight) {
    if (mVoc) mam_bow_destroy(mVoc);
    mVoc = nullptr;
    mK = k;
    mL = L;
    mScoring = scoring;
    mWeighting = weighting;
    const int rc = mam_bow_create(mDevice, k, L, weighting, scoring, (int)parent.size(), parent.data(), isLeaf.data(),
                                  desc.data(), weight.data(), &mVoc);
    if (rc < 0) throw std::runtime_error(std::string("mam_bow_create failed: ") + mam_last_error());
}

bool ORBVocabulary::loadFromTextFile(const std::string& filename) {
    std::ifstream f(filename);
    if (!f) return false;
    std::string s;
    if (!std::getline(f, s)) return false;
    std::stringstream ss(s);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    ss >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return false;
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    while (std::getline(f, s)) {
        if (s.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream ln(s);
        int pid = 0, isLeaf = 0;
        ln >> pid >> isLeaf;
        if (pid < 0 || pid >= (int)parent.size()) return false;
        parent.push_back(pid);
        leaf.push_back(isLeaf > 0 ? 1 : 0);
        for (int i = 0; i < 32; i++) {
            int v = 0;
            ln >> v;
            desc.push_back((uint8_t)v);
        }
        double w = 0.0;
        ln >> w;
        weight.push_back(w);
    }
    create(k, L, n1, n2, parent, leaf, desc, weight);
    return true;
}

unsigned int ORBVocabulary::size() const { return mVoc ? (unsigned int)mam_bow_words(mVoc) : 0u; }

void ORBVocabulary::transform(const Mat8U& features, BowVector& v, FeatureVector& fv, int levelsup) const {
    // TemplatedVocabulary.h:1125-1192, BowVector.cpp:34-84, FeatureVector.cpp:31-45
    v.clear();
    fv.clear();
    if (!mVoc || features.rows == 0) return;
    const int n = features.rows;
    std::vector<uint32_t> word(n), nid(n);
    std::vector<double> w(n);
    const int rc = mam_bow_transform(mVoc, n, features.data.data(), levelsup, word.data(), w.data(), nid.data());
    if (rc < 0) throw std::runtime_error(std::string("mam_bow_transform failed: ") + mam_last_error());
    const bool tf = mWeighting == 0 || mWeighting == 1;
    const bool must = mScoring != 5;   // every scoring object but DotProduct normalises
    for (int i = 0; i < n; i++) {
        if (!(w[i] > 0)) continue;   // stopped word
        if (tf) {
            auto it = v.lower_bound(word[i]);
            if (it != v.end() && it->first == word[i]) it->second += w[i];
            else v.insert(it, BowVector::value_type(word[i], w[i]));
        } else if (!v.count(word[i])) {
            v.insert(BowVector::value_type(word[i], w[i]));
        }
        fv[nid[i]].push_back((unsigned int)i);
    }
    if (tf && !v.empty() && !must) {
        const double nd = (double)v.size();
        for (auto& e : v) e.second /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (mScoring == 1) {
            for (auto& e : v) norm += e.second * e.second;
            norm = std::sqrt(norm);
        } else {
            for (auto& e : v) norm += std::fabs(e.second);
        }
        if (norm > 0.0)
            for (auto& e : v) e.second /= norm;
    }
}

}  // namespace MAM3SLAM
