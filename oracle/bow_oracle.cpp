// bow_oracle.cpp — TEST INFRASTRUCTURE ONLY (see orb_oracle.h header note).
//
// CPU restatement of DBoW2's vocabulary tree as ORB-SLAM3 uses it (ORBVocabulary, include/ORBVocabulary.h:29-30):
//   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420  loadFromTextFile (node order, children, word ids)
//   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1216-1259  transform(feature, word_id, weight, nid, levelsup)
//   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1192  transform(features, BowVector, FeatureVector, levelsup)
//   Thirdparty/DBoW2/DBoW2/BowVector.cpp:34-84              addWeight / addIfNotExist / normalize
//   Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45          addFeature
//   Thirdparty/DBoW2/DBoW2/FORB.cpp                          distance (Hamming, as double)
// Weighting: TF_IDF 0, TF 1, IDF 2, BINARY 3; scoring: L1_NORM 0, L2_NORM 1, ... DOT_PRODUCT 5 (ScoringObject.h).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

namespace {

struct Node {
    std::vector<int> children;
    uint8_t desc[32];
    double weight = 0.0;
    unsigned word_id = 0;
};

struct Vocab {
    int L = 0, weighting = 0, scoring = 0;
    std::vector<Node> nodes;
};

double forbDistance(const uint8_t* a, const uint8_t* b) {
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(a);
    const uint32_t* pb = reinterpret_cast<const uint32_t*>(b);
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        unsigned int v = pa[i] ^ pb[i];
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

Vocab build(int L, int weighting, int scoring, int n_nodes, const int32_t* parent, const uint8_t* is_leaf,
            const uint8_t* desc, const double* weight) {
    Vocab v;
    v.L = L;
    v.weighting = weighting;
    v.scoring = scoring;
    v.nodes.resize(1);
    unsigned nw = 0;
    for (int nid = 1; nid < n_nodes; nid++) {   // the loader's loop body, one text line per node
        v.nodes.resize(nid + 1);
        v.nodes[parent[nid]].children.push_back(nid);
        std::memcpy(v.nodes[nid].desc, desc + (size_t)nid * 32, 32);
        v.nodes[nid].weight = weight[nid];
        if (is_leaf[nid] > 0) v.nodes[nid].word_id = nw++;
    }
    return v;
}

// transform(feature, word_id, weight, nid, levelsup); nid_set = false where the reference leaves *nid unset
void transformOne(const Vocab& V, const uint8_t* feature, unsigned& word_id, double& weight, unsigned& nid,
                  bool& nid_set, int levelsup) {
    const int nid_level = V.L - levelsup;
    nid_set = false;
    if (nid_level <= 0) { nid = 0; nid_set = true; }
    unsigned final_id = 0;
    int current_level = 0;
    if (V.nodes[0].children.empty()) { word_id = 0; weight = 0.0; return; }
    do {
        ++current_level;
        const std::vector<int>& nodes = V.nodes[final_id].children;
        final_id = nodes[0];
        double best_d = forbDistance(feature, V.nodes[final_id].desc);
        for (size_t k = 1; k < nodes.size(); k++) {
            const double d = forbDistance(feature, V.nodes[nodes[k]].desc);
            if (d < best_d) { best_d = d; final_id = nodes[k]; }
        }
        if (current_level == nid_level) { nid = final_id; nid_set = true; }
    } while (!V.nodes[final_id].children.empty());
    word_id = V.nodes[final_id].word_id;
    weight = V.nodes[final_id].weight;
    if (!nid_set) nid = final_id;
}

}  // namespace

extern "C" {

// Per-feature outputs (as mam_bow_transform), plus the BowVector (words ascending, values) and the FeatureVector
// (node ids ascending, offsets, feature indices) of transform(features, v, fv, levelsup). Capacities: n each.
// Returns the BowVector size; *fv_nodes = the FeatureVector size.
// A built tree kept across calls (bench: the oracle's transform time without the tree build).
void* oracle_bow_build(int L, int weighting, int scoring, int n_nodes, const int32_t* parent, const uint8_t* is_leaf,
                       const uint8_t* vdesc, const double* vweight) {
    return new Vocab(build(L, weighting, scoring, n_nodes, parent, is_leaf, vdesc, vweight));
}

void oracle_bow_free(void* h) { delete static_cast<Vocab*>(h); }

int oracle_bow_run(const void* h, int n, const uint8_t* desc, int levelsup, uint32_t* out_word, double* out_weight,
                   uint32_t* out_nid, uint32_t* bow_words, double* bow_values, uint32_t* fv_ids, int32_t* fv_off,
                   uint32_t* fv_feats, int* fv_nodes) {
    const Vocab& V = *static_cast<const Vocab*>(h);
    const int weighting = V.weighting, scoring = V.scoring;
    std::map<unsigned, double> bow;
    std::map<unsigned, std::vector<unsigned>> fv;
    const bool must = scoring != 5;   // mustNormalize: every scoring but DOT_PRODUCT; L2_NORM with L2, else L1
    for (int i = 0; i < n; i++) {
        unsigned id = 0, nid = 0;
        double w = 0.0;
        bool set = false;
        transformOne(V, desc + (size_t)i * 32, id, w, nid, set, levelsup);
        out_word[i] = id;
        out_weight[i] = w;
        out_nid[i] = nid;
        if (!(w > 0)) continue;   // stopped word
        if (weighting == 0 || weighting == 1) {
            auto it = bow.lower_bound(id);
            if (it != bow.end() && it->first == id) it->second += w;
            else bow.insert(it, {id, w});
        } else {
            if (!bow.count(id)) bow.insert({id, w});
        }
        fv[nid].push_back((unsigned)i);
    }
    if ((weighting == 0 || weighting == 1) && !bow.empty() && !must) {
        const double nd = (double)bow.size();
        for (auto& e : bow) e.second /= nd;
    }
    if (must) {   // BowVector::normalize
        double norm = 0.0;
        if (scoring == 1) {
            for (auto& e : bow) norm += e.second * e.second;
            norm = std::sqrt(norm);
        } else {
            for (auto& e : bow) norm += std::fabs(e.second);
        }
        if (norm > 0.0)
            for (auto& e : bow) e.second /= norm;
    }
    int k = 0;
    for (auto& e : bow) { bow_words[k] = e.first; bow_values[k] = e.second; k++; }
    int m = 0, f = 0;
    fv_off[0] = 0;
    for (auto& e : fv) {
        fv_ids[m] = e.first;
        for (unsigned x : e.second) fv_feats[f++] = x;
        fv_off[++m] = f;
    }
    *fv_nodes = m;
    return k;
}

int oracle_bow_transform(int L, int weighting, int scoring, int n_nodes, const int32_t* parent, const uint8_t* is_leaf,
                         const uint8_t* vdesc, const double* vweight, int n, const uint8_t* desc, int levelsup,
                         uint32_t* out_word, double* out_weight, uint32_t* out_nid, uint32_t* bow_words,
                         double* bow_values, uint32_t* fv_ids, int32_t* fv_off, uint32_t* fv_feats, int* fv_nodes) {
    const Vocab V = build(L, weighting, scoring, n_nodes, parent, is_leaf, vdesc, vweight);
    return oracle_bow_run(&V, n, desc, levelsup, out_word, out_weight, out_nid, bow_words, bow_values, fv_ids, fv_off,
                          fv_feats, fv_nodes);
}

}  // extern "C"
