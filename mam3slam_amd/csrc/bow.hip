// bow.hip — DBoW2 vocabulary-tree transform on gfx950 + C-ABI (include/mam_bow.h).
//
// Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1216-1259 (transform of one feature: descend from the
// root, at every level the child with the smallest FORB::distance, the first one on ties; record the node at
// level L - levelsup), :1125-1192 (the per-feature loop), FORB::distance = Hamming distance of 32-byte descriptors.
//
// Layout: the children of every node are stored contiguously in file order as 48-byte records {descriptor, the
// child's own child range, node id}, so one level of a descent is one coalesced 48-byte load per lane (a lane per
// child), a group minimum of dist << 8 | position, and no dependent lookup of the chosen child's range.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/mam_bow.h"
#include "runtime.hpp"

namespace mam {
namespace bow {

struct __attribute__((aligned(16))) ChildRec {
    uint4 d0, d1;        // descriptor
    int32_t off, cnt;    // this child's children: records [off, off + cnt) (cnt = 0: a leaf)
    uint32_t node;       // node id
    uint32_t pad;
};

constexpr int GW = 16;   // lanes per feature (the reference's k <= 20: a level with more children loops)

__global__ __launch_bounds__(256) void k_bow_transform(const ChildRec* __restrict__ rec, int root_off, int root_cnt,
                                                       const uint32_t* __restrict__ word, const double* __restrict__ weight,
                                                       int nid_level, const uint8_t* __restrict__ desc, int stride,
                                                       const int32_t* __restrict__ counts, int nframes,
                                                       uint32_t* __restrict__ out_word, double* __restrict__ out_weight,
                                                       uint32_t* __restrict__ out_nid) {
    const long long g = ((long long)blockIdx.x * 256 + threadIdx.x) / GW;   // global feature slot
    const int f = (int)(g / stride);
    const int i = (int)(g - (long long)f * stride);
    if (f >= nframes) return;
    const int n = counts[2 * f];
    if (i >= n) return;   // group-uniform
    const int gl = threadIdx.x & (GW - 1);
    const uint4* D = reinterpret_cast<const uint4*>(desc + ((size_t)f * stride + i) * 32);
    const uint4 a0 = D[0], a1 = D[1];
    int off = root_off, cnt = root_cnt;
    uint32_t node = 0, nid = nid_level <= 0 ? 0u : 0xFFFFFFFFu;
    for (int level = 1; cnt > 0; level++) {
        unsigned best = 0xFFFFFFFFu;
        int boff = 0, bcnt = 0;
        uint32_t bnode = 0;
        for (int c0 = 0; c0 < cnt; c0 += GW) {
            const int c = c0 + gl;
            if (c < cnt) {
                const ChildRec r = rec[off + c];
                const int d = __popc(a0.x ^ r.d0.x) + __popc(a0.y ^ r.d0.y) + __popc(a0.z ^ r.d0.z) +
                              __popc(a0.w ^ r.d0.w) + __popc(a1.x ^ r.d1.x) + __popc(a1.y ^ r.d1.y) +
                              __popc(a1.z ^ r.d1.z) + __popc(a1.w ^ r.d1.w);
                const unsigned key = ((unsigned)d << 8) | (unsigned)c;
                if (key < best) {
                    best = key;
                    boff = r.off;
                    bcnt = r.cnt;
                    bnode = r.node;
                }
            }
        }
#pragma unroll
        for (int o = GW / 2; o >= 1; o >>= 1) {
            const unsigned ob = (unsigned)__shfl_xor((int)best, o, GW);
            const int ooff = __shfl_xor(boff, o, GW), ocnt = __shfl_xor(bcnt, o, GW);
            const uint32_t onode = (uint32_t)__shfl_xor((int)bnode, o, GW);
            if (ob < best) {
                best = ob;
                boff = ooff;
                bcnt = ocnt;
                bnode = onode;
            }
        }
        node = bnode;
        off = boff;
        cnt = bcnt;
        if (level == nid_level) nid = node;
    }
    if (gl == 0) {
        const size_t o = (size_t)f * stride + i;
        out_word[o] = word[node];
        out_weight[o] = weight[node];
        out_nid[o] = nid == 0xFFFFFFFFu ? node : nid;   // leaf shallower than nid_level: unset in the reference
    }
}

}  // namespace bow
}  // namespace mam

struct mam_bow_vocab {
    int device = 0;
    hipStream_t stream = nullptr;
    int k = 0, L = 0, weighting = 0, scoring = 0;
    int n_nodes = 0, n_words = 0;
    int root_off = 0, root_cnt = 0;
    mam::StageTimer timer{1};
    mam::DevBuf<mam::bow::ChildRec> rec;
    mam::DevBuf<uint32_t> word;
    mam::DevBuf<double> weight;
    mam::DevBuf<uint8_t> stage;
};

namespace {

int launch(mam_bow_vocab* v, int F, const uint8_t* desc, int stride, const int32_t* counts, int levelsup,
           uint32_t* ow, double* oweight, uint32_t* onid, hipStream_t s) {
    if (F <= 0 || stride <= 0) return MAM_OK;
    const long long threads = (long long)F * stride * mam::bow::GW;
    mam::StageTimer::Scope sc(&v->timer, s, 0);
    hipLaunchKernelGGL(mam::bow::k_bow_transform, dim3((int)((threads + 255) / 256)), dim3(256), 0, s, v->rec.p,
                       v->root_off, v->root_cnt, v->word.p, v->weight.p, v->L - levelsup, desc, stride, counts, F, ow,
                       oweight, onid);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

size_t carve_bytes(size_t count, size_t elem) { return (count * elem + 255) & ~(size_t)255; }

template <typename T>
T* carve(uint8_t*& p, size_t count) {
    T* r = reinterpret_cast<T*>(p);
    p += carve_bytes(count, sizeof(T));
    return r;
}

}  // namespace

extern "C" {

int mam_bow_create(int device, int k, int L, int weighting, int scoring, int n_nodes, const int32_t* parent,
                   const uint8_t* is_leaf, const uint8_t* desc, const double* weight, mam_bow_vocab** out) {
    if (!out || n_nodes < 1 || (n_nodes > 1 && (!parent || !is_leaf || !desc || !weight))) return MAM_ERR_ARG;
    *out = nullptr;
    for (int i = 1; i < n_nodes; i++)
        if (parent[i] < 0 || parent[i] >= i) {
            mam::set_last_error("vocabulary: every node's parent must precede it (text-file order)");
            return MAM_ERR_ARG;
        }
    int ndev = 0;
    MAM_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) { mam::set_last_error("no such HIP device"); return MAM_ERR_ARG; }
    MAM_DEVICE_SCOPE(device);
    // children in file order (m_nodes[pid].children.push_back(nid)), CSR by parent
    std::vector<int32_t> cnt(n_nodes, 0), off(n_nodes + 1, 0), pos(n_nodes, 0);
    for (int i = 1; i < n_nodes; i++) cnt[parent[i]]++;
    for (int i = 0; i < n_nodes; i++) off[i + 1] = off[i] + cnt[i];
    std::vector<int32_t> fill(off.begin(), off.end() - 1);
    for (int i = 1; i < n_nodes; i++) pos[i] = fill[parent[i]]++;
    std::vector<mam::bow::ChildRec> rec(std::max(n_nodes - 1, 1));
    std::vector<uint32_t> word(n_nodes, 0);
    std::vector<double> w(n_nodes, 0.0);
    int nw = 0;
    for (int i = 1; i < n_nodes; i++) {
        mam::bow::ChildRec& r = rec[pos[i]];
        std::memcpy(&r.d0, desc + (size_t)i * 32, 32);
        r.off = off[i];
        r.cnt = cnt[i];
        r.node = (uint32_t)i;
        r.pad = 0;
        w[i] = weight[i];
        if (is_leaf[i]) word[i] = (uint32_t)nw++;   // word ids in file order
    }
    mam_bow_vocab* v = new mam_bow_vocab();
    v->device = device;
    v->k = k; v->L = L; v->weighting = weighting; v->scoring = scoring;
    v->n_nodes = n_nodes;
    v->n_words = nw;
    v->root_off = off[0];
    v->root_cnt = cnt[0];
    int rc = v->rec.alloc(rec.size());
    if (!rc) rc = v->word.alloc(n_nodes);
    if (!rc) rc = v->weight.alloc(n_nodes);
    if (!rc && hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess) rc = MAM_ERR_DEVICE;
    if (!rc && (hipMemcpy(v->rec.p, rec.data(), rec.size() * sizeof(rec[0]), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(v->word.p, word.data(), word.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(v->weight.p, w.data(), w.size() * 8, hipMemcpyHostToDevice) != hipSuccess))
        rc = MAM_ERR_DEVICE;
    if (rc) {
        if (v->stream) (void)hipStreamDestroy(v->stream);
        delete v;
        return rc;
    }
    *out = v;
    return MAM_OK;
}

void mam_bow_destroy(mam_bow_vocab* v) {
    if (!v) return;
    ::mam::DeviceScope mam_dev_scope_(v->device);
    (void)hipStreamSynchronize(v->stream);
    (void)hipStreamDestroy(v->stream);
    delete v;
}

int mam_bow_words(mam_bow_vocab* v) { return v ? v->n_words : MAM_ERR_ARG; }

int mam_bow_transform_batch_device(mam_bow_vocab* v, int nframes, const uint8_t* desc, int stride,
                                   const int32_t* counts, int levelsup, uint32_t* ow, double* oweight, uint32_t* onid,
                                   void* stream) {
    if (!v || nframes < 0 || stride < 0 || (nframes > 0 && (!desc || !counts || !ow || !oweight || !onid)))
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(v->device);
    return launch(v, nframes, desc, stride, counts, levelsup, ow, oweight, onid,
                  stream ? (hipStream_t)stream : v->stream);
}

int mam_bow_transform(mam_bow_vocab* v, int n, const uint8_t* desc, int levelsup, uint32_t* ow, double* oweight,
                      uint32_t* onid) {
    if (!v || n < 0 || (n > 0 && (!desc || !ow || !oweight || !onid))) return MAM_ERR_ARG;
    if (n == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(v->device);
    const size_t bytes = carve_bytes((size_t)n * 32, 1) + carve_bytes(2, 4) + 2 * carve_bytes(n, 4) + carve_bytes(n, 8);
    if (int rc = v->stage.alloc(bytes)) return rc;
    uint8_t* p = v->stage.p;
    uint8_t* dd = carve<uint8_t>(p, (size_t)n * 32);
    int32_t* dc = carve<int32_t>(p, 2);
    uint32_t* dw = carve<uint32_t>(p, n);
    uint32_t* dn = carve<uint32_t>(p, n);
    double* dwt = carve<double>(p, n);
    const int32_t cnt[2] = {n, 0};
    MAM_HIP(hipMemcpyAsync(dd, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
    MAM_HIP(hipMemcpyAsync(dc, cnt, sizeof(cnt), hipMemcpyHostToDevice, v->stream));
    if (int rc = launch(v, 1, dd, n, dc, levelsup, dw, dwt, dn, v->stream)) return rc;
    MAM_HIP(hipMemcpyAsync(ow, dw, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    MAM_HIP(hipMemcpyAsync(oweight, dwt, (size_t)n * 8, hipMemcpyDeviceToHost, v->stream));
    MAM_HIP(hipMemcpyAsync(onid, dn, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    MAM_HIP(hipStreamSynchronize(v->stream));
    return MAM_OK;
}

int mam_bow_set_profiling(mam_bow_vocab* v, int enable) {
    if (!v) return MAM_ERR_ARG;
    v->timer.reset(enable != 0);
    return MAM_OK;
}

int mam_bow_stage_times(mam_bow_vocab* v, double* ms_out, int64_t* launches_out) {
    if (!v) return MAM_ERR_ARG;
    v->timer.collect();
    if (ms_out) ms_out[0] = v->timer.ms[0];
    if (launches_out) launches_out[0] = v->timer.n[0];
    return MAM_OK;
}

}  // extern "C"
