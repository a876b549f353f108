// Shared-map update exchange: each agent packs the deduplicated write-back of its step's LocalBundleAdjustment windows
// into one compact block, and every agent applies the all-gathered blocks in agent order (include/mam_exchange.h,
// SURVEY.md §8(e)); plus the windows' vertex estimates read from the shared tables.
// Reference semantics of the values: src/Optimizer.cc:1478-1494 (KeyFrame::SetPose(SE3f(q.cast<float>,
// t.cast<float>)), MapPoint::SetWorldPos(pos.cast<float>)).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/mam_exchange.h"
#include "../../include/mam_orb.h"
#include "runtime.hpp"

namespace mam {

// grid (ceil(max(P, L) / 256), n_windows): the window's vertex estimates from the shared tables, the float map values
// cast to double as the reference builds its graph (Optimizer.cc:1218, 1235: SE3Quat(GetPose().unit_quaternion()
// .cast<double>(), translation().cast<double>()); :1286: GetWorldPos().cast<double>())
__global__ __launch_bounds__(256) void k_read_windows(const float* __restrict__ kf, int64_t kf_cap,
                                                      const float* __restrict__ mp, int64_t mp_cap, int64_t mp_id_base,
                                                      const mam_map_window* __restrict__ win,
                                                      int32_t* __restrict__ status) {
    const mam_map_window& w = win[blockIdx.y];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < w.n_poses) {
        const int64_t id = w.pose_id[i];
        if (id < 0 || id >= kf_cap) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            const float* s = kf + id * 8;
            for (int k = 0; k < 4; k++) w.pose_q[4 * (size_t)i + k] = (double)s[k];
            for (int k = 0; k < 3; k++) w.pose_t[3 * (size_t)i + k] = (double)s[4 + k];
        }
    }
    if (i < w.n_points) {
        const int64_t r = w.point_id[i] - mp_id_base;
        if (r < 0 || r >= mp_cap) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            for (int k = 0; k < 3; k++) w.point_xyz[3 * (size_t)i + k] = (double)mp[r * 4 + k];
        }
    }
}

// ---- compact blocks: one per agent, the deduplicated write-back of all its windows (mam_exchange_pack_sources)
__host__ __device__ inline size_t compact_block_bytes(int kf_cap, int mp_cap) {
    return sizeof(mam_update_header) + (size_t)kf_cap * sizeof(mam_kf_update) + (size_t)mp_cap * sizeof(mam_mp_update);
}

// grid (ceil(max(n_kf, n_mp) / 256)): record i of each list from its source (window, vertex index)
__global__ __launch_bounds__(256) void k_pack_sources(const mam_map_window* __restrict__ win,
                                                      const int32_t* __restrict__ kf_src, int n_kf,
                                                      const int32_t* __restrict__ mp_src, int n_mp, int64_t mp_id_base,
                                                      int agent, uint8_t* __restrict__ block, int kf_cap, int mp_cap) {
    mam_update_header* h = reinterpret_cast<mam_update_header*>(block);
    mam_kf_update* K = reinterpret_cast<mam_kf_update*>(block + sizeof(mam_update_header));
    mam_mp_update* M = reinterpret_cast<mam_mp_update*>(block + sizeof(mam_update_header) +
                                                        (size_t)kf_cap * sizeof(mam_kf_update));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        mam_update_header hh;
        hh.n_kf = n_kf;
        hh.n_mp = n_mp;
        hh.agent = agent;
        hh.status = (n_kf > kf_cap || n_mp > mp_cap) ? MAM_ERR_CAPACITY : 0;
        *h = hh;
    }
    if (i < n_kf && i < kf_cap) {
        const mam_map_window& w = win[kf_src[2 * i]];
        const int v = kf_src[2 * i + 1];
        mam_kf_update u;
        u.row = (int32_t)w.pose_id[v];
        // KeyFrame::SetPose(SE3f(q.cast<float>(), t.cast<float>())) (Optimizer.cc:1478-1486): Sophus normalises the
        // float quaternion, coeffs / norm() with the norm as Eigen's SSE packet reduction sums the 4 floats,
        // (x^2 + z^2) + (y^2 + w^2) — the same order as Frame::SetPose in pose.hip
        float q[4];
        for (int k = 0; k < 4; k++) q[k] = (float)w.pose_q[4 * (size_t)v + k];
        const float nq = sqrtf((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
        for (int k = 0; k < 4; k++) u.q[k] = q[k] / nq;
        for (int k = 0; k < 3; k++) u.t[k] = (float)w.pose_t[3 * (size_t)v + k];
        K[i] = u;
    }
    if (i < n_mp && i < mp_cap) {
        const mam_map_window& w = win[mp_src[2 * i]];
        const int v = mp_src[2 * i + 1];
        mam_mp_update u;
        const int32_t row = (int32_t)(w.point_id[v] - mp_id_base);
        u.row = (w.point_bad && w.point_bad[v]) ? (int32_t)((uint32_t)row | 0x80000000u) : row;
        for (int k = 0; k < 3; k++) u.xyz[k] = (float)w.point_xyz[3 * (size_t)v + k];   // SetWorldPos(pos.cast<float>())
        M[i] = u;
    }
}

// one agent's compact block (launched per agent, in agent order); rows within a block are unique
__global__ __launch_bounds__(256) void k_apply_compact(const uint8_t* __restrict__ block, int kf_cap, int mp_cap,
                                                       float* __restrict__ kf, int64_t kf_rows, float* __restrict__ mp,
                                                       int64_t mp_rows, int32_t* __restrict__ status) {
    const mam_update_header h = *reinterpret_cast<const mam_update_header*>(block);
    if (h.status != 0 || h.n_kf < 0 || h.n_kf > kf_cap || h.n_mp < 0 || h.n_mp > mp_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(status, MAM_ERR_ARG);
        return;
    }
    const mam_kf_update* K = reinterpret_cast<const mam_kf_update*>(block + sizeof(mam_update_header));
    const mam_mp_update* M = reinterpret_cast<const mam_mp_update*>(block + sizeof(mam_update_header) +
                                                                    (size_t)kf_cap * sizeof(mam_kf_update));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < h.n_kf) {
        const mam_kf_update u = K[i];
        if (u.row >= 0 && u.row < kf_rows) {
            float* d = kf + (size_t)u.row * 8;
            for (int k = 0; k < 4; k++) d[k] = u.q[k];
            for (int k = 0; k < 3; k++) d[4 + k] = u.t[k];
            d[7] = 1.0f;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
    if (i < h.n_mp) {
        const mam_mp_update u = M[i];
        const int32_t row = (int32_t)((uint32_t)u.row & 0x7fffffffu);
        if (row < mp_rows) {
            float* d = mp + (size_t)row * 4;
            for (int k = 0; k < 3; k++) d[k] = u.xyz[k];
            d[3] = ((uint32_t)u.row & 0x80000000u) ? 1.0f : 0.0f;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
}

// ---- harness helpers
struct RowCopyArgs {
    int n_tables, n;
    mam_row_table t[8];
    int32_t src[64], dst[64];
    const int32_t* fa;
    const int32_t* fb;
    int64_t f_stride;
    int f_cols;
    uint8_t* flags;
    int64_t flags_stride;
};

// grid (n, n_tables + 1) x 256: block (i, k) copies row i of table k (16-byte chunks when the row and both addresses
// allow, else bytes); k = n_tables: the flags of row i
__global__ __launch_bounds__(256) void k_copy_rows(const RowCopyArgs a) {
    const int i = blockIdx.x, k = blockIdx.y;
    if (k < a.n_tables) {
        const mam_row_table& t = a.t[k];
        const uint8_t* s = reinterpret_cast<const uint8_t*>(t.src) + (t.src_row_offset + a.src[i]) * t.src_stride;
        uint8_t* d = reinterpret_cast<uint8_t*>(t.dst) + (int64_t)a.dst[i] * t.dst_stride;
        if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)t.row_bytes) & 15) == 0) {
            const int64_t nv = t.row_bytes / 16;
            for (int64_t j = threadIdx.x; j < nv; j += 256)
                reinterpret_cast<uint4*>(d)[j] = reinterpret_cast<const uint4*>(s)[j];
        } else {
            for (int64_t j = threadIdx.x; j < t.row_bytes; j += 256) d[j] = s[j];
        }
    } else if (a.flags) {
        const int32_t* x = a.fa + (int64_t)a.src[i] * a.f_stride;
        const int32_t* y = a.fb + (int64_t)a.src[i] * a.f_stride;
        uint8_t* f = a.flags + (int64_t)a.dst[i] * a.flags_stride;
        for (int j = threadIdx.x; j < a.f_cols; j += 256) f[j] = (x[j] >= 0 || y[j] >= 0) ? 1 : 0;
    }
}

// counter-based standard normal (splitmix64 -> two uniforms -> Box-Muller)
__device__ inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ inline float normal_at(uint64_t seed, uint64_t ctr) {
    const uint64_t r = splitmix64(seed ^ splitmix64(ctr));
    const float u1 = ((uint32_t)(r >> 40) + 1u) * (1.0f / 16777217.0f);   // (0, 1]
    const float u2 = (uint32_t)(r & 0xffffffu) * (1.0f / 16777216.0f);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// grid ceil(max(n_kf, n_mp) / 256) x 256
__global__ __launch_bounds__(256) void k_perturb(float* __restrict__ kf, int64_t kf_rows, const int64_t* __restrict__ kf_idx,
                                                 int n_kf, float* __restrict__ mp, int64_t mp_rows,
                                                 const int64_t* __restrict__ mp_idx, int n_mp, uint64_t seed, float sq,
                                                 float st, float sx, int32_t* __restrict__ status) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_kf) {
        const int64_t r = kf_idx[i];
        if (r < 0 || r >= kf_rows) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            float* v = kf + r * 8;
            float q[4];
            for (int k = 0; k < 4; k++) q[k] = v[k] + sq * normal_at(seed, 16 * (uint64_t)i + k);
            const float nrm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            const float sg = q[3] < 0.0f ? -1.0f : 1.0f;
            for (int k = 0; k < 4; k++) v[k] = sg * (q[k] / nrm);
            for (int k = 0; k < 3; k++) v[4 + k] += st * normal_at(seed, 16 * (uint64_t)i + 4 + k);
        }
    }
    if (i < n_mp) {
        const int64_t r = mp_idx[i];
        if (r < 0 || r >= mp_rows) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            for (int k = 0; k < 3; k++) mp[r * 4 + k] += sx * normal_at(seed ^ 0x5bd1e995ull, 4 * (uint64_t)i + k);
        }
    }
}

// ---- LBA windows from the keyframe ring: grid (ceil(S / 64), n_windows) x 64, one thread per MapPoint (its nn + 1
// edge slots, the poses by the first threads of each window)
struct RingArgs {
    const int32_t* pairs;
    int nn, n_fixed, S, nlevels;
    const mam_keypoint* keys;
    const int32_t* cnt;
    const float* tcw;    // [R][7]: q xyzw, t
    const float* mps;    // [R][S][20] (mam_fuse_mp: pos first)
    const int32_t* match;
    float inv_s2[8];
    const mam_ring_window* outs;
};

__global__ __launch_bounds__(64) void k_ring_windows(const RingArgs a) {
    const int w = blockIdx.y, p = blockIdx.x * 64 + threadIdx.x;
    const mam_ring_window& o = a.outs[w];
    const int NV = a.nn + 1;
    const int j = a.pairs[2 * (w * a.nn)];
    if (p < NV) {
        const int slot = p == 0 ? j : a.pairs[2 * (w * a.nn + p - 1) + 1];
        const float* T = a.tcw + 7 * (size_t)slot;
        for (int k = 0; k < 4; k++) o.pose_q[4 * p + k] = (double)T[k];
        for (int k = 0; k < 3; k++) o.pose_t[3 * p + k] = (double)T[4 + k];
        o.pose_fixed[p] = p >= NV - a.n_fixed ? 1 : 0;
    }
    if (p >= a.S) return;
    const int n = min(max(a.cnt[2 * j], 0), a.S);
    const bool valid = p < n;
    const float* M = a.mps + ((size_t)j * a.S + p) * 20;
    for (int k = 0; k < 3; k++) o.point_xyz[3 * (size_t)p + k] = valid ? (double)M[k] : 0.0;
    // the observations: count first (a MapPoint seen by fewer than two keyframes is left out), then the slots
    int nobs = valid ? 1 : 0;
    if (valid)
        for (int k = 0; k < a.nn; k++) {
            const int nb = a.pairs[2 * (w * a.nn + k) + 1];
            const int idx = a.match[(size_t)(w * a.nn + k) * a.S + p];
            nobs += (idx >= 0 && idx < min(a.cnt[2 * nb], a.S)) ? 1 : 0;
        }
    const bool keep = nobs >= 2;
    for (int v = 0; v < NV; v++) {
        const size_t e = (size_t)p * NV + v;
        int slot = j, idx = p;
        if (v > 0) {
            slot = a.pairs[2 * (w * a.nn + v - 1) + 1];
            idx = valid ? a.match[(size_t)(w * a.nn + v - 1) * a.S + p] : -1;
            if (idx >= min(a.cnt[2 * slot], a.S)) idx = -1;
        } else if (!valid) {
            idx = -1;
        }
        const bool act = keep && idx >= 0;
        o.edge_point[e] = p;
        o.edge_pose[e] = v;
        o.edge_active[e] = act ? 1 : 0;
        if (act) {
            const mam_keypoint& kp = a.keys[(size_t)slot * a.S + idx];
            o.edge_obs[2 * e] = (double)kp.x;
            o.edge_obs[2 * e + 1] = (double)kp.y;
            o.edge_inv_sigma2[e] = (double)a.inv_s2[min(max(kp.octave, 0), a.nlevels - 1)];
        } else {
            o.edge_obs[2 * e] = 0.0;
            o.edge_obs[2 * e + 1] = 0.0;
            o.edge_inv_sigma2[e] = 1.0;
        }
    }
}

// ---- LBA windows by the reference's window rule, compacted: grid (n_windows) x 256, one workgroup per window.
// Optimizer::LocalBundleAdjustment (Optimizer.cc:1118-1186): the local keyframes are the new keyframe and its
// covisible keyframes (GetVectorCovisibleKeyFrames: the connections KeyFrame::UpdateConnections keeps, weight = shared
// MapPoints >= 15, or the heaviest one when none reaches it, KeyFrame.cc:312-380), the local MapPoints those the new
// keyframe observes (the ring's MapPoints are the new keyframe's; a point seen by fewer than two keyframes is left
// out, as the fixed-shape form did), the fixed keyframes every other keyframe observing a local MapPoint. Poses: the
// new keyframe, its covisible keyframes by weight, then the fixed ones; points in keypoint order; edges
// point-major (the new keyframe's observation first, then the neighbours' in neighbour order) — only real
// observations, no inactive slots. counts[w] = {poses, points, edges, optimised poses}; pose_slot[w][i] the ring slot
// of pose i, point_src[w][i] the keypoint (MapPoint row of the new keyframe) of point i.
constexpr int RINGC_T = 256;
__device__ __forceinline__ int ringc_excl_scan(int v, int* wsum, int& total) {
    // block exclusive scan of RINGC_T values (wave inclusive scans by shuffle, then the wave totals)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(x, o, 64);
        if (lane >= o) x += u;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int pre = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < RINGC_T / 64; w++) {
        const int t = wsum[w];
        if (w < wid) pre += t;
        total += t;
    }
    __syncthreads();
    return pre + x - v;
}

__global__ __launch_bounds__(RINGC_T) void k_ring_windows_covis(const RingArgs a, int covis_th, int n_fixed,
                                                                int32_t* counts, int32_t* pose_slot,
                                                                int32_t* point_src) {
    extern __shared__ __attribute__((aligned(16))) uint32_t obsm[];   // [S]: bit k = observed by neighbour k
    __shared__ int wt[32], vpose[33], wsum[RINGC_T / 64], carry[2], hdr[4];
    const int w = blockIdx.x, t = threadIdx.x, nn = a.nn, S = a.S;
    int* claim = reinterpret_cast<int*>(obsm + S);                    // [S]: a neighbour keypoint's first claimant
    const mam_ring_window& o = a.outs[w];
    const int j = a.pairs[2 * (w * nn)];
    const int n = min(max(a.cnt[2 * j], 0), S);
    if (t < 32) wt[t] = 0;
    // observation masks: the forward Fuse matches of the new keyframe's MapPoints in each neighbour
    for (int p = t; p < S; p += RINGC_T) {
        uint32_t m = 0;
        if (p < n)
            for (int k = 0; k < nn; k++) {
                const int nb = a.pairs[2 * (w * nn + k) + 1];
                const int idx = a.match[(size_t)(w * nn + k) * S + p];
                if (idx >= 0 && idx < min(a.cnt[2 * nb], S)) m |= 1u << k;
            }
        obsm[p] = m;
    }
    // one MapPoint per neighbour keypoint: when two of the keyframe's MapPoints claim the same keypoint of a
    // neighbour, the reference's Fuse merges them (ORBmatcher.cc:1014-1122: the second finds the keypoint taken and
    // Replace()s one by the other); here the first claimant (lowest MapPoint index) keeps the observation and the later
    // claims are dropped
    for (int k = 0; k < nn; k++) {
        for (int q = t; q < S; q += RINGC_T) claim[q] = INT_MAX;
        __syncthreads();
        for (int p = t; p < n; p += RINGC_T)
            if ((obsm[p] >> k) & 1u) atomicMin(&claim[a.match[(size_t)(w * nn + k) * S + p]], p);
        __syncthreads();
        for (int p = t; p < n; p += RINGC_T)
            if (((obsm[p] >> k) & 1u) && claim[a.match[(size_t)(w * nn + k) * S + p]] != p) obsm[p] &= ~(1u << k);
        __syncthreads();
    }
    // the covisibility weights (shared MapPoints per neighbour)
    for (int p0 = 0; p0 < S; p0 += RINGC_T) {   // (uniform trip count: the ballots need every lane)
        const int p = p0 + t;
        const uint32_t m = p < S ? obsm[p] : 0u;
        for (int k = 0; k < nn; k++) {
            const int c = __popcll(__ballot((m >> k) & 1u));
            if ((t & 63) == 0 && c) atomicAdd(&wt[k], c);
        }
    }
    __syncthreads();
    // the window's keyframes (thread 0, <= 31 neighbours): the neighbours by covisibility weight, heaviest first (ties
    // by neighbour order: GetVectorCovisibleKeyFrames' order), the covisible ones (>= covis_th, or the heaviest when none
    // reaches it) local, the other observers fixed; with no fixed keyframe left the reference skips the LBA
    // (Optimizer.cc:1179-1183) — here the n_fixed least covisible local ones are fixed instead, the gauge anchor the
    // fixed cameras are
    if (t == 0) {
        int ord[32];
        int no = 0;
        for (int k = 0; k < nn; k++) {
            if (wt[k] <= 0) continue;
            int i = no++;
            while (i > 0 && wt[ord[i - 1]] < wt[k]) { ord[i] = ord[i - 1]; i--; }
            ord[i] = k;
        }
        int nloc = 0;
        while (nloc < no && wt[ord[nloc]] >= covis_th) nloc++;
        if (nloc == 0 && no > 0) nloc = 1;
        if (nloc == no) nloc = max(no - n_fixed, min(no, 1));
        for (int k = 0; k <= nn; k++) vpose[k] = -1;
        vpose[0] = 0;
        for (int i = 0; i < no; i++) vpose[1 + ord[i]] = 1 + i;
        hdr[0] = 1 + no;
        hdr[1] = 1 + nloc;
    }
    __syncthreads();
    const int np = hdr[0], nopt = hdr[1];
    if (t <= nn) {
        const int v = t, pi = vpose[v];
        if (pi >= 0) {
            const int slot = v == 0 ? j : a.pairs[2 * (w * nn + v - 1) + 1];
            const float* T = a.tcw + 7 * (size_t)slot;
            for (int k = 0; k < 4; k++) o.pose_q[4 * pi + k] = (double)T[k];
            for (int k = 0; k < 3; k++) o.pose_t[3 * pi + k] = (double)T[4 + k];
            o.pose_fixed[pi] = pi >= nopt ? 1 : 0;
            pose_slot[(size_t)w * (nn + 1) + pi] = slot;
        }
    }
    // points (kept: observed by the new keyframe and at least one neighbour) and their edges, compacted in order
    if (t == 0) { carry[0] = 0; carry[1] = 0; }
    __syncthreads();
    for (int p0 = 0; p0 < S; p0 += RINGC_T) {
        const int p = p0 + t;
        const uint32_t m = p < S ? obsm[p] : 0u;
        const bool keep = m != 0;
        const int ne = keep ? 1 + __popc(m) : 0;
        int tp, te;
        const int pi = ringc_excl_scan(keep ? 1 : 0, wsum, tp) + carry[0];
        const int e0 = ringc_excl_scan(ne, wsum, te) + carry[1];
        if (keep) {
            const float* M = a.mps + ((size_t)j * S + p) * 20;
            for (int k = 0; k < 3; k++) o.point_xyz[3 * (size_t)pi + k] = (double)M[k];
            point_src[(size_t)w * S + pi] = p;
            int e = e0;
            for (int v = 0; v <= nn; v++) {
                if (v > 0 && !((m >> (v - 1)) & 1u)) continue;
                const int slot = v == 0 ? j : a.pairs[2 * (w * nn + v - 1) + 1];
                const int idx = v == 0 ? p : a.match[(size_t)(w * nn + v - 1) * S + p];
                const mam_keypoint& kp = a.keys[(size_t)slot * S + idx];
                o.edge_point[e] = pi;
                o.edge_pose[e] = vpose[v];
                o.edge_obs[2 * (size_t)e] = (double)kp.x;
                o.edge_obs[2 * (size_t)e + 1] = (double)kp.y;
                o.edge_inv_sigma2[e] = (double)a.inv_s2[min(max(kp.octave, 0), a.nlevels - 1)];
                if (o.edge_active) o.edge_active[e] = 1;
                e++;
            }
        }
        __syncthreads();
        if (t == 0) { carry[0] += tp; carry[1] += te; }
        __syncthreads();
    }
    if (t == 0) {
        counts[4 * w] = np;
        counts[4 * w + 1] = carry[0];
        counts[4 * w + 2] = carry[1];
        counts[4 * w + 3] = nopt;
    }
}

}  // namespace mam

extern "C" int mam_ring_lba_windows(int n_windows, const int32_t* pairs, int nn, int n_fixed, const void* keys,
                                    const int32_t* cnt, const void* tcw, const void* mps, int S, const int32_t* match,
                                    const float* inv_level_sigma2, int nlevels, const mam_ring_window* outs,
                                    void* stream) {
    if (n_windows < 0 || nn < 1 || n_fixed < 0 || n_fixed > nn || S < 1 || nlevels < 1 || nlevels > 8 || !pairs ||
        !keys || !cnt || !tcw || !mps || !match || !inv_level_sigma2 || (n_windows > 0 && !outs))
        return MAM_ERR_ARG;
    if (n_windows == 0) return MAM_OK;
    mam::RingArgs a{};
    a.pairs = pairs;
    a.nn = nn;
    a.n_fixed = n_fixed;
    a.S = S;
    a.nlevels = nlevels;
    a.keys = reinterpret_cast<const mam_keypoint*>(keys);
    a.cnt = cnt;
    a.tcw = reinterpret_cast<const float*>(tcw);
    a.mps = reinterpret_cast<const float*>(mps);
    a.match = match;
    for (int l = 0; l < nlevels; l++) a.inv_s2[l] = inv_level_sigma2[l];
    a.outs = outs;
    const int np = std::max(S, nn + 1);
    hipLaunchKernelGGL(mam::k_ring_windows, dim3((np + 63) / 64, n_windows), dim3(64), 0, (hipStream_t)stream, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ring_lba_windows_covis(int n_windows, const int32_t* pairs, int nn, int covis_th, int n_fixed,
                                          const void* keys,
                                          const int32_t* cnt, const void* tcw, const void* mps, int S,
                                          const int32_t* match, const float* inv_level_sigma2, int nlevels,
                                          const mam_ring_window* outs, int32_t* counts, int32_t* pose_slot,
                                          int32_t* point_src, void* stream) {
    if (n_windows < 0 || nn < 1 || nn > 31 || n_fixed < 0 || S < 1 || nlevels < 1 || nlevels > 8 || !pairs || !keys ||
        !cnt || !tcw ||
        !mps || !match || !inv_level_sigma2 || (n_windows > 0 && (!outs || !counts || !pose_slot || !point_src)))
        return MAM_ERR_ARG;
    if ((size_t)S * 8 > 64 * 1024) return MAM_ERR_CAPACITY;
    if (n_windows == 0) return MAM_OK;
    mam::RingArgs a{};
    a.pairs = pairs;
    a.nn = nn;
    a.n_fixed = 0;
    a.S = S;
    a.nlevels = nlevels;
    a.keys = reinterpret_cast<const mam_keypoint*>(keys);
    a.cnt = cnt;
    a.tcw = reinterpret_cast<const float*>(tcw);
    a.mps = reinterpret_cast<const float*>(mps);
    a.match = match;
    for (int l = 0; l < nlevels; l++) a.inv_s2[l] = inv_level_sigma2[l];
    a.outs = outs;
    hipLaunchKernelGGL(mam::k_ring_windows_covis, dim3(n_windows), dim3(mam::RINGC_T), (size_t)S * 8,
                       (hipStream_t)stream, a, covis_th, n_fixed, counts, pose_slot, point_src);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_copy_rows(int n_tables, const mam_row_table* tables, int n, const int32_t* src_rows,
                             const int32_t* dst_rows, const int32_t* flag_a, const int32_t* flag_b, int64_t flag_stride,
                             int flag_cols, uint8_t* flags, int64_t flags_stride, void* stream) {
    if (n_tables < 0 || n < 0 || (n_tables > 0 && !tables) || (n > 0 && (!src_rows || !dst_rows)) ||
        (flags && (!flag_a || !flag_b || flag_cols < 0)))
        return MAM_ERR_ARG;
    if (n_tables > 8 || n > 64) return MAM_ERR_CAPACITY;
    if (n == 0 || (n_tables == 0 && !flags)) return MAM_OK;
    mam::RowCopyArgs a{};
    a.n_tables = n_tables;
    a.n = n;
    for (int k = 0; k < n_tables; k++) {
        if (tables[k].row_bytes < 0 || (tables[k].row_bytes > 0 && (!tables[k].src || !tables[k].dst))) return MAM_ERR_ARG;
        a.t[k] = tables[k];
    }
    for (int i = 0; i < n; i++) {
        a.src[i] = src_rows[i];
        a.dst[i] = dst_rows[i];
    }
    a.fa = flag_a;
    a.fb = flag_b;
    a.f_stride = flag_stride;
    a.f_cols = flag_cols;
    a.flags = flags;
    a.flags_stride = flags_stride;
    hipLaunchKernelGGL(mam::k_copy_rows, dim3(n, n_tables + (flags ? 1 : 0)), dim3(256), 0, (hipStream_t)stream, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_map_perturb(float* kf_table, int64_t kf_rows, const int64_t* kf_idx, int n_kf, float* mp_table,
                               int64_t mp_rows, const int64_t* mp_idx, int n_mp, uint64_t seed, float sigma_q,
                               float sigma_t, float sigma_x, int32_t* status, void* stream) {
    if (n_kf < 0 || n_mp < 0 || !status || (n_kf > 0 && (!kf_table || !kf_idx)) || (n_mp > 0 && (!mp_table || !mp_idx)))
        return MAM_ERR_ARG;
    const int n = std::max(n_kf, n_mp);
    if (n == 0) return MAM_OK;
    hipLaunchKernelGGL(mam::k_perturb, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, kf_table, kf_rows,
                       kf_idx, n_kf, mp_table, mp_rows, mp_idx, n_mp, (uint64_t)seed, sigma_q, sigma_t, sigma_x, status);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" size_t mam_exchange_compact_block_bytes(int kf_cap, int mp_cap) {
    return (kf_cap < 0 || mp_cap < 0) ? 0 : mam::compact_block_bytes(kf_cap, mp_cap);
}

extern "C" int mam_exchange_pack_sources(int n_windows, const mam_map_window* windows, const int32_t* kf_src, int n_kf,
                                         const int32_t* mp_src, int n_mp, int64_t mp_id_base, int agent, void* block,
                                         int kf_cap, int mp_cap, void* stream) {
    if (n_windows < 0 || n_kf < 0 || n_mp < 0 || kf_cap < 0 || mp_cap < 0 || !block ||
        ((n_kf || n_mp) && (!windows || n_windows == 0)) || (n_kf && !kf_src) || (n_mp && !mp_src))
        return MAM_ERR_ARG;
    if (n_kf > kf_cap || n_mp > mp_cap) return MAM_ERR_CAPACITY;
    const int n = std::max(1, std::max(n_kf, n_mp));
    hipLaunchKernelGGL(mam::k_pack_sources, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, windows, kf_src,
                       n_kf, mp_src, n_mp, mp_id_base, agent, reinterpret_cast<uint8_t*>(block), kf_cap, mp_cap);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_exchange_apply_compact(const void* gathered, int n_agents, int kf_cap, int mp_cap,
                                          float* kf_table, int64_t kf_rows, float* mp_table, int64_t mp_rows,
                                          int32_t* status, void* stream) {
    if (!gathered || n_agents < 1 || kf_cap < 0 || mp_cap < 0 || !kf_table || !mp_table || !status) return MAM_ERR_ARG;
    const size_t bb = mam::compact_block_bytes(kf_cap, mp_cap);
    const int n = std::max(1, std::max(kf_cap, mp_cap));
    for (int a = 0; a < n_agents; a++) {
        hipLaunchKernelGGL(mam::k_apply_compact, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const uint8_t*>(gathered) + (size_t)a * bb, kf_cap, mp_cap, kf_table,
                           kf_rows, mp_table, mp_rows, status);
        MAM_HIP(hipGetLastError());
    }
    return MAM_OK;
}

extern "C" int mam_map_read_windows(const float* kf_table, int64_t kf_cap, const float* mp_table, int64_t mp_cap,
                                    int64_t mp_id_base, int n_windows, const mam_map_window* windows, int max_rows,
                                    int32_t* status, void* stream) {
    if (!kf_table || !mp_table || !status || n_windows < 0 || max_rows < 0 || (n_windows > 0 && !windows))
        return MAM_ERR_ARG;
    if (n_windows == 0 || max_rows == 0) return MAM_OK;
    hipLaunchKernelGGL(mam::k_read_windows, dim3((max_rows + 255) / 256, n_windows), dim3(256), 0, (hipStream_t)stream,
                       kf_table, kf_cap, mp_table, mp_cap, mp_id_base, windows, status);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}
