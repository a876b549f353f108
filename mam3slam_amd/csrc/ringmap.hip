// The device-resident keyframe / MapPoint map of the LocalMapping leg (include/mam_ringmap.h): MapPoint identities
// shared across the ring's keyframes, their observation sets, LocalMapping's map edits and the LocalBundleAdjustment
// window build and write-back over them. Reference: src/LocalMapping.cc:95-172, 457-501, 504-828, 830-939;
// src/ORBmatcher.cc:1148-1338 (Fuse); src/MapPoint.cc:141-239 (AddObservation, EraseObservation, SetBadFlag),
// 248-297 (Replace), 329-403 (ComputeDistinctiveDescriptors), 426-494 (UpdateNormalAndDepth);
// src/KeyFrame.cc:312-380 (UpdateConnections); src/Optimizer.cc:1118-1186, 1413-1497 (LocalBundleAdjustment).
//
// Integer / byte work over R S rows: one thread per row or per keypoint, coalesced over the row tables; the only
// LDS-heavy kernels are the per-slot merge resolution (a hash of merge groups) and the window build (a bitmap of the
// MapPoints already taken). Every result is order-independent: atomics only take minima / maxima / ORs or count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "../../include/mam_ringmap.h"
#include "runtime.hpp"

namespace mam {
namespace rmap {

constexpr uint8_t F_INV = 1, F_TOUCH = 2, F_ERASED = 4, F_WRITTEN = 8, F_DEAD = 16, F_LOST = 32;
constexpr int32_t NO_CLAIM = 0x7f7f7f7f;   // hipMemset 0x7f

__device__ __forceinline__ int16_t* okp_row(const mam_ringmap& M, int id) { return M.okp + (size_t)id * M.R; }

__device__ __forceinline__ int nobs(const mam_ringmap& M, int id) {
    const int16_t* r = okp_row(M, id);
    int n = 0;
    for (int s = 0; s < M.R; s++) n += r[s] >= 0;
    return n;
}

// KeyFrame::GetCameraCenter in float (match.hip fuse_kf_of: Twc = Tcw^-1 as Sophus evaluates it)
__device__ __forceinline__ void camera_center(const float* T, float ow[3]) {
    const float px = -T[4], py = -T[5], pz = -T[6];
    const float qx = -T[0], qy = -T[1], qz = -T[2], w = T[3];
    float u0 = qy * pz - qz * py, u1 = qz * px - qx * pz, u2 = qx * py - qy * px;
    u0 = u0 + u0;
    u1 = u1 + u1;
    u2 = u2 + u2;
    ow[0] = (px + w * u0) + (qy * u2 - qz * u1);
    ow[1] = (py + w * u1) + (qz * u0 - qx * u2);
    ow[2] = (pz + w * u2) + (qx * u1 - qy * u0);
}

// ------------------------------------------------------------------------------------------------ union-find
__device__ __forceinline__ int uf_find(int* parent, int x) {
    while (true) {
        const int p = __hip_atomic_load(parent + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == x) return x;
        const int gp = __hip_atomic_load(parent + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (gp != p) __hip_atomic_store(parent + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // halving
        x = p;
    }
}

// the root without path compression: the flatten pass's only writes are each id's own final root (a halving store
// of another thread could overwrite an already flattened entry with an intermediate ancestor)
__device__ __forceinline__ int uf_root(const int* parent, int x) {
    while (true) {
        const int p = __hip_atomic_load(parent + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == x) return x;
        x = p;
    }
}

// link the larger root under the smaller: every component's root is its smallest id, whatever the union order
__device__ void uf_union(int* parent, int a, int b) {
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(parent + a, a, b) == a) return;
    }
}

// ------------------------------------------------------------------------------------------------ evict / repair
// KeyFrame::SetBadFlag of the slots' keyframes: every observation in them erased (flag LOST on the MapPoint)
__global__ __launch_bounds__(256) void k_evict_obs(const mam_ringmap M, int head, int W) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * M.S) return;
    const int s = head + t / M.S;
    const int e = s * M.S + t % M.S;
    const int m = M.mp_of[e];
    if (m >= 0) {
        okp_row(M, m)[s] = -1;
        M.mp_of[e] = -1;
        M.flag[m] = F_LOST;
    }
}

// Repair decision per live MapPoint (mode 0, after an eviction: MapPointCulling of the previous run's MapPoints and
// EraseObservation's bad rule for those that lost an observation; mode 1, after the LBA's erase: EraseObservation's
// rule for the flagged ones): -2 bad (SetBadFlag), >= 0 the new home row (the lowest remaining slot's keypoint) when
// the home keypoint lost its observation, -1 keep.
__global__ __launch_bounds__(256) void k_repair_decide(const mam_ringmap M, int mode, int run) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= M.R * M.S) return;
    int dec = -1;
    if (M.rec[id].valid) {
        const uint8_t f = M.flag[id];
        const int n = nobs(M, id);
        bool bad;
        if (mode == 0)
            bad = n <= 2 && ((f & F_LOST) || M.born[id] == run - 1);
        else
            bad = (f & F_ERASED) && n <= 2;
        if (n == 0) bad = true;
        if (bad) {
            dec = -2;
        } else if (M.mp_of[id] != id) {
            const int16_t* r = okp_row(M, id);
            for (int s = 0; s < M.R; s++)
                if (r[s] >= 0) {
                    dec = s * M.S + r[s];
                    break;
                }
        }
    }
    M.newid[id] = dec;
}

__global__ __launch_bounds__(256) void k_repair_apply(const mam_ringmap M) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= M.R * M.S) return;
    const int dec = M.newid[id];
    if (dec == -1) return;
    int16_t* r = okp_row(M, id);
    if (dec == -2) {   // SetBadFlag: every observation's EraseMapPointMatch, mpMap->EraseMapPoint
        for (int s = 0; s < M.R; s++) {
            const int k = r[s];
            if (k >= 0) {
                M.mp_of[s * M.S + k] = -1;
                r[s] = -1;
            }
        }
        M.rec[id].valid = 0;
        M.flag[id] |= F_DEAD;
        return;
    }
    // move the record to its new home row (a keypoint observing it: no live MapPoint is homed there)
    int16_t* r2 = okp_row(M, dec);
    for (int s = 0; s < M.R; s++) {
        const int k = r[s];
        r2[s] = (int16_t)k;
        r[s] = -1;
        if (k >= 0) M.mp_of[s * M.S + k] = dec;
    }
    M.rec[dec] = M.rec[id];
    M.born[dec] = M.born[id];
    M.rec[id].valid = 0;
    M.flag[id] |= F_DEAD;
}

__global__ __launch_bounds__(256) void k_flags(const mam_ringmap M) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < M.R * M.S) M.has_mp[e] = M.mp_of[e] >= 0 ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------ create
// CreateNewMapPoints: keypoint i1 of new keyframe w takes its first neighbour match; the neighbour keypoint's lowest
// claimant (w, i1) wins it
__global__ __launch_bounds__(256) void k_create_pick(const mam_ringmap M, int head, int W, const int32_t* pairs, int NN,
                                                     const int32_t* match) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * M.S) return;
    const int w = t / M.S, i1 = t % M.S, j = head + w;
    int target = -1;
    if (i1 < min(M.cnt[2 * j], M.S) && M.mp_of[j * M.S + i1] < 0) {
        for (int k = 0; k < NN; k++) {
            const int nb = pairs[2 * (w * NN + k) + 1];
            const int i2 = match[(size_t)(w * NN + k) * M.S + i1];
            if (i2 >= 0 && i2 < min(M.cnt[2 * nb], M.S) && M.mp_of[nb * M.S + i2] < 0) {
                target = nb * M.S + i2;
                break;
            }
        }
    }
    M.newid[j * M.S + i1] = target;
    if (target >= 0) atomicMin(M.claim + target, t);
}

__global__ __launch_bounds__(256) void k_create_accept(const mam_ringmap M, int head, int W, int run) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * M.S) return;
    const int w = t / M.S, i1 = t % M.S, j = head + w;
    const int id = j * M.S + i1;
    const int target = M.newid[id];
    if (target < 0 || M.claim[target] != t) return;
    const int nb = target / M.S, i2 = target % M.S;
    mam_fuse_mp r = M.kp_rec[id];
    r.valid = 1;
    M.rec[id] = r;
    M.born[id] = run;
    M.mp_of[id] = id;
    M.mp_of[target] = id;
    int16_t* o = okp_row(M, id);
    o[j] = (int16_t)i1;
    o[nb] = (int16_t)i2;
}

// ------------------------------------------------------------------------------------------------ gather
__global__ __launch_bounds__(256) void k_gather(const mam_ringmap M) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= M.R * M.S) return;
    const int m = M.mp_of[e];
    mam_fuse_mp r;
    if (m >= 0) {
        r = M.rec[m];
        r.valid = 1;
    } else {
        r = mam_fuse_mp{};
    }
    M.lists[e] = r;
}

// ------------------------------------------------------------------------------------------------ fuse side effects
struct FuseApplyArgs {
    int head, W, NN, NB;
    const int32_t* pairs;
    const int32_t* fwd;
    const int32_t* bwd;
};

// One proposal (MapPoint m -> keypoint t) per thread: forward items first, then backward; false where Fuse skips it
__device__ __forceinline__ bool fuse_proposal(const mam_ringmap& M, const FuseApplyArgs& a, int g, int* pm, int* pt) {
    const int S = M.S;
    const int nf = a.W * a.NN * S;
    int m, ts, t;
    if (g < nf) {
        const int b = g / S, i = g % S;
        const int w = b / a.NN, j = a.head + w, nb = a.pairs[2 * b + 1];
        if (i >= min(M.cnt[2 * j], S)) return false;
        const int idx = a.fwd[(size_t)b * S + i];
        if (idx < 0 || idx >= min(M.cnt[2 * nb], S)) return false;
        m = M.mp_of[j * S + i];
        ts = nb;
        t = nb * S + idx;
    } else {
        const int g2 = g - nf;
        const int b = g2 / S, i = g2 % S;
        const int w = b / a.NB, k = b % a.NB, j = a.head + w;
        const int nbk = a.pairs[2 * (w * a.NN + k) + 1];
        if (i >= min(M.cnt[2 * nbk], S)) return false;
        const int idx = a.bwd[(size_t)b * S + i];
        if (idx < 0 || idx >= min(M.cnt[2 * j], S)) return false;
        m = M.mp_of[nbk * S + i];
        if (m < 0) return false;
        const int16_t* r = okp_row(M, m);
        for (int k2 = 0; k2 < k; k2++)   // a fuse candidate once: from the first target keyframe holding it
            if (r[a.pairs[2 * (w * a.NN + k2) + 1]] >= 0) return false;
        ts = j;
        t = j * S + idx;
    }
    if (m < 0) return false;
    if (okp_row(M, m)[ts] >= 0) return false;   // IsInKeyFrame
    *pm = m;
    *pt = t;
    return true;
}

__global__ __launch_bounds__(256) void k_uf_init(const mam_ringmap M) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < M.R * M.S) M.parent[i] = i;
}

template <int PHASE>
__global__ __launch_bounds__(256) void k_fuse_proposals(const mam_ringmap M, const FuseApplyArgs a, int n) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    int m, t;
    if (!fuse_proposal(M, a, g, &m, &t)) return;
    const int q = M.mp_of[t];
    if (PHASE == 0) {
        if (q >= 0) {
            if (q != m) {   // Replace: one of the two survives
                uf_union(M.parent, m, q);
                M.flag[m] = F_INV;
                M.flag[q] = F_INV;
            }
        } else {   // AddObservation onto a free keypoint
            atomicMin(M.claim + t, m);
            M.flag[m] = F_INV;
        }
    } else if (q < 0) {
        const int c = M.claim[t];
        if (c != m) uf_union(M.parent, m, c);   // the later claimants find the first's MapPoint there
    }
}

__global__ __launch_bounds__(256) void k_uf_flatten(const mam_ringmap M) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M.R * M.S || !(M.flag[i] & F_INV)) return;
    const int r = uf_root(M.parent, i);
    __hip_atomic_store(M.parent + i, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_survivor(const mam_ringmap M) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M.R * M.S || !(M.flag[i] & F_INV)) return;
    const uint64_t key = ((uint64_t)nobs(M, i) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
    atomicMax((unsigned long long*)(M.surv + M.parent[i]), (unsigned long long)key);
}

__device__ __forceinline__ int survivor_of(const mam_ringmap& M, int root) {
    return (int)(0xFFFFFFFFu - (uint32_t)(M.surv[root] & 0xFFFFFFFFull));
}

// one workgroup per slot: per merge group of the slot's keypoints the winning keypoint (survivor's own, else the
// lowest member id's, else the lowest claimed keypoint); the slot's column of okp and its mp_of entries belong to it
constexpr int RES_T = 256;
__device__ __forceinline__ bool res_entry(const mam_ringmap& M, int s, int kp, int* grp, int* key, int* member) {
    const int e = s * M.S + kp;
    const int m = M.mp_of[e];
    if (m >= 0) {
        if (!(M.flag[m] & F_INV)) return false;
        const int r = M.parent[m];
        *grp = r;
        *key = m == survivor_of(M, r) ? 0 : ((1 << 28) | m);   // ids < 2^22 (R <= 128, S < 2^15)
        *member = m;
        return true;
    }
    const int c = M.claim[e];
    if (c == NO_CLAIM) return false;
    *grp = M.parent[c];
    *key = (2 << 28) | kp;
    *member = -1;
    return true;
}

__global__ __launch_bounds__(RES_T) void k_resolve_slots(const mam_ringmap M, int hs) {
    extern __shared__ int hsh[];   // [hs] group, [hs] min key
    int* hg = hsh;
    int* hk = hsh + hs;
    const int s = blockIdx.x;
    for (int i = threadIdx.x; i < hs; i += RES_T) {
        hg[i] = -1;
        hk[i] = INT_MAX;
    }
    __syncthreads();
    const int n = M.S;
    for (int kp = threadIdx.x; kp < n; kp += RES_T) {
        int g, key, mem;
        if (!res_entry(M, s, kp, &g, &key, &mem)) continue;
        int h = (int)(((uint32_t)g * 2654435761u) & (uint32_t)(hs - 1));
        while (true) {
            const int old = atomicCAS(hg + h, -1, g);
            if (old == -1 || old == g) {
                atomicMin(hk + h, key);
                break;
            }
            h = (h + 1) & (hs - 1);
        }
    }
    __syncthreads();
    for (int kp = threadIdx.x; kp < n; kp += RES_T) {
        int g, key, mem;
        if (!res_entry(M, s, kp, &g, &key, &mem)) continue;
        int h = (int)(((uint32_t)g * 2654435761u) & (uint32_t)(hs - 1));
        while (hg[h] != g) h = (h + 1) & (hs - 1);
        const bool win = hk[h] == key;
        const int sv = survivor_of(M, g);
        const int e = s * M.S + kp;
        if (mem >= 0) {
            if (win) {
                if (mem != sv) {   // ReplaceMapPointMatch + AddObservation
                    M.mp_of[e] = sv;
                    okp_row(M, mem)[s] = -1;
                    okp_row(M, sv)[s] = (int16_t)kp;
                }
            } else {   // the survivor is already in this keyframe: EraseMapPointMatch
                M.mp_of[e] = -1;
                okp_row(M, mem)[s] = -1;
            }
        } else if (win) {   // AddObservation + AddMapPoint
            M.mp_of[e] = sv;
            okp_row(M, sv)[s] = (int16_t)kp;
        }
    }
}

__global__ __launch_bounds__(256) void k_fuse_finalize(const mam_ringmap M) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M.R * M.S || !(M.flag[i] & F_INV)) return;
    if (survivor_of(M, M.parent[i]) != i) M.rec[i].valid = 0;   // mpMap->EraseMapPoint(this) after Replace
}

// ------------------------------------------------------------------------------------------------ refresh
__global__ __launch_bounds__(256) void k_touch(const mam_ringmap M, int head, int W) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * M.S) return;
    const int m = M.mp_of[head * M.S + t];
    if (m >= 0) M.flag[m] = F_TOUCH;   // benign: every writer stores the same value
}

__device__ __forceinline__ int desc_dist32(const uint8_t* a, const uint8_t* b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
    const uint4 a0 = x[0], a1 = x[1], b0 = y[0], b1 = y[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// UpdateNormalAndDepth (MapPoint.cc:426-494) of MapPoint id: observations in slot order, the reference keyframe =
// the home slot
// f(s, k) for every observation (slot s, keypoint k >= 0) of a MapPoint row, in slot order: 16-byte loads of eight
// slots when the row is 16-byte aligned (R a multiple of 8: c2's R = 96), else one slot a load
template <class F>
__device__ __forceinline__ void for_obs(const int16_t* r, int R, F f) {
    if ((R & 7) == 0) {
        const uint4* r4 = reinterpret_cast<const uint4*>(r);
        for (int q = 0; q < R / 8; q++) {
            const uint4 v = r4[q];
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const int k0 = (int16_t)(wv[h] & 0xffffu), k1 = (int16_t)(wv[h] >> 16);
                if (k0 >= 0) f(8 * q + 2 * h, k0);
                if (k1 >= 0) f(8 * q + 2 * h + 1, k1);
            }
        }
    } else {
        for (int s = 0; s < R; s++)
            if (r[s] >= 0) f(s, (int)r[s]);
    }
}

__device__ void normal_depth(const mam_ringmap& M, int id) {
    mam_fuse_mp& rec = M.rec[id];
    const int16_t* r = okp_row(M, id);
    const float P0 = rec.pos[0], P1 = rec.pos[1], P2 = rec.pos[2];
    float n0 = 0.0f, n1 = 0.0f, n2 = 0.0f;
    int n = 0;
    for_obs(r, M.R, [&](int s, int) {
        float ow[3];
        camera_center(M.tcw + 7 * (size_t)s, ow);
        const float a0 = P0 - ow[0], a1 = P1 - ow[1], a2 = P2 - ow[2];
        const float nr = sqrtf(a0 * a0 + (a1 * a1 + a2 * a2));   // Eigen's 3-term norm: e0 + (e1 + e2)
        n0 = n0 + a0 / nr;
        n1 = n1 + a1 / nr;
        n2 = n2 + a2 / nr;
        n++;
    });
    if (n == 0) return;
    const int hs = id / M.S, hk = id % M.S;
    float ow[3];
    camera_center(M.tcw + 7 * (size_t)hs, ow);
    const float c0 = P0 - ow[0], c1 = P1 - ow[1], c2 = P2 - ow[2];
    const float dist = sqrtf(c0 * c0 + (c1 * c1 + c2 * c2));
    const int level = min(max(M.keys[(size_t)hs * M.S + hk].octave, 0), M.nlevels - 1);
    const float maxd = dist * M.scale_factors[level];
    rec.max_distance = maxd;
    rec.min_distance = maxd / M.scale_factors[M.nlevels - 1];
    const float fn = (float)n;
    rec.normal[0] = n0 / fn;
    rec.normal[1] = n1 / fn;
    rec.normal[2] = n2 / fn;
}

// one wave per flagged MapPoint (waves stride over chunks of 64 ids): UpdateNormalAndDepth on lane 0 and, with DESC,
// ComputeDistinctiveDescriptors (MapPoint.cc:329-403): the observations' descriptors staged in LDS in slot order, lane
// i takes rows i and i + 64 of the N x N distance matrix and finds the row's median — element (N-1)/2 of the row
// sorted ascending, the diagonal 0 included — by a binary search over the distance value; the descriptor of the first
// row with the least median wins
constexpr int RF_T = 256, RF_NMAX = 128;
template <bool DESC>
__global__ __launch_bounds__(RF_T) void k_refresh(const mam_ringmap M, uint8_t bit) {
    __shared__ __attribute__((aligned(16))) uint8_t dsc[RF_T / 64][RF_NMAX][32];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nwaves = gridDim.x * (RF_T / 64);
    const int n_ids = M.R * M.S;
    for (int base = (blockIdx.x * (RF_T / 64) + wv) * 64; base < n_ids; base += nwaves * 64) {
        const int myid = base + lane;
        const bool want = myid < n_ids && (M.flag[myid] & bit) && M.rec[myid].valid;
        // UpdateNormalAndDepth: every lane its own MapPoint (a record's normal / depth fields, nothing another reads)
        if (want) normal_depth(M, myid);
        if (!DESC) continue;
        uint64_t todo = __ballot(want);
        while (todo) {
            const int l = __ffsll((unsigned long long)todo) - 1;
            todo &= todo - 1;
            const int id = base + l;
            const int16_t* r = okp_row(M, id);
            // the observations in slot order: lane l holds slots l and l + 64
            const int k0 = lane < M.R ? r[lane] : -1, k1 = lane + 64 < M.R ? r[lane + 64] : -1;
            const uint64_t b0 = __ballot(k0 >= 0), b1 = __ballot(k1 >= 0);
            const uint64_t below = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
            const int c0 = __popcll(b0);
            const int N = c0 + __popcll(b1);
            if (k0 >= 0) {
                const uint4* src = reinterpret_cast<const uint4*>(M.desc + ((size_t)lane * M.S + k0) * 32);
                uint4* dst = reinterpret_cast<uint4*>(dsc[wv][__popcll(b0 & below)]);
                dst[0] = src[0];
                dst[1] = src[1];
            }
            if (k1 >= 0) {
                const uint4* src = reinterpret_cast<const uint4*>(M.desc + ((size_t)(lane + 64) * M.S + k1) * 32);
                uint4* dst = reinterpret_cast<uint4*>(dsc[wv][c0 + __popcll(b1 & below)]);
                dst[0] = src[0];
                dst[1] = src[1];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const int med_k = (int)(0.5 * (double)(N - 1));
            uint32_t best = 0xFFFFFFFFu;   // (median << 8) | row
            for (int i = lane; i < N; i += 64) {
                const uint4* di = reinterpret_cast<const uint4*>(dsc[wv][i]);
                const uint4 a0 = di[0], a1 = di[1];
                int lo = 0, hi = 256;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    int c = 0;
                    for (int j = 0; j < N; j++) {
                        const uint4* dj = reinterpret_cast<const uint4*>(dsc[wv][j]);
                        const uint4 e0 = dj[0], e1 = dj[1];
                        const int d = __popc(a0.x ^ e0.x) + __popc(a0.y ^ e0.y) + __popc(a0.z ^ e0.z) +
                                      __popc(a0.w ^ e0.w) + __popc(a1.x ^ e1.x) + __popc(a1.y ^ e1.y) +
                                      __popc(a1.z ^ e1.z) + __popc(a1.w ^ e1.w);
                        c += d <= mid;
                    }
                    if (c > med_k) hi = mid;
                    else lo = mid + 1;
                }
                const uint32_t key = ((uint32_t)lo << 8) | (uint32_t)i;
                best = key < best ? key : best;
            }
            for (int o = 32; o >= 1; o >>= 1) {
                const uint32_t x = (uint32_t)__shfl_xor((int)best, o, 64);
                best = x < best ? x : best;
            }
            if (lane < 2 && N > 0) {
                const int row = (int)(best & 0xFFu);
                reinterpret_cast<uint4*>(M.rec[id].desc)[lane] = reinterpret_cast<const uint4*>(dsc[wv][row])[lane];
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// ------------------------------------------------------------------------------------------------ windows
constexpr int WIN_T = 1024;
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int& total) {
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
    for (int w = 0; w < WIN_T / 64; w++) {
        const int t = wsum[w];
        if (w < wid) pre += t;
        total += t;
    }
    __syncthreads();
    return pre + x - v;
}

struct WinArgs {
    int head, covis_th, pcap, ecap;
    const mam_ringmap_window* outs;
    int32_t* counts;
    int32_t* pose_slot;
    int32_t* point_id;
};

__global__ __launch_bounds__(WIN_T) void k_windows(const mam_ringmap M, const WinArgs a) {
    extern __shared__ uint32_t taken[];   // [R S / 32] MapPoint ids already local
    __shared__ int wt[128], first[128], posei[128], order[128], wsum[WIN_T / 64], hdr[8];
    const int w = blockIdx.x, j = a.head + w, t = threadIdx.x, R = M.R, S = M.S;
    const mam_ringmap_window& o = a.outs[w];
    const int nwords = (R * S + 31) / 32;
    for (int i = t; i < nwords; i += WIN_T) taken[i] = 0;
    if (t < 128) {
        wt[t] = 0;
        first[t] = INT_MAX;
        posei[t] = -1;
    }
    __syncthreads();
    // covisibility weights: shared MapPoints with every other keyframe (KeyFrame::UpdateConnections' KFcounter)
    for (int kp = t; kp < S; kp += WIN_T) {
        const int m = M.mp_of[j * S + kp];
        if (m < 0) continue;
        for_obs(okp_row(M, m), R, [&](int s, int) {
            if (s != j) atomicAdd(wt + s, 1);
        });
    }
    __syncthreads();
    if (t == 0) {   // GetVectorCovisibleKeyFrames: weight >= th, descending (ties: slot); none: the heaviest
        int nl = 0;
        order[nl++] = j;
        int nc = 0, smax = -1, wmax = 0;
        for (int s = 0; s < R; s++) {
            if (wt[s] > wmax) {
                wmax = wt[s];
                smax = s;
            }
            if (wt[s] < a.covis_th) continue;
            int i = nl + nc++;
            while (i > 1 && wt[order[i - 1]] < wt[s]) {
                order[i] = order[i - 1];
                i--;
            }
            order[i] = s;
        }
        nl += nc;
        if (nc == 0 && smax >= 0) order[nl++] = smax;
        for (int i = 0; i < nl; i++) posei[order[i]] = i;
        hdr[0] = nl;
        hdr[1] = 0;   // points
        hdr[2] = 0;   // overflow
    }
    __syncthreads();
    const int nloc = hdr[0];
    // local MapPoints: every MapPoint of every local keyframe, in keyframe order then keypoint order, once
    // (one keyframe chunk of WIN_T keypoints a pass; the next chunk's ids loaded before this one's scan)
    const int nch = (S + WIN_T - 1) / WIN_T;
    auto chunk_id = [&](int c) -> int {
        const int kp = (c % nch) * WIN_T + t;
        return (c < nloc * nch && kp < S) ? M.mp_of[order[c / nch] * S + kp] : -1;
    };
    int m_next = chunk_id(0), base = 0;   // (base: every thread's copy of the running count)
    for (int c = 0; c < nloc * nch; c++) {
        const int m = m_next;
        m_next = chunk_id(c + 1);
        bool nw = false;
        if (m >= 0) {
            const uint32_t bit = 1u << (m & 31);
            nw = !(atomicOr(taken + (m >> 5), bit) & bit);
        }
        int tot;
        const int pos = block_excl_scan(nw ? 1 : 0, wsum, tot) + base;   // (its barriers order the chunks' atomics)
        base += tot;
        if (nw && pos < a.pcap) {
            a.point_id[(size_t)w * a.pcap + pos] = m;
            const mam_fuse_mp& rc = M.rec[m];
            for (int cc = 0; cc < 3; cc++) o.point_xyz[3 * (size_t)pos + cc] = (double)rc.pos[cc];
        }
    }
    const int np_all = base;
    const int npts = min(np_all, a.pcap);
    __threadfence_block();
    __syncthreads();
    // fixed keyframes: the other observers of local MapPoints, by first encounter (MapPoint order, then slot order)
    for (int p = t; p < npts; p += WIN_T) {
        for_obs(okp_row(M, a.point_id[(size_t)w * a.pcap + p]), R, [&](int s, int) {
            if (posei[s] < 0) atomicMin(first + s, p);
        });
    }
    __syncthreads();
    if (t == 0) {
        int nf = 0;
        for (int s = 0; s < R; s++) {
            if (first[s] == INT_MAX) continue;
            int i = nloc + nf++;
            while (i > nloc && (first[order[i - 1]] > first[s] ||
                                (first[order[i - 1]] == first[s] && order[i - 1] > s))) {
                order[i] = order[i - 1];
                i--;
            }
            order[i] = s;
        }
        for (int i = nloc; i < nloc + nf; i++) posei[order[i]] = i;
        hdr[3] = nloc + nf;
        hdr[4] = 0;   // edges
    }
    __syncthreads();
    const int np = hdr[3];
    if (np == nloc || npts == 0 || np_all > a.pcap) {   // no fixed keyframe: the reference aborts the LBA
        if (t == 0) {
            const int c = np_all > a.pcap ? -1 : 0;
            for (int k = 0; k < 4; k++) a.counts[4 * w + k] = c;
        }
        return;
    }
    for (int i = t; i < np; i += WIN_T) {
        const int s = order[i];
        const float* T = M.tcw + 7 * (size_t)s;
        for (int c = 0; c < 4; c++) o.pose_q[4 * i + c] = (double)T[c];
        for (int c = 0; c < 3; c++) o.pose_t[3 * i + c] = (double)T[4 + c];
        o.pose_fixed[i] = i >= nloc ? 1 : 0;
        a.pose_slot[(size_t)w * R + i] = s;
    }
    // edges: per MapPoint in order, its observations in slot order
    int ebase = 0;   // (every thread's copy of the running edge count)
    for (int p0 = 0; p0 < npts; p0 += WIN_T) {
        const int p = p0 + t;
        int ne = 0;
        const int16_t* r = nullptr;
        if (p < npts) {
            r = okp_row(M, a.point_id[(size_t)w * a.pcap + p]);
            for_obs(r, R, [&](int, int) { ne++; });
        }
        int tot;
        int e = block_excl_scan(ne, wsum, tot) + ebase;
        ebase += tot;
        if (p < npts && e + ne <= a.ecap) {
            for_obs(r, R, [&](int s, int k) {
                const mam_keypoint& kp = M.keys[(size_t)s * S + k];
                o.edge_point[e] = p;
                o.edge_pose[e] = posei[s];
                o.edge_obs[2 * (size_t)e] = (double)kp.x;
                o.edge_obs[2 * (size_t)e + 1] = (double)kp.y;
                o.edge_inv_sigma2[e] = (double)M.inv_level_sigma2[min(max(kp.octave, 0), M.nlevels - 1)];
                e++;
            });
        }
    }
    if (t == 0) {
        const bool over = ebase > a.ecap;
        a.counts[4 * w] = over ? -1 : np;
        a.counts[4 * w + 1] = over ? -1 : npts;
        a.counts[4 * w + 2] = over ? -1 : ebase;
        a.counts[4 * w + 3] = over ? -1 : nloc;
    }
}

// ------------------------------------------------------------------------------------------------ write-back
struct WbArgs {
    int W, pcap;
    const mam_ringmap_window* wins;
    const mam_ringmap_result* res;
    const int32_t* counts;
    const int32_t* pose_slot;
    const int32_t* point_id;
};

// grid (ceil(max edges / 256), W): vToErase — chi2 > 5.991 or depth <= 0 -> EraseMapPointMatch + EraseObservation
__global__ __launch_bounds__(256) void k_wb_erase(const mam_ringmap M, const WbArgs a) {
    const int w = blockIdx.y, e = blockIdx.x * 256 + threadIdx.x;
    if (e >= a.counts[4 * w + 2]) return;
    const mam_ringmap_result& r = a.res[w];
    if (!(r.edge_chi2[e] > 5.991 || !r.edge_depth_ok[e])) return;
    const mam_ringmap_window& o = a.wins[w];
    const int m = a.point_id[(size_t)w * a.pcap + o.edge_point[e]];
    const int s = a.pose_slot[(size_t)w * M.R + o.edge_pose[e]];
    int16_t* row = okp_row(M, m);
    const int k = row[s];
    if (k < 0) return;
    M.mp_of[s * M.S + k] = -1;
    row[s] = -1;
    M.flag[m] = F_ERASED;
}

__device__ __forceinline__ int resolve_id(const mam_ringmap& M, int m) {
    const int d = M.newid[m];
    return d >= 0 ? d : (d == -2 ? -1 : m);
}

// grid (ceil(max(R, pcap) / 256), W): the last window writing each keyframe pose / MapPoint position
__global__ __launch_bounds__(256) void k_wb_last(const mam_ringmap M, const WbArgs a) {
    const int w = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (a.counts[4 * w + 2] <= 0) return;
    if (i < a.counts[4 * w + 3]) atomicMax(M.slot_last + a.pose_slot[(size_t)w * M.R + i], w);
    if (i < a.counts[4 * w + 1]) {
        const int m = resolve_id(M, a.point_id[(size_t)w * a.pcap + i]);
        if (m >= 0) atomicMax(M.lastw + m, w);
    }
}

__global__ __launch_bounds__(256) void k_wb_write(const mam_ringmap M, const WbArgs a) {
    const int w = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (a.counts[4 * w + 2] <= 0) return;
    const mam_ringmap_result& r = a.res[w];
    if (i < a.counts[4 * w + 3]) {
        const int s = a.pose_slot[(size_t)w * M.R + i];
        if (M.slot_last[s] == w) {
            // KeyFrame::SetPose(SE3f(q.cast<float>(), t.cast<float>())): Sophus renormalises the float quaternion,
            // norm summed (x^2 + z^2) + (y^2 + w^2) (as mam_exchange's k_pack_sources)
            float q[4];
            for (int c = 0; c < 4; c++) q[c] = (float)r.pose_q[4 * (size_t)i + c];
            const float nq = sqrtf((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
            float* T = M.tcw + 7 * (size_t)s;
            for (int c = 0; c < 4; c++) T[c] = q[c] / nq;
            for (int c = 0; c < 3; c++) T[4 + c] = (float)r.pose_t[3 * (size_t)i + c];
        }
    }
    if (i < a.counts[4 * w + 1]) {
        const int m = resolve_id(M, a.point_id[(size_t)w * a.pcap + i]);
        if (m >= 0 && M.lastw[m] == w) {
            for (int c = 0; c < 3; c++) M.rec[m].pos[c] = (float)r.point_xyz[3 * (size_t)i + c];   // SetWorldPos
            M.flag[m] |= F_WRITTEN;
        }
    }
}

// ------------------------------------------------------------------------------------------------ exchange
struct Header {
    int32_t n_kf, n_mp, agent, status;
};
struct KfRec {
    int32_t row;
    float q[4];
    float t[3];
};
static_assert(sizeof(Header) == 16 && sizeof(KfRec) == 32 && sizeof(mam_mp_record) == 48, "record sizes");

__host__ __device__ inline size_t block_bytes(int kf_cap, int mp_cap) {
    return sizeof(Header) + (size_t)kf_cap * sizeof(KfRec) + (size_t)mp_cap * sizeof(mam_mp_record);
}

constexpr int PK_CHUNK = 1024;
__device__ __forceinline__ bool pack_mp(const mam_ringmap& M, int id) {
    return (M.flag[id] & (F_WRITTEN | F_DEAD)) != 0;
}

// per 1024-row chunk: the MapPoint records it holds
__global__ __launch_bounds__(256) void k_pack_count(const mam_ringmap M) {
    __shared__ int red[4];
    const int c0 = blockIdx.x * PK_CHUNK;
    int n = 0;
    for (int i = c0 + threadIdx.x; i < min(c0 + PK_CHUNK, M.R * M.S); i += 256) n += pack_mp(M, i);
    for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) M.pack_off[1 + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void k_pack_scan(const mam_ringmap M, int nchunks) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        int acc = 0;
        M.pack_off[0] = 0;
        for (int c = 0; c < nchunks; c++) {
            acc += M.pack_off[1 + c];
            M.pack_off[1 + c] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void k_pack_write(const mam_ringmap M, int64_t row_kf, int64_t row_mp, int agent,
                                                    uint8_t* block, int kf_cap, int mp_cap, int nchunks) {
    __shared__ int wsum[4], base;
    Header* h = reinterpret_cast<Header*>(block);
    KfRec* K = reinterpret_cast<KfRec*>(block + sizeof(Header));
    mam_mp_record* P = reinterpret_cast<mam_mp_record*>(block + sizeof(Header) + (size_t)kf_cap * sizeof(KfRec));
    const int c = blockIdx.x;
    if (c == nchunks) {   // the keyframes (R <= 128: one block) and the header
        const int s = threadIdx.x;
        int f = (s < M.R && M.slot_last[s] >= 0) ? 1 : 0;
        int x = f;
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(x, o, 64);
            if ((threadIdx.x & 63) >= o) x += u;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < 4; w++) {
            if (w < (threadIdx.x >> 6)) pre += wsum[w];
            tot += wsum[w];
        }
        const int pos = pre + x - f;
        if (f && pos < kf_cap) {
            KfRec r;
            r.row = (int32_t)(row_kf + s);
            const float* T = M.tcw + 7 * (size_t)s;
            for (int k = 0; k < 4; k++) r.q[k] = T[k];
            for (int k = 0; k < 3; k++) r.t[k] = T[4 + k];
            K[pos] = r;
        }
        if (threadIdx.x == 0) {
            const int nmp = M.pack_off[nchunks];
            Header hh;
            hh.n_kf = min(tot, kf_cap);
            hh.n_mp = min(nmp, mp_cap);
            hh.agent = agent;
            hh.status = (tot > kf_cap || nmp > mp_cap) ? MAM_ERR_CAPACITY : 0;
            *h = hh;
        }
        return;
    }
    if (threadIdx.x == 0) base = M.pack_off[c];
    __syncthreads();
    for (int i0 = c * PK_CHUNK; i0 < min((c + 1) * PK_CHUNK, M.R * M.S); i0 += 256) {
        const int i = i0 + threadIdx.x;
        const int f = (i < M.R * M.S && pack_mp(M, i)) ? 1 : 0;
        int x = f;
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(x, o, 64);
            if ((threadIdx.x & 63) >= o) x += u;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < 4; w++) {
            if (w < (threadIdx.x >> 6)) pre += wsum[w];
            tot += wsum[w];
        }
        const int pos = base + pre + x - f;
        if (f && pos < mp_cap) {
            const mam_fuse_mp& rc = M.rec[i];
            mam_mp_record r{};
            const bool dead = !rc.valid;
            r.row = (int32_t)((uint32_t)(row_mp + i) | (dead ? 0x80000000u : 0u));
            for (int k = 0; k < 3; k++) {
                r.xyz[k] = rc.pos[k];
                r.normal[k] = rc.normal[k];
            }
            r.min_distance = rc.min_distance;
            r.max_distance = rc.max_distance;
            P[pos] = r;
        }
        __syncthreads();
        if (threadIdx.x == 0) base += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_apply(const uint8_t* block, int kf_cap, int mp_cap, float* kf, int64_t kf_rows,
                                               float* mp, int64_t mp_rows, int32_t* status) {
    const Header h = *reinterpret_cast<const Header*>(block);
    if (h.status != 0 || h.n_kf < 0 || h.n_kf > kf_cap || h.n_mp < 0 || h.n_mp > mp_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(status, MAM_ERR_ARG);
        return;
    }
    const KfRec* K = reinterpret_cast<const KfRec*>(block + sizeof(Header));
    const mam_mp_record* P =
        reinterpret_cast<const mam_mp_record*>(block + sizeof(Header) + (size_t)kf_cap * sizeof(KfRec));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < h.n_kf) {
        const KfRec r = K[i];
        if (r.row >= 0 && r.row < kf_rows) {
            float* d = kf + (size_t)r.row * 8;
            for (int k = 0; k < 4; k++) d[k] = r.q[k];
            for (int k = 0; k < 3; k++) d[4 + k] = r.t[k];
            d[7] = 1.0f;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
    if (i < h.n_mp) {
        const mam_mp_record r = P[i];
        const int64_t row = (int64_t)((uint32_t)r.row & 0x7fffffffu);
        if (row < mp_rows) {
            float* d = mp + (size_t)row * 12;
            for (int k = 0; k < 3; k++) d[k] = r.xyz[k];
            d[3] = ((uint32_t)r.row & 0x80000000u) ? 1.0f : 0.0f;
            for (int k = 0; k < 3; k++) d[4 + k] = r.normal[k];
            d[7] = r.min_distance;
            d[8] = r.max_distance;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
}

}  // namespace rmap
}  // namespace mam

// ------------------------------------------------------------------------------------------------ C-ABI
namespace {
using namespace mam::rmap;

bool map_ok(const mam_ringmap* m) {
    return m && m->R >= 1 && m->R <= 128 && m->S >= 1 && m->S <= 32767 && m->nlevels >= 1 && m->nlevels <= 8 &&
           m->mp_of && m->okp && m->rec && m->born && m->has_mp && m->lists && m->keys && m->desc && m->cnt &&
           m->tcw && m->kp_rec && m->parent && m->claim && m->surv && m->flag && m->newid && m->lastw &&
           m->slot_last && m->pack_off;
}
bool slots_ok(const mam_ringmap* m, int head, int W) {
    return W >= 1 && head >= 0 && head + W <= m->R;
}
inline dim3 grid_for(long long n) { return dim3((unsigned)((n + 255) / 256)); }
}  // namespace

extern "C" int mam_ringmap_evict(const mam_ringmap* map, int head, int W, int step, void* stream) {
    if (!map_ok(map) || !slots_ok(map, head, W)) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)M.R * M.S;
    MAM_HIP(hipMemsetAsync(M.flag, 0, (size_t)n, s));
    hipLaunchKernelGGL(k_evict_obs, grid_for((long long)W * M.S), dim3(256), 0, s, M, head, W);
    hipLaunchKernelGGL(k_repair_decide, grid_for(n), dim3(256), 0, s, M, 0, step);
    hipLaunchKernelGGL(k_repair_apply, grid_for(n), dim3(256), 0, s, M);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_flags(const mam_ringmap* map, void* stream) {
    if (!map_ok(map)) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipLaunchKernelGGL(k_flags, grid_for((long long)M.R * M.S), dim3(256), 0, (hipStream_t)stream, M);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_create(const mam_ringmap* map, int head, int W, const int32_t* pairs, int NN,
                                  const int32_t* match, int step, void* stream) {
    if (!map_ok(map) || !slots_ok(map, head, W) || !pairs || !match || NN < 1) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipStream_t s = (hipStream_t)stream;
    MAM_HIP(hipMemsetAsync(M.claim, 0x7f, (size_t)M.R * M.S * 4, s));
    hipLaunchKernelGGL(k_create_pick, grid_for((long long)W * M.S), dim3(256), 0, s, M, head, W, pairs, NN, match);
    hipLaunchKernelGGL(k_create_accept, grid_for((long long)W * M.S), dim3(256), 0, s, M, head, W, step);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_gather(const mam_ringmap* map, void* stream) {
    if (!map_ok(map)) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipLaunchKernelGGL(k_gather, grid_for((long long)M.R * M.S), dim3(256), 0, (hipStream_t)stream, M);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_fuse_apply(const mam_ringmap* map, int head, int W, const int32_t* pairs, int NN, int NB,
                                      const int32_t* fwd_idx, const int32_t* bwd_idx, void* stream) {
    if (!map_ok(map) || !slots_ok(map, head, W) || !pairs || NN < 1 || NB < 0 || NB > NN || !fwd_idx ||
        (NB > 0 && !bwd_idx))
        return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    int hs = 1;
    while (hs < 2 * M.S) hs <<= 1;
    if ((size_t)hs * 8 > 64 * 1024) return MAM_ERR_CAPACITY;
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)M.R * M.S;
    MAM_HIP(hipMemsetAsync(M.flag, 0, (size_t)n, s));
    MAM_HIP(hipMemsetAsync(M.claim, 0x7f, (size_t)n * 4, s));
    MAM_HIP(hipMemsetAsync(M.surv, 0, (size_t)n * 8, s));
    hipLaunchKernelGGL(k_uf_init, grid_for(n), dim3(256), 0, s, M);
    FuseApplyArgs a{head, W, NN, NB, pairs, fwd_idx, bwd_idx};
    const long long np = (long long)W * (NN + NB) * M.S;
    hipLaunchKernelGGL(k_fuse_proposals<0>, grid_for(np), dim3(256), 0, s, M, a, (int)np);
    hipLaunchKernelGGL(k_fuse_proposals<1>, grid_for(np), dim3(256), 0, s, M, a, (int)np);
    hipLaunchKernelGGL(k_uf_flatten, grid_for(n), dim3(256), 0, s, M);
    hipLaunchKernelGGL(k_survivor, grid_for(n), dim3(256), 0, s, M);
    hipLaunchKernelGGL(k_resolve_slots, dim3(M.R), dim3(RES_T), (size_t)hs * 8, s, M, hs);
    hipLaunchKernelGGL(k_fuse_finalize, grid_for(n), dim3(256), 0, s, M);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_refresh(const mam_ringmap* map, int head, int W, void* stream) {
    if (!map_ok(map) || !slots_ok(map, head, W)) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)M.R * M.S;
    MAM_HIP(hipMemsetAsync(M.flag, 0, (size_t)n, s));
    hipLaunchKernelGGL(k_touch, grid_for((long long)W * M.S), dim3(256), 0, s, M, head, W);
    hipLaunchKernelGGL(k_refresh<true>, dim3((unsigned)((n + 255) / 256)), dim3(RF_T), 0, s, M, F_TOUCH);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_windows(const mam_ringmap* map, int head, int W, int covis_th,
                                   const mam_ringmap_window* outs, int pcap, int ecap, int32_t* counts,
                                   int32_t* pose_slot, int32_t* point_id, void* stream) {
    if (!map_ok(map) || !slots_ok(map, head, W) || !outs || !counts || !pose_slot || !point_id || pcap < 1 ||
        ecap < 1)
        return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    const size_t lds = (size_t)((M.R * M.S + 31) / 32) * 4;
    if (lds > 64 * 1024) return MAM_ERR_CAPACITY;
    WinArgs a{head, covis_th, pcap, ecap, outs, counts, pose_slot, point_id};
    hipLaunchKernelGGL(k_windows, dim3(W), dim3(WIN_T), lds, (hipStream_t)stream, M, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_writeback(const mam_ringmap* map, int W, const mam_ringmap_window* wins,
                                     const mam_ringmap_result* res, const int32_t* counts, const int32_t* pose_slot,
                                     const int32_t* point_id, int pcap, int ecap, void* stream) {
    if (!map_ok(map) || W < 1 || !wins || !res || !counts || !pose_slot || !point_id || pcap < 1 || ecap < 1)
        return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)M.R * M.S;
    MAM_HIP(hipMemsetAsync(M.flag, 0, (size_t)n, s));
    MAM_HIP(hipMemsetAsync(M.lastw, 0xff, (size_t)n * 4, s));
    MAM_HIP(hipMemsetAsync(M.slot_last, 0xff, (size_t)M.R * 4, s));
    WbArgs a{W, pcap, wins, res, counts, pose_slot, point_id};
    hipLaunchKernelGGL(k_wb_erase, dim3((ecap + 255) / 256, W), dim3(256), 0, s, M, a);
    hipLaunchKernelGGL(k_repair_decide, grid_for(n), dim3(256), 0, s, M, 1, 0);
    hipLaunchKernelGGL(k_repair_apply, grid_for(n), dim3(256), 0, s, M);
    const int nl = std::max(M.R, pcap);
    hipLaunchKernelGGL(k_wb_last, dim3((nl + 255) / 256, W), dim3(256), 0, s, M, a);
    hipLaunchKernelGGL(k_wb_write, dim3((nl + 255) / 256, W), dim3(256), 0, s, M, a);
    hipLaunchKernelGGL(k_refresh<false>, dim3((unsigned)((n + 255) / 256)), dim3(RF_T), 0, s, M, F_WRITTEN);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" size_t mam_ringmap_block_bytes(int kf_cap, int mp_cap) {
    return (kf_cap < 0 || mp_cap < 0) ? 0 : block_bytes(kf_cap, mp_cap);
}

extern "C" int mam_ringmap_pack(const mam_ringmap* map, int64_t row_base_kf, int64_t row_base_mp, int agent,
                                void* block, int kf_cap, int mp_cap, void* stream) {
    if (!map_ok(map) || !block || kf_cap < 0 || mp_cap < 0) return MAM_ERR_ARG;
    const mam_ringmap M = *map;
    if (M.R > 256) return MAM_ERR_CAPACITY;
    hipStream_t s = (hipStream_t)stream;
    const int nchunks = (M.R * M.S + PK_CHUNK - 1) / PK_CHUNK;
    hipLaunchKernelGGL(k_pack_count, dim3(nchunks), dim3(256), 0, s, M);
    hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(64), 0, s, M, nchunks);
    hipLaunchKernelGGL(k_pack_write, dim3(nchunks + 1), dim3(256), 0, s, M, row_base_kf, row_base_mp, agent,
                       reinterpret_cast<uint8_t*>(block), kf_cap, mp_cap, nchunks);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_ringmap_apply(const void* gathered, int n_agents, int kf_cap, int mp_cap, float* kf_table,
                                 int64_t kf_rows, float* mp_table, int64_t mp_rows, int32_t* status, void* stream) {
    if (!gathered || n_agents < 1 || kf_cap < 0 || mp_cap < 0 || !kf_table || !mp_table || !status) return MAM_ERR_ARG;
    const size_t bb = block_bytes(kf_cap, mp_cap);
    const int n = std::max(1, std::max(kf_cap, mp_cap));
    for (int a = 0; a < n_agents; a++) {
        hipLaunchKernelGGL(k_apply, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const uint8_t*>(gathered) + (size_t)a * bb, kf_cap, mp_cap, kf_table,
                           kf_rows, mp_table, mp_rows, status);
        MAM_HIP(hipGetLastError());
    }
    return MAM_OK;
}
