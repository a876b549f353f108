// distribute.hpp — DistributeOctTree (reference src/ORBextractor.cc:555-779) on gfx950, shaped for single-frame
// latency. Included by orb_kernels.hip (namespace mam; lane/wave helpers, SortEl / stl_sort_wave from introsort.hpp).
//
// One workgroup of NT threads per (frame, level). The level's FAST candidates live in registers (KPT per thread,
// index k = j * NT + tid; beyond NT * KPT in global scratch), each with its current node id and the quadrant it went
// to in the last count pass. The node list lives in LDS as two ping-pong tables in LIST ORDER (node id == position).
// A quadtree round (ORBextractor.cc:605-677) or a final-phase expansion (:680-748) is:
//   scan    over the list: children per expanded node (creation bases), kept nodes (their rank) | 1 barrier inside
//   write   the new table: children of the expanded nodes in reverse creation order (push_front), then the kept
//           nodes in order — exactly the std::list the reference leaves — and the >1-key children in creation order
//           (the next final-phase candidates)                                                       | barrier
//   pass    every key to its node's new id (computed from the scan results, no per-key table) and at once its count
//           in the next round: the child quadrant of its node if that node expands (LDS atomics, aggregated per wave
//           by ballot)                                                                               | barrier
// The final phase's std::sort of (size, UL.x) with libstdc++'s tie behaviour is replayed by one wave
// (stl_sort_wave2) during the pass; the expansion cut (size >= N after an expansion) is a wave-level scan over the
// sorted candidates. Retain-best keeps the first max response in candidate order (:758-776).
#pragma once

namespace mam {
namespace dist {

// inclusive scan of a 32-bit value over the wave: DPP row shifts within rows of 16, then the gfx9 row broadcasts.
// Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

// exclusive scans of two values over the workgroup, one barrier: the per-wave totals alternate between two LDS
// buffers (`flip`), so a later call cannot overwrite partials an earlier one is still reading.
template <int NT>
__device__ __forceinline__ void block_scan2(uint32_t a, uint32_t b, uint32_t* part, int& flip, uint32_t& ea,
                                            uint32_t& eb, uint32_t& ta, uint32_t& tb) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t ia = wave_scan_incl(a), ib = wave_scan_incl(b);
    uint32_t* P = part + flip * 2 * NW;
    flip ^= 1;
    if (lane == 63) { P[w] = ia; P[NW + w] = ib; }
    __syncthreads();
    uint32_t pa = 0, pb = 0, sa = 0, sb = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint32_t x = P[i], y = P[NW + i];
        pa += i < w ? x : 0u;
        pb += i < w ? y : 0u;
        sa += x;
        sb += y;
    }
    ea = ia - a + pa;
    eb = ib - b + pb;
    ta = sa;
    tb = sb;
}

// child q (0 = n1 top-left, 1 = n2 top-right, 2 = n3 bottom-left, 3 = n4 bottom-right) of a node rectangle packed as
// {x0 | y0 << 16, x1 | y1 << 16} (ExtractorNode::DivideNode, ORBextractor.cc:480-536: half = ceil(extent / 2.f))
__device__ __forceinline__ uint2 child_rect2(uint2 r, int q) {
    const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
    const int cx0 = (q & 1) ? x0 + hx : x0, cx1 = (q & 1) ? x1 : x0 + hx;
    const int cy0 = (q & 2) ? y0 + hy : y0, cy1 = (q & 2) ? y1 : y0 + hy;
    return make_uint2((uint32_t)cx0 | ((uint32_t)cy0 << 16), (uint32_t)cx1 | ((uint32_t)cy1 << 16));
}
__device__ __forceinline__ int quad2(uint2 r, uint32_t key) {
    const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
    const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
    const bool right = x >= x0 + ((x1 - x0 + 1) >> 1), bottom = y >= y0 + ((y1 - y0 + 1) >> 1);
    return (right ? 1 : 0) | (bottom ? 2 : 0);
}

// cnt[t] += 1 for every active lane with t >= 0: lanes of the wave with the same target are counted by ballot and
// added by one leader (the early rounds send whole waves to the same few nodes: per-lane LDS atomics on one address
// serialise), up to AGG distinct targets per call; lanes left after that add one by one
#ifndef MAM_DIST_AGG
#define MAM_DIST_AGG 1   // distinct targets aggregated per wave in the count passes (0: plain LDS atomics; 1 measured best: 2 / 8 cost more issue than the conflicts they save)
#endif
template <int AGG>
__device__ __forceinline__ void agg_add(uint32_t* cnt, int t) {
#pragma unroll
    for (int it = 0; it < AGG; it++) {
        const uint64_t act = __ballot(t >= 0);
        if (!act) return;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const int lt = __builtin_amdgcn_readlane(t, leader);
        const uint64_t mm = __ballot(t == lt);
        if ((int)(threadIdx.x & 63) == leader) atomicAdd(cnt + lt, (uint32_t)__popcll(mm));
        if (t == lt) t = -1;
    }
    if (t >= 0) atomicAdd(cnt + t, 1u);
}

__host__ __device__ inline size_t a16(size_t b) { return (b + 15) & ~(size_t)15; }
// sort scratch: the wave sort's stack, stopper positions and move buffer for up to 4 elements per lane
#define MAM_DIST_SORT_E 4
__host__ __device__ inline size_t lds_bytes(int NC, int max_cells, int NT) {
    size_t s = a16((size_t)(max_cells + 1) * 4) + a16((size_t)4 * (NT / 64) * 4) + 64 +
               a16((size_t)MAM_SORT_WAVE2_SCRATCH(MAM_DIST_SORT_E) * 4);
    s += 2 * (a16((size_t)NC * 8) + a16((size_t)NC * 4) + a16((size_t)NC * 4) + a16((size_t)NC * 16));
    s += 3 * a16((size_t)NC * 4) + a16((size_t)NC * 8);
    return s;
}

}  // namespace dist

#ifdef MAM_DIST2_PROFILE
// per level: cycles by phase summed over launches (thread 0's clock after each phase), iteration counts, launches
// [0] init (+ the first count) [3] cut scan [4] kept scan [5] table write [6] the pass (remap + next count, wave 0's
// sort) [7] retain + output [8] final iterations [9] phase-1 rounds [10] sum of m [11] launches [12] wave 0's sort
__device__ unsigned long long g_d2prof[8][13];   // [12]: wave 0's sort alone
#define D2P(k)                                                                                         \
    do {                                                                                               \
        if (tid == 0) {                                                                                \
            const long long tn_ = clock64();                                                           \
            atomicAdd(&g_d2prof[l & 7][k], (unsigned long long)(tn_ - d2t));                           \
            d2t = tn_;                                                                                 \
        }                                                                                              \
    } while (0)
#define D2C(k, v) do { if (tid == 0) atomicAdd(&g_d2prof[l & 7][k], (unsigned long long)(v)); } while (0)
#else
#define D2P(k) do {} while (0)
#define D2C(k, v) do {} while (0)
#endif

// grid (levels, frames) x NT; levels l_first + blockIdx.x. ovf_key / ovf_node: per frame cand_per_frame u32 each
// (keys beyond NT * KPT of a level). lvl_counts[f][l] = {kept keypoints, lapping ones} or {-1, 0} on overflow.
template <int NT, int KPT>
__global__ __launch_bounds__(NT) void k_distribute2(const Geom* __restrict__ g, const int* __restrict__ cell_counts,
                                                    const uint32_t* __restrict__ cand, uint32_t* __restrict__ ovf_key,
                                                    uint32_t* __restrict__ ovf_node, uint32_t* __restrict__ out_key,
                                                    uint32_t* __restrict__ out_rank, int* __restrict__ lvl_counts,
                                                    int lap0, int lap1, int l_first) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using dist::a16;
    const int l = l_first + blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const LevelGeom& L = g->L[l];
    const int NC = g->node_cap;
    uint8_t* p8 = smem;
    auto take = [&](size_t bytes) { uint8_t* r = p8; p8 += a16(bytes); return r; };
    int* cellOff = (int*)take((size_t)(g->max_level_cells + 1) * 4);
    uint32_t* part = (uint32_t*)take((size_t)4 * (NT / 64) * 4);
    int* sh = (int*)take(64);
    int* sortscr = (int*)take((size_t)MAM_SORT_WAVE2_SCRATCH(MAM_DIST_SORT_E) * 4);
    uint2* rect0 = (uint2*)take((size_t)NC * 8);
    uint32_t* cnt0 = (uint32_t*)take((size_t)NC * 4);
    int* xr0 = (int*)take((size_t)NC * 4);
    uint4* chc0 = (uint4*)take((size_t)NC * 16);
    uint2* rect1 = (uint2*)take((size_t)NC * 8);
    uint32_t* cnt1 = (uint32_t*)take((size_t)NC * 4);
    int* xr1 = (int*)take((size_t)NC * 4);
    uint4* chc1 = (uint4*)take((size_t)NC * 16);
    uint32_t* nb = (uint32_t*)take((size_t)NC * 4);     // per node: creation | big-child base (expanded) or kept rank
    uint32_t* candl = (uint32_t*)take((size_t)NC * 4);  // final-phase candidates in creation order
    uint32_t* srt = (uint32_t*)take((size_t)NC * 4);    // expansion rank -> node; then the node's winning key
    SortEl* arr = (SortEl*)take((size_t)NC * 8);        // sort array; then the retain-best maxima
    int flip = 0;
    int* lc = lvl_counts + ((size_t)f * g->nlevels + l) * 2;
#ifdef MAM_DIST2_PROFILE
    long long d2t = clock64();
    D2C(11, 1);
#endif

    // ---- 0. this level's candidates in reference order (cells row-major, FAST order inside): cell offsets
    const int* cc = cell_counts + (size_t)f * g->cells_per_frame + L.cell_base;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < L.ncells; c0 += NT) {
        const int c = c0 + tid;
        const uint32_t v = c < L.ncells ? (uint32_t)cc[c] : 0u;
        uint32_t e, e2, t, t2;
        dist::block_scan2<NT>(v, 0u, part, flip, e, e2, t, t2);
        if (c < L.ncells) cellOff[c] = (int)(carry + e);
        carry += t;
    }
    const int n = (int)carry;
    if (n == 0) {
        if (tid == 0) { lc[0] = 0; lc[1] = 0; }
        return;
    }
    if (tid == 0) cellOff[L.ncells] = n;
    __syncthreads();
    const uint32_t* cbase = cand + (size_t)f * g->cand_per_frame + L.cand_base;
    uint32_t* OK = ovf_key + (size_t)f * g->cand_per_frame + L.cand_base;
    uint32_t* ON = ovf_node + (size_t)f * g->cand_per_frame + L.cand_base;
    auto fetch = [&](int k) -> uint32_t {
        int lo = 0, hi = L.ncells;   // last cell with cellOff[c] <= k
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (cellOff[mid] <= k) lo = mid;
            else hi = mid;
        }
        return cbase[(size_t)lo * L.cellcap + (k - cellOff[lo])];
    };
    const int nreg = n < NT * KPT ? n : NT * KPT;
    uint32_t kk[KPT], kn[KPT];
#pragma unroll
    for (int j = 0; j < KPT; j++) {
        const int k = j * NT + tid;
        kk[j] = k < nreg ? fetch(k) : 0u;
        kn[j] = 0;
    }
    for (int k = NT * KPT + tid; k < n; k += NT) OK[k] = fetch(k);
    // fn(key, node word, candidate index) over this thread's keys; node word = node | quadrant << 16
    auto for_keys = [&](auto&& fn) {
#pragma unroll
        for (int j = 0; j < KPT; j++) {
            const int k = j * NT + tid;
            if (k < nreg) fn(kk[j], kn[j], k);
        }
        for (int k = NT * KPT + tid; k < n; k += NT) {
            uint32_t nd = ON[k];
            fn(OK[k], nd, k);
            ON[k] = nd;
        }
    };

    // ---- 1. initial nodes (ORBextractor.cc:559-598), built in table 1, non-empty ones compacted into table 0
    const int N = L.nfeat;
    const int H = L.maxBY - L.minBY;
    const int nini = L.nini;
    for (int i = tid; i < nini; i += NT) {
        rect1[i] = make_uint2((uint32_t)(int)(L.hX * (float)i), (uint32_t)(int)(L.hX * (float)(i + 1)) | ((uint32_t)H << 16));
        cnt1[i] = 0;
    }
    __syncthreads();
    for_keys([&](uint32_t key, uint32_t& nd, int) {
        const int i = (int)((float)(key & 0xFFF) / L.hX);   // vpIniNodes[kp.pt.x / hX]
        nd = (uint32_t)i;
        dist::agg_add<(MAM_DIST_AGG < 4 ? MAM_DIST_AGG : 4)>(cnt1, i);
    });
    __syncthreads();
    int S = 0;
    {
        uint32_t kc = 0;
        for (int i0 = 0; i0 < nini; i0 += NT) {
            const int i = i0 + tid;
            const uint32_t c = i < nini ? cnt1[i] : 0u;
            uint32_t e, e2, t, t2;
            dist::block_scan2<NT>(c > 0 ? 1u : 0u, 0u, part, flip, e, e2, t, t2);
            if (c > 0) {
                const int np = (int)(kc + e);
                rect0[np] = rect1[i];
                cnt0[np] = c;
                xr0[np] = c > 1 ? 0 : -1;
                chc0[np] = make_uint4(0, 0, 0, 0);
                nb[i] = (uint32_t)np;
            }
            kc += t;
        }
        S = (int)kc;
    }
    __syncthreads();
    // the keys to their compacted initial nodes, and the first round's count (every node with > 1 keys divides)
    for_keys([&](uint32_t key, uint32_t& nd, int) {
        const int p = (int)nb[nd];
        int t = -1;
        if (xr0[p] >= 0) {
            const int q = dist::quad2(rect0[p], key);
            t = 4 * p + q;
            nd = (uint32_t)p | ((uint32_t)q << 16);
        } else {
            nd = (uint32_t)p;
        }
        dist::agg_add<MAM_DIST_AGG>(reinterpret_cast<uint32_t*>(chc0), t);
    });
    __syncthreads();
    D2P(0);

    // ---- 2. rounds
    int cur = 0, m = 0;
    bool final_phase = false;
    int guard = 0;
    while (true) {
        if (++guard > 4096) {   // unreachable for a correct rebuild (the list grows or the loop ends); never hang
            if (tid == 0) { lc[0] = -1; lc[1] = 0; }
            return;
        }
        const bool b = cur != 0;
        uint2* const R = b ? rect1 : rect0;
        uint32_t* const CN = b ? cnt1 : cnt0;
        int* const XR = b ? xr1 : xr0;
        uint4* const CH = b ? chc1 : chc0;
        uint2* const Rn = b ? rect0 : rect1;
        uint32_t* const CNn = b ? cnt0 : cnt1;
        int* const XRn = b ? xr0 : xr1;
        uint4* const CHn = b ? chc0 : chc1;
        if (final_phase && m == 0) break;
        uint32_t C = 0, M = 0;
        if (final_phase) {
            // ---- final phase (ORBextractor.cc:680-748): the candidates (last round's > 1-key children) were sorted
            // by wave 0 and counted by every key in the pass that ended the previous round
            D2C(8, 1);
            D2C(10, m);
            // expansion cut: after expanding ranks 0..r the list has S + sum (e - 1) nodes; stop at the first r where
            // that reaches N (:746-747). Wave 0 scans the ranks: creation / big-child bases, the cut, and marks the
            // candidates past the cut as not expanded.
            if (wid == 0) {
                uint32_t pc = 0;      // packed carry: children | big children << 16
                int rstop = m - 1;
                bool found = false;
                for (int r0 = 0; r0 < m; r0 += 64) {
                    const int r = r0 + lane;
                    int p = -1;
                    uint32_t v = 0;
                    if (r < m) {
                        p = (int)srt[r];
                        const uint4 c4 = CH[p];
                        v = (uint32_t)((c4.x > 0) + (c4.y > 0) + (c4.z > 0) + (c4.w > 0)) |
                            ((uint32_t)((c4.x > 1) + (c4.y > 1) + (c4.z > 1) + (c4.w > 1)) << 16);
                    }
                    const uint32_t incl = dist::wave_scan_incl(v) + pc;
                    const bool hit = !found && r < m && S + (int)(incl & 0xFFFF) - (r + 1) >= N;
                    const uint64_t hm = __ballot(hit);
                    const int rs = hm ? r0 + __ffsll((unsigned long long)hm) - 1 : -1;
                    if (r < m) {
                        if (found || (rs >= 0 && r > rs)) XR[p] = -1;
                        else nb[p] = incl - v;
                    }
                    if (!found && rs >= 0) {
                        rstop = rs;
                        found = true;
                        const uint32_t at = (uint32_t)__builtin_amdgcn_readlane((int)incl, rs - r0);
                        C = at & 0xFFFF;
                        M = at >> 16;
                    }
                    pc = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                }
                if (!found) { C = pc & 0xFFFF; M = pc >> 16; }
                (void)rstop;
                if (lane == 0) { sh[0] = (int)C; sh[1] = (int)M; }
            }
            __syncthreads();
            D2P(3);
            C = (uint32_t)sh[0];
            M = (uint32_t)sh[1];
        } else {
            // ---- phase-1 round (:605-677): every node with > 1 keys divides (counted in the previous pass)
            D2C(9, 1);
        }
        // kept nodes' ranks (and in phase 1 the creation / big-child bases) over the list in order
        uint32_t K = 0;
        {
            uint32_t c1 = 0, c2 = 0;
            for (int p0 = 0; p0 < S; p0 += NT) {
                const int p = p0 + tid;
                uint32_t v1 = 0, v2 = 0;
                bool ex = false;
                if (p < S) {
                    ex = XR[p] >= 0;
                    if (ex && !final_phase) {
                        const uint4 c4 = CH[p];
                        v1 = (uint32_t)((c4.x > 0) + (c4.y > 0) + (c4.z > 0) + (c4.w > 0)) |
                             ((uint32_t)((c4.x > 1) + (c4.y > 1) + (c4.z > 1) + (c4.w > 1)) << 16);
                    }
                    v2 = ex ? 0u : 1u;
                }
                uint32_t e1, e2, t1, t2;
                dist::block_scan2<NT>(v1, v2, part, flip, e1, e2, t1, t2);
                if (p < S) {
                    if (!ex) nb[p] = c2 + e2;
                    else if (!final_phase) nb[p] = c1 + e1;
                }
                c1 += t1;
                c2 += t2;
            }
            if (!final_phase) { C = c1 & 0xFFFF; M = c1 >> 16; }
            K = c2;
        }
        D2P(4);
        const int Snew = (int)(C + K);
        const bool fin = Snew >= N || Snew == S;
        const bool next_final = !fin && (final_phase || Snew + 3 * (int)M > N);
        // the new list: children in reverse creation order (push_front), then the kept nodes in order
        for (int p = tid; p < S; p += NT) {
            const uint2 rc = R[p];
            if (XR[p] >= 0) {
                const uint32_t pre = nb[p];
                const int cb = pre & 0xFFFF, bb = pre >> 16;
                const uint4 c4 = CH[p];
                const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
                int j = 0, jb = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (cq[q] > 0) {
                        const int np = (int)C - 1 - (cb + j);
                        Rn[np] = dist::child_rect2(rc, q);
                        CNn[np] = cq[q];
                        XRn[np] = cq[q] > 1 ? 0 : -1;
                        CHn[np] = make_uint4(0, 0, 0, 0);
                        if (cq[q] > 1) candl[bb + jb++] = (uint32_t)np;
                        j++;
                    }
                }
            } else {
                const int np = (int)C + (int)nb[p];
                Rn[np] = rc;
                CNn[np] = CN[p];
                XRn[np] = -1;
                CHn[np] = make_uint4(0, 0, 0, 0);
            }
        }
        __syncthreads();
        D2P(5);
        // the pass between rounds: every key to its node's new id (from the scan results), and — unless the list is
        // final — straight away its count in the next round (the new table's expanding nodes); in the final phase
        // wave 0 first sorts the next round's candidates by (size, UL.x) as libstdc++'s introsort orders them (ties
        // included) while the other waves run the pass
        const bool count_next = !fin;
        if (count_next && next_final && wid == 0) {
            const int mn = (int)M;
            for (int i = lane; i < mn; i += 64) {
                const int p = (int)candl[i];
                arr[i].key = (CNn[p] << 12) | (Rn[p].x & 0xFFFFu);
                arr[i].val = (uint32_t)p;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#ifdef MAM_DIST2_PROFILE
            const long long ts0 = clock64();
#endif
            if (mn <= 64) stl_sort_wave2<1>(arr, mn, sortscr);
            else if (mn <= 128) stl_sort_wave2<2>(arr, mn, sortscr);
            else if (mn <= 256) stl_sort_wave2<4>(arr, mn, sortscr);
            else if (lane == 0) stl_sort(arr, arr + mn);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#ifdef MAM_DIST2_PROFILE
            if (lane == 0) atomicAdd(&g_d2prof[l & 7][12], (unsigned long long)(clock64() - ts0));
#endif
            for (int i = lane; i < mn; i += 64) srt[mn - 1 - i] = arr[i].val;   // expansion rank: largest first
        }
        for_keys([&](uint32_t key, uint32_t& nd, int) {
            const int p = nd & 0xFFFF;
            int np;
            if (XR[p] >= 0) {
                const int q = nd >> 16;
                const uint4 c4 = CH[p];
                const int j = (q > 0 && c4.x > 0) + (q > 1 && c4.y > 0) + (q > 2 && c4.z > 0);
                np = (int)C - 1 - ((int)(nb[p] & 0xFFFF) + j);
            } else {
                np = (int)C + (int)nb[p];
            }
            int t = -1;
            if (count_next && XRn[np] >= 0) {
                const int q = dist::quad2(Rn[np], key);
                t = 4 * np + q;
                nd = (uint32_t)np | ((uint32_t)q << 16);
            } else {
                nd = (uint32_t)np;
            }
            if (count_next) dist::agg_add<MAM_DIST_AGG>(reinterpret_cast<uint32_t*>(CHn), t);
        });
        if (count_next) __syncthreads();
        D2P(6);
        S = Snew;
        m = (int)M;
        cur ^= 1;
        if (fin) break;
        final_phase = next_final;
    }

    // ---- 3. retain the best key per node: the first max response in candidate order (:758-776)
    const bool b = cur != 0;
    uint2* const R = b ? rect1 : rect0;
    (void)R;
    uint32_t* best = reinterpret_cast<uint32_t*>(arr);
    uint32_t* wk = srt;
    if (S > L.kp_cap) {
        if (tid == 0) { lc[0] = -1; lc[1] = 0; }
        return;
    }
    for (int p = tid; p < S; p += NT) best[p] = 0;
    __syncthreads();
    for_keys([&](uint32_t key, uint32_t& nd, int k) {
        atomicMax(&best[nd & 0xFFFF], ((key >> 24) << 24) | (0xFFFFFFu - (uint32_t)k));
    });
    __syncthreads();
    for_keys([&](uint32_t key, uint32_t& nd, int k) {
        const int p = nd & 0xFFFF;
        if (best[p] == (((key >> 24) << 24) | (0xFFFFFFu - (uint32_t)k))) wk[p] = key;
    });
    __syncthreads();
    // ---- 4. outputs in list order + lapping ranks (:1141-1162)
    uint32_t* ok = out_key + (size_t)f * g->kp_slots + L.kp_base;
    uint32_t* orr = out_rank + (size_t)f * g->kp_slots + L.kp_base;
    uint32_t st_carry = 0;
    for (int p0 = 0; p0 < S; p0 += NT) {
        const int p = p0 + tid;
        bool st = false;
        uint32_t kv = 0;
        if (p < S) {
            kv = wk[p];
            float xs = (float)((int)(kv & 0xFFF) + L.minBX);
            if (l != 0) xs = xs * L.scale;
            st = xs >= (float)lap0 && xs <= (float)lap1;
        }
        uint32_t e1, e2, t1, t2;
        dist::block_scan2<NT>(st ? 1u : 0u, 0u, part, flip, e1, e2, t1, t2);
        if (p < S) {
            const uint32_t rk = st_carry + e1;
            ok[p] = kv;
            orr[p] = st ? (0x80000000u | rk) : (uint32_t)(p - (int)rk);
        }
        st_carry += t1;
    }
    if (tid == 0) { lc[0] = S; lc[1] = (int)st_carry; }
    D2P(7);
}

}  // namespace mam
