// match.hip — gfx950 ORBmatcher hot-path searches + C-ABI (include/mam_match.h).
//
// Reference semantics (mono, Pinhole):
//   SearchByProjection(F, vpMapPoints)   src/ORBmatcher.cc:43-213   (greedy: a keypoint taken by an earlier
//                                        MapPoint of the same call is skipped by later ones, :88-90)
//   SearchByProjection(Cur, Last)        src/ORBmatcher.cc:1676-1887 + rotation histogram :1855-1884
//   SearchForTriangulation               src/ORBmatcher.cc:907-1146 (per idx1 independent; last equal wins)
//   Fuse(pKF, vpMapPoints, th)           src/ORBmatcher.cc:1148-1338, MapPoint::PredictScale src/MapPoint.cc:514-529
//   MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:329-403
//   Frame grid / GetFeaturesInArea       src/Frame.cc:385-416, 657-735
//
// Stages (one launch each, batched over frames):
//   k_grid     per frame: PosInGrid for every keypoint, LDS counting sort by cell (atomics) + per-cell insertion
//              sort by index -> cell-major list with ascending idx per cell = AssignFeaturesToGrid's cell vectors,
//              stored as 48-byte records (x, y, idx | octave, descriptor) for one-load candidate tests.
//   k_gather   16 lanes (one frame: 64) per search unit (MapPoint / last-frame entry): the window's candidates flattened in
//              GetFeaturesInArea's order (cells ix -> iy, index order inside) and dealt to the lanes; level +
//              radius filters, Hamming distance; only the candidates that can change a result kept (dist <=
//              TH_HIGH, or <= TH_HIGH / nnratio for the ratio test), placed in enumeration order by ballot into a
//              per-unit slot (entry = idx | dist<<16 | level<<25), longer lists into a per-frame overflow area.
//   k_resolve  per frame, one workgroup: the reference's sequential greedy loop replayed exactly as dependency
//              rounds — a unit resolves once every earlier unit sharing a candidate keypoint has; units ready in
//              the same round have disjoint candidates and commit in parallel. Then the rotation-histogram pass.
//   k_tri      SearchForTriangulation: one wave per idx1 of each shared vocabulary node; wave argmin on
//              (dist, -position) implements "dist <= bestDist, last equal wins".
//   k_fuse     Fuse(pKF, vpMapPoints): GW lanes per (keyframe, MapPoint): projection, distance / viewing-angle
//              tests, PredictScale, the window scan of k_gather with Fuse's level + reprojection tests, first minimum
//              distance; the replace-or-add side effects stay on the host (they never change another search).
//   k_distinct MapPoint::ComputeDistinctiveDescriptors: one wave per MapPoint, row medians by binary search.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/mam_match.h"
#include "camera.hpp"
#include "runtime.hpp"

#include <cstdio>

#ifndef MAM_GATHER_LANES
#define MAM_GATHER_LANES 16   // lanes per search unit in k_gather (64 / lanes units per wave)
#endif

namespace mam {

constexpr int NCELLS = MAM_GRID_COLS * MAM_GRID_ROWS;
constexpr int GRID_SORT_MAX = 8192;   // keypoints per frame the grid sort handles (LDS 32 KB)

// One keypoint in grid (cell-major) order: position, index | octave << 16, and its descriptor, so a window scan
// reads one 48-byte record per candidate (no dependent index -> descriptor load).
struct __attribute__((aligned(16))) GridEnt {
    float x, y;
    uint32_t io;              // keypoint index | octave << 16
    uint32_t pad;
    uint4 d0, d1;             // descriptor
};

struct ProjArgs {
    mam_frame_geom g;
    mam_frames_dev fr;
    int mode;                 // 0: local MapPoints, 1: last frame (motion model)
    int unit_stride;          // mp_stride / last_stride
    const int32_t* n_units;   // per frame
    // mode 0
    const mam_mp_track* mps;
    float th, th_far, nnratio;
    int far_points;
    // mode 1
    const mam_pose* tcw;
    mam_camera cam;
    const mam_last_entry* last;
    int check_ori;
    // > 0: TrackWithMotionModel's wider-window retry (Tracking.cc:2816-2824): only frames whose previous search (out_n,
    // on the same outputs) found fewer than retry_below matches search again, the others keep their result
    int retry_below;
    // scratch
    struct GridEnt* grid_ent; // [F][kp_stride] cell-major keypoint records (cell vectors of AssignFeaturesToGrid)
    int32_t* grid_start;      // [F][NCELLS+1]
    int32_t* cand_cnt;        // [F][unit_stride]
    int32_t* cand_off;        // [F][unit_stride]
    uint32_t* pool;           // [F][pool_per_frame]
    int32_t* pool_total;      // [F]
    int pool_per_frame;       // unit_stride * slot_cap + ovf_cap
    int slot_cap;             // candidate slots per unit
    int ovf_cap;              // per-frame overflow area for longer lists (pool_total = used)
    uint32_t* events;         // [F][unit_stride]
    int pool_lds;             // candidate entries the resolve stage stages in LDS
    int flat_lds;             // LDS bytes after the per-keypoint arrays (the flat resolve's unit + entry arrays)
    int32_t* out;             // [F][kp_stride]
    int32_t* out_n;           // [F]
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int desc_dist(const uint8_t* a, const uint8_t* b) {
    const uint4 a0 = reinterpret_cast<const uint4*>(a)[0], a1 = reinterpret_cast<const uint4*>(a)[1];
    const uint4 b0 = reinterpret_cast<const uint4*>(b)[0], b1 = reinterpret_cast<const uint4*>(b)[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ int frame_n(const mam_frames_dev& fr, int f) {
    int n = fr.counts[2 * f];
    return n < 0 ? 0 : (n > fr.kp_stride ? fr.kp_stride : n);
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ unsigned wave_minu(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    return v;
}

// ------------------------------------------------------------------------------------------------ grid
__global__ __launch_bounds__(1024) void k_grid(ProjArgs p) {
    __shared__ int cnt[NCELLS + 1];
    __shared__ int start[NCELLS + 1];
    __shared__ uint16_t cellOf[GRID_SORT_MAX];
    __shared__ uint16_t sorted[GRID_SORT_MAX];
    __shared__ int wsum[16];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = frame_n(p.fr, f);
    if (tid == 0) {   // per-call state of frame f (k_gather and k_resolve run after this kernel on the stream)
        p.out_n[f] = n > GRID_SORT_MAX ? MAM_ERR_CAPACITY : 0;
        p.pool_total[f] = 0;
    }
    if (n > GRID_SORT_MAX) return;
    const mam_keypoint* K = p.fr.keys + (size_t)f * p.fr.kp_stride;
    for (int c = tid; c <= NCELLS; c += 1024) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        // PosInGrid (Frame.cc:725-735): std::round (half away from zero)
        const int posX = (int)roundf((K[i].x - p.g.min_x) * p.g.grid_inv_w);
        const int posY = (int)roundf((K[i].y - p.g.min_y) * p.g.grid_inv_h);
        uint16_t cell = 0xFFFF;
        if (!(posX < 0 || posX >= MAM_GRID_COLS || posY < 0 || posY >= MAM_GRID_ROWS)) {
            cell = (uint16_t)(posX * MAM_GRID_ROWS + posY);   // ix-major, then iy: GetFeaturesInArea's order
            atomicAdd(&cnt[cell], 1);
        }
        cellOf[i] = cell;
    }
    __syncthreads();
    // exclusive scan of the 3072 cell counts: 3 cells per thread
    const int c0 = 3 * tid;
    const int a0 = cnt[c0], a1 = cnt[c0 + 1], a2 = cnt[c0 + 2];
    const int v = a0 + a1 + a2;
    const int incl = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
        if (w < wid) pre += wsum[w];
        tot += wsum[w];
    }
    const int base = pre + incl - v;
    start[c0] = base;
    start[c0 + 1] = base + a0;
    start[c0 + 2] = base + a0 + a1;
    if (tid == 0) start[NCELLS] = tot;
    __syncthreads();
    for (int c = tid; c < NCELLS; c += 1024) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int cell = cellOf[i];
        if (cell != 0xFFFF) sorted[start[cell] + atomicAdd(&cnt[cell], 1)] = (uint16_t)i;
    }
    __syncthreads();
    // atomics placed each cell's entries in arbitrary order: restore ascending keypoint index
    for (int c = tid; c < NCELLS; c += 1024) {
        const int b0 = start[c], b1 = start[c + 1];
        for (int k = b0 + 1; k < b1; k++) {
            const uint16_t val = sorted[k];
            int m = k - 1;
            while (m >= b0 && sorted[m] > val) { sorted[m + 1] = sorted[m]; m--; }
            sorted[m + 1] = val;
        }
    }
    __syncthreads();
    int32_t* gs = p.grid_start + (size_t)f * (NCELLS + 1);
    for (int c = tid; c <= NCELLS; c += 1024) gs[c] = start[c];
    const size_t off = (size_t)f * p.fr.kp_stride;
    const uint4* D = reinterpret_cast<const uint4*>(p.fr.desc + (size_t)f * p.fr.kp_stride * 32);
    for (int k = tid; k < tot; k += 1024) {
        const int i = sorted[k];
        GridEnt e;
        e.x = K[i].x;
        e.y = K[i].y;
        e.io = (uint32_t)i | ((uint32_t)(uint8_t)K[i].octave << 16);
        e.pad = 0;
        e.d0 = D[2 * i];
        e.d1 = D[2 * i + 1];
        p.grid_ent[off + k] = e;
    }
}

// ------------------------------------------------------------------------------------------------ gather
struct Window {
    float x, y, r;
    int minL, maxL;
    bool checkL;
    int cx0, cx1, cy0, cy1;
    const uint8_t* desc;
};

// GetFeaturesInArea's cell range (Frame.cc:665-687, KeyFrame.cc:712-726); false = the call returns empty.
__device__ __forceinline__ bool window_cells(const mam_frame_geom& g, Window* w) {
    const float r = w->r;
    w->cx0 = max(0, (int)floorf((w->x - g.min_x - r) * g.grid_inv_w));
    if (w->cx0 >= MAM_GRID_COLS) return false;
    w->cx1 = min(MAM_GRID_COLS - 1, (int)ceilf((w->x - g.min_x + r) * g.grid_inv_w));
    if (w->cx1 < 0) return false;
    w->cy0 = max(0, (int)floorf((w->y - g.min_y - r) * g.grid_inv_h));
    if (w->cy0 >= MAM_GRID_ROWS) return false;
    w->cy1 = min(MAM_GRID_ROWS - 1, (int)ceilf((w->y - g.min_y + r) * g.grid_inv_h));
    if (w->cy1 < 0) return false;
    return true;
}

// Search window of unit j of frame f; false = the reference `continue`s before or inside GetFeaturesInArea.
__device__ bool unit_window(const ProjArgs& p, int f, int j, Window* w) {
    if (j >= p.n_units[f]) return false;
    if (p.mode == 0) {
        const mam_mp_track& mp = p.mps[(size_t)f * p.unit_stride + j];
        if (!mp.track_in_view) return false;
        if (p.far_points && mp.track_depth > p.th_far) return false;
        if (mp.is_bad) return false;
        const int lvl = mp.scale_level;
        float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos (ORBmatcher.cc:215-221)
        if (p.th != 1.0f) r *= p.th;
        w->x = mp.proj_x;
        w->y = mp.proj_y;
        w->r = r * p.g.scale_factors[lvl];
        w->minL = lvl - 1;
        w->maxL = lvl;
        w->desc = mp.desc;
    } else {
        const mam_last_entry& L = p.last[(size_t)f * p.unit_stride + j];
        if (!L.valid) return false;
        const mam_pose& T = p.tcw[f];
        // Sophus SE3f action (so3.hpp:358-367, se3.hpp:321-324), evaluated as written
        const float qx = T.q[0], qy = T.q[1], qz = T.q[2], qw = T.q[3];
        const float px = L.pos[0], py = L.pos[1], pz = L.pos[2];
        float u0 = qy * pz - qz * py, u1 = qz * px - qx * pz, u2 = qx * py - qy * px;
        u0 += u0; u1 += u1; u2 += u2;
        const float c0 = qy * u2 - qz * u1, c1 = qz * u0 - qx * u2, c2 = qx * u1 - qy * u0;
        const float xc = ((px + qw * u0) + c0) + T.t[0];
        const float yc = ((py + qw * u1) + c1) + T.t[1];
        const float zc = ((pz + qw * u2) + c2) + T.t[2];
        const float invzc = (float)(1.0 / (double)zc);
        if (invzc < 0) return false;
        float u, v;
        cam::project_f(p.cam, xc, yc, zc, &u, &v);   // CurrentFrame.mpCamera->project(x3Dc) (ORBmatcher.cc:1713)
        if (u < p.g.min_x || u > p.g.max_x) return false;
        if (v < p.g.min_y || v > p.g.max_y) return false;
        w->x = u;
        w->y = v;
        w->r = p.th * p.g.scale_factors[L.octave];
        w->minL = L.octave - 1;
        w->maxL = L.octave + 1;
        w->desc = L.desc;
    }
    w->checkL = (w->minL > 0) || (w->maxL >= 0);
    return window_cells(p.g, w);
}

// A candidate is RELEVANT to its unit if its taken state can change the unit's result: dist <= TH_HIGH (it could
// be the pick) or, in the ratio-tested local search, dist <= TH_HIGH / nnratio (it could be the second best that
// fails the test). Irrelevant candidates never change a result (nor any other unit's), so only relevant ones are
// kept, in GetFeaturesInArea enumeration order.
__device__ __forceinline__ int rel_threshold(const ProjArgs& p) {
    return p.mode == 1 ? MAM_TH_HIGH
                       : (p.nnratio > 0.f ? min(256, (int)ceilf((float)MAM_TH_HIGH / p.nnratio) + 1) : 256);
}

// One pass over a unit's window by a group of GW lanes (64 / GW units per wave): the window's candidates (cells in
// ix -> iy order, each cell's keypoints in index order: GetFeaturesInArea's enumeration) are flattened and dealt
// to the group's lanes GW at a time; each lane finds its cell by a binary search over the group's cell-count scan,
// tests level / radius / distance, and a ballot (restricted to the group) places the relevant ones in order.
// Entries at positions < lim are written to dst. Returns the relevant count. Loop bounds are group-uniform, so a
// group is either wholly active or wholly idle in every iteration (the width-GW shuffles stay inside it).
template <int GW>
__device__ int gather_pass(const ProjArgs& p, int f, const Window& w, int rel, const uint4 u0, const uint4 u1,
                           uint32_t* dst, int lim) {
    const int lane = lane_id();
    const int gl = lane & (GW - 1);
    const int gb = lane & ~(GW - 1);   // first lane of the group
    const int ny = w.cy1 - w.cy0 + 1;
    const int ncell = (w.cx1 - w.cx0 + 1) * ny;
    const int32_t* gs = p.grid_start + (size_t)f * (NCELLS + 1);
    const GridEnt* G = p.grid_ent + (size_t)f * p.fr.kp_stride;
    const uint64_t below = (1ull << lane) - (1ull << gb);
    const uint64_t gmask = GW == 64 ? ~0ull : (((1ull << GW) - 1ull) << gb);
    int base = 0;
    for (int e0 = 0; e0 < ncell; e0 += GW) {
        const int e = e0 + gl;
        int k0 = 0, c = 0;
        if (e < ncell) {
            const int ix = w.cx0 + e / ny, iy = w.cy0 + e % ny;
            const int cell = ix * MAM_GRID_ROWS + iy;
            k0 = gs[cell];
            c = gs[cell + 1] - k0;
        }
        int incl = c;
#pragma unroll
        for (int o = 1; o < GW; o <<= 1) {
            const int t = __shfl_up(incl, o, GW);
            if (gl >= o) incl += t;
        }
        const int tot = __shfl(incl, GW - 1, GW);
        const int kb = k0 - (incl - c);   // record index of candidate t in this lane's cell = kb + t
        for (int t0 = 0; t0 < tot; t0 += GW) {
            const int t = t0 + gl;
            int m = 0;   // owner cell: first m with incl[m] > t
#pragma unroll
            for (int step = GW / 2; step >= 1; step >>= 1)
                if (__shfl(incl, m + step - 1, GW) <= t) m += step;
            const int k = __shfl(kb, m, GW) + t;
            bool ok = false;
            uint32_t ent = 0;
            if (t < tot) {
                const GridEnt ge = G[k];
                const int oct = (int)(ge.io >> 16);
                const bool lvl_ok = !w.checkL || (oct >= w.minL && (w.maxL < 0 || oct <= w.maxL));
                const float dx = ge.x - w.x, dy = ge.y - w.y;
                if (lvl_ok && fabsf(dx) < w.r && fabsf(dy) < w.r) {
                    const int dist = __popc(u0.x ^ ge.d0.x) + __popc(u0.y ^ ge.d0.y) + __popc(u0.z ^ ge.d0.z) +
                                     __popc(u0.w ^ ge.d0.w) + __popc(u1.x ^ ge.d1.x) + __popc(u1.y ^ ge.d1.y) +
                                     __popc(u1.z ^ ge.d1.z) + __popc(u1.w ^ ge.d1.w);
                    if (dist <= rel) {
                        ok = true;
                        ent = (ge.io & 0xFFFFu) | ((uint32_t)dist << 16) | ((uint32_t)oct << 25);
                    }
                }
            }
            const uint64_t bal = __ballot(ok) & gmask;
            const int o = base + __popcll(bal & below);
            if (ok && o < lim) dst[o] = ent;
            base += __popcll(bal);
        }
    }
    return base;
}

// GW lanes per unit (64 / GW units per wave). Lists go to a fixed slot of slot_cap entries per unit; a longer list
// is written again into the frame's overflow area (atomic allocation; the list stays contiguous and in order).
template <int GW>
__global__ __launch_bounds__(256) void k_gather(ProjArgs p, int nframes) {
    const long long gu = ((long long)blockIdx.x * 256 + threadIdx.x) / GW;   // global unit slot
    const int f = (int)(gu / p.unit_stride);
    const int j = (int)(gu - (long long)f * p.unit_stride);
    const bool live = f < nframes;
    const int gl = lane_id() & (GW - 1);
    int32_t* cntp = p.cand_cnt + (size_t)f * p.unit_stride + j;
    int32_t* offp = p.cand_off + (size_t)f * p.unit_stride + j;
    Window w;
    if (!live) return;
    if (p.retry_below > 0) {   // a frame the first search served (or reported an error for) is not searched again
        const int pn = p.out_n[f];
        if (pn < 0 || pn >= p.retry_below) return;
    }
    if (!unit_window(p, f, j, &w)) {
        if (gl == 0) { *cntp = 0; *offp = 0; }
        return;
    }
    uint32_t* fpool = p.pool + (size_t)f * p.pool_per_frame;
    const int rel = rel_threshold(p);
    const int CAP = p.slot_cap;
    const uint4 u0 = reinterpret_cast<const uint4*>(w.desc)[0], u1 = reinterpret_cast<const uint4*>(w.desc)[1];
    int total = gather_pass<GW>(p, f, w, rel, u0, u1, fpool + (size_t)j * CAP, CAP);
    int off = j * CAP;
    if (total > CAP) {
        int o2 = 0;
        if (gl == 0) o2 = atomicAdd(&p.pool_total[f], total);
        o2 = __shfl(o2, 0, GW);
        if (o2 + total <= p.ovf_cap) {
            off = p.unit_stride * CAP + o2;
            gather_pass<GW>(p, f, w, rel, u0, u1, fpool + off, total);
        } else {
            total = 0;   // capacity: pool_total > ovf_cap makes the resolve stage report the frame
        }
    }
    if (gl == 0) { *cntp = total; *offp = off; }
}

// ------------------------------------------------------------------------------------------------ resolve
__device__ __forceinline__ int rot_bin(float rot) {
    const float factor = 1.0f / MAM_HISTO_LENGTH;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == MAM_HISTO_LENGTH) bin = 0;
    return bin;
}

// Greedy resolve as dependency rounds. Unit u's outcome depends only on the taken-state of its candidate
// keypoints, which only earlier units sharing a candidate can change. Each round: every open unit writes its index
// into minU[k] (atomicMin) for each candidate k; a unit is READY when it is the minimum on all its candidates
// (every earlier unit sharing one is already final). Ready units have pairwise disjoint candidate sets, so they
// resolve and commit in parallel with exactly the sequential loop's result (ORBmatcher.cc:84-128 / :1745-1772):
// taken bits, out[] (a later round = a later unit overwrites: last writer wins), match counts, rotation events.
#ifdef MAM_RESOLVE_PROFILE
__device__ unsigned long long g_rprof[2][8];
#define RPROF(k) do { __syncthreads(); if (t == 0) { const long long tn = clock64(); atomicAdd(&g_rprof[p.mode][k], (unsigned long long)(tn - rp0)); rp0 = tn; } } while (0)
#else
#define RPROF(k) do {} while (0)
#endif
constexpr int RESOLVE_THREADS = 1024;

__host__ __device__ inline size_t a16(size_t b) { return (b + 15) & ~(size_t)15; }
// flat resolve carve after the per-keypoint arrays: ebase, best, second (u32 per unit), flags, notready (u8 per
// unit), entries (u32) and their units (u16)
__host__ __device__ inline size_t flat_carve_bytes(int nu, int ne) {
    return a16((size_t)(nu + 1) * 4) + 2 * a16((size_t)nu * 4) + 2 * a16((size_t)nu) + a16((size_t)ne * 4) +
           3 * a16((size_t)ne * 2);
}
constexpr int RESOLVE_POOL_LDS = 24576;   // candidate entries staged in LDS per frame (up to 96 KB)

__global__ __launch_bounds__(RESOLVE_THREADS) void k_resolve(ProjArgs p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int f = blockIdx.x, t = threadIdx.x;
    const int S = p.fr.kp_stride;
    const int nwords = (S + 31) / 32;
    uint32_t* takenb = reinterpret_cast<uint32_t*>(smem);                              // S bits
    int* minU = reinterpret_cast<int*>(smem + ((nwords * 4 + 15) & ~15));             // per keypoint
    int* minA = minU + ((S + 3) & ~3);                                                 // per keypoint
    int* outU = minA + ((S + 3) & ~3);                                                 // last assigner
    uint32_t* cpool = reinterpret_cast<uint32_t*>(outU + ((S + 3) & ~3));              // staged candidates
    __shared__ int hist[MAM_HISTO_LENGTH];
    __shared__ int top[3];
    __shared__ int s_nm, s_nev;
    const int n = frame_n(p.fr, f);
    int32_t* out = p.out + (size_t)f * S;
#ifdef MAM_RESOLVE_PROFILE
    long long rp0 = clock64();
#endif
    if (p.retry_below > 0) {   // as k_gather: frames with enough matches (or an error) keep the first search's result
        const int pn = p.out_n[f];
        if (pn < 0 || pn >= p.retry_below) return;
    }
    const int ptot = p.pool_total[f];
    __syncthreads();
    // reset for the next search on this context: a search that reuses the grid (mam_frames_dev.reuse_grid) skips
    // k_grid, which otherwise zeroes it
    if (t == 0) p.pool_total[f] = 0;
    if (n > GRID_SORT_MAX) {   // the grid stage could not sort this frame
        if (t == 0) p.out_n[f] = MAM_ERR_CAPACITY;
        return;
    }
    if (ptot > p.ovf_cap) {   // a list did not fit its slot nor the overflow area
        if (t == 0) p.out_n[f] = MAM_ERR_CAPACITY;
        return;
    }
    const int nu = p.n_units[f];
    // each thread owns units t, t + 1024, ... (at most UPT)
    constexpr int UPT = 4;
    if (nu > UPT * RESOLVE_THREADS) {
        if (t == 0) p.out_n[f] = MAM_ERR_CAPACITY;
        return;
    }
    const uint32_t* gpool = p.pool + (size_t)f * p.pool_per_frame;
    const int32_t* cc = p.cand_cnt + (size_t)f * p.unit_stride;
    const int32_t* co = p.cand_off + (size_t)f * p.unit_stride;
    uint32_t* ev = p.events + (size_t)f * p.unit_stride;
    const mam_keypoint* K = p.fr.keys + (size_t)f * S;
    // per-unit scalars first (global loads in flight together): list count / offset, nObs
    int ucnt[UPT], uoff[UPT], unobs[UPT];
#pragma unroll
    for (int k = 0; k < UPT; k++) {
        const int u = t + k * RESOLVE_THREADS;
        ucnt[k] = 0;
        uoff[k] = 0;
        unobs[k] = 0;
        if (u < nu) {
            ucnt[k] = cc[u];
            uoff[k] = co[u];
            unobs[k] = p.mode == 0 ? p.mps[(size_t)f * p.unit_stride + u].nobs
                                   : p.last[(size_t)f * p.unit_stride + u].nobs;
        }
    }
    for (int i = t; i < n; i += RESOLVE_THREADS) out[i] = -1;
    if (p.fr.taken) {
        const uint8_t* tk = p.fr.taken + (size_t)f * S;
        for (int w = t; w < nwords; w += RESOLVE_THREADS) {
            uint8_t v[32];
#pragma unroll
            for (int b = 0; b < 32; b++) v[b] = w * 32 + b < n ? tk[w * 32 + b] : 0;
            uint32_t bits = 0;
#pragma unroll
            for (int b = 0; b < 32; b++) bits |= (v[b] ? 1u : 0u) << b;
            takenb[w] = bits;
        }
    } else {
        for (int w = t; w < nwords; w += RESOLVE_THREADS) takenb[w] = 0;
    }
    for (int i = t; i < S; i += RESOLVE_THREADS) { minU[i] = 0x7FFFFFFF; minA[i] = 0x7FFFFFFF; outU[i] = -1; }
    if (t < MAM_HISTO_LENGTH) hist[t] = 0;
    if (t == 0) { s_nm = 0; s_nev = 0; }
    // A candidate is RELEVANT to its unit if its taken state can change the unit's result: dist <= TH_HIGH (it
    // could be the pick) or, in the ratio-tested local search, dist <= TH_HIGH / nnratio (it could be the second
    // best that fails the test). k_gather keeps only relevant candidates (same rel_threshold), so the lists are
    // staged as they are.
    int nm = 0;
    // ---- flat path: the candidate lists as one entry array (entry -> unit), every round a few passes over the
    //      entries dealt evenly to all threads; per-unit best / second best by LDS atomicMin on (dist << 16 | entry)
    //      (the first minimum in list order is the sequential loop's best, the first minimum of the rest its second
    //      best, ORBmatcher.cc:94-112). Falls back to the per-unit loop below when the entries do not fit in LDS.
    __shared__ int wtot4[UPT][RESOLVE_THREADS / 64];
    {
#pragma unroll
        for (int k = 0; k < UPT; k++) {
            const int incl = wave_incl_scan(ucnt[k]);
            if ((t & 63) == 63) wtot4[k][t >> 6] = incl;
        }
    }
    __syncthreads();
    int ebase_k[UPT], etotal = 0;
    {
        int carry = 0;
#pragma unroll
        for (int k = 0; k < UPT; k++) {
            int pre = 0, tot = 0;
            for (int w = 0; w < RESOLVE_THREADS / 64; w++) {
                const int v = wtot4[k][w];
                if (w < (t >> 6)) pre += v;
                tot += v;
            }
            ebase_k[k] = carry + pre + wave_incl_scan(ucnt[k]) - ucnt[k];
            carry += tot;
        }
        etotal = carry;
    }
    const size_t flat_bytes = flat_carve_bytes(nu, etotal);
    if (etotal <= 0xFFFF && flat_bytes <= (size_t)p.flat_lds) {
        uint8_t* fp = reinterpret_cast<uint8_t*>(cpool);
        int* ebase = reinterpret_cast<int*>(fp);                         fp += a16((size_t)(nu + 1) * 4);
        uint32_t* best = reinterpret_cast<uint32_t*>(fp);                 fp += a16((size_t)nu * 4);   // list offset first
        uint32_t* second = reinterpret_cast<uint32_t*>(fp);               fp += a16((size_t)nu * 4);
        uint8_t* flags = fp;                                              fp += a16((size_t)nu);       // 1 open, 2 taker
        uint8_t* notready = fp;                                           fp += a16((size_t)nu);
        uint32_t* epool = reinterpret_cast<uint32_t*>(fp);                fp += a16((size_t)etotal * 4);
        uint16_t* eunit = reinterpret_cast<uint16_t*>(fp);                fp += a16((size_t)etotal * 2);   // | taker << 15
        uint16_t* act0 = reinterpret_cast<uint16_t*>(fp);                 fp += a16((size_t)etotal * 2);   // active entries
        uint16_t* act1 = reinterpret_cast<uint16_t*>(fp);
        unsigned open = 0;
#pragma unroll
        for (int k = 0; k < UPT; k++) {
            const int u = t + k * RESOLVE_THREADS;
            if (u < nu) {
                const bool op = ucnt[k] > 0;
                ebase[u] = ebase_k[k];
                best[u] = (uint32_t)uoff[k];
                second[u] = 0xFFFFFFFFu;
                flags[u] = (op ? 1 : 0) | (unobs[k] > 0 ? 2 : 0);
                notready[u] = 0;
                if (op) open |= 1u << k;
            }
        }
        if (t == 0) ebase[nu] = etotal;
        __syncthreads();
        // entries in unit order: entry i belongs to the last unit with ebase <= i; all global loads of a pass in
        // flight together
        for (int i0 = 0; i0 < etotal; i0 += 4 * RESOLVE_THREADS) {
            uint32_t v[4];
            int uu[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int i = i0 + q * RESOLVE_THREADS + t;
                v[q] = 0;
                uu[q] = 0;
                if (i < etotal) {
                    int lo = 0, hi = nu;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (ebase[mid] <= i) lo = mid;
                        else hi = mid;
                    }
                    uu[q] = lo;
                    v[q] = gpool[best[lo] + (i - ebase[lo])];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int i = i0 + q * RESOLVE_THREADS + t;
                if (i < etotal) {
                    epool[i] = v[q];
                    eunit[i] = (uint16_t)(uu[q] | ((flags[uu[q]] & 2) << 14));
                    act0[i] = (uint16_t)i;
                }
            }
        }
        __syncthreads();
        for (int u = t; u < nu; u += RESOLVE_THREADS) best[u] = 0xFFFFFFFFu;
        RPROF(0);
        int round = 0;
        __shared__ int s_acnt;
        if (t == 0) s_acnt = 0;
        int acnt = etotal;   // entries of open units (every unit with entries is open in round 0)
        uint16_t* act = act0;
        uint16_t* nxt = act1;
        while (acnt > 0) {
#ifdef MAM_RESOLVE_PROFILE
            if (t == 0) atomicAdd(&g_rprof[p.mode][6], 1ull);
#endif
            const int stamp = (0xFFF - round) << 12;
            // (1) claims (see the per-unit loop below for minU / minA)
            for (int j = t; j < acnt; j += RESOLVE_THREADS) {
                const int i = act[j];
                const int ut = eunit[i], u = ut & 0x7FFF;
                const uint32_t e = epool[i];
                const int key = stamp | u;
                atomicMin(&minA[e & 0xFFFFu], key);
                if ((ut & 0x8000) && (int)((e >> 16) & 0x1FFu) <= MAM_TH_HIGH) atomicMin(&minU[e & 0xFFFFu], key);
            }
            __syncthreads();
            RPROF(3);
            // (2) readiness (one failing candidate makes its unit wait a round) and, speculatively for every open
            //     unit, its best untaken candidate (taken bits only change in the commit below)
            for (int j = t; j < acnt; j += RESOLVE_THREADS) {
                const int i = act[j];
                const int ut = eunit[i], u = ut & 0x7FFF;
                const uint32_t e = epool[i];
                const int key = stamp | u;
                const int dist = (int)((e >> 16) & 0x1FFu);
                const int idx = (int)(e & 0xFFFFu);
                const bool ok = minU[idx] >= key && (!(ut & 0x8000) || dist > MAM_TH_HIGH || minA[idx] >= key);
                if (!ok) notready[u] = 1;
                if (!((takenb[idx >> 5] >> (idx & 31)) & 1u)) atomicMin(&best[u], ((uint32_t)dist << 16) | (uint32_t)i);
            }
            __syncthreads();
            // (3) second best of the ready units (the ratio test of the local-map search)
            if (p.mode == 0) {
                for (int j = t; j < acnt; j += RESOLVE_THREADS) {
                    const int i = act[j];
                    const int u = eunit[i] & 0x7FFF;
                    if (notready[u]) continue;
                    const uint32_t b = best[u];
                    if (b == 0xFFFFFFFFu || (int)(b & 0xFFFFu) == i) continue;
                    const uint32_t e = epool[i];
                    const int idx = (int)(e & 0xFFFFu);
                    if ((takenb[idx >> 5] >> (idx & 31)) & 1u) continue;
                    atomicMin(&second[u], (((e >> 16) & 0x1FFu) << 16) | (uint32_t)i);
                }
                __syncthreads();
            }
            // (4) ready units commit (each thread its own units)
#pragma unroll
            for (int k = 0; k < UPT; k++) {
                if (!((open >> k) & 1u)) continue;
                const int u = t + k * RESOLVE_THREADS;
                if (notready[u]) {
                    notready[u] = 0;
                    best[u] = 0xFFFFFFFFu;
                    second[u] = 0xFFFFFFFFu;
                    continue;
                }
                open &= ~(1u << k);
                flags[u] = 0;
                const uint32_t b = best[u];
                if (b == 0xFFFFFFFFu) continue;
                const uint32_t eb = epool[b & 0xFFFFu];
                const int bestDist = (int)(b >> 16), bestLevel = (int)(eb >> 25), bestIdx = (int)(eb & 0xFFFFu);
                bool assign = bestDist <= MAM_TH_HIGH;
                if (assign && p.mode == 0) {
                    const uint32_t s2 = second[u];
                    const int bestDist2 = s2 == 0xFFFFFFFFu ? 256 : (int)(s2 >> 16);
                    const int bestLevel2 = s2 == 0xFFFFFFFFu ? -1 : (int)(epool[s2 & 0xFFFFu] >> 25);
                    if (bestLevel == bestLevel2 && bestDist > p.nnratio * bestDist2) assign = false;
                }
                if (!assign) continue;
                atomicMax(&outU[bestIdx], u);
                if ((unobs[k] > 0)) atomicOr(&takenb[bestIdx >> 5], 1u << (bestIdx & 31));
                nm++;
                if (p.mode == 1 && p.check_ori) ev[atomicAdd(&s_nev, 1)] = (uint32_t)bestIdx | ((uint32_t)u << 16);
            }
            __syncthreads();
            // (5) the entries of the units still open, in any order (positions carry no meaning; the entry
            //     index does): one LDS atomic per wave and pass
            for (int j0 = 0; j0 < acnt; j0 += RESOLVE_THREADS) {
                const int j = j0 + t;
                int i = 0;
                bool keep = false;
                if (j < acnt) {
                    i = act[j];
                    keep = flags[eunit[i] & 0x7FFF] & 1;
                }
                const uint64_t m = __ballot(keep);
                int base = 0;
                if ((t & 63) == 0 && m) base = atomicAdd(&s_acnt, __popcll(m));
                base = __shfl(base, 0, 64);
                if (keep) nxt[base + __popcll(m & ((1ull << (t & 63)) - 1ull))] = (uint16_t)i;
            }
            __syncthreads();
            acnt = s_acnt;
            __syncthreads();
            if (t == 0) s_acnt = 0;
            uint16_t* tmp = act;
            act = nxt;
            nxt = tmp;
            round++;
            RPROF(5);
        }
    } else {
        int mysum = 0;
    #pragma unroll
        for (int k = 0; k < UPT; k++) mysum += ucnt[k];
        // block exclusive scan of the per-thread counts
        __shared__ int wtot[RESOLVE_THREADS / 64];
        const int incl = wave_incl_scan(mysum);
        if ((t & 63) == 63) wtot[t >> 6] = incl;
        __syncthreads();
        int base = incl - mysum, total = 0;
        for (int w = 0; w < RESOLVE_THREADS / 64; w++) {
            if (w < (t >> 6)) base += wtot[w];
            total += wtot[w];
        }
        const bool staged = total <= p.pool_lds;
        if (staged) {
    #pragma unroll
            for (int k = 0; k < UPT; k++) {
                const uint32_t* lst = gpool + uoff[k];
                const int cnt = ucnt[k];
                int q = 0;
                for (; q + 4 <= cnt; q += 4) {   // four loads in flight per step
                    const uint32_t e0 = lst[q], e1 = lst[q + 1], e2 = lst[q + 2], e3 = lst[q + 3];
                    cpool[base + q] = e0;
                    cpool[base + q + 1] = e1;
                    cpool[base + q + 2] = e2;
                    cpool[base + q + 3] = e3;
                }
                for (; q < cnt; q++) cpool[base + q] = lst[q];
                uoff[k] = base;
                base += cnt;
            }
        }
        const uint32_t* pool = staged ? cpool : gpool;
        unsigned open = 0, taker = 0;
    #pragma unroll
        for (int k = 0; k < UPT; k++) {
            if (ucnt[k] > 0) {
                open |= 1u << k;
                if (unobs[k] > 0) taker |= 1u << k;
            }
        }
        __syncthreads();
        RPROF(0);
        // Claims carry the round in their high bits, (0xFFF - round) << 12 | unit, so a later round's claim is always
        // smaller than any earlier one and claims never need releasing: a value from an older round reads as "none".
        int round = 0;
        while (__syncthreads_or(open != 0)) {
    #ifdef MAM_RESOLVE_PROFILE
            if (t == 0) atomicAdd(&g_rprof[p.mode][6], 1ull);
    #endif
            const int stamp = (0xFFF - round) << 12;
            // (1) claims. minU[k]: earliest open unit that could TAKE k (nObs > 0 and dist <= TH_HIGH); minA[k]: earliest
            //     open unit to which k is relevant.
            for (int k = 0; k < UPT; k++) {
                if (!((open >> k) & 1u)) continue;
                const int key = stamp | (t + k * RESOLVE_THREADS);
                const uint32_t* lst = pool + uoff[k];
                const int cnt = ucnt[k];
                const bool tk = (taker >> k) & 1u;
                for (int q = 0; q < cnt; q++) {
                    const uint32_t e = lst[q];
                    const int dist = (int)((e >> 16) & 0x1FFu);
                    atomicMin(&minA[e & 0xFFFFu], key);
                    if (tk && dist <= MAM_TH_HIGH) atomicMin(&minU[e & 0xFFFFu], key);
                }
            }
            __syncthreads();
            RPROF(3);
            // (2) ready units resolve and commit
            for (int k = 0; k < UPT; k++) {
                if (!((open >> k) & 1u)) continue;
                const int u = t + k * RESOLVE_THREADS;
                const int key = stamp | u;
                const uint32_t* lst = pool + uoff[k];
                const int cnt = ucnt[k];
                // ready: no earlier open unit can take one of u's candidates, and (if u takes) no earlier open unit
                // looks at a keypoint u could take (a claim left from an older round is larger than any of this round's,
                // so it never blocks)
                const bool tk = (taker >> k) & 1u;
                bool ready = true;
                for (int q = 0; q < cnt && ready; q++) {
                    const uint32_t e = lst[q];
                    const int dist = (int)((e >> 16) & 0x1FFu);
                    const int mu = minU[e & 0xFFFFu], ma = minA[e & 0xFFFFu];
                    ready = mu >= key && (!tk || dist > MAM_TH_HIGH || ma >= key);
                }
                if (!ready) continue;
                open &= ~(1u << k);
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (int q = 0; q < cnt; q++) {
                    const uint32_t e = lst[q];
                    const int idx = (int)(e & 0xFFFFu);
                    if ((takenb[idx >> 5] >> (idx & 31)) & 1u) continue;
                    const int dist = (int)((e >> 16) & 0x1FFu);
                    const int lvl = (int)(e >> 25);
                    if (dist < bestDist) {
                        bestDist2 = bestDist; bestDist = dist;
                        bestLevel2 = bestLevel; bestLevel = lvl;
                        bestIdx = idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = lvl;
                        bestDist2 = dist;
                    }
                }
                bool assign = bestDist <= MAM_TH_HIGH;
                if (assign && p.mode == 0 && bestLevel == bestLevel2 && bestDist > p.nnratio * bestDist2) assign = false;
                if (!assign) continue;
                atomicMax(&outU[bestIdx], u);   // units that do not take may assign the same keypoint: last wins
                if (tk) atomicOr(&takenb[bestIdx >> 5], 1u << (bestIdx & 31));
                nm++;
                if (p.mode == 1 && p.check_ori) ev[atomicAdd(&s_nev, 1)] = (uint32_t)bestIdx | ((uint32_t)u << 16);
            }
            round++;
            RPROF(5);
        }
    }
    RPROF(1);
    atomicAdd(&s_nm, nm);
    __syncthreads();
    for (int i = t; i < n; i += RESOLVE_THREADS) out[i] = outU[i];
    __syncthreads();
    const int nev = s_nev;
    // (4) rotation consistency (ORBmatcher.cc:1855-1884, ComputeThreeMaxima :2012-2053); the bins of the
    //     committed matches are computed here, all in parallel
    if (p.mode == 1 && p.check_ori) {
        for (int e = t; e < nev; e += RESOLVE_THREADS) {
            const uint32_t v = ev[e];
            const int idx = (int)(v & 0xFFFFu), u = (int)(v >> 16);
            const int bin = rot_bin(p.last[(size_t)f * p.unit_stride + u].angle - K[idx].angle);
            ev[e] = (uint32_t)idx | ((uint32_t)bin << 16);
            atomicAdd(&hist[bin], 1);
        }
        __syncthreads();
        if (t == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < MAM_HISTO_LENGTH; i++) {
                const int sh = hist[i];
                if (sh > max1) { max3 = max2; max2 = max1; max1 = sh; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (sh > max2) { max3 = max2; max2 = sh; ind3 = ind2; ind2 = i; }
                else if (sh > max3) { max3 = sh; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            top[0] = ind1; top[1] = ind2; top[2] = ind3;
        }
        __syncthreads();
        int removed = 0;
        for (int e = t; e < nev; e += RESOLVE_THREADS) {
            const int bin = (int)(ev[e] >> 16);
            if (bin != top[0] && bin != top[1] && bin != top[2]) {
                const uint32_t idx = ev[e] & 0xFFFFu;
                out[idx] = MAM_MATCH_CLEARED;
                atomicAnd(&takenb[idx >> 5], ~(1u << (idx & 31)));   // the slot becomes NULL
                removed++;
            }
        }
        if (removed) atomicAdd(&s_nm, -removed);
        __syncthreads();
    }
    RPROF(2);
#ifdef MAM_RESOLVE_PROFILE
    if (t == 0) atomicAdd(&g_rprof[p.mode][7], 1ull);
#endif
    if (p.fr.taken_out) {
        // the frame's slot state after the call (mvpMapPoints[i] != NULL && Observations() > 0): what the next
        // search of the same frame reads as `taken`
        __syncthreads();
        uint8_t* to = p.fr.taken_out + (size_t)f * S;
        for (int i = t; i < S; i += RESOLVE_THREADS) to[i] = i < n ? (uint8_t)((takenb[i >> 5] >> (i & 31)) & 1u) : 0;
    }
    if (t == 0) p.out_n[f] = s_nm;
}

// ------------------------------------------------------------------------------------------------ triangulation
struct TriArgs {
    mam_frame_geom g;
    const mam_keypoint* keys1;
    const uint8_t* desc1;
    const uint8_t* has1;
    const mam_keypoint* keys2;
    const uint8_t* desc2;
    const uint8_t* has2;
    const uint32_t* feats1;
    const uint32_t* feats2;
    const int32_t* work;      // per work item: position in feats1
    const int32_t* work_n2;   // per work item: [begin, end) in feats2 (2 ints)
    int nwork;
    mam_camera cam1, cam2;    // pKF1->mpCamera, pKF2->mpCamera (pCamera1->epipolarConstrain(pCamera2, ...))
    float F[9];               // Pinhole pairs: F12
    float R12[9], t12[3];     // KannalaBrandt8 pairs: T12
    float ep[2];
    int coarse;
    int32_t* out;             // [n1]
};

// pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, sigma2[kp1.octave], sigma2[kp2.octave])
// (ORBmatcher.cc:1069): Pinhole.cpp:107-129 for a Pinhole KF1 (line of kp1 through F12, the 3.84 sigma2 test),
// KannalaBrandt8.cpp:216-220 (two-view triangulation, z1 > 1e-4) for a fisheye one. la/lb/lc: kp1's epipolar line,
// r1: kp1's unprojected ray (per idx1, computed once).
__device__ __forceinline__ bool tri_epipolar_ok(const TriArgs& a, const mam_keypoint& kp1, float la, float lb, float lc,
                                                const float r1[3], const mam_keypoint& kp2) {
    if (a.cam1.model == MAM_CAM_KANNALA_BRANDT8) {
        float r2[3];
        cam::kb8_unproject_f(a.cam2, kp2.x, kp2.y, r2);
        return cam::kb8_triangulate_matches(a.cam1, a.cam2, kp1.x, kp1.y, r1, kp2.x, kp2.y, r2, a.R12, a.t12,
                                            a.g.level_sigma2[kp1.octave], a.g.level_sigma2[kp2.octave]) > 0.0001f;
    }
    const float num = la * kp2.x + lb * kp2.y + lc;
    const float den = la * la + lb * lb;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * a.g.level_sigma2[kp2.octave];
}

__global__ __launch_bounds__(256) void k_tri(TriArgs a) {
    const int gw = (int)(((long long)blockIdx.x * 256 + threadIdx.x) >> 6);
    if (gw >= a.nwork) return;
    const int lane = lane_id();
    const uint32_t idx1 = a.feats1[a.work[gw]];
    if (a.has1[idx1]) return;
    const mam_keypoint kp1 = a.keys1[idx1];
    const uint8_t* d1 = a.desc1 + (size_t)idx1 * 32;
    const int b = a.work_n2[2 * gw], e = a.work_n2[2 * gw + 1];
    // epipolar line of kp1 in image 2 (Pinhole::epipolarConstrain, Pinhole.cpp:114-117) / kp1's ray (fisheye)
    const float la = kp1.x * a.F[0] + kp1.y * a.F[3] + a.F[6];
    const float lb = kp1.x * a.F[1] + kp1.y * a.F[4] + a.F[7];
    const float lc = kp1.x * a.F[2] + kp1.y * a.F[5] + a.F[8];
    float r1[3] = {0.0f, 0.0f, 1.0f};
    if (a.cam1.model == MAM_CAM_KANNALA_BRANDT8 && !a.coarse) cam::kb8_unproject_f(a.cam1, kp1.x, kp1.y, r1);
    unsigned best = 0xFFFFFFFFu;   // (dist << 16) | (0xFFFF - position): min = smallest dist, LAST position
    for (int i0 = b; i0 < e; i0 += 64) {
        const int i2 = i0 + lane;
        if (i2 < e) {
            const uint32_t idx2 = a.feats2[i2];
            if (!a.has2[idx2]) {
                const int dist = desc_dist(d1, a.desc2 + (size_t)idx2 * 32);
                if (dist <= MAM_TH_LOW) {
                    const mam_keypoint kp2 = a.keys2[idx2];
                    const float distex = a.ep[0] - kp2.x;
                    const float distey = a.ep[1] - kp2.y;
                    if (!(distex * distex + distey * distey < 100 * a.g.scale_factors[kp2.octave])) {
                        const bool ok = a.coarse != 0 || tri_epipolar_ok(a, kp1, la, lb, lc, r1, kp2);
                        if (ok) best = min(best, ((unsigned)dist << 16) | (0xFFFFu - (unsigned)(i2 - b)));
                    }
                }
            }
        }
    }
    best = wave_minu(best);
    if (lane == 0 && best != 0xFFFFFFFFu) a.out[idx1] = (int32_t)a.feats2[b + (int)(0xFFFFu - (best & 0xFFFFu))];
}

__global__ __launch_bounds__(256) void k_tri_rot(const mam_keypoint* keys1, const mam_keypoint* keys2, int n1,
                                                  int check_ori, int32_t* out, int32_t* nmatch) {
    __shared__ int hist[MAM_HISTO_LENGTH];
    __shared__ int top[3];
    __shared__ int red[4];
    const int tid = threadIdx.x;
    if (tid < MAM_HISTO_LENGTH) hist[tid] = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = tid; i < n1; i += 256) {
        if (out[i] >= 0) {
            cnt++;
            if (check_ori) atomicAdd(&hist[rot_bin(keys1[i].angle - keys2[out[i]].angle)], 1);
        }
    }
    __syncthreads();
    if (check_ori) {
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < MAM_HISTO_LENGTH; i++) {
                const int s = hist[i];
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
                else if (s > max3) { max3 = s; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            top[0] = ind1; top[1] = ind2; top[2] = ind3;
        }
        __syncthreads();
        for (int i = tid; i < n1; i += 256) {
            if (out[i] >= 0) {
                const int bin = rot_bin(keys1[i].angle - keys2[out[i]].angle);
                if (bin != top[0] && bin != top[1] && bin != top[2]) { out[i] = -1; cnt--; }
            }
        }
    }
    cnt = wave_sum(cnt);
    if (lane_id() == 0) red[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) *nmatch = red[0] + red[1] + red[2] + red[3];
}

// ---- batched SearchForTriangulation (CreateNewMapPoints' 30 searches per new keyframe, LocalMapping.cc:504-582):
// keyframe slots with device-resident features, FeatureVectors given as the BoW transform's per-feature node and
// weight (DBoW2 adds feature i to node nid iff its word weight > 0), pairs (kf1, kf2).
struct TriBatchArgs {
    mam_frame_geom g;
    mam_frames_dev kfs;
    const uint8_t* has_mp;
    const uint32_t* nid;
    const double* weight;
    const mam_pose* tcw;
    const int32_t* pairs;
    int npairs;
    mam_camera cam;
    int coarse, check_ori;
    unsigned long long* skey;   // [nkf][skey_stride] (nid << 32 | idx) ascending, ~0 past the FeatureVector
    int skey_stride;            // power of two >= kp_stride
    int32_t* nfv;               // [nkf] features in the FeatureVector
    unsigned long long* raw;    // [nkf][skey_stride] the unsorted keys skey was sorted from (the previous call's)
    int32_t* raw_ok;            // [nkf] raw / skey / nfv of the slot hold a sort of this stride's keys
    cam::PairGeom* pg;          // [npairs]
    int32_t* out;               // [npairs][kp_stride]
    int32_t* out_n;             // [npairs]
};

// grid (nkf) x 1024: every keyframe's FeatureVector as one sorted key array (node id, then feature index: the order
// the reference walks a FeatureVector, std::map by node + insertion order), bitonic sort in LDS. A keyframe slot whose
// keys equal, element for element, the keys of the slot's previous sort keeps that sort (a ring's older keyframes:
// only the run's new keyframes change between LocalMapping runs).
__global__ __launch_bounds__(1024) void k_tri_fv_sort(TriBatchArgs a) {
    extern __shared__ unsigned long long sk[];
    const int k = blockIdx.x, P = a.skey_stride;
    const int n = frame_n(a.kfs, k);
    const size_t base = (size_t)k * a.kfs.kp_stride;
    const bool had = a.raw_ok[k] != 0;
    int diff = had ? 0 : 1;
    for (int i = threadIdx.x; i < P; i += 1024) {
        unsigned long long v = ~0ull;
        if (i < n && a.weight[base + i] > 0.0) v = ((unsigned long long)a.nid[base + i] << 32) | (unsigned)i;
        sk[i] = v;
        if (had && a.raw[(size_t)k * P + i] != v) diff = 1;
    }
    if (!__syncthreads_or(diff)) return;   // the same keys: skey / nfv of the slot stand
    for (int i = threadIdx.x; i < P; i += 1024) a.raw[(size_t)k * P + i] = sk[i];
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < P / 2; i += 1024) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long x = sk[lo], y = sk[hi];
                if ((x > y) == up) { sk[lo] = y; sk[hi] = x; }
            }
            __syncthreads();
        }
    }
    int cnt = 0;
    for (int i = threadIdx.x; i < P; i += 1024) {
        a.skey[(size_t)k * P + i] = sk[i];
        cnt += sk[i] != ~0ull;
    }
    __shared__ int red[16];
    cnt = wave_sum(cnt);
    if (lane_id() == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < 16; w++) t += red[w];
        a.nfv[k] = t;
        a.raw_ok[k] = 1;
    }
}

// grid (ceil(npairs / 256)) x 256: the pair geometry of ORBmatcher.cc:913-930
__global__ __launch_bounds__(256) void k_tri_pair_geom(TriBatchArgs a) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= a.npairs) return;
    const mam_pose& t1 = a.tcw[a.pairs[2 * q]];
    const mam_pose& t2 = a.tcw[a.pairs[2 * q + 1]];
    cam::pair_geometry(t1.q, t1.t, t2.q, t2.t, a.cam, a.cam, &a.pg[q]);
}

// grid (npairs) x 512, one workgroup per pair (the pairs of one kf1 on one XCD: kf1's keys, descriptors and sorted
// FeatureVector stay in its L2). kf2's sorted FeatureVector keys are staged in LDS; the 32 groups of 16 lanes take
// contiguous ranges of kf1's sorted FeatureVector (node by node, in the order ORBmatcher.cc:974-1074 walks the two
// FeatureVectors) and look each new node up in kf2's keys by a binary search in LDS. Per idx1 the node's kf2
// candidates are dealt to the 16 lanes; (dist, last position) argmin over the lanes = "dist <= bestDist, last equal
// wins". Then, in the same workgroup, nmatches and the rotation-histogram filter when check_ori
// (ORBmatcher.cc:1114-1133).
#ifndef MAM_TRI_THREADS
#define MAM_TRI_THREADS 1024
#endif
constexpr int TRI_THREADS = MAM_TRI_THREADS;
__global__ __launch_bounds__(TRI_THREADS) void k_tri_pair(TriBatchArgs a) {
    extern __shared__ unsigned long long sk2[];   // [skey_stride] kf2's sorted keys, then kf2's has_mp bytes
    __shared__ int hist[MAM_HISTO_LENGTH];
    __shared__ int top[3];
    __shared__ int red[TRI_THREADS / 64];
    const int q = xcd_logical(blockIdx.x, gridDim.x);
    const int k1 = a.pairs[2 * q], k2 = a.pairs[2 * q + 1];
    const int S = a.kfs.kp_stride, tid = threadIdx.x;
    const int n1 = frame_n(a.kfs, k1);
    const int nfv1 = a.nfv[k1], nfv2 = a.nfv[k2];
    const size_t b1 = (size_t)k1 * S, b2 = (size_t)k2 * S;
    int32_t* out = a.out + (size_t)q * S;
    const unsigned long long* sk1 = a.skey + (size_t)k1 * a.skey_stride;
    uint8_t* has2 = reinterpret_cast<uint8_t*>(sk2 + a.skey_stride);
    for (int i = tid; i < nfv2; i += TRI_THREADS) sk2[i] = a.skey[(size_t)k2 * a.skey_stride + i];
    for (int i = tid; i < S; i += TRI_THREADS) has2[i] = a.has_mp[b2 + i];
    for (int i = tid; i < S; i += TRI_THREADS) out[i] = -1;
    if (tid < MAM_HISTO_LENGTH) hist[tid] = 0;
    __syncthreads();
    const cam::PairGeom& G = a.pg[q];
    const bool kb8 = a.cam.model == MAM_CAM_KANNALA_BRANDT8;
    const int grp = tid >> 4, sub = tid & 15, ngrp = TRI_THREADS / 16;
    const int per = (nfv1 + ngrp - 1) / ngrp;
    const int p0 = grp * per, p1 = min(nfv1, p0 + per);
    unsigned cur = 0xFFFFFFFFu;
    int b = 0, e = 0;
    // one position ahead: its key and has_mp are in flight while the current position's candidates are scored
    unsigned long long kn = p0 < p1 ? sk1[p0] : 0ull;
    uint8_t hn = p0 < p1 ? a.has_mp[b1 + (kn & 0xFFFFFFFFull)] : 1;
    for (int p = p0; p < p1; p++) {
        const unsigned long long k = kn;
        const uint8_t has1 = hn;
        if (p + 1 < p1) {
            kn = sk1[p + 1];
            hn = a.has_mp[b1 + (kn & 0xFFFFFFFFull)];
        }
        const unsigned nid = (unsigned)(k >> 32);
        const int idx1 = (int)(k & 0xFFFFFFFFull);
        if (nid != cur) {   // kf2's features of the node: [b, e) of its sorted keys
            cur = nid;
            const unsigned long long key = (unsigned long long)nid << 32;
            int lo = 0, hi = nfv2;
            while (lo < hi) {
                const int m = (lo + hi) >> 1;
                if (sk2[m] < key) lo = m + 1;
                else hi = m;
            }
            b = lo;
            hi = nfv2;
            while (lo < hi) {
                const int m = (lo + hi) >> 1;
                if (sk2[m] <= (key | 0xFFFFFFFFull)) lo = m + 1;
                else hi = m;
            }
            e = lo;
        }
        if (b == e || has1) continue;   // uniform over the group
        const mam_keypoint kp1 = a.kfs.keys[b1 + idx1];
        const uint8_t* d1 = a.kfs.desc + (b1 + idx1) * 32;
        const float la = kp1.x * G.F12[0] + kp1.y * G.F12[3] + G.F12[6];
        const float lb = kp1.x * G.F12[1] + kp1.y * G.F12[4] + G.F12[7];
        const float lc = kp1.x * G.F12[2] + kp1.y * G.F12[5] + G.F12[8];
        float r1[3] = {0.0f, 0.0f, 1.0f};
        if (kb8 && !a.coarse) cam::kb8_unproject_f(a.cam, kp1.x, kp1.y, r1);
        unsigned best = 0xFFFFFFFFu;
        for (int i2 = b + sub; i2 < e; i2 += 16) {
            const int idx2 = (int)(sk2[i2] & 0xFFFFFFFFull);
            if (has2[idx2]) continue;
            const int dist = desc_dist(d1, a.kfs.desc + (b2 + idx2) * 32);
            if (dist > MAM_TH_LOW) continue;
            const mam_keypoint kp2 = a.kfs.keys[b2 + idx2];
            const float distex = G.ep[0] - kp2.x;
            const float distey = G.ep[1] - kp2.y;
            if (distex * distex + distey * distey < 100 * a.g.scale_factors[kp2.octave]) continue;
            bool ok = a.coarse != 0;
            if (!ok) {
                if (kb8) {
                    float r2[3];
                    cam::kb8_unproject_f(a.cam, kp2.x, kp2.y, r2);
                    ok = cam::kb8_triangulate_matches(a.cam, a.cam, kp1.x, kp1.y, r1, kp2.x, kp2.y, r2, G.R12, G.t12,
                                                      a.g.level_sigma2[kp1.octave],
                                                      a.g.level_sigma2[kp2.octave]) > 0.0001f;
                } else {
                    const float num = la * kp2.x + lb * kp2.y + lc;
                    const float den = la * la + lb * lb;
                    ok = den != 0 && num * num / den < 3.84 * a.g.level_sigma2[kp2.octave];
                }
            }
            if (ok) best = min(best, ((unsigned)dist << 16) | (0xFFFFu - (unsigned)(i2 - b)));
        }
        for (int o = 8; o > 0; o >>= 1) best = min(best, (unsigned)__shfl_xor((int)best, o, 16));
        if (sub == 0 && best != 0xFFFFFFFFu) out[idx1] = (int)(sk2[b + (int)(0xFFFFu - (best & 0xFFFFu))] & 0xFFFFFFFFull);
    }
    __syncthreads();
    const mam_keypoint* keys1 = a.kfs.keys + b1;
    const mam_keypoint* keys2 = a.kfs.keys + b2;
    int cnt = 0;
    for (int i = tid; i < n1; i += TRI_THREADS) {
        if (out[i] >= 0) {
            cnt++;
            if (a.check_ori) atomicAdd(&hist[rot_bin(keys1[i].angle - keys2[out[i]].angle)], 1);
        }
    }
    __syncthreads();
    if (a.check_ori) {
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < MAM_HISTO_LENGTH; i++) {
                const int s = hist[i];
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
                else if (s > max3) { max3 = s; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            top[0] = ind1; top[1] = ind2; top[2] = ind3;
        }
        __syncthreads();
        for (int i = tid; i < n1; i += TRI_THREADS) {
            if (out[i] >= 0) {
                const int bin = rot_bin(keys1[i].angle - keys2[out[i]].angle);
                if (bin != top[0] && bin != top[1] && bin != top[2]) { out[i] = -1; cnt--; }
            }
        }
    }
    cnt = wave_sum(cnt);
    if (lane_id() == 0) red[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < TRI_THREADS / 64; w++) t += red[w];
        a.out_n[q] = t;
    }
}

__global__ void k_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = desc_dist(a + (size_t)i * 32, b + (size_t)i * 32);
}

// ------------------------------------------------------------------------------------------------ fuse
// ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight=false) (ORBmatcher.cc:1148-1338), mono Pinhole keyframe. A
// MapPoint's search reads nothing that the replace-or-add side effects of earlier MapPoints of the same call change
// (the MapPoints those touch are skipped by the caller's isBad / IsInKeyFrame re-check), so every MapPoint of every
// target keyframe is searched in parallel, GW lanes per MapPoint as in k_gather; the caller applies the results in
// list order.
struct FuseArgs {
    mam_frame_geom g;
    mam_frames_dev fr;
    const mam_fuse_kf* kfs;      // per item (NULL: from kf_tcw of the item's keyframe)
    mam_camera cam;
    const mam_fuse_mp* mps;
    int mp_stride;
    const int32_t* n_mps;
    float th;
    const GridEnt* grid_ent;
    const int32_t* grid_start;
    int32_t* out_idx;
    int32_t* out_dist;
    int32_t* out_n;
    // item indirection (mam_fuse_items_batch_device; NULL = item b is keyframe b with MapPoint list b)
    const int32_t* frame_of;     // keyframe of the frame set item b fuses into
    const int32_t* mp_of;        // MapPoint list item b fuses
    const mam_pose* kf_tcw;      // per keyframe of the set: GetPose()
    float log_scale_factor;      // mfLogScaleFactor
    const int32_t* grid_status;  // per keyframe of the set: k_grid's status (< 0: too many keypoints)
};

// KeyFrame::GetCameraCenter of a Tcw as Sophus computes Twc = Tcw^-1 in float: the conjugate quaternion applied to -t
// (match.py camera_center, the same operations in the same order)
__device__ __forceinline__ mam_fuse_kf fuse_kf_of(const mam_pose& T, float log_sf) {
    mam_fuse_kf k;
    k.tcw = T;
    const float px = -T.t[0], py = -T.t[1], pz = -T.t[2];
    const float qx = -T.q[0], qy = -T.q[1], qz = -T.q[2], w = T.q[3];
    float u0 = qy * pz - qz * py, u1 = qz * px - qx * pz, u2 = qx * py - qy * px;
    u0 = u0 + u0; u1 = u1 + u1; u2 = u2 + u2;
    k.ow[0] = (px + w * u0) + (qy * u2 - qz * u1);
    k.ow[1] = (py + w * u1) + (qz * u0 - qx * u2);
    k.ow[2] = (pz + w * u2) + (qx * u1 - qy * u0);
    k.log_scale_factor = log_sf;
    return k;
}

// (int) of a float as x86's cvttss2si computes it (NaN / out of range -> INT_MIN): PredictScale's (int)ceil(...)
__device__ __forceinline__ int cvt_i32_x86(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int)v : INT_MIN;
}

// The window of MapPoint mp in keyframe f; false where the reference `continue`s (ORBmatcher.cc:1179-1251).
__device__ bool fuse_window(const FuseArgs& p, int f, const mam_fuse_mp& mp, Window* w) {
    if (!mp.valid) return false;
    const mam_fuse_kf K = p.kfs ? p.kfs[f] : fuse_kf_of(p.kf_tcw[p.frame_of[f]], p.log_scale_factor);
    // Tcw * p3Dw: Sophus SE3f action, evaluated as written (as in unit_window)
    const float qx = K.tcw.q[0], qy = K.tcw.q[1], qz = K.tcw.q[2], qw = K.tcw.q[3];
    const float px = mp.pos[0], py = mp.pos[1], pz = mp.pos[2];
    float u0 = qy * pz - qz * py, u1 = qz * px - qx * pz, u2 = qx * py - qy * px;
    u0 += u0; u1 += u1; u2 += u2;
    const float c0 = qy * u2 - qz * u1, c1 = qz * u0 - qx * u2, c2 = qx * u1 - qy * u0;
    const float xc = ((px + qw * u0) + c0) + K.tcw.t[0];
    const float yc = ((py + qw * u1) + c1) + K.tcw.t[1];
    const float zc = ((pz + qw * u2) + c2) + K.tcw.t[2];
    if (zc < 0.0f) return false;
    float u, v;
    cam::project_f(p.cam, xc, yc, zc, &u, &v);   // pCamera->project(p3Dc) (ORBmatcher.cc:1210)
    if (!(u >= p.g.min_x && u < p.g.max_x && v >= p.g.min_y && v < p.g.max_y)) return false;   // KeyFrame::IsInImage
    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
    const float P0 = px - K.ow[0], P1 = py - K.ow[1], P2 = pz - K.ow[2];
    // Eigen's unrolled 3-term reductions (norm, dot): e0 + (e1 + e2)
    const float dist3D = sqrtf(P0 * P0 + (P1 * P1 + P2 * P2));
    if (dist3D < minD || dist3D > maxD) return false;
    const float dot = P0 * mp.normal[0] + (P1 * mp.normal[1] + P2 * mp.normal[2]);
    if ((double)dot < 0.5 * (double)dist3D) return false;
    // PredictScale (MapPoint.cc:514-529); log(float) as the correctly rounded float log
    const float ratio = mp.max_distance / dist3D;
#if defined(MAM_FUSE_EXPERIMENT) && (MAM_FUSE_EXPERIMENT & 2)
    int lvl = cvt_i32_x86(ceilf(logf(ratio) / K.log_scale_factor));   // timing experiment only
#else
    int lvl = cvt_i32_x86(ceilf((float)log((double)ratio) / K.log_scale_factor));
#endif
    if (lvl < 0) lvl = 0;
    else if (lvl >= p.g.nlevels) lvl = p.g.nlevels - 1;
    w->x = u;
    w->y = v;
    w->r = p.th * p.g.scale_factors[lvl];
    w->minL = lvl - 1;
    w->maxL = lvl;
    w->checkL = true;
    w->desc = mp.desc;
    return window_cells(p.g, w);
}

// Best keypoint of one MapPoint's window by a group of GW lanes: the window's candidates in GetFeaturesInArea order
// (as gather_pass deals them), the level and reprojection tests of ORBmatcher.cc:1267-1296, and the first minimum
// distance of the enumeration (dist < bestDist) as the group minimum of dist << 20 | position.
template <int GW>
__device__ void fuse_pass(const FuseArgs& p, int f, const Window& w, const uint4 u0, const uint4 u1, int* bdist,
                          int* bidx) {
    const int gl = lane_id() & (GW - 1);
    const int ny = w.cy1 - w.cy0 + 1;
    const int ncell = (w.cx1 - w.cx0 + 1) * ny;
    const int32_t* gs = p.grid_start + (size_t)f * (NCELLS + 1);
    const GridEnt* G = p.grid_ent + (size_t)f * p.fr.kp_stride;
    unsigned best = 0xFFFFFFFFu;
    int bi = -1;
    int base = 0;   // enumeration position of the chunk's first candidate
    for (int e0 = 0; e0 < ncell; e0 += GW) {
        const int e = e0 + gl;
        int k0 = 0, c = 0;
        if (e < ncell) {
            const int ix = w.cx0 + e / ny, iy = w.cy0 + e % ny;
            const int cell = ix * MAM_GRID_ROWS + iy;
            k0 = gs[cell];
            c = gs[cell + 1] - k0;
        }
        int incl = c;
#pragma unroll
        for (int o = 1; o < GW; o <<= 1) {
            const int t = __shfl_up(incl, o, GW);
            if (gl >= o) incl += t;
        }
        const int tot = __shfl(incl, GW - 1, GW);
        const int kb = k0 - (incl - c);
        for (int t0 = 0; t0 < tot; t0 += GW) {
            const int t = t0 + gl;
            int m = 0;
#pragma unroll
            for (int step = GW / 2; step >= 1; step >>= 1)
                if (__shfl(incl, m + step - 1, GW) <= t) m += step;
            const int k = __shfl(kb, m, GW) + t;
            if (t < tot) {
                const GridEnt ge = G[k];
                const int oct = (int)(ge.io >> 16);
                const float dx = ge.x - w.x, dy = ge.y - w.y;
                if (oct >= w.minL && oct <= w.maxL && fabsf(dx) < w.r && fabsf(dy) < w.r) {
                    const float ex = w.x - ge.x, ey = w.y - ge.y;
                    const float e2 = ex * ex + ey * ey;
                    if (!((double)(e2 * (1.0f / p.g.level_sigma2[oct])) > 5.99)) {
                        const int dist = __popc(u0.x ^ ge.d0.x) + __popc(u0.y ^ ge.d0.y) + __popc(u0.z ^ ge.d0.z) +
                                         __popc(u0.w ^ ge.d0.w) + __popc(u1.x ^ ge.d1.x) + __popc(u1.y ^ ge.d1.y) +
                                         __popc(u1.z ^ ge.d1.z) + __popc(u1.w ^ ge.d1.w);
                        const unsigned key = ((unsigned)dist << 20) | (unsigned)(base + t);
                        if (key < best) {
                            best = key;
                            bi = (int)(ge.io & 0xFFFFu);
                        }
                    }
                }
            }
        }
        base += tot;
    }
#pragma unroll
    for (int o = GW / 2; o >= 1; o >>= 1) {
        const unsigned ob = (unsigned)__shfl_xor((int)best, o, GW);
        const int oi = __shfl_xor(bi, o, GW);
        if (ob < best) {
            best = ob;
            bi = oi;
        }
    }
    *bdist = best == 0xFFFFFFFFu ? 256 : (int)(best >> 20);
    *bidx = bi;
}

template <int GW>
__global__ __launch_bounds__(256) void k_fuse(FuseArgs p, int nframes) {
    const long long gu = ((long long)blockIdx.x * 256 + threadIdx.x) / GW;   // global MapPoint slot
    const int f = (int)(gu / p.mp_stride);
    const int j = (int)(gu - (long long)f * p.mp_stride);
    if (f >= nframes) return;
    const int m = p.mp_of ? p.mp_of[f] : f;
    if (j >= p.n_mps[m]) return;   // group-uniform
    const int fk = p.frame_of ? p.frame_of[f] : f;   // the keyframe (its cell grid)
    if (p.grid_status && p.grid_status[fk] < 0) return;
    const size_t o = (size_t)f * p.mp_stride + j;
    const mam_fuse_mp& mp = p.mps[(size_t)m * p.mp_stride + j];
    Window w;
    int bd = 256, bi = -1;
#if defined(MAM_FUSE_EXPERIMENT) && (MAM_FUSE_EXPERIMENT & 1)
    if (fuse_window(p, f, mp, &w) && w.r < 0.f) {   // timing experiment only: no window scan
#else
    if (fuse_window(p, f, mp, &w)) {
#endif
        const uint4 u0 = reinterpret_cast<const uint4*>(mp.desc)[0], u1 = reinterpret_cast<const uint4*>(mp.desc)[1];
        fuse_pass<GW>(p, fk, w, u0, u1, &bd, &bi);
    }
    if ((lane_id() & (GW - 1)) == 0) {
        p.out_idx[o] = bd <= MAM_TH_LOW ? bi : -1;
        p.out_dist[o] = bd;
    }
}

// nFused per keyframe (a per-MapPoint atomicAdd on one counter per keyframe serialises in L2: ~7 ns per MapPoint)
__global__ __launch_bounds__(256) void k_fuse_count(FuseArgs p) {
    __shared__ int red[4];
    const int f = blockIdx.x, n = p.n_mps[p.mp_of ? p.mp_of[f] : f];
    const int32_t* idx = p.out_idx + (size_t)f * p.mp_stride;
    const int st = p.grid_status ? p.grid_status[p.frame_of[f]] : 0;
    int c = 0;
    if (st >= 0)
        for (int j = threadIdx.x; j < n; j += 256) c += idx[j] >= 0;
    c = wave_sum(c);
    if (lane_id() == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (p.grid_status) p.out_n[f] = st < 0 ? st : red[0] + red[1] + red[2] + red[3];
        else if (p.out_n[f] >= 0) p.out_n[f] = red[0] + red[1] + red[2] + red[3];
    }
}

// ------------------------------------------------------------------------------------------------ distinctive descriptor
// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403), one wave per MapPoint. Lane i takes row i of the
// N x N distance matrix (rows i, i + 64, ...) and finds the row's median, element (N-1)/2 of the sorted row, by a
// binary search over the distance value: 9 counting passes over the N descriptors, read at wave-uniform addresses.
// The chosen descriptor (smallest median, first on ties) is the wave minimum of median << 20 | i.
__global__ __launch_bounds__(256) void k_distinct(const int32_t* __restrict__ off, const uint8_t* __restrict__ descs,
                                                  int n, int32_t* __restrict__ out) {
    const int m = __builtin_amdgcn_readfirstlane((int)(((long long)blockIdx.x * 256 + threadIdx.x) >> 6));
    if (m >= n) return;
    const int lane = lane_id();
    const int b = off[m], N = off[m + 1] - b;
    if (N <= 0) {
        if (lane == 0) out[m] = -1;
        return;
    }
    const uint4* D = reinterpret_cast<const uint4*>(descs + (size_t)b * 32);
    const int k = (N - 1) >> 1;   // vDists[0.5*(N-1)]
    unsigned best = 0xFFFFFFFFu;
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        uint4 r0 = make_uint4(0u, 0u, 0u, 0u), r1 = r0;
        if (i < N) {
            r0 = D[2 * i];
            r1 = D[2 * i + 1];
        }
        int lo = 0, hi = 256;   // the median lies in [lo, hi]
        for (int it = 0; it < 9; it++) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < N; j++) {
                const uint4 c0 = D[2 * j], c1 = D[2 * j + 1];
                const int d = __popc(r0.x ^ c0.x) + __popc(r0.y ^ c0.y) + __popc(r0.z ^ c0.z) + __popc(r0.w ^ c0.w) +
                              __popc(r1.x ^ c1.x) + __popc(r1.y ^ c1.y) + __popc(r1.z ^ c1.z) + __popc(r1.w ^ c1.w);
                cnt += d <= mid;
            }
            if (cnt > k) hi = mid;
            else lo = mid + 1;
        }
        if (i < N) best = min(best, ((unsigned)lo << 20) | (unsigned)i);
    }
    best = wave_minu(best);
    if (lane == 0) out[m] = (int32_t)(best & 0xFFFFFu);
}

// ------------------------------------------------------------------------------------------------ frustum
// Tracking::SearchLocalPoints' projection loop (Tracking.cc:3119-3139): Frame::isInFrustum(pMP, 0.5) (Frame.cc:512-571,
// mono) + MapPoint::PredictScale(dist, Frame*) (MapPoint.cc:531-546) for every local MapPoint of every frame, one
// thread each, writing the mam_mp_track record the local-map search reads. Frame side per block: mRcw (Eigen
// toRotationMatrix of the Sophus quaternion) and mOw (Tcw.inverse().translation()), Frame.cc:472-479. Eigen's 3x3 * 3
// rows, norm() and dot() sum as e0 + (e1 + e2). Per-frame nToMatch by one atomic per block.
struct FrustumArgs {
    mam_frame_geom g;
    const mam_pose* tcw;
    mam_camera cam;
    float log_scale_factor, view_cos_limit;
    const mam_local_mp* mps;
    int mp_stride;
    const int32_t* n_mps;
    mam_mp_track* out;
    int32_t* out_n;
};

__global__ __launch_bounds__(256) void k_frustum(FrustumArgs a) {
    __shared__ float fr[15];   // R (9), t (3), Ow (3)
    __shared__ int wcount[4];
    const int f = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (threadIdx.x == 0) {
        const mam_pose T = a.tcw[f];
        const float qx = T.q[0], qy = T.q[1], qz = T.q[2], qw = T.q[3];
        const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
        const float twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
        const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
        fr[0] = 1.0f - (tyy + tzz); fr[1] = txy - twz; fr[2] = txz + twy;
        fr[3] = txy + twz; fr[4] = 1.0f - (txx + tzz); fr[5] = tyz - twx;
        fr[6] = txz - twy; fr[7] = tyz + twx; fr[8] = 1.0f - (txx + tyy);
        fr[9] = T.t[0]; fr[10] = T.t[1]; fr[11] = T.t[2];
        // Ow = conj(q) * (-t) (Sophus SO3 action, as unit_window evaluates it)
        const float px = T.t[0] * -1.0f, py = T.t[1] * -1.0f, pz = T.t[2] * -1.0f;
        const float ix = -qx, iy = -qy, iz = -qz;
        float u0 = iy * pz - iz * py, u1 = iz * px - ix * pz, u2 = ix * py - iy * px;
        u0 += u0; u1 += u1; u2 += u2;
        const float c0 = iy * u2 - iz * u1, c1 = iz * u0 - ix * u2, c2 = ix * u1 - iy * u0;
        fr[12] = ((px + qw * u0) + c0) + 0.0f;
        fr[13] = ((py + qw * u1) + c1) + 0.0f;
        fr[14] = ((pz + qw * u2) + c2) + 0.0f;
    }
    __syncthreads();
    const int n = a.n_mps[f];
    int in_view = 0;
    if (j < n && j < a.mp_stride) {
        const mam_local_mp& mp = a.mps[(size_t)f * a.mp_stride + j];
        mam_mp_track o;
        o.proj_x = -1.0f;
        o.proj_y = -1.0f;
        o.view_cos = 0.0f;
        o.track_depth = 0.0f;
        o.track_in_view = 0;
        o.scale_level = 0;
        o.is_bad = mp.is_bad;
        o.nobs = mp.nobs;
        const uint4* sd = reinterpret_cast<const uint4*>(mp.desc);
        uint4* od = reinterpret_cast<uint4*>(o.desc);
        od[0] = sd[0];
        od[1] = sd[1];
        if (!mp.seen && !mp.is_bad) {
            const float P0 = mp.pos[0], P1 = mp.pos[1], P2 = mp.pos[2];
            const float x = (fr[0] * P0 + (fr[1] * P1 + fr[2] * P2)) + fr[9];
            const float y = (fr[3] * P0 + (fr[4] * P1 + fr[5] * P2)) + fr[10];
            const float z = (fr[6] * P0 + (fr[7] * P1 + fr[8] * P2)) + fr[11];
            const float pc_dist = sqrtf(x * x + (y * y + z * z));
            if (z >= 0.0f) {
                float u, v;
                cam::project_f(a.cam, x, y, z, &u, &v);   // mpCamera->project(Pc) (Frame.cc:532)
                if (!(u < a.g.min_x || u > a.g.max_x || v < a.g.min_y || v > a.g.max_y)) {
                    o.proj_x = u;
                    o.proj_y = v;
                    const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
                    const float O0 = P0 - fr[12], O1 = P1 - fr[13], O2 = P2 - fr[14];
                    const float dist = sqrtf(O0 * O0 + (O1 * O1 + O2 * O2));
                    if (!(dist < minD || dist > maxD)) {
                        const float vc = (O0 * mp.normal[0] + (O1 * mp.normal[1] + O2 * mp.normal[2])) / dist;
                        if (!(vc < a.view_cos_limit)) {
                            // PredictScale; log(float) as the correctly rounded float log
                            const float ratio = mp.max_distance / dist;
                            int lvl = cvt_i32_x86(ceilf((float)log((double)ratio) / a.log_scale_factor));
                            if (lvl < 0) lvl = 0;
                            else if (lvl >= a.g.nlevels) lvl = a.g.nlevels - 1;
                            o.track_in_view = 1;
                            o.track_depth = pc_dist;
                            o.scale_level = lvl;
                            o.view_cos = vc;
                            in_view = 1;
                        }
                    }
                }
            }
        }
        a.out[(size_t)f * a.mp_stride + j] = o;
    }
    if (a.out_n) {
        const int c = __popcll(__ballot(in_view));
        if ((threadIdx.x & 63) == 0) wcount[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int s = wcount[0] + wcount[1] + wcount[2] + wcount[3];
            if (s) atomicAdd(&a.out_n[f], s);
        }
    }
}

}  // namespace mam

// ==================================================================================================== host
using mam::DevBuf;

struct mam_match_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    mam::StageTimer timer{7};
    int slot_cap = 32;        // candidate slots per unit (grows x4 when a host call overflows)
    size_t resolve_lds_max = 64 * 1024;
    // scratch
    DevBuf<mam::GridEnt> grid_ent;
    DevBuf<int32_t> grid_start, cand_cnt, cand_off, pool_total, out_n_tmp, grid_status;
    DevBuf<uint32_t> pool, events;
    // frames the grid scratch holds (mam_frames_dev.reuse_grid is accepted only for the same frames)
    const void* grid_keys = nullptr;
    const void* grid_counts = nullptr;
    int grid_nframes = 0, grid_stride = 0;
    // host-API staging
    DevBuf<uint8_t> stage;
    // batched triangulation scratch
    DevBuf<unsigned long long> tri_skey, tri_raw;
    DevBuf<int32_t> tri_nfv, tri_ok;
    int tri_P = 0, tri_nkf = 0;   // the stride / slot count tri_raw holds sorts of (else tri_ok is cleared)
    DevBuf<mam::cam::PairGeom> tri_pg;
};

namespace {

template <typename T>
T* carve(uint8_t*& p, size_t count) {
    T* r = reinterpret_cast<T*>(p);
    p += (count * sizeof(T) + 255) & ~(size_t)255;
    return r;
}

void set_pool(mam_match_ctx* c, mam::ProjArgs& a, int unit_stride) {
    a.slot_cap = c->slot_cap;
    a.ovf_cap = std::max(unit_stride * c->slot_cap / 2, 1 << 16);
    a.pool_per_frame = unit_stride * a.slot_cap + a.ovf_cap;
}

size_t carve_bytes(size_t count, size_t elem) { return (count * elem + 255) & ~(size_t)255; }

int ensure_scratch(mam_match_ctx* c, int F, int kp_stride, int unit_stride, int pool_per_frame) {
    if (int rc = c->grid_ent.alloc((size_t)F * kp_stride)) return rc;
    if (int rc = c->grid_start.alloc((size_t)F * (mam::NCELLS + 1))) return rc;
    if (int rc = c->cand_cnt.alloc((size_t)F * unit_stride)) return rc;
    if (int rc = c->cand_off.alloc((size_t)F * unit_stride)) return rc;
    if (int rc = c->pool_total.alloc(F)) return rc;
    if (int rc = c->pool.alloc((size_t)F * pool_per_frame)) return rc;
    if (int rc = c->events.alloc((size_t)F * unit_stride)) return rc;
    return MAM_OK;
}

// The frames' cell grid (k_grid, which also resets out_n / pool_total of every frame), or the one this context's
// previous search built over the same frames (mam_frames_dev.reuse_grid).
int build_grid(mam_match_ctx* c, mam::ProjArgs& a, int F, hipStream_t s) {
    if (a.fr.reuse_grid) {
        // AssignFeaturesToGrid runs once per Frame (Frame.cc:385-416): the previous search on this context built it
        if (c->grid_keys != (const void*)a.fr.keys || c->grid_counts != (const void*)a.fr.counts ||
            c->grid_nframes != F || c->grid_stride != a.fr.kp_stride) {
            mam::set_last_error("reuse_grid: this context's last search was not over the same frames");
            return MAM_ERR_ARG;
        }
        return MAM_OK;
    }
    mam::StageTimer::Scope sc(&c->timer, s, 0);
    hipLaunchKernelGGL(mam::k_grid, dim3(F), dim3(1024), 0, s, a);
    c->grid_keys = a.fr.keys;
    c->grid_counts = a.fr.counts;
    c->grid_nframes = F;
    c->grid_stride = a.fr.kp_stride;
    return MAM_OK;
}

// Shared launcher for both projection searches.
int launch_projection(mam_match_ctx* c, mam::ProjArgs& a, int F, hipStream_t s) {
    if (F <= 0) return MAM_OK;
    if (a.fr.kp_stride > mam::GRID_SORT_MAX || a.fr.kp_stride <= 0 || a.unit_stride <= 0) return MAM_ERR_ARG;
    if (int rc = ensure_scratch(c, F, a.fr.kp_stride, a.unit_stride, a.pool_per_frame)) return rc;
    a.grid_ent = c->grid_ent.p;
    a.grid_start = c->grid_start.p;
    a.cand_cnt = c->cand_cnt.p;
    a.cand_off = c->cand_off.p;
    a.pool = c->pool.p;
    a.pool_total = c->pool_total.p;
    a.events = c->events.p;
    if (int rc = build_grid(c, a, F, s)) return rc;
    {
        // batches: 16 lanes per unit (windows hold a few to a few tens of candidates, so four units share a wave and
        // their dependent global-memory round trips overlap: 0.38 -> 0.22 ms per 256 c1 frames); a single frame:
        // a whole wave per unit (fewer passes per unit, 26 -> 17 us)
        const long long units = (long long)F * a.unit_stride;
        mam::StageTimer::Scope sc(&c->timer, s, 1);
        if (F <= 4) {
            hipLaunchKernelGGL(mam::k_gather<64>, dim3((int)((units * 64 + 255) / 256)), dim3(256), 0, s, a, F);
        } else {
            constexpr int GW = MAM_GATHER_LANES;
            hipLaunchKernelGGL(mam::k_gather<GW>, dim3((int)((units * GW + 255) / 256)), dim3(256), 0, s, a, F);
        }
    }
    {
        mam::StageTimer::Scope sc(&c->timer, s, 2);
        const int S = a.fr.kp_stride;
        const size_t fixed = ((((S + 31) / 32) * 4 + 15) & ~15) + 12 * ((S + 3) & ~3);
        if (fixed + 4096 > c->resolve_lds_max) {
            mam::set_last_error("keypoint capacity too large for the resolve stage");
            return MAM_ERR_CAPACITY;
        }
        a.pool_lds = (int)std::min<size_t>((size_t)mam::RESOLVE_POOL_LDS, (c->resolve_lds_max - fixed) / 4);
        a.flat_lds = (int)(c->resolve_lds_max - fixed);
        hipLaunchKernelGGL(mam::k_resolve, dim3(F), dim3(mam::RESOLVE_THREADS), c->resolve_lds_max, s, a);
    }
    MAM_HIP(hipGetLastError());
#ifdef MAM_RESOLVE_PROFILE
    {
        static int calls = 0;
        if (++calls % 40 == 0) {
            unsigned long long h[2][8];
            MAM_HIP(hipStreamSynchronize(s));
            MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::g_rprof), sizeof(h)));
            for (int m = 0; m < 2; m++)
                fprintf(stderr, "resolve mode %d cycles per WG: setup %.0f claims %.0f resolve %.0f release %.0f loopexit %.0f "
                        "final %.0f; rounds/WG %.1f\n", m,
                        (double)h[m][0] / std::max(1ull, h[m][7]), (double)h[m][3] / std::max(1ull, h[m][7]),
                        (double)h[m][4] / std::max(1ull, h[m][7]), (double)h[m][5] / std::max(1ull, h[m][7]),
                        (double)h[m][1] / std::max(1ull, h[m][7]),
                        (double)h[m][2] / std::max(1ull, h[m][7]), (double)h[m][6] / std::max(1ull, h[m][7]));
        }
    }
#endif
    return MAM_OK;
}

bool geom_ok(const mam_frame_geom* g) { return g && g->nlevels >= 1 && g->nlevels <= MAM_MAX_LEVELS; }

int launch_fuse(mam_match_ctx* c, mam::FuseArgs& a, int F, hipStream_t s) {
    if (F <= 0) return MAM_OK;
    if (a.fr.kp_stride > mam::GRID_SORT_MAX || a.fr.kp_stride <= 0 || a.mp_stride <= 0) return MAM_ERR_ARG;
    const int G = a.frame_of ? a.fr.nframes : F;   // keyframes with a cell grid
    if (G <= 0) return MAM_ERR_ARG;
    if (int rc = c->grid_ent.alloc((size_t)G * a.fr.kp_stride)) return rc;
    if (int rc = c->grid_start.alloc((size_t)G * (mam::NCELLS + 1))) return rc;
    if (int rc = c->pool_total.alloc(G)) return rc;
    if (a.frame_of && (c->grid_status.alloc(G) != MAM_OK)) return MAM_ERR_DEVICE;
    mam::ProjArgs ga{};
    ga.g = a.g;
    ga.fr = a.fr;
    ga.grid_ent = c->grid_ent.p;
    ga.grid_start = c->grid_start.p;
    ga.pool_total = c->pool_total.p;
    ga.out_n = a.frame_of ? c->grid_status.p : a.out_n;
    a.grid_status = a.frame_of ? c->grid_status.p : nullptr;
    if (a.fr.reuse_grid) MAM_HIP(hipMemsetAsync(ga.out_n, 0, sizeof(int32_t) * (size_t)G, s));
    if (int rc = build_grid(c, ga, G, s)) return rc;
    a.grid_ent = c->grid_ent.p;
    a.grid_start = c->grid_start.p;
    {
        mam::StageTimer::Scope sc(&c->timer, s, 4);
        const long long units = (long long)F * a.mp_stride;
        if (F <= 4) {
            hipLaunchKernelGGL(mam::k_fuse<64>, dim3((int)((units * 64 + 255) / 256)), dim3(256), 0, s, a, F);
        } else {
            constexpr int GW = MAM_GATHER_LANES;
            hipLaunchKernelGGL(mam::k_fuse<GW>, dim3((int)((units * GW + 255) / 256)), dim3(256), 0, s, a, F);
        }
        hipLaunchKernelGGL(mam::k_fuse_count, dim3(F), dim3(256), 0, s, a);
    }
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

}  // namespace

extern "C" {

int mam_match_create(int device, mam_match_ctx** out) {
    if (!out) return MAM_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    MAM_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) { mam::set_last_error("no such HIP device"); return MAM_ERR_ARG; }
    MAM_DEVICE_SCOPE(device);
    mam_match_ctx* c = new mam_match_ctx();
    c->device = device;
    // the resolve stage may stage up to ~110 KB in LDS (gfx950: 160 KB per workgroup)
    c->resolve_lds_max = 64 * 1024;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::k_resolve), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024 - 1024) == hipSuccess)
        c->resolve_lds_max = 160 * 1024 - 1024;
    else
        (void)hipGetLastError();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        mam::set_last_error("hipStreamCreate failed");
        return MAM_ERR_DEVICE;
    }
    *out = c;
    return MAM_OK;
}

void mam_match_destroy(mam_match_ctx* c) {
    if (!c) return;
    ::mam::DeviceScope mam_dev_scope_(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int mam_descriptor_distance(mam_match_ctx* c, const uint8_t* a, const uint8_t* b, int n, int32_t* out) {
    if (!c || n < 0 || (n > 0 && (!a || !b || !out))) return MAM_ERR_ARG;
    if (n == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    const size_t bytes = carve_bytes((size_t)n * 32, 1) * 2 + carve_bytes(n, 4);
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    uint8_t* da = carve<uint8_t>(p, (size_t)n * 32);
    uint8_t* db = carve<uint8_t>(p, (size_t)n * 32);
    int32_t* dout = carve<int32_t>(p, n);
    MAM_HIP(hipMemcpyAsync(da, a, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    MAM_HIP(hipMemcpyAsync(db, b, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(mam::k_hamming, dim3((n + 255) / 256), dim3(256), 0, c->stream, da, db, n, dout);
    MAM_HIP(hipMemcpyAsync(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipStreamSynchronize(c->stream));
    return MAM_OK;
}

int mam_search_by_projection_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_frames_dev* fr,
                                          const mam_mp_track* mps, int mp_stride, const int32_t* n_mps, float th,
                                          int far_points, float th_far_points, float nnratio, int32_t* out,
                                          int32_t* out_n, void* stream) {
    if (!c || !geom_ok(g) || !fr || !mps || !n_mps || !out || !out_n || mp_stride <= 0) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    mam::ProjArgs a{};
    a.g = *g;
    a.fr = *fr;
    a.mode = 0;
    a.unit_stride = mp_stride;
    a.n_units = n_mps;
    a.mps = mps;
    a.th = th;
    a.th_far = th_far_points;
    a.nnratio = nnratio;
    a.far_points = far_points;
    set_pool(c, a, mp_stride);
    a.out = out;
    a.out_n = out_n;
    return launch_projection(c, a, fr->nframes, stream ? (hipStream_t)stream : c->stream);
}

int mam_search_by_projection_motion_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_frames_dev* fr,
                                                 const mam_pose* tcw, const mam_camera* cam,
                                                 const mam_last_entry* last, int last_stride, const int32_t* n_last,
                                                 float th, int check_ori, int32_t* out, int32_t* out_n, void* stream) {
    if (!c || !geom_ok(g) || !fr || !tcw || !cam || !last || !n_last || !out || !out_n || last_stride <= 0)
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    mam::ProjArgs a{};
    a.g = *g;
    a.fr = *fr;
    a.mode = 1;
    a.unit_stride = last_stride;
    a.n_units = n_last;
    a.tcw = tcw;
    a.cam = *cam;
    a.last = last;
    a.th = th;
    a.check_ori = check_ori;
    set_pool(c, a, last_stride);
    a.out = out;
    a.out_n = out_n;
    return launch_projection(c, a, fr->nframes, stream ? (hipStream_t)stream : c->stream);
}

int mam_track_motion_search_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_frames_dev* fr,
                                         const mam_pose* tcw, const mam_camera* cam, const mam_last_entry* last,
                                         int last_stride, const int32_t* n_last, float th, int check_ori,
                                         int min_matches, int32_t* out, int32_t* out_n, void* stream) {
    if (!c || !geom_ok(g) || !fr || !tcw || !cam || !last || !n_last || !out || !out_n || last_stride <= 0 ||
        min_matches < 0 || fr->reuse_grid)
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    mam::ProjArgs a{};
    a.g = *g;
    a.fr = *fr;
    a.mode = 1;
    a.unit_stride = last_stride;
    a.n_units = n_last;
    a.tcw = tcw;
    a.cam = *cam;
    a.last = last;
    a.th = th;
    a.check_ori = check_ori;
    set_pool(c, a, last_stride);
    a.out = out;
    a.out_n = out_n;
    if (int rc = launch_projection(c, a, fr->nframes, s)) return rc;
    if (min_matches == 0) return MAM_OK;
    // nmatches < 20: mvpMapPoints cleared and SearchByProjection(Cur, Last, 2 th) over the grid the first search built
    // (the resolve stage rewrites every output slot of a retried frame)
    a.fr.reuse_grid = 1;
    a.th = 2.0f * th;
    a.retry_below = min_matches;
    return launch_projection(c, a, fr->nframes, s);
}

// ---- synchronous single-frame forms over host buffers (reference semantics)
static int stage_frame(mam_match_ctx* c, int n, const mam_keypoint* keys, const uint8_t* desc, const uint8_t* taken,
                       size_t extra_bytes, uint8_t** extra, mam_frames_dev* fr, int32_t** dout, int32_t** dcount,
                       int32_t** dn) {
    const int S = std::max(n, 1);
    const size_t bytes = carve_bytes(S, sizeof(mam_keypoint)) + carve_bytes((size_t)S * 32, 1) + carve_bytes(S, 1) +
                         carve_bytes(S, 4) + carve_bytes(2, 4) + carve_bytes(4, 4) + extra_bytes + 256;
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    mam_keypoint* dk = carve<mam_keypoint>(p, S);
    uint8_t* dd = carve<uint8_t>(p, (size_t)S * 32);
    uint8_t* dt = carve<uint8_t>(p, S);
    *dout = carve<int32_t>(p, S);
    *dcount = carve<int32_t>(p, 2);
    *dn = carve<int32_t>(p, 4);
    *extra = p;
    if (n > 0) {
        MAM_HIP(hipMemcpyAsync(dk, keys, sizeof(mam_keypoint) * n, hipMemcpyHostToDevice, c->stream));
        MAM_HIP(hipMemcpyAsync(dd, desc, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
        if (taken) MAM_HIP(hipMemcpyAsync(dt, taken, n, hipMemcpyHostToDevice, c->stream));
    }
    const int32_t cnt[2] = {n, 0};
    MAM_HIP(hipMemcpyAsync(*dcount, cnt, sizeof(cnt), hipMemcpyHostToDevice, c->stream));
    fr->nframes = 1;
    fr->kp_stride = S;
    fr->keys = dk;
    fr->desc = dd;
    fr->counts = *dcount;
    fr->taken = taken ? dt : nullptr;
    fr->taken_out = nullptr;
    fr->reuse_grid = 0;
    return MAM_OK;
}

int mam_search_by_projection(mam_match_ctx* c, const mam_frame_geom* g, int n, const mam_keypoint* keys,
                             const uint8_t* desc, const uint8_t* taken, int n_mps, const mam_mp_track* mps, float th,
                             int far_points, float th_far_points, float nnratio, int32_t* out) {
    if (!c || !geom_ok(g) || n < 0 || n_mps < 0 || (n > 0 && (!keys || !desc || !out)) || (n_mps > 0 && !mps))
        return MAM_ERR_ARG;
    if (n > mam::GRID_SORT_MAX) return MAM_ERR_CAPACITY;
    MAM_DEVICE_SCOPE(c->device);
    for (int attempt = 0; attempt < 6; attempt++) {
        mam_frames_dev fr;
        uint8_t* extra;
        int32_t *dout, *dcount, *dn;
        const int U = std::max(n_mps, 1);
        if (int rc = stage_frame(c, n, keys, desc, taken, carve_bytes(U, sizeof(mam_mp_track)) + carve_bytes(1, 4),
                                 &extra, &fr, &dout, &dcount, &dn))
            return rc;
        mam_mp_track* dm = carve<mam_mp_track>(extra, U);
        int32_t* dnu = carve<int32_t>(extra, 1);
        if (n_mps > 0) MAM_HIP(hipMemcpyAsync(dm, mps, sizeof(mam_mp_track) * n_mps, hipMemcpyHostToDevice, c->stream));
        MAM_HIP(hipMemcpyAsync(dnu, &n_mps, 4, hipMemcpyHostToDevice, c->stream));
        if (int rc = mam_search_by_projection_batch_device(c, g, &fr, dm, U, dnu, th, far_points, th_far_points,
                                                           nnratio, dout, dn, c->stream))
            return rc;
        int32_t nm = 0;
        MAM_HIP(hipMemcpyAsync(&nm, dn, 4, hipMemcpyDeviceToHost, c->stream));
        if (n > 0) MAM_HIP(hipMemcpyAsync(out, dout, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
        MAM_HIP(hipStreamSynchronize(c->stream));
        if (nm == MAM_ERR_CAPACITY && c->slot_cap < (1 << 12)) { c->slot_cap *= 4; continue; }
        return nm;
    }
    return MAM_ERR_CAPACITY;
}

int mam_search_by_projection_motion(mam_match_ctx* c, const mam_frame_geom* g, int n, const mam_keypoint* keys,
                                    const uint8_t* desc, const uint8_t* taken, const mam_pose* tcw,
                                    const mam_pose* tlw, float mb, const mam_camera* cam, int n_last,
                                    const mam_last_entry* last, float th, int mono, int check_ori, int32_t* out) {
    (void)tlw; (void)mb;
    if (!c || !geom_ok(g) || !tcw || !cam || n < 0 || n_last < 0 || (n > 0 && (!keys || !desc || !out)) ||
        (n_last > 0 && !last))
        return MAM_ERR_ARG;
    if (!mono) { mam::set_last_error("stereo motion search is out of scope (mono agents only)"); return MAM_ERR_ARG; }
    if (n > mam::GRID_SORT_MAX) return MAM_ERR_CAPACITY;
    MAM_DEVICE_SCOPE(c->device);
    for (int attempt = 0; attempt < 6; attempt++) {
        mam_frames_dev fr;
        uint8_t* extra;
        int32_t *dout, *dcount, *dn;
        const int U = std::max(n_last, 1);
        if (int rc = stage_frame(c, n, keys, desc, taken,
                                 carve_bytes(U, sizeof(mam_last_entry)) + carve_bytes(1, 4) + carve_bytes(1, sizeof(mam_pose)),
                                 &extra, &fr, &dout, &dcount, &dn))
            return rc;
        mam_last_entry* dl = carve<mam_last_entry>(extra, U);
        int32_t* dnu = carve<int32_t>(extra, 1);
        mam_pose* dp = carve<mam_pose>(extra, 1);
        if (n_last > 0)
            MAM_HIP(hipMemcpyAsync(dl, last, sizeof(mam_last_entry) * n_last, hipMemcpyHostToDevice, c->stream));
        MAM_HIP(hipMemcpyAsync(dnu, &n_last, 4, hipMemcpyHostToDevice, c->stream));
        MAM_HIP(hipMemcpyAsync(dp, tcw, sizeof(mam_pose), hipMemcpyHostToDevice, c->stream));
        if (int rc = mam_search_by_projection_motion_batch_device(c, g, &fr, dp, cam, dl, U, dnu, th, check_ori, dout,
                                                                  dn, c->stream))
            return rc;
        int32_t nm = 0;
        MAM_HIP(hipMemcpyAsync(&nm, dn, 4, hipMemcpyDeviceToHost, c->stream));
        if (n > 0) MAM_HIP(hipMemcpyAsync(out, dout, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
        MAM_HIP(hipStreamSynchronize(c->stream));
        if (nm == MAM_ERR_CAPACITY && c->slot_cap < (1 << 12)) { c->slot_cap *= 4; continue; }
        return nm;
    }
    return MAM_ERR_CAPACITY;
}

// The search of one keyframe pair; geometry (F12 / R12, t12 / ep) and cameras already set in `ga`.
static int tri_search(mam_match_ctx* c, const mam_frame_geom* g, int n1, const mam_keypoint* keys1,
                      const uint8_t* desc1, const uint8_t* has1, const mam_featvec* fv1, int n2,
                      const mam_keypoint* keys2, const uint8_t* desc2, const uint8_t* has2, const mam_featvec* fv2,
                      const mam::TriArgs& ga, int check_ori, int coarse, int32_t* out) {
    if (!c || !geom_ok(g) || !fv1 || !fv2 || n1 < 0 || n2 < 0 || (n1 > 0 && (!keys1 || !desc1 || !has1 || !out)) ||
        (n2 > 0 && (!keys2 || !desc2 || !has2)))
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    for (int i = 0; i < n1; i++) out[i] = -1;
    if (n1 == 0) return 0;
    // shared vocabulary nodes: the reference's merge walk visits exactly the node ids present in both
    // FeatureVectors (ORBmatcher.cc:958-1108); flatten to one work item per idx1 entry.
    std::vector<int32_t> work, work_n2;
    int a1 = 0, a2 = 0;
    while (a1 < fv1->n_nodes && a2 < fv2->n_nodes) {
        const uint32_t id1 = fv1->node_ids[a1], id2 = fv2->node_ids[a2];
        if (id1 == id2) {
            for (int i1 = fv1->node_off[a1]; i1 < fv1->node_off[a1 + 1]; i1++) {
                work.push_back(i1);
                work_n2.push_back(fv2->node_off[a2]);
                work_n2.push_back(fv2->node_off[a2 + 1]);
            }
            a1++;
            a2++;
        } else if (id1 < id2) {
            a1++;
        } else {
            a2++;
        }
    }
    const int nw = (int)work.size();
    const int nf1 = fv1->node_off[fv1->n_nodes], nf2 = fv2->node_off[fv2->n_nodes];
    const size_t bytes = carve_bytes(n1, sizeof(mam_keypoint)) + carve_bytes((size_t)n1 * 32, 1) + carve_bytes(n1, 1) +
                         carve_bytes(std::max(n2, 1), sizeof(mam_keypoint)) + carve_bytes((size_t)std::max(n2, 1) * 32, 1) +
                         carve_bytes(std::max(n2, 1), 1) + carve_bytes(std::max(nf1, 1), 4) +
                         carve_bytes(std::max(nf2, 1), 4) + carve_bytes(std::max(nw, 1), 4) +
                         carve_bytes(2 * std::max(nw, 1), 4) + carve_bytes(n1, 4) + carve_bytes(1, 4);
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    mam::TriArgs a = ga;
    a.g = *g;
    mam_keypoint* dk1 = carve<mam_keypoint>(p, n1);
    uint8_t* dd1 = carve<uint8_t>(p, (size_t)n1 * 32);
    uint8_t* dh1 = carve<uint8_t>(p, n1);
    mam_keypoint* dk2 = carve<mam_keypoint>(p, std::max(n2, 1));
    uint8_t* dd2 = carve<uint8_t>(p, (size_t)std::max(n2, 1) * 32);
    uint8_t* dh2 = carve<uint8_t>(p, std::max(n2, 1));
    uint32_t* df1 = carve<uint32_t>(p, std::max(nf1, 1));
    uint32_t* df2 = carve<uint32_t>(p, std::max(nf2, 1));
    int32_t* dw = carve<int32_t>(p, std::max(nw, 1));
    int32_t* dw2 = carve<int32_t>(p, 2 * std::max(nw, 1));
    int32_t* dout = carve<int32_t>(p, n1);
    int32_t* dn = carve<int32_t>(p, 1);
    hipStream_t s = c->stream;
    MAM_HIP(hipMemcpyAsync(dk1, keys1, sizeof(mam_keypoint) * n1, hipMemcpyHostToDevice, s));
    MAM_HIP(hipMemcpyAsync(dd1, desc1, (size_t)n1 * 32, hipMemcpyHostToDevice, s));
    MAM_HIP(hipMemcpyAsync(dh1, has1, n1, hipMemcpyHostToDevice, s));
    if (n2 > 0) {
        MAM_HIP(hipMemcpyAsync(dk2, keys2, sizeof(mam_keypoint) * n2, hipMemcpyHostToDevice, s));
        MAM_HIP(hipMemcpyAsync(dd2, desc2, (size_t)n2 * 32, hipMemcpyHostToDevice, s));
        MAM_HIP(hipMemcpyAsync(dh2, has2, n2, hipMemcpyHostToDevice, s));
    }
    if (nf1 > 0) MAM_HIP(hipMemcpyAsync(df1, fv1->feats, 4 * (size_t)nf1, hipMemcpyHostToDevice, s));
    if (nf2 > 0) MAM_HIP(hipMemcpyAsync(df2, fv2->feats, 4 * (size_t)nf2, hipMemcpyHostToDevice, s));
    if (nw > 0) {
        MAM_HIP(hipMemcpyAsync(dw, work.data(), 4 * (size_t)nw, hipMemcpyHostToDevice, s));
        MAM_HIP(hipMemcpyAsync(dw2, work_n2.data(), 8 * (size_t)nw, hipMemcpyHostToDevice, s));
    }
    MAM_HIP(hipMemsetAsync(dout, 0xFF, 4 * (size_t)n1, s));
    a.keys1 = dk1; a.desc1 = dd1; a.has1 = dh1;
    a.keys2 = dk2; a.desc2 = dd2; a.has2 = dh2;
    a.feats1 = df1; a.feats2 = df2;
    a.work = dw; a.work_n2 = dw2; a.nwork = nw;
    a.coarse = coarse;
    a.out = dout;
    {
        mam::StageTimer::Scope sc(&c->timer, s, 3);
        if (nw > 0) hipLaunchKernelGGL(mam::k_tri, dim3((nw + 3) / 4), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mam::k_tri_rot, dim3(1), dim3(256), 0, s, dk1, dk2, n1, check_ori, dout, dn);
    }
    MAM_HIP(hipGetLastError());
    int32_t nm = 0;
    MAM_HIP(hipMemcpyAsync(out, dout, 4 * (size_t)n1, hipMemcpyDeviceToHost, s));
    MAM_HIP(hipMemcpyAsync(&nm, dn, 4, hipMemcpyDeviceToHost, s));
    MAM_HIP(hipStreamSynchronize(s));
    return nm;
}

int mam_search_for_triangulation(mam_match_ctx* c, const mam_frame_geom* g, int n1, const mam_keypoint* keys1,
                                 const uint8_t* desc1, const uint8_t* has1, const mam_featvec* fv1, int n2,
                                 const mam_keypoint* keys2, const uint8_t* desc2, const uint8_t* has2,
                                 const mam_featvec* fv2, const float* F12, const float* ep, int check_ori, int coarse,
                                 int32_t* out) {
    if (!F12 || !ep) return MAM_ERR_ARG;
    mam::TriArgs a{};   // Pinhole cameras (model 0): only F12 / ep are read
    for (int i = 0; i < 9; i++) a.F[i] = F12[i];
    a.ep[0] = ep[0];
    a.ep[1] = ep[1];
    return tri_search(c, g, n1, keys1, desc1, has1, fv1, n2, keys2, desc2, has2, fv2, a, check_ori, coarse, out);
}

int mam_triangulation_geometry(const mam_pose* t1w, const mam_pose* t2w, const mam_camera* cam1,
                               const mam_camera* cam2, float* R12, float* t12, float* F12, float* ep) {
    if (!t1w || !t2w || !cam1 || !cam2) return MAM_ERR_ARG;
    mam::cam::PairGeom pg;
    mam::cam::pair_geometry(t1w->q, t1w->t, t2w->q, t2w->t, *cam1, *cam2, &pg);
    if (R12) for (int i = 0; i < 9; i++) R12[i] = pg.R12[i];
    if (t12) for (int i = 0; i < 3; i++) t12[i] = pg.t12[i];
    if (F12) for (int i = 0; i < 9; i++) F12[i] = pg.F12[i];
    if (ep) { ep[0] = pg.ep[0]; ep[1] = pg.ep[1]; }
    return MAM_OK;
}

int mam_search_for_triangulation_kf(mam_match_ctx* c, const mam_frame_geom* g, const mam_tri_kf* kf1,
                                    const mam_tri_kf* kf2, int check_ori, int coarse, int32_t* out) {
    if (!kf1 || !kf2) return MAM_ERR_ARG;
    if ((kf1->cam.model != MAM_CAM_PINHOLE && kf1->cam.model != MAM_CAM_KANNALA_BRANDT8) ||
        (kf2->cam.model != MAM_CAM_PINHOLE && kf2->cam.model != MAM_CAM_KANNALA_BRANDT8))
        return MAM_ERR_ARG;
    mam::cam::PairGeom pg;
    mam::cam::pair_geometry(kf1->tcw.q, kf1->tcw.t, kf2->tcw.q, kf2->tcw.t, kf1->cam, kf2->cam, &pg);
    mam::TriArgs a{};
    a.cam1 = kf1->cam;
    a.cam2 = kf2->cam;
    for (int i = 0; i < 9; i++) { a.F[i] = pg.F12[i]; a.R12[i] = pg.R12[i]; }
    for (int i = 0; i < 3; i++) a.t12[i] = pg.t12[i];
    a.ep[0] = pg.ep[0];
    a.ep[1] = pg.ep[1];
    return tri_search(c, g, kf1->n, kf1->keys, kf1->desc, kf1->has_mp, &kf1->fv, kf2->n, kf2->keys, kf2->desc,
                      kf2->has_mp, &kf2->fv, a, check_ori, coarse, out);
}

int mam_search_for_triangulation_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_camera* cam,
                                              const mam_tri_batch* b, int check_ori, int coarse, int32_t* out_match12,
                                              int32_t* out_nmatches, void* stream) {
    if (!c || !geom_ok(g) || !cam || !b || !out_match12 || !out_nmatches || b->npairs < 0 || b->kfs.nframes < 0 ||
        b->kfs.kp_stride <= 0 || b->kfs.kp_stride > 8192 || !b->kfs.keys || !b->kfs.desc || !b->kfs.counts ||
        !b->has_mp || !b->nid || !b->weight || !b->tcw || (b->npairs > 0 && !b->pairs))
        return MAM_ERR_ARG;
    if (cam->model != MAM_CAM_PINHOLE && cam->model != MAM_CAM_KANNALA_BRANDT8) return MAM_ERR_ARG;
    if (b->npairs == 0 || b->kfs.nframes == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const int nkf = b->kfs.nframes, S = b->kfs.kp_stride;
    int P = 1;
    while (P < S) P <<= 1;
    const bool keep = c->tri_raw.p && c->tri_P == P && c->tri_nkf == nkf && c->tri_skey.n >= (size_t)nkf * P;
    if (int rc = c->tri_skey.alloc((size_t)nkf * P)) return rc;
    if (int rc = c->tri_raw.alloc((size_t)nkf * P)) return rc;
    if (int rc = c->tri_nfv.alloc(nkf)) return rc;
    if (int rc = c->tri_ok.alloc(nkf)) return rc;
    if (!keep) MAM_HIP(hipMemsetAsync(c->tri_ok.p, 0, sizeof(int32_t) * nkf, s));
    c->tri_P = P;
    c->tri_nkf = nkf;
    if (int rc = c->tri_pg.alloc(b->npairs)) return rc;
    mam::TriBatchArgs a{};
    a.g = *g;
    a.kfs = b->kfs;
    a.has_mp = b->has_mp;
    a.nid = b->nid;
    a.weight = b->weight;
    a.tcw = b->tcw;
    a.pairs = b->pairs;
    a.npairs = b->npairs;
    a.cam = *cam;
    a.coarse = coarse;
    a.check_ori = check_ori;
    a.skey = c->tri_skey.p;
    a.skey_stride = P;
    a.nfv = c->tri_nfv.p;
    a.raw = c->tri_raw.p;
    a.raw_ok = c->tri_ok.p;
    a.pg = c->tri_pg.p;
    a.out = out_match12;
    a.out_n = out_nmatches;
    {
        mam::StageTimer::Scope sc(&c->timer, s, 3);
        hipLaunchKernelGGL(mam::k_tri_fv_sort, dim3(nkf), dim3(1024), sizeof(unsigned long long) * P, s, a);
        hipLaunchKernelGGL(mam::k_tri_pair_geom, dim3((b->npairs + 255) / 256), dim3(256), 0, s, a);
        const size_t lds_pair = sizeof(unsigned long long) * P + (size_t)S;
        if (lds_pair > 65536 &&
            hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::k_tri_pair),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pair) != hipSuccess) {
            (void)hipGetLastError();
            mam::set_last_error("k_tri_pair: LDS request above the device limit");
            return MAM_ERR_CAPACITY;
        }
        hipLaunchKernelGGL(mam::k_tri_pair, dim3(b->npairs), dim3(mam::TRI_THREADS),
                           sizeof(unsigned long long) * P + (size_t)S, s, a);
    }
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

int mam_fuse_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_frames_dev* fr, const mam_fuse_kf* kfs,
                          const mam_camera* cam, const mam_fuse_mp* mps, int mp_stride, const int32_t* n_mps, float th,
                          int32_t* out_idx, int32_t* out_dist, int32_t* out_n, void* stream) {
    if (!c || !geom_ok(g) || !fr || !kfs || !cam || !mps || !n_mps || !out_idx || !out_dist || !out_n || mp_stride <= 0)
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    mam::FuseArgs a{};
    a.g = *g;
    a.fr = *fr;
    a.kfs = kfs;
    a.cam = *cam;
    a.mps = mps;
    a.mp_stride = mp_stride;
    a.n_mps = n_mps;
    a.th = th;
    a.out_idx = out_idx;
    a.out_dist = out_dist;
    a.out_n = out_n;
    return launch_fuse(c, a, fr->nframes, stream ? (hipStream_t)stream : c->stream);
}

int mam_fuse_items_batch_device(mam_match_ctx* c, const mam_frame_geom* g, const mam_frames_dev* fr,
                                const mam_pose* kf_tcw, float log_scale_factor, const mam_camera* cam, int n_items,
                                const int32_t* frame_of, const int32_t* mp_of, const mam_fuse_mp* mps, int mp_stride,
                                const int32_t* n_mps, float th, int32_t* out_idx, int32_t* out_dist,
                                int32_t* out_nfused, void* stream) {
    if (!c || !geom_ok(g) || !fr || !kf_tcw || !cam || n_items < 0 || !frame_of || !mp_of || !mps || !n_mps ||
        !out_idx || !out_dist || !out_nfused || mp_stride <= 0 || fr->nframes <= 0)
        return MAM_ERR_ARG;
    if (n_items == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    mam::FuseArgs a{};
    a.g = *g;
    a.fr = *fr;
    a.kfs = nullptr;
    a.cam = *cam;
    a.mps = mps;
    a.mp_stride = mp_stride;
    a.n_mps = n_mps;
    a.th = th;
    a.out_idx = out_idx;
    a.out_dist = out_dist;
    a.out_n = out_nfused;
    a.frame_of = frame_of;
    a.mp_of = mp_of;
    a.kf_tcw = kf_tcw;
    a.log_scale_factor = log_scale_factor;
    return launch_fuse(c, a, n_items, stream ? (hipStream_t)stream : c->stream);
}

int mam_fuse(mam_match_ctx* c, const mam_frame_geom* g, int n, const mam_keypoint* keys, const uint8_t* desc,
             const mam_fuse_kf* kf, const mam_camera* cam, int n_mps, const mam_fuse_mp* mps, float th,
             int32_t* out_idx, int32_t* out_dist) {
    if (!c || !geom_ok(g) || !kf || !cam || n < 0 || n_mps < 0 || (n > 0 && (!keys || !desc)) ||
        (n_mps > 0 && (!mps || !out_idx || !out_dist)))
        return MAM_ERR_ARG;
    if (n > mam::GRID_SORT_MAX) return MAM_ERR_CAPACITY;
    if (n_mps == 0) return 0;
    MAM_DEVICE_SCOPE(c->device);
    mam_frames_dev fr;
    uint8_t* extra;
    int32_t *dout, *dcount, *dn;
    const size_t eb = carve_bytes(n_mps, sizeof(mam_fuse_mp)) + 2 * carve_bytes(n_mps, 4) + carve_bytes(1, 4) +
                      carve_bytes(1, sizeof(mam_fuse_kf));
    if (int rc = stage_frame(c, n, keys, desc, nullptr, eb, &extra, &fr, &dout, &dcount, &dn)) return rc;
    mam_fuse_mp* dm = carve<mam_fuse_mp>(extra, n_mps);
    int32_t* di = carve<int32_t>(extra, n_mps);
    int32_t* dd = carve<int32_t>(extra, n_mps);
    int32_t* dnu = carve<int32_t>(extra, 1);
    mam_fuse_kf* dk = carve<mam_fuse_kf>(extra, 1);
    MAM_HIP(hipMemcpyAsync(dm, mps, sizeof(mam_fuse_mp) * n_mps, hipMemcpyHostToDevice, c->stream));
    MAM_HIP(hipMemcpyAsync(dnu, &n_mps, 4, hipMemcpyHostToDevice, c->stream));
    MAM_HIP(hipMemcpyAsync(dk, kf, sizeof(mam_fuse_kf), hipMemcpyHostToDevice, c->stream));
    if (int rc = mam_fuse_batch_device(c, g, &fr, dk, cam, dm, n_mps, dnu, th, di, dd, dn, c->stream)) return rc;
    int32_t nf = 0;
    MAM_HIP(hipMemcpyAsync(&nf, dn, 4, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipMemcpyAsync(out_idx, di, sizeof(int32_t) * n_mps, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipMemcpyAsync(out_dist, dd, sizeof(int32_t) * n_mps, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipStreamSynchronize(c->stream));
    return nf;
}

int mam_compute_distinctive_descriptors_batch_device(mam_match_ctx* c, int n_mps, const int32_t* off,
                                                     const uint8_t* descs, int32_t* out, void* stream) {
    if (!c || n_mps < 0 || (n_mps > 0 && (!off || !descs || !out))) return MAM_ERR_ARG;
    if (n_mps == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    {
        mam::StageTimer::Scope sc(&c->timer, s, 5);
        hipLaunchKernelGGL(mam::k_distinct, dim3((n_mps + 3) / 4), dim3(256), 0, s, off, descs, n_mps, out);
    }
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

int mam_compute_distinctive_descriptors(mam_match_ctx* c, int n_mps, const int32_t* off, const uint8_t* descs,
                                        int32_t* out) {
    if (!c || n_mps < 0 || (n_mps > 0 && (!off || !out))) return MAM_ERR_ARG;
    if (n_mps == 0) return MAM_OK;
    if (off[0] < 0) return MAM_ERR_ARG;
    for (int m = 0; m < n_mps; m++)
        if (off[m + 1] < off[m]) return MAM_ERR_ARG;
    const int total = off[n_mps];
    if (total > 0 && !descs) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    const size_t rows = (size_t)std::max(total, 1);
    const size_t bytes = carve_bytes((size_t)n_mps + 1, 4) + carve_bytes(rows * 32, 1) + carve_bytes(n_mps, 4);
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    int32_t* doff = carve<int32_t>(p, (size_t)n_mps + 1);
    uint8_t* dd = carve<uint8_t>(p, rows * 32);
    int32_t* dout = carve<int32_t>(p, n_mps);
    MAM_HIP(hipMemcpyAsync(doff, off, sizeof(int32_t) * ((size_t)n_mps + 1), hipMemcpyHostToDevice, c->stream));
    if (total > 0) MAM_HIP(hipMemcpyAsync(dd, descs, (size_t)total * 32, hipMemcpyHostToDevice, c->stream));
    if (int rc = mam_compute_distinctive_descriptors_batch_device(c, n_mps, doff, dd, dout, c->stream)) return rc;
    MAM_HIP(hipMemcpyAsync(out, dout, sizeof(int32_t) * n_mps, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipStreamSynchronize(c->stream));
    return MAM_OK;
}

int mam_is_in_frustum_batch_device(mam_match_ctx* c, const mam_frame_geom* g, int nframes, const mam_pose* tcw,
                                   const mam_camera* cam, float log_scale_factor, const mam_local_mp* mps,
                                   int mp_stride, const int32_t* n_mps, float view_cos_limit, mam_mp_track* out,
                                   int32_t* out_n_to_match, void* stream) {
    if (!c || !geom_ok(g) || nframes < 0 || !cam || mp_stride <= 0 || (nframes > 0 && (!tcw || !mps || !n_mps || !out)))
        return MAM_ERR_ARG;
    if (nframes == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    mam::FrustumArgs a{};
    a.g = *g;
    a.tcw = tcw;
    a.cam = *cam;
    a.log_scale_factor = log_scale_factor;
    a.view_cos_limit = view_cos_limit;
    a.mps = mps;
    a.mp_stride = mp_stride;
    a.n_mps = n_mps;
    a.out = out;
    a.out_n = out_n_to_match;
    mam::StageTimer::Scope sc(&c->timer, s, 6);
    if (out_n_to_match) MAM_HIP(hipMemsetAsync(out_n_to_match, 0, sizeof(int32_t) * (size_t)nframes, s));
    hipLaunchKernelGGL(mam::k_frustum, dim3((mp_stride + 255) / 256, nframes), dim3(256), 0, s, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

int mam_is_in_frustum(mam_match_ctx* c, const mam_frame_geom* g, const mam_pose* tcw, const mam_camera* cam,
                      float log_scale_factor, int n_mps, const mam_local_mp* mps, float view_cos_limit,
                      mam_mp_track* out) {
    if (!c || !geom_ok(g) || !tcw || !cam || n_mps < 0 || (n_mps > 0 && (!mps || !out))) return MAM_ERR_ARG;
    if (n_mps == 0) return 0;
    MAM_DEVICE_SCOPE(c->device);
    const size_t bytes = carve_bytes(sizeof(mam_pose), 1) + carve_bytes(n_mps, sizeof(mam_local_mp)) +
                         carve_bytes(n_mps, sizeof(mam_mp_track)) + carve_bytes(2, 4);
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    mam_pose* dT = carve<mam_pose>(p, 1);
    mam_local_mp* dm = carve<mam_local_mp>(p, n_mps);
    mam_mp_track* dout = carve<mam_mp_track>(p, n_mps);
    int32_t* dn = carve<int32_t>(p, 2);
    hipStream_t s = c->stream;
    MAM_HIP(hipMemcpyAsync(dT, tcw, sizeof(mam_pose), hipMemcpyHostToDevice, s));
    MAM_HIP(hipMemcpyAsync(dm, mps, sizeof(mam_local_mp) * (size_t)n_mps, hipMemcpyHostToDevice, s));
    MAM_HIP(hipMemcpyAsync(dn, &n_mps, sizeof(int32_t), hipMemcpyHostToDevice, s));
    if (int rc = mam_is_in_frustum_batch_device(c, g, 1, dT, cam, log_scale_factor, dm, n_mps, dn, view_cos_limit,
                                                dout, dn + 1, s))
        return rc;
    int32_t nt = 0;
    MAM_HIP(hipMemcpyAsync(out, dout, sizeof(mam_mp_track) * (size_t)n_mps, hipMemcpyDeviceToHost, s));
    MAM_HIP(hipMemcpyAsync(&nt, dn + 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MAM_HIP(hipStreamSynchronize(s));
    return nt;
}

int mam_match_set_profiling(mam_match_ctx* c, int enable) {
    if (!c) return MAM_ERR_ARG;
    c->timer.reset(enable != 0);
    return MAM_OK;
}

int mam_match_stage_times(mam_match_ctx* c, double* ms_out, int64_t* launches_out) {
    if (!c) return MAM_ERR_ARG;
    c->timer.collect();
    for (int i = 0; i < 7; i++) {
        if (ms_out) ms_out[i] = c->timer.ms[i];
        if (launches_out) launches_out[i] = c->timer.n[i];
    }
    return MAM_OK;
}

}  // extern "C"
