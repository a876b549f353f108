// orb_kernels.hip — gfx950 kernels of the ORB extraction hot path (MI355X, wave64).
//
// Stage map (reference call stack SURVEY.md §3.A):
//   k_pyr_down      ComputePyramid: cv::resize INTER_LINEAR 8U, level l from level l-1
//                   (src/ORBextractor.cc:1170-1195); one launch per level, batched over frames.
//   k_fast_cells    ComputeKeyPointsOctTree's per-cell FAST (src/ORBextractor.cc:805-872): one workgroup per
//                   35-px cell of every level of every frame; ROI staged in LDS, FAST-9 "strength" per
//                   pixel, in-cell 3x3 NMS at iniThFAST, retry at minThFAST only if the cell came out empty,
//                   ordered compaction (wave ballots + LDS scan) into per-cell candidate slots.
//   k_blur7         GaussianBlur(7x7, sigma 2, REFLECT_101) fixed-point (src/ORBextractor.cc:1132-1133): LDS
//                   tiles, separable integer passes, all levels in one launch.
//   k_distribute    DistributeOctTree (src/ORBextractor.cc:555-779): one workgroup per (frame, level); the
//                   quadtree rounds are rebuilt in parallel (list order reconstructed by scans), the
//                   final-phase std::sort replayed by mam::stl_sort; retain-best per node; lapping ranks.
//   k_describe      IC_Angle + computeOrbDescriptor + lapping placement (src/ORBextractor.cc:76-146,
//                   1122-1165): one wave per keypoint; rBRIEF bits built by __ballot.
//
// Integer/byte work throughout: HBM- and latency-bound, no MFMA.
#include <hip/hip_runtime.h>

#include "det_math.hpp"
#include "introsort.hpp"
#include "orb_common.hpp"

namespace mam {

__constant__ int8_t c_pattern[1024] = {
#include "orb_pattern.inc"
};

// Gaussian taps of cv::GaussianBlur(7x7, sigma=2) on 8U in fixed point (getGaussianKernelBitExact +
// getGaussianKernelFixedPoint_ED, 8 fractional bits).
#define GT0 18
#define GT1 34
#define GT2 48
#define GT3 56

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

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

// Exclusive scan over a 256-thread block. scr: >= 4 ints of LDS. All threads must call.
__device__ __forceinline__ int block_excl_scan(int v, int* scr, int* total) {
    const int incl = wave_incl_scan(v);
    const int w = wave_id();
    if (lane_id() == 63) scr[w] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int s = scr[i];
        if (i < w) pre += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return incl - v + pre;
}

__device__ __forceinline__ int block_sum(int v, int* scr) {
    int t;
    block_excl_scan(v, scr, &t);
    return t;
}

__device__ __forceinline__ int block_min(int v, int* scr) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    if (lane_id() == 0) scr[wave_id()] = v;
    __syncthreads();
    int r = min(min(scr[0], scr[1]), min(scr[2], scr[3]));
    __syncthreads();
    return r;
}

struct LevelSrc {
    const uint8_t* in0;
    size_t in_stride;
    size_t in_fstride;
    const uint8_t* pyr;
};

__device__ __forceinline__ const uint8_t* level_ptr(const Geom* g, const LevelSrc& s, int f, int l, int* pitch) {
    if (l == 0) {
        *pitch = (int)s.in_stride;
        return s.in0 + (size_t)f * s.in_fstride;
    }
    const LevelGeom& L = g->L[l];
    *pitch = L.pitch;
    return s.pyr + L.pyr_off + (size_t)f * L.frame_bytes;
}

// ------------------------------------------------------------------------------------------------ pyramid
// Column setup of one output quad dx..dx+3: its source columns sx[i] (and sx[i]+1) as byte offsets o[i] from the
// word-aligned column `base`, horizontal weights (right-edge replicate columns dx >= xmax folded in as a0 = 2048,
// a1 = 0: S[sx]*2048 + S[sx+1]*0 is the reference's S[sx]*2048) and which columns take the SIMD vertical formula
// (dx < xvec). The host guarantees o[i] + 1 <= 11 (three source words per row).
struct PyrQuad {
    int base;
    int o[4], a0[4], a1[4];
    bool vec[4];
};

__device__ __forceinline__ void pyr_quad_setup(const LevelGeom& L, int dx, int sx_shift, PyrQuad& c) {
    int sx[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int x = min(dx + i, L.w - 1);
        sx[i] = L.xofs[x] - sx_shift;
        const bool edge = dx + i >= L.xmax;
        c.a0[i] = edge ? 2048 : L.ialpha[2 * x];
        c.a1[i] = edge ? 0 : L.ialpha[2 * x + 1];
        c.vec[i] = dx + i < L.xvec;
    }
    c.base = sx[0] & ~3;
#pragma unroll
    for (int i = 0; i < 4; i++) c.o[i] = sx[i] - c.base;
}

// bytes o and o+1 of the 12-byte window w0:w1:w2 (o <= 10), as (b0, b1)
__device__ __forceinline__ void pyr_pair(uint32_t w0, uint32_t w1, uint32_t w2, int o, int& b0, int& b1) {
    const uint32_t lo = o < 4 ? w0 : (o < 8 ? w1 : w2);
    const uint32_t hi = o < 4 ? w1 : w2;
    const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(o & 3));
    b0 = (int)(v & 0xFFu);
    b1 = (int)((v >> 8) & 0xFFu);
}

// Four output pixels of one output row from source rows S0 (ry0) and S1 (ry1) (word-aligned row starts): exact-int
// horizontal pass (HResizeLinear), vertical pass with VResizeLinearVec_32s8u's mulhi formula for x < xvec and
// FixedPtCast<int,uchar,22> beyond. Three word loads per source row.
// nw: words in a source row; the words past it are read as 0 (only zero-weight edge columns reach them), so the
// last row of the caller's last frame is never read past
__device__ __forceinline__ uint32_t pyr_quad(const uint8_t* S0, const uint8_t* S1, const PyrQuad& c, int b0,
                                             int b1, int nw = 1 << 30) {
    const uint32_t* r0 = reinterpret_cast<const uint32_t*>(S0 + c.base);
    const uint32_t* r1 = reinterpret_cast<const uint32_t*>(S1 + c.base);
    const int wq = c.base >> 2;
    const bool h1 = wq + 1 < nw, h2 = wq + 2 < nw;
    const uint32_t x0 = r0[0], x1 = h1 ? r0[1] : 0u, x2 = h2 ? r0[2] : 0u;
    const uint32_t y0 = r1[0], y1 = h1 ? r1[1] : 0u, y2 = h2 ? r1[2] : 0u;
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int p0, p1, q0, q1;
        pyr_pair(x0, x1, x2, c.o[i], p0, p1);
        pyr_pair(y0, y1, y2, c.o[i], q0, q1);
        const int h0 = p0 * c.a0[i] + p1 * c.a1[i];
        const int h1 = q0 * c.a0[i] + q1 * c.a1[i];
        const int t0 = min(max(h0 >> 4, -32768), 32767);
        const int t1 = min(max(h1 >> 4, -32768), 32767);
        const int m0 = (t0 * b0) >> 16, m1 = (t1 * b1) >> 16;
        int sum = min(max(m0 + m1, -32768), 32767);
        sum = min(max(sum + 2, -32768), 32767);
        const int vs = sum >> 2;
        const int vf = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
        const int v = min(max(c.vec[i] ? vs : vf, 0), 255);
        packed |= (uint32_t)v << (8 * i);
    }
    return packed;
}

// One thread per output quad column and RQ consecutive output rows of the whole level (row-major over every frame's
// level): no LDS staging, every lane busy (the block kernel leaves most lanes idle on levels narrower than its
// 1024-pixel tiles), the quad's column coefficients pre-packed (LevelGeom.qcoef) and loaded once for its RQ rows, the
// three source words per row read straight from the level above, all RQ rows' loads issued before the first store.
// Requires word-aligned source rows (the host falls back to k_pyr_down otherwise).
template <int RQ>
__global__ __launch_bounds__(256) void k_pyr_flat(const Geom* __restrict__ g, int l, LevelSrc s, uint8_t* pyr) {
    const LevelGeom& L = g->L[l];
    const int nq = (L.w + 3) >> 2;
    const int nrg = (L.h + RQ - 1) / RQ;
    const int qi = blockIdx.x * 256 + threadIdx.x;
    const int f = blockIdx.y;
    if (qi >= nq * nrg) return;
    const int rg = qi / nq, q = qi - rg * nq;
    const uint4 c0 = L.qcoef[2 * q], c1 = L.qcoef[2 * q + 1];
    PyrQuad cq;
    cq.base = (int)(c0.x & 0xFFFu);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        cq.o[i] = (int)((c0.x >> (12 + 4 * i)) & 0xFu);
        cq.vec[i] = ((c0.x >> (28 + i)) & 1u) != 0;
    }
    const uint32_t pa[4] = {c0.y, c0.z, c0.w, c1.x};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        cq.a0[i] = (int)(pa[i] & 0xFFFFu);
        cq.a1[i] = (int)(pa[i] >> 16);
    }
    const int sh = g->L[l - 1].h;
    const int snw = (g->L[l - 1].w + 3) >> 2;
    int spitch;
    const uint8_t* src = level_ptr(g, s, f, l - 1, &spitch);
    uint32_t packed[RQ];
#pragma unroll
    for (int k = 0; k < RQ; k++) {
        const int dy = min(rg * RQ + k, L.h - 1);   // rows past the level repeat the last one (not stored)
        const int2 rc = L.rcoef[dy];
        const int sy = rc.x;
        const int ry0 = sy >= 0 ? (sy < sh ? sy : sh - 1) : 0;
        const int ry1 = sy + 1 >= 0 ? (sy + 1 < sh ? sy + 1 : sh - 1) : 0;
        packed[k] = pyr_quad(src + (size_t)ry0 * spitch, src + (size_t)ry1 * spitch, cq, (int)(short)(rc.y & 0xFFFF),
                             rc.y >> 16, snw);
    }
    uint8_t* o = pyr + L.pyr_off + (size_t)f * L.frame_bytes + 4 * q;
#pragma unroll
    for (int k = 0; k < RQ; k++) {
        const int dy = rg * RQ + k;
        if (dy >= L.h) break;
        uint8_t* od = o + (size_t)dy * L.pitch;
        if (4 * q + 4 <= L.w) {
            *reinterpret_cast<uint32_t*>(od) = packed[k];
        } else {
            for (int i = 0; i < 4 && 4 * q + i < L.w; i++) od[i] = (uint8_t)(packed[k] >> (8 * i));
        }
    }
}

// One workgroup per PYR_XB x PYR_RB output block: the source rows/columns the block reads are staged in LDS
// (32-bit loads where aligned), each thread owns one 4-pixel column quad for the block's rows and keeps its
// xofs/alpha coefficients in registers.
__global__ __launch_bounds__(256) void k_pyr_down(const Geom* __restrict__ g, int l, LevelSrc s, uint8_t* pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t rbuf[];
    const LevelGeom& L = g->L[l];
    const LevelGeom& P = g->L[l - 1];
    const int f = blockIdx.z;
    const int dx0 = blockIdx.x * PYR_XB, dy0 = blockIdx.y * PYR_RB;
    const int nx = min(PYR_XB, L.w - dx0), ny = min(PYR_RB, L.h - dy0);
    const int SW = g->pyr_seg_w;
    int spitch;
    const uint8_t* src = level_ptr(g, s, f, l - 1, &spitch);
    uint8_t* dst = pyr + L.pyr_off + (size_t)f * L.frame_bytes;
    const int sh = P.h;
    const int sxa = L.xofs[dx0] & ~3;
    const int sxb = min(L.xofs[dx0 + nx - 1] + 1, P.w - 1);
    const int segw = sxb - sxa + 1;
    const int ry_lo = min(max(L.yofs[dy0], 0), sh - 1);
    const int ry_hi = min(max(L.yofs[dy0 + ny - 1] + 1, 0), sh - 1);
    const int nrows = ry_hi - ry_lo + 1;
    const int tid = threadIdx.x;
    const bool aligned = ((spitch | (int)((uintptr_t)src & 3)) & 3) == 0;
    const int nw = aligned ? segw >> 2 : 0;   // whole words inside the segment
    for (int i0 = 0; i0 < nrows * nw; i0 += 8 * 256) {   // 8 global loads in flight per thread, then the stores
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int i = i0 + k * 256 + tid;
            const int r = i / max(nw, 1), c = i - r * nw;
            v[k] = i < nrows * nw ? *reinterpret_cast<const uint32_t*>(src + (size_t)(ry_lo + r) * spitch + sxa + 4 * c)
                                  : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int i = i0 + k * 256 + tid;
            const int r = i / max(nw, 1), c = i - r * nw;
            if (i < nrows * nw) *reinterpret_cast<uint32_t*>(rbuf + r * SW + 4 * c) = v[k];
        }
    }
    const int tail = segw - 4 * nw;
    for (int i = tid; i < nrows * tail; i += 256) {
        const int r = i / tail, c = 4 * nw + (i - r * tail);
        rbuf[r * SW + c] = src[(size_t)(ry_lo + r) * spitch + sxa + c];
    }
    __syncthreads();
    const int q = tid;   // PYR_XB / 4 == 256 quads
    if (4 * q >= nx) return;
    PyrQuad cq;
    pyr_quad_setup(L, dx0 + 4 * q, sxa, cq);
    for (int rr = 0; rr < ny; rr++) {
        const int dy = dy0 + rr;
        const int sy = L.yofs[dy];
        const int ry0 = sy >= 0 ? (sy < sh ? sy : sh - 1) : 0;
        const int ry1 = sy + 1 >= 0 ? (sy + 1 < sh ? sy + 1 : sh - 1) : 0;
        const uint32_t packed = pyr_quad(rbuf + (ry0 - ry_lo) * SW, rbuf + (ry1 - ry_lo) * SW, cq, L.ibeta[2 * dy],
                                         L.ibeta[2 * dy + 1]);
        uint8_t* o = dst + (size_t)dy * L.pitch + dx0 + 4 * q;
        if (dx0 + 4 * q + 4 <= L.w) {
            *reinterpret_cast<uint32_t*>(o) = packed;
        } else {
            for (int i = 0; i < 4 && dx0 + 4 * q + i < L.w; i++) o[i] = (uint8_t)(packed >> (8 * i));
        }
    }
}

// Whole pyramid of one frame in ONE launch: workgroup (band j, frame f) owns rows [own_lo, own_hi) of every level
// l >= 1 (an even split of each level's rows) and computes, in LDS, the rows [need_lo, need_hi) of every level that
// its owned rows of the higher levels depend on (host-derived from yofs, PyrBand). Level l is computed from level
// l-1's LDS rows (level 1 from the input frame in global memory), owned rows are stored to the pyramid buffer.
// Rows shared by two bands are computed by both: ~1.1-1.5x the arithmetic of the per-level launches, 7 dependent
// launches (and their per-launch latency, ~10 us each at one frame) become one. Arithmetic identical to
// k_pyr_down (pyr_quad). Thread t works on quad column q = t % nq for rows t / nq, t / nq + RG, ... so its
// column coefficients stay in registers for the whole level.

// A level's parameters for k_pyr_bands, staged once in LDS (the level loop reads no global memory but its stores)
struct PyrLvl {
    int w, h, pitch, sh;      // level size and pitch, the source level's height
    int sp, r0, qbase, rcoff;  // source LDS pitch and first row, the level's quads in the column table, row coefs
    int4 bl;                   // the band's rows of this level (needed [x, y), owned [z, w))
    uint8_t* gdst;             // the level in the pyramid buffer (this frame)
};

// One level of k_pyr_bands: rows [bl.x, bl.y) of level l from the LDS rows of level l-1 (first row P.r0, pitch
// P.sp); rc = this level's row coefficients {yofs, ibeta0 | ibeta1 << 16} for rows bl.x.. (LDS), qa / qb its quads'
// packed column coefficients (LevelGeom.qcoef: word 0..3 of the first uint4, word 0 of the second).
template <int NT>
__device__ __forceinline__ void pyr_band_level(const PyrLvl& P, const uint8_t* src, const int2* rc, const uint4* qa,
                                               const uint32_t* qb, uint8_t* lds_dst, bool keep, int tid) {
    const int dp = (P.w + 3) & ~3;
    const int nq = (P.w + 3) >> 2;
    const int RG = max(1, NT / nq);
    const int4 bl = P.bl;
    const int nrows = bl.y - bl.x;
    for (int t = tid; t < nq * RG; t += NT) {
        const int q = t % nq, rg = t / nq;
        PyrQuad c;
        {
            const uint4 c0 = qa[q];
            const uint32_t pa[4] = {c0.y, c0.z, c0.w, qb[q]};
            c.base = (int)(c0.x & 0xFFFu);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                c.o[i] = (int)((c0.x >> (12 + 4 * i)) & 0xFu);
                c.vec[i] = ((c0.x >> (28 + i)) & 1u) != 0;
                c.a0[i] = (int)(pa[i] & 0xFFFFu);
                c.a1[i] = (int)(pa[i] >> 16);
            }
        }
#pragma unroll 2
        for (int r = rg; r < nrows; r += RG) {
            const int dy = bl.x + r;
            const int2 yc = rc[r];
            const int sy = yc.x;
            const int ry0 = sy >= 0 ? (sy < P.sh ? sy : P.sh - 1) : 0;
            const int ry1 = sy + 1 >= 0 ? (sy + 1 < P.sh ? sy + 1 : P.sh - 1) : 0;
            const uint32_t packed = pyr_quad(src + (ry0 - P.r0) * P.sp, src + (ry1 - P.r0) * P.sp, c,
                                             (int)(short)(yc.y & 0xFFFF), yc.y >> 16);
            if (keep) *reinterpret_cast<uint32_t*>(lds_dst + r * dp + 4 * q) = packed;
            if (dy >= bl.z && dy < bl.w) {
                uint8_t* o = P.gdst + (size_t)dy * P.pitch + 4 * q;
                if (4 * q + 4 <= P.w) {
                    *reinterpret_cast<uint32_t*>(o) = packed;
                } else {
                    for (int i = 0; i < 4 && 4 * q + i < P.w; i++) o[i] = (uint8_t)(packed >> (8 * i));
                }
            }
        }
    }
}

#ifdef MAM_PYR_PROFILE
// cycles per phase summed over workgroups (thread 0): [0] prologue (level-0 rows + row / column coefficients staged),
// [l] level l, [9] workgroups
__device__ unsigned long long g_pyrprof[10];
#define PYRP(k)                                                                        \
    do {                                                                               \
        if (tid == 0) {                                                                \
            const long long tn_ = clock64();                                           \
            atomicAdd(&g_pyrprof[k], (unsigned long long)(tn_ - pt0));                 \
            pt0 = tn_;                                                                 \
        }                                                                              \
    } while (0)
#else
#define PYRP(k) do {} while (0)
#endif

// LDS: [even levels' rows (level 0 staged from the frame)] [odd levels' rows] [row coefficients of every level]
// [column coefficients of every level: qtot uint4, then qtot words]. The prologue puts everything with a global-memory
// latency in flight at once (level-0 rows, all row and column coefficients, the levels' parameters); the level loop
// then reads LDS only — each level is its compute and one barrier (a global load per level, the coefficient prefetch
// of the round-4 form, measured ~3-5 us per level at one frame: the chain of levels paid it seven times).
template <int NT>
__global__ __launch_bounds__(NT) void k_pyr_bands(const Geom* __restrict__ g, LevelSrc s, uint8_t* __restrict__ pyr,
                                                   const int4* __restrict__ bands, int buf1_off, int rc_off,
                                                   int qc_off, int qtot) {
    extern __shared__ __attribute__((aligned(16))) uint8_t pbuf[];
    __shared__ PyrLvl lv[MAM_MAX_LEVELS];
    const int j = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, NL = g->nlevels;
    const int4* B = bands + (size_t)j * NL;
    int2* rcoef = reinterpret_cast<int2*>(pbuf + rc_off);
    uint4* qa = reinterpret_cast<uint4*>(pbuf + qc_off);
    uint32_t* qb = reinterpret_cast<uint32_t*>(pbuf + qc_off + (size_t)qtot * 16);
#ifdef MAM_PYR_PROFILE
    long long pt0 = clock64();
    if (tid == 0) atomicAdd(&g_pyrprof[9], 1ull);
#endif
    // ---- prologue
    if (tid < NL) {
        // the levels' parameters (each thread sums the row / quad offsets of the levels below its own)
        const int l = tid;
        const LevelGeom& L = g->L[l];
        PyrLvl P;
        P.w = L.w;
        P.h = L.h;
        P.pitch = L.pitch;
        P.bl = B[l];
        P.gdst = pyr + L.pyr_off + (size_t)f * L.frame_bytes;
        P.sh = l > 0 ? g->L[l - 1].h : 0;
        P.sp = l > 0 ? ((g->L[l - 1].w + 3) & ~3) : 0;
        P.r0 = l > 0 ? B[l - 1].x : 0;
        int qb0 = 0, rc0 = 0;
        for (int k = 1; k < l; k++) {
            qb0 += (g->L[k].w + 3) >> 2;
            const int4 bk = B[k];
            rc0 += bk.y - bk.x;
        }
        P.qbase = qb0;
        P.rcoff = rc0;
        lv[l] = P;
    }
    {
        // level-0 rows [B[0].x, B[0].y), the band's row coefficients of every level, the column coefficients of every
        // level: loads first (8 per thread in flight), then the LDS stores
        const int4 b0 = B[0];
        const int w0 = g->L[0].w, p0 = (w0 + 3) & ~3;
        const uint8_t* in = s.in0 + (size_t)f * s.in_fstride;
        const int nr = b0.y - b0.x;
        if (((s.in_stride | (size_t)in | (size_t)w0) & 3) == 0) {
            const int wpr = w0 >> 2, nw = nr * wpr;
            for (int i0 = 0; i0 < nw; i0 += 8 * NT) {
                uint32_t v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int i = i0 + k * NT + tid;
                    const int r = i / wpr, c = i - r * wpr;
                    v[k] = i < nw ? *reinterpret_cast<const uint32_t*>(in + (size_t)(b0.x + r) * s.in_stride + 4 * c)
                                  : 0u;
                }
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int i = i0 + k * NT + tid;
                    const int r = i / wpr, c = i - r * wpr;
                    if (i < nw) *reinterpret_cast<uint32_t*>(pbuf + r * p0 + 4 * c) = v[k];
                }
            }
        } else {
            for (int i = tid; i < nr * w0; i += NT) {
                const int r = i / w0, c = i - r * w0;
                pbuf[r * p0 + c] = in[(size_t)(b0.x + r) * s.in_stride + c];
            }
        }
        const uint4* qg = g->L[1].qcoef;   // the levels' tables are contiguous from level 1 on
        for (int i = tid; i < qtot; i += NT) {
            const uint4 a = qg[2 * i];
            const uint32_t bw = qg[2 * i + 1].x;
            qa[i] = a;
            qb[i] = bw;
        }
        int off = 0;
        for (int l = 1; l < NL; l++) {
            const int4 bl = B[l];
            const int2* rg = g->L[l].rcoef;
            for (int r = tid; r < bl.y - bl.x; r += NT) rcoef[off + r] = rg[bl.x + r];
            off += bl.y - bl.x;
        }
    }
    __syncthreads();
    PYRP(0);
    for (int l = 1; l < NL; l++) {
        const PyrLvl& P = lv[l];
        const uint8_t* src = pbuf + ((l - 1) & 1 ? buf1_off : 0);
        pyr_band_level<NT>(P, src, rcoef + P.rcoff, qa + P.qbase, qb + P.qbase, pbuf + (l & 1 ? buf1_off : 0),
                           l + 1 < NL, tid);
        __syncthreads();
        PYRP(l);
    }
}

// ------------------------------------------------------------------------------------------------ FAST cells
// FAST-9/16 "strength" S = max over the 16 arcs of 9 contiguous circle pixels of min(v-p) (dark circle) or
// min(p-v) (bright circle). A pixel is a FAST corner at threshold t iff S > t, and OpenCV's cornerScore is then
// S-1 (fast_score.cpp: max(t, A, B) - 1), so one S map serves both thresholds.
// Two horizontally adjacent pixels per lane in packed fp16 (every difference of two bytes, -255..255, is exact in
// fp16): the ROI is staged as pixel pairs (p[c], p[c+1]), so one 32-bit LDS read gives a circle sample for both
// pixels, and the arc minima / maxima use gfx950's 3-input packed v_pk_minimum3_f16 / v_pk_maximum3_f16:
// arcs pairwise: max(arcmin[2i], arcmin[2i+1]) = min3(Q[2i+1], Q[2i+5], max(d[2i], d[2i+9])), Q = min of 4 samples.
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

__device__ __forceinline__ half2_t hmin3(half2_t a, half2_t b, half2_t c) {
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ half2_t hmax3(half2_t a, half2_t b, half2_t c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

// S of the pixel pair at inner pair column pc of ROI row r, i.e. pixels (r, 3 + 2pc) and (r, 4 + 2pc)
// (negative = 0). The ROI pixel pairs are split by column parity into planes E (pair at even column 2k) and O
// (odd column 2k + 1), interleaved per row (row = CW pairs of E then CW of O, compile-time pitch: every circle
// sample is one base address + an immediate offset), and consecutive lanes read consecutive words. Column
// 3 + 2pc + dx is E[pc + (3 + dx) / 2] for odd dx, O[pc + (2 + dx) / 2] for even dx.
template <int CW, int DY, int DX>
__device__ __forceinline__ half2_t fast_px(const half2_t* E) {
    if constexpr ((DX & 1) != 0) return E[DY * 2 * CW + (3 + DX) / 2];
    else return E[DY * 2 * CW + CW + (2 + DX) / 2];
}
template <int CW>
__device__ __forceinline__ half2_t fast_strength_h2(const half2_t* hp, int r, int pc) {
    // On the circle samples p_k themselves (no per-sample difference): min over an arc of (v - p) is v - max over the
    // arc of p, so S = max(v - min_k arcmax_p[k], max_k arcmin_p[k] - v). Exact in f16 (integers <= 255).
    const half2_t* E = hp + r * 2 * CW + pc;
    const half2_t v = fast_px<CW, 0, 0>(E);
    half2_t d[16];
    d[0] = fast_px<CW, 3, 0>(E);
    d[1] = fast_px<CW, 3, 1>(E);
    d[2] = fast_px<CW, 2, 2>(E);
    d[3] = fast_px<CW, 1, 3>(E);
    d[4] = fast_px<CW, 0, 3>(E);
    d[5] = fast_px<CW, -1, 3>(E);
    d[6] = fast_px<CW, -2, 2>(E);
    d[7] = fast_px<CW, -3, 1>(E);
    d[8] = fast_px<CW, -3, 0>(E);
    d[9] = fast_px<CW, -3, -1>(E);
    d[10] = fast_px<CW, -2, -2>(E);
    d[11] = fast_px<CW, -1, -3>(E);
    d[12] = fast_px<CW, 0, -3>(E);
    d[13] = fast_px<CW, 1, -3>(E);
    d[14] = fast_px<CW, 2, -2>(E);
    d[15] = fast_px<CW, 3, -1>(E);
    // The arcs starting at 2i and 2i+1 share the 8 samples 2i+1 .. 2i+8 (min M8 = min(Q[2i+1], Q[2i+5]) with Q[j] =
    // min of d[j .. j+3]), so max(arcmin[2i], arcmin[2i+1]) = min3(Q[2i+1], Q[2i+5], max(d[2i], d[2i+9])): eight
    // 3-input ops per direction instead of 32 for the sixteen arcs. Q at the odd starts from the four pair minima
    // P = min(d[4m+3], d[4m+4]): Q[4m+1] = min3(d[4m+1], d[4m+2], P[m]), Q[4m+3] = min3(P[m], d[4m+5], d[4m+6]).
    half2_t qn[8], qx[8];   // qn[i] = Q[2i+1] (min), qx[i] = the same window's max
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const half2_t pn = __builtin_elementwise_minimum(d[(4 * m + 3) & 15], d[(4 * m + 4) & 15]);
        const half2_t px = __builtin_elementwise_maximum(d[(4 * m + 3) & 15], d[(4 * m + 4) & 15]);
        qn[2 * m] = hmin3(d[4 * m + 1], d[4 * m + 2], pn);
        qx[2 * m] = hmax3(d[4 * m + 1], d[4 * m + 2], px);
        qn[2 * m + 1] = hmin3(pn, d[(4 * m + 5) & 15], d[(4 * m + 6) & 15]);
        qx[2 * m + 1] = hmax3(px, d[(4 * m + 5) & 15], d[(4 * m + 6) & 15]);
    }
    half2_t vb[8], va[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const half2_t a = d[2 * i], b = d[(2 * i + 9) & 15];
        vb[i] = hmin3(qn[i], qn[(i + 2) & 7], __builtin_elementwise_maximum(a, b));
        va[i] = hmax3(qx[i], qx[(i + 2) & 7], __builtin_elementwise_minimum(a, b));
    }
    const half2_t Bmax = __builtin_elementwise_maximum(hmax3(vb[0], vb[1], vb[2]),
                                                       hmax3(vb[3], vb[4], hmax3(vb[5], vb[6], vb[7])));
    const half2_t Amin = __builtin_elementwise_minimum(hmin3(va[0], va[1], va[2]),
                                                       hmin3(va[3], va[4], hmin3(va[5], va[6], va[7])));
    return __builtin_elementwise_maximum(v - Amin, Bmax - v);
}

// One workgroup (FAST_THREADS) per cell, everything on pixel pairs (two horizontally adjacent pixels per lane):
// (a) ROI -> LDS as f16 pixel pairs in two column-parity planes (compile-time pitch CW), 4 pairs per thread;
// (b) S of every inner pair into a half2 map with a zero guard ring (the 3-pixel ROI ring is never scored by
//     cv::FAST on the cell ROI, so it reads as 0);
// (c) NMS peak P = S if S > max of its 8 neighbours and S >= 2 (with t >= 1 OpenCV's "score > every neighbour's
//     score-or-0" is exactly S > t && S > max8(S) && S >= 2, for both thresholds), counted per (iteration, wave)
//     at both thresholds by ballot;
// (d) iniThFAST if any P > iniTh, else minThFAST; every wave reads all count entries with broadcast LDS reads;
// (e) corners written in row-major order (pair order = pixel order) at ballot prefix positions.
// Issue/latency-bound per workgroup (PMC: VALU busy ~11 %, a third of the wave cycles waiting, a third issue-stalled;
// the circle test is ~a quarter of the time, staging without global loads is no faster): DESIGN.md §3 / §6.
// One cell (cell_i of frame f) by one workgroup; smem: fast_lds_bytes() of dynamic LDS
template <int CW>
__device__ __forceinline__ void fast_cell_body(const Geom* __restrict__ g, const CellDesc* __restrict__ cells,
                                               const LevelSrc& s, uint32_t* __restrict__ cand,
                                               int* __restrict__ cell_counts, int iniTh, int minTh, int cell_i, int f,
                                               uint8_t* smem) {
    constexpr int T = FAST_THREADS, NW = FAST_THREADS / 64;
    const CellDesc c = cells[cell_i];
    const LevelGeom& L = g->L[c.level];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
#if defined(MAM_FAST_EXPERIMENT) && (MAM_FAST_EXPERIMENT & 4)
    if (tid == 0) cell_counts[(size_t)f * g->cells_per_frame + cell_i] = 0;   // timing experiment only
    return;
#endif
    int pitch;
    const uint8_t* lev = level_ptr(g, s, f, c.level, &pitch);
    const int rows = c.y1 - c.y0, cols = c.x1 - c.x0;
    const int bh = rows - 6, bw = cols - 6;
    const int pw = bw > 0 ? (bw + 1) >> 1 : 0;  // pixel pairs per inner row
    const int np = bh > 0 ? bh * pw : 0;
    constexpr int SC = CW;                      // S map pitch (pairs): pw + 2 <= CW (host-checked)
    // ---- LDS carve (fast_lds_bytes() on the host mirrors it)
    half2_t* hp = reinterpret_cast<half2_t*>(smem);                                // [rows][E: CW | O: CW]
    const int rmax = g->roi_max_rows;
    half2_t* Sh = reinterpret_cast<half2_t*>(smem + fast_off_s(rmax, CW));          // [bh+2][SC]
    uint16_t* pkm = reinterpret_cast<uint16_t*>(smem + fast_off_pk(rmax, CW));      // [np]
    int* cnt = reinterpret_cast<int*>(smem + fast_off_cnt(rmax, CW));               // [it*NW] packed
    const half2_t z = {(_Float16)0, (_Float16)0};
    // (a) stage 4 pairs per thread: bytes c0 .. c0+4 of one ROI row
    {
        const int qc = (cols + 3) >> 2, nq = rows * qc;
        const int dq = T / qc, dr = T - dq * qc;
        int r = tid / qc, q = tid - r * qc;
        const uint8_t* src = lev + (size_t)c.y0 * pitch + c.x0;
#pragma unroll 2
        for (int i = tid; i < nq; i += T) {
            // columns up to 4q + 4 <= cols + 3 stay inside the level row (cells end >= EDGE_THRESHOLD - 3 before
            // its right edge); values past the ROI only reach the discarded ring pixel of odd-width cells.
            // Unconditional loads: all in flight before the first use.
            const uint8_t* pr = src + (size_t)r * pitch + 4 * q;
            uint32_t w4;
            __builtin_memcpy(&w4, pr, 4);
            // byte b as the f16 0x64bb = 1024 + b (exact; the common offset cancels in every difference S takes):
            // one v_perm_b32 per pixel pair instead of per-byte conversions
            const uint32_t b4x = (uint32_t)pr[4] | 0x64646400u;
            constexpr uint32_t K64 = 0x64646464u;
            uint32_t* dE = reinterpret_cast<uint32_t*>(hp + r * 2 * CW + 2 * q);
            uint32_t* dO = dE + CW;
            dE[0] = __builtin_amdgcn_perm(K64, w4, 0x04010400u);   // (b0, b1)
            dO[0] = __builtin_amdgcn_perm(K64, w4, 0x04020401u);   // (b1, b2)
            dE[1] = __builtin_amdgcn_perm(K64, w4, 0x04030402u);   // (b2, b3)
            dO[1] = __builtin_amdgcn_perm(b4x, w4, 0x05040503u);   // (b3, b4)
            r += dq;
            q += dr;
            if (q >= qc) { q -= qc; r++; }
        }
        if (np > 0) {
            for (int i = tid; i < SC; i += T) { Sh[i] = z; Sh[(bh + 1) * SC + i] = z; }
            for (int i = tid; i < bh; i += T) { Sh[(i + 1) * SC] = z; Sh[(i + 1) * SC + pw + 1] = z; }
        }
    }
    __syncthreads();
#if defined(MAM_FAST_EXPERIMENT) && (MAM_FAST_EXPERIMENT & 2)
    // timing only: the count stays 0 (nothing downstream reads a candidate), the value kept live through the
    // cell's first candidate slot
    if (tid == 0) {
        cand[(size_t)f * g->cand_per_frame + L.cand_base + (size_t)c.slot * L.cellcap] = (uint32_t)(int)hp[tid].x;
        cell_counts[(size_t)f * g->cells_per_frame + cell_i] = 0;
    }
    return;
#endif
    const int pwm = max(pw, 1);
    const int dq = T / pwm, dr = T - dq * pwm;
    const int r_start = tid / pwm, p_start = tid - r_start * pwm;
    // (b) strength of every inner pair
    {
        int r = r_start, pc = p_start;
        for (int i = tid; i < np; i += T) {
#if defined(MAM_FAST_EXPERIMENT) && (MAM_FAST_EXPERIMENT & 1)
            half2_t S2 = hp[(r + 3) * 2 * CW + pc] - hp[(r + 3) * 2 * CW + CW + pc + 1];   // timing experiment only
#else
            half2_t S2 = fast_strength_h2<CW>(hp, r + 3, pc);
#endif
            S2 = __builtin_elementwise_maximum(S2, z);
            if (2 * pc + 1 >= bw) S2.y = (_Float16)0;   // odd width: the pair's second pixel is ring
            Sh[(r + 1) * SC + pc + 1] = S2;
            r += dq;
            pc += dr;
            if (pc >= pw) { pc -= pw; r++; }
        }
    }
    __syncthreads();
#if defined(MAM_FAST_EXPERIMENT) && (MAM_FAST_EXPERIMENT & 16)
    if (tid == 0) {   // timing only: up to S (count 0, the value kept live through the cell's first slot)
        cand[(size_t)f * g->cand_per_frame + L.cand_base + (size_t)c.slot * L.cellcap] = (uint32_t)(int)Sh[tid].x;
        cell_counts[(size_t)f * g->cells_per_frame + cell_i] = 0;
    }
    return;
#endif
    const int tlo = max(iniTh, 1), thi = max(minTh, 1);
    const int iters = (np + T - 1) / T;
    // (c) NMS peaks + per-(iteration, wave) counts at both thresholds, packed (hi << 16) | lo
    {
        int r = r_start, pc = p_start;
        for (int j = 0; j < iters; j++) {
            const int i = j * T + tid;
            int pk0 = 0, pk1 = 0;
            if (i < np) {
                const half2_t* q = Sh + (r + 1) * SC + pc + 1;
                const half2_t UL = q[-SC - 1], U = q[-SC], UR = q[-SC + 1];
                const half2_t ML = q[-1], M = q[0], MR = q[1];
                const half2_t DL = q[SC - 1], D = q[SC], DR = q[SC + 1];
                const half2_t up = hmax3(__builtin_shufflevector(UL, U, 1, 2), U, __builtin_shufflevector(U, UR, 1, 2));
                const half2_t dn = hmax3(__builtin_shufflevector(DL, D, 1, 2), D, __builtin_shufflevector(D, DR, 1, 2));
                const half2_t md = __builtin_elementwise_maximum(__builtin_shufflevector(ML, M, 1, 2),
                                                                 __builtin_shufflevector(M, MR, 1, 2));
                const half2_t m8 = hmax3(up, dn, md);
                pk0 = (M.x > m8.x && M.x >= (_Float16)2) ? (int)M.x : 0;
                pk1 = (M.y > m8.y && M.y >= (_Float16)2) ? (int)M.y : 0;
                pkm[i] = (uint16_t)(pk0 | (pk1 << 8));
                r += dq;
                pc += dr;
                if (pc >= pw) { pc -= pw; r++; }
            }
            const int chi = __popcll(__ballot(pk0 > tlo)) + __popcll(__ballot(pk1 > tlo));
            const int clo = __popcll(__ballot(pk0 > thi)) + __popcll(__ballot(pk1 > thi));
            if (lane == 0) cnt[j * NW + w] = (chi << 16) | clo;
        }
    }
    __syncthreads();
#if defined(MAM_FAST_EXPERIMENT) && (MAM_FAST_EXPERIMENT & 8)
    if (tid == 0) {   // timing only: up to NMS + counts (count 0, the value kept live through the cell's first slot)
        cand[(size_t)f * g->cand_per_frame + L.cand_base + (size_t)c.slot * L.cellcap] = (uint32_t)cnt[0];
        cell_counts[(size_t)f * g->cells_per_frame + cell_i] = 0;
    }
    return;
#endif
    // (d) cell totals and this wave's bases: every lane reads the entries (same address: LDS broadcast)
    int tot = 0, mybase_first = 0;
    const int nent = iters * NW;
    for (int e = 0; e < nent; e++) {
        const int v = cnt[e];
        if (e == w) mybase_first = tot;
        tot += v;
    }
    const int tot_hi = tot >> 16, tot_lo = tot & 0xFFFF;
    const bool use_hi = tot_hi > 0;
    const int th = use_hi ? tlo : thi;
    // (e) ordered emit; the base of entry (j, w) = base(j-1, w) + entries (j-1, w+1 .. NW-1) + (j, 0 .. w-1)
    uint32_t* out = cand + (size_t)f * g->cand_per_frame + L.cand_base + (size_t)c.slot * L.cellcap;
    {
        int r = r_start, pc = p_start;
        const uint64_t below = (1ull << lane) - 1ull;
        int basep = mybase_first;
        for (int j = 0; j < iters; j++) {
            if (j > 0) {
                for (int e = (j - 1) * NW + w; e < j * NW + w; e++) basep += cnt[e];
            }
            const int i = j * T + tid;
            int pk0 = 0, pk1 = 0;
            if (i < np) {
                const int v = pkm[i];
                pk0 = v & 0xFF;
                pk1 = v >> 8;
            }
            const bool f0 = pk0 > th, f1 = pk1 > th;
            const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
            int pos = (use_hi ? basep >> 16 : basep & 0xFFFF) + __popcll(m0 & below) + __popcll(m1 & below);
            if (i < np) {
                const uint32_t x = (uint32_t)(3 + 2 * pc + c.cj * L.wCell);
                const uint32_t y = (uint32_t)(r + 3 + c.ci * L.hCell);
                if (f0) out[pos++] = x | (y << 12) | ((uint32_t)(pk0 - 1) << 24);
                if (f1) out[pos] = (x + 1) | (y << 12) | ((uint32_t)(pk1 - 1) << 24);
                r += dq;
                pc += dr;
                if (pc >= pw) { pc -= pw; r++; }
            }
        }
    }
    if (tid == 0) cell_counts[(size_t)f * g->cells_per_frame + cell_i] = use_hi ? tot_hi : tot_lo;
}

#ifndef MAM_FAST_XCD
#define MAM_FAST_XCD 1
#endif
template <int CW>
__global__ __launch_bounds__(FAST_THREADS) void k_fast_cells(const Geom* __restrict__ g,
                                                             const CellDesc* __restrict__ cells, LevelSrc s,
                                                             uint32_t* __restrict__ cand,
                                                             int* __restrict__ cell_counts, int iniTh, int minTh,
                                                             int cell_first) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // XCD-aware order (as k_blur7): each XCD works a contiguous range of (frame, cell) ids, so the ROI rows adjacent
    // cells share (6-pixel overlaps, 128-byte lines spanning ~4 cells) are fetched into one L2 instead of up to four
    int cell_i = blockIdx.x, f = blockIdx.y;
    if (MAM_FAST_XCD) {
        const int logical = xcd_logical(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
        f = logical / gridDim.x;
        cell_i = logical - f * gridDim.x;
    }
    cell_i += cell_first;   // a launch over the cells [cell_first, cell_first + gridDim.x) of every frame
    fast_cell_body<CW>(g, cells, s, cand, cell_counts, iniTh, minTh, cell_i, f, smem);
}

// ---- FAST over chunks of a cell row (the band formulation): one workgroup per (frame, chunk of up to FAST_G
// consecutive cells of one cell row). The cells of a row share their ROI rows and their detection columns tile the
// row, so the chunk stages its ROI once (the cells' 6-pixel overlaps read once), computes the strength of every
// pixel once, then per cell: NMS with the neighbours outside the cell's detection area as 0 (cv::FAST on the cell
// ROI scores nothing outside it), the iniThFAST / minThFAST choice from the cell's counts and the cell's candidates
// in row-major order into its own slots — exactly k_fast_cells' outputs.
constexpr int FAST_G = 4;
struct ChunkDesc {
    int level;
    int cell0, ncell;   // first cell (index into the frame's cell table) and cells in the chunk (<= FAST_G)
    int x0, y0, x1, y1; // ROI: the first cell's x0 .. the last cell's x1, the row's y0 .. y1
    int ci, cj0;        // cell row, column of the first cell
};
__host__ __device__ inline size_t fastc_off_s(int rmax, int cw) { return fast_align16((size_t)rmax * 2 * cw * 4); }
__host__ __device__ inline size_t fastc_off_pk(int rmax, int cw) {
    return fastc_off_s(rmax, cw) + fast_align16((size_t)(rmax - 4) * cw * 4);
}
__host__ __device__ inline int fastc_max_entries(int rmax, int cw) {
    const int np = (rmax - 6) * (cw - 2);
    return (np + FAST_THREADS - 1) / FAST_THREADS * (FAST_THREADS / 64) * FAST_G;
}
__host__ __device__ inline size_t fastc_off_cnt(int rmax, int cw) {
    return fastc_off_pk(rmax, cw) + fast_align16((size_t)(rmax - 6) * cw * 2);
}
__host__ __device__ inline size_t fastc_lds_bytes(int rmax, int cw) {
    return fastc_off_cnt(rmax, cw) + (size_t)fastc_max_entries(rmax, cw) * 4;
}

template <int CW>
__global__ __launch_bounds__(FAST_THREADS) void k_fast_chunks(const Geom* __restrict__ g,
                                                              const ChunkDesc* __restrict__ chunks,
                                                              const CellDesc* __restrict__ cells, LevelSrc s,
                                                              uint32_t* __restrict__ cand,
                                                              int* __restrict__ cell_counts, int iniTh, int minTh,
                                                              int chunk_first) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int T = FAST_THREADS, NW = FAST_THREADS / 64;
    int ch_i = blockIdx.x, f = blockIdx.y;
    {
        const int logical = xcd_logical(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
        f = logical / gridDim.x;
        ch_i = logical - f * gridDim.x;
    }
    const ChunkDesc c = chunks[chunk_first + ch_i];
    const LevelGeom& L = g->L[c.level];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    int pitch;
    const uint8_t* lev = level_ptr(g, s, f, c.level, &pitch);
    const int rows = c.y1 - c.y0, cols = c.x1 - c.x0;
    const int bh = rows - 6, bw = cols - 6;
    const int pw = bw > 0 ? (bw + 1) >> 1 : 0;
    const int np = bh > 0 ? bh * pw : 0;
    const int wc = L.wCell, G = c.ncell;
    constexpr int SC = CW;
    half2_t* hp = reinterpret_cast<half2_t*>(smem);
    const int rmax = g->roi_max_rows;
    half2_t* Sh = reinterpret_cast<half2_t*>(smem + fastc_off_s(rmax, CW));
    uint16_t* pkm = reinterpret_cast<uint16_t*>(smem + fastc_off_pk(rmax, CW));
    int* cnt = reinterpret_cast<int*>(smem + fastc_off_cnt(rmax, CW));
    const half2_t z = {(_Float16)0, (_Float16)0};
    // (a) stage the chunk ROI as f16 pixel pairs (k_fast_cells' staging)
    {
        const int qc = (cols + 3) >> 2, nq = rows * qc;
        const int dq = T / qc, dr = T - dq * qc;
        int r = tid / qc, q = tid - r * qc;
        const uint8_t* src = lev + (size_t)c.y0 * pitch + c.x0;
#pragma unroll 2
        for (int i = tid; i < nq; i += T) {
            const uint8_t* pr = src + (size_t)r * pitch + 4 * q;
            uint32_t w4;
            __builtin_memcpy(&w4, pr, 4);
            const uint32_t b4x = (uint32_t)pr[4] | 0x64646400u;
            constexpr uint32_t K64 = 0x64646464u;
            uint32_t* dE = reinterpret_cast<uint32_t*>(hp + r * 2 * CW + 2 * q);
            uint32_t* dO = dE + CW;
            dE[0] = __builtin_amdgcn_perm(K64, w4, 0x04010400u);
            dO[0] = __builtin_amdgcn_perm(K64, w4, 0x04020401u);
            dE[1] = __builtin_amdgcn_perm(K64, w4, 0x04030402u);
            dO[1] = __builtin_amdgcn_perm(b4x, w4, 0x05040503u);
            r += dq;
            q += dr;
            if (q >= qc) { q -= qc; r++; }
        }
        if (np > 0) {
            for (int i = tid; i < SC; i += T) { Sh[i] = z; Sh[(bh + 1) * SC + i] = z; }
            for (int i = tid; i < bh; i += T) { Sh[(i + 1) * SC] = z; Sh[(i + 1) * SC + pw + 1] = z; }
        }
    }
    __syncthreads();
    const int pwm = max(pw, 1);
    const int dq = T / pwm, dr = T - dq * pwm;
    const int r_start = tid / pwm, p_start = tid - r_start * pwm;
    // (b) strength of every inner pair of the chunk, once
    {
        int r = r_start, pc = p_start;
        for (int i = tid; i < np; i += T) {
            half2_t S2 = fast_strength_h2<CW>(hp, r + 3, pc);
            S2 = __builtin_elementwise_maximum(S2, z);
            if (2 * pc + 1 >= bw) S2.y = (_Float16)0;
            Sh[(r + 1) * SC + pc + 1] = S2;
            r += dq;
            pc += dr;
            if (pc >= pw) { pc -= pw; r++; }
        }
    }
    __syncthreads();
    const int tlo = max(iniTh, 1), thi = max(minTh, 1);
    const int iters = (np + T - 1) / T;
    // the cell (within the chunk) of inner column ic, and whether ic is its cell's first / last detection column
    auto cell_of = [&](int ic) { return min(ic / wc, G - 1); };
    // (c) NMS peaks with the neighbours of other cells masked; per (iteration, wave, cell) counts at both thresholds
    {
        int r = r_start, pc = p_start;
        for (int j = 0; j < iters; j++) {
            const int i = j * T + tid;
            int pk0 = 0, pk1 = 0, k0 = 0, k1 = 0;
            if (i < np) {
                const half2_t* q = Sh + (r + 1) * SC + pc + 1;
                const int ic0 = 2 * pc, ic1 = 2 * pc + 1;
                k0 = cell_of(ic0);
                k1 = cell_of(ic1);
                // neighbour columns of pixel ic0: ic0 - 1 (pair pc - 1's .y) and ic1 (this pair's .y); of ic1: ic0
                // (this .x) and ic1 + 1 (pair pc + 1's .x). A neighbour in another cell reads as 0.
                const bool l0 = ic0 > 0 && cell_of(ic0 - 1) == k0, r0 = k1 == k0;
                const bool l1 = k0 == k1, r1 = ic1 + 1 < bw && cell_of(ic1 + 1) == k1;
                const half2_t UL = q[-SC - 1], U = q[-SC], UR = q[-SC + 1];
                const half2_t ML = q[-1], M = q[0], MR = q[1];
                const half2_t DL = q[SC - 1], D = q[SC], DR = q[SC + 1];
                const _Float16 zf = (_Float16)0;
                // pixel 0: columns ic0 - 1 (UL.y, ML.y, DL.y), ic0 (U.x, D.x), ic1 (U.y, M.y, D.y)
                const _Float16 a0 = l0 ? __builtin_elementwise_maximum(UL.y, __builtin_elementwise_maximum(ML.y, DL.y)) : zf;
                const _Float16 b0 = __builtin_elementwise_maximum(U.x, D.x);
                const _Float16 c0 = r0 ? __builtin_elementwise_maximum(U.y, __builtin_elementwise_maximum(M.y, D.y)) : zf;
                const _Float16 m0 = __builtin_elementwise_maximum(a0, __builtin_elementwise_maximum(b0, c0));
                // pixel 1: columns ic0 (U.x, M.x, D.x), ic1 (U.y, D.y), ic1 + 1 (UR.x, MR.x, DR.x)
                const _Float16 a1 = l1 ? __builtin_elementwise_maximum(U.x, __builtin_elementwise_maximum(M.x, D.x)) : zf;
                const _Float16 b1 = __builtin_elementwise_maximum(U.y, D.y);
                const _Float16 c1 = r1 ? __builtin_elementwise_maximum(UR.x, __builtin_elementwise_maximum(MR.x, DR.x)) : zf;
                const _Float16 m1 = __builtin_elementwise_maximum(a1, __builtin_elementwise_maximum(b1, c1));
                pk0 = (M.x > m0 && M.x >= (_Float16)2) ? (int)M.x : 0;
                pk1 = (M.y > m1 && M.y >= (_Float16)2) ? (int)M.y : 0;
                pkm[i] = (uint16_t)(pk0 | (pk1 << 8));
                r += dq;
                pc += dr;
                if (pc >= pw) { pc -= pw; r++; }
            }
            for (int k = 0; k < G; k++) {
                const int chi = __popcll(__ballot(k0 == k && pk0 > tlo)) + __popcll(__ballot(k1 == k && pk1 > tlo));
                const int clo = __popcll(__ballot(k0 == k && pk0 > thi)) + __popcll(__ballot(k1 == k && pk1 > thi));
                if (lane == 0) cnt[(j * NW + w) * FAST_G + k] = (chi << 16) | clo;
            }
        }
    }
    __syncthreads();
    // (d) per cell: totals, the threshold, this wave's first-entry bases
    int tot[FAST_G], base[FAST_G];
    const int nent = iters * NW;
#pragma unroll
    for (int k = 0; k < FAST_G; k++) { tot[k] = 0; base[k] = 0; }
    for (int e = 0; e < nent; e++) {
#pragma unroll
        for (int k = 0; k < FAST_G; k++) {
            const int v = k < G ? cnt[e * FAST_G + k] : 0;
            if (e == w) base[k] = tot[k];
            tot[k] += v;
        }
    }
    bool use_hi[FAST_G];
#pragma unroll
    for (int k = 0; k < FAST_G; k++) use_hi[k] = (tot[k] >> 16) > 0;
    // (e) ordered emit per cell: in the chunk's row-major pair order each cell's pixels keep their row-major order
    {
        int r = r_start, pc = p_start;
        const uint64_t below = (1ull << lane) - 1ull;
        const int xbase = 3 + c.cj0 * wc;
        for (int j = 0; j < iters; j++) {
            if (j > 0) {
                for (int e = (j - 1) * NW + w; e < j * NW + w; e++)
#pragma unroll
                    for (int k = 0; k < FAST_G; k++) base[k] += k < G ? cnt[e * FAST_G + k] : 0;
            }
            const int i = j * T + tid;
            int pk0 = 0, pk1 = 0, k0 = 0, k1 = 0;
            if (i < np) {
                const int v = pkm[i];
                pk0 = v & 0xFF;
                pk1 = v >> 8;
                k0 = cell_of(2 * pc);
                k1 = cell_of(2 * pc + 1);
            }
            int th0 = thi, th1 = thi, b0 = 0, b1 = 0;
#pragma unroll
            for (int k = 0; k < FAST_G; k++) {
                const int th = use_hi[k] ? tlo : thi;
                const int bk = use_hi[k] ? base[k] >> 16 : base[k] & 0xFFFF;
                if (k == k0) { th0 = th; b0 = bk; }
                if (k == k1) { th1 = th; b1 = bk; }
            }
            const bool f0 = i < np && pk0 > th0, f1 = i < np && pk1 > th1;
            int pos0 = b0, pos1 = b1 + ((f0 && k0 == k1) ? 1 : 0);
#pragma unroll
            for (int k = 0; k < FAST_G; k++) {
                const uint64_t m0 = __ballot(f0 && k0 == k), m1 = __ballot(f1 && k1 == k);
                const int before = __popcll(m0 & below) + __popcll(m1 & below);
                if (k == k0) pos0 += before;
                if (k == k1) pos1 += before;
            }
            if (i < np) {
                const uint32_t x = (uint32_t)(xbase + 2 * pc);
                const uint32_t y = (uint32_t)(r + 3 + c.ci * L.hCell);
                if (f0) {
                    uint32_t* out = cand + (size_t)f * g->cand_per_frame + L.cand_base + (size_t)cells[c.cell0 + k0].slot * L.cellcap;
                    out[pos0] = x | (y << 12) | ((uint32_t)(pk0 - 1) << 24);
                }
                if (f1) {
                    uint32_t* out = cand + (size_t)f * g->cand_per_frame + L.cand_base + (size_t)cells[c.cell0 + k1].slot * L.cellcap;
                    out[pos1] = (x + 1) | (y << 12) | ((uint32_t)(pk1 - 1) << 24);
                }
                r += dq;
                pc += dr;
                if (pc >= pw) { pc -= pw; r++; }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < FAST_G; k++)
        if (tid == k && k < G)
            cell_counts[(size_t)f * g->cells_per_frame + c.cell0 + k] = use_hi[k] ? tot[k] >> 16 : tot[k] & 0xFFFF;
}

// ------------------------------------------------------------------------------------------------ blur
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 u16_pair(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi, lo, sel));
}

__device__ __forceinline__ int refl101(int p, int n) {
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}
// BORDER_REFLECT_101 for -(n - 1) <= p <= 2n - 2 (one reflection), branch-free
__device__ __forceinline__ int refl101_1(int p, int n) {
    p = p < 0 ? -p : p;
    return p >= n ? 2 * n - 2 - p : p;
}

// Tile of BLUR_TILE_W x BLUR_TILE_H outputs. Input staged in LDS as bytes (rows y0-3 .. y0+H+2, cols x0-4 ..
// x0+W+3); interior tiles load aligned 32-bit words, border tiles reflect per byte (BORDER_REFLECT_101).
// Horizontal pass: 4 outputs per thread from 12 staged bytes -> u16 sums in LDS; vertical pass: 4 outputs per
// thread from 7 x 4 u16 -> one 32-bit store. Integer arithmetic exactly as the fixed-point separable filter.
constexpr int BLUR_IN_W = BLUR_TILE_W + 8;   // staged columns (x0-4 .. x0+W+3), multiple of 4
constexpr int BLUR_IN_H = BLUR_TILE_H + 6;

// Geometry of blur tile `tile` (frame-local index over every level)
struct BlurTile {
    const uint8_t* lev;
    int pitch, l, x0, y0, w, h;
    bool aligned;
};
__device__ __forceinline__ BlurTile blur_tile(const Geom* g, const LevelSrc& s, int f, int tile) {
    BlurTile t;
    t.l = 0;
    for (int i = 1; i < g->nlevels; i++)
        if (tile >= g->L[i].tile_base) t.l = i;
    const LevelGeom& L = g->L[t.l];
    tile -= L.tile_base;
    t.x0 = (tile % L.tiles_x) * BLUR_TILE_W;
    t.y0 = (tile / L.tiles_x) * BLUR_TILE_H;
    t.lev = level_ptr(g, s, f, t.l, &t.pitch);
    t.w = L.w;
    t.h = L.h;
    t.aligned = ((t.pitch | (int)((uintptr_t)t.lev & 3)) & 3) == 0;
    return t;
}

constexpr int BLUR_WPR = BLUR_IN_W / 4;
constexpr int BLUR_NWORDS = BLUR_IN_H * BLUR_WPR, BLUR_NIT = (BLUR_NWORDS + 255) / 256;

// Staged words of tile t into registers. Every word whose 4 columns lie inside the row is one aligned 32-bit load
// (row reflected per word); only the words straddling or past the left/right edge reflect per byte.
template <bool ONE_REFL>
__device__ __forceinline__ void blur_fetch_t(const BlurTile& t, int tid, uint32_t (&v)[BLUR_NIT]) {
#pragma unroll
    for (int k = 0; k < BLUR_NIT; k++) {
        const int i = k * 256 + tid;
        const int r = i / BLUR_WPR, c = i - r * BLUR_WPR;
        uint32_t word = 0u;
        if (i < BLUR_NWORDS) {
            const int y = t.y0 - 3 + r;
            const uint8_t* row = t.lev + (size_t)(ONE_REFL ? refl101_1(y, t.h) : refl101(y, t.h)) * t.pitch;
            const int gx = t.x0 - 4 + 4 * c;
            if (t.aligned && gx >= 0 && gx + 4 <= t.w) {
                word = *reinterpret_cast<const uint32_t*>(row + gx);
            } else {
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int x = min(gx + b, 2 * t.w - 2);
                    word |= (uint32_t)row[ONE_REFL ? refl101_1(x, t.w) : refl101(x, t.w)] << (8 * b);
                }
            }
        }
        v[k] = word;
    }
}
// Staged rows span [y0 - 3, y0 + BLUR_IN_H - 4] with y0 <= h - 1, staged columns [-4, 2w - 2] after the clamp: one
// reflection is enough when h >= BLUR_IN_H - 2 and w >= 5 (every level of the benchmark sizes); the general loop
// otherwise. The choice is uniform over the workgroup.
__device__ __forceinline__ void blur_fetch(const BlurTile& t, int tid, uint32_t (&v)[BLUR_NIT]) {
    if (t.h >= BLUR_IN_H - 2 && t.w >= 5) blur_fetch_t<true>(t, tid, v);
    else blur_fetch_t<false>(t, tid, v);
}

// Workgroup = BLUR_TPB consecutive tiles of one frame (possibly of different levels), software-pipelined: the next
// tile's words are loaded into registers while this tile's horizontal and vertical passes run, so the load latency
// of a tile is hidden behind the previous one's arithmetic.
constexpr size_t BLUR_LDS_BYTES = ((size_t)BLUR_IN_H * BLUR_IN_W + 15) / 16 * 16 + (size_t)BLUR_IN_H * BLUR_TILE_W * 2;
// Tile group `grp` (BLUR_TPB consecutive tiles) of frame f; tin / th_: the staged bytes and the horizontal sums (LDS)
__device__ __forceinline__ void blur_group_body(const Geom* __restrict__ g, const LevelSrc& s,
                                                uint8_t* __restrict__ blur, int f, int grp,
                                                uint8_t (*tin)[BLUR_IN_W], uint16_t (*th_)[BLUR_TILE_W]) {
    const int tid = threadIdx.x;
    const int tile0 = grp * BLUR_TPB;
    const int ntiles = min(BLUR_TPB, g->tiles_per_frame - tile0);
    uint32_t v[BLUR_NIT];
    BlurTile t = blur_tile(g, s, f, tile0);
    blur_fetch(t, tid, v);
    for (int j = 0; j < ntiles; j++) {
#pragma unroll
        for (int k = 0; k < BLUR_NIT; k++) {
            const int i = k * 256 + tid;
            const int r = i / BLUR_WPR, c = i - r * BLUR_WPR;
            if (i < BLUR_NWORDS) *reinterpret_cast<uint32_t*>(&tin[r][4 * c]) = v[k];
        }
        __syncthreads();   // tin complete; every thread is past the previous tile's vertical pass (th_ free)
        const LevelGeom& L = g->L[t.l];
        const int x0 = t.x0, y0 = t.y0, w = t.w, h = t.h;
        if (j + 1 < ntiles) {
            t = blur_tile(g, s, f, tile0 + j + 1);
            blur_fetch(t, tid, v);   // in flight during this tile's passes
        }
        // horizontal: output column x0+4q+k uses staged columns 4q+k+1 .. 4q+k+7
        constexpr int QPR = BLUR_TILE_W / 4;
        for (int i = tid; i < BLUR_IN_H * QPR; i += 256) {
            const int r = i / QPR, q = i - r * QPR;
            if (x0 + 4 * q >= w) continue;   // quad past the level's right edge: no output reads it
            const uint32_t wa = *reinterpret_cast<const uint32_t*>(&tin[r][4 * q]);
            const uint32_t wb = *reinterpret_cast<const uint32_t*>(&tin[r][4 * q + 4]);
            const uint32_t wc = *reinterpret_cast<const uint32_t*>(&tin[r][4 * q + 8]);
            // two outputs per packed u16 op: P_j = (p_j, p_j+1) by one v_perm_b32 each (selector 0x0c = a zero byte);
            // every partial sum stays <= 255 * 256 (fits 16 bits exactly)
            const u16x2 P1 = u16_pair(0u, wa, 0x0c020c01u), P2 = u16_pair(0u, wa, 0x0c030c02u);
            const u16x2 P3 = u16_pair(wb, wa, 0x0c040c03u), P4 = u16_pair(0u, wb, 0x0c010c00u);
            const u16x2 P5 = u16_pair(0u, wb, 0x0c020c01u), P6 = u16_pair(0u, wb, 0x0c030c02u);
            const u16x2 P7 = u16_pair(wc, wb, 0x0c040c03u), P8 = u16_pair(0u, wc, 0x0c010c00u);
            const u16x2 P9 = u16_pair(0u, wc, 0x0c020c01u);
            const u16x2 c0 = (u16x2)(unsigned short)GT0, c1 = (u16x2)(unsigned short)GT1;
            const u16x2 c2 = (u16x2)(unsigned short)GT2, c3 = (u16x2)(unsigned short)GT3;
            const u16x2 o01 = c0 * (P1 + P7) + c1 * (P2 + P6) + c2 * (P3 + P5) + c3 * P4;
            const u16x2 o23 = c0 * (P3 + P9) + c1 * (P4 + P8) + c2 * (P5 + P7) + c3 * P6;
            uint2 packed;
            packed.x = __builtin_bit_cast(uint32_t, o01);
            packed.y = __builtin_bit_cast(uint32_t, o23);
            *reinterpret_cast<uint2*>(&th_[r][4 * q]) = packed;
        }
        __syncthreads();
        uint8_t* out = blur + L.blur_off + (size_t)f * L.frame_bytes;
        // vertical: thread = one 4-column quad x BLUR_VR consecutive output rows; the BLUR_VR + 6 staged u16 rows it needs
        // are read once (sliding window) instead of 7 per output row
#ifndef MAM_BLUR_VR
#define MAM_BLUR_VR 4
#endif
        constexpr int BLUR_VR = MAM_BLUR_VR;
        static_assert(BLUR_TILE_H % BLUR_VR == 0, "row groups");
        for (int i = tid; i < (BLUR_TILE_H / BLUR_VR) * QPR; i += 256) {
            const int rg = i / QPR, q = i - rg * QPR;
            const int r = rg * BLUR_VR, x = x0 + 4 * q;
            if (y0 + r >= h || x >= w) continue;
            uint32_t col[BLUR_VR + 6][4];
    #pragma unroll
            for (int k = 0; k < BLUR_VR + 6; k++) {
                const uint2 v = *reinterpret_cast<const uint2*>(&th_[r + k][4 * q]);
                col[k][0] = v.x & 0xFFFF; col[k][1] = v.x >> 16; col[k][2] = v.y & 0xFFFF; col[k][3] = v.y >> 16;
            }
    #pragma unroll
            for (int rr = 0; rr < BLUR_VR; rr++) {
                const int y = y0 + r + rr;
                if (y >= h) break;
                uint32_t packed = 0;
    #pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t sum = GT0 * (col[rr][c] + col[rr + 6][c]) + GT1 * (col[rr + 1][c] + col[rr + 5][c]) +
                                         GT2 * (col[rr + 2][c] + col[rr + 4][c]) + GT3 * col[rr + 3][c];
                    const uint32_t v = (sum + 32768u) >> 16;
                    packed |= (v > 255u ? 255u : v) << (8 * c);
                }
                uint8_t* o = out + (size_t)y * L.pitch + x;
                if (x + 4 <= w) *reinterpret_cast<uint32_t*>(o) = packed;
                else
                    for (int c = 0; c < 4 && x + c < w; c++) o[c] = (uint8_t)(packed >> (8 * c));
            }
        }
    }
}

#ifndef MAM_BLUR_XCD
#define MAM_BLUR_XCD 1
#endif
// XCD-aware order: the hardware deals linear block ids round-robin over the 8 XCDs; remap them (bijectively, any grid
// size) so each XCD works a contiguous range of (frame, tile) ids, putting vertically adjacent tiles, whose staged halo
// rows overlap, on the same L2
__device__ __forceinline__ int blur_xcd_logical(int lin, int nlin) {
    if (!MAM_BLUR_XCD) return lin;
    const int q = nlin >> 3, rem = nlin & 7, x = lin & 7, k = lin >> 3;
    return x < rem ? x * (q + 1) + k : rem * (q + 1) + (x - rem) * q + k;
}
__global__ __launch_bounds__(256) void k_blur7(const Geom* __restrict__ g, LevelSrc s, uint8_t* __restrict__ blur) {
    __shared__ __attribute__((aligned(16))) uint8_t tin[BLUR_IN_H][BLUR_IN_W];
    __shared__ __attribute__((aligned(16))) uint16_t th_[BLUR_IN_H][BLUR_TILE_W];
    const int logical = blur_xcd_logical(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    const int f = logical / gridDim.x;
    blur_group_body(g, s, blur, f, logical - f * gridDim.x, tin, th_);
}

// Latency mode (a few frames): FAST over cells [cell_first, cell_first + ncells) and the blur of every level in ONE
// launch — blocks [0, ncells) of a frame row take a cell, blocks [ncells, ncells + ngroups) a blur tile group. Both
// stages read only the pyramid, so the blur runs beside FAST instead of in its own launch (one dependent launch less
// on the extraction's critical path). Dynamic LDS: max(fast_lds_bytes, BLUR_LDS_BYTES).
template <int CW>
__global__ __launch_bounds__(FAST_THREADS) void k_fast_blur(const Geom* __restrict__ g,
                                                            const CellDesc* __restrict__ cells, LevelSrc s,
                                                            uint32_t* __restrict__ cand, int* __restrict__ cell_counts,
                                                            int iniTh, int minTh, int cell_first, int ncells,
                                                            uint8_t* __restrict__ blur) {
    static_assert(FAST_THREADS == 256, "the blur tile group takes 256 threads");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int f = blockIdx.y;
    if ((int)blockIdx.x < ncells) {
        fast_cell_body<CW>(g, cells, s, cand, cell_counts, iniTh, minTh, cell_first + (int)blockIdx.x, f, smem);
    } else {
        blur_group_body(g, s, blur, f, (int)blockIdx.x - ncells, reinterpret_cast<uint8_t (*)[BLUR_IN_W]>(smem),
                        reinterpret_cast<uint16_t (*)[BLUR_TILE_W]>(
                            smem + ((size_t)BLUR_IN_H * BLUR_IN_W + 15) / 16 * 16));
    }
}

// ------------------------------------------------------------------------------------------------ distribute
// LDS-resident node table in LIST ORDER (node id == list position). Each round rebuilds the list:
// reference semantics (ORBextractor.cc:605-748): children are push_front'ed in creation order and the
// parent erased, so the new list = reverse(creation sequence) ++ (unexpanded nodes in order).
struct NodeBuf {
    uint16_t* x0;
    uint16_t* y0;
    uint16_t* x1;
    uint16_t* y1;
    uint32_t* cnt;
};

__device__ __forceinline__ int quad_of(const NodeBuf& A, int p, uint32_t key) {
    const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
    const int hx = (A.x1[p] - A.x0[p] + 1) >> 1;  // ceil((UR.x-UL.x)/2.f)
    const int hy = (A.y1[p] - A.y0[p] + 1) >> 1;
    const bool left = x < A.x0[p] + hx, top = y < A.y0[p] + hy;
    return left ? (top ? 0 : 2) : (top ? 1 : 3);
}

__device__ __forceinline__ void child_rect(const NodeBuf& A, int p, int q, int* x0, int* y0, int* x1, int* y1) {
    const int ax0 = A.x0[p], ay0 = A.y0[p], ax1 = A.x1[p], ay1 = A.y1[p];
    const int hx = (ax1 - ax0 + 1) >> 1, hy = (ay1 - ay0 + 1) >> 1;
    *x0 = (q & 1) ? ax0 + hx : ax0;
    *x1 = (q & 1) ? ax1 : ax0 + hx;
    *y0 = (q & 2) ? ay0 + hy : ay0;
    *y1 = (q & 2) ? ay1 : ay0 + hy;
}

#ifdef MAM_DIST_PROFILE
__device__ unsigned long long g_dprof[8];
#define DPROF(k) do { __syncthreads(); if (tid == 0) { const long long tn = clock64(); atomicAdd(&g_dprof[k], (unsigned long long)(tn - dp0)); dp0 = tn; } } while (0)
#else
#define DPROF(k) do {} while (0)
#endif

// LDSK: the level's candidate keys (K) and their node ids (KN) live in LDS (kcap entries); every pass over the
// candidates is then an LDS pass instead of a chain of global-memory round trips. Returns false (before any side
// effect) when the level has more than kcap candidates: the caller reruns it with K/KN in global scratch.
template <bool LDSK>
__device__ __forceinline__ bool distribute_impl(uint8_t* smem, const Geom* __restrict__ g,
                                                const int* __restrict__ cell_counts,
                                                const uint32_t* __restrict__ cand, uint32_t* __restrict__ keys,
                                                uint16_t* __restrict__ knode, uint32_t* __restrict__ out_key,
                                                uint32_t* __restrict__ out_rank, int* __restrict__ lvl_counts,
                                                int lap0, int lap1, int kcap) {
    const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const LevelGeom& L = g->L[l];
    const int NC = g->node_cap;
    // ---- LDS carve (all offsets multiples of 16 B)
    uint8_t* p8 = smem;
    auto take = [&](size_t bytes) { uint8_t* r = p8; p8 += (bytes + 15) & ~(size_t)15; return r; };
    // the two node tables as two named structs selected by value (a dynamically indexed array of pointer structs
    // would live in scratch memory: a global-memory round trip per access)
    NodeBuf nb0, nb1;
    for (int b = 0; b < 2; b++) {
        NodeBuf& t = b ? nb1 : nb0;
        t.x0 = (uint16_t*)take(NC * 2);
        t.y0 = (uint16_t*)take(NC * 2);
        t.x1 = (uint16_t*)take(NC * 2);
        t.y1 = (uint16_t*)take(NC * 2);
        t.cnt = (uint32_t*)take(NC * 4);
    }
    auto NBsel = [&](int b) -> NodeBuf { return b ? nb1 : nb0; };
    uint32_t* ch = (uint32_t*)take((size_t)NC * 16);
    int* xr = (int*)take(NC * 4);
    int* aux = (int*)take(NC * 4);       // E[r] then CB[r]
    int* candl = (int*)take(NC * 4);
    SortEl* arr = (SortEl*)take(NC * 8);
    int* cellOff = (int*)take((g->max_level_cells + 1) * 4);
    int* scr = (int*)take(64);
    int* sh = (int*)take(64);           // block-uniform scalars
    uint32_t* Kl = LDSK ? (uint32_t*)take((size_t)kcap * 4) : nullptr;
    uint16_t* KNl = LDSK ? (uint16_t*)take((size_t)kcap * 2) : nullptr;

#ifdef MAM_DIST_PROFILE
    long long dp0 = clock64();
#endif
    // ---- 0. gather this level's candidates in reference order (cells row-major, FAST order inside)
    const int* cc = cell_counts + (size_t)f * g->cells_per_frame + L.cell_base;
    int carry = 0;
    for (int c0 = 0; c0 < L.ncells; c0 += 256) {
        const int c = c0 + tid;
        const int v = c < L.ncells ? cc[c] : 0;
        int tot;
        const int pre = block_excl_scan(v, scr, &tot);
        if (c < L.ncells) cellOff[c] = carry + pre;
        carry += tot;
    }
    const int n = carry;
    if (LDSK && n > kcap) return false;
    const uint32_t* cbase = cand + (size_t)f * g->cand_per_frame + L.cand_base;
    uint32_t* K = LDSK ? Kl : keys + (size_t)f * g->cand_per_frame + L.cand_base;
    uint16_t* KN = LDSK ? KNl : knode + (size_t)f * g->cand_per_frame + L.cand_base;
    // candidate k -> its cell by binary search over the cell offsets; 4 independent global loads in flight per
    // thread (a cell-per-wave walk is a chain of ~ncells/4 dependent global round trips)
    if (tid == 0) cellOff[L.ncells] = n;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += 4 * 256) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = k0 + u * 256 + tid;
            v[u] = 0;
            if (k < n) {
                int lo = 0, hi = L.ncells;   // last cell with cellOff[c] <= k
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (cellOff[mid] <= k) lo = mid;
                    else hi = mid;
                }
                v[u] = cbase[(size_t)lo * L.cellcap + (k - cellOff[lo])];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = k0 + u * 256 + tid;
            if (k < n) K[k] = v[u];
        }
    }
    __syncthreads();
    int* lc = lvl_counts + ((size_t)f * g->nlevels + l) * 2;
    if (n == 0) {
        if (tid == 0) { lc[0] = 0; lc[1] = 0; }
        return true;
    }
    const int N = L.nfeat;
    const int H = L.maxBY - L.minBY;
    // ---- 1. initial nodes (ORBextractor.cc:559-598)
    int cur = 0;
    {
        const NodeBuf A = nb0;
        for (int i = tid; i < L.nini; i += 256) {
            A.x0[i] = (uint16_t)(int)(L.hX * (float)i);
            A.x1[i] = (uint16_t)(int)(L.hX * (float)(i + 1));
            A.y0[i] = 0;
            A.y1[i] = (uint16_t)H;
            A.cnt[i] = 0;
        }
        __syncthreads();
        for (int k = tid; k < n; k += 256) {
            const float x = (float)(K[k] & 0xFFF);
            const int i = (int)(x / L.hX);
            KN[k] = (uint16_t)i;
            atomicAdd(&A.cnt[i], 1u);
        }
        __syncthreads();
        // erase empty initial nodes, keep order
        const NodeBuf B = nb1;
        int keep_carry = 0;
        for (int i0 = 0; i0 < L.nini; i0 += 256) {
            const int i = i0 + tid;
            const bool ne = i < L.nini && A.cnt[i] > 0;
            int tot;
            const int pos = block_excl_scan(ne ? 1 : 0, scr, &tot);
            if (ne) {
                const int np = keep_carry + pos;
                B.x0[np] = A.x0[i]; B.y0[np] = A.y0[i]; B.x1[np] = A.x1[i]; B.y1[np] = A.y1[i];
                B.cnt[np] = A.cnt[i];
                ch[4 * i] = np;
            }
            keep_carry += tot;
        }
        __syncthreads();
        for (int k = tid; k < n; k += 256) KN[k] = (uint16_t)ch[4 * KN[k]];
        if (tid == 0) sh[0] = keep_carry;
        __syncthreads();
        cur = 1;
    }
    int S = sh[0];
    DPROF(0);

    // Rebuild the list given xr[p] (expansion rank, -1 = unexpanded) for p < S, NX expanded nodes whose
    // children were already counted into ch[4p..4p+3]; aux[r] = #non-empty children of rank r.
    // Produces the new list in the other buffer, remaps keys, builds candl (children with >1 keys in
    // creation order) and returns (via sh) the new size and #candidates.
    auto rebuild = [&](int NX) {
        const NodeBuf A = NBsel(cur);
        const NodeBuf B = NBsel(cur ^ 1);
        // exclusive scan of aux over ranks -> creation base (in place)
        int cb_carry = 0;
        for (int r0 = 0; r0 < NX; r0 += 256) {
            const int r = r0 + tid;
            const int v = r < NX ? aux[r] : 0;
            int tot;
            const int pre = block_excl_scan(v, scr, &tot);
            if (r < NX) aux[r] = cb_carry + pre;
            cb_carry += tot;
        }
        const int C = cb_carry;
        __syncthreads();
        int k_carry = 0;
        for (int p0 = 0; p0 < S; p0 += 256) {
            const int p = p0 + tid;
            const bool kept = p < S && xr[p] < 0;
            int tot;
            const int kr = block_excl_scan(kept ? 1 : 0, scr, &tot);
            if (p < S) {
                if (kept) {
                    const int np = C + k_carry + kr;
                    B.x0[np] = A.x0[p]; B.y0[np] = A.y0[p]; B.x1[np] = A.x1[p]; B.y1[np] = A.y1[p];
                    B.cnt[np] = A.cnt[p];
                    ch[4 * p] = np;
                } else {
                    int c = aux[xr[p]];
                    for (int q = 0; q < 4; q++) {
                        const uint32_t cq = ch[4 * p + q];
                        if (cq > 0) {
                            const int np = C - 1 - c;
                            int cx0, cy0, cx1, cy1;
                            child_rect(A, p, q, &cx0, &cy0, &cx1, &cy1);
                            B.x0[np] = (uint16_t)cx0; B.y0[np] = (uint16_t)cy0;
                            B.x1[np] = (uint16_t)cx1; B.y1[np] = (uint16_t)cy1;
                            B.cnt[np] = cq;
                            ch[4 * p + q] = np;
                            c++;
                        }
                    }
                }
            }
            k_carry += tot;
        }
        __syncthreads();
        for (int k = tid; k < n; k += 256) {
            const int p = KN[k];
            if (xr[p] < 0) KN[k] = (uint16_t)ch[4 * p];
            else KN[k] = (uint16_t)ch[4 * p + quad_of(A, p, K[k])];
        }
        // candidates for the next step: children with >1 keys, creation order = descending position
        int m_carry = 0;
        for (int c0 = 0; c0 < C; c0 += 256) {
            const int c = c0 + tid;
            const bool big = c < C && B.cnt[C - 1 - c] > 1;
            int tot;
            const int pos = block_excl_scan(big ? 1 : 0, scr, &tot);
            if (big) candl[m_carry + pos] = C - 1 - c;
            m_carry += tot;
        }
        if (tid == 0) { sh[0] = C + k_carry; sh[1] = m_carry; }
        __syncthreads();
        cur ^= 1;
    };

    bool finish = false;
    bool final_phase = false;
    int m = 0;
    int guard = 0;
    while (!finish) {
        if (++guard > 4096) {  // unreachable for a correct rebuild (S grows or the loop ends); never hang
            if (tid == 0) { lc[0] = -1; lc[1] = 0; }
            return true;
        }
        const int prevSize = S;
        if (!final_phase) {
            // ---- phase-1 round: every node with >1 keys divides (ORBextractor.cc:605-677)
            const NodeBuf A = NBsel(cur);
            int x_carry = 0;
            for (int p0 = 0; p0 < S; p0 += 256) {
                const int p = p0 + tid;
                const bool ex = p < S && A.cnt[p] > 1;
                int tot;
                const int pos = block_excl_scan(ex ? 1 : 0, scr, &tot);
                if (p < S) {
                    xr[p] = ex ? x_carry + pos : -1;
                    if (ex) { ch[4 * p] = 0; ch[4 * p + 1] = 0; ch[4 * p + 2] = 0; ch[4 * p + 3] = 0; }
                }
                x_carry += tot;
            }
            const int NX = x_carry;
            __syncthreads();
            for (int k = tid; k < n; k += 256) {
                const int p = KN[k];
                if (xr[p] >= 0) atomicAdd(&ch[4 * p + quad_of(A, p, K[k])], 1u);
            }
            __syncthreads();
            for (int p = tid; p < S; p += 256) {
                if (xr[p] >= 0)
                    aux[xr[p]] = (ch[4 * p] > 0) + (ch[4 * p + 1] > 0) + (ch[4 * p + 2] > 0) + (ch[4 * p + 3] > 0);
            }
            __syncthreads();
            rebuild(NX);
            S = sh[0];
            m = sh[1];
            if (S >= N || S == prevSize) finish = true;
            else if (S + m * 3 > N) final_phase = true;
            DPROF(1);
        } else {
            // ---- final phase (ORBextractor.cc:680-748): sort last round's >1-key children by
            // (size, UL.x) with libstdc++'s introsort, expand from the largest until size >= N.
            if (m == 0) break;
            const NodeBuf A = NBsel(cur);
            for (int i = tid; i < m; i += 256) {
                const int p = candl[i];
                arr[i].key = (A.cnt[p] << 12) | A.x0[p];
                arr[i].val = (uint32_t)p;
            }
            __syncthreads();
            DPROF(2);
            if (m <= 64) {
                // one wave replays libstdc++'s introsort (ties included) in registers; aux is dead here
                if (tid < 64) stl_sort_wave<1>(arr, m, aux);
            } else if (m <= 256) {
                if (tid < 64) stl_sort_wave<4>(arr, m, aux);
            } else if (tid == 0) {
                stl_sort(arr, arr + m);
            }
            __syncthreads();
            DPROF(3);
#ifdef MAM_DIST_PROFILE
            if (tid == 0) { atomicAdd(&g_dprof[6], (unsigned long long)m); atomicAdd(&g_dprof[7], 1ull); }
#endif
            for (int p = tid; p < S; p += 256) xr[p] = -1;
            __syncthreads();
            for (int i = tid; i < m; i += 256) {
                const int p = arr[i].val;
                xr[p] = i;  // sorted index for now
                ch[4 * p] = 0; ch[4 * p + 1] = 0; ch[4 * p + 2] = 0; ch[4 * p + 3] = 0;
            }
            __syncthreads();
            for (int k = tid; k < n; k += 256) {
                const int p = KN[k];
                if (xr[p] >= 0) atomicAdd(&ch[4 * p + quad_of(A, p, K[k])], 1u);
            }
            __syncthreads();
            // expansion rank r = m-1-i; grow(r) = sum_{r'<=r} (e(r')-1); stop at the first r with S+grow >= N
            int g_carry = 0;
            int rstop_local = m - 1;
            for (int r0 = 0; r0 < m; r0 += 256) {
                const int r = r0 + tid;
                int e = 0;
                if (r < m) {
                    const int p = arr[m - 1 - r].val;
                    e = (ch[4 * p] > 0) + (ch[4 * p + 1] > 0) + (ch[4 * p + 2] > 0) + (ch[4 * p + 3] > 0);
                    aux[r] = e;
                }
                int tot;
                const int pre = block_excl_scan(r < m ? e - 1 : 0, scr, &tot);
                if (r < m && S + g_carry + pre + (e - 1) >= N) rstop_local = min(rstop_local, r);
                g_carry += tot;
            }
            const int rstop = block_min(rstop_local, scr);
            const int NX = rstop + 1;
            for (int p = tid; p < S; p += 256) {
                const int i = xr[p];
                if (i >= 0) {
                    const int r = m - 1 - i;
                    xr[p] = r <= rstop ? r : -1;
                }
            }
            __syncthreads();
            rebuild(NX);
            S = sh[0];
            m = sh[1];
            if (S >= N || S == prevSize) finish = true;
            DPROF(4);
        }
    }

    // ---- retain the best key per node (first max response in candidate order, ORBextractor.cc:758-776)
    const NodeBuf A = NBsel(cur);
    (void)A;
    for (int p = tid; p < S; p += 256) ch[p] = 0;
    __syncthreads();
    for (int k = tid; k < n; k += 256) {
        const uint32_t v = ((K[k] >> 24) << 24) | (0xFFFFFFu - (uint32_t)k);
        atomicMax(&ch[KN[k]], v);
    }
    __syncthreads();
    // ---- outputs in list order + lapping ranks (ORBextractor.cc:1141-1162)
    uint32_t* ok = out_key + (size_t)f * g->kp_slots + L.kp_base;
    uint32_t* orr = out_rank + (size_t)f * g->kp_slots + L.kp_base;
    if (S > L.kp_cap) {
        if (tid == 0) { lc[0] = -1; lc[1] = 0; }
        return true;
    }
    int st_carry = 0;
    for (int p0 = 0; p0 < S; p0 += 256) {
        const int p = p0 + tid;
        bool st = false;
        uint32_t kv = 0;
        if (p < S) {
            const uint32_t k = 0xFFFFFFu - (ch[p] & 0xFFFFFFu);
            kv = K[k];
            float xs = (float)((int)(kv & 0xFFF) + L.minBX);
            if (l != 0) xs = xs * L.scale;
            st = xs >= (float)lap0 && xs <= (float)lap1;
        }
        int tot;
        const int rk = block_excl_scan(st ? 1 : 0, scr, &tot);
        if (p < S) {
            ok[p] = kv;
            orr[p] = st ? (0x80000000u | (uint32_t)(st_carry + rk)) : (uint32_t)(p - (st_carry + rk));
        }
        st_carry += tot;
    }
    if (tid == 0) { lc[0] = S; lc[1] = st_carry; }
    DPROF(5);
    return true;
}

__global__ __launch_bounds__(256) void k_distribute(const Geom* __restrict__ g, const int* __restrict__ cell_counts,
                                                    const uint32_t* __restrict__ cand, uint32_t* __restrict__ keys,
                                                    uint16_t* __restrict__ knode, uint32_t* __restrict__ out_key,
                                                    uint32_t* __restrict__ out_rank, int* __restrict__ lvl_counts,
                                                    int lap0, int lap1, int kcap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (!distribute_impl<true>(smem, g, cell_counts, cand, keys, knode, out_key, out_rank, lvl_counts, lap0, lap1, kcap))
        distribute_impl<false>(smem, g, cell_counts, cand, keys, knode, out_key, out_rank, lvl_counts, lap0, lap1, 0);
}

// ------------------------------------------------------------------------------------------------ describe
constexpr int DESC_R = 18;                          // max |rotated pattern offset| (rounded)
constexpr int DESC_ROWS = 2 * DESC_R + 1;            // 37 patch rows
constexpr int DESC_WPR = 10;                         // words per patch row: 37 bytes + up to 3 bytes of alignment
constexpr int DESC_NW = (DESC_ROWS * DESC_WPR + 63) / 64;   // words per lane

__global__ __launch_bounds__(256) void k_describe(const Geom* __restrict__ g, LevelSrc s,
                                                  const uint8_t* __restrict__ blur,
                                                  const uint32_t* __restrict__ out_key,
                                                  const uint32_t* __restrict__ out_rank,
                                                  const int* __restrict__ lvl_counts, int nframes,
                                                  mam_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                  int capacity, int32_t* __restrict__ counts, int fp_policy) {
#ifndef MAM_DESC_XCD
#define MAM_DESC_XCD 1
#endif
    // XCD-aware order: each XCD describes a contiguous range of (frame, keypoint) slots, so the patches of a frame's
    // nearby keypoints share its L2
    const int blk = MAM_DESC_XCD ? xcd_logical(blockIdx.x, gridDim.x) : blockIdx.x;
    const int gw = (blk * 256 + threadIdx.x) >> 6;
    const int lane = lane_id();
    const int f = gw / g->kp_slots;
    const int r = gw - f * g->kp_slots;
    if (f >= nframes) return;
    const int nl = g->nlevels;
    const int* lc = lvl_counts + (size_t)f * nl * 2;
    int l = 0;
    for (int i = 1; i < nl; i++)
        if (r >= g->L[i].kp_base) l = i;
    int ntot = 0, mono_before = 0, st_before = 0, mono_tot = 0;
    bool bad = false;
    for (int i = 0; i < nl; i++) {
        const int cnt = lc[2 * i], st = lc[2 * i + 1];
        if (cnt < 0) bad = true;
        ntot += cnt;
        mono_tot += cnt - st;
        if (i < l) { mono_before += cnt - st; st_before += st; }
    }
    const bool overflow = bad || ntot > capacity;
    if (r == 0 && lane == 0) {
        counts[2 * f] = overflow ? -2 : ntot;
        counts[2 * f + 1] = overflow ? 0 : mono_tot;
    }
    const LevelGeom& L = g->L[l];
    const int idx = r - L.kp_base;
    if (overflow || idx >= lc[2 * l]) return;
    const uint32_t kv = out_key[(size_t)f * g->kp_slots + r];
    const uint32_t rk = out_rank[(size_t)f * g->kp_slots + r];
    const int x = (int)(kv & 0xFFF) + L.minBX;
    const int y = (int)((kv >> 12) & 0xFFF) + L.minBY;
    const int score = (int)(kv >> 24);
    // IC_Angle on the unblurred level (ORBextractor.cc:76-103): integer moments over the radius-15 disk
    int pitch;
    const uint8_t* lev = level_ptr(g, s, f, l, &pitch);
    const uint8_t* center = lev + (size_t)y * pitch + x;
    // lane = (column u, half): the disk column u spans |v| <= vmax(u) (umax decreases with |v|), lanes 0..30 take
    // v in [-vmax, 0], lanes 32..62 take v in [1, vmax]; integer sums are order-independent
    // all 16 loads of a lane's column in flight at once (a v-loop would wait out one global latency per pixel);
    // umax is non-increasing, so vmax(u) = #{v in 1..15 : umax[v] >= |u|}
    // the blurred patch the rBRIEF tests sample (rotated pattern offsets: |offset| <= 13 (|cos| + |sin|) <= 18.4, so
    // rows y-18..y+18 and columns x-18..x+18), fetched into this wave's LDS slot in the same round trip as the IC
    // loads, before the angle is known; rows as DESC_WPR aligned words from the word holding column x-18
    const uint8_t* bl = blur + L.blur_off + (size_t)f * L.frame_bytes;
    const int bpitch = L.pitch;
    __shared__ uint32_t bpatch[4][DESC_ROWS * DESC_WPR];
    uint32_t* patch = bpatch[(threadIdx.x >> 6) & 3];
    const uintptr_t row0 = (uintptr_t)(bl + (size_t)(y - DESC_R) * bpitch + (x - DESC_R));
    const int shift = (int)(row0 & 3);   // byte offset of column x-18 in the first word of each row
    uint32_t pw[DESC_NW];
    {
        const uint8_t* base = reinterpret_cast<const uint8_t*>(row0 - (uintptr_t)shift);
#pragma unroll
        for (int k = 0; k < DESC_NW; k++) {
            const int i = k * 64 + lane;
            const int rr = i / DESC_WPR, c = i - rr * DESC_WPR;
            pw[k] = i < DESC_ROWS * DESC_WPR ? *reinterpret_cast<const uint32_t*>(base + (size_t)rr * bpitch + 4 * c) : 0u;
        }
    }
    int m10 = 0, m01 = 0;
    {
        const int col = lane & 31;
        int um[16];
#pragma unroll
        for (int k = 0; k < 16; k++) um[k] = g->umax[k];
        const int u = col - 15;
        const int au = u < 0 ? -u : u;
        int vmax = 0;
#pragma unroll
        for (int k = 1; k < 16; k++) vmax += au <= um[k] ? 1 : 0;
        const int v0 = lane < 32 ? -vmax : 1, n = col < 31 ? (lane < 32 ? vmax + 1 : vmax) : 0;
        const uint8_t* cp = center + u + (ptrdiff_t)v0 * pitch;
        int val[16];
#pragma unroll
        for (int k = 0; k < 16; k++) val[k] = k < n ? cp[(ptrdiff_t)k * pitch] : 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            m10 += val[k];
            m01 += (v0 + k) * val[k];
        }
        m10 *= u;
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    const float angle = fast_atan2((float)m01, (float)m10);
    // rBRIEF on the blurred level (ORBextractor.cc:107-146): lane owns pairs lane, lane+64, ...
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float a, b;   // a = (float)cos(angle), b = (float)sin(angle) under the fp policy (mam_orb.h MAM_FP_*)
    if (fp_policy & MAM_FP_TRIG_CORRECTLY_ROUNDED) det_sincos(angle * factorPI, &b, &a);
    else if (fp_policy & MAM_FP_TRIG_SSE2) glibc_sincosf<false>(angle * factorPI, &b, &a);
    else glibc_sincosf<true>(angle * factorPI, &b, &a);
    const bool desc_fma = !(fp_policy & MAM_FP_DESC_UNCONTRACTED);
#pragma unroll
    for (int k = 0; k < DESC_NW; k++) {
        const int i = k * 64 + lane;
        if (i < DESC_ROWS * DESC_WPR) patch[i] = pw[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // pixel (y + dy, x + dx) = patch byte (dy + 18) * 4 * DESC_WPR + shift + dx + 18
    const uint8_t* pc = reinterpret_cast<const uint8_t*>(patch) + DESC_R * 4 * DESC_WPR + shift + DESC_R;
    uint64_t words[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int pr = lane + 64 * k;
        int val[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const float px = (float)c_pattern[4 * pr + 2 * e];
            const float py = (float)c_pattern[4 * pr + 2 * e + 1];
            float fy, fx;
            if (desc_fma) {
                fy = __builtin_fmaf(px, b, py * a);
                fx = __builtin_fmaf(px, a, -(py * b));
            } else {
                const float t0 = px * b, t1 = py * a;
                fy = t0 + t1;
                const float t2 = px * a, t3 = py * b;
                fx = t2 - t3;
            }
            val[e] = pc[__float2int_rn(fy) * (4 * DESC_WPR) + __float2int_rn(fx)];
        }
        words[k] = __ballot(val[0] < val[1]);
    }
    // placement (ORBextractor.cc:1141-1162)
    int o;
    if (rk & 0x80000000u) o = ntot - 1 - (st_before + (int)(rk & 0x7FFFFFFFu));
    else o = mono_before + (int)rk;
    uint8_t* dd = desc + ((size_t)f * capacity + o) * 32;
    const uint64_t mine = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
    if (lane < 4) reinterpret_cast<uint64_t*>(dd)[lane] = mine;
    if (lane == 0) {
        mam_keypoint kp;
        float xs = (float)x, ys = (float)y;
        if (l != 0) { xs = xs * L.scale; ys = ys * L.scale; }
        kp.x = xs; kp.y = ys;
        kp.size = (float)L.psize;
        kp.angle = angle;
        kp.response = (float)score;
        kp.octave = l;
        kp.class_id = -1;
        kps[(size_t)f * capacity + o] = kp;
    }
}

}  // namespace mam
