// orb_extract.hip — host orchestration + C-ABI of the ORB extractor (include/mam_orb.h).
//
// Mirrors MAM3SLAM::ORBextractor (reference include/ORBextractor.h:43-100, src/ORBextractor.cc:409-469,
// 1086-1195): the constructor tables are computed on the host exactly as the reference does; the per-frame
// work runs as five kernel stages on the context's HIP stream (orb_kernels.hip). The same pipeline serves
// a single host frame (mam_orb_extract, synchronous, reference semantics) and device-resident batches of
// frames (mam_orb_extract_batch_device, asynchronous; used by multi-agent harnesses and bench.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <map>
#include <memory>
#include <vector>

#include "orb_common.hpp"
#include "runtime.hpp"
#include "orb_kernels.hip"
#include "distribute.hpp"

namespace {

thread_local std::string g_last_error;

inline int cvRoundF(float v) { return (int)lrintf(v); }
inline int cvRoundD(double v) { return (int)lrint(v); }
inline int cvFloorF(float v) { int i = (int)v; return i - (i > v); }
inline int cvCeilF(float v) { int i = (int)v; return i + (i < v); }
inline short satShortF(float v) {
    int iv = cvRoundF(v);
    return (short)(iv < -32768 ? -32768 : iv > 32767 ? 32767 : iv);
}

using mam::DevBuf;

}  // namespace

void mam::set_last_error(const std::string& s) { g_last_error = s; }

struct mam_orb_ctx {
    mam_orb_params prm{};
    int device = 0;
    hipStream_t stream = nullptr;
    // constructor tables (ORBextractor.cc:409-469)
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> nPerLevel, umax;
    // geometry for the current frame size
    int W = 0, H = 0, Fcap = 0;
    mam::Geom geom{};
    std::vector<mam::CellDesc> cells;
    DevBuf<mam::Geom> d_geom;
    DevBuf<mam::CellDesc> d_cells;
    DevBuf<int> d_tabs_i;
    DevBuf<short> d_tabs_s;
    DevBuf<uint4> d_qcoef;
    DevBuf<int2> d_rcoef;
    // per-batch device scratch
    DevBuf<uint8_t> d_pyr, d_blur, d_input;
    DevBuf<uint32_t> d_cand, d_keys, d_okey, d_orank;
    DevBuf<uint16_t> d_knode;
    DevBuf<uint32_t> d_knode32;   // k_distribute2's node words of keys beyond its register capacity
    DevBuf<int> d_cellcnt, d_lvlcnt;
    DevBuf<mam_keypoint> d_kps;
    DevBuf<uint8_t> d_desc;
    DevBuf<int32_t> d_counts;
    // mam_orb_extract's staging: the frame and one [counts | keypoints | descriptors] block, pinned on the host and
    // contiguous on the device, so a call is one upload, the pipeline, one download and one synchronisation
    mam::PinnedBuf h_in, h_out;
    DevBuf<uint8_t> d_out;
    size_t fast_lds = 0, dist_lds = 0;
    size_t dist2_lds[3] = {0, 0, 0};   // k_distribute2 LDS bytes for 256 / 512 / 1024 threads
    bool dist2_ok[3] = {false, false, false};   // the width's LDS fits a CU
    int dist_nt = -1;                  // DistributeOctTree width override (mam_orb_debug_set_option), -1 = auto
    int fork = -1;                     // latency-mode stream fork override (mam_orb_debug_set_option), -1 = auto
    // latency mode's side streams and their fork / join events (run_pipeline)
    hipStream_t side[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_pyr = nullptr, ev_side[2] = {nullptr, nullptr};
    int dist_kcap = 0;   // candidates per level k_distribute keeps in LDS (more: global scratch)
    int fast_cw = 0;   // k_fast_cells plane pitch instance
    // k_fast_chunks (cells of a row in chunks of up to FAST_G): chunk table, plane pitch instance, LDS, first chunk of
    // each level
    std::vector<mam::ChunkDesc> chunks;
    DevBuf<mam::ChunkDesc> d_chunks;
    int fastc_cw = 0;
    size_t fastc_lds = 0;
    int chunk_base[MAM_MAX_LEVELS + 1] = {};
    int fast_chunks = -1;   // k_fast_chunks instead of k_fast_cells (mam_orb_debug_set_option), -1 = automatic
    int fast_blur = -1;     // FAST + blur in one launch (k_fast_blur; mam_orb_debug_set_option), -1 = automatic
    // single-launch pyramid (k_pyr_bands): per band count, the band table and its LDS carve
    struct PyrPlan {
        int nb = 0;
        size_t lds = 0;
        int buf1_off = 0, rc_off = 0, qc_off = 0, qtot = 0;   // LDS carve: level rows, row / column coefficients
        DevBuf<int4> bands;
    };
    std::vector<std::vector<int>> h_yofs;       // resize row tables per level (host copy, l >= 1)
    std::map<int, std::unique_ptr<PyrPlan>> pyr_plans;
    // last-call bookkeeping for debug taps
    const uint8_t* last_in0 = nullptr;
    size_t last_stride = 0, last_fstride = 0;
    int last_nframes = 0;
    // profiling
    mam::StageTimer timer{MAM_STAGE_COUNT};
};

namespace {

int build_tables(mam_orb_ctx* c) {
    const mam_orb_params& p = c->prm;
    const int L = p.nlevels;
    const double scaleFactor = (double)p.scale_factor;   // member is double (ORBextractor.h:72)
    c->scale.assign(L, 0.f); c->sigma2.assign(L, 0.f); c->invScale.assign(L, 0.f); c->invSigma2.assign(L, 0.f);
    c->scale[0] = 1.0f; c->sigma2[0] = 1.0f;
    for (int i = 1; i < L; i++) {
        c->scale[i] = (float)((double)c->scale[i - 1] * scaleFactor);
        c->sigma2[i] = c->scale[i] * c->scale[i];
    }
    for (int i = 0; i < L; i++) { c->invScale[i] = 1.0f / c->scale[i]; c->invSigma2[i] = 1.0f / c->sigma2[i]; }
    c->nPerLevel.assign(L, 0);
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        c->nPerLevel[l] = cvRoundF(nDesired);
        sum += c->nPerLevel[l];
        nDesired *= factor;
    }
    c->nPerLevel[L - 1] = std::max(p.nfeatures - sum, 0);
    c->umax.assign(16, 0);
    int v, v0, vmax = cvFloorF(15 * sqrtf(2.f) / 2 + 1);
    int vmin = cvCeilF(15 * sqrtf(2.f) / 2);
    const double hp2 = 15 * 15;
    for (v = 0; v <= vmax; ++v) c->umax[v] = cvRoundD(sqrt(hp2 - v * v));
    for (v = 15, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
    return MAM_OK;
}

// OpenCV hal::resize INTER_LINEAR coefficient tables (see orb_kernels.hip k_pyr_down).
void resize_tables(int sw, int sh, int dw, int dh, std::vector<int>& xofs, std::vector<short>& ialpha,
                   std::vector<int>& yofs, std::vector<short>& ibeta, int* xmax_out, int* xvec_out) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    xofs.resize(dw); ialpha.resize(2 * dw); yofs.resize(dh); ibeta.resize(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloorF(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        ialpha[2 * dx] = satShortF((1.f - fx) * 2048);
        ialpha[2 * dx + 1] = satShortF(fx * 2048);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloorF(fy);
        fy -= sy;
        yofs[dy] = sy;
        ibeta[2 * dy] = satShortF((1.f - fy) * 2048);
        ibeta[2 * dy + 1] = satShortF(fy * 2048);
    }
    int xvec = 0;
    while (xvec <= dw - 16) xvec += 16;
    while (xvec < dw - 8) xvec += 8;
    *xmax_out = xmax;
    *xvec_out = xvec;
}

size_t distribute_lds_bytes(int NC, int max_cells) {
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t s = 0;
    for (int b = 0; b < 2; b++) s += 4 * a16(NC * 2) + a16(NC * 4);
    s += a16((size_t)NC * 16) + 3 * a16(NC * 4) + a16(NC * 8) + a16((max_cells + 1) * 4) + 64 + 64;
    return s;
}

int build_pyr_plan(mam_orb_ctx* c, int nb);
int pyr_forced_bands();
bool pyr_flat_enabled();
int pyr_rows_per_thread();

// Geometry for a W x H frame and capacity F (reallocates device scratch when either grows/changes).
int ensure_geometry(mam_orb_ctx* c, int W, int H, int F) {
    if (W == c->W && H == c->H && F <= c->Fcap) return MAM_OK;
    const bool geom_changed = (W != c->W || H != c->H);
    const int Fcap = std::max(F, geom_changed ? F : c->Fcap);
    const int L = c->prm.nlevels;
    mam::Geom& g = c->geom;
    if (geom_changed) {
        g = mam::Geom{};
        g.nlevels = L;
        for (int v = 0; v < 16; v++) g.umax[v] = c->umax[v];
        c->cells.clear();
        int cand = 0, kp = 0, tiles = 0, node_cap = 0, maxcells = 0, rmax = 0, cmax = 0;
        std::vector<int> ti;
        std::vector<short> ts;
        std::vector<size_t> tab_off(L, 0);
        for (int l = 0; l < L; l++) {
            mam::LevelGeom& lv = g.L[l];
            lv.w = cvRoundF((float)W * c->invScale[l]);
            lv.h = cvRoundF((float)H * c->invScale[l]);
            if (lv.w < 2 * mam::EDGE_THRESHOLD + 8 || lv.h < 2 * mam::EDGE_THRESHOLD + 8 || lv.w > 4095 || lv.h > 4095) {
                g_last_error = "frame size out of range for the level pyramid";
                return MAM_ERR_ARG;
            }
            lv.pitch = (lv.w + 63) & ~63;
            lv.frame_bytes = (long long)lv.h * lv.pitch;
            lv.scale = c->scale[l];
            lv.psize = (int)(mam::PATCH_SIZE * c->scale[l]);
            lv.nfeat = c->nPerLevel[l];
            // FAST cell grid, ComputeKeyPointsOctTree (ORBextractor.cc:785-823)
            lv.minBX = mam::EDGE_THRESHOLD - 3;
            lv.minBY = lv.minBX;
            lv.maxBX = lv.w - mam::EDGE_THRESHOLD + 3;
            lv.maxBY = lv.h - mam::EDGE_THRESHOLD + 3;
            const float width = (float)(lv.maxBX - lv.minBX), height = (float)(lv.maxBY - lv.minBY);
            lv.nCols = (int)(width / 35.f);
            lv.nRows = (int)(height / 35.f);
            if (lv.nCols < 1 || lv.nRows < 1) { g_last_error = "level too small for a FAST cell"; return MAM_ERR_ARG; }
            lv.wCell = (int)ceil(width / lv.nCols);
            lv.hCell = (int)ceil(height / lv.nRows);
            lv.cell_base = (int)c->cells.size();
            int cap = 0, slot = 0;
            for (int i = 0; i < lv.nRows; i++) {
                const float iniY = (float)(lv.minBY + i * lv.hCell);
                float maxY = iniY + lv.hCell + 6;
                if (iniY >= lv.maxBY - 3) continue;
                if (maxY > lv.maxBY) maxY = (float)lv.maxBY;
                for (int j = 0; j < lv.nCols; j++) {
                    const float iniX = (float)(lv.minBX + j * lv.wCell);
                    float maxX = iniX + lv.wCell + 6;
                    if (iniX >= lv.maxBX - 6) continue;
                    if (maxX > lv.maxBX) maxX = (float)lv.maxBX;
                    mam::CellDesc cd;
                    cd.level = l; cd.ci = i; cd.cj = j;
                    cd.x0 = (int)iniX; cd.y0 = (int)iniY; cd.x1 = (int)maxX; cd.y1 = (int)maxY;
                    cd.slot = slot++;
                    const int bh = cd.y1 - cd.y0 - 6, bw = cd.x1 - cd.x0 - 6;
                    if (bh > 0 && bw > 0) cap = std::max(cap, ((bh + 1) / 2) * ((bw + 1) / 2));
                    rmax = std::max(rmax, cd.y1 - cd.y0);
                    cmax = std::max(cmax, cd.x1 - cd.x0);
                    c->cells.push_back(cd);
                }
            }
            lv.ncells = slot;
            lv.cellcap = std::max(cap, 1);
            lv.cand_base = cand;
            lv.cand_cap = lv.ncells * lv.cellcap;
            cand += lv.cand_cap;
            maxcells = std::max(maxcells, lv.ncells);
            // DistributeOctTree initial nodes (ORBextractor.cc:559-560)
            lv.nini = (int)roundf((float)(lv.maxBX - lv.minBX) / (lv.maxBY - lv.minBY));
            if (lv.nini < 1) { g_last_error = "frame aspect gives zero initial octree nodes"; return MAM_ERR_ARG; }
            lv.hX = (float)(lv.maxBX - lv.minBX) / lv.nini;
            lv.kp_base = kp;
            lv.kp_cap = std::max(lv.nfeat + 3, 4 * lv.nini);
            kp += lv.kp_cap;
            node_cap = std::max(node_cap, std::max(lv.kp_cap, lv.nini) + 8);
            // blur tiles
            lv.tiles_x = (lv.w + mam::BLUR_TILE_W - 1) / mam::BLUR_TILE_W;
            lv.tiles_y = (lv.h + mam::BLUR_TILE_H - 1) / mam::BLUR_TILE_H;
            lv.tile_base = tiles;
            tiles += lv.tiles_x * lv.tiles_y;
        }
        if (cand >= (1 << 24)) { g_last_error = "too many FAST candidate slots"; return MAM_ERR_ARG; }
        g.cells_per_frame = (int)c->cells.size();
        g.cand_per_frame = cand;
        g.kp_slots = kp;
        g.tiles_per_frame = tiles;
        node_cap = std::max(node_cap, MAM_SORT_WAVE_SCRATCH(4));  // aux doubles as the wave sort's scratch
        g.node_cap = (node_cap + 3) & ~3;
        g.max_level_cells = maxcells;
        g.roi_max_rows = rmax;
        g.roi_max_cols = cmax;
        // resize tables for levels >= 1
        std::vector<int> xo, yo;
        std::vector<short> al, be;
        std::vector<size_t> ioff(L, 0), soff(L, 0);
        std::vector<int> xmaxv(L, 0), xvecv(L, 0);
        std::vector<uint4> qtab;
        std::vector<int2> rtab;
        std::vector<size_t> qoff(L, 0), roff(L, 0);
        c->h_yofs.assign(L, {});
        c->pyr_plans.clear();
        for (int l = 1; l < L; l++) {
            int xmax, xvec;
            resize_tables(g.L[l - 1].w, g.L[l - 1].h, g.L[l].w, g.L[l].h, xo, al, yo, be, &xmax, &xvec);
            c->h_yofs[l] = yo;
            ioff[l] = ti.size();
            ti.insert(ti.end(), xo.begin(), xo.end());
            ti.insert(ti.end(), yo.begin(), yo.end());
            soff[l] = ts.size();
            ts.insert(ts.end(), al.begin(), al.end());
            ts.insert(ts.end(), be.begin(), be.end());
            xmaxv[l] = xmax;
            xvecv[l] = xvec;
            // packed coefficients of k_pyr_flat (see LevelGeom.qcoef)
            {
                const int dw = g.L[l].w, dh = g.L[l].h, nq = (dw + 3) / 4;
                qoff[l] = qtab.size();
                for (int q = 0; q < nq; q++) {
                    uint32_t w0 = 0, pa[4] = {0, 0, 0, 0};
                    int sx[4];
                    for (int i = 0; i < 4; i++) sx[i] = xo[std::min(4 * q + i, dw - 1)];
                    const int base = sx[0] & ~3;
                    w0 = (uint32_t)base;
                    for (int i = 0; i < 4; i++) {
                        const int dx = 4 * q + i, x = std::min(dx, dw - 1);
                        const bool edge = dx >= xmax;
                        const int a0 = edge ? 2048 : al[2 * x], a1 = edge ? 0 : al[2 * x + 1];
                        w0 |= (uint32_t)(sx[i] - base) << (12 + 4 * i);
                        if (dx < xvec) w0 |= 1u << (28 + i);
                        pa[i] = (uint32_t)(a0 & 0xFFFF) | ((uint32_t)(a1 & 0xFFFF) << 16);
                    }
                    qtab.push_back(make_uint4(w0, pa[0], pa[1], pa[2]));
                    qtab.push_back(make_uint4(pa[3], 0, 0, 0));
                }
                roff[l] = rtab.size();
                for (int dy = 0; dy < dh; dy++)
                    rtab.push_back(make_int2(yo[dy], (be[2 * dy] & 0xFFFF) | ((int)be[2 * dy + 1] << 16)));
                if (xo[dw - 1] > 4095) { g_last_error = "level too wide for the packed resize table"; return MAM_ERR_ARG; }
            }
            // pyr_quad reads three source words per row: the four source columns of an output quad (and the +1 tap)
            // must lie within 12 bytes of the quad's word-aligned first column (scale factors up to ~2.6)
            for (int dx = 0; dx < g.L[l].w; dx += 4)
                if (xo[std::min(dx + 3, g.L[l].w - 1)] - (xo[dx] & ~3) > 10) {
                    g_last_error = "pyramid scale factor too large for the resize kernel";
                    return MAM_ERR_ARG;
                }
            // LDS staging bounds of k_pyr_down: source columns / rows one (PYR_XB x PYR_RB) output block reads
            const int sw = g.L[l - 1].w, sh = g.L[l - 1].h, dw = g.L[l].w, dh = g.L[l].h;
            for (int dx0 = 0; dx0 < dw; dx0 += mam::PYR_XB) {
                const int a = xo[dx0] & ~3, b = std::min(xo[std::min(dx0 + mam::PYR_XB, dw) - 1] + 1, sw - 1);
                g.pyr_seg_w = std::max(g.pyr_seg_w, ((b - a + 1) + 3) & ~3);
            }
            for (int dy0 = 0; dy0 < dh; dy0 += mam::PYR_RB) {
                const int a = std::min(std::max(yo[dy0], 0), sh - 1);
                const int b = std::min(std::max(yo[std::min(dy0 + mam::PYR_RB, dh) - 1] + 1, 0), sh - 1);
                g.pyr_rows = std::max(g.pyr_rows, b - a + 1);
            }
        }
        if (int rc = c->d_tabs_i.alloc(std::max<size_t>(ti.size(), 1))) return rc;
        if (int rc = c->d_tabs_s.alloc(std::max<size_t>(ts.size(), 1))) return rc;
        if (!ti.empty()) MAM_HIP(hipMemcpy(c->d_tabs_i.p, ti.data(), ti.size() * sizeof(int), hipMemcpyHostToDevice));
        if (!ts.empty()) MAM_HIP(hipMemcpy(c->d_tabs_s.p, ts.data(), ts.size() * sizeof(short), hipMemcpyHostToDevice));
        if (int rc = c->d_qcoef.alloc(std::max<size_t>(qtab.size(), 1))) return rc;
        if (int rc = c->d_rcoef.alloc(std::max<size_t>(rtab.size(), 1))) return rc;
        if (!qtab.empty()) MAM_HIP(hipMemcpy(c->d_qcoef.p, qtab.data(), qtab.size() * sizeof(uint4), hipMemcpyHostToDevice));
        if (!rtab.empty()) MAM_HIP(hipMemcpy(c->d_rcoef.p, rtab.data(), rtab.size() * sizeof(int2), hipMemcpyHostToDevice));
        for (int l = 1; l < L; l++) {
            mam::LevelGeom& lv = g.L[l];
            lv.qcoef = c->d_qcoef.p + qoff[l];
            lv.rcoef = c->d_rcoef.p + roff[l];
            lv.xofs = c->d_tabs_i.p + ioff[l];
            lv.yofs = c->d_tabs_i.p + ioff[l] + lv.w;
            lv.ialpha = c->d_tabs_s.p + soff[l];
            lv.ibeta = c->d_tabs_s.p + soff[l] + 2 * lv.w;
            lv.xmax = xmaxv[l];
            lv.xvec = xvecv[l];
        }
        if (int rc = c->d_cells.alloc(c->cells.size())) return rc;
        MAM_HIP(hipMemcpy(c->d_cells.p, c->cells.data(), c->cells.size() * sizeof(mam::CellDesc), hipMemcpyHostToDevice));
        c->fast_cw = 0;
        for (int cw : {24, 32, 40, 48})
            if (cw >= mam::fast_min_cw(cmax)) { c->fast_cw = cw; break; }
        if (c->fast_cw == 0) { g_last_error = "FAST cell too wide"; return MAM_ERR_ARG; }
        c->fast_lds = mam::fast_lds_bytes(rmax, c->fast_cw);
        // chunks: consecutive cells of one row (the cells table lists a row's cells in column order)
        c->chunks.clear();
        int chunk_cols = 0;
        for (int l = 0; l < L; l++) {
            c->chunk_base[l] = (int)c->chunks.size();
            const mam::LevelGeom& lv = g.L[l];
            for (int i0 = lv.cell_base; i0 < lv.cell_base + lv.ncells;) {
                int i1 = i0 + 1;
                while (i1 < lv.cell_base + lv.ncells && i1 - i0 < mam::FAST_G && c->cells[i1].ci == c->cells[i0].ci &&
                       c->cells[i1].cj == c->cells[i1 - 1].cj + 1)
                    i1++;
                mam::ChunkDesc ch;
                ch.level = l;
                ch.cell0 = i0;
                ch.ncell = i1 - i0;
                ch.x0 = c->cells[i0].x0; ch.y0 = c->cells[i0].y0;
                ch.x1 = c->cells[i1 - 1].x1; ch.y1 = c->cells[i0].y1;
                ch.ci = c->cells[i0].ci; ch.cj0 = c->cells[i0].cj;
                chunk_cols = std::max(chunk_cols, ch.x1 - ch.x0);
                c->chunks.push_back(ch);
                i0 = i1;
            }
        }
        c->chunk_base[L] = (int)c->chunks.size();
        c->fastc_cw = 0;
        for (int cw : {64, 80, 96, 112, 128, 160})
            if (cw >= mam::fast_min_cw(chunk_cols)) { c->fastc_cw = cw; break; }
        c->fastc_lds = c->fastc_cw ? mam::fastc_lds_bytes(rmax, c->fastc_cw) : 0;
        if (c->fastc_lds > 160 * 1024) c->fastc_cw = 0;   // (no chunk kernel for this geometry: k_fast_cells)
        if (int rc = c->d_chunks.alloc(std::max<size_t>(c->chunks.size(), 1))) return rc;
        if (!c->chunks.empty())
            MAM_HIP(hipMemcpy(c->d_chunks.p, c->chunks.data(), c->chunks.size() * sizeof(mam::ChunkDesc),
                              hipMemcpyHostToDevice));
        for (const void* fn : {reinterpret_cast<const void*>(&mam::k_fast_blur<24>),
                               reinterpret_cast<const void*>(&mam::k_fast_blur<32>),
                               reinterpret_cast<const void*>(&mam::k_fast_blur<40>),
                               reinterpret_cast<const void*>(&mam::k_fast_blur<48>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<64>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<80>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<96>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<112>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<128>),
                               reinterpret_cast<const void*>(&mam::k_fast_chunks<160>)})
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        {
            const int max_pairs = std::max(rmax - 6, 0) * ((std::max(cmax - 6, 0) + 1) / 2);
            if ((max_pairs + mam::FAST_THREADS - 1) / mam::FAST_THREADS * (mam::FAST_THREADS / 64) >
                mam::FAST_MAX_ENTRIES) {
                g_last_error = "FAST cell too large";
                return MAM_ERR_ARG;
            }
        }
        c->dist_lds = distribute_lds_bytes(g.node_cap, maxcells);
        // candidate keys + node ids in LDS (6 B each) up to a 64 KB workgroup (two per CU)
        c->dist_kcap = (int)std::min<size_t>(16384, c->dist_lds < 60 * 1024 ? (64 * 1024 - c->dist_lds) / 6 : 0) & ~63;
        c->dist_lds += (size_t)c->dist_kcap * 6 + 32;
        for (int i = 0; i < 3; i++) c->dist2_lds[i] = mam::dist::lds_bytes(g.node_cap, maxcells, 256 << i);
        if (g.node_cap > 16383) { g_last_error = "too many DistributeOctTree nodes (nfeatures too large)"; return MAM_ERR_ARG; }
        // the round-3 k_distribute (~60 B a node) is the fallback every geometry must fit; each k_distribute2 width
        // (~84 B a node at 1024 threads) runs only where its LDS fits (dist_threads falls back to the next narrower)
        if (c->fast_lds > 160 * 1024 || c->dist_lds > 160 * 1024) {
            g_last_error = "LDS budget exceeded (nfeatures or cell size too large)";
            return MAM_ERR_ARG;
        }
        for (int i = 0; i < 3; i++) c->dist2_ok[i] = c->dist2_lds[i] <= 160 * 1024;
        if (c->dist2_ok[0])
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::k_distribute2<256, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->dist2_lds[0]);
        if (c->dist2_ok[1])
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::k_distribute2<512, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->dist2_lds[1]);
        if (c->dist2_ok[2])
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::k_distribute2<1024, 8>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->dist2_lds[2]);
        for (int nb = 8; nb <= 64; nb += 8)
            if (int rc = build_pyr_plan(c, nb)) return rc;
        if (pyr_forced_bands() > 0 && pyr_forced_bands() % 8)
            if (int rc = build_pyr_plan(c, pyr_forced_bands())) return rc;
        c->W = W;
        c->H = H;
    }
    // per-frame buffer offsets for capacity Fcap
    long long pyr = 0, blur = 0;
    for (int l = 0; l < L; l++) {
        mam::LevelGeom& lv = g.L[l];
        lv.pyr_off = l == 0 ? 0 : pyr;
        if (l > 0) pyr += (long long)Fcap * lv.frame_bytes;
        lv.blur_off = blur;
        blur += (long long)Fcap * lv.frame_bytes;
    }
    const size_t cand = (size_t)Fcap * g.cand_per_frame;
    if (int rc = c->d_pyr.alloc(std::max<long long>(pyr, 64))) return rc;
    if (int rc = c->d_blur.alloc(blur + 64)) return rc;   // k_describe's patch prefetch reads up to 3 bytes past a row
    if (int rc = c->d_cand.alloc(cand)) return rc;
    if (int rc = c->d_keys.alloc(cand)) return rc;
    if (int rc = c->d_knode.alloc(cand)) return rc;
    if (int rc = c->d_knode32.alloc(cand)) return rc;
    if (int rc = c->d_cellcnt.alloc((size_t)Fcap * g.cells_per_frame)) return rc;
    if (int rc = c->d_lvlcnt.alloc((size_t)Fcap * L * 2)) return rc;
    if (int rc = c->d_okey.alloc((size_t)Fcap * g.kp_slots)) return rc;
    if (int rc = c->d_orank.alloc((size_t)Fcap * g.kp_slots)) return rc;
    if (int rc = c->d_geom.alloc(1)) return rc;
    MAM_HIP(hipMemcpy(c->d_geom.p, &g, sizeof(mam::Geom), hipMemcpyHostToDevice));
    c->Fcap = Fcap;
    return MAM_OK;
}

using StageScope = mam::StageTimer::Scope;

// k_pyr_bands plan for nb bands: band j owns rows [h*j/nb, h*(j+1)/nb) of every level >= 1 and needs, per level, the
// hull of its owned rows and the source rows (yofs of the level above, both taps, clamped) of the rows it needs one
// level up. Returns nullptr when a band would own no row of the top level or the LDS carve exceeds `lds_max`.
// Built for every candidate band count when the geometry is set up (no allocation or copy at launch time, so a
// launch can be captured into a HIP graph).
int build_pyr_plan(mam_orb_ctx* c, int nb) {
    const mam::Geom& g = c->geom;
    const int L = g.nlevels;
    if (L < 2 || nb < 1 || nb > g.L[L - 1].h) return MAM_OK;
    std::vector<int4> tab((size_t)nb * L);
    size_t buf[2] = {0, 0}, rows_max = 0;
    for (int j = 0; j < nb; j++) {
        int4* B = &tab[(size_t)j * L];
        for (int l = 0; l < L; l++) {
            const long long h = g.L[l].h;
            B[l].z = (int)(h * j / nb);
            B[l].w = (int)(h * (j + 1) / nb);
        }
        B[L - 1].x = B[L - 1].z;
        B[L - 1].y = B[L - 1].w;
        for (int l = L - 2; l >= 0; l--) {
            const std::vector<int>& yo = c->h_yofs[l + 1];
            const int sh = g.L[l].h;
            const int a = std::min(std::max(yo[B[l + 1].x], 0), sh - 1);
            const int b = std::min(std::max(yo[B[l + 1].y - 1] + 1, 0), sh - 1) + 1;
            B[l].x = l == 0 ? a : std::min(a, B[l].z);
            B[l].y = l == 0 ? b : std::max(b, B[l].w);
        }
        size_t rows = 0;
        for (int l = 0; l + 1 < L; l++)
            buf[l & 1] = std::max(buf[l & 1], (size_t)(B[l].y - B[l].x) * ((g.L[l].w + 3) & ~3));
        for (int l = 1; l < L; l++) rows += B[l].y - B[l].x;
        rows_max = std::max(rows_max, rows);
    }
    auto plan = std::make_unique<mam_orb_ctx::PyrPlan>();
    plan->nb = nb;
    plan->buf1_off = (int)((buf[0] + 15) & ~(size_t)15);
    plan->rc_off = (int)((plan->buf1_off + buf[1] + 15) & ~(size_t)15);
    // +16: pyr_quad's 12-byte window may run past the last row
    plan->qc_off = (int)((plan->rc_off + rows_max * 8 + 16 + 15) & ~(size_t)15);
    plan->qtot = 0;
    for (int l = 1; l < L; l++) plan->qtot += (g.L[l].w + 3) / 4;
    plan->lds = plan->qc_off + (size_t)plan->qtot * 20;
    if (plan->lds > 160 * 1024) return MAM_OK;
    if (int rc = plan->bands.alloc(tab.size())) return rc;
    MAM_HIP(hipMemcpy(plan->bands.p, tab.data(), tab.size() * sizeof(int4), hipMemcpyHostToDevice));
    c->pyr_plans[nb] = std::move(plan);
    return MAM_OK;
}

// output rows per k_pyr_flat thread (MAM_PYR_RQ = 1 / 2 / 4, default 4: one column-coefficient load per 4 rows and
// 4 quads' loads in flight; pyramid stage per 256 frames c1 0.394 / 0.377 / 0.387 ms, c2 0.939 / 0.823 / 0.787 ms)
int pyr_rows_per_thread() {
    static const int v = [] {
        const char* e = getenv("MAM_PYR_RQ");
        const int x = e ? atoi(e) : 4;
        return (x == 1 || x == 2) ? x : 4;
    }();
    return v;
}

// MAM_PYR_FLAT=0 forces the LDS block kernel for the per-level launches (experiments / parity cross-check)
bool pyr_flat_enabled() {
    static const bool on = [] {
        const char* e = getenv("MAM_PYR_FLAT");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int pyr_forced_bands() {
    static const int forced = [] {
        const char* e = getenv("MAM_PYR_BANDS");
        return e ? atoi(e) : -1;
    }();
    return forced;
}

mam_orb_ctx::PyrPlan* pyr_plan(mam_orb_ctx* c, int nb, size_t lds_max) {
    auto it = c->pyr_plans.find(nb);
    return it != c->pyr_plans.end() && it->second->lds <= lds_max ? it->second.get() : nullptr;
}

// The single-launch pyramid pays ~1.2-2x the arithmetic for one launch instead of nlevels-1: it wins for a few frames
// (latency-bound launches), the per-level launches win for batches (MI355X, c1: one frame 33 vs 54 us; batches: the
// per-level k_pyr_flat launches 0.37 ms per 256 frames vs 0.67 for the bands). Few frames: as many bands as fit
// (shortest chain per workgroup).
// MAM_PYR_BANDS=n forces n bands (0: per-level k_pyr_down launches).
mam_orb_ctx::PyrPlan* choose_pyr_plan(mam_orb_ctx* c, int F) {
    const int forced = pyr_forced_bands();
    if (forced == 0) return nullptr;
    if (forced > 0) return pyr_plan(c, forced, 160 * 1024);
    if (F > 4) return nullptr;
    for (int nb = 64; nb >= 8; nb -= 8)
        if (mam_orb_ctx::PyrPlan* p = pyr_plan(c, nb, 96 * 1024)) return p;
    return nullptr;
}

// DistributeOctTree kernel: k_distribute2 with 1024 threads per (frame, level) for a few frames (latency: a level's
// rounds are chains of barriers, more threads shorten the key passes), 256 for batches (occupancy). MAM_DIST_NT=0 the
// round-3 k_distribute, 256 / 512 / 1024 force a width.
int dist_threads(const mam_orb_ctx* c, int F) {
    static const int forced = [] {
        const char* e = getenv("MAM_DIST_NT");
        return e ? atoi(e) : -1;
    }();
    int v = c->dist_nt >= 0 ? c->dist_nt : forced;
    if (!(v == 0 || v == 256 || v == 512 || v == 1024)) v = F <= 4 ? 1024 : 256;
    // a width whose LDS does not fit this geometry (large extractors, e.g. Tracking.cc:606's 5x init extractor at
    // 1800-2500 features): the next narrower one, down to the round-3 kernel
    while (v > 0 && !c->dist2_ok[v == 1024 ? 2 : v == 512 ? 1 : 0]) v = v == 256 ? 0 : v / 2;
    return v;
}

// k_fast_chunks for every launch (MAM_FAST_CHUNKS=1 / the context option; default off until measured), when the
// geometry has a chunk plane pitch
bool fast_chunks_enabled(const mam_orb_ctx* c) {
    static const int env = [] {
        const char* e = getenv("MAM_FAST_CHUNKS");
        return e ? atoi(e) : -1;
    }();
    const int v = c->fast_chunks >= 0 ? c->fast_chunks : env;
    return v == 1 && c->fastc_cw > 0;
}

// FAST + blur in one launch (k_fast_blur) for up to 4 frames per call (latency: one dependent launch less);
// MAM_FAST_BLUR=0 / 1 or the context option override
bool fast_blur_enabled(const mam_orb_ctx* c, int F) {
    static const int env = [] {
        const char* e = getenv("MAM_FAST_BLUR");
        return e ? atoi(e) : -1;
    }();
    const int v = c->fast_blur >= 0 ? c->fast_blur : env;
    if (v == 0 || v == 1) return v == 1;
    return F <= 4;
}

// Latency mode (run_pipeline's three-stream dataflow) for up to 4 frames per call; MAM_ORB_FORK=0 / the context
// option turn it off (one stream, stages in order).
bool fork_enabled(const mam_orb_ctx* c, int F, int nt) {
    static const int env = [] {
        const char* e = getenv("MAM_ORB_FORK");
        return e ? atoi(e) : -1;
    }();
    const int v = c->fork >= 0 ? c->fork : env;
    if (v != 1 || nt == 0 || !c->side[0]) return false;   // default off: the cross-stream waits (~7-13 us each on
    return F <= 4;                                         // MI355X) cost more than the overlap gains (c1 0.117 vs 0.094 ms)
}

int run_pipeline(mam_orb_ctx* c, const uint8_t* d_in, int F, size_t stride, size_t fstride, int lap0, int lap1,
                 mam_keypoint* d_kps, uint8_t* d_desc, int capacity, int32_t* d_counts, hipStream_t s) {
    const mam::Geom& g = c->geom;
    const int L = g.nlevels;
    mam::LevelSrc src{d_in, stride, fstride, c->d_pyr.p};
    auto launch_pyramid = [&](hipStream_t s) {
        if (mam_orb_ctx::PyrPlan* pp = choose_pyr_plan(c, F)) {
            // a band's rows per level are few (c1: ~6-20): 1024 threads spread each level over ~1-3 rows per thread
            hipLaunchKernelGGL(mam::k_pyr_bands<1024>, dim3(pp->nb, F), dim3(1024), pp->lds, s, c->d_geom.p, src,
                               c->d_pyr.p, pp->bands.p, pp->buf1_off, pp->rc_off, pp->qc_off, pp->qtot);
        } else {
            // k_pyr_flat reads whole source words: level 0 rows must be word-aligned and a multiple of 4 wide (the
            // last word of the frame's last row must not run past the caller's buffer)
            const bool flat = pyr_flat_enabled() && ((stride | (size_t)d_in | (size_t)g.L[0].w) & 3) == 0;
            const size_t lds = (size_t)g.pyr_seg_w * g.pyr_rows + 16;   // pyr_quad's window past the last row
            for (int l = 1; l < L; l++) {
                const mam::LevelGeom& lv = g.L[l];
                if (flat) {
                    const int rq = pyr_rows_per_thread();
                    const long long nq = (long long)((lv.w + 3) / 4) * ((lv.h + rq - 1) / rq);
                    const dim3 pg((int)((nq + 255) / 256), F);
                    switch (rq) {
                        case 1: hipLaunchKernelGGL(mam::k_pyr_flat<1>, pg, dim3(256), 0, s, c->d_geom.p, l, src, c->d_pyr.p); break;
                        case 2: hipLaunchKernelGGL(mam::k_pyr_flat<2>, pg, dim3(256), 0, s, c->d_geom.p, l, src, c->d_pyr.p); break;
                        default: hipLaunchKernelGGL(mam::k_pyr_flat<4>, pg, dim3(256), 0, s, c->d_geom.p, l, src, c->d_pyr.p); break;
                    }
                } else {
                    dim3 grid((lv.w + mam::PYR_XB - 1) / mam::PYR_XB, (lv.h + mam::PYR_RB - 1) / mam::PYR_RB, F);
                    hipLaunchKernelGGL(mam::k_pyr_down, grid, dim3(256), lds, s, c->d_geom.p, l, src, c->d_pyr.p);
                }
            }
        }
    };
    auto launch_fast = [&](hipStream_t st, int cell_first, int ncells) {
        const dim3 fg(ncells, F), fb(mam::FAST_THREADS);
        switch (c->fast_cw) {
            case 24: hipLaunchKernelGGL(mam::k_fast_cells<24>, fg, fb, c->fast_lds, st, c->d_geom.p, c->d_cells.p, src,
                                        c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, cell_first); break;
            case 32: hipLaunchKernelGGL(mam::k_fast_cells<32>, fg, fb, c->fast_lds, st, c->d_geom.p, c->d_cells.p, src,
                                        c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, cell_first); break;
            case 40: hipLaunchKernelGGL(mam::k_fast_cells<40>, fg, fb, c->fast_lds, st, c->d_geom.p, c->d_cells.p, src,
                                        c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, cell_first); break;
            default: hipLaunchKernelGGL(mam::k_fast_cells<48>, fg, fb, c->fast_lds, st, c->d_geom.p, c->d_cells.p, src,
                                        c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, cell_first); break;
        }
    };
    const bool chunked = fast_chunks_enabled(c);
    // FAST over the cells of levels [l0, l1)
    auto launch_fast_levels = [&](hipStream_t st, int l0, int l1) {
        if (chunked) {
            const int c0 = c->chunk_base[l0], n = c->chunk_base[l1] - c0;
            if (n <= 0) return;
            const dim3 fg(n, F), fb(mam::FAST_THREADS);
#define MAM_FASTC(CW_)                                                                                                \
    case CW_: hipLaunchKernelGGL(mam::k_fast_chunks<CW_>, fg, fb, c->fastc_lds, st, c->d_geom.p, c->d_chunks.p,       \
                                 c->d_cells.p, src, c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast,                 \
                                 c->prm.min_th_fast, c0); break
            switch (c->fastc_cw) {
                MAM_FASTC(64); MAM_FASTC(80); MAM_FASTC(96); MAM_FASTC(112); MAM_FASTC(128); MAM_FASTC(160);
                default: break;
            }
#undef MAM_FASTC
            return;
        }
        const int cf = g.L[l0].cell_base, cl = l1 < L ? g.L[l1].cell_base : g.cells_per_frame;
        launch_fast(st, cf, cl - cf);
    };
    const int nt = dist_threads(c, F);
    auto launch_dist = [&](hipStream_t st, int l_first, int nl) {
        if (nt == 0) {   // the round-3 kernel (all levels)
            hipLaunchKernelGGL(mam::k_distribute, dim3(L, F), dim3(256), c->dist_lds, st, c->d_geom.p, c->d_cellcnt.p,
                               c->d_cand.p, c->d_keys.p, c->d_knode.p, c->d_okey.p, c->d_orank.p, c->d_lvlcnt.p, lap0,
                               lap1, c->dist_kcap);
            return;
        }
        const int li = nt == 1024 ? 2 : nt == 512 ? 1 : 0;
        const size_t lds = c->dist2_lds[li];
#define MAM_DIST2_LAUNCH(NT_, KPT_)                                                                                   \
    hipLaunchKernelGGL((mam::k_distribute2<NT_, KPT_>), dim3(nl, F), dim3(NT_), lds, st, c->d_geom.p, c->d_cellcnt.p, \
                       c->d_cand.p, c->d_keys.p, c->d_knode32.p, c->d_okey.p, c->d_orank.p, c->d_lvlcnt.p, lap0, lap1,  \
                       l_first)
        if (nt == 1024) MAM_DIST2_LAUNCH(1024, 8);
        else if (nt == 512) MAM_DIST2_LAUNCH(512, 16);
        else MAM_DIST2_LAUNCH(256, 16);
#undef MAM_DIST2_LAUNCH
    };
    if (fork_enabled(c, F, nt)) {
        // latency mode (a few frames): the stages as a dataflow over three streams. Level 0's FAST cells and its
        // DistributeOctTree need only the input frame, so they run beside the pyramid; the blur of every level runs
        // beside FAST + DistributeOctTree of levels >= 1; the descriptors join both.
        //   side A: FAST(level 0) -> DistributeOctTree(level 0)
        //   s:      pyramid -> FAST(levels >= 1) -> DistributeOctTree(levels >= 1) -> [join A, B] -> describe
        //   side B: [pyramid] -> blur (all levels)
        MAM_HIP(hipEventRecord(c->ev_fork, s));
        MAM_HIP(hipStreamWaitEvent(c->side[0], c->ev_fork, 0));
        launch_fast_levels(c->side[0], 0, 1);
        launch_dist(c->side[0], 0, 1);
        MAM_HIP(hipEventRecord(c->ev_side[0], c->side[0]));
        launch_pyramid(s);
        MAM_HIP(hipEventRecord(c->ev_pyr, s));
        MAM_HIP(hipStreamWaitEvent(c->side[1], c->ev_pyr, 0));
        hipLaunchKernelGGL(mam::k_blur7, dim3((g.tiles_per_frame + mam::BLUR_TPB - 1) / mam::BLUR_TPB, F), dim3(256), 0,
                           c->side[1], c->d_geom.p, src, c->d_blur.p);
        MAM_HIP(hipEventRecord(c->ev_side[1], c->side[1]));
        if (L > 1) {
            launch_fast_levels(s, 1, L);
            launch_dist(s, 1, L - 1);
        }
        MAM_HIP(hipStreamWaitEvent(s, c->ev_side[0], 0));
        MAM_HIP(hipStreamWaitEvent(s, c->ev_side[1], 0));
    } else {
        {
            StageScope sc(&c->timer, s, MAM_STAGE_PYRAMID);
            launch_pyramid(s);
        }
        if (!chunked && fast_blur_enabled(c, F)) {
            // one launch: every cell's FAST and the blur tile groups (the blur's time counts in the FAST stage)
            StageScope sc(&c->timer, s, MAM_STAGE_FAST);
            const int ng = (g.tiles_per_frame + mam::BLUR_TPB - 1) / mam::BLUR_TPB;
            const dim3 fg(g.cells_per_frame + ng, F), fb(mam::FAST_THREADS);
            const size_t lds = std::max(c->fast_lds, mam::BLUR_LDS_BYTES);
#define MAM_FASTB(CW_)                                                                                                \
    case CW_: hipLaunchKernelGGL(mam::k_fast_blur<CW_>, fg, fb, lds, s, c->d_geom.p, c->d_cells.p, src, c->d_cand.p,   \
                                 c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, 0, g.cells_per_frame,         \
                                 c->d_blur.p); break
            switch (c->fast_cw) {
                MAM_FASTB(24); MAM_FASTB(32); MAM_FASTB(40);
                default: hipLaunchKernelGGL(mam::k_fast_blur<48>, fg, fb, lds, s, c->d_geom.p, c->d_cells.p, src,
                                            c->d_cand.p, c->d_cellcnt.p, c->prm.ini_th_fast, c->prm.min_th_fast, 0,
                                            g.cells_per_frame, c->d_blur.p); break;
            }
#undef MAM_FASTB
        } else {
            // (blur and FAST both keep the CUs' issue slots busy in a batch: running the blur on a second stream
            // beside FAST + DistributeOctTree measured no gain there, so batches keep the stages in order)
            {
                StageScope sc(&c->timer, s, MAM_STAGE_BLUR);
                hipLaunchKernelGGL(mam::k_blur7, dim3((g.tiles_per_frame + mam::BLUR_TPB - 1) / mam::BLUR_TPB, F),
                                   dim3(256), 0, s, c->d_geom.p, src, c->d_blur.p);
            }
            {
                StageScope sc(&c->timer, s, MAM_STAGE_FAST);
                launch_fast_levels(s, 0, L);
            }
        }
        {
            StageScope sc(&c->timer, s, MAM_STAGE_DISTRIBUTE);
            launch_dist(s, 0, L);
        }
    }
    {
        StageScope sc(&c->timer, s, MAM_STAGE_DESCRIBE);
        const long long waves = (long long)F * g.kp_slots;
        const int blocks = (int)((waves + 3) / 4);
        hipLaunchKernelGGL(mam::k_describe, dim3(blocks), dim3(256), 0, s, c->d_geom.p, src, c->d_blur.p,
                           c->d_okey.p, c->d_orank.p, c->d_lvlcnt.p, F, d_kps, d_desc, capacity, d_counts,
                           c->prm.fp_policy);
    }
    MAM_HIP(hipGetLastError());
#ifdef MAM_PYR_PROFILE
    {
        static int callsp = 0;
        if (++callsp % 50 == 0) {
            unsigned long long h[10];
            MAM_HIP(hipStreamSynchronize(s));
            MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::g_pyrprof), sizeof(h)));
            const double n = h[9] ? (double)h[9] : 1.0;
            fprintf(stderr, "pyrprof W%d F%d bands/launch %.1f: prologue %.0f", g.L[0].w, F, n / 50.0, h[0] / n);
            for (int l = 1; l < 9; l++) fprintf(stderr, " l%d %.0f", l, h[l] / n);
            fprintf(stderr, "\n");
            unsigned long long zero[10] = {};
            MAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mam::g_pyrprof), zero, sizeof(zero)));
        }
    }
#endif
#ifdef MAM_DIST2_PROFILE
    {
        static int calls2 = 0;
        if (++calls2 % 50 == 0) {
            unsigned long long h[8][13];
            MAM_HIP(hipStreamSynchronize(s));
            MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::g_d2prof), sizeof(h)));
            for (int l = 0; l < 8; l++) {
                const double n = h[l][11] ? (double)h[l][11] : 1.0;
                fprintf(stderr, "d2prof W%d L%d l%d: init %.0f - %.0f - %.0f cut %.0f kept %.0f write %.0f "
                        "pass %.0f out %.0f | final its %.2f p1 rounds %.2f mean m %.1f | sort %.0f\n", g.L[0].w,
                        c->prm.nfeatures, l, h[l][0] / n, h[l][1] / n, h[l][2] / n, h[l][3] / n, h[l][4] / n, h[l][5] / n,
                        h[l][6] / n, h[l][7] / n, h[l][8] / n, h[l][9] / n, h[l][8] ? (double)h[l][10] / h[l][8] : 0.0,
                        h[l][12] / n);
            }
            unsigned long long zero[8][13] = {};
            MAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mam::g_d2prof), zero, sizeof(zero)));
        }
    }
#endif
#ifdef MAM_DIST_PROFILE
    {
        static int calls = 0;
        if (++calls % 20 == 0) {
            unsigned long long h[8];
            MAM_HIP(hipStreamSynchronize(s));
            MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::g_dprof), sizeof(h)));
            fprintf(stderr, "distribute cycles (sum over WGs): init %llu rounds %llu pre-sort %llu sort %llu final %llu "
                    "out %llu; sorts %llu mean m %.1f\n", h[0], h[1], h[2], h[3], h[4], h[5], h[7],
                    h[7] ? (double)h[6] / h[7] : 0.0);
        }
    }
#endif
    c->last_in0 = d_in;
    c->last_stride = stride;
    c->last_fstride = fstride;
    c->last_nframes = F;
    return MAM_OK;
}

bool valid_params(const mam_orb_params* p) {
    return p && p->nlevels >= 1 && p->nlevels <= MAM_MAX_LEVELS && p->nfeatures >= 0 && p->scale_factor > 1.0f &&
           p->ini_th_fast >= 0 && p->ini_th_fast <= 255 && p->min_th_fast >= 0 && p->min_th_fast <= 255;
}

}  // namespace

extern "C" {

const char* mam_last_error(void) { return g_last_error.c_str(); }

int mam_orb_create(const mam_orb_params* params, int device, mam_orb_ctx** out) {
    if (!out || !valid_params(params)) return MAM_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    MAM_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) { g_last_error = "no such HIP device"; return MAM_ERR_ARG; }
    MAM_DEVICE_SCOPE(device);
    mam_orb_ctx* c = new mam_orb_ctx();
    c->prm = *params;
    c->device = device;
    build_tables(c);
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; i++) e = hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_pyr, hipEventDisableTiming);
    for (int i = 0; i < 2 && e == hipSuccess; i++) e = hipEventCreateWithFlags(&c->ev_side[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        g_last_error = hipGetErrorString(e);
        delete c;
        return MAM_ERR_DEVICE;
    }
    *out = c;
    return MAM_OK;
}

void mam_orb_destroy(mam_orb_ctx* c) {
    if (!c) return;
    ::mam::DeviceScope mam_dev_scope_(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->d_geom.release(); c->d_cells.release(); c->d_chunks.release(); c->d_tabs_i.release(); c->d_tabs_s.release();
    c->d_pyr.release(); c->d_blur.release(); c->d_input.release();
    c->d_cand.release(); c->d_keys.release(); c->d_okey.release(); c->d_orank.release(); c->d_knode.release(); c->d_knode32.release();
    c->d_cellcnt.release(); c->d_lvlcnt.release(); c->d_kps.release(); c->d_desc.release(); c->d_counts.release(); c->d_out.release();
    for (int i = 0; i < 2; i++) {
        if (c->side[i]) { (void)hipStreamSynchronize(c->side[i]); (void)hipStreamDestroy(c->side[i]); }
        if (c->ev_side[i]) (void)hipEventDestroy(c->ev_side[i]);
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_pyr) (void)hipEventDestroy(c->ev_pyr);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mam_orb_levels(const mam_orb_ctx* c) { return c ? c->prm.nlevels : MAM_ERR_ARG; }

int mam_orb_scales(const mam_orb_ctx* c, float* out) {
    if (!c || !out) return MAM_ERR_ARG;
    const int L = c->prm.nlevels;
    for (int l = 0; l < L; l++) {
        out[l] = c->scale[l]; out[L + l] = c->invScale[l];
        out[2 * L + l] = c->sigma2[l]; out[3 * L + l] = c->invSigma2[l];
    }
    return MAM_OK;
}

int mam_orb_features_per_level(const mam_orb_ctx* c, int32_t* out) {
    if (!c || !out) return MAM_ERR_ARG;
    for (int l = 0; l < c->prm.nlevels; l++) out[l] = c->nPerLevel[l];
    return MAM_OK;
}

int mam_orb_max_keypoints(const mam_orb_ctx* c) {
    if (!c) return MAM_ERR_ARG;
    int s = 0;
    for (int l = 0; l < c->prm.nlevels; l++) s += c->nPerLevel[l] + 3;
    return s;
}

int mam_orb_extract_batch_device(mam_orb_ctx* c, const uint8_t* d_imgs, int nframes, int w, int h, size_t stride,
                                 size_t frame_stride, int lap0, int lap1, mam_keypoint* d_kps, uint8_t* d_desc,
                                 int capacity, int32_t* d_counts, void* stream) {
    if (!c || !d_imgs || nframes <= 0 || w <= 0 || h <= 0 || stride < (size_t)w || !d_kps || !d_desc || !d_counts ||
        capacity < 0)
        return MAM_ERR_ARG;
    if (nframes > 1 && frame_stride < stride * h) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    if (int rc = ensure_geometry(c, w, h, nframes)) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return run_pipeline(c, d_imgs, nframes, stride, frame_stride, lap0, lap1, d_kps, d_desc, capacity, d_counts, s);
}

int mam_orb_extract(mam_orb_ctx* c, const uint8_t* img, int w, int h, size_t stride, int lap0, int lap1,
                    mam_keypoint* kps, uint8_t* desc, int capacity, int* n_out, int* mono_out) {
    if (!c || !n_out || !mono_out) return MAM_ERR_ARG;
    *n_out = 0;
    *mono_out = 0;
    if (!img || w <= 0 || h <= 0) return MAM_ERR_EMPTY;
    if (stride < (size_t)w || capacity < 0) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    if (int rc = ensure_geometry(c, w, h, 1)) return rc;
    const int kcap = c->geom.kp_slots;
    // device / pinned block: counts (64 B) | kcap keypoints | kcap descriptors
    const size_t kp_off = 64, desc_off = (kp_off + sizeof(mam_keypoint) * (size_t)kcap + 15) & ~(size_t)15;
    const size_t out_bytes = desc_off + (size_t)kcap * 32;
    const size_t in_bytes = (size_t)w * h;
    if (int rc = c->d_input.alloc(in_bytes + 64)) return rc;   // k_pyr_flat may read up to 3 bytes past the frame
    if (int rc = c->d_out.alloc(out_bytes)) return rc;
    if (int rc = c->h_in.alloc(in_bytes)) return rc;
    if (int rc = c->h_out.alloc(out_bytes)) return rc;
    // MAM_ORB_HOST_PROFILE=1: the call's host phases (microseconds, averaged over 200 calls) on stderr
    static const bool hprof = [] {
        const char* e = getenv("MAM_ORB_HOST_PROFILE");
        return e && atoi(e) == 1;
    }();
    using hclock = std::chrono::steady_clock;
    hclock::time_point ht[7];
    if (hprof) ht[0] = hclock::now();
    if (stride == (size_t)w) std::memcpy(c->h_in.p, img, in_bytes);
    else
        for (int y = 0; y < h; y++) std::memcpy(c->h_in.p + (size_t)y * w, img + (size_t)y * stride, w);
    if (hprof) ht[1] = hclock::now();
    MAM_HIP(hipMemcpyAsync(c->d_input.p, c->h_in.p, in_bytes, hipMemcpyHostToDevice, c->stream));
    if (hprof) ht[2] = hclock::now();
    // the descriptor kernel writes the counts, keypoints and descriptors straight into the pinned host block (its
    // device mapping): no device-to-host copy launch after it (MAM_ORB_ZERO_COPY_OUT=0: the copy)
    static const bool zc_out = [] {
        const char* e = getenv("MAM_ORB_ZERO_COPY_OUT");
        return !(e && atoi(e) == 0);
    }();
    uint8_t* outp = c->d_out.p;
    if (zc_out) {
        void* dp = nullptr;
        MAM_HIP(hipHostGetDevicePointer(&dp, c->h_out.p, 0));
        outp = static_cast<uint8_t*>(dp);
    }
    int32_t* d_cnt = reinterpret_cast<int32_t*>(outp);
    mam_keypoint* d_kp = reinterpret_cast<mam_keypoint*>(outp + kp_off);
    uint8_t* d_ds = outp + desc_off;
    if (int rc = run_pipeline(c, c->d_input.p, 1, w, in_bytes, lap0, lap1, d_kp, d_ds, kcap, d_cnt, c->stream))
        return rc;
    if (hprof) ht[3] = hclock::now();
    if (!zc_out) MAM_HIP(hipMemcpyAsync(c->h_out.p, c->d_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
    if (hprof) ht[4] = hclock::now();
    MAM_HIP(hipStreamSynchronize(c->stream));
    if (hprof) ht[5] = hclock::now();
    struct HostProf {
        double acc[6] = {};
        int n = 0;
    };
    static HostProf hp;
    int32_t cnt[2];
    std::memcpy(cnt, c->h_out.p, sizeof(cnt));
    if (cnt[0] < 0) { g_last_error = "internal keypoint slot overflow"; return MAM_ERR_DEVICE; }
    *n_out = cnt[0];
    if (cnt[0] > capacity || (cnt[0] > 0 && (!kps || !desc))) return MAM_ERR_CAPACITY;
    *mono_out = cnt[1];
    if (cnt[0] > 0) {
        std::memcpy(kps, c->h_out.p + kp_off, sizeof(mam_keypoint) * (size_t)cnt[0]);
        std::memcpy(desc, c->h_out.p + desc_off, (size_t)cnt[0] * 32);
    }
    if (hprof) {
        ht[6] = hclock::now();
        for (int k = 0; k < 6; k++) hp.acc[k] += std::chrono::duration<double, std::micro>(ht[k + 1] - ht[k]).count();
        if (++hp.n == 200) {
            fprintf(stderr, "orb host %dx%d: memcpy-in %.1f h2d-enqueue %.1f pipeline-enqueue %.1f d2h-enqueue %.1f "
                    "sync-wait %.1f copy-out %.1f us (out %zu B)\n", w, h, hp.acc[0] / 200, hp.acc[1] / 200,
                    hp.acc[2] / 200, hp.acc[3] / 200, hp.acc[4] / 200, hp.acc[5] / 200, out_bytes);
            hp = HostProf{};
        }
    }
    return MAM_OK;
}

int mam_orb_get_level(mam_orb_ctx* c, int frame, int level, uint8_t* out, int* w_out, int* h_out) {
    if (!c || level < 0 || level >= c->prm.nlevels || frame < 0 || frame >= c->last_nframes || !c->last_in0)
        return MAM_ERR_ARG;
    const mam::LevelGeom& lv = c->geom.L[level];
    if (w_out) *w_out = lv.w;
    if (h_out) *h_out = lv.h;
    if (!out) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    MAM_HIP(hipStreamSynchronize(c->stream));
    const uint8_t* src;
    size_t pitch;
    if (level == 0) { src = c->last_in0 + (size_t)frame * c->last_fstride; pitch = c->last_stride; }
    else { src = c->d_pyr.p + lv.pyr_off + (size_t)frame * lv.frame_bytes; pitch = lv.pitch; }
    MAM_HIP(hipMemcpy2D(out, lv.w, src, pitch, lv.w, lv.h, hipMemcpyDeviceToHost));
    return MAM_OK;
}

int mam_orb_debug_blurred(mam_orb_ctx* c, int frame, int level, uint8_t* out) {
    if (!c || !out || level < 0 || level >= c->prm.nlevels || frame < 0 || frame >= c->last_nframes)
        return MAM_ERR_ARG;
    const mam::LevelGeom& lv = c->geom.L[level];
    MAM_DEVICE_SCOPE(c->device);
    MAM_HIP(hipStreamSynchronize(c->stream));
    MAM_HIP(hipMemcpy2D(out, lv.w, c->d_blur.p + lv.blur_off + (size_t)frame * lv.frame_bytes, lv.pitch, lv.w, lv.h,
                        hipMemcpyDeviceToHost));
    return lv.w * lv.h;
}

int mam_orb_debug_candidates(mam_orb_ctx* c, int frame, int level, uint32_t* out, int capacity) {
    if (!c || level < 0 || level >= c->prm.nlevels || frame < 0 || frame >= c->last_nframes) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    MAM_HIP(hipStreamSynchronize(c->stream));
    const mam::LevelGeom& lv = c->geom.L[level];
    std::vector<int> cnt(lv.ncells);
    MAM_HIP(hipMemcpy(cnt.data(), c->d_cellcnt.p + (size_t)frame * c->geom.cells_per_frame + lv.cell_base,
                      sizeof(int) * lv.ncells, hipMemcpyDeviceToHost));
    std::vector<uint32_t> slots((size_t)lv.cand_cap);
    MAM_HIP(hipMemcpy(slots.data(), c->d_cand.p + (size_t)frame * c->geom.cand_per_frame + lv.cand_base,
                      sizeof(uint32_t) * lv.cand_cap, hipMemcpyDeviceToHost));
    int n = 0;
    for (int i = 0; i < lv.ncells; i++)
        for (int k = 0; k < cnt[i]; k++) {
            if (out && n < capacity) out[n] = slots[(size_t)i * lv.cellcap + k];
            n++;
        }
    return n;
}

int mam_orb_debug_set_option(mam_orb_ctx* c, int option, int value) {
    if (!c) return MAM_ERR_ARG;
    switch (option) {
        case MAM_ORB_OPT_DISTRIBUTE_THREADS:
            if (value != -1 && value != 0 && value != 256 && value != 512 && value != 1024) return MAM_ERR_ARG;
            c->dist_nt = value;
            return MAM_OK;
        case MAM_ORB_OPT_FAST_CHUNKS:
            if (value < -1 || value > 1) return MAM_ERR_ARG;
            c->fast_chunks = value;
            return MAM_OK;
        case MAM_ORB_OPT_FORK:
            if (value < -1 || value > 1) return MAM_ERR_ARG;
            c->fork = value;
            return MAM_OK;
        case MAM_ORB_OPT_FAST_BLUR:
            if (value < -1 || value > 1) return MAM_ERR_ARG;
            c->fast_blur = value;
            return MAM_OK;
        default: return MAM_ERR_ARG;
    }
}

int mam_orb_set_profiling(mam_orb_ctx* c, int enable) {
    if (!c) return MAM_ERR_ARG;
    c->timer.reset(enable != 0);
    return MAM_OK;
}

int mam_orb_stage_times(mam_orb_ctx* c, double* ms_out, int64_t* launches_out) {
    if (!c) return MAM_ERR_ARG;
    c->timer.collect();
    for (int i = 0; i < MAM_STAGE_COUNT; i++) {
        if (ms_out) ms_out[i] = c->timer.ms[i];
        if (launches_out) launches_out[i] = c->timer.n[i];
    }
    return MAM_OK;
}

}  // extern "C"
