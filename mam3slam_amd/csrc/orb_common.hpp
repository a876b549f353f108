// orb_common.hpp — geometry shared by the host orchestration and the gfx950 kernels of the ORB path.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/mam_orb.h"

namespace mam {

constexpr int EDGE_THRESHOLD = 19;
constexpr int PATCH_SIZE = 31;
constexpr int HALF_PATCH_SIZE = 15;
constexpr int PYR_XB = 1024;        // k_pyr_down output columns per workgroup (4 per thread)
constexpr int PYR_RB = 8;           // k_pyr_down output rows per workgroup
#ifndef MAM_BLUR_TW
#define MAM_BLUR_TW 64
#define MAM_BLUR_TH 64
#endif
constexpr int BLUR_TILE_W = MAM_BLUR_TW;   // k_blur7 output tile: 4 px per thread-quad
constexpr int BLUR_TILE_H = MAM_BLUR_TH;
#ifndef MAM_BLUR_TPB
#define MAM_BLUR_TPB 1
#endif
constexpr int BLUR_TPB = MAM_BLUR_TPB;   // k_blur7 tiles per workgroup (next tile's loads overlap this one's passes)

// One pyramid level of the current frame size (all frames in a batch share it).
struct LevelGeom {
    int w, h;               // level size: cvRound(W * invScale[l]) (ORBextractor.cc:1175)
    int pitch;              // row pitch of this level in the pyramid and blur buffers (bytes)
    int pad0;
    long long frame_bytes;  // h * pitch
    long long pyr_off;      // byte offset of frame 0 of this level in the pyramid buffer (l >= 1)
    long long blur_off;     // byte offset of frame 0 of this level in the blurred buffer
    // FAST cell grid (ORBextractor.cc:785-803)
    int minBX, minBY, maxBX, maxBY;
    int nCols, nRows, wCell, hCell;
    int cell_base;          // first entry of this level in the per-frame cell table
    int ncells;             // active cells of this level
    int cellcap;            // candidate slots per cell (bound on NMS survivors in a band)
    int cand_base;          // u32 offset of this level's candidate slots within a frame
    int cand_cap;           // ncells * cellcap
    int nfeat;              // mnFeaturesPerLevel[l]
    int nini;               // initial DistributeOctTree nodes round(W/H) (ORBextractor.cc:559)
    int kp_base;            // first keypoint slot of this level within a frame
    int kp_cap;             // keypoint slots for this level
    float scale;            // mvScaleFactor[l]
    float hX;               // (float)(maxX-minX)/nIni
    int psize;              // (int)(PATCH_SIZE * scale) (ORBextractor.cc:877)
    // bilinear resize tables from level l-1 (l >= 1), built exactly as OpenCV's hal::resize does
    const int* xofs;
    const short* ialpha;    // 2 per dx
    const int* yofs;
    const short* ibeta;     // 2 per dy
    int xmax;               // first dx using the right-edge replicate formula
    int xvec;               // first column using the scalar (>>22) vertical formula
    int tile_base;          // first blur tile of this level within a frame
    int tiles_x, tiles_y;
    int pad1;
    // packed resize coefficients (k_pyr_flat): per output quad two uint4 {base | o0..o3 << 12.. | vec << 28,
    // a0|a1<<16 x4}, per output row int2 {yofs, ibeta0 | ibeta1 << 16}
    const uint4* qcoef;
    const int2* rcoef;
};

struct Geom {
    int nlevels;
    int cells_per_frame;    // active FAST cells over all levels
    int cand_per_frame;     // u32 candidate slots per frame
    int kp_slots;           // keypoint slots per frame (sum of kp_cap)
    int tiles_per_frame;    // blur tiles per frame
    int node_cap;           // DistributeOctTree node capacity (LDS)
    int max_level_cells;
    int roi_max_rows, roi_max_cols;
    int pyr_seg_w, pyr_rows;   // k_pyr_down LDS staging: source bytes per row / source rows per block (max)
    int umax[16];
    LevelGeom L[MAM_MAX_LEVELS];
};

// k_fast_cells: workgroup size and LDS carve for ROIs up to rmax x cmax (two pixel-pair planes | S map | peaks |
// packed count entries). The host rejects geometries beyond FAST_MAX_ENTRIES.
#ifndef MAM_FAST_THREADS
#define MAM_FAST_THREADS 256
#endif
constexpr int FAST_THREADS = MAM_FAST_THREADS;
constexpr int FAST_MAX_ENTRIES = 64;   // (iteration, wave) count entries: ceil(pairs / threads) * waves
__host__ __device__ inline size_t fast_align16(size_t b) { return (b + 15) & ~(size_t)15; }
// plane pitch CW (pairs per parity plane row = S map pitch): one of FAST_CW_CHOICES, >= (cols + 1) / 2 + 2
__host__ __device__ inline int fast_min_cw(int cols) { return ((cols + 1) >> 1) + 2; }
__host__ __device__ inline size_t fast_off_s(int rmax, int cw) { return fast_align16((size_t)rmax * 2 * cw * 4); }
__host__ __device__ inline size_t fast_off_pk(int rmax, int cw) {
    return fast_off_s(rmax, cw) + fast_align16((size_t)(rmax - 4) * cw * 4);
}
__host__ __device__ inline size_t fast_off_cnt(int rmax, int cw) {
    return fast_off_pk(rmax, cw) + fast_align16((size_t)(rmax - 6) * cw * 2);
}
__host__ __device__ inline size_t fast_lds_bytes(int rmax, int cw) { return fast_off_cnt(rmax, cw) + FAST_MAX_ENTRIES * 4; }

// FAST cell descriptor: ROI rows [y0,y1) cols [x0,x1) of level `level`.
struct CellDesc {
    int level;
    int ci, cj;             // cell row / column index
    int x0, y0, x1, y1;
    int slot;               // index of this cell within its level (candidate slot block)
};

}  // namespace mam
