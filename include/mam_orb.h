/*
 * mam_orb.h — C-ABI drop-in boundary for MAM3SLAM's ORB extractor (gfx950 / MI355X).
 *
 * Replaces, one entry point each:
 *   MAM3SLAM::ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
 *                                              reference: include/ORBextractor.h:50-51, src/ORBextractor.cc:409-469
 *   ORBextractor::operator()(image, mask, keypoints, descriptors, vLappingArea)
 *                                              reference: include/ORBextractor.h:58-60, src/ORBextractor.cc:1086-1168
 *   ORBextractor::GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares / GetInverseScaleSigmaSquares
 *                                              reference: include/ORBextractor.h:62-82
 *   ORBextractor::mvImagePyramid (public member, read by stereo code)
 *                                              reference: include/ORBextractor.h:84, src/ORBextractor.cc:1170-1195
 *
 * No torch / OpenCV types cross this boundary: plain pointers, sizes and POD structs.
 * All functions return MAM_OK (0) or a negative MAM_ERR_* code, never throw.
 */
#ifndef MAM_ORB_H
#define MAM_ORB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Byte-for-byte the layout of cv::KeyPoint (pt.x, pt.y, size, angle, response, octave, class_id) = 28 B. */
typedef struct mam_keypoint {
    float x, y;
    float size;
    float angle;
    float response;
    int32_t octave;
    int32_t class_id;
} mam_keypoint;

/* The five ORBextractor constructor arguments (Settings.cc:443-451 keys ORBextractor.*) plus the floating-point
 * policy of the rBRIEF steering. fp_policy = 0 (the default, a zero-initialised struct) is the
 * reference binary's arithmetic: g++ 11.4 -O3 -march=native on an FMA + AVX2 x86-64 host, glibc 2.35
 * (ros:humble, Dockerfile:18):
 *   - sin/cos of the angle (src/ORBextractor.cc:111): glibc 2.35 sincosf, the ifunc's FMA build;
 *   - GET_VALUE (src/ORBextractor.cc:117-119): fma(x, b, y*a) and fma(x, a, -(y*b)), the contraction GCC emits
 *     (vfmadd231ss / vfmsub132ss, asm checked).
 * Flags select other hosts/builds: */
#define MAM_FP_DESC_UNCONTRACTED 1      /* GET_VALUE as two rounded products and a rounded sum (no FMA build) */
#define MAM_FP_TRIG_SSE2 2              /* glibc sincosf SSE2 build (host without FMA/AVX2) */
#define MAM_FP_TRIG_CORRECTLY_ROUNDED 4 /* (float) of the double-precision sin/cos (libm-independent) */
typedef struct mam_orb_params {
    int32_t nfeatures;
    float   scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    int32_t fp_policy;   /* MAM_FP_* flags; 0 = the reference binary */
} mam_orb_params;

enum {
    MAM_OK = 0,
    MAM_ERR_EMPTY = -1,     /* empty image: the reference returns -1 (ORBextractor.cc:1090-1091) */
    MAM_ERR_CAPACITY = -2,  /* caller-owned output buffer too small; *n_out holds the required count */
    MAM_ERR_DEVICE = -3,    /* HIP runtime error */
    MAM_ERR_ARG = -4        /* invalid argument (NULL pointer, nlevels out of range, ...) */
};

#define MAM_MAX_LEVELS 16
#define MAM_DESC_BYTES 32

typedef struct mam_orb_ctx mam_orb_ctx;

/* Create an extractor bound to HIP device `device`. Owns a HIP stream and device scratch. */
int mam_orb_create(const mam_orb_params* params, int device, mam_orb_ctx** out);
void mam_orb_destroy(mam_orb_ctx* ctx);

/* out[0..nlevels) scale, [nlevels..2n) inv scale, [2n..3n) sigma2, [3n..4n) inv sigma2. */
int mam_orb_scales(const mam_orb_ctx* ctx, float* out);
/* mnFeaturesPerLevel (ORBextractor.cc:434-445), nlevels ints. */
int mam_orb_features_per_level(const mam_orb_ctx* ctx, int32_t* out);
int mam_orb_levels(const mam_orb_ctx* ctx);

/* Upper bound on keypoints one frame can yield (nfeatures + 3*nlevels). */
int mam_orb_max_keypoints(const mam_orb_ctx* ctx);

/* Synchronous single-frame call with HOST buffers — the exact semantics of ORBextractor::operator().
 * img: 8-bit grey, w x h, row pitch `stride` bytes. lap0/lap1 = vLappingArea (Frame.cc:311 passes 0,1000).
 * kps/desc: caller-owned, `capacity` entries (desc = capacity*32 bytes).
 * On success *n_out = #keypoints, *mono_out = returned monoIndex. */
int mam_orb_extract(mam_orb_ctx* ctx, const uint8_t* img, int w, int h, size_t stride,
                    int lap0, int lap1, mam_keypoint* kps, uint8_t* desc, int capacity,
                    int* n_out, int* mono_out);

/* Batched, DEVICE-resident: `nframes` frames of the same w x h at d_imgs + f*frame_stride.
 * Outputs for frame f at d_kps + f*capacity, d_desc + f*capacity*32, d_counts[2f] = n, [2f+1] = monoIndex
 * (n = -2 when the frame overflowed `capacity`). Asynchronous on `stream` (NULL = the context's stream). */
int mam_orb_extract_batch_device(mam_orb_ctx* ctx, const uint8_t* d_imgs, int nframes, int w, int h,
                                 size_t stride, size_t frame_stride, int lap0, int lap1,
                                 mam_keypoint* d_kps, uint8_t* d_desc, int capacity, int32_t* d_counts,
                                 void* stream);

/* Copy pyramid level `level` of the last single-frame call into host `out` (w_l x h_l, pitch w_l).
 * w_out / h_out receive the level size. Mirrors the public ORBextractor::mvImagePyramid. */
int mam_orb_get_level(mam_orb_ctx* ctx, int frame, int level, uint8_t* out, int* w_out, int* h_out);

/* Stage timing (HIP events on the context's launch stream), for bench.py's roofline.
 * enable != 0 records an event pair around every stage launch; mam_orb_stage_times returns the
 * summed milliseconds and launch counts per stage since the last reset. */
enum { MAM_STAGE_PYRAMID = 0, MAM_STAGE_FAST = 1, MAM_STAGE_BLUR = 2, MAM_STAGE_DISTRIBUTE = 3,
       MAM_STAGE_DESCRIBE = 4, MAM_STAGE_COUNT = 5 };
int mam_orb_set_profiling(mam_orb_ctx* ctx, int enable);
int mam_orb_stage_times(mam_orb_ctx* ctx, double* ms_out, int64_t* launches_out);

/* Debug taps for staged parity tests (frame f of the last call): per-level FAST candidates as packed
 * u32 (x | y<<12 | score<<24, coordinates relative to the FAST border) in reference order, and the
 * per-level distributed keypoints before orientation. Returns the count or a negative error. */
int mam_orb_debug_candidates(mam_orb_ctx* ctx, int frame, int level, uint32_t* out, int capacity);
int mam_orb_debug_blurred(mam_orb_ctx* ctx, int frame, int level, uint8_t* out);

/* Implementation switches for parity tests and A/B runs (no effect on results):
 * MAM_ORB_OPT_DISTRIBUTE_THREADS: DistributeOctTree workgroup width, 256 / 512 / 1024 (k_distribute2), 0 (the
 * round-3 kernel) or -1 (automatic: 1024 for up to 4 frames per call, else 256).
 * MAM_ORB_OPT_FORK: latency mode for up to 4 frames per call (level 0's FAST + DistributeOctTree beside the pyramid,
 * the blur beside the other levels' FAST, on the context's side streams), 1 on / 0 off / -1 automatic (off: the
 * cross-stream waits cost more than the overlap gains on MI355X).
 * MAM_ORB_OPT_FAST_CHUNKS: FAST over chunks of up to 4 cells of a cell row (k_fast_chunks) instead of one workgroup per
 * cell (k_fast_cells): 1 on / 0 off / -1 automatic.
 * MAM_ORB_OPT_FAST_BLUR: FAST and the blur in one launch (k_fast_blur) instead of two: 1 on / 0 off / -1 automatic
 * (on for up to 4 frames per call). */
enum { MAM_ORB_OPT_DISTRIBUTE_THREADS = 1, MAM_ORB_OPT_FORK = 2, MAM_ORB_OPT_FAST_CHUNKS = 3, MAM_ORB_OPT_FAST_BLUR = 4 };
int mam_orb_debug_set_option(mam_orb_ctx* ctx, int option, int value);

/* Last HIP error string for MAM_ERR_DEVICE. */
const char* mam_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MAM_ORB_H */
