/*
 * orb_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference ORB path used as the
 * parity checker (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg). Never linked into
 * the product library (mam3slam_amd/).
 *
 * Parity status: the reference cannot be built here (OpenCV/Eigen/Boost absent) and
 * ships no golden vectors, so the OpenCV-4.5.4 primitives below are restated from their published
 * algorithms: "parity unpinned" against the reference binary. Hand-derived
 * known-answer tests pin the pieces that can be pinned (tests/test_oracle_kat.py).
 */
#ifndef MAM_ORB_ORACLE_H
#define MAM_ORB_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/mam_orb.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full ORBextractor::operator() restatement. Same argument meaning as mam_orb_extract. */
int oracle_orb_extract(const mam_orb_params* p, const uint8_t* img, int w, int h, size_t stride,
                       int lap0, int lap1, mam_keypoint* kps, uint8_t* desc, int capacity,
                       int* n_out, int* mono_out);

/* Constructor tables: scales[4*nlevels] (scale, inv, sigma2, invsigma2), nfeat[nlevels], umax[16]. */
int oracle_orb_tables(const mam_orb_params* p, float* scales, int32_t* nfeat, int32_t* umax);

/* Pyramid: level sizes and pixels (level l at out + offsets[l], pitch = level width). */
int oracle_orb_pyramid(const mam_orb_params* p, const uint8_t* img, int w, int h, size_t stride,
                       int32_t* sizes /* 2*nlevels */, uint8_t* out, size_t out_cap);

/* cv::resize(src, dst, Size(dw,dh), 0, 0, INTER_LINEAR), CV_8UC1. */
void oracle_resize_linear(const uint8_t* src, int sw, int sh, size_t sstride, uint8_t* dst, int dw, int dh);

/* cv::FAST(roi, kps, threshold, nonmax=true), TYPE_9_16, on an arbitrary ROI. out = packed (x | y<<12 | score<<24). */
int oracle_fast(const uint8_t* roi, int cols, int rows, size_t stride, int threshold, uint32_t* out, int cap);

/* cv::GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) on a continuous CV_8U image. */
void oracle_gaussian7(const uint8_t* src, int w, int h, uint8_t* dst);
void oracle_gaussian7_taps(int32_t* taps7);

/* cv::fastAtan2 (degrees). */
float oracle_fast_atan2(float y, float x);

/* Deterministic (float)cos((double)a), (float)sin((double)a) (DESIGN.md §Parity policy). */
void oracle_sincos(float a, float* s, float* c);
/* sin/cos of the rBRIEF steering angle under an fp_policy (mam_orb.h MAM_FP_*; 0 = glibc 2.35 sincosf, FMA build). */
void oracle_sincos_policy(int fp_policy, float a, float* s, float* c);

/* Per-level FAST candidates (reference order, packed as above, coordinates relative to minBorder)
 * and the DistributeOctTree output for level `level`. Returns counts via *ncand / *nkeep. */
int oracle_level_stage(const mam_orb_params* p, const uint8_t* img, int w, int h, size_t stride, int level,
                       uint32_t* cand, int cand_cap, int* ncand, uint32_t* kept, int kept_cap, int* nkeep);

/* DistributeOctTree on a caller-provided candidate list (packed as above). */
int oracle_distribute(const uint32_t* cand, int n, int minX, int maxX, int minY, int maxY, int N,
                      uint32_t* out, int cap);

/* libstdc++ std::sort on (key, payload) pairs compared by key only — used to validate the device
 * introsort emulation. */
void oracle_std_sort_pairs(uint32_t* keys, uint32_t* payload, int n);

#ifdef __cplusplus
}
#endif
#endif
