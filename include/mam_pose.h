/*
 * mam_pose.h — C-ABI drop-in boundary for Optimizer::PoseOptimization (gfx950 / MI355X).
 *
 * Replaces the g2o solve of the reference call (src/Optimizer.cc:814-1115) for mono agents with a Pinhole or
 * KannalaBrandt8 camera (include/mam_camera.h; project / projectJac of Pinhole.cpp:35-81, KannalaBrandt8.cpp:46-65,
 * 145-175): one VertexSE3Expmap, EdgeSE3ProjectXYZOnlyPose mono edges (include/OptimizableTypes.h:31-57,
 * src/OptimizableTypes.cpp:49-63) with RobustKernelHuber(sqrt(5.991)), BlockSolver_6_3 + LinearSolverDense
 * (Eigen LDLT, solvers/linear_solver_dense.h:65-118) + OptimizationAlgorithmLevenberg
 * (core/optimization_algorithm_levenberg.cpp:61-169); four rounds of optimize(10), each restarted from the
 * frame's pose, with the chi2 > 5.991 inlier/outlier classification between rounds (edges at level 1 leave
 * the next round) and the robust kernel dropped after round 2 (Optimizer.cc:1001-1100).
 *
 * Pointers become indices: the wrapper passes one edge per keypoint i with mvpMapPoints[i] != NULL, in
 * increasing i (the reference's insertion order, Optimizer.cc:856-895), and maps outlier[e] back to
 * mvbOutlier[i]. The pose comes back in double (SE3Quat); the wrapper casts to float as Frame::SetPose does.
 */
#ifndef MAM_POSE_H
#define MAM_POSE_H

#include <stddef.h>
#include <stdint.h>

#include "mam_camera.h"

#include "mam_match.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One mono observation. 24 bytes. Values are the reference's floats (cast to double on the device, as
 * Eigen's .cast<double>() does). */
typedef struct mam_pose_edge {
    float obs[2];       /* mvKeysUn[i].pt */
    float xw[3];        /* pMP->GetWorldPos() */
    float inv_sigma2;   /* mvInvLevelSigma2[mvKeysUn[i].octave] */
} mam_pose_edge;

/* Per-frame result. */
typedef struct mam_pose_result {
    double q[4];        /* optimised Tcw: unit quaternion x, y, z, w (SE3Quat, normalised, w >= 0) */
    double t[3];
    int32_t n_inliers;  /* PoseOptimization's return: nInitialCorrespondences - nBad (0 if < 3 edges) */
    int32_t rounds;     /* optimisation rounds run (4 unless fewer than 10 edges) */
    int32_t iterations; /* LM iterations over all rounds */
    int32_t lm_trials;  /* LM trials over all rounds */
} mam_pose_result;

typedef struct mam_pose_ctx mam_pose_ctx;

int mam_pose_create(int device, mam_pose_ctx** out);
void mam_pose_destroy(mam_pose_ctx* ctx);

/* One frame, host buffers, synchronous. tcw: the frame's current pose (Frame::GetPose()). outlier[n]:
 * mvbOutlier of edge e after the last round. Returns n_inliers (>= 0) or a negative MAM_ERR_*. */
int mam_pose_optimization(mam_pose_ctx* ctx, const mam_pose* tcw, const mam_camera* cam, int n,
                          const mam_pose_edge* edges, uint8_t* outlier, mam_pose_result* result);

/* Batched, device-resident, asynchronous on `stream` (NULL = the context's stream): frame f has n_edges[f]
 * edges at edges + f * edge_stride and pose tcw[f]; outliers at outlier + f * edge_stride, results[f]. */
int mam_pose_optimization_batch_device(mam_pose_ctx* ctx, int nframes, const mam_pose* tcw, const mam_camera* cam,
                                       const mam_pose_edge* edges, int edge_stride, const int32_t* n_edges,
                                       uint8_t* outlier, mam_pose_result* results, void* stream);

/* The frame side of the call for device-resident tracked frames (the Tracking sequence of bench.py):
 * Optimizer::PoseOptimization's edge build (Optimizer.cc:856-895): frame f's keypoints (kps + f * kp_stride,
 * kp_count[f * count_stride] of them) whose slot holds a MapPoint — match_local[i] >= 0 (index into local_mps of the
 * frame, SearchByProjection(F, vpMapPoints)'s match; may be NULL) else match_last[i] >= 0 (index into last, the motion
 * search's) — one edge each in increasing i with information inv_level_sigma2[octave] (host array of nlevels);
 * n_edges[f] (MAM_ERR_CAPACITY beyond edge_stride) and edge_kp (the keypoint of each edge). Asynchronous. */
int mam_pose_frame_edges_batch_device(mam_pose_ctx* ctx, int nframes, const mam_keypoint* kps, int kp_stride,
                                      const int32_t* kp_count, int count_stride, const float* inv_level_sigma2,
                                      int nlevels, const int32_t* match_last, const mam_last_entry* last,
                                      int last_stride, const int32_t* match_local, const mam_local_mp* local_mps,
                                      int local_stride, mam_pose_edge* edges, int edge_stride, int32_t* n_edges,
                                      int32_t* edge_kp, void* stream);

/* Tracking's use of the result: Frame::SetPose(SE3f(q.cast<float>(), t.cast<float>())) into tcw[f], and with discard
 * the outliers' slots emptied as TrackWithMotionModel does after its PoseOptimization (Tracking.cc:2840-2857):
 * match_last[i] = -1 and taken[i] = 0 (taken may be NULL) for the keypoint of every outlier edge. Asynchronous. */
int mam_pose_frame_update_batch_device(mam_pose_ctx* ctx, int nframes, const mam_pose_result* results, mam_pose* tcw,
                                       const uint8_t* outlier, const int32_t* edge_kp, int edge_stride,
                                       const int32_t* n_edges, int discard, int32_t* match_last, uint8_t* taken,
                                       int kp_stride, void* stream);

/* Largest edge_stride one frame's workgroup can hold (LDS). */
int mam_pose_max_edges(mam_pose_ctx* ctx);

int mam_pose_set_profiling(mam_pose_ctx* ctx, int enable);
/* ms_out/launches_out: [0] the optimisation kernel. */
int mam_pose_stage_times(mam_pose_ctx* ctx, double* ms_out, int64_t* launches_out);

#ifdef __cplusplus
}
#endif
#endif /* MAM_POSE_H */
