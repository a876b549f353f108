/*
 * mam_lba.h — C-ABI drop-in boundary for Optimizer::LocalBundleAdjustment's solve (gfx950 / MI355X).
 *
 * Replaces the g2o section of the reference call (src/Optimizer.cc:1188-1410):
 *   g2o::SparseOptimizer + BlockSolver_6_3 + LinearSolverEigen + OptimizationAlgorithmLevenberg,
 *   VertexSE3Expmap / VertexSBAPointXYZ vertices, EdgeSE3ProjectXYZ mono edges with RobustKernelHuber,
 *   optimizer.initializeOptimization(); optimizer.optimize(10); and the per-edge chi2()/isDepthPositive()
 *   read-back used for outlier rejection (:1413-1460).
 * g2o sources followed: core/optimization_algorithm_levenberg.cpp:61-194, core/block_solver.hpp:353-604,
 *   core/base_binary_edge.hpp:54-120, core/robust_kernel_impl.cpp:76-91, core/sparse_optimizer.cpp:166-190,
 *   355-436, types/se3quat.h, types/types_six_dof_expmap.h:73-76, src/OptimizableTypes.cpp:139-160,
 *   src/CameraModels/Pinhole.cpp:35-81, src/CameraModels/KannalaBrandt8.cpp:46-65, 145-175.
 *
 * The window construction (local / fixed keyframes, local MapPoints), the outlier erase and the write-back
 * under Map::mMutexMapUpdate stay in the host wrapper (mam3slam_amd/lba.py, the analogue of Optimizer.cc:1118-
 * 1186 and :1463-1497), exactly as SURVEY.md §8(b) assigns them.
 */
#ifndef MAM_LBA_H
#define MAM_LBA_H

#include <stddef.h>
#include <stdint.h>

#include "mam_camera.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The g2o graph in reference order. Poses: every KeyFrame vertex (local then fixed, any order); the Hessian
 * column order (g2o _ivMap) is recovered from pose_id / point_id (vertices sorted by id, non-fixed poses
 * first, then points), so callers pass ids exactly as the reference assigns them (KF mnId; MapPoint
 * mnId+maxKFid+1). Edges: insertion order (Optimizer.cc:1252-1331). Doubles are the float map values cast
 * to double, as the reference does (Optimizer.cc:1218, 1235, 1286). */
typedef struct mam_lba_problem {
    int32_t n_poses;
    const int64_t* pose_id;        /* vertex id */
    const uint8_t* pose_fixed;     /* setFixed: init KF / fixed cameras */
    const double* pose_q;          /* [n_poses][4] unit quaternion x, y, z, w (Tcw) */
    const double* pose_t;          /* [n_poses][3] */
    const int32_t* pose_cam;       /* [n_poses] index into cams (NULL = camera 0) */
    int32_t n_points;
    const int64_t* point_id;
    const double* point_xyz;       /* [n_points][3] */
    int32_t n_edges;
    const int32_t* edge_point;     /* vertex 0 (index into points) */
    const int32_t* edge_pose;      /* vertex 1 (index into poses) */
    const double* edge_obs;        /* [n_edges][2] keypoint (mvKeysUn) */
    const double* edge_inv_sigma2; /* information = invSigma2 * I2 */
    int32_t n_cams;
    const float* cams;             /* [n_cams][4] Pinhole fx, fy, cx, cy or [n_cams][8] KannalaBrandt8 fx, fy, cx, cy,
                                      k0..k3 (mvParameters, float), per cam_model */
    double huber_delta;            /* (double)(float)sqrt(5.991); <= 0: no robust kernel (setRobustKernel(0)) */
    int32_t iterations;            /* optimize(10) */
    const uint8_t* edge_active;    /* [n_edges] 1 = level 0, 0 = setLevel(1): left out of the optimisation
                                      (initializeOptimization(0)); NULL = all edges. A vertex left without active
                                      edges keeps its estimate. edge_chi2 of an inactive edge is not written. */
    int32_t cam_model;             /* MAM_CAM_PINHOLE (0) or MAM_CAM_KANNALA_BRANDT8 (1): EdgeSE3ProjectXYZ's
                                      pCamera->project / projectJac (Pinhole.cpp:35-81, KannalaBrandt8.cpp:46-65,
                                      145-175) */
    int32_t n_opt_poses;           /* number of poses with pose_fixed == 0: required by mam_lba_solve_batch_device
                                      (sizes the device work before the flags are read), ignored by mam_lba_solve */
} mam_lba_problem;

typedef struct mam_lba_result {
    double* pose_q;                /* [n_poses][4] (fixed poses copied through) */
    double* pose_t;                /* [n_poses][3] */
    double* point_xyz;             /* [n_points][3] */
    double* edge_chi2;             /* [n_edges] chi2() after optimisation (may be NULL) */
    uint8_t* edge_depth_ok;        /* [n_edges] isDepthPositive() (may be NULL) */
    int32_t iterations;            /* optimize() return: iterations run */
    int32_t lm_trials;             /* total Levenberg trials */
    double initial_chi2;           /* activeRobustChi2 before the first step */
    double final_chi2;             /* activeRobustChi2 at the end */
    int32_t status;                /* 0 ok, 1 aborted by stop flag, <0 MAM_ERR_* */
} mam_lba_result;

typedef struct mam_lba_ctx mam_lba_ctx;

int mam_lba_create(int device, mam_lba_ctx** out);
void mam_lba_destroy(mam_lba_ctx* ctx);

/* Host buffers in, host buffers out; synchronous. stop_flag (may be NULL) is the caller's `bool* pbStopFlag`
 * (one byte, written by another thread): a flag set before the call returns the initial estimate with status 1 and
 * no iteration, like g2o's force-stop test (sparse_optimizer.cpp:377); set during the solve, it is seen between
 * chunks of Levenberg trials (the control flow runs on the device). */
int mam_lba_solve(mam_lba_ctx* ctx, const mam_lba_problem* problem, const volatile uint8_t* stop_flag,
                  mam_lba_result* result);

/* Q independent solves in one set of launches, everything in device memory (the multi-agent / keyframe-batch path):
 * every array pointer of problems[q] and of results[q] (pose_q, pose_t, point_xyz, edge_chi2, edge_depth_ok) is
 * device memory; the problem and result structs themselves are host memory. Contract: poses in ascending pose_id and
 * points in ascending point_id order (g2o's Hessian order, sparse_optimizer.cpp:166-190; pose_id / point_id are not
 * read) and n_opt_poses set. The Levenberg control flow runs on the device: the call enqueues whole iterations of
 * every problem and reads the problems' states back once per chunk of trials (no host round trip per trial);
 * results[q].iterations / lm_trials / initial_chi2 / final_chi2 / status are filled on return. Synchronous. */
int mam_lba_solve_batch_device(mam_lba_ctx* ctx, int n_problems, const mam_lba_problem* problems,
                               mam_lba_result* results, void* stream);

int mam_lba_set_profiling(mam_lba_ctx* ctx, int enable);
/* CU mask (n_words 32-bit words, include/mam_stream.h) of the streams a batch solve splits its problem groups onto
 * besides the caller's stream (which the caller creates with the same mask); n_words 0: every CU. */
int mam_lba_set_cu_mask(mam_lba_ctx* ctx, int n_words, const uint32_t* mask);
/* [0] structure + linearize + blocks, [1] Schur, [2] dense solve, [3] back-substitution + update + chi2 */
int mam_lba_stage_times(mam_lba_ctx* ctx, double* ms_out, int64_t* launches_out);

#ifdef __cplusplus
}
#endif
#endif /* MAM_LBA_H */
