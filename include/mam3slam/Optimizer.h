/*
 * MAM3SLAM::Optimizer::LocalBundleAdjustment — the reference entry point (include/Optimizer.h:57,
 * src/Optimizer.cc:1116-1498) with the g2o solve replaced by the gfx950 solver (include/mam_lba.h).
 * The window build (local keyframes by covisibility, local MapPoints, fixed keyframes), the early returns
 * (no fixed keyframe, stop flag), the outlier erase (chi2 > 5.991 || depth <= 0) and the write-back under
 * Map::mMutexMapUpdate follow the reference line by line; only `optimizer.optimize(10)` runs on the GPU.
 * PoseOptimization: the edge setup and write-back of src/Optimizer.cc:814-1115 around the GPU solve.
 */
#ifndef MAM3SLAM_OPTIMIZER_H
#define MAM3SLAM_OPTIMIZER_H

#include <list>
#include <set>
#include <vector>

#include "../mam_lba.h"
#include "../mam_pose.h"
#include "Map.h"

namespace MAM3SLAM {

/* The g2o graph LocalBundleAdjustment builds, in the reference's insertion order (Optimizer.cc:1212-1394). */
struct LocalBAWindow {
    std::list<KeyFrame*> lLocalKeyFrames, lFixedCameras;
    std::list<MapPoint*> lLocalMapPoints;
    int num_fixedKF = 0;
    unsigned long maxKFid = 0;
    /* flattened problem (owned storage for mam_lba_problem) */
    std::vector<KeyFrame*> vpKF;                 /* pose vertices: local then fixed */
    std::vector<MapPoint*> vpMP;
    std::vector<int64_t> pose_id, point_id;
    std::vector<uint8_t> pose_fixed;
    std::vector<double> pose_q, pose_t, point_xyz, edge_obs, edge_inv_sigma2;
    std::vector<int32_t> pose_cam, edge_point, edge_pose;
    std::vector<float> cams;
    std::vector<const GeometricCamera*> camera_list;
    int32_t cam_model = 0;
    /* index of camera c in camera_list (appended with its parameters on first use); every camera of one window
     * must be of the same model (mam_lba_problem.cam_model) */
    int32_t cameraIndex(const GeometricCamera* c);
    mam_lba_problem Problem(int iterations = 10) const;
};

class Optimizer {
public:
    /* Optimizer::PoseOptimization(Frame*) (include/Optimizer.h, src/Optimizer.cc:814-1115), mono frames (Pinhole or KannalaBrandt8): one
     * edge per keypoint with a MapPoint (in keypoint order), the 4-round g2o solve on the GPU (include/mam_pose.h),
     * pFrame->mvbOutlier and the pose written back. Returns nInitialCorrespondences - nBad (0 below 3). */
    static int PoseOptimization(Frame* pFrame);

    static void LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF,
                                      int& num_OptKF, int& num_MPs, int& num_edges);

    /* Optimizer.cc:1118-1180 + vertex/edge setup :1212-1394. Returns false where the reference returns before
     * optimizing because no keyframe is fixed (:1182-1186). */
    static bool BuildLocalBAWindow(KeyFrame* pKF, Map* pMap, LocalBAWindow& w);
    /* Optimizer.cc:1413-1497, the part of LocalBundleAdjustment after the solve: erase the observations of edges with
     * chi2 > 5.991 or a non-positive depth, then under Map::mMutexMapUpdate write the local keyframes' poses (q / t
     * per pose of w.vpKF, local ones first) and the local points (x per point of w.vpMP) back. */
    static void ApplyLocalBAResult(const LocalBAWindow& w, Map* pMap, const double* q, const double* t,
                                   const double* x, const double* chi2, const uint8_t* depth);

    /* The merge-window (welding) LocalBundleAdjustment, Optimizer.cc:3505-3952 (used when maps are merged,
     * LoopClosing.cc:2670): vpFixedKF fixed, vpAdjustKF optimised, their MapPoints; optimize(5) with Huber
     * (delta sqrt(5.99)), then the edges with chi2 > 5.991 or negative depth set to level 1 and every robust kernel
     * removed, optimize(10) over level 0; outlier erase and write-back of the adjusted keyframes and the points. */
    static void LocalBundleAdjustment(KeyFrame* pMainKF, std::vector<KeyFrame*> vpAdjustKF,
                                      std::vector<KeyFrame*> vpFixedKF, bool* pbStopFlag);

    /* GlobalBundleAdjustemnt / BundleAdjustment (Optimizer.cc:52-390), mono: every non-bad keyframe (the map's
     * initial keyframe fixed) and MapPoint with at least one edge, optimize(nIterations) with Huber kernels if
     * bRobust; written back directly when nLoopKF is the origin keyframe's id, else into mTcwGBA / mPosGBA with
     * mnBAGlobalForKF = nLoopKF. */
    static void GlobalBundleAdjustemnt(Map* pMap, int nIterations = 5, bool* pbStopFlag = nullptr,
                                       const unsigned long nLoopKF = 0, const bool bRobust = true);
    static void BundleAdjustment(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                 int nIterations = 5, bool* pbStopFlag = nullptr, const unsigned long nLoopKF = 0,
                                 const bool bRobust = true);
    /* Optimizer.cc:88-275: the graph BundleAdjustment builds; vbNotIncludedMP[i] = MapPoint i has no edge. */
    static void BuildBAWindow(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                              LocalBAWindow& w, std::vector<bool>& vbNotIncludedMP);

    /* Optimizer.cc:3531-3724: the merge window's vertices (fixed then adjusted keyframes, their MapPoints in
     * GetMapPoints() order) and mono edges; marks mnBALocalForMerge. lLocalKeyFrames = the adjusted keyframes. */
    static void BuildMergeBAWindow(KeyFrame* pMainKF, const std::vector<KeyFrame*>& vpAdjustKF,
                                   const std::vector<KeyFrame*>& vpFixedKF, LocalBAWindow& w);
};

}  // namespace MAM3SLAM
#endif
