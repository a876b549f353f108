/*
 * MAM3SLAM::ORBmatcher — the reference class (include/ORBmatcher.h:40-93) for the hot-path searches, running on
 * gfx950 through include/mam_match.h. Same constructor, same signatures, same side effects on
 * Frame::mvpMapPoints / vMatchedPairs, same return values. The matcher is a cheap value object like the
 * reference's (constructed on the stack at each call site); device state lives in one per-thread context.
 *
 * Scope: mono agents, Pinhole or KannalaBrandt8 camera (the frame's / keyframe's mpCamera; the KB8 epipolar test and
 * two-view triangulation of SearchForTriangulation included). bMono=false (stereo motion search) and
 * bOnlyStereo=true are not on this path and throw std::invalid_argument / return 0 respectively.
 */
#ifndef MAM3SLAM_ORBMATCHER_H
#define MAM3SLAM_ORBMATCHER_H

#include <utility>
#include <vector>

#include "Map.h"

namespace MAM3SLAM {

class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6f, bool checkOri = true);

    /* ORBmatcher.cc:2058-2074 for one pair; DescriptorDistances for a batch (one launch). */
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b);
    static void DescriptorDistances(const uint8_t* a, const uint8_t* b, int n, int* out);

    /* Tracking::SearchLocalPoints: ORBmatcher.cc:43-213. */
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3,
                           const bool bFarPoints = false, const float thFarPoints = 50.0f);

    /* Tracking::TrackWithMotionModel: ORBmatcher.cc:1676-1887. */
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);

    /* LocalMapping::CreateNewMapPoints: ORBmatcher.cc:907-1146. */
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               const bool bOnlyStereo, const bool bCoarse = false);

    /* LocalMapping::SearchInNeighbors: ORBmatcher.cc:1148-1338 (mono keyframe; bRight=true throws). The search
     * runs on the GPU for every MapPoint at once; the replace-or-add side effects follow in list order. */
    int Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th = 3.0, const bool bRight = false);

    /* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403) for every non-bad MapPoint of the list in one
     * launch (the loop at the end of SearchInNeighbors, LocalMapping.cc:923-935). */
    static void ComputeDistinctiveDescriptors(const std::vector<MapPoint*>& vpMapPoints);

    /* The epipolar quantities SearchForTriangulation derives from the poses (ORBmatcher.cc:913-930,
     * Pinhole.cpp:107-112): F12 row-major and the epipole of KF1's centre in KF2. */
    static void ComputeF12(KeyFrame* pKF1, KeyFrame* pKF2, float F12[9], float ep[2]);

    static const int TH_LOW;
    static const int TH_HIGH;
    static const int HISTO_LENGTH;

protected:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace MAM3SLAM
#endif
