/*
 * Minimal map model: the fields and methods of the reference's Frame, KeyFrame, MapPoint and Map that the hot
 * path reads or writes, with the reference's names, so the ORBmatcher / LocalBundleAdjustment wrappers keep
 * the reference signatures. In the reference these are the real classes (src/Frame.cc, src/KeyFrame.cc,
 * src/MapPoint.cc, src/Map.cc); INTEGRATION.md shows the wrappers compiled against them instead.
 *
 * Scope: mono agents (mvuRight = -1, no second camera), Pinhole or KannalaBrandt8 camera, no IMU. Mutex discipline follows the
 * reference where the hot path takes locks (observations, pose, Map::mMutexMapUpdate).
 */
#ifndef MAM3SLAM_MAP_H
#define MAM3SLAM_MAP_H

#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <vector>

#include "Types.h"

namespace MAM3SLAM {

class ORBextractor;
class ORBVocabulary;
class KeyFrame;
class MapPoint;
class Map;

/* Frame (src/Frame.cc:289-382, mono constructor without BoW / IMU). */
class Frame {
public:
    Frame() = default;
    Frame(const ImageView& imGray, ORBextractor* extractor, const GeometricCamera* pCamera, unsigned long id = 0);

    void SetPose(const SE3f& Tcw) { mTcw = Tcw; mbHasPose = true; }
    const SE3f& GetPose() const { return mTcw; }

    /* mam_frame_geom view of the static image bounds / grid / scale tables (Frame.cc:341-342, 782-809). */
    mam_frame_geom Geom() const;

    unsigned long mnId = 0;
    int N = 0;
    std::vector<KeyPoint> mvKeys, mvKeysUn;
    Mat8U mDescriptors;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    int monoLeft = -1;

    int mnScaleLevels = 0;
    float mfScaleFactor = 0.f;
    float mfLogScaleFactor = 0.f;   /* log(mfScaleFactor) (Frame.cc:313) */
    std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;

    float mnMinX = 0.f, mnMaxX = 0.f, mnMinY = 0.f, mnMaxY = 0.f;
    float mfGridElementWidthInv = 0.f, mfGridElementHeightInv = 0.f;

    const GeometricCamera* mpCamera = nullptr;
    SE3f mTcw;
    bool mbHasPose = false;
};

/* KeyFrame (src/KeyFrame.cc): the copy of a Frame plus covisibility, BA bookkeeping and the BoW feature
 * vector SearchForTriangulation walks. */
class KeyFrame {
public:
    KeyFrame(const Frame& F, Map* pMap, unsigned long id);

    SE3f GetPose();
    SE3f GetPoseInverse();
    void SetPose(const SE3f& Tcw);
    void GetCameraCenter(float Ow[3]);

    std::vector<MapPoint*> GetMapPointMatches();
    std::set<MapPoint*> GetMapPoints();                   /* KeyFrame.cc:325-340: non-NULL, non-bad */
    MapPoint* GetMapPoint(size_t idx);
    void AddMapPoint(MapPoint* pMP, size_t idx);
    void ReplaceMapPointMatch(const int& idx, MapPoint* pMP);   /* KeyFrame.cc:320-323 */
    void EraseMapPointMatch(int idx);
    void EraseMapPointMatch(MapPoint* pMP);

    /* mvpOrderedConnectedKeyFrames (set by the caller's covisibility graph; KeyFrame.cc:237-241). */
    void SetVectorCovisibleKeyFrames(const std::vector<KeyFrame*>& v) { mvpOrderedConnectedKeyFrames = v; }
    std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() { return mvpOrderedConnectedKeyFrames; }

    bool isBad() const { return mbBad; }
    void SetBadFlag() { mbBad = true; }
    Map* GetMap() const { return mpMap; }
    mam_frame_geom Geom() const;

    unsigned long mnId;
    unsigned long mnBALocalForKF = 0, mnBAFixedForKF = 0, mnBALocalForMerge = 0;
    /* global BA results kept for the loop closer (Optimizer.cc:299-300) */
    SE3f mTcwGBA;
    unsigned long mnBAGlobalForKF = 0;
    const int N;
    std::vector<KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight;
    Mat8U mDescriptors;
    int mnScaleLevels;
    float mfLogScaleFactor;
    std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    float mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv;
    const GeometricCamera* mpCamera;
    /* DBoW2::BowVector / FeatureVector (node id -> feature indices, ascending node ids), set by ComputeBoW. */
    std::map<unsigned int, double> mBowVec;
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;
    ORBVocabulary* mpORBvocabulary = nullptr;
    /* KeyFrame.cc:98-107: transform(mDescriptors, mBowVec, mFeatVec, 4) once (on the GPU). */
    void ComputeBoW();

private:
    std::mutex mMutexPose, mMutexFeatures;
    SE3f mTcw, mTwc;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<KeyFrame*> mvpOrderedConnectedKeyFrames;
    bool mbBad = false;
    Map* mpMap;
};

/* MapPoint (src/MapPoint.cc). Observations keyed by KeyFrame* exactly like the reference (std::map order). */
class MapPoint {
public:
    MapPoint(const float Pos[3], KeyFrame* pRefKF, Map* pMap, unsigned long id);

    void GetWorldPos(float Pos[3]);
    void SetWorldPos(const float Pos[3]);
    std::map<KeyFrame*, std::tuple<int, int>> GetObservations();
    int Observations();
    void AddObservation(KeyFrame* pKF, int idx);          /* MapPoint.cc:133-166, mono */
    void EraseObservation(KeyFrame* pKF);                 /* MapPoint.cc:168-201 */
    std::tuple<int, int> GetIndexInKeyFrame(KeyFrame* pKF);
    bool IsInKeyFrame(KeyFrame* pKF);                     /* MapPoint.cc:420-424 */
    void SetBadFlag();                                    /* MapPoint.cc:216-239 */
    bool isBad();
    void Replace(MapPoint* pMP);                          /* MapPoint.cc:248-300 */
    MapPoint* GetReplaced();                              /* MapPoint.cc:241-246 */
    void IncreaseVisible(int n = 1);
    void IncreaseFound(int n = 1);
    /* MapPoint.cc:329-403 on the GPU (one MapPoint; ORBmatcher::ComputeDistinctiveDescriptors batches many). */
    void ComputeDistinctiveDescriptors();
    void UpdateNormalAndDepth();                          /* MapPoint.cc:426-493 */
    void SetDescriptor(const uint8_t d[32]);
    void GetDescriptor(uint8_t d[32]);
    Map* GetMap() const { return mpMap; }
    void GetNormal(float n[3]);
    float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }
    float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }
    /* mfMinDistance / mfMaxDistance as stored (Fuse's PredictScale reads the latter). */
    float GetMinDistance();
    float GetMaxDistance();

    unsigned long mnId;
    unsigned long mnBALocalForKF = 0, mnBALocalForMerge = 0;
    float mPosGBA[3] = {0.f, 0.f, 0.f};   /* global BA result kept for the loop closer (Optimizer.cc:386-387) */
    unsigned long mnBAGlobalForKF = 0;
    /* Tracking fields written by Frame::isInFrustum (Frame.cc:512-586), read by SearchByProjection. */
    bool mbTrackInView = false;
    float mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackDepth = 0.f, mTrackViewCos = 0.f;
    int mnTrackScaleLevel = 0;

private:
    std::mutex mMutexPos, mMutexFeatures;
    float mWorldPos[3];
    float mNormalVector[3] = {0.f, 0.f, 0.f};
    float mfMinDistance = 0.f, mfMaxDistance = 0.f;
    uint8_t mDescriptor[32] = {0};
    std::map<KeyFrame*, std::tuple<int, int>> mObservations;
    int nObs = 0;
    int mnVisible = 1, mnFound = 1;
    bool mbBad = false;
    MapPoint* mpReplaced = nullptr;
    KeyFrame* mpRefKF;
    Map* mpMap;
};

/* Map (src/Map.cc): init keyframe id, the map-update mutex, change counter. */
class Map {
public:
    explicit Map(unsigned long initKFid = 0) : mnInitKFid(initKFid) {}
    unsigned long GetInitKFid() const { return mnInitKFid; }
    bool IsInertial() const { return false; }
    void EraseMapPoint(MapPoint* pMP) { std::lock_guard<std::mutex> l(mMutexMap); mspMapPoints.erase(pMP); }
    void AddMapPoint(MapPoint* pMP) { std::lock_guard<std::mutex> l(mMutexMap); mspMapPoints.insert(pMP); }
    /* Map.cc: AddKeyFrame (the first one is the origin), GetAllKeyFrames / GetAllMapPoints (std::set order) */
    void AddKeyFrame(KeyFrame* pKF) {
        std::lock_guard<std::mutex> l(mMutexMap);
        if (mspKeyFrames.empty()) mpKFinitial = pKF;
        mspKeyFrames.insert(pKF);
    }
    std::vector<KeyFrame*> GetAllKeyFrames() {
        std::lock_guard<std::mutex> l(mMutexMap);
        return std::vector<KeyFrame*>(mspKeyFrames.begin(), mspKeyFrames.end());
    }
    std::vector<MapPoint*> GetAllMapPoints() {
        std::lock_guard<std::mutex> l(mMutexMap);
        return std::vector<MapPoint*>(mspMapPoints.begin(), mspMapPoints.end());
    }
    KeyFrame* GetOriginKF() { return mpKFinitial; }
    void IncreaseChangeIndex() { std::lock_guard<std::mutex> l(mMutexMap); mnMapChange++; }
    int GetMapChangeIndex() { std::lock_guard<std::mutex> l(mMutexMap); return mnMapChange; }

    std::mutex mMutexMapUpdate;

private:
    unsigned long mnInitKFid;
    std::mutex mMutexMap;
    std::set<MapPoint*> mspMapPoints;
    std::set<KeyFrame*> mspKeyFrames;
    KeyFrame* mpKFinitial = nullptr;
    int mnMapChange = 0;
};

}  // namespace MAM3SLAM
#endif
