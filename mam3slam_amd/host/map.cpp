// Host-side value types and the minimal map model (include/mam3slam/Types.h, Map.h).
// Follows src/Frame.cc, src/KeyFrame.cc, src/MapPoint.cc of the reference for the members the hot path uses.
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "mam3slam/Map.h"
#include "../csrc/camera.hpp"
#include "mam3slam/ORBextractor.h"
#include "mam3slam/ORBVocabulary.h"
#include "mam3slam/ORBmatcher.h"

namespace MAM3SLAM {

namespace {
thread_local int t_device = 0;
}
void SetDevice(int device) { t_device = device; }
int GetDevice() { return t_device; }

// ---- SE3f (Sophus::SE3f) ----------------------------------------------------------------------------------

void SE3f::rotationMatrix(float R[9]) const {
    // Eigen QuaternionBase::toRotationMatrix
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    const float tx = 2.f * x, ty = 2.f * y, tz = 2.f * z;
    const float twx = tx * w, twy = ty * w, twz = tz * w;
    const float txx = tx * x, txy = ty * x, txz = tz * x;
    const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.f - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.f - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.f - (txx + tyy);
}

// Sophus SO3 action (so3.hpp:358-367): uv = 2 q.vec x p; p + w uv + q.vec x uv
static void quatRotate(const float q[4], const float p[3], float out[3]) {
    float uv[3] = {q[1] * p[2] - q[2] * p[1], q[2] * p[0] - q[0] * p[2], q[0] * p[1] - q[1] * p[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const float c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; i++) out[i] = p[i] + q[3] * uv[i] + c[i];
}

static void quatNormalize(float q[4]) {
    const float n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (n2 > 0.f) {
        const float n = std::sqrt(n2);
        for (int i = 0; i < 4; i++) q[i] /= n;
    }
}

void SE3f::map(const float p[3], float out[3]) const {
    quatRotate(q, p, out);
    for (int i = 0; i < 3; i++) out[i] += t[i];
}

SE3f SE3f::inverse() const {
    // se3.hpp:208-211: invR = conjugate; t' = invR * (-t)
    SE3f r;
    r.q[0] = -q[0]; r.q[1] = -q[1]; r.q[2] = -q[2]; r.q[3] = q[3];
    const float mt[3] = {t[0] * -1.f, t[1] * -1.f, t[2] * -1.f};
    quatRotate(r.q, mt, r.t);
    return r;
}

SE3f SE3f::operator*(const SE3f& o) const {
    // se3.hpp:304-308 with the SO3 product of so3.hpp:325-339 (renormalised by the SO3 constructor)
    const float *a = q, *b = o.q;
    SE3f r;
    r.q[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    r.q[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    r.q[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    r.q[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    quatNormalize(r.q);
    float rt[3];
    quatRotate(q, o.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = t[i] + rt[i];
    return r;
}

mam_pose SE3f::toC() const {
    mam_pose p;
    std::memcpy(p.q, q, sizeof(p.q));
    std::memcpy(p.t, t, sizeof(p.t));
    return p;
}

mam_camera GeometricCamera::toC() const {
    mam_camera c{};
    c.fx = mvParameters[0]; c.fy = mvParameters[1]; c.cx = mvParameters[2]; c.cy = mvParameters[3];
    if (mnType == CAM_FISHEYE) {
        for (int k = 0; k < 4; k++) c.k[k] = mvParameters[4 + k];
        c.model = MAM_CAM_KANNALA_BRANDT8;
        c.precision = precision;
    }
    return c;
}

void GeometricCamera::project(const float v[3], float uv[2]) const {
    mam::cam::project_f(toC(), v[0], v[1], v[2], &uv[0], &uv[1]);
}

void GeometricCamera::unproject(const float p[2], float ray[3]) const {
    if (mnType == CAM_FISHEYE) {
        mam::cam::kb8_unproject_f(toC(), p[0], p[1], ray);
        return;
    }
    ray[0] = (p[0] - mvParameters[2]) / mvParameters[0];
    ray[1] = (p[1] - mvParameters[3]) / mvParameters[1];
    ray[2] = 1.f;
}

void GeometricCamera::toK(float K[9]) const {
    K[0] = mvParameters[0]; K[1] = 0.f;             K[2] = mvParameters[2];
    K[3] = 0.f;             K[4] = mvParameters[1]; K[5] = mvParameters[3];
    K[6] = 0.f;             K[7] = 0.f;             K[8] = 1.f;
}

// ---- Frame ------------------------------------------------------------------------------------------------

static mam_frame_geom makeGeom(float minX, float maxX, float minY, float maxY, float invW, float invH,
                               const std::vector<float>& scales, const std::vector<float>& sigma2) {
    mam_frame_geom g;
    std::memset(&g, 0, sizeof(g));
    g.min_x = minX; g.max_x = maxX; g.min_y = minY; g.max_y = maxY;
    g.grid_inv_w = invW; g.grid_inv_h = invH;
    g.nlevels = (int32_t)scales.size();
    if (g.nlevels > MAM_MAX_LEVELS) throw std::invalid_argument("too many pyramid levels");
    for (int i = 0; i < g.nlevels; i++) {
        g.scale_factors[i] = scales[i];
        g.level_sigma2[i] = sigma2[i];
    }
    return g;
}

Frame::Frame(const ImageView& imGray, ORBextractor* extractor, const GeometricCamera* pCamera, unsigned long id)
    : mnId(id), mpCamera(pCamera) {
    // Frame.cc:289-382 (mono): scale info, ExtractORB(0, imGray, 0, 1000), N, undistortion (identity: the
    // synthetic pinhole agents have zero distortion), grid bounds.
    mnScaleLevels = extractor->GetLevels();
    mfScaleFactor = extractor->GetScaleFactor();
    mfLogScaleFactor = std::log(mfScaleFactor);
    mvScaleFactors = extractor->GetScaleFactors();
    mvInvScaleFactors = extractor->GetInverseScaleFactors();
    mvLevelSigma2 = extractor->GetScaleSigmaSquares();
    mvInvLevelSigma2 = extractor->GetInverseScaleSigmaSquares();

    std::vector<int> vLapping = {0, 1000};
    monoLeft = (*extractor)(imGray, ImageView(), mvKeys, mDescriptors, vLapping);
    N = (int)mvKeys.size();
    mvKeysUn = mvKeys;
    mvpMapPoints.assign(N, nullptr);
    mvbOutlier.assign(N, false);

    // ComputeImageBounds without distortion (Frame.cc:801-807), grid inverses (Frame.cc:341-342)
    mnMinX = 0.0f;
    mnMaxX = (float)imGray.cols;
    mnMinY = 0.0f;
    mnMaxY = (float)imGray.rows;
    mfGridElementWidthInv = static_cast<float>(MAM_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
    mfGridElementHeightInv = static_cast<float>(MAM_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
}

mam_frame_geom Frame::Geom() const {
    return makeGeom(mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv, mvScaleFactors,
                    mvLevelSigma2);
}

// ---- KeyFrame ---------------------------------------------------------------------------------------------

KeyFrame::KeyFrame(const Frame& F, Map* pMap, unsigned long id)
    : mnId(id), N(F.N), mvKeys(F.mvKeys), mvKeysUn(F.mvKeysUn), mvuRight(F.N, -1.0f), mDescriptors(F.mDescriptors),
      mnScaleLevels(F.mnScaleLevels), mfLogScaleFactor(F.mfLogScaleFactor), mvScaleFactors(F.mvScaleFactors), mvLevelSigma2(F.mvLevelSigma2),
      mvInvLevelSigma2(F.mvInvLevelSigma2), mnMinX(F.mnMinX), mnMaxX(F.mnMaxX), mnMinY(F.mnMinY), mnMaxY(F.mnMaxY),
      mfGridElementWidthInv(F.mfGridElementWidthInv), mfGridElementHeightInv(F.mfGridElementHeightInv),
      mpCamera(F.mpCamera), mvpMapPoints(F.mvpMapPoints), mpMap(pMap) {
    SetPose(F.GetPose());
}

SE3f KeyFrame::GetPose() {
    std::lock_guard<std::mutex> l(mMutexPose);
    return mTcw;
}

SE3f KeyFrame::GetPoseInverse() {
    std::lock_guard<std::mutex> l(mMutexPose);
    return mTwc;
}

void KeyFrame::SetPose(const SE3f& Tcw) {
    std::lock_guard<std::mutex> l(mMutexPose);   // KeyFrame.cc:109-116
    mTcw = Tcw;
    mTwc = mTcw.inverse();
}

void KeyFrame::GetCameraCenter(float Ow[3]) {
    std::lock_guard<std::mutex> l(mMutexPose);
    std::memcpy(Ow, mTwc.t, sizeof(float) * 3);
}

std::vector<MapPoint*> KeyFrame::GetMapPointMatches() {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    return mvpMapPoints;
}

std::set<MapPoint*> KeyFrame::GetMapPoints() {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    std::set<MapPoint*> s;
    for (MapPoint* pMP : mvpMapPoints)
        if (pMP && !pMP->isBad()) s.insert(pMP);
    return s;
}

MapPoint* KeyFrame::GetMapPoint(size_t idx) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    return mvpMapPoints[idx];
}

void KeyFrame::AddMapPoint(MapPoint* pMP, size_t idx) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    mvpMapPoints[idx] = pMP;
}

void KeyFrame::ReplaceMapPointMatch(const int& idx, MapPoint* pMP) { mvpMapPoints[idx] = pMP; }

void KeyFrame::EraseMapPointMatch(int idx) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    mvpMapPoints[idx] = nullptr;
}

void KeyFrame::EraseMapPointMatch(MapPoint* pMP) {
    const std::tuple<int, int> idx = pMP->GetIndexInKeyFrame(this);   // KeyFrame.cc:309-317
    if (std::get<0>(idx) != -1) mvpMapPoints[std::get<0>(idx)] = nullptr;
    if (std::get<1>(idx) != -1) mvpMapPoints[std::get<1>(idx)] = nullptr;
}

void KeyFrame::ComputeBoW() {
    if ((mBowVec.empty() || mFeatVec.empty()) && mpORBvocabulary)
        mpORBvocabulary->transform(mDescriptors, mBowVec, mFeatVec, 4);
}

mam_frame_geom KeyFrame::Geom() const {
    return makeGeom(mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv, mvScaleFactors,
                    mvLevelSigma2);
}

// ---- MapPoint ---------------------------------------------------------------------------------------------

MapPoint::MapPoint(const float Pos[3], KeyFrame* pRefKF, Map* pMap, unsigned long id)
    : mnId(id), mpRefKF(pRefKF), mpMap(pMap) {
    std::memcpy(mWorldPos, Pos, sizeof(mWorldPos));
}

void MapPoint::GetWorldPos(float Pos[3]) {
    std::lock_guard<std::mutex> l(mMutexPos);
    std::memcpy(Pos, mWorldPos, sizeof(mWorldPos));
}

void MapPoint::SetWorldPos(const float Pos[3]) {
    std::lock_guard<std::mutex> l(mMutexPos);
    std::memcpy(mWorldPos, Pos, sizeof(mWorldPos));
}

std::map<KeyFrame*, std::tuple<int, int>> MapPoint::GetObservations() {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    return mObservations;
}

int MapPoint::Observations() {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    return nObs;
}

void MapPoint::AddObservation(KeyFrame* pKF, int idx) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    std::tuple<int, int> indexes(-1, -1);
    auto it = mObservations.find(pKF);
    if (it != mObservations.end()) indexes = it->second;
    std::get<0>(indexes) = idx;
    mObservations[pKF] = indexes;
    if (pKF->mvuRight[idx] >= 0) nObs += 2;
    else nObs++;
}

void MapPoint::EraseObservation(KeyFrame* pKF) {
    bool bBad = false;
    {
        std::lock_guard<std::mutex> l(mMutexFeatures);
        auto it = mObservations.find(pKF);
        if (it != mObservations.end()) {
            const int leftIndex = std::get<0>(it->second), rightIndex = std::get<1>(it->second);
            if (leftIndex != -1) {
                if (pKF->mvuRight[leftIndex] >= 0) nObs -= 2;
                else nObs--;
            }
            if (rightIndex != -1) nObs--;
            mObservations.erase(it);
            if (mpRefKF == pKF) mpRefKF = mObservations.empty() ? nullptr : mObservations.begin()->first;
            if (nObs <= 2) bBad = true;
        }
    }
    if (bBad) SetBadFlag();
}

std::tuple<int, int> MapPoint::GetIndexInKeyFrame(KeyFrame* pKF) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    auto it = mObservations.find(pKF);
    return it != mObservations.end() ? it->second : std::tuple<int, int>(-1, -1);
}

bool MapPoint::IsInKeyFrame(KeyFrame* pKF) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    return mObservations.count(pKF) != 0;
}

void MapPoint::SetBadFlag() {
    std::map<KeyFrame*, std::tuple<int, int>> obs;
    {
        std::lock_guard<std::mutex> l1(mMutexFeatures);
        std::lock_guard<std::mutex> l2(mMutexPos);
        mbBad = true;
        obs.swap(mObservations);
    }
    for (auto& o : obs) {
        if (std::get<0>(o.second) != -1) o.first->EraseMapPointMatch(std::get<0>(o.second));
        if (std::get<1>(o.second) != -1) o.first->EraseMapPointMatch(std::get<1>(o.second));
    }
    if (mpMap) mpMap->EraseMapPoint(this);
}

bool MapPoint::isBad() {
    std::lock_guard<std::mutex> l1(mMutexFeatures);
    std::lock_guard<std::mutex> l2(mMutexPos);
    return mbBad;
}

MapPoint* MapPoint::GetReplaced() {
    std::lock_guard<std::mutex> l1(mMutexFeatures);
    std::lock_guard<std::mutex> l2(mMutexPos);
    return mpReplaced;
}

void MapPoint::Replace(MapPoint* pMP) {
    // MapPoint.cc:248-300: pMP takes over this point's observations (or the keyframe slot is cleared where pMP is
    // already observed), then recomputes its descriptor; this point becomes bad
    if (pMP->mnId == this->mnId) return;
    int nvisible, nfound;
    std::map<KeyFrame*, std::tuple<int, int>> obs;
    {
        std::lock_guard<std::mutex> l1(mMutexFeatures);
        std::lock_guard<std::mutex> l2(mMutexPos);
        obs = mObservations;
        mObservations.clear();
        mbBad = true;
        nvisible = mnVisible;
        nfound = mnFound;
        mpReplaced = pMP;
    }
    for (auto& o : obs) {
        KeyFrame* pKF = o.first;
        const int leftIndex = std::get<0>(o.second), rightIndex = std::get<1>(o.second);
        if (!pMP->IsInKeyFrame(pKF)) {
            if (leftIndex != -1) {
                pKF->ReplaceMapPointMatch(leftIndex, pMP);
                pMP->AddObservation(pKF, leftIndex);
            }
            if (rightIndex != -1) {
                pKF->ReplaceMapPointMatch(rightIndex, pMP);
                pMP->AddObservation(pKF, rightIndex);
            }
        } else {
            if (leftIndex != -1) pKF->EraseMapPointMatch(leftIndex);
            if (rightIndex != -1) pKF->EraseMapPointMatch(rightIndex);
        }
    }
    pMP->IncreaseFound(nfound);
    pMP->IncreaseVisible(nvisible);
    pMP->ComputeDistinctiveDescriptors();
    if (mpMap) mpMap->EraseMapPoint(this);
}

void MapPoint::IncreaseVisible(int n) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    mnVisible += n;
}

void MapPoint::IncreaseFound(int n) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    mnFound += n;
}

void MapPoint::ComputeDistinctiveDescriptors() { ORBmatcher::ComputeDistinctiveDescriptors(std::vector<MapPoint*>{this}); }

float MapPoint::GetMinDistance() {
    std::lock_guard<std::mutex> l(mMutexPos);
    return mfMinDistance;
}

float MapPoint::GetMaxDistance() {
    std::lock_guard<std::mutex> l(mMutexPos);
    return mfMaxDistance;
}

void MapPoint::SetDescriptor(const uint8_t d[32]) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    std::memcpy(mDescriptor, d, 32);
}

void MapPoint::GetDescriptor(uint8_t d[32]) {
    std::lock_guard<std::mutex> l(mMutexFeatures);
    std::memcpy(d, mDescriptor, 32);
}

void MapPoint::GetNormal(float n[3]) {
    std::lock_guard<std::mutex> l(mMutexPos);
    std::memcpy(n, mNormalVector, sizeof(mNormalVector));
}

static float norm3(const float v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

void MapPoint::UpdateNormalAndDepth() {
    // MapPoint.cc:426-493 (mono: left indices only)
    std::map<KeyFrame*, std::tuple<int, int>> observations;
    KeyFrame* pRefKF;
    float Pos[3];
    {
        std::lock_guard<std::mutex> l1(mMutexFeatures);
        std::lock_guard<std::mutex> l2(mMutexPos);
        if (mbBad) return;
        observations = mObservations;
        pRefKF = mpRefKF;
        std::memcpy(Pos, mWorldPos, sizeof(Pos));
    }
    if (observations.empty() || !pRefKF) return;
    float normal[3] = {0.f, 0.f, 0.f};
    int n = 0;
    for (auto& o : observations) {
        if (std::get<0>(o.second) != -1) {
            float Owi[3];
            o.first->GetCameraCenter(Owi);
            const float ni[3] = {Pos[0] - Owi[0], Pos[1] - Owi[1], Pos[2] - Owi[2]};
            const float nn = norm3(ni);
            for (int k = 0; k < 3; k++) normal[k] = normal[k] + ni[k] / nn;
            n++;
        }
    }
    float Oref[3];
    pRefKF->GetCameraCenter(Oref);
    const float PC[3] = {Pos[0] - Oref[0], Pos[1] - Oref[1], Pos[2] - Oref[2]};
    const float dist = norm3(PC);
    auto it = observations.find(pRefKF);
    if (it == observations.end() || std::get<0>(it->second) < 0) return;
    const int level = pRefKF->mvKeysUn[std::get<0>(it->second)].octave;
    const float levelScaleFactor = pRefKF->mvScaleFactors[level];
    const int nLevels = pRefKF->mnScaleLevels;
    {
        std::lock_guard<std::mutex> l3(mMutexPos);
        mfMaxDistance = dist * levelScaleFactor;
        mfMinDistance = mfMaxDistance / pRefKF->mvScaleFactors[nLevels - 1];
        for (int k = 0; k < 3; k++) mNormalVector[k] = normal[k] / (float)n;
    }
}

}  // namespace MAM3SLAM
