// MAM3SLAM::Optimizer::LocalBundleAdjustment (include/mam3slam/Optimizer.h).
// Window build, outlier erase and write-back follow src/Optimizer.cc:1116-1498 line by line (mono agents); the
// g2o `optimizer.optimize(10)` is mam_lba_solve on the GPU (include/mam_lba.h).
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

#include "mam3slam/Optimizer.h"

namespace MAM3SLAM {

namespace {

struct ThreadLBA {
    mam_lba_ctx* ctx = nullptr;
    int device = -1;
    ~ThreadLBA() {
        if (ctx) mam_lba_destroy(ctx);
    }
};
thread_local ThreadLBA t_lba;

struct ThreadPose {
    mam_pose_ctx* ctx = nullptr;
    int device = -1;
    ~ThreadPose() {
        if (ctx) mam_pose_destroy(ctx);
    }
};
thread_local ThreadPose t_pose;

// Sophus::SO3f's normalize() (so3.hpp:481-487): coeffs / norm(), the norm of the 4-float vector as Eigen's SSE packet
// reduction sums it, (x^2 + z^2) + (y^2 + w^2) (predux<Packet4f>: movehl add, then the two lanes) — one order for
// every SE3f built from an optimised quaternion (Frame and KeyFrame SetPose), as csrc/pose.hip and csrc/exchange.hip
void sophus_normalize(float q[4]) {
    const float n = std::sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
    for (int j = 0; j < 4; j++) q[j] /= n;
}

// contexts follow the thread's device (SetDevice): recreated when it changes
mam_pose_ctx* poseCtx() {
    if (t_pose.ctx && t_pose.device != GetDevice()) {
        mam_pose_destroy(t_pose.ctx);
        t_pose.ctx = nullptr;
    }
    if (!t_pose.ctx) {
        const int rc = mam_pose_create(GetDevice(), &t_pose.ctx);
        if (rc < 0) throw std::runtime_error(std::string("mam_pose_create failed: ") + mam_last_error());
        t_pose.device = GetDevice();
    }
    return t_pose.ctx;
}

mam_lba_ctx* lbaCtx() {
    if (t_lba.ctx && t_lba.device != GetDevice()) {
        mam_lba_destroy(t_lba.ctx);
        t_lba.ctx = nullptr;
    }
    if (!t_lba.ctx) {
        const int rc = mam_lba_create(GetDevice(), &t_lba.ctx);
        if (rc < 0) throw std::runtime_error(std::string("mam_lba_create failed: ") + mam_last_error());
        t_lba.device = GetDevice();
    }
    return t_lba.ctx;
}

}  // namespace

int Optimizer::PoseOptimization(Frame* pFrame) {
    // Set MapPoint vertices (Optimizer.cc:845-895, mono branch): one edge per keypoint with a MapPoint, in order
    const int N = pFrame->N;
    std::vector<mam_pose_edge> edges;
    std::vector<int> idx;
    edges.reserve(N);
    idx.reserve(N);
    if ((int)pFrame->mvbOutlier.size() != N) pFrame->mvbOutlier.assign(N, false);
    for (int i = 0; i < N; i++) {
        MapPoint* pMP = pFrame->mvpMapPoints[i];
        if (!pMP) continue;
        pFrame->mvbOutlier[i] = false;
        const KeyPoint& kpUn = pFrame->mvKeysUn[i];
        mam_pose_edge e;
        e.obs[0] = kpUn.pt.x;
        e.obs[1] = kpUn.pt.y;
        pMP->GetWorldPos(e.xw);
        e.inv_sigma2 = pFrame->mvInvLevelSigma2[kpUn.octave];
        edges.push_back(e);
        idx.push_back(i);
    }
    const mam_pose tcw = pFrame->GetPose().toC();
    const mam_pinhole cam = pFrame->mpCamera->toC();
    std::vector<uint8_t> outlier(std::max<size_t>(edges.size(), 1));
    mam_pose_result res;
    const int n = mam_pose_optimization(poseCtx(), &tcw, &cam, (int)edges.size(), edges.data(), outlier.data(), &res);
    if (n < 0) throw std::runtime_error(std::string("mam_pose_optimization failed: ") + mam_last_error());
    if (edges.size() < 3) return 0;   // :997-998 (pose untouched)
    for (size_t e = 0; e < idx.size(); e++) pFrame->mvbOutlier[idx[e]] = outlier[e] != 0;
    // Recover optimized pose (:1103-1107): SE3<float>(Quaterniond.cast<float>(), t.cast<float>())
    SE3f pose;
    for (int j = 0; j < 4; j++) pose.q[j] = (float)res.q[j];
    for (int j = 0; j < 3; j++) pose.t[j] = (float)res.t[j];
    sophus_normalize(pose.q);
    pFrame->SetPose(pose);
    return n;
}

int32_t LocalBAWindow::cameraIndex(const GeometricCamera* c) {
    for (size_t i = 0; i < camera_list.size(); i++)
        if (camera_list[i] == c) return (int32_t)i;
    const int32_t model = c->GetType() == GeometricCamera::CAM_FISHEYE ? MAM_CAM_KANNALA_BRANDT8 : MAM_CAM_PINHOLE;
    if (camera_list.empty()) cam_model = model;
    else if (model != cam_model)
        throw std::invalid_argument("LocalBundleAdjustment: Pinhole and KannalaBrandt8 keyframes in one window");
    camera_list.push_back(c);
    for (int k = 0; k < c->size(); k++) cams.push_back(c->mvParameters[k]);
    return (int32_t)(camera_list.size() - 1);
}

mam_lba_problem LocalBAWindow::Problem(int iterations) const {
    mam_lba_problem p{};
    p.n_poses = (int32_t)vpKF.size();
    p.pose_id = pose_id.data();
    p.pose_fixed = pose_fixed.data();
    p.pose_q = pose_q.data();
    p.pose_t = pose_t.data();
    p.pose_cam = pose_cam.data();
    p.n_points = (int32_t)vpMP.size();
    p.point_id = point_id.data();
    p.point_xyz = point_xyz.data();
    p.n_edges = (int32_t)edge_point.size();
    p.edge_point = edge_point.data();
    p.edge_pose = edge_pose.data();
    p.edge_obs = edge_obs.data();
    p.edge_inv_sigma2 = edge_inv_sigma2.data();
    p.n_cams = (int32_t)camera_list.size();
    p.cam_model = cam_model;
    p.cams = cams.data();
    p.huber_delta = (double)(float)std::sqrt(5.991);   // const float thHuberMono = sqrt(5.991) (:1275)
    p.iterations = iterations;
    p.edge_active = nullptr;
    return p;
}

bool Optimizer::BuildLocalBAWindow(KeyFrame* pKF, Map* pMap, LocalBAWindow& w) {
    w = LocalBAWindow();
    // Local KeyFrames: first breadth search from the current keyframe (:1118-1132)
    w.lLocalKeyFrames.push_back(pKF);
    pKF->mnBALocalForKF = pKF->mnId;
    Map* pCurrentMap = pKF->GetMap();
    const std::vector<KeyFrame*> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
    for (KeyFrame* pKFi : vNeighKFs) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad() && pKFi->GetMap() == pCurrentMap) w.lLocalKeyFrames.push_back(pKFi);
    }
    // Local MapPoints seen in local KeyFrames (:1134-1160)
    w.num_fixedKF = 0;
    for (KeyFrame* pKFi : w.lLocalKeyFrames) {
        if (pKFi->mnId == pMap->GetInitKFid()) w.num_fixedKF = 1;
        const std::vector<MapPoint*> vpMPs = pKFi->GetMapPointMatches();
        for (MapPoint* pMP : vpMPs) {
            if (pMP && !pMP->isBad() && pMP->GetMap() == pCurrentMap && pMP->mnBALocalForKF != pKF->mnId) {
                w.lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
        }
    }
    // Fixed KeyFrames: observers of local MapPoints that are not local (:1162-1178)
    for (MapPoint* pMP : w.lLocalMapPoints) {
        const auto observations = pMP->GetObservations();
        for (const auto& obs : observations) {
            KeyFrame* pKFi = obs.first;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad() && pKFi->GetMap() == pCurrentMap) w.lFixedCameras.push_back(pKFi);
            }
        }
    }
    w.num_fixedKF = (int)w.lFixedCameras.size() + w.num_fixedKF;
    if (w.num_fixedKF == 0) return false;   // :1182-1186

    // Vertices (:1212-1243): local keyframes (init KF fixed), then fixed cameras
    auto camIndex = [&](const GeometricCamera* c) { return w.cameraIndex(c); };
    std::map<KeyFrame*, int32_t> kfIndex;
    auto addPose = [&](KeyFrame* pKFi, bool fixed) {
        const SE3f Tcw = pKFi->GetPose();
        kfIndex[pKFi] = (int32_t)w.vpKF.size();
        w.vpKF.push_back(pKFi);
        w.pose_id.push_back((int64_t)pKFi->mnId);
        w.pose_fixed.push_back(fixed ? 1 : 0);
        for (int k = 0; k < 4; k++) w.pose_q.push_back((double)Tcw.q[k]);   // unit_quaternion().cast<double>()
        for (int k = 0; k < 3; k++) w.pose_t.push_back((double)Tcw.t[k]);
        w.pose_cam.push_back(camIndex(pKFi->mpCamera));
        if (pKFi->mnId > w.maxKFid) w.maxKFid = pKFi->mnId;
    };
    for (KeyFrame* pKFi : w.lLocalKeyFrames) addPose(pKFi, pKFi->mnId == pMap->GetInitKFid());
    for (KeyFrame* pKFi : w.lFixedCameras) addPose(pKFi, true);

    // MapPoint vertices and mono edges (:1245-1394), edge insertion order = point order x observation order
    for (MapPoint* pMP : w.lLocalMapPoints) {
        float pos[3];
        pMP->GetWorldPos(pos);
        const int32_t pi = (int32_t)w.vpMP.size();
        w.vpMP.push_back(pMP);
        w.point_id.push_back((int64_t)(pMP->mnId + w.maxKFid + 1));
        for (int k = 0; k < 3; k++) w.point_xyz.push_back((double)pos[k]);
        const auto observations = pMP->GetObservations();
        for (const auto& obs : observations) {
            KeyFrame* pKFi = obs.first;
            if (pKFi->isBad() || pKFi->GetMap() != pCurrentMap) continue;
            const int leftIndex = std::get<0>(obs.second);
            if (leftIndex == -1) continue;
            if (pKFi->mvuRight[leftIndex] >= 0)
                throw std::invalid_argument("LocalBundleAdjustment: stereo observations are out of scope");
            auto it = kfIndex.find(pKFi);
            if (it == kfIndex.end()) continue;   // unreachable: every observer is local or fixed
            const KeyPoint& kpUn = pKFi->mvKeysUn[leftIndex];
            w.edge_point.push_back(pi);
            w.edge_pose.push_back(it->second);
            w.edge_obs.push_back((double)kpUn.pt.x);
            w.edge_obs.push_back((double)kpUn.pt.y);
            w.edge_inv_sigma2.push_back((double)pKFi->mvInvLevelSigma2[kpUn.octave]);
        }
    }
    return true;
}

void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF,
                                      int& num_OptKF, int& num_MPs, int& num_edges) {
    LocalBAWindow w;
    const bool ok = BuildLocalBAWindow(pKF, pMap, w);
    num_fixedKF = w.num_fixedKF;
    if (!ok) return;
    num_OptKF = (int)w.lLocalKeyFrames.size();
    (void)num_MPs;                             // never written by the reference either
    num_edges = (int)w.edge_point.size();
    if (pbStopFlag && *pbStopFlag) return;     // :1406-1408

    const mam_lba_problem prob = w.Problem(10);
    std::vector<double> q(w.pose_q.size()), t(w.pose_t.size()), x(w.point_xyz.size()), chi2(w.edge_point.size());
    std::vector<uint8_t> depth(w.edge_point.size());
    mam_lba_result res;
    res.pose_q = q.data();
    res.pose_t = t.data();
    res.point_xyz = x.data();
    res.edge_chi2 = chi2.data();
    res.edge_depth_ok = depth.data();
    // g2o polls the force-stop flag between iterations (setForceStopFlag, :1203-1204); so does the solver
    static_assert(sizeof(bool) == 1, "pbStopFlag is read as one byte");
    const int rc = mam_lba_solve(lbaCtx(), &prob, reinterpret_cast<const volatile uint8_t*>(pbStopFlag), &res);
    if (rc < 0) throw std::runtime_error(std::string("mam_lba_solve failed: ") + mam_last_error());

    ApplyLocalBAResult(w, pMap, q.data(), t.data(), x.data(), chi2.data(), depth.data());
}

void Optimizer::ApplyLocalBAResult(const LocalBAWindow& w, Map* pMap, const double* q, const double* t,
                                   const double* x, const double* chi2, const uint8_t* depth) {
    // Check inlier observations (:1413-1430)
    std::vector<std::pair<KeyFrame*, MapPoint*>> vToErase;
    vToErase.reserve(w.edge_point.size());
    for (size_t i = 0; i < w.edge_point.size(); i++) {
        MapPoint* pMP = w.vpMP[w.edge_point[i]];
        if (pMP->isBad()) continue;
        if (chi2[i] > 5.991 || !depth[i]) vToErase.push_back(std::make_pair(w.vpKF[w.edge_pose[i]], pMP));
    }

    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);   // :1463
    for (auto& e : vToErase) {                                   // :1465-1474
        e.first->EraseMapPointMatch(e.second);
        e.second->EraseObservation(e.first);
    }
    // Recover optimized data (:1478-1494): local keyframes, then points
    size_t k = 0;
    for (KeyFrame* pKFi : w.lLocalKeyFrames) {
        SE3f Tiw;
        for (int j = 0; j < 4; j++) Tiw.q[j] = (float)q[4 * k + j];
        for (int j = 0; j < 3; j++) Tiw.t[j] = (float)t[3 * k + j];
        sophus_normalize(Tiw.q);   // Sophus::SE3f(Quaternionf, t) normalises the quaternion (so3.hpp:481-487)
        pKFi->SetPose(Tiw);
        k++;
    }
    size_t p = 0;
    for (MapPoint* pMP : w.lLocalMapPoints) {
        const float pos[3] = {(float)x[3 * p], (float)x[3 * p + 1], (float)x[3 * p + 2]};
        pMP->SetWorldPos(pos);
        pMP->UpdateNormalAndDepth();
        p++;
    }
    pMap->IncreaseChangeIndex();
}

void Optimizer::BuildBAWindow(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                              LocalBAWindow& w, std::vector<bool>& vbNotIncludedMP) {
    w = LocalBAWindow();
    vbNotIncludedMP.assign(vpMP.size(), false);
    if (vpKFs.empty()) return;
    Map* pMap = vpKFs[0]->GetMap();
    auto camIndex = [&](const GeometricCamera* c) { return w.cameraIndex(c); };
    std::map<KeyFrame*, int32_t> kfIndex;
    // KeyFrame vertices (:100-117): the initial keyframe fixed
    for (KeyFrame* pKF : vpKFs) {
        if (pKF->isBad()) continue;
        const SE3f Tcw = pKF->GetPose();
        const bool fixed = pKF->mnId == pMap->GetInitKFid();
        kfIndex[pKF] = (int32_t)w.vpKF.size();
        w.vpKF.push_back(pKF);
        w.pose_id.push_back((int64_t)pKF->mnId);
        w.pose_fixed.push_back(fixed ? 1 : 0);
        for (int k = 0; k < 4; k++) w.pose_q.push_back((double)Tcw.q[k]);
        for (int k = 0; k < 3; k++) w.pose_t.push_back((double)Tcw.t[k]);
        w.pose_cam.push_back(camIndex(pKF->mpCamera));
        if (pKF->mnId > w.maxKFid) w.maxKFid = pKF->mnId;
        (fixed ? w.lFixedCameras : w.lLocalKeyFrames).push_back(pKF);
    }
    w.num_fixedKF = (int)w.lFixedCameras.size();
    // MapPoint vertices and mono edges (:122-275); a point without edges is removed again (:266-270)
    for (size_t i = 0; i < vpMP.size(); i++) {
        MapPoint* pMP = vpMP[i];
        if (pMP->isBad()) continue;
        const int32_t pi = (int32_t)w.vpMP.size();
        const size_t e0 = w.edge_point.size();
        for (const auto& obs : pMP->GetObservations()) {
            KeyFrame* pKF = obs.first;
            if (pKF->isBad() || pKF->mnId > w.maxKFid) continue;
            auto it = kfIndex.find(pKF);
            if (it == kfIndex.end()) continue;   // optimizer.vertex(pKF->mnId) == NULL
            const int leftIndex = std::get<0>(obs.second);
            if (leftIndex == -1) continue;
            if (pKF->mvuRight[leftIndex] >= 0)
                throw std::invalid_argument("BundleAdjustment: stereo observations are out of scope");
            const KeyPoint& kpUn = pKF->mvKeysUn[leftIndex];
            w.edge_point.push_back(pi);
            w.edge_pose.push_back(it->second);
            w.edge_obs.push_back((double)kpUn.pt.x);
            w.edge_obs.push_back((double)kpUn.pt.y);
            w.edge_inv_sigma2.push_back((double)pKF->mvInvLevelSigma2[kpUn.octave]);
        }
        if (w.edge_point.size() == e0) {
            vbNotIncludedMP[i] = true;
            continue;
        }
        float pos[3];
        pMP->GetWorldPos(pos);
        w.vpMP.push_back(pMP);
        w.lLocalMapPoints.push_back(pMP);
        w.point_id.push_back((int64_t)(pMP->mnId + w.maxKFid + 1));
        for (int k = 0; k < 3; k++) w.point_xyz.push_back((double)pos[k]);
    }
}

void Optimizer::GlobalBundleAdjustemnt(Map* pMap, int nIterations, bool* pbStopFlag, const unsigned long nLoopKF,
                                       const bool bRobust) {
    const std::vector<KeyFrame*> vpKFs = pMap->GetAllKeyFrames();
    const std::vector<MapPoint*> vpMP = pMap->GetAllMapPoints();
    BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust);
}

void Optimizer::BundleAdjustment(const std::vector<KeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                 int nIterations, bool* pbStopFlag, const unsigned long nLoopKF, const bool bRobust) {
    if (vpKFs.empty()) return;
    Map* pMap = vpKFs[0]->GetMap();
    LocalBAWindow w;
    std::vector<bool> vbNotIncludedMP;
    BuildBAWindow(vpKFs, vpMP, w, vbNotIncludedMP);
    mam_lba_problem prob = w.Problem(nIterations);
    prob.huber_delta = bRobust ? (double)(float)std::sqrt(5.99) : 0.0;   // thHuber2D (:119, :166-171)
    std::vector<double> q(w.pose_q.size()), t(w.pose_t.size()), x(w.point_xyz.size());
    mam_lba_result res{q.data(), t.data(), x.data(), nullptr, nullptr, 0, 0, 0, 0, 0};
    const int rc = mam_lba_solve(lbaCtx(), &prob, reinterpret_cast<const volatile uint8_t*>(pbStopFlag), &res);
    if (rc < 0) throw std::runtime_error(std::string("mam_lba_solve failed: ") + mam_last_error());
    // Recover optimized data (:283-389)
    KeyFrame* pOrigin = pMap->GetOriginKF();
    const bool direct = pOrigin && nLoopKF == pOrigin->mnId;
    for (size_t k = 0; k < w.vpKF.size(); k++) {
        KeyFrame* pKF = w.vpKF[k];
        SE3f T;
        for (int j = 0; j < 4; j++) T.q[j] = (float)q[4 * k + j];
        for (int j = 0; j < 3; j++) T.t[j] = (float)t[3 * k + j];
        sophus_normalize(T.q);
        if (direct) {
            pKF->SetPose(T);
        } else {
            pKF->mTcwGBA = T;
            pKF->mnBAGlobalForKF = nLoopKF;
        }
    }
    for (size_t p = 0; p < w.vpMP.size(); p++) {
        MapPoint* pMP = w.vpMP[p];
        if (pMP->isBad()) continue;
        const float pos[3] = {(float)x[3 * p], (float)x[3 * p + 1], (float)x[3 * p + 2]};
        if (direct) {
            pMP->SetWorldPos(pos);
            pMP->UpdateNormalAndDepth();
        } else {
            for (int j = 0; j < 3; j++) pMP->mPosGBA[j] = pos[j];
            pMP->mnBAGlobalForKF = nLoopKF;
        }
    }
}

void Optimizer::BuildMergeBAWindow(KeyFrame* pMainKF, const std::vector<KeyFrame*>& vpAdjustKF,
                                   const std::vector<KeyFrame*>& vpFixedKF, LocalBAWindow& w) {
    w = LocalBAWindow();
    Map* pCurrentMap = pMainKF->GetMap();
    auto camIndex = [&](const GeometricCamera* c) { return w.cameraIndex(c); };
    std::map<KeyFrame*, int32_t> kfIndex;
    std::vector<MapPoint*> vpMPs;
    // fixed, then non-fixed keyframe vertices with their MapPoints (:3531-3605)
    auto addKF = [&](KeyFrame* pKFi, bool fixed) {
        if (pKFi->isBad() || pKFi->GetMap() != pCurrentMap) return;
        pKFi->mnBALocalForMerge = pMainKF->mnId;
        const SE3f Tcw = pKFi->GetPose();
        kfIndex[pKFi] = (int32_t)w.vpKF.size();
        w.vpKF.push_back(pKFi);
        w.pose_id.push_back((int64_t)pKFi->mnId);
        w.pose_fixed.push_back(fixed ? 1 : 0);
        for (int k = 0; k < 4; k++) w.pose_q.push_back((double)Tcw.q[k]);
        for (int k = 0; k < 3; k++) w.pose_t.push_back((double)Tcw.t[k]);
        w.pose_cam.push_back(camIndex(pKFi->mpCamera));
        if (pKFi->mnId > w.maxKFid) w.maxKFid = pKFi->mnId;
        (fixed ? w.lFixedCameras : w.lLocalKeyFrames).push_back(pKFi);
        for (MapPoint* pMPi : pKFi->GetMapPoints())
            if (pMPi && !pMPi->isBad() && pMPi->GetMap() == pCurrentMap && pMPi->mnBALocalForMerge != pMainKF->mnId) {
                vpMPs.push_back(pMPi);
                pMPi->mnBALocalForMerge = pMainKF->mnId;
            }
    };
    for (KeyFrame* pKFi : vpFixedKF) addKF(pKFi, true);
    for (KeyFrame* pKFi : vpAdjustKF) addKF(pKFi, false);
    w.num_fixedKF = (int)w.lFixedCameras.size();
    // MapPoint vertices and mono edges (:3634-3724)
    for (MapPoint* pMPi : vpMPs) {
        if (pMPi->isBad()) continue;
        float pos[3];
        pMPi->GetWorldPos(pos);
        const int32_t pi = (int32_t)w.vpMP.size();
        w.vpMP.push_back(pMPi);
        w.lLocalMapPoints.push_back(pMPi);
        w.point_id.push_back((int64_t)(pMPi->mnId + w.maxKFid + 1));
        for (int k = 0; k < 3; k++) w.point_xyz.push_back((double)pos[k]);
        for (const auto& obs : pMPi->GetObservations()) {
            KeyFrame* pKF = obs.first;
            const int idx = std::get<0>(obs.second);
            if (pKF->isBad() || pKF->mnId > w.maxKFid || pKF->mnBALocalForMerge != pMainKF->mnId || idx == -1 ||
                !pKF->GetMapPoint(idx))
                continue;
            if (pKF->mvuRight[idx] >= 0)
                throw std::invalid_argument("LocalBundleAdjustment(merge): stereo observations are out of scope");
            const KeyPoint& kpUn = pKF->mvKeysUn[idx];
            w.edge_point.push_back(pi);
            w.edge_pose.push_back(kfIndex.at(pKF));
            w.edge_obs.push_back((double)kpUn.pt.x);
            w.edge_obs.push_back((double)kpUn.pt.y);
            w.edge_inv_sigma2.push_back((double)pKF->mvInvLevelSigma2[kpUn.octave]);
        }
    }
}

void Optimizer::LocalBundleAdjustment(KeyFrame* pMainKF, std::vector<KeyFrame*> vpAdjustKF,
                                      std::vector<KeyFrame*> vpFixedKF, bool* pbStopFlag) {
    LocalBAWindow w;
    BuildMergeBAWindow(pMainKF, vpAdjustKF, vpFixedKF, w);
    if (pbStopFlag && *pbStopFlag) return;   // :3725-3727
    const size_t E = w.edge_point.size();
    std::vector<double> q(w.pose_q.size()), t(w.pose_t.size()), x(w.point_xyz.size()), chi2(E);
    std::vector<uint8_t> depth(E), active(E, 1);
    const volatile uint8_t* stop = reinterpret_cast<const volatile uint8_t*>(pbStopFlag);
    // optimize(5) with Huber kernels, delta thHuber2D = sqrt(5.99) as float (:3627, :3675-3677, :3730-3731)
    mam_lba_problem prob = w.Problem(5);
    prob.huber_delta = (double)(float)std::sqrt(5.99);
    mam_lba_result res{q.data(), t.data(), x.data(), chi2.data(), depth.data(), 0, 0, 0, 0, 0};
    int rc = mam_lba_solve(lbaCtx(), &prob, stop, &res);
    if (rc < 0) throw std::runtime_error(std::string("mam_lba_solve failed: ") + mam_last_error());
    if (!(pbStopFlag && *pbStopFlag)) {   // bDoMore (:3733-3737)
        // chi2 > 5.991 or negative depth -> setLevel(1); every kernel removed (:3742-3757); a level-1 edge keeps
        // the chi2 of the first optimisation (chi2() reads its last computed error)
        for (size_t i = 0; i < E; i++) {
            if (w.vpMP[w.edge_point[i]]->isBad()) continue;
            if (chi2[i] > 5.991 || !depth[i]) active[i] = 0;
        }
        // initializeOptimization(0); optimize(10), from the first optimisation's estimates (:3778-3779)
        const std::vector<double> q1 = q, t1 = t, x1 = x;
        mam_lba_problem p2 = prob;
        p2.pose_q = q1.data();
        p2.pose_t = t1.data();
        p2.point_xyz = x1.data();
        p2.huber_delta = 0.0;
        p2.iterations = 10;
        p2.edge_active = active.data();
        rc = mam_lba_solve(lbaCtx(), &p2, stop, &res);
        if (rc < 0) throw std::runtime_error(std::string("mam_lba_solve failed: ") + mam_last_error());
    }
    // outliers (:3788-3807), erase under the map mutex (:3832-3843), recover the adjusted keyframes and the points
    // (:3868-3951)
    std::vector<std::pair<KeyFrame*, MapPoint*>> vToErase;
    for (size_t i = 0; i < E; i++) {
        MapPoint* pMP = w.vpMP[w.edge_point[i]];
        if (pMP->isBad()) continue;
        if (chi2[i] > 5.991 || !depth[i]) vToErase.push_back(std::make_pair(w.vpKF[w.edge_pose[i]], pMP));
    }
    std::unique_lock<std::mutex> lock(pMainKF->GetMap()->mMutexMapUpdate);
    for (auto& e : vToErase) {
        e.first->EraseMapPointMatch(e.second);
        e.second->EraseObservation(e.first);
    }
    for (size_t k = 0; k < w.vpKF.size(); k++) {
        if (w.pose_fixed[k]) continue;
        KeyFrame* pKFi = w.vpKF[k];
        if (pKFi->isBad()) continue;
        SE3f Tiw;
        for (int j = 0; j < 4; j++) Tiw.q[j] = (float)q[4 * k + j];
        for (int j = 0; j < 3; j++) Tiw.t[j] = (float)t[3 * k + j];
        sophus_normalize(Tiw.q);
        pKFi->SetPose(Tiw);
    }
    for (size_t p = 0; p < w.vpMP.size(); p++) {
        MapPoint* pMPi = w.vpMP[p];
        if (pMPi->isBad()) continue;
        const float pos[3] = {(float)x[3 * p], (float)x[3 * p + 1], (float)x[3 * p + 2]};
        pMPi->SetWorldPos(pos);
        pMPi->UpdateNormalAndDepth();
    }
}

}  // namespace MAM3SLAM
