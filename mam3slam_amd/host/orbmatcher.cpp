// MAM3SLAM::ORBmatcher over the gfx950 searches (include/mam3slam/ORBmatcher.h, include/mam_match.h).
// The wrapper only marshals: object pointers -> indices and flags going in, indices -> pointers coming out, with
// the reference's side effects on Frame::mvpMapPoints (src/ORBmatcher.cc:43-213, 907-1146, 1676-1887) and on the
// keyframe / MapPoint graph (Fuse, :1148-1338).
#include <cstring>
#include <stdexcept>
#include <string>

#include "mam3slam/ORBmatcher.h"

namespace MAM3SLAM {

const int ORBmatcher::TH_HIGH = MAM_TH_HIGH;
const int ORBmatcher::TH_LOW = MAM_TH_LOW;
const int ORBmatcher::HISTO_LENGTH = MAM_HISTO_LENGTH;

namespace {

void throwOn(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " + mam_last_error());
}

// One device context per thread (the reference builds a matcher on the stack at every call site; device
// state must outlive it). The device is the calling thread's current HIP device (0 unless set).
struct ThreadCtx {
    mam_match_ctx* ctx = nullptr;
    ~ThreadCtx() {
        if (ctx) mam_match_destroy(ctx);
    }
};
thread_local ThreadCtx t_ctx;
thread_local int t_ctx_device = -1;

mam_match_ctx* ctx() {
    if (t_ctx.ctx && t_ctx_device != GetDevice()) {
        mam_match_destroy(t_ctx.ctx);
        t_ctx.ctx = nullptr;
    }
    if (!t_ctx.ctx) {
        throwOn(mam_match_create(GetDevice(), &t_ctx.ctx), "mam_match_create");
        t_ctx_device = GetDevice();
    }
    return t_ctx.ctx;
}

}  // namespace

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    DescriptorDistances(a, b, 1, &d);
    return d;
}

void ORBmatcher::DescriptorDistances(const uint8_t* a, const uint8_t* b, int n, int* out) {
    static_assert(sizeof(int) == sizeof(int32_t), "int32 output");
    throwOn(mam_descriptor_distance(ctx(), a, b, n, reinterpret_cast<int32_t*>(out)), "mam_descriptor_distance");
}

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th,
                                   const bool bFarPoints, const float thFarPoints) {
    const int n = F.N;
    std::vector<mam_mp_track> mps(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); i++) {
        MapPoint* pMP = vpMapPoints[i];
        mam_mp_track& t = mps[i];
        std::memset(&t, 0, sizeof(t));
        if (!pMP) { t.is_bad = 1; continue; }
        t.track_in_view = pMP->mbTrackInView ? 1 : 0;
        t.proj_x = pMP->mTrackProjX;
        t.proj_y = pMP->mTrackProjY;
        t.view_cos = pMP->mTrackViewCos;
        t.track_depth = pMP->mTrackDepth;
        t.scale_level = pMP->mnTrackScaleLevel;
        t.is_bad = pMP->isBad() ? 1 : 0;
        t.nobs = pMP->Observations();
        pMP->GetDescriptor(t.desc);
    }
    // the keypoint-taken test of ORBmatcher.cc:88-90
    std::vector<uint8_t> taken(n > 0 ? n : 1, 0);
    for (int i = 0; i < n; i++) taken[i] = (F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0) ? 1 : 0;
    std::vector<int32_t> out(n > 0 ? n : 1, -1);
    const mam_frame_geom g = F.Geom();
    const int nm = mam_search_by_projection(ctx(), &g, n, reinterpret_cast<const mam_keypoint*>(F.mvKeysUn.data()),
                                            F.mDescriptors.data.data(), taken.data(), (int)mps.size(), mps.data(), th,
                                            bFarPoints ? 1 : 0, thFarPoints, mfNNratio, out.data());
    throwOn(nm, "mam_search_by_projection");
    for (int i = 0; i < n; i++)
        if (out[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[out[i]];
    return nm;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
    if (!bMono) throw std::invalid_argument("SearchByProjection(Frame, Frame): stereo is out of scope (mono agents)");
    const int n = CurrentFrame.N;
    std::vector<mam_last_entry> last(LastFrame.N);
    for (int i = 0; i < LastFrame.N; i++) {
        mam_last_entry& e = last[i];
        std::memset(&e, 0, sizeof(e));
        MapPoint* pMP = LastFrame.mvpMapPoints[i];
        if (!pMP || LastFrame.mvbOutlier[i]) continue;   // ORBmatcher.cc:1697-1701
        e.valid = 1;
        pMP->GetWorldPos(e.pos);
        e.angle = LastFrame.mvKeysUn[i].angle;
        e.octave = LastFrame.mvKeys[i].octave;
        e.nobs = pMP->Observations();
        pMP->GetDescriptor(e.desc);
    }
    std::vector<uint8_t> taken(n > 0 ? n : 1, 0);
    for (int i = 0; i < n; i++)
        taken[i] = (CurrentFrame.mvpMapPoints[i] && CurrentFrame.mvpMapPoints[i]->Observations() > 0) ? 1 : 0;
    std::vector<int32_t> out(n > 0 ? n : 1, -1);
    const mam_frame_geom g = CurrentFrame.Geom();
    const mam_pose tcw = CurrentFrame.GetPose().toC();
    const mam_pinhole cam = CurrentFrame.mpCamera->toC();
    const int nm = mam_search_by_projection_motion(
        ctx(), &g, n, reinterpret_cast<const mam_keypoint*>(CurrentFrame.mvKeysUn.data()),
        CurrentFrame.mDescriptors.data.data(), taken.data(), &tcw, nullptr, 0.f, &cam, (int)last.size(), last.data(),
        th, 1, mbCheckOrientation ? 1 : 0, out.data());
    throwOn(nm, "mam_search_by_projection_motion");
    for (int i = 0; i < n; i++) {
        if (out[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[out[i]];
        else if (out[i] == MAM_MATCH_CLEARED) CurrentFrame.mvpMapPoints[i] = nullptr;
    }
    return nm;
}

void ORBmatcher::ComputeF12(KeyFrame* pKF1, KeyFrame* pKF2, float F12[9], float ep[2]) {
    // ORBmatcher.cc:913-930 (T12, the epipole) and Pinhole.cpp:107-112 (F12), as the device search computes them
    const mam_pose t1 = pKF1->GetPose().toC(), t2 = pKF2->GetPose().toC();
    const mam_camera c1 = pKF1->mpCamera->toC(), c2 = pKF2->mpCamera->toC();
    throwOn(mam_triangulation_geometry(&t1, &t2, &c1, &c2, nullptr, nullptr, F12, ep), "mam_triangulation_geometry");
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2,
                                       std::vector<std::pair<size_t, size_t>>& vMatchedPairs, const bool bOnlyStereo,
                                       const bool bCoarse) {
    vMatchedPairs.clear();
    if (bOnlyStereo) return 0;   // mono keyframes: every candidate fails the stereo test (ORBmatcher.cc:1000-1002)
    const int n1 = pKF1->N, n2 = pKF2->N;
    std::vector<uint8_t> has1(n1 > 0 ? n1 : 1, 0), has2(n2 > 0 ? n2 : 1, 0);
    for (int i = 0; i < n1; i++) has1[i] = pKF1->GetMapPoint(i) ? 1 : 0;
    for (int i = 0; i < n2; i++) has2[i] = pKF2->GetMapPoint(i) ? 1 : 0;
    auto flatten = [](const std::map<unsigned int, std::vector<unsigned int>>& fv, std::vector<uint32_t>& ids,
                      std::vector<int32_t>& off, std::vector<uint32_t>& feats) {
        ids.clear();
        off.assign(1, 0);
        feats.clear();
        for (const auto& node : fv) {
            ids.push_back(node.first);
            feats.insert(feats.end(), node.second.begin(), node.second.end());
            off.push_back((int32_t)feats.size());
        }
        if (feats.empty()) feats.push_back(0);
        if (ids.empty()) ids.push_back(0);
    };
    std::vector<uint32_t> i1, f1, i2, f2;
    std::vector<int32_t> o1, o2;
    flatten(pKF1->mFeatVec, i1, o1, f1);
    flatten(pKF2->mFeatVec, i2, o2, f2);
    mam_tri_kf k1{}, k2{};
    k1.n = n1;
    k1.keys = reinterpret_cast<const mam_keypoint*>(pKF1->mvKeysUn.data());
    k1.desc = pKF1->mDescriptors.data.data();
    k1.has_mp = has1.data();
    k1.fv = mam_featvec{(int32_t)pKF1->mFeatVec.size(), i1.data(), o1.data(), f1.data()};
    k1.tcw = pKF1->GetPose().toC();
    k1.cam = pKF1->mpCamera->toC();
    k2.n = n2;
    k2.keys = reinterpret_cast<const mam_keypoint*>(pKF2->mvKeysUn.data());
    k2.desc = pKF2->mDescriptors.data.data();
    k2.has_mp = has2.data();
    k2.fv = mam_featvec{(int32_t)pKF2->mFeatVec.size(), i2.data(), o2.data(), f2.data()};
    k2.tcw = pKF2->GetPose().toC();
    k2.cam = pKF2->mpCamera->toC();
    std::vector<int32_t> out(n1 > 0 ? n1 : 1, -1);
    const mam_frame_geom g = pKF2->Geom();
    const int nm = mam_search_for_triangulation_kf(ctx(), &g, &k1, &k2, mbCheckOrientation ? 1 : 0, bCoarse ? 1 : 0,
                                                   out.data());
    throwOn(nm, "mam_search_for_triangulation_kf");
    vMatchedPairs.reserve(nm);
    for (int i = 0; i < n1; i++)   // ORBmatcher.cc:1135-1143: ascending idx1
        if (out[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)out[i]));
    return nm;
}

int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th, const bool bRight) {
    if (bRight) throw std::invalid_argument("Fuse(bRight=true): stereo is out of scope (mono agents)");
    mam_fuse_kf kf;
    kf.tcw = pKF->GetPose().toC();
    pKF->GetCameraCenter(kf.ow);
    kf.log_scale_factor = pKF->mfLogScaleFactor;
    const size_t M = vpMapPoints.size();
    std::vector<mam_fuse_mp> mps(M);
    for (size_t i = 0; i < M; i++) {
        mam_fuse_mp& m = mps[i];
        std::memset(&m, 0, sizeof(m));
        MapPoint* pMP = vpMapPoints[i];
        if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;   // ORBmatcher.cc:1181-1196
        m.valid = 1;
        pMP->GetWorldPos(m.pos);
        pMP->GetNormal(m.normal);
        m.max_distance = pMP->GetMaxDistance();
        m.min_distance = pMP->GetMinDistance();
        pMP->GetDescriptor(m.desc);
    }
    std::vector<int32_t> idx(M > 0 ? M : 1, -1), dist(M > 0 ? M : 1, 256);
    const mam_frame_geom g = pKF->Geom();
    const mam_pinhole cam = pKF->mpCamera->toC();
    throwOn(mam_fuse(ctx(), &g, pKF->N, reinterpret_cast<const mam_keypoint*>(pKF->mvKeysUn.data()),
                     pKF->mDescriptors.data.data(), &kf, &cam, (int)M, mps.data(), th, idx.data(), dist.data()),
            "mam_fuse");
    // ORBmatcher.cc:1177-1335 in list order; the isBad / IsInKeyFrame tests see the effects of earlier MapPoints
    int nFused = 0;
    for (size_t i = 0; i < M; i++) {
        MapPoint* pMP = vpMapPoints[i];
        if (!pMP) continue;
        if (pMP->isBad()) continue;
        else if (pMP->IsInKeyFrame(pKF)) continue;
        if (idx[i] < 0) continue;   // a geometric `continue` or bestDist > TH_LOW
        const int bestIdx = idx[i];
        MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

void ORBmatcher::ComputeDistinctiveDescriptors(const std::vector<MapPoint*>& vpMapPoints) {
    // MapPoint.cc:331-366: the descriptors of the non-bad observing keyframes, in observation (std::map) order
    std::vector<int32_t> off(1, 0);
    std::vector<uint8_t> descs;
    std::vector<MapPoint*> todo;
    for (MapPoint* pMP : vpMapPoints) {
        if (!pMP || pMP->isBad()) continue;
        const std::map<KeyFrame*, std::tuple<int, int>> observations = pMP->GetObservations();
        const size_t before = descs.size();
        for (const auto& o : observations) {
            KeyFrame* pKF = o.first;
            if (pKF->isBad()) continue;
            for (const int i : {std::get<0>(o.second), std::get<1>(o.second)})
                if (i != -1) descs.insert(descs.end(), pKF->mDescriptors.ptr(i), pKF->mDescriptors.ptr(i) + 32);
        }
        if (descs.size() == before) continue;   // no descriptor: unchanged (:343-344, :365-366)
        todo.push_back(pMP);
        off.push_back((int32_t)(descs.size() / 32));
    }
    if (todo.empty()) return;
    std::vector<int32_t> best(todo.size());
    throwOn(mam_compute_distinctive_descriptors(ctx(), (int)todo.size(), off.data(), descs.data(), best.data()),
            "mam_compute_distinctive_descriptors");
    for (size_t m = 0; m < todo.size(); m++) todo[m]->SetDescriptor(descs.data() + (size_t)(off[m] + best[m]) * 32);
}

}  // namespace MAM3SLAM
