/*
 * mam_match.h — C-ABI drop-in boundary for MAM3SLAM's ORBmatcher hot-path searches (gfx950 / MI355X).
 *
 * Replaces (mono agents, Pinhole or KannalaBrandt8 camera, include/mam_camera.h):
 *   ORBmatcher::DescriptorDistance(a, b)                          reference: src/ORBmatcher.cc:2058-2074
 *   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
 *                                                                 reference: src/ORBmatcher.cc:43-213, 215-221
 *   ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th, bMono)
 *                                                                 reference: src/ORBmatcher.cc:1676-1887, 2012-2053
 *   ORBmatcher::SearchForTriangulation(KF1, KF2, vMatchedPairs, bOnlyStereo=false, bCoarse)
 *                                                                 reference: src/ORBmatcher.cc:907-1146
 *   ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight=false)          reference: src/ORBmatcher.cc:1148-1338
 *   MapPoint::ComputeDistinctiveDescriptors()                     reference: src/MapPoint.cc:329-403
 *   with Frame::GetFeaturesInArea / PosInGrid / AssignFeaturesToGrid (src/Frame.cc:385-416, 657-735) built
 *   on the device, and GeometricCamera::project / epipolarConstrain (src/CameraModels/Pinhole.cpp:35-41, 107-129,
 *   src/CameraModels/KannalaBrandt8.cpp:67-84, 116-143, 216-220, 306-406).
 *
 * Pointers/objects of the reference become indices: a Frame's mvpMapPoints is passed as `taken` flags
 * (1 = slot holds a MapPoint with Observations() > 0, the only property the searches read) and results come
 * back as per-keypoint indices of the matched MapPoint / last-frame keypoint (-1 = untouched). The
 * ORBmatcher wrapper (mam3slam_amd/match.py) maps indices back to objects.
 *
 * Every search exists in two forms: a synchronous host-pointer call with the reference's one-frame
 * semantics, and a batched device-pointer call (many frames / keyframe pairs per launch, asynchronous on a
 * stream) used by the multi-agent harness and bench.py.
 */
#ifndef MAM_MATCH_H
#define MAM_MATCH_H

#include <stddef.h>
#include <stdint.h>

#include "mam_camera.h"
#include "mam_orb.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MAM_GRID_COLS 64 /* FRAME_GRID_COLS, include/Frame.h */
#define MAM_GRID_ROWS 48 /* FRAME_GRID_ROWS */
#define MAM_TH_HIGH 100
#define MAM_TH_LOW 50
#define MAM_HISTO_LENGTH 30
/* out_kp_to_last value for a keypoint the rotation check un-assigned: the reference sets
 * CurrentFrame.mvpMapPoints[i] = NULL there (ORBmatcher.cc:1876-1881), clearing whatever it held. */
#define MAM_MATCH_CLEARED (-2)

/* Frame-level geometry shared by every frame of a call (one agent = one camera). */
typedef struct mam_frame_geom {
    float min_x, max_x, min_y, max_y;   /* mnMinX.. (Frame.cc:782-809) */
    float grid_inv_w, grid_inv_h;       /* mfGridElementWidthInv / HeightInv (Frame.cc:341-342) */
    int32_t nlevels;
    float scale_factors[MAM_MAX_LEVELS];/* mvScaleFactors */
    float level_sigma2[MAM_MAX_LEVELS]; /* mvLevelSigma2 */
} mam_frame_geom;

/* MapPoint fields SearchByProjection(F, vpMapPoints) reads (ORBmatcher.cc:49-90), filled by
 * Frame::isInFrustum (Frame.cc:512-586). 64 bytes. */
typedef struct mam_mp_track {
    float proj_x, proj_y;     /* mTrackProjX / mTrackProjY */
    float view_cos;           /* mTrackViewCos */
    float track_depth;        /* mTrackDepth */
    int32_t track_in_view;    /* mbTrackInView */
    int32_t scale_level;      /* mnTrackScaleLevel */
    int32_t is_bad;           /* isBad() */
    int32_t nobs;             /* Observations() */
    uint8_t desc[32];         /* GetDescriptor() */
} mam_mp_track;

/* MapPoint fields Tracking::SearchLocalPoints and Frame::isInFrustum read (Tracking.cc:3103-3139, Frame.cc:512-571,
 * MapPoint::PredictScale MapPoint.cc:531-546). 80 bytes. */
typedef struct mam_local_mp {
    float pos[3];             /* GetWorldPos() */
    float max_distance;       /* mfMaxDistance (GetMaxDistanceInvariance() = 1.2f * it; PredictScale's ratio) */
    float normal[3];          /* GetNormal() */
    float min_distance;       /* mfMinDistance (GetMinDistanceInvariance() = 0.8f * it) */
    int32_t is_bad;           /* isBad() */
    int32_t nobs;             /* Observations() */
    int32_t seen;             /* mnLastFrameSeen == CurrentFrame.mnId: already in the frame (skipped, not in view) */
    int32_t pad;
    uint8_t desc[32];         /* GetDescriptor() */
} mam_local_mp;

/* Sophus::SE3f as stored: unit quaternion (x, y, z, w) + translation. */
typedef struct mam_pose {
    float q[4];
    float t[3];
} mam_pose;

/* Cameras: mam_camera (mam_camera.h) — Pinhole or KannalaBrandt8; mam_pinhole is its round-1 name. Every
 * projection below goes through the camera's project (Pinhole.cpp:35-41 / KannalaBrandt8.cpp:67-84). */

/* Last-frame entry for SearchByProjection(Cur, Last) (ORBmatcher.cc:1695-1712). 64 bytes. */
typedef struct mam_last_entry {
    float pos[3];             /* pMP->GetWorldPos() */
    float angle;              /* LastFrame.mvKeysUn[i].angle */
    int32_t octave;           /* LastFrame.mvKeys[i].octave */
    int32_t valid;            /* mvpMapPoints[i] != NULL && !mvbOutlier[i] */
    int32_t nobs;             /* pMP->Observations() */
    int32_t pad;
    uint8_t desc[32];         /* pMP->GetDescriptor() */
} mam_last_entry;

/* MapPoint fields ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight=false) reads (ORBmatcher.cc:1179-1256). 80 bytes. */
typedef struct mam_fuse_mp {
    float pos[3];             /* GetWorldPos() */
    float max_distance;       /* mfMaxDistance: GetMaxDistanceInvariance() = 1.2f * it, PredictScale's ratio */
    float normal[3];          /* GetNormal() */
    float min_distance;       /* mfMinDistance: GetMinDistanceInvariance() = 0.8f * it */
    int32_t valid;            /* pMP != NULL && !pMP->isBad() && !pMP->IsInKeyFrame(pKF) (ORBmatcher.cc:1181-1196) */
    int32_t pad[3];
    uint8_t desc[32];         /* GetDescriptor() */
} mam_fuse_mp;

/* The keyframe side of a Fuse: Tcw, camera centre and mfLogScaleFactor (log of the float scale factor). */
typedef struct mam_fuse_kf {
    mam_pose tcw;             /* GetPose() */
    float ow[3];              /* GetCameraCenter() */
    float log_scale_factor;   /* mfLogScaleFactor (MapPoint::PredictScale, MapPoint.cc:514-529) */
} mam_fuse_kf;

/* DBoW2::FeatureVector flattened: node ids ascending, node_off[n_nodes+1] into feats (feature indices). */
typedef struct mam_featvec {
    int32_t n_nodes;
    const uint32_t* node_ids;
    const int32_t* node_off;
    const uint32_t* feats;
} mam_featvec;

typedef struct mam_match_ctx mam_match_ctx;

int mam_match_create(int device, mam_match_ctx** out);
void mam_match_destroy(mam_match_ctx* ctx);

/* DescriptorDistance over n pairs (rows of a and b, 32 B each). Host pointers. */
int mam_descriptor_distance(mam_match_ctx* ctx, const uint8_t* a, const uint8_t* b, int n, int32_t* out);

/* SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints) with ORBmatcher(nnratio).
 * F: n keypoints (mvKeysUn), descriptors n x 32, taken[n] (may be NULL).
 * out_kp_to_mp[n]: index of the MapPoint assigned to keypoint i in this call, else -1.
 * Returns nmatches (>= 0) or a negative MAM_ERR_*. */
int mam_search_by_projection(mam_match_ctx* ctx, const mam_frame_geom* geom, int n, const mam_keypoint* keys,
                             const uint8_t* desc, const uint8_t* taken, int n_mps, const mam_mp_track* mps,
                             float th, int far_points, float th_far_points, float nnratio, int32_t* out_kp_to_mp);

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono) with ORBmatcher(nnratio, checkOri).
 * out_kp_to_last[n_cur]: index i of the last-frame entry whose MapPoint was assigned, MAM_MATCH_CLEARED (-2)
 * if the assignment was removed by the rotation-consistency pass (slot must become NULL), else -1 (untouched). tlw/mb are only read when !mono (bForward/bBackward, ORBmatcher.cc:1688-1692). */
int mam_search_by_projection_motion(mam_match_ctx* ctx, const mam_frame_geom* geom, int n_cur,
                                    const mam_keypoint* keys, const uint8_t* desc, const uint8_t* taken,
                                    const mam_pose* tcw, const mam_pose* tlw, float mb, const mam_camera* cam,
                                    int n_last, const mam_last_entry* last, float th, int mono, int check_ori,
                                    int32_t* out_kp_to_last);

/* SearchForTriangulation(KF1, KF2, pairs, bOnlyStereo=false, bCoarse) with ORBmatcher(nnratio, checkOri)
 * for mono Pinhole keyframes. F12 (row-major 3x3, float) is the epipolarConstrain fundamental matrix
 * K1^-T [t12]x R12 K2^-1 and ep the epipole of KF1's centre in KF2 — both per pair, computed by the
 * wrapper. has_mp1/has_mp2: GetMapPoint(idx) != NULL. out_match12[n1]: idx2 or -1; returns nmatches. */
int mam_search_for_triangulation(mam_match_ctx* ctx, const mam_frame_geom* geom, int n1, const mam_keypoint* keys1,
                                 const uint8_t* desc1, const uint8_t* has_mp1, const mam_featvec* fv1, int n2,
                                 const mam_keypoint* keys2, const uint8_t* desc2, const uint8_t* has_mp2,
                                 const mam_featvec* fv2, const float* F12, const float* ep, int check_ori,
                                 int coarse, int32_t* out_match12);

/* The keyframe side of SearchForTriangulation(pKF1, pKF2, ...): mvKeysUn, mDescriptors, GetMapPoint(i) != NULL,
 * mFeatVec, GetPose() and mpCamera. */
typedef struct mam_tri_kf {
    int32_t n;
    const mam_keypoint* keys;
    const uint8_t* desc;
    const uint8_t* has_mp;
    mam_featvec fv;
    mam_pose tcw;
    mam_camera cam;
} mam_tri_kf;

/* SearchForTriangulation(pKF1, pKF2, pairs, bOnlyStereo=false, bCoarse) for mono keyframes with Pinhole or
 * KannalaBrandt8 cameras (ORBmatcher.cc:907-1146): the pair geometry of ORBmatcher.cc:913-930 (T12, the epipole) is
 * computed here (mam_triangulation_geometry), then pCamera1->epipolarConstrain(pCamera2, ...): the F12 line test
 * (Pinhole.cpp:107-129) or the two-view triangulation (KannalaBrandt8.cpp:216-220, 306-406). out_match12[kf1->n]:
 * idx2 or -1; returns nmatches. */
int mam_search_for_triangulation_kf(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_tri_kf* kf1,
                                    const mam_tri_kf* kf2, int check_ori, int coarse, int32_t* out_match12);

/* SearchForTriangulation's pair geometry (ORBmatcher.cc:913-930, Pinhole.cpp:109-112): T12 = T1w * T2w^-1 as R12
 * (row-major 3x3) and t12, F12 = K1^T^-1 [t12]x R12 K2^-1 (row-major; meaningful for Pinhole cameras) and ep = cam2's
 * projection of KF1's centre. Any output may be NULL. Host-only arithmetic, no device work. */
int mam_triangulation_geometry(const mam_pose* t1w, const mam_pose* t2w, const mam_camera* cam1,
                               const mam_camera* cam2, float* R12, float* t12, float* F12, float* ep);

/* ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight=false) for a mono keyframe (ORBmatcher.cc:1148-1338):
 * the per-MapPoint search. keys/desc = pKF->mvKeysUn / mDescriptors (n keypoints). out_idx[i] = the keypoint
 * MapPoint i fuses with (bestDist <= TH_LOW), else -1; out_dist[i] = bestDist (256 = no candidate passed). The
 * replace-or-add side effects (:1311-1330) are the caller's, applied in list order with the isBad / IsInKeyFrame
 * tests re-evaluated: they never change another MapPoint's search. Returns the number of
 * MapPoints with out_idx >= 0. */
int mam_fuse(mam_match_ctx* ctx, const mam_frame_geom* geom, int n, const mam_keypoint* keys, const uint8_t* desc,
             const mam_fuse_kf* kf, const mam_camera* cam, int n_mps, const mam_fuse_mp* mps, float th,
             int32_t* out_idx, int32_t* out_dist);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403) for n_mps MapPoints at once: MapPoint m's observed
 * descriptors are rows desc_off[m] .. desc_off[m+1]-1 of descs (32 B each), in the caller's observation order (the
 * reference's std::map<KeyFrame*> order, non-bad keyframes). out_best[m] = the row (relative to desc_off[m]) with
 * the least median Hamming distance to the others, first on ties; -1 for a MapPoint without descriptors. */
int mam_compute_distinctive_descriptors(mam_match_ctx* ctx, int n_mps, const int32_t* desc_off, const uint8_t* descs,
                                        int32_t* out_best);

/* ---- batched device-resident forms (asynchronous on `stream`; NULL = the context's stream) ---------- */

/* A batch of frames laid out as the extractor's batched output: frame f's keypoints at
 * keys + f*kp_stride, descriptors at desc + f*kp_stride*32, count counts[2f]. */
typedef struct mam_frames_dev {
    int32_t nframes;
    int32_t kp_stride;
    const mam_keypoint* keys;
    const uint8_t* desc;
    const int32_t* counts;
    const uint8_t* taken;     /* [nframes][kp_stride] or NULL */
    uint8_t* taken_out;       /* [nframes][kp_stride] or NULL: the slot state after a projection search (1 =
                                 mvpMapPoints[i] holds a MapPoint with Observations() > 0, rotation-cleared
                                 slots 0), i.e. the `taken` input of the frame's next search */
    int32_t reuse_grid;       /* nonzero: the frames' cell grid (AssignFeaturesToGrid, Frame.cc:385-416 — built once
                                 per Frame in the reference) is the one this context built in its previous search
                                 over the same keys/counts/nframes/kp_stride; the search skips rebuilding it
                                 (MAM_ERR_ARG if the context's last search was over other frames) */
} mam_frames_dev;

/* A batch of keyframes in device memory for SearchForTriangulation (LocalMapping::CreateNewMapPoints runs it against
 * the new keyframe's 30 best covisible keyframes, LocalMapping.cc:504-582). kfs: the keyframe slots in the extractor's
 * batched layout (nframes = keyframes; taken / taken_out / reuse_grid unused). has_mp[k][i]: GetMapPoint(i) != NULL.
 * The FeatureVector of slot k is given as the BoW transform's per-feature node and weight
 * (mam_bow_transform_batch_device out_nid / out_weight at levelsup 4): feature i belongs to node nid[k][i] iff
 * weight[k][i] > 0 (DBoW2 does not add stopped words). pairs[q] = (kf1 slot, kf2 slot). */
typedef struct mam_tri_batch {
    mam_frames_dev kfs;
    const uint8_t* has_mp;     /* [nkf][kp_stride] */
    const uint32_t* nid;       /* [nkf][kp_stride] */
    const double* weight;      /* [nkf][kp_stride] */
    const mam_pose* tcw;       /* [nkf] GetPose() */
    int32_t npairs;
    const int32_t* pairs;      /* [npairs][2] */
} mam_tri_batch;

/* npairs SearchForTriangulation(pKF1, pKF2, pairs, false, bCoarse) in one set of launches, every keyframe with camera
 * `cam` (Pinhole or KannalaBrandt8): out_match12[q][i] = idx2 or -1 for i < kf1's count (kp_stride entries per pair),
 * out_nmatches[q]. Asynchronous on `stream` (NULL = the context's). kp_stride <= 8192. */
int mam_search_for_triangulation_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_camera* cam,
                                              const mam_tri_batch* batch, int check_ori, int coarse,
                                              int32_t* out_match12, int32_t* out_nmatches, void* stream);

/* Frame f matches n_mps[f] MapPoints at mps + f*mp_stride. Outputs at out_kp_to_mp + f*kp_stride and
 * out_nmatches[f]. */
int mam_search_by_projection_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_frames_dev* frames,
                                          const mam_mp_track* mps, int mp_stride, const int32_t* n_mps, float th,
                                          int far_points, float th_far_points, float nnratio,
                                          int32_t* out_kp_to_mp, int32_t* out_nmatches, void* stream);

/* Frame f (current) matches n_last[f] last-frame entries at last + f*last_stride with pose tcw[f]. */
int mam_search_by_projection_motion_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom,
                                                 const mam_frames_dev* frames, const mam_pose* tcw,
                                                 const mam_camera* cam, const mam_last_entry* last, int last_stride,
                                                 const int32_t* n_last, float th, int check_ori,
                                                 int32_t* out_kp_to_last, int32_t* out_nmatches, void* stream);

/* Tracking::TrackWithMotionModel's search (Tracking.cc:2811-2824), per frame of the batch: SearchByProjection(Cur,
 * Last, th, check_ori); where it found fewer than min_matches (the reference's 20) matches, the frame's matches are
 * cleared (fill(mvpMapPoints, NULL)) and the search runs again with 2 * th. out / out_nmatches hold each frame's final
 * search (the count the reference then tests against 20 before PoseOptimization). frames->reuse_grid must be 0 (the
 * call builds the grid). Asynchronous; min_matches = 0 is the plain batch search. */
int mam_track_motion_search_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_frames_dev* frames,
                                         const mam_pose* tcw, const mam_camera* cam, const mam_last_entry* last,
                                         int last_stride, const int32_t* n_last, float th, int check_ori,
                                         int min_matches, int32_t* out_kp_to_last, int32_t* out_nmatches,
                                         void* stream);

/* Fuse into many keyframes in one launch (SearchInNeighbors' forward direction, LocalMapping.cc:881-890): keyframe f
 * (frames: its keypoints) with kfs[f] searches n_mps[f] MapPoints at mps + f*mp_stride. Outputs at
 * out_idx / out_dist + f*mp_stride and out_nfused[f]. */
/* Fuse(pKF, vpMapPoints, th) for n_items (keyframe, MapPoint list) pairs over one device-resident keyframe set:
 * SearchInNeighbors' two directions (LocalMapping.cc:881-918), the current keyframe's MapPoints into each target
 * keyframe and the targets' fuse candidates into the current keyframe, where one keyframe and one MapPoint list serve
 * many pairs. Item b fuses MapPoint list mp_of[b] (mps + mp_of[b] * mp_stride, n_mps[mp_of[b]] entries) into keyframe
 * frame_of[b] of `frames` (its pose kf_tcw[frame_of[b]] = GetPose(), the camera centre derived as
 * KeyFrame::GetCameraCenter does; log_scale_factor = mfLogScaleFactor); every keyframe's cell grid is built once per
 * call. Results as mam_fuse_batch_device's per item: out_idx / out_dist + b * mp_stride, out_nfused[b]. */
int mam_fuse_items_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_frames_dev* frames,
                                const mam_pose* kf_tcw, float log_scale_factor, const mam_camera* cam, int n_items,
                                const int32_t* frame_of, const int32_t* mp_of, const mam_fuse_mp* mps, int mp_stride,
                                const int32_t* n_mps, float th, int32_t* out_idx, int32_t* out_dist,
                                int32_t* out_nfused, void* stream);

int mam_fuse_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_frames_dev* frames,
                          const mam_fuse_kf* kfs, const mam_camera* cam, const mam_fuse_mp* mps, int mp_stride,
                          const int32_t* n_mps, float th, int32_t* out_idx, int32_t* out_dist, int32_t* out_nfused,
                          void* stream);

/* ComputeDistinctiveDescriptors over device arrays (desc_off[n_mps+1], descs, out_best[n_mps]). */
int mam_compute_distinctive_descriptors_batch_device(mam_match_ctx* ctx, int n_mps, const int32_t* desc_off,
                                                     const uint8_t* descs, int32_t* out_best, void* stream);

/* Tracking::SearchLocalPoints' projection loop (Tracking.cc:3119-3139): Frame::isInFrustum(pMP, view_cos_limit)
 * (Frame.cc:512-571, mono) + MapPoint::PredictScale(dist, Frame*) (MapPoint.cc:531-546) for n_mps local
 * MapPoints of a frame with pose tcw (Sophus SE3f: mRcw = rotationMatrix(), mOw = inverse().translation()).
 * out[i] = the track fields SearchByProjection(F, vpMapPoints) reads (proj_x/proj_y = -1 where the projection left
 * the image; view_cos/track_depth/scale_level are 0 for a MapPoint not in view; is_bad, nobs and desc copied).
 * log_scale_factor = mfLogScaleFactor (log of the float scale factor). Returns nToMatch (MapPoints in view). */
int mam_is_in_frustum(mam_match_ctx* ctx, const mam_frame_geom* geom, const mam_pose* tcw, const mam_camera* cam,
                      float log_scale_factor, int n_mps, const mam_local_mp* mps, float view_cos_limit,
                      mam_mp_track* out);

/* Batched: frame f (pose tcw[f]) projects n_mps[f] MapPoints at mps + f*mp_stride into out + f*mp_stride (the mps
 * input of mam_search_by_projection_batch_device); out_n_to_match[f] (may be NULL) = nToMatch. */
int mam_is_in_frustum_batch_device(mam_match_ctx* ctx, const mam_frame_geom* geom, int nframes, const mam_pose* tcw,
                                   const mam_camera* cam, float log_scale_factor, const mam_local_mp* mps,
                                   int mp_stride, const int32_t* n_mps, float view_cos_limit, mam_mp_track* out,
                                   int32_t* out_n_to_match, void* stream);

int mam_match_set_profiling(mam_match_ctx* ctx, int enable);
/* ms_out/launches_out (7 entries): [0] grid build, [1] candidate gather, [2] greedy resolve, [3] triangulation,
 * [4] fuse, [5] distinctive descriptors, [6] frustum (isInFrustum + PredictScale). */
int mam_match_stage_times(mam_match_ctx* ctx, double* ms_out, int64_t* launches_out);

#ifdef __cplusplus
}
#endif
#endif /* MAM_MATCH_H */
