/*
 * mam_ringmap.h — the device-resident keyframe / MapPoint map LocalMapping works on (the harness around the
 * LocalBundleAdjustment hot path): MapPoint identities shared across keyframes, their
 * observation sets, and the map edits of the reference's LocalMapping run between two LocalBundleAdjustment calls,
 * so that the timed LBA windows are the reference's windows (Optimizer.cc:1118-1186) over a real covisibility graph.
 *
 * The map holds the keyframes of a ring of R slots (S keypoint slots each). A MapPoint is identified by its home
 * row id = slot * S + keypoint (the keypoint of its reference keyframe, MapPoint::mpRefKF); its record
 * (mam_fuse_mp: position, mfMaxDistance, normal, mfMinDistance, valid, descriptor — the fields ORBmatcher::Fuse
 * reads) lives at that row. Observations (MapPoint::mObservations, one keypoint per keyframe):
 *   mp_of[s S + k] = id of the MapPoint keypoint k of slot s observes (KeyFrame::mvpMapPoints), -1 none;
 *   okp[id R + s]  = keypoint of MapPoint id in slot s (-1: not observed), meaningful for live ids.
 * Invariants: rec[id].valid <=> live MapPoint homed at id, and then mp_of[id] == id; mp_of[e] = m >= 0 => okp[m R +
 * slot(e)] == keypoint(e). Observation order (the reference iterates std::map<KeyFrame*, ...> by pointer): ascending
 * slot. All edits are deterministic (no result depends on the order device threads run).
 *
 * One LocalMapping run processes the W keyframes a step inserted, at ring slots H = [head, head + W) (their
 * keypoints / descriptors / pose already copied into the slots), in the reference's order (LocalMapping::Run,
 * LocalMapping.cc:95-172): mam_ringmap_evict (the slots' previous keyframes leave the map: KeyFrame::SetBadFlag's
 * EraseObservation + MapPointCulling), mam_ringmap_create (CreateNewMapPoints' MapPoints from the SearchForTriangulation
 * matches), mam_ringmap_gather (the Fuse inputs), mam_ringmap_fuse_apply (Fuse's Replace / AddObservation side
 * effects), mam_ringmap_refresh (SearchInNeighbors' ComputeDistinctiveDescriptors + UpdateNormalAndDepth),
 * mam_ringmap_windows (LocalBundleAdjustment's window build), and after the solve mam_ringmap_writeback (outlier
 * erase, SetPose, SetWorldPos + UpdateNormalAndDepth, Optimizer.cc:1413-1497) and mam_ringmap_pack (the write-back as
 * exchange records). The rules each function restates, and where the batch of W keyframes deviates from the
 * reference's one-keyframe-at-a-time order, are documented per function; tests/ringmap_host.py restates every one
 * on the host and tests/test_ringmap_gpu.py compares the whole map state after each call.
 */
#ifndef MAM_RINGMAP_H
#define MAM_RINGMAP_H

#include <stddef.h>
#include <stdint.h>

#include "mam_match.h"
#include "mam_orb.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The map (DEVICE pointers; the caller owns every buffer). */
typedef struct mam_ringmap {
    int32_t R, S;                 /* ring slots (<= 128), keypoint slots per keyframe (<= 32767) */
    int32_t nlevels;              /* <= 8 */
    float scale_factors[8];       /* mvScaleFactors */
    float inv_level_sigma2[8];    /* mvInvLevelSigma2 */
    int32_t* mp_of;               /* [R S] */
    int16_t* okp;                 /* [R S][R] */
    mam_fuse_mp* rec;             /* [R S] MapPoint records at their home rows */
    int32_t* born;                /* [R S] step of creation */
    uint8_t* has_mp;              /* [R S] mp_of >= 0 (SearchForTriangulation's input flags) */
    mam_fuse_mp* lists;           /* [R S] per slot, per keypoint: the record of the MapPoint it observes (valid 0:
                                     none) — KeyFrame::GetMapPointMatches() as Fuse's MapPoint lists */
    const mam_keypoint* keys;     /* [R][S] mvKeysUn */
    const uint8_t* desc;          /* [R][S][32] */
    const int32_t* cnt;           /* [R][2] keypoint count in [2 s] */
    float* tcw;                   /* [R][7] Tcw q xyzw, t (KeyFrame::GetPose; the write-back's SetPose) */
    const mam_fuse_mp* kp_rec;    /* [R][S] per keypoint: the MapPoint CreateNewMapPoints makes there (position,
                                     descriptor; the harness's stand-in for the triangulated point) */
    /* scratch (R S each unless noted): */
    int32_t* parent;              /* union-find parents */
    int32_t* claim;               /* per keypoint: the lowest claimant */
    uint64_t* surv;               /* per component root: (observations << 32) | ~id of its survivor */
    uint8_t* flag;                /* per id: phase flags (involved / touched / erased / written / dead) */
    int32_t* newid;               /* per id: repair decision (-1 keep, -2 bad, >= 0 new home) / creation target */
    int32_t* lastw;               /* per id: last window writing its position */
    int32_t* slot_last;           /* [R] last window optimising the slot's pose */
    int32_t* pack_off;            /* [R S / 1024 + 2] pack scan scratch */
} mam_ringmap;

/* KeyFrame::SetBadFlag of the keyframes leaving slots [head, head + W) — every observation in them erased
 * (MapPoint::EraseObservation) — and MapPointCulling (LocalMapping.cc:457-501) over the map: a MapPoint left with
 * <= 2 observations is SetBadFlag'ed (mono nThObs = 2; every live MapPoint was created in an earlier step; the
 * found-ratio test needs Tracking's counters and is not restated). A surviving MapPoint whose home keypoint left moves
 * to its lowest remaining slot (EraseObservation's new mpRefKF = the first remaining observation). Asynchronous. */
int mam_ringmap_evict(const mam_ringmap* map, int head, int W, int step, void* stream);

/* has_mp from mp_of (all slots). Asynchronous. */
int mam_ringmap_flags(const mam_ringmap* map, void* stream);

/* CreateNewMapPoints (LocalMapping.cc:504-828) from the batch's SearchForTriangulation matches: new keyframe w
 * (slot head + w) against its NN neighbours pairs[(w NN + k) 2 + 1] (k in search order), match[(w NN + k) S + i1] =
 * the neighbour keypoint of keypoint i1 (-1 none). Keypoint i1 takes its first match in neighbour order; a neighbour
 * keypoint claimed by several new keyframes goes to the lowest (w, i1); the losing claims make no MapPoint (in the
 * reference the later keyframe's search would not have offered the taken keypoint). A MapPoint is created at home
 * (slot head + w, i1) with the two observations, record = kp_rec there, born = step. The triangulation's geometric
 * checks are not restated (the stand-in position is the scene point of the keypoint). Asynchronous. */
int mam_ringmap_create(const mam_ringmap* map, int head, int W, const int32_t* pairs, int NN, const int32_t* match,
                       int step, void* stream);

/* Fuse's MapPoint lists: lists[e] = rec[mp_of[e]] (valid 1) or valid 0. Asynchronous. */
int mam_ringmap_gather(const mam_ringmap* map, void* stream);

/* SearchInNeighbors' Fuse side effects (LocalMapping.cc:830-939, ORBmatcher.cc:1148-1338). Proposals: forward item
 * (w NN + k): MapPoint mp_of[(head + w) S + i] -> keypoint fwd_idx[(w NN + k) S + i] of neighbour k; backward item
 * (w NB + k), k < NB: MapPoint mp_of[nb_k S + i] of the k-th neighbour -> keypoint bwd_idx[(w NB + k) S + i] of the new
 * keyframe, skipped when an earlier backward neighbour observes the MapPoint (vpFuseCandidates' dedup). A proposal of a
 * MapPoint already observed in the target keyframe is skipped (IsInKeyFrame). A proposal onto a keypoint holding
 * another MapPoint merges the two (Replace); proposals onto a free keypoint claim it (AddObservation), and several
 * claimants of one keypoint merge (the later ones find the first's MapPoint there). Merges are resolved over their
 * connected components: the survivor is the member with the most observations (Observations() >, ties: lowest id),
 * it takes every member's observations and claimed keypoints with one keypoint per keyframe (its own first, then the
 * lowest member id's, then the lowest claimed keypoint); the other keypoints lose their MapPoint
 * (EraseMapPointMatch) and the other members die (mpMap->EraseMapPoint). The W keyframes' proposals are resolved
 * together. Asynchronous. */
int mam_ringmap_fuse_apply(const mam_ringmap* map, int head, int W, const int32_t* pairs, int NN, int NB,
                           const int32_t* fwd_idx, const int32_t* bwd_idx, void* stream);

/* SearchInNeighbors' "update points" (LocalMapping.cc:917-930): ComputeDistinctiveDescriptors (MapPoint.cc:329-403)
 * and UpdateNormalAndDepth (:426-494) of every MapPoint the keyframes in [head, head + W) observe. Asynchronous. */
int mam_ringmap_refresh(const mam_ringmap* map, int head, int W, void* stream);

/* LocalBundleAdjustment's window of new keyframe w (Optimizer.cc:1118-1186) into window w's buffers:
 * local keyframes = the keyframe + GetVectorCovisibleKeyFrames (KeyFrame::UpdateConnections, KeyFrame.cc:312-380:
 * weight = shared MapPoints, those >= covis_th by weight descending — ties by slot — or the heaviest when none
 * reaches it); local MapPoints = every MapPoint of every local keyframe, in local keyframe order then keypoint order,
 * each once; fixed keyframes = the other observers of local MapPoints, in order of first encounter (MapPoint order,
 * then slot order). Poses: local then fixed; edges: per MapPoint in order, its observations in slot order.
 * counts[4 w ..] = {poses, points, edges, optimised poses}; all zero when the window has no fixed keyframe (the
 * reference aborts, :1182-1185) or no MapPoint; -1 when it exceeds the caps (poses <= R, points <= pcap, edges <=
 * ecap). pose_slot[w R + i] = slot of pose i; point_id[w pcap + i] = MapPoint id of point i. */
typedef struct mam_ringmap_window {
    double* pose_q;               /* [R][4] */
    double* pose_t;               /* [R][3] */
    uint8_t* pose_fixed;          /* [R] */
    double* point_xyz;            /* [pcap][3] */
    int32_t* edge_point;          /* [ecap] */
    int32_t* edge_pose;
    double* edge_obs;             /* [ecap][2] */
    double* edge_inv_sigma2;
} mam_ringmap_window;

int mam_ringmap_windows(const mam_ringmap* map, int head, int W, int covis_th, const mam_ringmap_window* outs,
                        int pcap, int ecap, int32_t* counts, int32_t* pose_slot, int32_t* point_id, void* stream);

/* The write-back of the batch's solved windows (Optimizer.cc:1413-1497), windows applied in order: every edge with
 * chi2 > 5.991 or a non-positive depth erases its observation (EraseMapPointMatch + EraseObservation; a MapPoint
 * left with <= 2 observations is SetBadFlag'ed, one whose home keypoint was erased moves to its lowest remaining
 * slot); every optimised keyframe's pose from the last window optimising it (SetPose(SE3f(q.cast<float>,
 * t.cast<float>)), the quaternion renormalised as Sophus does); every local MapPoint's position from the last window
 * holding it (SetWorldPos(pos.cast<float>)) and UpdateNormalAndDepth. res[w] = window w's solve results (DEVICE
 * arrays, mam_lba_result layout on the device: pose_q, pose_t, point_xyz, edge_chi2, edge_depth_ok); windows with
 * counts[4 w + 2] <= 0 are skipped. The touched rows are flagged for mam_ringmap_pack. Asynchronous. */
typedef struct mam_ringmap_result {
    const double* pose_q;
    const double* pose_t;
    const double* point_xyz;
    const double* edge_chi2;
    const uint8_t* edge_depth_ok;
} mam_ringmap_result;

int mam_ringmap_writeback(const mam_ringmap* map, int W, const mam_ringmap_window* wins,
                          const mam_ringmap_result* res, const int32_t* counts, const int32_t* pose_slot,
                          const int32_t* point_id, int pcap, int ecap, void* stream);

/* The write-back as one exchange block (mam_exchange.h's compact layout with 48-byte MapPoint records): header |
 * kf_cap KeyFrame records (row = row_base_kf + slot) | mp_cap MapPoint records (row = row_base_mp + id, bit 31 = bad;
 * position, normal, mfMinDistance, mfMaxDistance), every keyframe / MapPoint the last writeback changed, in slot / id
 * order. Asynchronous. */
typedef struct mam_mp_record {
    int32_t row;
    float xyz[3];
    float normal[3];
    float min_distance;
    float max_distance;
    int32_t pad[3];
} mam_mp_record;

size_t mam_ringmap_block_bytes(int kf_cap, int mp_cap);
int mam_ringmap_pack(const mam_ringmap* map, int64_t row_base_kf, int64_t row_base_mp, int agent, void* block,
                     int kf_cap, int mp_cap, void* stream);
/* Apply n_agents gathered blocks in agent order to replica tables kf_table [kf_rows][8] (q, t, valid) and mp_table
 * [mp_rows][12] (xyz, bad, normal, min, max, pad). Rows outside the tables or a bad header set *status. */
int mam_ringmap_apply(const void* gathered, int n_agents, int kf_cap, int mp_cap, float* kf_table, int64_t kf_rows,
                      float* mp_table, int64_t mp_rows, int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAM_RINGMAP_H */
