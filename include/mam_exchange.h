/*
 * mam_exchange.h — shared-map update exchange between agents (one agent per GPU), SURVEY.md §8(e).
 *
 * In the reference every agent's LocalMapping thread writes KeyFrame poses and MapPoint positions of a merged
 * Atlas map under Map::mMutexMapUpdate (src/Optimizer.cc:1463-1497: KeyFrame::SetPose, MapPoint::SetWorldPos,
 * erase of outlier observations -> MapPoint::SetBadFlag), and the other agents read them through shared
 * pointers. With one process per GPU there is no shared memory: after each LocalBundleAdjustment an agent packs
 * its write-back as fixed-size records, the records of all agents are all-gathered over RCCL (xGMI), and every
 * agent applies them to its device-resident copy of the shared tables in agent-id order. The reference's
 * interleaving is racy (last writer under the mutex wins); here the order is fixed (agent 0 first, highest
 * agent last), so every replica ends with identical bytes.
 *
 * Buffer layout for one agent (one all-gather block): record 0 is a header (kind MAM_UPDATE_HEADER, id = number
 * of records that follow, agent = producer), records 1..capacity the updates. The gathered buffer is
 * n_agents such blocks back to back (torch.distributed.all_gather_into_tensor order = rank order).
 */
#ifndef MAM_EXCHANGE_H
#define MAM_EXCHANGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MAM_UPDATE_HEADER = 0, MAM_UPDATE_KF = 1, MAM_UPDATE_MP = 2 };

/* 64 bytes. KF: v = Tcw unit quaternion x, y, z, w then translation (what KeyFrame::SetPose receives,
 * Optimizer.cc:1478-1486). MP: v[0..2] = world position (MapPoint::SetWorldPos, :1489-1494), bad = the point
 * was marked bad by the outlier erase. */
typedef struct mam_map_update {
    int64_t id;
    int32_t kind;
    int32_t agent;
    float v[7];
    int32_t bad;
    float reserved[4];
} mam_map_update;

/* Pack one LocalBundleAdjustment write-back (DEVICE pointers, asynchronous on `stream`):
 *   poses: n_poses entries, pose_q [n][4] / pose_t [n][3] f64 (mam_lba_result order), pose_id, pose_fixed — only
 *          non-fixed poses are written back by the reference, so only those are packed;
 *   points: n_points entries, point_xyz [n][3] f64, point_id, point_bad (may be NULL).
 * Values are converted exactly like the write-back: quaternion and translation cast to float and the quaternion
 * renormalised in float (Sophus::SE3f constructor), positions cast to float.
 * out: capacity+1 records (header + updates). Returns MAM_ERR_CAPACITY if the update does not fit. */
int mam_exchange_pack_lba(const double* pose_q, const double* pose_t, const int64_t* pose_id,
                          const uint8_t* pose_fixed, int n_poses, const double* point_xyz, const int64_t* point_id,
                          const uint8_t* point_bad, int n_points, int agent, mam_map_update* out, int capacity,
                          void* stream);

/* An LBA window as the shared map sees it (DEVICE pointers): the vertex ids (pose_id = KeyFrame table row, point_id -
 * mp_id_base = MapPoint table row) and the window's double-precision vertex arrays — the LBA inputs for
 * mam_map_read_windows, the LBA results for mam_exchange_pack_windows. pose_fixed selects what the write-back
 * carries (non-fixed poses), point_bad may be NULL. */
typedef struct mam_map_window {
    int32_t n_poses;
    int32_t n_points;
    const int64_t* pose_id;
    const uint8_t* pose_fixed;
    const int64_t* point_id;
    const uint8_t* point_bad;
    double* pose_q;
    double* pose_t;
    double* point_xyz;
} mam_map_window;

/* Build the vertex estimates of n_windows LBA windows from the shared tables (Optimizer.cc:1218, 1235, 1286: the
 * float KeyFrame pose / MapPoint position cast to double): windows is a DEVICE array of descriptors; max_rows >=
 * every window's max(n_poses, n_points). Ids outside the tables set *status to MAM_ERR_ARG. Asynchronous. */
int mam_map_read_windows(const float* kf_table, int64_t kf_cap, const float* mp_table, int64_t mp_cap,
                         int64_t mp_id_base, int n_windows, const mam_map_window* windows, int max_rows,
                         int32_t* status, void* stream);

/* mam_exchange_pack_lba for n_windows LBA results in one launch: window w (DEVICE descriptor array, result arrays)
 * goes to block w of out (capacity + 1 records each); MapPoint record ids are point_id - mp_id_base. The blocks are
 * applied like agents' blocks (mam_exchange_apply with n_agents = all gathered windows, in order). */
int mam_exchange_pack_windows(int n_windows, const mam_map_window* windows, int64_t mp_id_base, int agent,
                              mam_map_update* out, int capacity, void* stream);

/* Apply gathered blocks (n_agents x (capacity+1) records, DEVICE) to device tables, agent 0 first:
 *   kf_table [kf_cap][8] floats (q xyzw, t, 1.0 = written), mp_table [mp_cap][4] floats (xyz, bad flag).
 * Records with an id outside the table or a malformed header set *status (device int32) to MAM_ERR_ARG and are
 * skipped. Asynchronous on `stream`. */
int mam_exchange_apply(const mam_map_update* gathered, int n_agents, int capacity, float* kf_table, int64_t kf_cap,
                       float* mp_table, int64_t mp_cap, int32_t* status, void* stream);

/* ---- Compact blocks: one per agent per step, the write-back of ALL its LBA windows of the step, deduplicated (each
 * KeyFrame / MapPoint once, with the value of the last window that optimised it: the value the per-window blocks,
 * applied in window order, would leave), in records sized to what changes. Block = header (16 B) | kf_cap KeyFrame
 * records (32 B) | mp_cap MapPoint records (16 B); gathered = n_agents blocks back to back, applied in agent order. */
typedef struct mam_update_header {
    int32_t n_kf, n_mp, agent, status;   /* status: MAM_ERR_CAPACITY when the lists did not fit */
} mam_update_header;
typedef struct mam_kf_update {
    int32_t row;                         /* KeyFrame table row (= pose_id) */
    float q[4];                          /* Tcw unit quaternion x, y, z, w as KeyFrame::SetPose stores it */
    float t[3];
} mam_kf_update;
typedef struct mam_mp_update {
    int32_t row;                         /* MapPoint table row (point_id - mp_id_base); bit 31 = marked bad */
    float xyz[3];                        /* MapPoint::SetWorldPos(pos.cast<float>()) */
} mam_mp_update;

size_t mam_exchange_compact_block_bytes(int kf_cap, int mp_cap);

/* Pack the deduplicated write-back of n_windows LBA results (DEVICE window descriptors, as for
 * mam_exchange_pack_windows): KeyFrame record i from kf_src[2 i] = window, kf_src[2 i + 1] = pose index in it (a
 * non-fixed pose), MapPoint record i from mp_src[2 i], mp_src[2 i + 1] (DEVICE arrays; the host builds them with the
 * windows: every vertex once, from the last window holding it). Asynchronous. */
int mam_exchange_pack_sources(int n_windows, const mam_map_window* windows, const int32_t* kf_src, int n_kf,
                              const int32_t* mp_src, int n_mp, int64_t mp_id_base, int agent, void* block,
                              int kf_cap, int mp_cap, void* stream);

/* Apply n_agents gathered compact blocks (DEVICE) to the tables, agent 0 first (rows within a block are unique).
 * A block with status != 0 or counts beyond the caps, or rows outside the tables, set *status to MAM_ERR_ARG. */
int mam_exchange_apply_compact(const void* gathered, int n_agents, int kf_cap, int mp_cap, float* kf_table,
                               int64_t kf_rows, float* mp_table, int64_t mp_rows, int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAM_EXCHANGE_H */
