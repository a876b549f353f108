/*
 * mam_exchange.h — shared-map update exchange between agents (one agent per GPU), SURVEY.md §8(e).
 *
 * In the reference every agent's LocalMapping thread writes KeyFrame poses and MapPoint positions of a merged
 * Atlas map under Map::mMutexMapUpdate (src/Optimizer.cc:1463-1497: KeyFrame::SetPose, MapPoint::SetWorldPos,
 * erase of outlier observations -> MapPoint::SetBadFlag), and the other agents read them through shared
 * pointers. With one process per GPU there is no shared memory: after its LocalBundleAdjustment windows an agent
 * packs their write-back as fixed-size records, the records of all agents are all-gathered over RCCL (xGMI), and
 * every agent applies them to its device-resident copy of the shared tables in agent-id order. The reference's
 * interleaving is racy (last writer under the mutex wins); here the order is fixed (agent 0 first, highest
 * agent last), so every replica ends with identical bytes.
 *
 * Per step each agent sends ONE compact block: the write-back of all its LocalBundleAdjustment windows of the step,
 * deduplicated (mam_exchange_pack_sources); the gathered buffer is n_agents such blocks back to back
 * (torch.distributed.all_gather_into_tensor order = rank order), applied by mam_exchange_apply_compact.
 */
#ifndef MAM_EXCHANGE_H
#define MAM_EXCHANGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* An LBA window as the shared map sees it (DEVICE pointers): the vertex ids (pose_id = KeyFrame table row, point_id -
 * mp_id_base = MapPoint table row) and the window's double-precision vertex arrays — the LBA inputs for
 * mam_map_read_windows, the LBA results for mam_exchange_pack_sources. pose_fixed selects what the write-back
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

/* ---- Compact blocks: one per agent per step, the write-back of ALL its LBA windows of the step, deduplicated (each
 * KeyFrame / MapPoint once, with the value of the last window that optimised it: the value the per-window blocks,
 * applied in window order, would leave), in records sized to what changes. Block = header (16 B) | kf_cap KeyFrame
 * records (32 B) | mp_cap MapPoint records (16 B); gathered = n_agents blocks back to back, applied in agent order. */
typedef struct mam_update_header {
    int32_t n_kf, n_mp, agent, status;   /* status: MAM_ERR_CAPACITY when the lists did not fit */
} mam_update_header;
typedef struct mam_kf_update {
    int32_t row;                         /* KeyFrame table row (= pose_id) */
    float q[4];                          /* Tcw unit quaternion x, y, z, w as KeyFrame::SetPose stores it: the
                                            optimised double quaternion cast to float and renormalised as Sophus
                                            does (coeffs / norm(), norm summed (x^2 + z^2) + (y^2 + w^2)) */
    float t[3];
} mam_kf_update;
typedef struct mam_mp_update {
    int32_t row;                         /* MapPoint table row (point_id - mp_id_base); bit 31 = marked bad */
    float xyz[3];                        /* MapPoint::SetWorldPos(pos.cast<float>()) */
} mam_mp_update;

size_t mam_exchange_compact_block_bytes(int kf_cap, int mp_cap);

/* Pack the deduplicated write-back of n_windows LBA results (DEVICE window descriptors): KeyFrame record i from
 * kf_src[2 i] = window, kf_src[2 i + 1] = pose index in it (a non-fixed pose), MapPoint record i from mp_src[2 i],
 * mp_src[2 i + 1] (DEVICE arrays; the host builds them with the windows: every vertex once, from the last window
 * holding it). Asynchronous. */
int mam_exchange_pack_sources(int n_windows, const mam_map_window* windows, const int32_t* kf_src, int n_kf,
                              const int32_t* mp_src, int n_mp, int64_t mp_id_base, int agent, void* block,
                              int kf_cap, int mp_cap, void* stream);

/* Apply n_agents gathered compact blocks (DEVICE) to the tables, agent 0 first (rows within a block are unique).
 * A block with status != 0 or counts beyond the caps, or rows outside the tables, set *status to MAM_ERR_ARG. */
int mam_exchange_apply_compact(const void* gathered, int n_agents, int kf_cap, int mp_cap, float* kf_table,
                               int64_t kf_rows, float* mp_table, int64_t mp_rows, int32_t* status, void* stream);

/* ---- Device-side helpers of the harness around the path (bench.py / mam3slam_amd/mapping.py; no reference
 * counterpart): keyframes entering the LocalMapping queue and the synthetic map's new state, without host-side
 * tensor work inside the timed step. */

/* One table of a row copy: row r of the destination (dst + r * dst_stride) gets row src_row_offset + s of the source,
 * row_bytes bytes (DEVICE pointers; strides and sizes in bytes). */
typedef struct mam_row_table {
    const void* src;
    void* dst;
    int64_t row_bytes;
    int64_t src_stride;
    int64_t dst_stride;
    int64_t src_row_offset;
} mam_row_table;

/* Copy n <= 64 rows (src_rows[i] -> dst_rows[i], HOST arrays passed by value) of n_tables <= 8 tables in one launch;
 * with flags != NULL also flags[dst_rows[i] * flags_stride + j] = (flag_a[src_rows[i] * flag_stride + j] >= 0 ||
 * flag_b[...] >= 0) for j < flag_cols (a keyframe's "has a MapPoint" flags from Tracking's match lists).
 * Asynchronous. */
int mam_copy_rows(int n_tables, const mam_row_table* tables, int n, const int32_t* src_rows, const int32_t* dst_rows,
                  const int32_t* flag_a, const int32_t* flag_b, int64_t flag_stride, int flag_cols, uint8_t* flags,
                  int64_t flags_stride, void* stream);

/* The synthetic map's new keyframes at a perturbed state, deterministic in seed: KeyFrame rows kf_idx[i] (DEVICE
 * int64) get q += N(0, sigma_q) per component, renormalised, w >= 0, and t += N(0, sigma_t); MapPoint rows mp_idx[i]
 * get xyz += N(0, sigma_x) (counter-based normals). Rows outside the tables set *status to MAM_ERR_ARG.
 * Asynchronous. */
int mam_map_perturb(float* kf_table, int64_t kf_rows, const int64_t* kf_idx, int n_kf, float* mp_table,
                    int64_t mp_rows, const int64_t* mp_idx, int n_mp, uint64_t seed, float sigma_q, float sigma_t,
                    float sigma_x, int32_t* status, void* stream);

/* The LocalBundleAdjustment windows of the keyframes Tracking inserted are built on the device map
 * (include/mam_ringmap.h: mam_ringmap_windows, the reference's window rule over MapPoints shared by the keyframes). */

#ifdef __cplusplus
}
#endif
#endif /* MAM_EXCHANGE_H */
