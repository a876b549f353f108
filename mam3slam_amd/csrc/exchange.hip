// Shared-map update exchange: each agent packs the deduplicated write-back of its step's LocalBundleAdjustment windows
// into one compact block, and every agent applies the all-gathered blocks in agent order (include/mam_exchange.h,
// SURVEY.md §8(e)); plus the windows' vertex estimates read from the shared tables.
// Reference semantics of the values: src/Optimizer.cc:1478-1494 (KeyFrame::SetPose(SE3f(q.cast<float>,
// t.cast<float>)), MapPoint::SetWorldPos(pos.cast<float>)).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/mam_exchange.h"
#include "../../include/mam_orb.h"
#include "runtime.hpp"

namespace mam {

// grid (ceil(max(P, L) / 256), n_windows): the window's vertex estimates from the shared tables, the float map values
// cast to double as the reference builds its graph (Optimizer.cc:1218, 1235: SE3Quat(GetPose().unit_quaternion()
// .cast<double>(), translation().cast<double>()); :1286: GetWorldPos().cast<double>())
__global__ __launch_bounds__(256) void k_read_windows(const float* __restrict__ kf, int64_t kf_cap,
                                                      const float* __restrict__ mp, int64_t mp_cap, int64_t mp_id_base,
                                                      const mam_map_window* __restrict__ win,
                                                      int32_t* __restrict__ status) {
    const mam_map_window& w = win[blockIdx.y];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < w.n_poses) {
        const int64_t id = w.pose_id[i];
        if (id < 0 || id >= kf_cap) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            const float* s = kf + id * 8;
            for (int k = 0; k < 4; k++) w.pose_q[4 * (size_t)i + k] = (double)s[k];
            for (int k = 0; k < 3; k++) w.pose_t[3 * (size_t)i + k] = (double)s[4 + k];
        }
    }
    if (i < w.n_points) {
        const int64_t r = w.point_id[i] - mp_id_base;
        if (r < 0 || r >= mp_cap) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            for (int k = 0; k < 3; k++) w.point_xyz[3 * (size_t)i + k] = (double)mp[r * 4 + k];
        }
    }
}

// ---- compact blocks: one per agent, the deduplicated write-back of all its windows (mam_exchange_pack_sources)
__host__ __device__ inline size_t compact_block_bytes(int kf_cap, int mp_cap) {
    return sizeof(mam_update_header) + (size_t)kf_cap * sizeof(mam_kf_update) + (size_t)mp_cap * sizeof(mam_mp_update);
}

// grid (ceil(max(n_kf, n_mp) / 256)): record i of each list from its source (window, vertex index)
__global__ __launch_bounds__(256) void k_pack_sources(const mam_map_window* __restrict__ win,
                                                      const int32_t* __restrict__ kf_src, int n_kf,
                                                      const int32_t* __restrict__ mp_src, int n_mp, int64_t mp_id_base,
                                                      int agent, uint8_t* __restrict__ block, int kf_cap, int mp_cap) {
    mam_update_header* h = reinterpret_cast<mam_update_header*>(block);
    mam_kf_update* K = reinterpret_cast<mam_kf_update*>(block + sizeof(mam_update_header));
    mam_mp_update* M = reinterpret_cast<mam_mp_update*>(block + sizeof(mam_update_header) +
                                                        (size_t)kf_cap * sizeof(mam_kf_update));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        mam_update_header hh;
        hh.n_kf = n_kf;
        hh.n_mp = n_mp;
        hh.agent = agent;
        hh.status = (n_kf > kf_cap || n_mp > mp_cap) ? MAM_ERR_CAPACITY : 0;
        *h = hh;
    }
    if (i < n_kf && i < kf_cap) {
        const mam_map_window& w = win[kf_src[2 * i]];
        const int v = kf_src[2 * i + 1];
        mam_kf_update u;
        u.row = (int32_t)w.pose_id[v];
        // KeyFrame::SetPose(SE3f(q.cast<float>(), t.cast<float>())) (Optimizer.cc:1478-1486): Sophus normalises the
        // float quaternion, coeffs / norm() with the norm as Eigen's SSE packet reduction sums the 4 floats,
        // (x^2 + z^2) + (y^2 + w^2) — the same order as Frame::SetPose in pose.hip
        float q[4];
        for (int k = 0; k < 4; k++) q[k] = (float)w.pose_q[4 * (size_t)v + k];
        const float nq = sqrtf((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
        for (int k = 0; k < 4; k++) u.q[k] = q[k] / nq;
        for (int k = 0; k < 3; k++) u.t[k] = (float)w.pose_t[3 * (size_t)v + k];
        K[i] = u;
    }
    if (i < n_mp && i < mp_cap) {
        const mam_map_window& w = win[mp_src[2 * i]];
        const int v = mp_src[2 * i + 1];
        mam_mp_update u;
        const int32_t row = (int32_t)(w.point_id[v] - mp_id_base);
        u.row = (w.point_bad && w.point_bad[v]) ? (int32_t)((uint32_t)row | 0x80000000u) : row;
        for (int k = 0; k < 3; k++) u.xyz[k] = (float)w.point_xyz[3 * (size_t)v + k];   // SetWorldPos(pos.cast<float>())
        M[i] = u;
    }
}

// one agent's compact block (launched per agent, in agent order); rows within a block are unique
__global__ __launch_bounds__(256) void k_apply_compact(const uint8_t* __restrict__ block, int kf_cap, int mp_cap,
                                                       float* __restrict__ kf, int64_t kf_rows, float* __restrict__ mp,
                                                       int64_t mp_rows, int32_t* __restrict__ status) {
    const mam_update_header h = *reinterpret_cast<const mam_update_header*>(block);
    if (h.status != 0 || h.n_kf < 0 || h.n_kf > kf_cap || h.n_mp < 0 || h.n_mp > mp_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(status, MAM_ERR_ARG);
        return;
    }
    const mam_kf_update* K = reinterpret_cast<const mam_kf_update*>(block + sizeof(mam_update_header));
    const mam_mp_update* M = reinterpret_cast<const mam_mp_update*>(block + sizeof(mam_update_header) +
                                                                    (size_t)kf_cap * sizeof(mam_kf_update));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < h.n_kf) {
        const mam_kf_update u = K[i];
        if (u.row >= 0 && u.row < kf_rows) {
            float* d = kf + (size_t)u.row * 8;
            for (int k = 0; k < 4; k++) d[k] = u.q[k];
            for (int k = 0; k < 3; k++) d[4 + k] = u.t[k];
            d[7] = 1.0f;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
    if (i < h.n_mp) {
        const mam_mp_update u = M[i];
        const int32_t row = (int32_t)((uint32_t)u.row & 0x7fffffffu);
        if (row < mp_rows) {
            float* d = mp + (size_t)row * 4;
            for (int k = 0; k < 3; k++) d[k] = u.xyz[k];
            d[3] = ((uint32_t)u.row & 0x80000000u) ? 1.0f : 0.0f;
        } else {
            atomicExch(status, MAM_ERR_ARG);
        }
    }
}

}  // namespace mam

extern "C" size_t mam_exchange_compact_block_bytes(int kf_cap, int mp_cap) {
    return (kf_cap < 0 || mp_cap < 0) ? 0 : mam::compact_block_bytes(kf_cap, mp_cap);
}

extern "C" int mam_exchange_pack_sources(int n_windows, const mam_map_window* windows, const int32_t* kf_src, int n_kf,
                                         const int32_t* mp_src, int n_mp, int64_t mp_id_base, int agent, void* block,
                                         int kf_cap, int mp_cap, void* stream) {
    if (n_windows < 0 || n_kf < 0 || n_mp < 0 || kf_cap < 0 || mp_cap < 0 || !block ||
        ((n_kf || n_mp) && (!windows || n_windows == 0)) || (n_kf && !kf_src) || (n_mp && !mp_src))
        return MAM_ERR_ARG;
    if (n_kf > kf_cap || n_mp > mp_cap) return MAM_ERR_CAPACITY;
    const int n = std::max(1, std::max(n_kf, n_mp));
    hipLaunchKernelGGL(mam::k_pack_sources, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, windows, kf_src,
                       n_kf, mp_src, n_mp, mp_id_base, agent, reinterpret_cast<uint8_t*>(block), kf_cap, mp_cap);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_exchange_apply_compact(const void* gathered, int n_agents, int kf_cap, int mp_cap,
                                          float* kf_table, int64_t kf_rows, float* mp_table, int64_t mp_rows,
                                          int32_t* status, void* stream) {
    if (!gathered || n_agents < 1 || kf_cap < 0 || mp_cap < 0 || !kf_table || !mp_table || !status) return MAM_ERR_ARG;
    const size_t bb = mam::compact_block_bytes(kf_cap, mp_cap);
    const int n = std::max(1, std::max(kf_cap, mp_cap));
    for (int a = 0; a < n_agents; a++) {
        hipLaunchKernelGGL(mam::k_apply_compact, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const uint8_t*>(gathered) + (size_t)a * bb, kf_cap, mp_cap, kf_table,
                           kf_rows, mp_table, mp_rows, status);
        MAM_HIP(hipGetLastError());
    }
    return MAM_OK;
}

extern "C" int mam_map_read_windows(const float* kf_table, int64_t kf_cap, const float* mp_table, int64_t mp_cap,
                                    int64_t mp_id_base, int n_windows, const mam_map_window* windows, int max_rows,
                                    int32_t* status, void* stream) {
    if (!kf_table || !mp_table || !status || n_windows < 0 || max_rows < 0 || (n_windows > 0 && !windows))
        return MAM_ERR_ARG;
    if (n_windows == 0 || max_rows == 0) return MAM_OK;
    hipLaunchKernelGGL(mam::k_read_windows, dim3((max_rows + 255) / 256, n_windows), dim3(256), 0, (hipStream_t)stream,
                       kf_table, kf_cap, mp_table, mp_cap, mp_id_base, windows, status);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}
