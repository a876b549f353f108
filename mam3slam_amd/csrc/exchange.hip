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

// ---- harness helpers
struct RowCopyArgs {
    int n_tables, n;
    mam_row_table t[8];
    int32_t src[64], dst[64];
    const int32_t* fa;
    const int32_t* fb;
    int64_t f_stride;
    int f_cols;
    uint8_t* flags;
    int64_t flags_stride;
};

// grid (n, n_tables + 1) x 256: block (i, k) copies row i of table k (16-byte chunks when the row and both addresses
// allow, else bytes); k = n_tables: the flags of row i
__global__ __launch_bounds__(256) void k_copy_rows(const RowCopyArgs a) {
    const int i = blockIdx.x, k = blockIdx.y;
    if (k < a.n_tables) {
        const mam_row_table& t = a.t[k];
        const uint8_t* s = reinterpret_cast<const uint8_t*>(t.src) + (t.src_row_offset + a.src[i]) * t.src_stride;
        uint8_t* d = reinterpret_cast<uint8_t*>(t.dst) + (int64_t)a.dst[i] * t.dst_stride;
        if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)t.row_bytes) & 15) == 0) {
            const int64_t nv = t.row_bytes / 16;
            for (int64_t j = threadIdx.x; j < nv; j += 256)
                reinterpret_cast<uint4*>(d)[j] = reinterpret_cast<const uint4*>(s)[j];
        } else {
            for (int64_t j = threadIdx.x; j < t.row_bytes; j += 256) d[j] = s[j];
        }
    } else if (a.flags) {
        const int32_t* x = a.fa + (int64_t)a.src[i] * a.f_stride;
        const int32_t* y = a.fb + (int64_t)a.src[i] * a.f_stride;
        uint8_t* f = a.flags + (int64_t)a.dst[i] * a.flags_stride;
        for (int j = threadIdx.x; j < a.f_cols; j += 256) f[j] = (x[j] >= 0 || y[j] >= 0) ? 1 : 0;
    }
}

// counter-based standard normal (splitmix64 -> two uniforms -> Box-Muller)
__device__ inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ inline float normal_at(uint64_t seed, uint64_t ctr) {
    const uint64_t r = splitmix64(seed ^ splitmix64(ctr));
    const float u1 = ((uint32_t)(r >> 40) + 1u) * (1.0f / 16777217.0f);   // (0, 1]
    const float u2 = (uint32_t)(r & 0xffffffu) * (1.0f / 16777216.0f);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// grid ceil(max(n_kf, n_mp) / 256) x 256
__global__ __launch_bounds__(256) void k_perturb(float* __restrict__ kf, int64_t kf_rows, const int64_t* __restrict__ kf_idx,
                                                 int n_kf, float* __restrict__ mp, int64_t mp_rows,
                                                 const int64_t* __restrict__ mp_idx, int n_mp, uint64_t seed, float sq,
                                                 float st, float sx, int32_t* __restrict__ status) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_kf) {
        const int64_t r = kf_idx[i];
        if (r < 0 || r >= kf_rows) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            float* v = kf + r * 8;
            float q[4];
            for (int k = 0; k < 4; k++) q[k] = v[k] + sq * normal_at(seed, 16 * (uint64_t)i + k);
            const float nrm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            const float sg = q[3] < 0.0f ? -1.0f : 1.0f;
            for (int k = 0; k < 4; k++) v[k] = sg * (q[k] / nrm);
            for (int k = 0; k < 3; k++) v[4 + k] += st * normal_at(seed, 16 * (uint64_t)i + 4 + k);
        }
    }
    if (i < n_mp) {
        const int64_t r = mp_idx[i];
        if (r < 0 || r >= mp_rows) {
            atomicExch(status, MAM_ERR_ARG);
        } else {
            for (int k = 0; k < 3; k++) mp[r * 4 + k] += sx * normal_at(seed ^ 0x5bd1e995ull, 4 * (uint64_t)i + k);
        }
    }
}

}  // namespace mam

extern "C" int mam_copy_rows(int n_tables, const mam_row_table* tables, int n, const int32_t* src_rows,
                             const int32_t* dst_rows, const int32_t* flag_a, const int32_t* flag_b, int64_t flag_stride,
                             int flag_cols, uint8_t* flags, int64_t flags_stride, void* stream) {
    if (n_tables < 0 || n < 0 || (n_tables > 0 && !tables) || (n > 0 && (!src_rows || !dst_rows)) ||
        (flags && (!flag_a || !flag_b || flag_cols < 0)))
        return MAM_ERR_ARG;
    if (n_tables > 8 || n > 64) return MAM_ERR_CAPACITY;
    if (n == 0 || (n_tables == 0 && !flags)) return MAM_OK;
    mam::RowCopyArgs a{};
    a.n_tables = n_tables;
    a.n = n;
    for (int k = 0; k < n_tables; k++) {
        if (tables[k].row_bytes < 0 || (tables[k].row_bytes > 0 && (!tables[k].src || !tables[k].dst))) return MAM_ERR_ARG;
        a.t[k] = tables[k];
    }
    for (int i = 0; i < n; i++) {
        a.src[i] = src_rows[i];
        a.dst[i] = dst_rows[i];
    }
    a.fa = flag_a;
    a.fb = flag_b;
    a.f_stride = flag_stride;
    a.f_cols = flag_cols;
    a.flags = flags;
    a.flags_stride = flags_stride;
    hipLaunchKernelGGL(mam::k_copy_rows, dim3(n, n_tables + (flags ? 1 : 0)), dim3(256), 0, (hipStream_t)stream, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

extern "C" int mam_map_perturb(float* kf_table, int64_t kf_rows, const int64_t* kf_idx, int n_kf, float* mp_table,
                               int64_t mp_rows, const int64_t* mp_idx, int n_mp, uint64_t seed, float sigma_q,
                               float sigma_t, float sigma_x, int32_t* status, void* stream) {
    if (n_kf < 0 || n_mp < 0 || !status || (n_kf > 0 && (!kf_table || !kf_idx)) || (n_mp > 0 && (!mp_table || !mp_idx)))
        return MAM_ERR_ARG;
    const int n = std::max(n_kf, n_mp);
    if (n == 0) return MAM_OK;
    hipLaunchKernelGGL(mam::k_perturb, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, kf_table, kf_rows,
                       kf_idx, n_kf, mp_table, mp_rows, mp_idx, n_mp, (uint64_t)seed, sigma_q, sigma_t, sigma_x, status);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

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
