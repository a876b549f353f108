// runtime.hpp — host-side helpers shared by the translation units of libmam_gpu.so: device buffers,
// HIP error capture (mam_last_error), and HIP-event stage timers for bench.py's live roofline.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/mam_orb.h"

namespace mam {

void set_last_error(const std::string& s);   // defined in orb_extract.hip (one thread_local string)

#define MAM_HIP(call)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            ::mam::set_last_error(std::string(#call) + ": " + hipGetErrorString(e_));            \
            return MAM_ERR_DEVICE;                                                               \
        }                                                                                        \
    } while (0)

// Switches the calling thread to a context's device for the duration of one C-ABI call and restores the caller's
// current device on return: an agent thread that drives GPU g keeps GPU g current across library calls.
struct DeviceScope {
    int prev = -1;
    bool ok = false;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(device) == hipSuccess;
        if (!ok) set_last_error("hipSetDevice failed");
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

#define MAM_DEVICE_SCOPE(dev)                               \
    ::mam::DeviceScope mam_dev_scope_(dev);                 \
    if (!mam_dev_scope_.ok) return MAM_ERR_DEVICE

// XCD-aware block order: the hardware deals linear workgroup ids round-robin over the 8 XCDs (each with its own L2);
// map the linear id bijectively (any grid size) to a logical id so that each XCD works one contiguous range.
__host__ __device__ inline int xcd_logical(int lin, int nlin) {
    const int q = nlin >> 3, rem = nlin & 7, x = lin & 7, k = lin >> 3;
    return x < rem ? x * (q + 1) + k : rem * (q + 1) + (x - rem) * q + k;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (count <= n && p) return MAM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (count == 0) return MAM_OK;
        MAM_HIP(hipMalloc(&p, count * sizeof(T)));
        n = count;
        return MAM_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
};

// Pinned host staging buffer (grows, never shrinks): lets a solve upload all its inputs with one copy.
struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t n = 0;
    int alloc(size_t bytes) {
        if (bytes <= n && p) return MAM_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (bytes == 0) return MAM_OK;
        MAM_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), bytes, hipHostMallocDefault));
        n = bytes;
        return MAM_OK;
    }
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// Accumulates per-stage kernel time with HIP event pairs recorded on the launch stream.
struct StageTimer {
    struct Ev {
        int stage;
        hipEvent_t a, b;
    };
    bool enabled = false;
    int nstages;
    std::vector<Ev> pending;
    std::vector<hipEvent_t> pool;
    std::vector<double> ms;
    std::vector<long long> n;
    explicit StageTimer(int ns) : nstages(ns), ms(ns, 0.0), n(ns, 0) {}
    ~StageTimer() {
        for (auto& e : pending) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
    hipEvent_t take() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void reset(bool en) {
        enabled = en;
        for (int i = 0; i < nstages; i++) { ms[i] = 0; n[i] = 0; }
        for (auto& e : pending) { pool.push_back(e.a); pool.push_back(e.b); }
        pending.clear();
    }
    void collect() {
        for (auto& e : pending) {
            (void)hipEventSynchronize(e.b);
            float t = 0.f;
            (void)hipEventElapsedTime(&t, e.a, e.b);
            ms[e.stage] += t;
            n[e.stage] += 1;
            pool.push_back(e.a);
            pool.push_back(e.b);
        }
        pending.clear();
    }
    struct Scope {
        StageTimer* t;
        hipStream_t s;
        int stage;
        hipEvent_t a = nullptr;
        Scope(StageTimer* t_, hipStream_t s_, int st) : t(t_), s(s_), stage(st) {
            if (t && t->enabled) { a = t->take(); (void)hipEventRecord(a, s); }
        }
        ~Scope() {
            if (t && t->enabled) {
                hipEvent_t b = t->take();
                (void)hipEventRecord(b, s);
                t->pending.push_back({stage, a, b});
            }
        }
    };
};

}  // namespace mam
