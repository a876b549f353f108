// Known-bytes probe for the FETCH_SIZE counter (scripts/fetch_probe.py): each kernel reads every byte of a fresh
// buffer exactly once with one load shape, so FETCH_SIZE x 1024 / bytes is the counter's scale for that shape.
#include <hip/hip_runtime.h>
#include <cstdint>

extern "C" {

// 16-byte loads, consecutive lanes consecutive (the wide coalesced case)
__global__ void probe_wide(const uint4* __restrict__ p, size_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
// 4-byte loads, consecutive lanes consecutive
__global__ void probe_dword(const uint32_t* __restrict__ p, size_t n4, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) sink[0] = acc;
}
// 1-byte loads, consecutive lanes consecutive
__global__ void probe_byte(const uint8_t* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) sink[0] = acc;
}
// the FAST staging shape: an image of `pitch`-byte rows cut into 44-byte-wide, 41-row ROIs (one 256-thread workgroup
// each); a thread loads 4 bytes (+ the next byte, as the kernel's pr[4]) of one ROI row
__global__ void probe_roi(const uint8_t* __restrict__ img, int pitch, int rows, uint32_t* __restrict__ sink) {
    const int roi_w = 44, roi_h = 41;
    const int rois_x = pitch / roi_w;
    const int rx = blockIdx.x % rois_x, ry = blockIdx.x / rois_x;
    const uint8_t* src = img + (size_t)ry * roi_h * pitch + rx * roi_w;
    const int qc = roi_w / 4, nq = roi_h * qc;
    uint32_t acc = 0;
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        const int r = i / qc, q = i - r * qc;
        const uint8_t* pr = src + (size_t)r * pitch + 4 * q;
        uint32_t w;
        __builtin_memcpy(&w, pr, 4);
        acc ^= w ^ (q + 1 < qc ? pr[4] : 0u);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int fetch_probe_run(int kind, const void* p, size_t bytes, int pitch, uint32_t* sink) {
    const int grid = 4096, block = 256;
    switch (kind) {
        case 0: hipLaunchKernelGGL(probe_wide, dim3(grid), dim3(block), 0, 0, (const uint4*)p, bytes / 16, sink); break;
        case 1: hipLaunchKernelGGL(probe_dword, dim3(grid), dim3(block), 0, 0, (const uint32_t*)p, bytes / 4, sink); break;
        case 2: hipLaunchKernelGGL(probe_byte, dim3(grid), dim3(block), 0, 0, (const uint8_t*)p, bytes, sink); break;
        default: {
            const int rows = (int)(bytes / (size_t)pitch);
            const int nroi = (pitch / 44) * (rows / 41);
            hipLaunchKernelGGL(probe_roi, dim3(nroi), dim3(256), 0, 0, (const uint8_t*)p, pitch, rows, sink);
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
}
