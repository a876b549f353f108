// streams.hip — CU-partitioned streams (include/mam_stream.h): the two SLAM legs on disjoint CU sets.
#include <hip/hip_runtime.h>

#include "../../include/mam_stream.h"
#include "runtime.hpp"

extern "C" int mam_device_cu_count(int device, int* n_cus) {
    if (!n_cus) return MAM_ERR_ARG;
    MAM_HIP(hipDeviceGetAttribute(n_cus, hipDeviceAttributeMultiprocessorCount, device));
    return MAM_OK;
}

extern "C" int mam_cu_mask_split(int n_cus, int eighths, int complement, uint32_t* mask, int n_words) {
    if (!mask || n_cus <= 0 || n_words < (n_cus + 31) / 32 || eighths < 2 || eighths > 6 || (eighths & 1)) {
        mam::set_last_error("mam_cu_mask_split: bad arguments");
        return MAM_ERR_ARG;
    }
    for (int w = 0; w < n_words; w++) mask[w] = 0u;
    for (int i = 0; i < n_cus; i++) {
        const bool in = (i / 4) % 8 < eighths;
        if (in != (complement != 0)) mask[i >> 5] |= 1u << (i & 31);
    }
    return MAM_OK;
}

extern "C" int mam_stream_create_cu_mask(int n_words, const uint32_t* mask, void** stream) {
    if (!mask || !stream || n_words <= 0) return MAM_ERR_ARG;
    hipStream_t s = nullptr;
    MAM_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask));
    *stream = s;
    return MAM_OK;
}

extern "C" int mam_stream_destroy(void* stream) {
    if (!stream) return MAM_ERR_ARG;
    MAM_HIP(hipStreamDestroy((hipStream_t)stream));
    return MAM_OK;
}
