/*
 * mam_stream.h — CU-partitioned HIP streams for running the Tracking and LocalMapping legs side by side.
 *
 * The reference runs Tracking and LocalMapping as two threads on the host's cores (src/System.cc:234-252,
 * LocalMapping::Run in its own std::thread); on one MI355X the two legs' kernels would otherwise compete for every CU,
 * and LocalMapping's latency-bound LBA chain (~50 dependent launches per step) waits behind Tracking's chip-filling
 * launches. A stream created with a CU mask dispatches only to the CUs in the mask, so the legs can be given disjoint
 * CU sets (hipExtStreamCreateWithCUMask).
 */
#ifndef MAM_STREAM_H
#define MAM_STREAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CUs of device `device` (hipDeviceAttributeMultiprocessorCount). */
int mam_device_cu_count(int device, int* n_cus);

/* A CU mask of n_cus bits (n_words = ceil(n_cus / 32) words) selecting the CUs i with (i / 4) % 8 < eighths
 * (complement = 1: the others). eighths must be even (2, 4, 6): then every XCD keeps the same share of its CUs under
 * either bit-to-XCD mapping (contiguous 32-bit runs per XCD or interleaved bits), and no XCD is left without CUs. */
int mam_cu_mask_split(int n_cus, int eighths, int complement, uint32_t* mask, int n_words);

/* A stream on the current device that dispatches only to the CUs set in mask (n_words 32-bit words); *stream is a
 * hipStream_t. */
int mam_stream_create_cu_mask(int n_words, const uint32_t* mask, void** stream);
int mam_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif

#endif
