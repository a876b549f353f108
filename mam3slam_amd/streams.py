"""CU-partitioned HIP streams (include/mam_stream.h): the Tracking and LocalMapping legs on disjoint CU sets.

The reference runs the two legs as host threads (src/System.cc:234-252); here they share one GPU, and a stream
created with a CU mask dispatches only to its CUs, so LocalMapping's latency-bound LBA chain never queues behind
Tracking's chip-filling launches (and Tracking's waves never share a SIMD with it)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib

_SIGS = {
    "mam_device_cu_count": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "mam_cu_mask_split": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]),
    "mam_stream_create_cu_mask": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    "mam_stream_destroy": (C.c_int, [C.c_void_p]),
}

_streams = []   # the created streams live as long as the process (torch's ExternalStream does not own them)


def cu_count(device_index: int = 0) -> int:
    n = C.c_int()
    check(lib().mam_device_cu_count(int(device_index), C.byref(n)), "mam_device_cu_count")
    return n.value


def cu_mask(n_cus: int, eighths: int, complement: bool = False) -> np.ndarray:
    """The CUs i with (i / 4) % 8 < eighths (complement: the others) as uint32 words; eighths 2, 4 or 6."""
    nw = (n_cus + 31) // 32
    m = np.zeros(nw, np.uint32)
    check(lib().mam_cu_mask_split(int(n_cus), int(eighths), 1 if complement else 0, m.ctypes.data, nw),
          "mam_cu_mask_split")
    return m


def masked_stream(device, mask: np.ndarray):
    """A torch ExternalStream over a HIP stream that dispatches only to the CUs in mask."""
    import torch

    m = np.ascontiguousarray(mask, np.uint32)
    h = C.c_void_p()
    with torch.cuda.device(device):
        check(lib().mam_stream_create_cu_mask(len(m), m.ctypes.data, C.byref(h)), "mam_stream_create_cu_mask")
    s = torch.cuda.ExternalStream(h.value, device=device)
    _streams.append(s)
    return s
