"""ORBextractor — Python mirror of MAM3SLAM::ORBextractor over the C-ABI (include/mam_orb.h).

Reference interface (include/ORBextractor.h:43-100):
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
    int operator()(InputArray image, InputArray mask, vector<KeyPoint>& kps, OutputArray desc,
                   vector<int>& vLappingArea)            -> returns monoIndex, -1 on empty image
    GetLevels / GetScaleFactor / GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
    GetInverseScaleSigmaSquares, public mvImagePyramid

Here `extractor(image, mask, lapping_area)` returns (keypoints, descriptors, monoIndex): keypoints is a
numpy structured array with cv::KeyPoint's fields, descriptors an (N, 32) uint8 array. Every call runs the
HIP path; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import KeyPoint, MamError, OrbParams, check, lib, MAM_ERR_EMPTY

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == C.sizeof(KeyPoint) == 28


class ORBextractor:
    HARRIS_SCORE, FAST_SCORE = 0, 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0, fp_policy: int = 0):
        self._p = OrbParams(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST), int(minThFAST),
                            int(fp_policy))
        self._ctx = C.c_void_p()
        check(lib().mam_orb_create(C.byref(self._p), int(device), C.byref(self._ctx)), "mam_orb_create")
        self.nfeatures, self.nlevels = int(nfeatures), int(nlevels)
        self._last_shape = None

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            lib().mam_orb_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self) -> C.c_void_p:
        return self._ctx

    # ---- getters (ORBextractor.h:62-82)
    def _scales(self):
        out = np.zeros(4 * self.nlevels, np.float32)
        check(lib().mam_orb_scales(self._ctx, out.ctypes.data_as(C.c_void_p)), "mam_orb_scales")
        return out.reshape(4, self.nlevels)

    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return float(self._p.scale_factor)

    def GetScaleFactors(self):
        return [float(v) for v in self._scales()[0]]

    def GetInverseScaleFactors(self):
        return [float(v) for v in self._scales()[1]]

    def GetScaleSigmaSquares(self):
        return [float(v) for v in self._scales()[2]]

    def GetInverseScaleSigmaSquares(self):
        return [float(v) for v in self._scales()[3]]

    def features_per_level(self) -> np.ndarray:
        out = np.zeros(self.nlevels, np.int32)
        check(lib().mam_orb_features_per_level(self._ctx, out.ctypes.data_as(C.c_void_p)), "features_per_level")
        return out

    def max_keypoints(self) -> int:
        return check(lib().mam_orb_max_keypoints(self._ctx), "max_keypoints")

    # ---- operator() (ORBextractor.cc:1086-1168)
    def __call__(self, image: np.ndarray | None, mask=None, lapping_area=(0, 1000)):
        if image is None or getattr(image, "size", 0) == 0:
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8), MAM_ERR_EMPTY
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise MamError("ORBextractor expects a CV_8UC1 image (2-D uint8)")
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = self.max_keypoints()
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n, mono = C.c_int(), C.c_int()
        rc = lib().mam_orb_extract(self._ctx, img.ctypes.data_as(C.c_void_p), w, h, C.c_size_t(img.strides[0]),
                                   int(lapping_area[0]), int(lapping_area[1]), kps.ctypes.data_as(C.c_void_p),
                                   desc.ctypes.data_as(C.c_void_p), cap, C.byref(n), C.byref(mono))
        if rc == MAM_ERR_EMPTY:
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8), MAM_ERR_EMPTY
        check(rc, "mam_orb_extract")
        self._last_shape = (w, h)
        return kps[:n.value].copy(), desc[:n.value].copy(), mono.value

    # ---- public mvImagePyramid (ORBextractor.h:84)
    @property
    def mvImagePyramid(self):
        levels = []
        for l in range(self.nlevels):
            w, h = C.c_int(), C.c_int()
            check(lib().mam_orb_get_level(self._ctx, 0, l, None, C.byref(w), C.byref(h)), "get_level")
            out = np.zeros((h.value, w.value), np.uint8)
            check(lib().mam_orb_get_level(self._ctx, 0, l, out.ctypes.data_as(C.c_void_p), None, None), "get_level")
            levels.append(out)
        return levels

    # ---- batched, device-resident path (multi-agent harness / bench)
    def extract_batch_device(self, d_imgs: int, nframes: int, w: int, h: int, stride: int, frame_stride: int,
                             d_kps: int, d_desc: int, capacity: int, d_counts: int, stream: int = 0,
                             lapping_area=(0, 1000)):
        """All pointers are device addresses (e.g. torch tensor .data_ptr()). Asynchronous on `stream`."""
        return check(lib().mam_orb_extract_batch_device(self._ctx, C.c_void_p(d_imgs), nframes, w, h,
                                                        C.c_size_t(stride), C.c_size_t(frame_stride),
                                                        int(lapping_area[0]), int(lapping_area[1]),
                                                        C.c_void_p(d_kps), C.c_void_p(d_desc), capacity,
                                                        C.c_void_p(d_counts), C.c_void_p(stream)),
                     "mam_orb_extract_batch_device")

    # ---- profiling / debug taps
    def set_profiling(self, enable: bool):
        check(lib().mam_orb_set_profiling(self._ctx, 1 if enable else 0), "set_profiling")

    def stage_times(self):
        ms = np.zeros(5, np.float64)
        n = np.zeros(5, np.int64)
        check(lib().mam_orb_stage_times(self._ctx, ms.ctypes.data_as(C.c_void_p), n.ctypes.data_as(C.c_void_p)),
              "stage_times")
        names = ["pyramid", "fast", "blur", "distribute", "describe"]
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(names)}

    def set_distribute_threads(self, nt: int):
        """DistributeOctTree kernel width (parity tests / A/B): 256, 512, 1024, 0 (round-3 kernel), -1 automatic."""
        check(lib().mam_orb_debug_set_option(self._ctx, 1, int(nt)), "mam_orb_debug_set_option")

    def set_fork(self, on: int):
        """Latency-mode stream fork for up to 4 frames per call: 1 on, 0 off, -1 automatic."""
        check(lib().mam_orb_debug_set_option(self._ctx, 2, int(on)), "mam_orb_debug_set_option")

    def set_fast_chunks(self, on: int):
        """FAST over chunks of a cell row (k_fast_chunks) instead of one workgroup per cell: 1 on, 0 off, -1 auto."""
        check(lib().mam_orb_debug_set_option(self._ctx, 3, int(on)), "mam_orb_debug_set_option")

    def set_fast_blur(self, on: int):
        """FAST and the blur in one launch (k_fast_blur) instead of two: 1 on, 0 off, -1 automatic (few frames)."""
        check(lib().mam_orb_debug_set_option(self._ctx, 4, int(on)), "mam_orb_debug_set_option")

    def debug_candidates(self, level: int, frame: int = 0) -> np.ndarray:
        n = check(lib().mam_orb_debug_candidates(self._ctx, frame, level, None, 0), "debug_candidates")
        out = np.zeros(max(n, 1), np.uint32)
        check(lib().mam_orb_debug_candidates(self._ctx, frame, level, out.ctypes.data_as(C.c_void_p), n),
              "debug_candidates")
        return out[:n]

    def debug_blurred(self, level: int, frame: int = 0) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        check(lib().mam_orb_get_level(self._ctx, frame, level, None, C.byref(w), C.byref(h)), "get_level")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().mam_orb_debug_blurred(self._ctx, frame, level, out.ctypes.data_as(C.c_void_p)), "debug_blurred")
        return out

    def level(self, level: int, frame: int = 0) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        check(lib().mam_orb_get_level(self._ctx, frame, level, None, C.byref(w), C.byref(h)), "get_level")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().mam_orb_get_level(self._ctx, frame, level, out.ctypes.data_as(C.c_void_p), None, None),
              "get_level")
        return out
