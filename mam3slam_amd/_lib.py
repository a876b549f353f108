"""ctypes loader for libmam_gpu.so — the only way the Python host code reaches the GPU path.

There is no CPU fallback: if the HIP library is missing or does not load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MAM3SLAM_GPU_LIB: load an alternative build (kernel-variant experiments); default the in-tree product
LIB_PATH = os.environ.get("MAM3SLAM_GPU_LIB") or os.path.join(HERE, "libmam_gpu.so")


class MamError(RuntimeError):
    pass


class KeyPoint(C.Structure):
    """cv::KeyPoint layout (28 B) — include/mam_orb.h mam_keypoint."""

    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("fp_policy", C.c_int32)]


MAM_OK, MAM_ERR_EMPTY, MAM_ERR_CAPACITY, MAM_ERR_DEVICE, MAM_ERR_ARG = 0, -1, -2, -3, -4

_lib = None

# Every symbol declared in include/*.h, with (restype, argtypes). tests/test_abi.py checks the headers
# against this table and that the library exports each one.
_vp, _i32, _sz, _f32p, _i32p = C.c_void_p, C.c_int, C.c_size_t, C.POINTER(C.c_float), C.POINTER(C.c_int32)
SIGNATURES = {
    "mam_last_error": (C.c_char_p, []),
    "mam_orb_create": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "mam_orb_destroy": (None, [_vp]),
    "mam_orb_scales": (C.c_int, [_vp, _vp]),
    "mam_orb_features_per_level": (C.c_int, [_vp, _vp]),
    "mam_orb_levels": (C.c_int, [_vp]),
    "mam_orb_max_keypoints": (C.c_int, [_vp]),
    "mam_orb_extract": (C.c_int, [_vp, _vp, _i32, _i32, _sz, _i32, _i32, _vp, _vp, _i32, _vp, _vp]),
    "mam_orb_extract_batch_device": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _sz, _sz, _i32, _i32, _vp, _vp, _i32,
                                               _vp, _vp]),
    "mam_orb_get_level": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _vp]),
    "mam_orb_set_profiling": (C.c_int, [_vp, _i32]),
    "mam_orb_stage_times": (C.c_int, [_vp, _vp, _vp]),
    "mam_orb_debug_candidates": (C.c_int, [_vp, _i32, _i32, _vp, _i32]),
    "mam_orb_debug_blurred": (C.c_int, [_vp, _i32, _i32, _vp]),
    "mam_orb_debug_set_option": (C.c_int, [_vp, _i32, _i32]),
}


def _match_sigs():
    from .exchange import _SIGS as ex_sigs
    from .lba import _SIGS as lba_sigs
    from .match import _SIGS
    from .pose import _SIGS as pose_sigs
    from .bow import _SIGS as bow_sigs
    from .streams import _SIGS as stream_sigs
    from .ringmap import _SIGS as ringmap_sigs

    return {**_SIGS, **lba_sigs, **ex_sigs, **pose_sigs, **bow_sigs, **stream_sigs, **ringmap_sigs}


def lib() -> C.CDLL:
    """Load libmam_gpu.so (building it first if a hipcc is present and the .so is stale/missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        from . import build as _build

        _build.build()
    if not os.path.exists(LIB_PATH):
        raise MamError(f"HIP library {LIB_PATH} missing: run `python -m mam3slam_amd.build`")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in all_signatures().items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def all_signatures() -> dict:
    d = dict(SIGNATURES)
    d.update(_match_sigs())
    return d


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = lib().mam_last_error()
        raise MamError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")
    return rc
