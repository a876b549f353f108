"""mam3slam_amd — MI355X-native (gfx950) drop-in for MAM3SLAM's per-frame ORB + local-BA hot path.

The product is libmam_gpu.so (HIP kernels + C-ABI, include/*.h); this package is the thin host mirror of
the reference's C++ interfaces (ORBextractor, ORBmatcher, Optimizer::LocalBundleAdjustment) over it.
"""
from ._lib import MamError, lib  # noqa: F401
from .orb import KP_DTYPE, ORBextractor  # noqa: F401

__all__ = ["ORBextractor", "KP_DTYPE", "MamError", "lib"]
