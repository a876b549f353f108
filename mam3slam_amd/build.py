"""Build the gfx950 shared library (libmam_gpu.so) in-tree with hipcc, and the C++ host API library
(libmam3slam.so: MAM3SLAM::ORBextractor / ORBmatcher / Optimizer over the C-ABI) with g++.

Invoked by __graft_entry__.build() and by the tests. The library is the product: HIP kernels + host
orchestration + C-ABI (include/mam_orb.h). No torch extension, no JIT cache: the .so sits next to this file
so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmam_gpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# Translation units linked into libmam_gpu.so (each includes its own kernels).
SOURCES = ["orb_extract.hip", "match.hip", "lba.hip", "exchange.hip", "pose.hip", "bow.hip", "streams.hip", "ringmap.hip"]

FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # parity: no FMA contraction, IEEE f32 division/sqrt (DESIGN.md §Parity policy)
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall",
    "-Wno-unused-function",
    "-Werror=return-type",
]


HOST = os.path.join(HERE, "host")
HOST_LIB = os.path.join(HERE, "libmam3slam.so")
INCLUDE = os.path.join(HERE, "..", "include")
CXX = os.environ.get("CXX", "g++")
HOST_FLAGS = ["-std=c++17", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-Wall", "-Wextra", "-Wno-unused-parameter"]


def _sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _deps():
    out = []
    for root, _, files in os.walk(CSRC):
        out += [os.path.join(root, f) for f in files]
    for root, _, files in os.walk(INCLUDE):
        out += [os.path.join(root, f) for f in files]
    return out


def _host_sources():
    return sorted(os.path.join(HOST, f) for f in os.listdir(HOST) if f.endswith(".cpp"))


def host_needs_build() -> bool:
    if not os.path.exists(HOST_LIB):
        return True
    t = os.path.getmtime(HOST_LIB)
    deps = _host_sources() + [os.path.join(r, f) for r, _, fs in os.walk(INCLUDE) for f in fs] + [LIB]
    deps += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]   # camera.hpp, det_math.hpp
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_host(force: bool = False, verbose: bool = False) -> str:
    """libmam3slam.so links libmam_gpu.so from the same directory (rpath $ORIGIN)."""
    if not force and not host_needs_build():
        return HOST_LIB
    cmd = [CXX, *HOST_FLAGS, "-I", INCLUDE, "-o", HOST_LIB + ".tmp", *_host_sources(), "-L", HERE, "-l:libmam_gpu.so",
           "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host build failed ({r.returncode}):\n{r.stderr[-8000:]}")
    os.replace(HOST_LIB + ".tmp", HOST_LIB)
    return HOST_LIB


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build():
        _build_gpu(verbose)
    build_host(force=force, verbose=verbose)
    return LIB


def _build_gpu(verbose: bool) -> None:
    cmd = [HIPCC, *FLAGS, "-o", LIB + ".tmp", *_sources()]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-8000:]}")
    os.replace(LIB + ".tmp", LIB)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
