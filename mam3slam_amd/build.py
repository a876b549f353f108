"""Build the gfx950 shared library (libmam_gpu.so) in-tree with hipcc.

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
SOURCES = ["orb_extract.hip", "match.hip", "lba.hip"]

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
]


def _sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _deps():
    out = []
    for root in (CSRC, os.path.join(HERE, "..", "include")):
        for f in os.listdir(root):
            out.append(os.path.join(root, f))
    return out


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    cmd = [HIPCC, *FLAGS, "-o", LIB + ".tmp", *_sources()]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-8000:]}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
