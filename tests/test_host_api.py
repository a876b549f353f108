"""The C++ host API (include/mam3slam/*.h: ORBextractor, ORBmatcher, Optimizer::LocalBundleAdjustment with the
reference signatures) — compiled with g++ against libmam3slam.so and exercised by tests/cpp/test_host_api.cpp.

CPU: window build / map bookkeeping / SE3 algebra (no device calls). GPU: the wrappers end to end vs the oracle.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_host_api.cpp")
OUT_DIR = os.path.join(ROOT, "tests", "cpp", "_build")
BIN = os.path.join(OUT_DIR, "test_host_api")


def _binary():
    from mam3slam_amd import build as b
    from oracle import oracle_py

    b.build()
    oracle_py.build()
    os.makedirs(OUT_DIR, exist_ok=True)
    deps = [SRC, b.HOST_LIB, b.LIB]
    if os.path.exists(BIN) and all(os.path.getmtime(d) <= os.path.getmtime(BIN) for d in deps):
        return BIN
    pkg, orc = os.path.join(ROOT, "mam3slam_amd"), os.path.join(ROOT, "oracle")
    cmd = ["g++", "-std=c++17", "-O1", "-ffp-contract=off", "-Wall", "-I", os.path.join(ROOT, "include"), SRC, "-o",
           BIN, "-L", pkg, "-l:libmam3slam.so", "-l:libmam_gpu.so", "-L", orc, "-l:liboracle.so",
           f"-Wl,-rpath,{pkg}:{orc}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return BIN


def _run(mode, timeout):
    r = subprocess.run([_binary(), mode], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.startswith("OK"), r.stdout
    return r.stdout


def test_host_api_cpu():
    _run("cpu", 120)


@pytest.mark.gpu
def test_host_api_gpu(gpu_lib):
    _run("gpu", 600)
