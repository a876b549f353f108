"""The C++ host API (include/mam3slam/*.h: ORBextractor, ORBmatcher, Optimizer::LocalBundleAdjustment with the
reference signatures) — compiled with g++ against libmam3slam.so and exercised by tests/cpp/test_host_api.cpp.

CPU: window build / map bookkeeping / SE3 algebra and a two-thread Tracking / LocalMapping run on one map (no device
calls), also under AddressSanitizer + UBSan and ThreadSanitizer builds of libmam3slam.so and the test (host code only:
libmam_gpu.so is linked unsanitised and not called). GPU: the wrappers end to end vs the oracle, and Tracking calls
concurrent with LocalBundleAdjustment on separate thread-local contexts.
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


SAN_FLAGS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "tsan": ["-fsanitize=thread"]}


def _sanitized_binary(kind):
    """libmam3slam.so and the test built with -fsanitize (tests/cpp/_build/<kind>/), linked to the regular
    libmam_gpu.so and liboracle.so."""
    from mam3slam_amd import build as b
    from oracle import oracle_py

    b.build()
    oracle_py.build()
    d = os.path.join(OUT_DIR, kind)
    os.makedirs(d, exist_ok=True)
    lib, exe = os.path.join(d, "libmam3slam.so"), os.path.join(d, "test_host_api")
    srcs = b._host_sources()
    hdrs = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(ROOT, "include")) for f in fs]
    deps = srcs + hdrs + [SRC, b.LIB, __file__]
    if os.path.exists(exe) and all(os.path.getmtime(x) <= os.path.getmtime(exe) for x in deps):
        return exe
    pkg, orc = os.path.join(ROOT, "mam3slam_amd"), os.path.join(ROOT, "oracle")
    fl = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off", *SAN_FLAGS[kind]]
    r = subprocess.run(["g++", *fl, "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"), "-o", lib, *srcs, "-L", pkg,
                        "-l:libmam_gpu.so", f"-Wl,-rpath,{pkg}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run(["g++", *fl, "-I", os.path.join(ROOT, "include"), SRC, "-o", exe, "-L", d, "-l:libmam3slam.so",
                        "-L", pkg, "-l:libmam_gpu.so", "-L", orc, "-l:liboracle.so", f"-Wl,-rpath,{d}:{pkg}:{orc}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _run(mode, timeout, binary=None, env=None):
    e = {**os.environ, "MAM3SLAM_SETTINGS_DIR": os.path.join(ROOT, "mam3slam_amd", "data", "settings"), **(env or {})}
    r = subprocess.run([binary or _binary(), mode], capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.startswith("OK"), r.stdout
    return r.stdout


def test_host_api_cpu():
    _run("cpu", 120)


def test_host_api_cpu_asan():
    out = _run("cpu", 300, _sanitized_binary("asan"),
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out


def test_host_api_cpu_tsan():
    out = _run("cpu", 600, _sanitized_binary("tsan"), {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "WARNING: ThreadSanitizer" not in out


@pytest.mark.gpu
def test_host_api_gpu(gpu_lib):
    _run("gpu", 600)
