"""CPU: the algorithm of k_distribute2 (the latency-mode DistributeOctTree kernel, mam3slam_amd/csrc/distribute.hpp),
restated phase by phase on the host (tests/cpp/distribute2_model.cpp), gives the oracle's DistributeOctTree output —
the kept keys in list order (ORBextractor.cc:555-779) — on every level of real frames at the extractor shapes the GPU
tests use and on random, clustered candidate sets that drive the final phase through many sorts. The GPU parity tests
(tests/test_orb_gpu.py) then check the kernel itself."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from mam3slam_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("dist2") / "libdist2.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests/cpp/distribute2_model.cpp")], check=True)
    lib = C.CDLL(so)
    lib.dist2_model.restype = C.c_int
    lib.dist2_model.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]

    def run(cand, minx, maxx, miny, maxy, n_keep):
        cand = np.ascontiguousarray(cand, np.uint32)
        out = np.zeros(len(cand) + 8, np.uint32)
        m = lib.dist2_model(cand.ctypes.data, len(cand), minx, maxx, miny, maxy, n_keep, out.ctypes.data, len(out))
        assert m >= 0
        return out[:m].copy()

    return run


def _level_box(w, h, l, scales):
    lw, lh = int(np.rint(np.float32(w) * scales[1][l])), int(np.rint(np.float32(h) * scales[1][l]))
    return 16, lw - 16, 16, lh - 16


@pytest.mark.parametrize("w,h,nfeat", [(640, 480, 1000), (1280, 720, 2000), (960, 960, 700), (640, 480, 5000)])
def test_model_matches_oracle_on_frames(oracle, model, w, h, nfeat):
    p = oracle.params(nfeat)
    scales, nper, _ = oracle.tables(p)
    for fr in range(2):
        img = synth.make_frame(w, h, agent=2, frame=fr)
        for l in range(8):
            cand, kept = oracle.level_stage(img, l, p)
            box = _level_box(w, h, l, scales)
            got = model(cand, *box, int(nper[l]))
            assert np.array_equal(got, kept), (w, h, nfeat, fr, l, len(got), len(kept))


def test_model_matches_oracle_random(oracle, model):
    """Clustered random candidates (many equal-size nodes with equal UL.x: the sort's tie behaviour decides) over
    a range of keep counts, so the final phase runs from one to many iterations."""
    rng = np.random.default_rng(5)
    for trial in range(300):
        W = int(rng.integers(60, 1300))
        H = int(rng.integers(40, min(700, 2 * W - 1)))   # round(W / H) >= 1 initial nodes, as the extractor requires
        n = int(rng.integers(1, 3000))
        nc = int(rng.integers(1, 40))
        cx, cy = rng.integers(0, W, nc), rng.integers(0, H, nc)
        k = rng.integers(0, nc, n)
        spread = rng.integers(1, 60)
        x = np.clip(cx[k] + rng.integers(-spread, spread + 1, n), 0, W - 1)
        y = np.clip(cy[k] + rng.integers(-spread, spread + 1, n), 0, H - 1)
        s = rng.integers(7, 60, n)
        cand = (x | (y << 12) | (s << 24)).astype(np.uint32)
        N = int(rng.integers(1, 600))
        box = (16, 16 + W, 16, 16 + H)
        want = oracle.distribute(cand, *box, N)
        got = model(cand, *box, N)
        assert np.array_equal(got, want), (trial, W, H, n, N, len(got), len(want))
