"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the CPU oracle on seeded inputs,
stored together with the inputs). They are SELF-GENERATED (the reference ships no fixtures and cannot be built
here): they pin the oracle against regressions, not against the reference. The LBA oracle is cross-checked
independently by tests/test_lba_dense_xcheck.py (a dense numpy restatement).

CPU: the oracle still reproduces every fixture exactly (pins the restatement against regressions).
GPU: the HIP path reproduces them — bit-exact keypoints / descriptors / match indices, LBA within 1e-4.
"""
import os

import numpy as np
import pytest

from mam3slam_amd.match import LAST_ENTRY_DTYPE, MP_TRACK_DTYPE
from mam3slam_amd.orb import KP_DTYPE

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _kp(a):
    return np.ascontiguousarray(a).view(KP_DTYPE).reshape(-1)


def _frame(keys, desc, w, h, taken=None):
    from mam3slam_amd import scene

    F = scene.make_frame_data(_kp(keys), desc, int(w), int(h))
    F.taken = None if taken is None or taken.ndim == 0 else taken
    return F


def _featvec(ids, off, feats):
    return {int(ids[i]): [int(x) for x in feats[off[i]:off[i + 1]]] for i in range(len(ids))}


def _tri_frames(z, scene_cam=None):
    w, h = int(z["w"]), int(z["h"])
    K1 = _frame(z["tri_keys1"], z["tri_desc1"], w, h)
    K2 = _frame(z["tri_keys2"], z["tri_desc2"], w, h)
    K1.has_mp, K2.has_mp = z["tri_has1"], z["tri_has2"]
    K1.featvec = _featvec(z["tri_ids1"], z["tri_off1"], z["tri_feats1"])
    K2.featvec = _featvec(z["tri_ids2"], z["tri_off2"], z["tri_feats2"])
    return K1, K2


def _lba_problem(z):
    from mam3slam_amd.lba import LBAProblem

    return LBAProblem(**{k[2:]: z[k] for k in z.files if k.startswith("p_")})


# ---------------------------------------------------------------------------------------------- CPU: oracle pin

def test_oracle_reproduces_orb_golden(oracle):
    z = _load("orb.npz")
    for i in range(3):
        k, d, m = oracle.extract(z[f"img{i}"], oracle.params(int(z[f"nfeat{i}"])))
        assert np.array_equal(k.view(np.uint8).reshape(-1, 28), z[f"kps{i}"]), i
        assert np.array_equal(d, z[f"desc{i}"]) and m == int(z[f"mono{i}"]), i


def test_oracle_simd_reproduces_orb_golden(oracle):
    """The CPU baseline's AVX2 column (oracle/orb_simd.cpp: resize, blur, FAST) gives the golden bytes too."""
    z = _load("orb.npz")
    for i in range(3):
        k, d, m = oracle.extract(z[f"img{i}"], oracle.params(int(z[f"nfeat{i}"])), simd=True)
        assert np.array_equal(k.view(np.uint8).reshape(-1, 28), z[f"kps{i}"]), i
        assert np.array_equal(d, z[f"desc{i}"]) and m == int(z[f"mono{i}"]), i


def test_oracle_reproduces_match_golden(oracle):
    from mam3slam_amd import scene

    z = _load("match.npz")
    w, h = int(z["w"]), int(z["h"])
    F = _frame(z["local_keys"], z["local_desc"], w, h, z["local_taken"])
    mps = np.ascontiguousarray(z["local_mps"]).view(MP_TRACK_DTYPE).reshape(-1)
    n, o = oracle.search_by_projection(F, mps, 3.0, False, 50.0, 0.8)
    assert n == int(z["local_n"]) and np.array_equal(o, z["local_out"])
    F = _frame(z["motion_keys"], z["motion_desc"], w, h, z["motion_taken"])
    F.pose = (z["motion_q"], z["motion_t"])
    last = np.ascontiguousarray(z["motion_last"]).view(LAST_ENTRY_DTYPE).reshape(-1)
    n, o = oracle.search_by_projection_motion(F, last, scene.pinhole(w, h), 15.0, True)
    assert n == int(z["motion_n"]) and np.array_equal(o, z["motion_out"])
    K1, K2 = _tri_frames(z)
    n, o = oracle.search_for_triangulation(K1, K2, z["tri_F12"], z["tri_ep"], False, False)
    assert n == int(z["tri_n"]) and np.array_equal(o, z["tri_out"])


def test_oracle_reproduces_lba_golden(oracle):
    z = _load("lba.npz")
    r = oracle.lba_solve(_lba_problem(z))
    assert (r.iterations, r.lm_trials) == (int(z["r_iterations"]), int(z["r_trials"]))
    for a, b in ((r.pose_q, "r_pose_q"), (r.pose_t, "r_pose_t"), (r.point_xyz, "r_point_xyz"),
                 (r.edge_chi2, "r_edge_chi2")):
        assert np.array_equal(a, z[b]), b


# ---------------------------------------------------------------------------------------------- GPU vs golden

@pytest.mark.gpu
def test_gpu_orb_golden(gpu_lib):
    from mam3slam_amd import ORBextractor

    z = _load("orb.npz")
    for i in range(3):
        ext = ORBextractor(int(z[f"nfeat{i}"]), 1.2, 8, 20, 7)
        k, d, m = ext(z[f"img{i}"])
        assert np.array_equal(k.view(np.uint8).reshape(-1, 28), z[f"kps{i}"]), i
        assert np.array_equal(d, z[f"desc{i}"]) and m == int(z[f"mono{i}"]), i


@pytest.mark.gpu
def test_gpu_match_golden(gpu_lib):
    from mam3slam_amd import scene
    from mam3slam_amd.match import ORBmatcher

    z = _load("match.npz")
    w, h = int(z["w"]), int(z["h"])
    F = _frame(z["local_keys"], z["local_desc"], w, h, z["local_taken"])
    mps = np.ascontiguousarray(z["local_mps"]).view(MP_TRACK_DTYPE).reshape(-1)
    n, o = ORBmatcher(0.8).SearchByProjection(F, mps, 3.0, False, 50.0)
    assert n == int(z["local_n"]) and np.array_equal(o, z["local_out"])
    F = _frame(z["motion_keys"], z["motion_desc"], w, h, z["motion_taken"])
    F.pose = (z["motion_q"], z["motion_t"])
    last = np.ascontiguousarray(z["motion_last"]).view(LAST_ENTRY_DTYPE).reshape(-1)
    n, o = ORBmatcher(0.9, True).SearchByProjectionMotion(F, last, scene.pinhole(w, h), 15.0, True)
    assert n == int(z["motion_n"]) and np.array_equal(o, z["motion_out"])
    K1, K2 = _tri_frames(z)
    n, pairs = ORBmatcher(0.6, False).SearchForTriangulation(K1, K2, z["tri_F12"], z["tri_ep"], False, False)
    ref = z["tri_out"]
    assert n == int(z["tri_n"])
    assert np.array_equal(pairs, np.stack([np.nonzero(ref >= 0)[0], ref[ref >= 0]], 1))


@pytest.mark.gpu
def test_gpu_lba_golden(gpu_lib):
    from mam3slam_amd.lba import LBASolver

    z = _load("lba.npz")
    r = LBASolver().solve(_lba_problem(z))
    assert (r.iterations, r.lm_trials) == (int(z["r_iterations"]), int(z["r_trials"]))
    for a, b in ((r.pose_t, "r_pose_t"), (r.point_xyz, "r_point_xyz"), (r.pose_q, "r_pose_q")):
        ref = z[b]
        rel = np.linalg.norm(a - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-9)
        assert rel.max() <= 1e-4, b   # north-star tolerance on BA floats
