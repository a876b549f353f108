"""GPU parity: ORBmatcher::Fuse (ORBmatcher.cc:1148-1338) and MapPoint::ComputeDistinctiveDescriptors
(MapPoint.cc:329-403) on the HIP path (C-ABI) vs the CPU oracle — index-exact.

Fuse is compared per MapPoint: the keypoint it fuses with (-1 if none) and the best Hamming distance over the
candidates that pass the level and reprojection tests. The replace-or-add side effects are host code
(MAM3SLAM::ORBmatcher::Fuse, checked in tests/cpp/test_host_api.cpp). Inputs are real ORB features with synthetic
MapPoints around them (scene.fuse_mappoints): re-projections within a few pixels, normals inside and outside the
60-degree cone, distance-invariance ranges that predict the keypoint's level, descriptors 0..60 bits away, invalid
entries, points behind the camera / outside the image / outside their range, and non-finite ranges.
"""
import numpy as np
import pytest

from mam3slam_amd import scene, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    out = []
    for (w, h, nf, fr) in [(640, 480, 1000, 2), (640, 480, 1000, 9), (1280, 720, 2000, 4)]:
        img = synth.make_frame(w, h, agent=3, frame=fr)
        k, d, _ = oracle.extract(img, oracle.params(nf))
        out.append((w, h, k, d))
    return out


def _kf(frame, rng):
    w, h, k, d = frame
    KF = scene.make_frame_data(k, d, w, h)
    KF.pose = scene.small_pose(rng, rot=0.4, trans=0.5)
    return KF


def _check(got, ref, tag):
    ng, ig, dg = got
    no, io, do = ref
    bad = np.nonzero((ig != io) | (dg != do))[0]
    assert ng == no and len(bad) == 0, (f"{tag}: fused {ng} vs {no}, {len(bad)} MapPoints differ, first {bad[:5]} "
                                        f"gpu={ig[bad[:5]]}/{dg[bad[:5]]} oracle={io[bad[:5]]}/{do[bad[:5]]}")


@pytest.mark.parametrize("fi", [0, 1, 2])
@pytest.mark.parametrize("th", [1.0, 3.0, 7.5])
def test_fuse(gpu_lib, oracle, frames, fi, th):
    from mam3slam_amd.match import ORBmatcher

    M = ORBmatcher()
    w, h = frames[fi][:2]
    cam = scene.pinhole(w, h)
    for seed in range(3):
        rng = np.random.default_rng(500 * fi + seed)
        KF = _kf(frames[fi], rng)
        mps = scene.fuse_mappoints(KF, cam, rng)
        got = M.Fuse(KF, mps, cam, th)
        _check(got, oracle.fuse(KF, mps, cam, th), f"seed {seed}")
        assert got[0] > len(mps) // 4   # the scene produces real fusions


def test_fuse_edges(gpu_lib, oracle, frames):
    from mam3slam_amd.match import ORBmatcher

    M = ORBmatcher()
    w, h, k, d = frames[0]
    cam = scene.pinhole(w, h)
    rng = np.random.default_rng(77)
    KF = _kf(frames[0], rng)
    mps = scene.fuse_mappoints(KF, cam, rng)
    n, idx, dist = M.Fuse(KF, mps[:0], cam)
    assert n == 0 and len(idx) == 0
    inv = mps.copy()
    inv["valid"] = 0
    n, idx, dist = M.Fuse(KF, inv, cam)
    assert n == 0 and (idx == -1).all() and (dist == 256).all()
    # a keyframe without keypoints
    empty = scene.make_frame_data(k[:0], d[:0], w, h)
    empty.pose = KF.pose
    _check(M.Fuse(empty, mps, cam), oracle.fuse(empty, mps, cam), "empty keyframe")
    # non-finite distance ranges: PredictScale of an infinite / NaN ratio ((int) of a non-finite float is INT_MIN on
    # x86 -> level 0); NaN normals (every comparison false: no `continue`)
    odd = mps.copy()
    sel = rng.choice(len(odd), 60, replace=False)
    odd["max_distance"][sel[:20]] = np.inf
    odd["max_distance"][sel[20:40]] = np.nan
    odd["normal"][sel[40:]] = np.nan
    _check(M.Fuse(KF, odd, cam), oracle.fuse(KF, odd, cam), "non-finite")
    # the keyframe turned around: (nearly) everything behind the camera
    back = scene.make_frame_data(k, d, w, h)
    back.pose = (np.array([0, 1, 0, 0], np.float32), np.zeros(3, np.float32))
    _check(M.Fuse(back, mps, cam), oracle.fuse(back, mps, cam), "behind")


def test_fuse_batch_device(gpu_lib, oracle, frames):
    """Six target keyframes in one launch (SearchInNeighbors' forward direction), then again reusing the grid."""
    import torch

    from mam3slam_amd.match import FUSE_MP_DTYPE, FramesDev, FuseKF, ORBmatcher, fuse_kf
    from mam3slam_amd.orb import KP_DTYPE

    M = ORBmatcher()
    dev = torch.device("cuda")
    cam = scene.pinhole(640, 480)
    cases = []
    for i in range(6):
        rng = np.random.default_rng(900 + i)
        KF = _kf(frames[i % 2], rng)
        cases.append((KF, scene.fuse_mappoints(KF, cam, rng)))
    B = len(cases)
    S = max(len(c[0].keys) for c in cases)
    U = max(len(c[1]) for c in cases)
    keys = np.zeros((B, S), KP_DTYPE)
    desc = np.zeros((B, S, 32), np.uint8)
    cnt = np.zeros((B, 2), np.int32)
    mps = np.zeros((B, U), FUSE_MP_DTYPE)
    nm = np.zeros(B, np.int32)
    kfs = (FuseKF * B)()
    for b, (KF, m) in enumerate(cases):
        keys[b, :len(KF.keys)] = KF.keys
        desc[b, :len(KF.keys)] = KF.desc
        cnt[b, 0] = len(KF.keys)
        mps[b, :len(m)] = m
        nm[b] = len(m)
        kfs[b] = fuse_kf(KF.pose)
    t_keys = torch.from_numpy(keys.view(np.uint8).reshape(B, -1)).to(dev)
    t_desc = torch.from_numpy(desc).to(dev)
    t_cnt = torch.from_numpy(cnt).to(dev)
    t_mps = torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).to(dev)
    t_nm = torch.from_numpy(nm).to(dev)
    t_kfs = torch.from_numpy(np.frombuffer(kfs, np.uint8).copy()).to(dev)
    t_idx = torch.zeros((B, U), dtype=torch.int32, device=dev)
    t_dist = torch.zeros((B, U), dtype=torch.int32, device=dev)
    t_n = torch.zeros(B, dtype=torch.int32, device=dev)
    fr = FramesDev(B, S, t_keys.data_ptr(), t_desc.data_ptr(), t_cnt.data_ptr(), None, None, 0)
    for reuse in (0, 1):
        fr.reuse_grid = reuse
        torch.cuda.synchronize()
        M.fuse_batch_device(cases[0][0], fr, t_kfs.data_ptr(), cam, t_mps.data_ptr(), U, t_nm.data_ptr(), 3.0,
                            t_idx.data_ptr(), t_dist.data_ptr(), t_n.data_ptr())
        torch.cuda.synchronize()
        gi, gd, gn = t_idx.cpu().numpy(), t_dist.cpu().numpy(), t_n.cpu().numpy()
        for b, (KF, m) in enumerate(cases):
            _check((int(gn[b]), gi[b, :len(m)], gd[b, :len(m)]), oracle.fuse(KF, m, cam, 3.0), f"frame {b} reuse {reuse}")


def _obs_sets(rng, sizes):
    """Per MapPoint a run of observed descriptors: one base descriptor with 0..80 flipped bits per row, some exact
    duplicate rows (median ties)."""
    off = np.zeros(len(sizes) + 1, np.int32)
    off[1:] = np.cumsum(sizes)
    descs = np.zeros((int(off[-1]), 32), np.uint8)
    for m, n in enumerate(sizes):
        if n == 0:
            continue
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        rows = scene.flip_bits(np.repeat(base[None], n, 0), rng, int(rng.integers(0, 80)))
        if n > 3 and rng.random() < 0.3:
            rows[rng.integers(0, n)] = rows[rng.integers(0, n)]
        if n > 2 and rng.random() < 0.1:
            rows[:] = rows[0]
        descs[off[m]:off[m + 1]] = rows
    return off, descs


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_distinctive_descriptors(gpu_lib, oracle, seed):
    from mam3slam_amd.match import ORBmatcher

    rng = np.random.default_rng(seed)
    sizes = [0, 1, 2, 3, 4, 5, 8, 31, 63, 64, 65, 66, 127, 128, 129, 300] + list(rng.integers(1, 40, 400))
    off, descs = _obs_sets(rng, sizes)
    got = ORBmatcher().ComputeDistinctiveDescriptors(off, descs)
    ref = oracle.distinctive_descriptors(off, descs)
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, f"{len(bad)} MapPoints differ, first {bad[:5]}: gpu {got[bad[:5]]} oracle {ref[bad[:5]]}"
    assert got[0] == -1 and (got[1:] >= 0).all()


def test_distinctive_descriptors_batch_device(gpu_lib, oracle):
    import torch

    from mam3slam_amd.match import ORBmatcher

    rng = np.random.default_rng(11)
    sizes = rng.integers(1, 50, 3000)
    off, descs = _obs_sets(rng, sizes)
    t_off = torch.from_numpy(off).cuda()
    t_d = torch.from_numpy(descs).cuda()
    t_out = torch.full((len(sizes),), -5, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    ORBmatcher().distinctive_batch_device(len(sizes), t_off.data_ptr(), t_d.data_ptr(), t_out.data_ptr(),
                                          stream=s.cuda_stream)
    s.synchronize()
    assert np.array_equal(t_out.cpu().numpy(), oracle.distinctive_descriptors(off, descs))
