"""GPU parity: ORBmatcher hot-path searches (HIP via the C-ABI) vs the CPU oracle — index-exact.

Inputs are real ORB features (oracle extraction of seeded synthetic frames) wrapped in synthetic map
structures (mam3slam_amd/scene.py) that exercise the reference's control flow: greedy keypoint taking
(ORBmatcher.cc:88-90, 1747-1749), duplicate MapPoints, pre-taken keypoints, ratio test, rotation histogram
(:1855-1884), "last equal wins" in SearchForTriangulation (:1017).
"""
import numpy as np
import pytest

from mam3slam_amd import scene, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    out = []
    for (w, h, nf, fr) in [(640, 480, 1000, 0), (640, 480, 1000, 7), (1280, 720, 2000, 3)]:
        img = synth.make_frame(w, h, agent=5, frame=fr)
        k, d, _ = oracle.extract(img, oracle.params(nf))
        out.append((w, h, k, d))
    return out


def _matcher(nnratio=0.8, ori=True):
    from mam3slam_amd.match import ORBmatcher

    return ORBmatcher(nnratio, ori)


def test_descriptor_distance(gpu_lib, oracle):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    b[:10] = a[:10]
    b[10:20] = ~a[10:20]
    got = _matcher().DescriptorDistance(a, b)
    ref = np.array([oracle.descriptor_distance(a[i], b[i]) for i in range(len(a))])
    assert np.array_equal(got, ref)
    assert (got[:10] == 0).all() and (got[10:20] == 256).all()


@pytest.mark.parametrize("fi", [0, 1, 2])
@pytest.mark.parametrize("th", [1, 3, 15])
def test_search_by_projection_local(gpu_lib, oracle, frames, fi, th):
    w, h, k, d = frames[fi]
    M = _matcher(0.8)
    for seed in range(3):
        rng = np.random.default_rng(100 * fi + seed)
        F = scene.make_frame_data(k, d, w, h, rng, taken_frac=0.1 * seed)
        mps = scene.local_mappoints(F, rng)
        far = seed == 2
        ng, og = M.SearchByProjection(F, mps, th, far, 30.0)
        no, oo = oracle.search_by_projection(F, mps, th, far, 30.0, 0.8)
        assert ng == no, (seed, ng, no)
        diff = np.nonzero(og != oo)[0]
        assert len(diff) == 0, f"seed {seed}: {len(diff)} keypoints differ, first {diff[:5]} gpu={og[diff[:5]]} " \
                               f"oracle={oo[diff[:5]]}"


def test_search_by_projection_nnratio_and_edges(gpu_lib, oracle, frames):
    w, h, k, d = frames[0]
    rng = np.random.default_rng(9)
    F = scene.make_frame_data(k, d, w, h, rng)
    mps = scene.local_mappoints(F, rng, kflip=40)
    for nn in (0.6, 0.9, 1.0):
        M = _matcher(nn)
        ng, og = M.SearchByProjection(F, mps, 5)
        no, oo = oracle.search_by_projection(F, mps, 5, nnratio=nn)
        assert ng == no and np.array_equal(og, oo), nn
    M = _matcher(0.8)
    # every keypoint already taken -> no match; no MapPoints -> 0
    F.taken = np.ones(len(k), np.uint8)
    ng, og = M.SearchByProjection(F, mps, 3)
    assert ng == 0 and (og == -1).all()
    F.taken = None
    ng, og = M.SearchByProjection(F, mps[:0], 3)
    assert ng == 0 and (og == -1).all()


@pytest.mark.parametrize("fi", [0, 2])
@pytest.mark.parametrize("th,ori", [(7, True), (15, True), (15, False), (30, True)])
def test_search_by_projection_motion(gpu_lib, oracle, frames, fi, th, ori):
    w, h, k, d = frames[fi]
    cam = scene.pinhole(w, h)
    M = _matcher(0.9, ori)
    for seed in range(3):
        rng = np.random.default_rng(1000 + seed)
        F = scene.make_frame_data(k, d, w, h, rng, taken_frac=0.05 * seed)
        F.pose = scene.small_pose(rng)
        last = scene.motion_last_frame(F, cam, rng)
        ng, og = M.SearchByProjectionMotion(F, last, cam, th, True)
        no, oo = oracle.search_by_projection_motion(F, last, cam, th, ori)
        assert ng == no, (seed, ng, no)
        diff = np.nonzero(og != oo)[0]
        assert len(diff) == 0, f"seed {seed}: {len(diff)} differ, first {diff[:5]} gpu={og[diff[:5]]} oracle={oo[diff[:5]]}"


@pytest.mark.parametrize("fi", [0, 1, 2])
@pytest.mark.parametrize("ori,coarse", [(False, False), (True, False), (False, True)])
def test_search_for_triangulation(gpu_lib, oracle, frames, fi, ori, coarse):
    w, h, k, d = frames[fi]
    cam = scene.pinhole(w, h)
    M = _matcher(0.6, ori)
    for seed in range(2):
        rng = np.random.default_rng(2000 + seed)
        F = scene.make_frame_data(k, d, w, h)
        KF1, KF2, F12, ep = scene.keyframe_pair(F, cam, rng)
        ng, pairs = M.SearchForTriangulation(KF1, KF2, F12, ep, False, coarse)
        no, oo = oracle.search_for_triangulation(KF1, KF2, F12, ep, ori, coarse)
        ref_pairs = np.stack([np.nonzero(oo >= 0)[0], oo[oo >= 0]], 1)
        assert ng == no
        assert np.array_equal(pairs, ref_pairs)


def test_projection_batch_device(gpu_lib, oracle, frames):
    import torch

    from mam3slam_amd.match import MP_TRACK_DTYPE, FramesDev

    w, h, k, d = frames[0]
    Fn = 5
    M = _matcher(0.8)
    S = 1100
    keys = np.zeros((Fn, S), k.dtype)
    desc = np.zeros((Fn, S, 32), np.uint8)
    counts = np.zeros((Fn, 2), np.int32)
    mp_list, FD = [], []
    for f in range(Fn):
        rng = np.random.default_rng(50 + f)
        sel = np.sort(rng.choice(len(k), size=len(k) - 7 * f, replace=False))
        F = scene.make_frame_data(k[sel], d[sel], w, h)
        keys[f, :len(sel)] = F.keys
        desc[f, :len(sel)] = F.desc
        counts[f, 0] = len(sel)
        mp_list.append(scene.local_mappoints(F, rng))
        FD.append(F)
    ms = max(len(m) for m in mp_list)
    mps = np.zeros((Fn, ms), MP_TRACK_DTYPE)
    nmps = np.array([len(m) for m in mp_list], np.int32)
    for f in range(Fn):
        mps[f, :nmps[f]] = mp_list[f]
    dev = torch.device("cuda")
    t_keys = torch.from_numpy(keys.view(np.uint8).reshape(Fn, -1)).to(dev)
    t_desc = torch.from_numpy(desc).to(dev)
    t_cnt = torch.from_numpy(counts).to(dev)
    t_mps = torch.from_numpy(mps.view(np.uint8).reshape(Fn, -1)).to(dev)
    t_nmps = torch.from_numpy(nmps).to(dev)
    t_out = torch.zeros((Fn, S), dtype=torch.int32, device=dev)
    t_nm = torch.zeros(Fn, dtype=torch.int32, device=dev)
    fr = FramesDev(Fn, S, t_keys.data_ptr(), t_desc.data_ptr(), t_cnt.data_ptr(), None)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    M.search_by_projection_batch_device(FD[0], fr, t_mps.data_ptr(), ms, t_nmps.data_ptr(), 3.0, t_out.data_ptr(),
                                        t_nm.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    out, nm = t_out.cpu().numpy(), t_nm.cpu().numpy()
    for f in range(Fn):
        no, oo = oracle.search_by_projection(FD[f], mp_list[f], 3.0, nnratio=0.8)
        assert nm[f] == no
        assert np.array_equal(out[f, :counts[f, 0]], oo)


def test_motion_batch_device_taken_out(gpu_lib, oracle, frames):
    """Batched motion search with `taken` in and `taken_out`: matches index-exact per frame, and taken_out is the
    slot state the reference leaves in CurrentFrame.mvpMapPoints (ORBmatcher.cc:1768-1771 assign, :1876-1881
    rotation clear), read as `taken` (slot set and Observations() > 0) by the next search."""
    import torch

    from mam3slam_amd.match import LAST_ENTRY_DTYPE, FramesDev

    w, h, k, d = frames[0]
    cam = scene.pinhole(w, h)
    Fn, S = 4, 1100
    M = _matcher(0.9, True)
    keys = np.zeros((Fn, S), k.dtype)
    desc = np.zeros((Fn, S, 32), np.uint8)
    counts = np.zeros((Fn, 2), np.int32)
    taken = np.zeros((Fn, S), np.uint8)
    FD, lasts = [], []
    tcw = np.zeros(Fn, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for f in range(Fn):
        rng = np.random.default_rng(70 + f)
        sel = np.sort(rng.choice(len(k), size=len(k) - 5 * f, replace=False))
        F = scene.make_frame_data(k[sel], d[sel], w, h, rng, taken_frac=0.04 * f)
        F.pose = scene.small_pose(rng)
        keys[f, :len(sel)], desc[f, :len(sel)], counts[f, 0] = F.keys, F.desc, len(sel)
        if F.taken is not None:
            taken[f, :len(sel)] = F.taken
        tcw[f]["q"], tcw[f]["t"] = F.pose
        FD.append(F)
        lasts.append(scene.motion_last_frame(F, cam, rng))
    ls = max(len(x) for x in lasts)
    last = np.zeros((Fn, ls), LAST_ENTRY_DTYPE)
    for f in range(Fn):
        last[f, :len(lasts[f])] = lasts[f]
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    t_keys, t_desc, t_cnt = T(keys.view(np.uint8).reshape(Fn, -1)), T(desc), T(counts)
    t_taken, t_last, t_tcw = T(taken), T(last.view(np.uint8).reshape(Fn, -1)), T(tcw.view(np.uint8))
    t_nlast = T(np.array([len(x) for x in lasts], np.int32))
    t_out = torch.zeros((Fn, S), dtype=torch.int32, device=dev)
    t_nm = torch.zeros(Fn, dtype=torch.int32, device=dev)
    t_tout = torch.full((Fn, S), 7, dtype=torch.uint8, device=dev)
    fr = FramesDev(Fn, S, t_keys.data_ptr(), t_desc.data_ptr(), t_cnt.data_ptr(), t_taken.data_ptr(),
                   t_tout.data_ptr())
    M.search_motion_batch_device(FD[0], fr, t_tcw.data_ptr(), cam, t_last.data_ptr(), ls, t_nlast.data_ptr(), 15.0,
                                 t_out.data_ptr(), t_nm.data_ptr())
    torch.cuda.synchronize()
    out, nm, tout = t_out.cpu().numpy(), t_nm.cpu().numpy(), t_tout.cpu().numpy()
    for f in range(Fn):
        n = counts[f, 0]
        no, oo = oracle.search_by_projection_motion(FD[f], lasts[f], cam, 15.0, True)
        assert nm[f] == no
        assert np.array_equal(out[f, :n], oo)
        exp = np.where(oo >= 0, lasts[f]["nobs"][np.maximum(oo, 0)] > 0, (oo == -1) & (taken[f, :n] > 0))
        assert np.array_equal(tout[f, :n], exp.astype(np.uint8)), f
        assert not tout[f, n:].any()


def test_reuse_grid_shared_context(gpu_lib, oracle, frames):
    """The local-map search on the motion search's context reuses its cell grid (FramesDev.reuse_grid): same results
    as a fresh build; a reuse request over other frames is refused (MAM_ERR_ARG)."""
    import torch

    from mam3slam_amd._lib import MamError
    from mam3slam_amd.match import MP_TRACK_DTYPE, FramesDev, ORBmatcher

    w, h, k, d = frames[0]
    cam = scene.pinhole(w, h)
    Fn, S = 3, 1100
    keys = np.zeros((Fn, S), k.dtype)
    desc = np.zeros((Fn, S, 32), np.uint8)
    counts = np.zeros((Fn, 2), np.int32)
    FD, mp_list = [], []
    for f in range(Fn):
        rng = np.random.default_rng(90 + f)
        sel = np.sort(rng.choice(len(k), size=len(k) - 3 * f, replace=False))
        F = scene.make_frame_data(k[sel], d[sel], w, h)
        keys[f, :len(sel)], desc[f, :len(sel)], counts[f, 0] = F.keys, F.desc, len(sel)
        FD.append(F)
        mp_list.append(scene.local_mappoints(F, rng))
    ms = max(len(m) for m in mp_list)
    mps = np.zeros((Fn, ms), MP_TRACK_DTYPE)
    for f in range(Fn):
        mps[f, :len(mp_list[f])] = mp_list[f]
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    t_keys, t_desc, t_cnt = T(keys.view(np.uint8).reshape(Fn, -1)), T(desc), T(counts)
    t_mps, t_nmps = T(mps.view(np.uint8).reshape(Fn, -1)), T(np.array([len(m) for m in mp_list], np.int32))
    outs = []
    owner = ORBmatcher(0.8, True)
    sharer = ORBmatcher(0.8, True, share=owner)
    for reuse, M in ((0, owner), (1, sharer)):
        t_out = torch.zeros((Fn, S), dtype=torch.int32, device=dev)
        t_nm = torch.zeros(Fn, dtype=torch.int32, device=dev)
        fr = FramesDev(Fn, S, t_keys.data_ptr(), t_desc.data_ptr(), t_cnt.data_ptr(), None, None, reuse)
        M.search_by_projection_batch_device(FD[0], fr, t_mps.data_ptr(), ms, t_nmps.data_ptr(), 1.0, t_out.data_ptr(),
                                            t_nm.data_ptr())
        torch.cuda.synchronize()
        outs.append((t_out.cpu().numpy(), t_nm.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    for f in range(Fn):
        no, oo = oracle.search_by_projection(FD[f], mp_list[f], 1.0, nnratio=0.8)
        assert outs[1][1][f] == no and np.array_equal(outs[1][0][f, :counts[f, 0]], oo)
    # reuse over a different frame set (fewer frames) is refused
    fr_bad = FramesDev(Fn - 1, S, t_keys.data_ptr(), t_desc.data_ptr(), t_cnt.data_ptr(), None, None, 1)
    t_out = torch.zeros((Fn, S), dtype=torch.int32, device=dev)
    t_nm = torch.zeros(Fn, dtype=torch.int32, device=dev)
    with pytest.raises(MamError):
        sharer.search_by_projection_batch_device(FD[0], fr_bad, t_mps.data_ptr(), ms, t_nmps.data_ptr(), 1.0,
                                                 t_out.data_ptr(), t_nm.data_ptr())


def _frustum_frame(frames, fi, seed):
    w, h, k, d = frames[fi]
    rng = np.random.default_rng(900 + 10 * fi + seed)
    F = scene.make_frame_data(k, d, w, h)
    F.pose = scene.small_pose(rng, rot=0.2, trans=0.5)
    cam = scene.pinhole(w, h)
    return F, cam, scene.local_world_mappoints(F, cam, rng)


def _assert_tracks_equal(tg, to, what):
    for f in ("proj_x", "proj_y", "track_in_view", "is_bad", "nobs", "desc"):
        assert np.array_equal(tg[f], to[f]), f"{what}: {f}"
    v = to["track_in_view"] == 1
    for f in ("view_cos", "track_depth", "scale_level"):
        assert np.array_equal(tg[f][v], to[f][v]), f"{what}: {f}"


@pytest.mark.parametrize("fi", [0, 2])
def test_is_in_frustum(gpu_lib, oracle, frames, fi):
    """Frame::isInFrustum + PredictScale (SearchLocalPoints' projection loop): track fields bit-exact, nToMatch equal;
    every level predicted somewhere, and the reject branches (behind, outside, distance, angle, bad, seen) hit."""
    M = _matcher(0.8)
    levels = set()
    for seed in range(3):
        F, cam, mps = _frustum_frame(frames, fi, seed)
        ng, tg = M.IsInFrustum(F, mps, cam)
        no, to = oracle.is_in_frustum(F, mps, cam)
        assert ng == no and 0 < ng < len(mps), (ng, no, len(mps))
        _assert_tracks_equal(tg, to, f"seed {seed}")
        levels |= set(to["scale_level"][to["track_in_view"] == 1].tolist())
        assert (to["proj_x"] == -1).any() and ((to["proj_x"] != -1) & (to["track_in_view"] == 0)).any()
    assert levels == set(range(8)), levels


def test_frustum_then_local_search_batch(gpu_lib, oracle, frames):
    """SearchLocalPoints end to end on the device: isInFrustum for a batch of frames feeds the batched local-map
    search (th 1, nnratio 0.8) directly in HBM; per-frame matches index-exact vs the oracle chain."""
    import torch

    from mam3slam_amd.match import LOCAL_MP_DTYPE, MP_TRACK_DTYPE, FramesDev, Pose

    w, h, k, d = frames[0]
    M = _matcher(0.8)
    B = 4
    Fs, mpl, cam = [], [], None
    for s in range(B):
        F, cam, mps = _frustum_frame(frames, 0, 10 + s)
        Fs.append(F)
        mpl.append(mps)
    cap = len(k)
    S = max(len(m) for m in mpl)
    mp_all = np.zeros((B, S), LOCAL_MP_DTYPE)
    tcw = np.zeros(B, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for s in range(B):
        mp_all[s, :len(mpl[s])] = mpl[s]
        tcw[s]["q"], tcw[s]["t"] = Fs[s].pose
    dev = torch.device("cuda", 0)
    keys = np.zeros((B, cap), k.dtype)
    keys[:] = k
    desc = np.zeros((B, cap, 32), np.uint8)
    desc[:] = d
    d_keys = torch.from_numpy(keys.view(np.uint8).reshape(B, -1).copy()).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_cnt = torch.tensor([[len(k), 0]] * B, dtype=torch.int32, device=dev)
    d_mps = torch.from_numpy(mp_all.view(np.uint8).reshape(B, -1).copy()).to(dev)
    d_n = torch.tensor([len(m) for m in mpl], dtype=torch.int32, device=dev)
    d_tcw = torch.from_numpy(tcw.view(np.uint8).copy()).to(dev)
    d_tr = torch.zeros((B, S * MP_TRACK_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_ntm = torch.zeros(B, dtype=torch.int32, device=dev)
    d_out = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(B, dtype=torch.int32, device=dev)
    M.is_in_frustum_batch_device(Fs[0], B, d_tcw.data_ptr(), cam, d_mps.data_ptr(), S, d_n.data_ptr(),
                                 d_tr.data_ptr(), d_ntm.data_ptr())
    fr = FramesDev(B, cap, d_keys.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(), None, None)
    M.search_by_projection_batch_device(Fs[0], fr, d_tr.data_ptr(), S, d_n.data_ptr(), 1.0, d_out.data_ptr(),
                                        d_nm.data_ptr())
    torch.cuda.synchronize()
    tr = d_tr.cpu().numpy().view(MP_TRACK_DTYPE).reshape(B, S)
    out, nm, ntm = d_out.cpu().numpy(), d_nm.cpu().numpy(), d_ntm.cpu().numpy()
    for s in range(B):
        n = len(mpl[s])
        no, to = oracle.is_in_frustum(Fs[s], mpl[s], cam)
        assert ntm[s] == no
        _assert_tracks_equal(tr[s, :n], to, f"frame {s}")
        nmo, oo = oracle.search_by_projection(Fs[s], to, 1.0, False, 50.0, 0.8)
        assert nm[s] == nmo and np.array_equal(out[s, :len(k)], oo), s
