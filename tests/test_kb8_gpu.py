"""GPU parity with the KannalaBrandt8 camera (the testMultiAgentSystem agents' camera, test/settingsForTest_00.yaml:
960 x 960, 700 / 1500 features) on every projecting stage of the path: SearchByProjection(Cur, Last)
(ORBmatcher.cc:1713), Frame::isInFrustum (Frame.cc:532) + the local-map search, Fuse (ORBmatcher.cc:1210),
SearchForTriangulation with KannalaBrandt8::epipolarConstrain (two-view triangulation, KannalaBrandt8.cpp:216-220,
306-406), PoseOptimization and LocalBundleAdjustment (EdgeSE3ProjectXYZ[OnlyPose] with KannalaBrandt8::project /
projectJac, KannalaBrandt8.cpp:46-65, 145-175).

Bars as for the Pinhole tests: index-exact searches and bit-exact track fields (the float projection is the
reference build's, pinned to glibc 2.35 and g++ 11.4 by tests/cpp/test_glibc_camera.cpp); pose and BA within 1e-4
with identical control flow. The fisheye projection's double cos / sin differ between the device and glibc by at
most an ulp, far inside the BA tolerance.
"""
import numpy as np
import pytest

from mam3slam_amd import scene, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    out = []
    for (nf, fr) in [(700, 0), (1500, 5)]:
        img = synth.make_frame(960, 960, agent=1, frame=fr)
        k, d, _ = oracle.extract(img, oracle.params(nf))
        out.append((960, 960, k, d))
    return out


@pytest.fixture(scope="module")
def cam():
    return scene.kannala_brandt8(960, 960)


def _matcher(nnratio=0.8, ori=True):
    from mam3slam_amd.match import ORBmatcher

    return ORBmatcher(nnratio, ori)


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("th,ori", [(15, True), (30, False)])
def test_kb8_search_by_projection_motion(gpu_lib, oracle, frames, cam, fi, th, ori):
    w, h, k, d = frames[fi]
    M = _matcher(0.9, ori)
    total = 0
    for seed in range(3):
        rng = np.random.default_rng(3000 + seed)
        F = scene.make_frame_data(k, d, w, h, rng, taken_frac=0.05 * seed)
        F.pose = scene.small_pose(rng)
        last = scene.motion_last_frame(F, cam, rng)
        ng, og = M.SearchByProjectionMotion(F, last, cam, th, True)
        no, oo = oracle.search_by_projection_motion(F, last, cam, th, ori)
        assert ng == no, (seed, ng, no)
        diff = np.nonzero(og != oo)[0]
        assert len(diff) == 0, f"seed {seed}: {len(diff)} differ, first {diff[:5]} gpu={og[diff[:5]]} oracle={oo[diff[:5]]}"
        total += ng
    assert total > 0


@pytest.mark.parametrize("fi", [0, 1])
def test_kb8_is_in_frustum_and_local_search(gpu_lib, oracle, frames, cam, fi):
    from mam3slam_amd.match import MP_TRACK_DTYPE

    M = _matcher(0.8)
    w, h, k, d = frames[fi]
    for seed in range(2):
        rng = np.random.default_rng(3100 + 10 * fi + seed)
        F = scene.make_frame_data(k, d, w, h)
        F.pose = scene.small_pose(rng, rot=0.2, trans=0.5)
        mps = scene.local_world_mappoints(F, cam, rng)
        ng, tg = M.IsInFrustum(F, mps, cam)
        no, to = oracle.is_in_frustum(F, mps, cam)
        assert ng == no and 0 < ng < len(mps), (ng, no, len(mps))
        for f in ("proj_x", "proj_y", "track_in_view", "is_bad", "nobs", "desc"):
            assert np.array_equal(tg[f], to[f]), f
        v = to["track_in_view"] == 1
        for f in ("view_cos", "track_depth", "scale_level"):
            assert np.array_equal(tg[f][v], to[f][v]), f
        tracks = np.ascontiguousarray(to, MP_TRACK_DTYPE)
        ns, og = M.SearchByProjection(F, tracks, 1.0)
        nso, oo = oracle.search_by_projection(F, tracks, 1.0, nnratio=0.8)
        assert ns == nso and np.array_equal(og, oo) and ns > 0


@pytest.mark.parametrize("fi", [0, 1])
def test_kb8_fuse(gpu_lib, oracle, frames, cam, fi):
    M = _matcher()
    w, h, k, d = frames[fi]
    for seed in range(2):
        rng = np.random.default_rng(3200 + 10 * fi + seed)
        KF = scene.make_frame_data(k, d, w, h)
        KF.pose = scene.small_pose(rng, rot=0.4, trans=0.5)
        mps = scene.fuse_mappoints(KF, cam, rng)
        ng, ig, dg = M.Fuse(KF, mps, cam, 3.0)
        no, io, do = oracle.fuse(KF, mps, cam, 3.0)
        bad = np.nonzero((ig != io) | (dg != do))[0]
        assert ng == no and len(bad) == 0, (ng, no, bad[:5])
        assert ng > len(mps) // 4


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("ori,coarse", [(False, False), (True, False), (False, True)])
def test_kb8_search_for_triangulation(gpu_lib, oracle, frames, cam, fi, ori, coarse):
    """KannalaBrandt8::epipolarConstrain (unproject Newton + tanf, JacobiSVD two-view triangulation, both
    re-projections) inside the search: the pairs equal the oracle's, and the geometric test is selective (fewer
    matches than with bCoarse, which skips it)."""
    w, h, k, d = frames[fi]
    M = _matcher(0.6, ori)
    for seed in range(2):
        rng = np.random.default_rng(3300 + seed)
        F = scene.make_frame_data(k, d, w, h)
        KF1, KF2 = scene.keyframe_pair_3d(F, cam, rng)
        ng, pairs = M.SearchForTriangulationKF(KF1, KF2, cam, cam, False, coarse)
        no, oo = oracle.search_for_triangulation_kf(KF1, KF2, cam, cam, ori, coarse)
        ref_pairs = np.stack([np.nonzero(oo >= 0)[0], oo[oo >= 0]], 1)
        assert ng == no and np.array_equal(pairs, ref_pairs), (ng, no)
        assert ng > 20
        if not coarse:
            nc, _ = M.SearchForTriangulationKF(KF1, KF2, cam, cam, False, True)
            assert nc > ng


@pytest.mark.parametrize("fi", [0, 1])
def test_pinhole_kf_triangulation_equals_f12_path(gpu_lib, oracle, frames, fi):
    """The keyframe-level entry (geometry computed by the library) equals the F12 / epipole entry fed the same
    geometry (mam_triangulation_geometry), and both equal the oracle."""
    from mam3slam_amd.match import triangulation_geometry

    w, h, k, d = frames[fi]
    pin = scene.pinhole(w, h, 450.0)
    M = _matcher(0.6, True)
    rng = np.random.default_rng(3400 + fi)
    F = scene.make_frame_data(k, d, w, h)
    KF1, KF2 = scene.keyframe_pair_3d(F, pin, rng)
    _, _, F12, ep = triangulation_geometry(KF1.pose, KF2.pose, pin)
    n1, p1 = M.SearchForTriangulationKF(KF1, KF2, pin)
    n2, p2 = M.SearchForTriangulation(KF1, KF2, F12, ep)
    no, oo = oracle.search_for_triangulation_kf(KF1, KF2, pin, pin, True, False)
    assert n1 == n2 == no and np.array_equal(p1, p2) and n1 > 20
    assert np.array_equal(p1, np.stack([np.nonzero(oo >= 0)[0], oo[oo >= 0]], 1))


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("noise,ofrac", [(1.0, 0.08), (2.5, 0.25)])
def test_kb8_pose_optimization(gpu_lib, oracle, frames, cam, fi, noise, ofrac):
    from mam3slam_amd import pose
    from mam3slam_amd.pose import PoseOptimizer

    w, h, k, d = frames[fi]
    P = PoseOptimizer()
    for seed in range(2):
        F = scene.make_frame_data(k, d, w, h)
        xyz, _ = scene.pose_problem(F, cam, np.random.default_rng(3500 + seed), noise=noise, outlier_frac=ofrac)
        idx = np.nonzero(F.map_point >= 0)[0]
        edges = pose.make_edges(F.keys, 1.0 / F.level_sigma2, idx, xyz[F.map_point[idx]])
        ng, og, (qg, tg), sg = P.optimize(F.pose, cam, edges)
        no, oo, (qo, to), so = oracle.pose_optimization_edges(F.pose, cam, edges)
        assert ng == no and np.array_equal(og, oo), (seed, ng, no)
        assert sg["rounds"] == so["rounds"]
        for a, b in ((qg, qo), (tg, to)):
            assert np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)) <= 1e-4


@pytest.mark.parametrize("cfg", [dict(n_opt=10, n_fixed=3, n_points=300, obs_per_point=6, seed=21),
                                 dict(n_opt=50, n_fixed=10, n_points=3000, obs_per_point=8, seed=22)],
                         ids=["10kf", "50kf"])
def test_kb8_local_bundle_adjustment(gpu_lib, oracle, cam, cfg):
    from mam3slam_amd.lba import LBASolver, synthetic_problem

    prob = synthetic_problem(**cfg, camera=cam)
    assert prob.cam_model == 1 and prob.cams.shape == (1, 8)
    rg = LBASolver().solve(prob)
    ro = oracle.lba_solve(prob)
    assert rg.status == 0 and ro.status == 0
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
    for a, b in ((rg.pose_t, ro.pose_t), (rg.pose_q, ro.pose_q), (rg.point_xyz, ro.point_xyz)):
        num = np.linalg.norm(np.asarray(a) - np.asarray(b), axis=-1)
        den = np.maximum(np.linalg.norm(np.asarray(b), axis=-1), 1e-9)
        assert float((num / den).max()) <= 1e-4
    assert ro.final_chi2 < ro.initial_chi2


@pytest.mark.parametrize("model", ["pinhole", "kb8"])
@pytest.mark.parametrize("ori", [False, True])
def test_search_for_triangulation_batch_device(gpu_lib, oracle, frames, cam, model, ori):
    """The batched device form (CreateNewMapPoints' searches over keyframe slots in HBM, FeatureVectors as per-feature
    node + weight): every pair's matches equal the oracle's SearchForTriangulation on the same keyframes, with stopped
    words (weight 0) left out of the FeatureVectors and keyframes of different sizes."""
    import torch

    from mam3slam_amd.match import FramesDev, TriBatch

    dev = torch.device("cuda", 0)
    w, h, k, d = frames[1]
    c = cam if model == "kb8" else scene.pinhole(w, h, 450.0)
    M = _matcher(0.6, ori)
    rng = np.random.default_rng(3600 + ori)
    F = scene.make_frame_data(k, d, w, h)
    kfs = []
    for j in range(3):   # three pairs of keyframes generated around the frame, 6 slots
        KF1, KF2 = scene.keyframe_pair_3d(F, c, rng)
        kfs += [KF1, KF2]
    S = max(len(x.keys) for x in kfs) + 5
    nkf = len(kfs)
    keys = np.zeros((nkf, S), kfs[0].keys.dtype)
    desc = np.zeros((nkf, S, 32), np.uint8)
    cnt = np.zeros((nkf, 2), np.int32)
    has = np.zeros((nkf, S), np.uint8)
    nid = np.zeros((nkf, S), np.uint32)
    wt = np.zeros((nkf, S), np.float64)
    tcw = np.zeros(nkf, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for s_, KF in enumerate(kfs):
        n = len(KF.keys)
        keys[s_, :n], desc[s_, :n], cnt[s_, 0] = KF.keys, KF.desc, n
        has[s_, :n] = KF.has_mp
        stopped = rng.random(n) < 0.05   # stopped words: not in the FeatureVector
        fv = {}
        for node, feats in KF.featvec.items():
            for i in feats:
                nid[s_, i] = node
                if not stopped[i]:
                    wt[s_, i] = 1.0
                    fv.setdefault(node, []).append(i)
        KF.featvec = fv
        tcw[s_]["q"], tcw[s_]["t"] = KF.pose
    pairs = np.array([[0, 1], [2, 3], [4, 5], [1, 0], [0, 3], [5, 2]], np.int32)
    t = {n: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for n, v in
         dict(keys=keys.view(np.uint8), desc=desc, cnt=cnt, has=has, nid=nid, wt=wt, tcw=tcw.view(np.uint8),
              pairs=pairs).items()}
    out = torch.full((len(pairs), S), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
    b = TriBatch()
    b.kfs = FramesDev(nkf, S, t["keys"].data_ptr(), t["desc"].data_ptr(), t["cnt"].data_ptr(), None, None, 0)
    b.has_mp, b.nid, b.weight, b.tcw = t["has"].data_ptr(), t["nid"].data_ptr(), t["wt"].data_ptr(), t["tcw"].data_ptr()
    b.npairs, b.pairs = len(pairs), t["pairs"].data_ptr()
    M.search_for_triangulation_batch_device(kfs[0], c, b, out.data_ptr(), nm.data_ptr())
    torch.cuda.synchronize()
    og, ng = out.cpu().numpy(), nm.cpu().numpy()
    total = 0
    for q, (a1, a2) in enumerate(pairs):
        no, oo = oracle.search_for_triangulation_kf(kfs[a1], kfs[a2], c, c, ori, False)
        n1 = len(kfs[a1].keys)
        assert ng[q] == no and np.array_equal(og[q, :n1], oo), (q, ng[q], no)
        total += no
    assert total > 100
