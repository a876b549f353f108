"""GPU parity: LocalBundleAdjustment solve (HIP, FP64) vs the g2o restatement oracle.

Bar (BASELINE.json north_star): poses and points within 1e-4 relative; the Levenberg control flow (iterations,
trials) identical; the outlier set the reference erases (chi2 > 5.991 || depth <= 0, Optimizer.cc:1413-1460)
identical except for edges whose chi2 sits within 1e-6 of the threshold.
"""
import numpy as np
import pytest

from mam3slam_amd.lba import LBASolver, synthetic_problem

pytestmark = pytest.mark.gpu

CASES = [
    dict(n_opt=6, n_fixed=2, n_points=120, obs_per_point=4, seed=3),
    dict(n_opt=10, n_fixed=3, n_points=300, obs_per_point=6, seed=1),
    # dense 20-KF system: 8 tile columns, 36 tiles in the LDS pool; the first columns hold 5-7 tiles below the
    # diagonal, so their tall panels run as two items on two waves (the diagonal factored redundantly in both)
    dict(n_opt=20, n_fixed=5, n_points=1000, obs_per_point=8, seed=7, init_kf_local=False),
    dict(n_opt=50, n_fixed=10, n_points=3000, obs_per_point=8, seed=11),   # BASELINE configs[2]
    dict(n_opt=50, n_fixed=10, n_points=3000, obs_per_point=12, seed=12, outlier_frac=0.15),
]


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    num = np.linalg.norm(a - b, axis=-1)
    den = np.maximum(np.linalg.norm(b, axis=-1), 1e-9)
    return float((num / den).max()) if len(a) else 0.0


@pytest.fixture(scope="module")
def solver(gpu_lib):
    return LBASolver()


@pytest.mark.parametrize("cfg", CASES, ids=lambda c: f"{c['n_opt']}kf_{c['n_points']}mp_s{c['seed']}")
def test_lba_matches_oracle(solver, oracle, cfg):
    prob = synthetic_problem(**cfg)
    rg = solver.solve(prob)
    ro = oracle.lba_solve(prob)
    assert rg.status == 0 and ro.status == 0
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert abs(rg.initial_chi2 - ro.initial_chi2) <= 1e-9 * ro.initial_chi2
    assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
    assert _rel(rg.pose_t, ro.pose_t) <= 1e-4
    assert _rel(rg.pose_q, ro.pose_q) <= 1e-4
    assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
    og, oo = rg.outliers(), ro.outliers()
    near = np.abs(ro.edge_chi2 - 5.991) <= 1e-6 * 5.991
    assert not np.any((og != oo) & ~near)
    assert ro.final_chi2 < ro.initial_chi2


def test_lba_fixed_only_points(solver, oracle):
    # every keyframe fixed: the solve reduces to independent 3x3 point systems
    prob = synthetic_problem(n_opt=4, n_fixed=4, n_points=100, obs_per_point=4, seed=5)
    prob.pose_fixed[:] = 1
    rg, ro = solver.solve(prob), oracle.lba_solve(prob)
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
    # fixed poses pass through SE3Quat(q, t), which renormalises (se3quat.h:60-63); otherwise untouched
    assert _rel(rg.pose_q, ro.pose_q) <= 1e-15 and _rel(rg.pose_q, prob.pose_q) < 1e-6


def test_lba_stop_flag(solver, oracle):
    prob = synthetic_problem(n_opt=8, n_fixed=2, n_points=200, seed=9)
    stop = np.ones(1, np.uint8)   # bool pbStopFlag
    rg = solver.solve(prob, stop)
    ro = oracle.lba_solve(prob, stop)
    assert rg.iterations == ro.iterations == 0 and rg.status == ro.status == 1
    assert _rel(rg.point_xyz, prob.point_xyz) == 0.0


def _stage2(prob, r, iterations=10):
    """The merge-window LBA's second optimisation (Optimizer.cc:3742-3779): chi2 > 5.991 or negative depth ->
    setLevel(1), every robust kernel removed, optimize(10) over level 0 from the first optimisation's estimates."""
    import dataclasses

    active = ~((r.edge_chi2 > 5.991) | ~r.edge_depth_ok.astype(bool))
    return dataclasses.replace(prob, pose_q=np.array(r.pose_q), pose_t=np.array(r.pose_t),
                               point_xyz=np.array(r.point_xyz), huber_delta=0.0, iterations=iterations,
                               edge_active=active.astype(np.uint8)), active


@pytest.mark.parametrize("seed", [4, 13])
def test_lba_merge_schedule(solver, oracle, seed):
    """Welding LBA schedule (Optimizer.cc:3730-3779): optimize(5) with Huber delta sqrt(5.99), then level-1 outliers
    and no kernels for optimize(10). Each side runs both stages on its own estimates."""
    prob = synthetic_problem(n_opt=12, n_fixed=4, n_points=600, obs_per_point=6, seed=seed, outlier_frac=0.12)
    prob.huber_delta = float(np.float32(np.sqrt(5.99)))
    prob.iterations = 5
    rg1, ro1 = solver.solve(prob), oracle.lba_solve(prob)
    pg, ag = _stage2(prob, rg1)
    po, ao = _stage2(prob, ro1)
    assert np.array_equal(ag, ao) and (~ao).sum() > 10
    rg, ro = solver.solve(pg), oracle.lba_solve(po)
    assert rg.status == 0 and ro.status == 0
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2 and ro.final_chi2 < ro.initial_chi2
    assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
    assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
    assert np.allclose(rg.edge_chi2[ao], ro.edge_chi2[ao], rtol=1e-6, atol=1e-9)
    # a point whose every edge is at level 1 keeps its stage-1 estimate
    ep = np.asarray(prob.edge_point)
    alive = np.zeros(len(prob.point_id), bool)
    alive[ep[ao]] = True
    if (~alive).any():
        assert np.array_equal(np.asarray(rg.point_xyz)[~alive], np.asarray(rg1.point_xyz)[~alive])


def test_lba_batch_device(solver, oracle):
    """mam_lba_solve_batch_device: problems of different sizes and schedules (Huber / no kernel, level-1 edges, all
    poses fixed) solved together, each problem's own Levenberg control flow on the device; every problem matches the
    oracle on the same (id-ordered) graph."""
    import torch

    from mam3slam_amd.lba import DeviceBatch, id_ordered

    probs = [synthetic_problem(**CASES[0]), synthetic_problem(**CASES[3]),
             synthetic_problem(n_opt=12, n_fixed=4, n_points=600, obs_per_point=6, seed=4, outlier_frac=0.12),
             synthetic_problem(n_opt=4, n_fixed=4, n_points=100, obs_per_point=4, seed=5)]
    probs[2].huber_delta = 0.0
    probs[2].edge_active = (np.arange(len(probs[2].edge_point)) % 7 != 3).astype(np.uint8)
    probs[3].pose_fixed[:] = 1
    B = DeviceBatch(probs, torch.device("cuda", 0))
    stats = solver.solve_batch_device(B)
    for i, p in enumerate(probs):
        ro = oracle.lba_solve(id_ordered(p)[0])
        rg = B.result(i)
        assert stats[i]["status"] == 0 and ro.status == 0
        assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials), i
        assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
        assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
        assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
        act = np.ones(len(p.edge_point), bool) if p.edge_active is None else p.edge_active.astype(bool)
        assert np.allclose(rg.edge_chi2[act], ro.edge_chi2[act], rtol=1e-6, atol=1e-9)
        assert np.array_equal(rg.edge_depth_ok, ro.edge_depth_ok)
    # a second call on the same batch reproduces the first bit for bit
    first = [B.result(i) for i in range(len(probs))]
    solver.solve_batch_device(B)
    for i in range(len(probs)):
        assert np.array_equal(B.result(i).point_xyz, first[i].point_xyz)


def test_lba_batch_same_shape(solver, oracle):
    """Problems of one shape in one device batch (the ring's covisibility windows: 21 optimised + 10 fixed poses, dense
    covisibility): every problem's arena scratch is its own. Regression: a hand-kept size formula that lagged the carve
    (the pose sums' POSE_SPLIT partials) let problem q's pose sums overrun problem q + 1's structure."""
    import torch

    from mam3slam_amd.lba import DeviceBatch, id_ordered

    probs = [synthetic_problem(n_opt=21, n_fixed=10, n_points=1500, obs_per_point=12, seed=40 + i, init_kf_local=False)
             for i in range(4)]
    B = DeviceBatch(probs, torch.device("cuda", 0))
    stats = solver.solve_batch_device(B)
    for i, p in enumerate(probs):
        ro = oracle.lba_solve(id_ordered(p)[0])
        rg = B.result(i)
        assert stats[i]["status"] == 0 and ro.status == 0
        assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials), i
        assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
        assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
        assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4


@pytest.mark.parametrize("alone", [False, True])
def test_lba_dense_column_chain(solver, oracle, alone, monkeypatch):
    """Dense reduced systems past the LDS tile pool go to the column-chain factorization (ldlt_mw: 8 workgroups per
    problem claim block columns in order; cross-workgroup flags and panels through agent-coherent loads / stores):
    nt 14, 19, 22, 24 batched (and alone with MAM_LBA_MW=2), the oracle's control flow and solution; a second batch solve reproduces the
    first bit for bit (the flags' launch tags advance, nothing is reset)."""
    import torch

    from mam3slam_amd.lba import DeviceBatch, id_ordered

    sizes = (36, 50, 58, 63) if not alone else (58,)
    if alone:
        monkeypatch.setenv("MAM_LBA_MW", "2")   # (batches only by default)
    probs = [synthetic_problem(n_opt=n, n_fixed=8, n_points=1200, obs_per_point=14, seed=80 + n, init_kf_local=False)
             for n in sizes]
    if alone:
        for p in probs:
            rg, ro = solver.solve(p), oracle.lba_solve(p)
            assert rg.status == 0 and ro.status == 0
            assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
            assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
            assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
            assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
        return
    B = DeviceBatch(probs, torch.device("cuda", 0))
    stats = solver.solve_batch_device(B)
    first = []
    for i, p in enumerate(probs):
        ro = oracle.lba_solve(id_ordered(p)[0])
        rg = B.result(i)
        first.append(rg.point_xyz.copy())
        assert stats[i]["status"] == 0 and ro.status == 0
        assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials), i
        assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
        assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
        assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
    solver.solve_batch_device(B)
    for i in range(len(probs)):
        assert np.array_equal(B.result(i).point_xyz, first[i])


def test_lba_dense_register_form(solver, oracle, monkeypatch):
    """Dense reduced systems past the LDS tile pool (every pose pair shares landmarks): the register form of the
    factorization (k_ldlt_reg, MAM_LBA_REG=1) holds 128 tiles in registers, the next ones in LDS and the rest in place in S; nt 15
    (all in registers), 19 (registers + LDS), 21 (+ 54 tiles in S). Batched and alone, the oracle's control flow and
    solution."""
    import torch

    from mam3slam_amd.lba import DeviceBatch, id_ordered

    monkeypatch.setenv("MAM_LBA_REG", "1")
    probs = [synthetic_problem(n_opt=n, n_fixed=8, n_points=1200, obs_per_point=14, seed=60 + n, init_kf_local=False)
             for n in (40, 50, 56)]
    B = DeviceBatch(probs, torch.device("cuda", 0))
    stats = solver.solve_batch_device(B)
    for i, p in enumerate(probs):
        ro = oracle.lba_solve(id_ordered(p)[0])
        for rg, st in ((B.result(i), stats[i]["status"]), (None, None)):
            if rg is None:
                rg = solver.solve(p)
                ro = oracle.lba_solve(p)
                st = rg.status
            assert st == 0 and ro.status == 0
            assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials), i
            assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
            assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
            assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4


@pytest.mark.parametrize("pw", ["2", "4", "8"])
def test_lba_points_per_workgroup(solver, oracle, pw, monkeypatch):
    """The point kernels at 2 / 4 / 8 points per workgroup (a lone window of many observations a point takes 2, batches
    8; MAM_LBA_PW forces one): the same Levenberg control flow and solution as the oracle at each."""
    monkeypatch.setenv("MAM_LBA_PW", pw)
    prob = synthetic_problem(n_opt=21, n_fixed=10, n_points=1200, obs_per_point=14, seed=31, init_kf_local=False)
    rg, ro = solver.solve(prob), oracle.lba_solve(prob)
    assert rg.status == 0 and ro.status == 0
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2
    assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
    assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4


def test_lba_size_bound(solver):
    """A problem whose dense pose x landmark table would exceed 4 GiB (1100 optimised poses x 1M points) is refused
    with MAM_ERR_CAPACITY and a message naming the sizes, before any scratch allocation."""
    from mam3slam_amd._lib import MamError
    from mam3slam_amd.lba import LBAProblem

    P, L = 1100, 1_000_000
    q = np.zeros((P, 4))
    q[:, 3] = 1.0
    prob = LBAProblem(pose_id=np.arange(P), pose_fixed=np.zeros(P, np.uint8), pose_q=q, pose_t=np.zeros((P, 3)),
                      point_id=np.arange(L), point_xyz=np.tile([0.0, 0.0, 5.0], (L, 1)),
                      edge_point=np.arange(P, dtype=np.int32), edge_pose=np.arange(P, dtype=np.int32),
                      edge_obs=np.zeros((P, 2)), edge_inv_sigma2=np.ones(P),
                      cams=np.array([[500.0, 500.0, 320.0, 240.0]], np.float32))
    with pytest.raises(MamError, match="rc=-2.*too large"):
        solver.solve(prob)
    # the context stays usable
    small = synthetic_problem(n_opt=5, n_fixed=2, n_points=100, obs_per_point=4, seed=3)
    assert solver.solve(small).status == 0


def test_lba_arena_reuse(solver, oracle):
    # the pose x point table and S are not cleared between batches (lba.hip k_struct_init / eidx_at): a small window
    # solved in the arena a large one left behind, then the large one again, must both match the oracle exactly as
    # fresh solves do
    big = synthetic_problem(n_opt=50, n_fixed=10, n_points=3000, obs_per_point=8, seed=21)
    small = synthetic_problem(n_opt=7, n_fixed=2, n_points=400, obs_per_point=5, seed=22)
    for prob in (big, small, big):
        rg, ro = solver.solve(prob), oracle.lba_solve(prob)
        assert rg.status == 0 and ro.status == 0
        assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
        assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4
        assert _rel(rg.pose_t, ro.pose_t) <= 1e-4


@pytest.mark.parametrize("n_opt", [200])
def test_lba_map_scale(solver, oracle, n_opt):
    """Map scale (the welding / global BA the reference runs over hundreds of keyframes — its own run
    reaches 478, output/KF_traj.txt): a 200-keyframe graph of the shared synthetic map (all its keyframes optimised
    but the map's first) solved by the same device LM — S is 1200 x 1200, beyond the LDS tile pool (40 tile columns),
    so the factorization takes the HBM form — against the oracle on the same graph; the time is printed."""
    import time

    from mam3slam_amd import world as W

    wd = W.make_world(n_kf=n_opt + 60, seed=21)
    prob = W.window(wd, 0, n_opt=n_opt)[0]
    assert int((np.asarray(prob.pose_fixed) == 0).sum()) >= n_opt - 1
    solver.solve(prob)   # warm (allocations)
    t0 = time.perf_counter()
    rg = solver.solve(prob)
    ms = (time.perf_counter() - t0) * 1e3
    ro = oracle.lba_solve(prob)
    print(f"\nmap-scale LBA: {n_opt} KF, {len(prob.point_id)} MP, {len(prob.edge_point)} edges: {ms:.1f} ms on the GPU, "
          f"{rg.iterations} iterations / {rg.lm_trials} trials")
    assert rg.status == 0 and ro.status == 0
    assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials)
    assert abs(rg.final_chi2 - ro.final_chi2) <= 1e-6 * ro.final_chi2 and ro.final_chi2 < ro.initial_chi2
    assert _rel(rg.pose_t, ro.pose_t) <= 1e-4 and _rel(rg.pose_q, ro.pose_q) <= 1e-4
    assert _rel(rg.point_xyz, ro.point_xyz) <= 1e-4


def test_lba_map_scale_478(solver):
    """The reference run's map size (478 keyframes, output/KF_traj.txt) on the device alone (S 2868 x 2868; the
    oracle's dense factorization would take minutes on one core): solved without a capacity error, chi2 reduced."""
    import time

    from mam3slam_amd import world as W

    wd = W.make_world(n_kf=540, seed=22)
    prob = W.window(wd, 0, n_opt=478)[0]
    t0 = time.perf_counter()
    rg = solver.solve(prob)
    ms = (time.perf_counter() - t0) * 1e3
    print(f"\nmap-scale LBA: 478 KF, {len(prob.point_id)} MP, {len(prob.edge_point)} edges: {ms:.1f} ms on the GPU, "
          f"{rg.iterations} iterations / {rg.lm_trials} trials")
    assert rg.status == 0 and rg.final_chi2 < rg.initial_chi2
