"""GPU: LocalBundleAdjustment windows built from the keyframes Tracking inserted (mam_ring_lba_windows on the
NewMapPointsLeg ring: the new keyframe and its 30 neighbours, its keypoints' MapPoints, their observations from the
run's forward Fuse matches) — the assembly byte-exact against a host restatement from the same ring buffers, and the
device solve against the oracle on the assembled graph (identical Levenberg control flow, 1e-4)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    num = np.linalg.norm(a - b, axis=-1)
    den = np.maximum(np.linalg.norm(b, axis=-1), 1e-9)
    return float((num / den).max()) if len(a) else 0.0


@pytest.mark.parametrize("cfg,B,W", [("c1", 16, 2), ("c3", 2, 2)])
def test_ring_windows_match_oracle(gpu_lib, oracle, cfg, B, W):
    import torch

    import bench
    from mam3slam_amd.mapping import NewMapPointsLeg, RingLBA
    from mam3slam_amd.match import FUSE_MP_DTYPE
    from mam3slam_amd.orb import KP_DTYPE

    dev = torch.device("cuda", 0)
    tr = bench.TrackingLeg(dict(bench.CONFIGS[cfg]), B, 1, 0, dev)
    nm = NewMapPointsLeg(tr, W, dev)
    for step in range(nm.R // nm.W + 2):   # the ring past one turn: every neighbour a tracked keyframe
        tr.step()
        nm.ingest(step)
        nm.launch(nm.pending)
    rl = RingLBA(nm)
    rl.assemble(nm.stream)
    rl.solve(nm.stream)
    torch.cuda.synchronize()
    S, NN, NV = nm.S, nm.NN, rl.NV
    keys = nm.keys.cpu().numpy().view(KP_DTYPE).reshape(nm.R, S)
    cnt = nm.cnt.cpu().numpy()[:, 0]
    tcw = nm.tcw.cpu().numpy().view(np.float32).reshape(nm.R, 7)
    mps = nm.fmp.cpu().numpy().view(FUSE_MP_DTYPE).reshape(nm.R, S)
    match = nm.fwd_idx.cpu().numpy()
    pairs = nm.pairs[nm.head].cpu().numpy()
    inv_s2 = (np.float32(1.0) / np.asarray(tr.F0.level_sigma2, np.float32)).astype(np.float32)
    for w in range(W):
        prob = rl.window(w)
        j = int(pairs[w * NN, 0])
        slots = [j] + [int(pairs[w * NN + k, 1]) for k in range(NN)]
        assert np.array_equal(prob.pose_q, tcw[slots, :4].astype(np.float64))
        assert np.array_equal(prob.pose_t, tcw[slots, 4:7].astype(np.float64))
        assert np.array_equal(prob.pose_fixed, (np.arange(NV) >= NV - rl.n_fixed).astype(np.uint8))
        n = int(cnt[j])
        xyz = np.zeros((S, 3))
        xyz[:n] = mps[j, :n]["pos"].astype(np.float64)
        assert np.array_equal(prob.point_xyz, xyz)
        act = np.zeros((S, NV), np.uint8)
        obs = np.zeros((S, NV, 2))
        w2 = np.ones((S, NV))
        for p in range(n):
            idx = [p] + [int(match[w * NN + k, p]) for k in range(NN)]
            ok = [True] + [0 <= idx[v] < min(int(cnt[slots[v]]), S) for v in range(1, NV)]
            if sum(ok) < 2:
                continue
            for v in range(NV):
                if ok[v]:
                    kp = keys[slots[v], idx[v]]
                    act[p, v] = 1
                    obs[p, v] = (kp["x"], kp["y"])
                    w2[p, v] = inv_s2[kp["octave"]]
        assert np.array_equal(prob.edge_active, act.reshape(-1))
        assert np.array_equal(prob.edge_obs, obs.reshape(-1, 2)) and np.array_equal(prob.edge_inv_sigma2, w2.reshape(-1))
        assert np.array_equal(prob.edge_point, np.repeat(np.arange(S), NV))
        assert np.array_equal(prob.edge_pose, np.tile(np.arange(NV), S))
        n_act = int(act.sum())
        assert n_act > 4 * n, (n_act, n)   # a real multi-view graph: several observations per MapPoint on average
        q, t, x, its, trials, st, ic, fc = rl.result(w)
        ro = oracle.lba_solve(prob)
        assert st == 0 and ro.status == 0
        assert (its, trials) == (ro.iterations, ro.lm_trials), (w, its, trials, ro.iterations, ro.lm_trials)
        assert abs(fc - ro.final_chi2) <= 1e-6 * ro.final_chi2 and fc < ic
        assert _rel(t, ro.pose_t) <= 1e-4 and _rel(q, ro.pose_q) <= 1e-4 and _rel(x, ro.point_xyz) <= 1e-4
