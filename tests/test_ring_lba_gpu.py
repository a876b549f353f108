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


def _ring(cfg, B, W):
    import torch

    import bench
    from mam3slam_amd.mapping import NewMapPointsLeg

    dev = torch.device("cuda", 0)
    tr = bench.TrackingLeg(dict(bench.CONFIGS[cfg]), B, 1, 0, dev)
    nm = NewMapPointsLeg(tr, W, dev)
    for step in range(nm.R // nm.W + 2):   # the ring past one turn: every neighbour a tracked keyframe
        tr.step()
        nm.ingest(step)
        nm.launch(nm.pending)
    return tr, nm


@pytest.mark.parametrize("cfg,B,W", [("c1", 16, 2), ("c3", 2, 2)])
def test_ring_windows_covisibility_rule(gpu_lib, oracle, cfg, B, W):
    """The reference's window rule (Optimizer.cc:1118-1186) on the ring, compacted: local keyframes = the new keyframe
    + the neighbours sharing >= 15 of its MapPoints by weight (the heaviest when none does), fixed = the other
    neighbours that observe one (the n_fixed least covisible when that leaves none fixed), points = its MapPoints seen
    by >= 2 keyframes, edges = their real observations, a neighbour keypoint claimed by several MapPoints kept by the
    first — every array, the
    sizes and the slot / keypoint maps byte-exact against a host restatement from the ring buffers; the solve against
    the oracle on the assembled graph (identical Levenberg control flow, 1e-4)."""
    import torch

    from mam3slam_amd.mapping import RingLBA
    from mam3slam_amd.match import FUSE_MP_DTYPE
    from mam3slam_amd.orb import KP_DTYPE

    tr, nm = _ring(cfg, B, W)
    rl = RingLBA(nm)
    rl.assemble(nm.stream)
    rl.solve(nm.stream)
    torch.cuda.synchronize()
    S, NN = nm.S, nm.NN
    keys = nm.keys.cpu().numpy().view(KP_DTYPE).reshape(nm.R, S)
    cnt = nm.cnt.cpu().numpy()[:, 0]
    tcw = nm.tcw.cpu().numpy().view(np.float32).reshape(nm.R, 7)
    mps = nm.fmp.cpu().numpy().view(FUSE_MP_DTYPE).reshape(nm.R, S)
    match = nm.fwd_idx.cpu().numpy()
    pairs = nm.pairs[nm.head].cpu().numpy()
    inv_s2 = (np.float32(1.0) / np.asarray(tr.F0.level_sigma2, np.float32)).astype(np.float32)
    pose_slot, point_src = rl.pose_slot.cpu().numpy(), rl.point_src.cpu().numpy()
    n_local_total = 0
    for w in range(W):
        j = int(pairs[w * NN, 0])
        nbs = [int(pairs[w * NN + k, 1]) for k in range(NN)]
        n = min(int(cnt[j]), S)
        mask = np.zeros((n, NN), bool)
        for k in range(NN):
            idx = match[w * NN + k, :n]
            mask[:, k] = (idx >= 0) & (idx < min(int(cnt[nbs[k]]), S))
            # one MapPoint per neighbour keypoint: the first claimant keeps it (Fuse merges the others)
            seen = set()
            for p in range(n):
                if mask[p, k]:
                    if int(idx[p]) in seen:
                        mask[p, k] = False
                    seen.add(int(idx[p]))
        wt = mask.sum(0)
        order = sorted((k for k in range(NN) if wt[k] > 0), key=lambda k: (-wt[k], k))   # covisibility order
        nloc = sum(1 for k in order if wt[k] >= RingLBA.COVIS_TH)
        if nloc == 0 and order:
            nloc = 1
        if nloc == len(order):   # no fixed observer: the least covisible n_fixed are the gauge anchor
            nloc = max(len(order) - rl.n_fixed, min(len(order), 1))
        views = [0] + [1 + k for k in order]
        vpose = {v: i for i, v in enumerate(views)}
        slots = [j if v == 0 else nbs[v - 1] for v in views]
        nopt = 1 + nloc
        n_local_total += nopt
        kept = [p for p in range(n) if mask[p].any()]
        ep, eo, obs, w2 = [], [], [], []
        for i, p in enumerate(kept):
            for v in [0] + [1 + k for k in range(NN) if mask[p, k]]:
                slot = j if v == 0 else nbs[v - 1]
                kp = keys[slot, p if v == 0 else int(match[w * NN + v - 1, p])]
                ep.append(i)
                eo.append(vpose[v])
                obs.append((kp["x"], kp["y"]))
                w2.append(inv_s2[kp["octave"]])
        assert tuple(rl.sizes[w]) == (len(views), len(kept), len(ep), nopt)
        assert np.array_equal(pose_slot[w, :len(views)], slots)
        assert np.array_equal(point_src[w, :len(kept)], kept)
        prob = rl.window(w)
        assert np.array_equal(prob.pose_q, tcw[slots, :4].astype(np.float64))
        assert np.array_equal(prob.pose_t, tcw[slots, 4:7].astype(np.float64))
        assert np.array_equal(prob.pose_fixed, (np.arange(len(views)) >= nopt).astype(np.uint8))
        assert np.array_equal(prob.point_xyz, mps[j, kept]["pos"].astype(np.float64))
        assert np.array_equal(prob.edge_point, ep) and np.array_equal(prob.edge_pose, eo)
        assert np.array_equal(prob.edge_obs, np.array(obs, np.float64).reshape(-1, 2))
        assert np.array_equal(prob.edge_inv_sigma2, np.array(w2, np.float64))
        assert len(ep) > 3 * len(kept), (len(ep), len(kept))   # a multi-view graph
        q, t, x, its, trials, st, ic, fc = rl.result(w)
        ro = oracle.lba_solve(prob)
        assert st == 0 and ro.status == 0
        assert (its, trials) == (ro.iterations, ro.lm_trials), (w, its, trials, ro.iterations, ro.lm_trials)
        assert abs(fc - ro.final_chi2) <= 1e-6 * ro.final_chi2 and fc < ic
        assert _rel(t, ro.pose_t) <= 1e-4 and _rel(q, ro.pose_q) <= 1e-4 and _rel(x, ro.point_xyz) <= 1e-4
    assert n_local_total > 2 * W   # covisible neighbours were found (not only the keyframe itself)
    assert all(int(v[0]) > int(v[3]) for v in rl.sizes)   # every window has fixed keyframes


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
    rl = RingLBA(nm, rule="sequence")
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
