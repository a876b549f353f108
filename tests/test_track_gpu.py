"""GPU: the per-frame Tracking sequence bench.py times — TrackWithMotionModel (SearchByProjection(Cur, Last, th 15),
Optimizer::PoseOptimization, outlier discard: Tracking.cc:2786-2862) then TrackLocalMap (isInFrustum +
SearchByProjection(F, localMPs, th 1), PoseOptimization: Tracking.cc:2878-2901) — on device-resident frames, every
stage against the oracle on the stage's own inputs: the searches index-exact, the PoseOptimization edges exact, its
outlier sets identical and its pose within 1e-4, the discard and Frame::SetPose exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", ["c1", "c3"])
def test_tracking_sequence_matches_oracle(gpu_lib, oracle, cfg):
    import torch

    import bench
    from mam3slam_amd import scene
    from mam3slam_amd.match import LAST_ENTRY_DTYPE, MP_TRACK_DTYPE
    from mam3slam_amd.orb import KP_DTYPE
    from mam3slam_amd.pose import POSE_EDGE_DTYPE, POSE_RESULT_DTYPE, make_edges, set_pose_float

    dev = torch.device("cuda", 0)
    B = 8
    tr = bench.TrackingLeg(dict(bench.CONFIGS[cfg]), B, 2, 0, dev)
    tr.step()
    torch.cuda.synchronize()
    cap = tr.cap
    kps = tr.d_kps.cpu().numpy().view(KP_DTYPE).reshape(B, cap)
    desc = tr.d_desc.cpu().numpy()
    cnt = tr.d_cnt.cpu().numpy()
    out1, out2 = tr.d_out1.cpu().numpy(), tr.d_out2.cpu().numpy()
    taken = tr.d_taken.cpu().numpy()
    pn = tr.d_pn.cpu().numpy()
    pout = tr.d_pout.cpu().numpy()
    pres = tr.d_pres.cpu().numpy().view(POSE_RESULT_DTYPE).reshape(2, B)
    pe2 = tr.d_pe.cpu().numpy().view(POSE_EDGE_DTYPE).reshape(B, cap)
    tcw = tr.d_tcw.cpu().numpy().view(np.float32).reshape(B, 7)
    tracks = tr.d_mps.cpu().numpy().view(MP_TRACK_DTYPE).reshape(B, -1)
    n_out = 0
    for f in range(B):
        n = int(cnt[f, 0])
        F = scene.make_frame_data(kps[f, :n], desc[f, :n], tr.W, tr.H)
        # TrackWithMotionModel: motion search at the motion model's guess
        F.pose = tr.poses_init[f]
        last = np.ascontiguousarray(tr.lasts[f], LAST_ENTRY_DTYPE)
        _, o1 = oracle.search_by_projection_motion(F, last, tr.cam, 15.0, True)
        assert (o1 >= 0).sum() >= 20, "TrackWithMotionModel's wider-window retry (nmatches < 20) is not reproduced"
        idx = np.nonzero(o1 >= 0)[0]
        e1 = make_edges(F.keys, tr.inv_s2, idx, last["pos"][o1[idx]])
        assert int(pn[0, f]) == len(e1)
        r1, ol1, (q1, t1), _ = oracle.pose_optimization_edges(tr.poses_init[f], tr.cam, e1)
        assert np.array_equal(pout[0, f, :len(e1)], ol1), f
        assert int(pres[0, f]["n_inliers"]) == r1
        assert np.abs(pres[0, f]["t"] - t1).max() <= 1e-4 * max(np.abs(t1).max(), 1.0)
        assert np.abs(pres[0, f]["q"] - q1).max() <= 1e-4
        n_out += int(ol1.sum())
        # outliers discarded (mvpMapPoints[i] = NULL); the slots the local-map search may not take
        o1 = o1.copy()
        o1[idx[ol1 == 1]] = -1
        assert np.array_equal(out1[f, :n], o1), f
        tk = ((o1 >= 0) & (last["nobs"][np.maximum(o1, 0)] > 0)).astype(np.uint8)
        assert np.array_equal(taken[f, :n], tk), f
        # TrackLocalMap at the GPU's optimised pose (Frame::SetPose of call 1)
        F.pose = set_pose_float(pres[0, f]["q"], pres[0, f]["t"])
        nv, to = oracle.is_in_frustum(F, tr.mpls[f], tr.cam)
        tg = tracks[f, :len(tr.mpls[f])]
        assert np.array_equal(tg["proj_x"], to["proj_x"]) and np.array_equal(tg["proj_y"], to["proj_y"]), f
        F.taken = tk
        _, o2 = oracle.search_by_projection(F, to, 1.0, False, 50.0, 0.8)
        assert np.array_equal(out2[f, :n], o2), f
        # PoseOptimization with every match: the local-map search's where it made one, else the motion search's
        has = (o2 >= 0) | (o1 >= 0)
        idx2 = np.nonzero(has)[0]
        mp = np.ascontiguousarray(tr.mpls[f])
        pos = np.where((o2[idx2] >= 0)[:, None], mp["pos"][np.maximum(o2[idx2], 0)], last["pos"][np.maximum(o1[idx2], 0)])
        e2 = make_edges(F.keys, tr.inv_s2, idx2, pos)
        assert int(pn[1, f]) == len(e2) and np.array_equal(pe2[f, :len(e2)], e2), f
        r2, ol2, (q2, t2), _ = oracle.pose_optimization_edges(F.pose, tr.cam, e2)
        assert np.array_equal(pout[1, f, :len(e2)], ol2), f
        assert np.abs(pres[1, f]["t"] - t2).max() <= 1e-4 * max(np.abs(t2).max(), 1.0)
        # the frame's final pose is call 2's, as Frame::SetPose stores it
        qf, tf = set_pose_float(pres[1, f]["q"], pres[1, f]["t"])
        assert np.array_equal(tcw[f, :4], qf) and np.array_equal(tcw[f, 4:], tf), f
        # and it is the rendering camera's pose up to the noise of the synthetic MapPoints
        assert np.abs(tf - tr.poses[f][1]).max() < 0.02, (tf, tr.poses[f][1])
    assert n_out > 0   # the last frame's outlier block is rejected somewhere
