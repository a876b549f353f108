"""GPU: the LocalMapping leg bench.py times (mam3slam_amd/mapping.py) — windows read from the shared map, batched
LocalBundleAdjustment, write-backs packed / gathered / applied — against the oracle and the numpy exchange
restatement. Byte-exact for the map reads and the exchange; <= 1e-4 with identical Levenberg control flow for LBA."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_mapping_leg_matches_oracle(gpu_lib, oracle):
    import torch

    from mam3slam_amd.mapping import LocalMappingLeg
    from oracle import exchange_oracle as X

    dev = torch.device("cuda", 0)
    M = LocalMappingLeg(3, 0, 1, dev, max_gpus=1)
    for step, perturb in ((0, False), (1, True)):
        if perturb:
            M.new_keyframes(step)
        kf0, mp0 = M.kf_table.cpu().numpy().copy(), M.mp_table.cpu().numpy().copy()
        M.run(step, new_keyframes=False)
        torch.cuda.synchronize()
        assert int(M.status.item()) == 0
        kf_ref, mp_ref = kf0.copy(), mp0.copy()
        for w in range(M.W):
            prob = M.window_inputs(w)
            # the graph's estimates are the float map values cast to double (Optimizer.cc:1218, 1286)
            assert np.array_equal(prob.pose_q, kf0[M.kf_ids[w], :4].astype(np.float64))
            assert np.array_equal(prob.pose_t, kf0[M.kf_ids[w], 4:7].astype(np.float64))
            assert np.array_equal(prob.point_xyz, mp0[M.mp_ids[w], :3].astype(np.float64))
            rg = M.window_result(w)
            ro = oracle.lba_solve(prob)
            assert (rg.iterations, rg.lm_trials) == (ro.iterations, ro.lm_trials), (step, w)
            rel = np.abs(rg.point_xyz - ro.point_xyz).max() / np.abs(ro.point_xyz).max()
            assert rel <= 1e-4 and np.abs(rg.pose_t - ro.pose_t).max() <= 1e-4 * np.abs(ro.pose_t).max()
            # the window's write-back (Optimizer.cc:1478-1494), windows in order: what the compact block must leave
            X.writeback(kf_ref, mp_ref, rg.pose_q, rg.pose_t, prob.pose_id, prob.pose_fixed, rg.point_xyz,
                        prob.point_id - M.mp_base)
        assert np.array_equal(M.kf_table.cpu().numpy(), kf_ref)
        assert np.array_equal(M.mp_table.cpu().numpy(), mp_ref)
    # the next step's windows read the applied map
    assert not np.array_equal(M.window_inputs(1).point_xyz, M.probs[1].point_xyz)
