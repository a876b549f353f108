"""CPU: the C oracle's LocalBundleAdjustment (oracle/lba_oracle.cpp — which also made the self-generated golden
fixture tests/golden/lba.npz) against an independent dense restatement (oracle/lba_dense_numpy.py: the whole Hessian,
numpy LU, no Schur complement). Same Levenberg iterations and trials, poses and points within 1e-6 relative: a
regression in the oracle's Schur / LDL^T / ordering code would show up here, where the golden fixture only pins the
oracle against itself."""
import numpy as np
import pytest


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_lba_matches_dense_restatement(oracle, seed):
    from mam3slam_amd.lba import synthetic_problem
    from oracle import lba_dense_numpy

    prob = synthetic_problem(n_opt=5, n_fixed=2, n_points=60, obs_per_point=4, seed=seed)
    r = oracle.lba_solve(prob)
    d = lba_dense_numpy.solve(prob)
    assert (r.iterations, r.lm_trials) == (d["iterations"], d["lm_trials"])
    scale = float(np.abs(d["point_xyz"]).max())
    assert np.abs(r.point_xyz - d["point_xyz"]).max() <= 1e-6 * scale
    assert np.abs(r.pose_t - d["pose_t"]).max() <= 1e-6 * max(1.0, float(np.abs(d["pose_t"]).max()))
    # q and -q are the same rotation
    dq = np.minimum(np.abs(r.pose_q - d["pose_q"]).max(1), np.abs(r.pose_q + d["pose_q"]).max(1))
    assert dq.max() <= 1e-6
