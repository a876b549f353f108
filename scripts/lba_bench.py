"""Standalone LocalBundleAdjustment timing (BASELINE configs[2] window: 50 KF / 3000 MP): wall time per solve
on an idle GPU, per-stage GPU time, LM iterations/trials, and the oracle solve time for the same problem.

    python scripts/lba_bench.py [--solves 20] [--obs 8] [--oracle]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solves", type=int, default=20)
    ap.add_argument("--obs", type=int, default=8)
    ap.add_argument("--kf", type=int, default=50)
    ap.add_argument("--points", type=int, default=3000)
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args()
    from mam3slam_amd.lba import LBASolver, synthetic_problem

    prob = synthetic_problem(n_opt=a.kf, n_fixed=10, n_points=a.points, obs_per_point=a.obs, seed=1)
    S = LBASolver()
    r = S.solve(prob)   # warm-up (allocations, code objects)
    S.set_profiling(True)
    ts = []
    for _ in range(a.solves):
        t = time.perf_counter()
        r = S.solve(prob)
        ts.append((time.perf_counter() - t) * 1e3)
    st = S.stage_times()
    out = {"kf": a.kf, "points": a.points, "edges": int(len(prob.edge_point)), "iterations": r.iterations,
           "trials": r.lm_trials, "ms_per_solve_median": float(np.median(ts)), "ms_per_solve_min": float(min(ts)),
           "stage_ms_per_solve": {k: v[0] / a.solves for k, v in st.items()},
           "stage_launches_per_solve": {k: v[1] / a.solves for k, v in st.items()}}
    if a.oracle:
        from oracle import oracle_py

        t = time.perf_counter()
        ro = oracle_py.lba_solve(prob)
        out["oracle_ms"] = (time.perf_counter() - t) * 1e3
        rel = np.abs(ro.point_xyz - r.point_xyz).max() / np.abs(ro.point_xyz).max()
        out["max_point_rel_diff_vs_oracle"] = float(rel)
        out["same_control_flow"] = (ro.iterations, ro.lm_trials) == (r.iterations, r.lm_trials)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
