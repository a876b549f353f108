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
    ap.add_argument("--batch", type=int, default=0, help="also time Q problems solved together on the device path")
    ap.add_argument("--world", action="store_true",
                    help="windows of the shared synthetic map (mam3slam_amd/world.py, banded covisibility) instead of "
                         "synthetic_problem's random covisibility")
    a = ap.parse_args()
    if a.batch:
        import torch

        torch.cuda.init()   # torch's HIP runtime first: it does not attach after the library has initialised HIP
    from mam3slam_amd.lba import LBASolver, synthetic_problem

    if a.world:
        from mam3slam_amd import world as W

        wd = W.make_world(n_kf=25 * max(a.batch, 1) + 80, seed=7)
        mk = lambda q: W.window(wd, 25 * q, n_opt=a.kf)[0]   # noqa: E731
    else:
        mk = lambda q: synthetic_problem(n_opt=a.kf, n_fixed=10, n_points=a.points, obs_per_point=a.obs,  # noqa: E731
                                         seed=1 + q)
    prob = mk(0)
    S = LBASolver()
    r = S.solve(prob)   # warm-up (allocations, code objects)
    ts = []
    for _ in range(a.solves):   # wall time with no stage events in the stream
        t = time.perf_counter()
        r = S.solve(prob)
        ts.append((time.perf_counter() - t) * 1e3)
    S.set_profiling(True)   # per-stage GPU time from a second, profiled pass
    for _ in range(a.solves):
        S.solve(prob)
    st = S.stage_times()
    S.set_profiling(False)
    out = {"kf": a.kf, "points": int(len(prob.point_id)), "edges": int(len(prob.edge_point)), "world": a.world,
           "iterations": r.iterations,
           "trials": r.lm_trials, "ms_per_solve_median": float(np.median(ts)), "ms_per_solve_min": float(min(ts)),
           "stage_ms_per_solve": {k: v[0] / a.solves for k, v in st.items()},
           "stage_launches_per_solve": {k: v[1] / a.solves for k, v in st.items()}}
    if a.batch:
        import torch

        from mam3slam_amd.lba import DeviceBatch

        probs = [mk(q) for q in range(a.batch)]
        for Q in sorted({1, a.batch}):
            B = DeviceBatch(probs[:Q], torch.device("cuda", 0))
            S.solve_batch_device(B)
            torch.cuda.synchronize()
            tb = []
            for _ in range(max(3, a.solves // 2)):
                t = time.perf_counter()
                S.solve_batch_device(B)
                tb.append((time.perf_counter() - t) * 1e3)
            out[f"device_batch_{Q}"] = {"ms_per_batch_median": float(np.median(tb)),
                                        "solves_per_s": Q / (float(np.median(tb)) * 1e-3),
                                        "trials": [s["lm_trials"] for s in B.stats]}
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
