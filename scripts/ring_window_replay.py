"""Replay LBA windows dumped by ring_leg_probe.py --dump (npz): trim each to its compacted prefix and solve it with
the single-problem API (--mode single), the device batch API (--mode batch) or the CPU oracle (--mode oracle)."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def load(path):
    from mam3slam_amd.lba import HUBER_MONO, LBAProblem

    z = np.load(path)
    out = []
    w = 0
    while f"w{w}_edge_point" in z.files:
        g = lambda f: z[f"w{w}_{f}"]  # noqa: E731
        ep = g("edge_point")
        d = np.where(np.diff(ep) < 0)[0]
        E = int(d[0] + 1) if len(d) else len(ep)
        L = int(ep[:E].max() + 1)
        P = len(g("pose_fixed"))
        meta = g("meta")
        out.append(LBAProblem(pose_id=np.arange(P, dtype=np.int64), pose_fixed=g("pose_fixed")[:P], pose_q=g("pose_q")[:P],
                              pose_t=g("pose_t")[:P], point_id=np.arange(L, dtype=np.int64) + P, point_xyz=g("point_xyz")[:L],
                              edge_point=ep[:E], edge_pose=g("edge_pose")[:E], edge_obs=g("edge_obs")[:E],
                              edge_inv_sigma2=g("edge_inv_sigma2")[:E], cams=g("cams"), huber_delta=float(meta[0]),
                              iterations=int(meta[1]), edge_active=None, cam_model=int(meta[2])).contiguous())
        w += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--mode", choices=("single", "batch", "oracle"), default="single")
    ap.add_argument("--windows", type=int, default=0, help="how many windows (0: all)")
    ap.add_argument("--repeat", type=int, default=1, help="the windows repeated this many times in the batch")
    ap.add_argument("--solves", type=int, default=1, help="batch solves (timed after the first)")
    a = ap.parse_args()
    probs = load(a.npz)
    if a.windows:
        probs = probs[:a.windows]
    probs = probs * a.repeat
    for i, p in enumerate(probs):
        print(f"window {i}: P {len(p.pose_id)} opt {int((p.pose_fixed == 0).sum())} L {len(p.point_id)} "
              f"E {len(p.edge_point)}", flush=True)
    if a.mode == "oracle":
        from oracle import oracle_py as oracle
        oracle.build()
        for i, p in enumerate(probs):
            t0 = time.perf_counter()
            r = oracle.lba_solve(p)
            print(f"oracle {i}: status {r.status} its {r.iterations} trials {r.lm_trials} chi2 {r.initial_chi2:.6g} -> "
                  f"{r.final_chi2:.6g} ({time.perf_counter() - t0:.1f} s)", flush=True)
        return
    import torch

    from mam3slam_amd.lba import LBASolver

    torch.zeros(1, device="cuda")   # torch's HIP runtime first (as bench.py and the tests do)
    s = LBASolver()
    if a.mode == "single":
        for i, p in enumerate(probs):
            r = s.solve(p)
            ts = []
            for _ in range(a.solves - 1):
                t0 = time.perf_counter()
                s.solve(p)
                ts.append((time.perf_counter() - t0) * 1e3)
            med = f" ms per solve median {np.median(ts):.3f} min {min(ts):.3f}" if ts else ""
            print(f"single {i}: status {r.status} its {r.iterations} trials {r.lm_trials} chi2 {r.initial_chi2:.6g} -> "
                  f"{r.final_chi2:.6g}{med}", flush=True)
    else:
        from mam3slam_amd.lba import DeviceBatch

        B = DeviceBatch(probs, torch.device("cuda", 0))
        st = s.solve_batch_device(B)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.solves - 1):
            t0 = time.perf_counter()
            s.solve_batch_device(B)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        if ts:
            print(f"batch of {len(probs)}: ms per solve median {np.median(ts):.3f} min {min(ts):.3f}", flush=True)
        for i in range(min(len(probs), 4)):
            r = B.result(i)
            print(f"batch {i}: {st[i]} chi2 {r.initial_chi2:.6g} -> {r.final_chi2:.6g}", flush=True)


if __name__ == "__main__":
    main()
