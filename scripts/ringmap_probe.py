#!/usr/bin/env python3
"""Probe of the device map LocalMapping leg (mapping.NewMapPointsLeg + RingMappingLeg over ringmap.RingMap): runs
`--runs` LocalMapping runs after tracking steps and prints, per run, the map's size (MapPoints, observations per
MapPoint, MapPoints per keyframe), the windows' shape (optimised / fixed keyframes, points, edges) and the host time
of the run; with --check, the first solved window of the last run against the oracle; with --dump, the last run's
solved windows as an npz scripts/ring_window_replay.py replays."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--kf-every", type=int, default=8)
    ap.add_argument("--runs", type=int, default=12)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dump", default=None, help="npz of the last run's solved windows (scripts/ring_window_replay.py)")
    a = ap.parse_args()
    import torch

    import bench
    from mam3slam_amd.mapping import NewMapPointsLeg, RingMappingLeg

    dev = torch.device("cuda", 0)
    cfg = dict(bench.CONFIGS[a.config])
    tr = bench.TrackingLeg(cfg, a.batch, 2, 0, dev)
    W = max(1, a.batch // a.kf_every)
    nm = NewMapPointsLeg(tr, W, dev)
    leg = RingMappingLeg(nm, 0, 1, dev)
    rows = []
    for r in range(a.runs):
        tr.step()
        item = nm.ingest(r)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        leg.run(r, item)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        sz = leg.rl.sizes
        v = sz[:, 2] > 0
        st = nm.map.stats()
        nk, nmp, hst = leg.exchange_counts()
        row = {"run": r, "ms": round(ms, 2), "windows_solved": int(v.sum()),
               "opt_kf": float(sz[v, 3].mean()) if v.any() else 0, "fixed_kf": float((sz[v, 0] - sz[v, 3]).mean()) if v.any() else 0,
               "points": float(sz[v, 1].mean()) if v.any() else 0, "edges": float(sz[v, 2].mean()) if v.any() else 0,
               "trials": float(np.mean([s[1] for s in leg.stats])), **st, "exch_kf": nk, "exch_mp": nmp,
               "exch_status": hst, "tri_matches": float(nm.nmatch.float().mean().item()),
               "fwd_fused": float(nm.fwd_n.float().mean().item()), "bwd_fused": float(nm.bwd_n.float().mean().item())}
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"rows": rows}
    # the last run's first window: covisibility weights of its keyframe with every ring slot (host, from the map)
    snap = nm.map.snapshot()
    R, S = nm.R, nm.S
    mp_of = snap["mp_of"].reshape(R, S)
    j = nm.head
    wt = np.zeros(R, np.int64)
    for m in mp_of[j][mp_of[j] >= 0]:
        wt += snap["okp"][m] >= 0
    wt[j] = 0
    order = np.argsort(-wt)
    res["weights_kf0"] = [(int(s), int(wt[s]), int(nm.slot_pos[s])) for s in order]
    print("pos j", int(nm.slot_pos[j]), "weights (slot, w, pos):", res["weights_kf0"][:40], flush=True)
    print("n >= 15:", int((wt >= 15).sum()), "n > 0:", int((wt > 0).sum()), "sizes:", leg.rl.sizes.tolist()[:4], flush=True)
    if a.check:
        from oracle import oracle_py

        w = leg.first_valid()
        prob = leg.window_inputs(w)
        rg = leg.window_result(w)
        t0 = time.perf_counter()
        ro = oracle_py.lba_solve(prob)
        res["oracle_ms"] = (time.perf_counter() - t0) * 1e3
        res["same_control_flow"] = (ro.iterations, ro.lm_trials) == (rg.iterations, rg.lm_trials)
        res["rel"] = float(np.abs(ro.point_xyz - rg.point_xyz).max() / np.abs(ro.point_xyz).max())
        print(json.dumps({k: v for k, v in res.items() if k != "rows"}), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)
    if a.dump:
        z = {}
        for i, w in enumerate(leg.rl.valid):
            p = leg.window_inputs(w)
            for f in ("pose_fixed", "pose_q", "pose_t", "point_xyz", "edge_point", "edge_pose", "edge_obs",
                      "edge_inv_sigma2", "cams"):
                z[f"w{i}_{f}"] = getattr(p, f)
            z[f"w{i}_meta"] = np.array([p.huber_delta, p.iterations, p.cam_model], np.float64)
        np.savez_compressed(a.dump, **z)


if __name__ == "__main__":
    main()
