#!/usr/bin/env python3
"""PoseOptimization on the GPU (one workgroup per frame) vs the oracle on one host core, c1 / c2 frame shapes.

    python scripts/pose_bench.py [--config c1|c2] [--batch 256] [--reps 20] [--oracle]

Prints one JSON line: ms per batch launch (HIP events on the launch stream), frames/s, single-frame latency,
LM iterations / trials per frame, and (--oracle) the oracle's ms per frame and the parity of the batch.
"""
from __future__ import annotations

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
    ap.add_argument("--config", default="c1", choices=["c1", "c2"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--no-single", action="store_true", help="batch launches only (counter passes: one shape)")
    args = ap.parse_args()
    import torch

    from mam3slam_amd import ORBextractor, pose, scene, synth

    W, H, NF = (640, 480, 1000) if args.config == "c1" else (1280, 720, 2000)
    ext = ORBextractor(NF, 1.2, 8, 20, 7)
    cam = scene.pinhole(W, H)
    B = args.batch
    kinds = []
    for i in range(4):
        k, d, _ = ext(synth.make_frame(W, H, agent=0, frame=i))
        kinds.append((k, d))
    edges_l, poses = [], []
    for f in range(B):
        k, d = kinds[f % 4]
        F = scene.make_frame_data(k, d, W, H)
        xyz, _ = scene.pose_problem(F, cam, np.random.default_rng(f))
        idx = np.nonzero(F.map_point >= 0)[0]
        edges_l.append(pose.make_edges(F.keys, 1.0 / F.level_sigma2, idx, xyz[F.map_point[idx]]))
        poses.append(F.pose)
    S = max(len(e) for e in edges_l)
    E = np.zeros((B, S), pose.POSE_EDGE_DTYPE)
    for f, e in enumerate(edges_l):
        E[f, :len(e)] = e
    tcw = np.zeros(B, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for f, (q, t) in enumerate(poses):
        tcw[f]["q"], tcw[f]["t"] = q, t
    dev = torch.device("cuda")
    t_e = torch.from_numpy(E.view(np.uint8).reshape(B, -1)).to(dev)
    t_n = torch.tensor([len(e) for e in edges_l], dtype=torch.int32, device=dev)
    t_p = torch.from_numpy(tcw.view(np.uint8)).to(dev)
    t_o = torch.zeros((B, S), dtype=torch.uint8, device=dev)
    t_r = torch.zeros((B, pose.POSE_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    P = pose.PoseOptimizer()
    st = torch.cuda.Stream()

    def run(nf):
        P.optimize_batch_device(nf, t_p.data_ptr(), cam, t_e.data_ptr(), S, t_n.data_ptr(), t_o.data_ptr(),
                                t_r.data_ptr(), stream=st.cuda_stream)

    for _ in range(3):
        run(B)
        if not args.no_single:
            run(1)
    torch.cuda.synchronize()
    P.set_profiling(True)
    for _ in range(args.reps):
        run(B)
    torch.cuda.synchronize()
    ms_b = P.stage_times()["pose"][0] / args.reps
    ms_1, lat = None, None
    if not args.no_single:
        P.set_profiling(True)
        for _ in range(args.reps):
            run(1)
        torch.cuda.synchronize()
        ms_1 = P.stage_times()["pose"][0] / args.reps
        P.set_profiling(False)
        lat = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            run(1)
            st.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
    res = t_r.cpu().numpy().view(pose.POSE_RESULT_DTYPE).reshape(B)
    out = {"config": args.config, "batch": B, "edges_per_frame": float(np.mean([len(e) for e in edges_l])),
           "ms_per_batch_launch": ms_b, "frames_per_s": B / (ms_b * 1e-3), "ms_b1_launch": ms_1,
           "ms_b1_wall": float(np.median(lat)) if lat else None, "iterations_per_frame": float(res["iterations"].mean()),
           "lm_trials_per_frame": float(res["lm_trials"].mean())}
    out["roofline"] = roofline(out["edges_per_frame"], out["iterations_per_frame"], out["lm_trials_per_frame"], B, ms_b)
    if args.oracle:
        from oracle import oracle_py

        # every frame of the batch: the outlier sets on their own, then the full contract
        n = B
        t0 = time.perf_counter()
        ok = same_sets = 0
        outs = t_o.cpu().numpy()
        for f in range(n):
            no, oo, (qo, to), _ = oracle_py.pose_optimization_edges(poses[f], cam, edges_l[f])
            sets = bool(np.array_equal(oo, outs[f, :len(edges_l[f])]))
            same_sets += int(sets)
            ok += int(sets and no == res[f]["n_inliers"] and
                      np.max(np.abs(res[f]["q"] - qo)) < 1e-4 and np.max(np.abs(res[f]["t"] - to)) < 1e-4)
        out["oracle_ms_per_frame"] = (time.perf_counter() - t0) * 1e3 / n
        out["parity_frames"] = f"{ok}/{n}"
        out["outlier_sets_equal"] = f"{same_sets}/{n}"
    print(json.dumps(out), flush=True)



# algorithmic FP64 flops per active edge (Pinhole; a division or square root counts as one flop):
#   linearisation pass (build_system): T.map(Xw) 33, projection 7, error 2, chi 5, Huber 4, Jacobian 4, J*SE3deriv 10,
#     robust weights 5, weighted rows 10, H (21 entries of two products) 60, b 20, chi sum 1  -> 161
#   trial pass (active_chi at the candidate pose): map 33, projection 7, error 2, chi 5, Huber 4, sum 1  -> 52
FLOP_BUILD_EDGE, FLOP_TRIAL_EDGE = 161, 52
FP64_VALU_PEAK_TFS = 78.6   # MI355X vector FP64 (MI355X_MICROARCH.md); PoseOptimization is VALU FP64, not MFMA
# the newest round's counter pass (scripts/gpu_pose_pmc.sh, copied by scripts/collect_profiles.py)
PMC_FILE = next((f"profiles/{r}/pose_pmc_c2.json" for r in ("r06", "r05", "r04")
                 if os.path.exists(os.path.join(ROOT, f"profiles/{r}/pose_pmc_c2.json"))), "profiles/r04/pose_pmc_c2.json")


def roofline(edges, iterations, trials, frames, ms_launch) -> dict:
    """FP64 VALU roofline of one k_pose_opt launch: algorithmic flops = frames x edges x (iterations x 161 + trials x
    52) (every edge counted active: the outlier rounds deactivate a few per cent, so an upper bound) / launch time,
    against the vector FP64 peak of the whole chip and of the CUs the launch occupies (one workgroup per frame)."""
    fl = frames * edges * (iterations * FLOP_BUILD_EDGE + trials * FLOP_TRIAL_EDGE)
    ach = fl / (ms_launch * 1e-3) / 1e12
    r = {"bound": "fp64_valu", "kernel": "k_pose_opt", "unit": "TFLOP/s", "achieved": ach, "peak": FP64_VALU_PEAK_TFS,
         "frac": ach / FP64_VALU_PEAK_TFS, "frac_of_cus_used": ach / (FP64_VALU_PEAK_TFS * min(frames, 256) / 256.0),
         "flop_per_launch": fl, "avg_launch_ms": ms_launch,
         "limiter": "latency: one workgroup (8 waves) per frame; per LM iteration a linearisation pass over the "
                    "edges + a 28-value block reduction, per trial the serial 6x6 LDL^T + SE3 exp on wave 0 and a "
                    "chi2 pass + reduction (scripts/gpu_pose_pmc.sh for the VALU counters)"}
    path = os.path.join(ROOT, PMC_FILE)
    if os.path.exists(path):
        try:
            pj = json.load(open(path))
            e = next((v for k, v in pj.items() if "k_pose_opt" in k), None)
            if e:
                r["pmc"] = {k: e[k] for k in ("valu_busy", "SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64",
                                              "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                              "SQ_INSTS_VALU_TRANS_F64", "us_mean") if k in e}
                r["pmc_file"] = PMC_FILE
                f64 = sum(e.get(f"SQ_INSTS_VALU_{c}_F64", 0.0) for c in ("ADD", "MUL", "FMA", "TRANS"))
                if f64 and e.get("us_mean"):
                    # wave-instructions x 4 cycles (wave64 on a 16-lane FP64 unit) over the chip's SIMD-cycles
                    r["pmc"]["fp64_pipe_busy"] = f64 * 4 / (1024 * e["us_mean"] * 1e-6 * 2.4e9)
                    r["pmc"]["valu_pipe_busy"] = e.get("SQ_INSTS_VALU", 0.0) * 4 / (1024 * e["us_mean"] * 1e-6 * 2.4e9)
        except Exception:
            pass
    return r


def section(tr, reps=20, oracle=True) -> dict:
    """Optimizer::PoseOptimization after the motion-model search (Tracking.cc:2836), measured beside bench.py's step
    (not part of the headline metric): every frame's edges are its motion-search matches (keypoint, last-frame
    MapPoint position), one workgroup per frame, B frames per launch; plus the single-frame launch and the oracle on
    one host core (same edges). `tr` is bench.py's TrackingLeg after a step."""
    import torch

    from mam3slam_amd import pose, scene
    from mam3slam_amd.orb import KP_DTYPE

    B, dev, cam = tr.B, tr.dev, tr.cam
    out1 = tr.d_out1.cpu().numpy()
    sf, s2 = scene.scale_tables()
    inv_s2 = (np.float32(1.0) / s2).astype(np.float32)
    edges_l = []
    for f in range(B):
        n = int(tr.cnt_h[f, 0])
        o = out1[f, :n]
        idx = np.nonzero(o >= 0)[0]
        edges_l.append(pose.make_edges(tr.kps_h[f, :n].view(KP_DTYPE), inv_s2, idx, tr.lasts[f]["pos"][o[idx]]))
    S = max(len(e) for e in edges_l)
    E = np.zeros((B, S), pose.POSE_EDGE_DTYPE)
    for f, e in enumerate(edges_l):
        E[f, :len(e)] = e
    P = pose.PoseOptimizer(device=dev.index or 0)
    t_e = torch.from_numpy(E.view(np.uint8).reshape(B, -1)).to(dev)
    t_n = torch.tensor([len(e) for e in edges_l], dtype=torch.int32, device=dev)
    tcw = np.zeros(B, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for f in range(B):
        # the motion model's guess the step itself starts from (TrackingLeg.poses_init: the frame's pose 0.3 deg / 2 cm
        # off). (Rounds 3-4 started this section from a small pose around the identity instead, far from the frames'
        # poses: 26 iterations / 45 LM trials a frame, not the step's workload.)
        tcw[f]["q"], tcw[f]["t"] = tr.poses_init[f]
    t_p = torch.from_numpy(tcw.view(np.uint8)).to(dev)
    t_o = torch.zeros((B, S), dtype=torch.uint8, device=dev)
    t_r = torch.zeros((B, pose.POSE_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    stream = tr.tstream.cuda_stream

    def run(nf):
        P.optimize_batch_device(nf, t_p.data_ptr(), cam, t_e.data_ptr(), S, t_n.data_ptr(), t_o.data_ptr(),
                                t_r.data_ptr(), stream=stream)

    run(B)
    run(1)
    torch.cuda.synchronize(dev)
    P.set_profiling(True)
    for _ in range(reps):
        run(B)
    torch.cuda.synchronize(dev)
    ms_b = P.stage_times()["pose"][0] / reps
    P.set_profiling(True)
    for _ in range(reps):
        run(1)
    torch.cuda.synchronize(dev)
    ms_1 = P.stage_times()["pose"][0] / reps
    P.set_profiling(False)
    res = t_r.cpu().numpy().view(pose.POSE_RESULT_DTYPE).reshape(B)
    info = {"frames_per_launch": B, "edges_per_frame": float(np.mean([len(e) for e in edges_l])),
            "ms_per_launch": ms_b, "frames_per_s": B / (ms_b * 1e-3), "ms_single_frame_launch": ms_1,
            "iterations_per_frame": float(res["iterations"].mean()),
            "lm_trials_per_frame": float(res["lm_trials"].mean()),
            "inliers_per_frame": float(res["n_inliers"].mean())}
    info["roofline"] = roofline(info["edges_per_frame"], info["iterations_per_frame"], info["lm_trials_per_frame"],
                                B, ms_b)
    if oracle:
        from oracle import oracle_py

        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0 and n < B:
            oracle_py.pose_optimization_edges((tcw[n]["q"], tcw[n]["t"]), cam, edges_l[n])
            n += 1
        info["cpu_ms_per_frame"] = (time.perf_counter() - t0) * 1e3 / n
        info["cpu_sample"] = f"{n} frames, oracle C++ restatement, 1 thread"
    return info


if __name__ == "__main__":
    main()
