#!/usr/bin/env python3
"""bench.py — tracked frames/s of the MI355X ORB hot path (BASELINE.json metric), one JSON line on rank 0.

Step = one pass of the hot path over one batch of synthetic frames resident in HBM: ORB extraction of B
frames (pyramid -> FAST cells -> blur -> DistributeOctTree -> orientation + rBRIEF + lapping placement) and
the per-frame matching stage that follows it in Tracking (when built). N GPUs = N agents, one process per
GPU, each with its own frame stream (independent units: weak scaling, no data-path collective).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config c1|c2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE.json configs[1]: single-agent mono 640x480, 1000 features, 8 levels, extract + match
    "c1": dict(width=640, height=480, nfeatures=1000),
    # configs[2] frame geometry: 1280x720, 2000 features
    "c2": dict(width=1280, height=720, nfeatures=2000),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy


def level_sizes(w, h, nlevels=8, scale=1.2):
    s = [1.0]
    for _ in range(nlevels - 1):
        s.append(float(np.float32(np.float64(np.float32(s[-1])) * np.float64(np.float32(scale)))))
    return [(int(np.rint(np.float32(w) * (np.float32(1.0) / np.float32(x)))),
             int(np.rint(np.float32(h) * (np.float32(1.0) / np.float32(x))))) for x in s]


def stage_bytes(w, h, n_kp, n_cand):
    """Algorithmic HBM bytes per frame for each stage."""
    lv = level_sizes(w, h)
    P = sum(a * b for a, b in lv)
    P_ge1 = P - w * h
    P_le6 = P - lv[-1][0] * lv[-1][1]
    return {
        "pyramid": P_le6 + P_ge1,                 # read levels 0..6, write levels 1..7
        "fast": P + 4 * n_cand,                   # read every level once, write packed candidates
        "blur": 2 * P,                            # read + write every level
        "distribute": 4 * n_cand + 8 * n_kp,      # read candidates, write kept keypoints + ranks
        "describe": n_kp * (961 + 37 * 37 + 60),  # 31x31 moment patch + 37x37 blurred patch + 60 B out
    }


def cpu_baseline(cfg, seconds=10.0):
    """Oracle (single-thread C++ restatement of the reference path) on a bounded sample of the workload."""
    from mam3slam_amd import synth
    from oracle import oracle_py

    p = oracle_py.params(cfg["nfeatures"])
    frames = [synth.make_frame(cfg["width"], cfg["height"], agent=0, frame=i) for i in range(8)]
    oracle_py.extract(frames[0], p)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        oracle_py.extract(frames[n % len(frames)], p)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 10) or n >= 2000:
            break
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} frames {cfg['width']}x{cfg['height']}/{cfg['nfeatures']} ORB extract, oracle C++ "
                      f"restatement single-threaded, {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="frames per step per GPU")
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mam3slam_amd import ORBextractor, synth
    from mam3slam_amd.orb import KP_DTYPE

    cfg = CONFIGS[args.config]
    W, H, NF, B = cfg["width"], cfg["height"], cfg["nfeatures"], args.batch
    ext = ORBextractor(NF, 1.2, 8, 20, 7, device=local)
    cap = ext.max_keypoints()
    frames = np.stack([synth.make_frame(W, H, agent=rank, frame=i) for i in range(B)])
    d_img = torch.from_numpy(frames).to(dev)
    d_kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros((B, 2), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        ext.extract_batch_device(d_img.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                 d_cnt.data_ptr(), stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    cnt = d_cnt.cpu().numpy()
    n_kp = float(cnt[:, 0].mean())
    n_cand = float(sum(len(ext.debug_candidates(l, f)) for l in range(8) for f in range(min(B, 4)))) / min(B, 4)

    ext.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    stages = ext.stage_times()
    ext.set_profiling(False)
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    T = float(t.item())
    frames_total = world * B * args.steps

    # roofline of the dominant stage: algorithmic bytes per launch / average launch duration (HIP events)
    sb = stage_bytes(W, H, n_kp, n_cand)
    dom = max(stages, key=lambda k: stages[k][0])
    ms_tot, launches = stages[dom]
    avg_ms = ms_tot / max(launches, 1)
    bytes_per_launch = sb[dom] * B
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get(dom)
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": "tracked frames/sec (ORB extract+match+localBA) at 1/2/4/8 GPUs vs CPU ref",
            "value": frames_total / T,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": T / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: mono {W}x{H}, {NF} features, 8 levels, ORB extract "
                                   f"(match stage not yet in step)",
                       "frames_per_step_per_gpu": B, "width": W, "height": H, "nfeatures": NF,
                       "keypoints_per_frame": n_kp, "candidates_per_frame": n_cand,
                       "parallelism": f"agents{world} (one agent per GPU)"},
            "stages_ms_per_step": {k: v[0] / max(v[1], 1) for k, v in stages.items()},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_ms},
        }
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
