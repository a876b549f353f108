#!/usr/bin/env python3
"""bench.py — tracked frames/s of the MI355X ORB + local-BA hot path (BASELINE.json metric); one JSON line.

Step = one pass of the hot path over one batch of B synthetic frames resident in HBM, i.e. what Tracking does
per frame, batched:
  1. ORB extraction (pyramid, per-cell FAST, DistributeOctTree, orientation, rBRIEF, lapping placement)
  2. SearchByProjection(CurrentFrame, LastFrame, th=15)     (TrackWithMotionModel, Tracking.cc:2810)
  3. SearchByProjection(F, localMapPoints, th=1), nnratio 0.8 (SearchLocalPoints, Tracking.cc:3146-3156),
     with the keypoints matched in (2) taken
and for --config c2 additionally one LocalBundleAdjustment (50 KF / 3000 MP, BASELINE configs[2]) per step,
solved concurrently on its own HIP stream (the LocalMapping thread's work, Optimizer.cc:1116), followed by the
shared-map exchange: the LBA write-back packed into fixed-size records, all-gathered over RCCL, applied in agent
order.
N GPUs = N agents, one process per GPU, each with its own frame stream: independent units, weak scaling; the only
collective is that exchange (c2).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config c1|c2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE.json configs[1]: single-agent mono 640x480, 1000 features, 8 levels, extract + match
    "c1": dict(width=640, height=480, nfeatures=1000, lba=False),
    # BASELINE.json configs[2]: 1280x720, 2000 features + LocalBundleAdjustment (50 KF / 3000 MapPoints)
    "c2": dict(width=1280, height=720, nfeatures=2000, lba=True),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
# what actually limits each stage: the byte/integer path has no MFMA work and most stages issue far
# more VALU work per byte than the HBM roofline can see
ROOFLINE_NOTES = {
    "fast": "VALU issue: FAST-9 strength is ~85 packed-f16 min3/max3 ops per pixel pair (DESIGN.md §3)",
    "pyramid": "LDS-staged bilinear resize, latency-bound at 8 small launches",
    "describe": "one wave per keypoint: LDS-free gathers from the blurred level (latency)",
    "resolve": "one workgroup per frame, greedy dependency rounds (latency, LDS atomics)",
}
FP64_PEAK_TFS = 78.6    # MI355X FP64 vector (spec)


def level_sizes(w, h, nlevels=8, scale=1.2):
    s = [np.float32(1.0)]
    for _ in range(nlevels - 1):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    return [(int(np.rint(np.float32(w) * (np.float32(1.0) / x))), int(np.rint(np.float32(h) * (np.float32(1.0) / x))))
            for x in s]


def stage_bytes(w, h, n_kp, n_cand, n_last, n_mps, cand_motion, cand_local):
    """Algorithmic HBM bytes per frame for each kernel stage."""
    lv = level_sizes(w, h)
    P = sum(a * b for a, b in lv)
    P_ge1 = P - w * h
    P_le6 = P - lv[-1][0] * lv[-1][1]
    return {
        "pyramid": P_le6 + P_ge1,                  # read levels 0..6, write levels 1..7
        "fast": P + 4 * n_cand,                    # read every level once, write packed candidates
        "blur": 2 * P,                             # read + write every level
        "distribute": 4 * n_cand + 8 * n_kp,       # read candidates, write kept keypoints + ranks
        "describe": n_kp * (961 + 37 * 37 + 60),   # 31x31 moment disk + 37x37 blurred patch + 60 B out
        "grid": n_kp * (28 + 32 + 48),             # once per frame (the local search reuses it): keypoints +
                                                   # descriptors in, 48-B cell-ordered records out
        "gather": n_last * 64 + n_mps * 64 + (cand_motion + cand_local) * (2 + 28 + 32 + 4),
        "resolve": (cand_motion + cand_local) * 4 + (n_last + n_mps) * 8 + 2 * n_kp * 4,
    }


def cpu_baseline(cfg, seconds=10.0):
    """The oracle (single-thread C++ restatement of the reference path) on a bounded sample of the same
    step workload: extraction + motion search + local-map search per frame."""
    from mam3slam_amd import scene, synth
    from oracle import oracle_py

    p = oracle_py.params(cfg["nfeatures"])
    W, H = cfg["width"], cfg["height"]
    items = []
    for i in range(4):
        img = synth.make_frame(W, H, agent=0, frame=i)
        k, d, _ = oracle_py.extract(img, p)
        rng = np.random.default_rng(i)
        F = scene.make_frame_data(k, d, W, H)
        F.pose = scene.small_pose(rng)
        cam = scene.pinhole(W, H)
        items.append((img, scene.motion_last_frame(F, cam, rng), scene.local_mappoints(F, rng), F.pose, cam))
    n, t0 = 0, time.perf_counter()
    while True:
        img, last, mps, pose, cam = items[n % len(items)]
        k, d, _ = oracle_py.extract(img, p)
        F = scene.make_frame_data(k, d, W, H)
        F.pose = pose
        _, out = oracle_py.search_by_projection_motion(F, last, cam, 15.0, True)
        F.taken = (out >= 0).astype(np.uint8)
        oracle_py.search_by_projection(F, mps, 1.0, nnratio=0.8)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 5) or n >= 2000:
            break
    res = {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"{n} frames {W}x{H}/{cfg['nfeatures']}: extract + SearchByProjection(motion, th 15) + "
                     f"SearchByProjection(local map, th 1) on the oracle C++ restatement, single thread, {el:.1f}s"}
    if cfg["lba"]:
        from mam3slam_amd.lba import synthetic_problem

        prob = synthetic_problem(n_opt=50, n_fixed=10, n_points=3000, seed=1)
        t1 = time.perf_counter()
        r = oracle_py.lba_solve(prob)
        lba_ms = (time.perf_counter() - t1) * 1e3
        res["lba_ms"] = lba_ms
        res["sample"] += f"; LocalBundleAdjustment 50 KF/3000 MP ({len(prob.edge_point)} edges, {r.iterations} it) " \
                         f"{lba_ms:.1f} ms"
    return res


def pose_section(args, B, W, H, NF, cam, kps_h, cnt_h, d_out1, lasts, dev, stream):
    """Optimizer::PoseOptimization after the motion-model search (Tracking.cc:2836), measured beside the step (it is
    not part of the headline metric): every frame's edges are its motion-search matches (keypoint, last-frame
    MapPoint position), one workgroup per frame, B frames per launch; plus the single-frame launch and the oracle
    on one host core (same edges)."""
    import torch

    from mam3slam_amd import pose, scene
    from mam3slam_amd.orb import KP_DTYPE

    out1 = d_out1.cpu().numpy()
    sf, s2 = scene.scale_tables()
    inv_s2 = (np.float32(1.0) / s2).astype(np.float32)
    edges_l = []
    for f in range(B):
        n = int(cnt_h[f, 0])
        o = out1[f, :n]
        idx = np.nonzero(o >= 0)[0]
        edges_l.append(pose.make_edges(kps_h[f, :n].view(KP_DTYPE), inv_s2, idx, lasts[f]["pos"][o[idx]]))
    S = max(len(e) for e in edges_l)
    E = np.zeros((B, S), pose.POSE_EDGE_DTYPE)
    for f, e in enumerate(edges_l):
        E[f, :len(e)] = e
    P = pose.PoseOptimizer(device=dev.index or 0)
    t_e = torch.from_numpy(E.view(np.uint8).reshape(B, -1)).to(dev)
    t_n = torch.tensor([len(e) for e in edges_l], dtype=torch.int32, device=dev)
    tcw = np.zeros(B, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    rng = np.random.default_rng(7)
    for f in range(B):
        tcw[f]["q"], tcw[f]["t"] = scene.small_pose(rng)   # the motion model's guess around the frame's pose
    t_p = torch.from_numpy(tcw.view(np.uint8)).to(dev)
    t_o = torch.zeros((B, S), dtype=torch.uint8, device=dev)
    t_r = torch.zeros((B, pose.POSE_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)

    def run(nf):
        P.optimize_batch_device(nf, t_p.data_ptr(), cam, t_e.data_ptr(), S, t_n.data_ptr(), t_o.data_ptr(),
                                t_r.data_ptr(), stream=stream.cuda_stream)

    run(B)
    run(1)
    torch.cuda.synchronize(dev)
    reps = max(args.steps, 5)
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
    if not args.no_cpu_baseline and int(os.environ.get("RANK", "0")) == 0:
        from oracle import oracle_py

        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0 and n < B:
            oracle_py.pose_optimization_edges((tcw[n]["q"], tcw[n]["t"]), cam, edges_l[n])
            n += 1
        info["cpu_ms_per_frame"] = (time.perf_counter() - t0) * 1e3 / n
        info["cpu_sample"] = f"{n} frames, oracle C++ restatement, 1 thread"
    return info


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """`--gpus N` without a launcher: start N rank processes (one per GPU) under torch.distributed.run as CHILD
    processes of this one, which has not touched the GPU, and return their exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="frames per step per GPU (independent frame streams)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="c2 (1280x720/2000 + LocalBundleAdjustment) is BASELINE.json's headline metric config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-graph", action="store_true", help="launch the tracking step eagerly instead of a HIP graph")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the B=1 latency section (profiling runs: every launch then covers one lane's batch)")
    ap.add_argument("--no-pose", action="store_true", help="skip the PoseOptimization section")
    ap.add_argument("--no-sin", action="store_true",
                    help="skip the SearchInNeighbors section (Fuse + ComputeDistinctiveDescriptors)")
    ap.add_argument("--lanes", type=int, default=4,
                    help="independent sub-batches (agent groups) per GPU, each with its own contexts and HIP stream, "
                         "so one group's latency-bound stages overlap another's compute")
    ap.add_argument("--launch-check", action="store_true",
                    help="rendezvous + barrier over gloo on the CPU and exit (tests the --gpus N launcher, no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # before any HIP call: the ranks are children, never an exec of this process
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")

    import torch
    import torch.distributed as dist

    if args.launch_check:
        if world > 1:
            dist.init_process_group(backend="gloo")
            t = torch.tensor([rank], dtype=torch.int64)
            dist.all_reduce(t)
            dist.barrier()
            dist.destroy_process_group()
            if rank == 0:
                print(json.dumps({"launch_check": "ok", "world": world, "rank_sum": int(t.item())}), flush=True)
        else:
            print(json.dumps({"launch_check": "ok", "world": 1, "rank_sum": 0}), flush=True)
        return
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mam3slam_amd import ORBextractor, scene, synth
    from mam3slam_amd.match import LAST_ENTRY_DTYPE, MP_TRACK_DTYPE, FramesDev, ORBmatcher, Pose
    from mam3slam_amd.orb import KP_DTYPE

    cfg = CONFIGS[args.config]
    W, H, NF, B = cfg["width"], cfg["height"], cfg["nfeatures"], args.batch
    NL = max(1, args.lanes)
    if B % NL:
        raise SystemExit(f"--batch {B} is not a multiple of --lanes {NL}")
    BL = B // NL
    ext = ORBextractor(NF, 1.2, 8, 20, 7, device=local)
    cap = ext.max_keypoints()
    frames = np.stack([synth.make_frame(W, H, agent=rank, frame=i) for i in range(B)])
    d_img = torch.from_numpy(frames).to(dev)
    d_kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros((B, 2), dtype=torch.int32, device=dev)
    # one explicit stream orders extraction -> motion search -> local search (NULL would mean each library
    # context's own stream: unordered with each other)
    tstream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(tstream)
    stream = tstream.cuda_stream

    # lanes: frames [l * BL, (l + 1) * BL) run on lane l's stream with lane l's contexts
    lanes = []
    for l in range(NL):
        lanes.append({"lo": l * BL, "ext": ext if l == 0 else ORBextractor(NF, 1.2, 8, 20, 7, device=local),
                      "stream": tstream if l == 0 else torch.cuda.Stream(dev)})

    def extract_lane(ln):
        lo = ln["lo"]
        ln["ext"].extract_batch_device(d_img[lo].data_ptr(), BL, W, H, W, W * H, d_kps[lo].data_ptr(),
                                       d_desc[lo].data_ptr(), cap, d_cnt[lo].data_ptr(), stream=ln["stream"].cuda_stream)

    def extract():
        for ln in lanes:
            extract_lane(ln)

    def fork():
        for ln in lanes[1:]:
            ln["stream"].wait_stream(tstream)

    def join():
        for ln in lanes[1:]:
            tstream.wait_stream(ln["stream"])

    # ---- per-frame map structures around the frame's own features (built once; resident in HBM)
    fork()
    extract()
    join()
    torch.cuda.synchronize(dev)
    kps_h = d_kps.cpu().numpy().view(KP_DTYPE).reshape(B, cap)
    desc_h = d_desc.cpu().numpy()
    cnt_h = d_cnt.cpu().numpy()
    cam = scene.pinhole(W, H)
    lasts, mpss, poses = [], [], []
    F0 = None
    for f in range(B):
        rng = np.random.default_rng(1000 * rank + f)
        F = scene.make_frame_data(kps_h[f, :cnt_h[f, 0]], desc_h[f, :cnt_h[f, 0]], W, H)
        F.pose = scene.small_pose(rng)
        F0 = F0 or F
        lasts.append(scene.motion_last_frame(F, cam, rng))
        mpss.append(scene.local_mappoints(F, rng))
        poses.append(F.pose)
    Ls, Ms = max(len(x) for x in lasts), max(len(x) for x in mpss)
    last = np.zeros((B, Ls), LAST_ENTRY_DTYPE)
    mps = np.zeros((B, Ms), MP_TRACK_DTYPE)
    tcw = np.zeros(B, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for f in range(B):
        last[f, :len(lasts[f])] = lasts[f]
        mps[f, :len(mpss[f])] = mpss[f]
        tcw[f]["q"], tcw[f]["t"] = poses[f]
    d_last = torch.from_numpy(last.view(np.uint8).reshape(B, -1).copy()).to(dev)
    d_mps = torch.from_numpy(mps.view(np.uint8).reshape(B, -1).copy()).to(dev)
    d_tcw = torch.from_numpy(tcw.view(np.uint8).copy()).to(dev)
    d_nlast = torch.tensor([len(x) for x in lasts], dtype=torch.int32, device=dev)
    d_nmps = torch.tensor([len(x) for x in mpss], dtype=torch.int32, device=dev)
    d_out1 = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    d_out2 = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    d_nm1 = torch.zeros(B, dtype=torch.int32, device=dev)
    d_nm2 = torch.zeros(B, dtype=torch.int32, device=dev)
    d_taken = torch.zeros((B, cap), dtype=torch.uint8, device=dev)
    tcw_bytes = tcw.dtype.itemsize
    for ln in lanes:
        lo = ln["lo"]
        ln["mm"] = ORBmatcher(0.9, True, device=local)
        # the local-map search shares the motion search's context and reuses the frames' cell grid it built
        # (AssignFeaturesToGrid runs once per Frame in the reference)
        ln["ml"] = ORBmatcher(0.8, True, device=local, share=ln["mm"])
        # the motion search leaves the frame's slot state in d_taken (taken_out): the local search's `taken` input
        ln["fr1"] = FramesDev(BL, cap, d_kps[lo].data_ptr(), d_desc[lo].data_ptr(), d_cnt[lo].data_ptr(), None,
                              d_taken[lo].data_ptr())
        ln["fr2"] = FramesDev(BL, cap, d_kps[lo].data_ptr(), d_desc[lo].data_ptr(), d_cnt[lo].data_ptr(),
                              d_taken[lo].data_ptr(), None, 1)
    m_motion, m_local = lanes[0]["mm"], lanes[0]["ml"]

    def match_lane(ln):
        lo, st = ln["lo"], ln["stream"]
        ln["mm"].search_motion_batch_device(F0, ln["fr1"], d_tcw.data_ptr() + lo * tcw_bytes, cam,
                                            d_last[lo].data_ptr(), Ls, d_nlast[lo:].data_ptr(), 15.0,
                                            d_out1[lo].data_ptr(), d_nm1[lo:].data_ptr(), stream=st.cuda_stream)
        ln["ml"].search_by_projection_batch_device(F0, ln["fr2"], d_mps[lo].data_ptr(), Ms, d_nmps[lo:].data_ptr(),
                                                   1.0, d_out2[lo].data_ptr(), d_nm2[lo:].data_ptr(),
                                                   stream=st.cuda_stream)

    def match():
        for ln in lanes:
            match_lane(ln)

    def track_launch():
        fork()
        extract()
        match()
        join()

    lba_solver, lba_prob = None, None
    if cfg["lba"]:
        from mam3slam_amd.lba import LBASolver, synthetic_problem

        from mam3slam_amd.exchange import MapUpdateExchange

        lba_solver = LBASolver(device=local)
        lba_prob = synthetic_problem(n_opt=50, n_fixed=10, n_points=3000, seed=1 + rank)
        # shared-map exchange after every LBA: the agents' windows overlap in id space (a merged
        # map), so replicas see conflicting writes resolved in agent order
        exch = MapUpdateExchange(capacity=4096, device=dev)
        d_pose_id = torch.from_numpy(lba_prob.pose_id).to(dev)
        d_pose_fixed = torch.from_numpy(lba_prob.pose_fixed).to(dev)
        d_point_id = torch.from_numpy(lba_prob.point_id - (int(lba_prob.pose_id.max()) + 1)).to(dev)
        kf_cap, mp_cap = 1024, 1 << 16
        d_kf_table = torch.zeros((kf_cap, 8), dtype=torch.float32, device=dev)
        d_mp_table = torch.zeros((mp_cap, 4), dtype=torch.float32, device=dev)
        d_xstatus = torch.zeros(1, dtype=torch.int32, device=dev)

    lba_stats = {"n": 0, "ms": 0.0, "its": 0, "res": None}

    def lba_worker():
        t = time.perf_counter()
        r = lba_solver.solve(lba_prob)
        lba_stats["ms"] += (time.perf_counter() - t) * 1e3
        lba_stats["n"] += 1
        lba_stats["its"] = r.iterations
        lba_stats["res"] = r

    def exchange_updates():
        r = lba_stats["res"]
        bad = None   # bad flags come from the host-side erase (nObs <= 2); the synthetic window tracks no counts
        d_q = torch.from_numpy(r.pose_q).to(dev)
        d_t = torch.from_numpy(r.pose_t).to(dev)
        d_x = torch.from_numpy(r.point_xyz).to(dev)
        exch.pack_lba(d_q.data_ptr(), d_t.data_ptr(), d_pose_id.data_ptr(), d_pose_fixed.data_ptr(), len(r.pose_q),
                      d_x.data_ptr(), d_point_id.data_ptr(), bad, len(r.point_xyz), stream=stream)
        exch.gather()
        exch.apply(d_kf_table.data_ptr(), kf_cap, d_mp_table.data_ptr(), mp_cap, d_xstatus.data_ptr(), stream=stream)

    graph = None

    def track():
        if graph is not None:
            graph.replay()
        else:
            track_launch()

    def step():
        th = None
        if lba_solver is not None:
            th = threading.Thread(target=lba_worker)
            th.start()
        track()
        if th is not None:
            th.join()
            exchange_updates()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if not args.no_graph:
        # the tracking step (~30 launches) replayed as one HIP graph: no per-launch host gaps
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=tstream):
            track_launch()
        torch.cuda.synchronize(dev)
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
    cnt = d_cnt.cpu().numpy()
    n_kp = float(cnt[:, 0].mean())
    nf_probe = min(B, 4)
    n_cand = float(sum(len(ext.debug_candidates(l, f)) for l in range(8) for f in range(nf_probe))) / nf_probe
    nm1, nm2 = d_nm1.cpu().numpy(), d_nm2.cpu().numpy()
    if (nm1 < 0).any() or (nm2 < 0).any() or (cnt[:, 0] < 0).any():
        raise RuntimeError(f"device error codes in outputs: {nm1.min()} {nm2.min()} {cnt[:, 0].min()}")

    lba_stats.update(n=0, ms=0.0)
    if lba_solver is not None:
        lba_solver.set_profiling(True)
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
    # per-stage kernel times (HIP events around every launch, on the stream it runs on) from the same number of
    # eager tracking steps after the timed region: events cannot sit inside the replayed graph
    # The lanes run one after another here (synchronised in between), so every launch is timed standalone, as
    # in a --lanes 1 rocprofv3 kernel trace; stage_ms_per_step sums the lanes (work per step, not wall time).
    objs = [o for ln in lanes for o in (ln["ext"], ln["mm"])]   # ml shares mm's context (and its stage timer)
    for o in objs:
        o.set_profiling(True)
    torch.cuda.synchronize(dev)
    for _ in range(args.steps):
        for ln in lanes:
            ln["stream"].wait_stream(tstream)
            extract_lane(ln)
            match_lane(ln)
            tstream.wait_stream(ln["stream"])
            torch.cuda.synchronize(dev)
    stages = {}
    for ln in lanes:
        for k, v in ln["ext"].stage_times().items():
            a = stages.get(k, (0.0, 0))
            stages[k] = (a[0] + v[0], a[1] + v[1])
        sm = ln["mm"].stage_times()   # both searches of the lane (one context)
        for k in ("grid", "gather", "resolve"):
            a = stages.get(k, (0.0, 0))
            stages[k] = (a[0] + sm[k][0], a[1] + sm[k][1])
    for o in objs:
        o.set_profiling(False)
    lba_stage = lba_solver.stage_times() if lba_solver is not None else None
    # single-frame latency (B = 1, one HIP graph, synchronised per frame): the per-frame view of the north-star target
    ext.set_profiling(False)
    m_motion.set_profiling(False)
    m_local.set_profiling(False)
    fr1_1 = FramesDev(1, cap, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(), None, d_taken.data_ptr())
    fr2_1 = FramesDev(1, cap, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(), d_taken.data_ptr(), None, 1)

    def one_frame_launch():
        ext.extract_batch_device(d_img.data_ptr(), 1, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                 d_cnt.data_ptr(), stream=stream)
        m_motion.search_motion_batch_device(F0, fr1_1, d_tcw.data_ptr(), cam, d_last.data_ptr(), Ls,
                                            d_nlast.data_ptr(), 15.0, d_out1.data_ptr(), d_nm1.data_ptr(),
                                            stream=stream)
        m_local.search_by_projection_batch_device(F0, fr2_1, d_mps.data_ptr(), Ms, d_nmps.data_ptr(), 1.0,
                                                  d_out2.data_ptr(), d_nm2.data_ptr(), stream=stream)

    def measure_latency():
        one_frame_launch()
        torch.cuda.synchronize(dev)
        g1 = None
        if not args.no_graph:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=tstream):
                one_frame_launch()
            torch.cuda.synchronize(dev)

        def one_frame():
            if g1 is not None:
                g1.replay()
            else:
                one_frame_launch()
            torch.cuda.synchronize(dev)

        for _ in range(5):
            one_frame()
        lat = []
        for _ in range(50):
            t1 = time.perf_counter()
            one_frame()
            lat.append((time.perf_counter() - t1) * 1e3)
        return float(np.median(lat))

    latency_ms = None if args.no_latency else measure_latency()
    pose_info = None if args.no_pose else pose_section(args, B, W, H, NF, cam, kps_h, cnt_h, d_out1, lasts, dev,
                                                       tstream)
    sin_info = None
    if not args.no_sin:
        # LocalMapping::SearchInNeighbors' Hamming work, measured beside the step like the pose
        # section: Fuse into 30 target keyframes + Fuse of 8000 candidates + ComputeDistinctiveDescriptors
        from scripts import fuse_bench

        sin_info = fuse_bench.run(args.config, reps=max(args.steps, 5), device=dev.index or 0,
                                  oracle=not args.no_cpu_baseline and rank == 0)
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    T = float(t.item())
    frames_total = world * B * args.steps

    # roofline of the dominant kernel stage: algorithmic bytes per launch / mean launch duration (HIP events
    # recorded around each launch on the stream it runs on)
    mean_last = float(np.mean([len(x) for x in lasts]))
    mean_mps = float(np.mean([len(x) for x in mpss]))
    sb = stage_bytes(W, H, n_kp, n_cand, mean_last, mean_mps, cand_motion=mean_last * 6.0, cand_local=mean_mps * 3.0)
    per_step_ms = {k: v[0] / args.steps for k, v in stages.items()}
    dom = max(stages, key=lambda k: stages[k][0])
    ms_tot, launches = stages[dom]
    avg_ms = ms_tot / max(launches, 1)
    launches_per_step = launches / args.steps
    bytes_per_launch = sb[dom] * B / launches_per_step
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get(dom)
        except Exception:
            traffic = None

    if rank == 0:
        workload = (f"{args.config}: mono {W}x{H}, {NF} features, 8 levels; step = {B} frames x (ORB extract + "
                    f"SearchByProjection motion th15 + SearchByProjection local map th1)")
        if cfg["lba"]:
            workload += " + 1 LocalBundleAdjustment 50KF/3000MP per step (concurrent stream)"
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
            "config": {"workload": workload, "frames_per_step_per_gpu": B, "width": W, "height": H,
                       "nfeatures": NF, "keypoints_per_frame": n_kp, "fast_candidates_per_frame": n_cand,
                       "last_frame_points": mean_last, "local_map_points": mean_mps,
                       "matches_motion_per_frame": float(nm1.mean()), "matches_local_per_frame": float(nm2.mean()),
                       "parallelism": f"agents{world} (one agent per GPU, independent)",
                       "lanes": NL,
                       "launch": "hip graph per tracking step" if graph is not None else "eager"},
            "stage_ms_per_step": per_step_ms,
            "latency_ms_per_frame_b1": latency_ms,
            "roofline": {"bound": "hbm", "kernel": dom, "limiter": ROOFLINE_NOTES.get(dom), "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": avg_ms},
        }
        if pose_info is not None:
            out["pose_optimization"] = pose_info
        if sin_info is not None:
            out["search_in_neighbors"] = sin_info
        if cfg["lba"]:
            out["lba"] = {"solves": lba_stats["n"], "ms_per_solve_wall": lba_stats["ms"] / max(lba_stats["n"], 1),
                          "iterations": lba_stats["its"], "edges": int(len(lba_prob.edge_point)),
                          "stage_ms_total": {k: v[0] for k, v in lba_stage.items()}}
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
            out["cpu_baseline"]["latency_ms_per_frame"] = 1e3 / out["cpu_baseline"]["value"]
            if latency_ms:
                out["speedup_latency_b1"] = out["cpu_baseline"]["latency_ms_per_frame"] / latency_ms
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
