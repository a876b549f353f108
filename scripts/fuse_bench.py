#!/usr/bin/env python3
"""LocalMapping::SearchInNeighbors' Hamming work (LocalMapping.cc:830-939) on the GPU vs the oracle on one host core:

  forward   Fuse of the current keyframe's MapPoints into T target keyframes (one batched launch, :881-890)
  backward  Fuse of the targets' fuse candidates into the current keyframe (:896-918)
  update    ComputeDistinctiveDescriptors of the current keyframe's MapPoints (:923-935)

    python scripts/fuse_bench.py [--config c1|c2] [--targets 30] [--reps 20] [--oracle]

Prints one JSON line: ms per stage (HIP events on the launch stream, grid build included), the GPU total, and with
--oracle the oracle's ms for the same work and the parity of every output.
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


def run(config="c2", targets=30, candidates=8000, reps=20, oracle=False, device=0) -> dict:
    """One SearchInNeighbors workload (see the module docstring); returns the JSON object."""
    import torch

    from mam3slam_amd import ORBextractor, scene, synth
    from mam3slam_amd.match import FUSE_MP_DTYPE, FramesDev, FuseKF, ORBmatcher, fuse_kf
    from mam3slam_amd.orb import KP_DTYPE

    W, H, NF = (640, 480, 1000) if config == "c1" else (1280, 720, 2000)
    ext = ORBextractor(NF, 1.2, 8, 20, 7, device=device)
    cam = scene.pinhole(W, H)
    T = targets
    feats = [ext(synth.make_frame(W, H, agent=1, frame=i))[:2] for i in range(4)]
    cases = []
    for i in range(T + 1):   # T targets + the current keyframe (backward direction)
        k, d = feats[i % 4]
        rng = np.random.default_rng(i)
        KF = scene.make_frame_data(k, d, W, H)
        KF.pose = scene.small_pose(rng, rot=0.3, trans=0.5)
        cases.append((KF, scene.fuse_mappoints(KF, cam, rng)))
    cur, cur_mps = cases[T][0], scene.fuse_mappoints(cases[T][0], cam, np.random.default_rng(99), frac=1.0,
                                                     n_out=candidates // 10)
    cur_mps = np.resize(cur_mps, candidates)   # vpFuseCandidates: the targets' MapPoints, deduplicated
    dev = torch.device("cuda", device)

    def device_batch(items):
        B = len(items)
        S = max(len(c[0].keys) for c in items)
        U = max(len(c[1]) for c in items)
        keys = np.zeros((B, S), KP_DTYPE)
        desc = np.zeros((B, S, 32), np.uint8)
        cnt = np.zeros((B, 2), np.int32)
        mps = np.zeros((B, U), FUSE_MP_DTYPE)
        nm = np.zeros(B, np.int32)
        kfs = (FuseKF * B)()
        for b, (KF, m) in enumerate(items):
            keys[b, :len(KF.keys)] = KF.keys
            desc[b, :len(KF.keys)] = KF.desc
            cnt[b, 0] = len(KF.keys)
            mps[b, :len(m)] = m
            nm[b] = len(m)
            kfs[b] = fuse_kf(KF.pose)
        t = dict(keys=torch.from_numpy(keys.view(np.uint8).reshape(B, -1)).to(dev),
                 desc=torch.from_numpy(desc).to(dev), cnt=torch.from_numpy(cnt).to(dev),
                 mps=torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).to(dev), nm=torch.from_numpy(nm).to(dev),
                 kfs=torch.from_numpy(np.frombuffer(kfs, np.uint8).copy()).to(dev),
                 idx=torch.zeros((B, U), dtype=torch.int32, device=dev),
                 dist=torch.zeros((B, U), dtype=torch.int32, device=dev),
                 n=torch.zeros(B, dtype=torch.int32, device=dev))
        t["fr"] = FramesDev(B, S, t["keys"].data_ptr(), t["desc"].data_ptr(), t["cnt"].data_ptr(), None, None, 0)
        t["U"] = U
        return t

    fwd = device_batch(cases[:T])
    bwd = device_batch([(cur, cur_mps)])
    # update: the current keyframe's MapPoints with 2..30 observations each
    rng = np.random.default_rng(7)
    n_upd = len(cur.keys)
    sizes = rng.integers(2, 31, n_upd)
    off = np.zeros(n_upd + 1, np.int32)
    off[1:] = np.cumsum(sizes)
    descs = scene.flip_bits(np.repeat(cur.desc[np.arange(n_upd)], sizes, 0), rng, 40)
    t_off = torch.from_numpy(off).to(dev)
    t_desc = torch.from_numpy(descs).to(dev)
    t_best = torch.zeros(n_upd, dtype=torch.int32, device=dev)
    M = ORBmatcher(device=device)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)

    def fuse(t):
        M.fuse_batch_device(cur, t["fr"], t["kfs"].data_ptr(), cam, t["mps"].data_ptr(), t["U"], t["nm"].data_ptr(),
                            3.0, t["idx"].data_ptr(), t["dist"].data_ptr(), t["n"].data_ptr(), stream=st.cuda_stream)

    def update():
        M.distinctive_batch_device(n_upd, t_off.data_ptr(), t_desc.data_ptr(), t_best.data_ptr(), stream=st.cuda_stream)

    for _ in range(3):
        fuse(fwd)
        fuse(bwd)
        update()
    torch.cuda.synchronize(dev)
    ms = {}
    for name, fn in (("forward", lambda: fuse(fwd)), ("backward", lambda: fuse(bwd)), ("update", update)):
        M.set_profiling(True)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        stt = M.stage_times()
        ms[name] = sum(v[0] for v in stt.values()) / reps
    M.set_profiling(False)
    t0 = time.perf_counter()
    for _ in range(reps):
        fuse(fwd)
        fuse(bwd)
        update()
        st.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / reps
    out = {"config": config, "targets": T, "mps_per_target": float(np.mean([len(c[1]) for c in cases[:T]])),
           "candidates": len(cur_mps), "update_mps": n_upd, "update_obs_per_mp": float(sizes.mean()),
           "ms_forward": ms["forward"], "ms_backward": ms["backward"], "ms_update": ms["update"],
           "ms_total_kernels": ms["forward"] + ms["backward"] + ms["update"], "ms_total_wall": wall}
    if oracle:
        from oracle import oracle_py

        gi, gd, gn = fwd["idx"].cpu().numpy(), fwd["dist"].cpu().numpy(), fwd["n"].cpu().numpy()
        ok = 0
        t0 = time.perf_counter()
        for b, (KF, m) in enumerate(cases[:T]):
            n, i, d = oracle_py.fuse(KF, m, cam, 3.0)
            ok += int(n == gn[b] and np.array_equal(i, gi[b, :len(m)]) and np.array_equal(d, gd[b, :len(m)]))
        t1 = time.perf_counter()
        n, i, d = oracle_py.fuse(cur, cur_mps, cam, 3.0)
        t2 = time.perf_counter()
        bi, bd, bn = bwd["idx"].cpu().numpy()[0], bwd["dist"].cpu().numpy()[0], int(bwd["n"].cpu().numpy()[0])
        ok_b = n == bn and np.array_equal(i, bi[:len(cur_mps)]) and np.array_equal(d, bd[:len(cur_mps)])
        best = oracle_py.distinctive_descriptors(off, descs)
        t3 = time.perf_counter()
        ok_u = np.array_equal(best, t_best.cpu().numpy())
        out.update({"oracle_ms_forward": (t1 - t0) * 1e3, "oracle_ms_backward": (t2 - t1) * 1e3,
                    "oracle_ms_update": (t3 - t2) * 1e3, "oracle_ms_total": (t3 - t0) * 1e3,
                    "parity": {"forward_keyframes": f"{ok}/{T}", "backward": bool(ok_b), "update": bool(ok_u)}})
        out["speedup_wall"] = out["oracle_ms_total"] / wall
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2"])
    ap.add_argument("--targets", type=int, default=30)   # nn = 30 for monocular agents (LocalMapping.cc:833-835)
    ap.add_argument("--candidates", type=int, default=8000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run(a.config, a.targets, a.candidates, a.reps, a.oracle)), flush=True)


if __name__ == "__main__":
    main()
