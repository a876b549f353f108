#!/usr/bin/env python3
"""KeyFrame::ComputeBoW (DBoW2 transform, levelsup 4) on the GPU vs the oracle on one host core, with a synthetic
ORB-SLAM3-sized vocabulary (k = 10, L = 6: ~10^6 words; the real ORBvoc.txt is a missing blob).

    python scripts/bow_bench.py [--config c1|c2] [--keyframes 64] [--reps 20] [--oracle]

Prints one JSON line: ms per batched launch (all keyframes) and per single-keyframe launch (HIP events on the
launch stream), and with --oracle the oracle's ms per keyframe (tree build excluded) and the parity of every output.
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


def run(config="c2", keyframes=64, reps=20, oracle=False, device=0, L=6) -> dict:
    import torch

    from mam3slam_amd import ORBextractor, bow, synth

    W, H, NF = (640, 480, 1000) if config == "c1" else (1280, 720, 2000)
    ext = ORBextractor(NF, 1.2, 8, 20, 7, device=device)
    descs = [ext(synth.make_frame(W, H, agent=4, frame=i))[1] for i in range(4)]
    t0 = time.perf_counter()
    v = bow.synthetic_vocabulary(10, L, np.random.default_rng(0), early_leaf=0.02)
    t_voc = time.perf_counter() - t0
    voc = bow.ORBVocabulary(v, device=device)
    B = keyframes
    S = max(len(d) for d in descs)
    D = np.zeros((B, S, 32), np.uint8)
    cnt = np.zeros((B, 2), np.int32)
    for f in range(B):
        d = descs[f % 4]
        D[f, :len(d)] = d
        cnt[f, 0] = len(d)
    dev = torch.device("cuda", device)
    t_d, t_c = torch.from_numpy(D).to(dev), torch.from_numpy(cnt).to(dev)
    t_w = torch.zeros((B, S), dtype=torch.int32, device=dev)
    t_x = torch.zeros((B, S), dtype=torch.float64, device=dev)
    t_n = torch.zeros((B, S), dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)

    def launch(nf):
        voc.transform_batch_device(nf, t_d.data_ptr(), S, t_c.data_ptr(), 4, t_w.data_ptr(), t_x.data_ptr(),
                                   t_n.data_ptr(), stream=st.cuda_stream)

    for _ in range(3):
        launch(B)
        launch(1)
    torch.cuda.synchronize(dev)
    ms = {}
    for name, nf in (("batch", B), ("one", 1)):
        voc.set_profiling(True)
        for _ in range(reps):
            launch(nf)
        torch.cuda.synchronize(dev)
        ms[name] = voc.stage_times()["transform"][0] / reps
    voc.set_profiling(False)
    out = {"config": config, "words": voc.size(), "nodes": v.n_nodes, "features_per_keyframe": float(cnt[:, 0].mean()),
           "keyframes_per_launch": B, "ms_per_batch_launch": ms["batch"], "keyframes_per_s": B / (ms["batch"] * 1e-3),
           "ms_single_keyframe_launch": ms["one"], "vocab_build_s": t_voc}
    if oracle:
        from oracle import oracle_py

        gw, gx, gn = t_w.cpu().numpy().view(np.uint32), t_x.cpu().numpy(), t_n.cpu().numpy().view(np.uint32)
        tree = oracle_py.BowTree(v)
        ok = 0
        nk = 4
        t1 = time.perf_counter()
        for f in range(nk):
            n = int(cnt[f, 0])
            (wo, xo, no), _, _ = oracle_py.bow_transform(v, D[f, :n], 4, tree)
            ok += int(np.array_equal(wo, gw[f, :n]) and np.array_equal(xo, gx[f, :n]) and np.array_equal(no, gn[f, :n]))
        t2 = time.perf_counter()
        out["oracle_ms_per_keyframe"] = (t2 - t1) * 1e3 / nk
        out["parity_keyframes"] = f"{ok}/{nk}"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2"])
    ap.add_argument("--keyframes", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run(a.config, a.keyframes, a.reps, a.oracle)), flush=True)


if __name__ == "__main__":
    main()
