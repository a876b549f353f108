"""Standalone timing of the batched SearchForTriangulation (mam_search_for_triangulation_batch_device): a ring of
keyframe slots (2000 features each, FeatureVectors from the synthetic frame's vocabulary nodes) and CreateNewMapPoints'
pairs (each of the newest W keyframes against 30 others), HIP events around each call; prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nkf", type=int, default=96)
    ap.add_argument("--new", type=int, default=32)
    ap.add_argument("--nn", type=int, default=30)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ori", type=int, default=1)
    args = ap.parse_args()
    import torch

    from mam3slam_amd import scene, synth
    from mam3slam_amd.match import FramesDev, ORBmatcher, TriBatch
    from oracle import oracle_py as O

    O.build()

    dev = torch.device("cuda", 0)
    w, h = 1280, 720
    img = synth.make_frame(w, h, agent=0, frame=0)
    k, d, _ = O.extract(img, O.params(2000))
    cam = scene.pinhole(w, h, 700.0)
    rng = np.random.default_rng(7)
    F = scene.make_frame_data(k, d, w, h)
    kfs = []
    while len(kfs) < args.nkf:
        a, b = scene.keyframe_pair_3d(F, cam, rng)
        kfs += [a, b]
    kfs = kfs[:args.nkf]
    S = max(len(x.keys) for x in kfs)
    nkf = len(kfs)
    keys = np.zeros((nkf, S), kfs[0].keys.dtype)
    desc = np.zeros((nkf, S, 32), np.uint8)
    cnt = np.zeros((nkf, 2), np.int32)
    has = np.zeros((nkf, S), np.uint8)
    nid = np.zeros((nkf, S), np.uint32)
    wt = np.zeros((nkf, S), np.float64)
    tcw = np.zeros(nkf, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
    for s_, KF in enumerate(kfs):
        n = len(KF.keys)
        keys[s_, :n], desc[s_, :n], cnt[s_, 0] = KF.keys, KF.desc, n
        has[s_, :n] = KF.has_mp
        for node, feats in KF.featvec.items():
            for i in feats:
                nid[s_, i] = node
                wt[s_, i] = 1.0
        tcw[s_]["q"], tcw[s_]["t"] = KF.pose
    pairs = []
    for i in range(args.new):
        others = [j for j in range(nkf) if j != i]
        for j in rng.choice(others, args.nn, replace=False):
            pairs.append((i, int(j)))
    pairs = np.array(pairs, np.int32)
    t = {n: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for n, v in
         dict(keys=keys.view(np.uint8), desc=desc, cnt=cnt, has=has, nid=nid, wt=wt, tcw=tcw.view(np.uint8),
              pairs=pairs).items()}
    out = torch.full((len(pairs), S), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
    b = TriBatch()
    b.kfs = FramesDev(nkf, S, t["keys"].data_ptr(), t["desc"].data_ptr(), t["cnt"].data_ptr(), None, None, 0)
    b.has_mp, b.nid, b.weight, b.tcw = t["has"].data_ptr(), t["nid"].data_ptr(), t["wt"].data_ptr(), t["tcw"].data_ptr()
    b.npairs, b.pairs = len(pairs), t["pairs"].data_ptr()
    M = ORBmatcher(0.6, bool(args.ori))
    ms = []
    st = torch.cuda.Stream(dev)   # a real stream handle (the default stream's is 0, which means the context's own)
    for r in range(args.reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        M.search_for_triangulation_batch_device(kfs[0], cam, b, out.data_ptr(), nm.data_ptr(), stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        if r >= 3:
            ms.append(e0.elapsed_time(e1))
    # parity on a sample of pairs
    og, ng = out.cpu().numpy(), nm.cpu().numpy()
    bad = 0
    for q in rng.choice(len(pairs), 8, replace=False):
        a1, a2 = pairs[q]
        no, oo = O.search_for_triangulation_kf(kfs[a1], kfs[a2], cam, cam, bool(args.ori), False)
        n1 = len(kfs[a1].keys)
        bad += int(not (ng[q] == no and np.array_equal(og[q, :n1], oo)))
    print(json.dumps({"npairs": len(pairs), "nkf": nkf, "features": S, "ms_median": float(np.median(ms)),
                      "ms_min": float(np.min(ms)), "matches_per_pair": float(ng.mean()), "parity_bad_pairs": bad}))


if __name__ == "__main__":
    main()
