"""Diagnostic: CreateNewMapPoints searches of a config's keyframe ring — per pair the frames' sequence distance, the
oracle's matches with the camera's epipolar test, without it (coarse) and with the frames' true poses."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from mam3slam_amd.mapping import NewMapPointsLeg  # noqa: E402
from oracle import oracle_py as oracle  # noqa: E402

cfg, B, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda", 0)
conf = dict(bench.CONFIGS[cfg])
tr = bench.TrackingLeg(conf, B, 1, 0, dev)
nm = NewMapPointsLeg(tr, W, dev)
nfr = tr.P * tr.B
slot_frame = {k: k % nfr for k in range(nm.R)}
K = max(1, tr.B // W)
steps = nm.R // nm.W + 4
for step in range(steps):
    tr.step()
    nm.ingest(step)
    head = nm.pending
    fr = (np.arange(W) * K + step % K) % tr.B + tr.p * tr.B
    for i in range(W):
        slot_frame[(head + i) % nm.R] = int(fr[i])
    nm.launch(nm.pending)
torch.cuda.synchronize()
nmatch = nm.nmatch.cpu().numpy()
pairs = nm.pairs[nm.head].cpu().numpy()
rows = []
for q in range(0, nm.npairs):
    K1, K2 = nm.pair_inputs(q)
    a, b = (slot_frame[int(x)] for x in pairs[q])
    n0, _ = oracle.search_for_triangulation_kf(K1, K2, tr.cam, tr.cam, False, False)
    nc, _ = oracle.search_for_triangulation_kf(K1, K2, tr.cam, tr.cam, False, True)
    K1.pose, K2.pose = tr.pool["poses"][a], tr.pool["poses"][b]
    nt, _ = oracle.search_for_triangulation_kf(K1, K2, tr.cam, tr.cam, False, False)
    free1 = int((K1.has_mp == 0).sum())
    rows.append((a, b, int(nmatch[q]), n0, nc, nt, free1, len(K1.keys)))
    print(f"pair {q:3d} frames {a:3d} {b:3d} d={a - b:4d} gpu {int(nmatch[q]):4d} oracle {n0:4d} coarse {nc:4d} "
          f"true-pose {nt:4d} free {free1}/{len(K1.keys)}")
r = np.array(rows)
print("mean gpu", r[:, 2].mean(), "coarse", r[:, 4].mean(), "true-pose", r[:, 5].mean())
