#!/usr/bin/env python3
"""Per-stage GPU time of the extractor on one standalone 64-frame launch (the bench's stage-pass shape), for
library variants (MAM3SLAM_GPU_LIB):  python scripts/fast_stage.py [--config c1|c2] [--batch 64] [--reps 10]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from mam3slam_amd import ORBextractor, synth

    W, H, NF = (640, 480, 1000) if a.config == "c1" else (1280, 720, 2000)
    dev = torch.device("cuda", 0)
    ext = ORBextractor(NF, 1.2, 8, 20, 7)
    cap = ext.max_keypoints()
    B = a.batch
    imgs = torch.from_numpy(np.stack([synth.make_frame(W, H, 0, i) for i in range(B)])).to(dev)
    kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros((B, 2), dtype=torch.int32, device=dev)
    run = lambda: ext.extract_batch_device(imgs.data_ptr(), B, W, H, W, W * H, kps.data_ptr(), desc.data_ptr(), cap,  # noqa: E731
                                           cnt.data_ptr())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ext.set_profiling(True)
    for _ in range(a.reps):
        run()
    torch.cuda.synchronize()
    st = ext.stage_times()
    ext.set_profiling(False)
    print(json.dumps({"config": a.config, "batch": B, "ms_per_launch": {k: v[0] / max(v[1], 1) for k, v in st.items()},
                      "keypoints_mean": float(cnt[:, 0].float().mean().item())}))


if __name__ == "__main__":
    main()
