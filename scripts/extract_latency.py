"""Single-frame ORBextractor latency (the north star's per-frame extraction): the host C-ABI call a Frame constructor
makes (mam_orb_extract: host image in, host keypoints / descriptors out, synchronous) and the device-resident batch
call at B = 1, per config. Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

  python scripts/extract_latency.py [--reps 300] [--configs c1,c3,c2]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = {"c1": (640, 480, 1000), "c3": (640, 480, 700), "c2": (1280, 720, 2000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--configs", default="c1,c3,c2")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from mam3slam_amd import ORBextractor, synth
    from mam3slam_amd._lib import lib

    out = {}
    for name in a.configs.split(","):
        W, H, NF = CFG[name]
        ext = ORBextractor(NF, 1.2, 8, 20, 7, device=0)
        img = np.ascontiguousarray(synth.make_frame(W, H, agent=0, frame=3))
        cap = ext.max_keypoints()
        kps = np.zeros(cap * 28, np.uint8)
        desc = np.zeros((cap, 32), np.uint8)
        n, mono = C.c_int(), C.c_int()
        L = lib()

        def raw():
            rc = L.mam_orb_extract(ext.ctx, img.ctypes.data, W, H, C.c_size_t(W), 0, 1000, kps.ctypes.data,
                                   desc.ctypes.data, cap, C.byref(n), C.byref(mono))
            assert rc == 0, rc

        for _ in range(20):
            raw()
            ext(img)
        t_raw, t_py = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            raw()
            t_raw.append((time.perf_counter() - t0) * 1e3)
            t0 = time.perf_counter()
            ext(img)
            t_py.append((time.perf_counter() - t0) * 1e3)
        # device-resident, B = 1, on a torch stream (no host copies)
        dev = torch.device("cuda", 0)
        d_img = torch.from_numpy(img).to(dev)
        d_kps = torch.zeros(cap * 28, dtype=torch.uint8, device=dev)
        d_desc = torch.zeros(cap * 32, dtype=torch.uint8, device=dev)
        d_cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)

        def dev_call():
            ext.extract_batch_device(d_img.data_ptr(), 1, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                     d_cnt.data_ptr(), stream=s.cuda_stream)

        for _ in range(20):
            dev_call()
        torch.cuda.synchronize()
        t_dev = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            dev_call()
            s.synchronize()
            t_dev.append((time.perf_counter() - t0) * 1e3)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            dev_call()
        torch.cuda.synchronize()
        t_g = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            t_g.append((time.perf_counter() - t0) * 1e3)
        med = lambda v: float(np.median(v))
        out[name] = {"host_api_raw_ms": med(t_raw), "host_api_python_ms": med(t_py), "device_b1_eager_ms": med(t_dev),
                     "device_b1_graph_ms": med(t_g), "keypoints": int(n.value),
                     "p90_host_api_raw_ms": float(np.percentile(t_raw, 90))}
        print(name, json.dumps(out[name]), flush=True)
        ext.close()
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
