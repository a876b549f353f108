"""Probe of the ring LocalMapping leg at a config's full batch: every phase synchronised and printed, each
assembled window validated on the host (vertex indices inside the problem, sizes inside the buffers) before the solve,
so a malformed window stops the probe instead of reaching the LBA kernels."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mam3slam_amd.mapping import NewMapPointsLeg, RingMappingLeg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--n-fixed", type=int, default=10)
ap.add_argument("--dump", default=None, help="write the first assembled windows (npz) and stop before solving")
a = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[a.config])
tr = bench.TrackingLeg(cfg, a.batch, 4, 0, dev)
W = max(1, a.batch // 8)
nm = NewMapPointsLeg(tr, W, dev)
leg = RingMappingLeg(nm, 0, 1, dev)
leg.rl.n_fixed = a.n_fixed
print("legs", "W", W, "R", nm.R, "S", nm.S, "sets", leg.nheads, flush=True)
prev = None
for step in range(a.steps):
    tr.step()
    torch.cuda.synchronize()
    if prev is not None:
        st = leg.rl.sets[prev // W]
        torch.cuda.synchronize()
        cnt = st["counts"].cpu().numpy()
        bad = []
        for w in range(W):
            P, L, E, nopt = (int(v) for v in cnt[w])
            if not (0 < P <= leg.rl.NV and 0 <= nopt <= P and 0 <= L <= nm.S and 0 <= E <= nm.S * leg.rl.NV):
                bad.append((w, "sizes", P, L, E, nopt))
                continue
            b = st["bufs"][w]
            ep, eo = b["edge_point"][:E].cpu().numpy(), b["edge_pose"][:E].cpu().numpy()
            if E and (ep.min() < 0 or ep.max() >= L or eo.min() < 0 or eo.max() >= P):
                bad.append((w, "edges", int(ep.min()), int(ep.max()), int(eo.min()), int(eo.max()), P, L))
            fx = b["pose_fixed"][:P].cpu().numpy()
            if not np.array_equal(fx, (np.arange(P) >= nopt).astype(np.uint8)):
                bad.append((w, "fixed"))
        print(f"step {step} head {prev}: sizes P {cnt[:, 0].min()}-{cnt[:, 0].max()} L {cnt[:, 1].min()}-{cnt[:, 1].max()}"
              f" E {cnt[:, 2].min()}-{cnt[:, 2].max()} opt {cnt[:, 3].min()}-{cnt[:, 3].max()} bad {bad[:4]}", flush=True)
        if bad:
            sys.exit(2)
        if a.dump:
            leg.rl.cur = prev // W
            arrs = {}
            for w in range(4):
                pr = leg.rl.window(w)
                for f in ("pose_fixed", "pose_q", "pose_t", "point_xyz", "edge_point", "edge_pose", "edge_obs",
                          "edge_inv_sigma2", "cams"):
                    arrs[f"w{w}_{f}"] = np.asarray(getattr(pr, f))
                arrs[f"w{w}_meta"] = np.array([pr.huber_delta, pr.iterations, pr.cam_model], np.float64)
            np.savez(a.dump, **arrs)
            print("dumped", a.dump, flush=True)
            sys.exit(0)
        t0 = time.perf_counter()
        try:
            leg.run(step, head=prev)
        except RuntimeError as e:
            import ctypes as C

            from mam3slam_amd._lib import lib

            L = lib()
            L.mam_last_error.restype = C.c_char_p
            print("FAILED", e, "last error:", L.mam_last_error(), flush=True)
            raise
        torch.cuda.synchronize()
        print(f"  solved {time.perf_counter() - t0:.4f} s stats {leg.stats[:3]} status {int(leg.status.item())}"
              f" records kf {leg.n_kf_upd} mp {leg.n_mp_upd}", flush=True)
    nm.ingest(step)
    nm.launch(nm.pending)
    prev = nm.take()
    torch.cuda.synchronize()
    print(f"step {step}: ingested + searched + assembled head {prev}", flush=True)
print("DONE")
