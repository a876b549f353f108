#!/usr/bin/env python3
"""bench.py — tracked frames/s of the MI355X ORB + local-BA hot path (BASELINE.json metric); one JSON line.

A step is one pass of the hot path over B synthetic frames resident in HBM, one frame from each of B frame streams
(agent sequences) on this GPU, with the keyframe cadence of the reference's Tracking -> LocalMapping hand-off:

  Tracking, every frame, one HIP graph; frames start at the motion model's guess of the pose of
  the camera that rendered them (synth.frame_pose):
    1. ORB extraction (pyramid, per-cell FAST, DistributeOctTree, orientation, rBRIEF, lapping placement)
    2. TrackWithMotionModel (Tracking.cc:2786-2862): SearchByProjection(CurrentFrame, LastFrame, th=15),
       Optimizer::PoseOptimization, outliers' slots emptied
    3. TrackLocalMap (Tracking.cc:2878-2901): Frame::isInFrustum + MapPoint::PredictScale for every local MapPoint,
       SearchByProjection(F, localMapPoints, th=1) (nnratio 0.8, matched keypoints taken), PoseOptimization
  LocalMapping (c2), concurrently on its own streams: every stream inserts a keyframe every K frames (--kf-every), so
  B/K keyframes per step, each getting ComputeBoW and CreateNewMapPoints' 30 SearchForTriangulation against its
  covisible keyframes, then LocalBundleAdjustment (LocalMapping.cc:162-172) on its 50-keyframe window of a shared
  map in HBM (mam3slam_amd/mapping.py): window read from the map, the B/K solves batched with the Levenberg control
  on the device, the write-backs all-gathered over RCCL and applied to every GPU's map, which the next step's windows
  read.
N GPUs = N processes, each with its own B streams and B/K windows (weak scaling); the one collective is the map
exchange.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config c1|c2] [--kf-every K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

# One hardware queue per stream: the step uses 4 tracking lanes + the tracking / LocalMapping / triangulation / LBA
# group streams; with HIP's default of 4 queues, streams share queues and serialise behind each other
# (c2: 17.7-18.1k frames/s at 4 queues, 18.3k at 16). Set before the first HIP call (here and in spawned ranks).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE.json configs[1]: single-agent mono 640x480, 1000 features, 8 levels, extract + match
    "c1": dict(width=640, height=480, nfeatures=1000, lba=False),
    # BASELINE.json configs[2]: 1280x720, 2000 features + LocalBundleAdjustment (50 KF / ~3000 MapPoints windows)
    # path: 13 px of travel and 0.25 deg of roll per frame over a 4096-px wider scene — keyframes 8 frames apart are
    # 104 px apart, so a keyframe shares >= 15 MapPoints with the ~50 keyframes around it and fewer with the farther
    # ones (the covisibility graph LocalBundleAdjustment's window rule needs: local and fixed keyframes)
    "c2": dict(width=1280, height=720, nfeatures=2000, lba=True, path=(13.0, 0.25, 4096)),
    # BASELINE.json configs[3]: the testMultiAgentSystem agents (test/settingsForTest_00.yaml: KannalaBrandt8, 700
    # features) at 640x480, two agents in total (both on one GPU at --gpus 1, one per GPU at --gpus 2)
    # pool_frames: the two streams' keyframes over 16 steps are 32 distinct views (synth.frame_pose at the fisheye's
    # focal length: 0.53 deg of parallax per frame), so CreateNewMapPoints' neighbours beyond the nearest two pass
    # KannalaBrandt8's parallax test (cos < 0.9998, ~1.15 deg: KannalaBrandt8.cpp:316)
    # (path: 24 px / 0.25 deg per frame, as c2's: keyframes far enough apart that the ring holds covisible and fixed
    # ones)
    "c3": dict(width=640, height=480, nfeatures=700, lba=True, camera="kb8", agents=2, pool_frames=32, frame_stride=1,
               coherent_map=True, path=(24.0, 0.25, 1024)),
    # BASELINE.json configs[4]: 8 synthetic mono agents at 1280x720 / 2000 features, shared-map local BA, one agent
    # per GPU at --gpus 8 (all 8 on one GPU at --gpus 1); neighbouring agents' LBA windows overlap (keyframes and
    # MapPoints of the merged map), so the exchange resolves cross-GPU write conflicts in GPU order
    # (pool_frames: 9 sets of the 8 agents' frames — coprime with the keyframe cadence, so the keyframes the ring
    # holds are 72 different views: no identical keyframes in CreateNewMapPoints' neighbourhoods)
    "c4": dict(width=1280, height=720, nfeatures=2000, lba=True, agents=8, pool_frames=72, path=(40.0, 0.25, 2944)),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFS = 78.6    # MI355X FP64 vector / matrix (spec)
# what limits each stage; the byte/integer path has no MFMA work
# the limiter of a stage when no counter file of the config is present (with one, bench.py writes the limiter from
# that config's counters: profiles/traffic_<config>.json)
ROOFLINE_NOTES = {
    "fast": "latency / issue: per-cell workgroups over ~630 pixel pairs each (no PMC file for this config)",
    "pyramid": "bilinear resize, latency-bound at 7 dependent launches",
    "describe": "one wave per keypoint: IC-angle loads + the 37x37 blurred patch in LDS, two dependent round trips",
    "resolve": "one workgroup per frame, greedy dependency rounds (latency, LDS atomics)",
}


def level_sizes(w, h, nlevels=8, scale=1.2):
    s = [np.float32(1.0)]
    for _ in range(nlevels - 1):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    return [(int(np.rint(np.float32(w) * (np.float32(1.0) / x))), int(np.rint(np.float32(h) * (np.float32(1.0) / x))))
            for x in s]


LATENCY_STAGES = ("resolve",)


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
        "grid": n_kp * (28 + 32 + 48),             # keypoints + descriptors in, 48-B cell-ordered records out
        "gather": n_last * 64 + n_mps * 64 + (cand_motion + cand_local) * (2 + 28 + 32 + 4),
        "resolve": (cand_motion + cand_local) * 4 + (n_last + n_mps) * 8 + 2 * n_kp * 4,
        "frustum": n_mps * (80 + 64),              # mam_local_mp in, mam_mp_track out
    }


def lba_flops(E, L, Np, m_avg, trials, iterations):
    """Algorithmic FP64 flops of one LocalBundleAdjustment: per iteration E*420 (linearize + H
    blocks), per trial Schur sum_l m_l (m_l + 1) / 2 * 216 + L (60 + 144 m) + (6 Np)^3 / 3 + L (36 m + 18) + E * 60."""
    n = 6 * Np
    per_trial = L * m_avg * (m_avg + 1) / 2 * 216 + L * (60 + 144 * m_avg) + n ** 3 / 3 + L * (36 * m_avg + 18) + E * 60
    return iterations * E * 420 + trials * per_trial


def schur_flops(prob) -> float:
    """Algorithmic FP64 flops of one Schur complement of the window (block_solver.hpp:372-439's work): per landmark
    with m observations from optimised poses, the m (m + 1) / 2 pose-pair blocks W_i V^-1 W_j^T at 6 x 3 x 6 (216
    flops each)."""
    fixed = np.asarray(prob.pose_fixed).astype(bool)
    ep, eo = np.asarray(prob.edge_point), np.asarray(prob.edge_pose)
    m = np.bincount(ep[~fixed[eo]], minlength=1).astype(np.float64)
    return float((m * (m + 1) / 2).sum() * 216.0)


def ldlt_tile_flops(prob) -> float:
    """Algorithmic FP64 flops of one tile-skipping LDL^T factorization + solve of the window's reduced camera system
    (what k_ldlt_tiles must compute given the structure): S's 16x16 tiles that are non-zero (pose blocks sharing a
    landmark) plus the symbolic fill; per panel the diagonal tile's LDL^T and inverse (2 * 16^3 / 3 each), each panel
    tile L21 = A21 M (2 * 16^3), each trailing update L(r) D L(c)^T of two non-zero panel tiles (2 * 16^3, half for a
    diagonal tile), and the forward / backward solves (2 * 2 * 256 per non-zero tile)."""
    fixed = np.asarray(prob.pose_fixed).astype(bool)
    hp = -np.ones(len(fixed), int)
    hp[~fixed] = np.arange(int((~fixed).sum()))
    Np = int((~fixed).sum())
    nt = (6 * Np + 15) // 16
    if nt == 0:
        return 0.0
    T = np.eye(nt, dtype=bool)
    obs = {}
    for pt, po in zip(np.asarray(prob.edge_point), np.asarray(prob.edge_pose)):
        if hp[po] >= 0:
            obs.setdefault(int(pt), set()).add(int(hp[po]))
    blocks = set()
    for v in obs.values():
        v = sorted(v)
        for a in range(len(v)):
            for b in range(a, len(v)):
                blocks.add((v[b], v[a]))
    for i2, i1 in blocks:
        for r in range(6 * i2 // 16, (6 * i2 + 5) // 16 + 1):
            for c in range(6 * i1 // 16, (6 * i1 + 5) // 16 + 1):
                T[max(r, c), min(r, c)] = True
    tile = 2.0 * 16 ** 3
    fl = 0.0
    for c in range(nt):
        rows = [r for r in range(c + 1, nt) if T[r, c]]
        fl += 2 * tile / 3 + len(rows) * tile
        for a in rows:
            for b in rows:
                if b <= a:
                    T[a, b] = True
                    fl += tile / 2 if a == b else tile
    return fl + 4.0 * 256 * int(np.tril(T).sum())


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


# ------------------------------------------------------------------------------------------------------ tracking
class TrackingLeg:
    """B frames resident in HBM, split into lanes (sub-batches with their own contexts and HIP stream, captured
    together into one HIP graph) so one lane's latency-bound stages overlap another's compute."""

    def __init__(self, cfg, B, lanes, rank, dev, new_stream=None):
        import torch

        from mam3slam_amd import ORBextractor, scene, synth
        from mam3slam_amd.match import LAST_ENTRY_DTYPE, LOCAL_MP_DTYPE, MP_TRACK_DTYPE, FramesDev, ORBmatcher
        from mam3slam_amd.orb import KP_DTYPE

        self.dev, self.B, self.NL = dev, B, lanes
        W, H, NF = cfg["width"], cfg["height"], cfg["nfeatures"]
        self.W, self.H, self.NF = W, H, NF
        BL = B // lanes
        self.BL = BL
        di = dev.index or 0
        self.ext = ORBextractor(NF, 1.2, 8, 20, 7, device=di)
        cap = self.ext.max_keypoints()
        self.cap = cap
        cam = scene.kannala_brandt8(W, H) if cfg.get("camera") == "kb8" else scene.pinhole(W, H)
        self.cam = cam
        # a pool of P = ceil(pool_frames / B) frame sets: step s tracks set s mod P, so the keyframes a stream inserts over P
        # steps are different views (CreateNewMapPoints' neighbours then have parallax); set p, stream i renders frame
        # (p B + i) x frame_stride of the agent's sequence. P = 1: the same B frames every step.
        P, fs = max(1, -(-int(cfg.get("pool_frames", 1)) // B)), max(1, int(cfg.get("frame_stride", 1)))
        self.P, self.p = P, 0
        nfr = P * B
        fidx = [g * fs for g in range(nfr)]
        # frames rendered through the camera they are tracked with (the KannalaBrandt8 agents see the scene through the
        # fisheye: synth.make_frame_camera; the Pinhole frames are make_frame's crops, the same images)
        # (the fisheye's views at the canvas scale of its own focal length: the texture as dense in its image centre as
        # in a Pinhole frame of make_frame, not minified ~2.3x into a mass of FAST corners)
        fscene = float(cam.fx) if cam.is_kb8 else 500.0
        path = cfg.get("path")   # the camera path over the scene (synth.DEFAULT_MOTION unless the config sets one)
        if cam.is_kb8:
            frames = np.stack([synth.make_frame_camera(W, H, cam, agent=rank, frame=k, f=fscene, path=path)
                               for k in fidx])
        else:
            frames = np.stack([synth.make_frame(W, H, agent=rank, frame=k, path=path) for k in fidx])
        self.d_img_pool = torch.from_numpy(frames).to(dev)
        self.d_img = self.d_img_pool[:B].clone() if P > 1 else self.d_img_pool
        self.d_kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
        self.d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
        self.d_cnt = torch.zeros((B, 2), dtype=torch.int32, device=dev)
        # one explicit stream orders extraction -> motion search -> frustum -> local search
        # (new_stream: the streams' factory — CU-masked streams under --cu-split)
        new_stream = new_stream or (lambda: torch.cuda.Stream(dev))
        self.tstream = new_stream()
        self.lanes = []
        for l in range(lanes):
            self.lanes.append({"lo": l * BL, "ext": self.ext if l == 0 else ORBextractor(NF, 1.2, 8, 20, 7, device=di),
                               "stream": self.tstream if l == 0 else new_stream()})
        # every set's keypoints (the scene's MapPoints are placed on them)
        kps_l, desc_l, cnt_l = [], [], []
        for p in range(P):
            with torch.cuda.stream(self.tstream):
                if P > 1:
                    self.d_img.copy_(self.d_img_pool[p * B:(p + 1) * B])
                self._fork()
                self._extract()
                self._join()
            torch.cuda.synchronize(dev)
            kps_l.append(self.d_kps.clone())
            desc_l.append(self.d_desc.clone())
            cnt_l.append(self.d_cnt.clone())
        self.d_kps_pool, self.d_desc_pool, self.d_cnt_pool = torch.cat(kps_l), torch.cat(desc_l), torch.cat(cnt_l)
        if P > 1:
            self.d_img.copy_(self.d_img_pool[:B])
        kps_h = self.d_kps_pool.cpu().numpy().view(KP_DTYPE).reshape(nfr, cap)
        desc_h = self.d_desc_pool.cpu().numpy()
        cnt_h = self.d_cnt_pool.cpu().numpy()
        lasts, mpls, poses, poses_init = [], [], [], []
        F0 = None
        for f in range(nfr):
            rng = np.random.default_rng(1000 * rank + f)
            F = scene.make_frame_data(kps_h[f, :cnt_h[f, 0]], desc_h[f, :cnt_h[f, 0]], W, H)
            # the pose of the camera that rendered the frame (synth.frame_pose: the canvas as a plane in front of a
            # translating, rolling camera), so keyframes' poses and image content agree (SearchForTriangulation's
            # epipolar tests between keyframes pass for real correspondences, KannalaBrandt8 included)
            F.pose = synth.frame_pose(W, H, fidx[f], f=fscene, path=path)
            F0 = F0 or F
            # the last frame's and the local map's MapPoints re-project onto the frame's keypoints under that pose:
            # 45 % of the keypoints each (together ~70 % of the frame tracked, as ORB-SLAM's monocular tracking keeps
            # a few hundred map points per 1000 features; the rest is what CreateNewMapPoints triangulates)
            # (coherent_map: the MapPoints on the scene regions the map covers, the same in every view)
            cm = cfg.get("coherent_map", False)
            lasts.append(scene.motion_last_frame(F, cam, rng, frac=0.45,
                                                 sel=scene.coherent_selection(F, cam, 0.45, 1) if cm else None))
            mpls.append(scene.local_world_mappoints(F, cam, rng, frac=0.45,
                                                    sel=scene.coherent_selection(F, cam, 0.45, 2) if cm else None))
            poses.append(F.pose)
            # the motion model's guess mVelocity * LastFrame.GetPose() (Tracking.cc:2796): the true pose, 0.3 deg /
            # 2 cm off
            poses_init.append(scene.perturb_pose(F.pose, rng, rot=0.005, trans=0.02))
        self.F0 = F0
        # host copies of every set; frames / kps_h / cnt_h / desc_h / lasts / mpls / poses / poses_init: the set the
        # device buffers hold (the last step's)
        self.pool = dict(frames=frames, kps_h=kps_h, cnt_h=cnt_h, desc_h=desc_h, lasts=lasts, mpls=mpls, poses=poses,
                         poses_init=poses_init)
        self._set_views()
        Ls, Ms = max(len(x) for x in lasts), max(len(x) for x in mpls)
        self.Ls, self.Ms = Ls, Ms
        last = np.zeros((nfr, Ls), LAST_ENTRY_DTYPE)
        mpw = np.zeros((nfr, Ms), LOCAL_MP_DTYPE)
        tcw = np.zeros(nfr, dtype=np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,))]))
        for f in range(nfr):
            last[f, :len(lasts[f])] = lasts[f]
            mpw[f, :len(mpls[f])] = mpls[f]
            tcw[f]["q"], tcw[f]["t"] = poses_init[f]
        self.tcw_bytes = tcw.dtype.itemsize
        self.d_last_pool = torch.from_numpy(last.view(np.uint8).reshape(nfr, -1).copy()).to(dev)
        self.d_mpw_pool = torch.from_numpy(mpw.view(np.uint8).reshape(nfr, -1).copy()).to(dev)
        self.d_tcw_init_pool = torch.from_numpy(tcw.view(np.uint8).reshape(nfr, -1).copy()).to(dev)
        self.d_nlast_pool = torch.tensor([len(x) for x in lasts], dtype=torch.int32, device=dev)
        self.d_nmps_pool = torch.tensor([len(x) for x in mpls], dtype=torch.int32, device=dev)

        def work(t):   # the step's buffer: set 0's slice (advance copies the next set in), the pool itself when P = 1
            return t[:B].clone() if P > 1 else t

        self.d_last, self.d_mpw = work(self.d_last_pool), work(self.d_mpw_pool)
        self.d_mps = torch.zeros((B, Ms * MP_TRACK_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        # the motion model's guess (input of the step, never written) and the frame's pose as Tracking refines it
        self.d_tcw_init = work(self.d_tcw_init_pool).view(-1)
        self.d_tcw = self.d_tcw_init.clone()
        self.d_nlast, self.d_nmps = work(self.d_nlast_pool), work(self.d_nmps_pool)
        self.d_ntm = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_out1 = torch.zeros((B, cap), dtype=torch.int32, device=dev)
        self.d_out2 = torch.zeros((B, cap), dtype=torch.int32, device=dev)
        self.d_nm1 = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_nm2 = torch.zeros(B, dtype=torch.int32, device=dev)
        self.d_taken = torch.zeros((B, cap), dtype=torch.uint8, device=dev)
        # Optimizer::PoseOptimization after each search (Tracking.cc:2836, 2901): edges, their keypoints, outliers
        # and results of both calls
        from mam3slam_amd.pose import POSE_EDGE_DTYPE, POSE_RESULT_DTYPE, PoseOptimizer

        self.inv_s2 = (np.float32(1.0) / F0.level_sigma2).astype(np.float32)
        self.d_pe = torch.zeros((B, cap * POSE_EDGE_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.d_pk = torch.zeros((B, cap), dtype=torch.int32, device=dev)
        self.d_pout = torch.zeros((2, B, cap), dtype=torch.uint8, device=dev)
        self.d_pn = torch.zeros((2, B), dtype=torch.int32, device=dev)
        self.d_pres = torch.zeros((2, B, POSE_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        for ln in self.lanes:
            lo = ln["lo"]
            ln["mm"] = ORBmatcher(0.9, True, device=di)
            # the local-map search shares the motion search's context and reuses the cell grid it built
            ln["ml"] = ORBmatcher(0.8, True, device=di, share=ln["mm"])
            ln["fr1"] = FramesDev(BL, cap, self.d_kps[lo].data_ptr(), self.d_desc[lo].data_ptr(),
                                  self.d_cnt[lo].data_ptr(), None, self.d_taken[lo].data_ptr())
            ln["fr2"] = FramesDev(BL, cap, self.d_kps[lo].data_ptr(), self.d_desc[lo].data_ptr(),
                                  self.d_cnt[lo].data_ptr(), self.d_taken[lo].data_ptr(), None, 1)
            ln["po"] = PoseOptimizer(device=di)
            if ln["po"].max_edges() < cap:
                raise RuntimeError(f"PoseOptimization holds {ln['po'].max_edges()} edges per frame, frames have {cap}")
        self.graph = None

    def _set_views(self):
        B, p = self.B, self.p
        for k, v in self.pool.items():
            setattr(self, k, v[p * B:(p + 1) * B])

    def advance(self):
        """Move to the next frame set (P > 1): its images, last-frame and local-map MapPoints, motion-model guesses
        copied into the step's buffers on the tracking stream — the new frames of the step arriving."""
        import torch

        if self.P == 1:
            return
        self.p = (self.p + 1) % self.P
        with torch.cuda.stream(self.tstream):
            self._copy_set(self.p)
        self._set_views()

    def _copy_set(self, p):
        sl = slice(p * self.B, (p + 1) * self.B)
        for w, src in ((self.d_img, self.d_img_pool), (self.d_last, self.d_last_pool), (self.d_mpw, self.d_mpw_pool),
                       (self.d_tcw_init.view(self.B, -1), self.d_tcw_init_pool), (self.d_nlast, self.d_nlast_pool),
                       (self.d_nmps, self.d_nmps_pool)):
            w.copy_(src[sl])

    def _fork(self):
        for ln in self.lanes[1:]:
            ln["stream"].wait_stream(self.tstream)

    def _join(self):
        for ln in self.lanes[1:]:
            self.tstream.wait_stream(ln["stream"])

    def _extract_lane(self, ln):
        lo, BL, W, H = ln["lo"], self.BL, self.W, self.H
        ln["ext"].extract_batch_device(self.d_img[lo].data_ptr(), BL, W, H, W, W * H, self.d_kps[lo].data_ptr(),
                                       self.d_desc[lo].data_ptr(), self.cap, self.d_cnt[lo].data_ptr(),
                                       stream=ln["stream"].cuda_stream)

    def _extract(self):
        for ln in self.lanes:
            self._extract_lane(ln)

    def _pose_lane(self, ln, k, lo=None, nf=None, st=None):
        """Optimizer::PoseOptimization(&mCurrentFrame) of the lane's frames: call k = 0 after the motion search
        (TrackWithMotionModel, Tracking.cc:2836, then its outlier discard :2840-2857), k = 1 after the local-map search
        (TrackLocalMap, :2901); edges from the frames' slots (Optimizer.cc:856-895), the pose written back as
        Frame::SetPose does."""
        lo = ln["lo"] if lo is None else lo
        BL = self.BL if nf is None else nf
        st = ln["stream"].cuda_stream if st is None else st
        cap = self.cap
        po = ln["po"]
        tcw = self.d_tcw.data_ptr() + lo * self.tcw_bytes
        pe, pk = self.d_pe[lo].data_ptr(), self.d_pk[lo].data_ptr()
        pn, pout, pres = self.d_pn[k, lo:].data_ptr(), self.d_pout[k, lo].data_ptr(), self.d_pres[k, lo].data_ptr()
        po.frame_edges_batch_device(BL, self.d_kps[lo].data_ptr(), cap, self.d_cnt[lo].data_ptr(), 2, self.inv_s2,
                                    self.d_out1[lo].data_ptr(), self.d_last[lo].data_ptr(), self.Ls,
                                    self.d_out2[lo].data_ptr() if k == 1 else None,
                                    self.d_mpw[lo].data_ptr() if k == 1 else None, self.Ms, pe, cap, pn, pk, stream=st)
        po.optimize_batch_device(BL, tcw, self.cam, pe, cap, pn, pout, pres, stream=st)
        po.frame_update_batch_device(BL, pres, tcw, pout, pk, cap, pn, k == 0, self.d_out1[lo].data_ptr(),
                                     self.d_taken[lo].data_ptr(), cap, stream=st)

    def _match_lane(self, ln, lo=None, nf=None, st=None, fr1=None, fr2=None):
        """The lane's frames (or nf frames from lo, frame sets fr1 / fr2, stream st) after extraction."""
        lo = ln["lo"] if lo is None else lo
        BL = self.BL if nf is None else nf
        st = ln["stream"].cuda_stream if st is None else st
        fr1 = ln["fr1"] if fr1 is None else fr1
        fr2 = ln["fr2"] if fr2 is None else fr2
        tcw0 = self.d_tcw_init.data_ptr() + lo * self.tcw_bytes
        tcw = self.d_tcw.data_ptr() + lo * self.tcw_bytes
        # TrackWithMotionModel: the current frame at the motion model's guess, SearchByProjection(Cur, Last, th 15)
        # (again at th 30 for a frame with fewer than 20 matches), PoseOptimization, outliers discarded
        ln["mm"].track_motion_search_batch_device(self.F0, fr1, tcw0, self.cam, self.d_last[lo].data_ptr(), self.Ls,
                                                  self.d_nlast[lo:].data_ptr(), 15.0, self.d_out1[lo].data_ptr(),
                                                  self.d_nm1[lo:].data_ptr(), min_matches=20, stream=st)
        self._pose_lane(ln, 0, lo, BL, st)
        # TrackLocalMap: SearchLocalPoints (isInFrustum + SearchByProjection(F, localMPs, th 1)) at the optimised pose,
        # then PoseOptimization with every match
        ln["ml"].is_in_frustum_batch_device(self.F0, BL, tcw, self.cam, self.d_mpw[lo].data_ptr(), self.Ms,
                                            self.d_nmps[lo:].data_ptr(), self.d_mps[lo].data_ptr(),
                                            self.d_ntm[lo:].data_ptr(), stream=st)
        ln["ml"].search_by_projection_batch_device(self.F0, fr2, self.d_mps[lo].data_ptr(), self.Ms,
                                                   self.d_nmps[lo:].data_ptr(), 1.0, self.d_out2[lo].data_ptr(),
                                                   self.d_nm2[lo:].data_ptr(), stream=st)
        self._pose_lane(ln, 1, lo, BL, st)

    def launch(self):
        self.d_tcw.copy_(self.d_tcw_init)   # every step tracks its frames from the motion model's guess
        self._fork()
        self._extract()
        for ln in self.lanes:
            self._match_lane(ln)
        self._join()

    def capture(self):
        import torch

        if self.P == 1:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=self.tstream):
                self.launch()
            return
        # one graph per frame set: its frames' copy-in + the step
        self.graphs = []
        for p in range(self.P):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.tstream, pool=self.graphs[0].pool() if self.graphs else None):
                self._copy_set(p)
                self.launch()
            self.graphs.append(g)
        self.graph = self.graphs

    def step(self):
        import torch

        if self.graph is not None and self.P > 1:
            self.p = (self.p + 1) % self.P
            self._set_views()
            self.graphs[self.p].replay()
            return
        self.advance()
        if self.graph is not None:
            self.graph.replay()
        else:
            with torch.cuda.stream(self.tstream):
                self.launch()

    def stage_pass(self, steps):
        """Per-stage kernel time (HIP events on the launch stream) over `steps` eager steps with the lanes run one
        after another, so every launch is timed standalone (as in a --lanes 1 rocprofv3 kernel trace)."""
        import torch

        objs = [o for ln in self.lanes for o in (ln["ext"], ln["mm"], ln["po"])]
        for o in objs:
            o.set_profiling(True)
        torch.cuda.synchronize(self.dev)
        with torch.cuda.stream(self.tstream):
            for _ in range(steps):
                self.d_tcw.copy_(self.d_tcw_init)
                for ln in self.lanes:
                    ln["stream"].wait_stream(self.tstream)
                    self._extract_lane(ln)
                    self._match_lane(ln)
                    self.tstream.wait_stream(ln["stream"])
                    torch.cuda.synchronize(self.dev)
        stages = {}
        for ln in self.lanes:
            for k, v in ln["ext"].stage_times().items():
                a = stages.get(k, (0.0, 0))
                stages[k] = (a[0] + v[0], a[1] + v[1])
            sm = ln["mm"].stage_times()
            for k in ("grid", "gather", "resolve", "frustum"):
                a = stages.get(k, (0.0, 0))
                stages[k] = (a[0] + sm[k][0], a[1] + sm[k][1])
            sp = ln["po"].stage_times()["pose"]
            a = stages.get("pose", (0.0, 0))
            stages["pose"] = (a[0] + sp[0], a[1] + sp[1])
        for o in objs:
            o.set_profiling(False)
        return stages


# ------------------------------------------------------------------------------------------------------ sections
def latency_section(tr):
    """Single-frame latency: (a) one frame through the device-resident HIP graph (extract + motion search + frustum +
    local search); (b) ORBextractor::operator() through the host C-ABI (mam_orb_extract: host image in, host
    keypoints / descriptors out, synchronous), the drop-in path a Frame constructor calls."""
    import torch

    from mam3slam_amd.match import FramesDev

    dev, cap = tr.dev, tr.cap
    fr1 = FramesDev(1, cap, tr.d_kps.data_ptr(), tr.d_desc.data_ptr(), tr.d_cnt.data_ptr(), None,
                    tr.d_taken.data_ptr())
    fr2 = FramesDev(1, cap, tr.d_kps.data_ptr(), tr.d_desc.data_ptr(), tr.d_cnt.data_ptr(), tr.d_taken.data_ptr(),
                    None, 1)
    ln = tr.lanes[0]
    st = tr.tstream.cuda_stream

    def one_frame_launch():
        tr.d_tcw[:1].copy_(tr.d_tcw_init[:1])
        tr.ext.extract_batch_device(tr.d_img.data_ptr(), 1, tr.W, tr.H, tr.W, tr.W * tr.H, tr.d_kps.data_ptr(),
                                    tr.d_desc.data_ptr(), cap, tr.d_cnt.data_ptr(), stream=st)
        tr._match_lane(ln, 0, 1, st, fr1, fr2)

    with torch.cuda.stream(tr.tstream):
        one_frame_launch()
    torch.cuda.synchronize(dev)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=tr.tstream):
        one_frame_launch()
    torch.cuda.synchronize(dev)
    for _ in range(5):
        g1.replay()
        torch.cuda.synchronize(dev)
    lat = []
    for _ in range(50):
        t1 = time.perf_counter()
        g1.replay()
        torch.cuda.synchronize(dev)
        lat.append((time.perf_counter() - t1) * 1e3)
    # ORBextractor::operator() through the C-ABI as the C++ wrapper calls it (mam_orb_extract into the caller's
    # preallocated keypoint / descriptor buffers), and through the Python mirror (which allocates its outputs per call)
    import ctypes as C

    from mam3slam_amd._lib import lib

    img = np.ascontiguousarray(tr.frames[0])
    L = lib()
    cap = tr.ext.max_keypoints()
    kbuf, dbuf = np.zeros(cap * 28, np.uint8), np.zeros((cap, 32), np.uint8)
    n_o, m_o = C.c_int(), C.c_int()

    def raw():
        rc = L.mam_orb_extract(tr.ext.ctx, img.ctypes.data, tr.W, tr.H, C.c_size_t(tr.W), 0, 1000, kbuf.ctypes.data,
                               dbuf.ctypes.data, cap, C.byref(n_o), C.byref(m_o))
        assert rc == 0, rc

    for _ in range(5):
        raw()
        tr.ext(img)
    host, py = [], []
    for _ in range(50):
        t1 = time.perf_counter()
        raw()
        host.append((time.perf_counter() - t1) * 1e3)
        t1 = time.perf_counter()
        tr.ext(img)
        py.append((time.perf_counter() - t1) * 1e3)
    return {"device_graph_ms": float(np.median(lat)), "host_api_extract_ms": float(np.median(host)),
            "host_api_extract_ms_p90": float(np.percentile(host, 90)),
            "host_api_extract_python_ms": float(np.median(py)),
            "note": "host_api_extract_ms: mam_orb_extract (host frame in, host keypoints / descriptors out, "
                    "synchronous) into preallocated buffers, median of 50 after 5 warm calls; _python_ms: the same "
                    "through the Python ORBextractor mirror (output arrays allocated per call)"}


def ingest_section(tr, reps=5):
    """The PCIe legs the device-resident step leaves out: B frames host -> device from pinned memory, and the
    keypoints + descriptors + counts device -> host, each timed alone (events on the copy stream); DESIGN.md §6
    quotes the PCIe-inclusive rate."""
    import torch

    dev = tr.dev
    h_img = torch.from_numpy(tr.frames).pin_memory()
    h_kps = torch.empty(tuple(tr.d_kps.shape), dtype=torch.uint8).pin_memory()
    h_desc = torch.empty(tuple(tr.d_desc.shape), dtype=torch.uint8).pin_memory()
    h_cnt = torch.empty(tuple(tr.d_cnt.shape), dtype=torch.int32).pin_memory()
    s = torch.cuda.Stream(dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    h2d, d2h = [], []
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(s):
        for _ in range(reps):
            e[0].record(s)
            tr.d_img.copy_(h_img, non_blocking=True)
            e[1].record(s)
            h_kps.copy_(tr.d_kps, non_blocking=True)
            h_desc.copy_(tr.d_desc, non_blocking=True)
            h_cnt.copy_(tr.d_cnt, non_blocking=True)
            e[2].record(s)
            s.synchronize()
            h2d.append(e[0].elapsed_time(e[1]))
            d2h.append(e[1].elapsed_time(e[2]))
    bi = tr.frames.nbytes
    bo = tr.d_kps.numel() + tr.d_desc.numel() + 4 * tr.d_cnt.numel()
    m_in, m_out = float(np.median(h2d)), float(np.median(d2h))
    return {"h2d_ms_per_step": m_in, "d2h_ms_per_step": m_out, "h2d_bytes_per_step": int(bi),
            "d2h_bytes_per_step": int(bo), "h2d_GBs": bi / (m_in * 1e-3) / 1e9, "d2h_GBs": bo / (m_out * 1e-3) / 1e9}


def ring_lba_section(newmp, check=True):
    """LocalBundleAdjustment of the last LocalMapping run's keyframes (mapping.RingLBA over the device map): each new
    keyframe's window by the reference's rule — local = the keyframe + its covisible keyframes, local MapPoints = every
    MapPoint of every local keyframe, fixed = their other observers — assembled on the device and solved by the batch
    device API, standalone after the timed region (whose LocalMapping leg assembles and solves the same windows beside
    Tracking; no write-back here), assembly and solve (incl. its size read-back) timed apart; with check, the first
    solved window against the oracle on the same graph."""
    import torch

    from mam3slam_amd.mapping import RingLBA

    rl = RingLBA(newmp)
    torch.cuda.synchronize()
    for _ in range(3):   # warm (the solver context's arena, its trials-per-solve estimate for the read-back chunk)
        rl.assemble(newmp.stream)
        rl.solve(newmp.stream)
    torch.cuda.synchronize()
    reps, ms_asm, ms_solve = 5, 0.0, 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        rl.assemble(newmp.stream)
        newmp.stream.synchronize()
        t1 = time.perf_counter()
        rl.solve(newmp.stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ms_asm += (t1 - t0) * 1e3 / reps
        ms_solve += (t2 - t1) * 1e3 / reps
    ms = ms_asm + ms_solve
    v = rl.valid
    sz = rl.sizes[v] if v else np.zeros((1, 4))   # per solved window: poses, points, edges, optimised poses
    res = {"windows": newmp.W, "windows_solved": len(v), "rule": "covisibility (device map)",
           "covisibility_threshold": rl.COVIS_TH,
           "poses_mean": float(sz[:, 0].mean()), "optimised_poses_mean": float(sz[:, 3].mean()),
           "points_mean": float(sz[:, 1].mean()), "observations_mean": float(sz[:, 2].mean()),
           "ms_per_batch": ms, "ms_assemble": ms_asm, "ms_solve": ms_solve,
           "trials_all": [t for _, t, _ in rl.stats]}
    if check and v:
        from oracle import oracle_py

        w = v[0]
        prob = rl.window(w)
        _, _, _, its, trials, st, ic, fc = rl.result(w)
        ro = oracle_py.lba_solve(prob)
        q, t, x = rl.result(w)[:3]
        rel = float(np.abs(x - ro.point_xyz).max() / max(np.abs(ro.point_xyz).max(), 1e-12))
        res.update({"iterations": its, "trials": trials, "status": st, "chi2": [ic, fc]})
        res["oracle_same_control_flow"] = (its, trials) == (ro.iterations, ro.lm_trials)
        res["oracle_max_point_rel_diff"] = rel
    return res


def parity_section(tr, mapping, newmp=None):
    """In-run parity against the oracle, stage by stage on each stage's own inputs from the timed region: one frame's
    extraction; its TrackWithMotionModel (motion search, PoseOptimization, outlier discard) and TrackLocalMap
    (isInFrustum + local-map search at the optimised pose, PoseOptimization); one CreateNewMapPoints search; one
    LocalBundleAdjustment window: bit-exact / index-exact / identical outlier sets and LM control flow, floats within
    1e-4."""
    from mam3slam_amd import scene
    from mam3slam_amd.match import LAST_ENTRY_DTYPE, MP_TRACK_DTYPE
    from mam3slam_amd.pose import POSE_RESULT_DTYPE, make_edges, set_pose_float
    from oracle import oracle_py

    out = {}
    f = min(1, tr.B - 1)
    ko, do, _ = oracle_py.extract(tr.frames[f], oracle_py.params(tr.NF))
    n = int(tr.cnt_h[f, 0])
    kg = tr.kps_h[f, :n]
    dg = tr.d_desc[f, :n].cpu().numpy()
    out["extract_bit_exact"] = bool(len(ko) == n and all(np.array_equal(kg[k], ko[k])
                                                         for k in ("x", "y", "angle", "response", "octave"))
                                    and np.array_equal(dg, do))
    F = scene.make_frame_data(kg, dg, tr.W, tr.H)
    # TrackWithMotionModel
    F.pose = tr.poses_init[f]
    last = np.ascontiguousarray(tr.lasts[f], LAST_ENTRY_DTYPE)
    _, o1, _ = oracle_py.track_motion_search(F, last, tr.cam, 15.0, True)
    idx = np.nonzero(o1 >= 0)[0]
    e1 = make_edges(F.keys, tr.inv_s2, idx, last["pos"][o1[idx]])
    res = tr.d_pres[:, f].cpu().numpy().view(POSE_RESULT_DTYPE).reshape(2)
    pout = tr.d_pout[:, f].cpu().numpy()
    _, ol1, (q1, t1), _ = oracle_py.pose_optimization_edges(tr.poses_init[f], tr.cam, e1)
    o1 = o1.copy()
    o1[idx[ol1 == 1]] = -1
    out["motion_search_index_exact"] = bool(np.array_equal(tr.d_out1[f, :n].cpu().numpy(), o1))
    d1 = float(max(np.abs(res[0]["t"] - t1).max() / max(np.abs(t1).max(), 1.0), np.abs(res[0]["q"] - q1).max()))
    # TrackLocalMap at the optimised pose
    F.pose = set_pose_float(res[0]["q"], res[0]["t"])
    no, to = oracle_py.is_in_frustum(F, tr.mpls[f], tr.cam)
    tg = tr.d_mps[f].cpu().numpy().view(MP_TRACK_DTYPE)[:len(tr.mpls[f])]
    v = to["track_in_view"] == 1
    out["frustum_exact"] = bool(int(tr.d_ntm[f].item()) == no and np.array_equal(tg["proj_x"], to["proj_x"]) and
                                np.array_equal(tg["proj_y"], to["proj_y"]) and
                                np.array_equal(tg["scale_level"][v], to["scale_level"][v]))
    # the local search's `taken` input: the slots the motion search filled with a MapPoint with observations, less the
    # discarded outliers
    F.taken = tr.d_taken[f, :n].cpu().numpy()
    nmo, oo = oracle_py.search_by_projection(F, to, 1.0, False, 50.0, 0.8)
    out["local_search_index_exact"] = bool(int(tr.d_nm2[f].item()) == nmo and
                                           np.array_equal(tr.d_out2[f, :n].cpu().numpy(), oo))
    idx2 = np.nonzero((oo >= 0) | (o1 >= 0))[0]
    mp = np.ascontiguousarray(tr.mpls[f])
    pos = np.where((oo[idx2] >= 0)[:, None], mp["pos"][np.maximum(oo[idx2], 0)], last["pos"][np.maximum(o1[idx2], 0)])
    e2 = make_edges(F.keys, tr.inv_s2, idx2, pos)
    _, ol2, (q2, t2), _ = oracle_py.pose_optimization_edges(F.pose, tr.cam, e2)
    d2 = float(max(np.abs(res[1]["t"] - t2).max() / max(np.abs(t2).max(), 1.0), np.abs(res[1]["q"] - q2).max()))
    out["pose_optimization_same_outliers"] = bool(np.array_equal(pout[0, :len(e1)], ol1) and
                                                  np.array_equal(pout[1, :len(e2)], ol2))
    out["pose_optimization_max_rel_diff"] = max(d1, d2)
    out["pose_optimization_edges"] = [len(e1), len(e2)]
    if newmp is not None:
        # the first of the last step's CreateNewMapPoints searches that found matches (FeatureVectors from the device
        # BoW); none with a match fails the parity (a vacuous comparison proves nothing)
        nmv = newmp.nmatch.cpu().numpy()
        qs = np.nonzero(nmv[:newmp.npairs] > 0)[0]
        qp = int(qs[0]) if len(qs) else 0
        K1, K2 = newmp.pair_inputs(qp)
        t0 = time.perf_counter()
        no, oo = oracle_py.search_for_triangulation_kf(K1, K2, tr.cam, tr.cam, False, False)
        tri_ms = (time.perf_counter() - t0) * 1e3
        n1 = len(K1.keys)
        out["triangulation_index_exact"] = bool(len(qs) > 0 and no > 0 and int(nmv[qp]) == no and
                                                np.array_equal(newmp.out[qp, :n1].cpu().numpy(), oo))
        out["triangulation_pair"] = {"pair": qp, "matches": int(no), "n1": n1, "n2": len(K2.keys),
                                     "oracle_ms": tri_ms}
        # SearchInNeighbors: forward item 0 (keyframe 0's MapPoints into its nearest neighbour) and backward item 0
        ok, fused = True, []
        for backward, gi, gd, gn in ((False, newmp.fwd_idx, newmp.fwd_dist, newmp.fwd_n),
                                     (True, newmp.bwd_idx, newmp.bwd_dist, newmp.bwd_n)):
            KF, mps = newmp.fuse_inputs(backward, 0)
            nf, io, do_ = oracle_py.fuse(KF, mps, tr.cam, 3.0)
            ok = ok and int(gn[0].item()) == nf and np.array_equal(gi[0, :len(mps)].cpu().numpy(), io) and \
                np.array_equal(gd[0, :len(mps)].cpu().numpy(), do_)
            fused.append(int(nf))
        out["fuse_index_exact"] = bool(ok)
        out["fuse_items"] = {"forward_fused": fused[0], "backward_fused": fused[1]}
    solved = mapping is not None and (not hasattr(mapping, "rl") or len(mapping.rl.valid) > 0)
    if mapping is not None and not solved:
        # no window of the last run had a fixed keyframe (the reference aborts those LBAs): nothing to compare
        out["lba_window"] = None
    if solved:
        w = mapping.first_valid() if hasattr(mapping, "first_valid") else 0
        prob = mapping.window_inputs(w)
        rg = mapping.window_result(w)
        t0 = time.perf_counter()
        ro = oracle_py.lba_solve(prob)
        lba_cpu_ms = (time.perf_counter() - t0) * 1e3
        rel = float(np.abs(ro.point_xyz - rg.point_xyz).max() / max(np.abs(ro.point_xyz).max(), 1e-12))
        out["lba_same_control_flow"] = bool((ro.iterations, ro.lm_trials) == (rg.iterations, rg.lm_trials))
        out["lba_max_point_rel_diff"] = rel
        out["lba_window"] = {"iterations": int(ro.iterations), "trials": int(ro.lm_trials),
                             "edges": int(len(prob.edge_point)), "oracle_ms": lba_cpu_ms}
    return out


def host_info():
    """The host the CPU baseline ran on: CPU model, cores online, the affinity list of this process."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = []

    def ranges(v):
        out, i = [], 0
        while i < len(v):
            j = i
            while j + 1 < len(v) and v[j + 1] == v[j] + 1:
                j += 1
            out.append(f"{v[i]}-{v[j]}" if j > i else f"{v[i]}")
            i = j + 1
        return ",".join(out)

    return {"cpu_model": model, "nproc_online": os.cpu_count(), "affinity": ranges(aff), "affinity_count": len(aff),
            "threads_used": 1}


def cpu_baseline(tr, cfg, lba_window_ms, K, seconds=10.0, newmp=None):
    """The oracle (single-thread C++ restatement of the reference path) on a bounded sample of the same per-frame
    work — extraction, TrackWithMotionModel (motion search, PoseOptimization, outlier discard) and TrackLocalMap
    (isInFrustum + local-map search, PoseOptimization) — plus 1/K of a keyframe's LocalMapping work: a
    LocalBundleAdjustment of a window of the timed region (its oracle time measured in parity_section on the same
    inputs), its 30 SearchForTriangulation and ComputeBoW."""
    from mam3slam_amd import scene
    from mam3slam_amd.match import LAST_ENTRY_DTYPE
    from mam3slam_amd.pose import make_edges, set_pose_float
    from oracle import oracle_py

    p = oracle_py.params(cfg["nfeatures"])
    W, H = cfg["width"], cfg["height"]
    lasts = [np.ascontiguousarray(x, LAST_ENTRY_DTYPE) for x in tr.lasts]
    mpls = [np.ascontiguousarray(x) for x in tr.mpls]
    # the extraction in two columns: the scalar restatement, and with the AVX2 resize / blur / FAST the reference's
    # OpenCV build runs (oracle/orb_simd.cpp; identical outputs) — the sample's extractions use the AVX2 one, the
    # scalar one is timed on the same frames beside it (outside the sample's clock)
    n, t0 = 0, time.perf_counter()
    ext_s = ext_scalar_s = 0.0
    while True:
        f = n % len(tr.frames)
        te = time.perf_counter()
        k, d, _ = oracle_py.extract(tr.frames[f], p, simd=True)
        ext_s += time.perf_counter() - te
        ts = time.perf_counter()
        oracle_py.extract(tr.frames[f], p)
        ts = time.perf_counter() - ts
        ext_scalar_s += ts
        t0 += ts
        F = scene.make_frame_data(k, d, W, H)
        F.pose = tr.poses_init[f]
        last = lasts[f]
        _, o1, _ = oracle_py.track_motion_search(F, last, tr.cam, 15.0, True)
        idx = np.nonzero(o1 >= 0)[0]
        _, ol1, (q, t), _ = oracle_py.pose_optimization_edges(
            F.pose, tr.cam, make_edges(F.keys, tr.inv_s2, idx, last["pos"][o1[idx]]))
        o1[idx[ol1 == 1]] = -1
        F.pose = set_pose_float(q, t)
        F.taken = ((o1 >= 0) & (last["nobs"][np.maximum(o1, 0)] > 0)).astype(np.uint8)
        _, tracks = oracle_py.is_in_frustum(F, mpls[f], tr.cam)
        _, o2 = oracle_py.search_by_projection(F, tracks, 1.0, nnratio=0.8)
        idx2 = np.nonzero((o2 >= 0) | (o1 >= 0))[0]
        pos = np.where((o2[idx2] >= 0)[:, None], mpls[f]["pos"][np.maximum(o2[idx2], 0)],
                       last["pos"][np.maximum(o1[idx2], 0)])
        oracle_py.pose_optimization_edges(F.pose, tr.cam, make_edges(F.keys, tr.inv_s2, idx2, pos))
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 5) or n >= 2000:
            break
    track_ms = el * 1e3 / n
    per_frame_ms = track_ms + (lba_window_ms / K if lba_window_ms is not None else 0.0)
    tri_ms = None
    if newmp is not None:
        # one new keyframe's LocalMapping search work on the oracle: its 30 SearchForTriangulation (the device BoW's
        # FeatureVectors) and its ComputeBoW (the oracle's DBoW2 transform over the same vocabulary)
        tri_ms = 0.0
        for q in range(newmp.NN):
            K1, K2 = newmp.pair_inputs(q)
            t2 = time.perf_counter()
            oracle_py.search_for_triangulation_kf(K1, K2, tr.cam, tr.cam, False, False)
            tri_ms += (time.perf_counter() - t2) * 1e3
        tree = oracle_py.BowTree(newmp.voc.v)   # built once, as ORBVocabulary is loaded once (not timed)
        d = newmp.desc[newmp.head, :int(newmp.cnt[newmp.head, 0].item())].cpu().numpy()
        t2 = time.perf_counter()
        oracle_py.bow_transform(newmp.voc.v, d, 4, tree=tree)
        bow_ms = (time.perf_counter() - t2) * 1e3
        # its SearchInNeighbors: Fuse into its 30 neighbours, its fuse candidates into it, and the distinctive
        # descriptors of its MapPoints (the update's share of one keyframe)
        sin_ms = 0.0
        for q in range(newmp.NN):
            KF, mps = newmp.fuse_inputs(False, q)
            t2 = time.perf_counter()
            oracle_py.fuse(KF, mps, tr.cam, 3.0)
            sin_ms += (time.perf_counter() - t2) * 1e3
        for q in range(newmp.NB_BACK):
            KF, mps = newmp.fuse_inputs(True, q)
            t2 = time.perf_counter()
            oracle_py.fuse(KF, mps, tr.cam, 3.0)
            sin_ms += (time.perf_counter() - t2) * 1e3
        # ComputeDistinctiveDescriptors of the keyframe's MapPoints (their observations' descriptors from the map)
        off, descs = newmp.distinctive_inputs(newmp.head)
        t2 = time.perf_counter()
        oracle_py.distinctive_descriptors(off, descs)
        sin_ms += (time.perf_counter() - t2) * 1e3
        per_frame_ms += (tri_ms + bow_ms + sin_ms) / K
    ext_ms, ext_scalar_ms = ext_s * 1e3 / n, ext_scalar_s * 1e3 / n
    res = {"value": 1e3 / per_frame_ms, "unit": "frames/s", "cores": 1, "kind": "port",
           "value_scalar_extract": 1e3 / (per_frame_ms - ext_ms + ext_scalar_ms),
           "tracking_ms_per_frame": track_ms, "extract_ms_per_frame": ext_ms,
           "extract_ms_per_frame_scalar": ext_scalar_ms, "host": host_info(),
           "columns": "value: the extraction with the AVX2 resize / blur / FAST (oracle/orb_simd.cpp, the OpenCV SIMD "
                      "paths the reference links; byte-identical outputs); value_scalar_extract: with the scalar "
                      "restatement. Every GPU / CPU ratio in this line (north_star included) uses value.",
           "sample": f"{n} frames {W}x{H}/{cfg['nfeatures']}: extract (AVX2 primitives) + SearchByProjection(motion, "
                     f"th 15; 30 below 20 matches) + "
                     f"PoseOptimization + isInFrustum + SearchByProjection(local map, th 1) + PoseOptimization on the "
                     f"oracle C++ restatement (g++ -O3 -march=x86-64-v3, the reference's CMake -O3 -march=native "
                     f"level), single thread, {el:.1f}s"}
    if lba_window_ms is not None:
        res["lba_ms_per_window"] = lba_window_ms
        res["sample"] += f"; + LocalBundleAdjustment of a timed-region window ({lba_window_ms:.1f} ms) / {K} frames"
    if tri_ms is not None:
        res["new_keyframe_search_ms"] = {"triangulation_30_pairs": tri_ms, "compute_bow": bow_ms,
                                         "search_in_neighbors": sin_ms}
        res["sample"] += (f"; + one new keyframe's 30 SearchForTriangulation ({tri_ms:.1f} ms), ComputeBoW "
                          f"({bow_ms:.2f} ms) and SearchInNeighbors ({sin_ms:.1f} ms) / {K} frames")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per step per GPU (independent frame streams); default 256, c3 / c4: their 2 / 8 "
                         "agents / N")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="c2 (1280x720/2000 + LocalBundleAdjustment) is BASELINE.json's headline metric config")
    ap.add_argument("--kf-every", type=int, default=8,
                    help="keyframe cadence: each stream inserts a keyframe (one LocalBundleAdjustment) every K frames")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-graph", action="store_true", help="launch the tracking step eagerly instead of a HIP graph")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-frame latency and ingest sections")
    ap.add_argument("--no-pose", action="store_true", help="skip the PoseOptimization section")
    ap.add_argument("--no-sin", action="store_true", help="skip the SearchInNeighbors section")
    ap.add_argument("--no-overlap", action="store_true", help="skip timing each leg alone")
    ap.add_argument("--lm-windows", default="ring", choices=("ring", "world"),
                    help="the timed LocalMapping leg's LBA windows: ring = the keyframes the step tracked (RingMappingLeg, "
                         "the reference's window rule), world = the synthetic shared map's windows (LocalMappingLeg)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="tracking sub-batches (own contexts and stream, one graph); default 4, or 2 with LocalMapping "
                         "beside Tracking (c2: 23.9k vs 22.9k frames/s at 2 / 4 lanes, same box: fewer concurrent "
                         "tracking launches leave the LBA's latency-bound kernels more of the chip)")
    ap.add_argument("--cu-split", type=int, default=0, choices=(0, 2, 4, 6),
                    help="LocalMapping's LBA on eighths/8 of every XCD's CUs, Tracking and the keyframe searches on the "
                         "rest (CU-masked streams; 0: every stream on every CU)")
    ap.add_argument("--profile-timed", action="store_true",
                    help="record LocalMapping's stage events inside the timed region (default: a second pass)")
    ap.add_argument("--launch-check", action="store_true",
                    help="rendezvous + barrier over gloo on the CPU and exit (tests the --gpus N launcher, no GPU)")
    args = ap.parse_args()
    parity_failed = [False]

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
    # MAM_BENCH_ONE_DEVICE=1 + MAM_DIST_BACKEND=gloo (tests only): every rank on GPU 0, the exchange over gloo — the
    # whole multi-rank path on a one-GPU box (RCCL refuses two ranks on one device)
    if os.environ.get("MAM_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("MAM_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend=backend)

    cfg = CONFIGS[args.config]
    agents_total = cfg.get("agents")
    B = args.batch if args.batch is not None else (max(1, agents_total // world) if agents_total else 256)
    lanes = args.lanes if args.lanes is not None else (2 if cfg["lba"] else 4)
    NL, K = min(max(1, lanes), B), max(1, args.kf_every)
    if B % NL:
        raise SystemExit(f"--batch {B} is not a multiple of --lanes {NL}")
    # keyframe cadence: B/K new keyframes (LBA windows) per step; with fewer streams than K, one every K/B steps
    map_every = max(1, K // B)
    tr_stream = lm_stream = lm_mask = None
    if args.cu_split and cfg["lba"]:
        from mam3slam_amd import streams

        ncu = streams.cu_count(dev.index or 0)
        lm_mask = streams.cu_mask(ncu, args.cu_split)
        tr_mask = streams.cu_mask(ncu, args.cu_split, complement=True)
        tr_stream = lambda: streams.masked_stream(dev, tr_mask)  # noqa: E731
        lm_stream = streams.masked_stream(dev, lm_mask)
    tr = TrackingLeg(cfg, B, NL, rank, dev, new_stream=tr_stream)
    mapping = newmp = None
    if cfg["lba"]:
        from mam3slam_amd.mapping import LocalMappingLeg, NewMapPointsLeg, RingMappingLeg

        newmp = NewMapPointsLeg(tr, max(1, B // K), dev, stream=tr_stream() if tr_stream else None)
        if args.lm_windows == "ring":
            mapping = RingMappingLeg(newmp, rank, world, dev, stream=lm_stream)
            if lm_mask is not None:
                mapping.solver.set_cu_mask(lm_mask)
        else:
            mapping = LocalMappingLeg(max(1, B // K), rank, world, dev, camera=tr.cam if cfg.get("camera") else None,
                                      width=tr.W, height=tr.H)

    lba_ev = []   # (start, end) events of each LocalMapping run on its stream

    def mapping_worker(step_idx, item):
        # one LocalMapping run (LocalMapping::Run for the keyframes one step inserted), serial on LocalMapping's
        # stream: the keyframes into the ring, ComputeBoW, MapPointCulling, CreateNewMapPoints, SearchInNeighbors and
        # their map edits (NewMapPointsLeg.process), then the LocalBundleAdjustment windows, their solve and
        # write-back and the exchange of the write-back (RingMappingLeg.run; the world leg: its synthetic map's
        # windows) — the run's span on the stream from events recorded around it (the exchange tail included)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t_m = time.perf_counter()
        e0.record(mapping.stream)
        if args.lm_windows == "ring":
            mapping.run(step_idx, item)
        else:
            newmp.process(mapping.stream, item)
            mapping.run(step_idx)
        e1.record(mapping.stream)
        lba_ev.append((e0, e1))
        host_s["mapping_run"] += time.perf_counter() - t_m

    def lba_ms():
        torch.cuda.synchronize(dev)
        return [a.elapsed_time(b) for a, b in lba_ev]

    step_no = [0]
    # LocalMapping runs beside Tracking as in the reference (its own thread and stream, fed through a queue: the
    # keyframe queue LocalMapping::InsertKeyFrame fills): one run in progress and one waiting at most, so Tracking
    # blocks only when LocalMapping falls two runs behind. (Joining each run before the next tracking step would chain
    # search(i-1) -> LBA(i) -> tracking(i+1) and make the step the sum of the legs.)
    import queue

    runs = queue.Queue(maxsize=1)
    worker = [None]
    failure = []

    def mapping_loop():
        while True:
            item = runs.get()
            try:
                if item is None:
                    return
                if not failure:
                    mapping_worker(*item)
            except BaseException as e:   # re-raised by finish_mapping on the main thread
                failure.append(e)
            finally:
                runs.task_done()

    def finish_mapping():
        if worker[0] is not None:
            runs.join()
        if failure:
            raise failure[0]

    host_s = {"queue_wait": 0.0, "tracking_launch": 0.0, "keyframe_ingest_launch": 0.0, "mapping_run": 0.0}

    def step():
        t_a = time.perf_counter()
        tr.step()
        t_b = time.perf_counter()
        t_c = t_b
        if mapping is not None and (step_no[0] + 1) % map_every == 0:
            # the step's new keyframes into a staging set (tracking stream), then the run queued for LocalMapping's
            # thread: put blocks while one run is in progress and one waits (Tracking blocks when LocalMapping falls
            # two runs behind)
            item = newmp.ingest(step_no[0])
            if worker[0] is None:
                worker[0] = threading.Thread(target=mapping_loop, daemon=True)
                worker[0].start()
            if failure:
                raise failure[0]
            t_c = time.perf_counter()
            runs.put((step_no[0] // map_every, item))
        t_d = time.perf_counter()
        host_s["tracking_launch"] += t_b - t_a
        host_s["keyframe_ingest_launch"] += t_c - t_b
        host_s["queue_wait"] += t_d - t_c
        step_no[0] += 1

    for _ in range(args.warmup):
        step()
    finish_mapping()
    torch.cuda.synchronize(dev)
    if not args.no_graph:
        tr.capture()   # the tracking step (~40 launches) replayed as one HIP graph
        torch.cuda.synchronize(dev)
        for _ in range(2):
            step()
        finish_mapping()
        torch.cuda.synchronize(dev)
    cnt = tr.d_cnt.cpu().numpy()
    n_kp = float(cnt[:, 0].mean())
    nf_probe = min(tr.BL, 4)   # frames lane 0's extractor (tr.ext) processed
    n_cand = float(sum(len(tr.ext.debug_candidates(l, f)) for l in range(8) for f in range(nf_probe))) / nf_probe
    nm1, nm2, ntm = tr.d_nm1.cpu().numpy(), tr.d_nm2.cpu().numpy(), tr.d_ntm.cpu().numpy()
    if (nm1 < 0).any() or (nm2 < 0).any() or (cnt[:, 0] < 0).any():
        raise RuntimeError(f"device error codes in outputs: {nm1.min()} {nm2.min()} {cnt[:, 0].min()}")

    def set_profiling(on):
        # LocalMapping's per-stage HIP events (8 event records per LM trial on the LBA stream, 2 per search batch,
        # the map edits') and the all-gather's wall time
        mapping.time_gather = on
        newmp.profile = on
        mapping.solver.set_profiling(on)
        newmp.matcher.set_profiling(on)
        newmp.voc.set_profiling(on)

    lba_ev.clear()
    for k in host_s:
        host_s[k] = 0.0
    if mapping is not None:
        mapping.host_s = {}
    if mapping is not None and args.profile_timed:
        set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    finish_mapping()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # host time per timed step by phase (the main thread: queue wait, the tracking graph launch, the keyframe ingest +
    # search launch; the LocalMapping thread: its run) — where a host-bound step would show
    host_ms = {k: v * 1e3 / args.steps for k, v in host_s.items()}
    if mapping is not None:
        host_ms.update({"mapping_" + k: v * 1e3 / args.steps for k, v in mapping.host_s.items()})
    lba_stage = None
    tri_stage = None
    if mapping is not None and not args.profile_timed:
        # the stage times come from a second pass of the same steps with the events on, outside the timed region
        timed_lba_ev = list(lba_ev)
        set_profiling(True)
        for _ in range(args.steps):
            step()
        finish_mapping()
        torch.cuda.synchronize(dev)
        lba_ev[:] = timed_lba_ev
    if mapping is not None:
        lba_stage = mapping.solver.stage_times()
        mapping.solver.set_profiling(False)
        mst = newmp.matcher.stage_times()
        tri_stage = {"triangulation": mst["triangulation"], "compute_bow": newmp.voc.stage_times()["transform"],
                     "search_in_neighbors": (mst["fuse"][0] + mst["distinctive"][0] + mst["grid"][0],
                                             mst["fuse"][1] + mst["distinctive"][1])}
        newmp.matcher.set_profiling(False)
        newmp.voc.set_profiling(False)
        stv = int(mapping.status.cpu().numpy()[0])
        if stv != 0 or any(s[2] < 0 for s in mapping.stats):
            raise RuntimeError(f"LocalMapping leg status {stv} / {mapping.stats}")
    overlap = None
    if mapping is not None and not args.no_overlap:
        # each leg alone over the same number of steps (outside the timed region): Tracking's step (the HIP graph),
        # then LocalMapping's run (the LocalBundleAdjustment windows + exchange) — how much of the combined step is
        # overlap and how much is the legs contending for CUs
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            tr.step()
        torch.cuda.synchronize(dev)
        tr_only = (time.perf_counter() - t1) * 1e3 / args.steps
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(args.steps):   # the last run's keyframes again (re-inserted: the same LocalMapping work)
            if args.lm_windows == "ring":
                mapping.run(10_000 + i)
            else:
                newmp.process(mapping.stream, newmp.last_item)
                mapping.run(10_000 + i)
        torch.cuda.synchronize(dev)
        lm_only = (time.perf_counter() - t1) * 1e3 / args.steps
        overlap = {"combined_ms_per_step": el * 1e3 / args.steps, "tracking_only_ms_per_step": tr_only,
                   "local_mapping_only_ms_per_step": lm_only,
                   "note": "the same steps with one leg only (tracking: the step's HIP graph; LocalMapping: its "
                           "LocalBundleAdjustment windows + exchange, no concurrent tracking), rank-local wall time"}
    stages = tr.stage_pass(args.steps)
    lat = None if args.no_latency else latency_section(tr)
    ingest = None if args.no_latency else ingest_section(tr)
    pose_info = None
    if not args.no_pose:
        from scripts import pose_bench

        pose_info = pose_bench.section(tr, reps=max(args.steps, 5), oracle=not args.no_cpu_baseline and rank == 0)
    sin_info = None
    if not args.no_sin:
        from scripts import fuse_bench

        sin_info = fuse_bench.run(args.config, reps=max(args.steps, 5), device=dev.index or 0,
                                  oracle=not args.no_cpu_baseline and rank == 0)
    ring = ring_lba_section(newmp) if newmp is not None and rank == 0 else None
    parity = parity_section(tr, mapping, newmp) if rank == 0 else None
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    T = float(t.item())
    frames_total = world * B * args.steps

    # roofline of the dominant kernel stage: algorithmic bytes per launch / mean launch duration (HIP events on the
    # stream each launch runs on)
    mean_last = float(np.mean([len(x) for x in tr.lasts]))
    mean_mps = float(np.mean([len(x) for x in tr.mpls]))
    sb = stage_bytes(tr.W, tr.H, n_kp, n_cand, mean_last, mean_mps, cand_motion=mean_last * 6.0,
                     cand_local=mean_mps * 3.0)
    per_step_ms = {k: v[0] / args.steps for k, v in stages.items()}
    # the HBM roofline is over the byte-moving stages (PoseOptimization is FP64 compute: per_step_ms only; `resolve`,
    # one workgroup per frame doing dependency rounds on LDS atomics, is latency with a few KB a frame: per_step_ms)
    dom = max((k for k in stages if k in sb and k not in LATENCY_STAGES), key=lambda k: stages[k][0])
    ms_tot, launches = stages[dom]
    avg_ms = ms_tot / max(launches, 1)
    launches_per_step = launches / args.steps
    bytes_per_launch = sb[dom] * B / launches_per_step
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = traffic_raw = None
    pmc_counters = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):   # PMC passes of the same launches (scripts/gpu_fast_pmc.sh)
        try:
            tj = json.load(open(tpath))
            traffic, traffic_raw = tj.get(dom), tj.get("raw", {}).get(dom)
            # the passes' launch shape (gpu_fast_pmc.sh: --lanes 1 --batch 64) scaled to this run's launches of
            # tr.BL frames (the stage's bytes are per frame)
            fl = float(tj.get("frames_per_launch", 64))
            if traffic is not None:
                traffic *= tr.BL / fl
            if traffic_raw is not None:
                traffic_raw *= tr.BL / fl
            pmc_counters = {k: tj.get(k, {}).get(dom) for k in ("valu_busy", "wave_frac_wait", "wave_frac_issue_stall")}
        except Exception:
            traffic = traffic_raw = None
    limiter = ROOFLINE_NOTES.get(dom)
    if pmc_counters and all(v is not None for v in pmc_counters.values()):
        # the limiter as this config's counters give it (scripts/gpu_fast_pmc.sh -> profiles/traffic_<config>.json)
        limiter = (f"latency / issue: per standalone launch VALU busy {100 * pmc_counters['valu_busy']:.1f}%, "
                   f"{100 * pmc_counters['wave_frac_wait']:.0f}% of wave cycles waiting (s_waitcnt, barriers), "
                   f"{100 * pmc_counters['wave_frac_issue_stall']:.0f}% issue-stalled; HBM traffic "
                   f"{(traffic or 0) / 1e6:.1f} MB (raw FETCH {(traffic_raw or 0) / 1e6:.1f} MB) vs "
                   f"{sb[dom] * B / (launches / args.steps) / 1e6:.1f} MB algorithmic per launch "
                   f"(profiles/traffic_{args.config}.json)")

    if rank == 0:
        W, H, NF = tr.W, tr.H, tr.NF
        camd = "KannalaBrandt8 (test YAML)" if cfg.get("camera") == "kb8" else "Pinhole"
        workload = (f"{args.config}: mono {W}x{H}, {NF} features, 8 levels, {camd}; step = {B} frame streams x (ORB "
                    f"extract + TrackWithMotionModel: SearchByProjection motion th15 (th30 below 20 matches) + "
                    f"PoseOptimization + outlier "
                    f"discard; TrackLocalMap: isInFrustum + SearchByProjection local map th1 + PoseOptimization)")
        if agents_total:
            workload += f"; {agents_total} agents in total, {B} per GPU"
        if mapping is not None:
            workload += (f" + a keyframe every {K} frames per stream: {mapping.W} new keyframes per "
                         f"{'step' if map_every == 1 else f'{map_every} steps'}, each with "
                         f"ComputeBoW + 30 SearchForTriangulation (CreateNewMapPoints) + SearchInNeighbors (Fuse both ways + "
                         f"ComputeDistinctiveDescriptors) and ")
            if args.lm_windows == "ring":
                sz = mapping.rl.sizes[mapping.rl.valid]
                # (a short run's windows may all lack a fixed keyframe: the reference skips those LBAs)
                shape = (f"~{float(np.mean(sz[:, 3])):.1f} optimised KF; every MapPoint of every local keyframe, "
                         f"~{int(np.mean(sz[:, 1]))}; fixed = their other observers, "
                         f"{float(np.mean(sz[:, 0] - sz[:, 3])):.1f} KF; ~{int(np.mean(sz[:, 2]))} observations"
                         if len(sz) else "no window of the last run had a fixed keyframe")
                workload += (f"MapPoint creation, Fuse's Replace / AddObservation and the MapPoints' descriptor / "
                             f"normal / depth update on the device map the ring's keyframes share, and a "
                             f"LocalBundleAdjustment window of the keyframe by the reference's window rule over that "
                             f"map (local = the keyframe + its covisible keyframes, {shape}), batched, its write-back "
                             f"(outlier erase, poses, positions, normals / depth ranges) applied to the map, "
                             f"concurrent with tracking; write-backs exchanged (all-gather) and applied to the "
                             f"replica every GPU holds")
            else:
                workload += (f"a LocalBundleAdjustment window (50 KF + fixed, "
                             f"~{int(np.mean([len(p.point_id) for p in mapping.probs]))} MapPoints) of the synthetic "
                             f"shared map, batched, concurrent with tracking; write-backs exchanged and applied to "
                             f"the map the next windows read")
        out = {
            "metric": "tracked frames/sec (ORB extract+match+localBA) at 1/2/4/8 GPUs vs CPU ref",
            "value": frames_total / T,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": T / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if agents_total else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": workload, "frames_per_step_per_gpu": B, "width": W, "height": H,
                       "nfeatures": NF, "keyframe_every": K if mapping is not None else None,
                       "keypoints_per_frame": n_kp, "fast_candidates_per_frame": n_cand,
                       "last_frame_points": mean_last, "local_map_points": mean_mps,
                       "local_points_in_view": float(ntm.mean()),
                       "matches_motion_per_frame": float(nm1.mean()), "matches_local_per_frame": float(nm2.mean()),
                       "parallelism": f"agents{world} (one process per GPU; {B} frame streams per GPU)",
                       "lanes": NL, "launch": "hip graph per tracking step" if tr.graph is not None else "eager",
                       "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")},
            "stage_ms_per_step": per_step_ms,
            "roofline": {"bound": "hbm", "kernel": dom, "limiter": limiter, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_raw_fetch": traffic_raw, "pmc": pmc_counters,
                         "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_ms},
        }
        if lat is not None:
            out["latency_ms_per_frame_b1"] = lat["device_graph_ms"]
            out["latency"] = lat
        if ingest is not None:
            out["ingest"] = ingest
        if overlap is not None:
            out["overlap"] = overlap
        out["host_ms_per_step"] = host_ms
        if ring is not None:
            out["ring_lba"] = ring
            if parity is not None:
                parity["ring_lba_same_control_flow"] = ring.get("oracle_same_control_flow")
                parity["ring_lba_max_point_rel_diff"] = ring.get("oracle_max_point_rel_diff")
        vw = []
        if mapping is not None:
            # the last run's solved windows (a window without fixed keyframes is not solved: Optimizer.cc:1182-1185)
            vw = list(mapping.rl.valid) if args.lm_windows == "ring" else list(range(mapping.W))
        if mapping is not None and not vw:
            out["lba"] = {"windows_per_step": mapping.W, "windows_solved_last_run": 0,
                          "note": "no window of the last LocalMapping run had a fixed keyframe (the reference aborts "
                                  "those LocalBundleAdjustments, Optimizer.cc:1182-1185)"}
        if mapping is not None and vw:
            probs_v = [mapping.probs[w] for w in vw]
            its = [mapping.stats[w][0] for w in vw]
            trials = [mapping.stats[w][1] for w in vw]
            E = float(np.mean([mapping.edges[w] for w in vw]))
            L = float(np.mean([len(p.point_id) for p in probs_v]))
            Np = float(np.mean([int((p.pose_fixed == 0).sum()) for p in probs_v]))
            fl = lba_flops(E, L, Np, E / L, float(np.mean(trials)), float(np.mean(its)))
            spans = lba_ms()
            solve_ms = float(np.mean(spans)) if spans else None
            if args.lm_windows == "ring":
                nkr, nmr, xst = mapping.exchange_counts()
            else:
                nkr, nmr, xst = mapping.n_kf_upd, mapping.n_mp_upd, 0
            out["lba"] = {"windows_per_step": mapping.W, "windows_solved_last_run": len(vw), "ms_per_step_span": solve_ms,
                          "ms_per_window_span": solve_ms / mapping.W if solve_ms else None,
                          "span_note": "LocalMapping run per step on its stream (events around it: the keyframe "
                                       "searches it waits on, the LBA windows, the pack / all-gather / apply of "
                                       "their write-backs), concurrent with tracking",
                          "iterations_mean": float(np.mean(its)), "trials_mean": float(np.mean(trials)),
                          "edges_per_window": E, "points_per_window": L, "opt_keyframes": Np,
                          "algorithmic_gflop_per_window": fl / 1e9,
                          "achieved_fp64_tflops": (fl * len(vw)) / (solve_ms * 1e-3) / 1e12 if solve_ms else None,
                          "fp64_peak_tflops": FP64_PEAK_TFS,
                          "stage_ms_total": {k: v[0] for k, v in lba_stage.items()},
                          "stage_launches": {k: v[1] for k, v in lba_stage.items()},
                          "exchange_bytes_per_step": int(mapping.exch.send.numel() * world),
                          "exchange": {"bytes_per_rank_block": int(mapping.exch.block_bytes),
                                       "keyframe_records": nkr, "mappoint_records": nmr, "status": xst,
                                       "bytes_per_window": mapping.exch.block_bytes / mapping.W,
                                       "allgather_ms_median": float(np.median(mapping.exch.gather_ms))
                                       if mapping.exch.gather_ms else None,
                                       "note": "one fixed-size all_gather_into_tensor per step of each GPU's "
                                               "deduplicated write-back (32-B KeyFrame records; MapPoint records: "
                                               "48 B with normal and depth range on the device map, 16 B on the "
                                               "world leg); "
                                               "gather time = host wall around the collective with the stream "
                                               "synchronised, from the untimed profiling pass"}}
            # the LocalBundleAdjustment's roofline: its dominant kernel, the tile LDL^T (one workgroup per window,
            # FP64 MFMA), from the profiled pass's solve-stage events (the first stream group's launches: windows
            # [0, Q / G) of the batch) and the tile structure of those windows
            G = 2 if len(vw) >= 4 else 1
            g0 = probs_v[:len(vw) // G]
            fl_ldlt = [ldlt_tile_flops(p) for p in g0]
            ms_solve, n_solve = lba_stage["solve"]
            tr_mean = float(np.mean(trials[:len(g0)]))
            ach = args.steps * tr_mean * sum(fl_ldlt) / (ms_solve * 1e-3) / 1e12 if ms_solve else None
            # the FP64-MFMA counter pass over the windows this leg solves (ring: profiles/r05's 32 ring windows;
            # the synthetic world's windows: the round-4 pass over its batch of 32)
            mrel = next((f"profiles/{r}/{f}" for r in ("r06", "r05", "r04")
                         for f in (("lba_mfma_f64_ring.json",) if args.lm_windows == "ring" else ("lba_mfma_f64.json",))
                         if os.path.exists(os.path.join(ROOT, f"profiles/{r}/{f}"))), "profiles/r04/lba_mfma_f64.json")
            mpath = os.path.join(ROOT, mrel)
            mfma = None
            if os.path.exists(mpath):
                try:
                    mj = json.load(open(mpath))
                    mfma = {k: v for k, v in mj.items() if "k_ldlt" in k}
                except Exception:
                    mfma = None
            out["roofline_lba"] = {
                "bound": "mfma", "unit": "TFLOP/s", "achieved": ach,
                "kernel": ("k_ldlt_any + k_ldlt_mw" if args.lm_windows == "ring" else "k_ldlt_any"),
                "peak": FP64_PEAK_TFS, "frac": ach / FP64_PEAK_TFS if ach else None,
                "frac_of_cus_used": (ach / (FP64_PEAK_TFS * min(256, len(g0) * (8 if args.lm_windows == "ring" else 1)) / 256.0)
                                     if ach else None),
                "flop_per_factorization": float(np.mean(fl_ldlt)), "windows_per_launch": len(g0),
                "avg_launch_ms": ms_solve / max(n_solve, 1), "launches": n_solve,
                "mfma_counters": mfma, "mfma_counters_file": mrel if mfma else None,
                "limiter": ("latency: the device map's windows are dense (every optimised pose pair shares a MapPoint), so "
                            "the solve stage is k_ldlt_mw's column chain — 8 workgroups a window, a panel workgroup "
                            "factoring every 16-wide block column in turn (~10 us a column: the ready column's "
                            "agent-coherent load, the last update, the diagonal tile's 16 pivot steps, the panel rows, "
                            "the publish) while the others stream the earlier updates (DESIGN §3)"
                            if args.lm_windows == "ring" else
                            "latency: one workgroup per window factors the tile pattern as a dataflow of per-tile and "
                            "per-panel tasks (two chains of 6-9 block columns + the separator's 3-4 under the split "
                            "pose order); per column ~6.4k cycles: the critical tile update (4 FP64 MFMAs + operand "
                            "loads) ~1.5k, the tall panel's 16 dependent pivot steps ~2.3k, stores + flag ~1.2k "
                            "(scripts/gpu_ldlt_trace.sh)"),
                "note": "algorithmic = tile-skipping LDL^T + solves (ldlt_tile_flops); frac_of_cus_used prices "
                        "against the FP64 MFMA peak of the CUs the launch's workgroups occupy (one per window; eight "
                        "per dense window of the ring leg)"}
            # the Schur stage (k_schur_blk: FP64 VALU products of each landmark's pose pairs), the same windows
            fl_schur = [schur_flops(p) for p in g0]
            ms_schur, n_schur = lba_stage["schur"]
            ach_s = args.steps * tr_mean * sum(fl_schur) / (ms_schur * 1e-3) / 1e12 if ms_schur else None
            out["roofline_lba_schur"] = {
                "bound": "fp64", "kernel": "k_schur_blk", "unit": "TFLOP/s", "achieved": ach_s,
                "peak": FP64_PEAK_TFS, "frac": ach_s / FP64_PEAK_TFS if ach_s else None,
                "flop_per_schur": float(np.mean(fl_schur)), "windows_per_launch": len(g0),
                "avg_launch_ms": ms_schur / max(n_schur, 1), "launches": n_schur,
                "note": "algorithmic = sum over landmarks of m (m + 1) / 2 pose-pair blocks x 216 flops (schur_flops), "
                        "one Schur per LM trial; time = the solver's schur stage events (k_schur_blk and its "
                        "setup), the first stream group's launches"}
        if newmp is not None:
            nmv = newmp.nmatch.cpu().numpy()
            tri_b = newmp.algorithmic_bytes()
            tri_ms = tri_stage["triangulation"][0] / args.steps
            out["new_keyframes"] = {
                "keyframes_per_step": newmp.W, "searches_per_step": newmp.npairs, "neighbours": newmp.NN,
                "matches_per_search": float(nmv.mean()),
                "ms_per_step_triangulation": tri_ms,
                "ms_per_step_compute_bow": tri_stage["compute_bow"][0] / args.steps,
                "ms_per_step_search_in_neighbors": tri_stage["search_in_neighbors"][0] / args.steps,
                "fused_per_forward_fuse": float(newmp.fwd_n.float().mean().item()),
                "fused_per_backward_fuse": float(newmp.bwd_n.float().mean().item()),
                "candidate_pairs_per_search": tri_b["candidate_pairs"] / newmp.npairs,
                "map_edits_ms_last_profiled_run": newmp.profiled_map_ms(),
                "map": newmp.map.stats(),
                "algorithmic_bytes_per_step_triangulation": tri_b["bytes"],
                "achieved_GBs_triangulation": tri_b["bytes"] / (tri_ms * 1e-3) / 1e9 if tri_ms > 0 else None,
                "note": "ComputeBoW (levelsup 4, synthetic k=10 L=6 vocabulary) + MapPointCulling + "
                        "CreateNewMapPoints' SearchForTriangulation against the 30 nearest older keyframes of the "
                        "agent's sequence and the MapPoints of its matches + SearchInNeighbors (Fuse into the 30, Fuse "
                        "of 4 neighbours' MapPoints back, Replace / AddObservation, ComputeDistinctiveDescriptors + "
                        "UpdateNormalAndDepth) on the device map, on LocalMapping's stream before the LBA windows of "
                        "the same keyframes (stage times on that stream, concurrent with tracking, from a second "
                        "untimed pass of the same steps with the HIP events on; --profile-timed records them inside "
                        "the timed region; map: MapPoints alive, observations per MapPoint, MapPoints per keyframe); "
                        "algorithmic bytes per SURVEY §8(d): "
                        "sum over shared BoW nodes of |f1| x |f2| x 32 B of descriptors + the two FeatureVectors' "
                        "keypoints, flags and keys (the last run's pairs)"}
        if pose_info is not None:
            out["pose_optimization"] = pose_info
        if sin_info is not None:
            out["search_in_neighbors"] = sin_info
        if parity is not None:
            out["parity"] = parity
            # every exactness flag must hold and every float difference stay inside the north star's 1e-4
            bad = [k for k, v in parity.items() if isinstance(v, bool) and not v]
            bad += [k for k in ("lba_max_point_rel_diff", "pose_optimization_max_rel_diff", "ring_lba_max_point_rel_diff")
                    if parity.get(k) is not None and not parity[k] <= 1e-4]
            out["parity_ok"] = not bad
            if bad:
                out["invalid"] = "parity failed: " + ", ".join(bad)
        if not args.no_cpu_baseline:
            lba_cpu = parity.get("lba_window", {}).get("oracle_ms") if parity else None
            out["cpu_baseline"] = cpu_baseline(tr, cfg, lba_cpu, K, args.cpu_seconds, newmp)
            out["cpu_baseline"]["ms_per_frame"] = 1e3 / out["cpu_baseline"]["value"]
            if lat is not None:
                out["speedup_latency_b1"] = out["cpu_baseline"]["tracking_ms_per_frame"] / lat["device_graph_ms"]
            if lat is not None and (mapping is None or vw):
                # the north star's per-frame figure: ORBextractor (the host-API call a Frame constructor makes, B = 1)
                # + a lone LocalBundleAdjustment window every K frames, GPU vs the oracle on the same inputs. With a
                # LocalMapping leg the window is one of its timed-region windows; without one (c1) a 50-keyframe window
                # of the synthetic map (BASELINE configs[2]'s LBA shape) at this config's camera, its oracle time and
                # parity here
                from mam3slam_amd.lba import LBASolver

                win_note = "the same timed-region window"
                win_parity = None
                if mapping is not None:
                    prob = probs_v[0]
                else:
                    from mam3slam_amd import world as WD
                    from oracle import oracle_py

                    wd = WD.make_world(n_kf=120, seed=7, width=W, height=H)
                    prob = WD.window(wd, 25, n_opt=50)[0]
                    t1 = time.perf_counter()
                    ro = oracle_py.lba_solve(prob)
                    lba_cpu = (time.perf_counter() - t1) * 1e3
                    win_note = (f"a 50-keyframe window of the synthetic map ({len(prob.pose_id)} KF incl. fixed, "
                                f"{len(prob.point_id)} MapPoints, {len(prob.edge_point)} edges; the 50-KF LBA shape of BASELINE "
                                f"configs[2]) "
                                f"at this config's camera")
                sol = LBASolver(device=dev.index or 0)
                rg = sol.solve(prob)
                if mapping is None:
                    rel = float(np.abs(ro.point_xyz - rg.point_xyz).max() / max(np.abs(ro.point_xyz).max(), 1e-12))
                    win_parity = {"same_control_flow": bool((ro.iterations, ro.lm_trials) == (rg.iterations, rg.lm_trials)),
                                  "max_point_rel_diff": rel, "iterations": int(ro.iterations),
                                  "trials": int(ro.lm_trials)}
                    if parity is not None:
                        parity["north_star_lba_same_control_flow"] = win_parity["same_control_flow"]
                        parity["north_star_lba_max_point_rel_diff"] = rel
                        bad = not win_parity["same_control_flow"] or not rel <= 1e-4
                        if bad:
                            out["parity_ok"] = False
                            out["invalid"] = (out.get("invalid", "parity failed:") + " north_star_lba")
                # the C-ABI call alone (mam_lba_solve on host arrays, the structs built once, as the C++
                # Optimizer::LocalBundleAdjustment wrapper calls it), and through the Python mirror
                import ctypes as C

                from mam3slam_amd.lba import alloc_result

                cP = prob.as_c()
                cR, _arrs = alloc_result(prob)
                ts, tp = [], []
                for i in range(9):
                    t1 = time.perf_counter()
                    rc = sol._L.mam_lba_solve(sol._ctx, C.byref(cP), None, C.byref(cR))
                    t2 = time.perf_counter()
                    sol.solve(prob)
                    t3 = time.perf_counter()
                    assert rc == 0, rc
                    if i >= 2:
                        ts.append((t2 - t1) * 1e3)
                        tp.append((t3 - t2) * 1e3)
                lone = float(np.median(ts))
                ext_gpu, ext_cpu = lat["host_api_extract_ms"], out["cpu_baseline"]["extract_ms_per_frame"]
                g, c_ = ext_gpu + lone / K, ext_cpu + lba_cpu / K
                out["north_star"] = {
                    "extract_ms_gpu_host_api": ext_gpu, "extract_ms_cpu": ext_cpu,
                    "lba_lone_window_ms_gpu": lone, "lba_lone_window_ms_gpu_python": float(np.median(tp)),
                    "lba_window_ms_cpu": lba_cpu, "keyframe_every": K,
                    "per_frame_ms_gpu": g, "per_frame_ms_cpu": c_, "ratio": c_ / g,
                    "ratio_scalar_extract": (out["cpu_baseline"]["extract_ms_per_frame_scalar"] + lba_cpu / K) / g,
                    "lba_window": win_note, "lba_window_parity": win_parity,
                    "note": "ORBextractor per frame + one LocalBundleAdjustment window per K frames (the window alone "
                            "through mam_lba_solve, host arrays in and out; median of 7 after warm solves; the C-ABI "
                            "calls as a C++ caller makes them, the Python mirrors' times beside them), target "
                            ">= 50x; ratio: against the CPU extraction with the AVX2 primitives (cpu_baseline.value's "
                            "column), ratio_scalar_extract: against the scalar restatement's"}
        print(json.dumps(out), flush=True)
        if out.get("invalid"):
            print(out["invalid"], file=sys.stderr)
            parity_failed[0] = True
    if world > 1:
        dist.destroy_process_group()
    if parity_failed[0]:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
