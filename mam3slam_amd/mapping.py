"""The LocalMapping leg of a multi-agent step on one GPU: LocalBundleAdjustment of the new keyframes' windows over a
shared map resident in HBM, and the exchange that keeps the map identical on every GPU.

Per step (one call of `run`), for the W keyframes the agents on this GPU inserted:
  1. `new_keyframes`: each window's newest keyframe enters the map at the motion model's guess and its new MapPoints
     at their first triangulation (a deterministic perturbation of those map entries) — the work a new keyframe
     brings to LocalMapping (LocalMapping.cc:162-172 runs one LBA per processed keyframe);
  2. the windows' vertex estimates are read from the shared map tables (mam_map_read_windows: the graph build of
     Optimizer.cc:1218-1286 takes the float map values cast to double);
  3. all W LocalBundleAdjustment solves run together (mam_lba_solve_batch_device: Levenberg control on the device);
  4. the write-backs (Optimizer.cc:1463-1497) are packed (mam_exchange_pack_windows), all-gathered across GPUs
     (RCCL over xGMI) and applied in (GPU, window) order to the map every GPU holds — which the next step's windows
     read. Overlapping windows (shared keyframes / MapPoints) resolve deterministically: later blocks win.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import world as W
from .exchange import MapUpdateExchange, MapWindow
from .lba import LBASolver, _Problem, _Result


class LocalMappingLeg:
    def __init__(self, n_windows: int, rank: int, world_size: int, device, max_gpus: int = 8, n_opt: int = 50,
                 stride: int = 25, seed: int = 7, stream=None):
        import torch

        self.dev = device
        self.W = int(n_windows)
        self.rank, self.world_size = rank, world_size
        # one world for every world size (weak scaling: the same windows per GPU for any N)
        n_kf = (max_gpus * self.W + 1) * stride + n_opt + 8
        self.world = W.make_world(n_kf=n_kf, seed=seed)
        self.mp_base = self.world.n_kf          # MapPoint vertex id = mnId + maxKFid + 1
        self.starts = [(rank * self.W + w) * stride for w in range(self.W)]
        self.solver = LBASolver(device=device.index or 0)
        self.stream = stream if stream is not None else torch.cuda.Stream(device, priority=-1)
        self.kf_table = torch.from_numpy(self.world.kf_table).to(device)
        self.mp_table = torch.from_numpy(self.world.mp_table).to(device)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        self._keep = []
        self.probs, self.kf_ids, self.mp_ids = [], [], []
        self.c_probs = (_Problem * self.W)()
        self.c_res = (_Result * self.W)()
        rd = (MapWindow * self.W)()
        pk = (MapWindow * self.W)()
        self.res = []
        self.inputs = []
        max_rows, cap = 0, 0

        def dev(a):
            t = torch.from_numpy(np.array(a, copy=True)).to(device)
            self._keep.append(t)
            return t

        for w, s in enumerate(self.starts):
            p, kfs, mps = W.window(self.world, s, n_opt=n_opt)
            self.probs.append(p)
            self.kf_ids.append(kfs)
            self.mp_ids.append(mps)
            P, L, E = len(p.pose_id), len(p.point_id), len(p.edge_point)
            max_rows = max(max_rows, P, L)
            cap = max(cap, int((p.pose_fixed == 0).sum()) + L)
            pid, fix, mid = dev(p.pose_id), dev(p.pose_fixed), dev(p.point_id)
            q_in = torch.zeros((P, 4), dtype=torch.float64, device=device)
            t_in = torch.zeros((P, 3), dtype=torch.float64, device=device)
            x_in = torch.zeros((L, 3), dtype=torch.float64, device=device)
            out = dict(pose_q=torch.zeros((P, 4), dtype=torch.float64, device=device),
                       pose_t=torch.zeros((P, 3), dtype=torch.float64, device=device),
                       point_xyz=torch.zeros((L, 3), dtype=torch.float64, device=device),
                       edge_chi2=torch.zeros(E, dtype=torch.float64, device=device),
                       edge_depth_ok=torch.zeros(E, dtype=torch.uint8, device=device))
            self._keep += [q_in, t_in, x_in]
            self.inputs.append((q_in, t_in, x_in))
            self.res.append(out)
            cp = p.as_c()
            cp.pose_id = cp.point_id = None
            cp.pose_fixed = fix.data_ptr()
            cp.pose_q, cp.pose_t, cp.point_xyz = q_in.data_ptr(), t_in.data_ptr(), x_in.data_ptr()
            cp.pose_cam = None
            cp.edge_point, cp.edge_pose = dev(p.edge_point).data_ptr(), dev(p.edge_pose).data_ptr()
            cp.edge_obs, cp.edge_inv_sigma2 = dev(p.edge_obs).data_ptr(), dev(p.edge_inv_sigma2).data_ptr()
            cp.cams = dev(p.cams).data_ptr()
            cp.edge_active = None
            self.c_probs[w] = cp
            r = self.c_res[w]
            r.pose_q, r.pose_t = out["pose_q"].data_ptr(), out["pose_t"].data_ptr()
            r.point_xyz = out["point_xyz"].data_ptr()
            r.edge_chi2, r.edge_depth_ok = out["edge_chi2"].data_ptr(), out["edge_depth_ok"].data_ptr()
            for d, (q, t, x) in ((rd[w], (q_in, t_in, x_in)),
                                 (pk[w], (out["pose_q"], out["pose_t"], out["point_xyz"]))):
                d.n_poses, d.n_points = P, L
                d.pose_id, d.pose_fixed, d.point_id, d.point_bad = pid.data_ptr(), fix.data_ptr(), mid.data_ptr(), None
                d.pose_q, d.pose_t, d.point_xyz = q.data_ptr(), t.data_ptr(), x.data_ptr()
        self.max_rows = max_rows
        self.cap = cap
        self.d_read = dev(np.frombuffer(bytes(rd), np.uint8))
        self.d_pack = dev(np.frombuffer(bytes(pk), np.uint8))
        self.exch = MapUpdateExchange(capacity=self.W * (cap + 1) - 1, device=device)
        # the new keyframe of window w: its last local keyframe; its new MapPoints: those homed there
        self.new_kf = torch.tensor([min(s + n_opt - 1, self.world.n_kf - 1) for s in self.starts], device=device)
        homes = [np.nonzero(self.world.home == int(k))[0] for k in self.new_kf.cpu().numpy()]
        self.new_mp = torch.from_numpy(np.concatenate(homes).astype(np.int64)).to(device)
        self.new_mp_win = torch.from_numpy(np.concatenate([np.full(len(h), w) for w, h in enumerate(homes)])).to(device)
        self.stats = None
        self.windows_solved = 0

    @property
    def edges(self):
        return [len(p.edge_point) for p in self.probs]

    def new_keyframes(self, step: int):
        """Enter every window's new keyframe and its new MapPoints at a perturbed state (deterministic in step)."""
        import torch

        g = torch.Generator(device=self.dev)
        g.manual_seed(1_000_003 * (step + 1) + 7919 * self.rank)
        nk = self.new_kf
        dq = torch.randn((len(nk), 4), generator=g, device=self.dev) * 0.004
        q = self.kf_table[nk, :4] + dq
        q = q / q.norm(dim=1, keepdim=True)
        q = torch.where(q[:, 3:4] < 0, -q, q)
        self.kf_table[nk, :4] = q
        self.kf_table[nk, 4:7] += torch.randn((len(nk), 3), generator=g, device=self.dev) * 0.012
        self.mp_table[self.new_mp, :3] += torch.randn((len(self.new_mp), 3), generator=g, device=self.dev) * 0.017

    def run(self, step: int, new_keyframes: bool = True):
        """One LocalMapping step on self.stream (synchronous: returns when the map holds every GPU's write-backs)."""
        import torch

        with torch.cuda.stream(self.stream):
            s = self.stream.cuda_stream
            if new_keyframes:
                self.new_keyframes(step)
            self.exch.read_windows(self.kf_table.data_ptr(), self.world.n_kf, self.mp_table.data_ptr(), self.world.n_mp,
                                   self.mp_base, self.d_read.data_ptr(), self.W, self.max_rows,
                                   self.status.data_ptr(), stream=s)
            check = self.solver._L.mam_lba_solve_batch_device(self.solver._ctx, self.W, C.byref(self.c_probs),
                                                               C.byref(self.c_res), C.c_void_p(s))
            if check != 0:
                raise RuntimeError(f"mam_lba_solve_batch_device: {check}")
            self.stats = [(int(r.iterations), int(r.lm_trials), int(r.status)) for r in self.c_res]
            self.windows_solved += self.W
            self.exch.pack_windows(self.d_pack.data_ptr(), self.W, self.mp_base, self.cap, stream=s)
            self.exch.gather()
            self.exch.apply(self.kf_table.data_ptr(), self.world.n_kf, self.mp_table.data_ptr(), self.world.n_mp,
                            self.status.data_ptr(), stream=s, n_agents=self.world_size * self.W, capacity=self.cap)
        return self.stats

    def window_inputs(self, w: int):
        """Host copy of window w's LBA problem with the inputs it was last solved from (parity / CPU timing)."""
        import dataclasses

        q, t, x = self.inputs[w]
        return dataclasses.replace(self.probs[w], pose_q=q.cpu().numpy(), pose_t=t.cpu().numpy(),
                                   point_xyz=x.cpu().numpy())

    def window_result(self, w: int):
        o = {k: v.cpu().numpy() for k, v in self.res[w].items()}
        it, tr, st = self.stats[w]
        r = self.c_res[w]
        from .lba import LBAResult

        return LBAResult(o["pose_q"], o["pose_t"], o["point_xyz"], o["edge_chi2"], o["edge_depth_ok"], it, tr,
                         float(r.initial_chi2), float(r.final_chi2), st)
