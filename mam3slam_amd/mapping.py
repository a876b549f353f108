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
                 stride: int = 25, seed: int = 7, stream=None, camera=None, width: int = 1280, height: int = 720):
        import torch

        self.dev = device
        self.W = int(n_windows)
        self.rank, self.world_size = rank, world_size
        # one world for every world size (weak scaling: the same windows per GPU for any N)
        n_kf = (max_gpus * self.W + 1) * stride + n_opt + 8
        self.world = W.make_world(n_kf=n_kf, seed=seed, width=width, height=height, camera=camera)
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
        # the exchange's fixed block size must be the same on every rank (a collective over blocks of different
        # sizes fails or hangs): the largest window of any rank
        import torch.distributed as dist

        if world_size > 1 and dist.is_available() and dist.is_initialized():
            on_gpu = dist.get_backend() == "nccl"
            t = torch.tensor([cap], dtype=torch.int64, device=device if on_gpu else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cap = int(t.item())
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


class NewMapPointsLeg:
    """LocalMapping::ProcessNewKeyFrame's ComputeBoW and CreateNewMapPoints' SearchForTriangulation against the new
    keyframe's 30 neighbours (LocalMapping.cc:504-582, nn = 30 for monocular; ORBmatcher(0.6, false): no rotation
    check), for the W keyframes the agents on this GPU insert per step, on the device.

    The keyframes live in a ring of R slots in HBM (keypoints, descriptors, MapPoint flags, pose, BoW node + weight at
    levelsup 4): `ingest` copies the step's new keyframes out of the tracking buffers (on the tracking stream, after
    the step that tracked them: the reference's Tracking -> LocalMapping hand-off); `run` computes their BoW (DBoW2
    transform, synthetic k=10 L=6 vocabulary — ORBvoc.txt is a missing blob) and searches each against the 30 slots
    inserted before it (the synthetic map has no covisibility graph: the most recent keyframes stand in for the best
    covisible ones). The triangulation and MapPoint creation that follow the search (LocalMapping.cc:590-828) are
    outside the hot path; the map's new MapPoints enter through LocalMappingLeg.new_keyframes."""

    NN = 30

    def __init__(self, tr, n_new: int, device, seed: int = 0):
        import torch

        from . import bow
        from .match import FramesDev, ORBmatcher, TriBatch

        self.dev, self.tr, self.W = device, tr, int(n_new)
        # new slots + at least NN older ones + one spare group (the next ingest writes while a search may run),
        # a multiple of W
        self.R = self.W * (2 + -(-self.NN // self.W))
        R, S = self.R, tr.cap
        self.S = S
        self.keys = torch.zeros((R, S * 28), dtype=torch.uint8, device=device)
        self.desc = torch.zeros((R, S, 32), dtype=torch.uint8, device=device)
        self.cnt = torch.zeros((R, 2), dtype=torch.int32, device=device)
        self.has_mp = torch.zeros((R, S), dtype=torch.uint8, device=device)
        self.tcw = torch.zeros((R, tr.tcw_bytes), dtype=torch.uint8, device=device)
        self.nid = torch.zeros((R, S), dtype=torch.int32, device=device)
        self.weight = torch.zeros((R, S), dtype=torch.float64, device=device)
        self.word = torch.zeros((R, S), dtype=torch.int32, device=device)
        self.voc = bow.ORBVocabulary(bow.synthetic_vocabulary(10, 6, np.random.default_rng(seed), early_leaf=0.02),
                                     device=device.index or 0)
        self.matcher = ORBmatcher(0.6, False, device=device.index or 0)
        self.head = 0
        self.ready = {h: torch.cuda.Event() for h in range(0, self.R, self.W)}
        # completion of the search run at each head (None until one was issued there)
        self.done = {h: None for h in range(0, self.R, self.W)}
        self.stream = torch.cuda.Stream(device, priority=-1)
        # pairs for each head position: new slot j = head + i searches the NN slots inserted before it
        self.pairs = {}
        for head in range(0, R, self.W):
            p = []
            for i in range(self.W):
                j = (head + i) % R
                for k in range(1, self.NN + 1):
                    p.append((j, (j - k) % R))
            self.pairs[head] = torch.tensor(np.array(p, np.int32), device=device)
        self.npairs = self.W * self.NN
        self.out = torch.zeros((self.npairs, S), dtype=torch.int32, device=device)
        self.nmatch = torch.zeros(self.npairs, dtype=torch.int32, device=device)
        self._FramesDev, self._TriBatch = FramesDev, TriBatch
        # initial ring: the first R frames, BoW on the device, no MapPoints yet
        with torch.cuda.stream(tr.tstream):
            fr = torch.arange(R, device=device) % tr.B
            self.keys.copy_(tr.d_kps[fr])
            self.desc.copy_(tr.d_desc[fr])
            self.cnt.copy_(tr.d_cnt[fr])
            self.tcw.copy_(tr.d_tcw.view(tr.B, -1)[fr])
            self.voc.transform_batch_device(R, self.desc.data_ptr(), S, self.cnt.data_ptr(), 4, self.word.data_ptr(),
                                            self.weight.data_ptr(), self.nid.data_ptr(), stream=tr.tstream.cuda_stream)
            for ev in self.ready.values():
                ev.record(tr.tstream)
        self.pending = None

    def ingest(self, step: int):
        """Copy step `step`'s new keyframes (frames f = step mod K + i K) into the ring at the next head; on the
        tracking stream after the tracking step. Their BoW is computed by the next `run`."""
        import torch

        tr, W, R = self.tr, self.W, self.R
        K = max(1, tr.B // W)
        head = (self.head + W) % R   # the run at self.head was launched right after its ingest
        fr = (torch.arange(W, device=self.dev) * K + step % K) % tr.B
        sl = slice(head, head + W)
        # the latest search that read these slots is the one two heads back (R >= 2 W + NN): it must be done
        prev = self.done[(head - 2 * W) % R]
        with torch.cuda.stream(tr.tstream):
            if prev is not None:
                tr.tstream.wait_event(prev)
            self.keys[sl] = tr.d_kps[fr]
            self.desc[sl] = tr.d_desc[fr]
            self.cnt[sl] = tr.d_cnt[fr]
            self.tcw[sl] = tr.d_tcw.view(tr.B, -1)[fr]
            # GetMapPoint(i) != NULL: the keypoints Tracking matched (motion model or local map)
            self.has_mp[sl] = ((tr.d_out1[fr] >= 0) | (tr.d_out2[fr] >= 0)).to(torch.uint8)
            self.ready[head].record(tr.tstream)
        self.pending = head

    def take(self):
        """The ring head of the keyframes ingested since the last take (None if none): the next run's work. Called
        by the thread that starts the run, so a run never sees a later ingest."""
        h, self.pending = self.pending, None
        return h

    def launch(self, head):
        """Start the run of the keyframes ingested at `head` on this leg's own stream as soon as they are ingested (a
        search of one step's keyframes overlaps the LocalBundleAdjustment of the previous step's: different agents'
        keyframes, as with the reference's per-agent LocalMapping threads); `wait(stream, head)` orders a consumer of
        the same keyframes after it."""
        import torch

        self.run(self.stream, head)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.done[head] = ev

    def wait(self, stream, head):
        if head is not None and self.done[head] is not None:
            stream.wait_event(self.done[head])

    def run(self, stream, head):
        """ComputeBoW of the new keyframes at `head` + their W x 30 SearchForTriangulation, asynchronous on
        `stream`."""
        if head is None:
            return
        stream.wait_event(self.ready[head])
        self.head = head
        W, S, h = self.W, self.S, self.head
        s = stream.cuda_stream
        self.voc.transform_batch_device(W, self.desc[h].data_ptr(), S, self.cnt[h].data_ptr(), 4,
                                        self.word[h].data_ptr(), self.weight[h].data_ptr(), self.nid[h].data_ptr(),
                                        stream=s)
        b = self._TriBatch()
        b.kfs = self._FramesDev(self.R, S, self.keys.data_ptr(), self.desc.data_ptr(), self.cnt.data_ptr(), None, None, 0)
        b.has_mp, b.nid, b.weight = self.has_mp.data_ptr(), self.nid.data_ptr(), self.weight.data_ptr()
        b.tcw = self.tcw.data_ptr()
        pairs = self.pairs[h]
        b.npairs, b.pairs = int(pairs.shape[0]), pairs.data_ptr()
        self.matcher.search_for_triangulation_batch_device(self.tr.F0, self.tr.cam, b, self.out.data_ptr(),
                                                           self.nmatch.data_ptr(), False, stream=s)

    def algorithmic_bytes(self):
        """SURVEY §8(d) bytes of the last run's searches: per pair, sum over the BoW nodes both FeatureVectors hold of
        |f1| x |f2| descriptor pairs x 32 B, plus per FeatureVector feature its sorted key (8 B), MapPoint flag (1 B),
        keypoint (28 B) and descriptor (32 B) once."""
        nid = self.nid.cpu().numpy().view(np.uint32)
        w = self.weight.cpu().numpy()
        cnt = self.cnt.cpu().numpy()[:, 0]
        per_slot = []
        for k in range(self.R):
            n = int(min(max(cnt[k], 0), self.S))
            v = nid[k, :n][w[k, :n] > 0]
            u, c = np.unique(v, return_counts=True)
            per_slot.append(dict(zip(u.tolist(), c.tolist())))
        cand, fv = 0, 0
        for a, b in self.pairs[self.head].cpu().numpy():
            A, B = per_slot[a], per_slot[b]
            cand += sum(c * B[u] for u, c in A.items() if u in B)
            fv += sum(A.values()) + sum(B.values())
        return {"candidate_pairs": int(cand), "bytes": int(cand * 32 + fv * (8 + 1 + 28 + 32))}

    def pair_inputs(self, q: int):
        """Host FrameData of pair q of the last run (keys, desc, has_mp, FeatureVector from the device BoW, pose)."""
        from .match import FrameData
        from .orb import KP_DTYPE

        out = []
        for slot in self.pairs[self.head][q].cpu().numpy():
            n = int(self.cnt[slot, 0].item())
            keys = self.keys[slot].cpu().numpy().view(KP_DTYPE)[:n]
            F = FrameData(keys=keys, desc=self.desc[slot, :n].cpu().numpy(), width=self.tr.W, height=self.tr.H,
                          scale_factors=self.tr.F0.scale_factors, level_sigma2=self.tr.F0.level_sigma2)
            F.has_mp = self.has_mp[slot, :n].cpu().numpy()
            nid, w = self.nid[slot, :n].cpu().numpy(), self.weight[slot, :n].cpu().numpy()
            fv = {}
            for i in range(n):
                if w[i] > 0:
                    fv.setdefault(int(np.uint32(nid[i])), []).append(i)
            F.featvec = dict(sorted(fv.items()))
            t = self.tcw[slot].cpu().numpy().view(np.float32)
            F.pose = (t[:4].copy(), t[4:7].copy())
            out.append(F)
        return out
