"""The LocalMapping leg of a multi-agent step on one GPU: LocalBundleAdjustment of the new keyframes' windows over a
shared map resident in HBM, and the exchange that keeps the map identical on every GPU.

Per step (one call of `run`), for the W keyframes the agents on this GPU inserted:
  1. `new_keyframes`: each window's newest keyframe enters the map at the motion model's guess and its new MapPoints
     at their first triangulation (a deterministic perturbation of those map entries) — the work a new keyframe
     brings to LocalMapping (LocalMapping.cc:162-172 runs one LBA per processed keyframe);
  2. the windows' vertex estimates are read from the shared map tables (mam_map_read_windows: the graph build of
     Optimizer.cc:1218-1286 takes the float map values cast to double);
  3. all W LocalBundleAdjustment solves run together (mam_lba_solve_batch_device: Levenberg control on the device);
  4. the write-backs (Optimizer.cc:1463-1497) of all W windows are packed as one deduplicated block per GPU
     (mam_exchange_pack_sources: every optimised KeyFrame and MapPoint once, from the last window holding it, in
     32-byte / 16-byte records), all-gathered across GPUs (RCCL over xGMI) and applied in GPU order to the map every
     GPU holds — which the next step's windows read. Overlapping windows (shared keyframes / MapPoints) resolve
     deterministically: the later window within a GPU, the higher GPU across GPUs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import world as W
from .exchange import CompactExchange, MapWindow, dedup_sources
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
        max_rows = 0

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
        # the write-back of all W windows as one deduplicated record set (every optimised KeyFrame / MapPoint once, from
        # the last window holding it), and the exchange's fixed block size: it must be the same on every rank (a
        # collective over blocks of different sizes fails or hangs), the largest of any rank
        kf_src, mp_src = dedup_sources([(p.pose_id, p.pose_fixed, p.point_id) for p in self.probs])
        self.n_kf_upd, self.n_mp_upd = len(kf_src), len(mp_src)
        self.d_kf_src, self.d_mp_src = dev(kf_src), dev(mp_src)
        caps = [self.n_kf_upd, self.n_mp_upd]
        import torch.distributed as dist

        if world_size > 1 and dist.is_available() and dist.is_initialized():
            on_gpu = dist.get_backend() == "nccl"
            t = torch.tensor(caps, dtype=torch.int64, device=device if on_gpu else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            caps = [int(v) for v in t.tolist()]
        self.d_read = dev(np.frombuffer(bytes(rd), np.uint8))
        self.d_pack = dev(np.frombuffer(bytes(pk), np.uint8))
        self.exch = CompactExchange(caps[0], caps[1], device=device)
        self.time_gather = False
        # the new keyframe of window w: its last local keyframe; its new MapPoints: those homed there
        self.new_kf = torch.tensor([min(s + n_opt - 1, self.world.n_kf - 1) for s in self.starts], device=device)
        homes = [np.nonzero(self.world.home == int(k))[0] for k in self.new_kf.cpu().numpy()]
        self.new_mp = torch.from_numpy(np.concatenate(homes).astype(np.int64)).to(device)
        self.new_mp_win = torch.from_numpy(np.concatenate([np.full(len(h), w) for w, h in enumerate(homes)])).to(device)
        self.stats = None
        self.windows_solved = 0
        self.host_s = {}

    @property
    def edges(self):
        return [len(p.edge_point) for p in self.probs]

    def new_keyframes(self, step: int):
        """Enter every window's new keyframe and its new MapPoints at a perturbed state (deterministic in step)."""
        # one HIP launch (mam_map_perturb): q + N(0, 0.004) renormalised with w >= 0, t + N(0, 0.012), new MapPoints +
        # N(0, 0.017), counter-based normals seeded by (step, rank)
        import torch

        from .exchange import map_perturb

        # on torch's current stream (run() makes it self.stream): ordered with the caller's tensor reads
        map_perturb(self.kf_table.data_ptr(), self.world.n_kf, self.new_kf.data_ptr(), len(self.new_kf),
                    self.mp_table.data_ptr(), self.world.n_mp, self.new_mp.data_ptr(), len(self.new_mp),
                    1_000_003 * (step + 1) + 7919 * self.rank, 0.004, 0.012, 0.017, self.status.data_ptr(),
                    stream=torch.cuda.current_stream(self.dev).cuda_stream)

    def run(self, step: int, head=None, new_keyframes: bool = True):
        """One LocalMapping step (head: unused, the ring leg's argument): the solves are synchronous (mam_lba_solve_batch_device returns with the Levenberg
        state read back), the pack / all-gather / apply are queued: on return the map tables are final for work
        ordered after self.stream (a consumer on another stream waits on it)."""
        import time

        import torch

        with torch.cuda.stream(self.stream):
            t0 = time.perf_counter()
            s = self.stream.cuda_stream
            if new_keyframes:
                self.new_keyframes(step)
            self.exch.read_windows(self.kf_table.data_ptr(), self.world.n_kf, self.mp_table.data_ptr(), self.world.n_mp,
                                   self.mp_base, self.d_read.data_ptr(), self.W, self.max_rows,
                                   self.status.data_ptr(), stream=s)
            t1 = time.perf_counter()
            check = self.solver._L.mam_lba_solve_batch_device(self.solver._ctx, self.W, C.byref(self.c_probs),
                                                               C.byref(self.c_res), C.c_void_p(s))
            t2 = time.perf_counter()
            if check != 0:
                raise RuntimeError(f"mam_lba_solve_batch_device: {check}")
            self.stats = [(int(r.iterations), int(r.lm_trials), int(r.status)) for r in self.c_res]
            self.windows_solved += self.W
            self.exch.pack(self.d_pack.data_ptr(), self.W, self.d_kf_src.data_ptr(), self.n_kf_upd,
                           self.d_mp_src.data_ptr(), self.n_mp_upd, self.mp_base, stream=s)
            self.exch.gather(timed=self.time_gather)
            self.exch.apply(self.kf_table.data_ptr(), self.world.n_kf, self.mp_table.data_ptr(), self.world.n_mp,
                            self.status.data_ptr(), stream=s)
            t3 = time.perf_counter()
        # host wall per phase (the solve returns after its last read-back: it includes the GPU time of everything
        # queued before it on the stream — the keyframe searches it waits for)
        for k, v in (("launch", t1 - t0), ("solve", t2 - t1), ("exchange", t3 - t2)):
            self.host_s[k] = self.host_s.get(k, 0.0) + v
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
    transform, synthetic k=10 L=6 vocabulary — ORBvoc.txt is a missing blob) and searches each against its 30
    neighbours (the synthetic map has no covisibility graph: the keyframes nearest in the agent's frame sequence stand
    in for the best covisible ones; the keyframes' poses are those of the camera that rendered them,
    synth.frame_pose, refined by Tracking's PoseOptimization); then SearchInNeighbors (LocalMapping.cc:830-939):
    Fuse of the keyframe's MapPoints into its 30 neighbours, Fuse of the neighbours' fuse candidates into the keyframe
    and ComputeDistinctiveDescriptors of its MapPoints (`search_in_neighbors`). The triangulation and MapPoint creation that follow the search (LocalMapping.cc:590-828) are
    outside the hot path; the map's new MapPoints enter through LocalMappingLeg.new_keyframes."""

    NN = 30

    def __init__(self, tr, n_new: int, device, seed: int = 0, stream=None):
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
        self.stream = stream if stream is not None else torch.cuda.Stream(device, priority=-1)
        # pairs for each head position. With at least NN + 1 keyframes per ingest (c2: 32), new keyframe i (frame
        # i K + s of the agent's sequence) searches the NN keyframes of the same ingest nearest to it in the sequence
        # (frames i' K + s, |i - i'| smallest, earlier first on a tie): the covisible keyframes
        # GetBestCovisibilityKeyFrames(30) returns for a camera moving through one scene. With fewer, slot j = head + i
        # searches the NN slots inserted before it.
        self.pairs = {}
        for head in range(0, R, self.W):
            p = []
            for i in range(self.W):
                j = (head + i) % R
                if self.W > self.NN:
                    near = sorted((x for x in range(self.W) if x != i), key=lambda x: (abs(x - i), x))[:self.NN]
                    p += [(j, (head + x) % R) for x in near]
                else:
                    p += [(j, (j - k) % R) for k in range(1, self.NN + 1)]
            self.pairs[head] = torch.tensor(np.array(p, np.int32), device=device)
        self.npairs = self.W * self.NN
        self.out = torch.zeros((self.npairs, S), dtype=torch.int32, device=device)
        self.nmatch = torch.zeros(self.npairs, dtype=torch.int32, device=device)
        self._init_search_in_neighbors(seed)
        self._FramesDev, self._TriBatch = FramesDev, TriBatch
        # initial ring: the first R frames, BoW on the device, no MapPoints yet
        with torch.cuda.stream(tr.tstream):
            fr = torch.arange(R, device=device) % (tr.P * tr.B)   # the pool's frames in order, at their guessed poses
            self.keys.copy_(tr.d_kps_pool[fr])
            self.desc.copy_(tr.d_desc_pool[fr])
            self.cnt.copy_(tr.d_cnt_pool[fr])
            self.tcw.copy_(tr.d_tcw_init_pool.view(tr.P * tr.B, -1)[fr])
            self.fmp.copy_(self.fmp_frames[fr])
            self.cnt_col.copy_(self.cnt[:, 0])
            self.voc.transform_batch_device(R, self.desc.data_ptr(), S, self.cnt.data_ptr(), 4, self.word.data_ptr(),
                                            self.weight.data_ptr(), self.nid.data_ptr(), stream=tr.tstream.cuda_stream)
            for ev in self.ready.values():
                ev.record(tr.tstream)
        self.pending = None
        self.ring = None   # a RingMappingLeg assembling each run's LocalBundleAdjustment windows

    def ingest(self, step: int):
        """Copy step `step`'s new keyframes (frames f = step mod K + i K) into the ring at the next head; on the
        tracking stream after the tracking step. Their BoW is computed by the next `run`."""
        tr, W, R = self.tr, self.W, self.R
        K = max(1, tr.B // W)
        head = (self.head + W) % R   # the run at self.head was launched right after its ingest
        fr = [(i * K + step % K) % tr.B for i in range(W)]
        # the latest search that read these slots is the one two heads back (R >= 2 W + NN): it must be done
        prev = self.done[(head - 2 * W) % R]
        if prev is not None:
            tr.tstream.wait_event(prev)
        # one launch (mam_copy_rows): keypoints, descriptors, counts, pose, MapPoints of the frames (the pool set just
        # tracked), and GetMapPoint(i) != NULL — the keypoints Tracking matched (motion model or local map)
        self._ingest_rows(tr, fr, list(range(head, head + W)), tr.p * tr.B, tr.tstream.cuda_stream)
        self.ready[head].record(tr.tstream)
        self.pending = head

    def _ingest_rows(self, tr, fr, slots, fmp_offset, stream, flags=True):
        from .exchange import copy_rows

        S = self.S
        tables = [(tr.d_kps.data_ptr(), self.keys.data_ptr(), S * 28, S * 28, S * 28, 0),
                  (tr.d_desc.data_ptr(), self.desc.data_ptr(), S * 32, S * 32, S * 32, 0),
                  (tr.d_cnt.data_ptr(), self.cnt.data_ptr(), 8, 8, 8, 0),
                  (tr.d_cnt.data_ptr(), self.cnt_col.data_ptr(), 4, 8, 4, 0),
                  (tr.d_tcw.data_ptr(), self.tcw.data_ptr(), tr.tcw_bytes, tr.tcw_bytes, tr.tcw_bytes, 0),
                  (self.fmp_frames.data_ptr(), self.fmp.data_ptr(), self.fmp.shape[1], self.fmp_frames.shape[1],
                   self.fmp.shape[1], fmp_offset)]
        fl = (tr.d_out1.data_ptr(), tr.d_out2.data_ptr(), 4 * tr.cap, S, self.has_mp.data_ptr(), S) if flags else None
        for i in range(0, len(fr), 64):
            copy_rows(tables, fr[i:i + 64], slots[i:i + 64], fl, stream=stream)

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
        self.search_in_neighbors(stream, h)
        if self.ring is not None:   # the LocalBundleAdjustment windows of these keyframes (RingMappingLeg)
            self.ring.assemble(stream, h)

    # ------------------------------------------------------------------------------------------ SearchInNeighbors
    NB_BACK = 4   # neighbours whose MapPoints form a keyframe's fuse candidates

    def _init_search_in_neighbors(self, seed):
        """MapPoints of every tracked frame (the ring copies them with the keyframe) and the update's observation
        descriptors. A keyframe's MapPoints: its keypoints on the scene plane (synth.PLANE_DEPTH, world coordinates
        under the pose of the camera that rendered the frame), as MapPoint::UpdateNormalAndDepth leaves them
        (MapPoint.cc:426-494: normal = viewing direction, mfMaxDistance = distance x scale factor of the keypoint's
        level, mfMinDistance = mfMaxDistance / scale factor of the last level), descriptor = the keypoint's."""
        import torch

        from . import synth
        from .match import FUSE_MP_DTYPE, quat_to_rot

        tr, S = self.tr, self.S
        sf = tr.F0.scale_factors.astype(np.float64)
        # every frame of the tracking leg's frame pool (P sets of B: tr.pool)
        pool = tr.pool
        nfr = len(pool["poses"])
        fmp = np.zeros((nfr, S), FUSE_MP_DTYPE)
        desc_h = pool["desc_h"]
        for f in range(nfr):
            n = int(pool["cnt_h"][f, 0])
            k = pool["kps_h"][f, :n]
            q, t = pool["poses"][f]
            R = quat_to_rot(q).astype(np.float64)
            Ow = -R.T @ t.astype(np.float64)
            ray_c = np.concatenate([tr.cam.unproject_np(k["x"], k["y"]), np.ones((n, 1))], 1)
            ray_w = ray_c @ R   # R^T d
            sc = (synth.PLANE_DEPTH - Ow[2]) / ray_w[:, 2]
            X = Ow[None, :] + sc[:, None] * ray_w
            d = X - Ow[None, :]
            dist = np.linalg.norm(d, axis=1)
            m = fmp[f, :n]
            m["pos"] = X.astype(np.float32)
            m["normal"] = (d / dist[:, None]).astype(np.float32)
            m["max_distance"] = (dist * sf[k["octave"]]).astype(np.float32)
            m["min_distance"] = (m["max_distance"] / np.float32(sf[-1])).astype(np.float32)
            m["valid"] = 1
            m["desc"] = desc_h[f, :n]
        self.fmp_frames = torch.from_numpy(fmp.view(np.uint8).reshape(nfr, -1)).to(self.dev)
        self.fmp = torch.zeros((self.R, S * FUSE_MP_DTYPE.itemsize), dtype=torch.uint8, device=self.dev)
        self.cnt_col = torch.zeros(self.R, dtype=torch.int32, device=self.dev)
        W, NN, NBK = self.W, self.NN, self.NB_BACK
        # items per ring head: forward (slot's MapPoints -> each of its NN neighbours), backward (the NB_BACK nearest
        # neighbours' MapPoints -> the slot)
        self.sin_items = {}
        for head, pr in self.pairs.items():
            pr = pr.cpu().numpy()
            fwd_frame, fwd_mp = pr[:, 1], pr[:, 0]
            bwd_frame = np.repeat(pr[::NN, 0], NBK)
            bwd_mp = pr.reshape(W, NN, 2)[:, :NBK, 1].reshape(-1)
            self.sin_items[head] = tuple(torch.tensor(np.ascontiguousarray(a, np.int32), device=self.dev)
                                         for a in (fwd_frame, fwd_mp, bwd_frame, bwd_mp))
        nf, nb = W * NN, W * NBK
        self.fwd_idx = torch.zeros((nf, S), dtype=torch.int32, device=self.dev)
        self.fwd_dist = torch.zeros((nf, S), dtype=torch.int32, device=self.dev)
        self.fwd_n = torch.zeros(nf, dtype=torch.int32, device=self.dev)
        self.bwd_idx = torch.zeros((nb, S), dtype=torch.int32, device=self.dev)
        self.bwd_dist = torch.zeros((nb, S), dtype=torch.int32, device=self.dev)
        self.bwd_n = torch.zeros(nb, dtype=torch.int32, device=self.dev)
        # update: the W keyframes' MapPoints, 2..12 observations each, the observing keypoints' descriptors (the
        # keyframe's with up to 20 flipped bits: views of the point from other keyframes)
        from .scene import flip_bits

        rng = np.random.default_rng(seed + 11)
        n_upd = int(sum(int(tr.cnt_h[f % tr.B, 0]) for f in range(W)))
        sizes = rng.integers(2, 13, n_upd)
        off = np.zeros(n_upd + 1, np.int32)
        off[1:] = np.cumsum(sizes)
        base = np.concatenate([desc_h[f % tr.B, :int(tr.cnt_h[f % tr.B, 0])] for f in range(W)])
        descs = flip_bits(np.repeat(base, sizes, 0), rng, 20)
        self.upd_n = n_upd
        self.upd_off = torch.from_numpy(off).to(self.dev)
        self.upd_desc = torch.from_numpy(descs).to(self.dev)
        self.upd_best = torch.zeros(n_upd, dtype=torch.int32, device=self.dev)

    def search_in_neighbors(self, stream, head):
        """SearchInNeighbors of the keyframes at `head` (after their CreateNewMapPoints searches, on `stream`):
        forward Fuse of each keyframe's MapPoints into its NN neighbours, backward Fuse of its NB_BACK nearest
        neighbours' MapPoints (the fuse candidates) into it, ComputeDistinctiveDescriptors of the keyframes' MapPoints
        (UpdateNormalAndDepth and the map updates Fuse implies are host-side bookkeeping, not searched)."""
        fwd_frame, fwd_mp, bwd_frame, bwd_mp = self.sin_items[head]
        s = stream.cuda_stream
        fr = self._FramesDev(self.R, self.S, self.keys.data_ptr(), self.desc.data_ptr(), self.cnt.data_ptr(), None,
                             None, 0)
        tcw = self.tcw.data_ptr()
        import torch

        m = self.matcher   # (cnt_col: MapPoints of list m = ring slot m's keypoints, kept by the ingest)
        m.fuse_items_batch_device(self.tr.F0, fr, tcw, self.tr.cam, len(fwd_frame), fwd_frame.data_ptr(),
                                  fwd_mp.data_ptr(), self.fmp.data_ptr(), self.S, self.cnt_col.data_ptr(), 3.0,
                                  self.fwd_idx.data_ptr(), self.fwd_dist.data_ptr(), self.fwd_n.data_ptr(), stream=s)
        m.fuse_items_batch_device(self.tr.F0, fr, tcw, self.tr.cam, len(bwd_frame), bwd_frame.data_ptr(),
                                  bwd_mp.data_ptr(), self.fmp.data_ptr(), self.S, self.cnt_col.data_ptr(), 3.0,
                                  self.bwd_idx.data_ptr(), self.bwd_dist.data_ptr(), self.bwd_n.data_ptr(), stream=s)
        m.distinctive_batch_device(self.upd_n, self.upd_off.data_ptr(), self.upd_desc.data_ptr(),
                                   self.upd_best.data_ptr(), stream=s)

    def fuse_inputs(self, backward: bool, b: int):
        """Host (KeyFrame FrameData with pose, MapPoints) of forward / backward Fuse item b of the last run."""
        from .match import FUSE_MP_DTYPE, FrameData
        from .orb import KP_DTYPE

        fwd_frame, fwd_mp, bwd_frame, bwd_mp = self.sin_items[self.head]
        slot = int((bwd_frame if backward else fwd_frame)[b].item())
        ms = int((bwd_mp if backward else fwd_mp)[b].item())
        n = int(self.cnt[slot, 0].item())
        keys = self.keys[slot].cpu().numpy().view(KP_DTYPE)[:n]
        KF = FrameData(keys=keys, desc=self.desc[slot, :n].cpu().numpy(), width=self.tr.W, height=self.tr.H,
                       scale_factors=self.tr.F0.scale_factors, level_sigma2=self.tr.F0.level_sigma2)
        t = self.tcw[slot].cpu().numpy().view(np.float32)
        KF.pose = (t[:4].copy(), t[4:7].copy())
        nm = int(self.cnt[ms, 0].item())
        mps = self.fmp[ms].cpu().numpy().view(FUSE_MP_DTYPE)[:nm]
        return KF, mps

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


class RingWindow(C.Structure):
    """mam_ring_window: one assembled window's device arrays."""
    _fields_ = [("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("pose_fixed", C.c_void_p), ("point_xyz", C.c_void_p),
                ("edge_point", C.c_void_p), ("edge_pose", C.c_void_p), ("edge_obs", C.c_void_p),
                ("edge_inv_sigma2", C.c_void_p), ("edge_active", C.c_void_p)]


class RingLBA:
    """LocalBundleAdjustment over the keyframes Tracking inserted (Optimizer.cc:1118-1331 on the NewMapPointsLeg ring):
    per new keyframe of the last run, its window solved with the batch device API (mam_lba_solve_batch_device).

    rule "covisibility" (the reference's window rule, mam_ring_lba_windows_covis): the new keyframe and its covisible
    ring neighbours by weight (weight = its MapPoints a neighbour observes, from the run's forward Fuse matches: >= 15
    as KeyFrame::UpdateConnections keeps them, the heaviest when none reaches it) optimised, every other neighbour
    observing one of its MapPoints fixed; the problem compacted to the real observations (sizes read back once per
    batch). The ring's searched neighbours are the new keyframe's 30 nearest in its sequence, all of them covisible in
    the synthetic scene, so the reference's rule would leave no fixed keyframe (it then skips the LBA,
    Optimizer.cc:1179-1183): the n_fixed least covisible neighbours are fixed instead, as the gauge anchor. rule "sequence" (mam_ring_lba_windows): the NN neighbours nearest in sequence, the last n_fixed of them
    fixed, a fixed S x (NN + 1) edge-slot shape with unobserved slots inactive."""

    COVIS_TH = 15

    def __init__(self, nm, n_fixed: int = 10, iterations: int = 10, solver=None, rule: str = "covisibility",
                 sets: int = 1):
        import torch

        from .lba import HUBER_MONO

        if rule not in ("covisibility", "sequence"):
            raise ValueError(rule)
        self.nm, self.dev, self.rule = nm, nm.dev, rule
        W, NN, S = nm.W, nm.NN, nm.S
        self.NV, self.n_fixed = NN + 1, int(n_fixed)
        NV, E = self.NV, S * (NN + 1)
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=self.dev)  # noqa: E731
        cam = nm.tr.cam
        self.cams = torch.from_numpy(np.ascontiguousarray(cam.params(), np.float32)[None]).to(self.dev)
        # `sets` buffer sets (a window batch each: a set assembled while an earlier one is solved)
        self.sets = []
        for _ in range(max(1, int(sets))):
            bufs = []
            wins = (RingWindow * W)()
            c_probs = (_Problem * W)()
            c_res = (_Result * W)()
            for w in range(W):
                b = dict(pose_q=z((NV, 4), torch.float64), pose_t=z((NV, 3), torch.float64),
                         pose_fixed=z(NV, torch.uint8), point_xyz=z((S, 3), torch.float64),
                         edge_point=z(E, torch.int32), edge_pose=z(E, torch.int32), edge_obs=z((E, 2), torch.float64),
                         edge_inv_sigma2=z(E, torch.float64), edge_active=z(E, torch.uint8),
                         out_q=z((NV, 4), torch.float64), out_t=z((NV, 3), torch.float64),
                         out_xyz=z((S, 3), torch.float64), out_chi2=z(E, torch.float64), out_depth=z(E, torch.uint8))
                bufs.append(b)
                for f in RingWindow._fields_:
                    setattr(wins[w], f[0], b[f[0]].data_ptr())
                P = c_probs[w]
                P.n_poses, P.n_points, P.n_edges, P.n_cams = NV, S, E, 1
                P.pose_id = P.point_id = P.pose_cam = None
                P.pose_fixed, P.pose_q, P.pose_t = b["pose_fixed"].data_ptr(), b["pose_q"].data_ptr(), b["pose_t"].data_ptr()
                P.point_xyz = b["point_xyz"].data_ptr()
                P.edge_point, P.edge_pose = b["edge_point"].data_ptr(), b["edge_pose"].data_ptr()
                P.edge_obs, P.edge_inv_sigma2 = b["edge_obs"].data_ptr(), b["edge_inv_sigma2"].data_ptr()
                P.edge_active = b["edge_active"].data_ptr() if rule == "sequence" else None
                P.cams = self.cams.data_ptr()
                P.huber_delta, P.iterations = HUBER_MONO, int(iterations)
                P.cam_model = 1 if cam.is_kb8 else 0
                P.n_opt_poses = NV - self.n_fixed
                R = c_res[w]
                R.pose_q, R.pose_t, R.point_xyz = b["out_q"].data_ptr(), b["out_t"].data_ptr(), b["out_xyz"].data_ptr()
                R.edge_chi2, R.edge_depth_ok = b["out_chi2"].data_ptr(), b["out_depth"].data_ptr()
            st = dict(bufs=bufs, c_probs=c_probs, c_res=c_res,
                      d_wins=torch.from_numpy(np.frombuffer(bytes(wins), np.uint8).copy()).to(self.dev),
                      # covisibility windows: per window {poses, points, edges, optimised poses}, the ring slot of
                      # each pose, the new keyframe's keypoint of each point (device), and the host copy of the first two
                      counts=z((W, 4), torch.int32), pose_slot=z((W, NV), torch.int32), point_src=z((W, S), torch.int32),
                      meta_h=torch.zeros((W, 4 + NV), dtype=torch.int32).pin_memory(), sizes=None, slots=None,
                      stats=None)
            self.sets.append(st)
        self.cur = 0   # the set window() / result() / stats describe: the last solved
        s2 = np.asarray(nm.tr.F0.level_sigma2, np.float32)
        self.inv_s2 = (C.c_float * len(s2))(*[float(np.float32(1.0) / x) for x in s2])
        self.nlevels = len(s2)
        self.solver = solver or LBASolver(device=self.dev.index or 0)

    # the last solved set's views (what ring_lba_section and the tests read)
    @property
    def bufs(self):
        return self.sets[self.cur]["bufs"]

    @property
    def c_probs(self):
        return self.sets[self.cur]["c_probs"]

    @property
    def c_res(self):
        return self.sets[self.cur]["c_res"]

    @property
    def sizes(self):
        return self.sets[self.cur]["sizes"]

    @property
    def stats(self):
        return self.sets[self.cur]["stats"]

    @property
    def pose_slot(self):
        return self.sets[self.cur]["pose_slot"]

    @property
    def point_src(self):
        return self.sets[self.cur]["point_src"]

    def assemble(self, stream, set_index: int = 0):
        """The windows of the keyframes of the leg's last run (after its search_in_neighbors on `stream`)."""
        from ._lib import check
        from .exchange import _bind

        nm, st = self.nm, self.sets[set_index]
        if self.rule == "covisibility":
            check(_bind().mam_ring_lba_windows_covis(
                nm.W, nm.pairs[nm.head].data_ptr(), nm.NN, self.COVIS_TH, self.n_fixed, nm.keys.data_ptr(),
                nm.cnt.data_ptr(), nm.tcw.data_ptr(), nm.fmp.data_ptr(), nm.S, nm.fwd_idx.data_ptr(), self.inv_s2,
                self.nlevels, st["d_wins"].data_ptr(), st["counts"].data_ptr(), st["pose_slot"].data_ptr(),
                st["point_src"].data_ptr(), stream.cuda_stream), "mam_ring_lba_windows_covis")
        else:
            check(_bind().mam_ring_lba_windows(nm.W, nm.pairs[nm.head].data_ptr(), nm.NN, self.n_fixed, nm.keys.data_ptr(), nm.cnt.data_ptr(),
                     nm.tcw.data_ptr(), nm.fmp.data_ptr(), nm.S, nm.fwd_idx.data_ptr(), self.inv_s2, self.nlevels,
                     st["d_wins"].data_ptr(), stream.cuda_stream), "mam_ring_lba_windows")

    def solve(self, stream, set_index: int = 0):
        import torch

        st = self.sets[set_index]
        if self.rule == "covisibility":
            # the compacted sizes and the pose slots: one small read-back (the problem descriptors are host structs)
            with torch.cuda.stream(stream):
                st["meta_h"][:, :4].copy_(st["counts"], non_blocking=True)
                st["meta_h"][:, 4:].copy_(st["pose_slot"], non_blocking=True)
            stream.synchronize()
            meta = st["meta_h"].numpy()
            st["sizes"], st["slots"] = meta[:, :4].copy(), meta[:, 4:].copy()
            for w in range(self.nm.W):
                P = st["c_probs"][w]
                P.n_poses, P.n_points, P.n_edges, P.n_opt_poses = (int(v) for v in st["sizes"][w])
            # a window with no local MapPoint observed twice, or no fixed keyframe, is not solved — the reference's
            # LocalBundleAdjustment returns there (Optimizer.cc:1179-1183); its sizes are zeroed
            sz = st["sizes"]
            valid = [w for w in range(self.nm.W) if sz[w, 1] > 0 and sz[w, 2] > 0 and sz[w, 0] > sz[w, 3]]
            for w in range(self.nm.W):
                if w not in valid:
                    sz[w] = 0
                    P = st["c_probs"][w]
                    P.n_poses = P.n_points = P.n_edges = P.n_opt_poses = 0
        else:
            valid = list(range(self.nm.W))
        st["valid"] = valid
        stats = [(0, 0, 0)] * self.nm.W
        if valid:
            if len(valid) == self.nm.W:
                probs, res = st["c_probs"], st["c_res"]
            else:
                probs = (_Problem * len(valid))(*[st["c_probs"][w] for w in valid])
                res = (_Result * len(valid))(*[st["c_res"][w] for w in valid])
            rc = self.solver._L.mam_lba_solve_batch_device(self.solver._ctx, len(valid), C.byref(probs),
                                                           C.byref(res), C.c_void_p(stream.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"mam_lba_solve_batch_device: {rc}")
            for i, w in enumerate(valid):
                if res is not st["c_res"]:
                    st["c_res"][w] = res[i]
                r = st["c_res"][w]
                stats[w] = (int(r.iterations), int(r.lm_trials), int(r.status))
        st["stats"] = stats
        self.cur = set_index
        return stats

    def _size(self, w: int):
        P = self.c_probs[w]
        return int(P.n_poses), int(P.n_points), int(P.n_edges)

    def window(self, w: int):
        """Host LBAProblem of window w as assembled (ids = array order; the compacted prefix of the buffers)."""
        from .lba import HUBER_MONO, LBAProblem

        b = {k: v.cpu().numpy() for k, v in self.bufs[w].items()}
        P, L, E = self._size(w)
        act = b["edge_active"][:E] if self.rule == "sequence" else None
        return LBAProblem(pose_id=np.arange(P, dtype=np.int64), pose_fixed=b["pose_fixed"][:P], pose_q=b["pose_q"][:P],
                          pose_t=b["pose_t"][:P], point_id=np.arange(L, dtype=np.int64) + P,
                          point_xyz=b["point_xyz"][:L], edge_point=b["edge_point"][:E], edge_pose=b["edge_pose"][:E],
                          edge_obs=b["edge_obs"][:E], edge_inv_sigma2=b["edge_inv_sigma2"][:E],
                          cams=self.cams.cpu().numpy(), huber_delta=HUBER_MONO, iterations=int(self.c_probs[w].iterations),
                          edge_active=act, cam_model=int(self.c_probs[w].cam_model)).contiguous()

    def result(self, w: int):
        b = self.bufs[w]
        r = self.c_res[w]
        P, L, _ = self._size(w)
        return (b["out_q"].cpu().numpy()[:P], b["out_t"].cpu().numpy()[:P], b["out_xyz"].cpu().numpy()[:L],
                int(r.iterations), int(r.lm_trials), int(r.status), float(r.initial_chi2), float(r.final_chi2))


class RingMappingLeg:
    """The LocalMapping leg over the keyframes Tracking inserted: per step, the LocalBundleAdjustment windows of the
    keyframes whose searches the NewMapPointsLeg ran (RingLBA, the reference's window rule, assembled on the
    NewMapPointsLeg's stream right after those searches, one buffer set per ring head), solved together
    (mam_lba_solve_batch_device), and their write-back (Optimizer.cc:1463-1497) exchanged: every optimised KeyFrame
    once (the last window optimising it) and every window's MapPoints as 32-byte / 16-byte records
    (mam_exchange_pack_sources), one all-gather across GPUs, applied in rank order to the shared map every GPU holds
    (rows: rank x ring slot for KeyFrames, (rank x ring slot) x S + keypoint for MapPoints).

    The interface of LocalMappingLeg (bench.py reads the same fields)."""

    def __init__(self, nm, rank: int, world_size: int, device, iterations: int = 10, stream=None):
        import torch
        import torch.distributed as dist

        from .exchange import CompactExchange, MapWindow

        self.nm, self.dev = nm, device
        self.W, self.rank, self.world_size = nm.W, rank, world_size
        self.nheads = nm.R // nm.W
        self.rl = RingLBA(nm, iterations=iterations, sets=self.nheads)
        nm.ring = self   # the NewMapPointsLeg assembles each run's windows right after its searches
        self.solver = self.rl.solver
        self.stream = stream if stream is not None else torch.cuda.Stream(device, priority=-1)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        NV, S, R = self.rl.NV, nm.S, nm.R
        # the shared map every GPU holds: KeyFrame rows [q xyzw, t, valid], MapPoint rows [xyz, bad]
        self.kf_rows, self.mp_rows = world_size * R, world_size * R * S
        self.kf_table = torch.zeros((self.kf_rows, 8), dtype=torch.float32, device=device)
        self.mp_table = torch.zeros((self.mp_rows, 4), dtype=torch.float32, device=device)
        kf_cap, mp_cap = self.W * NV, self.W * S   # the same on every rank (same W, NN, S)
        self.exch = CompactExchange(kf_cap, mp_cap, device=device)
        # per buffer set: the windows' global vertex ids (device, computed per step) and the pack descriptors
        self.pose_gid = [torch.zeros((self.W, NV), dtype=torch.int64, device=device) for _ in range(self.nheads)]
        self.point_gid = [torch.zeros((self.W, S), dtype=torch.int64, device=device) for _ in range(self.nheads)]
        self.d_pack = []
        for k, st in enumerate(self.rl.sets):
            pk = (MapWindow * self.W)()
            for w in range(self.W):
                b = st["bufs"][w]
                d = pk[w]
                d.n_poses, d.n_points = NV, S
                d.pose_id, d.pose_fixed = self.pose_gid[k][w].data_ptr(), b["pose_fixed"].data_ptr()
                d.point_id, d.point_bad = self.point_gid[k][w].data_ptr(), None
                d.pose_q, d.pose_t, d.point_xyz = b["out_q"].data_ptr(), b["out_t"].data_ptr(), b["out_xyz"].data_ptr()
            self.d_pack.append(torch.from_numpy(np.frombuffer(bytes(pk), np.uint8).copy()).to(device))
        self.src_h = torch.zeros(2 * (kf_cap + mp_cap), dtype=torch.int32).pin_memory()
        self.src_d = torch.zeros(2 * (kf_cap + mp_cap), dtype=torch.int32, device=device)
        self.n_kf_upd = self.n_mp_upd = 0
        self.time_gather = False
        self.stats = None
        self.windows_solved = 0
        self.host_s = {}
        self.last = None   # the buffer set of the last solve
        self._probs = None
        if world_size > 1 and dist.is_available() and dist.is_initialized():
            dist.barrier()

    def assemble(self, stream, head):
        self.rl.assemble(stream, head // self.W)

    def run(self, step: int, head=None):
        """One LocalMapping step: the windows of the keyframes at `head` (their searches and assembly ordered before
        this on the caller's wait), solved synchronously, then the pack / all-gather / apply queued on self.stream."""
        import time

        import torch

        if head is None:
            if self.last is None:   # no keyframe run yet: nothing to solve
                self.stats = [(0, 0, 0)] * self.W
                return self.stats
            head = self.last * self.W
        k = head // self.W
        with torch.cuda.stream(self.stream):
            t0 = time.perf_counter()
            s = self.stream.cuda_stream
            t1 = time.perf_counter()
            self.stats = self.rl.solve(self.stream, k)
            t2 = time.perf_counter()
            self.windows_solved += self.W
            self.last = k
            self._probs = None
            st = self.rl.sets[k]
            sizes, slots = st["sizes"], st["slots"]
            R, S = self.nm.R, self.nm.S
            base = self.rank * R
            # global ids: KeyFrame row = rank R + ring slot; MapPoint row = (rank R + the new keyframe's slot) S + keypoint
            self.pose_gid[k].copy_(st["pose_slot"].to(torch.int64) + base)
            self.point_gid[k].copy_((st["pose_slot"][:, :1].to(torch.int64) + base) * S + st["point_src"].to(torch.int64))
            # the write-back sources: every optimised KeyFrame once (from the last window optimising it), every
            # window's MapPoints (a keyframe's own: no two windows share one)
            kf = {}
            for w in range(self.W):
                for i in range(int(sizes[w, 3])):
                    kf[base + int(slots[w, i])] = (w, i)
            kf_src = np.array([kf[g] for g in sorted(kf)], np.int32).reshape(-1, 2)
            mp_src = np.concatenate([np.stack([np.full(int(sizes[w, 1]), w), np.arange(int(sizes[w, 1]))], 1)
                                     for w in range(self.W)]).astype(np.int32)
            self.n_kf_upd, self.n_mp_upd = len(kf_src), len(mp_src)
            nk = 2 * len(kf_src)
            src = self.src_h.numpy()
            src[:nk] = kf_src.reshape(-1)
            src[nk:nk + 2 * len(mp_src)] = mp_src.reshape(-1)
            n_all = nk + 2 * len(mp_src)
            self.src_d[:n_all].copy_(self.src_h[:n_all], non_blocking=True)
            self.exch.pack(self.d_pack[k].data_ptr(), self.W, self.src_d.data_ptr(), len(kf_src),
                           self.src_d.data_ptr() + 4 * nk, len(mp_src), 0, stream=s)
            self.exch.gather(timed=self.time_gather)
            self.exch.apply(self.kf_table.data_ptr(), self.kf_rows, self.mp_table.data_ptr(), self.mp_rows,
                            self.status.data_ptr(), stream=s)
            t3 = time.perf_counter()
        for key, v in (("launch", t1 - t0), ("solve", t2 - t1), ("exchange", t3 - t2)):
            self.host_s[key] = self.host_s.get(key, 0.0) + v
        return self.stats

    @property
    def probs(self):
        """Host LBAProblems of the last solved windows (built on first use after a solve)."""
        if self._probs is None:
            self._probs = [self.rl.window(w) for w in range(self.W)]
        return self._probs

    @property
    def edges(self):
        return [int(v) for v in self.rl.sizes[:, 2]]

    def window_inputs(self, w: int):
        return self.rl.window(w)

    def window_result(self, w: int):
        from .lba import LBAResult

        P, L, E = self.rl._size(w)
        b = self.rl.bufs[w]
        r = self.rl.c_res[w]
        it, tr, st = self.stats[w]
        return LBAResult(b["out_q"].cpu().numpy()[:P], b["out_t"].cpu().numpy()[:P], b["out_xyz"].cpu().numpy()[:L],
                         b["out_chi2"].cpu().numpy()[:E], b["out_depth"].cpu().numpy()[:E], it, tr,
                         float(r.initial_chi2), float(r.final_chi2), st)
