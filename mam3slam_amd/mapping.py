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
    """LocalMapping's keyframe work on the device, for the W keyframes the agents on this GPU insert per LocalMapping
    run (LocalMapping::Run, LocalMapping.cc:95-172, one run = the step's W new keyframes): ProcessNewKeyFrame's
    ComputeBoW (DBoW2 transform, synthetic k=10 L=6 vocabulary — ORBvoc.txt is a missing blob), MapPointCulling,
    CreateNewMapPoints (SearchForTriangulation against the keyframe's NN = 30 neighbours, LocalMapping.cc:504-582,
    ORBmatcher(0.6, false), and the MapPoints of its matches) and SearchInNeighbors (Fuse of the keyframe's MapPoints
    into its neighbours, Fuse of its NB_BACK nearest neighbours' MapPoints into it, and the Replace / AddObservation
    side effects, ComputeDistinctiveDescriptors + UpdateNormalAndDepth of its MapPoints, LocalMapping.cc:830-939) —
    the searches on the matcher kernels, the map edits on the device map (ringmap.RingMap, include/mam_ringmap.h).

    The keyframes live in a ring of R slots in HBM (keypoints, descriptors, pose, BoW node + weight, and per keypoint
    the scene point a new MapPoint made there gets: `fmp`, the stand-in for the triangulated position); the map's
    MapPoints are shared across the slots (RingMap: mp_of / okp / records). `ingest` copies a step's new keyframes out
    of the tracking buffers into a staging set (on the tracking stream, after the step that tracked them: the
    reference's Tracking -> LocalMapping hand-off); `process` (on LocalMapping's stream) moves them into the next W
    ring slots — the keyframes there leave the map (KeyFrame::SetBadFlag) — and runs the keyframe work. A new
    keyframe's neighbours (GetBestCovisibilityKeyFrames(30) for a camera moving through one scene) are the NN older
    ring keyframes nearest to it along the agent's frame sequence (same view last; ties: the more recent first);
    the W keyframes of one run see the map as the run started (they are processed together, as concurrent agents'
    LocalMapping threads would)."""

    NN = 30
    NB_BACK = 4   # the neighbours whose MapPoints are the backward Fuse's candidates
    NSTAGE = 3

    def __init__(self, tr, n_new: int, device, seed: int = 0, stream=None):
        import torch

        from . import bow
        from .match import FUSE_MP_DTYPE, FramesDev, ORBmatcher, TriBatch
        from .ringmap import RingMap

        self.dev, self.tr, self.W = device, tr, int(n_new)
        # the new slots + at least NN older ones + one spare group, a multiple of W
        self.R = self.W * (2 + -(-self.NN // self.W))
        R, S = self.R, tr.cap
        self.S = S
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=device)  # noqa: E731
        self.keys = z((R, S * 28), torch.uint8)
        self.desc = z((R, S, 32), torch.uint8)
        self.cnt = z((R, 2), torch.int32)
        self.has_mp = z((R, S), torch.uint8)
        self.tcw = z((R, tr.tcw_bytes), torch.uint8)
        self.nid = z((R, S), torch.int32)
        self.weight = z((R, S), torch.float64)
        self.word = z((R, S), torch.int32)
        self.cnt_col = z(R, torch.int32)
        self.fmp = z((R, S * FUSE_MP_DTYPE.itemsize), torch.uint8)
        self.tcw_search = z((R, tr.tcw_bytes), torch.uint8)   # the poses the last run's searches read
        # staging sets: a step's keyframes between the ingest and the run that moves them into the ring
        W = self.W
        self.stage = [dict(keys=z((W, S * 28), torch.uint8), desc=z((W, S, 32), torch.uint8), cnt=z((W, 2), torch.int32),
                           tcw=z((W, tr.tcw_bytes), torch.uint8), fmp=z((W, S * FUSE_MP_DTYPE.itemsize), torch.uint8),
                           ready=torch.cuda.Event(), used=None)
                      for _ in range(self.NSTAGE)]
        self.voc = bow.ORBVocabulary(bow.synthetic_vocabulary(10, 6, np.random.default_rng(seed), early_leaf=0.02),
                                     device=device.index or 0)
        self.matcher = ORBmatcher(0.6, False, device=device.index or 0)
        self.stream = stream if stream is not None else torch.cuda.Stream(device, priority=-1)
        self.npairs = W * self.NN
        NB = min(self.NB_BACK, self.NN)
        self.NB = NB
        self.out = z((self.npairs, S), torch.int32)
        self.nmatch = z(self.npairs, torch.int32)
        self.fwd_idx = z((self.npairs, S), torch.int32)
        self.fwd_dist = z((self.npairs, S), torch.int32)
        self.fwd_n = z(self.npairs, torch.int32)
        self.bwd_idx = z((W * NB, S), torch.int32)
        self.bwd_dist = z((W * NB, S), torch.int32)
        self.bwd_n = z(W * NB, torch.int32)
        # per run: pairs [W NN][2], fuse items (fwd frame, fwd list [W NN], bwd frame, bwd list [W NB]) in one buffer
        self.n_items = 2 * self.npairs + 2 * self.npairs + 2 * W * NB
        self.items_h = torch.zeros(self.n_items, dtype=torch.int32).pin_memory()
        self.items_d = z(self.n_items, torch.int32)
        o = 2 * self.npairs
        self.pairs_d = self.items_d[:o].view(self.npairs, 2)
        self.fwd_frame, self.fwd_list = self.items_d[o:o + self.npairs], self.items_d[o + self.npairs:o + 2 * self.npairs]
        o += 2 * self.npairs
        self.bwd_frame, self.bwd_list = self.items_d[o:o + W * NB], self.items_d[o + W * NB:o + 2 * W * NB]
        self._items_ev = None
        self._init_scene_points()
        self._FramesDev, self._TriBatch = FramesDev, TriBatch
        # trajectory position (pool frame index) and insertion order of each slot: the neighbour rule's inputs
        self.slot_pos = np.zeros(R, np.int64)
        self.slot_age = np.arange(R, dtype=np.int64) - R
        # initial ring: the first R frames of the pool, BoW on the device, no MapPoint yet
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
        torch.cuda.synchronize(device)
        self.slot_pos[:] = np.arange(R) % (tr.P * tr.B)
        self.map = RingMap(R, S, tr.F0.scale_factors, tr.F0.level_sigma2, self.keys, self.desc, self.cnt, self.tcw,
                           self.fmp, self.has_mp, device)
        self.next_head = 0
        self.ingests = 0
        self.runs = 0
        self.head = 0          # the head of the last processed run
        self.pending = None    # the last ingest's item (tests / launch)
        self.last_item = None  # the last processed item
        self.map_ms = []       # per profiled run: the map edits' GPU time (HIP events on the run's stream)
        self.profile = False

    # ------------------------------------------------------------------------------------------ scene points
    def _init_scene_points(self):
        """Per pool frame and keypoint, the MapPoint a triangulation there makes (the stand-in for
        GeometricTools::Triangulate, LocalMapping.cc:701): the keypoint's ray on the scene plane (synth.PLANE_DEPTH,
        world coordinates under the pose of the camera that rendered the frame), normal = viewing direction, depth
        range as UpdateNormalAndDepth leaves it for one view, descriptor = the keypoint's."""
        import torch

        from . import synth
        from .match import FUSE_MP_DTYPE, quat_to_rot

        tr, S = self.tr, self.S
        sf = tr.F0.scale_factors.astype(np.float64)
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

    # ------------------------------------------------------------------------------------------ ingest
    def ingest(self, step: int):
        """Copy step `step`'s new keyframes (frames f = step mod K + i K of the tracking batch) into a staging set, on
        the tracking stream after the step that tracked them; returns the run item (head, staging set, the frames'
        pool indices), also kept as self.pending."""
        from .exchange import copy_rows

        tr, W = self.tr, self.W
        K = max(1, tr.B // W)
        fr = [(i * K + step % K) % tr.B for i in range(W)]
        k = self.ingests % self.NSTAGE
        st = self.stage[k]
        if st["used"] is not None:   # the run that read this set last has moved it into the ring
            tr.tstream.wait_event(st["used"])
        S = self.S
        tables = [(tr.d_kps.data_ptr(), st["keys"].data_ptr(), S * 28, S * 28, S * 28, 0),
                  (tr.d_desc.data_ptr(), st["desc"].data_ptr(), S * 32, S * 32, S * 32, 0),
                  (tr.d_cnt.data_ptr(), st["cnt"].data_ptr(), 8, 8, 8, 0),
                  (tr.d_tcw.data_ptr(), st["tcw"].data_ptr(), tr.tcw_bytes, tr.tcw_bytes, tr.tcw_bytes, 0),
                  (self.fmp_frames.data_ptr(), st["fmp"].data_ptr(), self.fmp.shape[1], self.fmp_frames.shape[1],
                   self.fmp.shape[1], tr.p * tr.B)]
        for i in range(0, W, 64):
            copy_rows(tables, fr[i:i + 64], list(range(i, min(W, i + 64))), stream=tr.tstream.cuda_stream)
        st["ready"].record(tr.tstream)
        item = (self.next_head, k, [tr.p * tr.B + f for f in fr])
        self.next_head = (self.next_head + W) % self.R
        self.ingests += 1
        self.pending = item
        return item

    def take(self):
        h, self.pending = self.pending, None
        return h

    def launch(self, item):
        """process() on this leg's own stream (tests; the bench's LocalMapping thread calls process on its stream)."""
        if item is not None:
            self.process(self.stream, item)

    def wait(self, stream, item):
        pass

    def _pairs(self, head: int, pos_new):
        """Each new keyframe's NN neighbours: the older ring slots nearest along the frame sequence (a keyframe of
        the same view last), the more recently inserted first on a tie, then the lower slot."""
        R, W, NN = self.R, self.W, self.NN
        new = set(range(head, head + W))
        older = np.array([s for s in range(R) if s not in new])
        pairs = np.zeros((W, NN, 2), np.int32)
        for w in range(W):
            d = np.abs(self.slot_pos[older] - pos_new[w])
            key = np.lexsort((older, -self.slot_age[older], d, d == 0))
            nb = older[key[:NN]]
            pairs[w, :, 0] = head + w
            pairs[w, :, 1] = nb
        return pairs.reshape(-1, 2)

    def process(self, stream, item, run: int | None = None, hook=None):
        """LocalMapping's keyframe work for the keyframes of `item`, asynchronous on `stream` (a torch stream): the
        keyframes into ring slots [head, head + W) (the previous ones leave the map), ComputeBoW, MapPointCulling,
        CreateNewMapPoints, SearchInNeighbors. hook(phase) (tests): called after each phase's launches ("insert",
        "evict", "search", "create", "fuse_search", "fuse_apply", "refresh")."""
        import torch

        if item is None:
            return
        head, k, frames = item
        self.last_item = item
        W, S, R = self.W, self.S, self.R
        run = self.runs if run is None else run
        self.runs += 1
        st = self.stage[k]
        s = stream.cuda_stream
        stream.wait_event(st["ready"])
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if self.profile else None
        with torch.cuda.stream(stream):
            # the keyframes into the ring (InsertKeyFrame), the staging set free again
            sl = slice(head, head + W)
            self.keys[sl].copy_(st["keys"])
            self.desc[sl].copy_(st["desc"])
            self.cnt[sl].copy_(st["cnt"])
            self.tcw[sl].copy_(st["tcw"])
            self.fmp[sl].copy_(st["fmp"])
            self.cnt_col[sl].copy_(st["cnt"][:, 0])
            if st["used"] is None:
                st["used"] = torch.cuda.Event()
            st["used"].record(stream)
            pos = np.asarray(frames, np.int64)
            pairs = self._pairs(head, pos)
            self.slot_pos[sl] = pos
            self.slot_age[sl] = self.ingests + np.arange(W)
            NN, NB = self.NN, self.NB
            items = np.concatenate([pairs.reshape(-1), pairs[:, 1], pairs[:, 0],
                                    np.repeat(pairs[::NN, 0], NB), pairs.reshape(W, NN, 2)[:, :NB, 1].reshape(-1)])
            if self._items_ev is not None:   # the previous run's copy out of the pinned buffer has finished
                self._items_ev.synchronize()
            self.items_h.numpy()[:] = items
            self.items_d.copy_(self.items_h, non_blocking=True)
            self._items_ev = torch.cuda.Event()
            self._items_ev.record(stream)
            self.head = head
            self.run_index = run
            if hook:
                hook("insert")
            if ev:
                ev[0].record(stream)
            # KeyFrame::SetBadFlag of the slots' previous keyframes + MapPointCulling
            self.map.evict(head, W, run, s)
            self.map.flags(s)
            if hook:
                hook("evict")
            if ev:
                ev[1].record(stream)
            self.tcw_search.copy_(self.tcw)   # (the parity checks' view: the write-back moves the poses later)
            self.voc.transform_batch_device(W, self.desc[head].data_ptr(), S, self.cnt[head].data_ptr(), 4,
                                            self.word[head].data_ptr(), self.weight[head].data_ptr(),
                                            self.nid[head].data_ptr(), stream=s)
            b = self._TriBatch()
            b.kfs = self._FramesDev(R, S, self.keys.data_ptr(), self.desc.data_ptr(), self.cnt.data_ptr(), None, None, 0)
            b.has_mp, b.nid, b.weight = self.has_mp.data_ptr(), self.nid.data_ptr(), self.weight.data_ptr()
            b.tcw = self.tcw.data_ptr()
            b.npairs, b.pairs = self.npairs, self.pairs_d.data_ptr()
            self.matcher.search_for_triangulation_batch_device(self.tr.F0, self.tr.cam, b, self.out.data_ptr(),
                                                               self.nmatch.data_ptr(), False, stream=s)
            if hook:
                hook("search")
            if ev:
                ev[2].record(stream)
            self.map.create(head, W, self.pairs_d.data_ptr(), NN, self.out.data_ptr(), run, s)
            self.map.gather(s)
            if hook:
                hook("create")
            if ev:
                ev[3].record(stream)
            self.search_in_neighbors(stream)
            if hook:
                hook("fuse_search")
            if ev:
                ev[4].record(stream)
            self.map.fuse_apply(head, W, self.pairs_d.data_ptr(), NN, NB, self.fwd_idx.data_ptr(),
                                self.bwd_idx.data_ptr(), s)
            if hook:
                hook("fuse_apply")
            self.map.refresh(head, W, s)
            if hook:
                hook("refresh")
            if ev:
                ev[5].record(stream)
                self._ev = ev

    def profiled_map_ms(self):
        """GPU ms of the last profiled run's map edits (evict + flags, create + gather, fuse apply + refresh; HIP
        events on the run's stream), None when the run was not profiled."""
        ev = getattr(self, "_ev", None)
        if not ev:
            return None
        ev[-1].synchronize()
        return ev[0].elapsed_time(ev[1]) + ev[2].elapsed_time(ev[3]) + ev[4].elapsed_time(ev[5])

    # ------------------------------------------------------------------------------------------ SearchInNeighbors
    def search_in_neighbors(self, stream):
        """SearchInNeighbors' searches of the run's keyframes (after their CreateNewMapPoints MapPoints): forward Fuse
        of each keyframe's MapPoints into its NN neighbours, backward Fuse of its NB nearest neighbours' MapPoints
        into it — the MapPoint lists gathered from the map (KeyFrame::GetMapPointMatches, valid 0 where a keypoint has
        none). The side effects follow in RingMap.fuse_apply."""
        s = stream.cuda_stream
        fr = self._FramesDev(self.R, self.S, self.keys.data_ptr(), self.desc.data_ptr(), self.cnt.data_ptr(), None,
                             None, 0)
        tcw = self.tcw.data_ptr()
        lists = self.map.lists.data_ptr()
        m = self.matcher   # (cnt_col: list m's length = ring slot m's keypoints)
        m.fuse_items_batch_device(self.tr.F0, fr, tcw, self.tr.cam, self.npairs, self.fwd_frame.data_ptr(),
                                  self.fwd_list.data_ptr(), lists, self.S, self.cnt_col.data_ptr(), 3.0,
                                  self.fwd_idx.data_ptr(), self.fwd_dist.data_ptr(), self.fwd_n.data_ptr(), stream=s)
        m.fuse_items_batch_device(self.tr.F0, fr, tcw, self.tr.cam, self.W * self.NB, self.bwd_frame.data_ptr(),
                                  self.bwd_list.data_ptr(), lists, self.S, self.cnt_col.data_ptr(), 3.0,
                                  self.bwd_idx.data_ptr(), self.bwd_dist.data_ptr(), self.bwd_n.data_ptr(), stream=s)

    # ------------------------------------------------------------------------------------------ host views
    def _frame(self, slot: int, search_pose: bool = False):
        from .match import FrameData
        from .orb import KP_DTYPE

        n = int(self.cnt[slot, 0].item())
        keys = self.keys[slot].cpu().numpy().view(KP_DTYPE)[:n]
        F = FrameData(keys=keys, desc=self.desc[slot, :n].cpu().numpy(), width=self.tr.W, height=self.tr.H,
                      scale_factors=self.tr.F0.scale_factors, level_sigma2=self.tr.F0.level_sigma2)
        t = (self.tcw_search if search_pose else self.tcw)[slot].cpu().numpy().view(np.float32)
        F.pose = (t[:4].copy(), t[4:7].copy())
        return F

    def fuse_inputs(self, backward: bool, b: int, lists=None):
        """Host (KeyFrame FrameData with pose, MapPoint list) of forward / backward Fuse item b of the last run (the
        lists as the run gathered them, or `lists` [R S] FUSE_MP_DTYPE)."""
        from .match import FUSE_MP_DTYPE

        slot = int((self.bwd_frame if backward else self.fwd_frame)[b].item())
        ms = int((self.bwd_list if backward else self.fwd_list)[b].item())
        KF = self._frame(slot, search_pose=True)
        nm = int(self.cnt[ms, 0].item())
        if lists is None:
            lists = self.map.lists.cpu().numpy().view(FUSE_MP_DTYPE).reshape(self.R, self.S)
        return KF, lists[ms, :nm].copy()

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
        for a, b in self.pairs_d.cpu().numpy():
            A, B = per_slot[a], per_slot[b]
            cand += sum(c * B[u] for u, c in A.items() if u in B)
            fv += sum(A.values()) + sum(B.values())
        return {"candidate_pairs": int(cand), "bytes": int(cand * 32 + fv * (8 + 1 + 28 + 32))}

    def pair_inputs(self, q: int, has_mp=None):
        """Host FrameData of pair q of the last run (keys, desc, has_mp — the map's flags the search read, or
        `has_mp` [R][S] — FeatureVector from the device BoW, pose)."""
        if has_mp is None:
            has_mp = self.has_mp.cpu().numpy()
        out = []
        for slot in self.pairs_d[q].cpu().numpy():
            F = self._frame(int(slot), search_pose=True)
            n = len(F.keys)
            F.has_mp = has_mp[slot, :n].copy()
            nid, w = self.nid[slot, :n].cpu().numpy(), self.weight[slot, :n].cpu().numpy()
            fv = {}
            for i in range(n):
                if w[i] > 0:
                    fv.setdefault(int(np.uint32(nid[i])), []).append(i)
            F.featvec = dict(sorted(fv.items()))
            out.append(F)
        return out

    def distinctive_inputs(self, slot: int):
        """(offsets, descriptors) of the MapPoints keyframe `slot` observes — their observations' descriptors in slot
        order — ComputeDistinctiveDescriptors' inputs on the host (the CPU baseline; synchronises)."""
        R, S = self.R, self.S
        mp_of = self.map.mp_of.cpu().numpy().reshape(R, S)
        okp = self.map.okp.cpu().numpy()
        desc = self.desc.cpu().numpy()
        off, ds = [0], []
        for m in mp_of[slot][mp_of[slot] >= 0]:
            for s in np.nonzero(okp[m] >= 0)[0]:
                ds.append(desc[s, okp[m, s]])
            off.append(len(ds))
        return np.array(off, np.int32), (np.stack(ds) if ds else np.zeros((0, 32), np.uint8))


class RingLBA:
    """LocalBundleAdjustment of each new keyframe of the last LocalMapping run (Optimizer.cc:1118-1497 on the device
    map, ringmap.RingMap): its window by the reference's rule (mam_ringmap_windows: local = the keyframe + its
    covisible keyframes by weight, local MapPoints = every MapPoint of every local keyframe, fixed = their other
    observers; windows with no fixed keyframe are not solved, as the reference aborts), the W windows solved as one
    batch (mam_lba_solve_batch_device; the sizes read back once per batch), and their write-back (mam_ringmap_writeback:
    outlier erase, SetPose, SetWorldPos + UpdateNormalAndDepth)."""

    COVIS_TH = 15

    def __init__(self, nm, iterations: int = 10, solver=None, pcap: int = 16384, ecap: int = 262144):
        import torch

        from .lba import HUBER_MONO
        from .ringmap import RingMapResult, RingMapWindow

        self.nm, self.dev = nm, nm.dev
        W, R = nm.W, nm.R
        self.pcap, self.ecap = int(pcap), int(ecap)
        P, E = self.pcap, self.ecap
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=self.dev)  # noqa: E731
        cam = nm.tr.cam
        self.cams = torch.from_numpy(np.ascontiguousarray(cam.params(), np.float32)[None]).to(self.dev)
        self.bufs = []
        wins = (RingMapWindow * W)()
        ress = (RingMapResult * W)()
        self.c_probs = (_Problem * W)()
        self.c_res = (_Result * W)()
        for w in range(W):
            b = dict(pose_q=z((R, 4), torch.float64), pose_t=z((R, 3), torch.float64), pose_fixed=z(R, torch.uint8),
                     point_xyz=z((P, 3), torch.float64), edge_point=z(E, torch.int32), edge_pose=z(E, torch.int32),
                     edge_obs=z((E, 2), torch.float64), edge_inv_sigma2=z(E, torch.float64),
                     out_q=z((R, 4), torch.float64), out_t=z((R, 3), torch.float64), out_xyz=z((P, 3), torch.float64),
                     out_chi2=z(E, torch.float64), out_depth=z(E, torch.uint8))
            self.bufs.append(b)
            for f in RingMapWindow._fields_:
                setattr(wins[w], f[0], b[f[0]].data_ptr())
            r = ress[w]
            r.pose_q, r.pose_t, r.point_xyz = b["out_q"].data_ptr(), b["out_t"].data_ptr(), b["out_xyz"].data_ptr()
            r.edge_chi2, r.edge_depth_ok = b["out_chi2"].data_ptr(), b["out_depth"].data_ptr()
            Pb = self.c_probs[w]
            Pb.pose_id = Pb.point_id = Pb.pose_cam = None
            Pb.pose_fixed, Pb.pose_q, Pb.pose_t = b["pose_fixed"].data_ptr(), b["pose_q"].data_ptr(), b["pose_t"].data_ptr()
            Pb.point_xyz = b["point_xyz"].data_ptr()
            Pb.edge_point, Pb.edge_pose = b["edge_point"].data_ptr(), b["edge_pose"].data_ptr()
            Pb.edge_obs, Pb.edge_inv_sigma2 = b["edge_obs"].data_ptr(), b["edge_inv_sigma2"].data_ptr()
            Pb.edge_active = None
            Pb.n_cams, Pb.cams = 1, self.cams.data_ptr()
            Pb.huber_delta, Pb.iterations = HUBER_MONO, int(iterations)
            Pb.cam_model = 1 if cam.is_kb8 else 0
            Rs = self.c_res[w]
            Rs.pose_q, Rs.pose_t, Rs.point_xyz = b["out_q"].data_ptr(), b["out_t"].data_ptr(), b["out_xyz"].data_ptr()
            Rs.edge_chi2, Rs.edge_depth_ok = b["out_chi2"].data_ptr(), b["out_depth"].data_ptr()
        self.d_wins = torch.from_numpy(np.frombuffer(bytes(wins), np.uint8).copy()).to(self.dev)
        self.d_res = torch.from_numpy(np.frombuffer(bytes(ress), np.uint8).copy()).to(self.dev)
        self.counts = z((W, 4), torch.int32)
        self.pose_slot = z((W, R), torch.int32)
        self.point_id = z((W, P), torch.int32)
        self.meta_h = torch.zeros((W, 4 + R), dtype=torch.int32).pin_memory()
        self.sizes = np.zeros((W, 4), np.int64)
        self.slots = np.zeros((W, R), np.int64)
        self.valid = []
        self.stats = [(0, 0, 0)] * W
        self.solver = solver or LBASolver(device=self.dev.index or 0)

    def assemble(self, stream):
        """The windows of the run's keyframes (after its map edits on `stream`)."""
        nm = self.nm
        nm.map.windows(nm.head, nm.W, self.COVIS_TH, self.d_wins.data_ptr(), self.pcap, self.ecap,
                       self.counts.data_ptr(), self.pose_slot.data_ptr(), self.point_id.data_ptr(), stream.cuda_stream)

    def solve(self, stream):
        import torch

        W = self.nm.W
        with torch.cuda.stream(stream):
            self.meta_h[:, :4].copy_(self.counts, non_blocking=True)
            self.meta_h[:, 4:].copy_(self.pose_slot, non_blocking=True)
        stream.synchronize()
        meta = self.meta_h.numpy()
        self.sizes, self.slots = meta[:, :4].astype(np.int64), meta[:, 4:].astype(np.int64)
        if (self.sizes < 0).any():
            w = int(np.nonzero((self.sizes < 0).any(1))[0][0])
            raise RuntimeError(f"ring LBA window {w} exceeds the buffers (points <= {self.pcap}, edges <= {self.ecap})")
        for w in range(W):
            P = self.c_probs[w]
            P.n_poses, P.n_points, P.n_edges, P.n_opt_poses = (int(v) for v in self.sizes[w])
        # windows the reference would not solve (no fixed keyframe, no MapPoint) come back empty
        valid = [w for w in range(W) if self.sizes[w, 2] > 0]
        self.valid = valid
        stats = [(0, 0, 0)] * W
        if valid:
            if len(valid) == W:
                probs, res = self.c_probs, self.c_res
            else:
                probs = (_Problem * len(valid))(*[self.c_probs[w] for w in valid])
                res = (_Result * len(valid))(*[self.c_res[w] for w in valid])
            rc = self.solver._L.mam_lba_solve_batch_device(self.solver._ctx, len(valid), C.byref(probs),
                                                           C.byref(res), C.c_void_p(stream.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"mam_lba_solve_batch_device: {rc}")
            for i, w in enumerate(valid):
                if res is not self.c_res:
                    self.c_res[w] = res[i]
                r = self.c_res[w]
                stats[w] = (int(r.iterations), int(r.lm_trials), int(r.status))
        self.stats = stats
        return stats

    def writeback(self, stream):
        nm = self.nm
        nm.map.writeback(nm.W, self.d_wins.data_ptr(), self.d_res.data_ptr(), self.counts.data_ptr(),
                         self.pose_slot.data_ptr(), self.point_id.data_ptr(), self.pcap, self.ecap, stream.cuda_stream)

    def _size(self, w: int):
        return int(self.sizes[w, 0]), int(self.sizes[w, 1]), int(self.sizes[w, 2])

    def window(self, w: int):
        """Host LBAProblem of window w as assembled (ids = array order)."""
        from .lba import HUBER_MONO, LBAProblem

        P, L, E = self._size(w)
        b = {k: v.cpu().numpy() for k, v in self.bufs[w].items() if not k.startswith("out")}
        return LBAProblem(pose_id=np.arange(P, dtype=np.int64), pose_fixed=b["pose_fixed"][:P], pose_q=b["pose_q"][:P],
                          pose_t=b["pose_t"][:P], point_id=np.arange(L, dtype=np.int64) + P,
                          point_xyz=b["point_xyz"][:L], edge_point=b["edge_point"][:E], edge_pose=b["edge_pose"][:E],
                          edge_obs=b["edge_obs"][:E], edge_inv_sigma2=b["edge_inv_sigma2"][:E],
                          cams=self.cams.cpu().numpy(), huber_delta=HUBER_MONO,
                          iterations=int(self.c_probs[w].iterations), edge_active=None,
                          cam_model=int(self.c_probs[w].cam_model)).contiguous()

    def result(self, w: int):
        b = self.bufs[w]
        r = self.c_res[w]
        P, L, _ = self._size(w)
        return (b["out_q"].cpu().numpy()[:P], b["out_t"].cpu().numpy()[:P], b["out_xyz"].cpu().numpy()[:L],
                int(r.iterations), int(r.lm_trials), int(r.status), float(r.initial_chi2), float(r.final_chi2))


class RingMappingLeg:
    """The LocalMapping leg over the keyframes Tracking inserted: per run, the LocalBundleAdjustment windows of the
    keyframes the NewMapPointsLeg just processed (RingLBA: the reference's window rule over the device map), solved
    together, their write-back applied to the map (outlier erase, poses, positions, normals / depth ranges), and the
    write-back exchanged: packed as records (every changed KeyFrame and MapPoint, 32 / 48 bytes:
    mam_ringmap_pack), all-gathered across GPUs (RCCL over xGMI), applied in rank order to the replica of every
    GPU's map each GPU holds (rows: rank x ring slot for KeyFrames, (rank x R + home slot) x S + keypoint for
    MapPoints).

    The interface of LocalMappingLeg (bench.py reads the same fields)."""

    def __init__(self, nm, rank: int, world_size: int, device, iterations: int = 10, stream=None,
                 mp_cap: int | None = None, pcap: int = 16384, ecap: int = 262144):
        import torch
        import torch.distributed as dist

        from .ringmap import RingMapExchange

        self.nm, self.dev = nm, device
        self.W, self.rank, self.world_size = nm.W, rank, world_size
        self.rl = RingLBA(nm, iterations=iterations, pcap=pcap, ecap=ecap)
        self.solver = self.rl.solver
        self.stream = stream if stream is not None else torch.cuda.Stream(device, priority=-1)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        R, S = nm.R, nm.S
        self.kf_rows, self.mp_rows = world_size * R, world_size * R * S
        self.kf_table = torch.zeros((self.kf_rows, 8), dtype=torch.float32, device=device)
        self.mp_table = torch.zeros((self.mp_rows, 12), dtype=torch.float32, device=device)
        self.exch = RingMapExchange(R, mp_cap if mp_cap is not None else R * S // 2, device)
        self.time_gather = False
        self.stats = None
        self.windows_solved = 0
        self.host_s = {}
        self.last = None
        self._probs = None
        self.n_kf_upd = self.n_mp_upd = 0
        if world_size > 1 and dist.is_available() and dist.is_initialized():
            dist.barrier()

    def run(self, step: int, item=None):
        """One LocalMapping run: the keyframe work of `item` (NewMapPointsLeg.process), the windows, the solve (host
        synchronous: the sizes and the Levenberg state are read back), the write-back, and the exchange queued on
        self.stream. item None: the last item again (the same keyframes re-inserted)."""
        import time

        import torch

        if item is None:
            item = self.last
            if item is None:
                self.stats = [(0, 0, 0)] * self.W
                return self.stats
        self.last = item
        nm, st = self.nm, self.stream
        t0 = time.perf_counter()
        nm.process(st, item)
        self.rl.assemble(st)
        t1 = time.perf_counter()
        self.stats = self.rl.solve(st)
        t2 = time.perf_counter()
        self.windows_solved += len(self.rl.valid)
        self._probs = None
        with torch.cuda.stream(st):
            self.rl.writeback(st)
            R, S = nm.R, nm.S
            nm.map.pack(self.rank * R, self.rank * R * S, self.rank, self.exch.send.data_ptr(), self.exch.kf_cap,
                        self.exch.mp_cap, st.cuda_stream)
            self.exch.gather(st, timed=self.time_gather)
            self.exch.apply(self.kf_table.data_ptr(), self.kf_rows, self.mp_table.data_ptr(), self.mp_rows,
                            self.status.data_ptr(), st.cuda_stream)
        t3 = time.perf_counter()
        for key, v in (("launch", t1 - t0), ("solve", t2 - t1), ("exchange", t3 - t2)):
            self.host_s[key] = self.host_s.get(key, 0.0) + v
        return self.stats

    def exchange_counts(self):
        """(KeyFrame records, MapPoint records, status) of the last packed block (synchronises)."""
        h = self.exch.header()
        self.n_kf_upd, self.n_mp_upd = int(h["n_kf"]), int(h["n_mp"])
        return self.n_kf_upd, self.n_mp_upd, int(h["status"])

    @property
    def probs(self):
        """Host LBAProblems of the last solved windows (built on first use after a solve; empty windows included)."""
        if self._probs is None:
            self._probs = [self.rl.window(w) for w in range(self.W)]
        return self._probs

    @property
    def edges(self):
        return [int(v) for v in self.rl.sizes[:, 2]]

    def first_valid(self):
        if not self.rl.valid:
            raise RuntimeError("no LocalBundleAdjustment window was solved in the last run")
        return self.rl.valid[0]

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
