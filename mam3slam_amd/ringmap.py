"""The device-resident keyframe / MapPoint map of the LocalMapping leg (include/mam_ringmap.h, csrc/ringmap.hip).

MapPoint identities shared across the keyframe ring, their observation sets, and the map edits LocalMapping makes
around each LocalBundleAdjustment (LocalMapping.cc:95-172): eviction of the keyframes leaving the ring + MapPoint
culling, CreateNewMapPoints' new points, Fuse's Replace / AddObservation side effects, the MapPoints' descriptor /
normal / depth refresh, the reference's LBA window build (Optimizer.cc:1118-1186) and its write-back
(Optimizer.cc:1413-1497), and the write-back as exchange records for the other GPUs.

Rows: a MapPoint id is its home row slot * S + keypoint; `rec` holds the records (FUSE_MP_DTYPE: position,
mfMaxDistance, normal, mfMinDistance, valid, descriptor), `mp_of` the MapPoint of each keyframe keypoint and `okp`
(int16 [R S][R]) the keypoint of each MapPoint in each slot (-1 none). tests/ringmap_host.py restates every call.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib
from .match import FUSE_MP_DTYPE

MP_RECORD_DTYPE = np.dtype([("row", "<i4"), ("xyz", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_distance", "<f4"),
                            ("max_distance", "<f4"), ("pad", "<i4", (3,))])
KF_RECORD_DTYPE = np.dtype([("row", "<i4"), ("q", "<f4", (4,)), ("t", "<f4", (3,))])
HEADER_DTYPE = np.dtype([("n_kf", "<i4"), ("n_mp", "<i4"), ("agent", "<i4"), ("status", "<i4")])
assert MP_RECORD_DTYPE.itemsize == 48 and KF_RECORD_DTYPE.itemsize == 32


class RingMapC(C.Structure):
    """mam_ringmap (device pointers)."""
    _fields_ = [("R", C.c_int32), ("S", C.c_int32), ("nlevels", C.c_int32), ("scale_factors", C.c_float * 8),
                ("inv_level_sigma2", C.c_float * 8)] + [(k, C.c_void_p) for k in (
                    "mp_of", "okp", "rec", "born", "has_mp", "lists", "keys", "desc", "cnt", "tcw", "kp_rec", "parent",
                    "claim", "surv", "flag", "newid", "lastw", "slot_last", "pack_off")]


class RingMapWindow(C.Structure):
    """mam_ringmap_window: one window's LBA problem arrays (device)."""
    _fields_ = [(k, C.c_void_p) for k in ("pose_q", "pose_t", "pose_fixed", "point_xyz", "edge_point", "edge_pose",
                                           "edge_obs", "edge_inv_sigma2")]


class RingMapResult(C.Structure):
    """mam_ringmap_result: one window's solve results (device)."""
    _fields_ = [(k, C.c_void_p) for k in ("pose_q", "pose_t", "point_xyz", "edge_chi2", "edge_depth_ok")]


_V, _I, _I64 = C.c_void_p, C.c_int, C.c_int64
_SIGS = {
    "mam_ringmap_evict": (_I, [_V, _I, _I, _I, _V]),
    "mam_ringmap_flags": (_I, [_V, _V]),
    "mam_ringmap_create": (_I, [_V, _I, _I, _V, _I, _V, _I, _V]),
    "mam_ringmap_gather": (_I, [_V, _V]),
    "mam_ringmap_fuse_apply": (_I, [_V, _I, _I, _V, _I, _I, _V, _V, _V]),
    "mam_ringmap_refresh": (_I, [_V, _I, _I, _V]),
    "mam_ringmap_windows": (_I, [_V, _I, _I, _I, _V, _I, _I, _V, _V, _V, _V]),
    "mam_ringmap_writeback": (_I, [_V, _I, _V, _V, _V, _V, _V, _I, _I, _V]),
    "mam_ringmap_block_bytes": (C.c_size_t, [_I, _I]),
    "mam_ringmap_pack": (_I, [_V, _I64, _I64, _I, _V, _I, _I, _V]),
    "mam_ringmap_apply": (_I, [_V, _I, _I, _I, _V, _I64, _V, _I64, _V, _V]),
}


def _bind():
    L = lib()
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


def block_bytes(kf_cap: int, mp_cap: int) -> int:
    return HEADER_DTYPE.itemsize + kf_cap * KF_RECORD_DTYPE.itemsize + mp_cap * MP_RECORD_DTYPE.itemsize


class RingMap:
    """The map state over a keyframe ring (R slots of S keypoints): keys / desc / cnt / tcw / kp_rec are the ring's
    device tensors (owned by the caller: NewMapPointsLeg), the rest is allocated here."""

    def __init__(self, R: int, S: int, scale_factors, level_sigma2, keys, desc, cnt, tcw, kp_rec, has_mp, device):
        import torch

        self.R, self.S, self.dev = int(R), int(S), device
        if not (1 <= self.R <= 128 and 1 <= self.S <= 32767):
            raise ValueError(f"ring {R} x {S} outside the map's bounds (R <= 128, S <= 32767)")
        n = self.R * self.S
        z = lambda shape, dt, fill=0: torch.full(shape, fill, dtype=dt, device=device)  # noqa: E731
        self.mp_of = z((n,), torch.int32, -1)
        self.okp = z((n, self.R), torch.int16, -1)
        self.rec = z((n, FUSE_MP_DTYPE.itemsize), torch.uint8)
        self.born = z((n,), torch.int32, -1 << 20)
        self.lists = z((n, FUSE_MP_DTYPE.itemsize), torch.uint8)
        self.parent = z((n,), torch.int32)
        self.claim = z((n,), torch.int32)
        self.surv = z((n,), torch.int64)
        self.flag = z((n,), torch.uint8)
        self.newid = z((n,), torch.int32)
        self.lastw = z((n,), torch.int32)
        self.slot_last = z((self.R,), torch.int32, -1)
        self.pack_off = z((n // 1024 + 3,), torch.int32)
        self.has_mp, self.keys, self.desc, self.cnt, self.tcw, self.kp_rec = has_mp, keys, desc, cnt, tcw, kp_rec
        c = RingMapC()
        c.R, c.S = self.R, self.S
        sf = np.asarray(scale_factors, np.float32)
        s2 = np.asarray(level_sigma2, np.float32)
        c.nlevels = len(sf)
        for i in range(len(sf)):
            c.scale_factors[i] = float(sf[i])
            c.inv_level_sigma2[i] = float(np.float32(1.0) / s2[i])
        for k in ("mp_of", "okp", "rec", "born", "has_mp", "lists", "keys", "desc", "cnt", "tcw", "kp_rec", "parent",
                  "claim", "surv", "flag", "newid", "lastw", "slot_last", "pack_off"):
            setattr(c, k, getattr(self, k).data_ptr())
        self.c = c
        self._L = _bind()

    def clear(self):
        """An empty map (no MapPoint)."""
        self.mp_of.fill_(-1)
        self.okp.fill_(-1)
        self.rec.zero_()
        self.born.fill_(-1 << 20)
        self.has_mp.zero_()

    # ---------------------------------------------------------------------------------------------- the run's calls
    def evict(self, head: int, W: int, run: int, stream: int):
        check(self._L.mam_ringmap_evict(C.byref(self.c), head, W, run, C.c_void_p(stream)), "mam_ringmap_evict")

    def flags(self, stream: int):
        check(self._L.mam_ringmap_flags(C.byref(self.c), C.c_void_p(stream)), "mam_ringmap_flags")

    def create(self, head: int, W: int, d_pairs: int, NN: int, d_match: int, run: int, stream: int):
        check(self._L.mam_ringmap_create(C.byref(self.c), head, W, C.c_void_p(d_pairs), NN, C.c_void_p(d_match), run,
                                         C.c_void_p(stream)), "mam_ringmap_create")

    def gather(self, stream: int):
        check(self._L.mam_ringmap_gather(C.byref(self.c), C.c_void_p(stream)), "mam_ringmap_gather")

    def fuse_apply(self, head: int, W: int, d_pairs: int, NN: int, NB: int, d_fwd: int, d_bwd: int, stream: int):
        check(self._L.mam_ringmap_fuse_apply(C.byref(self.c), head, W, C.c_void_p(d_pairs), NN, NB, C.c_void_p(d_fwd),
                                             C.c_void_p(d_bwd), C.c_void_p(stream)), "mam_ringmap_fuse_apply")

    def refresh(self, head: int, W: int, stream: int):
        check(self._L.mam_ringmap_refresh(C.byref(self.c), head, W, C.c_void_p(stream)), "mam_ringmap_refresh")

    def windows(self, head: int, W: int, covis_th: int, d_outs: int, pcap: int, ecap: int, d_counts: int,
                d_pose_slot: int, d_point_id: int, stream: int):
        check(self._L.mam_ringmap_windows(C.byref(self.c), head, W, covis_th, C.c_void_p(d_outs), pcap, ecap,
                                          C.c_void_p(d_counts), C.c_void_p(d_pose_slot), C.c_void_p(d_point_id),
                                          C.c_void_p(stream)), "mam_ringmap_windows")

    def writeback(self, W: int, d_wins: int, d_res: int, d_counts: int, d_pose_slot: int, d_point_id: int, pcap: int,
                  ecap: int, stream: int):
        check(self._L.mam_ringmap_writeback(C.byref(self.c), W, C.c_void_p(d_wins), C.c_void_p(d_res),
                                            C.c_void_p(d_counts), C.c_void_p(d_pose_slot), C.c_void_p(d_point_id),
                                            pcap, ecap, C.c_void_p(stream)), "mam_ringmap_writeback")

    def pack(self, row_base_kf: int, row_base_mp: int, agent: int, d_block: int, kf_cap: int, mp_cap: int,
             stream: int):
        check(self._L.mam_ringmap_pack(C.byref(self.c), int(row_base_kf), int(row_base_mp), int(agent),
                                       C.c_void_p(d_block), kf_cap, mp_cap, C.c_void_p(stream)), "mam_ringmap_pack")

    # ---------------------------------------------------------------------------------------------- host views
    def snapshot(self):
        """Host copy of the map state (synchronises): mp_of [R S], okp [R S][R], rec (FUSE_MP_DTYPE [R S]), born, and
        the ring's tcw [R][7]."""
        return {"mp_of": self.mp_of.cpu().numpy().copy(), "okp": self.okp.cpu().numpy().copy(),
                "rec": self.rec.cpu().numpy().view(FUSE_MP_DTYPE).reshape(-1).copy(),
                "born": self.born.cpu().numpy().copy(),
                "tcw": self.tcw.cpu().numpy().view(np.float32).reshape(self.R, 7).copy()}

    def stats(self):
        """MapPoints alive, observations per MapPoint, MapPoints per keyframe (host; synchronises)."""
        v = self.rec.cpu().numpy().view(FUSE_MP_DTYPE).reshape(-1)["valid"] != 0
        ob = (self.okp.cpu().numpy() >= 0).sum(1)
        per_kf = (self.mp_of.cpu().numpy().reshape(self.R, self.S) >= 0).sum(1)
        return {"mappoints": int(v.sum()), "observations_mean": float(ob[v].mean()) if v.any() else 0.0,
                "mappoints_per_keyframe": float(per_kf.mean())}


class RingMapExchange:
    """The write-back of a GPU's LocalMapping run as one block (mam_ringmap_pack: 32-byte KeyFrame and 48-byte
    MapPoint records — position, normal, mfMinDistance, mfMaxDistance, bad bit), one fixed-size all-gather over the
    ranks (RCCL over xGMI; gloo in the CPU tests), applied in rank order to the replica tables every GPU holds
    (mam_ringmap_apply)."""

    def __init__(self, kf_cap: int, mp_cap: int, device, group=None):
        import torch
        import torch.distributed as dist

        self.kf_cap, self.mp_cap = int(kf_cap), int(mp_cap)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.block_bytes = block_bytes(self.kf_cap, self.mp_cap)
        self.send = torch.zeros(self.block_bytes, dtype=torch.uint8, device=device)
        self.recv = self.send if self.world == 1 else torch.zeros(self.world * self.block_bytes, dtype=torch.uint8,
                                                                   device=device)
        self._L = _bind()
        self.gather_ms = []

    def gather(self, stream, timed: bool = False):
        """The all-gather on `stream` (a torch stream) after the pack queued on it."""
        import time

        import torch

        from .exchange import _all_gather

        with torch.cuda.stream(stream):
            if timed:
                stream.synchronize()
                t0 = time.perf_counter()
            _all_gather(self.recv, self.send, self.world, self.group)
            if timed:
                stream.synchronize()
                self.gather_ms.append((time.perf_counter() - t0) * 1e3)

    def apply(self, d_kf_table: int, kf_rows: int, d_mp_table: int, mp_rows: int, d_status: int, stream: int):
        check(self._L.mam_ringmap_apply(C.c_void_p(self.recv.data_ptr()), self.world, self.kf_cap, self.mp_cap,
                                        C.c_void_p(d_kf_table), int(kf_rows), C.c_void_p(d_mp_table), int(mp_rows),
                                        C.c_void_p(d_status), C.c_void_p(stream)), "mam_ringmap_apply")

    def header(self):
        return self.send[:16].cpu().numpy().view(HEADER_DTYPE)[0]
