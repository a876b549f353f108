"""Shared-map update exchange between agents, one agent per GPU (include/mam_exchange.h).

After each LocalBundleAdjustment an agent packs its write-back (optimised KeyFrame poses, MapPoint positions, bad
flags — what src/Optimizer.cc:1463-1497 writes into the shared Atlas under mMutexMapUpdate) into one fixed-size
block of 64-byte records on the GPU (`pack_lba`), the blocks of all agents are all-gathered
(`torch.distributed.all_gather_into_tensor`: RCCL over xGMI on MI355X, gloo on CPU), and every agent applies the
gathered blocks to its device-resident shared tables in agent-id order (`apply`), so all replicas hold identical
bytes. One collective per LBA, fixed size: no all-gatherv, no count exchange.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib

UPDATE_HEADER, UPDATE_KF, UPDATE_MP = 0, 1, 2
UPDATE_DTYPE = np.dtype([("id", "<i8"), ("kind", "<i4"), ("agent", "<i4"), ("v", "<f4", (7,)), ("bad", "<i4"),
                         ("reserved", "<f4", (4,))])
assert UPDATE_DTYPE.itemsize == 64
RECORD_BYTES = 64

_SIGS = {
    "mam_exchange_pack_lba": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p]),
    "mam_exchange_apply": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                     C.c_void_p, C.c_void_p]),
    "mam_exchange_pack_windows": (C.c_int, [C.c_int, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_void_p]),
    "mam_map_read_windows": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p,
                                       C.c_int, C.c_void_p, C.c_void_p]),
    "mam_exchange_compact_block_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "mam_exchange_pack_sources": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64,
                                            C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "mam_exchange_apply_compact": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64,
                                             C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
}

# compact blocks (include/mam_exchange.h): header | KeyFrame records | MapPoint records
HEADER_DTYPE = np.dtype([("n_kf", "<i4"), ("n_mp", "<i4"), ("agent", "<i4"), ("status", "<i4")])
KF_UPDATE_DTYPE = np.dtype([("row", "<i4"), ("q", "<f4", (4,)), ("t", "<f4", (3,))])
MP_UPDATE_DTYPE = np.dtype([("row", "<i4"), ("xyz", "<f4", (3,))])
assert HEADER_DTYPE.itemsize == 16 and KF_UPDATE_DTYPE.itemsize == 32 and MP_UPDATE_DTYPE.itemsize == 16


def compact_block_bytes(kf_cap: int, mp_cap: int) -> int:
    return HEADER_DTYPE.itemsize + kf_cap * KF_UPDATE_DTYPE.itemsize + mp_cap * MP_UPDATE_DTYPE.itemsize


def dedup_sources(windows):
    """The write-back of a batch of LBA windows as one deduplicated record set: `windows` = [(pose_id, pose_fixed,
    point_id)] per window, in the order the windows' results are applied. Every optimised KeyFrame and every MapPoint
    once, taken from the LAST window holding it — the value the per-window write-backs (Optimizer.cc:1463-1497),
    applied in window order, leave in the map. Returns (kf_src, mp_src): int32 [n][2] (window, vertex index), in
    ascending vertex id."""
    kf, mp = {}, {}
    for w, (pid, fixed, mid) in enumerate(windows):
        for i in np.nonzero(np.asarray(fixed) == 0)[0]:
            kf[int(pid[i])] = (w, int(i))
        for i, m in enumerate(np.asarray(mid)):
            mp[int(m)] = (w, i)
    kf_src = np.array([kf[k] for k in sorted(kf)], np.int32).reshape(-1, 2)
    mp_src = np.array([mp[k] for k in sorted(mp)], np.int32).reshape(-1, 2)
    return kf_src, mp_src


class MapWindow(C.Structure):
    """mam_map_window: an LBA window's vertex ids and double vertex arrays (device pointers)."""
    _fields_ = [("n_poses", C.c_int32), ("n_points", C.c_int32), ("pose_id", C.c_void_p), ("pose_fixed", C.c_void_p),
                ("point_id", C.c_void_p), ("point_bad", C.c_void_p), ("pose_q", C.c_void_p), ("pose_t", C.c_void_p),
                ("point_xyz", C.c_void_p)]


def _bind():
    L = lib()
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


def _as_torch_stream(stream: int, device):
    """A raw HIP stream handle as a torch stream (0 = the device's default stream)."""
    import torch

    cur = torch.cuda.current_stream(device)
    if int(stream) == cur.cuda_stream:
        return cur
    if int(stream) == 0:
        return torch.cuda.default_stream(device)
    return torch.cuda.ExternalStream(int(stream), device=device)


def _all_gather(recv, send, world, group):
    """all_gather_into_tensor of one block per rank (RCCL on the GPU; gloo on host tensors, or staged through the
    host for CUDA tensors in the one-GPU multi-rank tests)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        recv.copy_(send)
    elif dist.get_backend(group) == "gloo":
        if send.is_cuda:
            torch.cuda.current_stream(send.device).synchronize()
            parts = [torch.empty(send.numel(), dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, send.cpu(), group=group)
            recv.copy_(torch.cat(parts))
        else:
            dist.all_gather(list(recv.view(world, -1).unbind(0)), send, group=group)
    else:
        dist.all_gather_into_tensor(recv, send, group=group)


class CompactExchange:
    """The per-step exchange of the bench's LocalMapping leg: each rank packs the deduplicated write-back of all its
    windows (mam_exchange_pack_sources: 32-byte KeyFrame and 16-byte MapPoint records), one fixed-size all-gather of
    the blocks (capacities agreed at setup: the largest of any rank), every rank applies all blocks in rank order
    (mam_exchange_apply_compact)."""

    def __init__(self, kf_cap: int, mp_cap: int, device="cuda", group=None):
        import torch
        import torch.distributed as dist

        self.kf_cap, self.mp_cap = int(kf_cap), int(mp_cap)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.block_bytes = compact_block_bytes(self.kf_cap, self.mp_cap)
        self.send = torch.zeros(self.block_bytes, dtype=torch.uint8, device=device)
        self.recv = torch.zeros(self.world * self.block_bytes, dtype=torch.uint8, device=device)
        self._L = _bind()
        self._pack_stream = None
        self.gather_ms = []   # host wall of each all-gather (collective on torch's current stream, synchronised)

    def pack(self, d_windows: int, n_windows: int, d_kf_src: int, n_kf: int, d_mp_src: int, n_mp: int,
             mp_id_base: int, stream: int = 0):
        check(self._L.mam_exchange_pack_sources(int(n_windows), C.c_void_p(d_windows), C.c_void_p(d_kf_src), int(n_kf),
                                                C.c_void_p(d_mp_src), int(n_mp), int(mp_id_base), self.rank,
                                                C.c_void_p(self.send.data_ptr()), self.kf_cap, self.mp_cap,
                                                C.c_void_p(stream)), "mam_exchange_pack_sources")
        self._pack_stream = int(stream)

    def gather(self, timed: bool = False):
        import time

        import torch

        if self._pack_stream is not None and self.send.is_cuda:
            torch.cuda.current_stream(self.send.device).wait_stream(_as_torch_stream(self._pack_stream, self.send.device))
        if timed and self.send.is_cuda:
            torch.cuda.current_stream(self.send.device).synchronize()
            t0 = time.perf_counter()
        _all_gather(self.recv, self.send, self.world, self.group)
        if timed and self.send.is_cuda:
            torch.cuda.current_stream(self.send.device).synchronize()
            self.gather_ms.append((time.perf_counter() - t0) * 1e3)
        return self.recv

    def apply(self, d_kf_table: int, kf_rows: int, d_mp_table: int, mp_rows: int, d_status: int, stream: int = 0):
        import torch

        if self.send.is_cuda:
            _as_torch_stream(stream, self.send.device).wait_stream(torch.cuda.current_stream(self.send.device))
        check(self._L.mam_exchange_apply_compact(C.c_void_p(self.recv.data_ptr()), self.world, self.kf_cap,
                                                 self.mp_cap, C.c_void_p(d_kf_table), int(kf_rows),
                                                 C.c_void_p(d_mp_table), int(mp_rows), C.c_void_p(d_status),
                                                 C.c_void_p(stream)), "mam_exchange_apply_compact")


    def read_windows(self, d_kf_table: int, kf_cap: int, d_mp_table: int, mp_cap: int, mp_id_base: int,
                     d_windows: int, n_windows: int, max_rows: int, d_status: int, stream: int = 0):
        """The windows' LBA inputs from the (just applied) shared tables, on `stream` (mam_map_read_windows)."""
        check(self._L.mam_map_read_windows(C.c_void_p(d_kf_table), int(kf_cap), C.c_void_p(d_mp_table), int(mp_cap),
                                           int(mp_id_base), int(n_windows), C.c_void_p(d_windows), int(max_rows),
                                           C.c_void_p(d_status), C.c_void_p(stream)), "mam_map_read_windows")


class MapUpdateExchange:
    """Fixed-capacity all-gather of update blocks. `device` is where the send/receive buffers live (a CUDA device
    for the product path; "cpu" with the gloo backend for host-side tests of the collective)."""

    def __init__(self, capacity: int = 4096, device="cuda", group=None):
        import torch
        import torch.distributed as dist

        self.capacity = int(capacity)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        nbytes = (self.capacity + 1) * RECORD_BYTES
        self.send = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        self.recv = torch.zeros(self.world * nbytes, dtype=torch.uint8, device=device)
        self._L = None
        self._pack_stream = None   # raw HIP stream the last pack_lba ran on (the collective must wait for it)

    def _torch_stream(self, stream: int):
        import torch

        if stream is None or not self.send.is_cuda:
            return None
        cur = torch.cuda.current_stream(self.send.device)
        if int(stream) == cur.cuda_stream:
            return cur
        if int(stream) == 0:
            return torch.cuda.default_stream(self.send.device)
        return torch.cuda.ExternalStream(int(stream), device=self.send.device)

    @property
    def block_bytes(self) -> int:
        return (self.capacity + 1) * RECORD_BYTES

    def gather(self):
        """All-gather every agent's block into `recv` (rank order). Returns `recv`."""
        import torch
        import torch.distributed as dist

        # order the collective after the pack kernel: torch runs it on its current stream, pack_lba ran on a raw one
        if self._pack_stream is not None:
            ps = self._torch_stream(self._pack_stream)
            if ps is not None:
                torch.cuda.current_stream(self.send.device).wait_stream(ps)
        if self.world == 1:
            self.recv.copy_(self.send)
        elif dist.get_backend(self.group) == "gloo":
            if self.send.is_cuda:   # gloo gathers host tensors: stage through the host (tests of the multi-rank path)
                torch.cuda.current_stream(self.send.device).synchronize()
                parts = [torch.empty(self.send.numel(), dtype=torch.uint8) for _ in range(self.world)]
                dist.all_gather(parts, self.send.cpu(), group=self.group)
                self.recv.copy_(torch.cat(parts))
            else:
                dist.all_gather(list(self.recv.view(self.world, -1).unbind(0)), self.send, group=self.group)
        else:
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        return self.recv

    # ---- device kernels (product path)
    def _lib(self):
        if self._L is None:
            self._L = _bind()
        return self._L

    def pack_lba(self, d_pose_q: int, d_pose_t: int, d_pose_id: int, d_pose_fixed: int, n_poses: int,
                 d_point_xyz: int, d_point_id: int, d_point_bad: int | None, n_points: int, stream: int = 0,
                 agent: int | None = None):
        """Pack one LBA write-back (device pointers) into the send block on `stream`."""
        a = self.rank if agent is None else int(agent)
        check(self._lib().mam_exchange_pack_lba(
            C.c_void_p(d_pose_q), C.c_void_p(d_pose_t), C.c_void_p(d_pose_id), C.c_void_p(d_pose_fixed), n_poses,
            C.c_void_p(d_point_xyz), C.c_void_p(d_point_id), C.c_void_p(d_point_bad or 0), n_points, a,
            C.c_void_p(self.send.data_ptr()), self.capacity, C.c_void_p(stream)), "mam_exchange_pack_lba")
        self._pack_stream = int(stream)

    def apply(self, d_kf_table: int, kf_cap: int, d_mp_table: int, mp_cap: int, d_status: int, stream: int = 0,
              gathered: int | None = None, n_agents: int | None = None, capacity: int | None = None):
        """Apply the gathered blocks (default: `recv`) to the device tables, agent 0 first. `stream` is ordered after
        the collective (torch's current stream) before the apply kernel reads `recv`. With window blocks
        (pack_windows) pass the per-window capacity and n_agents = world x windows."""
        cap = self.capacity if capacity is None else int(capacity)
        nb = n_agents or self.world
        if gathered is None and nb * (cap + 1) * RECORD_BYTES > self.recv.numel():
            raise ValueError(f"apply: {nb} blocks of {cap + 1} records exceed the receive buffer")
        import torch

        if self.send.is_cuda:
            st = self._torch_stream(stream)
            if st is not None:
                st.wait_stream(torch.cuda.current_stream(self.send.device))
        check(self._lib().mam_exchange_apply(
            C.c_void_p(gathered or self.recv.data_ptr()), nb, cap,
            C.c_void_p(d_kf_table), int(kf_cap), C.c_void_p(d_mp_table), int(mp_cap), C.c_void_p(d_status),
            C.c_void_p(stream)), "mam_exchange_apply")

    def pack_windows(self, d_windows: int, n_windows: int, mp_id_base: int, capacity: int, stream: int = 0,
                     agent: int | None = None):
        """Pack n_windows LBA results (device descriptor array) into the send buffer, one block of `capacity` + 1
        records per window (the send buffer must hold n_windows blocks: construct with capacity = n_windows *
        (capacity + 1) - 1)."""
        a = self.rank if agent is None else int(agent)
        if n_windows * (capacity + 1) * RECORD_BYTES > self.send.numel():
            raise ValueError(f"pack_windows: {n_windows} blocks of {capacity + 1} records exceed the send buffer")
        check(self._lib().mam_exchange_pack_windows(int(n_windows), C.c_void_p(d_windows), int(mp_id_base), a,
                                                    C.c_void_p(self.send.data_ptr()), int(capacity),
                                                    C.c_void_p(stream)), "mam_exchange_pack_windows")
        self._pack_stream = int(stream)

    def read_windows(self, d_kf_table: int, kf_cap: int, d_mp_table: int, mp_cap: int, mp_id_base: int,
                     d_windows: int, n_windows: int, max_rows: int, d_status: int, stream: int = 0):
        """The windows' LBA inputs from the (just applied) shared tables, on `stream`."""
        check(self._lib().mam_map_read_windows(C.c_void_p(d_kf_table), int(kf_cap), C.c_void_p(d_mp_table),
                                               int(mp_cap), int(mp_id_base), int(n_windows), C.c_void_p(d_windows),
                                               int(max_rows), C.c_void_p(d_status), C.c_void_p(stream)),
              "mam_map_read_windows")

    @staticmethod
    def check_status(status_tensor):
        """Raise if an apply flagged a malformed block or an id outside the tables (synchronises)."""
        v = int(status_tensor.reshape(-1)[0].item())
        if v != 0:
            raise RuntimeError(f"mam_exchange_apply: status {v} (malformed header or id outside the tables)")
