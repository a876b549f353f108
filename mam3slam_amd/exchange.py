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
}


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
