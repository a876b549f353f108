"""Shared-map update exchange between agents, one agent per GPU (include/mam_exchange.h).

After each step's LocalBundleAdjustment windows an agent packs their write-back (optimised KeyFrame poses, MapPoint
positions, bad flags — what src/Optimizer.cc:1463-1497 writes into the shared Atlas under mMutexMapUpdate),
deduplicated over its windows, into one fixed-size compact block on the GPU (`CompactExchange.pack`), the blocks of
all agents are all-gathered (`torch.distributed.all_gather_into_tensor`: RCCL over xGMI on MI355X, gloo on CPU), and
every agent applies the gathered blocks to its device-resident shared tables in agent-id order
(`CompactExchange.apply`), so all replicas hold identical bytes. One collective per step, fixed size: no
all-gatherv, no count exchange.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib

_SIGS = {
    "mam_map_read_windows": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p,
                                       C.c_int, C.c_void_p, C.c_void_p]),
    "mam_exchange_compact_block_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "mam_exchange_pack_sources": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64,
                                            C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "mam_exchange_apply_compact": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64,
                                             C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
    "mam_copy_rows": (C.c_int, [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                C.c_int, C.c_void_p, C.c_int64, C.c_void_p]),
    "mam_map_perturb": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int,
                                  C.c_uint64, C.c_float, C.c_float, C.c_float, C.c_void_p, C.c_void_p]),
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


class RowTable(C.Structure):
    """mam_row_table: one table of a mam_copy_rows launch (device pointers, byte strides)."""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("row_bytes", C.c_int64), ("src_stride", C.c_int64),
                ("dst_stride", C.c_int64), ("src_row_offset", C.c_int64)]


def copy_rows(tables, src_rows, dst_rows, flags=None, stream: int = 0):
    """mam_copy_rows: rows src_rows[i] -> dst_rows[i] of every table [(src_ptr, dst_ptr, row_bytes, src_stride,
    dst_stride, src_row_offset)] in one launch (<= 8 tables, <= 64 rows); flags = (flag_a_ptr, flag_b_ptr,
    flag_stride_bytes, cols, flags_ptr, flags_stride_bytes) also sets flags[dst][j] = a[src][j] >= 0 or b[src][j] >= 0."""
    L = _bind()
    tb = (RowTable * max(1, len(tables)))(*[RowTable(*t) for t in tables])
    n = len(src_rows)
    sr = (C.c_int32 * max(1, n))(*[int(x) for x in src_rows])
    dr = (C.c_int32 * max(1, n))(*[int(x) for x in dst_rows])
    fa = fb = fl = None
    fs = fc = fls = 0
    if flags is not None:
        fa, fb, fs, fc, fl, fls = flags
        fs //= 4   # int32 elements
    check(L.mam_copy_rows(len(tables), tb, n, sr, dr, C.c_void_p(fa), C.c_void_p(fb), int(fs), int(fc), C.c_void_p(fl),
                          int(fls), C.c_void_p(stream)), "mam_copy_rows")


def map_perturb(d_kf_table: int, kf_rows: int, d_kf_idx: int, n_kf: int, d_mp_table: int, mp_rows: int, d_mp_idx: int,
                n_mp: int, seed: int, sigma_q: float, sigma_t: float, sigma_x: float, d_status: int, stream: int = 0):
    """mam_map_perturb: the synthetic map's new keyframes / MapPoints at a perturbed state (deterministic in seed)."""
    check(_bind().mam_map_perturb(C.c_void_p(d_kf_table), int(kf_rows), C.c_void_p(d_kf_idx), int(n_kf),
                                  C.c_void_p(d_mp_table), int(mp_rows), C.c_void_p(d_mp_idx), int(n_mp),
                                  int(seed) & 0xFFFFFFFFFFFFFFFF, float(sigma_q), float(sigma_t), float(sigma_x),
                                  C.c_void_p(d_status), C.c_void_p(stream)), "mam_map_perturb")


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
        if recv.data_ptr() != send.data_ptr():
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
        # one rank: the gathered blocks are its own block (no copy)
        self.recv = self.send if self.world == 1 else torch.zeros(self.world * self.block_bytes, dtype=torch.uint8,
                                                                   device=device)
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

    @staticmethod
    def check_status(status_tensor):
        """Raise if an apply flagged a malformed block or a row outside the tables (synchronises)."""
        v = int(status_tensor.reshape(-1)[0].item())
        if v != 0:
            raise RuntimeError(f"mam_exchange_apply_compact: status {v} (malformed header or row outside the tables)")
