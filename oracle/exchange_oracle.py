"""TEST INFRASTRUCTURE ONLY — numpy restatement of the shared-map update exchange (include/mam_exchange.h).

Packing follows the LocalBundleAdjustment write-back (src/Optimizer.cc:1478-1494): non-fixed poses only (the
reference writes back lLocalKeyFrames; fixed cameras are untouched), quaternion cast to float and renormalised in
float (Sophus::SE3f(Quaternionf, t) normalises, so3.hpp:481-487), positions cast to float. Application is in agent
order (deterministic replacement for the reference's mutex-ordered last-writer-wins, Optimizer.cc:1463).
Parity: the exchange has no reference counterpart to pin against (the reference shares pointers); the
restatement defines the contract and the GPU kernels must match it byte for byte.
"""
from __future__ import annotations

import numpy as np

UPDATE_HEADER, UPDATE_KF, UPDATE_MP = 0, 1, 2
UPDATE_DTYPE = np.dtype([("id", "<i8"), ("kind", "<i4"), ("agent", "<i4"), ("v", "<f4", (7,)), ("bad", "<i4"),
                         ("reserved", "<f4", (4,))])
ERR_CAPACITY, ERR_ARG = -2, -4


def pack_lba(pose_q, pose_t, pose_id, pose_fixed, point_xyz, point_id, point_bad, agent, capacity):
    out = np.zeros(capacity + 1, UPDATE_DTYPE)
    keep = np.nonzero(np.asarray(pose_fixed) == 0)[0]
    n_opt, n_pts = len(keep), len(point_id)
    total = n_opt + n_pts
    q = np.asarray(pose_q, np.float64)[keep].astype(np.float32)
    n = np.sqrt(((q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]) + q[:, 3] * q[:, 3]).astype(np.float32)
    q = (q / n[:, None]).astype(np.float32)
    t = np.asarray(pose_t, np.float64)[keep].astype(np.float32)
    k = min(n_opt, capacity)
    out["id"][1:1 + k] = np.asarray(pose_id)[keep][:k]
    out["kind"][1:1 + k] = UPDATE_KF
    out["agent"][1:1 + k] = agent
    out["v"][1:1 + k, :4] = q[:k]
    out["v"][1:1 + k, 4:] = t[:k]
    m = max(0, min(n_pts, capacity - n_opt))
    sl = slice(1 + n_opt, 1 + n_opt + m)
    out["id"][sl] = np.asarray(point_id)[:m]
    out["kind"][sl] = UPDATE_MP
    out["agent"][sl] = agent
    out["v"][sl, :3] = np.asarray(point_xyz, np.float64)[:m].astype(np.float32)
    if point_bad is not None:
        out["bad"][sl] = (np.asarray(point_bad)[:m] != 0).astype(np.int32)
    out["id"][0] = total if total <= capacity else ERR_CAPACITY
    out["kind"][0] = UPDATE_HEADER
    out["agent"][0] = agent
    return out


def apply(gathered, n_agents, capacity, kf_table, mp_table):
    """gathered: UPDATE_DTYPE [n_agents*(capacity+1)]; kf_table float32 [K,8]; mp_table float32 [M,4]. In place.
    Returns the status (0 or ERR_ARG)."""
    status = 0
    blocks = np.asarray(gathered).reshape(n_agents, capacity + 1)
    for a in range(n_agents):
        h = blocks[a, 0]
        cnt = int(h["id"])
        if int(h["kind"]) != UPDATE_HEADER or cnt < 0 or cnt > capacity:
            status = ERR_ARG
            continue
        for u in blocks[a, 1:1 + cnt]:
            i, kind = int(u["id"]), int(u["kind"])
            if kind == UPDATE_KF and 0 <= i < len(kf_table):
                kf_table[i, :7] = u["v"]
                kf_table[i, 7] = 1.0
            elif kind == UPDATE_MP and 0 <= i < len(mp_table):
                mp_table[i, :3] = u["v"][:3]
                mp_table[i, 3] = 1.0 if u["bad"] else 0.0
            else:
                status = ERR_ARG
    return status


# ---- compact blocks (mam_exchange_pack_sources / mam_exchange_apply_compact)
def pack_sources(results, kf_src, mp_src, mp_id_base, agent, kf_cap, mp_cap):
    """results: per window (pose_q, pose_t, pose_id, point_xyz, point_id, point_bad or None); returns the block bytes."""
    from mam3slam_amd.exchange import HEADER_DTYPE, KF_UPDATE_DTYPE, MP_UPDATE_DTYPE

    h = np.zeros(1, HEADER_DTYPE)
    K = np.zeros(kf_cap, KF_UPDATE_DTYPE)
    M = np.zeros(mp_cap, MP_UPDATE_DTYPE)
    nk, nm = len(kf_src), len(mp_src)
    h["n_kf"], h["n_mp"], h["agent"] = nk, nm, agent
    h["status"] = ERR_CAPACITY if (nk > kf_cap or nm > mp_cap) else 0
    for i, (w, v) in enumerate(np.asarray(kf_src)[:kf_cap]):
        pq, pt, pid = results[w][0], results[w][1], results[w][2]
        q = np.asarray(pq[v], np.float64).astype(np.float32)
        n = np.float32(np.sqrt(np.float32(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3])))
        K[i]["row"] = int(pid[v])
        K[i]["q"] = (q / n).astype(np.float32)
        K[i]["t"] = np.asarray(pt[v], np.float64).astype(np.float32)
    for i, (w, v) in enumerate(np.asarray(mp_src)[:mp_cap]):
        xyz, mid, bad = results[w][3], results[w][4], results[w][5]
        row = int(mid[v]) - int(mp_id_base)
        if bad is not None and bad[v]:
            row = row | -0x80000000
        M[i]["row"] = row
        M[i]["xyz"] = np.asarray(xyz[v], np.float64).astype(np.float32)
    return h.tobytes() + K.tobytes() + M.tobytes()


def apply_compact(gathered: bytes, n_agents, kf_cap, mp_cap, kf_table, mp_table):
    """In place, agent order; returns the status (0 or ERR_ARG)."""
    from mam3slam_amd.exchange import HEADER_DTYPE, KF_UPDATE_DTYPE, MP_UPDATE_DTYPE, compact_block_bytes

    bb = compact_block_bytes(kf_cap, mp_cap)
    status = 0
    for a in range(n_agents):
        blk = gathered[a * bb:(a + 1) * bb]
        h = np.frombuffer(blk[:16], HEADER_DTYPE)[0]
        if int(h["status"]) != 0 or not (0 <= h["n_kf"] <= kf_cap) or not (0 <= h["n_mp"] <= mp_cap):
            status = ERR_ARG
            continue
        K = np.frombuffer(blk[16:16 + 32 * kf_cap], KF_UPDATE_DTYPE)[:int(h["n_kf"])]
        M = np.frombuffer(blk[16 + 32 * kf_cap:], MP_UPDATE_DTYPE)[:int(h["n_mp"])]
        for u in K:
            r = int(u["row"])
            if 0 <= r < len(kf_table):
                kf_table[r, :4] = u["q"]
                kf_table[r, 4:7] = u["t"]
                kf_table[r, 7] = 1.0
            else:
                status = ERR_ARG
        for u in M:
            raw = int(u["row"])
            r = raw & 0x7FFFFFFF
            if r < len(mp_table):
                mp_table[r, :3] = u["xyz"]
                mp_table[r, 3] = 1.0 if raw < 0 else 0.0
            else:
                status = ERR_ARG
    return status
