"""TEST INFRASTRUCTURE ONLY — numpy restatement of the shared-map update exchange (include/mam_exchange.h).

Packing follows the LocalBundleAdjustment write-back (src/Optimizer.cc:1478-1494): non-fixed poses only (the
reference writes back lLocalKeyFrames; fixed cameras are untouched), quaternion cast to float and renormalised in
float (Sophus::SE3f(Quaternionf, t) normalises, so3.hpp:481-487, with Eigen's SSE reduction order), positions cast to
float. `writeback` is one window's write-back applied directly (the reference's sequential semantics); the compact
blocks (`pack_sources`, `apply_compact`) must leave the same tables. Application is in agent order (deterministic
replacement for the reference's mutex-ordered last-writer-wins, Optimizer.cc:1463).
Parity: the exchange has no reference counterpart to pin against (the reference shares pointers); the
restatement defines the contract and the GPU kernels must match it byte for byte.
"""
from __future__ import annotations

import numpy as np

ERR_CAPACITY, ERR_ARG = -2, -4


def sophus_normalize(q):
    """Sophus::SO3f::normalize (so3.hpp:481-487) of a float quaternion (x, y, z, w): coeffs / norm(), the norm of the
    4-float vector as Eigen's SSE packet reduction sums it (predux<Packet4f>: (x^2 + z^2) + (y^2 + w^2))."""
    q = np.asarray(q, np.float32)
    sq = (q * q).astype(np.float32)
    n = np.sqrt(np.float32(np.float32(sq[0] + sq[2]) + np.float32(sq[1] + sq[3])))
    return (q / np.float32(n)).astype(np.float32)


def writeback(kf_table, mp_table, pose_q, pose_t, pose_id, pose_fixed, point_xyz, point_row, point_bad=None):
    """One LocalBundleAdjustment window's write-back into the shared tables, in place (Optimizer.cc:1478-1494):
    every non-fixed pose KeyFrame::SetPose(SE3f(q.cast<float>(), t.cast<float>())) (Sophus renormalises q), every
    point MapPoint::SetWorldPos(pos.cast<float>()) and its bad flag. The reference applies the windows of several
    agents one after another under mMutexMapUpdate; applying windows in order with this function is the sequential
    semantics the compact blocks must reproduce."""
    for i in np.nonzero(np.asarray(pose_fixed) == 0)[0]:
        r = int(pose_id[i])
        kf_table[r, :4] = sophus_normalize(np.asarray(pose_q[i], np.float64).astype(np.float32))
        kf_table[r, 4:7] = np.asarray(pose_t[i], np.float64).astype(np.float32)
        kf_table[r, 7] = 1.0
    for i, r in enumerate(np.asarray(point_row)):
        mp_table[int(r), :3] = np.asarray(point_xyz[i], np.float64).astype(np.float32)
        mp_table[int(r), 3] = 1.0 if (point_bad is not None and point_bad[i]) else 0.0


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
        K[i]["row"] = int(pid[v])
        K[i]["q"] = sophus_normalize(np.asarray(pq[v], np.float64).astype(np.float32))
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
