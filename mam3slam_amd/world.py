"""A synthetic shared map (the merged Atlas several agents' LocalMapping threads optimise) and the LocalBundleAdjustment
windows cut from it, for the bench's LocalMapping leg and the exchange tests.

The reference's windows are cut from one map (Optimizer.cc:1118-1186: the keyframe and its covisible keyframes are
optimised, the other keyframes observing their MapPoints are fixed), so windows of different keyframes overlap and
their write-backs land on the same KeyFrames / MapPoints (Optimizer.cc:1463-1497). Here the map is a camera path
along a corridor: keyframe k at x = 0.1 k, MapPoints "homed" at a keyframe and observed by the 8 keyframes around it
(pixel noise at the keypoint's level, a fraction of gross outliers), with the poses and positions perturbed as a
running SLAM system leaves them. A window = `n_opt` consecutive keyframes + the keyframes outside it that observe its
points (fixed), as an id-ordered LBAProblem (keyframe id = index, MapPoint vertex id = n_kf + index, the reference's
mnId + maxKFid + 1).

The map state lives in two device tables shared with the exchange (include/mam_exchange.h): kf_table [n_kf][8] float
(Tcw quaternion xyzw, translation, written flag) and mp_table [n_mp][4] float (position, bad flag).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .lba import HUBER_MONO, LBAProblem, _rot_to_quat


@dataclass
class World:
    n_kf: int
    n_mp: int
    kf_table: np.ndarray     # float32 [n_kf][8]
    mp_table: np.ndarray     # float32 [n_mp][4]
    obs_kf: np.ndarray       # int32 [n_obs] observing keyframe, grouped by MapPoint (ascending), keyframe ascending
    obs_mp: np.ndarray       # int32 [n_obs]
    obs_uv: np.ndarray       # float32 [n_obs][2] keypoint
    obs_w: np.ndarray        # float32 [n_obs] invSigma2 of the keypoint's level
    mp_obs_off: np.ndarray   # int32 [n_mp + 1]
    home: np.ndarray         # int32 [n_mp] keyframe a MapPoint is homed at
    cam: np.ndarray          # float32 [1][4] pinhole fx, fy, cx, cy or [1][8] KannalaBrandt8 (cam_model 1)
    width: int
    height: int
    cam_model: int = 0


def _scale_tables():
    s = [np.float32(1.0)]
    for _ in range(7):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(1.2))))
    s = np.array(s, np.float32)
    return s, (np.float32(1.0) / (s * s)).astype(np.float32)


def make_world(n_kf: int = 800, pts_per_kf: int = 60, obs_span=(-3, 5), seed: int = 0, outlier_frac: float = 0.05,
               width: int = 1280, height: int = 720, f: float = 500.0, camera=None) -> World:
    """camera: a match.Camera (Pinhole / KannalaBrandt8) for the observations instead of the f-pinhole."""
    rng = np.random.default_rng(seed)
    scale, inv_s2 = _scale_tables()
    cam = np.array([[f, f, width / 2, height / 2]], np.float32) if camera is None else camera.params()[None, :]
    k = np.arange(n_kf)
    centres = np.stack([0.1 * k, 0.3 * np.sin(k / 7.0), np.zeros(n_kf)], 1)
    yaw = 0.05 * np.sin(k / 5.0)
    Rs = np.zeros((n_kf, 3, 3))
    Rs[:, 0, 0] = np.cos(yaw)
    Rs[:, 0, 2] = -np.sin(yaw)
    Rs[:, 1, 1] = 1.0
    Rs[:, 2, 0] = np.sin(yaw)
    Rs[:, 2, 2] = np.cos(yaw)
    ts = -np.einsum("kij,kj->ki", Rs, centres)
    # MapPoints homed at every keyframe, seen by keyframes home + obs_span
    n_mp = n_kf * pts_per_kf
    home = np.repeat(k, pts_per_kf).astype(np.int32)
    X = np.stack([centres[home, 0] + rng.uniform(-1.0, 1.0, n_mp), rng.uniform(-1.5, 1.5, n_mp),
                  rng.uniform(3.0, 8.0, n_mp)], 1)
    offs = np.arange(obs_span[0], obs_span[1])
    okf = (home[:, None] + offs[None, :]).reshape(-1)
    omp = np.repeat(np.arange(n_mp), len(offs))
    keep = (okf >= 0) & (okf < n_kf)
    okf, omp = okf[keep].astype(np.int32), omp[keep].astype(np.int32)
    Xc = np.einsum("nij,nj->ni", Rs[okf], X[omp]) + ts[okf]
    octv = rng.integers(0, 8, len(okf))
    if camera is None:
        u = f * Xc[:, 0] / Xc[:, 2] + width / 2
        v = f * Xc[:, 1] / Xc[:, 2] + height / 2
    else:
        u, v = camera.project_np(Xc).T
    u = u + rng.normal(0, 1, len(okf)) * scale[octv]
    v = v + rng.normal(0, 1, len(okf)) * scale[octv]
    u = u + 20.0 * (rng.random(len(okf)) < outlier_frac)
    obs_uv = np.stack([u, v], 1).astype(np.float32)          # mvKeysUn are float
    off = np.zeros(n_mp + 1, np.int32)
    np.add.at(off, omp + 1, 1)
    off = np.cumsum(off).astype(np.int32)
    # the map as a running system leaves it: poses ~0.5 deg / 2 cm off, points ~3 cm off, stored as float
    kf_table = np.zeros((n_kf, 8), np.float32)
    for i in range(n_kf):
        w = rng.normal(size=3)
        w *= np.deg2rad(0.5) / np.linalg.norm(w)
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / th
        dR = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
        q = _rot_to_quat(dR @ Rs[i])
        if q[3] < 0:
            q = -q
        q = q.astype(np.float32)
        q /= np.float32(np.linalg.norm(q.astype(np.float64)))
        kf_table[i, :4] = q
        kf_table[i, 4:7] = ts[i] + rng.normal(0, 0.02 / np.sqrt(3), 3)
        kf_table[i, 7] = 1.0
    mp_table = np.zeros((n_mp, 4), np.float32)
    mp_table[:, :3] = X + rng.normal(0, 0.03 / np.sqrt(3), X.shape)
    return World(n_kf, n_mp, kf_table, mp_table, okf, omp, obs_uv, inv_s2[octv].astype(np.float32), off, home, cam,
                 width, height, 0 if camera is None else int(camera.model))


def window(world: World, start: int, n_opt: int = 50, huber_delta: float = HUBER_MONO, iterations: int = 10):
    """The LocalBundleAdjustment graph of keyframes [start, start + n_opt) (Optimizer.cc:1118-1331), id-ordered:
    local keyframes optimised (keyframe 0, the map's init keyframe, fixed: :1220), the MapPoints they observe, the
    other keyframes observing those MapPoints fixed, one mono edge per observation by a window keyframe, per MapPoint
    in MapPoint order and keyframe order within it. Returns (LBAProblem with the map's current values, kf_ids,
    mp_ids) — the ids index world.kf_table / world.mp_table."""
    lo, hi = start, min(start + n_opt, world.n_kf)
    in_local = (world.obs_kf >= lo) & (world.obs_kf < hi)
    mps = np.unique(world.obs_mp[in_local])
    sel = np.isin(world.obs_mp, mps)
    okf, omp = world.obs_kf[sel], world.obs_mp[sel]
    kfs = np.unique(okf)
    fixed = ((kfs < lo) | (kfs >= hi) | (kfs == 0)).astype(np.uint8)
    kf_index = {int(x): i for i, x in enumerate(kfs)}
    mp_index = np.searchsorted(mps, omp)
    P = len(kfs)
    q = world.kf_table[kfs, :4].astype(np.float64)
    t = world.kf_table[kfs, 4:7].astype(np.float64)
    prob = LBAProblem(pose_id=kfs.astype(np.int64), pose_fixed=fixed, pose_q=q, pose_t=t,
                      point_id=(mps + world.n_kf).astype(np.int64),
                      point_xyz=world.mp_table[mps, :3].astype(np.float64),
                      edge_point=mp_index.astype(np.int32),
                      edge_pose=np.array([kf_index[int(x)] for x in okf], np.int32),
                      edge_obs=world.obs_uv[sel].astype(np.float64),
                      edge_inv_sigma2=world.obs_w[sel].astype(np.float64), cams=world.cam,
                      huber_delta=huber_delta, iterations=iterations, cam_model=world.cam_model).contiguous()
    assert P == len(prob.pose_id)
    return prob, kfs.astype(np.int64), mps.astype(np.int64)
