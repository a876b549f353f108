"""Synthetic matching / mapping inputs built around real extracted ORB features.

There is no dataset, vocabulary or map: the searches are fed structures generated from a frame's own
keypoints so that real matches exist, plus the adversarial cases the reference's control flow has
(duplicate MapPoints competing for one keypoint, pre-taken keypoints, bad / not-in-view points, wrong-level
predictions, Hamming ties, outliers behind the camera, empty windows).
"""
from __future__ import annotations

import os

import numpy as np

from .match import (FUSE_MP_DTYPE, LAST_ENTRY_DTYPE, LOCAL_MP_DTYPE, MP_TRACK_DTYPE, Camera, FrameData,
                    KannalaBrandt8, Pinhole, camera_center, epipole_12, fundamental_12)
from .orb import KP_DTYPE


def _backproject(cam: Camera, u, v, z):
    """Camera-frame points at depth z whose projections are the pixels (u, v) (Pinhole or KannalaBrandt8)."""
    r = cam.unproject_np(u, v)
    z = np.asarray(z, np.float64)
    return np.stack([r[..., 0] * z, r[..., 1] * z, z], -1)


def scale_tables(nlevels=8, scale=1.2):
    s = [np.float32(1.0)]
    for _ in range(nlevels - 1):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    s = np.array(s, np.float32)
    return s, (s * s).astype(np.float32)


def flip_bits(desc: np.ndarray, rng: np.random.Generator, kmax: int) -> np.ndarray:
    d = desc.copy()
    for i in range(len(d)):
        k = int(rng.integers(0, kmax + 1))
        for b in rng.choice(256, size=k, replace=False):
            d[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def make_frame_data(keys, desc, w, h, rng=None, taken_frac=0.0) -> FrameData:
    sf, s2 = scale_tables()
    taken = None
    if rng is not None and taken_frac > 0:
        taken = (rng.random(len(keys)) < taken_frac).astype(np.uint8)
    return FrameData(keys=np.ascontiguousarray(keys, KP_DTYPE), desc=np.ascontiguousarray(desc, np.uint8), width=w,
                     height=h, scale_factors=sf, level_sigma2=s2, taken=taken)


def local_mappoints(F: FrameData, rng: np.random.Generator, frac=0.8, dup_frac=0.15, n_random=60, kflip=14):
    """MapPoint track records around F's keypoints (what Frame::isInFrustum leaves in each MapPoint)."""
    n = len(F.keys)
    sel = rng.choice(n, size=int(n * frac), replace=False)
    m = len(sel)
    mps = np.zeros(m, MP_TRACK_DTYPE)
    k = F.keys[sel]
    mps["proj_x"] = k["x"] + rng.normal(0, 0.8, m).astype(np.float32)
    mps["proj_y"] = k["y"] + rng.normal(0, 0.8, m).astype(np.float32)
    mps["view_cos"] = rng.uniform(0.99, 1.0, m).astype(np.float32)
    mps["track_depth"] = rng.uniform(0.5, 60, m).astype(np.float32)
    mps["track_in_view"] = (rng.random(m) < 0.95).astype(np.int32)
    mps["scale_level"] = np.clip(k["octave"] + rng.integers(0, 2, m), 0, 7)
    mps["is_bad"] = (rng.random(m) < 0.02).astype(np.int32)
    mps["nobs"] = rng.integers(0, 6, m) * (rng.random(m) < 0.97) + (rng.random(m) < 0.97)
    mps["desc"] = flip_bits(F.desc[sel], rng, kflip)
    # duplicates: near-identical MapPoints competing for the same keypoint (greedy conflicts)
    nd = int(m * dup_frac)
    dup = mps[rng.choice(m, size=nd, replace=False)].copy()
    dup["proj_x"] += rng.normal(0, 0.5, nd).astype(np.float32)
    dup["desc"] = flip_bits(dup["desc"], rng, 3)
    # random points: mostly empty windows / no good match
    rnd = np.zeros(n_random, MP_TRACK_DTYPE)
    rnd["proj_x"] = rng.uniform(-20, F.width + 20, n_random)
    rnd["proj_y"] = rng.uniform(-20, F.height + 20, n_random)
    rnd["view_cos"] = rng.uniform(0.9, 1.0, n_random)
    rnd["track_in_view"] = 1
    rnd["scale_level"] = rng.integers(0, 8, n_random)
    rnd["nobs"] = 1
    rnd["desc"] = rng.integers(0, 256, (n_random, 32), dtype=np.uint8)
    allm = np.concatenate([mps, dup, rnd])
    return allm[rng.permutation(len(allm))]


def local_world_mappoints(F: FrameData, cam: Pinhole, rng: np.random.Generator, frac=0.8, dup_frac=0.15,
                          n_random=60, kflip=14, seen_frac=0.05, sel=None):
    """Local-map MapPoints in world coordinates around frame F (F.pose = Tcw): Tracking::mvpLocalMapPoints as
    SearchLocalPoints receives them (LOCAL_MP_DTYPE). Points back-project F's keypoints to depths 1.5-40 m, so
    Frame::isInFrustum re-projects them near their keypoints; their normals point from the camera centre with a
    spread (a few beyond the 60 deg viewing limit), the scale-invariance range brackets the current distance (a few
    outside it, so PredictScale sees every level), and the usual adversarial cases ride along: bad points, points
    already seen this frame, duplicates competing for one keypoint, points behind the camera or outside the image."""
    from .match import camera_center, quat_to_rot

    q, t = F.pose
    R = quat_to_rot(q).astype(np.float64)
    Ow = camera_center(F.pose).astype(np.float64)
    n = len(F.keys)
    if sel is None:   # the keypoints the local map's points project near (coherent_selection: scene-consistent)
        sel = rng.choice(n, size=int(n * frac), replace=False)
    m = len(sel)
    k = F.keys[sel]
    z = rng.uniform(1.5, 40.0, m)
    u = k["x"] + rng.normal(0, 0.8, m)
    v = k["y"] + rng.normal(0, 0.8, m)
    Xc = _backproject(cam, u, v, z)
    Xw = (Xc - t[None, :].astype(np.float64)) @ R
    mps = np.zeros(m, LOCAL_MP_DTYPE)
    mps["pos"] = Xw.astype(np.float32)
    d = Xw - Ow[None, :]
    dist = np.linalg.norm(d, axis=1)
    nrm = d / dist[:, None] + rng.normal(0, 0.35, (m, 3))
    mps["normal"] = (nrm / np.linalg.norm(nrm, axis=1)[:, None]).astype(np.float32)
    # mfMaxDistance = dist * 1.2^level_ref (the level the MapPoint was created at), mfMinDistance = max / 1.2^7
    lvl_ref = rng.integers(0, 8, m)
    maxd = dist * (1.2 ** lvl_ref) * rng.uniform(0.95, 1.05, m)
    out_rng = rng.random(m) < 0.05
    maxd[out_rng] = dist[out_rng] * rng.uniform(0.3, 0.8, out_rng.sum())
    mps["max_distance"] = maxd.astype(np.float32)
    mps["min_distance"] = (maxd / 1.2 ** 7).astype(np.float32)
    mps["is_bad"] = (rng.random(m) < 0.02).astype(np.int32)
    mps["seen"] = (rng.random(m) < seen_frac).astype(np.int32)
    mps["nobs"] = rng.integers(0, 6, m) * (rng.random(m) < 0.97) + (rng.random(m) < 0.97)
    mps["desc"] = flip_bits(F.desc[sel], rng, kflip)
    nd = int(m * dup_frac)
    dup = mps[rng.choice(m, size=nd, replace=False)].copy()
    dup["pos"] += rng.normal(0, 0.004, (nd, 3)).astype(np.float32)
    dup["desc"] = flip_bits(dup["desc"], rng, 3)
    rnd = np.zeros(n_random, LOCAL_MP_DTYPE)
    rnd["pos"] = (Ow[None, :] + rng.uniform(-30, 30, (n_random, 3))).astype(np.float32)
    rnd["normal"] = rng.normal(0, 1, (n_random, 3)).astype(np.float32)
    rnd["normal"] /= np.linalg.norm(rnd["normal"], axis=1)[:, None]
    rnd["max_distance"] = rng.uniform(5, 80, n_random).astype(np.float32)
    rnd["min_distance"] = rnd["max_distance"] / np.float32(1.2 ** 7)
    rnd["nobs"] = 1
    rnd["desc"] = rng.integers(0, 256, (n_random, 32), dtype=np.uint8)
    allm = np.concatenate([mps, dup, rnd])
    return allm[rng.permutation(len(allm))]


def pinhole(w, h, f=500.0) -> Pinhole:
    return Pinhole(np.float32(f), np.float32(f), np.float32(w / 2), np.float32(h / 2))


# the reference's test/settingsForTest_00.yaml (the testMultiAgentSystem agents' KannalaBrandt8 at 960 x 960) and its
# sibling settingsForTest_01.yaml: configuration data for BASELINE configs[3], kept in the package's data directory
TEST_SETTINGS = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "settings",
                              f"settingsForTest_0{i}.yaml") for i in (0, 1)]


def kannala_brandt8(w=960, h=960, settings: str | None = None) -> KannalaBrandt8:
    """Camera 1 of the test settings file (Camera.type KannalaBrandt8, Camera1.*), read with settings.Settings; other
    image sizes scale fx, cx by w / Camera.width and fy, cy by h / Camera.height (the distortion acts on the ray angle
    and is unchanged)."""
    from .settings import Settings

    return Settings(settings or TEST_SETTINGS[0]).camera_scaled(w, h)


def small_pose(rng, rot=0.01, trans=0.05):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(-rot, rot)
    q = np.append(axis * np.sin(ang / 2), np.cos(ang / 2)).astype(np.float32)
    q /= np.float32(np.linalg.norm(q))
    t = rng.uniform(-trans, trans, 3).astype(np.float32)
    return q.astype(np.float32), t


def perturb_pose(pose, rng, rot=0.005, trans=0.02):
    """(dq, dt) * pose for a random small (dq, dt): a motion model's guess near the true Tcw (float32)."""
    from .match import quat_to_rot

    dq, dt = small_pose(rng, rot=rot, trans=trans)
    ax, ay, az, aw = [float(x) for x in dq]
    bx, by, bz, bw = [float(x) for x in pose[0]]
    q = np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                  aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])
    q = (q / np.linalg.norm(q)).astype(np.float32)
    t = (quat_to_rot(dq).astype(np.float64) @ np.asarray(pose[1], np.float64) + dt).astype(np.float32)
    return q, t


def coherent_selection(F: FrameData, cam: Camera, frac: float, salt: int, cell: float = 0.25) -> np.ndarray:
    """Indices of F's keypoints whose scene point — the keypoint's ray on the canvas plane (synth.PLANE_DEPTH, world
    coordinates under F.pose) — lies in a "mapped" cell of the plane (cell x cell world units, ~13 px of a 640-wide
    view): a hash of the cell below `frac`. The same scene regions are mapped in every view, so a keyframe's keypoints
    without a MapPoint are mostly unmapped in its neighbours too (as in a real map; an independent draw per frame would
    leave only frac^2 of the correspondences free in both keyframes of a CreateNewMapPoints pair)."""
    from . import synth
    from .match import quat_to_rot

    q, t = F.pose
    R = quat_to_rot(q).astype(np.float64)
    Ow = -R.T @ t.astype(np.float64)
    n = len(F.keys)
    ray_c = np.concatenate([cam.unproject_np(F.keys["x"], F.keys["y"]), np.ones((n, 1))], 1)
    ray_w = ray_c @ R   # R^T d
    X = Ow[None, :] + ((synth.PLANE_DEPTH - Ow[2]) / ray_w[:, 2])[:, None] * ray_w
    ix = np.floor(X[:, 0] / cell).astype(np.int64).astype(np.uint64)
    iy = np.floor(X[:, 1] / cell).astype(np.int64).astype(np.uint64)
    z = ix * np.uint64(0x9E3779B97F4A7C15) ^ iy * np.uint64(0xC2B2AE3D27D4EB4F) ^ np.uint64(salt) * np.uint64(0x165667B1)
    z = (z ^ (z >> np.uint64(31))) * np.uint64(0xBF58476D1CE4E5B9)
    z = z ^ (z >> np.uint64(29))
    return np.nonzero((z >> np.uint64(40)).astype(np.float64) / float(1 << 24) < frac)[0]


def motion_last_frame(F: FrameData, cam: Pinhole, rng: np.random.Generator, frac=0.75, n_out=80, kflip=12,
                      sel=None):
    """LastFrame entries whose MapPoints re-project near F's keypoints under F.pose (Tcw); sel: the keypoints that
    get one (default: a random `frac` of them)."""
    from .match import quat_to_rot

    q, t = F.pose
    R = quat_to_rot(q)
    n = len(F.keys)
    if sel is None:
        sel = rng.choice(n, size=int(n * frac), replace=False)
    m = len(sel)
    k = F.keys[sel]
    z = rng.uniform(2.0, 12.0, m)
    u = k["x"] + rng.normal(0, 0.7, m)
    v = k["y"] + rng.normal(0, 0.7, m)
    Xc = _backproject(cam, u, v, z)
    Xw = (Xc - t[None, :].astype(np.float64)) @ R.astype(np.float64)   # R^T (Xc - t)
    last = np.zeros(m, LAST_ENTRY_DTYPE)
    last["pos"] = Xw.astype(np.float32)
    last["angle"] = ((k["angle"] + rng.normal(0, 4.0, m)) % 360).astype(np.float32)
    last["octave"] = np.clip(k["octave"] + rng.integers(-1, 2, m), 0, 7)
    last["valid"] = (rng.random(m) < 0.95).astype(np.int32)
    last["nobs"] = rng.integers(1, 8, m) * (rng.random(m) < 0.98)
    last["desc"] = flip_bits(F.desc[sel], rng, kflip)
    # a block with a consistent large rotation (a minority histogram bin) and pure outliers
    rot = rng.random(m) < 0.08
    last["angle"][rot] = (last["angle"][rot] + 90.0) % 360
    out = np.zeros(n_out, LAST_ENTRY_DTYPE)
    out["pos"] = rng.uniform(-8, 8, (n_out, 3)).astype(np.float32)
    out["angle"] = rng.uniform(0, 360, n_out)
    out["octave"] = rng.integers(0, 8, n_out)
    out["valid"] = 1
    out["nobs"] = 1
    out["desc"] = rng.integers(0, 256, (n_out, 32), dtype=np.uint8)
    allm = np.concatenate([last, out])
    return allm[rng.permutation(len(allm))]


def quantize(desc: np.ndarray, centroids: np.ndarray, node_ids: np.ndarray):
    """Nearest-centroid Hamming quantizer (a one-level stand-in for DBoW2's transform at levelsup=4)."""
    x = np.unpackbits(desc, axis=1).astype(np.int16)
    c = np.unpackbits(centroids, axis=1).astype(np.int16)
    d = (x[:, None, :] != c[None, :, :]).sum(-1)
    lab = d.argmin(1)
    fv = {}
    for i, l in enumerate(lab):
        fv.setdefault(int(node_ids[l]), []).append(i)
    return fv


def keyframe_pair(F: FrameData, cam: Pinhole, rng: np.random.Generator, n_nodes=24, kflip=10, baseline=0.3):
    """(KF1, KF2, F12, ep): KF2 sees KF1's features shifted by a horizontal disparity (x-translation rig), so
    the epipolar lines are near-horizontal and many pairs satisfy the constraint; plus extra features."""
    n = len(F.keys)
    k1 = F.keys.copy()
    sel = rng.choice(n, size=int(n * 0.8), replace=False)
    k2 = F.keys[sel].copy()
    disp = rng.uniform(3, 40, len(sel)).astype(np.float32)
    k2["x"] = np.clip(k2["x"] - disp, 0, F.width - 1)
    k2["y"] = k2["y"] + rng.normal(0, 0.8, len(sel)).astype(np.float32)
    k2["octave"] = np.clip(k2["octave"] + rng.integers(-1, 2, len(sel)), 0, 7)
    k2["angle"] = ((k2["angle"] + rng.normal(0, 5, len(sel))) % 360).astype(np.float32)
    d2 = flip_bits(F.desc[sel], rng, kflip)
    ne = n // 5
    ke = np.zeros(ne, KP_DTYPE)
    ke["x"] = rng.uniform(0, F.width - 1, ne)
    ke["y"] = rng.uniform(0, F.height - 1, ne)
    ke["octave"] = rng.integers(0, 8, ne)
    ke["angle"] = rng.uniform(0, 360, ne)
    ke["size"] = 31
    de = rng.integers(0, 256, (ne, 32), dtype=np.uint8)
    k2 = np.concatenate([k2, ke])
    d2 = np.concatenate([d2, de])
    perm = rng.permutation(len(k2))
    k2, d2 = k2[perm], d2[perm]
    centroids = rng.integers(0, 256, (n_nodes, 32), dtype=np.uint8)
    node_ids = np.sort(rng.choice(1_000_000, size=n_nodes, replace=False)).astype(np.uint32)
    KF1 = make_frame_data(k1, F.desc, F.width, F.height)
    KF2 = make_frame_data(k2, d2, F.width, F.height)
    KF1.has_mp = (rng.random(len(k1)) < 0.2).astype(np.uint8)
    KF2.has_mp = (rng.random(len(k2)) < 0.2).astype(np.uint8)
    KF1.featvec = quantize(KF1.desc, centroids, node_ids)
    KF2.featvec = quantize(KF2.desc, centroids, node_ids)
    q0 = np.array([0, 0, 0, 1], np.float32)
    KF1.pose = (q0, np.zeros(3, np.float32))
    KF2.pose = (q0, np.array([-baseline, 0.0, -0.05], np.float32))
    K = np.array([[cam.fx, 0, cam.cx], [0, cam.fy, cam.cy], [0, 0, 1]], np.float32)
    F12 = fundamental_12(KF1.pose, KF2.pose, K, K)
    ep = epipole_12(KF1.pose, KF2.pose, cam)
    return KF1, KF2, F12, ep


def keyframe_pair_3d(F: FrameData, cam: Camera, rng: np.random.Generator, n_nodes=24, kflip=10, baseline=0.3,
                     noise=0.6):
    """(KF1, KF2) for SearchForTriangulation with any camera model: KF1's keypoints back-projected to 2-12 m and
    re-projected into KF2 (baselined, slightly rotated; project_np) with pixel noise, so the pairs satisfy Pinhole
    epipolar lines or KannalaBrandt8 two-view triangulation up to the noise; plus random extra features, MapPoint
    flags and FeatureVectors from a one-level quantizer. Poses are set (Tcw)."""
    from .match import quat_to_rot

    n = len(F.keys)
    k1 = F.keys.copy()
    sel = rng.choice(n, size=int(n * 0.8), replace=False)
    z = rng.uniform(2.0, 12.0, len(sel))
    X1 = _backproject(cam, k1["x"][sel], k1["y"][sel], z)
    ang = 0.03
    q2 = np.array([0.0, np.sin(ang / 2), 0.0, np.cos(ang / 2)], np.float32)
    t2 = np.array([-baseline, 0.02, -0.05], np.float32)
    X2 = X1 @ quat_to_rot(q2).astype(np.float64).T + t2[None, :].astype(np.float64)
    uv = cam.project_np(X2) + rng.normal(0, noise, (len(sel), 2))
    ok = (X2[:, 2] > 0.1) & (uv[:, 0] >= 0) & (uv[:, 0] < F.width - 1) & (uv[:, 1] >= 0) & (uv[:, 1] < F.height - 1)
    sel, uv = sel[ok], uv[ok]
    k2 = F.keys[sel].copy()
    k2["x"] = uv[:, 0].astype(np.float32)
    k2["y"] = uv[:, 1].astype(np.float32)
    k2["octave"] = np.clip(k2["octave"] + rng.integers(-1, 2, len(sel)), 0, 7)
    k2["angle"] = ((k2["angle"] + rng.normal(0, 5, len(sel))) % 360).astype(np.float32)
    d2 = flip_bits(F.desc[sel], rng, kflip)
    ne = n // 5
    ke = np.zeros(ne, KP_DTYPE)
    ke["x"] = rng.uniform(0, F.width - 1, ne)
    ke["y"] = rng.uniform(0, F.height - 1, ne)
    ke["octave"] = rng.integers(0, 8, ne)
    ke["angle"] = rng.uniform(0, 360, ne)
    ke["size"] = 31
    de = rng.integers(0, 256, (ne, 32), dtype=np.uint8)
    k2 = np.concatenate([k2, ke])
    d2 = np.concatenate([d2, de])
    perm = rng.permutation(len(k2))
    k2, d2 = k2[perm], d2[perm]
    centroids = rng.integers(0, 256, (n_nodes, 32), dtype=np.uint8)
    node_ids = np.sort(rng.choice(1_000_000, size=n_nodes, replace=False)).astype(np.uint32)
    KF1 = make_frame_data(k1, F.desc, F.width, F.height)
    KF2 = make_frame_data(k2, d2, F.width, F.height)
    KF1.has_mp = (rng.random(len(k1)) < 0.2).astype(np.uint8)
    KF2.has_mp = (rng.random(len(k2)) < 0.2).astype(np.uint8)
    KF1.featvec = quantize(KF1.desc, centroids, node_ids)
    KF2.featvec = quantize(KF2.desc, centroids, node_ids)
    KF1.pose = (np.array([0, 0, 0, 1], np.float32), np.zeros(3, np.float32))
    KF2.pose = (q2, t2)
    return KF1, KF2


def pose_problem(F: FrameData, cam: Pinhole, rng: np.random.Generator, frac=0.7, outlier_frac=0.08, noise=1.0,
                 rot=0.02, trans=0.06):
    """Inputs of Optimizer::PoseOptimization around F's keypoints: a true pose, matched MapPoints (world positions)
    that re-project onto their keypoints with pixel noise (scaled by the keypoint's level), a fraction of gross
    outliers (points displaced so they re-project 15-60 px away) and an initial pose (F.pose) perturbed from the
    true one, as the motion model leaves it. Returns (mps_xyz float32[M,3], true pose); sets F.pose and
    F.map_point."""
    from .match import quat_to_rot

    qt, tt = small_pose(rng, rot=0.05, trans=0.3)
    Rt = quat_to_rot(qt).astype(np.float64)
    n = len(F.keys)
    sel = np.sort(rng.choice(n, size=int(n * frac), replace=False))
    m = len(sel)
    k = F.keys[sel]
    s = F.scale_factors[k["octave"]].astype(np.float64)
    z = rng.uniform(2.0, 20.0, m)
    u = k["x"] + rng.normal(0, noise, m) * s
    v = k["y"] + rng.normal(0, noise, m) * s
    bad = rng.random(m) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, m)
    r = rng.uniform(15.0, 60.0, m)
    u = np.where(bad, u + r * np.cos(ang), u)
    v = np.where(bad, v + r * np.sin(ang), v)
    Xc = _backproject(cam, u, v, z)
    Xw = (Xc - tt[None, :].astype(np.float64)) @ Rt   # Rt^T (Xc - t)
    mp = np.full(n, -1, np.int32)
    perm = rng.permutation(m)   # MapPoint table order unrelated to keypoint order
    mp[sel] = perm
    xyz = np.zeros((m, 3), np.float32)
    xyz[perm] = Xw.astype(np.float32)
    dq, dt = small_pose(rng, rot=rot, trans=trans)   # initial = (dq, dt) * true
    ax, ay, az, aw = [float(x) for x in dq]
    bx, by, bz, bw = [float(x) for x in qt]
    q0 = np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                   aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])
    q0 = (q0 / np.linalg.norm(q0)).astype(np.float32)
    t0 = (quat_to_rot(dq).astype(np.float64) @ tt.astype(np.float64) + dt).astype(np.float32)
    F.pose = (q0, t0)
    F.map_point = mp
    F.outlier = None
    return xyz, (qt, tt)


def fuse_mappoints(F: FrameData, cam: Pinhole, rng: np.random.Generator, frac=0.7, dup_frac=0.1, n_out=120, kflip=60):
    """MapPoints as ORBmatcher::Fuse(pKF, vpMapPoints) sees them (ORBmatcher.cc:1177-1256), around keyframe F's
    keypoints under F.pose: world positions that re-project within a few pixels (scaled by the level), normals
    inside the 60-degree cone (5 % reversed), distance-invariance ranges whose PredictScale lands on the keypoint's
    level or the one above, descriptors with 0..kflip flipped bits (so some fail TH_LOW), 5 % invalid, near
    duplicates, 3 % outside their distance range, and random points (behind the camera, outside the image)."""
    from .match import quat_to_rot

    q, t = F.pose
    R = quat_to_rot(q).astype(np.float64)
    n = len(F.keys)
    sel = rng.choice(n, size=int(n * frac), replace=False)
    m = len(sel)
    k = F.keys[sel]
    s = F.scale_factors[k["octave"]].astype(np.float64)
    z = rng.uniform(1.5, 25.0, m)
    u = k["x"] + rng.normal(0, 0.8, m) * s
    v = k["y"] + rng.normal(0, 0.8, m) * s
    Xc = _backproject(cam, u, v, z)
    Xw = (Xc - t[None, :].astype(np.float64)) @ R   # R^T (Xc - t)
    PO = Xw - camera_center(F.pose).astype(np.float64)[None, :]
    d = np.linalg.norm(PO, axis=1)
    nrm = PO / d[:, None] + rng.normal(0, 0.15, (m, 3))
    back = rng.random(m) < 0.05
    nrm[back] = -nrm[back]
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    # PredictScale = ceil(log(maxD / dist) / log 1.2): maxD = dist * 1.2^(level - x), x in (0.05, 0.95)
    lvl = k["octave"] + rng.integers(0, 2, m)
    maxd = d * 1.2 ** (lvl - rng.uniform(0.05, 0.95, m))
    mps = np.zeros(m, FUSE_MP_DTYPE)
    mps["pos"] = Xw.astype(np.float32)
    mps["normal"] = nrm.astype(np.float32)
    mps["max_distance"] = maxd.astype(np.float32)
    mps["min_distance"] = (maxd / float(F.scale_factors[-1])).astype(np.float32)
    far = rng.random(m) < 0.03
    mps["max_distance"][far] *= np.float32(0.5)
    mps["valid"] = (rng.random(m) < 0.95).astype(np.int32)
    mps["desc"] = flip_bits(F.desc[sel], rng, kflip)
    nd = int(m * dup_frac)
    dup = mps[rng.choice(m, size=nd, replace=False)].copy()
    dup["pos"] += rng.normal(0, 0.003, (nd, 3)).astype(np.float32)
    dup["desc"] = flip_bits(dup["desc"], rng, 6)
    out = np.zeros(n_out, FUSE_MP_DTYPE)
    out["pos"] = rng.uniform(-10, 10, (n_out, 3)).astype(np.float32)
    nr = rng.normal(size=(n_out, 3))
    out["normal"] = (nr / np.linalg.norm(nr, axis=1)[:, None]).astype(np.float32)
    out["max_distance"] = rng.uniform(1, 40, n_out).astype(np.float32)
    out["min_distance"] = out["max_distance"] / np.float32(F.scale_factors[-1])
    out["valid"] = 1
    out["desc"] = rng.integers(0, 256, (n_out, 32), dtype=np.uint8)
    allm = np.concatenate([mps, dup, out])
    return allm[rng.permutation(len(allm))]
