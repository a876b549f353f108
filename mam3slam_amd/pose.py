"""PoseOptimization — host mirror of Optimizer::PoseOptimization over the C-ABI (include/mam_pose.h).

Reference: static int Optimizer::PoseOptimization(Frame* pFrame)   (src/Optimizer.cc:814-1115)

`pose_optimization(F, mps_xyz)` is the reference call on a `FrameData` (mam3slam_amd/match.py): one mono edge per
keypoint i whose slot holds a MapPoint (`F.map_point[i] >= 0`; its world position `mps_xyz[F.map_point[i]]`), in
increasing i; it sets `F.pose` (float, as Frame::SetPose) and `F.outlier` (mvbOutlier) and returns the number of
inliers. `PoseOptimizer.optimize_batch_device` is the batched device-resident form (one workgroup per frame).
The same call with the reference signature over the C++ Frame model is `MAM3SLAM::Optimizer::PoseOptimization`
(include/mam3slam/Optimizer.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib
from .match import Pinhole, Pose

POSE_EDGE_DTYPE = np.dtype([("obs", "<f4", (2,)), ("xw", "<f4", (3,)), ("inv_sigma2", "<f4")])
POSE_RESULT_DTYPE = np.dtype([("q", "<f8", (4,)), ("t", "<f8", (3,)), ("n_inliers", "<i4"), ("rounds", "<i4"),
                              ("iterations", "<i4"), ("lm_trials", "<i4")])
assert POSE_EDGE_DTYPE.itemsize == 24 and POSE_RESULT_DTYPE.itemsize == 72


class PoseResult(C.Structure):
    _fields_ = [("q", C.c_double * 4), ("t", C.c_double * 3), ("n_inliers", C.c_int32), ("rounds", C.c_int32),
                ("iterations", C.c_int32), ("lm_trials", C.c_int32)]


_SIGS = {
    "mam_pose_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "mam_pose_destroy": (None, [C.c_void_p]),
    "mam_pose_optimization": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_void_p]),
    "mam_pose_optimization_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                     C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_pose_frame_edges_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                                    C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                    C.c_void_p]),
    "mam_pose_frame_update_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                     C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                     C.c_int, C.c_void_p]),
    "mam_pose_max_edges": (C.c_int, [C.c_void_p]),
    "mam_pose_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "mam_pose_stage_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
}


def pose_struct(pose) -> Pose:
    """(q xyzw, t) -> mam_pose (float, as Sophus::SE3f stores it)."""
    q, t = pose
    p = Pose()
    p.q[:] = [float(np.float32(v)) for v in q]
    p.t[:] = [float(np.float32(v)) for v in t]
    return p


def make_edges(keys: np.ndarray, inv_level_sigma2: np.ndarray, kp_index: np.ndarray, xyz: np.ndarray) -> np.ndarray:
    """Edges of Optimizer.cc:856-895 (mono branch): keypoint kp_index[e] observes world point xyz[e]."""
    e = np.zeros(len(kp_index), POSE_EDGE_DTYPE)
    k = keys[kp_index]
    e["obs"][:, 0] = k["x"]
    e["obs"][:, 1] = k["y"]
    e["xw"] = np.asarray(xyz, np.float32)
    e["inv_sigma2"] = np.asarray(inv_level_sigma2, np.float32)[k["octave"]]
    return e


class PoseOptimizer:
    """Context of the gfx950 PoseOptimization (one per tracking thread)."""

    def __init__(self, device: int = 0):
        self._L = lib()
        self._ctx = C.c_void_p()
        check(self._L.mam_pose_create(device, C.byref(self._ctx)), "mam_pose_create")

    def __del__(self):
        if getattr(self, "_ctx", None):
            self._L.mam_pose_destroy(self._ctx)
            self._ctx = None

    def max_edges(self) -> int:
        return check(self._L.mam_pose_max_edges(self._ctx), "mam_pose_max_edges")

    def optimize(self, pose, cam: Pinhole, edges: np.ndarray):
        """One frame: returns (n_inliers, outlier[n] uint8, (q float64[4], t float64[3]), stats dict)."""
        edges = np.ascontiguousarray(edges, POSE_EDGE_DTYPE)
        n = len(edges)
        out = np.zeros(max(n, 1), np.uint8)
        res = PoseResult()
        p = pose_struct(pose)
        rc = check(self._L.mam_pose_optimization(self._ctx, C.byref(p), C.byref(cam), n,
                                                  edges.ctypes.data if n else None, out.ctypes.data, C.byref(res)),
                   "mam_pose_optimization")
        stats = {"rounds": res.rounds, "iterations": res.iterations, "lm_trials": res.lm_trials}
        return rc, out[:n].copy(), (np.array(res.q[:]), np.array(res.t[:])), stats

    def optimize_batch_device(self, nframes: int, d_tcw: int, cam: Pinhole, d_edges: int, edge_stride: int,
                              d_n_edges: int, d_outlier: int, d_results: int, stream: int = 0):
        return check(self._L.mam_pose_optimization_batch_device(
            self._ctx, nframes, C.c_void_p(d_tcw), C.byref(cam), C.c_void_p(d_edges), edge_stride,
            C.c_void_p(d_n_edges), C.c_void_p(d_outlier), C.c_void_p(d_results), C.c_void_p(stream)),
            "mam_pose_optimization_batch_device")

    def frame_edges_batch_device(self, nframes: int, d_kps: int, kp_stride: int, d_count: int, count_stride: int,
                                 inv_level_sigma2: np.ndarray, d_match_last: int, d_last: int, last_stride: int,
                                 d_match_local: int | None, d_local: int | None, local_stride: int, d_edges: int,
                                 edge_stride: int, d_n_edges: int, d_edge_kp: int, stream: int = 0):
        """Optimizer::PoseOptimization's edge build for device-resident tracked frames (Optimizer.cc:856-895)."""
        inv = np.ascontiguousarray(inv_level_sigma2, np.float32)
        return check(self._L.mam_pose_frame_edges_batch_device(
            self._ctx, nframes, C.c_void_p(d_kps), kp_stride, C.c_void_p(d_count), count_stride,
            inv.ctypes.data, len(inv), C.c_void_p(d_match_last), C.c_void_p(d_last), last_stride,
            C.c_void_p(d_match_local) if d_match_local else None, C.c_void_p(d_local) if d_local else None,
            local_stride, C.c_void_p(d_edges), edge_stride, C.c_void_p(d_n_edges), C.c_void_p(d_edge_kp),
            C.c_void_p(stream)), "mam_pose_frame_edges_batch_device")

    def frame_update_batch_device(self, nframes: int, d_results: int, d_tcw: int, d_outlier: int, d_edge_kp: int,
                                  edge_stride: int, d_n_edges: int, discard: bool, d_match_last: int | None,
                                  d_taken: int | None, kp_stride: int, stream: int = 0):
        """Frame::SetPose from the result and, with discard, TrackWithMotionModel's outlier discard
        (Tracking.cc:2836-2857)."""
        return check(self._L.mam_pose_frame_update_batch_device(
            self._ctx, nframes, C.c_void_p(d_results), C.c_void_p(d_tcw), C.c_void_p(d_outlier),
            C.c_void_p(d_edge_kp), edge_stride, C.c_void_p(d_n_edges), 1 if discard else 0,
            C.c_void_p(d_match_last) if d_match_last else None, C.c_void_p(d_taken) if d_taken else None,
            kp_stride, C.c_void_p(stream)), "mam_pose_frame_update_batch_device")

    def set_profiling(self, enable: bool):
        check(self._L.mam_pose_set_profiling(self._ctx, 1 if enable else 0), "mam_pose_set_profiling")

    def stage_times(self):
        ms = np.zeros(1, np.float64)
        n = np.zeros(1, np.int64)
        check(self._L.mam_pose_stage_times(self._ctx, ms.ctypes.data, n.ctypes.data), "mam_pose_stage_times")
        return {"pose": (float(ms[0]), int(n[0]))}


def pose_optimization(F, mps_xyz: np.ndarray, cam: Pinhole, optimizer: PoseOptimizer | None = None) -> int:
    """Optimizer::PoseOptimization(pFrame) on a FrameData: F.map_point[i] >= 0 marks mvpMapPoints[i] (index into
    mps_xyz); F.pose is replaced by the optimised pose (float), F.outlier receives mvbOutlier."""
    opt = optimizer or PoseOptimizer()
    idx = np.nonzero(F.map_point >= 0)[0]
    edges = make_edges(F.keys, 1.0 / F.level_sigma2, idx, mps_xyz[F.map_point[idx]])
    n, out, (q, t), _ = opt.optimize(F.pose, cam, edges)
    outlier = np.zeros(len(F.keys), np.uint8) if getattr(F, "outlier", None) is None else F.outlier
    outlier[idx] = out
    F.outlier = outlier
    F.pose = set_pose_float(q, t)
    return n


def set_pose_float(q, t):
    """Frame::SetPose(Sophus::SE3f(q.cast<float>(), t.cast<float>())) (Optimizer.cc:1108-1111): Sophus normalises
    the float quaternion, coeffs / norm() with Eigen's SSE 4-float reduction ((x^2 + z^2) + (y^2 + w^2))."""
    qf = np.asarray(q, np.float64).astype(np.float32)
    sq = qf * qf
    n = np.sqrt(np.float32((sq[0] + sq[2]) + (sq[1] + sq[3])))
    return (qf / n).astype(np.float32), np.asarray(t, np.float64).astype(np.float32)
