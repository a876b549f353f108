"""ORBmatcher — Python mirror of MAM3SLAM::ORBmatcher's hot-path searches over the C-ABI (include/mam_match.h).

Reference interface (include/ORBmatcher.h:40-93, src/ORBmatcher.cc):
    ORBmatcher(float nnratio=0.6, bool checkOri=true)
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b)
    int SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, float th=3, bool bFarPoints=false,
                           float thFarPoints=50)
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, float th, bool bMono)
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, vector<pair<size_t,size_t>>& vMatchedPairs,
                               bool bOnlyStereo, bool bCoarse=false)
    int Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th=3.0, bool bRight=false)
and MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:329-403), batched over many MapPoints.
    TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30

Frames/KeyFrames are passed as FrameData (numpy views of the fields the searches read). Object pointers are
replaced by indices: the search results are per-keypoint indices into the MapPoint list / last frame
(-1 = untouched), exactly what the reference writes into Frame::mvpMapPoints.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ._lib import MamError, check, lib
from .orb import KP_DTYPE

TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30
GRID_COLS, GRID_ROWS = 64, 48
MAX_LEVELS = 16


class FrameGeom(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("grid_inv_w", C.c_float), ("grid_inv_h", C.c_float), ("nlevels", C.c_int32),
                ("scale_factors", C.c_float * MAX_LEVELS), ("level_sigma2", C.c_float * MAX_LEVELS)]


class Pose(C.Structure):
    _fields_ = [("q", C.c_float * 4), ("t", C.c_float * 3)]


class Camera(C.Structure):
    """mam_camera (include/mam_camera.h): GeometricCamera as a value, model 0 = Pinhole, 1 = KannalaBrandt8.
    project_np / unproject_np are float64 numpy forms for the synthetic-scene generators only (the searches and the
    solves project on the device, bit-exact with the reference's float code: mam3slam_amd/csrc/camera.hpp)."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("k", C.c_float * 4),
                ("model", C.c_int32), ("precision", C.c_float)]
    PINHOLE, KANNALA_BRANDT8 = 0, 1

    @property
    def is_kb8(self) -> bool:
        return self.model == Camera.KANNALA_BRANDT8

    def params(self) -> np.ndarray:
        """mvParameters (float32): 4 for a Pinhole, 8 for a KannalaBrandt8 (mam_lba_problem.cams rows)."""
        base = [self.fx, self.fy, self.cx, self.cy]
        return np.array(base + (list(self.k) if self.is_kb8 else []), np.float32)

    def project_np(self, X: np.ndarray) -> np.ndarray:
        X = np.asarray(X, np.float64)
        x, y, z = X[..., 0], X[..., 1], X[..., 2]
        if not self.is_kb8:
            return np.stack([self.fx * x / z + self.cx, self.fy * y / z + self.cy], -1)
        th = np.arctan2(np.sqrt(x * x + y * y), z)
        psi = np.arctan2(y, x)
        k = [float(v) for v in self.k]
        r = th + k[0] * th ** 3 + k[1] * th ** 5 + k[2] * th ** 7 + k[3] * th ** 9
        return np.stack([self.fx * r * np.cos(psi) + self.cx, self.fy * r * np.sin(psi) + self.cy], -1)

    def unproject_np(self, u, v) -> np.ndarray:
        """Rays (x/z, y/z) of pixels (KannalaBrandt8::unproject's Newton solve in float64)."""
        px = (np.asarray(u, np.float64) - self.cx) / self.fx
        py = (np.asarray(v, np.float64) - self.cy) / self.fy
        if not self.is_kb8:
            return np.stack([px, py], -1)
        thd = np.clip(np.sqrt(px * px + py * py), 0, np.pi / 2)
        k = [float(v) for v in self.k]
        th = thd.copy()
        for _ in range(20):
            t2 = th * th
            f = th * (1 + k[0] * t2 + k[1] * t2 ** 2 + k[2] * t2 ** 3 + k[3] * t2 ** 4) - thd
            df = 1 + 3 * k[0] * t2 + 5 * k[1] * t2 ** 2 + 7 * k[2] * t2 ** 3 + 9 * k[3] * t2 ** 4
            th = th - f / df
        sc = np.where(thd > 1e-8, np.tan(th) / np.maximum(thd, 1e-30), 1.0)
        return np.stack([px * sc, py * sc], -1)


class Pinhole(Camera):
    """Pinhole (src/CameraModels/Pinhole.cpp): mvParameters fx, fy, cx, cy."""

    def __init__(self, fx=0.0, fy=0.0, cx=0.0, cy=0.0):
        super().__init__(fx, fy, cx, cy, (C.c_float * 4)(), Camera.PINHOLE, 0.0)


class KannalaBrandt8(Camera):
    """KannalaBrandt8 (src/CameraModels/KannalaBrandt8.cpp): fx, fy, cx, cy, k0..k3; precision 1e-6
    (KannalaBrandt8.h:42-47)."""

    def __init__(self, fx=0.0, fy=0.0, cx=0.0, cy=0.0, k0=0.0, k1=0.0, k2=0.0, k3=0.0, precision=1e-6):
        super().__init__(fx, fy, cx, cy, (C.c_float * 4)(k0, k1, k2, k3), Camera.KANNALA_BRANDT8, precision)



class FeatVec(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("node_ids", C.c_void_p), ("node_off", C.c_void_p), ("feats", C.c_void_p)]


class TriKF(C.Structure):
    """mam_tri_kf: the keyframe side of SearchForTriangulation (keys, descriptors, MapPoint flags, FeatureVector,
    pose, camera)."""
    _fields_ = [("n", C.c_int32), ("keys", C.c_void_p), ("desc", C.c_void_p), ("has_mp", C.c_void_p),
                ("fv", FeatVec), ("tcw", Pose), ("cam", Camera)]


class FramesDev(C.Structure):
    _fields_ = [("nframes", C.c_int32), ("kp_stride", C.c_int32), ("keys", C.c_void_p), ("desc", C.c_void_p),
                ("counts", C.c_void_p), ("taken", C.c_void_p), ("taken_out", C.c_void_p), ("reuse_grid", C.c_int32)]


class TriBatch(C.Structure):
    """mam_tri_batch: keyframe slots in HBM + FeatureVectors as per-feature (node, weight) + pairs."""
    _fields_ = [("kfs", FramesDev), ("has_mp", C.c_void_p), ("nid", C.c_void_p), ("weight", C.c_void_p),
                ("tcw", C.c_void_p), ("npairs", C.c_int32), ("pairs", C.c_void_p)]


MP_TRACK_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("view_cos", "<f4"), ("track_depth", "<f4"),
                           ("track_in_view", "<i4"), ("scale_level", "<i4"), ("is_bad", "<i4"), ("nobs", "<i4"),
                           ("desc", "u1", (32,))])
LAST_ENTRY_DTYPE = np.dtype([("pos", "<f4", (3,)), ("angle", "<f4"), ("octave", "<i4"), ("valid", "<i4"),
                             ("nobs", "<i4"), ("pad", "<i4"), ("desc", "u1", (32,))])
assert MP_TRACK_DTYPE.itemsize == 64 and LAST_ENTRY_DTYPE.itemsize == 64
FUSE_MP_DTYPE = np.dtype([("pos", "<f4", (3,)), ("max_distance", "<f4"), ("normal", "<f4", (3,)),
                          ("min_distance", "<f4"), ("valid", "<i4"), ("pad", "<i4", (3,)), ("desc", "u1", (32,))])
assert FUSE_MP_DTYPE.itemsize == 80
# mam_local_mp: the MapPoint fields SearchLocalPoints / Frame::isInFrustum read (Tracking.cc:3103-3139)
LOCAL_MP_DTYPE = np.dtype([("pos", "<f4", (3,)), ("max_distance", "<f4"), ("normal", "<f4", (3,)),
                           ("min_distance", "<f4"), ("is_bad", "<i4"), ("nobs", "<i4"), ("seen", "<i4"),
                           ("pad", "<i4"), ("desc", "u1", (32,))])
assert LOCAL_MP_DTYPE.itemsize == 80


class FuseKF(C.Structure):
    _fields_ = [("tcw", Pose), ("ow", C.c_float * 3), ("log_scale_factor", C.c_float)]


def camera_center(pose):
    """KeyFrame::GetCameraCenter: translation of Tcw^-1 (Sophus: conjugate quaternion applied to -t), float32."""
    q = np.asarray(pose[0], np.float32)
    p = -np.asarray(pose[1], np.float32)
    qv, w = -q[:3], q[3]
    uv = np.cross(qv, p).astype(np.float32)
    uv = uv + uv
    return (p + w * uv + np.cross(qv, uv)).astype(np.float32)


def pose_c(pose) -> Pose:
    """(q xyzw, t) -> mam_pose."""
    T = Pose()
    for i in range(4):
        T.q[i] = float(pose[0][i])
    for i in range(3):
        T.t[i] = float(pose[1][i])
    return T


def triangulation_geometry(pose1, pose2, cam1: Camera, cam2: Camera | None = None):
    """SearchForTriangulation's pair geometry as the library computes it (mam_triangulation_geometry,
    ORBmatcher.cc:913-930): (R12 3x3, t12, F12 3x3, ep) float32."""
    cam2 = cam1 if cam2 is None else cam2
    R12, t12 = np.zeros(9, np.float32), np.zeros(3, np.float32)
    F12, ep = np.zeros(9, np.float32), np.zeros(2, np.float32)
    t1, t2 = pose_c(pose1), pose_c(pose2)
    check(_bind().mam_triangulation_geometry(C.byref(t1), C.byref(t2), C.byref(cam1), C.byref(cam2), _p(R12), _p(t12),
                                             _p(F12), _p(ep)), "mam_triangulation_geometry")
    return R12.reshape(3, 3), t12, F12.reshape(3, 3), ep


def fuse_kf(pose, scale_factor: float = 1.2) -> FuseKF:
    """The keyframe side of Fuse: Tcw, camera centre, mfLogScaleFactor = log of the float scale factor."""
    k = FuseKF()
    for i in range(4):
        k.tcw.q[i] = float(pose[0][i])
    for i in range(3):
        k.tcw.t[i] = float(pose[1][i])
    ow = camera_center(pose)
    for i in range(3):
        k.ow[i] = float(ow[i])
    k.log_scale_factor = float(np.log(np.float32(scale_factor)))
    return k

_SIGS = {
    "mam_match_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "mam_match_destroy": (None, [C.c_void_p]),
    "mam_descriptor_distance": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "mam_search_by_projection": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_int, C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_float,
                                           C.c_void_p]),
    "mam_search_by_projection_motion": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                                  C.c_int, C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p]),
    "mam_search_for_triangulation": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "mam_search_for_triangulation_kf": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                  C.c_void_p]),
    "mam_search_for_triangulation_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                            C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_triangulation_geometry": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p]),
    "mam_search_by_projection_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                        C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_float,
                                                        C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_search_by_projection_motion_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                               C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                                               C.c_float, C.c_int, C.c_void_p, C.c_void_p,
                                                               C.c_void_p]),
    "mam_track_motion_search_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                       C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                                       C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                                       C.c_void_p]),
    "mam_fuse": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                           C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]),
    "mam_fuse_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                        C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_fuse_items_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                              C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                              C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_compute_distinctive_descriptors": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_compute_distinctive_descriptors_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                                                   C.c_void_p, C.c_void_p]),
    "mam_is_in_frustum": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_int, C.c_void_p,
                                    C.c_float, C.c_void_p]),
    "mam_is_in_frustum_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
                                                 C.c_void_p, C.c_int, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p,
                                                 C.c_void_p]),
    "mam_match_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "mam_match_stage_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
}


def _bind():
    L = lib()
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


@dataclass
class FrameData:
    """The Frame / KeyFrame fields the searches read. keys = mvKeysUn (KP_DTYPE), desc = mDescriptors."""

    keys: np.ndarray
    desc: np.ndarray
    width: int
    height: int
    scale_factors: np.ndarray
    level_sigma2: np.ndarray
    taken: np.ndarray | None = None          # mvpMapPoints[i] && Observations() > 0  (Frame)
    has_mp: np.ndarray | None = None         # GetMapPoint(i) != NULL                   (KeyFrame)
    featvec: dict | None = None              # DBoW2::FeatureVector: node id -> list of feature indices
    pose: tuple | None = None                # (q xyzw float32[4], t float32[3]) = Tcw
    map_point: np.ndarray | None = None      # mvpMapPoints[i] as an index into a MapPoint table (-1 = NULL)
    outlier: np.ndarray | None = None        # mvbOutlier
    extra: dict = field(default_factory=dict)

    def geom(self) -> FrameGeom:
        g = FrameGeom()
        # ComputeImageBounds without distortion (Frame.cc:801-807) and the grid inverses (Frame.cc:341-342)
        g.min_x, g.max_x, g.min_y, g.max_y = 0.0, float(self.width), 0.0, float(self.height)
        g.grid_inv_w = float(np.float32(GRID_COLS) / np.float32(self.width))
        g.grid_inv_h = float(np.float32(GRID_ROWS) / np.float32(self.height))
        g.nlevels = len(self.scale_factors)
        for i, v in enumerate(self.scale_factors):
            g.scale_factors[i] = float(v)
        for i, v in enumerate(self.level_sigma2):
            g.level_sigma2[i] = float(v)
        return g


def flatten_featvec(fv: dict):
    ids = np.array(sorted(fv), dtype=np.uint32)
    off = np.zeros(len(ids) + 1, np.int32)
    feats = []
    for i, k in enumerate(ids):
        lst = sorted(fv[int(k)])
        feats.extend(lst)
        off[i + 1] = off[i] + len(lst)
    return ids, off, np.array(feats if feats else [0], dtype=np.uint32)


def quat_to_rot(q):
    x, y, z, w = [np.float32(v) for v in q]
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float32)


def fundamental_12(pose1, pose2, K1, K2):
    """F12 = K1^-T [t12]x R12 K2^-1 with T12 = T1w * T2w^-1 (ORBmatcher.cc:926-930, Pinhole.cpp:109-112)."""
    R1, t1 = quat_to_rot(pose1[0]), np.asarray(pose1[1], np.float32)
    R2, t2 = quat_to_rot(pose2[0]), np.asarray(pose2[1], np.float32)
    R12 = (R1 @ R2.T).astype(np.float32)
    t12 = (t1 - R12 @ t2).astype(np.float32)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], np.float32)
    F = np.linalg.inv(K1.T.astype(np.float64)).astype(np.float32) @ tx @ R12 @ np.linalg.inv(
        K2.astype(np.float64)).astype(np.float32)
    return F.astype(np.float32)


def epipole_12(pose1, pose2, cam2: Pinhole):
    """ep = KF2 camera projection of KF1's centre (ORBmatcher.cc:913-919)."""
    R1, t1 = quat_to_rot(pose1[0]), np.asarray(pose1[1], np.float32)
    R2, t2 = quat_to_rot(pose2[0]), np.asarray(pose2[1], np.float32)
    Cw = (-R1.T @ t1).astype(np.float32)
    C2 = (R2 @ Cw + t2).astype(np.float32)
    return np.array([cam2.fx * C2[0] / C2[2] + cam2.cx, cam2.fy * C2[1] / C2[2] + cam2.cy], np.float32)


class ORBmatcher:
    TH_HIGH, TH_LOW, HISTO_LENGTH = TH_HIGH, TH_LOW, HISTO_LENGTH

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0, share: "ORBmatcher" = None):
        """share: use another matcher's device context (its scratch and stream state), so a search can reuse the
        cell grid that matcher's last search built over the same frames (FramesDev.reuse_grid)."""
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self._L = _bind()
        self._owner = share is None
        if share is not None:
            self._share = share   # keep the owner alive
            self._ctx = share._ctx
        else:
            self._ctx = C.c_void_p()
            check(self._L.mam_match_create(int(device), C.byref(self._ctx)), "mam_match_create")

    def close(self):
        if not getattr(self, "_owner", False):
            self._ctx = C.c_void_p()
            return
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.mam_match_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    def DescriptorDistance(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        out = np.zeros(len(a), np.int32)
        check(self._L.mam_descriptor_distance(self._ctx, _p(a), _p(b), len(a), _p(out)), "descriptor_distance")
        return out

    def SearchByProjection(self, F: FrameData, mps: np.ndarray, th: float = 3, bFarPoints: bool = False,
                           thFarPoints: float = 50):
        """Local-map search (ORBmatcher.cc:43-213). Returns (nmatches, kp_to_mp)."""
        keys = np.ascontiguousarray(F.keys, KP_DTYPE)
        desc = np.ascontiguousarray(F.desc, np.uint8)
        taken = None if F.taken is None else np.ascontiguousarray(F.taken, np.uint8)
        mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
        out = np.full(max(len(keys), 1), -1, np.int32)
        g = F.geom()
        n = self._L.mam_search_by_projection(self._ctx, C.byref(g), len(keys), _p(keys), _p(desc), _p(taken),
                                             len(mps), _p(mps), float(th), int(bFarPoints), float(thFarPoints),
                                             self.mfNNratio, _p(out))
        check(n, "SearchByProjection")
        return n, out[:len(keys)]

    def SearchByProjectionMotion(self, Cur: FrameData, last: np.ndarray, cam: Pinhole, th: float, bMono: bool = True):
        """Motion-model search SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:1676-1887).
        `last` holds LastFrame's entries (LAST_ENTRY_DTYPE); Cur.pose = CurrentFrame Tcw."""
        if not bMono:
            raise MamError("stereo motion search is out of scope (mono agents only)")
        keys = np.ascontiguousarray(Cur.keys, KP_DTYPE)
        desc = np.ascontiguousarray(Cur.desc, np.uint8)
        taken = None if Cur.taken is None else np.ascontiguousarray(Cur.taken, np.uint8)
        last = np.ascontiguousarray(last, LAST_ENTRY_DTYPE)
        pose = Pose()
        for i in range(4):
            pose.q[i] = float(Cur.pose[0][i])
        for i in range(3):
            pose.t[i] = float(Cur.pose[1][i])
        out = np.full(max(len(keys), 1), -1, np.int32)
        g = Cur.geom()
        n = self._L.mam_search_by_projection_motion(self._ctx, C.byref(g), len(keys), _p(keys), _p(desc), _p(taken),
                                                    C.byref(pose), None, 0.0, C.byref(cam), len(last), _p(last),
                                                    float(th), 1, int(self.mbCheckOrientation), _p(out))
        check(n, "SearchByProjection(motion)")
        return n, out[:len(keys)]

    def SearchForTriangulation(self, KF1: FrameData, KF2: FrameData, F12: np.ndarray, ep: np.ndarray,
                               bOnlyStereo: bool = False, bCoarse: bool = False):
        """ORBmatcher.cc:907-1146 (mono Pinhole). Returns (nmatches, vMatchedPairs as (k,2) int array)."""
        if bOnlyStereo:
            return 0, np.zeros((0, 2), np.int64)
        k1 = np.ascontiguousarray(KF1.keys, KP_DTYPE)
        k2 = np.ascontiguousarray(KF2.keys, KP_DTYPE)
        d1 = np.ascontiguousarray(KF1.desc, np.uint8)
        d2 = np.ascontiguousarray(KF2.desc, np.uint8)
        h1 = np.ascontiguousarray(KF1.has_mp if KF1.has_mp is not None else np.zeros(len(k1)), np.uint8)
        h2 = np.ascontiguousarray(KF2.has_mp if KF2.has_mp is not None else np.zeros(len(k2)), np.uint8)
        i1, o1, f1 = flatten_featvec(KF1.featvec)
        i2, o2, f2 = flatten_featvec(KF2.featvec)
        fv1 = FeatVec(len(i1), i1.ctypes.data, o1.ctypes.data, f1.ctypes.data)
        fv2 = FeatVec(len(i2), i2.ctypes.data, o2.ctypes.data, f2.ctypes.data)
        F12 = np.ascontiguousarray(F12, np.float32).reshape(9)
        ep = np.ascontiguousarray(ep, np.float32).reshape(2)
        out = np.full(max(len(k1), 1), -1, np.int32)
        g = KF2.geom()
        n = self._L.mam_search_for_triangulation(self._ctx, C.byref(g), len(k1), _p(k1), _p(d1), _p(h1),
                                                 C.byref(fv1), len(k2), _p(k2), _p(d2), _p(h2), C.byref(fv2),
                                                 _p(F12), _p(ep), int(self.mbCheckOrientation), int(bCoarse), _p(out))
        check(n, "SearchForTriangulation")
        out = out[:len(k1)]
        idx = np.nonzero(out >= 0)[0]
        return n, np.stack([idx, out[idx]], 1).astype(np.int64)

    def search_for_triangulation_batch_device(self, F: FrameData, cam: Camera, batch: TriBatch, d_out: int,
                                              d_nmatches: int, bCoarse: bool = False, stream=None):
        """mam_search_for_triangulation_batch_device: batch.npairs SearchForTriangulation calls over device-resident
        keyframes; F supplies the frame geometry (scale / sigma tables, image bounds)."""
        g = F.geom()
        check(self._L.mam_search_for_triangulation_batch_device(self._ctx, C.byref(g), C.byref(cam), C.byref(batch),
                                                                 int(self.mbCheckOrientation), int(bCoarse),
                                                                 C.c_void_p(d_out), C.c_void_p(d_nmatches),
                                                                 C.c_void_p(stream or 0)),
              "SearchForTriangulation(batch)")

    def SearchForTriangulationKF(self, KF1: FrameData, KF2: FrameData, cam1: Camera, cam2: Camera | None = None,
                                 bOnlyStereo: bool = False, bCoarse: bool = False):
        """ORBmatcher.cc:907-1146 from the keyframes' poses (KF.pose) and cameras, Pinhole or KannalaBrandt8: the pair
        geometry of :913-930 and pCamera1->epipolarConstrain are computed by the library. Returns (nmatches,
        vMatchedPairs as (k,2) int array)."""
        if bOnlyStereo:
            return 0, np.zeros((0, 2), np.int64)
        cam2 = cam1 if cam2 is None else cam2
        keep = []
        kf = []
        for KF, cam in ((KF1, cam1), (KF2, cam2)):
            k = np.ascontiguousarray(KF.keys, KP_DTYPE)
            d = np.ascontiguousarray(KF.desc, np.uint8)
            h = np.ascontiguousarray(KF.has_mp if KF.has_mp is not None else np.zeros(len(k)), np.uint8)
            ids, off, feats = flatten_featvec(KF.featvec)
            keep += [k, d, h, ids, off, feats]
            t = TriKF()
            t.n = len(k)
            t.keys, t.desc, t.has_mp = _p(k), _p(d), _p(h)
            t.fv = FeatVec(len(ids), ids.ctypes.data, off.ctypes.data, feats.ctypes.data)
            t.tcw = pose_c(KF.pose)
            t.cam = cam
            kf.append(t)
        out = np.full(max(len(KF1.keys), 1), -1, np.int32)
        g = KF2.geom()
        n = self._L.mam_search_for_triangulation_kf(self._ctx, C.byref(g), C.byref(kf[0]), C.byref(kf[1]),
                                                    int(self.mbCheckOrientation), int(bCoarse), _p(out))
        check(n, "SearchForTriangulationKF")
        out = out[:len(KF1.keys)]
        idx = np.nonzero(out >= 0)[0]
        return n, np.stack([idx, out[idx]], 1).astype(np.int64)

    def Fuse(self, KF: FrameData, mps: np.ndarray, cam: Pinhole, th: float = 3.0, bRight: bool = False):
        """ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight) (ORBmatcher.cc:1148-1338): the per-MapPoint search of a
        mono keyframe. KF.pose = Tcw; mps: FUSE_MP_DTYPE (valid = non-NULL, not bad, not already in the keyframe).
        Returns (n, idx, dist): idx[i] = the keypoint MapPoint i fuses with (bestDist <= TH_LOW) or -1, dist[i] =
        bestDist (256 = no candidate). The replace-or-add side effects are the caller's, in list order."""
        if bRight:
            raise MamError("Fuse(bRight=true): stereo is out of scope (mono agents only)")
        keys = np.ascontiguousarray(KF.keys, KP_DTYPE)
        desc = np.ascontiguousarray(KF.desc, np.uint8)
        mps = np.ascontiguousarray(mps, FUSE_MP_DTYPE)
        kf = fuse_kf(KF.pose)
        idx = np.full(max(len(mps), 1), -1, np.int32)
        dist = np.full(max(len(mps), 1), 256, np.int32)
        g = KF.geom()
        n = self._L.mam_fuse(self._ctx, C.byref(g), len(keys), _p(keys), _p(desc), C.byref(kf), C.byref(cam), len(mps),
                             _p(mps), float(th), _p(idx), _p(dist))
        check(n, "Fuse")
        return n, idx[:len(mps)], dist[:len(mps)]

    def ComputeDistinctiveDescriptors(self, desc_off: np.ndarray, descs: np.ndarray) -> np.ndarray:
        """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403) for many MapPoints in one launch: MapPoint
        m's observed descriptors are rows desc_off[m] .. desc_off[m+1]-1 of descs. Returns the chosen row of each
        (relative to desc_off[m]; -1 = no descriptor)."""
        off = np.ascontiguousarray(desc_off, np.int32)
        d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
        n = len(off) - 1
        out = np.full(max(n, 1), -1, np.int32)
        check(self._L.mam_compute_distinctive_descriptors(self._ctx, n, _p(off), _p(d) if len(d) else None, _p(out)),
              "ComputeDistinctiveDescriptors")
        return out[:n]

    def IsInFrustum(self, F: FrameData, mps: np.ndarray, cam: Pinhole, viewingCosLimit: float = 0.5,
                    scale_factor: float = 1.2):
        """SearchLocalPoints' projection loop (Tracking.cc:3119-3139): Frame::isInFrustum(pMP, viewingCosLimit) +
        PredictScale for every local MapPoint (LOCAL_MP_DTYPE) of frame F (F.pose = Tcw). Returns (nToMatch, tracks):
        MP_TRACK_DTYPE records, the `mps` input of SearchByProjection."""
        mps = np.ascontiguousarray(mps, LOCAL_MP_DTYPE)
        out = np.zeros(max(len(mps), 1), MP_TRACK_DTYPE)
        T = Pose()
        for i in range(4):
            T.q[i] = float(F.pose[0][i])
        for i in range(3):
            T.t[i] = float(F.pose[1][i])
        g = F.geom()
        n = self._L.mam_is_in_frustum(self._ctx, C.byref(g), C.byref(T), C.byref(cam),
                                      float(np.log(np.float32(scale_factor))), len(mps), _p(mps),
                                      float(viewingCosLimit), _p(out))
        check(n, "isInFrustum")
        return n, out[:len(mps)]

    # ---- batched device-resident (bench / multi-agent harness)
    def is_in_frustum_batch_device(self, F: FrameData, nframes: int, d_tcw: int, cam: Pinhole, d_mps: int,
                                   mp_stride: int, d_nmps: int, d_out: int, d_nmatch: int = 0, stream: int = 0,
                                   view_cos_limit: float = 0.5, scale_factor: float = 1.2):
        g = F.geom()
        return check(self._L.mam_is_in_frustum_batch_device(
            self._ctx, C.byref(g), int(nframes), C.c_void_p(d_tcw), C.byref(cam),
            float(np.log(np.float32(scale_factor))), C.c_void_p(d_mps), int(mp_stride), C.c_void_p(d_nmps),
            float(view_cos_limit), C.c_void_p(d_out), C.c_void_p(d_nmatch or None), C.c_void_p(stream)),
            "is_in_frustum_batch_device")

    def search_by_projection_batch_device(self, F: FrameData, frames: FramesDev, d_mps: int, mp_stride: int,
                                          d_nmps: int, th: float, d_out: int, d_nmatch: int, stream: int = 0,
                                          far=False, th_far=50.0):
        g = F.geom()
        return check(self._L.mam_search_by_projection_batch_device(
            self._ctx, C.byref(g), C.byref(frames), C.c_void_p(d_mps), mp_stride, C.c_void_p(d_nmps), float(th),
            int(far), float(th_far), self.mfNNratio, C.c_void_p(d_out), C.c_void_p(d_nmatch), C.c_void_p(stream)),
            "search_by_projection_batch_device")

    def search_motion_batch_device(self, F: FrameData, frames: FramesDev, d_tcw: int, cam: Pinhole, d_last: int,
                                   last_stride: int, d_nlast: int, th: float, d_out: int, d_nmatch: int,
                                   stream: int = 0):
        g = F.geom()
        return check(self._L.mam_search_by_projection_motion_batch_device(
            self._ctx, C.byref(g), C.byref(frames), C.c_void_p(d_tcw), C.byref(cam), C.c_void_p(d_last),
            last_stride, C.c_void_p(d_nlast), float(th), int(self.mbCheckOrientation), C.c_void_p(d_out),
            C.c_void_p(d_nmatch), C.c_void_p(stream)), "search_motion_batch_device")

    def track_motion_search_batch_device(self, F: FrameData, frames: FramesDev, d_tcw: int, cam: Pinhole,
                                         d_last: int, last_stride: int, d_nlast: int, th: float, d_out: int,
                                         d_nmatch: int, min_matches: int = 20, stream: int = 0):
        """Tracking::TrackWithMotionModel's search (Tracking.cc:2811-2824): th, and 2 th for the frames that found
        fewer than min_matches."""
        g = F.geom()
        return check(self._L.mam_track_motion_search_batch_device(
            self._ctx, C.byref(g), C.byref(frames), C.c_void_p(d_tcw), C.byref(cam), C.c_void_p(d_last),
            last_stride, C.c_void_p(d_nlast), float(th), int(self.mbCheckOrientation), int(min_matches),
            C.c_void_p(d_out), C.c_void_p(d_nmatch), C.c_void_p(stream)), "track_motion_search_batch_device")

    def fuse_batch_device(self, F: FrameData, frames: FramesDev, d_kfs: int, cam: Pinhole, d_mps: int, mp_stride: int,
                          d_nmps: int, th: float, d_idx: int, d_dist: int, d_nfused: int, stream: int = 0):
        g = F.geom()
        return check(self._L.mam_fuse_batch_device(
            self._ctx, C.byref(g), C.byref(frames), C.c_void_p(d_kfs), C.byref(cam), C.c_void_p(d_mps), mp_stride,
            C.c_void_p(d_nmps), float(th), C.c_void_p(d_idx), C.c_void_p(d_dist), C.c_void_p(d_nfused),
            C.c_void_p(stream)), "fuse_batch_device")

    def fuse_items_batch_device(self, F: FrameData, frames: FramesDev, d_kf_tcw: int, cam: Camera, n_items: int,
                                d_frame_of: int, d_mp_of: int, d_mps: int, mp_stride: int, d_nmps: int, th: float,
                                d_idx: int, d_dist: int, d_nfused: int, stream: int = 0, scale_factor: float = 1.2):
        """Fuse of n_items (keyframe of `frames`, MapPoint list) pairs (mam_fuse_items_batch_device)."""
        g = F.geom()
        return check(self._L.mam_fuse_items_batch_device(
            self._ctx, C.byref(g), C.byref(frames), C.c_void_p(d_kf_tcw), float(np.log(np.float32(scale_factor))),
            C.byref(cam), int(n_items), C.c_void_p(d_frame_of), C.c_void_p(d_mp_of), C.c_void_p(d_mps), mp_stride,
            C.c_void_p(d_nmps), float(th), C.c_void_p(d_idx), C.c_void_p(d_dist), C.c_void_p(d_nfused),
            C.c_void_p(stream)), "fuse_items_batch_device")

    def distinctive_batch_device(self, n_mps: int, d_off: int, d_descs: int, d_out: int, stream: int = 0):
        return check(self._L.mam_compute_distinctive_descriptors_batch_device(
            self._ctx, int(n_mps), C.c_void_p(d_off), C.c_void_p(d_descs), C.c_void_p(d_out), C.c_void_p(stream)),
            "distinctive_batch_device")

    def set_profiling(self, enable: bool):
        check(self._L.mam_match_set_profiling(self._ctx, 1 if enable else 0), "match_set_profiling")

    def stage_times(self):
        ms = np.zeros(7, np.float64)
        n = np.zeros(7, np.int64)
        check(self._L.mam_match_stage_times(self._ctx, _p(ms), _p(n)), "match_stage_times")
        names = ["grid", "gather", "resolve", "triangulation", "fuse", "distinctive", "frustum"]
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(names)}
