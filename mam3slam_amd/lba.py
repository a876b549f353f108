"""LocalBundleAdjustment — host mirror of Optimizer::LocalBundleAdjustment over the C-ABI (include/mam_lba.h).

Reference: static void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap,
           int& num_fixedKF, int& num_OptKF, int& num_MPs, int& num_edges)   (src/Optimizer.cc:1116-1498)

`LBAProblem` is the g2o graph the reference builds (vertices, mono edges, Huber delta, 10 iterations);
`solve()` runs the Levenberg-Marquardt / Schur solve on the GPU (`stop_flag`: a one-byte array, the reference's
`bool* pbStopFlag`). The full call with the reference signature — window construction (Optimizer.cc:1118-1186),
solve, outlier erase (chi2 > 5.991 or depth <= 0, :1413-1460) and write-back as float (:1463-1497) — is the C++
host API `MAM3SLAM::Optimizer::LocalBundleAdjustment` (include/mam3slam/Optimizer.h).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import check, lib

HUBER_MONO = float(np.float32(np.sqrt(np.float32(5.991))))   # const float thHuberMono = sqrt(5.991)


class _Problem(C.Structure):
    _fields_ = [("n_poses", C.c_int32), ("pose_id", C.c_void_p), ("pose_fixed", C.c_void_p), ("pose_q", C.c_void_p),
                ("pose_t", C.c_void_p), ("pose_cam", C.c_void_p), ("n_points", C.c_int32), ("point_id", C.c_void_p),
                ("point_xyz", C.c_void_p), ("n_edges", C.c_int32), ("edge_point", C.c_void_p),
                ("edge_pose", C.c_void_p), ("edge_obs", C.c_void_p), ("edge_inv_sigma2", C.c_void_p),
                ("n_cams", C.c_int32), ("cams", C.c_void_p), ("huber_delta", C.c_double), ("iterations", C.c_int32),
                ("edge_active", C.c_void_p), ("cam_model", C.c_int32), ("n_opt_poses", C.c_int32)]


class _Result(C.Structure):
    _fields_ = [("pose_q", C.c_void_p), ("pose_t", C.c_void_p), ("point_xyz", C.c_void_p), ("edge_chi2", C.c_void_p),
                ("edge_depth_ok", C.c_void_p), ("iterations", C.c_int32), ("lm_trials", C.c_int32),
                ("initial_chi2", C.c_double), ("final_chi2", C.c_double), ("status", C.c_int32)]


_SIGS = {
    "mam_lba_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "mam_lba_destroy": (None, [C.c_void_p]),
    "mam_lba_solve": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_lba_solve_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_lba_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "mam_lba_set_cu_mask": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "mam_lba_stage_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
}


@dataclass
class LBAProblem:
    pose_id: np.ndarray          # int64 [P]
    pose_fixed: np.ndarray       # uint8 [P]
    pose_q: np.ndarray           # float64 [P,4] xyzw
    pose_t: np.ndarray           # float64 [P,3]
    point_id: np.ndarray         # int64 [L]
    point_xyz: np.ndarray        # float64 [L,3]
    edge_point: np.ndarray       # int32 [E]
    edge_pose: np.ndarray        # int32 [E]
    edge_obs: np.ndarray         # float64 [E,2]
    edge_inv_sigma2: np.ndarray  # float64 [E]
    cams: np.ndarray             # float32 [C,4] Pinhole / [C,8] KannalaBrandt8 (cam_model 1)
    pose_cam: np.ndarray | None = None
    huber_delta: float = HUBER_MONO
    iterations: int = 10
    edge_active: np.ndarray | None = None   # uint8 per edge: 0 = setLevel(1) (left out)
    cam_model: int = 0                        # MAM_CAM_PINHOLE / MAM_CAM_KANNALA_BRANDT8

    def contiguous(self):
        for k, dt in [("pose_id", np.int64), ("pose_fixed", np.uint8), ("pose_q", np.float64), ("pose_t", np.float64),
                      ("point_id", np.int64), ("point_xyz", np.float64), ("edge_point", np.int32),
                      ("edge_pose", np.int32), ("edge_obs", np.float64), ("edge_inv_sigma2", np.float64),
                      ("cams", np.float32)]:
            setattr(self, k, np.ascontiguousarray(getattr(self, k), dt))
        if self.pose_cam is not None:
            self.pose_cam = np.ascontiguousarray(self.pose_cam, np.int32)
        if self.edge_active is not None:
            self.edge_active = np.ascontiguousarray(self.edge_active, np.uint8)
        return self

    def as_c(self) -> _Problem:
        self.contiguous()
        P = _Problem()
        P.n_poses = len(self.pose_id)
        P.pose_id, P.pose_fixed = self.pose_id.ctypes.data, self.pose_fixed.ctypes.data
        P.pose_q, P.pose_t = self.pose_q.ctypes.data, self.pose_t.ctypes.data
        P.pose_cam = None if self.pose_cam is None else self.pose_cam.ctypes.data
        P.n_points = len(self.point_id)
        P.point_id, P.point_xyz = self.point_id.ctypes.data, self.point_xyz.ctypes.data
        P.n_edges = len(self.edge_point)
        P.edge_point, P.edge_pose = self.edge_point.ctypes.data, self.edge_pose.ctypes.data
        P.edge_obs, P.edge_inv_sigma2 = self.edge_obs.ctypes.data, self.edge_inv_sigma2.ctypes.data
        P.n_cams = len(self.cams)
        P.cams = self.cams.ctypes.data
        P.huber_delta = float(self.huber_delta)
        P.iterations = int(self.iterations)
        P.edge_active = None if self.edge_active is None else self.edge_active.ctypes.data
        P.cam_model = int(self.cam_model)
        P.n_opt_poses = int((self.pose_fixed == 0).sum())
        return P


@dataclass
class LBAResult:
    pose_q: np.ndarray
    pose_t: np.ndarray
    point_xyz: np.ndarray
    edge_chi2: np.ndarray
    edge_depth_ok: np.ndarray
    iterations: int
    lm_trials: int
    initial_chi2: float
    final_chi2: float
    status: int

    def outliers(self):
        """Edges the reference erases: chi2() > 5.991 || !isDepthPositive() (Optimizer.cc:1413-1429)."""
        return (self.edge_chi2 > 5.991) | (self.edge_depth_ok == 0)


def alloc_result(prob: LBAProblem):
    P, L, E = len(prob.pose_id), len(prob.point_id), len(prob.edge_point)
    arrs = dict(pose_q=np.zeros((P, 4)), pose_t=np.zeros((P, 3)), point_xyz=np.zeros((L, 3)),
                edge_chi2=np.zeros(E), edge_depth_ok=np.zeros(E, np.uint8))
    R = _Result()
    R.pose_q, R.pose_t = arrs["pose_q"].ctypes.data, arrs["pose_t"].ctypes.data
    R.point_xyz = arrs["point_xyz"].ctypes.data
    R.edge_chi2, R.edge_depth_ok = arrs["edge_chi2"].ctypes.data, arrs["edge_depth_ok"].ctypes.data
    return R, arrs


def wrap_result(R: _Result, arrs) -> LBAResult:
    return LBAResult(arrs["pose_q"], arrs["pose_t"], arrs["point_xyz"], arrs["edge_chi2"], arrs["edge_depth_ok"],
                     int(R.iterations), int(R.lm_trials), float(R.initial_chi2), float(R.final_chi2), int(R.status))


class LBASolver:
    def __init__(self, device: int = 0):
        L = lib()
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        self._L = L
        self._ctx = C.c_void_p()
        check(L.mam_lba_create(int(device), C.byref(self._ctx)), "mam_lba_create")

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.mam_lba_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, prob: LBAProblem, stop_flag: np.ndarray | None = None) -> LBAResult:
        P = prob.as_c()
        R, arrs = alloc_result(prob)
        sf = None if stop_flag is None else stop_flag.ctypes.data_as(C.c_void_p)
        check(self._L.mam_lba_solve(self._ctx, C.byref(P), sf, C.byref(R)), "mam_lba_solve")
        return wrap_result(R, arrs)

    def solve_batch_device(self, batch: "DeviceBatch", stream: int = 0):
        """All problems of `batch` (device-resident, id-ordered) in one set of launches; fills batch.stats."""
        check(self._L.mam_lba_solve_batch_device(self._ctx, len(batch.probs), C.byref(batch.c_probs),
                                                 C.byref(batch.c_res), C.c_void_p(stream)), "mam_lba_solve_batch_device")
        batch.stats = [dict(iterations=int(r.iterations), lm_trials=int(r.lm_trials), initial_chi2=float(r.initial_chi2),
                            final_chi2=float(r.final_chi2), status=int(r.status)) for r in batch.c_res]
        return batch.stats

    def set_cu_mask(self, mask):
        """The CU mask (uint32 words; None: every CU) of the streams a split batch solve adds (mam_lba_set_cu_mask)."""
        m = None if mask is None else np.ascontiguousarray(mask, np.uint32)
        check(self._L.mam_lba_set_cu_mask(self._ctx, 0 if m is None else len(m), None if m is None else m.ctypes.data),
              "lba_set_cu_mask")
        self._cu_mask = m

    def set_profiling(self, enable: bool):
        check(self._L.mam_lba_set_profiling(self._ctx, 1 if enable else 0), "lba_set_profiling")

    def stage_times(self):
        ms = np.zeros(4)
        n = np.zeros(4, np.int64)
        check(self._L.mam_lba_stage_times(self._ctx, ms.ctypes.data_as(C.c_void_p), n.ctypes.data_as(C.c_void_p)),
              "lba_stage_times")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(["linearize", "schur", "solve", "update"])}


def id_ordered(prob: LBAProblem):
    """The same g2o graph with poses and points listed in ascending id (the Hessian order the device batch path
    takes, sparse_optimizer.cpp:166-190); edges keep their insertion order. Returns (problem, pose_order,
    point_order): row i of the new problem is row pose_order[i] / point_order[i] of the old one."""
    import dataclasses

    po = np.argsort(prob.pose_id, kind="stable")
    pl = np.argsort(prob.point_id, kind="stable")
    ipo = np.empty_like(po)
    ipo[po] = np.arange(len(po))
    ipl = np.empty_like(pl)
    ipl[pl] = np.arange(len(pl))
    q = dataclasses.replace(prob, pose_id=prob.pose_id[po], pose_fixed=prob.pose_fixed[po], pose_q=prob.pose_q[po],
                            pose_t=prob.pose_t[po], point_id=prob.point_id[pl], point_xyz=prob.point_xyz[pl],
                            edge_point=ipl[prob.edge_point].astype(np.int32),
                            edge_pose=ipo[prob.edge_pose].astype(np.int32),
                            pose_cam=None if prob.pose_cam is None else prob.pose_cam[po])
    return q.contiguous(), po, pl


class DeviceBatch:
    """Q LocalBundleAdjustment problems resident in HBM (torch tensors), id-ordered, with device result arrays, for
    LBASolver.solve_batch_device (mam_lba_solve_batch_device)."""

    def __init__(self, probs, device):
        import torch

        self.probs = [id_ordered(p)[0] for p in probs]
        self._keep = []
        Q = len(self.probs)
        self.c_probs = (_Problem * Q)()
        self.c_res = (_Result * Q)()
        self.res = []

        def dev(a, dt=None):
            t = torch.from_numpy(np.ascontiguousarray(a if dt is None else a.astype(dt))).to(device)
            self._keep.append(t)
            return t.data_ptr()

        for i, p in enumerate(self.probs):
            P = p.as_c()   # host struct; pointers replaced by device copies
            P.pose_id = P.point_id = None
            P.pose_fixed = dev(p.pose_fixed)
            P.pose_q, P.pose_t, P.point_xyz = dev(p.pose_q), dev(p.pose_t), dev(p.point_xyz)
            P.pose_cam = None if p.pose_cam is None else dev(p.pose_cam)
            P.edge_point, P.edge_pose = dev(p.edge_point), dev(p.edge_pose)
            P.edge_obs, P.edge_inv_sigma2 = dev(p.edge_obs), dev(p.edge_inv_sigma2)
            P.cams = dev(p.cams)
            P.edge_active = None if p.edge_active is None else dev(p.edge_active)
            self.c_probs[i] = P
            Pn, L, E = len(p.pose_id), len(p.point_id), len(p.edge_point)
            out = dict(pose_q=torch.zeros((Pn, 4), dtype=torch.float64, device=device),
                       pose_t=torch.zeros((Pn, 3), dtype=torch.float64, device=device),
                       point_xyz=torch.zeros((L, 3), dtype=torch.float64, device=device),
                       edge_chi2=torch.zeros(E, dtype=torch.float64, device=device),
                       edge_depth_ok=torch.zeros(E, dtype=torch.uint8, device=device))
            self.res.append(out)
            R = self.c_res[i]
            R.pose_q, R.pose_t = out["pose_q"].data_ptr(), out["pose_t"].data_ptr()
            R.point_xyz = out["point_xyz"].data_ptr()
            R.edge_chi2, R.edge_depth_ok = out["edge_chi2"].data_ptr(), out["edge_depth_ok"].data_ptr()
        self.stats = None

    def result(self, i) -> LBAResult:
        """Problem i's result (host copies, id order) as an LBAResult."""
        o = {k: v.cpu().numpy() for k, v in self.res[i].items()}
        s = self.stats[i]
        return LBAResult(o["pose_q"], o["pose_t"], o["point_xyz"], o["edge_chi2"], o["edge_depth_ok"],
                         s["iterations"], s["lm_trials"], s["initial_chi2"], s["final_chi2"], s["status"])


# ------------------------------------------------------------------------------------------------ synthetic
def _rot_to_quat(R):
    R = np.asarray(R, np.float64)
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        return np.array([(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s])
    i = int(np.argmax(np.diag(R)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
    q = np.zeros(4)
    q[i] = 0.25 * s
    q[3] = (R[k, j] - R[j, k]) / s
    q[j] = (R[j, i] + R[i, j]) / s
    q[k] = (R[k, i] + R[i, k]) / s
    return q


def _quat_to_rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def synthetic_problem(n_opt=50, n_fixed=10, n_points=3000, obs_per_point=8, seed=0, outlier_frac=0.05,
                      width=1280, height=720, f=500.0, init_kf_local=True, camera=None) -> LBAProblem:
    """SURVEY.md §8(d) LBA workload: optimizable KFs on a circle (r = 5 m) looking inward + fixed KFs,
    points U[-2,2]^3 each seen by `obs_per_point` KFs, pixel noise N(0, scale[oct]), gross outliers +20 px,
    initial poses perturbed by ~0.5 deg / 2 cm and points by 3 cm. Values pass through float32 as the map
    stores them (Optimizer.cc:1218, 1286). camera: a match.Camera (Pinhole / KannalaBrandt8) instead of the
    f-pinhole centred in width x height."""
    rng = np.random.default_rng(seed)
    n_kf = n_opt + n_fixed
    scale = [1.0]
    for _ in range(7):
        scale.append(float(np.float32(np.float64(np.float32(scale[-1])) * np.float64(np.float32(1.2)))))
    scale = np.array(scale, np.float32)
    inv_sigma2 = (np.float32(1.0) / (scale * scale)).astype(np.float32)
    cam = np.array([[f, f, width / 2, height / 2]], np.float32) if camera is None else camera.params()[None, :]
    ang = np.linspace(0, 2 * np.pi, n_kf, endpoint=False) + rng.uniform(0, 0.05, n_kf)
    Rs, ts = [], []
    for a in ang:
        c = np.array([5 * np.cos(a), 0.3 * np.sin(3 * a), 5 * np.sin(a)])
        zc = -c / np.linalg.norm(c)
        xc = np.cross([0, 1, 0], zc)
        xc /= np.linalg.norm(xc)
        yc = np.cross(zc, xc)
        Rwc = np.stack([xc, yc, zc], 1)
        Rcw = Rwc.T
        Rs.append(Rcw)
        ts.append(-Rcw @ c)
    X = rng.uniform(-2, 2, (n_points, 3))
    pose_fixed = np.zeros(n_kf, np.uint8)
    pose_fixed[n_opt:] = 1
    if init_kf_local:
        pose_fixed[0] = 1          # the map's init KF inside the local window (Optimizer.cc:1220)
    # ids: KF mnId unique; point id = mnId + maxKFid + 1
    kf_ids = rng.choice(10 * n_kf, size=n_kf, replace=False).astype(np.int64)
    maxkf = int(kf_ids.max())
    mp_ids = rng.choice(20 * n_points, size=n_points, replace=False).astype(np.int64) + maxkf + 1
    kf_ptr = rng.permutation(n_kf)     # std::map<KeyFrame*,...> iteration order = pointer order
    ep, eo, eobs, einf = [], [], [], []
    for l in range(n_points):
        k_opt = rng.choice(n_opt, size=min(obs_per_point - 1, n_opt), replace=False)
        k_fix = rng.choice(np.arange(n_opt, n_kf), size=1) if n_fixed > 0 else np.arange(n_opt, n_opt + 1)[:0]
        ks = np.concatenate([k_opt, k_fix])
        ks = ks[np.argsort(kf_ptr[ks])]
        for k in ks:
            Xc = Rs[k] @ X[l] + ts[k]
            oct_ = int(rng.integers(0, 8))
            if camera is None:
                u = f * Xc[0] / Xc[2] + width / 2 + rng.normal(0, scale[oct_])
                v = f * Xc[1] / Xc[2] + height / 2 + rng.normal(0, scale[oct_])
            else:
                u, v = camera.project_np(Xc) + rng.normal(0, scale[oct_], 2)
            if rng.random() < outlier_frac:
                u += 20.0
            ep.append(l)
            eo.append(k)
            eobs.append([np.float32(u), np.float32(v)])   # mvKeysUn are float
            einf.append(inv_sigma2[oct_])
    q0, t0 = [], []
    for k in range(n_kf):
        R, t = Rs[k], ts[k]
        if not pose_fixed[k]:
            w = rng.normal(size=3)
            w *= np.deg2rad(0.5) / np.linalg.norm(w)
            th = np.linalg.norm(w)
            K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / th
            dR = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
            R = dR @ R
            t = t + rng.normal(0, 0.02 / np.sqrt(3), 3)
        q = _rot_to_quat(R)
        if q[3] < 0:
            q = -q
        q = q.astype(np.float32)                           # KeyFrame pose is Sophus::SE3f
        q /= np.float32(np.linalg.norm(q.astype(np.float64)))
        q0.append(q.astype(np.float64))
        t0.append(t.astype(np.float32).astype(np.float64))
    Xn = (X + rng.normal(0, 0.03 / np.sqrt(3), X.shape)).astype(np.float32).astype(np.float64)
    return LBAProblem(pose_id=kf_ids, pose_fixed=pose_fixed, pose_q=np.array(q0), pose_t=np.array(t0),
                      point_id=mp_ids, point_xyz=Xn, edge_point=np.array(ep, np.int32), edge_pose=np.array(eo, np.int32),
                      edge_obs=np.array(eobs, np.float64), edge_inv_sigma2=np.array(einf, np.float64), cams=cam,
                      cam_model=0 if camera is None else int(camera.model)).contiguous()
