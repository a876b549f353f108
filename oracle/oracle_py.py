"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/liboracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
The product package (mam3slam_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class KeyPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("fp_policy", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.oracle_fast_atan2.restype = C.c_float
        _lib.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
    return _lib


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini=20, mn=7, fp_policy=0) -> OrbParams:
    return OrbParams(nfeatures, scale_factor, nlevels, ini, mn, fp_policy)


def _u8p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def extract(img: np.ndarray, p: OrbParams | None = None, lap=(0, 1000), simd: bool = False):
    """ORBextractor::operator() on the oracle. Returns (keypoints structured array, desc (N,32) u8, mono). simd: with
    the AVX2 resize / blur / FAST (oracle/orb_simd.cpp; the same outputs)."""
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = p.nfeatures + 3 * p.nlevels + 64
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    mono = C.c_int(0)
    fn = lib().oracle_orb_extract_simd if simd else lib().oracle_orb_extract
    rc = fn(C.byref(p), _u8p(img), w, h, C.c_size_t(w), int(lap[0]), int(lap[1]), kps.ctypes.data_as(C.c_void_p),
            _u8p(desc), cap, C.byref(n), C.byref(mono))
    if rc != 0:
        raise RuntimeError(f"oracle_orb_extract rc={rc}")
    return kps[:n.value].copy(), desc[:n.value].copy(), mono.value


def tables(p: OrbParams | None = None):
    p = p or params()
    L = p.nlevels
    scales = np.zeros(4 * L, np.float32)
    nfeat = np.zeros(L, np.int32)
    umax = np.zeros(16, np.int32)
    rc = lib().oracle_orb_tables(C.byref(p), scales.ctypes.data_as(C.c_void_p), nfeat.ctypes.data_as(C.c_void_p),
                                 umax.ctypes.data_as(C.c_void_p))
    assert rc == 0
    return scales.reshape(4, L), nfeat, umax


def pyramid(img: np.ndarray, p: OrbParams | None = None):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    sizes = np.zeros(2 * p.nlevels, np.int32)
    cap = w * h * 4
    out = np.zeros(cap, np.uint8)
    rc = lib().oracle_orb_pyramid(C.byref(p), _u8p(img), w, h, C.c_size_t(w), sizes.ctypes.data_as(C.c_void_p),
                                  _u8p(out), C.c_size_t(cap))
    assert rc == 0
    levels, off = [], 0
    for l in range(p.nlevels):
        lw, lh = int(sizes[2 * l]), int(sizes[2 * l + 1])
        levels.append(out[off:off + lw * lh].reshape(lh, lw).copy())
        off += lw * lh
    return levels


def resize_linear(src: np.ndarray, dw: int, dh: int, simd: bool = False) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.uint8)
    fn = lib().oracle_resize_linear_simd if simd else lib().oracle_resize_linear
    fn(_u8p(src), sw, sh, C.c_size_t(sw), _u8p(dst), dw, dh)
    return dst


def fast(roi: np.ndarray, threshold: int, simd: bool = False) -> np.ndarray:
    roi = np.ascontiguousarray(roi, dtype=np.uint8)
    rows, cols = roi.shape
    cap = rows * cols
    out = np.zeros(max(cap, 1), np.uint32)
    fn = lib().oracle_fast_simd if simd else lib().oracle_fast
    n = fn(_u8p(roi), cols, rows, C.c_size_t(cols), threshold, out.ctypes.data_as(C.c_void_p), cap)
    return out[:n].copy()


def gaussian7(src: np.ndarray, simd: bool = False) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape
    dst = np.zeros_like(src)
    (lib().oracle_gaussian7_simd if simd else lib().oracle_gaussian7)(_u8p(src), w, h, _u8p(dst))
    return dst


def gaussian_taps():
    t = np.zeros(7, np.int32)
    lib().oracle_gaussian7_taps(t.ctypes.data_as(C.c_void_p))
    return t


def fast_atan2(y: float, x: float) -> float:
    return float(lib().oracle_fast_atan2(y, x))


def sincos(a: float):
    s, c = C.c_float(), C.c_float()
    lib().oracle_sincos(C.c_float(a), C.byref(s), C.byref(c))
    return s.value, c.value


def sincos_policy(fp_policy: int, a: float):
    s, c = C.c_float(), C.c_float()
    lib().oracle_sincos_policy(int(fp_policy), C.c_float(a), C.byref(s), C.byref(c))
    return s.value, c.value


def level_stage(img: np.ndarray, level: int, p: OrbParams | None = None):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = w * h
    cand = np.zeros(cap, np.uint32)
    kept = np.zeros(cap, np.uint32)
    nc, nk = C.c_int(), C.c_int()
    rc = lib().oracle_level_stage(C.byref(p), _u8p(img), w, h, C.c_size_t(w), level,
                                  cand.ctypes.data_as(C.c_void_p), cap, C.byref(nc),
                                  kept.ctypes.data_as(C.c_void_p), cap, C.byref(nk))
    assert rc == 0
    return cand[:nc.value].copy(), kept[:nk.value].copy()


def distribute(cand: np.ndarray, minx, maxx, miny, maxy, n_keep) -> np.ndarray:
    cand = np.ascontiguousarray(cand, dtype=np.uint32)
    cap = max(len(cand), 1) + 8
    out = np.zeros(cap, np.uint32)
    m = lib().oracle_distribute(cand.ctypes.data_as(C.c_void_p), len(cand), minx, maxx, miny, maxy, n_keep,
                                out.ctypes.data_as(C.c_void_p), cap)
    return out[:m].copy()


def std_sort_pairs(keys: np.ndarray, payload: np.ndarray):
    k = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    v = np.ascontiguousarray(payload, dtype=np.uint32).copy()
    lib().oracle_std_sort_pairs(k.ctypes.data_as(C.c_void_p), v.ctypes.data_as(C.c_void_p), len(k))
    return k, v


def unpack(packed: np.ndarray):
    packed = np.asarray(packed, dtype=np.uint32)
    return packed & 0xFFF, (packed >> 12) & 0xFFF, packed >> 24


# ---------------------------------------------------------------- matcher oracle (oracle/match_oracle.cpp)
def _vp(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def descriptor_distance(a, b) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().oracle_descriptor_distance(_vp(a), _vp(b)))


def search_by_projection(F, mps, th, far_points=False, th_far=50.0, nnratio=0.8):
    """F: mam3slam_amd.match.FrameData; mps: MP_TRACK_DTYPE array. Returns (nmatches, kp_to_mp)."""
    from mam3slam_amd.match import KP_DTYPE, MP_TRACK_DTYPE

    L = lib()
    L.oracle_search_by_projection.restype = C.c_int
    L.oracle_search_by_projection.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                              C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_float, C.c_void_p]
    keys = np.ascontiguousarray(F.keys, KP_DTYPE)
    desc = np.ascontiguousarray(F.desc, np.uint8)
    taken = None if F.taken is None else np.ascontiguousarray(F.taken, np.uint8)
    mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
    out = np.full(max(len(keys), 1), -1, np.int32)
    g = F.geom()
    n = L.oracle_search_by_projection(C.byref(g), len(keys), _vp(keys), _vp(desc), _vp(taken), len(mps), _vp(mps),
                                      float(th), int(far_points), float(th_far), float(nnratio), _vp(out))
    return n, out[:len(keys)]


def search_by_projection_motion(F, last, cam, th, check_ori=True):
    from mam3slam_amd.match import KP_DTYPE, LAST_ENTRY_DTYPE, Pose

    L = lib()
    L.oracle_search_by_projection_motion.restype = C.c_int
    L.oracle_search_by_projection_motion.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                     C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_float, C.c_int,
                                                     C.c_void_p]
    keys = np.ascontiguousarray(F.keys, KP_DTYPE)
    desc = np.ascontiguousarray(F.desc, np.uint8)
    taken = None if F.taken is None else np.ascontiguousarray(F.taken, np.uint8)
    last = np.ascontiguousarray(last, LAST_ENTRY_DTYPE)
    pose = Pose()
    for i in range(4):
        pose.q[i] = float(F.pose[0][i])
    for i in range(3):
        pose.t[i] = float(F.pose[1][i])
    out = np.full(max(len(keys), 1), -1, np.int32)
    g = F.geom()
    n = L.oracle_search_by_projection_motion(C.byref(g), len(keys), _vp(keys), _vp(desc), _vp(taken), C.byref(pose),
                                             C.byref(cam), len(last), _vp(last), float(th), int(check_ori), _vp(out))
    return n, out[:len(keys)]


def track_motion_search(F, last, cam, th=15.0, check_ori=True, min_matches=20):
    """Tracking::TrackWithMotionModel's search (Tracking.cc:2811-2824): SearchByProjection(Cur, Last, th); with fewer
    than 20 matches the current frame's MapPoints are cleared and the search runs again at 2 th. Returns (n, out,
    retried)."""
    n, out = search_by_projection_motion(F, last, cam, th, check_ori)
    if n < min_matches:
        n, out = search_by_projection_motion(F, last, cam, 2 * th, check_ori)
        return n, out, True
    return n, out, False


def search_for_triangulation(KF1, KF2, F12, ep, check_ori=False, coarse=False):
    from mam3slam_amd.match import KP_DTYPE, FeatVec, flatten_featvec

    L = lib()
    L.oracle_search_for_triangulation.restype = C.c_int
    L.oracle_search_for_triangulation.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                  C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    k1 = np.ascontiguousarray(KF1.keys, KP_DTYPE)
    k2 = np.ascontiguousarray(KF2.keys, KP_DTYPE)
    d1 = np.ascontiguousarray(KF1.desc, np.uint8)
    d2 = np.ascontiguousarray(KF2.desc, np.uint8)
    h1 = np.ascontiguousarray(KF1.has_mp, np.uint8)
    h2 = np.ascontiguousarray(KF2.has_mp, np.uint8)
    i1, o1, f1 = flatten_featvec(KF1.featvec)
    i2, o2, f2 = flatten_featvec(KF2.featvec)
    fv1 = FeatVec(len(i1), i1.ctypes.data, o1.ctypes.data, f1.ctypes.data)
    fv2 = FeatVec(len(i2), i2.ctypes.data, o2.ctypes.data, f2.ctypes.data)
    F12 = np.ascontiguousarray(F12, np.float32).reshape(9)
    ep = np.ascontiguousarray(ep, np.float32).reshape(2)
    out = np.full(max(len(k1), 1), -1, np.int32)
    g = KF2.geom()
    n = L.oracle_search_for_triangulation(C.byref(g), len(k1), _vp(k1), _vp(d1), _vp(h1), C.byref(fv1), len(k2),
                                          _vp(k2), _vp(d2), _vp(h2), C.byref(fv2), _vp(F12), _vp(ep), int(check_ori),
                                          int(coarse), _vp(out))
    return n, out[:len(k1)]


def search_for_triangulation_kf(KF1, KF2, cam1, cam2=None, check_ori=False, coarse=False):
    """SearchForTriangulation from poses + cameras (Pinhole or KannalaBrandt8), the oracle's own pair geometry."""
    from mam3slam_amd.match import KP_DTYPE, FeatVec, TriKF, flatten_featvec, pose_c

    L = lib()
    L.oracle_search_for_triangulation_kf.restype = C.c_int
    L.oracle_search_for_triangulation_kf.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    cam2 = cam1 if cam2 is None else cam2
    keep, kf = [], []
    for KF, cam in ((KF1, cam1), (KF2, cam2)):
        k = np.ascontiguousarray(KF.keys, KP_DTYPE)
        d = np.ascontiguousarray(KF.desc, np.uint8)
        h = np.ascontiguousarray(KF.has_mp if KF.has_mp is not None else np.zeros(len(k)), np.uint8)
        ids, off, feats = flatten_featvec(KF.featvec)
        keep += [k, d, h, ids, off, feats]
        t = TriKF()
        t.n = len(k)
        t.keys, t.desc, t.has_mp = _vp(k), _vp(d), _vp(h)
        t.fv = FeatVec(len(ids), ids.ctypes.data, off.ctypes.data, feats.ctypes.data)
        t.tcw = pose_c(KF.pose)
        t.cam = cam
        kf.append(t)
    out = np.full(max(len(KF1.keys), 1), -1, np.int32)
    g = KF2.geom()
    n = L.oracle_search_for_triangulation_kf(C.byref(g), C.byref(kf[0]), C.byref(kf[1]), int(check_ori), int(coarse),
                                             _vp(out))
    return n, out[:len(KF1.keys)]


def kb8_project(cam, X):
    """KannalaBrandt8::project(Vector3f) / Pinhole::project as the oracle evaluates it (float32 u, v)."""
    L = lib()
    L.oracle_kb8_project.restype = None
    L.oracle_kb8_project.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    X = np.ascontiguousarray(X, np.float32)
    uv = np.zeros(2, np.float32)
    L.oracle_kb8_project(C.byref(cam), _vp(X), _vp(uv))
    return uv


def kb8_unproject(cam, px, py):
    L = lib()
    L.oracle_kb8_unproject.restype = None
    L.oracle_kb8_unproject.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_void_p]
    r = np.zeros(3, np.float32)
    L.oracle_kb8_unproject(C.byref(cam), float(px), float(py), _vp(r))
    return r


def kb8_triangulate(cam1, cam2, kp1, kp2, R12, t12, sigma1, sigma2):
    """KannalaBrandt8::TriangulateMatches: z1 > 0 or the reference's negative codes -1..-5."""
    L = lib()
    L.oracle_kb8_triangulate.restype = C.c_float
    L.oracle_kb8_triangulate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_float, C.c_float]
    a = [np.ascontiguousarray(v, np.float32).reshape(-1) for v in (kp1, kp2, R12, t12)]
    return float(L.oracle_kb8_triangulate(C.byref(cam1), C.byref(cam2), *[_vp(v) for v in a], float(sigma1),
                                          float(sigma2)))


def fuse(KF, mps, cam, th=3.0):
    """ORBmatcher::Fuse per-MapPoint search. Returns (n, idx, dist) like mam3slam_amd.match.ORBmatcher.Fuse."""
    from mam3slam_amd.match import FUSE_MP_DTYPE, KP_DTYPE, fuse_kf

    L = lib()
    L.oracle_fuse.restype = C.c_int
    L.oracle_fuse.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                              C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
    keys = np.ascontiguousarray(KF.keys, KP_DTYPE)
    desc = np.ascontiguousarray(KF.desc, np.uint8)
    mps = np.ascontiguousarray(mps, FUSE_MP_DTYPE)
    kf = fuse_kf(KF.pose)
    idx = np.full(max(len(mps), 1), -1, np.int32)
    dist = np.full(max(len(mps), 1), 256, np.int32)
    g = KF.geom()
    n = L.oracle_fuse(C.byref(g), len(keys), _vp(keys), _vp(desc), C.byref(kf), C.byref(cam), len(mps), _vp(mps),
                      float(th), _vp(idx), _vp(dist))
    return n, idx[:len(mps)], dist[:len(mps)]


def is_in_frustum(F, mps, cam, view_cos_limit=0.5, scale_factor=1.2):
    """SearchLocalPoints' isInFrustum + PredictScale loop. Returns (nToMatch, MP_TRACK_DTYPE tracks)."""
    from mam3slam_amd.match import LOCAL_MP_DTYPE, MP_TRACK_DTYPE, Pose

    L = lib()
    L.oracle_is_in_frustum.restype = C.c_int
    L.oracle_is_in_frustum.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_int, C.c_void_p, C.c_float,
                                       C.c_void_p]
    mps = np.ascontiguousarray(mps, LOCAL_MP_DTYPE)
    out = np.zeros(max(len(mps), 1), MP_TRACK_DTYPE)
    T = Pose()
    for i in range(4):
        T.q[i] = float(F.pose[0][i])
    for i in range(3):
        T.t[i] = float(F.pose[1][i])
    g = F.geom()
    n = L.oracle_is_in_frustum(C.byref(g), C.byref(T), C.byref(cam), float(np.log(np.float32(scale_factor))), len(mps),
                               _vp(mps), float(view_cos_limit), _vp(out))
    return n, out[:len(mps)]


def distinctive_descriptors(desc_off, descs):
    L = lib()
    L.oracle_distinctive_descriptors.restype = C.c_int
    L.oracle_distinctive_descriptors.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    off = np.ascontiguousarray(desc_off, np.int32)
    d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
    n = len(off) - 1
    out = np.full(max(n, 1), -1, np.int32)
    L.oracle_distinctive_descriptors(n, _vp(off), _vp(d) if len(d) else None, _vp(out))
    return out[:n]


# ---------------------------------------------------------------- DBoW2 oracle (oracle/bow_oracle.cpp)
class BowTree:
    """A tree built once by the oracle (oracle_bow_build), for repeated transforms."""

    def __init__(self, v):
        L = lib()
        L.oracle_bow_build.restype = C.c_void_p
        L.oracle_bow_build.argtypes = [C.c_int] * 4 + [C.c_void_p] * 4
        L.oracle_bow_free.argtypes = [C.c_void_p]
        self._L = L
        self.h = L.oracle_bow_build(v.L, v.weighting, v.scoring, v.n_nodes, _vp(v.parent), _vp(v.is_leaf),
                                    _vp(v.desc), _vp(v.weight))

    def __del__(self):
        if getattr(self, "h", None):
            self._L.oracle_bow_free(self.h)
            self.h = None


def bow_transform(v, descs, levelsup=4, tree: BowTree | None = None):
    """v: mam3slam_amd.bow.VocabularyArrays. Returns ((word, weight, nid) per feature, bow dict, featvec dict)."""
    t = BowTree(v) if tree is None else tree
    L = lib()
    L.oracle_bow_run.restype = C.c_int
    L.oracle_bow_run.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int] + [C.c_void_p] * 9
    d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
    n = len(d)
    m = max(n, 1)
    w, x, nid = np.zeros(m, np.uint32), np.zeros(m, np.float64), np.zeros(m, np.uint32)
    bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
    fi, fo, ff = np.zeros(m, np.uint32), np.zeros(m + 1, np.int32), np.zeros(m, np.uint32)
    nf = C.c_int(0)
    nb = L.oracle_bow_run(t.h, n, _vp(d), int(levelsup), _vp(w), _vp(x), _vp(nid), _vp(bw), _vp(bv), _vp(fi), _vp(fo),
                          _vp(ff), C.byref(nf))
    bow = {int(bw[i]): float(bv[i]) for i in range(nb)}
    fv = {int(fi[j]): [int(q) for q in ff[fo[j]:fo[j + 1]]] for j in range(nf.value)}
    return (w[:n], x[:n], nid[:n]), bow, fv


# ---------------------------------------------------------------- LBA oracle (oracle/lba_oracle.cpp)
def lba_solve(prob, stop=None):
    """g2o LocalBundleAdjustment solve restatement. prob: mam3slam_amd.lba.LBAProblem."""
    from mam3slam_amd.lba import alloc_result, wrap_result

    L = lib()
    L.oracle_lba_solve.restype = C.c_int
    L.oracle_lba_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    P = prob.as_c()
    R, arrs = alloc_result(prob)
    sf = None if stop is None else stop.ctypes.data_as(C.c_void_p)
    rc = L.oracle_lba_solve(C.byref(P), sf, C.byref(R))
    assert rc == 0, rc
    return wrap_result(R, arrs)


# ---------------------------------------------------------------- PoseOptimization oracle (oracle/pose_oracle.cpp)
def pose_optimization_edges(pose, cam, edges):
    """g2o PoseOptimization restatement on explicit edges (mam3slam_amd.pose.POSE_EDGE_DTYPE).
    Returns (n_inliers, outlier uint8[n], (q float64[4], t float64[3]), stats)."""
    from mam3slam_amd.pose import POSE_EDGE_DTYPE, PoseResult, pose_struct

    L = lib()
    L.oracle_pose_optimization.restype = C.c_int
    L.oracle_pose_optimization.argtypes = [C.c_void_p] * 2 + [C.c_int] + [C.c_void_p] * 3
    e = np.ascontiguousarray(edges, POSE_EDGE_DTYPE)
    n = len(e)
    out = np.zeros(max(n, 1), np.uint8)
    res = PoseResult()
    p = pose_struct(pose)
    rc = L.oracle_pose_optimization(C.byref(p), C.byref(cam), n, e.ctypes.data if n else None, out.ctypes.data,
                                    C.byref(res))
    assert rc >= 0, rc
    stats = {"rounds": res.rounds, "iterations": res.iterations, "lm_trials": res.lm_trials}
    return rc, out[:n].copy(), (np.array(res.q[:]), np.array(res.t[:])), stats


def pose_optimization(F, mps_xyz, cam):
    """Optimizer::PoseOptimization(pFrame) on a FrameData (same conventions as mam3slam_amd.pose.pose_optimization):
    returns (n_inliers, outlier per keypoint, (q, t))."""
    from mam3slam_amd.pose import make_edges

    idx = np.nonzero(F.map_point >= 0)[0]
    edges = make_edges(F.keys, 1.0 / F.level_sigma2, idx, mps_xyz[F.map_point[idx]])
    n, out, qt, _ = pose_optimization_edges(F.pose, cam, edges)
    outl = np.zeros(len(F.keys), np.uint8)
    outl[idx] = out
    return n, outl, qt
