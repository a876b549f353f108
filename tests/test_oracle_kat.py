"""CPU: pin the oracle (oracle/orb_oracle.cpp) with hand-derived known answers.

The reference ships no golden vectors for this path and cannot be built here, so the
OpenCV-4.5.4 primitives are pinned by values derivable by hand from the reference source and the published
algorithms; everything else is "parity unpinned" (DESIGN.md §Oracle).
"""
import ctypes
import ctypes.util
import math
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_constructor_tables(oracle):
    scales, nfeat, umax = oracle.tables(oracle.params(1000))
    # mnFeaturesPerLevel (ORBextractor.cc:434-445) — SURVEY.md §8 table
    assert nfeat.tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert oracle.tables(oracle.params(2000))[1].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    assert oracle.tables(oracle.params(700))[1].tolist() == [152, 127, 106, 88, 73, 61, 51, 42]
    assert oracle.tables(oracle.params(1500))[1].tolist() == [326, 271, 226, 189, 157, 131, 109, 91]
    assert oracle.tables(oracle.params(5000))[1].tolist() == [1086, 905, 754, 628, 524, 436, 364, 303]
    # umax (ORBextractor.cc:453-468)
    assert umax.tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    # scale chain float(prev * (double)1.2f)
    s = [1.0]
    for _ in range(7):
        s.append(float(np.float32(np.float64(np.float32(s[-1])) * np.float64(np.float32(1.2)))))
    assert np.array_equal(scales[0], np.array(s, np.float32))
    assert np.array_equal(scales[1], np.float32(1.0) / scales[0])


def test_pyramid_sizes(oracle):
    img = np.zeros((480, 640), np.uint8)
    levels = oracle.pyramid(img)
    assert [l.shape[::-1] for l in levels] == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231),
                                               (257, 193), (214, 161), (179, 134)]
    assert sum(l.size for l in levels) == 950532
    img = np.zeros((720, 1280), np.uint8)
    assert sum(l.size for l in oracle.pyramid(img)) == 2853088


def test_gaussian_taps_and_impulse(oracle):
    taps = oracle.gaussian_taps()
    assert taps.tolist() == [18, 34, 48, 56, 48, 34, 18] and taps.sum() == 256
    # error-diffusion construction of getGaussianKernelFixedPoint_ED, recomputed here
    k = [math.exp(x * x * (-0.125 / 4.0)) for x in (-6, -4, -2)]
    s = 2 * sum(k) + 1
    err, ed = 0.0, []
    for v in k:
        adj = v / s * 256 + err
        r = round(adj)
        err = adj - r
        ed.append(r)
    assert ed == [18, 34, 48] and 256 - 2 * sum(ed) == 56
    img = np.zeros((15, 15), np.uint8)
    img[7, 7] = 255
    out = oracle.gaussian7(img)
    for y in range(15):
        for x in range(15):
            ky = taps[y - 4] if 4 <= y <= 10 else 0
            kx = taps[x - 4] if 4 <= x <= 10 else 0
            assert out[y, x] == (int(ky) * int(kx) * 255 + 32768) >> 16
    const = np.full((20, 30), 77, np.uint8)
    assert np.all(oracle.gaussian7(const) == 77)


def test_fast_atan2(oracle):
    assert oracle.fast_atan2(0.0, 1.0) == 0.0
    assert oracle.fast_atan2(1.0, 0.0) == 90.0
    assert oracle.fast_atan2(0.0, -1.0) == 180.0
    assert oracle.fast_atan2(-1.0, 0.0) == 270.0
    rng = np.random.default_rng(0)
    for _ in range(2000):
        y, x = rng.integers(-400000, 400000, 2)
        if x == 0 and y == 0:
            continue
        ref = math.degrees(math.atan2(y, x)) % 360.0
        got = oracle.fast_atan2(float(y), float(x))
        d = abs(got - ref)
        assert min(d, 360 - d) < 0.01, (y, x, got, ref)


def _fast_bruteforce(roi, t):
    """Textbook FAST-9/16 (segment test, cornerScore = max(t, best arc margin) - 1, strict 3x3 NMS inside the
    detection band) — an independent statement of App. A.1 used to pin the oracle's OpenCV restatement."""
    rows, cols = roi.shape
    circ = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
            (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    score = np.zeros((rows, cols), np.int32)
    corner = np.zeros((rows, cols), bool)
    for i in range(3, rows - 3):
        for j in range(3, cols - 3):
            v = int(roi[i, j])
            d = [v - int(roi[i + dy, j + dx]) for dx, dy in circ]
            A = max(min(d[(s + k) % 16] for k in range(9)) for s in range(16))
            B = max(min(-d[(s + k) % 16] for k in range(9)) for s in range(16))
            if max(A, B) > t:
                corner[i, j] = True
                score[i, j] = max(t, A, B) - 1
    out = []
    for i in range(3, rows - 3):
        for j in range(3, cols - 3):
            if corner[i, j]:
                s = score[i, j]
                nb = score[i - 1:i + 2, j - 1:j + 2].copy()
                nb[1, 1] = -1
                if (s > nb).all():
                    out.append(j | (i << 12) | (int(s) << 24))
    return np.array(out, np.uint32)


def test_fast_isolated_peak(oracle):
    roi = np.zeros((9, 9), np.uint8)
    roi[4, 4] = 100
    got = oracle.fast(roi, 20)
    assert got.tolist() == [4 | (4 << 12) | (99 << 24)]


@pytest.mark.parametrize("seed", range(6))
def test_fast_matches_definition(oracle, seed):
    rng = np.random.default_rng(seed)
    roi = rng.integers(0, 256, size=(24, 29)).astype(np.uint8)
    if seed % 2:
        from scipy.ndimage import uniform_filter

        roi = uniform_filter(roi.astype(np.float32), 2).astype(np.uint8)
    for t in (7, 20, 40):
        assert np.array_equal(oracle.fast(roi, t), _fast_bruteforce(roi, t)), (seed, t)


def test_distribute_reversed_list_order(oracle):
    # one initial node over [0,100]^2 split once into 4 single-key children: push_front n1..n4 leaves the
    # list [n4, n3, n2, n1] (ORBextractor.cc:626-671)
    def pk(x, y, s):
        return x | (y << 12) | (s << 24)

    cand = np.array([pk(10, 10, 5), pk(60, 10, 7), pk(10, 60, 9), pk(60, 60, 1)], np.uint32)
    out = oracle.distribute(cand, 0, 100, 0, 100, 4)
    assert out.tolist() == [pk(60, 60, 1), pk(10, 60, 9), pk(60, 10, 7), pk(10, 10, 5)]
    # retain best: two keys sharing the upper-left quadrant at N=1 -> the root split already gives
    # size >= N, nodes keep their max-response key (first max wins)
    cand = np.array([pk(10, 10, 5), pk(12, 11, 8), pk(13, 12, 8), pk(80, 80, 3)], np.uint32)
    out = oracle.distribute(cand, 0, 100, 0, 100, 1)
    assert out.tolist() == [pk(80, 80, 3), pk(12, 11, 8)]


def test_device_introsort_matches_libstdcxx(tmp_path):
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests/cpp/test_introsort.cpp")],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


def test_det_sincos_correctly_rounded(oracle):
    """det_sincos = (float)cos/sin of the float argument evaluated in double; compare with Python's libm
    double cos/sin rounded once to float over the rBRIEF argument range [0, 2*pi)."""
    rng = np.random.default_rng(1)
    xs = np.float32(rng.uniform(0, 2 * np.pi, 20000))
    bad = 0
    for x in xs:
        s, c = oracle.sincos(float(x))
        if s != float(np.float32(math.sin(float(x)))) or c != float(np.float32(math.cos(float(x)))):
            bad += 1
    assert bad == 0


def test_glibc_sincosf_restatement_exact(oracle, tmp_path):
    """The default steering trig (fp_policy 0) is glibc 2.35 sincosf, the reference image's libm (ros:humble =
    Ubuntu 22.04, as this container): the oracle's and the device's restatements equal this container's libm
    sincosf/sinf/cosf bit for bit on every 7th float of [0, 2*pi] (tests/cpp/test_glibc_sincosf.cpp; the full sweep,
    stride 1, is 1,086,918,684 floats, all equal: DESIGN.md §4)."""
    exe = tmp_path / "tgs"
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests/cpp/test_glibc_sincosf.cpp"), "-L", odir, "-l:liboracle.so",
                    f"-Wl,-rpath,{odir}", "-ldl"], check=True)
    r = subprocess.run([str(exe), "7"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


def test_glibc_sincosf_kat(oracle):
    """Known answers of glibc 2.35 sincosf (this container's libm) at the quadrant boundaries and the three code
    paths (tiny argument, |x| < pio4 polynomial, reduce_fast)."""
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    for f in ("sinf", "cosf"):
        getattr(libm, f).restype = ctypes.c_float
        getattr(libm, f).argtypes = [ctypes.c_float]
    for x in [0.0, 1e-5, 0.5, 0.78, 0.7853982, 1.5707964, 3.1415927, 4.712389, 6.2831855, 2.0943952, 5.759587]:
        s, c = oracle.sincos_policy(0, x)
        assert s == libm.sinf(x) and c == libm.cosf(x), x


def _pose_setup(oracle, seed, **kw):
    from mam3slam_amd import scene, synth

    img = synth.make_frame(640, 480, agent=1, frame=seed)
    k, d, _ = oracle.extract(img, oracle.params(1000))
    cam = scene.pinhole(640, 480)
    F = scene.make_frame_data(k, d, 640, 480)
    xyz, truth = scene.pose_problem(F, cam, np.random.default_rng(seed), **kw)
    return F, xyz, truth, cam


def test_pose_oracle_exact_geometry_recovers_truth(oracle):
    """KAT: noise- and outlier-free correspondences -> PoseOptimization converges to the true pose, no outliers."""
    F, xyz, (qt, tt), cam = _pose_setup(oracle, 0, noise=0.0, outlier_frac=0.0)
    n, outl, (q, t) = oracle.pose_optimization(F, xyz, cam)
    assert n == int((F.map_point >= 0).sum()) and outl.sum() == 0
    # the true pose and the points are float32: residual error ~1e-6
    assert np.allclose(q * np.sign(q[3]), qt * np.sign(qt[3]), atol=2e-6)
    assert np.allclose(t, tt, atol=2e-5)


def test_pose_oracle_flags_gross_outliers(oracle):
    F, xyz, _, cam = _pose_setup(oracle, 1, noise=0.5, outlier_frac=0.1)
    n, outl, _ = oracle.pose_optimization(F, xyz, cam)
    idx = np.nonzero(F.map_point >= 0)[0]
    # every displaced point (15-60 px at level scale >= 1, sigma^-2 <= 1) is above chi2 5.991
    assert outl[idx].sum() >= 0.08 * len(idx) and n == len(idx) - outl.sum()


def test_pose_oracle_too_few_correspondences(oracle):
    """nInitialCorrespondences < 3 -> return 0, pose untouched (Optimizer.cc:997-998)."""
    from mam3slam_amd.pose import POSE_EDGE_DTYPE

    from mam3slam_amd import scene

    cam = scene.pinhole(640, 480)
    q = np.array([0.0, 0.0, 0.0, 1.0], np.float32)
    t = np.array([0.1, -0.2, 0.3], np.float32)
    e = np.zeros(2, POSE_EDGE_DTYPE)
    e["obs"] = [[100, 100], [200, 300]]
    e["xw"] = [[0, 0, 5], [1, 1, 6]]
    e["inv_sigma2"] = 1.0
    n, out, (qo, to), st = oracle.pose_optimization_edges((q, t), cam, e)
    assert n == 0 and st["rounds"] == 0 and not out.any()
    assert np.array_equal(qo, q.astype(np.float64)) and np.array_equal(to, t.astype(np.float64))


def test_distinctive_oracle_median_rule(oracle):
    """ComputeDistinctiveDescriptors (MapPoint.cc:383-397): median = element (N-1)/2 of the sorted distance row,
    smallest median wins, first on ties."""
    a = np.zeros(32, np.uint8)
    b = a.copy()
    b[:2] = 0xFF     # 16 bits from a
    c = np.full(32, 0xFF, np.uint8)   # 256 from a, 240 from b
    # MapPoint 0 rows (c, a, b): medians c [0,240,256] -> 240, a [0,16,256] -> 16, b [0,16,240] -> 16 -> row 1
    # MapPoint 1 (N = 2): both medians are element 0 = 0 -> row 0; MapPoint 2: no rows -> -1
    # MapPoint 3 (c, a, a, c): every sorted row is [0, 0, 256, 256], element 1 = 0 -> row 0
    off = np.array([0, 3, 5, 5, 9], np.int32)
    d = np.stack([c, a, b, c, a, c, a, a, c])
    assert list(oracle.distinctive_descriptors(off, d)) == [1, 0, -1, 0]


def test_fuse_oracle_hand_example(oracle):
    """Fuse (ORBmatcher.cc:1177-1333) on a 3-keypoint keyframe at the identity pose."""
    from mam3slam_amd import scene
    from mam3slam_amd.match import FUSE_MP_DTYPE, Pinhole
    from mam3slam_amd.orb import KP_DTYPE

    keys = np.zeros(3, KP_DTYPE)
    keys["x"] = [100.0, 300.0, 302.0]
    keys["y"] = [100.0, 200.0, 200.0]
    keys["octave"] = [0, 1, 1]
    desc = np.zeros((3, 32), np.uint8)
    desc[1:] = 0x0F
    desc[2, 0] = 0x00    # 4 bits from keypoint 1
    KF = scene.make_frame_data(keys, desc, 640, 480)
    KF.pose = (np.array([0, 0, 0, 1], np.float32), np.zeros(3, np.float32))
    cam = Pinhole(500.0, 500.0, 320.0, 240.0)

    def mp(u, v, z, drow, lvl):
        m = np.zeros(1, FUSE_MP_DTYPE)
        X = np.array([(u - 320) / 500 * z, (v - 240) / 500 * z, z], np.float64)
        dist = np.linalg.norm(X)
        m["pos"] = X
        m["normal"] = X / dist
        m["max_distance"] = dist * 1.2 ** (lvl - 0.5)   # PredictScale -> lvl
        m["min_distance"] = m["max_distance"] / np.float32(1.2 ** 7)
        m["valid"] = 1
        m["desc"] = drow
        return m

    mps = np.concatenate([
        mp(300.5, 200.0, 4.0, desc[1], 1),    # keypoints 1 and 2 in the window: 1 is 0 bits away -> 1
        mp(301.5, 200.0, 4.0, desc[2], 1),    # -> 2 (0 bits)
        mp(300.5, 200.0, -4.0, desc[1], 1),   # behind the camera
        mp(100.2, 100.0, 3.0, ~desc[0], 0),   # 256 bits from keypoint 0: not < bestDist = 256
        mp(300.5, 200.0, 4.0, desc[1], 4),    # predicted level 4: the level-1 keypoints fail the level test
        mp(300.5, 200.0, 4.0, desc[1], 1),    # invalid (NULL / bad / already in the keyframe)
    ])
    mps["valid"][5] = 0
    n, idx, dist = oracle.fuse(KF, mps, cam, 3.0)
    assert n == 2 and list(idx) == [1, 2, -1, -1, -1, -1] and list(dist) == [0, 0, 256, 256, 256, 256]


def test_bow_oracle_hand_tree(oracle):
    """DBoW2 transform (TemplatedVocabulary.h:1216-1259) on a hand-built tree: root -> A, B; A -> A1, A2 (leaves);
    B leaf. Descent by the first minimum Hamming distance, the node at level L - levelsup, TF-IDF + L1."""
    from mam3slam_amd import bow

    z = np.zeros(32, np.uint8)
    A = z.copy()
    Bd = np.full(32, 0xFF, np.uint8)
    A1 = z.copy()
    A1[0] = 0x0F
    A2 = z.copy()
    A2[1] = 0xF0
    # nodes: 0 root, 1 A, 2 B (leaf, word 0), 3 A1 (word 1), 4 A2 (word 2)
    v = bow.VocabularyArrays(2, 2, bow.L1_NORM, bow.TF_IDF, [0, 0, 0, 1, 1], [0, 0, 1, 1, 1],
                             np.stack([z, A, Bd, A1, A2]), [0.0, 0.0, 2.0, 1.0, 3.0])
    f0 = A1.copy()                      # -> A (0 bits) -> A1 (0 bits): word 1
    f1 = A2.copy()                      # -> A -> A2: word 2
    f2 = np.full(32, 0xFF, np.uint8)    # -> B: word 0 (a leaf at level 1)
    f3 = z.copy()                       # A1 and A2 both 4 bits away: the first child, A1
    (w, x, nid), B, F = oracle.bow_transform(v, np.stack([f0, f1, f2, f3]), 1)   # node level 1
    assert list(w) == [1, 2, 0, 1] and list(x) == [1.0, 3.0, 2.0, 1.0] and list(nid) == [1, 1, 2, 1]
    assert B == {0: 2.0 / 7.0, 1: 2.0 / 7.0, 2: 3.0 / 7.0} and F == {1: [0, 1, 3], 2: [2]}
    assert bow.bow_from_words(w, x, nid) == (B, F)


def test_bow_text_round_trip(tmp_path):
    from mam3slam_amd import bow

    v = bow.synthetic_vocabulary(6, 3, np.random.default_rng(2), early_leaf=0.2)
    p = tmp_path / "v.txt"
    bow.save_to_text_file(v, str(p))
    r = bow.load_from_text_file(str(p))
    assert (r.k, r.L, r.scoring, r.weighting) == (6, 3, bow.L1_NORM, bow.TF_IDF)
    assert np.array_equal(r.parent, v.parent) and np.array_equal(r.is_leaf, v.is_leaf)
    assert np.array_equal(r.desc[1:], v.desc[1:]) and np.array_equal(r.weight, v.weight)


def _np_is_in_frustum(F, mps, cam, limit=np.float32(0.5)):
    """isInFrustum + PredictScale (Frame.cc:512-571, MapPoint.cc:531-546) restated in numpy float32, op for op in the
    oracle's order (Eigen rows / norm / dot as e0 + (e1 + e2)); log via float64 rounded to float32."""
    f32 = np.float32
    q, t = (np.asarray(F.pose[0], f32), np.asarray(F.pose[1], f32))
    qx, qy, qz, qw = q
    tx, ty, tz = f32(2) * qx, f32(2) * qy, f32(2) * qz
    twx, twy, twz, txx, txy, txz = tx * qw, ty * qw, tz * qw, tx * qx, ty * qx, tz * qx
    tyy, tyz, tzz = ty * qy, tz * qy, tz * qz
    R = np.array([f32(1) - (tyy + tzz), txy - twz, txz + twy, txy + twz, f32(1) - (txx + tzz), tyz - twx,
                  txz - twy, tyz + twx, f32(1) - (txx + tyy)], f32)
    p = -t
    iv = -q[:3]
    uv = np.array([iv[1] * p[2] - iv[2] * p[1], iv[2] * p[0] - iv[0] * p[2], iv[0] * p[1] - iv[1] * p[0]], f32)
    uv = uv + uv
    cr = np.array([iv[1] * uv[2] - iv[2] * uv[1], iv[2] * uv[0] - iv[0] * uv[2], iv[0] * uv[1] - iv[1] * uv[0]], f32)
    Ow = ((p + qw * uv) + cr) + f32(0)
    P = mps["pos"].astype(f32)
    Pc = [(R[3 * r] * P[:, 0] + (R[3 * r + 1] * P[:, 1] + R[3 * r + 2] * P[:, 2])) + t[r] for r in range(3)]
    pcd = np.sqrt(Pc[0] * Pc[0] + (Pc[1] * Pc[1] + Pc[2] * Pc[2]))
    with np.errstate(divide="ignore", invalid="ignore"):
        u = f32(cam.fx) * Pc[0] / Pc[2] + f32(cam.cx)
        v = f32(cam.fy) * Pc[1] / Pc[2] + f32(cam.cy)
    alive = (mps["seen"] == 0) & (mps["is_bad"] == 0) & ~(Pc[2] < 0)
    inimg = alive & ~((u < 0) | (u > f32(F.width)) | (v < 0) | (v > f32(F.height)))
    PO = [P[:, r] - Ow[r] for r in range(3)]
    dist = np.sqrt(PO[0] * PO[0] + (PO[1] * PO[1] + PO[2] * PO[2]))
    nr = mps["normal"].astype(f32)
    vc = (PO[0] * nr[:, 0] + (PO[1] * nr[:, 1] + PO[2] * nr[:, 2])) / dist
    ok = inimg & ~((dist < f32(0.8) * mps["min_distance"]) | (dist > f32(1.2) * mps["max_distance"])) & ~(vc < limit)
    ratio = mps["max_distance"].astype(f32) / dist
    lg = np.log(ratio.astype(np.float64)).astype(f32)
    lvl = np.ceil(lg / f32(np.log(f32(1.2)))).astype(np.int64)
    lvl = np.clip(lvl, 0, 7)
    return inimg, np.where(inimg, u, f32(-1)), np.where(inimg, v, f32(-1)), ok, pcd, vc, lvl


def test_is_in_frustum_oracle_vs_numpy(oracle):
    """The oracle's isInFrustum loop against an independent numpy float32 restatement of the same reference lines;
    every reject branch and every predicted level occurs."""
    from mam3slam_amd import scene, synth

    img = synth.make_frame(640, 480, agent=4, frame=2)
    k, d, _ = oracle.extract(img, oracle.params(1000))
    levels = set()
    for seed in range(4):
        rng = np.random.default_rng(70 + seed)
        F = scene.make_frame_data(k, d, 640, 480)
        F.pose = scene.small_pose(rng, rot=0.2, trans=0.5)
        cam = scene.pinhole(640, 480)
        mps = scene.local_world_mappoints(F, cam, rng)
        n, tr = oracle.is_in_frustum(F, mps, cam)
        inimg, u, v, ok, pcd, vc, lvl = _np_is_in_frustum(F, mps, cam)
        assert n == int(ok.sum()) and np.array_equal(tr["track_in_view"] == 1, ok)
        assert np.array_equal(tr["proj_x"], u) and np.array_equal(tr["proj_y"], v)
        assert np.array_equal(tr["track_depth"][ok], pcd[ok]) and np.array_equal(tr["view_cos"][ok], vc[ok])
        assert np.array_equal(tr["scale_level"][ok], lvl[ok])
        levels |= set(lvl[ok].tolist())
        assert (inimg & ~ok).any() and (~inimg).any()
    assert levels == set(range(8))


def test_glibc_camera_restatement_exact(oracle, tmp_path):
    """The camera restatements (mam3slam_amd/csrc/camera.hpp, shared by the oracle and gfx950) equal this container's
    glibc 2.35 libm (the reference image's) bit for bit — atanf on every 97th float, atan2f on 4M pairs, tanf on every
    97th float of [-2.4, 2.4] — and KannalaBrandt8::project(Vector3f) / unproject equal the reference's scalar code
    built as the reference is built (g++ 11.4 -O3 -march=x86-64-v3: FMA contraction; tests/cpp/kb8_codegen_probe.cpp)
    on 2M random points / pixels of the test-YAML camera."""
    probe = tmp_path / "probe.o"
    exe = tmp_path / "tgc"
    subprocess.run(["g++", "-O3", "-march=x86-64-v3", "-c", "-o", str(probe),
                    os.path.join(ROOT, "tests/cpp/kb8_codegen_probe.cpp")], check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests/cpp/test_glibc_camera.cpp"), str(probe), "-ldl"], check=True)
    r = subprocess.run([str(exe), "97"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


def test_kb8_project_unproject_kat(oracle):
    """KannalaBrandt8 (test/settingsForTest_00.yaml): unproject inverts project to float precision across the image,
    the principal point maps to the optical axis, and the projection matches a float64 evaluation of the model."""
    from mam3slam_amd import scene

    cam = scene.kannala_brandt8()
    r = oracle.kb8_unproject(cam, cam.cx, cam.cy)
    assert abs(r[0]) < 1e-6 and abs(r[1]) < 1e-6 and r[2] == 1.0
    rng = np.random.default_rng(4)
    for _ in range(200):
        # inside the lens' monotonic field (theta_d < ~1.2 rad: 380 px); beyond it the reference's Newton solve leaves
        # the valid branch exactly as the restatement does
        rad, phi = 380 * np.sqrt(rng.uniform()), rng.uniform(0, 2 * np.pi)
        u, v = cam.cx + rad * np.cos(phi), cam.cy + rad * np.sin(phi)
        ray = oracle.kb8_unproject(cam, u, v)
        uv = oracle.kb8_project(cam, ray * np.float32(rng.uniform(0.5, 20)))
        assert abs(uv[0] - u) < 2e-3 and abs(uv[1] - v) < 2e-3, (u, v, uv)
        X = np.array([rng.uniform(-3, 3), rng.uniform(-3, 3), rng.uniform(0.3, 9)], np.float32)
        ref = cam.project_np(X.astype(np.float64))
        assert np.abs(oracle.kb8_project(cam, X) - ref).max() < 2e-3


def test_kb8_triangulate_matches_kat(oracle):
    """KannalaBrandt8::TriangulateMatches on exact correspondences: z1 = the point's depth in camera 1; parallel rays
    -> -1; a point behind both cameras -> -2; a correspondence far off its epipolar curve -> -4 / -5."""
    from mam3slam_amd import scene
    from mam3slam_amd.match import quat_to_rot

    cam = scene.kannala_brandt8()
    s2 = np.float32(1.44)
    ang = 0.05
    q2 = np.array([0, np.sin(ang / 2), 0, np.cos(ang / 2)], np.float32)
    t2 = np.array([-0.4, 0.05, 0.02], np.float32)
    R2 = quat_to_rot(q2).astype(np.float64)
    # T12 = T1w T2w^-1 with T1w = I: R12 = R2^T, t12 = -R2^T t2
    R12 = R2.T.astype(np.float32)
    t12 = (-R2.T @ t2.astype(np.float64)).astype(np.float32)
    rng = np.random.default_rng(8)
    for _ in range(50):
        X = np.array([rng.uniform(-4, 4), rng.uniform(-4, 4), rng.uniform(3, 15)])
        kp1 = cam.project_np(X)
        kp2 = cam.project_np(R2 @ X + t2)
        if not (0 < kp2[0] < 960 and 0 < kp2[1] < 960):
            continue
        z1 = oracle.kb8_triangulate(cam, cam, kp1, kp2, R12, t12, s2, s2)
        assert z1 > 0 and abs(z1 - X[2]) < 0.02 * X[2], (z1, X)
        assert oracle.kb8_triangulate(cam, cam, kp1, kp2 + np.array([0, 25.0]), R12, t12, s2, s2) in (-4.0, -5.0,
                                                                                                      -2.0, -3.0)
    kp = cam.project_np(np.array([0.5, 0.2, 5.0]))
    assert oracle.kb8_triangulate(cam, cam, kp, kp, np.eye(3), np.zeros(3), s2, s2) == -1.0


def test_kb8_triangulation_search_oracle(oracle):
    """SearchForTriangulation with KannalaBrandt8 keyframes on the oracle: a 3D-consistent pair (scene.keyframe_pair_3d)
    matches many features, and the two-view test rejects some of what bCoarse (no geometric test) accepts."""
    from mam3slam_amd import scene, synth

    img = synth.make_frame(960, 960, agent=1, frame=0)
    k, d, _ = oracle.extract(img, oracle.params(700))
    cam = scene.kannala_brandt8()
    F = scene.make_frame_data(k, d, 960, 960)
    KF1, KF2 = scene.keyframe_pair_3d(F, cam, np.random.default_rng(1))
    n, out = oracle.search_for_triangulation_kf(KF1, KF2, cam, cam, False, False)
    nc, outc = oracle.search_for_triangulation_kf(KF1, KF2, cam, cam, False, True)
    assert n > 50 and nc > n


def test_pinhole_kf_triangulation_oracle_equals_f12_entry(oracle):
    """The oracle's keyframe-level entry (its own pair geometry) equals its F12 entry fed the C-ABI's geometry
    (mam_triangulation_geometry, host arithmetic in libmam_gpu.so): both sides compute T12 / ep / F12 identically."""
    from mam3slam_amd import scene, synth
    from mam3slam_amd.match import triangulation_geometry

    img = synth.make_frame(640, 480, agent=2, frame=3)
    k, d, _ = oracle.extract(img, oracle.params(1000))
    pin = scene.pinhole(640, 480)
    F = scene.make_frame_data(k, d, 640, 480)
    KF1, KF2 = scene.keyframe_pair_3d(F, pin, np.random.default_rng(2))
    _, _, F12, ep = triangulation_geometry(KF1.pose, KF2.pose, pin)
    n1, o1 = oracle.search_for_triangulation_kf(KF1, KF2, pin, pin, True, False)
    n2, o2 = oracle.search_for_triangulation(KF1, KF2, F12, ep, True, False)
    assert n1 == n2 and np.array_equal(o1, o2) and n1 > 50


def test_simd_primitives_equal_scalar(oracle):
    """oracle/orb_simd.cpp (AVX2 resize vertical pass, 7x7 fixed-point blur, FAST 9/16 with the run-length counters)
    byte- / keypoint-identical to the scalar restatement on random and synthetic images, odd sizes and borders
    included; the whole extractor on synthetic frames of the bench shapes."""
    from mam3slam_amd import synth

    rng = np.random.default_rng(5)
    imgs = [rng.integers(0, 256, (h, w), dtype=np.uint8) for h, w in ((7, 7), (9, 40), (37, 53), (120, 161))]
    imgs += [synth.make_frame(640, 480, agent=3, frame=1), synth.make_frame(333, 251, agent=4, frame=2)]
    for im in imgs:
        h, w = im.shape
        for dw, dh in ((round(w / 1.2), round(h / 1.2)), (max(1, w // 2), max(1, h // 2)), (w + 13, h + 5)):
            assert np.array_equal(oracle.resize_linear(im, dw, dh, simd=True), oracle.resize_linear(im, dw, dh))
        assert np.array_equal(oracle.gaussian7(im, simd=True), oracle.gaussian7(im))
        for th in (7, 20, 0, 60):
            assert np.array_equal(oracle.fast(im, th, simd=True), oracle.fast(im, th)), (im.shape, th)
    for (w, h, nf) in ((640, 480, 1000), (1280, 720, 2000)):
        img = synth.make_frame(w, h, agent=1, frame=2)
        k1, d1, m1 = oracle.extract(img, oracle.params(nf))
        k2, d2, m2 = oracle.extract(img, oracle.params(nf), simd=True)
        assert np.array_equal(k1.view(np.uint8), k2.view(np.uint8)) and np.array_equal(d1, d2) and m1 == m2
