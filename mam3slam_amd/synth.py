"""Deterministic synthetic mono frames (SURVEY.md §8(d) "Synthetic inputs").

There is no dataset in this environment: every benchmark and parity case runs on seeded textured
frames. Scene = random axis-aligned and rotated rectangles (grey levels U[20,235]) plus Gaussian-smoothed
noise, clamped to u8. Frame k of agent a is a crop of a larger canvas translated 2 px/frame with a
0.2 deg/frame roll, so consecutive frames share structure (useful for matching).

seed = 0x4D414D33 ^ (agent << 16) ^ frame  (the survey's convention).
"""
from __future__ import annotations

import functools

import numpy as np

_SEED_BASE = 0x4D414D33


def frame_seed(agent: int, frame: int) -> int:
    return (_SEED_BASE ^ (agent << 16) ^ frame) & 0xFFFFFFFF


def _smooth_noise(rng: np.random.Generator, h: int, w: int, sigma: float = 8.0) -> np.ndarray:
    from scipy.ndimage import gaussian_filter

    n = rng.normal(0.0, 1.0, size=(h, w)).astype(np.float32)
    n = gaussian_filter(n, 1.2)
    n *= sigma / max(float(n.std()), 1e-6)
    return n


@functools.lru_cache(maxsize=16)
def make_canvas(h: int, w: int, seed: int, n_rects: int | None = None) -> np.ndarray:
    """A textured float32 canvas of size h x w (cached; treat as read-only)."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w), float(rng.uniform(60, 190)), np.float32)
    if n_rects is None:
        n_rects = max(40, (h * w) // 2500)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    for _ in range(n_rects):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        rw, rh = rng.uniform(6, max(8, w / 8)), rng.uniform(6, max(8, h / 8))
        val = float(rng.uniform(20, 235))
        if rng.random() < 0.5:
            x0, x1 = int(cx - rw / 2), int(cx + rw / 2)
            y0, y1 = int(cy - rh / 2), int(cy + rh / 2)
            img[max(0, y0):max(0, y1), max(0, x0):max(0, x1)] = val
        else:
            th = rng.uniform(0, np.pi)
            c, s = np.cos(th), np.sin(th)
            x0, x1 = int(max(0, cx - rw - rh)), int(min(w, cx + rw + rh + 1))
            y0, y1 = int(max(0, cy - rw - rh)), int(min(h, cy + rw + rh + 1))
            if x1 <= x0 or y1 <= y0:
                continue
            dx = xx[y0:y1, x0:x1] - cx
            dy = yy[y0:y1, x0:x1] - cy
            u = dx * c + dy * s
            v = -dx * s + dy * c
            m = (np.abs(u) < rw / 2) & (np.abs(v) < rh / 2)
            img[y0:y1, x0:x1][m] = val
    img += _smooth_noise(rng, h, w)
    return img


# The camera path: `px` canvas pixels of translation and `deg` degrees of roll per frame index, over a canvas `extent`
# pixels wider than the view (frames up to extent / px). The default is the survey's 2 px / 0.2 deg per frame; a
# longer path (BASELINE configs[2]'s LocalMapping: keyframes far enough apart that the farther ones no longer share
# MapPoints, as a camera moving through a scene leaves them) uses a wider canvas.
DEFAULT_MOTION = (2.0, 0.2, 4 * 256)


def make_frame(w: int, h: int, agent: int = 0, frame: int = 0, motion: bool = True, path=None) -> np.ndarray:
    """u8 h x w frame; consecutive `frame` indices of one agent view one moving scene (path = (px, deg, extent) per
    frame, default DEFAULT_MOTION)."""
    px, deg, extent = path or DEFAULT_MOTION
    canvas_seed = frame_seed(agent, 0)
    margin = 64
    ch, cw = h + 2 * margin, w + 2 * margin + int(extent)
    canvas = make_canvas(ch, cw, canvas_seed)
    tx = px * frame if motion else 0.0
    ang = deg * frame if motion else 0.0
    if int(tx) > int(extent):
        raise ValueError(f"frame {frame} leaves the canvas (path {path})")
    if ang != 0.0:
        from scipy.ndimage import rotate

        sub = canvas[:, int(tx): int(tx) + w + 2 * margin]
        sub = rotate(sub, ang, reshape=False, order=1, mode="reflect")
        out = sub[margin:margin + h, margin:margin + w]
    else:
        out = canvas[margin:margin + h, margin + int(tx): margin + int(tx) + w]
    # per-frame sensor noise keeps frames distinct even without motion
    rng = np.random.default_rng(frame_seed(agent, frame) ^ 0x5A5A)
    out = out + rng.normal(0.0, 1.5, size=out.shape).astype(np.float32)
    return np.ascontiguousarray(np.clip(np.rint(out), 0, 255).astype(np.uint8))


# The camera that renders make_frame's images of the canvas, as a 3-D scene: the canvas is the plane z = PLANE_DEPTH in
# front of a Pinhole camera (fx = fy = f, principal point (w/2, h/2): scene.pinhole) that translates along x and rolls
# about its optical axis. make_frame maps canvas pixel P to image pixel p = R_k (P - o_k - c) + c with the crop offset
# o_k = (2k + margin, margin), c = ((w - 1)/2, (h - 1)/2) (scipy's rotation centre) and R_k = [[cos a, sin a],
# [-sin a, cos a]], a = 0.2 k degrees (scipy.ndimage.rotate turns the content counter-clockwise on screen). With the
# world point of canvas pixel P at ((P - o_0 - c) Z / f, Z), camera k = (R_k about z, t = (Z / f)(R_k (o_0 - o_k) + c -
# (w/2, h/2), 0)) projects it onto p exactly.
PLANE_DEPTH = 5.0


def frame_pose(w: int, h: int, frame: int, f: float = 500.0, depth: float = PLANE_DEPTH, motion: bool = True,
               path=None):
    """Tcw (q xyzw float32, t float32) of the camera that rendered make_frame(w, h, agent, frame, path=path) (any
    agent)."""
    px, deg, _ = path or DEFAULT_MOTION
    k = frame if motion else 0
    a = np.deg2rad(deg * k)
    ca, sa = np.cos(a), np.sin(a)
    R2 = np.array([[ca, sa], [-sa, ca]])
    d = np.array([-float(int(px * k)), 0.0])   # o_0 - o_k
    txy = depth / f * (R2 @ d + np.array([(w - 1) / 2.0 - w / 2.0, (h - 1) / 2.0 - h / 2.0]))
    # R = [[R2, 0], [0, 1]]: quaternion of a rotation about z by angle -a (R2 is that rotation in x-right, y-down axes)
    q = np.array([0.0, 0.0, np.sin(-a / 2.0), np.cos(-a / 2.0)])
    return q.astype(np.float32), np.array([txy[0], txy[1], 0.0], np.float32)


_RAYS = {}


def _camera_rays(w: int, h: int, cam, ss: int):
    """(x / z, y / z) of the ss x ss sub-pixel sample points of every pixel (pose-independent: cached per camera)."""
    key = (w, h, ss, tuple(cam.params().tolist()))
    if key not in _RAYS:
        rays = []
        for sy in range(ss):
            for sx in range(ss):
                yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
                r = cam.unproject_np(xx + (sx + 0.5) / ss - 0.5, yy + (sy + 0.5) / ss - 0.5)
                rays.append((r[..., 0].copy(), r[..., 1].copy()))
        _RAYS[key] = rays
    return _RAYS[key]


def make_frame_camera(w: int, h: int, cam, agent: int = 0, frame: int = 0, f: float = 500.0,
                      depth: float = PLANE_DEPTH, motion: bool = True, ss: int = 3, path=None) -> np.ndarray:
    """make_frame's scene seen through camera `cam` (a match.KannalaBrandt8 — the testMultiAgentSystem agents' fisheye —
    or a Pinhole) from the same pose, frame_pose(w, h, frame): every sample ray (cam.unproject_np) meets the canvas
    plane z = depth (the camera rolls about z and translates in x / y, so the plane is at camera depth `depth` too),
    where the canvas is sampled bilinearly (mirrored beyond its border); a pixel is the mean of ss x ss samples (the
    fisheye sees the canvas minified ~2.3x: point samples would alias, and a keypoint's descriptor would change with
    its sub-pixel phase from view to view). Keyframes of these frames see the scene through the camera they are
    tracked with, so SearchForTriangulation's camera-specific epipolar test (KannalaBrandt8::epipolarConstrain:
    two-view triangulation + reprojection) passes for true correspondences. The u8 quantisation and sensor noise are
    make_frame's."""
    from scipy.ndimage import map_coordinates

    canvas_seed = frame_seed(agent, 0)
    margin = 64
    ch, cw = h + 2 * margin, w + 2 * margin + int((path or DEFAULT_MOTION)[2])
    canvas = make_canvas(ch, cw, canvas_seed)
    q, t = frame_pose(w, h, frame, f, depth, motion, path=path)
    a = -2.0 * np.arctan2(float(q[2]), float(q[3]))             # roll of frame_pose's quaternion (about z by -a)
    ca, sa = np.cos(a), np.sin(a)
    acc = np.zeros((h, w), np.float64)
    for rx, ry in _camera_rays(w, h, cam, ss):
        dx, dy = rx * depth - float(t[0]), ry * depth - float(t[1])   # R^T (Xc - t), R = [[ca, sa], [-sa, ca]]
        xw, yw = ca * dx - sa * dy, sa * dx + ca * dy
        px = xw * f / depth + margin + (w - 1) / 2.0            # canvas pixel of the world point (frame_pose's model)
        py = yw * f / depth + margin + (h - 1) / 2.0
        acc += map_coordinates(canvas, [py, px], order=1, mode="mirror")
    out = (acc / (ss * ss)).astype(np.float32)
    rng = np.random.default_rng(frame_seed(agent, frame) ^ 0x5A5A)
    out = out + rng.normal(0.0, 1.5, size=out.shape).astype(np.float32)
    return np.ascontiguousarray(np.clip(np.rint(out), 0, 255).astype(np.uint8))


def canvas_point(w: int, h: int, frame: int, px: np.ndarray, py: np.ndarray, motion: bool = True):
    """Canvas pixel coordinates of image pixels (px, py) of make_frame(w, h, agent, frame) (the inverse warp)."""
    k = frame if motion else 0
    a = np.deg2rad(0.2 * k)
    ca, sa = np.cos(a), np.sin(a)
    cx, cy = (w - 1) / 2.0, (h - 1) / 2.0
    dx, dy = np.asarray(px, np.float64) - cx, np.asarray(py, np.float64) - cy
    margin = 64
    # R^-1 = R^T = [[cos, -sin], [sin, cos]]
    return ca * dx - sa * dy + cx + int(2.0 * k) + margin, sa * dx + ca * dy + cy + margin


def make_batch(w: int, h: int, n: int, agent: int = 0, start: int = 0) -> np.ndarray:
    return np.stack([make_frame(w, h, agent, start + i) for i in range(n)])
