"""Settings — Python mirror of MAM3SLAM::Settings (include/mam3slam/Settings.h): the reference's settings keys for the
extractor and camera 1 read from its OpenCV FileStorage YAML (src/Settings.cc:184-270 readCamera1, :443-451 readORB;
src/Agent.cc:22-29 File.version "1.0"). Reals are read as double and narrowed to float (readParameter<float>).
"""
from __future__ import annotations

import numpy as np

from .match import Camera, KannalaBrandt8, Pinhole


class Settings:
    def __init__(self, path: str):
        self.values: dict[str, str] = {}
        with open(path) as f:
            for n, line in enumerate(f):
                if n == 0 and line.strip().startswith("%YAML"):
                    continue
                q, cut = False, len(line)
                for i, ch in enumerate(line):
                    if ch == '"':
                        q = not q
                    elif ch == "#" and not q:
                        cut = i
                        break
                t = line[:cut].strip()
                if not t or t == "---" or ":" not in t:
                    continue
                k, v = t.split(":", 1)
                v = v.strip()
                if len(v) >= 2 and v[0] == '"' and v[-1] == '"':
                    v = v[1:-1]
                if k.strip():
                    self.values[k.strip()] = v
        if self.values.get("File.version") != "1.0":
            raise ValueError(f"{path}: not a File.version \"1.0\" settings file")
        model = self._str("Camera.type")
        f = self._float
        self.distortion: list = []
        if model in ("PinHole", "Rectified"):
            self.camera_type = model
            self.camera: Camera = Pinhole(f("Camera1.fx"), f("Camera1.fy"), f("Camera1.cx"), f("Camera1.cy"))
            if model == "PinHole" and "Camera1.k1" in self.values:
                self.distortion = [f("Camera1.k1"), f("Camera1.k2"), f("Camera1.p1"), f("Camera1.p2")]
                if "Camera1.k3" in self.values:
                    self.distortion.append(f("Camera1.k3"))
        elif model == "KannalaBrandt8":
            self.camera_type = model
            self.camera = KannalaBrandt8(f("Camera1.fx"), f("Camera1.fy"), f("Camera1.cx"), f("Camera1.cy"),
                                         f("Camera1.k1"), f("Camera1.k2"), f("Camera1.k3"), f("Camera1.k4"))
        else:
            raise ValueError(f"{path}: unknown Camera.type {model}")
        self.width, self.height, self.fps = self._int("Camera.width"), self._int("Camera.height"), \
            float(self._int("Camera.fps"))   # readParameter<int> (Settings.cc:410) into a float member
        self.n_features = self._int("ORBextractor.nFeatures")
        self.scale_factor = f("ORBextractor.scaleFactor")
        self.n_levels = self._int("ORBextractor.nLevels")
        self.ini_th_fast = self._int("ORBextractor.iniThFAST")
        self.min_th_fast = self._int("ORBextractor.minThFAST")

    def _str(self, k):
        if k not in self.values:
            raise KeyError(f"missing required parameter {k}")
        return self.values[k]

    def _float(self, k) -> float:
        return float(np.float32(float(self._str(k))))

    def _int(self, k) -> int:
        return int(self._str(k))

    def orb_args(self):
        """ORBextractor(nFeatures, scaleFactor, nLevels, iniThFAST, minThFAST) (Tracking.cc:600-606)."""
        return self.n_features, self.scale_factor, self.n_levels, self.ini_th_fast, self.min_th_fast

    def camera_scaled(self, w: int, h: int) -> Camera:
        """Camera 1 for w x h images: fx, cx scaled by w / Camera.width, fy, cy by h / Camera.height (the distortion
        acts on the ray angle and is unchanged) — the test YAML's 960 x 960 fisheye at the bench's image size."""
        d = lambda k: float(self._str(k))   # noqa: E731  (the YAML's value, double)
        sx, sy = w / self.width, h / self.height
        fx, fy, cx, cy = (np.float32(d("Camera1.fx") * sx), np.float32(d("Camera1.fy") * sy),
                          np.float32(d("Camera1.cx") * sx), np.float32(d("Camera1.cy") * sy))
        if self.camera.is_kb8:
            return KannalaBrandt8(fx, fy, cx, cy, *[np.float32(d(f"Camera1.k{i}")) for i in range(1, 5)])
        return Pinhole(fx, fy, cx, cy)
