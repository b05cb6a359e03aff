"""Frame sources and sinks for the reference-compatible drivers.

The reference reads with ``cv2.VideoCapture`` and writes ``mp4v`` with
``cv2.VideoWriter`` (``frame_differencing.py:39,63-65``;
``motion_compression_opt.py:39,50-52,121-122,135-136``). The codec is outside
the accelerated path. Here:

* ``*.npy`` clips (N x H x W x 3 uint8 BGR, memory-mapped) and
  ``synthetic://WxH?frames=N&seed=S&noisy=0|1&fps=F`` URIs are always readable;
* anything else goes through ``cv2.VideoCapture`` when OpenCV is importable;
* ``*.mp4`` outputs are written with ``cv2.VideoWriter(mp4v)`` when OpenCV is
  importable, otherwise as an ``.npy`` frame stream next to the requested name
  (same basename) so every output frame is still inspectable.
"""
from __future__ import annotations

import json
import os
import struct
from urllib.parse import parse_qs, urlparse

import numpy as np

try:  # optional: only used for real video files
    import cv2  # type: ignore
except Exception:  # pragma: no cover - cv2 is absent in this image
    cv2 = None

CAP_PROP_FPS = 5
CAP_PROP_FRAME_WIDTH = 3
CAP_PROP_FRAME_HEIGHT = 4
CAP_PROP_FRAME_COUNT = 7


class _ArraySource:
    def __init__(self, frames, fps: float):
        self._f = frames
        self._fps = float(fps)
        self._i = 0

    def isOpened(self) -> bool:
        return self._f is not None

    def get(self, prop: int) -> float:
        if prop == CAP_PROP_FPS:
            return self._fps
        if prop == CAP_PROP_FRAME_WIDTH:
            return float(self._f.shape[2])
        if prop == CAP_PROP_FRAME_HEIGHT:
            return float(self._f.shape[1])
        if prop == CAP_PROP_FRAME_COUNT:
            return float(len(self._f))
        return 0.0

    def read(self):
        if self._f is None or self._i >= len(self._f):
            return False, None
        fr = np.ascontiguousarray(self._f[self._i])
        self._i += 1
        return True, fr

    def release(self) -> None:
        self._f = None


class _SyntheticFrames:
    """Lazy sequence view over a SyntheticClip (frames generated on read)."""

    def __init__(self, clip, n):
        self._clip, self._n = clip, int(n)
        self.shape = (self._n, clip.H, clip.W, 3)

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        return self._clip.frame(int(i))


def video_name(path: str) -> str:
    """<basename without extension> (fd:45, fd:177); a synthetic URI is named WxH."""
    if path.startswith("synthetic://"):
        return urlparse(path).netloc
    return os.path.splitext(os.path.basename(path))[0]


def open_source(path: str):
    """cv2.VideoCapture-like object for ``path`` (isOpened/get/read/release)."""
    if path.startswith("synthetic://"):
        from .synthetic import SyntheticClip
        u = urlparse(path)
        w, h = (int(v) for v in u.netloc.lower().split("x"))
        q = {k: v[0] for k, v in parse_qs(u.query).items()}
        clip = SyntheticClip(w, h, seed=int(q.get("seed", 0)), noisy=q.get("noisy", "0") in ("1", "true"))
        return _ArraySource(_SyntheticFrames(clip, int(q.get("frames", 100))), float(q.get("fps", 30)))
    if not path.endswith(".npy") and cv2 is None:
        # an .mp4 this package wrote without OpenCV is the .npy stream next to it
        alt = os.path.splitext(path)[0] + ".npy"
        if os.path.exists(alt):
            path = alt
    if path.endswith(".npy"):
        if not os.path.exists(path):
            return _ArraySource(None, 0)
        arr = np.load(path, mmap_mode="r")
        fps = 30.0
        meta = os.path.splitext(path)[0] + ".json"
        if os.path.exists(meta):
            with open(meta) as f:
                fps = float(json.load(f).get("fps", fps))
        # N x H x W x 3 BGR frames, or N x H x W single-channel frames (mask videos)
        if arr.dtype != np.uint8 or not (arr.ndim == 3 or (arr.ndim == 4 and arr.shape[3] == 3)):
            return _ArraySource(None, 0)
        return _ArraySource(arr, fps)
    if cv2 is not None:
        return cv2.VideoCapture(path)
    return _ArraySource(None, 0)


class NpyStreamWriter:
    """Append frames to an .npy file whose header is rewritten on release."""

    _HDR = 256

    def __init__(self, path: str, fps: float, size, is_color: bool = True):
        self.path = path
        self.fps = float(fps)
        self.W, self.H = int(size[0]), int(size[1])
        self.is_color = is_color
        self.n = 0
        self._fp = open(path, "wb")
        self._write_header()
        with open(os.path.splitext(path)[0] + ".json", "w") as f:
            json.dump({"fps": self.fps, "width": self.W, "height": self.H}, f)

    def _write_header(self):
        shape = (self.n, self.H, self.W, 3) if self.is_color else (self.n, self.H, self.W)
        d = "{'descr': '|u1', 'fortran_order': False, 'shape': %r, }" % (shape,)
        pad = self._HDR - 10 - len(d) - 1
        hdr = b"\x93NUMPY\x01\x00" + struct.pack("<H", self._HDR - 10) + d.encode() + b" " * pad + b"\n"
        self._fp.seek(0)
        self._fp.write(hdr)
        self._fp.seek(0, 2)

    def isOpened(self) -> bool:
        return self._fp is not None

    def write(self, frame: np.ndarray) -> None:
        exp = (self.H, self.W, 3) if self.is_color else (self.H, self.W)
        if frame.shape != exp:  # cv2.VideoWriter silently drops mismatched frames
            return
        self._fp.write(np.ascontiguousarray(frame, dtype=np.uint8).tobytes())
        self.n += 1

    def release(self) -> None:
        if self._fp is not None:
            self._write_header()
            self._fp.close()
            self._fp = None


def open_sink(path: str, fps: float, size, is_color: bool = True):
    """cv2.VideoWriter(path, mp4v, fps, size)-like object."""
    if cv2 is not None and not path.endswith(".npy"):
        fourcc = cv2.VideoWriter_fourcc(*"mp4v")
        return cv2.VideoWriter(path, fourcc, fps, tuple(size), isColor=is_color)
    root, ext = os.path.splitext(path)
    return NpyStreamWriter(root + ".npy" if ext != ".npy" else path, fps, size, is_color)
