"""Frame sources and sinks for the reference-compatible drivers.

The reference reads with ``cv2.VideoCapture`` and writes ``mp4v`` with
``cv2.VideoWriter`` (``frame_differencing.py:39,63-65``;
``motion_compression_opt.py:39,50-52,121-122,135-136``). The codec is outside
the accelerated path. Here:

* ``*.npy`` clips (N x H x W x 3 uint8 BGR, memory-mapped) and
  ``synthetic://WxH?frames=N&seed=S&noisy=0|1&fps=F`` URIs are always readable;
* ``*.y4m`` (YUV4MPEG2, 4:2:0) videos are always readable: ``read()`` returns
  the BGR frame cv2.VideoCapture would (cvtColor YUV2BGR_I420, converted on
  the GPU by ``dvc_yuv420_to_bgr``), ``read_yuv()`` the raw 4:2:0 frame, which
  the FD driver hands to the GPU worker as is (in_format I420: the conversion
  runs in the worker's front stage, the decoded surface never round-trips);
* anything else goes through ``cv2.VideoCapture`` when OpenCV is importable;
* ``*.mp4`` outputs are written with ``cv2.VideoWriter(mp4v)`` when OpenCV is
  importable, otherwise as an ``.npy`` frame stream next to the requested name
  (same basename) so every output frame is still inspectable, or — with
  ``DVC_VIDEO_SINK=y4m`` or a ``.y4m`` name — as a YUV4MPEG2 video (colour
  frames 4:2:0 via ``dvc_bgr_to_i420`` on the GPU = cvtColor BGR2YUV_I420;
  single-channel frames as ``Cmono``) that any player or encoder reads.
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


class Y4mReader:
    """cv2.VideoCapture-like reader of a YUV4MPEG2 file with 4:2:0 chroma
    (C420jpeg / C420 / C420paldv / C420mpeg2 / no C tag). Frames are memory-mapped;
    ``pixel_format`` is "I420"."""

    pixel_format = "I420"

    def __init__(self, path: str, device: int = 0):
        self._mm, self._i, self.device = None, 0, int(device)
        try:
            with open(path, "rb") as f:
                head = f.readline(4096)
        except OSError:
            return
        tags = head.split()
        if not tags or tags[0] != b"YUV4MPEG2" or not head.endswith(b"\n"):
            return
        W = H = 0
        fps, chroma = 30.0, b"420jpeg"
        for t in tags[1:]:
            k, v = t[:1], t[1:]
            if k == b"W":
                W = int(v)
            elif k == b"H":
                H = int(v)
            elif k == b"F":
                num, den = v.split(b":")
                fps = int(num) / max(int(den), 1)
            elif k == b"C":
                chroma = v
        if W <= 0 or H <= 0 or W % 2 or H % 2 or not chroma.startswith(b"420"):
            return   # 4:4:4 / 4:2:2 / mono sources are not 4:2:0 surfaces
        self.W, self.H, self.fps = W, H, fps
        self._frame_bytes = W * H * 3 // 2
        raw = np.memmap(path, np.uint8, mode="r")
        off, frames = len(head), []
        while off < len(raw):   # FRAME[ params]\n + payload
            nl = off
            while nl < len(raw) and raw[nl] != 10:
                nl += 1
            if bytes(raw[off:off + 5]) != b"FRAME" or nl + 1 + self._frame_bytes > len(raw):
                break
            frames.append(nl + 1)
            off = nl + 1 + self._frame_bytes
        self._mm, self._offs = raw, frames

    def isOpened(self) -> bool:
        return self._mm is not None

    def get(self, prop: int) -> float:
        if self._mm is None:
            return 0.0
        return {CAP_PROP_FPS: self.fps, CAP_PROP_FRAME_WIDTH: float(self.W), CAP_PROP_FRAME_HEIGHT: float(self.H),
                CAP_PROP_FRAME_COUNT: float(len(self._offs))}.get(prop, 0.0)

    def read_yuv(self):
        """(ok, (H*3/2, W) uint8 I420 frame) — the decoder surface."""
        if self._mm is None or self._i >= len(self._offs):
            return False, None
        o = self._offs[self._i]
        self._i += 1
        return True, np.asarray(self._mm[o:o + self._frame_bytes]).reshape(self.H * 3 // 2, self.W)

    def read(self):
        """(ok, BGR frame) as cv2.VideoCapture.read() gives it (cvtColor on the GPU)."""
        ok, f = self.read_yuv()
        if not ok:
            return False, None
        from ._native import yuv420_to_bgr
        return True, yuv420_to_bgr(f, "I420", self.device)

    def release(self) -> None:
        self._mm = None


class Y4mWriter:
    """cv2.VideoWriter-like YUV4MPEG2 writer: colour frames (BGR) as 4:2:0
    (C420jpeg, cvtColor BGR2YUV_I420 on the GPU), single-channel frames as Cmono."""

    def __init__(self, path: str, fps: float, size, is_color: bool = True, device: int = 0):
        self.path, self.W, self.H = path, int(size[0]), int(size[1])
        self.is_color, self.device, self.n = is_color, int(device), 0
        num, den = (int(round(float(fps) * 1000)), 1000) if float(fps) != int(fps) else (int(fps), 1)
        self._fp = None
        if is_color and (self.W % 2 or self.H % 2):
            return   # 4:2:0 needs even sides (cv2.VideoWriter would fail to open as well)
        self._fp = open(path, "wb")
        self._fp.write(b"YUV4MPEG2 W%d H%d F%d:%d Ip A1:1 %s\n"
                       % (self.W, self.H, max(num, 1), den, b"C420jpeg" if is_color else b"Cmono"))

    def isOpened(self) -> bool:
        return self._fp is not None

    def write(self, frame: np.ndarray) -> None:
        if self._fp is None:
            return
        exp = (self.H, self.W, 3) if self.is_color else (self.H, self.W)
        if frame.shape != exp:   # cv2.VideoWriter silently drops mismatched frames
            return
        if self.is_color:
            from ._native import bgr_to_i420
            payload = bgr_to_i420(frame, self.device)
        else:
            payload = np.ascontiguousarray(frame, dtype=np.uint8)
        self._fp.write(b"FRAME\n")
        self._fp.write(payload.tobytes())
        self.n += 1

    def write_yuv(self, frame: np.ndarray) -> None:
        """A frame already in the stream's layout: (H*3/2, W) I420 for colour
        streams (e.g. the FD worker's DVC_FLAG_OUT_I420 outputs), (H, W) mono."""
        if self._fp is None:
            return
        exp = (self.H * 3 // 2, self.W) if self.is_color else (self.H, self.W)
        if frame.shape != exp:
            return
        self._fp.write(b"FRAME\n")
        self._fp.write(np.ascontiguousarray(frame, dtype=np.uint8).tobytes())
        self.n += 1

    def release(self) -> None:
        if self._fp is not None:
            self._fp.close()
            self._fp = None


def video_name(path: str) -> str:
    """<basename without extension> (fd:45, fd:177); a synthetic URI is named WxH."""
    if path.startswith("synthetic://"):
        return urlparse(path).netloc
    return os.path.splitext(os.path.basename(path))[0]


def open_source(path: str):
    """cv2.VideoCapture-like object for ``path`` (isOpened/get/read/release)."""
    if path.endswith(".y4m"):
        return Y4mReader(path, int(os.environ.get("DVC_DEVICE", os.environ.get("LOCAL_RANK", 0))))
    if path.startswith("synthetic://"):
        from .synthetic import SyntheticClip
        u = urlparse(path)
        w, h = (int(v) for v in u.netloc.lower().split("x"))
        q = {k: v[0] for k, v in parse_qs(u.query).items()}
        clip = SyntheticClip(w, h, seed=int(q.get("seed", 0)), noisy=q.get("noisy", "0") in ("1", "true"))
        return _ArraySource(_SyntheticFrames(clip, int(q.get("frames", 100))), float(q.get("fps", 30)))
    if not path.endswith(".npy") and cv2 is None:
        # an .mp4 this package wrote without OpenCV is the .npy / .y4m stream next to it
        for ext in (".npy", ".y4m"):
            alt = os.path.splitext(path)[0] + ext
            if os.path.exists(alt):
                return open_source(alt)
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
    root, ext = os.path.splitext(path)
    if ext == ".y4m" or (ext != ".npy" and cv2 is None and os.environ.get("DVC_VIDEO_SINK", "npy") == "y4m"):
        dev = int(os.environ.get("DVC_DEVICE", os.environ.get("LOCAL_RANK", 0)))
        return Y4mWriter(root + ".y4m", fps, size, is_color, dev)
    if cv2 is not None and ext != ".npy":
        fourcc = cv2.VideoWriter_fourcc(*"mp4v")
        return cv2.VideoWriter(path, fourcc, fps, tuple(size), isColor=is_color)
    return NpyStreamWriter(root + ".npy" if ext != ".npy" else path, fps, size, is_color)
