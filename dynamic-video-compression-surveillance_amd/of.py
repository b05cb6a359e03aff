"""One camera feed on one GPU: the per-frame worker of the optical-flow path.

``OFWorker`` owns a ``dvc_of`` handle (include/dvc.h) and replaces the bodies
of the two reference loops of ``motion_compression_opt.py`` fused per frame:
``temporal_smoothing_flow`` (``of:65-101``: gray, Farneback, |flow| > thr, the
30-frame vote, close/open, rectangles) and ``compress_with_motion``
(``of:141-185``: static 8x8 blocks DCT-quantised on Y, Cr, Cb, then grey).
``prime`` is the first-frame setup (``of:54-62``), ``step`` one frame.

Frames are H x W x 3 uint8 BGR: numpy arrays in host mode; device buffers
(torch tensors or raw addresses) with ``device_ptrs=True`` (asynchronous).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _buffers as B
from . import _native as N


def derive_of_params(width: int, height: int, flow_threshold: float = 0.5, alpha_fraction: float = 0.2,
                     window_size: int = 30, morph_kernel: int = 2, quantization_level: float = 100.0,
                     flags: int = 0, direct_sums: bool = False, in_format: str = "BGR",
                     chroma_rows: int = 0) -> N.OfParams:
    """dvc_of_params from the reference kwargs of ``temporal_smoothing_flow``
    (of:29-31) and the arguments it hard-codes: Farneback (0.3, 2, 9, 2, 5, 1.1,
    0) at of:72-81, ``QTY_aggressive`` = 100 at of:138. ``direct_sums``: direct
    per-pixel box sums instead of OpenCV's running sums (the default)."""
    p = N.OfParams()
    if direct_sums:
        flags |= N.DVC_FLAG_OF_DIRECT_SUMS
    p.width, p.height = int(width), int(height)
    p.flow_threshold = float(flow_threshold)
    p.quant = float(quantization_level)
    p.alpha_fraction = float(alpha_fraction)
    p.window = int(window_size)
    p.morph_kernel = int(morph_kernel)
    p.pyr_scale, p.levels, p.winsize, p.iterations, p.poly_n, p.poly_sigma = 0.3, 2, 9, 2, 5, 1.1
    p.flags = flags
    p.in_format = N.FORMATS[in_format]
    p.chroma_rows = int(chroma_rows)
    return p


class OFWorker:
    def __init__(self, width: int, height: int, *, device: int = 0, stream=None, device_ptrs: bool = False,
                 keep_planes: bool = False, ktiming: bool = False, max_batch: int = 1, **kwargs):
        flags = (N.DVC_FLAG_DEVICE_PTRS if device_ptrs else 0) | (N.DVC_FLAG_KEEP_PLANES if keep_planes else 0) \
            | (N.DVC_FLAG_KTIMING if ktiming else 0) | (N.DVC_FLAG_JOIN_STREAM if stream is not None else 0)
        self.params = derive_of_params(width, height, flags=flags, **kwargs)
        self.params.max_batch = int(max_batch)
        self.W, self.H = int(width), int(height)
        self.in_format = kwargs.get("in_format", "BGR")
        self.device = int(device)
        self.device_ptrs = device_ptrs
        self._lib = N.lib()
        h = ctypes.c_void_p()
        s = ctypes.c_void_p(int(stream)) if stream is not None else None
        N.check(self._lib.dvc_of_create(ctypes.byref(self.params), self.device, s, ctypes.byref(h)))
        self._h = h

    @property
    def _fshape(self):
        """Input frames: packed BGR, or a (H*3/2, W) 4:2:0 frame."""
        return (self.H, self.W, 3) if self.in_format == "BGR" else (self.H * 3 // 2, self.W)

    @property
    def _oshape(self):
        return (self.H, self.W, 3)

    @property
    def _pitch(self):
        return 3 * self.W if self.in_format == "BGR" else self.W

    def _dev(self, x, name, tail, n=None, batched=False) -> int:
        return B.device_buf(x, tail, self.device, name, n=n, batched=batched)

    def prime(self, frame) -> None:
        """of:54-62: previous gray := gray(frame 0); the vote window is emptied."""
        if self.device_ptrs:
            N.check(self._lib.dvc_of_prime(self._h, self._dev(frame, "frame", self._fshape)[0], self._pitch))
        else:
            f = B.host_in(frame, self._fshape, "frame")
            N.check(self._lib.dvc_of_prime(self._h, f.ctypes.data, self._pitch))

    def set_state(self, prev_gray, raw_masks) -> None:
        """Resume instead of :meth:`prime` (dvc_of_set_state): the previous gray
        (H x W, of:101) and the raw |flow| masks of the last frames, oldest
        first ((n, H, W), of:84) — :meth:`plane` with OF_PLANE_GRAY / _RAW
        exports them."""
        g = np.ascontiguousarray(prev_gray, dtype=np.uint8)
        m = np.ascontiguousarray(raw_masks, dtype=np.uint8)
        if m.ndim == 2:
            m = m[None]
        if g.shape != (self.H, self.W) or m.shape[1:] != (self.H, self.W):
            raise ValueError(f"state planes must be ({self.H}, {self.W})")
        N.check(self._lib.dvc_of_set_state(self._h, g.ctypes.data, m.ctypes.data if len(m) else None, len(m)))

    def step(self, frame, mask=None, compressed=None, want=("mask", "compressed")):
        """of:70-101 + of:151-183 for one frame. Host mode returns ``(mask,
        compressed)`` (H x W {0,255} and H x W x 3); device mode writes into the
        given buffers and returns None."""
        if self.device_ptrs:
            addr = self._dev(frame, "frame", self._fshape)[0]
            mk = self._dev(mask, "mask", (self.H, self.W))[0] if mask is not None else None
            cp = self._dev(compressed, "compressed", self._oshape)[0] if compressed is not None else None
            N.check(self._lib.dvc_of_step(self._h, addr, self._pitch, mk, cp))
            return None
        f = B.host_in(frame, self._fshape, "frame")
        mask = B.host_out(mask, (self.H, self.W), "mask", "mask" in want)
        compressed = B.host_out(compressed, self._oshape, "compressed", "compressed" in want)
        N.check(self._lib.dvc_of_step(self._h, f.ctypes.data, self._pitch,
                                      mask.ctypes.data if mask is not None else None,
                                      compressed.ctypes.data if compressed is not None else None))
        return mask, compressed

    def step_batch(self, frames, mask=None, compressed=None, want=("mask", "compressed")):
        """n consecutive frames (identical to n :meth:`step` calls). Host mode:
        (n, H, W, 3) uint8 in, ``(masks, compressed)`` out. Device mode: CUDA
        tensors on the handle's device or explicit ``(address, n)`` tuples;
        asynchronous, returns None."""
        fs, ms, os_ = int(np.prod(self._fshape)), self.W * self.H, 3 * self.W * self.H
        if self.device_ptrs:
            addr, n = self._dev(frames, "frames", self._fshape, batched=True)
            mk = self._dev(mask, "mask", (self.H, self.W), n=n, batched=True)[0] if mask is not None else None
            cp = self._dev(compressed, "compressed", self._oshape, n=n, batched=True)[0] \
                if compressed is not None else None
            N.check(self._lib.dvc_of_step_batch(self._h, addr, self._pitch, fs, n, mk, ms, cp, os_))
            return None
        if not isinstance(frames, np.ndarray) or frames.ndim != len(self._fshape) + 1:
            raise ValueError(f"frames: expected uint8 frames of shape (n, {', '.join(map(str, self._fshape))})")
        n = int(frames.shape[0])
        f = B.host_in(frames, (n,) + self._fshape, "frames")
        mask = B.host_out(mask, (n, self.H, self.W), "mask", "mask" in want)
        compressed = B.host_out(compressed, (n,) + self._oshape, "compressed", "compressed" in want)
        N.check(self._lib.dvc_of_step_batch(self._h, f.ctypes.data, self._pitch, fs, n,
                                            mask.ctypes.data if mask is not None else None, ms,
                                            compressed.ctypes.data if compressed is not None else None, os_))
        return mask, compressed

    def sync(self) -> None:
        N.check(self._lib.dvc_of_sync(self._h))

    def stats(self) -> dict:
        s = N.OfStats()
        N.check(self._lib.dvc_of_get_stats(self._h, ctypes.byref(s)))
        return {k: int(getattr(s, k)) for k, _ in N.OfStats._fields_}

    def plane(self, which: int) -> np.ndarray:
        """N.OF_PLANE_*: raw |flow| mask, vote-smoothed, close/open, rectangles, gray."""
        out = np.empty((self.H, self.W), np.uint8)
        N.check(self._lib.dvc_of_read_plane(self._h, int(which), out.ctypes.data))
        return out

    def flow(self) -> np.ndarray:
        """Farneback flow (H x W x 2 float32) of the last frame (needs keep_planes)."""
        out = np.empty((self.H, self.W, 2), np.float32)
        N.check(self._lib.dvc_of_read_flow(self._h, out.ctypes.data))
        return out

    def debug_read(self, what: int, level: int = 0) -> np.ndarray:
        """Farneback intermediates of the last frame at a pyramid level: 0 its
        polynomial expansion R (h, w, 5), 1 the previous frame's R, 2 the flow
        after the first iteration (h, w, 2)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        N.check(self._lib.dvc_of_debug_read(self._h, what, level, None, ctypes.byref(w), ctypes.byref(h)))
        out = np.empty((h.value, w.value, 5 if what in (0, 1) else 2), np.float32)
        N.check(self._lib.dvc_of_debug_read(self._h, what, level, out.ctypes.data, None, None))
        return out

    def ktime(self, reset: bool = False):
        """(total ms, launches) of the finest-level Farneback iterations, hipEvent-timed."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        N.check(self._lib.dvc_of_ktime(self._h, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0))
        return float(ms.value), int(n.value)

    def ktime_kernel(self) -> str:
        """The kernel that ran the level-0 iterations of the last batch (what
        :meth:`ktime` timed): "k_flow" (direct sums), "k_flow_scan" (the
        barrier-phased running-sum scan) or "k_flow_scan2" (the pipelined scan)."""
        if not hasattr(self._lib, "dvc_of_ktime_kernel"):   # an older build (DVC_LIB_PATH A/B)
            return "k_flow_scan2"
        k = self._lib.dvc_of_ktime_kernel(self._h)
        if k < 0:
            N.check(k)
        return {N.KTIME_FLOW: "k_flow", N.KTIME_FLOW_SCAN: "k_flow_scan", N.KTIME_FLOW_SCAN2: "k_flow_scan2"}[k]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.dvc_of_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
