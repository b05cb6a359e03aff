"""One camera feed on one GPU: the per-frame worker of the FD path.

``FDWorker`` owns a ``dvc_fd`` handle (include/dvc.h) and replaces the body of
the reference loop ``frame_differencing.py:85-138``: ``prime`` is the frame-0
preprocessing (``fd:67-81``), ``step`` one iteration (``fd:91-133``).

Frames are H x W x 3 uint8 BGR. In host mode they are numpy arrays; in device
mode (``device_ptrs=True``) they are device buffers — torch tensors on the
handle's device, or raw integer addresses — and ``step`` is asynchronous.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from . import _buffers as B
from . import _native as N


def derive_params(width: int, height: int, block_size: int = 4, motion_threshold: float = 0.5,
                  min_area: float = 500, kernel_size: int = 7, release_factor: float = 0.5,
                  quantization_level: float = 100, flags: int = 0, src_width: int = 0,
                  src_height: int = 0, in_format: str = "BGR", chroma_rows: int = 0) -> N.FdParams:
    """dvc_fd_params from the reference kwargs (frame_differencing.py:21-30).

    * ``ithresh = floor(motion_threshold)`` clamped to [-1, 255]: cv::threshold
      floors the threshold for 8U input (fd:97).
    * ``min_area2 = floor(2*min_area)``: ``contourArea > min_area`` is exactly
      ``2*area > floor(2*min_area)`` for the half-integer polygon areas (fd:103).
    * addWeighted receives (release_factor, 1 - release_factor, 0) as doubles and
      computes in float32 (fd:107).
    """
    p = N.FdParams()
    p.width, p.height = int(width), int(height)
    p.block = int(block_size)
    p.ithresh = max(-1, min(255, math.floor(motion_threshold)))
    p.min_area2 = math.floor(2.0 * float(min_area))
    p.ksize = int(kernel_size)
    p.anchor = int(kernel_size) // 2
    p.alpha = float(release_factor)
    p.beta = float(1 - release_factor)
    p.gamma = 0.0
    p.quant = float(quantization_level)
    p.prime_ksize = 25   # fd:77
    p.prime_sigma = 30.0
    p.flags = flags
    p.src_width, p.src_height = int(src_width or 0), int(src_height or 0)
    p.in_format = N.FORMATS[in_format]
    p.chroma_rows = int(chroma_rows)
    return p


class FDWorker:
    def __init__(self, width: int, height: int, *, device: int = 0, stream=None,
                 device_ptrs: bool = False, keep_planes: bool = False, ktiming: bool = False,
                 max_batch: int = 1, out_format: str = "BGR", fused: bool = True, **kwargs):
        """``width, height``: the scaled frame size (fd:60-61); frames handed to
        :meth:`prime`/:meth:`step` are ``src_width x src_height`` (the video's,
        default the same) and are resized on the GPU (fd:74,91).
        ``max_batch``: frames one device launch covers in :meth:`step_batch`
        (bit planes for NSLOT = 3 batches of max_batch frames in flight, the
        contour filter's working arrays for one, fd_api.hip). ``stream``: the
        caller's HIP stream (``torch.cuda.Stream.cuda_stream``), joined as
        dvc_fd_create documents. ``in_format`` (kwarg) "BGR" / "I420" / "NV12":
        the frames handed over (4:2:0 decoder surfaces are converted on the GPU);
        ``out_format`` "BGR" or "I420": overlay and compressed frames as the
        encoder's 4:2:0 input (DVC_FLAG_OUT_I420). ``fused=False``: outputs in
        one k_out pass instead of the fused front's speculative static-block
        outputs + k_fix (DVC_FLAG_FD_UNFUSED; same bytes)."""
        if out_format not in ("BGR", "I420"):
            raise ValueError(f"out_format {out_format!r}: BGR or I420")
        flags = (N.DVC_FLAG_DEVICE_PTRS if device_ptrs else 0) | (N.DVC_FLAG_KEEP_PLANES if keep_planes else 0) \
            | (N.DVC_FLAG_KTIMING if ktiming else 0) | (N.DVC_FLAG_JOIN_STREAM if stream is not None else 0) \
            | (N.DVC_FLAG_OUT_I420 if out_format == "I420" else 0) | (0 if fused else N.DVC_FLAG_FD_UNFUSED)
        self.out_format = out_format
        self.params = derive_params(width, height, flags=flags, **kwargs)
        self.params.max_batch = int(max_batch)
        self.W, self.H = int(width), int(height)
        self.SW = int(kwargs.get("src_width") or width)
        self.SH = int(kwargs.get("src_height") or height)
        self.in_format = kwargs.get("in_format", "BGR")
        self.device = int(device)
        self.device_ptrs = device_ptrs
        self._lib = N.lib()
        h = ctypes.c_void_p()
        s = ctypes.c_void_p(int(stream)) if stream is not None else None
        N.check(self._lib.dvc_fd_create(ctypes.byref(self.params), self.device, s, ctypes.byref(h)))
        self._h = h

    # -------------------------------------------------------------- frames --
    @property
    def _fshape(self):
        """Input frames (source size): packed BGR, or a (H*3/2, W) 4:2:0 frame."""
        return (self.SH, self.SW, 3) if self.in_format == "BGR" else (self.SH * 3 // 2, self.SW)

    @property
    def _pitch(self):
        return 3 * self.SW if self.in_format == "BGR" else self.SW

    @property
    def _oshape(self):
        """Output frames (scaled size): packed BGR, or (H*3/2, W) I420."""
        return (self.H, self.W, 3) if self.out_format == "BGR" else (self.H * 3 // 2, self.W)

    def _dev(self, x, name, n=None, batched=False, tail=None):
        addr, m = B.device_buf(x, tail or self._fshape, self.device, name, n=n, batched=batched)
        return addr, m

    def prime(self, frame) -> None:
        """fd:67-81: previous gray := GaussianBlur(gray(frame), 25x25, 30); acc := 0."""
        if self.device_ptrs:
            addr, _ = self._dev(frame, "frame")
            N.check(self._lib.dvc_fd_prime(self._h, addr, self._pitch))
        else:
            f = B.host_in(frame, self._fshape, "frame")
            N.check(self._lib.dvc_fd_prime(self._h, f.ctypes.data, self._pitch))

    def set_state(self, prev_gray, acc) -> None:
        """Resume instead of :meth:`prime` (dvc_fd_set_state): the previous
        blurred gray and the accumulated mask (fd:107,133), H x W uint8 each —
        what :meth:`plane` exports as PLANE_GRAY / PLANE_ACC."""
        g = np.ascontiguousarray(prev_gray, dtype=np.uint8)
        a = np.ascontiguousarray(acc, dtype=np.uint8)
        if g.shape != (self.H, self.W) or a.shape != (self.H, self.W):
            raise ValueError(f"state planes must be ({self.H}, {self.W})")
        N.check(self._lib.dvc_fd_set_state(self._h, g.ctypes.data, a.ctypes.data))

    def step(self, frame, overlay=None, compressed=None, acc=None, want=("overlay", "compressed")):
        """fd:91-133 for one frame.

        Host mode: returns ``(overlay, compressed)`` numpy frames (allocated if
        not given; a name missing from ``want`` is skipped). Device mode: writes
        into the given device buffers (None = not produced) and returns None.
        """
        if self.device_ptrs:
            addr, _ = self._dev(frame, "frame")
            ov = self._dev(overlay, "overlay", tail=self._oshape)[0] if overlay is not None else None
            cp = self._dev(compressed, "compressed", tail=self._oshape)[0] if compressed is not None else None
            ac = self._dev(acc, "acc", tail=(self.H, self.W))[0] if acc is not None else None
            N.check(self._lib.dvc_fd_step(self._h, addr, self._pitch, ov, cp, ac))
            return None
        f = B.host_in(frame, self._fshape, "frame")
        overlay = B.host_out(overlay, self._oshape, "overlay", "overlay" in want)
        compressed = B.host_out(compressed, self._oshape, "compressed", "compressed" in want)
        acc = B.host_out(acc, (self.H, self.W), "acc", False)
        N.check(self._lib.dvc_fd_step(self._h, f.ctypes.data, self._pitch,
                                      overlay.ctypes.data if overlay is not None else None,
                                      compressed.ctypes.data if compressed is not None else None,
                                      acc.ctypes.data if acc is not None else None))
        return overlay, compressed

    def step_batch(self, frames, overlay=None, compressed=None, want=("overlay", "compressed")):
        """fd:85-138 for n consecutive frames (identical to n :meth:`step` calls).

        Host mode: ``frames`` is an (n, H, W, 3) uint8 array; returns
        ``(overlay, compressed)`` arrays of the same shape (allocated if not
        given; a name missing from ``want`` is None). Device mode: ``frames``,
        ``overlay``, ``compressed`` are (n, H, W, 3) uint8 CUDA tensors on the
        handle's device (outputs may hold more frames), or explicit
        ``(address, n)`` tuples of dense frames; asynchronous, returns None.
        """
        fs, os_ = int(np.prod(self._fshape)), int(np.prod(self._oshape))
        if self.device_ptrs:
            addr, n = self._dev(frames, "frames", batched=True)
            ov = self._dev(overlay, "overlay", n=n, batched=True, tail=self._oshape)[0] if overlay is not None else None
            cp = self._dev(compressed, "compressed", n=n, batched=True, tail=self._oshape)[0] \
                if compressed is not None else None
            N.check(self._lib.dvc_fd_step_batch(self._h, addr, self._pitch, fs, n, ov, cp, os_))
            return None
        if not isinstance(frames, np.ndarray) or frames.ndim != len(self._fshape) + 1:
            raise ValueError(f"frames: expected uint8 frames of shape (n, {', '.join(map(str, self._fshape))})")
        n = int(frames.shape[0])
        f = B.host_in(frames, (n,) + self._fshape, "frames")
        overlay = B.host_out(overlay, (n,) + self._oshape, "overlay", "overlay" in want)
        compressed = B.host_out(compressed, (n,) + self._oshape, "compressed", "compressed" in want)
        N.check(self._lib.dvc_fd_step_batch(self._h, f.ctypes.data, self._pitch, fs, n,
                                            overlay.ctypes.data if overlay is not None else None,
                                            compressed.ctypes.data if compressed is not None else None, os_))
        return overlay, compressed

    # ------------------------------------------------------------- queries --
    def sync(self) -> None:
        N.check(self._lib.dvc_fd_sync(self._h))

    def stats(self) -> dict:
        s = N.FdStats()
        N.check(self._lib.dvc_fd_get_stats(self._h, ctypes.byref(s)))
        return {k: int(getattr(s, k)) for k, _ in N.FdStats._fields_}

    def plane(self, which: int) -> np.ndarray:
        out = np.empty((self.H, self.W), np.uint8)
        N.check(self._lib.dvc_fd_read_plane(self._h, int(which), out.ctypes.data))
        return out

    def ktime(self, reset: bool = False):
        """(total ms, launches) of the dominant HBM kernel, hipEvent-timed."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        N.check(self._lib.dvc_fd_ktime(self._h, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0))
        return float(ms.value), int(n.value)

    def ktime_kernel(self) -> str:
        """Which kernel ktime() timed in the last batch: "k_front_fused" (the fused
        front with the speculative outputs) or "k_out"."""
        if not hasattr(self._lib, "dvc_fd_ktime_kernel"):   # an older build (DVC_LIB_PATH A/B)
            return "k_out"
        k = self._lib.dvc_fd_ktime_kernel(self._h)
        if k < 0:
            N.check(k)
        return "k_front_fused" if k == N.KTIME_FRONT_FUSED else "k_out"

    def graph_stats(self) -> dict:
        """Batches launched as HIP graphs (the short-batch device path) and graphs built."""
        b, g = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(self._lib.dvc_fd_graph_stats(self._h, ctypes.byref(b), ctypes.byref(g)))
        return {"batches": int(b.value), "builds": int(g.value)}

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.dvc_fd_destroy(self._h)
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
