"""CPU oracle — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over ``oracle/liboracle_dvc.so`` (a plain-C restatement of the
reference's frame-differencing worker, ``frame_differencing.py:67-133``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker or the CPU baseline. The
product package (``dynamic-video-compression-surveillance_amd``) never imports
it and has no CPU fallback.

Parity status: the oracle's numpy-side orchestration is pinned by golden
vectors captured from the unmodified reference code (``tests/golden/``); its
OpenCV primitives are restated from OpenCV 4.11's published algorithms and are
"OCV-unverified" (cv2 is absent from this image) — see DESIGN.md §Parity.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_dvc.so")
_lib = None


class FdParams(ctypes.Structure):
    """Mirror of ``dvc_fd_params`` (include/dvc.h)."""

    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("block", ctypes.c_int32),
        ("ithresh", ctypes.c_int32),
        ("min_area2", ctypes.c_int64),
        ("ksize", ctypes.c_int32),
        ("anchor", ctypes.c_int32),
        ("alpha", ctypes.c_float),
        ("beta", ctypes.c_float),
        ("gamma", ctypes.c_float),
        ("quant", ctypes.c_float),
        ("prime_ksize", ctypes.c_int32),
        ("prime_sigma", ctypes.c_double),
        ("flags", ctypes.c_uint32),
        ("max_batch", ctypes.c_uint32),
        ("src_width", ctypes.c_int32),
        ("src_height", ctypes.c_int32),
        ("in_format", ctypes.c_int32),
        ("chroma_rows", ctypes.c_int32),
    ]


class FdStats(ctypes.Structure):
    _fields_ = [
        ("frames", ctypes.c_uint64),
        ("motion_px", ctypes.c_uint64),
        ("components", ctypes.c_uint64),
        ("static_blocks", ctypes.c_uint64),
    ]


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oc_gauss_kernel_q8.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_uint16)]
        L.oc_bgr2gray.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, u8p]
        L.oc_gaussian_q8.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint16), ctypes.c_int, u8p]
        L.oc_contour_filter.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, u8p, u8p]
        L.oc_contour_filter.restype = ctypes.c_int64
        L.oc_contour_filter_literal.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, u8p]
        L.oc_contour_filter_literal.restype = ctypes.c_int64
        L.oc_find_external_contours.argtypes = [u8p, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)),
                                                ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))]
        L.oc_find_external_contours.restype = ctypes.c_int64
        L.oc_contour_area2.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_int64]
        L.oc_contour_area2.restype = ctypes.c_int64
        L.oc_fill_contour.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.c_int64, ctypes.c_uint8]
        L.oc_free.argtypes = [ctypes.c_void_p]
        L.oc_dilate_rect.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
        L.oc_add_weighted_px.argtypes = [ctypes.c_uint8, ctypes.c_float, ctypes.c_uint8, ctypes.c_float, ctypes.c_float]
        L.oc_add_weighted_px.restype = ctypes.c_uint8
        L.oc_bgr2ycrcb_px.argtypes = [u8p, u8p]
        L.oc_ycrcb2bgr_px.argtypes = [u8p, u8p]
        L.oc_dct_matrix.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        fp = ctypes.POINTER(ctypes.c_float)
        L.oc_dct2d.argtypes = [fp, ctypes.c_int, fp, fp]
        L.oc_idct2d.argtypes = [fp, ctypes.c_int, fp, fp]
        L.oc_dct2d_rect.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp]
        L.oc_idct2d_rect.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, fp, fp]
        L.oc_dct_size_ok.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oc_resize_simd_end.argtypes = [ctypes.c_int]
        L.oc_resize_bgr.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int]
        L.oc_block_quant.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                     ctypes.c_float, u8p, ctypes.c_int]
        L.oc_fd_create.argtypes = [ctypes.POINTER(FdParams), ctypes.c_int]
        L.oc_fd_create.restype = ctypes.c_void_p
        L.oc_fd_destroy.argtypes = [ctypes.c_void_p]
        L.oc_fd_prime.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t]
        L.oc_fd_step.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, u8p, u8p, u8p]
        L.oc_fd_read_plane.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p]
        L.oc_fd_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(FdStats)]
        L.oc_fd_set_state.argtypes = [ctypes.c_void_p, u8p, u8p]
        L.oc_yuv420_to_bgr.argtypes = [u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, u8p, ctypes.c_size_t]
        L.oc_bgr_to_i420.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t, u8p, u8p,
                                     ctypes.c_size_t]
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


# ---------------------------------------------------------------- params ----
def fd_params(width, height, block_size=4, motion_threshold=0.5, min_area=500,
              kernel_size=7, release_factor=0.5, quantization_level=100,
              prime_ksize=25, prime_sigma=30.0, src_width=0, src_height=0) -> FdParams:
    """Host-side derivation of dvc_fd_params from the reference kwargs
    (frame_differencing.py:21-30); same rules as the product's host code.
    width/height are the scaled size (fd:60-61), src_* the video's (0: same)."""
    p = FdParams()
    p.src_width, p.src_height = int(src_width), int(src_height)
    p.width, p.height, p.block = int(width), int(height), int(block_size)
    p.ithresh = max(-1, min(255, math.floor(motion_threshold)))
    p.min_area2 = math.floor(2.0 * float(min_area))
    p.ksize = int(kernel_size)
    p.anchor = int(kernel_size) // 2
    p.alpha = float(release_factor)
    p.beta = float(1 - release_factor)
    p.gamma = 0.0
    p.quant = float(quantization_level)
    p.prime_ksize, p.prime_sigma = int(prime_ksize), float(prime_sigma)
    return p


# ------------------------------------------------------------- primitives ----
def gauss_taps_q8(n: int, sigma: float) -> np.ndarray:
    t = (ctypes.c_uint16 * n)()
    if lib().oc_gauss_kernel_q8(n, sigma, t) != 0:
        raise ValueError("bad kernel size")
    return np.array(t[:], dtype=np.uint16)


def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr)
    H, W = bgr.shape[:2]
    out = np.empty((H, W), np.uint8)
    lib().oc_bgr2gray(_u8(bgr), W * 3, W, H, _u8(out))
    return out


def gaussian_blur(gray: np.ndarray, n: int, sigma: float) -> np.ndarray:
    gray = np.ascontiguousarray(gray)
    H, W = gray.shape
    k = gauss_taps_q8(n, sigma)
    kc = (ctypes.c_uint16 * n)(*k.tolist())
    out = np.empty_like(gray)
    lib().oc_gaussian_q8(_u8(gray), W, H, kc, n, _u8(out))
    return out


def contour_filter(mask: np.ndarray, min_area2: int, literal: bool = False):
    """Returns (filtered, n_components[, filled]) — fd:100-104."""
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    H, W = mask.shape
    out = np.empty_like(mask)
    if literal:
        n = lib().oc_contour_filter_literal(_u8(mask), W, H, int(min_area2), _u8(out))
        return out, int(n)
    filled = np.empty_like(mask)
    n = lib().oc_contour_filter(_u8(mask), W, H, int(min_area2), _u8(out), _u8(filled))
    return out, int(n), filled


def find_external_contours(mask: np.ndarray):
    """Literal Suzuki-Abe RETR_EXTERNAL contours as a list of (N,2) int32 (x,y)."""
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    H, W = mask.shape
    xy = ctypes.POINTER(ctypes.c_int32)()
    off = ctypes.POINTER(ctypes.c_int32)()
    n = lib().oc_find_external_contours(_u8(mask), W, H, ctypes.byref(xy), ctypes.byref(off))
    offs = np.ctypeslib.as_array(off, shape=(n + 1,)).copy()
    npts = int(offs[-1])
    pts = np.ctypeslib.as_array(xy, shape=(max(npts, 1) * 2,)).copy()[: npts * 2].reshape(-1, 2) if npts else np.zeros((0, 2), np.int32)
    lib().oc_free(ctypes.cast(xy, ctypes.c_void_p))
    lib().oc_free(ctypes.cast(off, ctypes.c_void_p))
    return [pts[offs[i]:offs[i + 1]].copy() for i in range(n)]


def contour_area2(pts: np.ndarray) -> int:
    pts = np.ascontiguousarray(pts, dtype=np.int32)
    return int(lib().oc_contour_area2(pts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(pts)))


def fill_contour(img: np.ndarray, pts: np.ndarray, color: int = 255) -> None:
    assert img.dtype == np.uint8 and img.flags.c_contiguous
    pts = np.ascontiguousarray(pts, dtype=np.int32)
    H, W = img.shape
    lib().oc_fill_contour(_u8(img), W, H, pts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(pts), color)


def dilate(mask: np.ndarray, k: int, anchor: int | None = None) -> np.ndarray:
    mask = np.ascontiguousarray(mask)
    H, W = mask.shape
    out = np.empty_like(mask)
    lib().oc_dilate_rect(_u8(mask), W, H, k, k // 2 if anchor is None else anchor, _u8(out))
    return out


def add_weighted(a: np.ndarray, alpha: float, b: np.ndarray, beta: float, gamma: float) -> np.ndarray:
    f = lib().oc_add_weighted_px
    out = np.empty_like(a)
    for i, (x, y) in enumerate(zip(a.ravel().tolist(), b.ravel().tolist())):
        out.ravel()[i] = f(x, alpha, y, beta, gamma)
    return out


def bgr2ycrcb(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr)
    out = np.empty_like(bgr)
    f = lib().oc_bgr2ycrcb_px
    src, dst = bgr.reshape(-1, 3), out.reshape(-1, 3)
    for i in range(src.shape[0]):
        f(_u8(src[i]), _u8(dst[i]))
    return out


def ycrcb2bgr(ycc: np.ndarray) -> np.ndarray:
    ycc = np.ascontiguousarray(ycc)
    out = np.empty_like(ycc)
    f = lib().oc_ycrcb2bgr_px
    src, dst = ycc.reshape(-1, 3), out.reshape(-1, 3)
    for i in range(src.shape[0]):
        f(_u8(src[i]), _u8(dst[i]))
    return out


def dct_matrix(B: int) -> np.ndarray:
    m = (ctypes.c_float * (B * B))()
    lib().oc_dct_matrix(B, m)
    return np.array(m[:], dtype=np.float32).reshape(B, B)


class OddDCTError(RuntimeError):
    """cv2.dct / cv2.idct of an odd length > 1: OpenCV raises StsNotImplemented."""


def _dct_call(fn, block: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(block, dtype=np.float32)
    if x.ndim == 1:
        x = x.reshape(1, -1)
    bh, bw = x.shape
    if not lib().oc_dct_size_ok(bh, bw):
        raise OddDCTError("Odd-size DCT's are not implemented")
    Mh, Mw = dct_matrix(bh), dct_matrix(bw)
    y = np.empty_like(x)
    fp = ctypes.POINTER(ctypes.c_float)
    fn(x.ctypes.data_as(fp), bh, bw, Mh.ctypes.data_as(fp), Mw.ctypes.data_as(fp), y.ctypes.data_as(fp))
    return y.reshape(block.shape)


def dct2d(block: np.ndarray) -> np.ndarray:
    """cv2.dct of a float32 bh x bw block (orthonormal DCT-II rows then
    columns, the oracle's fmaf chains); odd sides > 1 raise OddDCTError."""
    return _dct_call(lib().oc_dct2d_rect, block)


def idct2d(block: np.ndarray) -> np.ndarray:
    """cv2.idct of a float32 bh x bw block."""
    return _dct_call(lib().oc_idct2d_rect, block)


def resize(bgr: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(bgr, (width, height)) INTER_LINEAR 8UC3 as the oracle restates it
    (oc_resize_bgr: copy / exact-2x area fast / fixed-point linear)."""
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w = bgr.shape[:2]
    out = np.empty((int(height), int(width), 3), np.uint8)
    lib().oc_resize_bgr(_u8(bgr), 3 * w, w, h, _u8(out), 3 * int(width), int(width), int(height))
    return out


def yuv420_to_bgr(frame: np.ndarray, fmt: str = "I420") -> np.ndarray:
    """cv2.cvtColor(frame, COLOR_YUV2BGR_I420 / COLOR_YUV2BGR_NV12) of a
    (H*3/2) x W uint8 4:2:0 frame (oracle/yuv_oracle.c; parity-unpinned vs cv2)."""
    frame = np.ascontiguousarray(frame, np.uint8)
    H, W = frame.shape[0] * 2 // 3, frame.shape[1]
    out = np.empty((H, W, 3), np.uint8)
    base = frame.ctypes.data
    p = ctypes.POINTER(ctypes.c_uint8)
    if fmt == "NV12":
        u, v, cp, cs = base + H * W, base + H * W + 1, W, 2
    else:
        u, v, cp, cs = base + H * W, base + H * W + (H // 2) * (W // 2), W // 2, 1
    lib().oc_yuv420_to_bgr(_u8(frame), W, ctypes.cast(u, p), ctypes.cast(v, p), cp, cs, W, H, _u8(out), 3 * W)
    return out


def bgr_to_i420(bgr: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(bgr, COLOR_BGR2YUV_I420): a (H*3/2) x W frame (Y, then U and V
    planes of H/2 x W/2), restated in oracle/yuv_oracle.c (parity-unpinned vs cv2)."""
    bgr = np.ascontiguousarray(bgr, np.uint8)
    H, W = bgr.shape[:2]
    out = np.empty((H * 3 // 2, W), np.uint8)
    base = out.ctypes.data
    p = ctypes.POINTER(ctypes.c_uint8)
    lib().oc_bgr_to_i420(_u8(bgr), 3 * W, W, H, _u8(out), W, ctypes.cast(base + H * W, p),
                         ctypes.cast(base + H * W + (H // 2) * (W // 2), p), W // 2)
    return out


def resize_simd_end(width_bytes: int) -> int:
    return int(lib().oc_resize_simd_end(int(width_bytes)))


def block_quant(block: np.ndarray, q: float) -> np.ndarray:
    """fd:122-125 for one BxB uint8 block of Y."""
    block = np.ascontiguousarray(block, dtype=np.uint8)
    B = block.shape[0]
    M = dct_matrix(B)
    out = np.empty_like(block)
    lib().oc_block_quant(_u8(block), B, B, M.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), q, _u8(out), B)
    return out


# ---------------------------------------------------------------- worker ----
class OracleFD:
    """The oracle's per-feed worker (fd:67-133), one frame per ``step``."""

    def __init__(self, width, height, literal: bool = False, **kwargs):
        self.W, self.H = int(width), int(height)
        self.params = fd_params(width, height, **kwargs)
        self._h = lib().oc_fd_create(ctypes.byref(self.params), 1 if literal else 0)
        if not self._h:
            raise ValueError("oracle rejected parameters")

    def close(self):
        if self._h:
            lib().oc_fd_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def prime(self, bgr: np.ndarray) -> None:
        bgr = np.ascontiguousarray(bgr)
        lib().oc_fd_prime(self._h, _u8(bgr), bgr.shape[1] * 3)

    def step(self, bgr: np.ndarray):
        """(overlay, compressed, acc) of one frame (source size in, scaled size out).
        Raises OddDCTError (with ``.overlay`` and ``.acc`` set) where the
        reference's cv2.dct raises (fd:122)."""
        bgr = np.ascontiguousarray(bgr)
        ov = np.empty((self.H, self.W, 3), np.uint8)
        cp = np.empty_like(ov)
        acc = np.empty((self.H, self.W), np.uint8)
        rc = lib().oc_fd_step(self._h, _u8(bgr), bgr.shape[1] * 3, _u8(ov), _u8(cp), _u8(acc))
        if rc == -6:
            e = OddDCTError("Odd-size DCT's are not implemented")
            e.overlay, e.acc = ov, acc
            raise e
        if rc != 0:
            raise RuntimeError(f"oracle step failed: {rc}")
        return ov, cp, acc

    def plane(self, which: int) -> np.ndarray:
        out = np.empty((self.H, self.W), np.uint8)
        lib().oc_fd_read_plane(self._h, which, _u8(out))
        return out

    def stats(self) -> dict:
        s = FdStats()
        lib().oc_fd_get_stats(self._h, ctypes.byref(s))
        return {k: int(getattr(s, k)) for k, _ in FdStats._fields_}

    def set_state(self, prev_gray: np.ndarray, acc: np.ndarray) -> None:
        """Load (previous blurred gray, accumulated mask) taken from another run
        mid-sequence: the next ``step`` checks one transition of a long run."""
        g = np.ascontiguousarray(prev_gray, np.uint8)
        a = np.ascontiguousarray(acc, np.uint8)
        assert g.shape == a.shape == (self.H, self.W)
        lib().oc_fd_set_state(self._h, _u8(g), _u8(a))


# ------------------------------------------------------------- optical flow --
class OfParams(ctypes.Structure):
    """Mirror of ``dvc_of_params`` (include/dvc.h)."""

    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("flow_threshold", ctypes.c_float),
        ("quant", ctypes.c_float),
        ("alpha_fraction", ctypes.c_double),
        ("window", ctypes.c_int32),
        ("morph_kernel", ctypes.c_int32),
        ("pyr_scale", ctypes.c_double),
        ("levels", ctypes.c_int32),
        ("winsize", ctypes.c_int32),
        ("iterations", ctypes.c_int32),
        ("poly_n", ctypes.c_int32),
        ("poly_sigma", ctypes.c_double),
        ("flags", ctypes.c_uint32),
        ("max_batch", ctypes.c_uint32),
        ("in_format", ctypes.c_int32),
        ("chroma_rows", ctypes.c_int32),
    ]


def of_params(width, height, flow_threshold=0.5, alpha_fraction=0.2, window_size=30, morph_kernel=2,
              quant=100.0, direct_sums=False) -> OfParams:
    """motion_compression_opt.py:29-31 kwargs + the hard-coded Farneback arguments (of:72-81).
    ``direct_sums``: direct per-pixel box sums instead of OpenCV's running sums."""
    p = OfParams()
    p.flags = 0x10 if direct_sums else 0
    p.width, p.height = int(width), int(height)
    p.flow_threshold, p.quant = float(flow_threshold), float(quant)
    p.alpha_fraction, p.window, p.morph_kernel = float(alpha_fraction), int(window_size), int(morph_kernel)
    p.pyr_scale, p.levels, p.winsize, p.iterations, p.poly_n, p.poly_sigma = 0.3, 2, 9, 2, 5, 1.1
    return p


def _of_lib():
    L = lib()
    if not getattr(L, "_of_ready", False):
        u8p = ctypes.POINTER(ctypes.c_uint8)
        fp = ctypes.POINTER(ctypes.c_float)
        L.oc_of_create.argtypes = [ctypes.POINTER(OfParams)]
        L.oc_of_create.restype = ctypes.c_void_p
        L.oc_of_destroy.argtypes = [ctypes.c_void_p]
        L.oc_of_prime.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t]
        L.oc_of_step.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, u8p, u8p, fp]
        L.oc_of_read_plane.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p]
        L.oc_of_set_state.argtypes = [ctypes.c_void_p, u8p, u8p, ctypes.c_int]
        L.oc_farneback.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, fp]
        L.oc_morph_close_open.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p]
        L.oc_morph_close_open_k.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
        L.oc_ellipse_element.argtypes = [ctypes.c_int, u8p]
        L.oc_rect_mask.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p]
        L.oc_rect_mask.restype = ctypes.c_int64
        L.oc_of_compress.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_float, u8p]
        L.oc_vote_threshold.argtypes = [ctypes.c_double, ctypes.c_int]
        L.oc_fb_levels.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int]
        L.oc_fb_level_poly.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_double, fp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oc_update_matrices.argtypes = [fp, fp, fp, ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, ctypes.c_int]
        L.oc_update_flow_box.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.oc_update_flow_box_sliding.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.oc_of_set_sliding.argtypes = [ctypes.c_int]
        L._of_ready = True
    return L


def farneback(prev: np.ndarray, nxt: np.ndarray, pyr_scale=0.3, levels=2, winsize=9, iterations=2, poly_n=5,
              poly_sigma=1.1, sliding=True) -> np.ndarray:
    prev, nxt = np.ascontiguousarray(prev, np.uint8), np.ascontiguousarray(nxt, np.uint8)
    H, W = prev.shape
    flow = np.empty((H, W, 2), np.float32)
    set_sliding(sliding)
    try:
        _of_lib().oc_farneback(_u8(prev), _u8(nxt), W, H, pyr_scale, levels, winsize, iterations, poly_n,
                               poly_sigma, flow.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    finally:
        set_sliding(True)
    return flow


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def fb_level_poly(gray: np.ndarray, k: int, pyr_scale=0.3, poly_n=5, poly_sigma=1.1) -> np.ndarray:
    """Smoothed, resized, polynomial-expanded level k of a gray image (h, w, 5)."""
    gray = np.ascontiguousarray(gray, np.uint8)
    H, W = gray.shape
    R = np.empty((H, W, 5), np.float32)
    w, h = ctypes.c_int(), ctypes.c_int()
    _of_lib().oc_fb_level_poly(_u8(gray), W, H, pyr_scale, k, poly_n, poly_sigma, _fp(R), ctypes.byref(w),
                               ctypes.byref(h))
    return R.reshape(-1)[: h.value * w.value * 5].reshape(h.value, w.value, 5).copy()


def fb_iteration(R0: np.ndarray, R1: np.ndarray, flow: np.ndarray, winsize=9, sliding=True) -> np.ndarray:
    """One FarnebackUpdateMatrices + FarnebackUpdateFlow_Blur step (flow_in -> flow_out),
    box sums in OpenCV's running order (sliding) or direct."""
    h, w = R0.shape[:2]
    R0, R1 = np.ascontiguousarray(R0, np.float32), np.ascontiguousarray(R1, np.float32)
    f = np.ascontiguousarray(flow, np.float32).copy()
    M = np.empty((h, w, 5), np.float32)
    _of_lib().oc_update_matrices(_fp(R0), _fp(R1), _fp(f), w, h, _fp(M), 0, h)
    (_of_lib().oc_update_flow_box_sliding if sliding else _of_lib().oc_update_flow_box)(_fp(M), w, h, winsize, _fp(f))
    return f


def morph_close_open(m: np.ndarray, k: int = 2) -> np.ndarray:
    """of:89-90 with getStructuringElement(MORPH_ELLIPSE, (k, k)) (of:62)."""
    m = np.ascontiguousarray(m, np.uint8)
    out = np.empty_like(m)
    _of_lib().oc_morph_close_open_k(_u8(m), m.shape[1], m.shape[0], int(k), _u8(out))
    return out


def ellipse_element(k: int) -> np.ndarray:
    """getStructuringElement(MORPH_ELLIPSE, (k, k)) as the oracle restates it (k x k, 0/1)."""
    el = np.empty((k, k), np.uint8)
    _of_lib().oc_ellipse_element(int(k), _u8(el))
    return el


def rect_mask(m: np.ndarray):
    m = np.ascontiguousarray(m, np.uint8)
    out = np.empty_like(m)
    n = _of_lib().oc_rect_mask(_u8(m), m.shape[1], m.shape[0], _u8(out))
    return out, int(n)


def of_compress(bgr: np.ndarray, mask: np.ndarray, quant=100.0) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr)
    mask = np.ascontiguousarray(mask, np.uint8)
    out = np.empty_like(bgr)
    H, W = mask.shape
    _of_lib().oc_of_compress(_u8(bgr), 3 * W, _u8(mask), W, H, quant, _u8(out))
    return out


def set_sliding(on: bool) -> None:
    """Box sums of a standalone oc_farneback call: OpenCV's incremental (sliding)
    accumulation (True, the default) or direct per-pixel sums (False). OracleOF
    handles choose by their own ``direct_sums`` argument."""
    _of_lib().oc_of_set_sliding(1 if on else 0)


def vote_threshold(alpha: float, L: int) -> int:
    return int(_of_lib().oc_vote_threshold(alpha, L))


class OracleOF:
    """The oracle's fused OF worker (of:60-101 + of:141-185), one frame per ``step``."""

    def __init__(self, width, height, **kwargs):
        self.W, self.H = int(width), int(height)
        self.params = of_params(width, height, **kwargs)
        self._h = _of_lib().oc_of_create(ctypes.byref(self.params))
        if not self._h:
            raise ValueError("oracle rejected parameters")

    def close(self):
        if self._h:
            _of_lib().oc_of_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def prime(self, bgr):
        bgr = np.ascontiguousarray(bgr)
        _of_lib().oc_of_prime(self._h, _u8(bgr), 3 * self.W)

    def step(self, bgr):
        bgr = np.ascontiguousarray(bgr)
        mask = np.empty((self.H, self.W), np.uint8)
        cp = np.empty_like(bgr)
        flow = np.empty((self.H, self.W, 2), np.float32)
        rc = _of_lib().oc_of_step(self._h, _u8(bgr), 3 * self.W, _u8(mask), _u8(cp),
                                  flow.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if rc != 0:
            raise RuntimeError(f"oracle OF step failed: {rc}")
        return mask, cp, flow

    def set_state(self, prev_gray: np.ndarray, raw_masks: np.ndarray) -> None:
        """Load (previous gray, raw |flow| masks of the last frames oldest first)
        taken from another run mid-sequence (the deque of of:84)."""
        g = np.ascontiguousarray(prev_gray, np.uint8)
        m = np.ascontiguousarray(raw_masks, np.uint8).reshape(-1, self.H, self.W)
        assert g.shape == (self.H, self.W)
        _of_lib().oc_of_set_state(self._h, _u8(g), _u8(m), int(m.shape[0]))

    def plane(self, which: int) -> np.ndarray:
        """0 raw |flow| mask, 1 voted, 2 close/open, 3 rectangles."""
        out = np.empty((self.H, self.W), np.uint8)
        _of_lib().oc_of_read_plane(self._h, which, _u8(out))
        return out
