"""ctypes binding of ``libdvc_hip.so`` — the C-ABI declared in ``include/dvc.h``.

The reference has no FFI: it calls ``cv2.*`` inside the per-frame loop of
``frame_differencing.py:85-138``. This module is the thin layer that replaces
those calls with one ``dvc_fd_step`` per frame (or one ``dvc_fd_step_batch``
per run of frames). There is deliberately no CPU
fallback: if the HIP library is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libdvc_hip.so")
SOURCES = ["fd_kernels.hip", "fd_api.hip", "of_kernels.hip", "of_api.hip", "yuv_kernels.hip", "diag.hip"]
HEADERS = ["fd_kernels.h", "dvc_device.h", "of_kernels.h", "host_common.h", "yuv_kernels.h", "yuv_px.h"]
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off"]

DVC_OK = 0
DVC_E_INVALID, DVC_E_HIP, DVC_E_STATE, DVC_E_NOMEM, DVC_E_UNSUPPORTED = -1, -2, -3, -4, -5
DVC_E_ODD_DCT = -6
DVC_FLAG_DEVICE_PTRS = 0x1
DVC_FLAG_KTIMING = 0x2
DVC_FLAG_KEEP_PLANES = 0x4
DVC_FLAG_JOIN_STREAM = 0x8
DVC_FLAG_OF_DIRECT_SUMS = 0x10
DVC_FLAG_OUT_I420 = 0x20
DVC_FLAG_FD_UNFUSED = 0x40
KTIME_OUT, KTIME_FRONT_FUSED = 0, 1         # dvc_fd_ktime_kernel: which kernel KTIMING timed
KTIME_FLOW, KTIME_FLOW_SCAN, KTIME_FLOW_SCAN2 = 2, 3, 4   # dvc_of_ktime_kernel: the level-0 flow kernel
FMT_BGR, FMT_I420, FMT_NV12 = 0, 1, 2      # DVC_FMT_* frame formats (video I/O)
FORMATS = {"BGR": FMT_BGR, "I420": FMT_I420, "NV12": FMT_NV12}

PLANE_GRAY, PLANE_MOTION, PLANE_FILTERED, PLANE_ACC, PLANE_DILATED = range(5)
OF_PLANE_RAW, OF_PLANE_SMOOTH, OF_PLANE_MORPH, OF_PLANE_RECT, OF_PLANE_GRAY = range(5)

# every symbol include/dvc.h declares (checked by tests/test_host.py::test_abi_exports_every_declared_symbol)
EXPORTS = [
    "dvc_abi_version", "dvc_last_error", "dvc_device_count", "dvc_fd_create", "dvc_fd_prime",
    "dvc_fd_step", "dvc_fd_sync", "dvc_fd_get_stats", "dvc_fd_read_plane", "dvc_fd_ktime",
    "dvc_fd_destroy", "dvc_gaussian_taps_q8", "dvc_contour_filter", "dvc_fd_step_batch",
    "dvc_of_create", "dvc_of_prime", "dvc_of_step", "dvc_of_step_batch", "dvc_of_sync", "dvc_of_get_stats",
    "dvc_of_read_plane", "dvc_of_read_flow", "dvc_of_ktime", "dvc_of_destroy", "dvc_of_compress",
    "dvc_of_debug_read", "dvc_host_alloc", "dvc_host_free", "dvc_yuv420_to_bgr", "dvc_bgr_to_i420",
    "dvc_copy_rate", "dvc_ofc_create", "dvc_ofc_run", "dvc_ofc_sync", "dvc_ofc_destroy",
    "dvc_fd_set_state", "dvc_of_set_state", "dvc_fd_ktime_kernel", "dvc_of_ktime_kernel",
    "dvc_fd_graph_stats",
]
ABI_VERSION = 7
MAX_BATCH = 512


class DvcError(RuntimeError):
    """A negative status from the C-ABI (message from dvc_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"dvc error {code}: {msg}")
        self.code = code


class FdParams(ctypes.Structure):
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


class OfParams(ctypes.Structure):
    """``dvc_of_params`` (include/dvc.h)."""
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


OfStats = FdStats   # same four counters (dvc_of_stats)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(PKG_DIR, "..", "include", "dvc.h")]
    if not force and os.path.exists(LIB_PATH):
        newest = max(os.path.getmtime(d) for d in deps if os.path.exists(d))
        if os.path.getmtime(LIB_PATH) >= newest:
            return LIB_PATH
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc, *HIPCC_FLAGS, "-o", tmp, *srcs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    """Load libdvc_hip.so. Raises (never falls back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("DVC_LIB_PATH") or LIB_PATH   # override: A/B runs of two builds
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the HIP path has no CPU fallback)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (same
    # SONAME). Loading torch first makes libdvc_hip.so bind to that instance, so
    # torch tensors/streams and this library share devices and streams; loading
    # /opt/rocm's copy first would leave torch without a usable GPU.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(path)
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    L.dvc_abi_version.restype = ctypes.c_int
    L.dvc_last_error.restype = ctypes.c_char_p
    L.dvc_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.dvc_fd_create.argtypes = [ctypes.POINTER(FdParams), ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.dvc_fd_prime.argtypes = [vp, u8p, ctypes.c_size_t]
    L.dvc_fd_set_state.argtypes = [vp, u8p, u8p]
    L.dvc_fd_set_state.restype = ctypes.c_int
    L.dvc_of_set_state.argtypes = [vp, u8p, u8p, ctypes.c_int]
    L.dvc_of_set_state.restype = ctypes.c_int
    L.dvc_fd_step.argtypes = [vp, u8p, ctypes.c_size_t, u8p, u8p, u8p]
    L.dvc_fd_sync.argtypes = [vp]
    L.dvc_fd_get_stats.argtypes = [vp, ctypes.POINTER(FdStats)]
    L.dvc_fd_read_plane.argtypes = [vp, ctypes.c_int, u8p]
    L.dvc_fd_ktime.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    if hasattr(L, "dvc_fd_ktime_kernel"):   # (an older build under DVC_LIB_PATH lacks it)
        L.dvc_fd_ktime_kernel.argtypes = [vp]
        L.dvc_fd_ktime_kernel.restype = ctypes.c_int
    if hasattr(L, "dvc_fd_graph_stats"):
        L.dvc_fd_graph_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.dvc_fd_graph_stats.restype = ctypes.c_int
    if hasattr(L, "dvc_of_ktime_kernel"):
        L.dvc_of_ktime_kernel.argtypes = [vp]
        L.dvc_of_ktime_kernel.restype = ctypes.c_int
    L.dvc_fd_destroy.argtypes = [vp]
    L.dvc_fd_destroy.restype = None
    L.dvc_gaussian_taps_q8.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_uint16)]
    L.dvc_fd_step_batch.argtypes = [vp, u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, u8p, u8p,
                                    ctypes.c_size_t]
    L.dvc_contour_filter.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int, u8p,
                                     ctypes.POINTER(ctypes.c_uint64)]
    L.dvc_of_create.argtypes = [ctypes.POINTER(OfParams), ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.dvc_of_prime.argtypes = [vp, u8p, ctypes.c_size_t]
    L.dvc_of_step.argtypes = [vp, u8p, ctypes.c_size_t, u8p, u8p]
    L.dvc_of_step_batch.argtypes = [vp, u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, u8p, ctypes.c_size_t,
                                    u8p, ctypes.c_size_t]
    L.dvc_of_sync.argtypes = [vp]
    L.dvc_of_get_stats.argtypes = [vp, ctypes.POINTER(OfStats)]
    L.dvc_of_read_plane.argtypes = [vp, ctypes.c_int, u8p]
    L.dvc_of_read_flow.argtypes = [vp, vp]
    L.dvc_of_ktime.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.dvc_of_destroy.argtypes = [vp]
    L.dvc_of_debug_read.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
    L.dvc_of_debug_read.restype = ctypes.c_int
    L.dvc_of_destroy.restype = None
    L.dvc_of_compress.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                  u8p]
    L.dvc_ofc_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, vp,
                                 ctypes.c_uint32, ctypes.POINTER(vp)]
    L.dvc_ofc_run.argtypes = [vp, u8p, ctypes.c_size_t, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_size_t,
                              ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t]
    L.dvc_ofc_sync.argtypes = [vp]
    L.dvc_ofc_destroy.argtypes = [vp]
    L.dvc_ofc_destroy.restype = None
    for name in ("dvc_ofc_create", "dvc_ofc_run", "dvc_ofc_sync"):
        getattr(L, name).restype = ctypes.c_int
    L.dvc_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
    L.dvc_host_alloc.restype = ctypes.c_int
    L.dvc_host_free.argtypes = [vp]
    L.dvc_host_free.restype = None
    L.dvc_yuv420_to_bgr.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                    vp, ctypes.c_uint32]
    L.dvc_bgr_to_i420.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, vp,
                                  ctypes.c_uint32]
    L.dvc_copy_rate.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double)]
    L.dvc_copy_rate.restype = ctypes.c_int
    L.dvc_yuv420_to_bgr.restype = ctypes.c_int
    L.dvc_bgr_to_i420.restype = ctypes.c_int
    for name in ("dvc_of_create", "dvc_of_prime", "dvc_of_step", "dvc_of_step_batch", "dvc_of_sync",
                 "dvc_of_get_stats", "dvc_of_read_plane", "dvc_of_read_flow", "dvc_of_ktime", "dvc_of_compress"):
        getattr(L, name).restype = ctypes.c_int
    for name in ("dvc_device_count", "dvc_fd_create", "dvc_fd_prime", "dvc_fd_step", "dvc_fd_sync",
                 "dvc_fd_get_stats", "dvc_fd_read_plane", "dvc_fd_ktime", "dvc_gaussian_taps_q8",
                 "dvc_contour_filter", "dvc_fd_step_batch"):
        getattr(L, name).restype = ctypes.c_int
    if L.dvc_abi_version() != ABI_VERSION:
        # a library with another dvc_fd_params / flag layout would corrupt
        # memory: refuse it unless the caller opts in explicitly (A/B of builds
        # from an older tree whose layout is known to match)
        if os.environ.get("DVC_ALLOW_ABI_MISMATCH") != "1":
            raise ImportError(f"{path}: ABI version {L.dvc_abi_version()} != {ABI_VERSION} "
                              "(set DVC_ALLOW_ABI_MISMATCH=1 to load it anyway)")
        import warnings
        warnings.warn(f"{path}: ABI version mismatch accepted (DVC_ALLOW_ABI_MISMATCH=1)")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != DVC_OK:
        msg = lib().dvc_last_error()
        raise DvcError(rc, msg.decode() if msg else "")


class _Pinned:
    """Owner of one dvc_host_alloc block (freed when the last view dies)."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib().dvc_host_alloc(int(nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)

    def __del__(self):
        try:
            lib().dvc_host_free(ctypes.c_void_p(self.ptr))
        except Exception:
            pass


def pinned(shape, dtype="uint8"):
    """A numpy array in page-locked host memory (dvc_host_alloc): host-pointer
    steps DMA such buffers directly, with no staging copy on the CPU."""
    import numpy as np
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    owner = _Pinned(max(count * dt.itemsize, 1))
    buf = (ctypes.c_uint8 * max(count * dt.itemsize, 1)).from_address(owner.ptr)
    buf._owner = owner          # every view of the array keeps the block alive
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


def contour_filter(mask, min_area2: int, device: int = 0):
    """fd:100-104 on the GPU for one host mask; returns (filtered, components)."""
    import numpy as np
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    H, W = m.shape
    out = np.empty_like(m)
    nc = ctypes.c_uint64()
    check(lib().dvc_contour_filter(m.ctypes.data, W, H, int(min_area2), int(device), out.ctypes.data,
                                   ctypes.byref(nc)))
    return out, int(nc.value)


def of_compress(bgr, mask, quant: float = 100.0, device: int = 0):
    """compress_with_motion for one frame with an arbitrary mask (of:151-183) on the GPU."""
    import numpy as np
    f = np.ascontiguousarray(bgr, dtype=np.uint8)
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    H, W = m.shape
    if f.shape != (H, W, 3):
        raise ValueError("frame and mask shapes differ")
    out = np.empty_like(f)
    check(lib().dvc_of_compress(f.ctypes.data, 3 * W, m.ctypes.data, W, H, float(quant), int(device),
                                out.ctypes.data))
    return out


class OFCompressor:
    """compress_with_motion's loop (of:141-185) on the GPU for chunks of frames
    (dvc_ofc): host numpy frames (n, H, W, 3) and decoded masks (n, H, W) or
    (n, H, W, 3) -> compressed frames (n, H, W, 3)."""

    def __init__(self, width: int, height: int, quant: float = 100.0, max_batch: int = 32, device: int = 0):
        self.W, self.H, self.max_batch = int(width), int(height), max(1, int(max_batch))
        h = ctypes.c_void_p()
        check(lib().dvc_ofc_create(self.W, self.H, float(quant), self.max_batch, int(device), None, 0,
                                   ctypes.byref(h)))
        self._h = h

    def run(self, frames, masks, out=None):
        import numpy as np
        f = np.ascontiguousarray(frames, dtype=np.uint8)
        m = np.ascontiguousarray(masks, dtype=np.uint8)
        if f.ndim == 3:
            f, m = f[None], m[None]
        n = f.shape[0]
        ch = 3 if m.ndim == 4 else 1
        if f.shape[1:] != (self.H, self.W, 3) or m.shape[:3] != (n, self.H, self.W):
            raise ValueError(f"frames {f.shape} / masks {m.shape} do not match {self.W}x{self.H}")
        if out is None:
            out = np.empty_like(f)
        if n:
            check(lib().dvc_ofc_run(self._h, f.ctypes.data, 3 * self.W, f[0].nbytes, m.ctypes.data, self.W * ch,
                                    m[0].nbytes, ch, n, out.ctypes.data, out[0].nbytes))
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().dvc_ofc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def yuv420_to_bgr(frames, fmt: str = "I420", device: int = 0):
    """cv2.cvtColor(COLOR_YUV2BGR_I420 / _NV12) on the GPU of host 4:2:0 frames:
    one (H*3/2, W) uint8 frame or an (n, H*3/2, W) stack -> (.., H, W, 3) BGR."""
    import numpy as np
    f = np.ascontiguousarray(frames, dtype=np.uint8)
    one = f.ndim == 2
    f = f[None] if one else f
    n, H, W = f.shape[0], f.shape[1] * 2 // 3, f.shape[2]
    if f.shape[1] != H * 3 // 2 or H % 2 or W % 2:
        raise ValueError(f"4:2:0 frames must be (H*3/2, W) with H, W even, got {f.shape[1:]}")
    out = np.empty((n, H, W, 3), np.uint8)
    check(lib().dvc_yuv420_to_bgr(f.ctypes.data, W, FORMATS[fmt], 0, W, H, n, f[0].nbytes, out.ctypes.data, 3 * W,
                                  3 * W * H, int(device), None, 0))
    return out[0] if one else out


def bgr_to_i420(frames, device: int = 0):
    """cv2.cvtColor(COLOR_BGR2YUV_I420) on the GPU of host BGR frames: (H, W, 3) or
    (n, H, W, 3) uint8 -> (.., H*3/2, W) I420."""
    import numpy as np
    f = np.ascontiguousarray(frames, dtype=np.uint8)
    one = f.ndim == 3
    f = f[None] if one else f
    n, H, W = f.shape[:3]
    if H % 2 or W % 2 or f.shape[3] != 3:
        raise ValueError(f"BGR frames must be (H, W, 3) with H, W even, got {f.shape[1:]}")
    out = np.zeros((n, H * 3 // 2, W), np.uint8)
    check(lib().dvc_bgr_to_i420(f.ctypes.data, 3 * W, 3 * W * H, W, H, n, out.ctypes.data, W, 0, out[0].nbytes,
                                int(device), None, 0))
    return out[0] if one else out


def copy_rate(device: int = 0, nbytes: int = 1 << 30, reps: int = 20, nontemporal: bool = True) -> float:
    """dvc_copy_rate: this GPU's hand-written streaming-copy rate in GB/s (bytes
    read + written), the practical HBM ceiling the bench quotes beside 8 TB/s."""
    g = ctypes.c_double()
    check(lib().dvc_copy_rate(int(device), int(nbytes), int(reps), int(bool(nontemporal)), ctypes.byref(g)))
    return g.value


def gaussian_taps_q8(n: int, sigma: float) -> list:
    t = (ctypes.c_uint16 * n)()
    check(lib().dvc_gaussian_taps_q8(n, sigma, t))
    return list(t)
