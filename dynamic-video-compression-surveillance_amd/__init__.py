"""dvc_amd — MI355X-native per-frame worker for dynamic surveillance compression.

Drop-in for the hot path of carlozamu/dynamic-video-compression-surveillance:
the frame-differencing worker (``frame_differencing.py``) and the optical-flow
worker (``motion_compression_opt.py``) run as hand-written
HIP kernels for gfx950 behind the C-ABI in ``include/dvc.h``; this package is
the Python host that keeps the reference's function signatures.

Import it as ``dvc_amd`` (the repo-root ``dvc_amd.py`` shim maps that name onto
this directory, whose name is not a Python identifier).
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401  (loading is lazy; no CPU fallback)
from .fd import FDWorker, derive_params  # noqa: F401
from .of import OFWorker, derive_of_params  # noqa: F401,E402
