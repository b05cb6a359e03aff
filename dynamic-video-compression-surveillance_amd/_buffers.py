"""Checks at the ctypes boundary.

Every buffer whose address crosses into the C-ABI (include/dvc.h) is checked
here first: the C side trusts dense frames of ``3*W`` bytes per row and
``3*W*H`` bytes per frame, so a sliced, permuted, short or wrongly placed
buffer must be refused in Python rather than read or written out of bounds on
the device or the host heap.

* host buffers: numpy ``uint8``, C-contiguous, writeable outputs, exact shape;
* device buffers: torch CUDA tensors, ``uint8``, contiguous, on the handle's
  device, the expected trailing shape and at least ``n`` frames; or, as an
  explicit opt-in for callers that manage raw allocations, an ``(address, n)``
  tuple / :class:`DevicePtr` whose layout the caller vouches for.
"""
from __future__ import annotations

import numpy as np


class DevicePtr:
    """A raw device address of ``n`` dense frames (explicit opt-in: unchecked)."""

    __slots__ = ("addr", "n")

    def __init__(self, addr: int, n: int = 1):
        self.addr, self.n = int(addr), int(n)


def _is_tensor(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def device_buf(x, tail: tuple, device: int, name: str, n: int | None = None, batched: bool = True):
    """(address, frames) of a device buffer of frames with trailing shape ``tail``.

    ``batched``: the buffer is ``(m,) + tail`` (``m >= n`` when ``n`` is given);
    otherwise exactly ``tail`` (one frame). Raises ValueError/TypeError."""
    if isinstance(x, DevicePtr):
        return x.addr, x.n
    if isinstance(x, tuple) and len(x) == 2 and all(isinstance(v, int) for v in x):
        return int(x[0]), int(x[1])
    if not _is_tensor(x):
        raise TypeError(f"{name}: device mode needs a torch CUDA tensor or an explicit (address, n) tuple, "
                        f"got {type(x).__name__}")
    import torch
    if not x.is_cuda:
        raise ValueError(f"{name}: tensor is on {x.device}, not a GPU")
    if x.device.index != int(device):
        raise ValueError(f"{name}: tensor is on cuda:{x.device.index}, the handle on cuda:{device}")
    if x.dtype != torch.uint8:
        raise ValueError(f"{name}: dtype {x.dtype}, expected torch.uint8")
    if not x.is_contiguous():
        raise ValueError(f"{name}: tensor is not contiguous")
    shape = tuple(x.shape)
    if batched:
        if len(shape) != len(tail) + 1 or shape[1:] != tuple(tail):
            raise ValueError(f"{name}: shape {shape}, expected (n,) + {tuple(tail)}")
        m = shape[0]
        if n is not None and m < n:
            raise ValueError(f"{name}: holds {m} frames, {n} needed")
        return int(x.data_ptr()), m
    if shape != tuple(tail) and shape != (1,) + tuple(tail):
        raise ValueError(f"{name}: shape {shape}, expected {tuple(tail)}")
    return int(x.data_ptr()), 1


def host_in(x, shape: tuple, name: str) -> np.ndarray:
    """A C-contiguous uint8 host array of exactly ``shape`` (copied if needed)."""
    if not isinstance(x, np.ndarray) or x.dtype != np.uint8 or x.shape != tuple(shape):
        raise ValueError(f"{name}: expected a uint8 numpy array of shape {tuple(shape)}")
    return np.ascontiguousarray(x)


def host_out(x, shape: tuple, name: str, allocate: bool):
    """An output host array: ``None`` -> a new array when ``allocate`` (else None);
    a given array must be writeable, C-contiguous uint8 of exactly ``shape``."""
    if x is None:
        return np.empty(shape, np.uint8) if allocate else None
    if (not isinstance(x, np.ndarray) or x.dtype != np.uint8 or x.shape != tuple(shape)
            or not x.flags.c_contiguous or not x.flags.writeable):
        raise ValueError(f"{name}: expected a writeable C-contiguous uint8 array of shape {tuple(shape)}")
    return x
