"""Deterministic synthetic surveillance clips.

The reference ships no sample media (``frame_differencing.py:201`` and
``motion_compression_opt.py:250`` point at absent files), so parity tests and
the benchmark run on generated feeds:

* static textured background ``B(x,y,c) = 28 + ((37x + 11(c+1)y + 29c) mod 200)``;
* ``n_objects`` axis-aligned rectangles / filled discs (6 at 640 px width, 12 at
  1920, 24 at 3840 unless given), side U[24,160]*(W/1920) px, constant random
  BGR colour, integer velocity U[-6,6]^2 (never zero), bouncing off the edges;
* variant ``noisy``: +-3 uniform integer noise on 0.5 % of the pixels of every
  frame (many sub-min_area components for the contour filter).

Everything is drawn from ``numpy.random.default_rng(seed)`` (PCG64), so a
(seed, W, H, frame index) always yields the same frame.
"""
from __future__ import annotations

import numpy as np


def default_objects(width: int) -> int:
    return 6 if width <= 640 else (12 if width <= 1920 else 24)


def background(width: int, height: int) -> np.ndarray:
    x = np.arange(width, dtype=np.int64)[None, :, None]
    y = np.arange(height, dtype=np.int64)[:, None, None]
    c = np.arange(3, dtype=np.int64)[None, None, :]
    return (28 + (37 * x + 11 * (c + 1) * y + 29 * c) % 200).astype(np.uint8)


def _tri(u: int, L: int) -> int:
    """Bouncing coordinate in [0, L]."""
    if L <= 0:
        return 0
    m = u % (2 * L)
    return m if m <= L else 2 * L - m


class SyntheticClip:
    def __init__(self, width: int, height: int, seed: int = 0, n_objects: int | None = None,
                 noisy: bool = False):
        self.W, self.H, self.seed, self.noisy = int(width), int(height), int(seed), bool(noisy)
        rng = np.random.default_rng(self.seed)
        n = default_objects(self.W) if n_objects is None else int(n_objects)
        scale = self.W / 1920.0
        self.objects = []
        for _ in range(n):
            kind = int(rng.integers(0, 2))  # 0 rect, 1 disc
            sw = max(2, int(round(rng.uniform(24, 160) * scale)))
            sh = sw if kind == 1 else max(2, int(round(rng.uniform(24, 160) * scale)))
            sw, sh = min(sw, self.W), min(sh, self.H)
            color = rng.integers(0, 256, 3).astype(np.uint8)
            px = int(rng.integers(0, self.W - sw + 1))
            py = int(rng.integers(0, self.H - sh + 1))
            while True:
                vx, vy = (int(v) for v in rng.integers(-6, 7, 2))
                if vx or vy:
                    break
            self.objects.append((kind, sw, sh, color, px, py, vx, vy))
        self._bg = background(self.W, self.H)
        self._disc_masks = {}

    def _disc(self, d: int) -> np.ndarray:
        m = self._disc_masks.get(d)
        if m is None:
            r = (d - 1) / 2.0
            yy, xx = np.mgrid[0:d, 0:d]
            m = (xx - r) ** 2 + (yy - r) ** 2 <= (d / 2.0) ** 2
            self._disc_masks[d] = m
        return m

    def frame(self, t: int) -> np.ndarray:
        f = self._bg.copy()
        for kind, sw, sh, color, px, py, vx, vy in self.objects:
            x = _tri(px + vx * t, self.W - sw)
            y = _tri(py + vy * t, self.H - sh)
            if kind == 0:
                f[y:y + sh, x:x + sw] = color
            else:
                f[y:y + sh, x:x + sw][self._disc(sw)] = color
        if self.noisy:
            rng = np.random.default_rng((self.seed, int(t), 1))
            npx = int(round(0.005 * self.W * self.H))
            idx = rng.choice(self.W * self.H, size=npx, replace=False)
            delta = rng.integers(-3, 4, size=(npx, 3))
            flat = f.reshape(-1, 3)
            flat[idx] = np.clip(flat[idx].astype(np.int16) + delta, 0, 255).astype(np.uint8)
        return f

    def frames(self, n: int, start: int = 0) -> np.ndarray:
        return np.stack([self.frame(start + i) for i in range(n)])


def clip(width: int, height: int, n_frames: int, seed: int = 0, noisy: bool = False,
         n_objects: int | None = None) -> np.ndarray:
    return SyntheticClip(width, height, seed=seed, noisy=noisy, n_objects=n_objects).frames(n_frames)
