"""Capture golden vectors of the OF path from the UNMODIFIED reference.

Runs ``/root/reference/motion_compression_opt.py`` (read-only, imported by path
with ``sys.dont_write_bytecode``): ``temporal_smoothing_flow`` then
``compress_with_motion`` on the videos it wrote, exactly as
``process_single_video_of`` chains them (of:209-231), under the in-memory cv2
shim of ``make_golden.py`` extended with the OF primitives. The shim's
videos are lossless (frames are kept as written), so the capture is the
reference's two passes with the mp4v round trip removed — the fused worker's
contract.

What this pins: the reference's numpy-side semantics — the deque vote
(``np.sum`` of the queued masks against ``alpha*len*255`` in float64),
``.astype(np.uint8)*255``, ``block_mask.mean() == 0`` gating of full blocks
only, float32 ``/QTY`` + ``np.round`` half-even, ``np.clip`` + truncating
uint8 assignment on all three channels, the merge / YCrCb->BGR / per-block
gray order — and, through independent shim implementations, the morphology
(a numpy ``getStructuringElement(MORPH_ELLIPSE)`` + ``morphologyEx``) and the
rectangles (literal Suzuki-Abe ``findContours`` + ``boundingRect`` +
``rectangle``), against the oracle's formulations of those steps.
Farneback itself is the oracle's restatement (cv2 is absent: OCV-unverified).

Container-only (needs /root/reference); outputs are committed fixtures.

    python tests/golden/make_golden_of.py
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from tests.golden.make_golden import make_cv2  # noqa: E402
from tests.golden.cases_of import CASES, FULL_ARRAYS  # noqa: E402

REF = "/root/reference/motion_compression_opt.py"


def make_cv2_of(clips: dict, written: dict):
    cv2 = make_cv2(clips, written)
    cv2.COLOR_GRAY2BGR = 8
    cv2.MORPH_ELLIPSE, cv2.MORPH_CLOSE, cv2.MORPH_OPEN = 2, 3, 2

    base_capture = cv2.VideoCapture

    class VideoCapture(base_capture):
        def __init__(self, path):
            super().__init__(path)
            if self.f is None and os.path.basename(path) in written:
                self.f = np.stack(written[os.path.basename(path)])

    cv2.VideoCapture = VideoCapture
    base_cvt = cv2.cvtColor

    def cvtColor(img, code):
        if code == cv2.COLOR_GRAY2BGR:
            return np.repeat(img[..., None], 3, axis=2)
        return base_cvt(img, code)

    def getStructuringElement(shape, ksize):
        # OpenCV getStructuringElement, MORPH_ELLIPSE branch
        assert shape == cv2.MORPH_ELLIPSE
        kw, kh = ksize
        r, c = kh // 2, kw // 2
        inv_r2 = 1.0 / (r * r) if r else 0.0
        el = np.zeros((kh, kw), np.uint8)
        for i in range(kh):
            dy = i - r
            if abs(dy) <= r:
                dx = int(round(c * np.sqrt((r * r - dy * dy) * inv_r2)))
                j1, j2 = max(c - dx, 0), min(c + dx + 1, kw)
                el[i, j1:j2] = 1
        return el

    def _morph(img, kernel, dilate):
        kh, kw = kernel.shape
        ay, ax = kh // 2, kw // 2
        H, W = img.shape
        out = np.full((H, W), 0 if dilate else 255, np.int32)
        for i in range(kh):
            for j in range(kw):
                if not kernel[i, j]:
                    continue
                dy, dx = i - ay, j - ax   # out(x, y) uses src(x + dx, y + dy); outside = ignored
                src = np.full((H, W), 0 if dilate else 255, np.int32)
                ys, yd = (slice(dy, H), slice(0, H - dy)) if dy >= 0 else (slice(0, H + dy), slice(-dy, H))
                xs, xd = (slice(dx, W), slice(0, W - dx)) if dx >= 0 else (slice(0, W + dx), slice(-dx, W))
                src[yd, xd] = img[ys, xs]
                out = np.maximum(out, src) if dilate else np.minimum(out, src)
        return out.astype(np.uint8)

    def morphologyEx(img, op, kernel):
        if op == cv2.MORPH_CLOSE:
            return _morph(_morph(img, kernel, True), kernel, False)
        if op == cv2.MORPH_OPEN:
            return _morph(_morph(img, kernel, False), kernel, True)
        raise ValueError(op)

    def calcOpticalFlowFarneback(prev, nxt, flow, pyr_scale, levels, winsize, iterations, poly_n, poly_sigma,
                                 flags):
        assert flow is None and flags == 0
        return O.farneback(prev, nxt, pyr_scale, levels, winsize, iterations, poly_n, poly_sigma)

    def cartToPolar(x, y):
        x = np.asarray(x, np.float32)
        y = np.asarray(y, np.float32)
        return np.sqrt(x * x + y * y).astype(np.float32), np.zeros_like(x)

    def boundingRect(cnt):
        p = np.asarray(cnt).reshape(-1, 2)
        x0, y0 = p.min(axis=0)
        x1, y1 = p.max(axis=0)
        return int(x0), int(y0), int(x1 - x0 + 1), int(y1 - y0 + 1)

    def rectangle(img, p1, p2, color, thickness):
        assert thickness == -1
        (xa, ya), (xb, yb) = p1, p2
        H, W = img.shape[:2]
        img[max(ya, 0):min(yb, H - 1) + 1, max(xa, 0):min(xb, W - 1) + 1] = color
        return img

    for fn in (cvtColor, getStructuringElement, morphologyEx, calcOpticalFlowFarneback, cartToPolar,
               boundingRect, rectangle):
        setattr(cv2, fn.__name__, fn)
    return cv2


def run_reference(frames: np.ndarray, **kwargs):
    clips = {"clip.mp4": frames}
    written: dict = {}
    sys.modules["cv2"] = make_cv2_of(clips, written)
    spec = importlib.util.spec_from_file_location("ref_motion_compression_opt", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with tempfile.TemporaryDirectory() as td:
        md = mod.temporal_smoothing_flow("clip.mp4", td, **kwargs)
        cp = mod.compress_with_motion(os.path.join(td, "overlay.mp4"), os.path.join(td, "mask.mp4"), td)
    del sys.modules["cv2"]
    assert md[0] == cp[0] == len(frames) - 1, (md, cp)
    return np.stack(written["mask.mp4"]), np.stack(written["compressed.mp4"])


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    arrays, meta = {}, {}
    for name, (mk, kw) in CASES.items():
        frames = mk()
        masks, comp = run_reference(frames, **kw)
        assert masks.shape == (len(frames) - 1,) + frames.shape[1:3], masks.shape
        if name in FULL_ARRAYS:
            arrays[f"{name}__mask"] = masks
            arrays[f"{name}__compressed"] = comp
        meta[name] = {"kwargs": kw, "n_frames": int(len(frames)), "input_sha256": [sha(f) for f in frames],
                      "mask_sha256": [sha(f) for f in masks], "compressed_sha256": [sha(f) for f in comp],
                      "mask_px": [int((f > 0).sum()) for f in masks]}
        print(f"{name}: {len(frames)} frames, kwargs={kw}, mask px/frame={meta[name]['mask_px']}")
    np.savez_compressed(os.path.join(HERE, "of_golden.npz"), **arrays)
    with open(os.path.join(HERE, "of_golden.json"), "w") as f:
        json.dump({"cases": meta,
                   "source": "reference motion_compression_opt.py:29-193 (temporal_smoothing_flow -> "
                             "compress_with_motion) under tests/golden/make_golden_of.py cv2 shim"}, f, indent=1)


if __name__ == "__main__":
    main()
