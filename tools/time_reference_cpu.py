"""Time the reference's own CPU path (missing #4) — container only.

Runs the UNMODIFIED reference orchestration (`/root/reference/frame_differencing.py`,
`filter_and_dilate_movements` with its defaults) on a synthetic 1080p clip and
reports the reference's own per-frame timing (its execution_times.txt,
fd:86,135,147-157). cv2 is absent from this image, so the cv2 calls go to an
in-memory shim. The golden-vector shim (`tests/golden/make_golden.py`) is
exact but slow where it calls the C oracle once per pixel (cvtColor) or per
block through ctypes, which would bill the shim to the reference; for timing,
those primitives are replaced here by vectorised numpy / scipy stand-ins of
the same shape and comparable cost to OpenCV's (their outputs are not
checked — this measures time, parity is the golden vectors' job). What is
measured is therefore the reference's Python loop and its numpy per-block loop
(fd:117-127) with the primitives at native-library speed. The GPU box has no
/root/reference: the figure is measured here, on this container's CPU, one
thread, and committed as profiles/r4_reference_cpu_container.json.

    python tools/time_reference_cpu.py [frames=6] [width=1920] [height=1080]
"""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
from scipy import ndimage  # noqa: E402

import tests.golden.make_golden as MG  # noqa: E402
from dvc_amd.synthetic import clip  # noqa: E402

_make_exact = MG.make_cv2


def _dct_mat(n):
    k = np.arange(n)[:, None]
    x = np.arange(n)[None, :]
    m = np.cos(np.pi * (2 * x + 1) * k / (2 * n)) * np.sqrt(2.0 / n)
    m[0] /= np.sqrt(2.0)
    return m.astype(np.float32)


def make_timing_cv2(clips, written):
    cv2 = _make_exact(clips, written)
    exact_find, exact_area, exact_draw = cv2.findContours, cv2.contourArea, cv2.drawContours

    def cvtColor(img, code):
        f = img.astype(np.float32)
        if code == cv2.COLOR_BGR2GRAY:
            return (f @ np.float32([0.114, 0.587, 0.299])).round().astype(np.uint8)
        if code == cv2.COLOR_BGR2YCrCb:
            y = f @ np.float32([0.114, 0.587, 0.299])
            cr = (f[..., 2] - y) * 0.713 + 128
            cb = (f[..., 0] - y) * 0.564 + 128
            return np.clip(np.stack([y, cr, cb], -1).round(), 0, 255).astype(np.uint8)
        y, cr, cb = f[..., 0], f[..., 1] - 128, f[..., 2] - 128
        bgr = np.stack([y + 1.773 * cb, y - 0.714 * cr - 0.344 * cb, y + 1.403 * cr], -1)
        return np.clip(bgr.round(), 0, 255).astype(np.uint8)

    def GaussianBlur(img, ksize, sigma):
        n = int(ksize[0])
        s = sigma if sigma > 0 else 0.3 * ((n - 1) * 0.5 - 1) + 0.8
        x = np.arange(n) - (n - 1) / 2
        k = np.exp(-x * x / (2 * s * s))
        k /= k.sum()
        f = ndimage.convolve1d(img.astype(np.float32), k, axis=0, mode="mirror")
        return ndimage.convolve1d(f, k, axis=1, mode="mirror").round().astype(np.uint8)

    def dilate(img, kernel, iterations=1):
        return ndimage.maximum_filter(img, size=kernel.shape[0])

    mats = {}

    def dct(block):
        m = mats.setdefault(block.shape[0], _dct_mat(block.shape[0]))
        return m @ block @ m.T

    def idct(block):
        m = mats.setdefault(block.shape[0], _dct_mat(block.shape[0]))
        return m.T @ block @ m

    for fn in (cvtColor, GaussianBlur, dilate, dct, idct):
        setattr(cv2, fn.__name__, fn)
    # findContours / contourArea / drawContours: the oracle's C, once per frame / contour
    cv2.findContours, cv2.contourArea, cv2.drawContours = exact_find, exact_area, exact_draw
    return cv2


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    frames = clip(W, H, n, seed=0)
    MG.make_cv2 = make_timing_cv2
    t0 = time.perf_counter()
    ov, cp, times = MG.run_reference(frames)
    wall = time.perf_counter() - t0
    lines = {k.strip(): v.strip() for k, v in (ln.split(":", 1) for ln in times.splitlines() if ":" in ln)}
    per_frame = float(lines["Average time per frame"].split()[0])
    out = {
        "what": "reference frame_differencing.filter_and_dilate_movements (defaults), unmodified; cv2 calls "
                "through a timing shim (numpy / scipy stand-ins for cvtColor, GaussianBlur, dilate, dct, idct; "
                "the C oracle for findContours / contourArea / drawContours)",
        "where": "this container's CPU (the GPU box has no /root/reference), 1 thread",
        "cpu": platform.processor() or platform.machine(),
        "workload": f"synthetic {W}x{H} clip (dvc_amd.synthetic.clip seed 0), {n} frames",
        "frames_processed": int(lines["Frames processed"]),
        "reference_avg_s_per_frame": per_frame,
        "reference_Mpx_per_s": round(W * H / per_frame / 1e6, 4) if per_frame else None,
        "wall_s": round(wall, 2),
        "outputs_written": [int(len(ov)), int(len(cp))],
        "note": "the per-block numpy loop (fd:117-127) runs once per 4x4 block: 129,600 iterations a 1080p frame",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
