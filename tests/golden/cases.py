"""Golden cases shared by make_golden.py (capture) and the parity tests (replay).

Inputs are regenerated from these factories (dvc_amd.synthetic / PCG64); the
fixture fd_golden.json keeps their SHA-256 so generator drift is caught.
"""
import numpy as np

from dvc_amd.synthetic import clip

CASES = {
    # name: (frames factory, reference kwargs of filter_and_dilate_movements)
    "s160_clean": (lambda: clip(160, 96, 10, seed=1, n_objects=3), {}),
    "s160_noisy_min20": (lambda: clip(160, 96, 8, seed=2, noisy=True, n_objects=3), {"min_area": 20}),
    "noise64_min100": (lambda: np.random.default_rng(4).integers(0, 256, (4, 48, 64, 3), dtype=np.uint8),
                       {"min_area": 100}),
    "s160_main_variant": (lambda: clip(160, 96, 8, seed=3, n_objects=3),
                          {"block_size": 8, "kernel_size": 10, "release_factor": 0.3}),
    "s160_thr3_k3": (lambda: clip(160, 96, 6, seed=5, noisy=True, n_objects=4),
                     {"motion_threshold": 3.5, "kernel_size": 3, "min_area": 10.5, "quantization_level": 40}),
    "s640_clean_seed0": (lambda: clip(640, 360, 8, seed=0), {}),
    "s640_noisy_seed6": (lambda: clip(640, 360, 6, seed=6, noisy=True), {}),
}
# cases whose every output pixel is stored in fd_golden.npz (the rest: SHA-256 per frame)
FULL_ARRAYS = ("s160_clean", "noise64_min100")
