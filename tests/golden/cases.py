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
    # geometry: partial edge blocks (fd:117-127), any block size, scale_factor (fd:60-61,74,91)
    "w162_h98_partial": (lambda: clip(162, 98, 12, seed=11, n_objects=3), {}),
    "w164_h100_main_variant": (lambda: clip(164, 100, 12, seed=12, n_objects=3),
                               {"block_size": 8, "kernel_size": 10, "release_factor": 0.3}),
    "main_config_scale0p5": (lambda: clip(328, 200, 10, seed=13, n_objects=3),      # fd:200-207 kwargs
                             {"block_size": 8, "kernel_size": 10, "release_factor": 0.3,
                              "quantization_level": 100, "scale_factor": 0.5}),
    "scale0p7_linear": (lambda: clip(200, 120, 10, seed=14, n_objects=3), {"scale_factor": 0.7}),
    "scale1p3_b6": (lambda: clip(120, 80, 10, seed=15, n_objects=2), {"scale_factor": 1.3, "block_size": 6}),
    "b16_partial": (lambda: clip(200, 120, 12, seed=16, n_objects=3), {"block_size": 16}),
    "b1_min20": (lambda: clip(64, 48, 11, seed=17, n_objects=2), {"block_size": 1, "min_area": 20}),
    "b2_w66": (lambda: clip(66, 50, 11, seed=20, n_objects=2), {"block_size": 2, "min_area": 20}),
    # the round-4 parameter ranges: blocks beyond 64 (partial edge blocks of 40 / 48 rows)
    # and dilation kernels beyond 63 (anchor 50 / 63)
    "s640_b80_k100": (lambda: clip(640, 360, 8, seed=21), {"block_size": 80, "kernel_size": 100}),
    "s320_b128_k127": (lambda: clip(320, 176, 8, seed=22, n_objects=3), {"block_size": 128, "kernel_size": 127}),
    # cv2.dct raises on an odd side > 1 (fd:122) and the loop ends (fd:140)
    "odd_b5_stops": (lambda: clip(160, 96, 12, seed=18, n_objects=3), {"block_size": 5}),
    "odd_w163_stops": (lambda: clip(163, 96, 14, seed=19, n_objects=3), {}),
}
# cases whose every output pixel is stored in fd_golden.npz (the rest: SHA-256 per frame)
FULL_ARRAYS = ("s160_clean", "noise64_min100", "w162_h98_partial", "odd_w163_stops")
