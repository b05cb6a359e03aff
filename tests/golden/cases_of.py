"""Golden cases of the OF path shared by make_golden_of.py (capture) and the
parity tests (replay). Inputs are regenerated from these factories; the fixture
of_golden.json keeps their SHA-256 so generator drift is caught. Sizes cover
pyramid depths 0, 1 and 2, sides that are not multiples of 8 (partial 8x8
edge blocks, skipped by compress_with_motion, of:159,177; rows that are not
whole dword quads) and morph_kernel values other than the default 2 (of:62)."""
import numpy as np

from dvc_amd.synthetic import clip

CASES = {
    # name: (frames factory, reference kwargs of temporal_smoothing_flow)
    "of_s160_clean": (lambda: clip(160, 96, 8, seed=1, n_objects=3), {}),                  # 1 level
    "of_noise64": (lambda: np.random.default_rng(4).integers(0, 256, (4, 48, 64, 3), dtype=np.uint8), {}),
    "of_s320_w4": (lambda: clip(320, 176, 12, seed=2, n_objects=3),                          # 2 levels, deque eviction
                   {"window_size": 4, "alpha_fraction": 0.5}),
    "of_s320_alpha0": (lambda: clip(320, 176, 4, seed=3, n_objects=2), {"alpha_fraction": 0.0}),
    "of_s640_seed0": (lambda: clip(640, 360, 5, seed=0), {}),                                # 3 levels
    "of_s640_noisy_thr03": (lambda: clip(640, 360, 5, seed=6, noisy=True), {"flow_threshold": 0.3}),
    "of_s162x98": (lambda: clip(162, 98, 6, seed=12, n_objects=3), {}),                      # partial blocks
    "of_s170x100_morph3": (lambda: clip(170, 100, 6, seed=13, n_objects=3), {"morph_kernel": 3}),
    "of_s133x75_morph5_w3": (lambda: clip(133, 75, 7, seed=14, n_objects=3),                  # odd sides
                             {"morph_kernel": 5, "window_size": 3, "alpha_fraction": 0.4}),
    "of_s330x186_morph4": (lambda: clip(330, 186, 5, seed=15, n_objects=4), {"morph_kernel": 4}),   # 2 levels
    # the round-4 ranges: vote windows beyond 127 (counts past 127, eviction at 200) and
    # elements beyond 31
    "of_noise64_w200": (lambda: np.random.default_rng(16).integers(0, 256, (212, 48, 64, 3), dtype=np.uint8),
                        {"window_size": 200, "alpha_fraction": 0.9}),
    "of_s160_morph40": (lambda: clip(160, 96, 6, seed=17, n_objects=3), {"morph_kernel": 40}),
}
# cases whose every output pixel is stored in of_golden.npz (the rest: SHA-256 per frame)
FULL_ARRAYS = ("of_s160_clean", "of_noise64", "of_s162x98", "of_s170x100_morph3")
