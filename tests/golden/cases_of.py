"""Golden cases of the OF path shared by make_golden_of.py (capture) and the
parity tests (replay). Inputs are regenerated from these factories; the fixture
of_golden.json keeps their SHA-256 so generator drift is caught. Sizes are
multiples of 8 (the GPU path's constraint) and cover pyramid depths 0, 1 and 2."""
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
}
# cases whose every output pixel is stored in of_golden.npz (the rest: SHA-256 per frame)
FULL_ARRAYS = ("of_s160_clean", "of_noise64")
