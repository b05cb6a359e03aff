"""Write n synthetic BGR frames (dvc_amd.synthetic, seed 0) as raw bytes for tools/stage_bench."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dvc_amd.synthetic import SyntheticClip  # noqa: E402

W, H, n, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
noisy = len(sys.argv) > 5 and sys.argv[5] == "noisy"
clip = SyntheticClip(W, H, seed=0, noisy=noisy)
with open(out, "wb") as f:
    for t in range(n):
        f.write(clip.frame(t).tobytes())
