"""Per-phase timing of the OF scan kernel from s_memtime stamps (debug build with
-DDVC_SCAN_STAMPS, e.g. gpurun_ab/libstamp.so via DVC_LIB_PATH): frame 0 of the
last level-0 launch, every (strip, row block): 0 step start, 1 after the vertical
sums, 2 after the left-strip wait, 3 after the chains / M, 4 after the barrier,
5 after the solve. Prints phase medians and the wavefront critical path."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dvc_amd  # noqa: E402
from dvc_amd.synthetic import SyntheticClip  # noqa: E402

W, H, n = 1920, 1080, int(os.environ.get("DVC_STAMP_FRAMES", "16"))
clip = SyntheticClip(W, H, seed=0)
fr = torch.from_numpy(np.stack([clip.frame(i) for i in range(n + 1)])).cuda()
w = dvc_amd.OFWorker(W, H, device=0, device_ptrs=True, max_batch=n)
mk = torch.empty((n, H, W), dtype=torch.uint8, device="cuda")
cp = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
w.prime(fr[0])
for _ in range(3):
    w.step_batch(fr[1:], mk, cp)
w.sync()
L = dvc_amd._native.lib()
buf = (ctypes.c_ulonglong * (32 * 96 * 8))()
assert L.dvc_debug_scan_stamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(32, 96, 8).astype(np.int64)
S, B = 30, 90
a = a[:S, :B]
t0 = a[:, :, 0][a[:, :, 0] > 0].min()
rel = (a - t0) / 2.1e3   # ~us at 2.1 GHz (s_memtime ticks = shader cycles)
ph = np.diff(a[:, :, :6], axis=2) / 2.1e3
names = ["vertical", "wait", "chain/M", "barrier", "solve"]
for i, nm in enumerate(names):
    print(f"{nm:10s} median {np.median(ph[:, :, i]):7.2f} us  p90 {np.percentile(ph[:, :, i], 90):7.2f}")
print(f"step total median {np.median(np.sum(ph, axis=2)):.2f} us")
sub = {"prefetch issue (0->6)": (0, 6), "vertical sums (6->7)": (6, 7), "barrier A (7->1)": (7, 1)}
for nm, (i, j) in sub.items():
    d = (a[:, :, j] - a[:, :, i]) / 2.1e3
    print(f"  {nm:24s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}")
print("strip 0 block starts (us):", np.round(rel[0, :6, 0], 2))
print("strip 15 block starts (us):", np.round(rel[15, :6, 0], 2))
print("last strip end:", round(rel[S - 1, B - 1, 5], 1), "us; strip starts:", np.round(rel[:, 0, 0], 1)[:10])
print("wait by strip (median over blocks):", np.round(np.median(ph[:, :, 1], axis=1), 2))
