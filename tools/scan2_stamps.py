"""Per-interval timing of the pipelined OF scan (k_flow_scan2) from s_memtime
stamps (debug build with -DDVC_SCAN2_STAMPS, loaded via DVC_LIB_PATH): frame 0
of the last level-0 launch, every (strip, interval). Chain wave: 0 start, 1
after the left-strip poll, 2 after the chain, 3 after the barrier. An M-wave
waves' arrivals at the interval's barrier: 4 wave 1 (vertical sums + M), 5
wave 4 (M only, on the chain's SIMD), 6 wave 10 (solve + M), 7 wave 15
(solve + M). With -DDVC_STAMP_DETAIL=1 (and DVC_STAMP_DETAIL=1 here) stamps
4..7 trace wave 10 instead: after stage 3, after the solve, after R1 row 0, at the barrier."""
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
assert L.dvc_debug_scan2_stamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(32, 96, 8).astype(np.int64)
S, NB = 30, 90
a = a[:S, :NB + 2]   # interval k at index k + 1 (k = -1 .. NB)
cyc = 2.1e3          # ~us at 2.1 GHz (s_memtime ticks = shader cycles)
st = a[:, 2:NB, :]   # steady state k = 1 .. NB - 2
prev3 = a[:, 1:NB - 1, 3]
rows = {
    "chain: poll wait": st[:, :, 1] - st[:, :, 0],
    "chain: chain": st[:, :, 2] - st[:, :, 1],
    "chain: barrier wait": st[:, :, 3] - st[:, :, 2],
    "wave 1 (V+G) done": st[:, :, 4] - prev3,
    "wave 4 (G) done": st[:, :, 5] - prev3,
    "wave 10 (S+G) done": st[:, :, 6] - prev3,
    "wave 15 (S+G) done": st[:, :, 7] - prev3,
    "interval": st[:, :, 3] - prev3,
}
if os.environ.get("DVC_STAMP_DETAIL") == "1":   # library built with -DDVC_STAMP_DETAIL=1: wave 10's steps
    rows = {k: v for k, v in rows.items() if k.startswith("chain") or k == "interval"}
    rows.update({
        "w10: to stage3 done": st[:, :, 4] - prev3,
        "w10: ldR0 + solve": st[:, :, 5] - st[:, :, 4],
        "w10: ldR1 row 0": st[:, :, 6] - st[:, :, 5],
        "w10: rest to barrier": st[:, :, 7] - st[:, :, 6],
    })
for nm, d in rows.items():
    d = d / cyc
    print(f"{nm:22s} median {np.median(d):7.3f} us  p10 {np.percentile(d, 10):7.3f}  p90 {np.percentile(d, 90):7.3f}"
          f"  strip0 {np.median(d[0]):7.3f}")
item = (a[:, NB + 1, 3] - a[:, 0, 0]) / cyc
print("item total (us) median", round(float(np.median(item)), 1), " strips' starts (us):",
      np.round((a[:, 0, 0] - a[:, 0, 0].min()) / cyc, 1)[:12])
