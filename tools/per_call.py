"""Per-call fixed cost of the FD worker, 1080p, device frames.

    python tools/per_call.py [--frames 766] [--batches 1,2,4,8,32]

For each frames-per-call b: one handle (max_batch = b), the same ping-pong
device sequence as bench.py, three ways of calling it:
  * "worker": FDWorker.step / step_batch with torch views (bench.py --per-frame);
  * "raw":    the C-ABI through ctypes with precomputed integer addresses;
  * "issue":  raw, the host time of the calls alone (the enqueue cost; the device
              may still be running when the loop ends).
Prints one JSON line per b: us per call and Mpx/s for each.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=766)
    ap.add_argument("--ring", type=int, default=64)
    ap.add_argument("--batches", default="1,2,4,8,32")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import dvc_amd
    from dvc_amd.synthetic import SyntheticClip
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    clip = SyntheticClip(W, H, seed=0)
    ring = [clip.frame(i) for i in range(args.ring)]
    order = list(range(args.ring)) + list(range(args.ring - 2, 0, -1))
    P = args.frames
    seq = torch.empty((P, H, W, 3), dtype=torch.uint8, device=dev)
    for j in range(P):
        seq[j].copy_(torch.from_numpy(ring[order[(j + 1) % len(order)]]))
    ov = torch.empty_like(seq)
    cp = torch.empty_like(seq)
    torch.cuda.synchronize()
    L = dvc_amd._native.lib()
    fs = W * H * 3
    for b in [int(x) for x in args.batches.split(",")]:
        w = dvc_amd.FDWorker(W, H, device=0, device_ptrs=True, max_batch=b)
        w.prime(torch.from_numpy(ring[0]).to(dev))
        h = w._h
        base_in, base_ov, base_cp = seq.data_ptr(), ov.data_ptr(), cp.data_ptr()
        calls = [(j, min(b, P - j)) for j in range(0, P, b)]

        def run_worker():
            for j, m in calls:
                if b == 1:
                    w.step(seq[j], ov[j], cp[j])
                else:
                    w.step_batch(seq[j:j + m], ov[j:j + m], cp[j:j + m])

        def run_raw():
            for j, m in calls:
                o = j * fs
                if b == 1:
                    rc = L.dvc_fd_step(h, base_in + o, 3 * W, base_ov + o, base_cp + o, None)
                else:
                    rc = L.dvc_fd_step_batch(h, base_in + o, 3 * W, fs, m, base_ov + o, base_cp + o, fs)
                if rc:
                    dvc_amd._native.check(rc)

        res = {"frames_per_call": b, "calls": len(calls), "frames": P}
        for name, fn in (("worker", run_worker), ("raw", run_raw)):
            fn()
            w.sync()
            best, issue = 1e9, 1e9
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                t1 = time.perf_counter()
                w.sync()
                t2 = time.perf_counter()
                best = min(best, t2 - t0)
                issue = min(issue, t1 - t0)
            res[name] = {"us_per_call": round(best / len(calls) * 1e6, 2),
                         "mpx_s": round(P * W * H / best / 1e6, 1)}
            if name == "raw":
                res["issue"] = {"us_per_call": round(issue / len(calls) * 1e6, 2)}
        w.close()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
