"""Drop-in driver throughput (GPU box): process_single_video_fd (or _of) end to
end as a user calls it — a 1080p Y4M (4:2:0) camera file in, the two output videos out
(.npy streams of BGR frames, or Y4M with DVC_VIDEO_SINK=y4m), file I/O and host
copies included. Prints one JSON line per run.
  python tools/bench_dropin.py [--frames N] [--sink npy|y4m] [--module NAME] [--dir /tmp/x]
"""
import argparse
import importlib
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def make_clip(path, W, H, n):
    from dvc_amd._native import bgr_to_i420
    from dvc_amd.synthetic import SyntheticClip
    c = SyntheticClip(W, H, seed=0)
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F30:1 Ip A1:1 C420jpeg\n" % (W, H))
        for t in range(n):
            f.write(b"FRAME\n" + bgr_to_i420(c.frame(t), 0).tobytes())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=150)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--sink", choices=("npy", "y4m"), default="npy")
    ap.add_argument("--path", choices=("fd", "of"), default="fd")
    ap.add_argument("--module", default="")
    ap.add_argument("--dir", default="/tmp/dvc_dropin")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    src = os.path.join(a.dir, "cam.y4m")
    if not os.path.exists(src):
        make_clip(src, a.width, a.height, a.frames)
    os.environ["DVC_VIDEO_SINK"] = a.sink
    module = a.module or ("frame_differencing" if a.path == "fd" else "motion_compression_opt")
    mod = importlib.import_module(f"dvc_amd.{module}")
    out = os.path.join(a.dir, "out")
    shutil.rmtree(out, ignore_errors=True)
    t0 = time.time()
    if a.path == "fd":
        mod.process_single_video_fd(src, out)
    else:
        mod.process_single_video_of(src, out)
    dt = time.time() - t0
    n = a.frames - 1
    print(json.dumps({"mode": f"drop-in process_single_video_{a.path}", "module": module, "source": "y4m I420 file",
                      "sink": a.sink, "frames": n, "seconds": round(dt, 3), "fps": round(n / dt, 1),
                      "Mpx_per_s": round(n * a.width * a.height / dt / 1e6, 1)}))
    shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
