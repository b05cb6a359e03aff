"""Benchmark: the frame-differencing hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
    python bench.py --width 3840 --height 2160       # configs[2]: 4K FD feed
    python bench.py --path of                        # configs[4]: 1080p OF (Farneback) path

Workload (BASELINE.json configs[1]): one synthetic 1920x1080 camera feed per
GPU (seed = rank), the full per-frame worker of frame_differencing.py:91-133 —
gray, 5x5 blur, absdiff/threshold, contour-area filter, 7x7 dilate,
accumulation, red overlay, static-block DCT quantisation, YCrCb round trip —
with the GUI's default kwargs (windows.py:154). Frames are device-resident: R
distinct synthetic frames (--ring; FD batch+1, OF 64) played ping-pong
(0..R-1..1) so every consecutive pair is real motion, materialised as one
contiguous (2R-2)-frame sequence (FD 1080p: 766 frames, 4.8 GB — far beyond
the 256 MB Infinity Cache); overlay and compressed outputs go to device buffers
of the same length. A step = one pass over that sequence through
dvc_fd_step_batch (launches of --batch frames, FD default 383 at 1080p: larger
grids keep the latency-bound contour filter occupied and amortise each call's
fixed serial tail — round 6 on one box: 8 → 244 k, 32 → 353 k, 128 → 389 k,
383 → 409 k Mpx/s, profiles/r6_bench_fd_batch*.json; --per-frame: one
dvc_fd_step per frame instead, 50 k, each call one HIP graph launch).

Feeds shard one per GPU with no data-path collective ("scaling": "weak");
RCCL carries only the end-of-run aggregate stats and the max-over-ranks time.

Timing: ``--runs`` (5) timed runs of exactly ``--steps`` steps each, each
bracketed by a barrier and a device sync; ``value`` is the median run (max over
ranks per run), every run's value under ``timing``. ``ranks`` records the
world size the process group saw and every rank's own frame count.

Extra JSON fields: ``roofline`` for the dominant kernel (FD: the fused k_front:
hipEvent time per launch on the front stream where it runs, in a second pass of
the same steps; k_out on the back stream when the one-pass output stage runs —
block sizes other than 4; ``copy``: the same bytes against this
box's hand-written copy rate, dvc_copy_rate) and
``cpu_baseline`` (the C oracle, one host core, a bounded sample of the same
feed, with ``all_cores``: one feed per available core up to the box's CPU
share; rank 0 at N=1 only).

``--path of`` runs the fused optical-flow worker of motion_compression_opt.py
(of:65-101 + of:141-185: gray, Farneback 3-level pyramid, vote, close/open,
rectangles, 8x8 three-channel compression) on the same device-resident
sequence; its dominant kernel is k_flow_scan2 at pyramid level 0 (OpenCV's
running box sums, a latency-bound recurrence: roofline on the VALU axis).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixels/s (frames/s × H×W) 1080p frame-diff path @1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# fused k_front / k_out (the dominant HBM kernel) algorithmic bytes per pixel per frame: read BGR 3 +
# acc>127 bit 1/8 (+ one static bit per block, negligible), write overlay 3 + compressed 3
BACK_BYTES_PER_PX_FRAME = 9.125
BACK_BYTES_PER_PX_LAUNCH = 0
# the fused front (block_size 4, BGR in and out: fd_kernels.h FrontOut) moves the same
# 9.125 B/px per frame — read BGR 3, write overlay 3 + compressed 3 (speculatively, as
# static blocks) + motion bits 1/8 — plus, once per launch, prev gray in 1 + gray out 1
FRONT_FUSED_BYTES_PER_PX_LAUNCH = 2
PIPE_BYTES_PER_PX = 13         # whole frame: + prev gray 1 read, new gray 1 written
# OF: k_flow at level 0, per pixel per launch (iterations = 2): read R(prev) 20 + R(cur) 20
# (+ flow in 8 on the 2nd), write flow 8 on the 1st / the motion bit 1/8 on the 2nd
OF_FLOW_BYTES_PER_PX = (48.0 + 48.125) / 2
OF_PIPE_BYTES_PER_PX = 11.25   # SURVEY.md §8d (config 5): frame I/O + state, not Farneback scratch
# k_flow is not HBM-bound: its work is FarnebackUpdateMatrices (f32) + the box sums
# and solve (f64) per pixel per iteration (oracle/of_oracle.c oc_update_matrices +
# oc_update_flow_box_sliding): 81 f32 + 33 f64 flops; an f64 op takes two f32 issue
# slots on gfx950 (FP64 vector = half the 157.3 TFLOP/s FP32 vector peak), so the
# VALU roofline counts FP32-equivalent flops against the FP32 vector peak
OF_FLOW_F32_FLOPS_PER_PX = 81
OF_FLOW_F64_FLOPS_PER_PX = 33
FP32_VECTOR_PEAK_TFLOPS = 157.3


def pingpong(n: int):
    return list(range(n)) + list(range(n - 2, 0, -1))


def pmc_traffic(path: str, kernel_prefix: str, workload: str, frames_per_launch: float):
    """HBM bytes per launch of a kernel from a committed rocprofv3 PMC summary of
    the same workload and launch size (tools/profile_round.sh), or None."""
    try:
        with open(path) as f:
            d = json.load(f)
        fpl = d.get("frames_per_launch")
        if d.get("workload") != workload or fpl is None or abs(fpl - frames_per_launch) > 0.5:
            return None
        k = d["kernels"][kernel_prefix]
        return float(k["hbm_bytes_per_launch"])
    except Exception:
        return None


def _cpu_feed(job):
    """One feed through the C oracle on this process's core: (frames, seconds)."""
    width, height, budget_s, max_frames, path, seed = job
    sys.path.insert(0, ROOT)
    import oracle  # checker / CPU baseline only
    from dvc_amd.synthetic import SyntheticClip
    clip = SyntheticClip(width, height, seed=seed)
    o = oracle.OracleFD(width, height) if path == "fd" else oracle.OracleOF(width, height)
    o.prime(clip.frame(0))
    frames = [clip.frame(t) for t in range(1, max_frames + 1)]
    n, t0 = 0, time.perf_counter()
    for f in frames:
        o.step(f)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    o.close()
    return n, dt


def cpu_baseline(width: int, height: int, budget_s: float, max_frames: int, path: str = "fd", cores: int = 1):
    """The C oracle on the host: `cores` independent feeds (seeds 0..cores-1) on
    as many processes, each a bounded sample of ~budget_s; value = the sum of
    their Mpx/s (the CPU analogue of feed-per-GPU)."""
    import oracle  # checker / CPU baseline only
    oracle.build()
    jobs = [(width, height, budget_s, max_frames, path, c) for c in range(max(1, cores))]
    if len(jobs) == 1:
        res = [_cpu_feed(jobs[0])]
    else:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(len(jobs)) as pool:   # fresh interpreters: no GPU state inherited
            res = pool.map(_cpu_feed, jobs)
    value = sum(n * width * height / dt for n, dt in res) / 1e6
    nf = sum(n for n, _ in res)
    secs = max(dt for _, dt in res)
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count()
    src = f"oracle/{'dvc' if path == 'fd' else 'of'}_oracle.c"
    return {"value": round(value, 3), "unit": "Mpixels/s", "cores": len(jobs), "kind": "port",
            "nproc": os.cpu_count(), "cpus_available": avail,
            "sample": f"C oracle ({src}, -O3, 1 thread per feed) on {len(jobs)} feed(s) of the same {width}x{height} "
                      f"synthetic workload (seeds 0..{len(jobs) - 1}), {nf} frames in {secs:.1f} s"}


def copy_bandwidth(local: int, nbytes=2 << 30, reps=20):
    """This GPU's streaming-copy rate in GB/s (bytes read + written), the
    practical ceiling SURVEY.md §8d asks the roofline to be quoted against
    beside the 8 TB/s spec: dvc_copy_rate, a hand-written 16-B-per-lane copy
    (the form MI355X_MICROARCH.md measures 6.29 TB/s with; tools/copy_sweep.hip
    picked its grid and unroll) of a 2 GiB buffer, with plain and with
    nontemporal loads and stores; the faster of the two."""
    import dvc_amd
    plain = dvc_amd._native.copy_rate(local, nbytes, reps, nontemporal=False)
    nt = dvc_amd._native.copy_rate(local, nbytes, reps, nontemporal=True)
    return max(plain, nt), {"plain": round(plain, 1), "nontemporal": round(nt, 1)}


def run_cpu_baseline(args):
    """One host core (the oracle is single-threaded per feed), and beside it every
    available core up to the box's CPU share, one feed per core."""
    W, H = args.width, args.height
    base = cpu_baseline(W, H, args.cpu_budget, 120, args.path, 1)
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    share = int(os.environ.get("DVC_CPU_SHARE", "16"))
    ncores = args.cpu_cores or max(1, min(avail, share))
    if ncores > 1:
        mc = cpu_baseline(W, H, args.cpu_budget, 120, args.path, ncores)
        mc["cap"] = (f"{ncores} of {avail} available CPUs: the GPU box's CPU share per GPU is {share} "
                     f"(DVC_CPU_SHARE)") if ncores < avail else "every available CPU"
        base["all_cores"] = mc
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--ring", type=int, default=0, help="distinct frames (0: batch+1 fd / 64 of)")
    ap.add_argument("--noisy", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=("fd", "of"), default="fd",
                    help="fd: frame_differencing.py worker (headline); of: motion_compression_opt.py worker")
    ap.add_argument("--block-size", type=int, default=4, help="FD block_size (fd:161; the __main__ variant uses 8)")
    ap.add_argument("--kernel-size", type=int, default=7, help="FD dilation kernel_size (__main__: 10)")
    ap.add_argument("--release-factor", type=float, default=0.5, help="FD release_factor (__main__: 0.3)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per device launch (max_batch; 0: fd 383 at 1080p, scaled by pixels / of 126)")
    ap.add_argument("--per-frame", action="store_true", help="one dvc_fd_step per frame instead of batches")
    ap.add_argument("--io", choices=("device", "host-pinned", "host-pageable"), default="device",
                    help="device: frames and outputs resident in HBM (the headline); host-*: frames from and "
                         "outputs to host memory through the C-ABI's host-pointer path (PCIe-inclusive; pinned = "
                         "dvc_host_alloc buffers DMA'd directly, pageable = numpy arrays staged by the library)")
    ap.add_argument("--feeds", type=int, default=1,
                    help="independent feeds per GPU, one handle and one host thread each (config 4's unit)")
    ap.add_argument("--of-direct", action="store_true",
                    help="OF: direct per-pixel box sums (DVC_FLAG_OF_DIRECT_SUMS) instead of OpenCV's running sums")
    ap.add_argument("--in-format", choices=("BGR", "I420", "NV12"), default="BGR",
                    help="frames as decoder surfaces: 4:2:0 YUV converted on the GPU in the worker's first "
                         "stage (cvtColor YUV2BGR, what VideoCapture.read() returns; video I/O, SURVEY §8f #1)")
    ap.add_argument("--out-format", choices=("BGR", "I420"), default="BGR",
                    help="FD outputs as the encoder's 4:2:0 input (cvtColor BGR2YUV_I420 of the frames fd:112,131 "
                         "hand to VideoWriter; DVC_FLAG_OUT_I420) instead of BGR")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU baseline's multi-core leg: this many feeds on this many host processes (0: every "
                         "available CPU up to the box's CPU share, DVC_CPU_SHARE, default 16)")
    ap.add_argument("--out-ring", type=int, default=2,
                    help="output buffer sets written in turn, one per step: the encoder side reads one set while "
                         "the next step writes the other (default 2); 1: every step overwrites the previous step's "
                         "outputs, so a fused-front batch waits for the fix-up of the batch two before it")
    ap.add_argument("--ktime-seconds", type=float, default=6.0,
                    help="minimum device time of the hipEvent pass that times the dominant kernel")
    ap.add_argument("--runs", type=int, default=5,
                    help="timed runs of --steps steps each; the line reports the median run (SURVEY.md §8d)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import dvc_amd
    from dvc_amd.synthetic import SyntheticClip

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # the CPU baseline (rank 0 at N=1 only) runs first, in fresh processes, so the
    # GPU phase below is one contiguous stretch of device work
    cpu_base = None
    if world == 1 and not args.no_cpu_baseline:
        cpu_base = run_cpu_baseline(args)
    # DVC_BENCH_ONE_DEVICE=1: rehearse the N > 1 flow on a one-GPU box (every
    # rank on cuda:0, gloo for the end-of-run reduction; RCCL refuses two ranks
    # on one device). The driver's multi-GPU runs never set it.
    one_dev = os.environ.get("DVC_BENCH_ONE_DEVICE") == "1"
    local = 0 if one_dev else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    W, H = args.width, args.height
    of = args.path == "of"
    host_io = args.io != "device"
    # FD: 383-frame launches at 1080p (scaled by pixel count for larger frames);
    # host I/O: 32-frame chunks (the library pipelines chunk uploads / downloads)
    fd_batch = max(31, min(383, 383 * 1920 * 1080 // (W * H)))
    R = args.ring or (64 if (of or host_io) else fd_batch + 1)
    order = pingpong(R)
    P = len(order)                 # frames per step (126 for R=64)
    # OF: the whole 126-frame step in one launch set (the coarse pyramid levels'
    # flow launches are latency-bound: more frames per launch amortise them;
    # interleaved sweep at 1080p: 16 -> 11.7 k, 32 -> 12.9 k, 64 -> 13.7 k,
    # 126 -> 14.3 k, 254 -> 14.6 k, 510 -> 14.7 k Mpx/s)
    batch = 1 if args.per_frame else max(1, min(args.batch or (126 if of else (32 if host_io else fd_batch)), P))
    F = max(1, args.feeds)

    # per feed: its own synthetic camera (seed = global feed index); frame j of
    # a step is ring frame order[(j + 1) % P] (frame 0 primes the feed)
    yuv = args.in_format != "BGR"

    def to_surface(fr):
        """BGR -> the 4:2:0 surface a decoder would hand over (cvtColor BGR2YUV_I420 on the GPU)."""
        i420 = dvc_amd._native.bgr_to_i420(fr, local)
        if args.in_format == "NV12":
            c = i420[H:].reshape(-1)
            u, v = c[:H * W // 4].reshape(H // 2, W // 2), c[H * W // 4:].reshape(H // 2, W // 2)
            i420 = np.concatenate([i420[:H], np.stack([u, v], -1).reshape(H // 2, W)])
        return i420

    def feed_inputs(f):
        clip = SyntheticClip(W, H, seed=rank * F + f, noisy=args.noisy)
        ring = [clip.frame(i) for i in range(R)]
        if yuv:
            ring = [to_surface(fr) for fr in ring]
        fshape = ring[0].shape
        idx = [order[(j + 1) % P] for j in range(P)]
        # OF writes a mask plane instead of the red overlay; I420 outputs are (H*3/2, W)
        oshape = (P, H, W) if of else ((P, H * 3 // 2, W) if args.out_format == "I420" else (P, H, W, 3))
        if args.io == "device":
            seq = torch.empty((P,) + fshape, dtype=torch.uint8, device=dev)
            for j in range(P):
                seq[j].copy_(torch.from_numpy(ring[idx[j]]))
            outs = [(torch.empty(oshape, dtype=torch.uint8, device=dev),
                     torch.empty((P, H, W, 3) if of else oshape[0:1] + oshape[1:], dtype=torch.uint8, device=dev))
                    for _ in range(max(1, args.out_ring))]
        else:
            alloc = dvc_amd._native.pinned if args.io == "host-pinned" else (lambda shp: np.empty(shp, np.uint8))
            seq = alloc((P,) + fshape)
            for j in range(P):
                seq[j] = ring[idx[j]]
            outs = [(alloc(oshape), alloc((P, H, W, 3) if of else oshape)) for _ in range(max(1, args.out_ring))]
        first = torch.from_numpy(ring[0]).to(dev) if args.io == "device" else ring[0]
        return seq, outs, first

    inputs = [feed_inputs(f) for f in range(F)]
    torch.cuda.synchronize()

    def make_worker(f, ktiming=False):
        cls = dvc_amd.OFWorker if of else dvc_amd.FDWorker
        kw = dict(direct_sums=args.of_direct, in_format=args.in_format) if of else \
            dict(block_size=args.block_size, kernel_size=args.kernel_size, release_factor=args.release_factor,
                 in_format=args.in_format, out_format=args.out_format)
        w = cls(W, H, device=local, device_ptrs=not host_io, ktiming=ktiming, max_batch=batch, **kw)
        w.prime(inputs[f][2])
        return w

    step_no = [0] * F

    def run_feed(w, f, n):
        seq, outs, _ = inputs[f]
        for _ in range(n):
            ov, cp = outs[step_no[f] % len(outs)]   # --out-ring: output sets used in turn, step by step
            step_no[f] += 1
            if args.per_frame:
                for j in range(P):
                    w.step(seq[j], ov[j], cp[j])
            else:
                w.step_batch(seq, ov, cp)

    def run_steps(ws, n):
        if len(ws) == 1:
            run_feed(ws[0], 0, n)
        else:   # one host thread per feed (ctypes releases the GIL)
            errs = []

            def go(f):
                try:
                    run_feed(ws[f], f, n)
                except Exception as e:  # re-raised below
                    errs.append(e)
            ths = [threading.Thread(target=go, args=(f,)) for f in range(len(ws))]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            if errs:
                raise errs[0]
        for w in ws:
            w.sync()

    ws = [make_worker(f) for f in range(F)]
    run_steps(ws, args.warmup)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # --runs timed runs of exactly --steps steps each, every one bracketed by a
    # barrier + device sync on both sides; the line reports the median run
    # (max over ranks per run), all runs listed beside it
    runs = max(1, args.runs)
    elapsed_runs = []
    st0 = [w.stats() for w in ws]   # counters before the timed runs (prime + warmup)
    has_gs = not of and hasattr(ws[0]._lib, "dvc_fd_graph_stats")
    g0 = ws[0].graph_stats()["batches"] if has_gs else 0
    for _ in range(runs):
        barrier()
        t0 = time.perf_counter()
        run_steps(ws, args.steps)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        elapsed_runs.append(t1 - t0)
    # counters of the timed runs alone (every run steps the same frames): per run
    sts = [w.stats() for w in ws]
    # FD: how the batches were launched — one HIP graph a batch (short batches of
    # device frames, fd_api.hip enqueue_graph) or on the four stage streams
    # batches of the timed runs that ran as one graph launch (feed 0)
    gstats = None
    if has_gs:
        nb = runs * args.steps * (P if args.per_frame else -(-P // batch))
        gstats = {"graph": ws[0].graph_stats()["batches"] - g0, "batches": nb}
    st = {k: sum(x[k] - x0[k] for x, x0 in zip(sts, st0)) / runs for k in sts[0]}
    for w in ws:
        w.close()

    # dominant kernel: hipEvent-timed launches (the fused front on the front
    # stream or k_out on the back stream / k_flow level 0 on the flow stream) of
    # feed 0 alone, same steps; at least ~--ktime-seconds of device time, so the
    # GPU phase is long enough for an outside utilisation sampler to see
    wk = make_worker(0, ktiming=True)
    run_steps([wk], 1)
    wk.ktime(reset=True)
    step_s = sorted(elapsed_runs)[len(elapsed_runs) // 2] / max(args.steps, 1)
    ksteps = max(1, min(args.steps, 10), int(args.ktime_seconds / max(step_s, 1e-6)))
    run_steps([wk], ksteps)
    kms, kn = wk.ktime()
    kkernel = wk.ktime_kernel()   # the library reports the kernel it launched (FD: front / k_out; OF: level 0)
    wk.close()
    kframes = ksteps * P

    # the end-of-run collective (RCCL at N > 1; feeds.reduce_runs): counters
    # summed, each run's time maxed, every rank's own frame count
    from dvc_amd.feeds import reduce_runs
    red = reduce_runs(st, elapsed_runs, rank, world, device="cpu" if one_dev else dev)
    vec = [red["totals"][k] for k in ("frames", "motion_px", "components", "static_blocks")]
    tmax = red["run_times_max"]
    ranks = {"world_size": red["world_size"], "backend": red["backend"], "frames_per_rank": red["frames_per_rank"],
             "scope": "one timed run"}
    run_times = sorted(tmax)
    elapsed_max = run_times[len(run_times) // 2] if len(run_times) % 2 else \
        0.5 * (run_times[len(run_times) // 2 - 1] + run_times[len(run_times) // 2])
    # frames every rank actually stepped in one timed run (the all-reduced
    # counter), not the nominal steps x P x feeds x world: a short rank is not
    # over-credited
    frames_total = float(vec[0])
    frames_nominal = args.steps * P * F * world
    value = frames_total * W * H / elapsed_max / 1e6

    if rank == 0:
        avg_ms = kms / max(kn, 1)
        res = f"{W}x{H}" if (W, H) != (1920, 1080) else "1080p"
        workload = f"{args.path}_{res}_single_feed_per_gpu" if F == 1 else f"{args.path}_{res}_{F}_feeds_per_gpu"
        if host_io:
            workload += f"_{args.io}_io"
        if args.per_frame:
            workload += "_per_frame"
        if args.noisy:
            workload += "_noisy"
        if yuv:
            workload += f"_{args.in_format.lower()}_input"
        if not of and args.out_format != "BGR":
            workload += f"_{args.out_format.lower()}_output"
        if of and args.of_direct:
            workload += "_direct_sums"
        if not of and (args.block_size, args.kernel_size, args.release_factor) != (4, 7, 0.5):
            workload += f"_b{args.block_size}_k{args.kernel_size}_r{args.release_factor:g}"
        if of:   # kn counts level-0 flow launches (iterations per batch)
            kname = kkernel   # the level-0 kernel the library launched (dvc_of_ktime_kernel)
            per_launch_frames = kframes * 2 / max(kn, 1)
            bytes_per_launch = OF_FLOW_BYTES_PER_PX * W * H * per_launch_frames
            traffic = pmc_traffic(os.path.join(ROOT, "profiles", "pmc_summary_of.json"), kname, workload,
                                  per_launch_frames)
        else:
            kname = kkernel
            per_launch_frames = kframes / max(kn, 1)
            # I420 outputs: 1.5 B/px each instead of 3; 4:2:0 input surfaces are read
            # in place (1.5 B/px instead of the BGR frame's 3)
            back = BACK_BYTES_PER_PX_FRAME - (3.0 if args.out_format == "I420" else 0.0) - (1.5 if yuv else 0.0)
            per_launch = FRONT_FUSED_BYTES_PER_PX_LAUNCH if kname == "k_front_fused" else BACK_BYTES_PER_PX_LAUNCH
            bytes_per_launch = (back * kframes + per_launch * kn) * W * H / max(kn, 1)
            traffic = pmc_traffic(os.path.join(ROOT, "profiles", "pmc_summary.json"),
                                  "k_front" if kname == "k_front_fused" else "k_out", workload, per_launch_frames)
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        # SURVEY §8d's per-pixel bytes for this configuration: frame in (BGR 3 / 4:2:0
        # 1.5), state 4, outputs 2 x (BGR 3 / I420 1.5)
        pipe = OF_PIPE_BYTES_PER_PX if of else (PIPE_BYTES_PER_PX - (1.5 if yuv else 0.0)
                                                - (3.0 if args.out_format == "I420" else 0.0))
        line = {
            "metric": METRIC if not of else "Mpixels/s (frames/s × H×W) 1080p optical-flow path; % HBM roofline",
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": workload, "path": "optical-flow (motion_compression_opt.py)" if of
                       else "frame-differencing (frame_differencing.py)",
                       "width": W, "height": H, "frames_per_step": P, "feeds_per_gpu": F,
                       "io": args.io + (" (PCIe-inclusive: frames up, both outputs down)" if host_io else ""),
                       "ring_frames": R, "noisy": args.noisy, "in_format": args.in_format,
                       "out_format": "mask + BGR" if of else args.out_format,
                       "launch": "per-frame" if args.per_frame else "batched", "frames_per_launch": batch,
                       "launch_path": None if gstats is None else
                       ("HIP graph a batch" if gstats["graph"] == gstats["batches"] else
                        "stage streams" if gstats["graph"] == 0 else
                        f"{gstats['graph']} of {gstats['batches']} batches as HIP graphs, the rest on the stage streams"),
                       "output_sets": max(1, args.out_ring),
                       "parallelism": f"feed-per-gpu x{world}",
                       "fps_per_gpu": round(args.steps * P * F / elapsed_max, 1),
                       "pipeline_bytes_per_px": pipe,
                       "pipeline_GBps_per_gpu": round(pipe * args.steps * P * F * W * H / elapsed_max / 1e9, 1)},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "frames_per_launch": round(per_launch_frames, 2),
                         "avg_launch_us": round(avg_ms * 1e3, 2), "launches_timed": kn,
                         "timed_with": "feed 0 alone"},
            "stats": {"scope": "one timed run, all ranks", "frames": int(vec[0]), "motion_px": int(vec[1]),
                      "components": int(vec[2]), "static_blocks": int(vec[3]), "frames_nominal": frames_nominal},
            "timing": {"runs": runs, "reported": "median run", "steps_per_run": args.steps,
                       "value_per_run": [round(frames_total * W * H / t / 1e6, 2) for t in
                                         tmax],
                       "ktime_pass": {"steps": ksteps, "launches": kn}},
            "ranks": ranks,
        }
        if traffic is not None:
            line["roofline"]["traffic_source"] = (
                "committed rocprofv3 PMC profile of the same workload and launch size (2 x FETCH_SIZE + "
                "WRITE_SIZE, tools/profile_round.sh): profiles/" + ("pmc_summary_of.json" if of else "pmc_summary.json"))
        # the same kernel's bytes (and the pipeline's) against this box's measured copy rate
        cp_gbs, cp_detail = copy_bandwidth(local)
        line["roofline"]["copy"] = {"GBps": round(cp_gbs, 1), "frac": round(achieved / cp_gbs, 4),
                                    "pipeline_frac": round(line["config"]["pipeline_GBps_per_gpu"] / cp_gbs, 4),
                                    "kernel": "dvc_copy_rate: hand-written 16 B/lane copy of 2 GiB", **cp_detail}
        if of:   # k_flow's binding axis is the VALU (serial f64 recurrences), not HBM
            px_it = W * H * per_launch_frames
            flops = px_it * (OF_FLOW_F32_FLOPS_PER_PX + 2 * OF_FLOW_F64_FLOPS_PER_PX)
            tf = flops / (avg_ms * 1e-3) / 1e12
            hbm = line["roofline"]
            line["roofline"] = {"bound": "valu", "kernel": kname, "achieved": round(tf, 3),
                                "peak": FP32_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s (FP32-equivalent)",
                                "frac": round(tf / FP32_VECTOR_PEAK_TFLOPS, 4),
                                "flops_per_launch": int(flops),
                                "flops_per_px_iteration": {"f32": OF_FLOW_F32_FLOPS_PER_PX,
                                                           "f64": OF_FLOW_F64_FLOPS_PER_PX},
                                "traffic": traffic, "frames_per_launch": hbm["frames_per_launch"],
                                "avg_launch_us": hbm["avg_launch_us"], "launches_timed": kn,
                                "timed_with": "feed 0 alone",
                                "hbm": {"achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": hbm["frac"], "copy": hbm.get("copy"),
                                        "algorithmic_bytes_per_launch": hbm["algorithmic_bytes_per_launch"]}}
        if cpu_base is not None:
            line["cpu_baseline"] = cpu_base
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
