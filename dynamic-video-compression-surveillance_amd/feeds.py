"""Independent camera feeds sharded one per GPU.

The reference processes videos one after another on one worker thread
(``windows.py:142-158``). Feeds are independent — within a feed frames are
sequential through ``prev_gray``/``accumulated_mask`` (``fd:107,133``), so the
feed is the parallel unit: one process per GPU (torchrun), each process owns
the feeds ``feeds[rank::world]`` with no per-frame communication. The only
collective is an end-of-run all-reduce of a few counters (RCCL on GPUs, gloo on
CPU), plus the max-over-ranks wall time.
"""
from __future__ import annotations

import hashlib
import os
from typing import Callable, Iterable, Sequence

import numpy as np

STAT_KEYS = ("frames", "motion_px", "components", "static_blocks")


def dist_env():
    """(rank, world, local_rank) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard(items: Sequence, rank: int, world: int) -> list:
    """Round-robin shard: rank r owns items r, r+world, ... (weak scaling by feed)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(items[rank::world])


def aggregate(stats: dict, elapsed_s: float | None = None, device=None) -> dict:
    """Sum the per-rank counters and max the wall time over all ranks.

    One all-reduce of a <= 64-byte vector at the end of a run (latency-bound over
    xGMI); identity when torch.distributed is not initialised.
    """
    import torch
    import torch.distributed as dist
    vals = [float(stats.get(k, 0)) for k in STAT_KEYS]
    vec = torch.tensor(vals, dtype=torch.float64, device=device)
    t = torch.tensor([float(elapsed_s or 0.0)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = {k: int(round(v)) for k, v in zip(STAT_KEYS, vec.tolist())}
    if elapsed_s is not None:
        out["elapsed_max_s"] = float(t.item())
    return out


def reduce_runs(stats: dict, run_times: Sequence[float], rank: int, world: int, device=None) -> dict:
    """bench.py's end-of-run collective: three float64 all-reduces when a
    process group is up (RCCL on device tensors at N > 1) — the counters summed
    over ranks, each timed run's wall time maxed (the slowest rank bounds the
    run), and every rank's own frame count (a zero vector with this rank's slot
    set, summed). Identity without a process group."""
    import torch
    import torch.distributed as dist
    vec = torch.tensor([float(stats.get(k, 0)) for k in STAT_KEYS], dtype=torch.float64, device=device)
    tmax = torch.tensor([float(t) for t in run_times], dtype=torch.float64, device=device)
    per_rank = torch.zeros(max(world, 1), dtype=torch.float64, device=device)
    per_rank[rank] = float(stats.get("frames", 0))
    up = dist.is_available() and dist.is_initialized()
    if up:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)       # per run: the slowest rank's time
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)        # end-of-run aggregate stats only
        dist.all_reduce(per_rank, op=dist.ReduceOp.SUM)   # each rank's own frame count
    return {"totals": {k: float(v) for k, v in zip(STAT_KEYS, vec.tolist())},
            "run_times_max": [float(x) for x in tmax.tolist()],
            "frames_per_rank": [int(round(x)) for x in per_rank.tolist()],
            "world_size": dist.get_world_size() if up else 1,
            "backend": dist.get_backend() if up else None}


def process_feeds(video_paths: Iterable[str], output_dir: str, technique: str = "Frame Differencing",
                  **kwargs) -> list:
    """Run this rank's shard of ``video_paths`` through the reference-compatible
    driver (windows.py:144-158 picks the technique by its combo-box label).
    Returns the paths this rank processed."""
    rank, world, local = dist_env()
    os.environ.setdefault("DVC_DEVICE", str(local))
    mine = shard(list(video_paths), rank, world)
    if technique == "Frame Differencing":           # windows.py:152-154
        from .frame_differencing import process_single_video_fd as run
    elif technique == "Optical Flow":               # windows.py:149-151
        if kwargs:
            raise TypeError("process_single_video_of takes no keyword arguments (of:195)")
        from .motion_compression_opt import process_single_video_of as run
    else:
        raise ValueError(f"Unknown technique selected: {technique!r}")   # windows.py:156
    for p in mine:
        run(p, output_dir, **kwargs)
    return mine


def run_feed(source: str, make_worker: Callable, read_ahead: int = 16) -> dict:
    """Stream one feed through a per-frame worker and return its counters.

    ``make_worker(width, height)`` returns an object with ``prime(frame)``,
    ``step_batch(frames) -> (overlay, compressed)``, ``stats()`` and
    ``close()`` — an :class:`~dvc_amd.fd.FDWorker` in the product (frames
    ``read_ahead`` at a time through one ``dvc_fd_step_batch`` call). Frame 0
    primes the feed (fd:67-77); every later frame is one iteration of fd:85-138.
    The returned dict holds the worker's counters plus ``digest``, a SHA-256
    over every output frame in order, so a feed's results can be compared
    across ranks and runs without shipping the frames.
    """
    from . import video_io
    cap = video_io.open_source(source)
    if not cap.isOpened():
        raise FileNotFoundError(source)
    W = int(cap.get(video_io.CAP_PROP_FRAME_WIDTH))
    H = int(cap.get(video_io.CAP_PROP_FRAME_HEIGHT))
    ok, first = cap.read()
    if not ok:
        raise ValueError(f"{source}: no frames")
    w = make_worker(W, H)
    digest = hashlib.sha256()
    try:
        w.prime(first)
        buf = []
        while True:
            ok, f = cap.read()
            if ok:
                buf.append(f)
            if buf and (not ok or len(buf) == read_ahead):
                ov, cp = w.step_batch(np.stack(buf))
                for t in range(len(buf)):
                    digest.update(np.ascontiguousarray(ov[t]).tobytes())
                    digest.update(np.ascontiguousarray(cp[t]).tobytes())
                buf = []
            if not ok:
                break
        st = dict(w.stats())
    finally:
        cap.release()
        w.close()
    st["digest"] = digest.hexdigest()
    return st


def run_feeds(sources: Sequence[str], make_worker: Callable, read_ahead: int = 16, device=None):
    """This rank's shard of ``sources`` through :func:`run_feed`, then the one
    end-of-run collective (:func:`aggregate`). Returns (per-feed results of this
    rank, aggregate over all ranks)."""
    import time
    rank, world, _ = dist_env()
    t0 = time.perf_counter()
    mine = {src: run_feed(src, make_worker, read_ahead) for src in shard(list(sources), rank, world)}
    total = {k: sum(r[k] for r in mine.values()) for k in STAT_KEYS}
    return mine, aggregate(total, elapsed_s=time.perf_counter() - t0, device=device)
