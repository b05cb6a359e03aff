"""The multi-GPU path's RCCL code, run once on the GPU box (world size 1).

bench.py at N > 1 initialises ``init_process_group("nccl", device_id=...)``
and reduces its end-of-run counters with three float64 all-reduces on device
tensors (``feeds.reduce_runs``); ``feeds.run_feeds`` / ``feeds.aggregate`` do
the same for the drop-in feed loop. A one-GPU box cannot run two RCCL ranks,
but it can run that exact code at world size 1, so the first SCALE run cannot
be the first time the nccl init and the device all-reduces execute. The child
is a fresh interpreter (multiprocessing spawn) so its RCCL state is its own;
the parent only reads its result.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

FEEDS = ["synthetic://160x96?frames=9&seed=1&noisy=1", "synthetic://160x96?frames=7&seed=2&noisy=0"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)   # as bench.py at N > 1
        import dvc_amd
        from dvc_amd.feeds import reduce_runs, run_feeds

        def make(W, H):
            return dvc_amd.FDWorker(W, H, device=0, max_batch=4, min_area=20)
        mine, agg = run_feeds(FEEDS, make, read_ahead=4, device=dev)
        stats = {k: sum(r[k] for r in mine.values()) for k in ("frames", "motion_px", "components", "static_blocks")}
        red = reduce_runs(stats, [0.25, 0.5, 0.125], 0, 1, device=dev)
        backend = dist.get_backend()
        dist.barrier()
        dist.destroy_process_group()
        q.put(("ok", backend, {k: r["digest"] for k, r in mine.items()}, stats, agg, red))
    except Exception as e:  # reported to the parent
        import traceback
        q.put(("error", repr(e), traceback.format_exc()))


@pytest.mark.timeout(240)
def test_rccl_world_size_one(gpu_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=200)
    p.join(60)
    assert res[0] == "ok", res[1:]
    assert p.exitcode == 0
    _, backend, digests, stats, agg, red = res
    assert backend == "nccl"
    assert stats["frames"] == 8 + 6
    for k, v in stats.items():
        assert agg[k] == v, k                      # sum over one rank = identity, through RCCL
        assert red["totals"][k] == v, k
    assert red["run_times_max"] == [0.25, 0.5, 0.125]
    assert red["frames_per_rank"] == [stats["frames"]]
    assert red["world_size"] == 1 and red["backend"] == "nccl"
    # the same feeds without a process group: identical outputs
    from dvc_amd.feeds import run_feed

    def make(W, H):
        return gpu_lib.FDWorker(W, H, device=0, max_batch=3, min_area=20)
    for src in FEEDS:
        assert run_feed(src, make, read_ahead=3)["digest"] == digests[src], src
