"""world_size-2 gloo test of the N>1 path on CPU.

Feeds shard one per rank (``feeds.shard``) and run with no data-path
collective; the only collective is the end-of-run aggregate (sum of counters,
max of wall time) — what bench.py does over RCCL. Each rank runs REAL per-feed
work through ``feeds.run_feed`` (the product's streaming loop), with the CPU
oracle standing in for the GPU worker (this is the CPU suite). Checked:

* every feed's output digest and counters equal a single-process run of the
  same feed (sharding changes nothing);
* the all-reduced counters equal the host sum over all feeds, on both ranks.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

FEEDS = [f"synthetic://96x64?frames=9&seed={i}&noisy={i % 2}" for i in range(5)]


class OracleWorker:
    """The C oracle behind FDWorker's interface (test infrastructure only)."""

    def __init__(self, W, H):
        import oracle
        self._o = oracle.OracleFD(W, H, min_area=20)

    def prime(self, f):
        self._o.prime(f)

    def step_batch(self, frames):
        import numpy as np
        outs = [self._o.step(f) for f in frames]
        return np.stack([o[0] for o in outs]), np.stack([o[1] for o in outs])

    def stats(self):
        return self._o.stats()

    def close(self):
        self._o.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dvc_amd.feeds import run_feeds
    from tests.test_distributed import OracleWorker
    mine, agg = run_feeds(FEEDS, OracleWorker, read_ahead=4)
    q.put((rank, mine, agg))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_feeds(oracle_lib):
    from dvc_amd.feeds import STAT_KEYS, run_feed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=150) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    (r0, m0, a0), (r1, m1, a1) = res
    assert list(m0) == FEEDS[0::2] and list(m1) == FEEDS[1::2]
    single = {src: run_feed(src, OracleWorker, read_ahead=3) for src in FEEDS}   # one process, other chunking
    for src, r in {**m0, **m1}.items():
        assert r == single[src], src
    assert a0 == a1
    for k in STAT_KEYS:
        assert a0[k] == sum(single[s][k] for s in FEEDS), k
    assert a0["frames"] == 5 * 8
    assert a0["elapsed_max_s"] > 0
