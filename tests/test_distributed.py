"""world_size-2 gloo test of the N>1 path on CPU: feeds shard one per rank with
no data-path collective; the only collective is the end-of-run aggregate
(sum of counters, max of wall time), exactly what bench.py does over RCCL."""
import os
import socket

import pytest
import torch.multiprocessing as mp


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
    from dvc_amd.feeds import aggregate, dist_env, shard
    r, w, _ = dist_env()
    feeds = [f"synthetic://64x48?seed={i}" for i in range(5)]
    mine = shard(feeds, r, w)
    # per-feed work is independent; emulate per-rank counters deterministically
    stats = {"frames": 10 * len(mine), "motion_px": 1000 + r, "components": 3 * (r + 1), "static_blocks": 7}
    agg = aggregate(stats, elapsed_s=1.5 + r)
    q.put((r, mine, agg))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo_aggregate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=90) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    (r0, m0, a0), (r1, m1, a1) = res
    assert m0 == ["synthetic://64x48?seed=0", "synthetic://64x48?seed=2", "synthetic://64x48?seed=4"]
    assert m1 == ["synthetic://64x48?seed=1", "synthetic://64x48?seed=3"]
    assert a0 == a1
    assert a0["frames"] == 50 and a0["motion_px"] == 2001 and a0["components"] == 9 and a0["static_blocks"] == 14
    assert a0["elapsed_max_s"] == 2.5
