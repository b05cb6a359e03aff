"""BASELINE.json configs[3] — 8 independent 1920x1080 feeds, one per GPU — run
as its unit on one GPU: 8 FD handles (seeds 0..7, the bench's device pointers
and 383-frame launches, ~8 GB of scratch each) driven concurrently from 8 host
threads, two passes of 766 frames each (4 launches per feed).

SURVEY.md §4.5: every feed's outputs must equal its 1-GPU run of the same
seed, and the aggregate stats must equal the per-feed sum.

* concurrent run: per-frame 64-bit digests of both outputs (computed on the
  device: a weighted sum of the frame's 64-bit words with odd weights, so any
  single changed word changes it) and the per-feed stats;
* isolated run of each feed afterwards, alone on the GPU and in differently
  sized calls (batch boundaries moved): the same digests and stats;
* at strided frames of the isolated run the oracle checks one transition, loaded
  with the handle's state before it (previous blurred gray + accumulated mask,
  fd:107,133 — the hand-off tests/test_bench_config.py uses): outputs, planes and
  the stats increment bit for bit.

Reference: feeds run one after another in windows.py:144-158; the per-feed state
is fd:107,133; the per-frame loop fd:85-138.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, BATCH, RING, FEEDS, PASSES = 1920, 1080, 383, 128, 8, 2
P = 2 * BATCH          # frames per pass (bench.py: 766 at 1080p)
FD_PLANES = {"motion": 1, "filtered": 2, "acc": 3, "dilated": 4}


def _pingpong(n):
    return list(range(n)) + list(range(n - 2, 0, -1))


def _feed(seed, dev):
    """Feed `seed`: RING distinct synthetic frames played ping-pong into a P-frame
    device sequence (every consecutive pair is real motion), as bench.py does."""
    import torch
    from dvc_amd.synthetic import SyntheticClip
    clip = SyntheticClip(W, H, seed=seed)
    order = _pingpong(RING)
    idx = [order[(j + 1) % len(order)] for j in range(P)]
    ring = torch.empty((RING, H, W, 3), dtype=torch.uint8, device=dev)
    for i in range(RING):
        ring[i].copy_(torch.from_numpy(clip.frame(i)))
    seq = ring[torch.tensor(idx, device=dev)].contiguous()
    first = ring[0].clone()
    del ring
    return clip, idx, seq, first


_WEIGHTS = {}


def _digests(x):
    """Per-frame 64-bit digests of (n, H, W, 3) uint8 device frames."""
    import torch
    n = x.shape[0]
    words = x.reshape(n, -1).view(torch.int64)
    key = (words.shape[1], x.device)
    if key not in _WEIGHTS:
        g = torch.Generator(device="cpu").manual_seed(1234)
        w = torch.randint(-(2 ** 62), 2 ** 62, (words.shape[1],), generator=g, dtype=torch.int64) * 2 + 1
        _WEIGHTS[key] = w.to(x.device)
    w = _WEIGHTS[key]
    out = []
    for a in range(0, n, 64):
        out.append((words[a:a + 64] * w).sum(dim=1))   # wraps mod 2^64
    return torch.cat(out).cpu().tolist()


def test_config4_eight_1080p_feeds_on_one_gpu(gpu_lib, oracle_lib):
    import torch
    dev = torch.device("cuda", 0)
    feeds = {s: _feed(s, dev) for s in range(FEEDS)}
    ov = {s: torch.empty((P, H, W, 3), dtype=torch.uint8, device=dev) for s in range(FEEDS)}
    cp = {s: torch.empty_like(ov[s]) for s in range(FEEDS)}

    # ---- concurrent: one handle and one host thread per feed
    conc, errs = {}, []
    barrier = threading.Barrier(FEEDS)

    def work(s):
        try:
            _, _, seq, first = feeds[s]
            w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=BATCH)
            w.prime(first)
            barrier.wait(timeout=60)            # all handles exist: the passes overlap
            dig = []
            for _ in range(PASSES):
                w.step_batch(seq, ov[s], cp[s])
                w.sync()
                dig.append((_digests(ov[s]), _digests(cp[s])))
            conc[s] = (dig, w.stats())
            w.close()
        except Exception as e:   # surfaced below
            errs.append((s, repr(e)))
            try:
                barrier.abort()
            except Exception:
                pass

    ths = [threading.Thread(target=work, args=(s,)) for s in range(FEEDS)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not errs, errs
    assert sorted(conc) == list(range(FEEDS))

    # ---- isolated: each feed alone, call boundaries moved, oracle at strided frames
    total = {k: 0 for k in ("frames", "motion_px", "components", "static_blocks")}
    for s in range(FEEDS):
        clip, idx, seq, first = feeds[s]
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=BATCH, keep_planes=True)
        w.prime(first)
        ref = oracle_lib.OracleFD(W, H)
        checks = sorted({(97 * (s + 1)) % (P - 2) + 1, P - 1 - 13 * s})   # two frames per pass, per feed
        dig = []
        for p in range(PASSES):
            a = 0
            for k in checks:
                if k > a:
                    w.step_batch(seq[a:k], ov[s][a:k], cp[s][a:k])
                st0 = w.stats()
                gray0, acc0 = w.plane(0), w.plane(3)
                w.step_batch(seq[k:k + 1], ov[s][k:k + 1], cp[s][k:k + 1])
                ref.set_state(gray0, acc0)
                r0 = ref.stats()
                rov, rcp, _ = ref.step(clip.frame(idx[k]))
                assert np.array_equal(ov[s][k].cpu().numpy(), rov), f"feed {s} pass {p} frame {k}: overlay != oracle"
                assert np.array_equal(cp[s][k].cpu().numpy(), rcp), f"feed {s} pass {p} frame {k}: compressed"
                for name, i in FD_PLANES.items():
                    assert np.array_equal(w.plane(i), ref.plane(i)), f"feed {s} frame {k}: {name} plane"
                d_gpu = {q: v - st0[q] for q, v in w.stats().items()}
                d_ref = {q: v - r0[q] for q, v in ref.stats().items()}
                assert d_gpu == d_ref, (s, k, d_gpu, d_ref)
                a = k + 1
            if a < P:
                w.step_batch(seq[a:], ov[s][a:], cp[s][a:])
            w.sync()
            dig.append((_digests(ov[s]), _digests(cp[s])))
        st = w.stats()
        w.close()
        ref.close()
        for p in range(PASSES):
            for what, i in (("overlay", 0), ("compressed", 1)):
                bad = [j for j, (x, y) in enumerate(zip(conc[s][0][p][i], dig[p][i])) if x != y]
                assert not bad, f"feed {s} pass {p}: {what} differs from its isolated run at frames {bad[:5]}"
        assert conc[s][1] == st, (s, conc[s][1], st)
        assert st["frames"] == PASSES * P
        for k in total:
            total[k] += st[k]
    # the aggregate the bench all-reduces (feeds.aggregate: identity without a process group)
    from dvc_amd.feeds import aggregate
    agg = aggregate({k: sum(conc[s][1][k] for s in conc) for k in total})
    assert agg == total, (agg, total)
    assert total["frames"] == FEEDS * PASSES * P
