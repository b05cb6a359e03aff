"""Several feeds on one GPU (BASELINE config 4's feed-per-stream unit; SURVEY §4.5,
§8e) and stream-ordered use of a handle.

* 4 FD handles driven concurrently from 4 host threads (ctypes releases the
  GIL), host and device mode mixed, one of them on a caller-supplied stream:
  every feed's outputs and stats equal its isolated run, and the isolated runs
  equal the oracle — concurrency changes nothing.
* determinism of the contour filter's atomics: the same feed on 3 handles at
  once gives identical outputs, labels' effects and stats.
* a device-pointer run ordered only by the caller's stream: the frames are
  produced by copies on that stream and the outputs consumed by copies on it,
  with no host synchronisation in between (dvc_fd_create's stream contract).
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, NF = 640, 360, 24


def _clip(seed):
    from dvc_amd.synthetic import clip
    return clip(W, H, NF, seed=seed, noisy=seed % 2 == 1)


def _oracle(oracle, frames):
    ref = oracle.OracleFD(W, H)
    ref.prime(frames[0])
    ov, cp = [], []
    for f in frames[1:]:
        o, c, _ = ref.step(f)
        ov.append(o)
        cp.append(c)
    st = ref.stats()
    ref.close()
    return np.stack(ov), np.stack(cp), st


def _host_feed(dvc_amd, frames, chunk=5):
    w = dvc_amd.FDWorker(W, H, max_batch=4)
    w.prime(frames[0])
    ovs, cps = [], []
    for a in range(1, len(frames), chunk):
        ov, cp = w.step_batch(frames[a:a + chunk])
        ovs.append(ov)
        cps.append(cp)
    st = w.stats()
    w.close()
    return np.concatenate(ovs), np.concatenate(cps), st


def _device_feed(dvc_amd, frames, stream=None):
    import torch
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(frames).to(dev)
    ov = torch.empty_like(d[1:])
    cp = torch.empty_like(d[1:])
    w = dvc_amd.FDWorker(W, H, device_ptrs=True, max_batch=6,
                         stream=stream.cuda_stream if stream is not None else None)
    w.prime(d[0])
    for a in range(0, NF - 1, 7):
        b = min(NF - 1, a + 7)
        w.step_batch(d[1 + a:1 + b], ov[a:b], cp[a:b])
    w.sync()
    st = w.stats()
    w.close()
    return ov.cpu().numpy(), cp.cpu().numpy(), st


def test_concurrent_feeds(gpu_lib, oracle_lib):
    import torch
    seeds = [0, 1, 2, 3]
    clips = {s: _clip(s) for s in seeds}
    runners = {0: lambda f: _host_feed(gpu_lib, f), 1: lambda f: _device_feed(gpu_lib, f),
               2: lambda f: _host_feed(gpu_lib, f, chunk=23),
               3: lambda f: _device_feed(gpu_lib, f, stream=torch.cuda.Stream(device=0))}
    iso = {s: runners[s](clips[s]) for s in seeds}
    for s in seeds:
        rov, rcp, rst = _oracle(oracle_lib, clips[s])
        assert np.array_equal(iso[s][0], rov) and np.array_equal(iso[s][1], rcp), f"feed {s} != oracle"
        assert iso[s][2] == rst, (s, iso[s][2], rst)
    out, errs = {}, []

    def work(s):
        try:
            out[s] = runners[s](clips[s])
        except Exception as e:  # surfaced below
            errs.append((s, repr(e)))

    for _ in range(2):
        ths = [threading.Thread(target=work, args=(s,)) for s in seeds]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=100)
        assert not errs, errs
        for s in seeds:
            assert np.array_equal(out[s][0], iso[s][0]), f"feed {s}: overlay differs under concurrency"
            assert np.array_equal(out[s][1], iso[s][1]), f"feed {s}: compressed differs under concurrency"
            assert out[s][2] == iso[s][2], (s, out[s][2], iso[s][2])


def test_contour_filter_deterministic(gpu_lib):
    """Same noisy feed on 3 handles concurrently: identical outputs and stats
    (the union-find atomics may race in order, never in result)."""
    frames = _clip(5)
    res, errs = [None] * 3, []

    def work(i):
        try:
            res[i] = _device_feed(gpu_lib, frames)
        except Exception as e:
            errs.append(repr(e))

    ths = [threading.Thread(target=work, args=(i,)) for i in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not errs, errs
    for r in res[1:]:
        assert np.array_equal(r[0], res[0][0]) and np.array_equal(r[1], res[0][1]) and r[2] == res[0][2]


def test_caller_stream_ordering(gpu_lib):
    """Frames written by copies on the caller's stream, outputs read back by
    copies on it; one reused device frame buffer, no host sync until the end."""
    import torch
    frames = _clip(2)
    host = gpu_lib.FDWorker(W, H)
    host.prime(frames[0])
    want = [host.step(f) for f in frames[1:]]
    host.close()
    pinned = torch.from_numpy(frames).pin_memory()
    s = torch.cuda.Stream(device=0)
    with torch.cuda.stream(s):
        dframe = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        ov = torch.empty_like(dframe)
        cp = torch.empty_like(dframe)
        got_ov = torch.empty((NF - 1, H, W, 3), dtype=torch.uint8, device="cuda:0")
        got_cp = torch.empty_like(got_ov)
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, stream=s.cuda_stream)
        dframe.copy_(pinned[0], non_blocking=True)
        w.prime(dframe)
        for t in range(1, NF):
            dframe.copy_(pinned[t], non_blocking=True)     # WAR on the previous step's input
            w.step(dframe, ov, cp)
            got_ov[t - 1].copy_(ov)                         # RAW on this step's outputs
            got_cp[t - 1].copy_(cp)
    s.synchronize()
    w.close()
    for t in range(NF - 1):
        assert np.array_equal(got_ov[t].cpu().numpy(), want[t][0]), f"overlay differs at {t + 1}"
        assert np.array_equal(got_cp[t].cpu().numpy(), want[t][1]), f"compressed differs at {t + 1}"


def test_device_mode_rejects_bad_buffers(gpu_lib):
    """Sliced / wrongly typed / short device buffers are refused before the C-ABI."""
    import torch
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=2)
    f = torch.zeros((3, H, W, 3), dtype=torch.uint8, device="cuda:0")
    w.prime(f[0])
    with pytest.raises(ValueError):
        w.step(f[0].permute(1, 0, 2), f[1], f[2])             # wrong shape
    with pytest.raises(ValueError):
        w.step(f[0, :, ::2], f[1], f[2])                      # not contiguous
    with pytest.raises(ValueError):
        w.step(f[0].float(), f[1], f[2])                      # dtype
    with pytest.raises(ValueError):
        w.step_batch(f, f[:2], f)                             # output holds 2 of 3 frames
    with pytest.raises(TypeError):
        w.step(int(f[0].data_ptr()), f[1], f[2])              # bare address: not an explicit opt-in
    with pytest.raises(ValueError):
        w.step(f[0].cpu(), f[1], f[2])                        # host tensor in device mode
    w.close()


def test_fd_handle_footprint(gpu_lib):
    """A 1080p FD handle at the bench's max_batch (383) stays under 10 GB of HBM:
    bit planes for three batches in flight, one contour-filter working set
    (its batches run one after another on the handle's stream) — several feeds
    per GPU fit (VERDICT r1 'what's weak' #7 measured ~22 GB)."""
    import torch
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    w = gpu_lib.FDWorker(1920, 1080, device=0, device_ptrs=True, max_batch=383)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    w.close()
    used = free0 - free1
    assert 1e9 < used < 10e9, f"handle footprint {used / 1e9:.2f} GB"
