"""GPU parity of the exact configurations behind the bench numbers (bench.py).

bench.py times device-pointer ``step_batch`` calls over a ping-pong sequence of
R distinct synthetic frames (FD 1080p: 383-frame launches over 766 frames; 4K:
95-frame launches over 190; OF 1080p: 16-frame launches over 126), three FD
batch slots / two OF slots and four (three) streams in flight. Here the same
sequence runs twice through that exact call pattern, and

* every output frame of the batched run equals the per-frame path's
  (``dvc_fd_step`` / ``dvc_of_step`` one frame at a time), on the device;
* the cumulative stats of both runs are equal;
* at strided frames the oracle checks one transition: it is loaded with the
  per-frame run's state before that frame (previous gray + accumulated mask;
  OF: previous gray + the raw-mask window) and steps the same frame — outputs,
  planes and the stats increment must match bit for bit. (Replaying the oracle
  over all 1532 frames would take minutes; the state hand-off checks the same
  transitions of the long run.)

Reference loop: frame_differencing.py:85-138; motion_compression_opt.py:65-101
+ 141-185.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FD_PLANES = {"motion": 1, "filtered": 2, "acc": 3, "dilated": 4}


def _pingpong(n):
    return list(range(n)) + list(range(n - 2, 0, -1))


def _sequence(W, H, R, noisy, seed, dev):
    """bench.py's device sequence: frame j of a pass is ring[order[(j+1) % P]]."""
    import torch
    from dvc_amd.synthetic import SyntheticClip
    clip = SyntheticClip(W, H, seed=seed, noisy=noisy)
    order = _pingpong(R)
    P = len(order)
    ring = [clip.frame(i) for i in range(R)]
    idx = [order[(j + 1) % P] for j in range(P)]
    seq = torch.empty((P, H, W, 3), dtype=torch.uint8, device=dev)
    for j in range(P):
        seq[j].copy_(torch.from_numpy(ring[idx[j]]), non_blocking=False)
    first = torch.from_numpy(ring[0]).to(dev)
    return ring, idx, seq, first


def _stat_delta(a, b):
    return {k: b[k] - a[k] for k in a}


@pytest.mark.parametrize("W,H,batch,noisy,stride", [
    (1920, 1080, 383, False, 97),
    (1920, 1080, 383, True, 131),
    (3840, 2160, 95, False, 47),
])
def test_fd_bench_config(gpu_lib, oracle_lib, W, H, batch, noisy, stride):
    import torch
    dev = torch.device("cuda", 0)
    R = batch + 1
    ring, idx, seq, first = _sequence(W, H, R, noisy, seed=0, dev=dev)
    P, passes = seq.shape[0], 2
    # the bench's call pattern: one step_batch per pass, launches of `batch`
    ovb = torch.empty((passes,) + tuple(seq.shape), dtype=torch.uint8, device=dev)
    cpb = torch.empty_like(ovb)
    wb = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch)
    wb.prime(first)
    for p in range(passes):
        wb.step_batch(seq, ovb[p], cpb[p])
    wb.sync()
    st_batch = wb.stats()
    wb.close()
    assert st_batch["frames"] == passes * P

    # per-frame run ordered on torch's stream (the handle joins it), so the
    # device-side comparisons below see each step's outputs
    cur = torch.cuda.current_stream(dev).cuda_stream
    wf = gpu_lib.FDWorker(W, H, device_ptrs=True, keep_planes=True, stream=cur)
    wf.prime(first)
    ov = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.empty_like(ov)
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(ring[0])                # the state before frame 0; later checks load the GPU's state
    checked = 0
    total = passes * P
    for k in range(total):
        p, j = divmod(k, P)
        check = k % stride == 0 or k == total - 1
        if check:
            st0 = wf.stats()
            if k > 0:
                gray0, acc0 = wf.plane(0), wf.plane(3)
        wf.step(seq[j], ov, cp)
        assert torch.equal(ov, ovb[p, j]), f"overlay: batched != per-frame at frame {k}"
        assert torch.equal(cp, cpb[p, j]), f"compressed: batched != per-frame at frame {k}"
        if check:
            if k > 0:
                ref.set_state(gray0, acc0)
            r0 = ref.stats()
            rov, rcp, racc = ref.step(ring[idx[j]])
            assert np.array_equal(ov.cpu().numpy(), rov), f"overlay != oracle at frame {k}"
            assert np.array_equal(cp.cpu().numpy(), rcp), f"compressed != oracle at frame {k}"
            for name, i in FD_PLANES.items():
                assert np.array_equal(wf.plane(i), ref.plane(i)), f"{name} plane != oracle at frame {k}"
            d_gpu, d_ref = _stat_delta(st0, wf.stats()), _stat_delta(r0, ref.stats())
            assert d_gpu == d_ref, (k, d_gpu, d_ref)
            checked += 1
    assert wf.stats() == st_batch
    wf.close()
    ref.close()
    assert checked >= 8


def test_of_bench_config(gpu_lib, oracle_lib):
    import torch
    dvc_amd = gpu_lib
    N = dvc_amd._native
    W, H, batch, R, stride = 1920, 1080, 126, 64, 61   # bench.py --path of defaults
    dev = torch.device("cuda", 0)
    ring, idx, seq, first = _sequence(W, H, R, False, seed=0, dev=dev)
    P, passes = seq.shape[0], 2
    mkb = torch.empty((passes, P, H, W), dtype=torch.uint8, device=dev)
    cpb = torch.empty((passes,) + tuple(seq.shape), dtype=torch.uint8, device=dev)
    wb = dvc_amd.OFWorker(W, H, device_ptrs=True, max_batch=batch)
    wb.prime(first)
    for p in range(passes):
        wb.step_batch(seq, mkb[p], cpb[p])
    wb.sync()
    st_batch = wb.stats()
    wb.close()

    wf = dvc_amd.OFWorker(W, H, device_ptrs=True, keep_planes=True, stream=torch.cuda.current_stream(dev).cuda_stream)
    wf.prime(first)
    mk = torch.empty((H, W), dtype=torch.uint8, device=dev)
    cp = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
    ref = oracle_lib.OracleOF(W, H)
    ref.prime(ring[0])                # the state before frame 0; later checks load the GPU's state
    window = []                       # raw |flow| masks of the last frames (the deque, of:84)
    gray = None
    total, checked = passes * P, 0
    for k in range(total):
        p, j = divmod(k, P)
        check = k % stride == 0 or k == total - 1
        gray0 = gray
        wf.step(seq[j], mk, cp)
        assert torch.equal(mk, mkb[p, j]), f"mask: batched != per-frame at frame {k}"
        assert torch.equal(cp, cpb[p, j]), f"compressed: batched != per-frame at frame {k}"
        if check:
            if k > 0:
                ref.set_state(gray0, np.stack(window[-30:]))
            rmk, rcp, rflow = ref.step(ring[idx[j]])
            assert np.array_equal(wf.flow().view(np.uint32), rflow.view(np.uint32)), f"flow != oracle at frame {k}"
            assert np.array_equal(mk.cpu().numpy(), rmk), f"mask != oracle at frame {k}"
            assert np.array_equal(cp.cpu().numpy(), rcp), f"compressed != oracle at frame {k}"
            checked += 1
        window.append(wf.plane(N.OF_PLANE_RAW))
        window = window[-30:]
        gray = wf.plane(N.OF_PLANE_GRAY)
    assert wf.stats() == st_batch
    wf.close()
    ref.close()
    assert checked >= 5


def test_fd_headline_launch_every_frame_vs_oracle(gpu_lib, oracle_lib):
    """The headline launch itself, every frame: one 383-frame dvc_fd_step_batch
    of bench.py's 1080p sequence (configs[1], device frames, one graph
    launch) against a sequential oracle replay of the same 383 frames —
    overlay and compressed frame bit for bit at every frame, and the stats.
    (~45 s of oracle time on one core; the strided transition checks above
    cover the second pass and the other configurations.)"""
    import torch
    dev = torch.device("cuda", 0)
    W, H, batch = 1920, 1080, 383
    ring, idx, seq, first = _sequence(W, H, batch + 1, False, seed=0, dev=dev)
    ov = torch.empty((batch, H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.empty_like(ov)
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch)
    w.prime(first)
    w.step_batch(seq[:batch], ov, cp)
    w.sync()
    st = w.stats()
    assert w.graph_stats()["batches"] == 1       # one graph launch (the shared contour-filter set)
    w.close()
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(ring[0])
    for t in range(batch):
        rov, rcp, _ = ref.step(ring[idx[t]])
        assert np.array_equal(ov[t].cpu().numpy(), rov), f"overlay != oracle at frame {t}"
        assert np.array_equal(cp[t].cpu().numpy(), rcp), f"compressed != oracle at frame {t}"
    assert st == ref.stats()
    ref.close()
