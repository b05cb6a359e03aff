"""GPU parity of the FD graph path (fd_api.hip enqueue_graph).

Batches of device frames read in place run as one HIP graph launch each — the
same kernels, arguments and dependencies as the stage streams; a batch of
<= 128 frames runs its contour filter on its slot's own working set (grown to
the batch), a longer one on the shared set after the set's previous user. Here: every output of a run
whose calls switch between short and long graph batches and stream batches
(frames at an odd address are staged, so they take the stage streams) equals
the stream-only run (DVC_FD_GRAPH=0) and the oracle;
per-frame calls that re-use one output set (the fused front's overlap waits)
and are read back on the caller's joined stream; the accumulated-mask copy
of dvc_fd_step.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H = 640, 360


@pytest.fixture(scope="module")
def clip91():
    from dvc_amd.synthetic import clip
    return clip(W, H, 91, seed=21)


@pytest.fixture(scope="module")
def clip430():
    from dvc_amd.synthetic import clip
    return clip(W, H, 430, seed=23)


def _run(gpu_lib, clip, sizes, graph, monkeypatch, out_format="BGR", staged=()):
    import torch
    monkeypatch.setenv("DVC_FD_GRAPH", "1" if graph else "0")
    dev = torch.device("cuda", 0)
    seq = torch.from_numpy(clip).to(dev)
    n = sum(sizes)
    oshape = (n, H, W, 3) if out_format == "BGR" else (n, H * 3 // 2, W)
    ov = torch.zeros(oshape, dtype=torch.uint8, device=dev)
    cp = torch.zeros_like(ov)
    w = gpu_lib.FDWorker(W, H, device=0, device_ptrs=True, max_batch=max(sizes), out_format=out_format)
    w.prime(seq[0])
    fb = H * W * 3
    odd = torch.empty(max(sizes) * fb + 1, dtype=torch.uint8, device=dev)
    j = 0
    for i, m in enumerate(sizes):
        src = seq[1 + j:1 + j + m]
        if i in staged:   # the same frames one byte off a dword boundary
            odd[1:1 + m * fb].copy_(src.reshape(-1))
            src = (odd.data_ptr() + 1, m)
        w.step_batch(src, ov[j:j + m], cp[j:j + m])
        j += m
    w.sync()
    res = ov.cpu().numpy(), cp.cpu().numpy(), w.stats(), w.graph_stats(), w.plane(gpu_lib._native.PLANE_ACC)
    w.close()
    return res


@pytest.mark.parametrize("out_format", ["BGR", "I420"])
def test_graph_and_stream_batches_agree(gpu_lib, oracle_lib, clip430, monkeypatch, out_format):
    # 430 - 1 frames: short graph batches (own filter sets, grown 1 -> 2 -> 4 -> 8),
    # long ones (shared set: 140 after a short one, 136 after a long one, 133
    # after a stream batch), stream batches (the staged 3 and 1) after short
    # and long graph batches
    sizes = [1, 1, 2, 3, 1, 8, 140, 136, 1, 133, 2, 1]
    staged = (3, 8)
    g = _run(gpu_lib, clip430, sizes, True, monkeypatch, out_format, staged)
    s = _run(gpu_lib, clip430, sizes, False, monkeypatch, out_format, staged)
    assert sum(sizes) == len(clip430) - 1
    assert g[3]["batches"] == len(sizes) - len(staged) and s[3]["batches"] == 0
    assert 1 <= g[3]["builds"] <= g[3]["batches"]   # a graph per slot and launch shape
    assert np.array_equal(g[0], s[0]) and np.array_equal(g[1], s[1])
    assert g[2] == s[2] and np.array_equal(g[4], s[4])
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(clip430[0])
    for t in range(1, len(clip430)):
        rov, rcp, racc = ref.step(clip430[t])
        if out_format == "I420":
            rov, rcp = oracle_lib.bgr_to_i420(rov), oracle_lib.bgr_to_i420(rcp)
        assert np.array_equal(g[0][t - 1], rov), f"overlay differs at frame {t}"
        assert np.array_equal(g[1][t - 1], rcp), f"compressed differs at frame {t}"
    assert g[2] == ref.stats()
    assert np.array_equal(g[4], racc)
    ref.close()


def test_graph_per_frame_one_output_set_joined_stream(gpu_lib, oracle_lib, clip91, monkeypatch):
    """Per-frame steps into ONE output set (every fused front overwrites the
    bytes the previous frame's fix-up writes), each frame's outputs copied out
    on the caller's stream right after its call (DVC_FLAG_JOIN_STREAM), and
    the accumulated mask of every frame through dvc_fd_step's acc pointer."""
    import torch
    monkeypatch.setenv("DVC_FD_GRAPH", "1")
    dev = torch.device("cuda", 0)
    n = 24
    seq = torch.from_numpy(clip91[:n + 1]).to(dev)
    user = torch.cuda.Stream(device=dev)
    ov = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.zeros_like(ov)
    acc = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    hist = torch.zeros((n, 3, H, W, 3), dtype=torch.uint8, device=dev)
    w = gpu_lib.FDWorker(W, H, device=0, device_ptrs=True, stream=user.cuda_stream)
    with torch.cuda.stream(user):
        w.prime(seq[0])
        for t in range(n):
            w.step(seq[t + 1], ov, cp, acc=acc)
            hist[t, 0].copy_(ov)
            hist[t, 1].copy_(cp)
            hist[t, 2, :, :, 0].copy_(acc)
    user.synchronize()
    st = w.graph_stats()
    w.close()
    assert st["batches"] == n
    h = hist.cpu().numpy()
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(clip91[0])
    for t in range(n):
        rov, rcp, racc = ref.step(clip91[t + 1])
        assert np.array_equal(h[t, 0], rov), f"overlay differs at frame {t + 1}"
        assert np.array_equal(h[t, 1], rcp), f"compressed differs at frame {t + 1}"
        assert np.array_equal(h[t, 2, :, :, 0], racc), f"acc differs at frame {t + 1}"
    ref.close()


def test_graph_path_1080p_per_frame(gpu_lib, oracle_lib, monkeypatch):
    """The bench's per-frame workload at 1080p: graph calls vs the oracle."""
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(1920, 1080, 9, seed=2)
    monkeypatch.setenv("DVC_FD_GRAPH", "1")
    dev = torch.device("cuda", 0)
    seq = torch.from_numpy(frames).to(dev)
    ov = torch.zeros((8, 1080, 1920, 3), dtype=torch.uint8, device=dev)
    cp = torch.zeros_like(ov)
    w = gpu_lib.FDWorker(1920, 1080, device=0, device_ptrs=True)
    w.prime(seq[0])
    for t in range(8):
        w.step(seq[t + 1], ov[t], cp[t])
    w.sync()
    assert w.graph_stats()["batches"] == 8
    st = w.stats()
    w.close()
    ovh, cph = ov.cpu().numpy(), cp.cpu().numpy()
    ref = oracle_lib.OracleFD(1920, 1080)
    ref.prime(frames[0])
    for t in range(8):
        rov, rcp, _ = ref.step(frames[t + 1])
        assert np.array_equal(ovh[t], rov) and np.array_equal(cph[t], rcp), f"frame {t + 1}"
    assert st == ref.stats()
    ref.close()


def test_long_batches_into_one_output_set(gpu_lib, oracle_lib, clip430, monkeypatch):
    """Long batches that re-use one output set take the stage streams (their
    front waits for the previous batch's whole chain); short ones between them
    the graph path. Every frame against the oracle."""
    import torch
    monkeypatch.setenv("DVC_FD_GRAPH", "1")
    dev = torch.device("cuda", 0)
    sizes = [140, 140, 1, 2, 136]
    seq = torch.from_numpy(clip430[:sum(sizes) + 1]).to(dev)
    ov = torch.zeros((max(sizes), H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.zeros_like(ov)
    w = gpu_lib.FDWorker(W, H, device=0, device_ptrs=True, max_batch=max(sizes))
    w.prime(seq[0])
    hov, hcp, j = [], [], 0
    for m in sizes:
        w.step_batch(seq[1 + j:1 + j + m], ov[:m], cp[:m])
        w.sync()
        hov.append(ov[:m].cpu().numpy())
        hcp.append(cp[:m].cpu().numpy())
        j += m
    st, gs = w.stats(), w.graph_stats()
    w.close()
    assert gs["batches"] == 3   # the first 140 (nothing in flight overlaps), the 1 and the 2
    hov, hcp = np.concatenate(hov), np.concatenate(hcp)
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(clip430[0])
    for t in range(sum(sizes)):
        rov, rcp, _ = ref.step(clip430[t + 1])
        assert np.array_equal(hov[t], rov), f"overlay differs at frame {t + 1}"
        assert np.array_equal(hcp[t], rcp), f"compressed differs at frame {t + 1}"
    assert st == ref.stats()
    ref.close()
