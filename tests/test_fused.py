"""GPU parity of the fused front (fd_kernels.h FrontOut) against the one-pass
output stage, through the C-ABI.

With block_size 4 and BGR or I420 outputs (BGR or 4:2:0 input), k_front writes every full 4x4
block of both outputs as if it were static (overlay = the frame, compressed =
(Y', Y', Y') of the quantised DCT, frame_differencing.py:110-130) while it has
the frame in registers, and k_fix4 rewrites the blocks the accumulated mask
makes non-static. The bytes must equal the unfused k_out pass
(DVC_FLAG_FD_UNFUSED) and the oracle, including when a caller reuses output
buffers across calls — a later batch's speculative stores must not land
before an earlier batch's k_fix4 of the same bytes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames_dev(W, H, n, seed, noisy, dev):
    import torch
    from dvc_amd.synthetic import clip
    fr = clip(W, H, n, seed=seed, noisy=noisy)
    return fr, torch.from_numpy(fr).to(dev)


@pytest.mark.parametrize("W,H,n,batch,seed,noisy", [
    (1920, 1080, 121, 40, 3, False),
    (640, 360, 61, 20, 4, True),
    (644, 362, 41, 13, 5, False),     # partial edge blocks: k_out_gen beside the fused front
    (1000, 200, 33, 32, 6, True),     # W % 256 != 0: tiles that run past the frame's right edge
])
def test_fused_equals_unfused(gpu_lib, W, H, n, batch, seed, noisy):
    """Every output frame of the fused path == the one-pass k_out path, batched."""
    import torch
    dev = torch.device("cuda", 0)
    _, seq = _frames_dev(W, H, n, seed, noisy, dev)
    outs = {}
    for fused in (True, False):
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch, fused=fused, ktiming=True)
        w.prime(seq[0])
        ov = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device=dev)
        cp = torch.empty_like(ov)
        w.step_batch(seq[1:], ov, cp)
        w.sync()
        assert w.ktime_kernel() == ("k_front_fused" if fused else "k_out")
        outs[fused] = (ov, cp, w.stats())
        w.close()
    (ovf, cpf, sf), (ovu, cpu_, su) = outs[True], outs[False]
    assert sf == su
    for t in range(n - 1):
        assert torch.equal(ovf[t], ovu[t]), f"overlay: fused != unfused at frame {t + 1}"
        assert torch.equal(cpf[t], cpu_[t]), f"compressed: fused != unfused at frame {t + 1}"


@pytest.mark.parametrize("W,H,SW,SH,n,batch,seed,noisy", [
    (960, 540, 1920, 1080, 33, 16, 11, False),   # fd:200-207: b=8, k=10, r=0.3, scale 0.5 (resized on the GPU)
    (1920, 1080, 0, 0, 25, 12, 12, True),
    (652, 364, 0, 0, 31, 10, 13, False),          # partial 8x8 edge blocks: k_out_gen beside the fused front
    (1000, 200, 0, 0, 21, 20, 14, True),          # tiles past the right edge
])
def test_fused_b8_equals_unfused(gpu_lib, W, H, SW, SH, n, batch, seed, noisy, monkeypatch):
    """block_size 8 (the reference's __main__ variant, fd:200-207): the fused
    front writes every full 8x8 block as static (4 lanes a block, k_front
    OB = 8) and k_out<8>'s per-block pass rewrites the non-static ones; every
    output frame == the one-pass k_out<8> path. (Opt-in: DVC_FD_FUSED8=1 when
    the handle is created.)"""
    import torch
    monkeypatch.setenv("DVC_FD_FUSED8", "1")
    dev = torch.device("cuda", 0)
    sw, sh = (SW, SH) if SW else (W, H)
    _, seq = _frames_dev(sw, sh, n, seed, noisy, dev)
    kw = dict(block_size=8, kernel_size=10, release_factor=0.3)
    if SW:
        kw.update(src_width=SW, src_height=SH)
    outs = {}
    for fused in (True, False):
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch, fused=fused, ktiming=True, **kw)
        w.prime(seq[0])
        ov = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device=dev)
        cp = torch.empty_like(ov)
        w.step_batch(seq[1:], ov, cp)
        w.sync()
        assert w.ktime_kernel() == ("k_front_fused" if fused else "k_out")
        outs[fused] = (ov, cp, w.stats())
        w.close()
    (ovf, cpf, sf), (ovu, cpu_, su) = outs[True], outs[False]
    assert sf == su
    for t in range(n - 1):
        assert torch.equal(ovf[t], ovu[t]), f"overlay: fused != unfused at frame {t + 1}"
        assert torch.equal(cpf[t], cpu_[t]), f"compressed: fused != unfused at frame {t + 1}"


def test_fused_b8_matches_oracle(gpu_lib, oracle_lib, monkeypatch):
    """The fused 8x8 path frame by frame against the CPU oracle (fd:200-207 kwargs)."""
    from dvc_amd.synthetic import clip
    monkeypatch.setenv("DVC_FD_FUSED8", "1")
    W, H, n = 640, 360, 9
    frames = clip(W, H, n, seed=21, noisy=True)
    kw = dict(block_size=8, kernel_size=10, release_factor=0.3)
    gpu = gpu_lib.FDWorker(W, H, **kw)
    ref = oracle_lib.OracleFD(W, H, **kw)
    gpu.prime(frames[0])
    ref.prime(frames[0])
    for t in range(1, n):
        ov, cp = gpu.step(frames[t])
        rov, rcp, _ = ref.step(frames[t])
        assert np.array_equal(ov, rov), f"overlay differs at frame {t}"
        assert np.array_equal(cp, rcp), f"compressed differs at frame {t}"
    assert gpu.stats() == ref.stats()
    gpu.close()
    ref.close()


def test_fused_one_output(gpu_lib):
    """Only one of the outputs requested: the other pointer is NULL in both kernels."""
    import torch
    dev = torch.device("cuda", 0)
    W, H, n = 640, 360, 25
    _, seq = _frames_dev(W, H, n, 8, False, dev)
    ref = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=8, fused=False)
    ref.prime(seq[0])
    rov = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device=dev)
    rcp = torch.empty_like(rov)
    ref.step_batch(seq[1:], rov, rcp)
    ref.sync()
    ref.close()
    for which in ("overlay", "compressed"):
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=8)
        w.prime(seq[0])
        out = torch.empty_like(rov)
        if which == "overlay":
            w.step_batch(seq[1:], out, None)
        else:
            w.step_batch(seq[1:], None, out)
        w.sync()
        w.close()
        assert torch.equal(out, rov if which == "overlay" else rcp), which


def test_fused_reused_output_buffers(gpu_lib, oracle_lib):
    """The bench's pattern and a ring-buffer caller's: chunks of frames stepped
    into TWO output buffers in turn with no sync between calls, so batch k
    writes the bytes batch k-2 wrote (and its k_fix rewrote). Different motion
    in every chunk: a stale k_fix landing after the next speculative stores
    would leave non-static blocks of the wrong frame. The final contents of both
    buffers must equal the per-frame unfused run and the oracle."""
    import torch
    dev = torch.device("cuda", 0)
    W, H, chunk, chunks = 640, 360, 9, 7
    n = 1 + chunk * chunks
    frames, seq = _frames_dev(W, H, n, 9, True, dev)
    ring = [(torch.empty((chunk, H, W, 3), dtype=torch.uint8, device=dev),
             torch.empty((chunk, H, W, 3), dtype=torch.uint8, device=dev)) for _ in range(2)]
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=chunk)
    w.prime(seq[0])
    for c in range(chunks):
        ov, cp = ring[c % 2]
        w.step_batch(seq[1 + c * chunk:1 + (c + 1) * chunk], ov, cp)
    w.sync()
    w.close()
    # reference: the oracle frame by frame; the last two chunks' outputs
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(frames[0])
    last = {}
    for t in range(1, n):
        rov, rcp, _ = ref.step(frames[t])
        c, j = divmod(t - 1, chunk)
        if c >= chunks - 2:
            last[(c, j)] = (rov, rcp)
    ref.close()
    for (c, j), (rov, rcp) in last.items():
        ov, cp = ring[c % 2]
        assert np.array_equal(ov[j].cpu().numpy(), rov), f"overlay != oracle: chunk {c} frame {j}"
        assert np.array_equal(cp[j].cpu().numpy(), rcp), f"compressed != oracle: chunk {c} frame {j}"


@pytest.mark.parametrize("fmt", ["NV12", "I420"])
def test_fused_yuv_surfaces(gpu_lib, oracle_lib, fmt):
    """4:2:0 decoder surfaces read in place: the fused front converts each
    block's quads once (gray and overlay) and k_fix4 converts the non-static
    blocks it rewrites; every byte equals the one-pass path's."""
    import ctypes
    import torch
    from dvc_amd.synthetic import clip
    from tests.test_video_io_gpu import _nv12, _surface
    N = gpu_lib._native
    W, H, pitch, crows, n, batch = 1280, 720, 1408, 736, 41, 20
    frames = clip(W, H, n, seed=12, noisy=True)
    i420 = np.stack([oracle_lib.bgr_to_i420(f) for f in frames])
    surf = np.stack([_surface(f if fmt == "I420" else _nv12(f, H, W), H, W, fmt, pitch, crows) for f in i420])
    d = torch.from_numpy(surf).cuda()
    L = N.lib()
    outs = {}
    for fused in (True, False):
        p = gpu_lib.fd.derive_params(W, H, in_format=fmt, chroma_rows=crows,
                                     flags=N.DVC_FLAG_DEVICE_PTRS | N.DVC_FLAG_KTIMING |
                                     (0 if fused else N.DVC_FLAG_FD_UNFUSED))
        p.max_batch = batch
        ov = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device="cuda")
        cp = torch.empty_like(ov)
        h = ctypes.c_void_p()
        N.check(L.dvc_fd_create(ctypes.byref(p), 0, None, ctypes.byref(h)))
        try:
            N.check(L.dvc_fd_prime(h, d[0].data_ptr(), pitch))
            N.check(L.dvc_fd_step_batch(h, d[1].data_ptr(), pitch, surf[0].nbytes, n - 1, ov.data_ptr(),
                                        cp.data_ptr(), 3 * W * H))
            N.check(L.dvc_fd_sync(h))
            kk = L.dvc_fd_ktime_kernel(h)
        finally:
            L.dvc_fd_destroy(h)
        assert kk == (N.KTIME_FRONT_FUSED if fused else N.KTIME_OUT)
        outs[fused] = (ov, cp)
    for t in range(n - 1):
        assert torch.equal(outs[True][0][t], outs[False][0][t]), f"overlay: fused != unfused at frame {t + 1}"
        assert torch.equal(outs[True][1][t], outs[False][1][t]), f"compressed: fused != unfused at frame {t + 1}"


def test_fused_nv12_per_frame_partial_rows(gpu_lib, oracle_lib):
    """NV12 surfaces stepped one frame a call (dvc_fd_step: one-frame batches of
    the fused front) with H % 4 = 2 (the last block row partial: k_out_gen beside
    k_fix4) and the same two output frames reused every call — each call's
    speculative stores wait for the previous call's fix-up — against the oracle
    on the converted frames."""
    import ctypes
    import torch
    from dvc_amd.synthetic import clip
    from tests.test_video_io_gpu import _nv12, _oracle_run, _surface
    N = gpu_lib._native
    W, H, pitch, crows, n = 640, 362, 704, 368, 9
    frames = clip(W, H, n, seed=14, noisy=True)
    i420 = np.stack([oracle_lib.bgr_to_i420(f) for f in frames])
    bgr = np.stack([oracle_lib.yuv420_to_bgr(f) for f in i420])
    outs, _ = _oracle_run(oracle_lib, bgr, W, H)
    surf = np.stack([_surface(_nv12(f, H, W), H, W, "NV12", pitch, crows) for f in i420])
    d = torch.from_numpy(surf).cuda()
    p = gpu_lib.fd.derive_params(W, H, in_format="NV12", chroma_rows=crows,
                                 flags=N.DVC_FLAG_DEVICE_PTRS | N.DVC_FLAG_KTIMING)
    L = N.lib()
    h = ctypes.c_void_p()
    N.check(L.dvc_fd_create(ctypes.byref(p), 0, None, ctypes.byref(h)))
    ov = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    cp = torch.empty_like(ov)
    try:
        N.check(L.dvc_fd_prime(h, d[0].data_ptr(), pitch))
        for t in range(1, n):
            N.check(L.dvc_fd_step(h, d[t].data_ptr(), pitch, ov.data_ptr(), cp.data_ptr(), None))
            N.check(L.dvc_fd_sync(h))
            assert L.dvc_fd_ktime_kernel(h) == N.KTIME_FRONT_FUSED
            assert np.array_equal(ov.cpu().numpy(), outs[t - 1][0]), f"overlay differs at frame {t}"
            assert np.array_equal(cp.cpu().numpy(), outs[t - 1][1]), f"compressed differs at frame {t}"
    finally:
        L.dvc_fd_destroy(h)


def test_fused_nv12_bench_scale(gpu_lib, oracle_lib):
    """The NV12 bench configuration (1080p, 383-frame launches, two launches a
    call, two calls into the same outputs): the fused front's outputs and stats
    equal the one-pass path's (itself pinned against the oracle by
    test_video_io_gpu.py) over 1532 frames."""
    import ctypes
    import torch
    from dvc_amd.synthetic import clip
    from tests.test_video_io_gpu import _nv12
    N = gpu_lib._native
    W, H, R, batch = 1920, 1080, 48, 383
    frames = clip(W, H, R, seed=3)
    nv = np.stack([_nv12(oracle_lib.bgr_to_i420(f), H, W) for f in frames])   # (R, 1.5H, W)
    order = list(range(R)) + list(range(R - 2, 0, -1))
    P = 766
    idx = torch.tensor([order[(j + 1) % len(order)] for j in range(P)], device="cuda")
    ring = torch.from_numpy(nv).cuda()
    seq = ring[idx].contiguous()
    L = N.lib()
    outs = {}
    for fused in (True, False):
        p = gpu_lib.fd.derive_params(W, H, in_format="NV12", chroma_rows=H,
                                     flags=N.DVC_FLAG_DEVICE_PTRS | (0 if fused else N.DVC_FLAG_FD_UNFUSED))
        p.max_batch = batch
        ov = torch.empty((P, H, W, 3), dtype=torch.uint8, device="cuda")
        cp = torch.empty_like(ov)
        h = ctypes.c_void_p()
        N.check(L.dvc_fd_create(ctypes.byref(p), 0, None, ctypes.byref(h)))
        try:
            N.check(L.dvc_fd_prime(h, ring[0].data_ptr(), W))
            for _ in range(2):
                N.check(L.dvc_fd_step_batch(h, seq.data_ptr(), W, nv[0].nbytes, P, ov.data_ptr(), cp.data_ptr(),
                                            3 * W * H))
            N.check(L.dvc_fd_sync(h))
            st = N.FdStats()
            N.check(L.dvc_fd_get_stats(h, ctypes.byref(st)))
        finally:
            L.dvc_fd_destroy(h)
        outs[fused] = (ov, cp, {k: int(getattr(st, k)) for k, _ in st._fields_})
    assert outs[True][2] == outs[False][2]
    for t in range(P):
        assert torch.equal(outs[True][0][t], outs[False][0][t]), f"overlay: fused != unfused at frame {t}"
        assert torch.equal(outs[True][1][t], outs[False][1][t]), f"compressed: fused != unfused at frame {t}"
    del outs, seq, ring


@pytest.mark.parametrize("W,H,n,batch,seed,noisy,fmt", [
    (1920, 1080, 61, 20, 21, False, "BGR"),
    (640, 360, 41, 13, 22, True, "BGR"),
    (1000, 200, 21, 20, 24, True, "BGR"),      # tiles past the right edge
    (1280, 720, 25, 12, 25, True, "NV12"),     # 4:2:0 surfaces read in place
    (648, 360, 21, 8, 26, False, "I420"),
])
def test_fused_i420_outputs_equal_unfused(gpu_lib, oracle_lib, W, H, n, batch, seed, noisy, fmt):
    """DVC_FLAG_OUT_I420 on the fused front: k_front writes every 4x4 block of
    both outputs as BGR2YUV_I420 of the static form (overlay = the frame,
    compressed = (Y', Y', Y') -> U = V = 128) and k_fix4 rewrites the
    non-static blocks as I420; every byte equals the one-pass k_out path."""
    import torch
    from dvc_amd.synthetic import clip
    from tests.test_video_io_gpu import _nv12
    dev = torch.device("cuda", 0)
    frames = clip(W, H, n, seed=seed, noisy=noisy)
    if fmt == "BGR":
        src = frames
    else:
        i420 = np.stack([oracle_lib.bgr_to_i420(f) for f in frames])
        src = i420 if fmt == "I420" else np.stack([_nv12(f, H, W) for f in i420])
    seq = torch.from_numpy(np.ascontiguousarray(src)).to(dev)
    outs = {}
    for fused in (True, False):
        w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch, fused=fused, ktiming=True, in_format=fmt,
                             out_format="I420")
        w.prime(seq[0])
        ov = torch.empty((n - 1, H * 3 // 2, W), dtype=torch.uint8, device=dev)
        cp = torch.empty_like(ov)
        for b0 in range(1, n, batch):
            b1 = min(n, b0 + batch)
            w.step_batch(seq[b0:b1], ov[b0 - 1:b1 - 1], cp[b0 - 1:b1 - 1])
        w.sync()
        assert w.ktime_kernel() == ("k_front_fused" if fused else "k_out")
        outs[fused] = (ov, cp, w.stats())
        w.close()
    (ovf, cpf, sf), (ovu, cpu_, su) = outs[True], outs[False]
    assert sf == su
    for t in range(n - 1):
        assert torch.equal(ovf[t], ovu[t]), f"overlay (I420): fused != unfused at frame {t + 1}"
        assert torch.equal(cpf[t], cpu_[t]), f"compressed (I420): fused != unfused at frame {t + 1}"


def test_fused_i420_outputs_match_oracle(gpu_lib, oracle_lib):
    """The fused I420 outputs at the bench's launch size against the oracle's
    BGR outputs converted by the oracle's BGR2YUV_I420 (fd:112,131)."""
    import torch
    from dvc_amd.synthetic import clip
    W, H, n = 1920, 1080, 9
    frames = clip(W, H, n, seed=27, noisy=True)
    dev = torch.device("cuda", 0)
    seq = torch.from_numpy(frames).to(dev)
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=n - 1, out_format="I420", ktiming=True)
    w.prime(seq[0])
    ov = torch.empty((n - 1, H * 3 // 2, W), dtype=torch.uint8, device=dev)
    cp = torch.empty_like(ov)
    w.step_batch(seq[1:], ov, cp)
    w.sync()
    assert w.ktime_kernel() == "k_front_fused"
    w.close()
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(frames[0])
    for t in range(1, n):
        rov, rcp, _ = ref.step(frames[t])
        assert np.array_equal(ov[t - 1].cpu().numpy(), oracle_lib.bgr_to_i420(rov)), f"overlay (I420) at {t}"
        assert np.array_equal(cp[t - 1].cpu().numpy(), oracle_lib.bgr_to_i420(rcp)), f"compressed (I420) at {t}"
    ref.close()
