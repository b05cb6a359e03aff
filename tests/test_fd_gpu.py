"""GPU parity: the HIP frame-differencing path vs the CPU oracle, through the C-ABI.

Bar (BASELINE.json north_star): uint8 motion/filtered/dilated/accumulated masks
bit-exact; overlay and compressed frames bit-exact as well (the DCT runs the
same float32 fmaf chain as the oracle, so no tolerance is needed against it).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PLANES = {"gray": 0, "motion": 1, "filtered": 2, "acc": 3, "dilated": 4}


def _run_pair(dvc_amd, oracle, frames, scale=None, **kw):
    """Per-frame GPU vs oracle on every plane, output and counter. ``scale``:
    (W, H) of the scaled frames (the frames given are the source size)."""
    SH, SW = frames.shape[1:3]
    W, H = scale or (SW, SH)
    if scale:
        kw = dict(kw, src_width=SW, src_height=SH)
    gpu = dvc_amd.FDWorker(W, H, device=0, keep_planes=True, **kw)
    ref = oracle.OracleFD(W, H, **kw)
    gpu.prime(frames[0])
    ref.prime(frames[0])
    for t in range(1, len(frames)):
        try:
            rov, rcp, racc = ref.step(frames[t])
        except oracle.OddDCTError as e:          # the reference stops here (fd:122, fd:140)
            from dvc_amd._native import DVC_E_ODD_DCT, DvcError
            ov = np.empty((H, W, 3), np.uint8)
            with pytest.raises(DvcError) as ei:
                gpu.step(frames[t], ov)
            assert ei.value.code == DVC_E_ODD_DCT
            assert np.array_equal(ov, e.overlay), f"overlay of the stopping frame {t} differs"
            assert gpu.stats()["frames"] == ref.stats()["frames"] == t - 1
            gpu.close()
            ref.close()
            return None
        ov, cp = gpu.step(frames[t])
        for name, idx in PLANES.items():
            g, r = gpu.plane(idx), ref.plane(idx)
            if not np.array_equal(g, r):
                d = np.argwhere(g != r)
                raise AssertionError(f"{name} plane differs at frame {t}: {len(d)} px, first {d[:5].tolist()}")
        assert np.array_equal(ov, rov), f"overlay differs at frame {t}: {(ov != rov).any(-1).sum()} px"
        if not np.array_equal(cp, rcp):
            diff = np.abs(cp.astype(int) - rcp.astype(int))
            raise AssertionError(f"compressed differs at frame {t}: {(diff > 0).any(-1).sum()} px, max {diff.max()}")
    gs, rs = gpu.stats(), ref.stats()
    assert gs == rs, (gs, rs)
    gpu.close()
    ref.close()
    return gs


@pytest.mark.parametrize("W,H,n,seed,noisy", [
    (640, 360, 12, 0, False),
    (640, 360, 8, 5, True),
    (1920, 1080, 4, 1, False),
    (1920, 1080, 3, 2, True),
    (3840, 2160, 3, 4, False),
])
def test_fd_parity_synthetic(gpu_lib, oracle_lib, W, H, n, seed, noisy):
    from dvc_amd.synthetic import clip
    st = _run_pair(gpu_lib, oracle_lib, clip(W, H, n, seed=seed, noisy=noisy))
    assert st["frames"] == n - 1


def test_fd_parity_main_variant(gpu_lib, oracle_lib):
    """frame_differencing.py:200-207 kwargs (block 8, kernel 10 = asymmetric anchor, release 0.3)."""
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(640, 360, 8, seed=7), block_size=8, kernel_size=10,
              release_factor=0.3, quantization_level=100)


def test_fd_parity_random_frames(gpu_lib, oracle_lib):
    """Pure-noise frames: frame 1 is one giant component riddled with holes."""
    rng = np.random.default_rng(11)
    frames = rng.integers(0, 256, (5, 96, 160, 3), dtype=np.uint8)
    _run_pair(gpu_lib, oracle_lib, frames)


def test_fd_parity_thresholds(gpu_lib, oracle_lib):
    from dvc_amd.synthetic import clip
    frames = clip(320, 240, 6, seed=9, noisy=True)
    for thr, ma in [(-1.0, 0), (3.7, 50), (254.5, 500), (0.5, -1)]:
        _run_pair(gpu_lib, oracle_lib, frames, motion_threshold=thr, min_area=ma)


def _masks():
    rng = np.random.default_rng(123)
    out = []
    for H, W, p in [(16, 16, 0.5), (64, 64, 0.3), (40, 132, 0.55), (100, 200, 0.45), (8, 256, 0.5),
                    (128, 68, 0.6), (200, 300, 0.1)]:
        out.append((rng.random((H, W)) < p).astype(np.uint8) * 255)
    m = np.zeros((120, 160), np.uint8)                # nested rings + holes + border contact
    for r0, v in [(2, 255), (10, 0), (18, 255), (26, 0), (34, 255)]:
        m[r0:120 - r0, r0:160 - r0] = v
    m[0:5, 100:140] = 255
    out.append(m)
    out.append(np.full((64, 64), 255, np.uint8))    # everything
    out.append(np.zeros((64, 64), np.uint8))        # nothing
    cb = (np.indices((48, 128)).sum(0) % 2 * 255).astype(np.uint8)  # checkerboard: max runs per row
    out.append(cb)
    tall = np.zeros((1080, 64), np.uint8)            # tall components: deep union-find chains
    tall[:, 10:14] = 255
    tall[:, 30] = 255
    tall[::2, 40:50] = 255
    out.append(tall)
    stripes = np.zeros((64, 4096), np.uint8)         # wide rows
    stripes[:, ::3] = 255
    out.append(stripes)
    return out


def test_contour_filter_masks(gpu_lib, oracle_lib):
    for i, m in enumerate(_masks()):
        for ma2 in (-1, 0, 6, 1000):
            g, gn = gpu_lib._native.contour_filter(m, ma2)
            r, rn, _ = oracle_lib.contour_filter(m, ma2)
            assert gn == rn, (i, ma2, gn, rn)
            assert np.array_equal(g, r), (i, ma2, int((g != r).sum()))


@pytest.mark.parametrize("W", [2048, 4096])
def test_contour_filter_over_budget_bands(gpu_lib, oracle_lib, W):
    """Bands with more runs + gaps than k_band's LDS node budget take the global
    union-find path: alternating-pixel rows (W/2 runs each), checkerboards,
    random dense blobs and rings across band seams, vs the oracle."""
    rng = np.random.default_rng(W)
    H = 48
    m = (rng.random((H, W)) < 0.45).astype(np.uint8)
    m[0:8, :] = 0
    m[0:8, 0::2] = 1                      # band 0: every other pixel, 8 rows
    m[16:24, :] = (np.indices((8, W)).sum(0) % 2).astype(np.uint8)   # checkerboard band
    m[30:44, 100:140] = 1                 # a filled square straddling a seam ...
    m[33:41, 110:130] = 0                 # ... with a hole (holes are filled, fd:104)
    for ma2 in (-1, 0, 10, 1000):
        g, gn = gpu_lib._native.contour_filter(m, ma2)
        r, rn, _ = oracle_lib.contour_filter(m, ma2)
        assert gn == rn, (ma2, gn, rn)
        assert np.array_equal(g, r), (ma2, int((g != r).sum()))


def test_contour_filter_random_sweep(gpu_lib, oracle_lib):
    rng = np.random.default_rng(5)
    for _ in range(60):
        H, W = 4 * int(rng.integers(1, 40)), 4 * int(rng.integers(1, 60))
        m = (rng.random((H, W)) < rng.uniform(0.05, 0.9)).astype(np.uint8) * 255
        ma2 = int(rng.integers(-1, 40))
        g, gn = gpu_lib._native.contour_filter(m, ma2)
        r, rn, _ = oracle_lib.contour_filter(m, ma2)
        assert gn == rn and np.array_equal(g, r), (H, W, ma2)


def test_device_mode_matches_host_mode(gpu_lib):
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(640, 360, 6, seed=2)
    host = gpu_lib.FDWorker(640, 360)
    host.prime(frames[0])
    outs = [host.step(f) for f in frames[1:]]
    dev = torch.from_numpy(frames).to("cuda:0")
    ov = torch.empty_like(dev[0])
    cp = torch.empty_like(dev[0])
    acc = torch.empty((360, 640), dtype=torch.uint8, device="cuda:0")
    w = gpu_lib.FDWorker(640, 360, device_ptrs=True, stream=torch.cuda.current_stream().cuda_stream)
    w.prime(dev[0])
    for t in range(1, 6):
        w.step(dev[t], ov, cp, acc)
        torch.cuda.synchronize()
        assert np.array_equal(ov.cpu().numpy(), outs[t - 1][0])
        assert np.array_equal(cp.cpu().numpy(), outs[t - 1][1])
    w.close()
    host.close()


def _oracle_sequence(oracle, frames, **kw):
    H, W = frames.shape[1:3]
    ref = oracle.OracleFD(W, H, **kw)
    ref.prime(frames[0])
    ovs, cps = [], []
    for t in range(1, len(frames)):
        ov, cp, _ = ref.step(frames[t])
        ovs.append(ov)
        cps.append(cp)
    planes = {name: ref.plane(idx) for name, idx in PLANES.items()}
    st = ref.stats()
    ref.close()
    return np.stack(ovs), np.stack(cps), planes, st


@pytest.mark.parametrize("W,H,n,max_batch,noisy", [
    (640, 360, 13, 5, True),      # chunks 5, 5, 2
    (640, 360, 9, 8, False),
    (1920, 1080, 6, 4, True),     # chunks 4, 1
])
def test_batch_matches_oracle(gpu_lib, oracle_lib, W, H, n, max_batch, noisy):
    """dvc_fd_step_batch (host mode): every frame's outputs, the last frame's planes
    and the stats equal the oracle's frame-by-frame run."""
    from dvc_amd.synthetic import clip
    frames = clip(W, H, n, seed=3, noisy=noisy)
    rov, rcp, rplanes, rst = _oracle_sequence(oracle_lib, frames)
    w = gpu_lib.FDWorker(W, H, keep_planes=True, max_batch=max_batch)
    w.prime(frames[0])
    ov, cp = w.step_batch(frames[1:])
    for t in range(n - 1):
        assert np.array_equal(ov[t], rov[t]), f"overlay differs at frame {t + 1}"
        assert np.array_equal(cp[t], rcp[t]), f"compressed differs at frame {t + 1}"
    for name, idx in PLANES.items():
        assert np.array_equal(w.plane(idx), rplanes[name]), f"{name} plane differs"
    assert w.stats() == rst
    w.close()


def test_batch_device_matches_steps(gpu_lib):
    """Device-mode batches (several calls, overlapping slots) == one step per frame."""
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(640, 360, 8, seed=6, noisy=True)
    order = [1, 2, 3, 4, 5, 6, 7, 6, 5, 4, 3, 2, 1, 2, 3, 4, 5]
    seq = torch.from_numpy(np.ascontiguousarray(frames[order])).to("cuda:0")
    f0 = torch.from_numpy(frames[0]).to("cuda:0")
    outs = []
    for mode in ("step", "batch"):
        ov = torch.empty_like(seq)
        cp = torch.empty_like(seq)
        w = gpu_lib.FDWorker(640, 360, device_ptrs=True, max_batch=3)
        w.prime(f0)
        if mode == "step":
            for j in range(len(order)):
                w.step(seq[j], ov[j], cp[j])
        else:
            for a, b in ((0, 7), (7, 8), (8, 17)):      # chunks 3,3,1 | 1 | 3,3,3
                w.step_batch(seq[a:b], ov[a:b], cp[a:b])
        w.sync()
        outs.append((ov.cpu().numpy(), cp.cpu().numpy(), w.stats(), w.plane(PLANES["acc"])))
        w.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
    assert np.array_equal(outs[0][3], outs[1][3])


def test_errors(gpu_lib):
    from dvc_amd._native import DvcError
    with pytest.raises(DvcError):
        gpu_lib.FDWorker(640, 360, block_size=129)  # the GPU path implements block sizes 1..128
    with pytest.raises(DvcError):
        gpu_lib.FDWorker(8, 360)                    # frames of at least 16 x 16
    w = gpu_lib.FDWorker(640, 360)
    with pytest.raises(DvcError):
        w.step(np.zeros((360, 640, 3), np.uint8))   # step before prime
    w.close()


def test_process_single_video_fd(gpu_lib, tmp_path):
    from dvc_amd.frame_differencing import process_single_video_fd
    calls = []
    process_single_video_fd("synthetic://320x240?frames=102&seed=3", str(tmp_path), progress_callback=calls.append)
    d = tmp_path / "320x240"
    assert calls == [50, 100]
    ov = np.load(d / "dilated_motion_mask_video.npy")
    cp = np.load(d / "compressed_final_video.npy")
    assert ov.shape == (101, 240, 320, 3) and cp.shape == ov.shape
    txt = (d / "execution_times.txt").read_text().splitlines()
    assert txt[0] == "Frame Differencing:" and txt[1] == "  Frames processed: 101"
    assert (d / "processing.log").exists()
    # per-frame time as fd:86,135 sums it: read -> write of every frame adds up
    # to the loop, so frames x average <= total (rounding of the 2/4 decimals)
    total = float(txt[2].split(":")[1].split()[0])
    avg = float(txt[3].split(":")[1].split()[0])
    assert 0 < avg and 101 * avg <= total + 101 * 5e-5 + 5e-3


def test_process_single_video_fd_chunks_and_odd_dct_stop(gpu_lib, tmp_path, monkeypatch, caplog):
    """The drop-in's reader / step / writer threads: chunks of 4 frames give the
    same output videos as one FDWorker.step per frame; a 3-px edge block stops
    the run as the reference does (fd:122, fd:140): the failing frame's overlay
    is written, its compressed frame is not, the error is logged."""
    from dvc_amd import frame_differencing as fdm
    from dvc_amd._native import DVC_E_ODD_DCT, DvcError
    from dvc_amd.synthetic import clip
    monkeypatch.setattr(fdm, "READ_AHEAD", 4)

    def per_frame(frames):
        w = gpu_lib.FDWorker(frames.shape[2], frames.shape[1])
        w.prime(frames[0])
        outs = []
        try:
            for f in frames[1:]:
                outs.append(w.step(f))
        except DvcError as e:
            assert e.code == DVC_E_ODD_DCT
            return outs, True
        finally:
            w.close()
        return outs, False

    for name, frames in (("cam", clip(320, 240, 11, seed=5)), ("odd", clip(643, 360, 12, seed=1003, n_objects=4))):
        np.save(tmp_path / f"{name}.npy", frames)
        fdm.process_single_video_fd(str(tmp_path / f"{name}.npy"), str(tmp_path / "out"))
        ref, stopped = per_frame(frames)
        ov = np.load(tmp_path / f"out/{name}/dilated_motion_mask_video.npy")
        cp = np.load(tmp_path / f"out/{name}/compressed_final_video.npy")
        assert len(cp) == len(ref) and len(ov) == len(ref) + (1 if stopped else 0)
        for t in range(len(ref)):
            assert np.array_equal(ov[t], ref[t][0]) and np.array_equal(cp[t], ref[t][1]), f"{name} frame {t + 1}"
        assert stopped == (name == "odd")
        if stopped:   # logged, not raised (fd:140-141); processing.log only if logging was unconfigured
            assert "Odd-size DCT" in caplog.text
        txt = (tmp_path / f"out/{name}/execution_times.txt").read_text()
        assert f"Frames processed: {len(cp)}" in txt


# ---------------------------------------------------------------- geometry ---
# Any frame size and block size (fd:117-127: partial edge blocks are their
# slices; an odd side > 1 of a static block stops the reference, fd:122/140),
# and scale_factor (fd:60-61, 74, 91: the GPU resizes).
@pytest.mark.parametrize("W,H,n,kw", [
    (960, 540, 12, dict(block_size=8, kernel_size=10, release_factor=0.3)),   # __main__ kwargs at 1080p / 2
    (1366, 768, 11, {}),                        # W % 4 = 2: re-pitched rows, 2-px edge blocks
    (641, 361, 11, {}),                         # 1-px edge blocks (length-1 DCTs)
    (643, 360, 12, {}),                         # 3-px edge blocks: stops at the first static one
    (162, 98, 11, dict(block_size=2, min_area=20)),
    (200, 120, 11, dict(block_size=16)),
    (200, 122, 11, dict(block_size=6, kernel_size=4)),
    (130, 70, 11, dict(block_size=1, min_area=10)),
    (258, 194, 11, dict(block_size=64)),
    (300, 200, 11, dict(block_size=5)),         # odd block: stops once a block is static
])
def test_fd_parity_geometry(gpu_lib, oracle_lib, W, H, n, kw):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(W, H, n, seed=W + H, n_objects=4), **kw)


@pytest.mark.parametrize("block", [4, 8])
@pytest.mark.parametrize("ksize", [64, 100, 127])
def test_fd_parity_large_dilation_fast_blocks(gpu_lib, oracle_lib, block, ksize):
    """k_dilate<4/8> with windows taller than 64 rows (its rows(std::true_type)
    branch: kernel_size above ~61 at b=4, ~57 at b=8), fd:106. One small moving
    object in a tall frame leaves most kept-mask rows empty (sparse kocc), and
    a second one touching the left/top edges puts the window across the frame
    border."""
    from dvc_amd.synthetic import clip
    frames = clip(320, 400, 7, seed=block * 131 + ksize, n_objects=1)
    frames[:, :40, :48] = frames[:, :1, :1]          # a flat corner ...
    for t in range(len(frames)):                     # ... with an object sliding along the edges
        frames[t, :24 + 3 * t, :20 + 4 * t] = (30 + 20 * t) % 256
    _run_pair(gpu_lib, oracle_lib, frames, block_size=block, kernel_size=ksize, min_area=30)


@pytest.mark.parametrize("SW,SH,W,H,kw", [
    (1920, 1080, 960, 540, dict(block_size=8, kernel_size=10, release_factor=0.3)),   # fd:200-207
    (640, 360, 448, 252, {}),                   # scale 0.7: INTER_LINEAR fixed point
    (320, 180, 416, 234, dict(block_size=6)),   # scale 1.3: upscale
    (641, 361, 320, 180, {}),                   # about 0.5 of odd sizes: linear, not the 2x area path
])
def test_fd_parity_scaled(gpu_lib, oracle_lib, SW, SH, W, H, kw):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(SW, SH, 9, seed=SW, n_objects=4), scale=(W, H), **kw)


@pytest.mark.parametrize("W,H,batch,kw", [
    (1366, 768, 5, {}),
    (962, 542, 4, dict(block_size=8)),
    (200, 122, 3, dict(block_size=6)),
])
def test_geometry_batch_device_matches_oracle(gpu_lib, oracle_lib, W, H, batch, kw):
    """Dense (n, H, W, 3) device frames of any width (rows not 4-byte aligned ->
    re-pitched on the device), batched, vs the oracle frame by frame."""
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(W, H, 10, seed=3, n_objects=5)
    rov, rcp, rplanes, rst = _oracle_sequence(oracle_lib, frames, **kw)
    d = torch.from_numpy(frames).to("cuda:0")
    ov = torch.empty_like(d[1:])
    cp = torch.empty_like(d[1:])
    w = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=batch, **kw)
    w.prime(d[0])
    w.step_batch(d[1:], ov, cp)
    w.sync()
    assert np.array_equal(ov.cpu().numpy(), rov) and np.array_equal(cp.cpu().numpy(), rcp)
    assert w.stats() == rst
    w.close()


def test_odd_stop_in_batch(gpu_lib, oracle_lib):
    """A batch crossing the stopping frame: frames before it complete, its
    overlay valid, stats count the completed frames (host and device mode)."""
    import torch
    from dvc_amd._native import DVC_E_ODD_DCT, DvcError
    from dvc_amd.synthetic import clip
    W, H = 643, 360
    frames = clip(W, H, 14, seed=9)
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(frames[0])
    rov = []
    for f in frames[1:]:
        try:
            rov.append(ref.step(f)[0])
        except oracle_lib.OddDCTError as e:
            rov.append(e.overlay)
            break
    k = ref.stats()["frames"]
    assert 0 < k < len(frames) - 2
    w = gpu_lib.FDWorker(W, H, max_batch=4)
    w.prime(frames[0])
    ov = np.empty((13, H, W, 3), np.uint8)
    with pytest.raises(DvcError) as ei:
        w.step_batch(frames[1:], ov, np.empty_like(ov))
    assert ei.value.code == DVC_E_ODD_DCT and w.stats()["frames"] == k
    assert all(np.array_equal(ov[t], rov[t]) for t in range(k + 1))
    with pytest.raises(DvcError):
        w.step(frames[1])                       # stopped until the next prime
    w.prime(frames[0])
    w.step(frames[1])
    w.close()
    d = torch.from_numpy(frames).to("cuda:0")
    wd = gpu_lib.FDWorker(W, H, device_ptrs=True, max_batch=5)
    wd.prime(d[0])
    dov = torch.empty_like(d[1:])
    wd.step_batch(d[1:], dov, torch.empty_like(dov))   # asynchronous: reported at the sync
    with pytest.raises(DvcError) as ei:
        wd.sync()
    assert ei.value.code == DVC_E_ODD_DCT and wd.stats()["frames"] == k
    assert all(np.array_equal(dov[t].cpu().numpy(), rov[t]) for t in range(k + 1))
    wd.close()


def test_contour_filter_any_width(gpu_lib, oracle_lib):
    rng = np.random.default_rng(77)
    for _ in range(40):
        H, W = int(rng.integers(4, 90)), int(rng.integers(4, 300))
        m = (rng.random((H, W)) < rng.uniform(0.05, 0.9)).astype(np.uint8) * 255
        ma2 = int(rng.integers(-1, 40))
        g, gn = gpu_lib._native.contour_filter(m, ma2)
        r, rn, _ = oracle_lib.contour_filter(m, ma2)
        assert gn == rn and np.array_equal(g, r), (H, W, ma2)
