"""GPU parity: the HIP optical-flow path vs the CPU oracle, through the C-ABI.

Every float and double expression of the Farneback restatement runs in the
same order on both sides (-ffp-contract=off), so the bar is bit-exact for the
flow itself (float32 per component), every mask plane (raw |flow| > thr, vote,
close/open, rectangles) and every compressed frame.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PLANES = {"raw": 0, "smooth": 1, "morph": 2, "rect": 3}


def _first_diff(g, r):
    d = np.argwhere(g != r)
    return f"{len(d)} differ, first {d[:4].tolist()}"


def _run_pair(dvc_amd, oracle, frames, batch=0, **kw):
    """Per-frame (batch=0) or batched GPU run vs the oracle; returns GPU stats."""
    H, W = frames.shape[1:3]
    okw = {k: v for k, v in kw.items()
           if k in ("flow_threshold", "alpha_fraction", "window_size", "morph_kernel", "direct_sums")}
    gpu = dvc_amd.OFWorker(W, H, device=0, keep_planes=True, max_batch=max(batch, 1), **kw)
    ref = oracle.OracleOF(W, H, **okw)
    gpu.prime(frames[0])
    ref.prime(frames[0])
    motion = comps = static = 0
    rmasks, rcps = [], []
    for t in range(1, len(frames)):
        rmask, rcp, rflow = ref.step(frames[t])
        rmasks.append(rmask)
        rcps.append(rcp)
        raw = ref.plane(0)
        motion += int((raw > 0).sum())
        comps += oracle.rect_mask(ref.plane(2))[1]
        full = rmask[:H // 8 * 8, :W // 8 * 8]        # partial edge blocks are never static (of:159)
        static += int((full.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3)) == 0).sum())
        if batch:
            continue
        mask, cp = gpu.step(frames[t])
        flow = gpu.flow()
        if not np.array_equal(flow.view(np.uint32), rflow.view(np.uint32)):
            err = np.abs(flow - rflow).max()
            raise AssertionError(f"flow differs at frame {t}: {_first_diff(flow, rflow)}, max abs {err}")
        for name, idx in PLANES.items():
            g, r = gpu.plane(idx), ref.plane(idx)
            assert np.array_equal(g, r), f"{name} plane differs at frame {t}: {_first_diff(g, r)}"
        assert np.array_equal(mask, rmask), f"mask differs at frame {t}"
        if not np.array_equal(cp, rcp):
            diff = np.abs(cp.astype(int) - rcp.astype(int))
            raise AssertionError(f"compressed differs at frame {t}: {(diff > 0).any(-1).sum()} px, max {diff.max()}")
    if batch:
        masks, cps = gpu.step_batch(frames[1:])
        for t in range(len(frames) - 1):
            assert np.array_equal(masks[t], rmasks[t]), f"batched mask differs at frame {t + 1}"
            assert np.array_equal(cps[t], rcps[t]), f"batched compressed differs at frame {t + 1}"
    st = gpu.stats()
    assert st == {"frames": len(frames) - 1, "motion_px": motion, "components": comps, "static_blocks": static}, st
    gpu.close()
    ref.close()
    return st


@pytest.mark.parametrize("W,H", [(160, 96), (640, 360), (333, 185), (170, 100)])
def test_of_stages(gpu_lib, oracle_lib, W, H):
    """Stage by stage on one frame pair: gray, the polynomial expansion of every
    pyramid level, the coarsest level's first iteration, the final flow."""
    from dvc_amd.synthetic import clip
    frames = clip(W, H, 2, seed=1)
    gpu = gpu_lib.OFWorker(W, H, keep_planes=True)
    gpu.prime(frames[0])
    gpu.step(frames[1])
    g0, g1 = oracle_lib.bgr2gray(frames[0]), oracle_lib.bgr2gray(frames[1])
    assert np.array_equal(gpu.plane(gpu_lib._native.OF_PLANE_GRAY), g1), "gray"
    L = int(oracle_lib._of_lib().oc_fb_levels(W, H, 0.3, 2))
    for k in range(L + 1):
        for what, g in ((1, g0), (0, g1)):
            got, want = gpu.debug_read(what, k), oracle_lib.fb_level_poly(g, k)
            assert got.shape == want.shape, (k, got.shape, want.shape)
            if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                raise AssertionError(f"R level {k} ({'prev' if what else 'cur'}): {_first_diff(got, want)}, "
                                     f"max abs {np.abs(got - want).max()}")
    R0, R1 = oracle_lib.fb_level_poly(g0, L), oracle_lib.fb_level_poly(g1, L)
    f1 = oracle_lib.fb_iteration(R0, R1, np.zeros(R0.shape[:2] + (2,), np.float32))   # OpenCV's running sums
    got = gpu.debug_read(2, L)
    assert np.array_equal(got.view(np.uint32), f1.view(np.uint32)), f"iteration 0 flow: {_first_diff(got, f1)}"
    want = oracle_lib.farneback(g0, g1)
    got = gpu.flow()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"final flow: {_first_diff(got, want)}"
    gpu.close()


@pytest.mark.parametrize("W,H,n,seed,noisy", [
    (160, 96, 6, 1, False),      # 1 pyramid level
    (320, 176, 6, 2, False),     # 2 levels
    (640, 360, 5, 0, False),     # 3 levels
    (640, 360, 4, 5, True),
    (328, 184, 4, 7, False),     # width not a multiple of 32 / 64
])
def test_of_parity_synthetic(gpu_lib, oracle_lib, W, H, n, seed, noisy):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(W, H, n, seed=seed, noisy=noisy))


@pytest.mark.parametrize("direct", [False, True])
def test_of_parity_1080p(gpu_lib, oracle_lib, direct):
    """Both box-sum orders: OpenCV's running sums (k_flow_scan2, the default) and
    direct per-pixel sums (k_flow, DVC_FLAG_OF_DIRECT_SUMS), each vs the oracle
    computing the same order."""
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(1920, 1080, 3, seed=3), direct_sums=direct)


@pytest.mark.parametrize("W,H,kw", [
    (328, 184, dict(direct_sums=True)),
    (640, 360, dict(direct_sums=True, window_size=5)),
    (96, 64, {}),                        # one strip, one pyramid level
    (136, 72, dict(batch=3)),            # partial last strip, batched
])
def test_of_box_orders(gpu_lib, oracle_lib, W, H, kw):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(W, H, 5, seed=W), **kw)


def test_of_parity_window_eviction(gpu_lib, oracle_lib):
    """window 3 over 9 frames: the deque drops masks (of:84, maxlen)."""
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(320, 176, 9, seed=4, n_objects=4), window_size=3, alpha_fraction=0.4)


def test_of_parity_long_run(gpu_lib, oracle_lib):
    """> 256 frames: the launchers reduce frame numbers modulo the ring periods
    (reduce_frame in of_kernels.hip); slots, the vote window and its eviction
    must carry on exactly, batched and per frame."""
    from dvc_amd.synthetic import clip
    frames = clip(64, 48, 301, seed=3, n_objects=2)
    _run_pair(gpu_lib, oracle_lib, frames, batch=16, window_size=7)
    _run_pair(gpu_lib, oracle_lib, frames[:271], window_size=5)


def test_of_parity_random_frames(gpu_lib, oracle_lib):
    rng = np.random.default_rng(11)
    _run_pair(gpu_lib, oracle_lib, rng.integers(0, 256, (4, 96, 128, 3), dtype=np.uint8), flow_threshold=2.0)


@pytest.mark.parametrize("batch", [2, 4])
def test_of_batched_equals_oracle(gpu_lib, oracle_lib, batch):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(320, 176, 10, seed=6, noisy=True), batch=batch, window_size=4)


def test_of_device_pointers(gpu_lib, oracle_lib):
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(320, 176, 5, seed=8)
    n, H, W = frames.shape[:3]
    d_in = torch.from_numpy(frames).to("cuda:0")
    d_mask = torch.empty((n - 1, H, W), dtype=torch.uint8, device="cuda:0")
    d_cp = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device="cuda:0")
    w = gpu_lib.OFWorker(W, H, device_ptrs=True, max_batch=4)
    w.prime(d_in[0])
    w.step_batch(d_in[1:], mask=d_mask, compressed=d_cp)
    w.sync()
    ref = oracle_lib.OracleOF(W, H)
    ref.prime(frames[0])
    for t in range(1, n):
        rmask, rcp, _ = ref.step(frames[t])
        assert np.array_equal(d_mask[t - 1].cpu().numpy(), rmask), t
        assert np.array_equal(d_cp[t - 1].cpu().numpy(), rcp), t
    w.close()


@pytest.mark.parametrize("density", [0.0, 0.002, 0.05, 1.0])
def test_of_compress_arbitrary_mask(gpu_lib, oracle_lib, density):
    """compress_with_motion (of:151-183) with a decoded-style mask of any content."""
    rng = np.random.default_rng(int(density * 1000) + 3)
    H, W = 120, 200
    bgr = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    mask = (rng.random((H, W)) < density).astype(np.uint8) * rng.integers(1, 256, (H, W), dtype=np.uint8)
    got = gpu_lib._native.of_compress(bgr, mask, 100.0)
    want = oracle_lib.of_compress(bgr, mask, 100.0)
    assert np.array_equal(got, want)


def test_of_rejects_unsupported(gpu_lib):
    with pytest.raises(gpu_lib._native.DvcError):
        gpu_lib.OFWorker(7, 360)            # frames of at least 8 x 8
    for k in (0, 65):                       # morph_kernel 1..64
        with pytest.raises(gpu_lib._native.DvcError):
            gpu_lib.OFWorker(640, 360, morph_kernel=k)
    w = gpu_lib.OFWorker(160, 96)
    with pytest.raises(gpu_lib._native.DvcError):
        w.step(np.zeros((96, 160, 3), np.uint8))   # step before prime
    w.close()


def test_process_single_video_of_dropin(gpu_lib, oracle_lib, tmp_path):
    """motion_compression_opt.process_single_video_of on a synthetic clip: the two
    reference passes (of:209-231) through .npy streams == the fused oracle worker."""
    from dvc_amd import motion_compression_opt as M
    from dvc_amd import video_io
    from dvc_amd.synthetic import clip
    uri = "synthetic://320x176?frames=7&seed=9"
    M.process_single_video_of(uri, str(tmp_path))
    out = tmp_path / "320x176"
    frames = clip(320, 176, 7, seed=9)
    ref = oracle_lib.OracleOF(320, 176)
    ref.prime(frames[0])
    ov = video_io.open_source(str(out / "overlay.mp4"))
    mk = video_io.open_source(str(out / "mask.mp4"))
    cp = video_io.open_source(str(out / "compressed.mp4"))
    for t in range(1, 7):
        rmask, rcp, _ = ref.step(frames[t])
        assert np.array_equal(ov.read()[1], frames[t])
        assert np.array_equal(mk.read()[1], rmask), t
        assert np.array_equal(cp.read()[1], rcp), t
    txt = open(out / "execution_times.txt").read()
    assert txt.startswith("Motion Detection:\n  Frames processed: 6\n") and "Compression:\n  Frames processed: 6\n" in txt


# ---------------------------------------------------------------- geometry ---
# The reference runs at any frame size (Farneback, the vote and the morphology
# are per pixel; compress_with_motion skips partial 8x8 blocks, of:159,177) and
# takes morph_kernel as a kwarg (of:29-31,62: getStructuringElement(MORPH_ELLIPSE)).
@pytest.mark.parametrize("W,H,n,kw", [
    (162, 98, 5, {}),                                   # W % 8 = 2, H % 8 = 2: partial blocks, 2-px quads
    (170, 100, 5, dict(morph_kernel=3)),
    (133, 75, 6, dict(morph_kernel=5, window_size=3, batch=2)),   # odd sides, batched
    (333, 185, 4, dict(morph_kernel=4)),                # even element: asymmetric anchor, 2 levels
    (97, 61, 5, dict(morph_kernel=1)),                  # 1x1 element (MORPH_RECT): identity
    (203, 117, 4, dict(morph_kernel=9, flow_threshold=0.3)),
])
def test_of_any_geometry(gpu_lib, oracle_lib, W, H, n, kw):
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(W, H, n, seed=W + H, n_objects=3), **kw)


def test_of_1366x768(gpu_lib, oracle_lib):
    """A common camera size that is not a multiple of 8 (1366 = 170 * 8 + 6)."""
    from dvc_amd.synthetic import clip
    _run_pair(gpu_lib, oracle_lib, clip(1366, 768, 3, seed=5))


@pytest.mark.parametrize("k", [3, 7])
def test_of_morph_kernel_planes(gpu_lib, oracle_lib, k):
    """The close/open plane itself (of:89-90) against the oracle's restatement of
    getStructuringElement + morphologyEx, on vote planes dense enough to matter."""
    rng = np.random.default_rng(k)
    frames = rng.integers(0, 256, (5, 72, 136, 3), dtype=np.uint8)
    _run_pair(gpu_lib, oracle_lib, frames, morph_kernel=k, flow_threshold=1.0, window_size=2)


@pytest.mark.parametrize("W,H,pad", [(170, 100, 0), (162, 98, 6), (320, 176, 4)])
def test_of_device_pointers_any_pitch(gpu_lib, oracle_lib, W, H, pad):
    """Device frames whose rows the kernels cannot read in place (3W % 4 != 0, or
    rows padded to a pitch that is not whole quads) are re-pitched on the GPU."""
    import torch
    from dvc_amd.synthetic import clip
    frames = clip(W, H, 5, seed=W, n_objects=3)
    n = len(frames)
    pitch = 3 * W + pad
    buf = np.zeros((n, H, pitch), np.uint8)
    buf[:, :, :3 * W] = frames.reshape(n, H, 3 * W)
    d_in = torch.from_numpy(buf).to("cuda:0")
    d_mask = torch.empty((n - 1, H, W), dtype=torch.uint8, device="cuda:0")
    d_cp = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device="cuda:0")
    w = gpu_lib.OFWorker(W, H, device_ptrs=True, max_batch=2)
    lib = gpu_lib._native.lib()
    gpu_lib._native.check(lib.dvc_of_prime(w._h, d_in[0].data_ptr(), pitch))
    gpu_lib._native.check(lib.dvc_of_step_batch(w._h, d_in[1].data_ptr(), pitch, H * pitch, n - 1,
                                                 d_mask.data_ptr(), H * W, d_cp.data_ptr(), 3 * H * W))
    w.sync()
    ref = oracle_lib.OracleOF(W, H)
    ref.prime(frames[0])
    for t in range(1, n):
        rmask, rcp, _ = ref.step(frames[t])
        assert np.array_equal(d_mask[t - 1].cpu().numpy(), rmask), t
        assert np.array_equal(d_cp[t - 1].cpu().numpy(), rcp), t
    w.close()


# ------------------------------------------------------------- compressor ----
def _gray(m3):
    m = m3.astype(np.uint32)
    return ((m[..., 0] * 1868 + m[..., 1] * 9617 + m[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


@pytest.mark.parametrize("W,H,ch", [(200, 120, 1), (203, 117, 3), (64, 64, 3), (1366, 10, 1)])
def test_ofc_batch_equals_per_frame(gpu_lib, oracle_lib, W, H, ch):
    """dvc_ofc (compress_with_motion's loop, of:141-185, n frames per call) ==
    dvc_of_compress per frame == the oracle, with 1- and 3-channel decoded masks:
    a 3-channel mask is grayed exactly first (of:147-149) — (1, 0, 0) grays to
    0, so such a pixel must not gate its block."""
    rng = np.random.default_rng(W * H + ch)
    n = 7
    frames = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    if ch == 1:
        masks = ((rng.random((n, H, W)) < 0.01) * rng.integers(1, 256, (n, H, W))).astype(np.uint8)
    else:
        masks = np.zeros((n, H, W, 3), np.uint8)
        sel = rng.random((n, H, W)) < 0.01
        masks[sel] = rng.integers(0, 256, (int(sel.sum()), 3))
        faint = rng.random((n, H, W)) < 0.02            # grays to 0: static
        masks[faint] = (1, 0, 0)
    c = gpu_lib._native.OFCompressor(W, H, max_batch=3)
    got = c.run(frames, masks)
    c.close()
    gm = masks if ch == 1 else _gray(masks)
    for t in range(n):
        want = oracle_lib.of_compress(frames[t], gm[t], 100.0)
        assert np.array_equal(got[t], want), t
        assert np.array_equal(gpu_lib._native.of_compress(frames[t], gm[t], 100.0), want), t


def test_compress_with_motion_dropin_chunks(gpu_lib, oracle_lib, tmp_path, monkeypatch):
    """The drop-in's second pass in chunks (READ_AHEAD 4 over 11 frame pairs)
    with a 3-channel mask video as VideoCapture decodes mask.mp4, at a size that
    is not a multiple of 8: == the oracle per frame on the grayed mask; the mask
    video being shorter ends the loop (of:144-145)."""
    from dvc_amd import motion_compression_opt as M
    monkeypatch.setattr(M, "READ_AHEAD", 4)
    rng = np.random.default_rng(7)
    W, H = 165, 99
    frames = rng.integers(0, 256, (11, H, W, 3), dtype=np.uint8)
    masks = np.zeros((10, H, W, 3), np.uint8)
    for t in range(10):
        y, x = rng.integers(0, H - 20), rng.integers(0, W - 30)
        masks[t, y:y + 20, x:x + 30] = 255
        masks[t, rng.random((H, W)) < 0.01] = (1, 0, 0)     # grays to 0
    np.save(tmp_path / "in.npy", frames)
    np.save(tmp_path / "mask.npy", masks)
    n, total, avg = M.compress_with_motion(str(tmp_path / "in.npy"), str(tmp_path / "mask.npy"), str(tmp_path))
    assert n == 10 and total > 0 and abs(avg - total / 10) < 1e-9
    got = np.load(tmp_path / "compressed.npy")
    gm = ((masks.astype(np.uint32) * np.array([1868, 9617, 4899])).sum(-1) + 8192 >> 14).astype(np.uint8)
    for t in range(10):
        assert np.array_equal(got[t], oracle_lib.of_compress(frames[t], gm[t], 100.0)), t


@pytest.mark.parametrize("W,H", [(640, 360), (333, 185)])
def test_of_upsample_forms_agree(gpu_lib, oracle_lib, W, H, monkeypatch):
    """k_flow_up_lds (coarse rows staged in LDS, the default, at 8 output
    rows a workgroup; 1, 3 and 16 via DVC_OF_UP_ROWS) and the gather form
    k_flow_up (DVC_OF_UP_GATHER, the fallback for levels too wide to stage)
    give the same flow bits, and all equal the oracle's."""
    from dvc_amd.synthetic import clip
    frames = clip(W, H, 4, seed=7)
    ref = oracle_lib.OracleOF(W, H)
    ref.prime(frames[0])
    rflows = [ref.step(frames[t])[2] for t in range(1, len(frames))]
    ref.close()
    for gather, rows in ((False, None), (False, "1"), (False, "3"), (False, "16"), (True, None)):
        if gather:
            monkeypatch.setenv("DVC_OF_UP_GATHER", "1")
        else:
            monkeypatch.delenv("DVC_OF_UP_GATHER", raising=False)
        if rows:
            monkeypatch.setenv("DVC_OF_UP_ROWS", rows)
        else:
            monkeypatch.delenv("DVC_OF_UP_ROWS", raising=False)
        gpu = gpu_lib.OFWorker(W, H, keep_planes=True)
        gpu.prime(frames[0])
        for t in range(1, len(frames)):
            gpu.step(frames[t])
            f = gpu.flow()
            assert np.array_equal(f.view(np.uint32), rflows[t - 1].view(np.uint32)), \
                f"gather={gather} rows={rows}: flow differs at frame {t}: {_first_diff(f, rflows[t - 1])}"
        gpu.close()


@pytest.mark.parametrize("W,H,n,batch", [(333, 185, 5, 0), (1920, 1080, 3, 2)])
def test_of_scan_forms_agree(gpu_lib, oracle_lib, W, H, n, batch, monkeypatch):
    """The pipelined k_flow_scan2 (the default for winsize 9) and the
    barrier-phased k_flow_scan it replaced (DVC_OF_SCAN2=0 at create: the
    form winsize != 9 takes) give the same flow bits, masks and compressed
    frames — a partial last strip (333 px) and a height that is not a multiple
    of the 12-row blocks (185, 1080 / 2^k) — and the library reports which one
    ran (dvc_of_ktime_kernel). At 333 x 185 both also equal the oracle."""
    from dvc_amd.synthetic import clip
    frames = clip(W, H, n, seed=W + H)
    runs = {}
    for scan2 in ("1", "0"):
        monkeypatch.setenv("DVC_OF_SCAN2", scan2)
        gpu = gpu_lib.OFWorker(W, H, keep_planes=True, max_batch=max(batch, 1))
        gpu.prime(frames[0])
        if batch:
            masks, cps = gpu.step_batch(frames[1:])
            runs[scan2] = ([gpu.flow()], list(masks), list(cps), gpu.stats())
        else:
            fl, ms, cs = [], [], []
            for t in range(1, n):
                m, c = gpu.step(frames[t])
                fl.append(gpu.flow())
                ms.append(m)
                cs.append(c)
            runs[scan2] = (fl, ms, cs, gpu.stats())
        assert gpu.ktime_kernel() == ("k_flow_scan2" if scan2 == "1" else "k_flow_scan")
        gpu.close()
    a, b = runs["1"], runs["0"]
    for k, (fa, fb) in enumerate(zip(a[0], b[0])):
        assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32)), f"flow differs (step {k}): {_first_diff(fa, fb)}"
    for t, (ma, mb) in enumerate(zip(a[1], b[1])):
        assert np.array_equal(ma, mb), f"mask differs at frame {t + 1}"
    for t, (ca, cb) in enumerate(zip(a[2], b[2])):
        assert np.array_equal(ca, cb), f"compressed differs at frame {t + 1}"
    assert a[3] == b[3]
    if not batch:
        ref = oracle_lib.OracleOF(W, H)
        ref.prime(frames[0])
        for t in range(1, n):
            rm, rc, rf = ref.step(frames[t])
            assert np.array_equal(a[0][t - 1].view(np.uint32), rf.view(np.uint32)), f"flow vs oracle, frame {t}"
            assert np.array_equal(a[1][t - 1], rm) and np.array_equal(a[2][t - 1], rc), f"outputs vs oracle, frame {t}"
        ref.close()


@pytest.mark.parametrize("scan2", ["1", "0"])
def test_of_scan_abort_drains(gpu_lib, oracle_lib, scan2, monkeypatch):
    """A strip hand-off wait that fails (fault injection: DVC_OF_FAULT=scan_abort
    raises the abort flag before every batch, the path a ~1 s poll timeout
    takes) drains the launch — every wave of a workgroup leaves the interval
    loop at the same barrier — and the error comes back from the
    call instead of a hang. A handle created afterwards runs bit-exact."""
    import time
    from dvc_amd._native import DVC_E_HIP, DvcError
    from dvc_amd.synthetic import clip
    W, H = 1920, 1080
    frames = clip(W, H, 5, seed=9)
    monkeypatch.setenv("DVC_OF_SCAN2", scan2)
    monkeypatch.setenv("DVC_OF_FAULT", "scan_abort")
    gpu = gpu_lib.OFWorker(W, H, max_batch=4)
    gpu.prime(frames[0])
    t0 = time.perf_counter()
    with pytest.raises(DvcError) as ei:
        gpu.step_batch(frames[1:])
    assert ei.value.code == DVC_E_HIP and "hand-off" in str(ei.value)
    assert time.perf_counter() - t0 < 20.0
    gpu.close()
    monkeypatch.delenv("DVC_OF_FAULT")
    gpu = gpu_lib.OFWorker(W, H, keep_planes=True)
    ref = oracle_lib.OracleOF(W, H)
    gpu.prime(frames[0])
    ref.prime(frames[0])
    m, c = gpu.step(frames[1])
    rm, rc, rf = ref.step(frames[1])
    assert np.array_equal(gpu.flow().view(np.uint32), rf.view(np.uint32))
    assert np.array_equal(m, rm) and np.array_equal(c, rc)
    gpu.close()
    ref.close()
