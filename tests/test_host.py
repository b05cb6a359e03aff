"""CPU tests of the host side: the C-ABI library loads and exports every symbol
include/dvc.h declares (no compute calls), parameter derivation, the reference's
execution_times.txt format, frame I/O, the synthetic generator, feed sharding."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "dvc.h")).read()
    return sorted(set(re.findall(r"\b(dvc_[a-z0-9_]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    import dvc_amd
    dvc_amd._native.build()
    L = dvc_amd._native.lib()
    declared = _declared_symbols()
    assert set(declared) == set(dvc_amd._native.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert L.dvc_abi_version() == dvc_amd._native.ABI_VERSION


def test_shipping_library_has_no_result_changing_knobs():
    """The stage-skip ablations (outputs wrong by design) and the CU-split
    experiment live only in variant builds (tools/build_variant.sh
    -DDVC_ABLATION / -DDVC_EXPERIMENTS), never in the default libdvc_hip.so."""
    import dvc_amd
    path = dvc_amd._native.build()
    blob = open(path, "rb").read()
    for knob in (b"DVC_FD_SKIP", b"DVC_OF_SKIP", b"DVC_CU_SPLIT"):
        assert knob not in blob, knob


def test_shipping_library_reads_no_tuning_knobs():
    """Launch-tuning knobs (grid sizes, chunks, priorities, LDS pads, A/B
    switches) are read from the environment only by experiment builds
    (csrc/tune.h): their names are absent from the shipping
    library, whose only environment reads are the per-handle path selectors
    and the fault injection the tests use."""
    import re
    import dvc_amd
    blob = open(dvc_amd._native.build(), "rb").read()
    names = set(re.findall(rb"DVC_[A-Z0-9_]{3,}", blob))
    allowed = {b"DVC_FD_GRAPH", b"DVC_FD_FUSED8", b"DVC_OF_SCAN2", b"DVC_OF_UP_ROWS", b"DVC_OF_UP_GATHER",
               b"DVC_OF_FAULT"}
    for n in (b"DVC_PRIO", b"DVC_FRONT_WAVES", b"DVC_FUSED_CHUNKS", b"DVC_OUT_WGS", b"DVC_FIX_WGS", b"DVC_CCL_CG",
              b"DVC_OF_SERIAL", b"DVC_OF_PRIO", b"DVC_OF_SCAN", b"DVC_OF_BH", b"DVC_FD_FUSED", b"DVC_ACC_GENERAL"):
        assert n not in names, n
    # (error texts name flags and formats: DVC_FLAG_*, DVC_FMT_*)
    assert all(n in allowed or n.startswith((b"DVC_FLAG_", b"DVC_FMT_")) for n in names), names


def test_abi_gaussian_taps_host_only():
    """dvc_gaussian_taps_q8 is pure host code: same taps as the oracle."""
    import dvc_amd
    import oracle
    for n, s in [(5, 0.0), (25, 30.0), (7, 1.2), (31, 5.0)]:
        assert dvc_amd._native.gaussian_taps_q8(n, s) == oracle.gauss_taps_q8(n, s).tolist()


def test_derive_params_matches_reference_semantics():
    from dvc_amd.fd import derive_params
    p = derive_params(1920, 1080)
    assert (p.block, p.ithresh, p.min_area2, p.ksize, p.anchor) == (4, 0, 1000, 7, 3)
    assert (p.alpha, p.beta, p.gamma, p.quant) == (0.5, 0.5, 0.0, 100.0)
    assert (p.prime_ksize, p.prime_sigma) == (25, 30.0)
    # fd:200-207 variant and edge thresholds
    p = derive_params(960, 540, block_size=8, kernel_size=10, release_factor=0.3, min_area=10.25,
                      motion_threshold=-3)
    assert (p.block, p.ksize, p.anchor, p.min_area2, p.ithresh) == (8, 10, 5, 20, -1)
    assert p.alpha == np.float32(0.3) and p.beta == np.float32(1 - 0.3)
    assert derive_params(16, 16, motion_threshold=999).ithresh == 255


def test_execution_times_format(tmp_path):
    """Parsed with the reference's own rules (performance_analysis.py:42-107, restated)."""
    from dvc_amd.frame_differencing import write_execution_times
    p = tmp_path / "execution_times.txt"
    write_execution_times(p, 99, 12.3456, 0.12345)
    lines = [ln.strip() for ln in open(p) if ln.strip()]
    assert lines[0] == "Frame Differencing:"
    pat = r":\s*([\d\.]+)"
    assert int(re.search(pat, lines[1]).group(1)) == 99
    assert float(re.search(pat, lines[2]).group(1)) == 12.35
    assert float(re.search(pat, lines[3]).group(1)) == 0.1235
    assert lines[4] == "Total video processing time: 12.35 seconds"


def test_npy_stream_writer_and_source(tmp_path):
    from dvc_amd import video_io
    frames = np.random.default_rng(0).integers(0, 256, (5, 24, 32, 3), dtype=np.uint8)
    w = video_io.open_sink(str(tmp_path / "out.mp4"), 25, (32, 24))
    for f in frames:
        w.write(f)
    w.write(np.zeros((10, 10, 3), np.uint8))   # wrong size: dropped like cv2.VideoWriter
    w.release()
    back = np.load(tmp_path / "out.npy")
    assert np.array_equal(back, frames)
    cap = video_io.open_source(str(tmp_path / "out.npy"))
    assert cap.isOpened() and cap.get(video_io.CAP_PROP_FPS) == 25.0
    assert cap.get(video_io.CAP_PROP_FRAME_WIDTH) == 32
    got = []
    while True:
        ok, f = cap.read()
        if not ok:
            break
        got.append(f)
    assert np.array_equal(np.stack(got), frames)
    assert not video_io.open_source(str(tmp_path / "missing.npy")).isOpened()


def test_synthetic_deterministic_and_moving():
    from dvc_amd.synthetic import SyntheticClip, background, clip
    a = clip(160, 96, 4, seed=3)
    b = clip(160, 96, 4, seed=3)
    assert np.array_equal(a, b)
    assert not np.array_equal(a[0], a[1])
    bg = background(8, 4)
    assert bg[0, 0].tolist() == [28, 28 + 29, 28 + 58]
    c = SyntheticClip(640, 360, seed=0, noisy=True)
    assert len(c.objects) == 6
    d = c.frame(1).astype(int) - SyntheticClip(640, 360, seed=0).frame(1).astype(int)
    assert 0 < (d != 0).any(-1).mean() < 0.01 and np.abs(d).max() <= 3


def _np_linear_tab(ssize, dsize):
    """Independent numpy restatement of resizeGeneric_'s INTER_LINEAR tables."""
    scale = 1.0 / (dsize / ssize)
    d = np.arange(dsize)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo, hi = s < 0, s >= ssize - 1
    f[lo | hi] = 0
    s[lo] = 0
    s[hi] = ssize - 1
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return s, a0, a1


def _np_resize(img, dw, dh):
    sh, sw = img.shape[:2]
    if (sw, sh) == (dw, dh):
        return img.copy()
    if sw == 2 * dw and sh == 2 * dh:
        f = img.astype(np.int64)
        return ((f[0::2, 0::2] + f[0::2, 1::2] + f[1::2, 0::2] + f[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    xs, xa, xb = _np_linear_tab(sw, dw)
    ys, ya, yb = _np_linear_tab(sh, dh)
    src = img.astype(np.int64)
    xs1 = np.minimum(xs + 1, sw - 1)
    Hrow = src[:, xs] * xa[None, :, None] + src[:, xs1] * xb[None, :, None]       # sh x dw x 3
    S0, S1 = Hrow[ys].reshape(dh, -1), Hrow[np.minimum(ys + 1, sh - 1)].reshape(dh, -1)
    b0, b1 = ya[:, None], yb[:, None]
    simd = ((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2
    scal = (S0 * b0 + S1 * b1 + (1 << 21)) >> 22
    w = 3 * dw
    x = 0
    while x <= w - 16:
        x += 16
    while x < w - 8:
        x += 8
    out = np.where(np.arange(w)[None, :] < x, simd, scal)
    return np.clip(out, 0, 255).astype(np.uint8).reshape(dh, dw, 3)


@pytest.mark.parametrize("sw,sh,dw,dh", [(10, 8, 10, 8), (10, 8, 5, 4), (200, 120, 140, 84), (120, 80, 156, 104),
                                         (64, 48, 37, 29), (33, 17, 66, 34), (1920, 1080, 960, 540),
                                         (1366, 768, 683, 384), (1365, 767, 682, 383)])
def test_oracle_resize_matches_numpy_restatement(oracle_lib, sw, sh, dw, dh):
    """cv2.resize INTER_LINEAR 8UC3 (fd:74,91): the C oracle vs an independent
    numpy restatement (copy / exact-2x area fast / fixed-point linear with the
    128-bit SIMD rounding prefix). OpenCV itself is absent: parity unpinned."""
    img = np.random.default_rng(sw * 7 + dh).integers(0, 256, (sh, sw, 3), dtype=np.uint8)
    assert np.array_equal(oracle_lib.resize(img, dw, dh), _np_resize(img, dw, dh))


def test_resize_simd_split():
    import oracle
    assert [oracle.resize_simd_end(w) for w in (3, 8, 9, 15, 16, 17, 24, 25, 2880, 360)] == \
        [0, 0, 8, 8, 16, 16, 16, 24, 2880, 352]


def test_video_name():
    from dvc_amd.video_io import video_name
    assert video_name("/a/b/cam01.mp4") == "cam01"
    assert video_name("synthetic://640x360?frames=5") == "640x360"


def test_unopenable_video_logs_and_returns(tmp_path, caplog):
    from dvc_amd.frame_differencing import filter_and_dilate_movements
    with caplog.at_level("ERROR"):
        assert filter_and_dilate_movements(str(tmp_path / "nope.npy"), str(tmp_path)) is None
    assert "Unable to open the video." in caplog.text


def test_shard():
    from dvc_amd.feeds import shard
    feeds = [f"cam{i}" for i in range(10)]
    parts = [shard(feeds, r, 4) for r in range(4)]
    assert sorted(sum(parts, [])) == sorted(feeds)
    assert parts[1] == ["cam1", "cam5", "cam9"]
    with pytest.raises(ValueError):
        shard(feeds, 4, 4)


def test_pingpong_order():
    import bench
    o = bench.pingpong(64)
    assert len(o) == 126 and o[0] == 0 and o[63] == 63 and o[-1] == 1
    assert all(abs(a - b) == 1 for a, b in zip(o, o[1:] + o[:1]))


def test_of_execution_times_format(tmp_path):
    """OF layout parsed with the reference's rules (performance_analysis.py:44-79, restated)."""
    from dvc_amd.motion_compression_opt import write_execution_times
    p = tmp_path / "execution_times.txt"
    write_execution_times(p, (99, 12.3456, 0.12345), (99, 1.5, 0.01515))
    lines = [ln.strip() for ln in open(p) if ln.strip()]
    pat = r":\s*([\d\.]+)"
    assert lines[0] == "Motion Detection:"
    assert int(re.search(pat, lines[1]).group(1)) == 99
    assert float(re.search(pat, lines[2]).group(1)) == 12.35
    assert float(re.search(pat, lines[3]).group(1)) == 0.1235
    ci = lines.index("Compression:")
    assert int(re.search(pat, lines[ci + 1]).group(1)) == 99
    assert float(re.search(pat, lines[ci + 2]).group(1)) == 1.5
    assert float(re.search(pat, lines[ci + 3]).group(1)) == 0.0152
    assert lines[-1] == "Total video processing time: 13.85 seconds"


def test_of_unopenable_video_returns_zeros(tmp_path, caplog):
    from dvc_amd.motion_compression_opt import compress_with_motion, temporal_smoothing_flow
    with caplog.at_level("ERROR"):
        assert temporal_smoothing_flow(str(tmp_path / "nope.npy"), str(tmp_path)) == (0, 0, 0)
        assert compress_with_motion(str(tmp_path / "a.npy"), str(tmp_path / "b.npy"), str(tmp_path)) == (0, 0, 0)
    assert "Unable to open video file" in caplog.text
    assert "Unable to open input video" in caplog.text


def test_gray_mask_stream_roundtrip(tmp_path):
    """mask.mp4 without OpenCV: a single-channel .npy stream, readable by its .mp4 name."""
    from dvc_amd import video_io
    w = video_io.open_sink(str(tmp_path / "mask.mp4"), 25, (32, 16), is_color=False)
    m = (np.arange(16 * 32).reshape(16, 32) % 2 * 255).astype(np.uint8)
    w.write(m)
    w.write(255 - m)
    w.release()
    src = video_io.open_source(str(tmp_path / "mask.mp4"))
    assert src.isOpened() and src.get(video_io.CAP_PROP_FRAME_WIDTH) == 32
    ok, f0 = src.read()
    ok1, f1 = src.read()
    assert ok and ok1 and np.array_equal(f0, m) and np.array_equal(f1, 255 - m)
    assert src.read()[0] is False


def test_div_rn_equals_ieee_division():
    """dvc_device.h div_rn: RN_f32(t/q) == (float)((double)t * RN_f64(1/q)) — the
    kernels' quantiser division (fd:123, of:166). Random and adversarial operands:
    quotients next to every half-integer (where rint would flip) and next to float
    midpoints; bit-exact against numpy's IEEE float32 division."""
    rng = np.random.default_rng(123)
    qs = np.array([100, 40, 3, 7, 0.7, 1e-3, 1e5, 64, 0.5, 1, 99.99, 1.0000001, 123456.7, 3.3e-5],
                  np.float32)
    qs = np.concatenate([qs, rng.uniform(0.01, 1000, 200).astype(np.float32),
                         np.float32(1) + np.arange(1, 200, dtype=np.float32) * np.float32(2 ** -23)])
    for q in qs:
        q = np.float32(q)
        t = np.concatenate([
            rng.uniform(-5000, 5000, 20000).astype(np.float32),
            (rng.uniform(-1, 1, 2000) * 1e-5).astype(np.float32),
            # t = (k + 0.5) * q and its float neighbours: quotients straddling rint boundaries
            ((np.arange(-60, 60) + 0.5) * q).astype(np.float32),
        ])
        t = np.concatenate([t, np.nextafter(t, np.float32(np.inf)), np.nextafter(t, np.float32(-np.inf))])
        want = t / q
        got = (t.astype(np.float64) * (1.0 / np.float64(q))).astype(np.float32)
        assert np.array_equal(want.view(np.uint32), got.view(np.uint32)), f"q={q}"
        assert np.array_equal(np.rint(want) * q, np.rint(got) * q)


def test_process_feeds_techniques(tmp_path):
    """feeds.process_feeds dispatches the reference GUI's two technique labels
    (windows.py:149-156); anything else is rejected before any GPU work."""
    from dvc_amd.feeds import process_feeds
    with pytest.raises(ValueError):
        process_feeds(["synthetic://64x48?frames=2"], str(tmp_path), technique="Background Subtraction")
    with pytest.raises(TypeError):
        process_feeds(["synthetic://64x48?frames=2"], str(tmp_path), technique="Optical Flow", min_area=3)


def _write_stream(path, n, fps, shape=(8, 16, 3), val=7):
    from dvc_amd import video_io
    w = video_io.open_sink(str(path), fps, (shape[1], shape[0]), is_color=len(shape) == 3)
    for _ in range(n):
        w.write(np.full(shape, val, np.uint8))
    w.release()


def test_performance_report(tmp_path, capsys):
    """performance_analysis.py:152-249 restated: CSV columns, durations, sizes, reduction."""
    import csv
    from dvc_amd import performance_analysis as pa
    from dvc_amd.frame_differencing import write_execution_times as fd_times
    from dvc_amd.motion_compression_opt import write_execution_times as of_times
    fd = tmp_path / "clipA"
    fd.mkdir()
    fd_times(fd / "execution_times.txt", 59, 3.0, 3.0 / 59)
    _write_stream(fd / "dilated_motion_mask_video.mp4", 60, 30)
    _write_stream(fd / "compressed_final_video.mp4", 30, 30)      # half the bytes
    of = tmp_path / "clipB"
    of.mkdir()
    of_times(of / "execution_times.txt", (99, 2.0, 0.0202), (99, 1.0, 0.0101))
    _write_stream(of / "overlay.mp4", 100, 25)
    _write_stream(of / "compressed.mp4", 100, 25)
    (tmp_path / "junk").mkdir()
    (tmp_path / "junk" / "execution_times.txt").write_text("nonsense\n")
    pa.main(["pa", str(tmp_path)])
    out = capsys.readouterr().out
    assert "Error parsing" in out and "CSV saved in" in out
    rows = list(csv.DictReader(open(tmp_path / "performance" / "performance_data.csv")))
    assert list(rows[0].keys()) == pa.FIELDNAMES
    a, b = rows
    assert a["video"] == "clipA" and int(a["md_frames"]) == 59 and int(a["cp_frames"]) == 0
    assert float(a["video_duration_seconds"]) == 2.0
    assert float(a["conversion_time_per_minute (s/min)"]) == 90.0
    hdr = 256   # NpyStreamWriter header
    assert int(a["original_size_bytes"]) == hdr + 60 * 8 * 16 * 3
    assert float(a["reduction_percentage (%)"]) == pytest.approx(100 * 30 * 384 / (hdr + 60 * 384))
    assert b["video"] == "clipB" and int(b["cp_frames"]) == 99
    assert float(b["total_processing_time (s)"]) == 3.0 and float(b["video_duration_seconds"]) == 4.0


def test_performance_report_parse_rules(tmp_path):
    from dvc_amd.performance_analysis import parse_execution_times
    p = tmp_path / "e.txt"
    p.write_text("Motion Detection:\nFrames processed: 5\nTotal time: 1.5 seconds\nAverage time per frame: 0.3 seconds\n")
    d = parse_execution_times(p)   # no Compression section, no total line: total = md + cp
    assert (d["cp_frames"], d["cp_time"], d["total_processing_time"]) == (0, 0, 1.5)
    p.write_text("")
    assert parse_execution_times(p) is None
