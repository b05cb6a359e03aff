"""Video I/O on the CPU: the 4:2:0 <-> BGR conversion oracle
(oracle/yuv_oracle.c, OpenCV 4.11 cvtColor restated) on known answers, and
the YUV4MPEG2 container reader/writer (no GPU calls).

Parity status: cv2 is not importable here, so the conversions are
parity-UNPINNED against OpenCV itself; the known answers below are the BT.601
limited-range values any conforming converter produces (black, white, the
primaries), and the GPU kernels are held bit-exact to this oracle
(tests/test_video_io_gpu.py)."""
import os

import numpy as np
import pytest


def _i420(Y, U, V):
    return np.concatenate([Y.ravel(), U.ravel(), V.ravel()]).reshape(Y.shape[0] * 3 // 2, Y.shape[1])


def test_yuv_oracle_known_answers(oracle_lib):
    o = oracle_lib
    H, W = 4, 6
    for y, u, v, bgr in [(16, 128, 128, (0, 0, 0)), (235, 128, 128, (255, 255, 255)), (0, 128, 128, (0, 0, 0)),
                         (126, 128, 128, (128, 128, 128)), (82, 90, 240, (0, 1, 255)), (145, 54, 34, (0, 255, 0)),
                         (41, 240, 110, (255, 0, 0))]:
        f = _i420(np.full((H, W), y, np.uint8), np.full((H // 2, W // 2), u, np.uint8),
                  np.full((H // 2, W // 2), v, np.uint8))
        out = o.yuv420_to_bgr(f)
        assert out.shape == (H, W, 3)
        assert np.abs(out.astype(int) - np.array(bgr)).max() <= 1, (y, u, v, out[0, 0])
    # BGR -> YUV on the primaries (BT.601 limited range)
    for bgr, yuv in [((0, 0, 0), (16, 128, 128)), ((255, 255, 255), (235, 128, 128)), ((0, 0, 255), (82, 90, 240)),
                     ((0, 255, 0), (145, 54, 34)), ((255, 0, 0), (41, 240, 110))]:
        f = o.bgr_to_i420(np.broadcast_to(np.array(bgr, np.uint8), (H, W, 3)).copy())
        assert (f[0, 0], f[H, 0], f[H + H // 4, 0]) == yuv, (bgr, f[0, 0], f[H, 0], f[H + H // 4, 0])


def test_yuv_oracle_layouts_and_roundtrip(oracle_lib):
    o = oracle_lib
    rng = np.random.default_rng(1)
    H, W = 10, 14
    Y = rng.integers(0, 256, (H, W), dtype=np.uint8)
    U = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
    V = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
    i420 = _i420(Y, U, V)
    nv12 = np.concatenate([Y, np.stack([U, V], -1).reshape(H // 2, W)])
    a, b = o.yuv420_to_bgr(i420), o.yuv420_to_bgr(nv12, "NV12")
    assert np.array_equal(a, b)
    # chroma sample (i, j) serves the 2x2 luma quad: equal luma in a quad -> equal BGR
    q = _i420(np.repeat(np.repeat(Y[::2, ::2], 2, 0), 2, 1), U, V)
    out = o.yuv420_to_bgr(q)
    assert np.array_equal(out[0::2, 0::2], out[1::2, 1::2])
    # smooth content survives BGR -> I420 -> BGR within the 4:2:0 / 8-bit error
    g = np.linspace(40, 200, W, dtype=np.float64)
    smooth = np.stack([np.tile(g, (H, 1)), np.tile(g[::-1], (H, 1)), np.full((H, W), 120.0)], -1).astype(np.uint8)
    back = o.yuv420_to_bgr(o.bgr_to_i420(smooth))
    assert np.abs(back.astype(int) - smooth.astype(int)).max() <= 24


def _write_y4m(path, frames_i420, W, H, fps="30:1", extra=b""):
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F%s Ip A1:1 C420jpeg%s\n" % (W, H, fps.encode(), extra))
        for fr in frames_i420:
            f.write(b"FRAME\n")
            f.write(fr.tobytes())


def test_y4m_reader_container(tmp_path, oracle_lib):
    from dvc_amd import video_io
    from dvc_amd.synthetic import clip
    W, H = 96, 64
    frames = clip(W, H, 5, seed=2)
    yuv = [oracle_lib.bgr_to_i420(f) for f in frames]
    p = str(tmp_path / "cam.y4m")
    _write_y4m(p, yuv, W, H, "25:1")
    cap = video_io.open_source(p)
    assert cap.isOpened() and cap.pixel_format == "I420"
    assert (cap.get(video_io.CAP_PROP_FRAME_WIDTH), cap.get(video_io.CAP_PROP_FRAME_HEIGHT)) == (W, H)
    assert cap.get(video_io.CAP_PROP_FPS) == 25.0 and cap.get(video_io.CAP_PROP_FRAME_COUNT) == 5
    for t in range(5):
        ok, f = cap.read_yuv()
        assert ok and f.shape == (H * 3 // 2, W) and np.array_equal(f, yuv[t])
    assert cap.read_yuv() == (False, None)
    assert video_io.video_name(p) == "cam"
    # an .mp4 name this package wrote as .y4m (no OpenCV) resolves to it
    assert video_io.open_source(str(tmp_path / "cam.mp4")).isOpened()
    # truncated last frame: dropped; bad header / 4:4:4: not opened
    with open(p, "ab") as f:
        f.write(b"FRAME\n" + bytes(10))
    assert video_io.open_source(p).get(video_io.CAP_PROP_FRAME_COUNT) == 5
    bad = str(tmp_path / "bad.y4m")
    with open(bad, "wb") as f:
        f.write(b"YUV4MPEG2 W8 H8 F30:1 C444\nFRAME\n" + bytes(192))
    assert not video_io.open_source(bad).isOpened()
    with open(bad, "wb") as f:
        f.write(b"NOTY4M W8 H8\n")
    assert not video_io.open_source(bad).isOpened()


def test_y4m_writer_mono_and_sink_selection(tmp_path, monkeypatch):
    from dvc_amd import video_io
    W, H = 10, 6
    w = video_io.open_sink(str(tmp_path / "mask.y4m"), 30, (W, H), is_color=False)
    assert isinstance(w, video_io.Y4mWriter) and w.isOpened()
    m = (np.arange(W * H).reshape(H, W) % 256).astype(np.uint8)
    w.write(m)
    w.write(np.zeros((H, W + 1), np.uint8))       # wrong size: dropped like cv2.VideoWriter
    w.release()
    data = open(str(tmp_path / "mask.y4m"), "rb").read()
    head, rest = data.split(b"\n", 1)
    assert head.split() == [b"YUV4MPEG2", b"W10", b"H6", b"F30:1", b"Ip", b"A1:1", b"Cmono"]
    assert rest == b"FRAME\n" + m.tobytes()
    # default sink without OpenCV: lossless .npy; DVC_VIDEO_SINK=y4m selects YUV4MPEG2
    if video_io.cv2 is None:
        s = video_io.open_sink(str(tmp_path / "out.mp4"), 30, (W, H))
        assert isinstance(s, video_io.NpyStreamWriter)
        s.release()
        monkeypatch.setenv("DVC_VIDEO_SINK", "y4m")
        s = video_io.open_sink(str(tmp_path / "out2.mp4"), 30, (W, H), is_color=False)
        assert isinstance(s, video_io.Y4mWriter) and s.path.endswith("out2.y4m")
        s.release()
    # odd sides cannot be 4:2:0
    assert not video_io.Y4mWriter(str(tmp_path / "odd.y4m"), 30, (9, 6)).isOpened()
    assert os.path.exists(str(tmp_path / "mask.y4m"))
