"""BASELINE.json configs[0] at its stated length: one 640x360 synthetic
100-frame clip through the HIP path, against the CPU oracle.

configs[0] names the reference's own CPU-runnable case
(frame_differencing.py with the GUI defaults, windows.py:154). Here the same
clip runs (a) frame by frame through dvc_fd_step, every plane and both outputs
compared with the oracle at every frame, (b) as 32-frame device batches
(the drop-in's read-ahead), and (c) end to end through the drop-in
``process_single_video_fd`` (fd:161-196): its two output videos frame for
frame and ``execution_times.txt`` (fd:152-157: 99 processed frames, frame 0
primes the feed, fd:67-81).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, N = 640, 360, 100


@pytest.fixture(scope="module")
def clip100():
    from dvc_amd.synthetic import clip
    return clip(W, H, N, seed=0)


@pytest.fixture(scope="module")
def oracle_outs(oracle_lib, clip100):
    ref = oracle_lib.OracleFD(W, H)
    ref.prime(clip100[0])
    outs = [ref.step(f)[:2] for f in clip100[1:]]
    st = ref.stats()
    ref.close()
    return outs, st


def test_config0_per_frame_every_plane(gpu_lib, oracle_lib, clip100):
    from tests.test_fd_gpu import _run_pair
    st = _run_pair(gpu_lib, oracle_lib, clip100)
    assert st["frames"] == N - 1
    assert st["components"] > 0 and st["motion_px"] > 0


def test_config0_device_batches(gpu_lib, oracle_outs, clip100):
    import torch
    outs, st = oracle_outs
    dev = torch.device("cuda", 0)
    seq = torch.from_numpy(clip100).to(dev)
    ov = torch.empty((N - 1, H, W, 3), dtype=torch.uint8, device=dev)
    cp = torch.empty_like(ov)
    w = gpu_lib.FDWorker(W, H, device=0, device_ptrs=True, max_batch=32)
    w.prime(seq[0])
    w.step_batch(seq[1:], ov, cp)     # 99 frames: launches of 32, 32, 32, 3
    w.sync()
    ovh, cph = ov.cpu().numpy(), cp.cpu().numpy()
    for t in range(N - 1):
        assert np.array_equal(ovh[t], outs[t][0]), f"overlay differs at frame {t + 1}"
        assert np.array_equal(cph[t], outs[t][1]), f"compressed differs at frame {t + 1}"
    assert w.stats() == st
    w.close()


def test_config0_dropin_process_single_video_fd(gpu_lib, oracle_outs, clip100, tmp_path, monkeypatch):
    from dvc_amd import frame_differencing as fdm
    from dvc_amd import video_io
    outs, _ = oracle_outs
    monkeypatch.delenv("DVC_VIDEO_SINK", raising=False)
    src = str(tmp_path / "clip0.npy")
    np.save(src, clip100)
    out_dir = str(tmp_path / "out")
    fdm.process_single_video_fd(src, out_dir)
    for name, k in (("dilated_motion_mask_video", 0), ("compressed_final_video", 1)):
        cap = video_io.open_source(os.path.join(out_dir, "clip0", name + ".mp4"))
        assert cap.isOpened() and cap.get(video_io.CAP_PROP_FRAME_COUNT) == N - 1
        for t in range(N - 1):
            ok, f = cap.read()
            assert ok and np.array_equal(f, outs[t][k]), f"{name} frame {t + 1}"
        cap.release()
    lines = open(os.path.join(out_dir, "clip0", "execution_times.txt")).read().split("\n")
    assert lines[0] == "Frame Differencing:"
    assert lines[1] == f"  Frames processed: {N - 1}"
    assert lines[2].startswith("  Total time: ") and lines[2].endswith(" seconds")
    assert lines[3].startswith("  Average time per frame: ")
    assert lines[5].startswith("Total video processing time: ")
