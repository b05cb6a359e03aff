"""The drop-in drivers' error convention against the reference's (CPU, no GPU).

* ``motion_compression_opt.temporal_smoothing_flow`` / ``compress_with_motion``:
  the reference's frame loops (``of:65-101``, ``of:141-185``) have no ``try``,
  so an error inside them reaches the caller; an unopenable video is logged
  and returns ``(0, 0, 0)`` (``of:40-42, 123-128``).
* ``frame_differencing.filter_and_dilate_movements``: the reference's loop is
  inside ``try/except`` (``fd:84-145``): the error is logged, the loop stops,
  the function returns normally.

The GPU worker is replaced by stubs that fail on their first step (the
product path itself has no CPU fallback).
"""
import logging

import numpy as np
import pytest


class _Boom(RuntimeError):
    pass


class _FailingOF:
    def __init__(self, *a, **k):
        self.closed = False

    def prime(self, f):
        pass

    def step_batch(self, *a, **k):
        raise _Boom("step failed")

    def close(self):
        self.closed = True


class _FailingComp(_FailingOF):
    def run(self, *a, **k):
        raise _Boom("compress failed")


def test_of_flow_loop_error_propagates(tmp_path, monkeypatch):
    import dvc_amd.motion_compression_opt as mco
    made = []
    monkeypatch.setattr(mco, "OFWorker", lambda *a, **k: made.append(_FailingOF()) or made[-1])
    monkeypatch.setattr(mco.ChunkPipeline, "__init__", _np_pipeline_init(mco.ChunkPipeline.__init__))
    with pytest.raises(_Boom):
        mco.temporal_smoothing_flow("synthetic://64x48?frames=6&seed=1", str(tmp_path))
    assert made and made[0].closed            # released on the way out


def test_of_compress_loop_error_propagates(tmp_path, monkeypatch):
    import dvc_amd.motion_compression_opt as mco
    monkeypatch.setattr(mco.N, "OFCompressor", lambda *a, **k: _FailingComp())
    monkeypatch.setattr(mco.ChunkPipeline, "__init__", _np_pipeline_init(mco.ChunkPipeline.__init__))
    src = "synthetic://64x48?frames=6&seed=2"
    with pytest.raises(_Boom):
        mco.compress_with_motion(src, src, str(tmp_path))


def test_of_unopenable_video_returns_zeros(tmp_path, caplog):
    import dvc_amd.motion_compression_opt as mco
    with caplog.at_level(logging.ERROR):
        assert mco.temporal_smoothing_flow(str(tmp_path / "missing.mp4"), str(tmp_path)) == (0, 0, 0)
        assert mco.compress_with_motion(str(tmp_path / "a.mp4"), str(tmp_path / "b.mp4"), str(tmp_path)) == (0, 0, 0)
    assert "Unable to open" in caplog.text


def test_fd_loop_error_is_logged_and_stops(tmp_path, monkeypatch, caplog):
    import dvc_amd.frame_differencing as fdm

    class _FailingFD(_FailingOF):
        _fshape = _oshape = (48, 64, 3)

        def step_batch(self, *a, **k):
            raise _Boom("fd step failed")

        def step(self, *a, **k):
            raise _Boom("fd step failed")

    monkeypatch.setattr(fdm, "FDWorker", lambda *a, **k: _FailingFD())
    monkeypatch.setattr(fdm.ChunkPipeline, "__init__", _np_pipeline_init(fdm.ChunkPipeline.__init__))
    with caplog.at_level(logging.ERROR):
        fdm.filter_and_dilate_movements("synthetic://64x48?frames=6&seed=3", str(tmp_path))   # returns normally
    assert "fd step failed" in caplog.text


def _np_pipeline_init(orig):
    """ChunkPipeline with plain numpy buffers (its default is page-locked memory, a GPU call)."""
    def init(self, R, in_shape, out_shapes, read, emit, alloc=None):
        orig(self, R, in_shape, out_shapes, read, emit, alloc=lambda s: np.zeros(s, np.uint8))
    return init
