"""Host logic of the drop-in drivers' reader / step / writer threads
(dvc_amd/_dropin.py) with plain numpy buffers and a CPU "step": chunking,
order, end of video at and off chunk boundaries, the failing-frame hand-off of
the odd-DCT stop, and error propagation from either thread (no GPU)."""
import threading

import numpy as np
import pytest

from dvc_amd._dropin import ChunkPipeline


def _source(n, shape=(2, 3)):
    frames = [np.full(shape, t, np.uint8) for t in range(n)]
    it = iter(frames)

    def read():
        f = next(it, None)
        return (f is not None), f
    return frames, read


def _run(n, R, fail_at=None):
    """Drive the pipeline like frame_differencing: out = in + 1, stop at fail_at."""
    frames, read = _source(n)
    written, failed = [], []

    def emit(i, outs, done, failing):
        assert threading.current_thread().name == "dvc-writer"
        written.extend(outs[0][t].copy() for t in range(done))
        if failing:
            failed.append(outs[0][done].copy())

    pipe = ChunkPipeline(R, (2, 3), [(2, 3)], read, emit, alloc=lambda s: np.zeros(s, np.uint8))
    pipe.start()
    handed = 0
    try:
        while True:
            i, n_ = pipe.next_chunk()
            if n_ == 0:
                break
            j = pipe.out_buffer()
            pipe.outs[j][0][:n_] = pipe.ins[i][:n_] + 1
            done = n_ if fail_at is None or handed + n_ <= fail_at else fail_at - handed
            pipe.write(i, j, done, done < n_)
            handed += done
            if done < n_ or n_ < R:
                break
        pipe.finish()
    finally:
        pipe.stop()
    return frames, written, failed


@pytest.mark.parametrize("n,R", [(10, 4), (12, 4), (3, 8), (1, 1), (0, 4), (25, 1)])
def test_chunks_in_order(n, R):
    frames, written, failed = _run(n, R)
    assert len(written) == n and not failed
    for t, w in enumerate(written):
        assert np.array_equal(w, frames[t] + 1)


def test_failing_frame_handoff():
    frames, written, failed = _run(11, 4, fail_at=6)   # frame 6 (second chunk) stops the run
    assert len(written) == 6 and len(failed) == 1
    assert np.array_equal(failed[0], frames[6] + 1)


def test_reader_error_surfaces():
    def read():
        raise IOError("disk gone")
    pipe = ChunkPipeline(4, (2,), [(2,)], read, lambda *a: None, alloc=lambda s: np.zeros(s, np.uint8))
    pipe.start()
    with pytest.raises(IOError, match="disk gone"):
        pipe.next_chunk()
    pipe.stop()


def test_writer_error_surfaces():
    _, read = _source(20)

    def emit(i, outs, done, failing):
        raise ValueError("sink full")
    pipe = ChunkPipeline(4, (2, 3), [(2, 3)], read, emit, alloc=lambda s: np.zeros(s, np.uint8))
    pipe.start()
    with pytest.raises(ValueError, match="sink full"):
        for _ in range(ChunkPipeline.NBUF + 2):   # the writer fails on the first chunk
            i, n = pipe.next_chunk()
            pipe.write(i, pipe.out_buffer(), n)
        pipe.finish()
    pipe.stop()


def test_frame_times_sum_to_loop_time():
    """execution_times.txt's per-frame time (fd:86,135): one entry per written
    frame, positive, and frames x average <= the wall time around the loop —
    the reference's sequential loop gives exactly that sum."""
    import time

    frames, read = _source(23)
    slow_read = lambda: (time.sleep(0.002), read())[1]   # noqa: E731
    pipe = ChunkPipeline(4, (2, 3), [(2, 3)], slow_read, lambda i, outs, done, failing: time.sleep(0.003),
                         alloc=lambda s: np.zeros(s, np.uint8))
    t0 = time.time()
    pipe.start()
    try:
        while True:
            i, n = pipe.next_chunk()
            if n == 0:
                break
            j = pipe.out_buffer()
            time.sleep(0.004)                               # the "step"
            pipe.write(i, j, n)
            if n < 4:
                break
        pipe.finish()
    finally:
        pipe.stop()
    total = time.time() - t0
    ft = pipe.frame_times()
    assert len(ft) == 23 and all(t > 0 for t in ft)
    assert sum(ft) <= total + 1e-6
    assert sum(ft) >= 0.5 * total                           # the loop is the run



def test_two_videos_in_lockstep():
    """compress_with_motion reads the input and mask videos together (of:142-
    145) and stops at the shorter one: a list of input shapes gives one chunk
    array per video."""
    a = iter([np.full((2, 3), t, np.uint8) for t in range(9)])
    b = iter([np.full((2,), 100 + t, np.uint8) for t in range(7)])

    def read():
        x, y = next(a, None), next(b, None)
        return (x is not None and y is not None), (x, y)
    got = []
    pipe = ChunkPipeline(3, [(2, 3), (2,)], [(2,)], read,
                         lambda i, outs, done, failing: got.extend(outs[0][t].copy() for t in range(done)),
                         alloc=lambda s: np.zeros(s, np.uint8))
    pipe.start()
    try:
        while True:
            i, n = pipe.next_chunk()
            if n == 0:
                break
            fa, fb = pipe.ins[i]
            j = pipe.out_buffer()
            pipe.outs[j][0][:n] = fa[:n, :, 0] + fb[:n]
            pipe.write(i, j, n)
            if n < 3:
                break
        pipe.finish()
    finally:
        pipe.stop()
    assert len(got) == 7
    for t, g in enumerate(got):
        assert np.array_equal(g, np.full((2,), 100 + 2 * t, np.uint8))
