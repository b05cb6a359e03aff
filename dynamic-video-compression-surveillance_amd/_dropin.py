"""Host side of the drop-in drivers' frame loops (``frame_differencing.py:85-138``,
``motion_compression_opt.py:65-101``) in three threads.

The reference reads a frame, processes it and writes it, one after the other.
Here a reader thread fills page-locked chunks of R frames (``cap.read()``),
the calling thread steps each chunk with one ``step_batch`` call on the GPU,
and a writer thread emits the outputs (``VideoWriter.write``): reading chunk
c+1 and writing chunk c-1 overlap chunk c's step instead of adding to it.
Three buffers each way; file I/O, frame copies and the ctypes calls release
the GIL. An input chunk is recycled after the writer is done with it (the
OF driver writes the input frames as its overlay video).

Per-frame time (``frame_times``): the reference times each frame from its
``cap.read()`` to its last ``write`` (``frame_differencing.py:86,135``); its loop
is sequential, so that interval is also the time the frame adds to the run and
the per-frame times sum to the loop's wall time. The pipeline keeps that
second meaning: a frame's time is the wall-clock interval between the write
completion of the frame before it and its own (the first frame's starts at the
pipeline's first read), spread evenly over the frames of a chunk. So
frames x average = the loop's wall time <= the run's total time, as in the
reference; a frame's read-to-write latency inside the pipeline (about three
chunk periods) is not what the file reports.
"""
from __future__ import annotations

import queue
import threading
import time

from ._native import pinned


class ChunkPipeline:
    NBUF = 3

    def __init__(self, R, in_shape, out_shapes, read, emit, alloc=None):
        """``read()`` -> (ok, frame) (cap.read); ``emit(i, outs, done, failing)``
        writes the first ``done`` frames of input chunk ``i`` / output buffers
        ``outs`` (on the writer thread). ``alloc(shape)``: the buffers, default
        page-locked uint8 arrays (``_native.pinned``). ``in_shape`` may be a
        list of shapes: then ``read()`` returns (ok, (frame_a, frame_b, ..)) —
        several videos read in lockstep (compress_with_motion, of:142-143) —
        and ``ins[i]`` is a tuple of chunk arrays."""
        self.R, self.read, self.emit = R, read, emit
        alloc = alloc or pinned
        self.multi = isinstance(in_shape, list)
        shapes = in_shape if self.multi else [in_shape]
        self.ins = [tuple(alloc((R,) + tuple(sh)) for sh in shapes) for _ in range(self.NBUF)]
        if not self.multi:
            self.ins = [x[0] for x in self.ins]
        self.outs = [tuple(alloc((R,) + tuple(s)) for s in out_shapes) for _ in range(self.NBUF)]
        self.free_in, self.free_out = queue.Queue(), queue.Queue()
        for k in range(self.NBUF):
            self.free_in.put(k)
            self.free_out.put(k)
        self.filled, self.to_write = queue.Queue(), queue.Queue()
        self.error = None
        self._stop = threading.Event()
        self.reader = self.writer = None
        self.t0 = None
        self.departures = []             # (time the chunk's last write returned, frames in it)

    def start(self):
        self.t0 = time.time()
        self.reader = threading.Thread(target=self._read_loop, name="dvc-reader", daemon=True)
        self.writer = threading.Thread(target=self._write_loop, name="dvc-writer", daemon=True)
        self.reader.start()
        self.writer.start()
        return self.reader, self.writer

    def _read_loop(self):
        try:
            while not self._stop.is_set():
                i = self.free_in.get()
                if i is None:
                    return
                n = 0
                while n < self.R:
                    ok, f = self.read()
                    if not ok:
                        break
                    if self.multi:
                        for buf, x in zip(self.ins[i], f):
                            buf[n] = x
                    else:
                        self.ins[i][n] = f
                    n += 1
                self.filled.put((i, n))
                if n < self.R:           # end of the video
                    return
        except Exception as e:           # surfaced by next_chunk
            self.error = e
            self.filled.put((None, 0))

    def _write_loop(self):
        try:
            while True:
                item = self.to_write.get()
                if item is None:
                    return
                i, j, done, failing = item
                self.emit(i, self.outs[j], done, failing)
                self.departures.append((time.time(), done))
                self.free_out.put(j)
                self.free_in.put(i)
        except Exception as e:           # surfaced by next_chunk / out_buffer / finish
            self.error = e
            self.free_out.put(None)
            self.free_in.put(None)       # the reader stops
            self.filled.put((None, 0))   # a caller waiting for a chunk wakes up

    def next_chunk(self):
        """(input chunk index, frames in it); 0 frames at the end of the video."""
        i, n = self.filled.get()
        if self.error is not None:
            raise self.error
        return i, n

    def out_buffer(self):
        j = self.free_out.get()
        if j is None:
            raise self.error
        return j

    def write(self, i, j, done, failing=False):
        self.to_write.put((i, j, done, failing))

    def finish(self):
        """Wait until every chunk handed to write() is written."""
        self.to_write.put(None)
        self.writer.join()
        if self.error is not None:
            raise self.error

    def frame_times(self):
        """Seconds per written frame (module docstring): chunk c's frames share
        the interval since chunk c-1's writes completed."""
        out, prev = [], self.t0
        for t, done in self.departures:
            if done > 0:
                out.extend([(t - prev) / done] * done)
                prev = t
        return out

    def stop(self):
        self._stop.set()
        self.free_in.put(None)
        self.to_write.put(None)
        for t in (self.reader, self.writer):
            if t is not None:
                t.join(timeout=60)
