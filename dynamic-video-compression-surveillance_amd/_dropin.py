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
"""
from __future__ import annotations

import queue
import threading

from ._native import pinned


class ChunkPipeline:
    NBUF = 3

    def __init__(self, R, in_shape, out_shapes, read, emit, alloc=None):
        """``read()`` -> (ok, frame) (cap.read); ``emit(i, outs, done, failing)``
        writes the first ``done`` frames of input chunk ``i`` / output buffers
        ``outs`` (on the writer thread). ``alloc(shape)``: the buffers, default
        page-locked uint8 arrays (``_native.pinned``)."""
        self.R, self.read, self.emit = R, read, emit
        alloc = alloc or pinned
        self.ins = [alloc((R,) + tuple(in_shape)) for _ in range(self.NBUF)]
        self.outs = [tuple(alloc((R,) + tuple(s)) for s in out_shapes) for _ in range(self.NBUF)]
        self.free_in, self.free_out = queue.Queue(), queue.Queue()
        for k in range(self.NBUF):
            self.free_in.put(k)
            self.free_out.put(k)
        self.filled, self.to_write = queue.Queue(), queue.Queue()
        self.error = None
        self._stop = threading.Event()
        self.reader = self.writer = None

    def start(self):
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

    def stop(self):
        self._stop.set()
        self.free_in.put(None)
        self.to_write.put(None)
        for t in (self.reader, self.writer):
            if t is not None:
                t.join(timeout=60)
