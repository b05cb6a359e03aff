"""Drop-in for the reference's ``frame_differencing.py`` (FD path).

Public surface, kwargs, defaults and side effects are the reference's:

* ``setup_logging(output_dir)``                      — ``frame_differencing.py:7-19``
* ``filter_and_dilate_movements(video_path, ...)``   — ``frame_differencing.py:21-159``
* ``process_single_video_fd(video_path, ...)``       — ``frame_differencing.py:161-196``

Outputs go to ``<output_dir>/<video basename>/``: ``dilated_motion_mask_video``
and ``compressed_final_video`` (mp4v through OpenCV when importable, else an
``.npy`` frame stream of the same basename), ``execution_times.txt`` in the
reference's exact format, and ``processing.log``. Errors are logged and the
functions return ``None`` (``fd:40-42, 68-71, 140-145``).

The per-frame work (``fd:91-133``, resize included) runs on the GPU through
``FDWorker`` — the HIP kernels in ``csrc/`` — never through a CPU fallback. The
frames are read ahead ``DVC_READ_AHEAD`` (default 32) at a time into
page-locked buffers and stepped with one ``dvc_fd_step_batch`` call per group
(identical results to one call per frame, which the batch tests prove): the
device runs the group as launches over tiles x frames and the host copies
overlap with the computation, instead of a synchronous round trip per frame.
"""
from __future__ import annotations

import logging
import os
import time

from . import video_io
from ._dropin import ChunkPipeline
from ._native import DVC_E_ODD_DCT, DvcError
from .fd import FDWorker

LOG_FORMAT = "%(asctime)s - %(levelname)s - %(message)s"
READ_AHEAD = int(os.environ.get("DVC_READ_AHEAD", "32"))


def setup_logging(output_dir):
    """fd:7-19: ``processing.log`` (truncated) plus the console. Like the
    reference it relies on ``basicConfig``, so it is a no-op when the process
    has configured logging already (e.g. the GUI's handler)."""
    os.makedirs(output_dir, exist_ok=True)
    log_path = os.path.join(output_dir, "processing.log")
    sinks = [logging.FileHandler(log_path, mode="w"), logging.StreamHandler()]
    logging.basicConfig(level=logging.INFO, format=LOG_FORMAT, handlers=sinks)
    logging.info(f"Logging configured. Log file saved in: {log_path}")


def _device() -> int:
    return int(os.environ.get("DVC_DEVICE", os.environ.get("LOCAL_RANK", 0)))


def _feed_dir(output_dir, video_path) -> str:
    """<output_dir>/<basename without extension> (fd:45-46, fd:177-178)."""
    return os.path.join(output_dir, video_io.video_name(video_path))


class _Writers:
    """The two mp4v outputs of fd:63-65 plus the progress callback of fd:137-138.
    ``yuv``: both sinks are Y4M videos and take the worker's I420 frames as they
    are (no BGR round trip through the host)."""

    def __init__(self, out_dir, fps, size, progress_callback):
        self.mask = video_io.open_sink(os.path.join(out_dir, "dilated_motion_mask_video.mp4"), fps, size)
        self.final = video_io.open_sink(os.path.join(out_dir, "compressed_final_video.mp4"), fps, size)
        self.callback = progress_callback
        self.frames = 0
        self.yuv = isinstance(self.mask, video_io.Y4mWriter) and isinstance(self.final, video_io.Y4mWriter)

    def emit(self, overlay, compressed):
        put = (lambda s, f: s.write_yuv(f)) if self.yuv else (lambda s, f: s.write(f))
        put(self.mask, overlay)
        if compressed is None:       # the frame whose block loop raised: overlay only (fd:112 < fd:122)
            return
        put(self.final, compressed)
        self.frames += 1
        if self.callback is not None and self.frames % 50 == 0:
            self.callback(self.frames)

    def release(self):
        self.mask.release()
        self.final.release()


def filter_and_dilate_movements(video_path, output_dir,
                                block_size=4,
                                search_area=16,
                                motion_threshold=0.5,
                                min_area=500,
                                kernel_size=7,
                                release_factor=0.5,
                                quantization_level=100,
                                scale_factor=1.0,
                                progress_callback=None):
    """fd:21-159. ``search_area`` is accepted and unused, as in the reference."""
    t_start = time.time()
    cap = video_io.open_source(video_path)
    if not cap.isOpened():
        logging.error("Unable to open the video.")
        return
    out_dir = _feed_dir(output_dir, video_path)
    os.makedirs(out_dir, exist_ok=True)
    setup_logging(out_dir)
    times_path = os.path.join(out_dir, "execution_times.txt")

    fps = int(cap.get(video_io.CAP_PROP_FPS))
    src_w = int(cap.get(video_io.CAP_PROP_FRAME_WIDTH))
    src_h = int(cap.get(video_io.CAP_PROP_FRAME_HEIGHT))
    out_w, out_h = int(src_w * scale_factor), int(src_h * scale_factor)   # fd:60-61
    sinks = _Writers(out_dir, fps, (out_w, out_h), progress_callback)

    # a 4:2:0 source (Y4M; a hardware decoder's surfaces) goes to the worker as
    # is: it converts on the GPU exactly as VideoCapture.read() would (fd:87)
    yuv = getattr(cap, "pixel_format", "BGR") != "BGR"
    read = cap.read_yuv if yuv else cap.read
    ok, first = read()
    if not ok:
        logging.error("Unable to read the first frame of the video.")
        cap.release()
        return

    per_frame_s = []
    worker = None
    reader = writer = None
    try:
        R = max(1, READ_AHEAD)
        blk = block_size
        i420 = sinks.yuv and blk in (4, 8) and out_w % blk == 0 and out_h % blk == 0
        worker = FDWorker(out_w, out_h, device=_device(), src_width=src_w, src_height=src_h, max_batch=R,
                          block_size=block_size, motion_threshold=motion_threshold, min_area=min_area,
                          kernel_size=kernel_size, release_factor=release_factor,
                          quantization_level=quantization_level, in_format=cap.pixel_format if yuv else "BGR",
                          out_format="I420" if i420 else "BGR")
        if not i420:
            sinks.yuv = False
        worker.prime(first)                                     # fd:67-81 (resize on the GPU)

        def emit(i, ov_cp, done, failing):                      # writer thread: fd:112,131,137-138
            ov, cp = ov_cp
            for t in range(done):
                sinks.emit(ov[t], cp[t])
            if failing:
                sinks.emit(ov[done], None)

        pipe = ChunkPipeline(R, worker._fshape, [worker._oshape, worker._oshape], read, emit)
        reader, writer = pipe.start()
        handed = 0                                              # frames given to the writer
        while True:
            i, n = pipe.next_chunk()                            # fd:87-89, R frames ahead
            if n == 0:
                break
            j = pipe.out_buffer()
            ov, cp = pipe.outs[j]
            stop = None
            try:                                                # fd:91-133, n times
                worker.step_batch(pipe.ins[i][:n], ov[:n], cp[:n])
                done = n
            except DvcError as e:
                if e.code != DVC_E_ODD_DCT:
                    raise
                stop, done = e, worker.stats()["frames"] - handed
            pipe.write(i, j, done, stop is not None)
            handed += done
            if stop is not None:
                pipe.finish()
                raise RuntimeError("OpenCV(4.11.0) (-213:The function/feature is not implemented) "
                                   "Odd-size DCT's are not implemented in function 'apply'") from stop
            if n < R:
                break
        pipe.finish()
    except Exception as e:
        logging.error("Error during processing: " + str(e), exc_info=True)
    finally:
        if reader is not None:
            pipe.stop()
            # fd:86,135 per frame: read -> last write, as the run sees it (_dropin.py)
            per_frame_s = pipe.frame_times()[:sinks.frames]
        cap.release()
        sinks.release()
        if worker is not None:
            worker.close()

    total_time = time.time() - t_start
    avg = sum(per_frame_s) / len(per_frame_s) if per_frame_s else 0
    write_execution_times(times_path, sinks.frames, total_time, avg)
    logging.info(f"Execution statistics saved in: {times_path}")


def write_execution_times(path, frame_count, total_time, avg_time_per_frame):
    """fd:152-157, byte-identical layout (parsed by performance_analysis.py:44-109)."""
    lines = ["Frame Differencing:",
             f"  Frames processed: {frame_count}",
             f"  Total time: {total_time:.2f} seconds",
             f"  Average time per frame: {avg_time_per_frame:.4f} seconds",
             "",
             f"Total video processing time: {total_time:.2f} seconds"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def process_single_video_fd(video_path,
                            output_dir,
                            block_size=4,
                            search_area=16,
                            motion_threshold=0.5,
                            min_area=500,
                            kernel_size=7,
                            release_factor=0.5,
                            quantization_level=100,
                            scale_factor=1.0,
                            progress_callback=None):
    """fd:161-196: the per-video entry point the GUI calls (windows.py:154) —
    prepares the feed's folder and log, then runs the worker with every kwarg."""
    options = dict(block_size=block_size, search_area=search_area, motion_threshold=motion_threshold,
                   min_area=min_area, kernel_size=kernel_size, release_factor=release_factor,
                   quantization_level=quantization_level, scale_factor=scale_factor,
                   progress_callback=progress_callback)
    name = video_io.video_name(video_path)
    out_dir = _feed_dir(output_dir, video_path)
    os.makedirs(out_dir, exist_ok=True)
    setup_logging(out_dir)
    logging.info(f"=== Start processing (Frame Differencing) for '{name}' ===")
    filter_and_dilate_movements(video_path, output_dir, **options)
    logging.info(f"=== Processing successfully completed for '{name}'. ===")
