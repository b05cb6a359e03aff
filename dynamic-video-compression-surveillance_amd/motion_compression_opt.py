"""Drop-in for the reference's ``motion_compression_opt.py`` (OF path).

Same public surface, kwargs, defaults, return values and side effects:

* ``setup_logging(output_dir)``                        — ``of:8-27``
* ``temporal_smoothing_flow(video_path, output_dir, ...)`` — ``of:29-109``:
  writes ``overlay.mp4`` (the input frames) and ``mask.mp4`` (the rectangle
  mask), returns ``(frames, total_s, avg_s)``
* ``compress_with_motion(input_video, mask_video, output_dir)`` — ``of:111-193``:
  writes ``compressed.mp4``, returns ``(frames, total_s, avg_s)``
* ``process_single_video_of(video_path, output_dir)``  — ``of:195-247``:
  both steps plus ``execution_times.txt`` in the reference's format

Videos are mp4v through OpenCV when it is importable, else ``.npy`` frame
streams of the same basename (``video_io``); with the lossless streams the
two passes give exactly the fused worker's output. Error convention as the
reference's: a video that cannot be opened, or a first frame that cannot be
read, is logged and the function returns ``(0, 0, 0)`` (``of:40-42, 55-58,
123-128``); an error inside either frame loop propagates to the caller, since
neither ``of:65-101`` nor ``of:141-185`` has a ``try`` (outputs are still
released on the way out).

The per-frame work runs on the GPU: ``OFWorker`` (Farneback, vote, close/open,
rectangles; of:70-97) and ``OFCompressor`` / ``dvc_ofc_run`` (of:141-185) —
never a CPU fallback. Both loops run in chunks through ``ChunkPipeline``
(reader / GPU / writer threads). ``avg_s`` is total / frames, as of:106,190
compute it.
"""
from __future__ import annotations

import logging
import os
import time

from . import _native as N
from ._dropin import ChunkPipeline
from . import video_io
from .of import OFWorker

READ_AHEAD = int(os.environ.get("DVC_READ_AHEAD", "32"))


LOG_FORMAT = "%(asctime)s - %(levelname)s - %(message)s"


def _file_sinks(logger) -> set:
    return {h.baseFilename for h in logger.handlers if isinstance(h, logging.FileHandler)}


def setup_logging(output_dir):
    """of:8-27 behaviour: the root logger gets one truncating ``processing.log``
    sink per folder, at INFO; handlers installed by others (the GUI's) stay."""
    os.makedirs(output_dir, exist_ok=True)
    target = os.path.join(output_dir, "processing.log")
    root = logging.getLogger()
    if os.path.abspath(target) not in _file_sinks(root):
        sink = logging.FileHandler(target, mode="w")
        sink.setFormatter(logging.Formatter(LOG_FORMAT))
        root.addHandler(sink)
    root.setLevel(logging.INFO)
    root.info(f"Logging configured. Log file saved in: {target}")


def _device() -> int:
    return int(os.environ.get("DVC_DEVICE", os.environ.get("LOCAL_RANK", 0)))


def temporal_smoothing_flow(video_path, output_dir, flow_threshold=0.5, alpha_fraction=0.2,
                            window_size=30, morph_kernel=2, save_name="overlay.mp4",
                            mask_save_name="mask.mp4"):
    """of:29-109: Farneback motion mask with temporal vote, close/open and rectangles."""
    start_time = time.time()
    cap = video_io.open_source(video_path)
    if not cap.isOpened():
        logging.error(f"Error: Unable to open video file: {video_path}")
        return 0, 0, 0
    fps = cap.get(video_io.CAP_PROP_FPS)
    width = int(cap.get(video_io.CAP_PROP_FRAME_WIDTH))
    height = int(cap.get(video_io.CAP_PROP_FRAME_HEIGHT))
    out_overlay = video_io.open_sink(os.path.join(output_dir, save_name), fps, (width, height))
    out_mask = video_io.open_sink(os.path.join(output_dir, mask_save_name), fps, (width, height), is_color=False)

    ret, first_frame = cap.read()
    if not ret:
        logging.error("Error: Unable to read the first frame.")
        cap.release()
        return 0, 0, 0
    frame_count = 0
    worker = pipe = None
    try:
        # of:65-101 for READ_AHEAD frames per dvc_of_step_batch call (identical
        # to one step per frame): a reader thread reads ahead into page-locked
        # chunks, a writer thread writes the overlay (the frames themselves,
        # of:99) and mask videos while the next chunk runs (_dropin.py)
        R = max(1, READ_AHEAD)
        worker = OFWorker(width, height, device=_device(), flow_threshold=flow_threshold,
                          alpha_fraction=alpha_fraction, window_size=window_size, morph_kernel=morph_kernel,
                          max_batch=R)
        worker.prime(first_frame)

        def emit(i, outs, done, failing):
            for t in range(done):
                out_overlay.write(pipe.ins[i][t])
                out_mask.write(outs[0][t])

        pipe = ChunkPipeline(R, (height, width, 3), [(height, width)], cap.read, emit)
        pipe.start()
        while True:
            i, n = pipe.next_chunk()
            if n == 0:
                break
            j = pipe.out_buffer()
            worker.step_batch(pipe.ins[i][:n], mask=pipe.outs[j][0][:n], want=("mask",))
            pipe.write(i, j, n)
            frame_count += n
            if n < R:
                break
        pipe.finish()
    finally:   # of:65-101 has no try: an error propagates to the caller (outputs are still released here)
        if pipe is not None:
            pipe.stop()
        cap.release()
        out_overlay.release()
        out_mask.release()
        if worker is not None:
            worker.close()
    total_time = time.time() - start_time
    avg_time = total_time / frame_count if frame_count > 0 else 0
    logging.info(f"Temporal smoothing flow completed for '{os.path.basename(video_path)}' in "
                 f"{total_time:.2f} seconds. Frames processed: {frame_count}")
    return frame_count, total_time, avg_time


def compress_with_motion(input_video, mask_video, output_dir, quantization_level=100):
    """of:111-193: static 8x8 blocks (mask all zero) DCT-quantised on Y, Cr, Cb, then grey.

    The loop of:141-185 runs READ_AHEAD frame pairs per ``dvc_ofc_run`` call
    (``_native.OFCompressor``; identical to one call per frame): a reader thread
    reads the input and mask videos in lockstep into page-locked chunks (of:142-
    143, stopping at the shorter one), the GPU grays 3-channel masks (of:147-149)
    and compresses the chunk, a writer thread writes ``compressed.mp4`` (of:185)."""
    start_time = time.time()
    logging.info(f"Starting motion-based compression for: {os.path.basename(input_video)}")
    cap_input = video_io.open_source(input_video)
    cap_mask = video_io.open_source(mask_video)
    if not cap_input.isOpened():
        logging.error(f"Error: Unable to open input video: {input_video}")
        return 0, 0, 0
    if not cap_mask.isOpened():
        logging.error(f"Error: Unable to open mask video: {mask_video}")
        return 0, 0, 0
    fps = cap_input.get(video_io.CAP_PROP_FPS)
    width = int(cap_input.get(video_io.CAP_PROP_FRAME_WIDTH))
    height = int(cap_input.get(video_io.CAP_PROP_FRAME_HEIGHT))
    out = video_io.open_sink(os.path.join(output_dir, "compressed.mp4"), fps, (width, height))
    frame_count = 0
    comp = pipe = None
    try:
        ret_in, frame_in = cap_input.read()
        ret_mask, frame_mask = cap_mask.read()
        if ret_in and ret_mask:
            first = [(frame_in, frame_mask)]

            def read_pair():   # of:142-145: both videos, stop at the first missing frame
                if first:
                    return True, first.pop()
                ok_a, a = cap_input.read()
                ok_b, b = cap_mask.read()
                return (ok_a and ok_b), (a, b)

            R = max(1, READ_AHEAD)
            mshape = tuple(frame_mask.shape)   # (H, W) or (H, W, 3) as decoded
            comp = N.OFCompressor(width, height, float(quantization_level), max_batch=R, device=_device())

            def emit(i, outs, done, failing):
                for t in range(done):
                    out.write(outs[0][t])

            pipe = ChunkPipeline(R, [(height, width, 3), mshape], [(height, width, 3)], read_pair, emit)
            pipe.start()
            while True:
                i, n = pipe.next_chunk()
                if n == 0:
                    break
                j = pipe.out_buffer()
                frames, masks = pipe.ins[i]
                comp.run(frames[:n], masks[:n], out=pipe.outs[j][0][:n])
                pipe.write(i, j, n)
                frame_count += n
                if n < R:
                    break
            pipe.finish()
    finally:   # of:141-185 has no try either: errors propagate
        if pipe is not None:
            pipe.stop()
        if comp is not None:
            comp.close()
        cap_input.release()
        cap_mask.release()
        out.release()
    total_time = time.time() - start_time
    avg_time = total_time / frame_count if frame_count > 0 else 0
    logging.info(f"Motion-based compression completed for '{os.path.basename(input_video)}' in "
                 f"{total_time:.2f} seconds. Frames processed: {frame_count}")
    return frame_count, total_time, avg_time


def write_execution_times(path, md, cp):
    """of:233-244, byte-identical layout (parsed by performance_analysis.py)."""
    with open(path, "w") as f:
        f.write("Motion Detection:\n")
        f.write(f"  Frames processed: {md[0]}\n")
        f.write(f"  Total time: {md[1]:.2f} seconds\n")
        f.write(f"  Average time per frame: {md[2]:.4f} seconds\n\n")
        f.write("Compression:\n")
        f.write(f"  Frames processed: {cp[0]}\n")
        f.write(f"  Total time: {cp[1]:.2f} seconds\n")
        f.write(f"  Average time per frame: {cp[2]:.4f} seconds\n\n")
        f.write(f"Total video processing time: {md[1] + cp[1]:.2f} seconds\n")


def process_single_video_of(video_path, output_dir):
    """of:195-247."""
    video_name = video_io.video_name(video_path)
    video_output_dir = os.path.join(output_dir, video_name)
    os.makedirs(video_output_dir, exist_ok=True)
    setup_logging(video_output_dir)
    logging.info(f"=== Processing for video '{video_name}' started ===")

    logging.info("Step 1/2: Starting motion detection...")
    md = temporal_smoothing_flow(video_path, video_output_dir, flow_threshold=0.5, alpha_fraction=0.2,
                                 window_size=30, morph_kernel=2, save_name="overlay.mp4",
                                 mask_save_name="mask.mp4")
    logging.info(f"Step 1/2: Motion detection completed (elapsed: {md[1]:.2f} s, avg per frame: {md[2]:.4f} s).")

    logging.info("Step 2/2: Starting compression...")
    cp = compress_with_motion(os.path.join(video_output_dir, "overlay.mp4"),
                              os.path.join(video_output_dir, "mask.mp4"), video_output_dir)
    logging.info(f"Step 2/2: Compression completed (elapsed: {cp[1]:.2f} s, avg per frame: {cp[2]:.4f} s).")

    execution_times_path = os.path.join(video_output_dir, "execution_times.txt")
    write_execution_times(execution_times_path, md, cp)
    logging.info(f"Execution times logged in: {execution_times_path}")
    logging.info(f"=== Processing of '{video_name}' completed successfully. ===")
