"""Drop-in for the reference's ``frame_differencing.py`` (FD path).

Same public surface, same kwargs and defaults, same side effects:

* ``setup_logging(output_dir)``                      — ``frame_differencing.py:7-19``
* ``filter_and_dilate_movements(video_path, ...)``   — ``frame_differencing.py:21-159``
* ``process_single_video_fd(video_path, ...)``       — ``frame_differencing.py:161-196``

Outputs go to ``<output_dir>/<video basename>/``: ``dilated_motion_mask_video``
and ``compressed_final_video`` (mp4v through OpenCV when importable, else an
``.npy`` frame stream of the same basename), ``execution_times.txt`` in the
reference's exact format, and ``processing.log``. Errors are logged and the
functions return ``None``, as the reference does (``fd:40-42, 68-71, 140-145``).

The per-frame work (``fd:91-133``) runs on the GPU through ``FDWorker`` — the
HIP kernels in ``csrc/`` — never through a CPU fallback.
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np

from . import video_io
from .fd import FDWorker


def setup_logging(output_dir):
    """fd:7-19: processing.log + console; a no-op basicConfig if logging is set up."""
    os.makedirs(output_dir, exist_ok=True)
    log_file = os.path.join(output_dir, "processing.log")
    logging.basicConfig(level=logging.INFO,
                        format="%(asctime)s - %(levelname)s - %(message)s",
                        handlers=[logging.FileHandler(log_file, mode='w'),
                                  logging.StreamHandler()])
    logging.info(f"Logging configured. Log file saved in: {log_file}")


def resize_frame(frame: np.ndarray, size) -> np.ndarray:
    """cv2.resize(frame, (sw, sh)) with INTER_LINEAR (fd:74,91).

    * dsize == ssize: OpenCV copies the frame (the GUI default scale 1.0).
    * exact 2x downscale: OpenCV turns INTER_LINEAR into the fast INTER_AREA
      path, ``(a + b + c + d + 2) >> 2`` per 2x2 block.
    Other scale factors are not implemented and raise.
    """
    sw, sh = int(size[0]), int(size[1])
    h, w = frame.shape[:2]
    if (sw, sh) == (w, h):
        return frame
    if sw * 2 == w and sh * 2 == h:
        f = frame.astype(np.uint16)
        s = f[0::2, 0::2] + f[0::2, 1::2] + f[1::2, 0::2] + f[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    raise NotImplementedError(f"scale to {sw}x{sh} from {w}x{h}: only 1.0 and exact 0.5 are implemented")


def _device() -> int:
    return int(os.environ.get("DVC_DEVICE", os.environ.get("LOCAL_RANK", 0)))


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
    start_time = time.time()
    cap = video_io.open_source(video_path)
    if not cap.isOpened():
        logging.error("Unable to open the video.")
        return

    video_name = video_io.video_name(video_path)
    video_output_dir = os.path.join(output_dir, video_name)
    os.makedirs(video_output_dir, exist_ok=True)
    setup_logging(video_output_dir)

    mask_output_path = os.path.join(video_output_dir, "dilated_motion_mask_video.mp4")
    final_output_path = os.path.join(video_output_dir, "compressed_final_video.mp4")
    time_log_path = os.path.join(video_output_dir, "execution_times.txt")

    fps = int(cap.get(video_io.CAP_PROP_FPS))
    width = int(cap.get(video_io.CAP_PROP_FRAME_WIDTH))
    height = int(cap.get(video_io.CAP_PROP_FRAME_HEIGHT))
    scaled_width = int(width * scale_factor)
    scaled_height = int(height * scale_factor)

    mask_out = video_io.open_sink(mask_output_path, fps, (scaled_width, scaled_height))
    final_out = video_io.open_sink(final_output_path, fps, (scaled_width, scaled_height))

    ret, prev_frame = cap.read()
    if not ret:
        logging.error("Unable to read the first frame of the video.")
        cap.release()
        return

    frame_count = 0
    frame_processing_times = []
    worker = None
    try:
        prev_frame = resize_frame(prev_frame, (scaled_width, scaled_height))
        worker = FDWorker(scaled_width, scaled_height, device=_device(),
                          block_size=block_size, motion_threshold=motion_threshold, min_area=min_area,
                          kernel_size=kernel_size, release_factor=release_factor,
                          quantization_level=quantization_level)
        worker.prime(prev_frame)
        overlay = np.empty((scaled_height, scaled_width, 3), np.uint8)
        compressed = np.empty_like(overlay)
        while True:
            frame_start = time.time()
            ret, curr_frame = cap.read()
            if not ret:
                break
            curr_frame = resize_frame(curr_frame, (scaled_width, scaled_height))
            worker.step(curr_frame, overlay, compressed)
            mask_out.write(overlay)
            final_out.write(compressed)
            frame_count += 1
            frame_processing_times.append(time.time() - frame_start)
            if progress_callback is not None and frame_count % 50 == 0:
                progress_callback(frame_count)
    except Exception as e:
        logging.error("Error during processing: " + str(e), exc_info=True)
    finally:
        cap.release()
        mask_out.release()
        final_out.release()
        if worker is not None:
            worker.close()

    total_time = time.time() - start_time
    avg_time_per_frame = (sum(frame_processing_times) / len(frame_processing_times)
                          if frame_processing_times else 0)
    write_execution_times(time_log_path, frame_count, total_time, avg_time_per_frame)
    logging.info(f"Execution statistics saved in: {time_log_path}")


def write_execution_times(path, frame_count, total_time, avg_time_per_frame):
    """fd:152-157, byte-identical layout (parsed by performance_analysis.py:44-109)."""
    with open(path, "w") as f:
        f.write("Frame Differencing:\n")
        f.write(f"  Frames processed: {frame_count}\n")
        f.write(f"  Total time: {total_time:.2f} seconds\n")
        f.write(f"  Average time per frame: {avg_time_per_frame:.4f} seconds\n\n")
        f.write(f"Total video processing time: {total_time:.2f} seconds\n")


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
    """fd:161-196."""
    video_name = video_io.video_name(video_path)
    video_output_dir = os.path.join(output_dir, video_name)
    os.makedirs(video_output_dir, exist_ok=True)

    setup_logging(video_output_dir)
    logging.info(f"=== Start processing (Frame Differencing) for '{video_name}' ===")

    filter_and_dilate_movements(video_path,
                                output_dir,
                                block_size=block_size,
                                search_area=search_area,
                                motion_threshold=motion_threshold,
                                min_area=min_area,
                                kernel_size=kernel_size,
                                release_factor=release_factor,
                                quantization_level=quantization_level,
                                scale_factor=scale_factor,
                                progress_callback=progress_callback)

    logging.info(f"=== Processing successfully completed for '{video_name}'. ===")
