"""Per-run performance report over an output folder.

Same surface and outputs as the reference's ``performance_analysis.py``: for
every ``<output_folder>/<video>/execution_times.txt`` written by the FD or OF
driver it reads the timings, the duration of the "original" output video and
the sizes of the original / compressed outputs, and writes
``<output_folder>/performance/performance_data.csv`` with the reference's
columns (``performance_analysis.py:213-248``) plus the two charts
(``:251-286``) when matplotlib is importable.

Differences, both because this image has no OpenCV:
* videos are opened through :mod:`video_io`, so an output written as an
  ``.npy`` frame stream (no ``mp4v`` encoder here) is found by its ``.mp4``
  name, its duration is frames / fps from the stream's sidecar;
* sizes of such streams are raw frame bytes, so the "reduction" column only
  means codec compression when the outputs really are ``mp4v`` files.
"""
from __future__ import annotations

import csv
import logging
import os
import re
import sys

from . import video_io

_NUM = re.compile(r":\s*([\d\.]+)")

FIELDNAMES = [   # performance_analysis.py:213-227
    "video",
    "md_frames",
    "md_time (s)",
    "md_avg (s/frame)",
    "cp_frames",
    "cp_time (s)",
    "cp_avg (s/frame)",
    "total_processing_time (s)",
    "video_duration_seconds",
    "conversion_time_per_minute (s/min)",
    "original_size_bytes",
    "compressed_size_bytes",
    "reduction_percentage (%)",
]


def _section(lines, start):
    """(frames, total_s, avg_s) from the three lines after a section title."""
    return (int(_NUM.search(lines[start + 1]).group(1)), float(_NUM.search(lines[start + 2]).group(1)),
            float(_NUM.search(lines[start + 3]).group(1)))


def parse_execution_times(file_path):
    """Timings of one ``execution_times.txt`` (performance_analysis.py:9-113).

    OF layout (``Motion Detection:`` then ``Compression:``) fills md_* and
    cp_*; FD layout (``Frame Differencing:``) fills md_* with cp_* = 0. The
    total is the ``Total video processing time:`` line, else md + cp. Any
    failure prints ``Error parsing <path>: <reason>`` and returns None."""
    try:
        with open(file_path, "r") as f:
            lines = [ln.strip() for ln in f if ln.strip() != ""]
        total = [ln for ln in lines if ln.startswith("Total video processing time:")]
        if lines[0].startswith("Motion Detection:"):
            md = _section(lines, 0)
            ci = next((i for i, ln in enumerate(lines) if ln.startswith("Compression:")), None)
            cp = _section(lines, ci) if ci is not None else (0, 0, 0)
        elif lines[0].startswith("Frame Differencing:"):
            md = _section(lines, 0)
            cp = (0, 0.0, 0.0)
        else:
            raise ValueError("Unrecognized format of execution_times.txt")
        tot = float(_NUM.search(total[0]).group(1)) if total else md[1] + cp[1]
    except Exception as e:  # the reference reports and skips (:110-112)
        print(f"Error parsing {file_path}: {e}")
        return None
    return {"md_frames": md[0], "md_time": md[1], "md_avg": md[2], "cp_frames": cp[0], "cp_time": cp[1],
            "cp_avg": cp[2], "total_processing_time": tot}


def _resolve(path):
    """``path`` if it exists, else the ``.npy`` stream video_io wrote in its place."""
    if os.path.isfile(path):
        return path
    alt = os.path.splitext(path)[0] + ".npy"
    return alt if os.path.isfile(alt) else None


def get_video_duration(video_path):
    """frames / fps of a video (0 when unreadable), performance_analysis.py:115-126."""
    p = _resolve(video_path)
    if p is None:
        return 0
    cap = video_io.open_source(p)
    duration = 0
    if cap.isOpened():
        fps = cap.get(video_io.CAP_PROP_FPS)
        n = cap.get(video_io.CAP_PROP_FRAME_COUNT)
        if fps > 0:
            duration = n / fps
        cap.release()
    return duration


def get_file_size(file_path):
    """Bytes of a file, 0 when missing (performance_analysis.py:128-133)."""
    p = _resolve(file_path)
    try:
        return os.path.getsize(p) if p else 0
    except OSError:
        return 0


def get_original_and_compressed_paths(subfolder):
    """OF outputs (overlay.mp4, compressed.mp4) if present, else the FD ones
    (dilated_motion_mask_video.mp4, compressed_final_video.mp4), else (None, None)
    (performance_analysis.py:135-150)."""
    for orig, comp in (("overlay.mp4", "compressed.mp4"),
                       ("dilated_motion_mask_video.mp4", "compressed_final_video.mp4")):
        o, c = os.path.join(subfolder, orig), os.path.join(subfolder, comp)
        if _resolve(o) and _resolve(c):
            return o, c
    return None, None


def collect(output_folder):
    """One row dict per processed video under ``output_folder`` (:166-206)."""
    rows = []
    for item in sorted(os.listdir(output_folder)):   # sorted: deterministic row order
        sub = os.path.join(output_folder, item)
        exec_file = os.path.join(sub, "execution_times.txt")
        if not (os.path.isdir(sub) and os.path.isfile(exec_file)):
            continue
        d = parse_execution_times(exec_file)
        if d is None:
            continue
        d["video"] = item
        orig, comp = get_original_and_compressed_paths(sub)
        if orig is None:
            print(f"Warning: video files not found in {sub}")
            continue
        dur = get_video_duration(orig)
        d["video_duration_seconds"] = dur
        d["conversion_time_per_minute"] = d["total_processing_time"] * 60 / dur if dur > 0 else 0
        o, c = get_file_size(orig), get_file_size(comp)
        d["original_size_bytes"], d["compressed_size_bytes"] = o, c
        d["reduction_percentage"] = (o - c) / o * 100 if o > 0 else 0
        rows.append(d)
    return rows


def write_csv(rows, csv_file):
    keys = ["video", "md_frames", "md_time", "md_avg", "cp_frames", "cp_time", "cp_avg", "total_processing_time",
            "video_duration_seconds", "conversion_time_per_minute", "original_size_bytes", "compressed_size_bytes",
            "reduction_percentage"]
    with open(csv_file, mode="w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDNAMES)
        w.writeheader()
        for d in rows:
            w.writerow({name: d.get(k, "") for name, k in zip(FIELDNAMES, keys)})


def write_charts(rows, folder):
    """The line and bar charts (:251-286); skipped (returns []) without matplotlib."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        logging.info("matplotlib not importable: charts skipped")
        return []
    videos = [d["video"] for d in rows]
    red = [d["reduction_percentage"] for d in rows]
    avg = sum(red) / len(red)
    charts = (   # (file, title, y label, draw)
        ("conversion_times_line_chart.png", "Total Conversion Time and per Minute per Video", "Time (s)",
         lambda: [plt.plot(videos, [d[k] for d in rows], marker="o", label=lab)
                  for k, lab in (("total_processing_time", "Total Conversion Time (s)"),
                                 ("conversion_time_per_minute", "Conversion Time per Minute (s/min)"))]),
        ("reduction_percentage_bar_chart.png", "Compression Percentage per Video", "Reduction (%)",
         lambda: (plt.bar(videos, red, color="cornflowerblue", label="Reduction (%)"),
                  plt.axhline(y=avg, color="red", linestyle="--", label=f"Average Reduction ({avg:.2f}%)"))),
    )
    out = []
    for name, title, ylab, draw in charts:
        plt.figure(figsize=(10, 6))
        draw()
        plt.xlabel("Video")
        plt.ylabel(ylab)
        plt.title(title)
        plt.xticks(rotation=45, ha="right")
        plt.legend()
        plt.tight_layout()
        out.append(os.path.join(folder, name))
        plt.savefig(out[-1])
        plt.close()
    return out


def main(argv=None):
    """``python -m <package>.performance_analysis <output_folder>`` (:152-288)."""
    argv = sys.argv if argv is None else argv
    if len(argv) < 2:
        print("Usage: python performance_analysis.py <output_folder>")
        sys.exit(1)
    output_folder = argv[1]
    if not os.path.isdir(output_folder):
        print(f"Invalid output folder: {output_folder}")
        sys.exit(1)
    perf = os.path.join(output_folder, "performance")
    os.makedirs(perf, exist_ok=True)
    rows = collect(output_folder)
    if not rows:
        print("No performance data found.")
        sys.exit(1)
    csv_file = os.path.join(perf, "performance_data.csv")
    write_csv(rows, csv_file)
    print(f"CSV saved in: {csv_file}")
    for p in write_charts(rows, perf):
        print(f"Chart saved in: {p}")
    print("Performance analysis completed successfully.")


if __name__ == "__main__":
    main()
