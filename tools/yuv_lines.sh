#!/bin/bash
# GPU box: the YUV bench lines kept under profiles/ (in-place surfaces).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/yuv_lines
timeout -k 10 300 python3 -u bench.py --in-format NV12 > gpurun_out/yuv_lines/nv12.json
timeout -k 10 300 python3 -u bench.py --in-format I420 > gpurun_out/yuv_lines/i420.json
timeout -k 10 300 python3 -u bench.py --in-format NV12 --out-format I420 > gpurun_out/yuv_lines/nv12_i420.json
timeout -k 10 300 python3 -u bench.py --io host-pinned --in-format NV12 --out-format I420 --steps 20 --warmup 2 \
    > gpurun_out/yuv_lines/pinned_nv12_i420.json
timeout -k 10 300 python3 -u bench.py --io host-pinned --steps 20 --warmup 2 > gpurun_out/yuv_lines/pinned_bgr.json
