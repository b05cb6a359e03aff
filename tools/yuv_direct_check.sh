#!/bin/bash
# GPU box: YUV-input parity tests, then in-place vs staged 4:2:0 input (A/B).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_video_io_gpu.py \
    > gpurun_out/yuv_tests.log 2>&1
for r in 1 2; do
  for m in 1 0; do
    DVC_FD_YUV_DIRECT=$m timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 3 \
        --in-format NV12 > gpurun_out/yuv_ab_${m}_$r.json
  done
done
