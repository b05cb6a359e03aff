#!/bin/bash
# GPU box: NV12-input FD bench with k_front tile heights 16 / 32 / 64 rows
# (DVC_FRONT_NW 4 / 8 / 16: fewer converted halo rows), interleaved, then a
# kernel trace of the default NV12 run.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/yuv_nw
for r in 1 2; do
  for nw in 4 8 16; do
    DVC_FRONT_NW=$nw timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 3 \
        --in-format NV12 > gpurun_out/yuv_nw/nw${nw}_$r.json
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/yuv_nw/trace -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --in-format NV12 > gpurun_out/yuv_nw/trace.log 2>&1
