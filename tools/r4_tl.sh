#!/bin/bash
# GPU box: kernel-trace timeline of the bench under the given environment
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
rm -rf gpurun_out/tl/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 5 --warmup 2 --ktime-seconds 0.2 "$@" > gpurun_out/tl/bench.log 2>&1
f=$(find gpurun_out/tl -name "t_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f k_front 3000 2
