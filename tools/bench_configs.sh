#!/bin/bash
# GPU box: the bench lines of every single-GPU BASELINE.json config, plus a
# rocprofv3 kernel-trace summary of each, under gpurun_out/configs/.
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/configs
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-budget 10 > $OUT/fd_1080p.json
timeout -k 10 300 python3 bench.py --width 3840 --height 2160 --steps 5 --warmup 1 --cpu-budget 10 --batch 31 > $OUT/fd_4k.json
timeout -k 10 300 python3 bench.py --path of --steps 3 --warmup 1 --cpu-budget 10 > $OUT/of_1080p.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/of_trace -o t --output-format csv -- \
    python3 bench.py --path of --no-cpu-baseline --steps 2 --warmup 1 > $OUT/of_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fd4k_trace -o t --output-format csv -- \
    python3 bench.py --width 3840 --height 2160 --batch 31 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/fd4k_trace.log 2>&1
