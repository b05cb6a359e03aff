#!/bin/bash
# GPU box: round-4 evidence for the FD headline: the bench line (median of 5
# runs, CPU baseline included), the kernel trace and the two PMC passes of the
# same workload (tools/profile_round.sh), and the OF bench line.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r4}
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench_fd_1080p.json 2> gpurun_out/${TAG}_bench_fd.err
tools/profile_round.sh ${TAG}fd fd_1080p_single_feed_per_gpu
timeout -k 10 300 python3 bench.py --path of --no-cpu-baseline --ktime-seconds 2 > gpurun_out/${TAG}_bench_of_1080p.json 2> gpurun_out/${TAG}_bench_of.err
cat gpurun_out/${TAG}_bench_fd_1080p.json gpurun_out/${TAG}_bench_of_1080p.json
