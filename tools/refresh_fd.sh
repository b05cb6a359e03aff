#!/bin/bash
# GPU box: the FD bench lines kept under profiles/ (default 1080p, 4K, noisy)
# and the kernel-trace + PMC profile of the default workload.
#   tools/refresh_fd.sh <tag>
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py > gpurun_out/${TAG}_bench_fd_1080p.json 2> gpurun_out/${TAG}_bench_fd_1080p.err
timeout -k 10 300 python3 -u bench.py --width 3840 --height 2160 > gpurun_out/${TAG}_bench_fd_4k.json 2> gpurun_out/${TAG}_bench_fd_4k.err
timeout -k 10 300 python3 -u bench.py --noisy > gpurun_out/${TAG}_bench_fd_noisy.json 2> gpurun_out/${TAG}_bench_fd_noisy.err
bash tools/profile_round.sh ${TAG}fd fd_1080p_single_feed_per_gpu
