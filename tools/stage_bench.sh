#!/bin/bash
# Build and run tools/stage_bench.hip under rocprofv3 (GPU box). Output under gpurun_out/stage/.
#   tools/stage_bench.sh [W H n reps fused]
set -e
cd "$(dirname "$0")/.."
W=${1:-1920}; H=${2:-1080}; N=${3:-63}; REPS=${4:-6}; FUSED=${5:-1}
mkdir -p gpurun_out/stage
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o gpurun_out/stage/stage_bench \
    tools/stage_bench.hip dynamic-video-compression-surveillance_amd/csrc/fd_kernels.hip
python3 tools/make_frames.py $W $H $((N + 1)) /tmp/frames.raw
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stage/prof$FUSED -o s --output-format csv -- \
    gpurun_out/stage/stage_bench $W $H $N $REPS /tmp/frames.raw $FUSED
cut -d, -f1-4 $(find gpurun_out/stage/prof$FUSED -name "s_kernel_stats.csv" | head -1)
