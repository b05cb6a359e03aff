#!/bin/bash
# GPU box: kernel trace of the fused pipeline + stage ablations (DVC_FD_SKIP).
cd "$(dirname "$0")/.."
# The skip masks exist only in the ablation build (the shipping library has
# no result-changing knobs): build it first, on the CPU side, with
#   tools/build_variant.sh build/libdvc_ablation.so -DDVC_ABLATION
ABL=${ABL:-build/libdvc_ablation.so}
[ -f "$ABL" ] || { echo "missing $ABL (tools/build_variant.sh $ABL -DDVC_ABLATION)"; exit 1; }
export DVC_LIB_PATH=$ABL
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
A="--steps 20 --warmup 3 --runs 1 --ktime-seconds 1"
export DVC_FUSED_CHUNKS=${CH:-8}
tools/ab_env.sh 1 "DVC_FD_SKIP=0" "DVC_FD_SKIP=2" "DVC_FD_SKIP=4" "DVC_FD_SKIP=8" "DVC_FD_SKIP=6" "DVC_FD_SKIP=12" -- $A > gpurun_out/r4_ablate.txt 2>&1
cat gpurun_out/r4_ablate.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 5 --warmup 2 --ktime-seconds 0.2 > gpurun_out/tr/bench.log 2>&1
f=$(find gpurun_out/tr -name "t_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f k_front 3000 3 > gpurun_out/r4_timeline.txt
cat gpurun_out/r4_timeline.txt
cat $(find gpurun_out/tr -name "t_kernel_stats.csv" | head -1) | cut -c1-160
