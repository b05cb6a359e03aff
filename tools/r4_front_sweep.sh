#!/bin/bash
# GPU box: fused-front launch-shape sweep (interleaved, one box): prefetch depth
# and frame chunks, in the pipeline and the front alone (DVC_FD_SKIP=14).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A="--steps 20 --warmup 3 --runs 1 --ktime-seconds 1"
tools/ab_env.sh 1 "DVC_FD_FUSED=0" "DVC_FD_FUSED=1" "DVC_FRONT_PF=2" "DVC_FUSED_CHUNKS=2" "DVC_FUSED_CHUNKS=4" \
   "DVC_FUSED_CHUNKS=8" "DVC_FRONT_PF=2 DVC_FUSED_CHUNKS=3" -- $A > gpurun_out/r4_sweep.txt 2>&1
tools/ab_env.sh 1 "DVC_FD_SKIP=14" "DVC_FD_SKIP=14 DVC_FRONT_PF=2" "DVC_FD_SKIP=14 DVC_FUSED_CHUNKS=4" \
   "DVC_FD_SKIP=14 DVC_FUSED_CHUNKS=8" "DVC_FD_SKIP=14 DVC_FD_FUSED=0" "DVC_FD_SKIP=7 DVC_FD_FUSED=0" -- $A >> gpurun_out/r4_sweep.txt 2>&1
cat gpurun_out/r4_sweep.txt
