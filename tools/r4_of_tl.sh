#!/bin/bash
# GPU box: kernel-trace timeline of the OF bench (steady state around k_of_out).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/oftr && rm -rf gpurun_out/oftr/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/oftr -o t --output-format csv -- \
    python3 bench.py --path of --no-cpu-baseline --runs 1 --steps ${STEPS:-4} --warmup 2 --ktime-seconds 0.2 > gpurun_out/oftr/bench.log 2>&1
f=$(find gpurun_out/oftr -name "t_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f ${ANCHOR:-k_of_out} ${GAP:-20000} ${SHOW:-2} > gpurun_out/r4_of_timeline.txt
cat gpurun_out/r4_of_timeline.txt
tail -c 1500 gpurun_out/oftr/bench.log | grep -o '"value": [0-9.]*' | head -1
