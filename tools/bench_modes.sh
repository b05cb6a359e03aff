#!/bin/bash
# Extra bench lines beside the device-resident headline (run on the GPU box):
# host-pointer I/O (PCIe-inclusive), per-frame launches, several feeds per GPU,
# the multi-core CPU baseline. Each step has its own time limit.
set -o pipefail
out=${1:-gpurun_out/modes}
mkdir -p "$out"
run() { name=$1; shift; timeout -k 10 240 python bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "FAILED $name"; return 1; }; echo "$name: $(python -c "import json;d=json.load(open('$out/$name.json'));print(d['value'], d['config'].get('fps_per_gpu'), d.get('cpu_baseline',{}).get('value'))")"; }
run fd_device --steps 20 --warmup 3 --no-cpu-baseline &&
run fd_host_pinned --io host-pinned --steps 6 --warmup 1 --no-cpu-baseline &&
run fd_host_pageable --io host-pageable --steps 4 --warmup 1 --no-cpu-baseline &&
run fd_per_frame --per-frame --steps 3 --warmup 1 --no-cpu-baseline &&
run fd_2feeds --feeds 2 --steps 10 --warmup 2 --no-cpu-baseline &&
run fd_4feeds --feeds 4 --steps 6 --warmup 2 --no-cpu-baseline &&
run fd_cpu16 --steps 5 --warmup 1 --cpu-cores 16 --cpu-budget 12
