#!/bin/bash
# GPU box: k_front launch-shape sweep, alone (DVC_FD_SKIP=14) and in the full
# pipeline, interleaved over rounds (default 1080p bench config).
#   tools/front_sweep.sh [rounds] "<env variant>" ...
set -e
cd "$(dirname "$0")/.."
# The skip masks exist only in the ablation build (the shipping library has
# no result-changing knobs): build it first, on the CPU side, with
#   tools/build_variant.sh build/libdvc_ablation.so -DDVC_ABLATION
ABL=${ABL:-build/libdvc_ablation.so}
[ -f "$ABL" ] || { echo "missing $ABL (tools/build_variant.sh $ABL -DDVC_ABLATION)"; exit 1; }
export DVC_LIB_PATH=$ABL
R=${1:-2}; shift || true
OUT=gpurun_out/front_sweep
mkdir -p $OUT
vars=("$@")
[ ${#vars[@]} -eq 0 ] && vars=("X=0")
for r in $(seq 1 $R); do
  for skip in 14 0; do
    for v in "${vars[@]}"; do
      env $v DVC_FD_SKIP=$skip timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $OUT/run.json 2> $OUT/run.err
      python3 -c "import json; d=json.load(open('$OUT/run.json')); print('round $r skip $skip [$v]', round(d['ms_per_step'],3), 'ms/step', round(d['value']))"
    done
  done
done
