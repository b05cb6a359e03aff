#!/bin/bash
# GPU box: OF stage ablation (DVC_OF_SKIP bit mask: 2 flow, 4 vote + mask
# morphology / rectangles, 8 k_of_out), interleaved over rounds, default OF
# bench config.   tools/ablate_of.sh [rounds]
set -e
cd "$(dirname "$0")/.."
# The skip masks exist only in the ablation build (the shipping library has
# no result-changing knobs): build it first, on the CPU side, with
#   tools/build_variant.sh build/libdvc_ablation.so -DDVC_ABLATION
ABL=${ABL:-build/libdvc_ablation.so}
[ -f "$ABL" ] || { echo "missing $ABL (tools/build_variant.sh $ABL -DDVC_ABLATION)"; exit 1; }
export DVC_LIB_PATH=$ABL
R=${1:-2}
OUT=gpurun_out/ablate_of
mkdir -p $OUT
for r in $(seq 1 $R); do
  for m in 0 2 4 8 12 14; do
    DVC_OF_SKIP=$m timeout -k 10 150 python3 bench.py --path of --no-cpu-baseline --steps 10 --warmup 2 > $OUT/skip$m.json 2> $OUT/skip$m.err
    python3 -c "import json; d=json.load(open('$OUT/skip$m.json')); print('round $r skip $m', round(d['ms_per_step'],3), 'ms/step', round(d['value']), d['unit'])"
  done
done
