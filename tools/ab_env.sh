#!/bin/bash
# Interleaved A/B of bench.py under environment variants (GPU box):
#   tools/ab_env.sh <rounds> "<env A>" "<env B>" ... -- [bench args]
# prints value per variant per round. Tuning knobs (csrc/tune.h) are read only
# by an experiment build: tools/build_variant.sh build/libdvc_exp.so
# -DDVC_EXPERIMENTS on the CPU side, then DVC_LIB_PATH=build/libdvc_exp.so here.
R=$1; shift
vars=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do vars+=("$1"); shift; done
shift
for r in $(seq 1 $R); do
  for v in "${vars[@]}"; do
    val=$(env $v timeout -k 10 120 python bench.py --no-cpu-baseline "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'])") || { echo "FAIL $v"; exit 1; }
    echo "round $r [$v] $val"
  done
done
