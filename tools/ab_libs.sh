#!/bin/bash
# Interleaved A/B of bench.py over library builds (GPU box):
#   tools/ab_libs.sh <rounds> <lib A> <lib B> ... -- [bench args]
# prints value per library per round (DVC_LIB_PATH selects the build).
R=$1; shift
libs=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do libs+=("$1"); shift; done
shift
for r in $(seq 1 $R); do
  for l in "${libs[@]}"; do
    val=$(DVC_LIB_PATH=$l timeout -k 10 150 python bench.py --no-cpu-baseline --runs 1 "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'])") || { echo "FAIL $l"; exit 1; }
    echo "round $r [$l] $val"
  done
done
