#!/bin/bash
# Interleaved A/B of bench.py argument variants (GPU box):
#   tools/ab_args.sh <rounds> "<args A>" "<args B>" ...
# prints value and roofline frac per variant per round.
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    val=$(timeout -k 10 120 python bench.py --no-cpu-baseline $v 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'])") || { echo "FAIL $v"; exit 1; }
    echo "round $r [$v] $val"
  done
done
