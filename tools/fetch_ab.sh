#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE per kernel of one bench.py workload under
# environment variants (one counter group per rocprofv3 run, MI355X_MICROARCH.md § HBM).
#   tools/fetch_ab.sh <tag> "<env A>" "<env B>" ... -- [bench args]
# summaries: gpurun_out/fetch_<tag>/<i>/pmc_summary.json (variant i, 0-based)
set -e
cd "$(dirname "$0")/.."
TAG=$1; shift
vars=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do vars+=("$1"); shift; done
shift
export TMPDIR=/tmp
i=0
for v in "${vars[@]}"; do
  OUT=gpurun_out/fetch_$TAG/$i
  mkdir -p $OUT
  echo "$v" > $OUT/env.txt
  env $v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/fetch.log 2>&1
  env $v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/write.log 2>&1
  FPL=$(python3 -c "import json; print(json.loads([l for l in open('$OUT/fetch.log') if l.startswith('{\"metric\"')][-1])['roofline']['frames_per_launch'])")
  python3 tools/pmc_summary.py $OUT/fetch/f_counter_collection.csv $OUT/write/w_counter_collection.csv \
      $OUT/pmc_summary.json "ab" "$FPL" > /dev/null
  i=$((i + 1))
done
