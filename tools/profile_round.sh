#!/bin/bash
# GPU box: kernel-trace stats + the two PMC passes (FETCH_SIZE, WRITE_SIZE; one
# counter group per run, MI355X_MICROARCH.md § HBM) of one bench.py workload,
# summaries under gpurun_out/prof_<tag>/ (copy the ones to keep into profiles/).
#   tools/profile_round.sh <tag> <workload name> [bench.py args...]
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r1}
WL=${2:-fd_1080p_single_feed_per_gpu}
shift 2 || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 5 --warmup 2 --ktime-seconds 0.2 "$@" > $OUT/bench_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 2 --warmup 1 --ktime-seconds 0.1 "$@" > $OUT/bench_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 2 --warmup 1 --ktime-seconds 0.1 "$@" > $OUT/bench_write.log 2>&1
FPL=$(python3 -c "import json; print(json.loads([l for l in open('$OUT/bench_fetch.log') if l.startswith('{\"metric\"')][-1])['roofline']['frames_per_launch'])")
python3 tools/pmc_summary.py $OUT/fetch/f_counter_collection.csv $OUT/write/w_counter_collection.csv \
    $OUT/pmc_summary.json "$WL" "$FPL" > /dev/null
