#!/bin/bash
# GPU box: the round's closing evidence at HEAD — the -m gpu suite and smoke(),
# then tools/refresh_r4.sh (bench lines, kernel traces, PMC, SQ counters,
# drop-in drivers) under gpurun_out/<tag>/.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r4}
mkdir -p gpurun_out
bash tools/gpu_suite.sh || { tail -30 gpurun_out/gpu_suite.log; tail gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log; tail -1 gpurun_out/smoke.log
bash tools/refresh_r4.sh $TAG
