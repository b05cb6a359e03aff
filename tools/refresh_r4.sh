#!/bin/bash
# GPU box: the HEAD evidence set kept under profiles/ — bench lines (FD 1080p,
# 4K, noisy, NV12 input; OF 1080p, NV12 input), kernel-trace + PMC profiles of
# the FD and OF headline workloads, the OF SQ counters, the drop-in drivers.
#   tools/refresh_r4.sh <tag>      (outputs under gpurun_out/<tag>/)
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r4}
O=gpurun_out/$TAG
mkdir -p $O
b() { local name=$1; shift; timeout -k 10 400 python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err; tail -c 300 $O/bench_$name.json; echo; }
# profiles first: the bench lines' `traffic` reads profiles/pmc_summary*.json
bash tools/profile_round.sh ${TAG}fd fd_1080p_single_feed_per_gpu
bash tools/profile_round.sh ${TAG}of of_1080p_single_feed_per_gpu --path of
cp gpurun_out/prof_${TAG}fd/pmc_summary.json profiles/pmc_summary.json
cp gpurun_out/prof_${TAG}of/pmc_summary.json profiles/pmc_summary_of.json
b fd_1080p
b of_1080p --path of
b fd_4k --width 3840 --height 2160
b fd_noisy --noisy
b fd_nv12_input --in-format NV12
b of_nv12_input --path of --in-format NV12
bash tools/of_pmc.sh
for p in fd of; do
  timeout -k 10 300 python3 tools/bench_dropin.py --path $p --frames 300 --sink y4m --dir /tmp/dvc_dropin_$p >> $O/dropin_driver.jsonl
done
cat $O/dropin_driver.jsonl
