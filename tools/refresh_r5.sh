#!/bin/bash
# GPU box: the round-5 HEAD evidence set kept under profiles/ (one refresh a
# round): bench lines — FD 1080p (configs[1], headline), 4K, noisy, NV12 input,
# the operating points the product uses (32-frame launches = the drop-in's
# DVC_READ_AHEAD, per-frame calls, one output set), the reference's __main__
# variant (b=8, k=10, r=0.3) and I420 outputs; OF 1080p (configs[4]) and NV12 —
# kernel traces + PMC of the FD and OF headline workloads, SQ counters of both,
# the drop-in drivers and the N > 1 launch rehearsal.
#   tools/refresh_r5.sh [tag]      (outputs under gpurun_out/<tag>/)
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r5}
O=gpurun_out/$TAG
mkdir -p $O
b() { local name=$1; shift; timeout -k 10 400 python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err; python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
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
b fd_batch32 --batch 32 --runs 3
b fd_batch128 --batch 128 --runs 3
b fd_per_frame --per-frame --runs 3 --steps 5 --warmup 1
b fd_out_ring1 --out-ring 1 --runs 3
b fd_b8_k10_r0.3 --block-size 8 --kernel-size 10 --release-factor 0.3 --runs 3
b fd_i420_output --out-format I420 --runs 3
b fd_nv12_input_i420_output --in-format NV12 --out-format I420 --runs 3
bash tools/of_pmc.sh > $O/of_pmc.log 2>&1
python3 tools/pmc_table.py $(find gpurun_out/of_pmc/p1 -name "p_counter_collection.csv" | head -1) \
    $(find gpurun_out/of_pmc/p2 -name "p_counter_collection.csv" | head -1) > $O/of_sq_counters.txt 2>&1 || true
bash tools/fd_sq_pmc.sh > $O/fd_sq.log 2>&1 && cp gpurun_out/fd_pmc/table.txt $O/fd_sq_counters.txt
for p in fd of; do
  timeout -k 10 300 python3 tools/bench_dropin.py --path $p --frames 300 --sink y4m --dir /tmp/dvc_dropin_$p >> $O/dropin_driver.jsonl
done
bash tools/rehearse_ranks.sh && cp gpurun_out/ranks/n2.json $O/ranks_n2.json && cp gpurun_out/ranks/n4.json $O/ranks_n4.json
echo done
