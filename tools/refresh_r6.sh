#!/bin/bash
# GPU box: the round-6 HEAD evidence set kept under profiles/ (the closing
# refresh, after the round's last code change), in two parts (each within one
# gpurun call):
#   tools/refresh_r6.sh a   kernel traces + PMC of the FD and OF headline
#                           workloads (the bench lines' `traffic` reads
#                           profiles/pmc_summary*.json), SQ counters, the FD
#                           and OF headline lines, 4K, noisy, NV12 and I420 input
#   tools/refresh_r6.sh b   the operating points (per-frame calls and 8- /
#                           32-frame launches through the graph path, 128, one
#                           output set), the __main__ variant, I420 outputs,
#                           OF NV12, the per-call sweep, the drop-in drivers
#                           and the N > 1 launch rehearsal
# Outputs under gpurun_out/r6/.
set -e
cd "$(dirname "$0")/.."
PART=${1:-a}
O=gpurun_out/r6
mkdir -p $O
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 400 python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err; python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
if [ "$PART" = a ]; then
  bash tools/profile_round.sh r6fd fd_1080p_single_feed_per_gpu
  bash tools/profile_round.sh r6of of_1080p_single_feed_per_gpu --path of
  cp gpurun_out/prof_r6fd/pmc_summary.json profiles/pmc_summary.json
  cp gpurun_out/prof_r6of/pmc_summary.json profiles/pmc_summary_of.json
  cp gpurun_out/prof_r6fd/pmc_summary.json $O/pmc_summary.json
  cp gpurun_out/prof_r6of/pmc_summary.json $O/pmc_summary_of.json
  cp $(find gpurun_out/prof_r6fd/trace -name "t_kernel_stats.csv" | head -1) $O/fd_kernel_stats.csv
  cp $(find gpurun_out/prof_r6of/trace -name "t_kernel_stats.csv" | head -1) $O/of_kernel_stats.csv
  python3 tools/timeline.py $(find gpurun_out/prof_r6of/trace -name "t_kernel_trace.csv" | head -1) k_of_out 20000 1 \
      > $O/of_timeline.txt 2>&1 || true
  bash tools/fd_sq_pmc.sh > $O/fd_sq.log 2>&1 && cp gpurun_out/fd_pmc/table.txt $O/fd_sq_counters.txt
  bash tools/of_pmc.sh > $O/of_pmc.log 2>&1
  python3 tools/pmc_table.py $(find gpurun_out/of_pmc/p1 -name "p_counter_collection.csv" | head -1) \
      $(find gpurun_out/of_pmc/p2 -name "p_counter_collection.csv" | head -1) > $O/of_sq_counters.txt 2>&1 || true
  b fd_1080p
  b of_1080p --path of
  b fd_4k --width 3840 --height 2160
  b fd_noisy --noisy
  b fd_nv12_input --in-format NV12
  b fd_i420_input --in-format I420
else
  b fd_1080p_box_b
  b fd_per_frame --per-frame --runs 3 --steps 10 --warmup 2
  b fd_batch8 --batch 8 --runs 3
  b fd_batch32 --batch 32 --runs 3
  b fd_batch128 --batch 128 --runs 3
  b fd_out_ring1 --out-ring 1 --runs 3
  b fd_b8_k10_r0.3 --block-size 8 --kernel-size 10 --release-factor 0.3 --runs 3
  b fd_i420_output --out-format I420 --runs 3
  b fd_nv12_input_i420_output --in-format NV12 --out-format I420 --runs 3
  b of_nv12_input --path of --in-format NV12
  timeout -k 10 300 python3 -u tools/per_call.py > $O/per_call.jsonl
  for p in fd of; do
    timeout -k 10 300 python3 tools/bench_dropin.py --path $p --frames 300 --sink y4m --dir /tmp/dvc_dropin_$p >> $O/dropin_driver.jsonl
  done
  bash tools/rehearse_ranks.sh && cp gpurun_out/ranks/n2.json $O/ranks_n2.json && cp gpurun_out/ranks/n4.json $O/ranks_n4.json
fi
echo done
