#!/bin/bash
# GPU box: SQ instruction/wait counters of the FD pipeline kernels (the
# headline bench workload), one counter group per rocprofv3 run ->
# gpurun_out/fd_pmc/p1/ and the per-kernel table gpurun_out/fd_pmc/table.txt
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/fd_pmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $OUT/p1 -o p --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --runs 1 --ktime-seconds 0.1 > $OUT/p1.log 2>&1
python3 tools/pmc_table.py $(find $OUT/p1 -name "p_counter_collection.csv" | head -1) > $OUT/table.txt
cat $OUT/table.txt
