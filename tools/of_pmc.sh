#!/bin/bash
# GPU box: SQ instruction/wait counters of the OF kernels (bench --path of),
# one counter group per rocprofv3 run -> gpurun_out/of_pmc/p{1,2}/
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/of_pmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/p1 -o p --output-format csv -- \
    python3 bench.py --path of --no-cpu-baseline --steps 1 --warmup 1 --ktime-seconds 0.1 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
    -d $OUT/p2 -o p --output-format csv -- \
    python3 bench.py --path of --no-cpu-baseline --steps 1 --warmup 1 --ktime-seconds 0.1 > $OUT/p2.log 2>&1
