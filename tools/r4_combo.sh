#!/bin/bash
# GPU box: FD 4:2:0 fused-front parity + NV12 A/B, OF parity + A/B (scratch iteration)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_video_io_gpu.py tests/test_fused.py tests/test_of_gpu.py tests/test_golden_of.py tests/test_bench_config.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_combo_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4_combo_tests.log; exit 1; }
tail -2 gpurun_out/r4_combo_tests.log
tools/ab_env.sh 2 "DVC_FD_FUSED=0" "DVC_X=0" -- --in-format NV12 --steps 20 --warmup 3 --runs 1 --ktime-seconds 1 > gpurun_out/r4_nv12_ab.txt 2>&1; cat gpurun_out/r4_nv12_ab.txt
tools/ab_env.sh 2 "DVC_LIB_PATH=build/ab/lib_head.so" "DVC_X=0" "DVC_LIB_PATH=build/ab/lib_pipe2.so" -- --path of --steps 6 --warmup 2 --runs 1 --ktime-seconds 1 > gpurun_out/r4_of_ab.txt 2>&1; cat gpurun_out/r4_of_ab.txt
