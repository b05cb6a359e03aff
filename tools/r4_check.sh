#!/bin/bash
# GPU box: parity tests (args: test files; default the round-4 set), then an
# interleaved A/B of the fused front against the one-pass k_out
# (DVC_FD_FUSED=0), 1080p bench config, and one bench line.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TESTS=${@:-tests/test_fused.py tests/test_rccl.py tests/test_wide.py tests/test_golden.py tests/test_golden_of.py tests/test_bench_config.py tests/test_fd_gpu.py tests/test_of_gpu.py}
timeout -k 10 700 python3 -u -m pytest $TESTS -x -v -m gpu \
    --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 || { tail -30 gpurun_out/r4_tests.log; exit 1; }
tail -3 gpurun_out/r4_tests.log
tools/ab_env.sh 2 "DVC_FD_FUSED=1" "DVC_FD_FUSED=0" -- --steps 20 --warmup 3 --runs 1 --ktime-seconds 1 > gpurun_out/r4_ab.txt 2>&1
cat gpurun_out/r4_ab.txt
timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --runs 3 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
cat gpurun_out/r4_bench.json
