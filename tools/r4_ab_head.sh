#!/bin/bash
# GPU box: parity tests (TESTS), then an interleaved A/B of the working tree's
# library against build/ab/lib_head.so (the committed HEAD) on bench ARGS1/ARGS2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_fd_gpu.py tests/test_fused.py tests/test_golden.py tests/test_bench_config.py}
timeout -k 10 700 python3 -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_abh_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4_abh_tests.log; exit 1; }
tail -2 gpurun_out/r4_abh_tests.log
for a in "${ARGS1:---steps 20 --warmup 3 --runs 1 --ktime-seconds 1}" "${ARGS2:---in-format NV12 --steps 20 --warmup 3 --runs 1 --ktime-seconds 1}"; do
  echo "== $a"
  tools/ab_env.sh ${ROUNDS:-3} "DVC_LIB_PATH=build/ab/lib_head.so" "DVC_X=0" -- $a 2>&1
done > gpurun_out/r4_abh.txt
cat gpurun_out/r4_abh.txt
