#!/bin/bash
# GPU box, one iteration: parity tests (TESTS), an interleaved A/B (VARIANTS,
# default fused vs unfused) and the kernel-trace timeline of the default build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_fused.py tests/test_bench_config.py}
if [ "$TESTS" != "none" ]; then
timeout -k 10 600 python3 -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4_tests.log; exit 1; }
tail -2 gpurun_out/r4_tests.log
fi
A="--steps 20 --warmup 3 --runs 1 --ktime-seconds 1"
eval "tools/ab_env.sh ${ROUNDS:-2} ${VARIANTS:-\"DVC_FD_FUSED=1\" \"DVC_FD_FUSED=0\"} -- $A" > gpurun_out/r4_ab.txt 2>&1
cat gpurun_out/r4_ab.txt
rm -rf gpurun_out/tr/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr -o t --output-format csv -- \
    python3 bench.py --no-cpu-baseline --runs 1 --steps 5 --warmup 2 --ktime-seconds 0.2 > gpurun_out/tr/bench.log 2>&1
f=$(find gpurun_out/tr -name "t_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f ${ANCHOR:-k_front} 3000 3 > gpurun_out/r4_timeline.txt
cat gpurun_out/r4_timeline.txt
