# OF: parity tests, then the scan kernel at 512 / 256 threads and the direct-sum kernel (bench.py --path of)
mkdir -p gpurun_out/ofs
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_of_gpu.py tests/test_of_sliding.py > gpurun_out/ofs/tests.log 2>&1 || exit 1
for c in 512 256; do
  DVC_OF_SCAN=$c timeout -k 10 120 python -u bench.py --path of --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ofs/bench_$c.json 2> gpurun_out/ofs/bench_$c.err || exit 1
done
timeout -k 10 120 python -u bench.py --path of --of-direct --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ofs/bench_direct.json 2> gpurun_out/ofs/bench_direct.err
