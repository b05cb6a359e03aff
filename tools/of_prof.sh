# TEMP: scan-kernel phase cycle counters (DVC_OF_SCAN_PROF)
mkdir -p gpurun_out/ofp
DVC_OF_SCAN_PROF=1 timeout -k 10 120 python -u bench.py --path of --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ofp/b.json 2> gpurun_out/ofp/b.err
