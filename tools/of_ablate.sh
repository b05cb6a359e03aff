# TEMP: timing ablations of k_flow_scan (results are wrong by design; timing only)
mkdir -p gpurun_out/abl
for a in 0 2 6 7 15 22 23 31; do
  DVC_OF_ABLATE=$a timeout -k 10 120 python -u bench.py --path of --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl/a$a.json 2> gpurun_out/abl/a$a.err || exit 1
done
