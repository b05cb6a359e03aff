#!/bin/bash
# GPU box: FD stage ablation (DVC_FD_SKIP bit mask: 1 front, 2 contour filter,
# 4 dilate + accumulate, 8 output), interleaved over rounds, default 1080p bench
# config; plus the FETCH_SIZE access-width calibration (tools/calib_fetch.hip).
#   tools/ablate_stages.sh [rounds] [extra bench args]
set -e
cd "$(dirname "$0")/.."
# The skip masks exist only in the ablation build (the shipping library has
# no result-changing knobs): build it first, on the CPU side, with
#   tools/build_variant.sh build/libdvc_ablation.so -DDVC_ABLATION
ABL=${ABL:-build/libdvc_ablation.so}
[ -f "$ABL" ] || { echo "missing $ABL (tools/build_variant.sh $ABL -DDVC_ABLATION)"; exit 1; }
export DVC_LIB_PATH=$ABL
R=${1:-2}; shift || true
OUT=gpurun_out/ablate
mkdir -p $OUT
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $OUT/calib tools/calib_fetch.hip
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib_prof -o c --output-format csv -- \
    $OUT/calib 1536 > $OUT/calib.log 2>&1
for r in $(seq 1 $R); do
  for m in 0 2 4 6 1 8 14 13; do
    DVC_FD_SKIP=$m timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 "$@" > $OUT/skip$m.json 2> $OUT/skip$m.err
    python3 -c "import json; d=json.load(open('$OUT/skip$m.json')); print('round $r skip $m', round(d['ms_per_step'],3), 'ms/step', round(d['value']), d['unit'])"
  done
done
