#!/bin/bash
# GPU box: OF kernel times with the flow stream skipped (DVC_OF_SKIP=2: the
# pyramid and mask stages alone) and with the mask stages skipped (=12: the
# pyramid and the flow), kernel-trace stats under gpurun_out/of_isolate/.
set -e
cd "$(dirname "$0")/.."
# The skip masks exist only in the ablation build (the shipping library has
# no result-changing knobs): build it first, on the CPU side, with
#   tools/build_variant.sh build/libdvc_ablation.so -DDVC_ABLATION
ABL=${ABL:-build/libdvc_ablation.so}
[ -f "$ABL" ] || { echo "missing $ABL (tools/build_variant.sh $ABL -DDVC_ABLATION)"; exit 1; }
export DVC_LIB_PATH=$ABL
OUT=gpurun_out/of_isolate
mkdir -p $OUT
export TMPDIR=/tmp
for m in 2 12; do
  DVC_OF_SKIP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/skip$m -o t --output-format csv -- \
      python3 bench.py --path of --no-cpu-baseline --runs 1 --steps 6 --warmup 2 > $OUT/skip$m.log 2>&1
done
