#!/bin/bash
# GPU box: isolated FD stages (tools/stage_bench.hip) under a kernel trace and
# the FETCH_SIZE / WRITE_SIZE passes, plus the FETCH_SIZE width calibration
# (tools/calib_fetch.hip). Output under gpurun_out/stage_prof/.
#   tools/stage_prof.sh [W H n]
set -e
cd "$(dirname "$0")/.."
W=${1:-1920}; H=${2:-1080}; N=${3:-63}
OUT=gpurun_out/stage_prof
mkdir -p $OUT
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o $OUT/stage_bench \
    tools/stage_bench.hip dynamic-video-compression-surveillance_amd/csrc/fd_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $OUT/calib tools/calib_fetch.hip
python3 tools/make_frames.py $W $H $((N + 1)) /tmp/frames.raw
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o s --output-format csv -- \
    $OUT/stage_bench $W $H $N 4 /tmp/frames.raw > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- \
    $OUT/stage_bench $W $H $N 3 /tmp/frames.raw > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- \
    $OUT/stage_bench $W $H $N 3 /tmp/frames.raw > $OUT/write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib_prof -o c --output-format csv -- \
    $OUT/calib 1536 > $OUT/calib.log 2>&1
echo done
