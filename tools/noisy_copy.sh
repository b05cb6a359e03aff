#!/bin/bash
# GPU box: the noisy (CCL-stress) FD line and the default lines with the
# measured copy rate beside the roofline.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/nc
timeout -k 10 300 python3 -u bench.py > gpurun_out/nc/fd.json
timeout -k 10 300 python3 -u bench.py --noisy > gpurun_out/nc/fd_noisy.json
timeout -k 10 300 python3 -u bench.py --width 3840 --height 2160 > gpurun_out/nc/fd_4k.json
timeout -k 10 300 python3 -u bench.py --path of > gpurun_out/nc/of.json
