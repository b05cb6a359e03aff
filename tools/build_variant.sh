#!/bin/bash
# Build libdvc_hip.so with extra compiler flags into another path (A/B and
# debug builds, e.g. -DDVC_SCAN_STAMPS):  tools/build_variant.sh <out.so> [flags...]
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
C=dynamic-video-compression-surveillance_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off "$@" -o "$OUT" \
    $C/fd_kernels.hip $C/fd_api.hip $C/of_kernels.hip $C/of_api.hip $C/yuv_kernels.hip $C/diag.hip
