#!/bin/bash
# GPU box: PMC passes over the isolated stages (tools/stage_bench.hip, fused mode)
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/stage_pmc
mkdir -p $OUT
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o $OUT/sb \
    tools/stage_bench.hip dynamic-video-compression-surveillance_amd/csrc/fd_kernels.hip
python3 tools/make_frames.py 1920 1080 384 /tmp/frames.raw
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $OUT/$1 -o p --output-format csv -- $OUT/sb 1920 1080 383 3 /tmp/frames.raw 1 > $OUT/$1.log 2>&1; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU"
python3 - <<'PY'
import csv, glob, collections
out = collections.defaultdict(dict)
for d in ("fetch", "write", "sq1"):
    f = glob.glob(f"gpurun_out/stage_pmc/{d}/**/p_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dvc::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k in acc:
        for c, v in acc[k].items():
            out[k][c] = v / len(n[k])
for k, cs in out.items():
    print(k[:30], " ".join(f"{c}={v:.3g}" for c, v in sorted(cs.items())))
PY
