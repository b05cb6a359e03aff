#!/bin/bash
# GPU box: does a smaller FD batch let k_out's re-read of the frames k_front
# read hit the Infinity Cache? Per batch size: bench value (device frames,
# 1080p) and one FETCH_SIZE pass -> k_out / k_front fetched MB per frame
# (VERDICT r1 "next" 5c). Results in gpurun_out/ic_sweep/.
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/ic_sweep
mkdir -p $OUT
export TMPDIR=/tmp
for b in 8 16 32 64 383; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 3 --batch $b > $OUT/bench_b$b.json
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_b$b -o f --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch $b > $OUT/fetch_b$b.log 2>&1
done
python3 - <<'PY' > $OUT/summary.txt
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import per_kernel
for b in (8, 16, 32, 64, 383):
    v = json.loads(open(f"gpurun_out/ic_sweep/bench_b{b}.json").read().strip().splitlines()[-1])["value"]
    f = per_kernel(f"gpurun_out/ic_sweep/f_b{b}/f_counter_collection.csv", "FETCH_SIZE")
    mb = {k: 2 * 1024 * sum(x) / len(x) / b / 1e6 for k, x in f.items() if k in ("k_out", "k_front")}
    print(f"batch {b:4d}: {v:10.1f} Mpx/s  fetch MB/frame (x2 corrected) " +
          " ".join(f"{k} {m:.2f}" for k, m in sorted(mb.items())))
PY
cat $OUT/summary.txt
