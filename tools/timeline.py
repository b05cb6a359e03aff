#!/usr/bin/env python3
"""Steady-state timeline of a rocprofv3 kernel trace (CSV): per-stream busy time
and per-kernel mean duration over the last `tail` fraction of the trace.
    tools/timeline.py <t_kernel_trace.csv> [tail_fraction=0.5]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
             r["Stream_Id"]) for r in rows), key=lambda x: x[0])
t0, t1 = ks[0][0], max(k[1] for k in ks)
lo = t1 - (t1 - t0) * frac
ks = [k for k in ks if k[0] >= lo]
span = max(k[1] for k in ks) - ks[0][0]
busy, dur, cnt = defaultdict(int), defaultdict(int), defaultdict(int)
for s, e, n, st in ks:
    busy[st] += e - s
    dur[n] += e - s
    cnt[n] += 1
print(f"window {span / 1e3:.1f} us, {len(ks)} kernels")
for st, b in sorted(busy.items()):
    print(f"  stream {st}: busy {b / 1e3:9.1f} us ({100 * b / span:5.1f}%)")
for n in sorted(dur, key=lambda n: -dur[n]):
    print(f"  {n:40s} n={cnt[n]:4d} mean {dur[n] / cnt[n] / 1e3:8.1f} us  total {dur[n] / 1e3:9.1f}")
