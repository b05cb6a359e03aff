#!/usr/bin/env python3
"""Steady-state view of a rocprofv3 kernel trace (CSV) of a pipelined run:
finds the longest burst of `anchor` kernel launches whose consecutive ends are
< `gap_us` apart, prints the period (mean anchor end-to-end spacing) and, for
the middle launches of the burst, every kernel in order with its stream.
    tools/timeline.py <t_kernel_trace.csv> [anchor=k_out] [gap_us=2000] [show=3]"""
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_out"
gap = float(sys.argv[3]) if len(sys.argv) > 3 else 2000.0
show = int(sys.argv[4]) if len(sys.argv) > 4 else 3
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("dvc::", "").replace("void ", ""), r["Stream_Id"]) for r in rows)
an = [k for k in ks if anchor in k[2]]
best, cur = (0, 0), 0
for i in range(1, len(an) + 1):
    if i == len(an) or (an[i][1] - an[i - 1][1]) / 1e3 > gap:
        if i - cur > best[1] - best[0]:
            best = (cur, i)
        cur = i
a, b = best
if b - a < 2:
    sys.exit("no burst")
period = (an[b - 1][1] - an[a][1]) / 1e3 / (b - 1 - a)
print(f"burst of {b - a} {anchor} launches, period {period:.1f} us")
m = a + (b - a) // 2 - show // 2
lo, hi = an[m][0], an[min(m + show, b - 1)][1]
win = [k for k in ks if lo <= k[0] <= hi]
for s, e, n, st in win:
    print(f"  {st:>3} {n:16s} {(s - lo) / 1e3:8.1f} {(e - lo) / 1e3:8.1f} {(e - s) / 1e3:7.1f}")
