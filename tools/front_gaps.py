#!/usr/bin/env python3
"""Gaps between consecutive fused fronts in a rocprofv3 kernel trace (CSV) of
the graph path: fronts launched from slot graphs run on the four slot streams
in turn (the KTIMING pass runs them all on one stream and is left out).
Prints the median / p10 / p90 gap (one front's end to the next one's start),
the median front duration and the median front-to-front period, in us.
    tools/front_gaps.py <t_kernel_trace.csv> [label]"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
label = sys.argv[2] if len(sys.argv) > 2 else ""
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"])
            for r in rows if "k_front<" in r["Kernel_Name"])
# the graph-path fronts: a run of fronts whose streams rotate (not all one stream)
best, cur = [], []
for k in ks:
    if cur and k[2] == cur[-1][2]:
        best, cur = max(best, cur, key=len), []
    cur.append(k)
best = max(best, cur, key=len)[4:]   # past the first slot round
if len(best) < 3:
    sys.exit("no rotating run of fronts")
# (gaps over 1 ms are the bench's step / run boundaries, not the pipeline's)
idx = [i for i in range(1, len(best)) if best[i][0] - best[i - 1][1] < 1_000_000]
gaps = sorted((best[i][0] - best[i - 1][1]) / 1e3 for i in idx)
per = [(best[i][1] - best[i - 1][1]) / 1e3 for i in idx]
dur = [(k[1] - k[0]) / 1e3 for k in best]
q = lambda p: gaps[min(len(gaps) - 1, int(p * len(gaps)))]
print(f"{label} fronts {len(best)}: gap median {st.median(gaps):.1f} p10 {q(0.1):.1f} p90 {q(0.9):.1f}, "
      f"front median {st.median(dur):.1f}, period median {st.median(per):.1f} (us)")
