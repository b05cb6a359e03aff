"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/pmc_summary.json.

    python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json> [workload [frames_per_launch]]

``workload`` (bench.py's config.workload of the profiled command) and
``frames_per_launch`` (its roofline.frames_per_launch) are recorded so bench.py
only quotes the traffic for the workload and launch size it was measured on.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md § HBM: on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads;
WRITE_SIZE is exact for streaming stores). Both counters are in KiB.
Infinity-Cache hits are counted too, so these are L2-miss bytes, an upper
bound on HBM traffic.
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    """{kernel: sorted per-launch values} over the launches of each kernel's
    LARGEST grid (a kernel launched per pyramid level, like k_flow, is quoted
    for its finest level — the launch bench.py times)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    grid = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"]
        key = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("dvc::", "").split("<")[0]
        g = int(r.get("Grid_Size", 0) or 0)
        grid[key] = max(grid.get(key, 0), g)
        acc[(key, g)][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: sorted(acc[(k, g)].values()) for k, g in grid.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB*1024, mean over the launches of each kernel's largest grid; "
                   "gfx950 FETCH_SIZE halves wide streaming reads (MI355X_MICROARCH.md), other access widths "
                   "uncalibrated; Infinity-Cache hits included",
           "workload": sys.argv[4] if len(sys.argv) > 4 else None,
           "frames_per_launch": float(sys.argv[5]) if len(sys.argv) > 5 else None,
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fm = sum(f) / len(f) * 1024 if f else None   # mean: k_flow alternates two iteration kinds
        wm = sum(w) / len(w) * 1024 if w else None
        out["kernels"][k] = {
            "launches": max(len(f), len(w)),
            "fetch_bytes_raw": fm,
            "write_bytes": wm,
            "hbm_bytes_per_launch": (2 * fm + wm) if (fm is not None and wm is not None) else None,
        }
    with open(sys.argv[3], "w") as fp:
        json.dump(out, fp, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
