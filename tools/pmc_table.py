"""Per-kernel table of rocprofv3 --pmc counter CSVs (mean per dispatch).

    python tools/pmc_table.py <counter_collection.csv> [more.csv ...]
"""
import collections
import csv
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("dvc::", "")
            names[r["Dispatch_Id"]] = k
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d, cs in per.items():
            for c, v in cs.items():
                acc[names[d]][c].append(v)
    cols = sorted({c for k in acc.values() for c in k})
    print("kernel".ljust(28) + "".join(c.replace("SQ_", "")[:14].rjust(15) for c in cols))
    for k in sorted(acc):
        print(k[:28].ljust(28) + "".join((f"{sum(acc[k][c]) / len(acc[k][c]):15.4g}" if acc[k][c] else " " * 15)
                                          for c in cols))


if __name__ == "__main__":
    main()
