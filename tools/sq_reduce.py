"""Reduce a rocprofv3 --pmc counter_collection.csv to per-dispatch-mean
counter values of the kernels whose name contains a pattern (dev tool)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, pat = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in rows:
        k = r.get("Kernel_Name", "")
        if pat not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = {}
    for k, c in acc.items():
        n = max(1, len(disp[k]))
        out[k[:90]] = {"dispatches": n, **{name: v / n for name, v in c.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
