#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (mean over
dispatches) and print one row per kernel with every counter seen."""
import csv
import sys
from collections import defaultdict


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        disp = defaultdict(lambda: defaultdict(float))
        names = {}
        with open(p) as f:
            for r in csv.DictReader(f):
                key = (r["Dispatch_Id"])
                names[key] = r["Kernel_Name"]
                disp[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for key, cs in disp.items():
            for c, v in cs.items():
                acc[names[key]][c].append(v)
    for k, cs in acc.items():
        short = k.split("(")[0][-90:]
        print(short)
        for c, vs in sorted(cs.items()):
            print(f"    {c:32s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")


if __name__ == "__main__":
    main(sys.argv[1:])
