#!/usr/bin/env python3
"""Kernel-trace utilisation summary: time per kernel class split by grid
size (workgroups), plus the idle gaps between consecutive dispatches.
usage: trace_util.py KERNEL_TRACE_CSV [last_n_steps_fraction]"""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        wg = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-50:], wg))
rows.sort()
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
rows = rows[int(len(rows) * (1 - frac)):]
span = rows[-1][1] - rows[0][0]
busy = sum(e - s for s, e, _, _ in rows)
gaps = sum(max(0, rows[i + 1][0] - rows[i][1]) for i in range(len(rows) - 1))
print(f"dispatches {len(rows)} span {span / 1e6:.2f} ms busy {busy / 1e6:.2f} ms gaps {gaps / 1e6:.2f} ms")
bins = [(0, 64), (64, 256), (256, 512), (512, 1024), (1024, 1 << 30)]
acc = defaultdict(float)
for s, e, k, wg in rows:
    for lo, hi in bins:
        if lo <= wg < hi:
            acc[(lo, hi)] += e - s
for b in bins:
    print(f"  workgroups [{b[0]:5d},{b[1] if b[1] < 1 << 30 else 'inf'}): {acc[b] / 1e6:8.2f} ms")
small = defaultdict(lambda: [0, 0.0])
for s, e, k, wg in rows:
    if wg < 512:
        small[k][0] += 1
        small[k][1] += e - s
print("kernels with < 512 workgroups (time):")
for k, (n, t) in sorted(small.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"  {k:50s} n={n:5d} {t / 1e6:8.3f} ms")
