#!/usr/bin/env python3
"""Per-step kernel statistics of the steady-state steps of a rocprofv3 --kernel-trace run
(bench.py --profile-only): the steps are delimited by the iteration-counter launches
(k_counter_add, one per network per step), and only the last STEPS complete steps count, so
warm-up, planning and one-time launches (weight bounds of the frozen VGG19, graph capture)
stay out of the per-step numbers that run_kernel_stats.csv spreads over the whole run.

    python scripts/steady_stats.py gpurun_out/<tag>_prof_seq/run_kernel_trace.csv [STEPS] > out.csv"""
import collections
import csv
import sys


def main(path, steps=5):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ca = [i for i, r in enumerate(rows) if "k_counter_add" in r["Kernel_Name"]]
    per = 2   # (G and D counters)
    starts = ca[::per]
    if len(starts) < steps + 1:
        raise SystemExit(f"{len(starts)} step marks, need {steps + 1}")
    t0 = int(rows[starts[-steps - 1]]["Start_Timestamp"])
    t1 = int(rows[starts[-1]]["Start_Timestamp"])
    acc = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        s = int(r["Start_Timestamp"])
        if t0 <= s < t1:
            a = acc[r["Kernel_Name"]]
            a[0] += 1
            a[1] += (int(r["End_Timestamp"]) - s) / 1e3
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "CallsPerStep", "UsPerStep", "AverageUs"])
    for n, (c, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        w.writerow([n, round(c / steps, 2), round(t / steps, 2), round(t / c, 2)])
    tot = sum(t for _, t in acc.values()) / steps
    launches = sum(c for c, _ in acc.values()) / steps
    print(f"# {steps} steady steps: {tot / 1e3:.3f} ms of kernels per step in {launches:.1f} launches, "
          f"step span {(t1 - t0) / steps / 1e6:.3f} ms", file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
