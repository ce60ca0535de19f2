"""Compare split-K reduce durations per argument set across scripts/gpu_r6_reduce.sh runs:
python scripts/diag/reduce_cmp.py gpurun_out/r6_reduce_before gpurun_out/r6_reduce ..."""
import collections
import csv
import sys


def agg(d):
    rows = [r for r in csv.DictReader(open(d + '/kt/kt_kernel_trace.csv')) if 'splitk_reduce' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    t = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
    args = [l for l in open(d + '/args.txt') if l.startswith('[reduce]')]
    a = collections.defaultdict(list)
    for x, y in zip(args, t):
        a[x.split(' tpo')[0].replace('[reduce] ', '') + ' | C ' + x.split(' C ', 1)[1].strip()].append(y)
    return a


runs = [agg(d) for d in sys.argv[1:]]
tot = [0.0] * len(runs)
for k in sorted(runs[0], key=lambda k: -sum(runs[0][k])):
    vals = []
    for i, r in enumerate(runs):
        tot[i] += sum(r.get(k, [0]))
        vals.append(sum(r[k]) / len(r[k]) if k in r else float('nan'))
    print(" -> ".join(f"{v:6.1f}" for v in vals) + f" us x{len(runs[0][k]):2d}  {k}")
print("per step (3 steps traced): " + " -> ".join(f"{t / 3:.0f} us" for t in tot))
