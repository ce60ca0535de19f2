import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/run_kernel_stats.csv')))
steps = [int(r['Calls']) // 2 for r in rows if 'k_adam' in r['Name']][0]
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('steps', steps, 'kernel ms/step %.3f' % (tot / 1e6 / steps))
agg = {}
for r in rows:
    key = r['Name'].split('(')[0].replace('void ', '')
    if 'conv_gemm' in key:
        key = 'conv_gemm (all)'
    agg[key] = agg.get(key, 0) + float(r['TotalDurationNs'])
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:18]:
    print(f"{v / 1e6 / steps:8.3f} ms/step  {k}")
