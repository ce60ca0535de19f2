# Round 6: the data-parallel step at world size 1 through RCCL, HIP graph vs eager launches
# (same box, alternating), next to the plain N=1 graph step; then the bucket-ready timeline.
set -o pipefail
mkdir -p gpurun_out/r6_dist
export TMPDIR=/tmp
O=gpurun_out/r6_dist
B="python bench.py --steps 30 --warmup 8 --no-cpu-baseline --no-twin --no-core --no-pmc-leg"
for r in 1 2; do
  timeout -k 10 300 $B > $O/plain_$r.json 2> $O/plain_$r.err || exit 1
  timeout -k 10 300 $B --dist > $O/dist_graph_$r.json 2> $O/dist_graph_$r.err || exit 1
  timeout -k 10 300 $B --dist --no-graph > $O/dist_eager_$r.json 2> $O/dist_eager_$r.err || exit 1
  for f in plain dist_graph dist_eager; do
    echo "$f $r $(python -c "import json;d=json.loads(open('$O/${f}_$r.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['config']['hip_graph'],d['config']['process_group'])")"
  done
done
timeout -k 10 300 python scripts/diag/bucket_timeline.py > $O/bucket_timeline.txt 2> $O/bucket_timeline.err
echo rc=$?
