# eager vs graph at N=1, and the data-parallel path (RCCL, world size 1) with and without graph capture
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-core"
timeout -k 10 300 $B --no-graph > gpurun_out/d_eager.json 2> gpurun_out/d_eager.err && \
timeout -k 10 300 $B --dist --no-graph > gpurun_out/d_dist_eager.json 2> gpurun_out/d_dist_eager.err && \
timeout -k 10 300 $B --dist > gpurun_out/d_dist_graph.json 2> gpurun_out/d_dist_graph.err
echo rc=$?
