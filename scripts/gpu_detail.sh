set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DG_BENCH_DETAIL=1 timeout -k 10 600 python bench.py --steps 10 --warmup 4 --no-cpu-baseline --no-core > gpurun_out/detail.json 2> gpurun_out/detail.err
echo rc=$?
