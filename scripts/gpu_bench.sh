set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
DG_BENCH_DETAIL=1 timeout -k 10 600 python bench.py --steps 20 --warmup 6 --cpu-steps 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 5 --warmup 3 > gpurun_out/prof.log 2>&1
echo rc=$?
