# Round profile set: the bench line (with the CPU baseline), rocprofv3 kernel stats, and the two
# PMC traffic passes of the conv engine (FETCH_SIZE and WRITE_SIZE in separate runs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 30 --warmup 8 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/prof.log 2>&1 && \
bash scripts/gpu_pmc_bench.sh
