set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/prof.log 2>&1
echo rc=$?
