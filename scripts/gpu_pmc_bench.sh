# HBM traffic of the conv engine per training step (roofline.traffic):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), eager launches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 bench.py --profile-only --no-graph --steps 3 --warmup 2 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 bench.py --profile-only --no-graph --steps 3 --warmup 2 > gpurun_out/pmc_write.log 2>&1
echo rc=$?
