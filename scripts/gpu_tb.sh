# GPU tests then the bench (no CPU leg): the build -> measure loop
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/test.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo rc=$?
