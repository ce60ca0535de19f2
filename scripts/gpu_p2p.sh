set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_sr_gpu.py tests/test_fullsize_gpu.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/p2p.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo rc=$?
