set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_REPS=5
timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/cfg_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_step_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo rc=$?
