set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_sr_gpu.py tests/test_step_gpu.py tests/test_conv_gpu.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/sr.log 2>&1
echo rc=$?
