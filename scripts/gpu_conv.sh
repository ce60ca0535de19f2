set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -q -m gpu -x > gpurun_out/test_conv.log 2>&1 && \
timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1
echo rc=$?
