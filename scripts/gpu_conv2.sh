set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_conv_gpu.py -q -m gpu -x > gpurun_out/test_conv.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/test_conv.log; exit 1; }
DG_CONV_MATH=fp32 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/conv_bench_fp32.log 2>&1 && \
DG_CONV_MATH=bf16x6 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/conv_bench_x6.log 2>&1
echo rc=$?
