set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_conv_gpu.py -q -m gpu -x > gpurun_out/test_conv.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; tail -30 gpurun_out/test_conv.log; exit $rc; fi
DG_CONV_MATH=bf16x6 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/conv_bench_x6.log 2>&1
echo rc=$?
