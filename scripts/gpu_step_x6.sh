set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DG_CONV_MATH=bf16x6 timeout -k 10 400 python -m pytest tests/test_step_gpu.py -q -m gpu -x > gpurun_out/test_step_x6.log 2>&1; echo "step tests rc=$?"
DG_CONV_MATH=bf16x6 DG_BENCH_DETAIL=1 timeout -k 10 600 python bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/bench_x6.json 2> gpurun_out/bench_x6.err && \
DG_CONV_MATH=fp32 timeout -k 10 600 python bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err
echo rc=$?
