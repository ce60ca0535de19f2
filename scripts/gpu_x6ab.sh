set -o pipefail
mkdir -p gpurun_out
L="G.down2,G.down4,G.up4,G.up6,G.up7,D.down2,D.conv"
timeout -k 10 400 python -m pytest tests/test_conv_gpu.py -q -m gpu -x > gpurun_out/test_conv.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/test_conv.log; exit 1; }
for c in 0 4 5 6; do
  DG_CONV_MATH=bf16x6 DG_LAYERS=$L DG_FORCE_X6CFG=$c timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/x6ab_$c.log 2>&1 || exit 2
done
echo rc=0
