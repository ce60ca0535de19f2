set -o pipefail
mkdir -p gpurun_out
L="G.down3,G.down4,G.up4,G.up5,G.up6,D.down3,D.conv"
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -q -m gpu -x > gpurun_out/test_conv.log 2>&1 && \
timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/ab_default.log 2>&1 && \
DG_LAYERS=$L DG_FORCE_CFG=0 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/ab_cfg0.log 2>&1 && \
DG_LAYERS=$L DG_FORCE_CFG=5 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/ab_cfg5.log 2>&1
echo rc=$?
