set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_pool_gpu.py tests/test_planes_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_x6h_tests.log 2>&1 && \
bash scripts/gpu_ab_lib.sh ${AB_VARIANT:-rowmajor} > gpurun_out/ab_x6h_bench.txt 2>&1 && \
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/ab_x6h_layers_new.md 2>/dev/null && \
DG_LIB=$PWD/denoise-gan_amd/lib/libdgan_${AB_VARIANT:-rowmajor}.so timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/ab_x6h_layers_old.md 2>/dev/null
echo rc=$?
