set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_sr_gpu.py tests/test_step_gpu.py tests/test_x3_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6/c4_tests.log 2>&1; rc=$?
tail -n 6 gpurun_out/r6/c4_tests.log
[ $rc -ne 0 ] && exit $rc
TAG=l1 bash scripts/gpu_r6_ab.sh "base" "launder|DG_LIB=@L/libdgan_launder.so" "ng0|DG_XCD_NG=0" "ng8|DG_XCD_NG=8"
