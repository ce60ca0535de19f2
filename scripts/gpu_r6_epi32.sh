# Round 6: an epilogue change (the fp32 kernel LDS-staged epilogue; then the row-block loops not unrolled): the -m gpu suite,
# then a same-box A/B against the previous commit's library (libdgan_head.so).
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider \
    -rf > gpurun_out/r6/epi32_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r6/epi32_tests.log
[ $rc -ne 0 ] && exit $rc
TAG=${T:-epi32} bash scripts/gpu_r6_ab.sh "new" "head|DG_LIB=@L/libdgan_head.so"
