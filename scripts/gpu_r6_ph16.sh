# Round 6: the 16 x 16 patch (conv_x6h.hip PH 16): the fp16x3 kernel tests, then a same-box A/B
# of the bench with the 8 x 16 patch forced against the planner's pick.
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r6/ph16_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/r6/ph16_tests.log
[ $rc -ne 0 ] && exit $rc
TAG=ph16 bash scripts/gpu_r6_ab.sh "ph16" "ph8|DG_X3H_PH=8"
