# Round 6: input staging before the target's VGG19 fork (DG_STAGE_FIRST=1) vs after it -- same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DG_STAGE_FIRST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_overlap_gpu.py > gpurun_out/r6_sf_tests.log 2>&1 || { tail -20 gpurun_out/r6_sf_tests.log; exit 1; }
tail -1 gpurun_out/r6_sf_tests.log
EXTRA="--steps 60" TAG=sf bash scripts/gpu_r6_ab.sh "base" "first|DG_STAGE_FIRST=1" || exit 1
echo rc=0
