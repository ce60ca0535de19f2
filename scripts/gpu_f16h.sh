# fp16 halo tiles: parity (fp16 conv cases, SR steps) then same-box SRGAN A/B against the generic fp16 tiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp16_gpu.py > gpurun_out/f16h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f16h_tests.log; [ $rc -eq 0 ] || exit $rc
EXTRA="--model srgan --no-pmc-leg" bash scripts/gpu_ab_env.sh "DG_PLAN_DISABLE=halo_f16"
