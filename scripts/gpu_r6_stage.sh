# Round 6: fused input staging (dg_stage_pair) and the BN finalize operand prefetch -- GPU tests of
# the touched paths, then a same-box A/B: the four-launch staging (DG_STAGE_SPLIT=1) and the
# previous BN finalize (variant library libdgan_bnold.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_abi.py tests/test_boundary_gpu.py tests/test_overlap_gpu.py tests/test_bn_gpu.py > gpurun_out/r6_stage_tests.log 2>&1 || { tail -30 gpurun_out/r6_stage_tests.log; exit 1; }
tail -1 gpurun_out/r6_stage_tests.log
TAG=stage bash scripts/gpu_r6_ab.sh "new" "split|DG_STAGE_SPLIT=1" "bnold|DG_LIB=@L/libdgan_bnold.so" || exit 1
python - <<'PY'
import json
L={t: json.loads(open(f"gpurun_out/r6_ab_stage/{t}_1.json").read().strip().splitlines()[-1])["losses"] for t in ("new","split","bnold")}
print("losses bit-equal new/split/bnold:", L["new"] == L["split"] == L["bnold"], L["new"])
PY
echo rc=0
