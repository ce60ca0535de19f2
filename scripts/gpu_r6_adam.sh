# Round 6: G's Adam per down block beside the backward and D's Adam on D's stream (ADAM_TAIL) --
# GPU tests of the step paths, then a same-box A/B against round 5's Adam placement (DG_NO_ADAM_TAIL=1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_overlap_gpu.py tests/test_boundary_gpu.py tests/test_step_gpu.py tests/test_golden_gpu.py > gpurun_out/r6_adam_tests.log 2>&1 || { tail -30 gpurun_out/r6_adam_tests.log; exit 1; }
tail -1 gpurun_out/r6_adam_tests.log
TAG=adam bash scripts/gpu_r6_ab.sh "tail" "old|DG_NO_ADAM_TAIL=1" || exit 1
python - <<'PY'
import json
for t in ("tail", "old"):
    d = json.loads(open(f"gpurun_out/r6_ab_adam/{t}_1.json").read().strip().splitlines()[-1])
    print(t, "graph_equals_eager", d["graph_equals_eager"]["equal"], "losses", d["losses"])
PY
echo rc=0
