# same-box A/B of an environment switch: GPU tests, then the bench alternating base / "$1"=1, twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/test.log 2>&1 || { echo tests failed; exit 1; }
tail -1 gpurun_out/test.log
B="python bench.py --steps 30 --warmup 8 --no-cpu-baseline"
for r in 1 2; do
  for v in base "$1"; do
    if [ "$v" = base ]; then e=""; else e="$v=${AB_VAL:-1}"; fi
    env $e timeout -k 10 300 $B > gpurun_out/abe_${v}_$r.json 2> gpurun_out/abe_${v}_$r.err || exit 1
    echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/abe_${v}_$r.json').read().strip().splitlines()[-1]);print(d['value'],d['core']['value'],d['roofline']['conv_launch_ms_per_step'])")"
  done
done
