# Round 6: run-to-run determinism, the -m gpu suite (one process), then one default bench line.
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
T=${TAG:-check}
REPS=3 timeout -k 10 300 python -u scripts/diag/determinism.py > $O/${T}_det.log 2>&1; rc=$?
grep -v amdgpu.ids $O/${T}_det.log
[ $rc -ne 0 ] && exit $rc
grep -q DIFFER $O/${T}_det.log && exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider \
    -rf --durations=15 ${TESTS:-} > $O/${T}_tests.log 2>&1; rc=$?
tail -n 25 $O/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 30 --warmup 8 --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
python -c "import json;d=json.loads(open('$O/${T}_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['graph_equals_eager'],d['roofline']['p2p_convs']['frac'],d['roofline']['frac'],d['core'],d['fp32_exact']['value'])"
