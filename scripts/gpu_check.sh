# GPU round trip used while iterating: the -m gpu suite, then a short bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/check_tests.log 2>&1
rc=$?
tail -3 gpurun_out/check_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/check_bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], 'core', d['core']['value'], 'conv ms', d['roofline']['conv_launch_ms_per_step'], 'frac', d['roofline']['frac'])"
