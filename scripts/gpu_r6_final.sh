# Round-6 measurement set (one GPU call): the -m gpu suite and smoke(), the four
# BASELINE workloads' bench lines (CPU baseline + live PMC traffic each), rocprofv3
# kernel stats of the three GAN steps (pix2pix also with one stream, DG_NO_OVERLAP=1: per-kernel durations
# without the side streams' concurrency), per-layer conv tables, and the per-conv-call
# PMC traffic table of the pix2pix step.  TAG names the outputs; SKIP_TESTS=1 skips
# the test suite (a re-measurement of an already tested tree).
set -o pipefail
TAG=${1:-r6_final}
mkdir -p gpurun_out
export TMPDIR=/tmp
# PART=1: tests, smoke and the four bench lines; PART=2: profiles, layer tables, PMC table
# (gpurun's 1200 s per call); unset: everything
if [ -z "$SKIP_TESTS" ] && [ "${PART:-0}" != 2 ]; then
  timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ "${PART:-0}" != 2 ]; then
timeout -k 10 500 python bench.py --steps 30 --warmup 8 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 400 python bench.py --model srgan --steps 30 --warmup 8 > gpurun_out/${TAG}_bench_srgan.json 2> gpurun_out/${TAG}_bench_srgan.err && \
timeout -k 10 500 python bench.py --model fsrgan --steps 10 --warmup 4 > gpurun_out/${TAG}_bench_fsrgan.json 2> gpurun_out/${TAG}_bench_fsrgan.err && \
timeout -k 10 400 python bench.py --model autoencoder --steps 30 --warmup 8 > gpurun_out/${TAG}_bench_autoencoder.json 2> gpurun_out/${TAG}_bench_autoencoder.err || exit 1
fi
[ "${PART:-0}" = 1 ] && { echo rc=0; exit 0; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/${TAG}_prof.log 2>&1 && \
DG_NO_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_seq -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/${TAG}_prof_seq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_srgan -o run --output-format csv -- python3 bench.py --model srgan --profile-only --steps 10 --warmup 4 > gpurun_out/${TAG}_prof_srgan.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_fsrgan -o run --output-format csv -- python3 bench.py --model fsrgan --profile-only --steps 6 --warmup 3 > gpurun_out/${TAG}_prof_fsrgan.log 2>&1 && \
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/${TAG}_layers_full.md 2> gpurun_out/${TAG}_layers_full.err && \
timeout -k 10 300 python scripts/layer_table.py --content 0 --steps 3 > gpurun_out/${TAG}_layers_core.md 2> gpurun_out/${TAG}_layers_core.err && \
timeout -k 10 300 python scripts/layer_table.py --model fsrgan --steps 2 > gpurun_out/${TAG}_layers_fsrgan.md 2> gpurun_out/${TAG}_layers_fsrgan.err && \
timeout -k 10 300 python scripts/layer_table.py --model srgan --steps 3 > gpurun_out/${TAG}_layers_srgan.md 2> gpurun_out/${TAG}_layers_srgan.err && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmcl_f -o pmc --output-format csv -- python3 scripts/pmc_layers.py run --out gpurun_out/${TAG}_marks_f.json > gpurun_out/${TAG}_pmcl_f.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmcl_w -o pmc --output-format csv -- python3 scripts/pmc_layers.py run --out gpurun_out/${TAG}_marks_w.json > gpurun_out/${TAG}_pmcl_w.log 2>&1 && \
python scripts/pmc_layers.py table --fetch gpurun_out/${TAG}_pmcl_f --write gpurun_out/${TAG}_pmcl_w --marks gpurun_out/${TAG}_marks_f.json > gpurun_out/${TAG}_pmc_layers.md
echo rc=$?
