# Per-layer conv tables (HIP events per conv call) with and without the VGG19 term,
# then rocprofv3 kernel stats of the bench step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/layers_full.md 2> gpurun_out/layers_full.err && \
timeout -k 10 300 python scripts/layer_table.py --content 0 --steps 3 > gpurun_out/layers_core.md 2> gpurun_out/layers_core.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/prof.log 2>&1
echo rc=$?
