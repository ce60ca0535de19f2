# Round-3 measurement set (one GPU call): the four BASELINE workloads' bench lines (each with
# its CPU baseline and the live PMC traffic leg), the pix2pix per-layer conv tables, and
# rocprofv3 kernel stats of the pix2pix, SRGAN and FastSRGAN steps.  TAG names the outputs
# (gpurun_out/<TAG>_*).
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 30 --warmup 8 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 400 python bench.py --model srgan --steps 30 --warmup 8 > gpurun_out/${TAG}_bench_srgan.json 2> gpurun_out/${TAG}_bench_srgan.err && \
timeout -k 10 500 python bench.py --model fsrgan --steps 10 --warmup 4 > gpurun_out/${TAG}_bench_fsrgan.json 2> gpurun_out/${TAG}_bench_fsrgan.err && \
timeout -k 10 400 python bench.py --model autoencoder --steps 30 --warmup 8 > gpurun_out/${TAG}_bench_autoencoder.json 2> gpurun_out/${TAG}_bench_autoencoder.err && \
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/${TAG}_layers_full.md 2> gpurun_out/${TAG}_layers_full.err && \
timeout -k 10 300 python scripts/layer_table.py --content 0 --steps 3 > gpurun_out/${TAG}_layers_core.md 2> gpurun_out/${TAG}_layers_core.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/${TAG}_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_srgan -o run --output-format csv -- python3 bench.py --model srgan --profile-only --steps 10 --warmup 4 > gpurun_out/${TAG}_prof_srgan.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_fsrgan -o run --output-format csv -- python3 bench.py --model fsrgan --profile-only --steps 6 --warmup 3 > gpurun_out/${TAG}_prof_fsrgan.log 2>&1
echo rc=$?
