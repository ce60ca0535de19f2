set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_LAYERS=${DG_LAYERS:-D.conv}
export DG_REPS=3
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmc3.log 2>&1
echo rc=$?
