set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_LAYERS=${DG_LAYERS:-D.conv}
export DG_REPS=5
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/pmcc1 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmcc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pmcc2 -o kt --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmcc2.log 2>&1
echo rc=$?
