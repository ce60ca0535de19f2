set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_LAYERS=${DG_LAYERS:-D.conv}
export DG_REPS=3
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmc.log 2>&1
echo rc=$?
