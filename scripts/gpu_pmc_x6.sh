set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_LAYERS=${DG_LAYERS:-V.b3cx,V.b1c2}
export DG_REPS=3
export DG_CONV_MATH=bf16x6
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmcx1 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmcx1.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmcx2 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmcx2.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM GRBM_COUNT -d gpurun_out/pmcx3 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/pmcx3.log 2>&1
echo rc=$?
