# Round 6: determinism of the final tree, and wave-state PMC of the fp16x3 implicit-GEMM kernels
# (WGRAD 128x256 and the FWD / DGRAD tiles) on the pix2pix bs32 shapes (scripts/conv_bench.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/diag/determinism.py > gpurun_out/r6_end_determinism.txt 2>&1 || { tail -5 gpurun_out/r6_end_determinism.txt; exit 1; }
tail -3 gpurun_out/r6_end_determinism.txt
export DG_MATH=f16x3 DG_BS=32 DG_REPS=3 DG_LAYERS=G.up7,G.up6,D.conv,G.down3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/wpmc1 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/wpmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d gpurun_out/wpmc2 -o pmc --output-format csv -- python3 scripts/conv_bench.py > gpurun_out/wpmc2.log 2>&1
echo rc=$?
