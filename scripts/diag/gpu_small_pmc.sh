# PMC passes over scripts/diag/small_bench.py (small-Cin conv kernels vs the generic GEMM path)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/spmc1 -o pmc --output-format csv -- python3 scripts/diag/small_bench.py --iters 3 > gpurun_out/spmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM -d gpurun_out/spmc2 -o pmc --output-format csv -- python3 scripts/diag/small_bench.py --iters 3 > gpurun_out/spmc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/spmc3 -o pmc --output-format csv -- python3 scripts/diag/small_bench.py --iters 3 > gpurun_out/spmc3.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run --output-format csv -- python3 scripts/diag/small_bench.py --iters 3 > gpurun_out/sprof.log 2>&1
