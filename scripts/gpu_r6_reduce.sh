# Round 6: why do some split-K reduces of the pix2pix bs16 step take 25-35 us for 16 MB of
# partials?  (1) every reduce launch's arguments (DG_TRACE_REDUCE), (2) per-dispatch SQ counters
# of the reduce kernels in one step.
set -o pipefail
O=gpurun_out/r6_reduce
mkdir -p $O
export TMPDIR=/tmp
DG_TRACE_REDUCE=1 timeout -k 10 300 python3 scripts/pmc_layers.py run --out $O/marks.json 2> $O/args.txt || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    --kernel-include-regex splitk_reduce -d $O/pmc -o pmc --output-format csv -- \
    python3 scripts/pmc_layers.py run --out $O/marks2.json > $O/pmc.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex splitk_reduce -d $O/kt -o kt --output-format csv -- \
    python3 scripts/pmc_layers.py run --out $O/marks3.json > $O/kt.log 2>&1 || exit 1
echo rc=0
