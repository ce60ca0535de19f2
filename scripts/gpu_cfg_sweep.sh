# Per-layer conv timing under each planner choice (conv_bench at the fused
# step's batch of 32): default plan, fp32 kernel, and each bf16x6 tile config
# forced -- to check the planner's choices after kernel changes.
set -o pipefail
mkdir -p gpurun_out/sweep
export DG_BS=${DG_BS:-32} DG_REPS=${DG_REPS:-7}
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/sweep/default.log 2>&1 || exit 1
DG_CONV_MATH=fp32 timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/sweep/fp32.log 2>&1 || exit 1
for c in 0 1 2 3 4 5; do
  DG_FORCE_X6CFG=$c timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/sweep/x6_$c.log 2>&1 || exit 1
done
echo sweep done
