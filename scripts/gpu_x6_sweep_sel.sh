# selected layers under each bf16x6 tile config forced (DG_FORCE_X6CFG), batch 32
set -o pipefail
mkdir -p gpurun_out/sweepx
export DG_BS=${DG_BS:-32} DG_REPS=${DG_REPS:-7} DG_LAYERS=${DG_LAYERS:-G.down2,G.down3,D.down2,D.down3,G.up6,G.up7}
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/sweepx/default.log 2>&1 || exit 1
for c in 0 1 2 3 4 5; do
  DG_FORCE_X6CFG=$c timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/sweepx/x6_$c.log 2>&1 || exit 1
done
echo sweep done
