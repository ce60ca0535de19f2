# narrow-channel layers (Cin 3/6, Cout 3) under each fp32 tile config forced (DG_FORCE_CFG)
set -o pipefail
mkdir -p gpurun_out/sweep32
export DG_BS=${DG_BS:-32} DG_REPS=${DG_REPS:-7} DG_LAYERS=G.down1,G.last,D.down1,V.b1c1
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/sweep32/default.log 2>&1 || exit 1
for c in 0 1 2 3 4 5 6; do
  DG_FORCE_CFG=$c timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/sweep32/cfg_$c.log 2>&1 || exit 1
done
echo sweep done
