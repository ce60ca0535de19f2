set -o pipefail
mkdir -p gpurun_out
L=${L:-"G.down2,G.down4,G.up4,G.up6,G.up7,D.down2,D.conv"}
for c in ${CFGS:-0 4 5}; do
  DG_LAYERS=$L DG_FORCE_X6CFG=$c timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/x6ab_$c.log 2>&1 || exit 2
done
echo rc=0
