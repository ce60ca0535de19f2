set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DG_REPS=5
export DG_LAYERS=V.b1c2,V.b2c1,V.b2c2,D.down2,G.up7,G.down2,V.b3cx
for c in 1 6 2 7 3 8; do
  DG_FORCE_X6CFG=$c timeout -k 10 300 python scripts/conv_bench.py > gpurun_out/cfg_$c.log 2>&1 || exit 1
done
echo rc=0
