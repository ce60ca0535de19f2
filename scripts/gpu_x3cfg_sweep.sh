# fp16x3 implicit-GEMM tile sweep (DG_FORCE_X3CFG 0..6 against the planner's choice) on the
# G / D stride-2 layers at the train step's bs32, one process per config.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DG_MATH=f16x3 DG_BS=32 DG_REPS=20
export DG_LAYERS=G.down2,G.down3,G.down4,G.up5,G.up6,G.up7,D.down2,D.down3,D.conv
OUT=gpurun_out/x3cfg_sweep.txt
: > $OUT
for c in plan 0 1 2 3 4 5 6; do
  echo "## cfg $c" >> $OUT
  if [ $c = plan ]; then timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1
  else DG_FORCE_X3CFG=$c timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1; fi
done
echo done
