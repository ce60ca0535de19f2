# fp16x3 halo patches-per-block sweep (DG_X3H_PTILES) on VGG19's shallow layers at bs16
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DG_MATH=f16x3 DG_BS=16 DG_REPS=20 DG_LAYERS=V.b1c2,V.b2c1,V.b2c2
OUT=gpurun_out/x3h_pt_sweep.txt
: > $OUT
for pt in plan 1 2 4 8 16; do
  echo "## ptiles $pt" >> $OUT
  if [ $pt = plan ]; then timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1
  else DG_X3H_PTILES=$pt timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1; fi
done
echo done
