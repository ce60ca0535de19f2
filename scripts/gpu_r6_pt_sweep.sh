# Round 6: patches per block (DG_X3H_PTILES) of the fp16x3 halo kernel's stride-2 phase plans
# (G / D down-block input gradients, the U-Net up-block forwards) and the PatchGAN's KT 4 halo,
# at the step's bs32, against the planner's pick
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DG_MATH=f16x3 DG_BS=32 DG_REPS=20 DG_LAYERS=G.down2,G.down3,G.down4,G.up5,G.up6,G.up7,D.down2,D.down3,D.conv
OUT=gpurun_out/x3h2_pt_sweep.txt
: > $OUT
for pt in plan 1 2 4 16 32; do
  echo "## ptiles $pt" >> $OUT
  if [ $pt = plan ]; then DG_PLAN_DEBUG=1 timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1
  else DG_X3H_PTILES=$pt timeout -k 10 120 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1; fi
done
echo done
