# Round 6: a 4-wave 128 x 256 fp16x3 implicit-GEMM tile (64 x 128 per wave, one wave per SIMD; kX3Cfgs 7 in the
# variant library libdgan_w4.so) against the planner's tiles, per layer at bs32, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DG_LIB=$PWD/denoise-gan_amd/lib/libdgan_w4.so
DG_FORCE_X3CFG=7 DG_FORCE_X3=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x3_gpu.py > gpurun_out/r6_w4_tests.log 2>&1 || { tail -30 gpurun_out/r6_w4_tests.log; exit 1; }
tail -1 gpurun_out/r6_w4_tests.log
export DG_MATH=f16x3 DG_BS=32 DG_REPS=20 DG_LAYERS=G.down2,G.down3,G.down4,G.down5,G.up4,G.up5,G.up6,G.up7,D.down2,D.down3,D.conv
OUT=gpurun_out/r6_w4_sweep.txt
: > $OUT
for r in 1 2; do
  for v in plan 7; do
    echo "## cfg $v round $r" >> $OUT
    if [ $v = plan ]; then timeout -k 10 150 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1
    else DG_FORCE_X3CFG=7 timeout -k 10 150 python scripts/conv_bench.py >> $OUT 2>&1 || exit 1; fi
  done
done
echo rc=0
