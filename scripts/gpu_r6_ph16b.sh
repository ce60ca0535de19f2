# Round 6: per-layer table of the pix2pix step with the 8 x 16 patch, the 16 x 16 patch, and the
# 16 x 16 patch with three weight buffers (libdgan_nb3.so), for the VGG19 rows.
set -o pipefail
O=gpurun_out/r6_ph16b
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
DG_X3H_PH=8 timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/ph8.md 2> $O/ph8.err || exit 1
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/ph16.md 2> $O/ph16.err || exit 1
DG_LIB=$L/libdgan_nb3.so timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/nb3.md 2> $O/nb3.err || exit 1
DG_X3H_PH=8 timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/ph8b.md 2> $O/ph8b.err || exit 1
tail -n 4 $O/ph8.md $O/ph16.md $O/nb3.md $O/ph8b.md
DG_X3H_PH=8 TAG=wx bash scripts/gpu_r6_ab.sh "wx|DG_X3H_PH=8" "nowx|DG_X3H_PH=8 DG_PLAN_DISABLE=wgrad_extra"
