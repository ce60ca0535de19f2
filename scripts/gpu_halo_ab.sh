# generic vs halo-tiled bf16x6 kernel on the VGG19 3x3 shapes (conv_bench, same box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base DG_NO_HALO=1; do
  echo "== $v" >> gpurun_out/halo_ab.txt
  env $([ "$v" = base ] || echo $v) DG_BS=32 DG_LAYERS=V.b2c2,V.b3cx,V.b4cx,G.down3,G.down4,G.up5,G.up6 timeout -k 10 120 python scripts/conv_bench.py >> gpurun_out/halo_ab.txt 2>&1 || exit 1
done
