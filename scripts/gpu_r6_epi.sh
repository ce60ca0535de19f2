# Round 6: (1) split-K reduce durations at the 256K-thread target, (2) same-box A/B of the epilogue
# with its LDS passes not unrolled (default) against the unrolled form (libdgan_epiu.so), (3) the
# per-layer tables of both.
set -o pipefail
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
bash scripts/gpu_r6_reduce.sh || exit 1
TAG=epi bash scripts/gpu_r6_ab.sh "epi" "epiu|DG_LIB=@L/libdgan_epiu.so" || exit 1
O=gpurun_out/r6_epi
mkdir -p $O
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/epi.md 2> $O/epi.err || exit 1
DG_LIB=$L/libdgan_epiu.so timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/epiu.md 2> $O/epiu.err || exit 1
tail -n 4 $O/epi.md $O/epiu.md
