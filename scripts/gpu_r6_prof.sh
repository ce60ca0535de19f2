# Round 6: one-stream kernel stats of the pix2pix bs16 step, and a same-box A/B of the five-stream
# step against one stream (DG_NO_OVERLAP=1) after the epilogue code-size changes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_prof
mkdir -p $O
DG_NO_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > $O/seq.log 2>&1 || exit 1
TAG=ovl bash scripts/gpu_r6_ab.sh "ovl" "one|DG_NO_OVERLAP=1"
