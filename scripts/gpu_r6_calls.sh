# Round 6: where each conv call of the pix2pix bs16 step spends its time -- every dispatch between
# the call's dg_mark brackets with its duration (rocprofv3 --kernel-trace), plus the per-layer table.
set -o pipefail
O=gpurun_out/r6_${TAG:-calls}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- \
    python3 scripts/pmc_layers.py run --out $O/marks.json > $O/kt.log 2>&1 || exit 1
python scripts/pmc_layers.py kernels --trace $O/kt --marks $O/marks.json > $O/calls.txt || exit 1
if [ -z "$NO_LAYERS" ]; then
timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > $O/layers_full.md 2> $O/layers_full.err || exit 1
tail -n 4 $O/layers_full.md
fi
echo rc=0
