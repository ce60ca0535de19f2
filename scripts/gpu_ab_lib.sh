# same-box A/B of variant libraries (scripts/build_variant.py): bench rounds base, variants..., repeated
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=denoise-gan_amd/lib
B="python bench.py --steps 30 --warmup 8 --no-cpu-baseline --no-core --no-pmc-leg"
for r in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/$L/libdgan_$v.so"; fi
    DG_LIB=$lib timeout -k 10 300 $B > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err || exit 1
    echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/ab_${v}_$r.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['conv_launch_ms_per_step'])")"
  done
done
