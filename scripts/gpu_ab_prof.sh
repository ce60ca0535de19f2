# same-box per-kernel A/B of variant libraries: rocprofv3 kernel stats of a short bench per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$L/libdgan_$v.so"; fi
  DG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$v -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 4 > gpurun_out/abp_$v.log 2>&1 || exit 1
done
echo done
