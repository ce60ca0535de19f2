# Round 6: NBUF variants of the fp16x3 implicit-GEMM tiles (DG_X3_NB45 / DG_X3_NB12 = 3): x3 kernel
# tests on each variant, same-box bench A/B (two alternating rounds), per-layer tables
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
for v in "$@"; do
  DG_LIB=$L/libdgan_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_x3_gpu.py > gpurun_out/r6_t_$v.log 2>&1 || { tail -20 gpurun_out/r6_t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r6_t_$v.log)"
done
bash scripts/gpu_ab_lib.sh "$@" || exit 1
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$L/libdgan_$v.so"; fi
  DG_LIB=$lib timeout -k 10 300 python scripts/layer_table.py --content 1 --steps 3 > gpurun_out/r6_lt_$v.md 2> gpurun_out/r6_lt_$v.err || exit 1
  echo "$v $(tail -4 gpurun_out/r6_lt_$v.md | head -2 | tr '\n' ' ')"
done
echo rc=0
