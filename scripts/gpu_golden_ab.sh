# the bs16 golden test under environment variants (diagnosis of numerics changes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base "$@"; do
  echo "== $v" >> gpurun_out/golden_ab.txt
  env $([ "$v" = base ] || echo $v) timeout -k 10 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread -m gpu "tests/test_golden_gpu.py::test_pix2pix_bs16_matches_golden" -s 2>&1 | grep -E "vs golden|passed|failed|^E .*Assert" >> gpurun_out/golden_ab.txt
done
exit 0
