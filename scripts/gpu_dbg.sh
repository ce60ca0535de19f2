set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sr_gpu.py -v -m gpu -k "geometries" --timeout 300 --timeout-method thread > gpurun_out/geo.log 2>&1
echo rc=$?
