# Round 6: which library makes the pix2pix bs16 step non-deterministic run to run?
set -o pipefail
mkdir -p gpurun_out/r6_det
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
for lib in libdgan.so libdgan_nofield.so libdgan_nokern.so; do
  echo "== $lib"; DG_LIB=$L/$lib CONTENT=0 REPS=3 timeout -k 10 300 python -u scripts/diag/determinism.py 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== round-5 python, this library"
cp scripts/diag/determinism.py bisect/744e2fa/scripts/diag/determinism_r6.py
(cd bisect/744e2fa && DG_LIB=$L/libdgan.so CONTENT=0 REPS=3 timeout -k 10 300 python -u scripts/diag/determinism_r6.py 2>&1 | grep -v amdgpu.ids) || exit 1
echo "== round-5 python, round-5 library"
(cd bisect/744e2fa && CONTENT=0 REPS=3 timeout -k 10 300 python -u scripts/diag/determinism_r6.py 2>&1 | grep -v amdgpu.ids) || exit 1
