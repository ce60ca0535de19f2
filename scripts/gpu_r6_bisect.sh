# Round 6: the FastSRGAN bs2 mixed_float16 step test on the trees between the
# round-4 end and 3621845, each with its own library (git worktrees under bisect/, built in the
# build container): where did G conv2d/kernel's GPU-vs-emulation distance move?
set -o pipefail
mkdir -p gpurun_out/r6_bisect
export TMPDIR=/tmp
for c in a25c5ac d309e52 d6893a1 63e6bde c8cbf4c 3621845; do
  (cd bisect/$c && timeout -k 10 300 python -u -m pytest tests/test_fp16_gpu.py -k "fsrgan_fp16_step or srgan_fp16_step" \
      -s -q -p no:cacheprovider > ../../gpurun_out/r6_bisect/$c.log 2>&1)
  echo "$c: $(grep -c passed gpurun_out/r6_bisect/$c.log) $(grep -m1 'G conv2d/kernel' gpurun_out/r6_bisect/$c.log)"
done
echo done
