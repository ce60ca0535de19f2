# Round 6: same-box A/B of one epilogue copy in the persistent fp16x3 halo loop (libdgan_epi1.so:
# 85 -> 56 KB of code, but 26-51 VGPRs spilled to scratch in the BN 128 kernels) against two copies.
TAG=epi1 bash scripts/gpu_r6_ab.sh "two" "one|DG_LIB=@L/libdgan_epi1.so"
