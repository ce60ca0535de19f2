// Round 6 diagnostic: the cost of the per-workgroup max atomics (block_atomic_absmax) that
// measured-max producers end with -- the split-K reduce with a max output took 28-36 us against
// 10-12 us without (gpurun_out/r6_reduce).  Each variant: G workgroups of 256 threads, each
// reads 16 KiB (a stand-in for its share of a reduce) and ends with one atomicMax of its max into
// S shards placed STRIDE floats apart.  hipcc --offload-arch=gfx950 -O3 atomic_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) k_var(const float4 *x, long n4, unsigned *m, int shards, int stride, int mode) {
    float v = 0.f;
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n4; e += (long)gridDim.x * 256) {
        float4 q = x[e];
        v = fmaxf(v, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
    }
    __shared__ float red[4];
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        unsigned *w = m + (blockIdx.x % shards) * stride;
        const unsigned u = __float_as_uint(v);
        if (mode == 0) atomicMax(w, u);
        else if (mode == 1) {
            if (u > __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(w, u);
        } else if (mode == 3) {
            __hip_atomic_fetch_max(w, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // mode 2: no atomic (a plain store of the block's max to its own slot)
        else m[blockIdx.x * stride + 4096 * 32] = u;
    }
}

int main() {
    const long n4 = 4L << 20;   // 64 MiB of input
    float4 *x;
    unsigned *m;
    hipMalloc(&x, n4 * 16);
    hipMalloc(&m, (4096 * 32 + 8192 * 32) * 4);
    std::vector<float> h(n4 * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000003) * 1e-3f;
    hipMemcpy(x, h.data(), n4 * 16, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct V { const char *name; int shards, stride, mode; };
    const V vs[] = {{"no atomic (plain store per block)", 1, 1, 2},
                    {"1 shard", 1, 1, 0},
                    {"8 shards, adjacent (current layout)", 8, 1, 0},
                    {"8 shards, adjacent, load-check (current code)", 8, 1, 1},
                    {"8 shards, 128 B apart", 8, 32, 0},
                    {"8 shards, 128 B apart, load-check", 8, 32, 1},
                    {"64 shards, 128 B apart", 64, 32, 0},
                    {"8 shards, adjacent, workgroup scope", 8, 1, 3}};
    for (int grid : {256, 512, 1024, 2048, 4096}) {
        for (const V &v : vs) {
            float best = 1e9;
            for (int r = 0; r < 20; ++r) {
                hipMemsetAsync(m, 0, (4096 * 32 + 8192 * 32) * 4, 0);
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k_var, dim3(grid), dim3(256), 0, 0, x, n4, m, v.shards, v.stride, v.mode);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (r >= 3 && ms < best) best = ms;
            }
            unsigned hm[64 * 32];
            hipMemcpy(hm, m, sizeof(hm), hipMemcpyDeviceToHost);
            unsigned mx = 0;
            for (int i = 0; i < 64 * 32; ++i) mx = hm[i] > mx ? hm[i] : mx;
            printf("grid %5d  %-48s %8.2f us  (max %g)\n", grid, v.name, best * 1e3, *(float *)&mx);
        }
    }
    return 0;
}
