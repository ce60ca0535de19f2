// Shared helpers for libdgan (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "dgan.h"

namespace dg {

void set_error(const char *fmt, ...);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float act_fwd(float v, int act, float alpha) {
    switch (act) {
    case DG_ACT_LRELU: return v > 0.f ? v : v * alpha;
    case DG_ACT_RELU: return v > 0.f ? v : 0.f;
    case DG_ACT_TANH: return tanhf(v);
    case DG_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
    }
}

// derivative of the activation expressed through its OUTPUT z
// (LeakyReLU/ReLU: TF uses `features > 0 ? g : alpha*g`, sign(z) == sign(features);
//  tanh: 1 - z^2; sigmoid: z (1 - z)).
__device__ __forceinline__ float act_grad_from_out(float z, int act, float alpha) {
    switch (act) {
    case DG_ACT_LRELU: return z > 0.f ? 1.f : alpha;
    case DG_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case DG_ACT_TANH: return 1.f - z * z;
    case DG_ACT_SIGMOID: return z * (1.f - z);
    default: return 1.f;
    }
}

// Counter-based hash for dropout masks; restated bit-for-bit in oracle/p2p_oracle.py.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__host__ __device__ __forceinline__ bool dropout_keep(uint32_t seed, uint32_t step, uint32_t idx, float rate) {
    uint32_t h = mix32(seed ^ mix32(step * 0x9E3779B9U + 0x632BE5ABU) ^ mix32(idx + 0x85EBCA6BU));
    float u = (float)(h >> 8) * (1.0f / 16777216.0f);
    return u >= rate;
}

}  // namespace dg

#define DG_ARG(cond, ...)                                  \
    do {                                                   \
        if (!(cond)) {                                     \
            dg::set_error(__VA_ARGS__);                    \
            return DG_ERR_ARG;                             \
        }                                                  \
    } while (0)

#define DG_LAUNCHED(name)                                                        \
    do {                                                                         \
        hipError_t e__ = hipGetLastError();                                      \
        if (e__ != hipSuccess) {                                                 \
            dg::set_error("%s: launch failed: %s", name, hipGetErrorString(e__)); \
            return DG_ERR_HIP;                                                   \
        }                                                                        \
    } while (0)

static inline unsigned dg_cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }
