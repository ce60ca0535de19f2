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

// ---- bf16x6 plane layout (k_split3): per pixel row, per 16-channel group,
// hi[16] mid[16] lo[16] -- the producers that write a consumer's planes
// directly use these (conv epilogues, max pool)
// (lo_src -> bits 15:0, hi_src -> bits 31:16), round-to-nearest-even
__device__ __forceinline__ unsigned cvt_pk_bf16(float lo_src, float hi_src) {
    unsigned r;
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo_src), "v"(hi_src));
    return r;
}

// exact three-way split of the pair (x0, x1) into packed bf16 planes
__device__ __forceinline__ void split3(float x0, float x1, unsigned &h, unsigned &m, unsigned &l) {
    h = cvt_pk_bf16(x0, x1);
    const float r0 = x0 - __uint_as_float(h << 16);
    const float r1 = x1 - __uint_as_float(h & 0xffff0000u);
    m = cvt_pk_bf16(r0, r1);
    const float s0 = r0 - __uint_as_float(m << 16);
    const float s1 = r1 - __uint_as_float(m & 0xffff0000u);
    l = cvt_pk_bf16(s0, s1);
}

typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));

// fp16x3 operand planes (include/dgan.h DG_MATH_F16X3, the forward GEMMs of 3x3
// stride-1 layers): a pre-scaled value s*x = h + l is held as two fp16 pieces,
// h = fp16(s*x), l = fp16(s*x - h) (both RNE), |l| <= 2^-11 |s*x|; a product is
// h.h' + h.l' + l.h' (the dropped l.l' and l's own rounding each < 2^-22 |x x'|).
// Activation rows hold, per 32-channel group, h[32] l[32] (4 B per element);
// weight rows, per 16-column group, h[16] l[16].  The scales keep both operands
// inside fp16's normal range: activations x 2^-4 (|x| < 2^20), weights x 2^8; the
// GEMM multiplies its accumulators by F16X3_OSCALE.  A plane tensor in this
// format is passed to the device helpers below with a NEGATIVE channel count.
constexpr float F16X3_XS = 0.0625f;
constexpr float F16X3_WS = 256.f;
constexpr float F16X3_OSCALE = 1.f / (F16X3_XS * F16X3_WS);
__device__ __forceinline__ void split_x3(float x, float s, _Float16 &h, _Float16 &l) {
    const float v = x * s;
    h = (_Float16)v;
    l = (_Float16)(v - (float)h);
}
// Gradient operands (DG_MATH_F16X3 input gradients) have no static range: their planes
// are scaled by 2^(14 - e) with bound = m * g < 2^e read from device memory -- m a
// measured max |value| (atomicMax by the producer of the previous gradient), g a weight
// bound (max over input channels of sum |w|, NULL = 1) -- so the scaled values stay below
// 2^14 (fp16 max 65504) while values down to 2^-28 of the bound keep 22 bits
// A measured max is kept as X3_SHARDS floats (one per workgroup shard) X3_SHARD_STRIDE floats
// apart -- a 128-byte line each -- in an X3_SLOT-float slot; its value is their max.  Device-wide
// atomics to one line serialize at about 10 ns each whatever word they hit: with the 8 shards in
// one 32-byte run (round 5) a 2048-workgroup split-K reduce spent 20 us of its 30 on them; one
// line per shard costs nothing measurable (round 6, scripts/diag/atomic_bench.hip,
// profiles/r6/atomic_bench.txt).
constexpr int X3_SHARDS = 8;
constexpr int X3_SHARD_STRIDE = 32;
constexpr int X3_SLOT = X3_SHARDS * X3_SHARD_STRIDE;
// Activations use the same form when a scale source is given (dg_conv_set_act_scale,
// dg_bn_fwd_train_seg_x): a BN forward's bound of its output, a measured max, or a conv
// output's bound m * g + c (m: measured max |input|, g: max over output channels of sum |w|,
// c: max |bias|) -- a static 2^-4 would leave |x| < 2 with a subnormal low piece (an absolute
// floor of 2^-21 instead of 22 bits)
__device__ __forceinline__ float x3_bound_scale(float b) {
    if (!(b > 0.f) || !(b <= 3.0e38f)) return 1.f;
    int e;
    (void)frexpf(b, &e);   // b < 2^e
    return ldexpf(1.f, 14 - e);
}
__device__ __forceinline__ float x3_grad_scale(const float *m, const float *g, const float *c = nullptr) {
    float mm = m[0];
#pragma unroll
    for (int i = 1; i < X3_SHARDS; ++i) mm = fmaxf(mm, m[i * X3_SHARD_STRIDE]);
    return x3_bound_scale(mm * (g ? *g : 1.f) + (c ? *c : 0.f));
}
// the raw terms of a scale source, loaded at kernel entry and combined in the epilogue (the
// GEMM kernels: the loads then complete under the main loop instead of stalling each block's tail)
struct X3Raw {
    float m[X3_SHARDS];
    float g, c;
    bool on;
};
__device__ __forceinline__ X3Raw x3_raw(const float *m, const float *g, const float *c) {
    X3Raw r;
    r.on = m != nullptr;
#pragma unroll
    for (int i = 0; i < X3_SHARDS; ++i) r.m[i] = m ? m[i * X3_SHARD_STRIDE] : 0.f;
    r.g = g ? *g : 1.f;
    r.c = c ? *c : 0.f;
    return r;
}
__device__ __forceinline__ float x3_raw_scale(const X3Raw &r, float dflt) {
    if (!r.on) return dflt;
    float mm = r.m[0];
#pragma unroll
    for (int i = 1; i < X3_SHARDS; ++i) mm = fmaxf(mm, r.m[i]);
    return x3_bound_scale(mm * r.g + r.c);
}
// |v| into a sharded device max (non-negative floats order as their bit patterns): a
// butterfly over each wave's lanes, the waves' maxima through LDS, then one vector atomic into
// the workgroup's shard (a read-before-atomic test measured slower once the shards sit on their
// own lines).  Every thread of the workgroup must call it.
__device__ __forceinline__ void block_atomic_absmax(float *dst, float v) {
    __shared__ float red[16];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = (blockDim.x + 63) >> 6;
        for (int i = 1; i < nw; ++i) v = fmaxf(v, red[i]);
        unsigned *w = reinterpret_cast<unsigned *>(dst) +
                      ((blockIdx.x + blockIdx.y * gridDim.x) & (X3_SHARDS - 1)) * X3_SHARD_STRIDE;
        atomicMax(w, __float_as_uint(v));
    }
}

// planes of one output element / of 4 consecutive elements (col % 4 == 0) for the
// consuming conv: C > 0 bf16x6 planes, C < 0 fp16x3 activation planes (-C channels)
// (xs: the fp16x3 scale -- F16X3_XS for activations, x3_grad_scale for gradients)
__device__ __forceinline__ void store_planes1(unsigned short *yp, int C, long pix, int col, float x,
                                              float xs = F16X3_XS) {
    if (C < 0) {
        _Float16 *d = reinterpret_cast<_Float16 *>(yp) + pix * 2 * (-C) + (col >> 5) * 64 + (col & 31);
        split_x3(x, xs, d[0], d[32]);
        return;
    }
    unsigned h, m, l;
    split3(x, 0.f, h, m, l);
    unsigned short *d = yp + pix * 3 * C + (col >> 4) * 48 + (col & 15);
    d[0] = (unsigned short)h;
    d[16] = (unsigned short)m;
    d[32] = (unsigned short)l;
}
__device__ __forceinline__ void store_planes4(unsigned short *yp, int C, long pix, int col, f32x4 v,
                                              float xs = F16X3_XS) {
    if (C < 0) {
        _Float16 *d = reinterpret_cast<_Float16 *>(yp) + pix * 2 * (-C) + (col >> 5) * 64 + (col & 31);
        f16x4_t h, l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            _Float16 a, b;
            split_x3(v[q], xs, a, b);
            h[q] = a;
            l[q] = b;
        }
        *reinterpret_cast<f16x4_t *>(d) = h;
        *reinterpret_cast<f16x4_t *>(d + 32) = l;
        return;
    }
    unsigned h0, m0, l0, h1, m1, l1;
    split3(v[0], v[1], h0, m0, l0);
    split3(v[2], v[3], h1, m1, l1);
    unsigned short *d = yp + pix * 3 * C + (col >> 4) * 48 + (col & 15);
    *reinterpret_cast<u32x2_t *>(d) = u32x2_t{h0, h1};
    *reinterpret_cast<u32x2_t *>(d + 16) = u32x2_t{m0, m1};
    *reinterpret_cast<u32x2_t *>(d + 32) = u32x2_t{l0, l1};
}

// fp16 operand copy of a DG_MATH_FP16 GEMM operand ([rows][C], round-to-nearest-even like the
// conversion pass k_split_f16) of 4 consecutive elements / of one element
__device__ __forceinline__ void store_f16x4(_Float16 *d, f32x4 v) {
    *reinterpret_cast<f16x4_t *>(d) = f16x4_t{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
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
