// BatchNormalization (+ fused activation / dropout) for the training step.
//
// Reference semantics: Keras BatchNormalization() in training mode, as built
// at pix2pix.py:119 (down blocks), :135 (up blocks), :211 (D), followed by
// LeakyReLU (alpha 0.3, :121/:213) or Dropout(0.5)+ReLU (:137-140).  TF's
// FusedBatchNormV3 normalises with the biased batch variance and feeds the
// Bessel-corrected one into the moving average.
//
// All reductions are per channel over the M = N*H*W rows of an NHWC tensor
// and deterministic: fixed row chunks -> per-chunk partials -> an ordered,
// parallel finalize.  Streaming passes move float4 per lane whenever the
// channel count and strides allow it (V = 4), else one float (V = 1).
// Statistics inside a chunk use sums shifted by the chunk's first row (no
// catastrophic cancellation); chunks are combined with Chan's formula.
#include "common.h"
#include <algorithm>

namespace dg {

struct BnPlan {
    int R;       // row chunks
    long rows;   // rows per chunk
};

static BnPlan bn_plan(long M, int C) {
    // row chunks of >= 64 rows, at most 256 (measured: more, shorter chunks
    // slow the partial passes down); the finalize kernels hold a channel's
    // R partials in the registers of 16 lanes
    (void)C;
    BnPlan p;
    long r = std::min<long>(256, std::max<long>(1, (M + 63) / 64));
    p.rows = (M + r - 1) / r;
    p.R = (int)((M + p.rows - 1) / p.rows);
    return p;
}

// ws layout (floats) for S row segments of M rows each (independent
// statistics per segment: e.g. the G(x) and G(y) halves of one batched
// generator pass, pix2pix.py:44 / :90):
//   forward  [3*S*R*C partials (n, mean, M2)] [S*R*C unused] [4*S*C scale / shift]
//   backward [4*S*R*C partials (sums, maxima)] [6*S*C coefficients]
static size_t bn_ws_floats(long M, int C, int S = 1) {
    BnPlan p = bn_plan(M, C);
    return (size_t)4 * S * p.R * C + (size_t)6 * S * C + 64;
}

// the forward's per-channel scale / shift (z = act(y * scale + shift)), one rounding sequence
// for the forward (k_bn_stats_final) and the backward passes that recompute act'(z) from y
// (RZ), so both evaluate t = y * scale + shift to the same float.  shift keeps the rounding of
// rounds 1-4 (b - mu*g*inv: the SR family's fp16 step tests sit on rounding ties of it)
__device__ __forceinline__ void bn_scale_shift(float g, float inv, float mu, float b, float &sc, float &sh) {
    sc = g * inv;
    sh = b - mu * g * inv;
}

// segment of global row r (S is 1 or 2 in practice: a loop, no 64-bit divide)
__device__ __forceinline__ int seg_of(long &r, long M) {
    int s = 0;
    while (r >= M) { r -= M; ++s; }
    return s;
}

// block geometry of the partial passes: CPB channel slots (V channels each) x RL row lanes
struct PartGeom {
    int V, cpb, rl, cg;
};
static PartGeom part_geom(int C, int V) {
    PartGeom g;
    g.V = V;
    int slots = (C + V - 1) / V;
    int cpb = 1;
    while (cpb < slots && cpb < 64) cpb <<= 1;
    g.cpb = cpb;
    g.rl = 256 / cpb;
    g.cg = (slots + cpb - 1) / cpb;
    return g;
}

template <int V>
__device__ __forceinline__ void loadv(const float *p, float (&v)[V]) {
    if constexpr (V == 4) {
        f32x4 t = *reinterpret_cast<const f32x4 *>(p);
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
        v[0] = p[0];
    }
}

template <int V>
__device__ __forceinline__ void storev(float *p, const float (&v)[V]) {
    if constexpr (V == 4) {
        f32x4 t = {v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4 *>(p) = t;
    } else {
        p[0] = v[0];
    }
}

// per (segment, chunk, channel): n, mean, M2; grid (channel groups, chunks, segments)
template <int V>
__global__ void __launch_bounds__(256)
k_bn_stats_partial(const float *__restrict__ y, int ld, long M, int C, long rows, int cpb, float *__restrict__ pn,
                   float *__restrict__ pmean, float *__restrict__ pm2, float *__restrict__ pbd, float *zbound) {
    // pbd (may be NULL): per chunk max |y - K| + |chunk mean - K| >= max |y - chunk mean|, the
    // term of the output bound that scales fp16x3 z planes (k_bn_stats_final); zbound zeroed here
    __shared__ float s1s[256 * V], s2s[256 * V], dms[256 * V];
    if (zbound && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < X3_SHARDS)
        zbound[threadIdx.x * X3_SHARD_STRIDE] = 0.f;
    const int slot = threadIdx.x % cpb, rl = threadIdx.x / cpb, RL = 256 / cpb;
    const int c0 = (blockIdx.x * cpb + slot) * V;
    y += (long)blockIdx.z * M * ld;
    const long pbase = (long)blockIdx.z * gridDim.y;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = min(M, r0 + rows);
    float s1[V], s2[V], K[V], dm[V];
#pragma unroll
    for (int q = 0; q < V; ++q) s1[q] = s2[q] = dm[q] = 0.f;
    const bool cok = c0 < C;
    if (cok) {
        loadv<V>(y + r0 * ld + c0, K);
        // U rows' loads in flight per lane, summed in row order (deterministic)
        constexpr int U = 8;
        long r = r0 + rl;
        for (; r + (U - 1) * RL < r1; r += U * RL) {
            float v[U][V];
#pragma unroll
            for (int u = 0; u < U; ++u) loadv<V>(y + (r + u * RL) * ld + c0, v[u]);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    float d = v[u][q] - K[q];
                    s1[q] += d;
                    s2[q] += d * d;
                    dm[q] = fmaxf(dm[q], fabsf(d));
                }
        }
        for (; r < r1; r += RL) {
            float v[V];
            loadv<V>(y + r * ld + c0, v);
#pragma unroll
            for (int q = 0; q < V; ++q) {
                float d = v[q] - K[q];
                s1[q] += d;
                s2[q] += d * d;
                dm[q] = fmaxf(dm[q], fabsf(d));
            }
        }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
        s1s[threadIdx.x * V + q] = s1[q]; s2s[threadIdx.x * V + q] = s2[q]; dms[threadIdx.x * V + q] = dm[q];
    }
    __syncthreads();
    if (rl != 0 || !cok) return;
    for (int l = 1; l < RL; ++l) {
        const int t = threadIdx.x + l * cpb;
#pragma unroll
        for (int q = 0; q < V; ++q) {
            s1[q] += s1s[t * V + q]; s2[q] += s2s[t * V + q]; dm[q] = fmaxf(dm[q], dms[t * V + q]);
        }
    }
    const float n = (float)(r1 - r0);
#pragma unroll
    for (int q = 0; q < V; ++q) {
        const long o = (pbase + blockIdx.y) * C + c0 + q;
        pn[o] = n;
        pmean[o] = K[q] + s1[q] / n;
        pm2[o] = fmaxf(s2[q] - s1[q] * s1[q] / n, 0.f);
        if (pbd) pbd[o] = dm[q] + fabsf(s1[q] / n);
    }
}

// finalize: block = 16 channels x 16 lanes; lane l holds the chunk partials
// l, l + 16, ... (R <= 256: at most 16 per lane, all loads issued at once, each
// wave-load 16 consecutive channels of 4 chunk rows); Chan's combine as sums
// (mean = sum n_i mean_i / n, M2 = sum M2_i + n_i (mean_i - mean)^2) over the
// registers; the 16 lane sums of a channel added in a fixed order (deterministic)
constexpr int FIN_C = 16, FIN_L = 16, FIN_K = 16;
static_assert(FIN_L * FIN_K >= 256, "bn_plan's 256 chunks fit the finalize lanes");

__device__ __forceinline__ float lane_sum16(float v, float *sh, int cl, int ln) {
    sh[ln * FIN_C + cl] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < FIN_L; ++l) s += sh[l * FIN_C + cl];
    __syncthreads();
    return s;
}

// two (or four: sum, sum, max, max) 16-lane reductions through one LDS round, each
// in lane_sum16's order (bit-identical to separate calls, fewer barriers)
__device__ __forceinline__ void lane_sum16x2(float a, float b, float &sa, float &sb, float *sh, int cl, int ln) {
    sh[ln * FIN_C + cl] = a;
    sh[256 + ln * FIN_C + cl] = b;
    __syncthreads();
    sa = 0.f; sb = 0.f;
#pragma unroll
    for (int l = 0; l < FIN_L; ++l) { sa += sh[l * FIN_C + cl]; sb += sh[256 + l * FIN_C + cl]; }
    __syncthreads();
}
__device__ __forceinline__ void lane_red16x4(float (&v)[4], float *sh, int cl, int ln) {
#pragma unroll
    for (int j = 0; j < 4; ++j) sh[j * 256 + ln * FIN_C + cl] = v[j];
    __syncthreads();
    float r[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int l = 0; l < FIN_L; ++l) {
        r[0] += sh[l * FIN_C + cl];
        r[1] += sh[256 + l * FIN_C + cl];
        r[2] = fmaxf(r[2], sh[512 + l * FIN_C + cl]);
        r[3] = fmaxf(r[3], sh[768 + l * FIN_C + cl]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = r[j];
}

// segments in order: segment s's statistics normalise its rows, and the moving
// averages take the segments' updates one after the other (the reference's
// separate BN calls, e.g. G(x) then G(y))
__global__ void __launch_bounds__(256)
k_bn_stats_final(const float *pn, const float *pmean, const float *pm2, int R, int C, int S, const float *gamma,
                 const float *beta, float *save_mean, float *save_invstd, float *mm, float *mv, float momentum,
                 float eps, float *scale, float *shift, const float *pbd, float keep_scale, float *zbound,
                 const float *cp_bound) {
    // zbound (pbd set): max over channels and segments of (|scale| max |y - mean| + |beta|) x the
    // dropout keep scale >= max |z| (ReLU / LeakyReLU do not grow |t|), and the bound of the
    // tensor copied beside z (cp_bound, a max slot), into one of X3_SHARDS floats (zeroed by the
    // partial pass): the scale of the z planes (k_bn_apply)
    __shared__ float sh[2 * 256];
    const int cl = threadIdx.x % FIN_C, ln = threadIdx.x / FIN_C;
    const int c = blockIdx.x * FIN_C + cl;
    const bool cok = c < C;
    float mmc = 0.f, mvc = 0.f, zbn = 0.f;
    float gpar = 1.f, bpar = 0.f;   // (gamma / beta with the partials' load round, not after the reductions)
    if (ln == 0 && cok) {
        if (mm) mmc = mm[c];
        if (mv) mvc = mv[c];
        if (gamma) gpar = gamma[c];
        if (beta) bpar = beta[c];
    }
    for (int sg = 0; sg < S; ++sg) {
        const long o = (long)sg * R * C;
        float vn[FIN_K], vm[FIN_K], vq[FIN_K], vb[FIN_K];
#pragma unroll
        for (int k = 0; k < FIN_K; ++k) {
            const int r = ln + k * FIN_L;
            const bool ok = cok && r < R;
            const long i = o + (long)(ok ? r : 0) * C + (cok ? c : 0);
            vn[k] = ok ? pn[i] : 0.f;
            vm[k] = ok ? pmean[i] : 0.f;
            vq[k] = ok ? pm2[i] : 0.f;
            vb[k] = ok && pbd ? pbd[i] : 0.f;   // (in the same load round: the chunk bounds)
        }
        float sn = 0.f, sm = 0.f;
#pragma unroll
        for (int k = 0; k < FIN_K; ++k) { sn += vn[k]; sm += vn[k] * vm[k]; }
        float n, msum;
        lane_sum16x2(sn, sm, n, msum, sh, cl, ln);
        const float mu = n > 0.f ? msum / n : 0.f;
        float q = 0.f;
#pragma unroll
        for (int k = 0; k < FIN_K; ++k) {
            const float d = vm[k] - mu;
            q += vq[k] + vn[k] * d * d;
        }
        const float m2 = lane_sum16(q, sh, cl, ln);
        float dmax = 0.f;   // max |y - mu| over the segment's rows: chunk bound + |chunk mean - mu|
        if (pbd) {
#pragma unroll
            for (int k = 0; k < FIN_K; ++k) {
                const int r = ln + k * FIN_L;
                if (cok && r < R) dmax = fmaxf(dmax, vb[k] + fabsf(vm[k] - mu));
            }
            sh[ln * FIN_C + cl] = dmax;
            __syncthreads();
#pragma unroll
            for (int l = 0; l < FIN_L; ++l) dmax = fmaxf(dmax, sh[l * FIN_C + cl]);
            __syncthreads();
        }
        if (ln != 0 || !cok) continue;
        const float var = n > 0.f ? m2 / n : 0.f;
        const float inv = 1.f / sqrtf(var + eps);
        const int sc = sg * C + c;
        if (save_mean) save_mean[sc] = mu;
        if (save_invstd) save_invstd[sc] = inv;
        bn_scale_shift(gpar, inv, mu, bpar, scale[sc], shift[sc]);
        zbn = fmaxf(zbn, (fabsf(gpar * inv) * dmax + fabsf(bpar)) * keep_scale);
        mmc -= (mmc - mu) * (1.f - momentum);
        const float unb = n > 1.f ? m2 / (n - 1.f) : m2;
        mvc -= (mvc - unb) * (1.f - momentum);
    }
    if (ln == 0 && cok) {
        if (mm) mm[c] = mmc;
        if (mv) mv[c] = mvc;
    }
    if (zbound) {   // the block's 16 channels (and the copied tensor's bound), one vector atomic
        sh[threadIdx.x] = ln == 0 ? zbn : 0.f;
        __syncthreads();
        if (threadIdx.x == 0) {
            float b = 0.f;
            for (int i = 0; i < FIN_C; ++i) b = fmaxf(b, sh[i]);
            if (cp_bound && blockIdx.x == 0)
                for (int i = 0; i < X3_SHARDS; ++i) b = fmaxf(b, cp_bound[i * X3_SHARD_STRIDE]);
            atomicMax(reinterpret_cast<unsigned *>(zbound) + (blockIdx.x & (X3_SHARDS - 1)) * X3_SHARD_STRIDE,
                      __float_as_uint(b));
        }
    }
}

// S segments of M rows: segment s uses its own scale / shift ([S][C]) and
// dropout seed (seed + s * seed_stride; the mask index restarts per segment)
template <int V>
__global__ void __launch_bounds__(256)
k_bn_apply(const float *__restrict__ y, int ld, long M, int S, int C, const float *__restrict__ scale,
           const float *__restrict__ shift, float *__restrict__ z, int ldz, int act, float alpha, float drop_rate,
           uint32_t seed, uint32_t seed_stride, const int32_t *step_dev, unsigned short *zp0, int zp0C, int zp0col,
           unsigned short *zp1, int zp1C, int zp1col, _Float16 *__restrict__ zh, const float *__restrict__ res,
           int ldres, const float *zbound, const float *__restrict__ cp, int ldcp, int cpC, int cpcol) {
    // zbound: the planes' scale source (fp16x3 planes; NULL: F16X3_XS); cp: cpC channels of a
    // second tensor (the U-Net skip half of the concat, pix2pix.py:188) whose planes go to zp0 at
    // column cpcol with the same scale -- one scale for the whole consumer operand
    const float xs = zbound ? x3_grad_scale(zbound, nullptr) : F16X3_XS;
    const uint32_t step = step_dev ? (uint32_t)*step_dev : 0u;
    const float keep_scale = drop_rate > 0.f ? 1.f / (1.f - drop_rate) : 1.f;
    const int CV = C / V;
    const long total = (long)S * M * CV;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long r = e / CV;
        const int c = (int)(e - r * CV) * V;
        long rr = r;
        const int sg = seg_of(rr, M);
        float v[V], o[V], sc[V], sh[V];
        loadv<V>(y + r * ld + c, v);
        loadv<V>(scale + sg * C + c, sc);
        loadv<V>(shift + sg * C + c, sh);
        const uint32_t sd = seed + (uint32_t)sg * seed_stride;
#pragma unroll
        for (int q = 0; q < V; ++q) {
            float t = __builtin_fmaf(v[q], sc[q], sh[q]);
            if (drop_rate > 0.f)
                t = dropout_keep(sd, step, (uint32_t)(rr * C + c + q), drop_rate) ? t * keep_scale : 0.f;
            o[q] = act_fwd(t, act, alpha);
        }
        if (res) {   // a residual Add fused after the block (srgan.py:165, fsrgan.py:176): z = act(BN(y)) + res
            float rv[V];
            loadv<V>(res + r * ldres + c, rv);
#pragma unroll
            for (int q = 0; q < V; ++q) o[q] += rv[q];
        }
        storev<V>(z + r * ldz + c, o);
        // the consuming fp16 conv's operand copy of z ([rows][C])
        if (zh) {
            if constexpr (V == 4) store_f16x4(zh + r * C + c, f32x4{o[0], o[1], o[2], o[3]});
            else zh[r * C + c] = (_Float16)o[0];
        }
        // (V = 4) bf16x6 planes of z for up to two consuming convs, at channel
        // column col of their [rows][3 C] packed x planes (a concat's slice)
        if constexpr (V == 4) {
            if (zp0) store_planes4(zp0, zp0C, r, zp0col + c, f32x4{o[0], o[1], o[2], o[3]}, xs);
            if (zp1) store_planes4(zp1, zp1C, r, zp1col + c, f32x4{o[0], o[1], o[2], o[3]}, xs);
        }
    }
    if constexpr (V == 4) {
        if (cp) {
            const int CP4 = cpC / 4;
            const long tc = (long)S * M * CP4;
            for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < tc; e += (long)gridDim.x * blockDim.x) {
                const long r = e / CP4;
                const int c = (int)(e - r * CP4) * 4;
                store_planes4(zp0, zp0C, r, cpcol + c, *reinterpret_cast<const f32x4 *>(cp + r * ldcp + c), xs);
            }
        }
    }
}

// inference: coefficients recomputed per element from the moving statistics
__global__ void __launch_bounds__(256)
k_bn_apply_infer(const float *__restrict__ y, int ld, long M, int C, const float *gamma, const float *beta,
                 const float *mm, const float *mv, float eps, float *__restrict__ z, int ldz, int act, float alpha) {
    const long total = M * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        long r = e / C;
        int c = (int)(e - r * C);
        const float inv = 1.f / sqrtf(mv[c] + eps);
        const float g = gamma ? gamma[c] : 1.f;
        const float b = beta ? beta[c] : 0.f;
        z[r * ldz + c] = act_fwd((y[r * ld + c] - mm[c]) * inv * g + b, act, alpha);
    }
}

// the block output z, read only for act' (z NULL: a linear BN, act' = 1 -- the
// fused BN + residual Add never writes its own z)
template <int V>
__device__ __forceinline__ void load_z(const float *__restrict__ z, long off, float (&zv)[V]) {
    if (z) {
        loadv<V>(z + off, zv);
    } else {
#pragma unroll
        for (int q = 0; q < V; ++q) zv[q] = 0.f;
    }
}

// backward: partial sums of dbn and dbn*xhat per (chunk, channel); MX: also the maxima of the
// fp16x3 dy bound (pd / pv set) -- without them the pass keeps round 3's register / LDS footprint.
// RZ: act'(z) from the sign of t = y * scale + shift (the forward's, bn_scale_shift from gamma,
// offs, mean, invstd) instead of reading z -- ReLU / LeakyReLU without dropout, where
// sign(z) = sign(t); one tensor fewer per element
template <int V, bool MX, bool RZ = false>
__global__ void __launch_bounds__(256)
k_bn_bwd_partial(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz,
                 const float *__restrict__ y, int ldy, long M, int C, long rows, int cpb,
                 const float *__restrict__ mean, const float *__restrict__ invstd, int act, float alpha, float dscale,
                 float *__restrict__ p1, float *__restrict__ p2, float *__restrict__ pd, float *__restrict__ pv,
                 float *__restrict__ bound, const float *__restrict__ gamma, const float *__restrict__ offs) {
    // pd / pv (may be NULL): per chunk max |dbn| and max |y - mean|, the terms of the bound
    // on |dy| that scales its fp16x3 planes (k_bn_bwd_final); bound zeroed here for it
    __shared__ float a1s[256 * V], a2s[256 * V], dms[MX ? 256 * V : 1], vms[MX ? 256 * V : 1];
    if (bound && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < X3_SHARDS)
        bound[threadIdx.x * X3_SHARD_STRIDE] = 0.f;
    const int slot = threadIdx.x % cpb, rl = threadIdx.x / cpb, RL = 256 / cpb;
    const int c0 = (blockIdx.x * cpb + slot) * V;
    {   // segment blockIdx.z: its rows and its saved statistics
        const long ro = (long)blockIdx.z * M;
        dz += ro * lddz; y += ro * ldy;
        if (z) z += ro * ldz;
        mean += (long)blockIdx.z * C; invstd += (long)blockIdx.z * C;
    }
    const long pbase = (long)blockIdx.z * gridDim.y;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = min(M, r0 + rows);
    float a1[V], a2[V], dm[V], vm[V], mu[V], inv[V], fs[V], fh[V];
#pragma unroll
    for (int q = 0; q < V; ++q) a1[q] = a2[q] = dm[q] = vm[q] = 0.f;
    const bool cok = c0 < C;
    if (cok) {
        loadv<V>(mean + c0, mu);
        loadv<V>(invstd + c0, inv);
        if constexpr (RZ) {
#pragma unroll
            for (int q = 0; q < V; ++q)
                bn_scale_shift(gamma ? gamma[c0 + q] : 1.f, inv[q], mu[q], offs ? offs[c0 + q] : 0.f, fs[q], fh[q]);
        }
        auto acc_row = [&](const float (&dv)[V], const float (&zv)[V], const float (&yv)[V]) {
#pragma unroll
            for (int q = 0; q < V; ++q) {
                const float zq = RZ ? __builtin_fmaf(yv[q], fs[q], fh[q]) : zv[q];
                float dbn = dv[q] * act_grad_from_out(zq, act, alpha) * dscale;
                a1[q] += dbn;
                a2[q] += dbn * (yv[q] - mu[q]) * inv[q];
                if constexpr (MX) {
                    dm[q] = fmaxf(dm[q], fabsf(dbn));
                    vm[q] = fmaxf(vm[q], fabsf(yv[q] - mu[q]));
                }
            }
        };
        // U rows' loads in flight per lane, summed in row order (deterministic)
        constexpr int U = 4;
        long r = r0 + rl;
        for (; r + (U - 1) * RL < r1; r += U * RL) {
            float dv[U][V], zv[U][V], yv[U][V];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                loadv<V>(dz + (r + u * RL) * lddz + c0, dv[u]);
                load_z<V>(RZ ? nullptr : z, (r + u * RL) * ldz + c0, zv[u]);
                loadv<V>(y + (r + u * RL) * ldy + c0, yv[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc_row(dv[u], zv[u], yv[u]);
        }
        for (; r < r1; r += RL) {
            float dv[V], zv[V], yv[V];
            loadv<V>(dz + r * lddz + c0, dv);
            load_z<V>(RZ ? nullptr : z, r * ldz + c0, zv);
            loadv<V>(y + r * ldy + c0, yv);
            acc_row(dv, zv, yv);
        }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
        a1s[threadIdx.x * V + q] = a1[q]; a2s[threadIdx.x * V + q] = a2[q];
        if constexpr (MX) { dms[threadIdx.x * V + q] = dm[q]; vms[threadIdx.x * V + q] = vm[q]; }
    }
    __syncthreads();
    if (rl != 0 || !cok) return;
    for (int l = 1; l < RL; ++l) {
        const int t = threadIdx.x + l * cpb;
#pragma unroll
        for (int q = 0; q < V; ++q) {
            a1[q] += a1s[t * V + q]; a2[q] += a2s[t * V + q];
            if constexpr (MX) { dm[q] = fmaxf(dm[q], dms[t * V + q]); vm[q] = fmaxf(vm[q], vms[t * V + q]); }
        }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
        const long o = (pbase + blockIdx.y) * C + c0 + q;
        p1[o] = a1[q];
        p2[o] = a2[q];
        if constexpr (MX) { pd[o] = dm[q]; pv[o] = vm[q]; }
    }
}

// per segment s: coef[s] = [A | B | D | mean | scale | shift] ([S][6][C]); dgamma / dbeta = the
// sum over the segments (the reference's calls share the BN variables)
__global__ void __launch_bounds__(256)
k_bn_bwd_final(const float *p1, const float *p2, const float *pd, const float *pv, int R, int C, int S, long M,
               const float *gamma, const float *mean, const float *invstd, float *dgamma, float *dbeta, float beta,
               float *coef, float *bound, int rz, const float *offs) {
    // rz: also coef rows 4 / 5 = the forward's scale / shift (bn_scale_shift), for k_bn_bwd_apply's
    // act'(z) recomputed from y
    // bound (pd, pv set): max over channels and segments of |A| max|dbn| + |B| max|y - mean| + |D|
    // >= max |dy|, into one of X3_SHARDS floats (zeroed by the partial pass)
    // one load round and one LDS round per segment: p1 / p2 (and pd / pv) together
    __shared__ float sh[4 * 256];
    const int cl = threadIdx.x % FIN_C, ln = threadIdx.x / FIN_C;
    const int c = blockIdx.x * FIN_C + cl;
    float t1 = 0.f, t2 = 0.f, bnd = 0.f;
    // the per-channel operands with the partials' load round (S <= 2 segments: the forward's
    // statistics of both), not after the reductions
    float g = 1.f, off = 0.f, inv0 = 0.f, mu0 = 0.f, inv1 = 0.f, mu1 = 0.f;
    if (ln == 0 && c < C) {
        if (gamma) g = gamma[c];
        if (rz && offs) off = offs[c];
        inv0 = invstd[c]; mu0 = mean[c];
        if (S > 1) { inv1 = invstd[C + c]; mu1 = mean[C + c]; }
    }
    for (int sg = 0; sg < S; ++sg) {
        const long o = (long)sg * R * C;
        float v1[FIN_K], v2[FIN_K], vd[FIN_K], vv[FIN_K];
#pragma unroll
        for (int k = 0; k < FIN_K; ++k) {
            const int r = ln + k * FIN_L;
            const bool ok = c < C && r < R;
            const long i = o + (long)(ok ? r : 0) * C + (c < C ? c : 0);
            v1[k] = ok ? p1[i] : 0.f;
            v2[k] = ok ? p2[i] : 0.f;
            vd[k] = ok && pd ? pd[i] : 0.f;
            vv[k] = ok && pd ? pv[i] : 0.f;
        }
        float red[4] = {0.f, 0.f, 0.f, 0.f};   // sum, sum, max, max (maxima of non-negative values)
#pragma unroll
        for (int k = 0; k < FIN_K; ++k) {
            red[0] += v1[k];
            red[1] += v2[k];
            red[2] = fmaxf(red[2], vd[k]);
            red[3] = fmaxf(red[3], vv[k]);
        }
        lane_red16x4(red, sh, cl, ln);
        const float a1 = red[0], a2 = red[1], md = red[2], mv = red[3];
        if (ln != 0 || c >= C) continue;
        t1 += a1;
        t2 += a2;
        // dy = k1 (dbn - m1 - xhat m2), xhat = (y - mean) invstd  ==>  dy = A dbn + B (y - mean) + D
        const int sc = sg * C + c;
        const float inv = sg == 0 ? inv0 : (sg == 1 ? inv1 : invstd[sc]);
        const float mu = sg == 0 ? mu0 : (sg == 1 ? mu1 : mean[sc]);
        const float k1 = g * inv;
        const float m1 = a1 / (float)M, m2 = a2 / (float)M;
        float *cf = coef + (long)sg * 6 * C;
        cf[c] = k1;
        cf[C + c] = -k1 * m2 * inv;
        cf[2 * C + c] = -k1 * m1;
        cf[3 * C + c] = mu;
        if (rz) bn_scale_shift(g, inv, mu, off, cf[4 * C + c], cf[5 * C + c]);
        bnd = fmaxf(bnd, fabsf(k1) * md + fabsf(cf[C + c]) * mv + fabsf(cf[2 * C + c]));
    }
    if (ln == 0 && c < C) {
        if (dbeta) dbeta[c] = t1 + (beta != 0.f ? beta * dbeta[c] : 0.f);
        if (dgamma) dgamma[c] = t2 + (beta != 0.f ? beta * dgamma[c] : 0.f);
    }
    if (bound) {   // the block's 16 channels, one vector atomic (non-negative floats order as uints)
        sh[threadIdx.x] = ln == 0 ? bnd : 0.f;
        __syncthreads();
        if (threadIdx.x == 0) {
            float b = 0.f;
            for (int i = 0; i < FIN_C; ++i) b = fmaxf(b, sh[i]);
            atomicMax(reinterpret_cast<unsigned *>(bound) + (blockIdx.x & (X3_SHARDS - 1)) * X3_SHARD_STRIDE,
                      __float_as_uint(b));
        }
    }
}

template <int V, bool RZ = false>
__global__ void __launch_bounds__(256)
k_bn_bwd_apply(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz,
               const float *__restrict__ y, int ldy, long M, int S, int C, int act, float alpha, float dscale,
               const float *__restrict__ coef, float *__restrict__ dy, int lddy, unsigned short *__restrict__ dyp,
               _Float16 *__restrict__ dyh, const float *__restrict__ dyb) {
    // dyb (may be NULL): dy's bound -- its planes are then the consumer's fp16x3 planes,
    // scaled by x3_grad_scale(dyb) (k_bn_bwd_final)
    const float xs = dyb ? x3_grad_scale(dyb, nullptr) : 1.f;
    const int pC = dyb ? -C : C;
    // coef[s] = [A | B | D | mean] per channel:  dy = A * dbn + B * (y - mean) + D
    // dyp (V = 4, C % 16 == 0): dy's bf16x6 planes too, in the packed layout
    // the consuming conv reads (no split pass before its backward GEMMs)
    const int CV = C / V;
    const long total = (long)S * M * CV;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long r = e / CV;
        const int c = (int)(e - r * CV) * V;
        long rr = r;
        const float *cf = coef + (long)seg_of(rr, M) * 6 * C;
        float dv[V], zv[V], yv[V], A[V], B[V], D[V], Mu[V], o[V];
        loadv<V>(dz + r * lddz + c, dv);
        load_z<V>(RZ ? nullptr : z, r * ldz + c, zv);
        loadv<V>(y + r * ldy + c, yv);
        loadv<V>(cf + c, A);
        loadv<V>(cf + C + c, B);
        loadv<V>(cf + 2 * C + c, D);
        loadv<V>(cf + 3 * C + c, Mu);
        if constexpr (RZ) {   // act'(z) from t = y * scale + shift (the forward's rounding)
            float fs[V], fh[V];
            loadv<V>(cf + 4 * C + c, fs);
            loadv<V>(cf + 5 * C + c, fh);
#pragma unroll
            for (int q = 0; q < V; ++q) zv[q] = __builtin_fmaf(yv[q], fs[q], fh[q]);
        }
#pragma unroll
        for (int q = 0; q < V; ++q)
            o[q] = A[q] * (dv[q] * act_grad_from_out(zv[q], act, alpha) * dscale) + B[q] * (yv[q] - Mu[q]) + D[q];
        if (dy) storev<V>(dy + r * lddy + c, o);
        if constexpr (V == 4) {
            if (dyp) store_planes4(dyp, pC, r, c, f32x4{o[0], o[1], o[2], o[3]}, xs);
            if (dyh) store_f16x4(dyh + r * C + c, f32x4{o[0], o[1], o[2], o[3]});
        } else {
            if (dyh) dyh[r * C + c] = (_Float16)o[0];
        }
    }
}

template <int V>
__global__ void __launch_bounds__(256)
k_act_bwd(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz, long M, int C, int act,
          float alpha, float *__restrict__ dy, int lddy) {
    const int CV = C / V;
    const long total = M * CV;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long r = e / CV;
        const int c = (int)(e - r * CV) * V;
        float dv[V], zv[V], o[V];
        loadv<V>(dz + r * lddz + c, dv);
        loadv<V>(z + r * ldz + c, zv);
#pragma unroll
        for (int q = 0; q < V; ++q) o[q] = dv[q] * act_grad_from_out(zv[q], act, alpha);
        storev<V>(dy + r * lddy + c, o);
    }
}

static unsigned ew_grid(long n) { return (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n, 256), 8192)); }

// float4 path usable: channels and every stride multiple of 4, 16-byte aligned bases
static bool vec4_ok(int C, std::initializer_list<std::pair<const void *, int>> ts) {
    if (C % 4) return false;
    for (auto &t : ts)
        if (t.first && ((((uintptr_t)t.first) & 15) || (t.second % 4))) return false;
    return true;
}

}  // namespace dg

extern "C" {

int dg_bn_workspace_size(int M, int C, size_t *bytes) { return dg_bn_workspace_size_seg(1, M, C, bytes); }

int dg_bn_workspace_size_seg(int S, int M, int C, size_t *bytes) {
    DG_ARG(bytes && S >= 1 && M >= 0 && C > 0, "bad arguments");
    *bytes = dg::bn_ws_floats(M, C, S) * sizeof(float);
    return DG_OK;
}

int dg_bn_fwd_train(int M, int C, const float *y, int ldy, const float *gamma, const float *beta, float *save_mean,
                    float *save_invstd, float *moving_mean, float *moving_var, float momentum, float eps, float *z,
                    int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed, const int32_t *step_dev,
                    void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_fwd_train_seg(1, M, C, y, ldy, gamma, beta, save_mean, save_invstd, moving_mean, moving_var,
                               momentum, eps, z, ldz, act, alpha, drop_rate, drop_seed, 0u, step_dev, nullptr, 0, 0,
                               nullptr, 0, 0, ws, ws_bytes, stream);
}

int dg_bn_fwd_train_pl(int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                       float *save_mean, float *save_invstd, float *moving_mean, float *moving_var, float momentum,
                       float eps, float *z, int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed,
                       const int32_t *step_dev, void *zp0, int zp0C, int zp0col, void *zp1, int zp1C, int zp1col,
                       void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_fwd_train_seg(1, M, C, y, ldy, gamma, beta, save_mean, save_invstd, moving_mean, moving_var,
                               momentum, eps, z, ldz, act, alpha, drop_rate, drop_seed, 0u, step_dev, zp0, zp0C,
                               zp0col, zp1, zp1C, zp1col, ws, ws_bytes, stream);
}

int dg_bn_fwd_train_seg(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                        float *save_mean, float *save_invstd, float *moving_mean, float *moving_var, float momentum,
                        float eps, float *z, int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed,
                        uint32_t drop_seed_stride, const int32_t *step_dev, void *zp0, int zp0C, int zp0col,
                        void *zp1, int zp1C, int zp1col, void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_fwd_train_seg_h(S, M, C, y, ldy, gamma, beta, save_mean, save_invstd, moving_mean, moving_var,
                                 momentum, eps, z, ldz, act, alpha, drop_rate, drop_seed, drop_seed_stride, step_dev,
                                 zp0, zp0C, zp0col, zp1, zp1C, zp1col, nullptr, 0, nullptr, ws, ws_bytes, stream);
}

int dg_bn_fwd_train_seg_h(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                          float *save_mean, float *save_invstd, float *moving_mean, float *moving_var, float momentum,
                          float eps, float *z, int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed,
                          uint32_t drop_seed_stride, const int32_t *step_dev, void *zp0, int zp0C, int zp0col,
                          void *zp1, int zp1C, int zp1col, const float *res, int ldres, void *z_f16, void *ws,
                          size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_fwd_train_seg_x(S, M, C, y, ldy, gamma, beta, save_mean, save_invstd, moving_mean, moving_var,
                                 momentum, eps, z, ldz, act, alpha, drop_rate, drop_seed, drop_seed_stride, step_dev,
                                 zp0, zp0C, zp0col, zp1, zp1C, zp1col, nullptr, nullptr, 0, 0, 0, nullptr, res, ldres,
                                 z_f16, ws, ws_bytes, stream);
}

int dg_bn_fwd_train_seg_x(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                          float *save_mean, float *save_invstd, float *moving_mean, float *moving_var, float momentum,
                          float eps, float *z, int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed,
                          uint32_t drop_seed_stride, const int32_t *step_dev, void *zp0, int zp0C, int zp0col,
                          void *zp1, int zp1C, int zp1col, float *z_bound, const float *cp, int ldcp, int cpC,
                          int cpcol, const float *cp_bound, const float *res, int ldres, void *z_f16, void *ws,
                          size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(y && z && ws, "NULL tensor");
    DG_ARG(!z_bound || !res, "bound-scaled planes of a BN fused with a residual Add are not supported");
    DG_ARG(!cp || (z_bound && zp0 && zp0C < 0 && cpC > 0 && cpC % 32 == 0 && cpcol % 32 == 0 && ldcp % 4 == 0 &&
                   cpcol + cpC <= -zp0C && (((uintptr_t)cp) & 15) == 0),
           "copied planes: fp16x3 zp0 with a bound, cpC and cpcol multiples of 32 inside zp0, float4 rows");
    DG_ARG(!res || ldres >= C, "residual pixel stride smaller than channels");
    DG_ARG(!z_f16 || (((uintptr_t)z_f16) & 7) == 0, "fp16 copy must be 8-byte aligned");
    DG_ARG(S >= 1 && S <= 8 && M > 0 && C > 0 && ldy >= C && ldz >= C, "bad shape");
    DG_ARG(ws_bytes >= dg::bn_ws_floats(M, C, S) * sizeof(float), "workspace too small");
    DG_ARG(drop_rate >= 0.f && drop_rate < 1.f, "bad dropout rate");
    hipStream_t s = (hipStream_t)stream;
    dg::BnPlan bp = dg::bn_plan(M, C);
    float *w = (float *)ws;
    const size_t RC = (size_t)S * bp.R * C;
    float *pn = w, *pmean = w + RC, *pm2 = w + 2 * RC;
    float *scale = w + 3 * RC, *shift = scale + (size_t)S * C;
    const bool v4y = dg::vec4_ok(C, {{y, ldy}});
    // (z_bound: the chunk bounds go to the forward's unused partial slot)
    float *pbd = z_bound ? w + 3 * RC : nullptr;
    scale = w + 4 * RC;
    shift = scale + (size_t)S * C;
    if (v4y) {
        dg::PartGeom pg = dg::part_geom(C, 4);
        hipLaunchKernelGGL(dg::k_bn_stats_partial<4>, dim3(pg.cg, bp.R, S), dim3(256), 0, s, y, ldy, (long)M, C,
                           bp.rows, pg.cpb, pn, pmean, pm2, pbd, z_bound);
    } else {
        dg::PartGeom pg = dg::part_geom(C, 1);
        hipLaunchKernelGGL(dg::k_bn_stats_partial<1>, dim3(pg.cg, bp.R, S), dim3(256), 0, s, y, ldy, (long)M, C,
                           bp.rows, pg.cpb, pn, pmean, pm2, pbd, z_bound);
    }
    DG_LAUNCHED("bn_stats_partial");
    const float keep = drop_rate > 0.f ? 1.f / (1.f - drop_rate) : 1.f;
    hipLaunchKernelGGL(dg::k_bn_stats_final, dim3(dg_cdiv(C, dg::FIN_C)), dim3(256), 0, s, pn, pmean, pm2, bp.R, C, S,
                       gamma, beta, save_mean, save_invstd, moving_mean, moving_var, momentum, eps, scale, shift, pbd,
                       keep, z_bound, cp_bound);
    DG_LAUNCHED("bn_stats_final");
    const bool av4 = dg::vec4_ok(C, {{y, ldy}, {z, ldz}, {res, ldres}});
    unsigned short *p0 = (unsigned short *)zp0, *p1 = (unsigned short *)zp1;
    // (planes C < 0: the consumer's fp16x3 planes of -C channels, 32-channel groups)
    auto pl_ok = [&](const unsigned short *p, int pc, int col) {
        const int g = pc < 0 ? 32 : 16, apc = pc < 0 ? -pc : pc;
        return !p || (av4 && apc % g == 0 && col % g == 0 && C % g == 0 && col + C <= apc && (((uintptr_t)p) & 15) == 0);
    };
    DG_ARG(pl_ok(p0, zp0C, zp0col) && pl_ok(p1, zp1C, zp1col),
           "z planes need float4-aligned tensors, C and the column a multiple of 16 (fp16x3: 32), col + C <= planes C, "
           "16-byte alignment");
    const long MT = (long)S * M;
    DG_ARG(!cp || av4, "copied planes need float4-aligned tensors");
    if (av4)
        hipLaunchKernelGGL(dg::k_bn_apply<4>, dim3(dg::ew_grid(MT * C / 4)), dim3(256), 0, s, y, ldy, (long)M, S, C,
                           scale, shift, z, ldz, act, alpha, drop_rate, drop_seed, drop_seed_stride, step_dev, p0,
                           zp0C, zp0col, p1, zp1C, zp1col, (_Float16 *)z_f16, res, ldres, z_bound, cp, ldcp, cpC,
                           cpcol);
    else
        hipLaunchKernelGGL(dg::k_bn_apply<1>, dim3(dg::ew_grid(MT * C)), dim3(256), 0, s, y, ldy, (long)M, S, C, scale,
                           shift, z, ldz, act, alpha, drop_rate, drop_seed, drop_seed_stride, step_dev, p0, zp0C,
                           zp0col, p1, zp1C, zp1col, (_Float16 *)z_f16, res, ldres, z_bound, nullptr, 0, 0, 0);
    DG_LAUNCHED("bn_apply");
    return DG_OK;
}

int dg_bn_fwd_infer(int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                    const float *moving_mean, const float *moving_var, float eps, float *z, int ldz, int act,
                    float alpha, dg_stream_t stream) {
    DG_ARG(y && z && moving_mean && moving_var, "NULL tensor");
    DG_ARG(M > 0 && C > 0 && ldy >= C && ldz >= C, "bad shape");
    hipLaunchKernelGGL(dg::k_bn_apply_infer, dim3(dg::ew_grid((long)M * C)), dim3(256), 0, (hipStream_t)stream, y,
                       ldy, (long)M, C, gamma, beta, moving_mean, moving_var, eps, z, ldz, act, alpha);
    DG_LAUNCHED("bn_apply_infer");
    return DG_OK;
}

int dg_bn_bwd(int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y, int ldy,
              const float *gamma, const float *save_mean, const float *save_invstd, int act, float alpha,
              float drop_rate, float *dy, int lddy, float *dgamma, float *dbeta, float beta, void *ws,
              size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_bwd_seg(1, M, C, dz, lddz, z, ldz, y, ldy, gamma, save_mean, save_invstd, act, alpha, drop_rate, dy,
                         lddy, nullptr, dgamma, dbeta, beta, ws, ws_bytes, stream);
}

int dg_bn_bwd_pl(int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y, int ldy,
                 const float *gamma, const float *save_mean, const float *save_invstd, int act, float alpha,
                 float drop_rate, float *dy, int lddy, void *dy_planes, float *dgamma, float *dbeta, float beta,
                 void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_bwd_seg(1, M, C, dz, lddz, z, ldz, y, ldy, gamma, save_mean, save_invstd, act, alpha, drop_rate, dy,
                         lddy, dy_planes, dgamma, dbeta, beta, ws, ws_bytes, stream);
}

int dg_bn_bwd_seg(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y, int ldy,
                  const float *gamma, const float *save_mean, const float *save_invstd, int act, float alpha,
                  float drop_rate, float *dy, int lddy, void *dy_planes, float *dgamma, float *dbeta, float beta,
                  void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_bwd_seg_h(S, M, C, dz, lddz, z, ldz, y, ldy, gamma, save_mean, save_invstd, act, alpha, drop_rate, dy,
                           lddy, dy_planes, nullptr, dgamma, dbeta, beta, ws, ws_bytes, stream);
}

int dg_bn_bwd_seg_h(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y, int ldy,
                    const float *gamma, const float *save_mean, const float *save_invstd, int act, float alpha,
                    float drop_rate, float *dy, int lddy, void *dy_planes, void *dy_f16, float *dgamma, float *dbeta,
                    float beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_bn_bwd_seg_x(S, M, C, dz, lddz, z, ldz, y, ldy, gamma, save_mean, save_invstd, act, alpha, drop_rate, dy,
                           lddy, dy_planes, DG_PLANES_BF16X6, nullptr, dy_f16, dgamma, dbeta, beta, ws, ws_bytes,
                           stream);
}

}  // extern "C"

namespace dg {
// rz: act'(z) from y and the forward's scale / shift (gamma, offs, save_mean, save_invstd) -- z
// is not read (dg_bn_bwd_seg_r)
static int bn_bwd_impl(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y,
                       int ldy, const float *gamma, const float *offs, bool rz, const float *save_mean,
                       const float *save_invstd, int act, float alpha, float drop_rate, float *dy, int lddy,
                       void *dy_planes, int dy_planes_format, float *dy_bound, void *dy_f16, float *dgamma,
                       float *dbeta, float beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(!dy_f16 || (((uintptr_t)dy_f16) & 7) == 0, "fp16 copy must be 8-byte aligned");
    // dy NULL: only its planes are written (every consumer reads dy_planes)
    // z NULL: allowed for a linear BN without dropout (act' = 1, z is not read), and with rz
    DG_ARG(dz && (z || rz || (act == DG_ACT_NONE && drop_rate == 0.f)) && y && save_mean && save_invstd &&
           (dy || dy_planes) && ws, "NULL tensor");
    if (rz) z = nullptr;
    DG_ARG(dy_planes_format == DG_PLANES_BF16X6 || dy_planes_format == DG_PLANES_F16X3, "bad plane format");
    const bool x3 = dy_planes && dy_planes_format == DG_PLANES_F16X3;
    DG_ARG(!x3 || (dy_bound && C % 32 == 0), "fp16x3 dy planes need a bound buffer (8 floats) and C %% 32 == 0");
    if (!z) ldz = C;
    DG_ARG(S >= 1 && S <= 8 && M > 0 && C > 0 && lddz >= C && ldz >= C && ldy >= C && (!dy || lddy >= C), "bad shape");
    DG_ARG(ws_bytes >= dg::bn_ws_floats(M, C, S) * sizeof(float), "workspace too small");
    if (drop_rate > 0.f && act != DG_ACT_RELU) {
        dg::set_error("dropout backward needs a ReLU after it (mask recovered from the output)");
        return DG_ERR_UNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    const float dscale = drop_rate > 0.f ? 1.f / (1.f - drop_rate) : 1.f;
    dg::BnPlan bp = dg::bn_plan(M, C);
    float *w = (float *)ws;
    const size_t RC = (size_t)S * bp.R * C;
    float *p1 = w, *p2 = w + RC, *coef = w + 4 * RC;
    float *pd = x3 ? w + 2 * RC : nullptr, *pv = x3 ? w + 3 * RC : nullptr, *bnd = x3 ? dy_bound : nullptr;
    const bool v4 = dg::vec4_ok(C, {{dz, lddz}, {z, ldz}, {y, ldy}, {save_mean, 4}, {save_invstd, 4}});
    {
        const dg::PartGeom pg = dg::part_geom(C, v4 ? 4 : 1);
        const dim3 grid(pg.cg, bp.R, S);
#define DG_BNP(V_, MX_, RZ_)                                                                                    \
    hipLaunchKernelGGL((dg::k_bn_bwd_partial<V_, MX_, RZ_>), grid, dim3(256), 0, s, dz, lddz, z, ldz, y, ldy, (long)M, \
                       C, bp.rows, pg.cpb, save_mean, save_invstd, act, alpha, dscale, p1, p2, pd, pv, bnd, gamma, offs)
        if (rz) {
            if (v4 && x3) DG_BNP(4, true, true);
            else if (v4) DG_BNP(4, false, true);
            else if (x3) DG_BNP(1, true, true);
            else DG_BNP(1, false, true);
        } else {
            if (v4 && x3) DG_BNP(4, true, false);
            else if (v4) DG_BNP(4, false, false);
            else if (x3) DG_BNP(1, true, false);
            else DG_BNP(1, false, false);
        }
#undef DG_BNP
    }
    DG_LAUNCHED("bn_bwd_partial");
    hipLaunchKernelGGL(dg::k_bn_bwd_final, dim3(dg_cdiv(C, dg::FIN_C)), dim3(256), 0, s, p1, p2, pd, pv, bp.R, C, S,
                       (long)M, gamma, save_mean, save_invstd, dgamma, dbeta, beta, coef, bnd, rz ? 1 : 0, offs);
    DG_LAUNCHED("bn_bwd_final");
    const bool av4 = dg::vec4_ok(C, {{dz, lddz}, {z, ldz}, {y, ldy}, {dy, lddy}});
    unsigned short *dyp = (unsigned short *)dy_planes;
    DG_ARG(!dyp || (av4 && C % 16 == 0 && (((uintptr_t)dyp) & 15) == 0),
           "dy planes need C %% 16 == 0, float4-aligned tensors and a 16-byte aligned plane buffer");
    const long MT = (long)S * M;
#define DG_BNA(V_, RZ_)                                                                                    \
    hipLaunchKernelGGL((dg::k_bn_bwd_apply<V_, RZ_>), dim3(dg::ew_grid(MT * C / V_)), dim3(256), 0, s, dz, lddz, z, \
                       ldz, y, ldy, (long)M, S, C, act, alpha, dscale, coef, dy, lddy, dyp, (_Float16 *)dy_f16, bnd)
    if (av4 && rz) DG_BNA(4, true);
    else if (av4) DG_BNA(4, false);
    else if (rz) DG_BNA(1, true);
    else DG_BNA(1, false);
#undef DG_BNA
    DG_LAUNCHED("bn_bwd_apply");
    return DG_OK;
}
}  // namespace dg

extern "C" {

int dg_bn_bwd_seg_x(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz, const float *y, int ldy,
                    const float *gamma, const float *save_mean, const float *save_invstd, int act, float alpha,
                    float drop_rate, float *dy, int lddy, void *dy_planes, int dy_planes_format, float *dy_bound,
                    void *dy_f16, float *dgamma, float *dbeta, float beta, void *ws, size_t ws_bytes,
                    dg_stream_t stream) {
    return dg::bn_bwd_impl(S, M, C, dz, lddz, z, ldz, y, ldy, gamma, nullptr, false, save_mean, save_invstd, act,
                           alpha, drop_rate, dy, lddy, dy_planes, dy_planes_format, dy_bound, dy_f16, dgamma, dbeta,
                           beta, ws, ws_bytes, stream);
}

int dg_bn_bwd_seg_r(int S, int M, int C, const float *dz, int lddz, const float *y, int ldy, const float *gamma,
                    const float *bn_beta, const float *save_mean, const float *save_invstd, int act, float alpha,
                    float *dy, int lddy, void *dy_planes, int dy_planes_format, float *dy_bound, void *dy_f16,
                    float *dgamma, float *dbeta, float beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(act == DG_ACT_RELU || act == DG_ACT_LRELU || act == DG_ACT_NONE,
           "act'(z) recomputed from y needs ReLU / LeakyReLU / linear (sign(z) = sign(y * scale + shift))");
    return dg::bn_bwd_impl(S, M, C, dz, lddz, nullptr, C, y, ldy, gamma, bn_beta, true, save_mean, save_invstd, act,
                           alpha, 0.f, dy, lddy, dy_planes, dy_planes_format, dy_bound, dy_f16, dgamma, dbeta, beta,
                           ws, ws_bytes, stream);
}



int dg_act_bwd(int M, int C, const float *dz, int lddz, const float *z, int ldz, int act, float alpha, float *dy,
               int lddy, dg_stream_t stream) {
    DG_ARG(dz && z && dy, "NULL tensor");
    DG_ARG(M >= 0 && C > 0 && lddz >= C && ldz >= C && lddy >= C, "bad shape");
    if (M == 0) return DG_OK;
    if (dg::vec4_ok(C, {{dz, lddz}, {z, ldz}, {dy, lddy}}))
        hipLaunchKernelGGL(dg::k_act_bwd<4>, dim3(dg::ew_grid((long)M * C / 4)), dim3(256), 0, (hipStream_t)stream, dz,
                           lddz, z, ldz, (long)M, C, act, alpha, dy, lddy);
    else
        hipLaunchKernelGGL(dg::k_act_bwd<1>, dim3(dg::ew_grid((long)M * C)), dim3(256), 0, (hipStream_t)stream, dz,
                           lddz, z, ldz, (long)M, C, act, alpha, dy, lddy);
    DG_LAUNCHED("act_bwd");
    return DG_OK;
}

}  // extern "C"
