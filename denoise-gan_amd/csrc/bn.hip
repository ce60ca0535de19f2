// BatchNormalization (+ fused activation / dropout) for the training step.
//
// Reference semantics: Keras BatchNormalization() in training mode, as built
// at pix2pix.py:119 (down blocks), :135 (up blocks), :211 (D), followed by
// LeakyReLU (alpha 0.3, :121/:213) or Dropout(0.5)+ReLU (:137-140).  TF's
// FusedBatchNormV3 normalises with the biased batch variance and feeds the
// Bessel-corrected one into the moving average.
//
// All reductions are per channel over the M = N*H*W rows of an NHWC tensor
// and deterministic: fixed row chunks -> (n, mean, M2) partials (Chan
// merge, shifted sums inside a chunk) -> ordered finalize.  A block is
// 64 channels x 4 row lanes, so each wave reads 256 contiguous bytes of a row.
#include "common.h"
#include <algorithm>

namespace dg {

struct BnPlan {
    int cg;      // channel groups of 64
    int R;       // row chunks
    long rows;   // rows per chunk
};

static BnPlan bn_plan(long M, int C) {
    BnPlan p;
    p.cg = (C + 63) / 64;
    // ~512 blocks in the partial pass, >= 64 rows each; the finalize combines
    // R partials per channel with 4 lanes, so R stays small
    long r = std::max<long>(1, 512 / p.cg);
    r = std::min<long>(r, std::max<long>(1, (M + 63) / 64));
    p.rows = (M + r - 1) / r;
    p.R = (int)((M + p.rows - 1) / p.rows);
    return p;
}

// ws layout (floats): [3*R*C partials] [2*C scale/shift or 3*C bwd coefs]
static size_t bn_ws_floats(long M, int C) {
    BnPlan p = bn_plan(M, C);
    return (size_t)3 * p.R * C + (size_t)4 * C + 64;
}

__device__ __forceinline__ void chan_merge(float &n, float &mean, float &m2, float nb, float meanb, float m2b) {
    if (nb == 0.f) return;
    if (n == 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
    float nn = n + nb;
    float d = meanb - mean;
    mean += d * (nb / nn);
    m2 += m2b + d * d * (n * nb / nn);
    n = nn;
}

__global__ void __launch_bounds__(256)
k_bn_stats_partial(const float *__restrict__ y, int ld, long M, int C, long rows, float *__restrict__ pn,
                   float *__restrict__ pmean, float *__restrict__ pm2) {
    __shared__ float sn[256], smean[256], sm2[256];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int rl = threadIdx.x >> 6;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = min(M, r0 + rows);
    float cnt = 0.f, mean = 0.f, m2 = 0.f;
    if (c < C && r0 < r1) {
        const float K = y[r0 * ld + c];
        float s1 = 0.f, s2 = 0.f;
        for (long r = r0 + rl; r < r1; r += 4) {
            float d = y[r * ld + c] - K;
            s1 += d;
            s2 += d * d;
            cnt += 1.f;
        }
        if (cnt > 0.f) {
            mean = K + s1 / cnt;
            m2 = fmaxf(s2 - s1 * s1 / cnt, 0.f);
        }
    }
    sn[threadIdx.x] = cnt; smean[threadIdx.x] = mean; sm2[threadIdx.x] = m2;
    __syncthreads();
    if (rl == 0 && c < C) {
        float n = sn[threadIdx.x], mu = smean[threadIdx.x], q = sm2[threadIdx.x];
        for (int k = 1; k < 4; ++k) {
            int t = threadIdx.x + 64 * k;
            chan_merge(n, mu, q, sn[t], smean[t], sm2[t]);
        }
        const long o = (long)blockIdx.y * C + c;
        pn[o] = n; pmean[o] = mu; pm2[o] = q;
    }
}

// finalize: block = 64 channels x 4 lanes; two parallel passes over the R
// chunk partials (Chan's combine written as sums: mean = sum n_i mean_i / n,
// M2 = sum M2_i + n_i (mean_i - mean)^2), no serial merge chain
__global__ void __launch_bounds__(256)
k_bn_stats_final(const float *pn, const float *pmean, const float *pm2, int R, int C, const float *gamma,
                 const float *beta, float *save_mean, float *save_invstd, float *mm, float *mv, float momentum,
                 float eps, float *scale, float *shift) {
    __shared__ float s0[256], s1[256];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int l4 = threadIdx.x >> 6;
    const int c64 = threadIdx.x & 63;
    float sn = 0.f, sm = 0.f;
    if (c < C)
        for (int r = l4; r < R; r += 4) {
            const float n = pn[(long)r * C + c];
            sn += n;
            sm += n * pmean[(long)r * C + c];
        }
    s0[threadIdx.x] = sn; s1[threadIdx.x] = sm;
    __syncthreads();
    const float n = s0[c64] + s0[c64 + 64] + s0[c64 + 128] + s0[c64 + 192];
    const float mu = n > 0.f ? (s1[c64] + s1[c64 + 64] + s1[c64 + 128] + s1[c64 + 192]) / n : 0.f;
    __syncthreads();
    float q = 0.f;
    if (c < C)
        for (int r = l4; r < R; r += 4) {
            const float d = pmean[(long)r * C + c] - mu;
            q += pm2[(long)r * C + c] + pn[(long)r * C + c] * d * d;
        }
    s0[threadIdx.x] = q;
    __syncthreads();
    if (l4 != 0 || c >= C) return;
    const float m2 = s0[c64] + s0[c64 + 64] + s0[c64 + 128] + s0[c64 + 192];
    const float var = n > 0.f ? m2 / n : 0.f;
    const float inv = 1.f / sqrtf(var + eps);
    if (save_mean) save_mean[c] = mu;
    if (save_invstd) save_invstd[c] = inv;
    const float g = gamma ? gamma[c] : 1.f;
    const float b = beta ? beta[c] : 0.f;
    scale[c] = g * inv;
    shift[c] = b - mu * g * inv;
    if (mm) mm[c] -= (mm[c] - mu) * (1.f - momentum);
    if (mv) {
        const float unb = n > 1.f ? m2 / (n - 1.f) : m2;
        mv[c] -= (mv[c] - unb) * (1.f - momentum);
    }
}

template <bool VEC4>
__global__ void __launch_bounds__(256)
k_bn_apply(const float *__restrict__ y, int ld, long M, int C, const float *__restrict__ scale,
           const float *__restrict__ shift, float *__restrict__ z, int ldz, int act, float alpha, float drop_rate,
           uint32_t seed, const int32_t *step_dev) {
    const uint32_t step = step_dev ? (uint32_t)*step_dev : 0u;
    const float keep_scale = drop_rate > 0.f ? 1.f / (1.f - drop_rate) : 1.f;
    const long stride = (long)gridDim.x * blockDim.x;
    if constexpr (VEC4) {
        const int C4 = C >> 2;
        const long total = M * C4;
        for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
            long r = e / C4;
            int c = (int)(e - r * C4) * 4;
            f32x4 v = *reinterpret_cast<const f32x4 *>(y + r * ld + c);
            f32x4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float t = v[q] * scale[c + q] + shift[c + q];
                if (drop_rate > 0.f) t = dropout_keep(seed, step, (uint32_t)(r * C + c + q), drop_rate) ? t * keep_scale : 0.f;
                o[q] = act_fwd(t, act, alpha);
            }
            *reinterpret_cast<f32x4 *>(z + r * ldz + c) = o;
        }
    } else {
        const long total = M * C;
        for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
            long r = e / C;
            int c = (int)(e - r * C);
            float t = y[r * ld + c] * scale[c] + shift[c];
            if (drop_rate > 0.f) t = dropout_keep(seed, step, (uint32_t)e, drop_rate) ? t * keep_scale : 0.f;
            z[r * ldz + c] = act_fwd(t, act, alpha);
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

// backward: partial sums of dbn and dbn*xhat per (chunk, channel)
__global__ void __launch_bounds__(256)
k_bn_bwd_partial(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz,
                 const float *__restrict__ y, int ldy, long M, int C, long rows, const float *__restrict__ mean,
                 const float *__restrict__ invstd, int act, float alpha, float dscale, float *__restrict__ p1,
                 float *__restrict__ p2) {
    __shared__ float s1[256], s2[256];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int rl = threadIdx.x >> 6;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = min(M, r0 + rows);
    float a1 = 0.f, a2 = 0.f;
    if (c < C) {
        const float mu = mean[c], inv = invstd[c];
        for (long r = r0 + rl; r < r1; r += 4) {
            float dbn = dz[r * lddz + c] * act_grad_from_out(z[r * ldz + c], act, alpha) * dscale;
            float xh = (y[r * ldy + c] - mu) * inv;
            a1 += dbn;
            a2 += dbn * xh;
        }
    }
    s1[threadIdx.x] = a1; s2[threadIdx.x] = a2;
    __syncthreads();
    if (rl == 0 && c < C) {
        float b1 = s1[threadIdx.x] + s1[threadIdx.x + 64] + s1[threadIdx.x + 128] + s1[threadIdx.x + 192];
        float b2 = s2[threadIdx.x] + s2[threadIdx.x + 64] + s2[threadIdx.x + 128] + s2[threadIdx.x + 192];
        const long o = (long)blockIdx.y * C + c;
        p1[o] = b1; p2[o] = b2;
    }
}

__global__ void __launch_bounds__(256)
k_bn_bwd_final(const float *p1, const float *p2, int R, int C, long M, const float *gamma, const float *invstd,
               float *dgamma, float *dbeta, float beta, float *coef) {
    __shared__ float s0[256], s1[256];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int l4 = threadIdx.x >> 6;
    const int c64 = threadIdx.x & 63;
    float a1 = 0.f, a2 = 0.f;
    if (c < C)
        for (int r = l4; r < R; r += 4) { a1 += p1[(long)r * C + c]; a2 += p2[(long)r * C + c]; }
    s0[threadIdx.x] = a1; s1[threadIdx.x] = a2;
    __syncthreads();
    if (l4 != 0 || c >= C) return;
    a1 = s0[c64] + s0[c64 + 64] + s0[c64 + 128] + s0[c64 + 192];
    a2 = s1[c64] + s1[c64 + 64] + s1[c64 + 128] + s1[c64 + 192];
    if (dbeta) dbeta[c] = a1 + (beta != 0.f ? beta * dbeta[c] : 0.f);
    if (dgamma) dgamma[c] = a2 + (beta != 0.f ? beta * dgamma[c] : 0.f);
    const float g = gamma ? gamma[c] : 1.f;
    coef[c] = g * invstd[c];
    coef[C + c] = a1 / (float)M;
    coef[2 * C + c] = a2 / (float)M;
}

__global__ void __launch_bounds__(256)
k_bn_bwd_apply(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz,
               const float *__restrict__ y, int ldy, long M, int C, const float *__restrict__ mean,
               const float *__restrict__ invstd, int act, float alpha, float dscale, const float *__restrict__ coef,
               float *__restrict__ dy, int lddy) {
    const long total = M * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        long r = e / C;
        int c = (int)(e - r * C);
        float dbn = dz[r * lddz + c] * act_grad_from_out(z[r * ldz + c], act, alpha) * dscale;
        float xh = (y[r * ldy + c] - mean[c]) * invstd[c];
        dy[r * lddy + c] = coef[c] * (dbn - coef[C + c] - xh * coef[2 * C + c]);
    }
}

__global__ void __launch_bounds__(256)
k_act_bwd(const float *__restrict__ dz, int lddz, const float *__restrict__ z, int ldz, long M, int C, int act,
          float alpha, float *__restrict__ dy, int lddy) {
    const long total = M * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        long r = e / C;
        int c = (int)(e - r * C);
        dy[r * lddy + c] = dz[r * lddz + c] * act_grad_from_out(z[r * ldz + c], act, alpha);
    }
}

static unsigned ew_grid(long n) { return (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n, 256), 8192)); }

}  // namespace dg

extern "C" {

int dg_bn_workspace_size(int M, int C, size_t *bytes) {
    DG_ARG(bytes && M >= 0 && C > 0, "bad arguments");
    *bytes = dg::bn_ws_floats(M, C) * sizeof(float);
    return DG_OK;
}

int dg_bn_fwd_train(int M, int C, const float *y, int ldy, const float *gamma, const float *beta, float *save_mean,
                    float *save_invstd, float *moving_mean, float *moving_var, float momentum, float eps, float *z,
                    int ldz, int act, float alpha, float drop_rate, uint32_t drop_seed, const int32_t *step_dev,
                    void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(y && z && ws, "NULL tensor");
    DG_ARG(M > 0 && C > 0 && ldy >= C && ldz >= C, "bad shape");
    DG_ARG(ws_bytes >= dg::bn_ws_floats(M, C) * sizeof(float), "workspace too small");
    DG_ARG(drop_rate >= 0.f && drop_rate < 1.f, "bad dropout rate");
    hipStream_t s = (hipStream_t)stream;
    dg::BnPlan bp = dg::bn_plan(M, C);
    float *w = (float *)ws;
    float *pn = w, *pmean = w + (size_t)bp.R * C, *pm2 = w + (size_t)2 * bp.R * C;
    float *scale = w + (size_t)3 * bp.R * C, *shift = scale + C;
    hipLaunchKernelGGL(dg::k_bn_stats_partial, dim3(bp.cg, bp.R), dim3(256), 0, s, y, ldy, (long)M, C, bp.rows, pn,
                       pmean, pm2);
    DG_LAUNCHED("bn_stats_partial");
    hipLaunchKernelGGL(dg::k_bn_stats_final, dim3(bp.cg), dim3(256), 0, s, pn, pmean, pm2, bp.R, C, gamma,
                       beta, save_mean, save_invstd, moving_mean, moving_var, momentum, eps, scale, shift);
    DG_LAUNCHED("bn_stats_final");
    bool vec = (C % 4 == 0) && (ldy % 4 == 0) && (ldz % 4 == 0) && ((((uintptr_t)y) | ((uintptr_t)z)) & 15) == 0;
    if (vec)
        hipLaunchKernelGGL(dg::k_bn_apply<true>, dim3(dg::ew_grid((long)M * C / 4)), dim3(256), 0, s, y, ldy, (long)M,
                           C, scale, shift, z, ldz, act, alpha, drop_rate, drop_seed, step_dev);
    else
        hipLaunchKernelGGL(dg::k_bn_apply<false>, dim3(dg::ew_grid((long)M * C)), dim3(256), 0, s, y, ldy, (long)M, C,
                           scale, shift, z, ldz, act, alpha, drop_rate, drop_seed, step_dev);
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
    DG_ARG(dz && z && y && save_mean && save_invstd && dy && ws, "NULL tensor");
    DG_ARG(M > 0 && C > 0 && lddz >= C && ldz >= C && ldy >= C && lddy >= C, "bad shape");
    DG_ARG(ws_bytes >= dg::bn_ws_floats(M, C) * sizeof(float), "workspace too small");
    if (drop_rate > 0.f && act != DG_ACT_RELU) {
        dg::set_error("dropout backward needs a ReLU after it (mask recovered from the output)");
        return DG_ERR_UNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    const float dscale = drop_rate > 0.f ? 1.f / (1.f - drop_rate) : 1.f;
    dg::BnPlan bp = dg::bn_plan(M, C);
    float *w = (float *)ws;
    float *p1 = w, *p2 = w + (size_t)bp.R * C, *coef = w + (size_t)3 * bp.R * C;
    hipLaunchKernelGGL(dg::k_bn_bwd_partial, dim3(bp.cg, bp.R), dim3(256), 0, s, dz, lddz, z, ldz, y, ldy, (long)M, C,
                       bp.rows, save_mean, save_invstd, act, alpha, dscale, p1, p2);
    DG_LAUNCHED("bn_bwd_partial");
    hipLaunchKernelGGL(dg::k_bn_bwd_final, dim3(bp.cg), dim3(256), 0, s, p1, p2, bp.R, C, (long)M, gamma,
                       save_invstd, dgamma, dbeta, beta, coef);
    DG_LAUNCHED("bn_bwd_final");
    hipLaunchKernelGGL(dg::k_bn_bwd_apply, dim3(dg::ew_grid((long)M * C)), dim3(256), 0, s, dz, lddz, z, ldz, y, ldy,
                       (long)M, C, save_mean, save_invstd, act, alpha, dscale, coef, dy, lddy);
    DG_LAUNCHED("bn_bwd_apply");
    return DG_OK;
}

int dg_act_bwd(int M, int C, const float *dz, int lddz, const float *z, int ldz, int act, float alpha, float *dy,
               int lddy, dg_stream_t stream) {
    DG_ARG(dz && z && dy, "NULL tensor");
    DG_ARG(M >= 0 && C > 0 && lddz >= C && ldz >= C && lddy >= C, "bad shape");
    if (M == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_act_bwd, dim3(dg::ew_grid((long)M * C)), dim3(256), 0, (hipStream_t)stream, dz, lddz, z,
                       ldz, (long)M, C, act, alpha, dy, lddy);
    DG_LAUNCHED("act_bwd");
    return DG_OK;
}

}  // extern "C"
