// Error reporting, version, and the small data-movement / optimizer kernels.
#include "common.h"
#include "conv_impl.h"
#include <cstdarg>
#include <cstdio>
#include <algorithm>

namespace dg {

static thread_local char g_err[512] = "no error";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Keras Adam as TF's ApplyAdam kernel computes it (train_pix2pix.py:68-69 ->
// ResourceApplyAdam): alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1);
// v += (g^2-v)(1-b2); p -= m*alpha/(sqrt(v)+eps) -- epsilon is added to
// sqrt(v), not to the bias-corrected v-hat.  One flat arena, float4 bulk.
__global__ void __launch_bounds__(256)
k_adam(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m, float *__restrict__ v, long n,
       float lr, float b1, float b2, float eps, float gscale, const int32_t *iter, long decay_steps,
       float decay_rate, int staircase, const float *ls) {
    if (ls) {   // dynamic loss scale: skip the step on non-finite gradients, else unscale
        if (ls[2] == 0.f) return;
        gscale /= ls[0];
    }
    const int it = iter ? *iter : 0;
    if (decay_steps > 0) {  // ExponentialDecay evaluated at optimizer.iterations (before the increment)
        float e = (float)it / (float)decay_steps;
        if (staircase) e = floorf(e);
        lr = lr * powf(decay_rate, e);
    }
    const float t = (float)(it + 1);
    const float lr_t = lr * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
    const long n4 = n >> 2;
    const long stride = (long)gridDim.x * blockDim.x;
    // U float4 groups per lane per round, all 4U loads issued before the first use (the
    // single-group loop waited a full HBM latency per 64 B of the 28 B/element stream)
    constexpr int U = 4;
    auto upd = [&](f32x4 gg, f32x4 &mm, f32x4 &vv, f32x4 &pp) __attribute__((always_inline)) {
        gg *= gscale;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mm[q] += (gg[q] - mm[q]) * (1.f - b1);
            vv[q] += (gg[q] * gg[q] - vv[q]) * (1.f - b2);
            pp[q] -= (mm[q] * lr_t) / (sqrtf(vv[q]) + eps);
        }
    };
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f32x4 gg[U], mm[U], vv[U], pp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            gg[u] = reinterpret_cast<const f32x4 *>(g)[i + u * stride];
            mm[u] = reinterpret_cast<f32x4 *>(m)[i + u * stride];
            vv[u] = reinterpret_cast<f32x4 *>(v)[i + u * stride];
            pp[u] = reinterpret_cast<f32x4 *>(p)[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            upd(gg[u], mm[u], vv[u], pp[u]);
            reinterpret_cast<f32x4 *>(m)[i + u * stride] = mm[u];
            reinterpret_cast<f32x4 *>(v)[i + u * stride] = vv[u];
            reinterpret_cast<f32x4 *>(p)[i + u * stride] = pp[u];
        }
    }
    for (; i < n4; i += stride) {
        f32x4 gg = reinterpret_cast<const f32x4 *>(g)[i];
        f32x4 mm = reinterpret_cast<f32x4 *>(m)[i];
        f32x4 vv = reinterpret_cast<f32x4 *>(v)[i];
        f32x4 pp = reinterpret_cast<f32x4 *>(p)[i];
        upd(gg, mm, vv, pp);
        reinterpret_cast<f32x4 *>(m)[i] = mm;
        reinterpret_cast<f32x4 *>(v)[i] = vv;
        reinterpret_cast<f32x4 *>(p)[i] = pp;
    }
    for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float gg = g[i] * gscale;
        float mm = m[i] + (gg - m[i]) * (1.f - b1);
        float vv = v[i] + (gg * gg - v[i]) * (1.f - b2);
        m[i] = mm; v[i] = vv;
        p[i] -= (mm * lr_t) / (sqrtf(vv) + eps);
    }
}

__global__ void k_counter_add(int32_t *c, int32_t inc, const float *ls) {
    if (!ls || ls[2] != 0.f) *c += inc;
}

// ---- dynamic loss scale (tf.keras mixed_precision LossScaleOptimizer, loss_scale='dynamic',
// srgan.py:64-67): state ls = {scale, good steps, finite flag, 0} on the device ----
__global__ void __launch_bounds__(256) k_scale_by(float *x, long n, const float *ls) {
    const float sc = ls[0];
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) x[e] *= sc;
}

// every thread that sees a non-finite gradient stores 0 to the flag (same value: race-free)
__global__ void __launch_bounds__(256) k_check_finite(const float *g, long n, float *ls) {
    bool bad = false;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
        bad |= !isfinite(g[e]);
    if (bad) ls[2] = 0.f;
}

// DynamicLossScale.update: finite -> good steps + 1, doubling the scale after `period`
// of them; non-finite -> halve (not below 1) and restart the count.  Re-arms the flag.
__global__ void k_loss_scale_update(float *ls, int period, float mult) {
    float sc = ls[0], good = ls[1];
    if (ls[2] != 0.f) {
        good += 1.f;
        if (good >= (float)period) {
            const float nx = sc * mult;
            if (isfinite(nx)) sc = nx;
            good = 0.f;
        }
    } else {
        sc = fmaxf(sc / mult, 1.f);
        good = 0.f;
    }
    ls[0] = sc;
    ls[1] = good;
    ls[2] = 1.f;
}

__global__ void __launch_bounds__(256)
k_channel_concat(long npix, const float *a, int lda, int ca, const float *b, int ldb, int cb, float *out, int ldo) {
    const int C = ca + cb;
    const long total = npix * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        long pix = e / C;
        int c = (int)(e - pix * C);
        out[pix * ldo + c] = c < ca ? a[pix * lda + c] : b[pix * ldb + (c - ca)];
    }
}

__global__ void __launch_bounds__(256)
k_strided_copy(long npix, int C, const float *src, int lds, float *dst, int ldd) {
    if (C <= 4) {   // (a few channels: one pixel per lane, no per-element index division)
        for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x)
            for (int c = 0; c < C; ++c) dst[p * ldd + c] = src[p * lds + c];
        return;
    }
    const long total = npix * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        long pix = e / C;
        int c = (int)(e - pix * C);
        dst[pix * ldd + c] = src[pix * lds + c];
    }
}

// the pix2pix step's input staging in one pass over the pixels (trainer.Pix2PixTrainer.step):
// cat = [x | y] (D(real)'s input, pix2pix.py:200), catx[:, 0:C] = x (D(fake)'s input, whose other
// half G(x) fills), gx / gy = x / y (the 2N-image G batch of the identity pass, pix2pix.py:44,90)
__global__ void __launch_bounds__(256)
k_stage_pair(long npix, int C, const float *__restrict__ x, const float *__restrict__ y, float *__restrict__ cat,
             int ldcat, float *__restrict__ catx, int ldcatx, float *__restrict__ gx, float *__restrict__ gy) {
    for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
        float xv[4], yv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (c < C) { xv[c] = x[p * C + c]; yv[c] = y[p * C + c]; }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c >= C) break;
            cat[p * ldcat + c] = xv[c];
            cat[p * ldcat + C + c] = yv[c];
            if (catx) catx[p * ldcatx + c] = xv[c];
            if (gx) gx[p * C + c] = xv[c];
            if (gy) gy[p * C + c] = yv[c];
        }
    }
}

__global__ void __launch_bounds__(256) k_fill(float *p, long n, float v) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) p[e] = v;
}

static unsigned grid_for(long n) { return (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n, 256), 8192)); }

}  // namespace dg

// an empty dispatch that marks a position in the stream's kernel sequence (profiling:
// scripts/pmc_layers.py attributes per-dispatch PMC counters to the library calls between
// two marks); `id` only makes the dispatch's arguments distinct
__global__ void k_mark(int id) { (void)id; }

extern "C" {

const char *dg_last_error_string(void) { return dg::g_err; }
int dg_version(void) { return 1; }
static_assert(dg::X3_SLOT == DG_MAX_SLOT, "include/dgan.h DG_MAX_SLOT is the library's max-slot size");
int dg_max_slot_floats(void) { return dg::X3_SLOT; }

#ifndef DG_SOURCE_SHA
#define DG_SOURCE_SHA "unknown"
#endif
// the sources this binary was built from (dgan/build.py passes source_sha(): sha256 over
// csrc/* and include/dgan.h), the target and the compiler
const char *dg_build_info(void) {
    return "source_sha=" DG_SOURCE_SHA ";arch=gfx950;hip=" __VERSION__;
}

int dg_mark(int id, dg_stream_t stream) {
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, (hipStream_t)stream, id);
    DG_LAUNCHED("mark");
    return DG_OK;
}

int dg_adam(float *p, const float *g, float *m, float *v, int64_t n, float lr, float beta1, float beta2, float eps,
            float grad_scale, const int32_t *iter_dev, dg_stream_t stream) {
    DG_ARG(p && g && m && v, "NULL tensor");
    DG_ARG(n >= 0, "negative size");
    DG_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0, "adam buffers must be 16B aligned");
    if (n == 0) return DG_OK;
    unsigned grid = (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n / 4 + 1, 256), 4096));
    hipLaunchKernelGGL(dg::k_adam, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)n, lr, beta1,
                       beta2, eps, grad_scale, iter_dev, 0L, 1.f, 0, (const float *)nullptr);
    DG_LAUNCHED("adam");
    return DG_OK;
}

int dg_adam_sched(float *p, const float *g, float *m, float *v, int64_t n, float lr, int64_t decay_steps,
                  float decay_rate, int staircase, float beta1, float beta2, float eps, float grad_scale,
                  const int32_t *iter_dev, dg_stream_t stream) {
    DG_ARG(p && g && m && v, "NULL tensor");
    DG_ARG(n >= 0, "negative size");
    DG_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0, "adam buffers must be 16B aligned");
    if (n == 0) return DG_OK;
    unsigned grid = (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n / 4 + 1, 256), 4096));
    hipLaunchKernelGGL(dg::k_adam, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)n, lr, beta1,
                       beta2, eps, grad_scale, iter_dev, (long)decay_steps, decay_rate, staircase,
                       (const float *)nullptr);
    DG_LAUNCHED("adam_sched");
    return DG_OK;
}

int dg_adam_ls(float *p, const float *g, float *m, float *v, int64_t n, float lr, int64_t decay_steps,
               float decay_rate, int staircase, float beta1, float beta2, float eps, float grad_scale,
               const int32_t *iter_dev, const float *loss_scale, dg_stream_t stream) {
    DG_ARG(p && g && m && v && loss_scale, "NULL tensor");
    DG_ARG(n >= 0, "negative size");
    DG_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0, "adam buffers must be 16B aligned");
    if (n == 0) return DG_OK;
    unsigned grid = (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n / 4 + 1, 256), 4096));
    hipLaunchKernelGGL(dg::k_adam, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)n, lr, beta1,
                       beta2, eps, grad_scale, iter_dev, (long)decay_steps, decay_rate, staircase, loss_scale);
    DG_LAUNCHED("adam_ls");
    return DG_OK;
}

int dg_counter_add_ls(int32_t *counter_dev, int32_t inc, const float *loss_scale, dg_stream_t stream) {
    DG_ARG(counter_dev, "NULL counter");
    hipLaunchKernelGGL(dg::k_counter_add, dim3(1), dim3(1), 0, (hipStream_t)stream, counter_dev, inc, loss_scale);
    DG_LAUNCHED("counter_add_ls");
    return DG_OK;
}

int dg_scale_by(int64_t n, float *x, const float *loss_scale, dg_stream_t stream) {
    DG_ARG((x || n == 0) && loss_scale, "NULL tensor");
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_scale_by, dim3(dg::grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, (long)n,
                       loss_scale);
    DG_LAUNCHED("scale_by");
    return DG_OK;
}

int dg_check_finite(int64_t n, const float *g, float *loss_scale, dg_stream_t stream) {
    DG_ARG((g || n == 0) && loss_scale, "NULL tensor");
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_check_finite, dim3(std::min<unsigned>(dg::grid_for(n), 2048)), dim3(256), 0,
                       (hipStream_t)stream, g, (long)n, loss_scale);
    DG_LAUNCHED("check_finite");
    return DG_OK;
}

int dg_loss_scale_update(float *loss_scale, int period, float multiplier, dg_stream_t stream) {
    DG_ARG(loss_scale && period > 0 && multiplier > 1.f, "bad arguments");
    hipLaunchKernelGGL(dg::k_loss_scale_update, dim3(1), dim3(1), 0, (hipStream_t)stream, loss_scale, period,
                       multiplier);
    DG_LAUNCHED("loss_scale_update");
    return DG_OK;
}

int dg_counter_add(int32_t *counter_dev, int32_t inc, dg_stream_t stream) {
    DG_ARG(counter_dev, "NULL counter");
    hipLaunchKernelGGL(dg::k_counter_add, dim3(1), dim3(1), 0, (hipStream_t)stream, counter_dev, inc,
                       (const float *)nullptr);
    DG_LAUNCHED("counter_add");
    return DG_OK;
}

int dg_channel_concat(int64_t npix, const float *a, int lda, int ca, const float *b, int ldb, int cb, float *out,
                      int ldo, dg_stream_t stream) {
    DG_ARG(a && b && out, "NULL tensor");
    DG_ARG(lda >= ca && ldb >= cb && ldo >= ca + cb, "bad strides");
    long total = (long)npix * (ca + cb);
    if (total == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_channel_concat, dim3(dg::grid_for(total)), dim3(256), 0, (hipStream_t)stream, (long)npix,
                       a, lda, ca, b, ldb, cb, out, ldo);
    DG_LAUNCHED("channel_concat");
    return DG_OK;
}

int dg_stage_pair(int64_t npix, int C, const float *x, const float *y, float *cat, int ldcat, float *catx, int ldcatx,
                  float *gx, float *gy, dg_stream_t stream) {
    DG_ARG(x && y && cat, "NULL tensor");
    DG_ARG(C >= 1 && C <= 4, "1 to 4 channels");
    DG_ARG(ldcat >= 2 * C && (!catx || ldcatx >= C), "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_stage_pair, dim3(dg::grid_for(npix)), dim3(256), 0, (hipStream_t)stream, (long)npix, C, x,
                       y, cat, ldcat, catx, ldcatx, gx, gy);
    DG_LAUNCHED("stage_pair");
    return DG_OK;
}

int dg_strided_copy(int64_t npix, int C, const float *src, int lds, float *dst, int ldd, dg_stream_t stream) {
    DG_ARG(src && dst, "NULL tensor");
    DG_ARG(lds >= C && ldd >= C, "bad strides");
    long total = (long)npix * C;
    if (total == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_strided_copy, dim3(dg::grid_for(C <= 4 ? (long)npix : total)), dim3(256), 0, (hipStream_t)stream, (long)npix, C,
                       src, lds, dst, ldd);
    DG_LAUNCHED("strided_copy");
    return DG_OK;
}

int dg_to_f16(int64_t n, const float *src, void *dst, dg_stream_t stream) {
    DG_ARG((src && dst) || n == 0, "NULL tensor");
    DG_ARG(n % 8 == 0 && (((uintptr_t)src) & 15) == 0 && (((uintptr_t)dst) & 15) == 0,
           "n %% 8 == 0 and 16-byte aligned buffers");
    if (n == 0) return DG_OK;
    // rows of 8 elements: the operand conversion pass of the fp16 GEMMs, RNE
    dg::launch_split_f16(src, 8, (long)(n / 8), 8, dst, (hipStream_t)stream);
    DG_LAUNCHED("to_f16");
    return DG_OK;
}

int dg_fill(float *p, int64_t n, float value, dg_stream_t stream) {
    DG_ARG(p || n == 0, "NULL tensor");
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_fill, dim3(dg::grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, (long)n, value);
    DG_LAUNCHED("fill");
    return DG_OK;
}

}  // extern "C"
