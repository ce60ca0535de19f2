// pix2pix losses: values and gradients in three launches.
//
//   Pix2Pix.generator_loss (pix2pix.py:74-94):
//     gan      = w_gan * BCE_logits(1, D(x, G(x)))                      (:75)
//     var      = w_tv  * mean_b(total_variation(target - gen))           (:78)
//     l1       = w_l1  * mean|target - gen|                              (:81)
//     l2       = w_l2  * mean (target - gen)^2                           (:84)
//     content  = w_content * <VGG MSE, supplied by the caller>           (:87)
//     identity = w_id  * mean|G(target) - target|                        (:90)
//     total    = gan + l2 + content + var + l1 + identity                (:92)
//   Pix2Pix.discriminator_loss (:96-103): BCE(1, real) + BCE(0, fake).
//
// BCE with logits is TF's sigmoid_cross_entropy_with_logits
// max(z,0) - z*y + log1p(exp(-|z|)), averaged over every logit (Keras
// SUM_OVER_BATCH_SIZE).  total_variation is per image sum |dh| + |dw| over
// all channels (tf.image.total_variation).  d|x|/dx at 0 is 0 (tf.sign).
// Reductions are deterministic (fixed grid, ordered final sum).
#include "common.h"
#include <algorithm>

namespace dg {

constexpr int LOSS_IMG_BLOCKS = 1024;
constexpr int LOSS_LOGIT_BLOCKS = 64;

__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ float block_sum(float v, float *red) {
    // 256 threads: wave reduce then 4 partials
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

struct LossArgs {
    int B, H, W, C;
    const float *gen; int ldgen;
    const float *tgt; int ldtgt;
    const float *ident; int ldident;
    const float *zr; const float *zf; int nlog;
    float w_gan, w_l1, w_l2, w_tv, w_id, w_content;
    const float *content;
    float *out;
    float *dgen; int lddgen;
    float *dident; int lddident;
    float *dzr_d, *dzf_d, *dzf_g;
    float *part_img;    // [LOSS_IMG_BLOCKS][4]
    float *part_log;    // [LOSS_LOGIT_BLOCKS][3]
};

__global__ void __launch_bounds__(256) k_loss_img(const LossArgs a) {
    __shared__ float red[4];
    const long npix = (long)a.B * a.H * a.W;
    const long total = npix * a.C;
    const float inv_n = 1.f / (float)total;
    const float tv_scale = a.w_tv / (float)a.B;
    float s_l1 = 0.f, s_l2 = 0.f, s_tv = 0.f, s_id = 0.f;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long pix = e / a.C;
        const int c = (int)(e - pix * a.C);
        const int w = (int)(pix % a.W);
        const int h = (int)((pix / a.W) % a.H);
        auto dval = [&](long px) { return a.tgt[px * a.ldtgt + c] - a.gen[px * a.ldgen + c]; };
        const float d = dval(pix);
        s_l1 += fabsf(d);
        s_l2 += d * d;
        float gtv = 0.f;  // d TV / d d(pix)
        if (h + 1 < a.H) {
            float dd = dval(pix + a.W) - d;
            s_tv += fabsf(dd);
            gtv -= sgn(dd);
        }
        if (w + 1 < a.W) {
            float dd = dval(pix + 1) - d;
            s_tv += fabsf(dd);
            gtv -= sgn(dd);
        }
        if (h > 0) gtv += sgn(d - dval(pix - a.W));
        if (w > 0) gtv += sgn(d - dval(pix - 1));
        if (a.dgen) {
            // L = ... ; d = t - g  =>  dL/dg = -dL/dd
            float gd = a.w_l1 * sgn(d) * inv_n + a.w_l2 * 2.f * d * inv_n + tv_scale * gtv;
            a.dgen[pix * a.lddgen + c] = -gd;
        }
        if (a.ident) {
            float di = a.ident[pix * a.ldident + c] - a.tgt[pix * a.ldtgt + c];
            s_id += fabsf(di);
            if (a.dident) a.dident[pix * a.lddident + c] = a.w_id * sgn(di) * inv_n;
        }
    }
    float r;
    r = block_sum(s_l1, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 4 + 0] = r;
    r = block_sum(s_l2, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 4 + 1] = r;
    r = block_sum(s_tv, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 4 + 2] = r;
    r = block_sum(s_id, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 4 + 3] = r;
}

__device__ __forceinline__ float bce_logits(float z, float y) { return fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z))); }
__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + expf(-z)); }

__global__ void __launch_bounds__(256) k_loss_logits(const LossArgs a) {
    __shared__ float red[4];
    const float inv_n = 1.f / (float)a.nlog;
    float s_r1 = 0.f, s_f0 = 0.f, s_f1 = 0.f;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < a.nlog; e += gridDim.x * blockDim.x) {
        const float zr = a.zr[e], zf = a.zf[e];
        s_r1 += bce_logits(zr, 1.f);
        s_f0 += bce_logits(zf, 0.f);
        s_f1 += bce_logits(zf, 1.f);
        if (a.dzr_d) a.dzr_d[e] = (sigmoidf(zr) - 1.f) * inv_n;
        if (a.dzf_d) a.dzf_d[e] = sigmoidf(zf) * inv_n;
        if (a.dzf_g) a.dzf_g[e] = a.w_gan * (sigmoidf(zf) - 1.f) * inv_n;
    }
    float r;
    r = block_sum(s_r1, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 0] = r;
    r = block_sum(s_f0, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 1] = r;
    r = block_sum(s_f1, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 2] = r;
}

// fixed-order block sum over 256 threads (tree in LDS): deterministic
__device__ __forceinline__ float tree_sum256(float v, float *sh) {
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    const float r = sh[0];
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(256) k_loss_final(const LossArgs a, int nimg_blocks, int nlog_blocks) {
    __shared__ float sh[256];
    float v[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < nimg_blocks; b += 256)
        for (int q = 0; q < 4; ++q) v[q] += a.part_img[b * 4 + q];
    for (int b = threadIdx.x; b < nlog_blocks; b += 256)
        for (int q = 0; q < 3; ++q) v[4 + q] += a.part_log[b * 3 + q];
    float t[7];
    for (int q = 0; q < 7; ++q) t[q] = tree_sum256(v[q], sh);
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const float l1 = t[0], l2 = t[1], tv = t[2], id = t[3], r1 = t[4], f0 = t[5], f1 = t[6];
    const float n = (float)((long)a.B * a.H * a.W * a.C);
    const float nl = (float)a.nlog;
    const float gan = a.w_gan * f1 / nl;
    const float L1 = a.w_l1 * l1 / n;
    const float L2 = a.w_l2 * l2 / n;
    const float var = a.w_tv * tv / (float)a.B;
    const float ident = a.ident ? a.w_id * id / n : 0.f;
    const float cont = a.content ? a.w_content * a.content[0] : 0.f;
    const float disc = r1 / nl + f0 / nl;
    // tuple order of train_step (train_pix2pix.py:71)
    a.out[0] = gan + L2 + cont + var + L1 + ident;
    a.out[1] = gan;
    a.out[2] = L1;
    a.out[3] = L2;
    a.out[4] = cont;
    a.out[5] = disc;
    a.out[6] = var;
    a.out[7] = ident;
}

}  // namespace dg

extern "C" {

int dg_p2p_loss_workspace_size(int B, int H, int W, int C, int n_logits, size_t *bytes) {
    DG_ARG(bytes, "NULL argument");
    (void)B; (void)H; (void)W; (void)C; (void)n_logits;
    *bytes = (size_t)(dg::LOSS_IMG_BLOCKS * 4 + dg::LOSS_LOGIT_BLOCKS * 3 + 64) * sizeof(float);
    return DG_OK;
}

int dg_p2p_loss(int B, int H, int W, int C, const float *gen, int ldgen, const float *tgt, int ldtgt,
                const float *ident, int ldident, const float *logit_real, const float *logit_fake, int n_logits,
                const float *weights, const float *content_value, float *out, float *dgen, int lddgen, float *dident,
                int lddident, float *dlogit_real_d, float *dlogit_fake_d, float *dlogit_fake_g, void *ws,
                size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(gen && tgt && logit_real && logit_fake && weights && out && ws, "NULL tensor");
    DG_ARG(B > 0 && H > 0 && W > 0 && C > 0 && n_logits > 0, "bad shape");
    DG_ARG(ldgen >= C && ldtgt >= C && (!ident || ldident >= C), "bad strides");
    size_t need;
    dg_p2p_loss_workspace_size(B, H, W, C, n_logits, &need);
    DG_ARG(ws_bytes >= need, "workspace too small");
    dg::LossArgs a{};
    a.B = B; a.H = H; a.W = W; a.C = C;
    a.gen = gen; a.ldgen = ldgen; a.tgt = tgt; a.ldtgt = ldtgt; a.ident = ident; a.ldident = ldident;
    a.zr = logit_real; a.zf = logit_fake; a.nlog = n_logits;
    a.w_gan = weights[0]; a.w_l1 = weights[1]; a.w_l2 = weights[2]; a.w_tv = weights[3]; a.w_id = weights[4];
    a.w_content = weights[5];
    a.content = content_value; a.out = out;
    a.dgen = dgen; a.lddgen = lddgen; a.dident = dident; a.lddident = lddident;
    a.dzr_d = dlogit_real_d; a.dzf_d = dlogit_fake_d; a.dzf_g = dlogit_fake_g;
    a.part_img = (float *)ws;
    a.part_log = a.part_img + dg::LOSS_IMG_BLOCKS * 4;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(dg::k_loss_img, dim3(dg::LOSS_IMG_BLOCKS), dim3(256), 0, s, a);
    DG_LAUNCHED("loss_img");
    hipLaunchKernelGGL(dg::k_loss_logits, dim3(dg::LOSS_LOGIT_BLOCKS), dim3(256), 0, s, a);
    DG_LAUNCHED("loss_logits");
    hipLaunchKernelGGL(dg::k_loss_final, dim3(1), dim3(256), 0, s, a, dg::LOSS_IMG_BLOCKS, dg::LOSS_LOGIT_BLOCKS);
    DG_LAUNCHED("loss_final");
    return DG_OK;
}

}  // extern "C"
