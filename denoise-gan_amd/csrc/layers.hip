// Layer kernels of the SRGAN / FastSRGAN / Autoencoder generators and
// discriminators and of the frozen VGG19 feature extractor (content loss):
//
//   PReLU(shared_axes=[1,2]) with an optional tf.nn.depth_to_space(., 2)
//       in front of it                      srgan.py:137-139, :152, fsrgan.py:197-199, :207
//   residual Add                             srgan.py:165, :170; fsrgan.py:187, :212
//   DepthwiseConv2D(3, s1, 'same', bias)     fsrgan.py:162-167
//   MaxPool2D(2, 2)                          autoencoder.py:111-115 (and VGG19's block pools)
//   UpSampling2D(2, 'nearest') + ReLU        autoencoder.py:117-131
//   vgg19.preprocess_input((x+1)*255/2)      srgan.py:71-73, fsrgan.py:74-76, pix2pix.py:45-51
//   content MSE on VGG features / 12.75      srgan.py:74-76
//   the SR-GAN loss set (adv / mae / mse / tv / disc) with gradients
//                                            train_srgan.py:84-96, train_fsrgan.py:86-96,
//                                            train_autoencoder.py:84-100
//
// Every activation is NHWC fp32 with an explicit pixel stride.  All
// per-channel reductions are deterministic: fixed row chunks -> per-chunk
// partials -> an ordered final sum.  Input-gradient outputs take `beta`
// (dx = new + beta * dx) so a tensor with several consumers accumulates its
// gradient in place.
#include "common.h"
#include <cstring>
#include <initializer_list>
#include <algorithm>

namespace dg {

static unsigned lgrid(long n) { return (unsigned)std::max<long>(1, std::min<long>(dg_cdiv(n, 256), 16384)); }

// row chunking of the per-channel partial reductions: 64 channels x 4 row lanes per block
struct RedPlan {
    int R;      // row chunks (grid.y)
    long rows;  // rows per chunk
};
static RedPlan red_plan(long M) {
    RedPlan p;
    long r = std::min<long>(512, std::max<long>(1, (M + 255) / 256));
    p.rows = (M + r - 1) / r;
    p.R = (int)((M + p.rows - 1) / p.rows);
    return p;
}

// The depthwise filter gradient's ten outputs (9 taps, bias) in one launch:
// out_q[c] = sum over the R row chunks of part[r][q][c] (+ beta out_q[c]).
// Block (q, 16 channels): 16 row lanes sum rows r = lane, lane + 16, ... in
// order (eight loads in flight), then the lanes are added in lane order.
// (One thread per channel summing all R rows, one launch per output, took
// 121 us per launch, 7.3 ms of FastSRGAN's step.)
__global__ void __launch_bounds__(256) k_rows_final10(const float *part, int R, int C, float *dk, float *dbias,
                                                     float beta) {
    __shared__ float red[256];
    const int q = blockIdx.x;
    float *out = q < 9 ? dk + (size_t)q * C : dbias;
    if (!out) return;   // block-uniform
    const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c = blockIdx.y * 16 + cl;
    float s = 0.f;
    if (c < C) {
        const float *pp = part + (size_t)q * C + c;
        const long rs = 10L * C;
#pragma unroll 8
        for (int r = rl; r < R; r += 16) s += pp[(long)r * rs];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (rl == 0 && c < C) {
        float t = red[cl];
        for (int l = 1; l < 16; ++l) t += red[l * 16 + cl];
        out[c] = beta != 0.f ? t + beta * out[c] : t;
    }
}

// --------------------------------------------------------------------------
// PReLU with optional depth_to_space (block B).  Input y [N,H,W,C*B*B],
// output z [N,H*B,W*B,C]; TF depth_to_space (NHWC, DCR):
//   z[n, h*B+i, w*B+j, c] = y[n, h, w, (i*B + j)*C + c]
// PReLU = relu(x) - alpha*relu(-x)  (Keras): x>0 ? x : alpha[c]*x; its
// gradient is 1 / alpha / 0 for x >0 / <0 / ==0, d alpha = -relu(-x).
// --------------------------------------------------------------------------
// A/B switch: DG_PLAN_DISABLE containing "prelu4" keeps the one-channel kernels
static bool plan_off_prelu4() {
    static const bool off = [] {
        const char *l = getenv("DG_PLAN_DISABLE");
        return l && strstr(l, "prelu4");
    }();
    return off;
}

struct ShufGeom {
    int H, W, C, B;
};
__device__ __forceinline__ long shuf_out_pix(long pix, int ch, const ShufGeom &g, int &c) {
    const int q = ch / g.C;
    c = ch - q * g.C;
    const int i = q / g.B, j = q - i * g.B;
    const long hw = (long)g.H * g.W;
    const long n = pix / hw;
    const int r = (int)(pix - n * hw);
    const int h = r / g.W, w = r - h * g.W;
    return (n * g.H * g.B + (long)h * g.B + i) * ((long)g.W * g.B) + (long)w * g.B + j;
}

// float4 path: C % 4 == 0, every row stride % 4 == 0 and every base 16-byte aligned
static bool prelu_v4(int C, std::initializer_list<std::pair<const void *, int>> ts) {
    if (C % 4) return false;
    for (const auto &t : ts)
        if ((t.second % 4) || (((uintptr_t)t.first) & 15)) return false;
    return !plan_off_prelu4();
}

// zh: the consuming fp16 conv's operand copy of z ([output pixels][C]), or NULL
__global__ void __launch_bounds__(256) k_prelu_fwd(long npix, ShufGeom g, const float *__restrict__ y, int ldy,
                                                  const float *__restrict__ alpha, float *__restrict__ z, int ldz,
                                                  _Float16 *__restrict__ zh) {
    const int CB = g.C * g.B * g.B;
    const long total = npix * CB;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long pix = e / CB;
        const int ch = (int)(e - pix * CB);
        int c;
        const long op = shuf_out_pix(pix, ch, g, c);
        const float v = y[pix * ldy + ch];
        const float o = v > 0.f ? v : alpha[c] * v;
        z[op * ldz + c] = o;
        if (zh) zh[op * g.C + c] = (_Float16)o;
    }
}

// four channels per thread (C % 4 == 0, float4-aligned rows): the four share one
// depth_to_space sub-position, so their z elements are adjacent too
__global__ void __launch_bounds__(256) k_prelu_fwd4(long npix, ShufGeom g, const float *__restrict__ y, int ldy,
                                                   const float *__restrict__ alpha, float *__restrict__ z, int ldz,
                                                   _Float16 *__restrict__ zh) {
    const int CB4 = g.C * g.B * g.B / 4;
    const long total = npix * CB4;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long pix = e / CB4;
        const int ch = (int)(e - pix * CB4) * 4;
        int c;
        const long op = shuf_out_pix(pix, ch, g, c);
        const f32x4 v = *reinterpret_cast<const f32x4 *>(y + pix * ldy + ch);
        const f32x4 a = *reinterpret_cast<const f32x4 *>(alpha + c);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = v[q] > 0.f ? v[q] : a[q] * v[q];
        *reinterpret_cast<f32x4 *>(z + op * ldz + c) = o;
        if (zh) store_f16x4(zh + op * g.C + c, o);
    }
}

// dy = dz * prelu'(y) (+beta*dy); partial d alpha sums over row chunks
__global__ void __launch_bounds__(256) k_prelu_bwd(long npix, ShufGeom g, const float *__restrict__ y, int ldy,
                                                  const float *__restrict__ alpha, const float *__restrict__ dz,
                                                  int lddz, float *__restrict__ dy, int lddy, float beta, long rows,
                                                  float *__restrict__ part, _Float16 *__restrict__ dyh) {
    const int CB = g.C * g.B * g.B;
    const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int ch = blockIdx.x * 64 + cl;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = std::min<long>(npix, r0 + rows);
    float acc = 0.f;
    int c = 0;
    if (ch < CB) {
        for (long pix = r0 + rl; pix < r1; pix += 4) {
            const long op = shuf_out_pix(pix, ch, g, c);
            const float v = y[pix * ldy + ch];
            const float gz = dz[op * lddz + c];
            const float d = v > 0.f ? gz : (v < 0.f ? alpha[c] * gz : 0.f);
            float *o = dy + pix * lddy + ch;
            const float r = beta != 0.f ? d + beta * *o : d;
            *o = r;
            if (dyh) dyh[pix * CB + ch] = (_Float16)r;   // the producing fp16 conv's dy copy
            acc += gz * fminf(v, 0.f);
        }
    }
    __shared__ float red[4][64];
    red[rl][cl] = acc;
    __syncthreads();
    if (rl == 0 && ch < CB) {
        float s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
        part[(long)blockIdx.y * CB + ch] = s;  // per input channel; folded over the B*B sub-positions below
    }
}

// four channels per thread, 16 channel quads x 16 row lanes per block (sixteen rows'
// loads in flight per channel quad); the row lanes' sums are added in lane order
__global__ void __launch_bounds__(256) k_prelu_bwd4(long npix, ShufGeom g, const float *__restrict__ y, int ldy,
                                                   const float *__restrict__ alpha, const float *__restrict__ dz,
                                                   int lddz, float *__restrict__ dy, int lddy, float beta, long rows,
                                                   float *__restrict__ part, _Float16 *__restrict__ dyh) {
    const int CB = g.C * g.B * g.B;
    const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int ch = (blockIdx.x * 16 + cl) * 4;
    const long r0 = (long)blockIdx.y * rows;
    const long r1 = std::min<long>(npix, r0 + rows);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (ch < CB) {
        int c = 0;
        shuf_out_pix(r0, ch, g, c);
        const f32x4 a = *reinterpret_cast<const f32x4 *>(alpha + c);
        for (long pix = r0 + rl; pix < r1; pix += 16) {
            int cc;
            const long op = shuf_out_pix(pix, ch, g, cc);
            const f32x4 v = *reinterpret_cast<const f32x4 *>(y + pix * ldy + ch);
            const f32x4 gz = *reinterpret_cast<const f32x4 *>(dz + op * lddz + c);
            float *o = dy + pix * lddy + ch;
            f32x4 r;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                r[q] = v[q] > 0.f ? gz[q] : (v[q] < 0.f ? a[q] * gz[q] : 0.f);
                acc[q] += gz[q] * fminf(v[q], 0.f);
            }
            if (beta != 0.f) r += beta * *reinterpret_cast<const f32x4 *>(o);
            *reinterpret_cast<f32x4 *>(o) = r;
            if (dyh) store_f16x4(dyh + pix * CB + ch, r);   // the producing fp16 conv's dy copy
        }
    }
    __shared__ f32x4 red[16][16];
    red[rl][cl] = acc;
    __syncthreads();
    if (rl == 0 && ch < CB) {
        f32x4 sum = red[0][cl];
        for (int l = 1; l < 16; ++l) sum += red[l][cl];
        *reinterpret_cast<f32x4 *>(part + (long)blockIdx.y * CB + ch) = sum;
    }
}

// d alpha[c] = sum_r sum_q part[r][q*C + c]  (+ beta * dalpha).  Block = 16 channels x
// 16 row lanes: lane rl sums rows r = rl, rl + 16, ... (the B*B sub-positions of a row
// together, eight rows' loads in flight), then the lanes are added in lane order.
// (One thread per channel summing all R*BB partials serially: 357 us per call in
// FastSRGAN, one block for its 32 channels.)
__global__ void __launch_bounds__(256) k_prelu_alpha_final(const float *part, int R, int C, int BB, float *dalpha,
                                                          float beta) {
    __shared__ float red[256];
    const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + cl;
    float s = 0.f;
    if (c < C) {
        const long rs = (long)C * BB;
#pragma unroll 8
        for (int r = rl; r < R; r += 16) {
            const float *pp = part + (long)r * rs + c;
            float t = pp[0];
            for (int q = 1; q < BB; ++q) t += pp[q * C];
            s += t;
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (rl == 0 && c < C) {
        float t = red[cl];
        for (int l = 1; l < 16; ++l) t += red[l * 16 + cl];
        dalpha[c] = beta != 0.f ? t + beta * dalpha[c] : t;
    }
}

// --------------------------------------------------------------------------
// elementwise helpers
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_add(long npix, int C, const float *a, int lda, const float *b, int ldb,
                                            float *out, int ldo, _Float16 *__restrict__ outh) {
    const long total = npix * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / C;
        const int c = (int)(e - p * C);
        const float o = a[p * lda + c] + b[p * ldb + c];
        out[p * ldo + c] = o;
        if (outh) outh[p * C + c] = (_Float16)o;   // the consuming fp16 conv's operand copy
    }
}

__global__ void __launch_bounds__(256) k_accumulate(long npix, int C, const float *src, int lds, float *dst, int ldd,
                                                   float beta) {
    const long total = npix * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / C;
        const int c = (int)(e - p * C);
        float *o = dst + p * ldd + c;
        const float v = src[p * lds + c];
        *o = beta != 0.f ? v + beta * *o : v;
    }
}

__global__ void __launch_bounds__(256) k_act_fwd(long npix, int C, const float *x, int ldx, int act, float alpha,
                                                float *z, int ldz) {
    const long total = npix * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / C;
        const int c = (int)(e - p * C);
        z[p * ldz + c] = act_fwd(x[p * ldx + c], act, alpha);
    }
}

// --------------------------------------------------------------------------
// MaxPool2D(2, strides 2, 'valid' == 'same' for even sizes).  Ho = H/2.
// The gradient goes to the first maximum of each window in row-major order
// (TF's MaxPoolGrad routes to the forward argmax).  Rows/cols beyond 2*Ho
// (odd sizes, 'valid') get zero gradient.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_maxpool_fwd(int N, int H, int W, int C, const float *x, int ldx, float *y,
                                                    int ldy) {
    const int Ho = H / 2, Wo = W / 2;
    const long total = (long)N * Ho * Wo * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long op = e / C;
        const int c = (int)(e - op * C);
        const int wo = (int)(op % Wo);
        const long t = op / Wo;
        const int ho = (int)(t % Ho);
        const long n = t / Ho;
        const long ip = (n * H + 2 * ho) * W + 2 * wo;
        const float a = x[ip * ldx + c], b = x[(ip + 1) * ldx + c];
        const float d = x[(ip + W) * ldx + c], f = x[(ip + W + 1) * ldx + c];
        y[op * ldy + c] = fmaxf(fmaxf(a, b), fmaxf(d, f));
    }
}

// one thread per (window, channel): the window's four input gradients; rows/cols past
// 2*Ho / 2*Wo (odd sizes) get their zero gradient from the tail pass below
__global__ void __launch_bounds__(256) k_maxpool_bwd(int N, int H, int W, int C, const float *x, int ldx,
                                                    const float *dy, int lddy, float *dx, int lddx, float beta,
                                                    int act, float alpha) {
    const int Ho = H / 2, Wo = W / 2;
    const long total = (long)N * Ho * Wo * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long op = e / C;
        const int c = (int)(e - op * C);
        const int wo = (int)(op % Wo);
        const long t = op / Wo;
        const int ho = (int)(t % Ho);
        const long n = t / Ho;
        const long p0 = (n * H + 2 * ho) * W + 2 * wo;
        const long pp[4] = {p0, p0 + 1, p0 + W, p0 + W + 1};
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = x[pp[q] * ldx + c];
        int am = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
            if (v[q] > v[am]) am = q;
        const float gy = dy[op * lddy + c];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float g = q == am ? gy * act_grad_from_out(v[q], act, alpha) : 0.f;
            float *o = dx + pp[q] * lddx + c;
            *o = beta != 0.f ? g + beta * *o : g;
        }
    }
}

// float4 over channels (C % 4 == 0, 16-byte rows): one thread per (window,
// 4 channels).  yp / dxp: optional bf16x6 planes of the output / input
// gradient (C % 16 == 0) for the conv that consumes it -- no split pass.
// (ypC: the planes' channel argument of store_planes4 -- C, or -C for fp16x3 planes)
// (fp16x3 planes: scaled from the source (sm, sg, sc) when given -- the producing conv's output
// source, a bound of the pooled values too -- else F16X3_XS)
__global__ void __launch_bounds__(256) k_maxpool_fwd4(int N, int H, int W, int C, const float *x, int ldx, float *y,
                                                     int ldy, unsigned short *yp, int ypC, const float *sm,
                                                     const float *sg, const float *sc) {
    const float xs = sm ? x3_grad_scale(sm, sg, sc) : F16X3_XS;
    const int Ho = H / 2, Wo = W / 2, C4 = C >> 2;
    const int total = N * Ho * Wo * C4;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int op = e / C4;
        const int c = (e - op * C4) * 4;
        const int wo = op % Wo, t = op / Wo, ho = t % Ho, n = t / Ho;
        const long ip = ((long)n * H + 2 * ho) * W + 2 * wo;
        const f32x4 a = *reinterpret_cast<const f32x4 *>(x + ip * ldx + c);
        const f32x4 b = *reinterpret_cast<const f32x4 *>(x + (ip + 1) * ldx + c);
        const f32x4 d = *reinterpret_cast<const f32x4 *>(x + (ip + W) * ldx + c);
        const f32x4 f = *reinterpret_cast<const f32x4 *>(x + (ip + W + 1) * ldx + c);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = fmaxf(fmaxf(a[q], b[q]), fmaxf(d[q], f[q]));
        *reinterpret_cast<f32x4 *>(y + (long)op * ldy + c) = o;
        if (yp) store_planes4(yp, ypC, op, c, o, xs);
    }
}

__global__ void __launch_bounds__(256) k_maxpool_bwd4(int N, int H, int W, int C, const float *x, int ldx,
                                                     const float *dy, int lddy, float *dx, int lddx, float beta,
                                                     int act, float alpha, unsigned short *dxp) {
    const int Ho = H / 2, Wo = W / 2, C4 = C >> 2;
    const int total = N * Ho * Wo * C4;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int op = e / C4;
        const int c = (e - op * C4) * 4;
        const int wo = op % Wo, t = op / Wo, ho = t % Ho, n = t / Ho;
        const long p0 = ((long)n * H + 2 * ho) * W + 2 * wo;
        const long pp[4] = {p0, p0 + 1, p0 + W, p0 + W + 1};
        f32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const f32x4 *>(x + pp[q] * ldx + c);
        const f32x4 gy = *reinterpret_cast<const f32x4 *>(dy + (long)op * lddy + c);
        int am[4] = {0, 0, 0, 0};  // first maximum per channel
#pragma unroll
        for (int q = 1; q < 4; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (v[q][k] > v[am[k]][k]) am[k] = q;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 g;
#pragma unroll
            for (int k = 0; k < 4; ++k) g[k] = am[k] == q ? gy[k] * act_grad_from_out(v[q][k], act, alpha) : 0.f;
            f32x4 *o = reinterpret_cast<f32x4 *>(dx + pp[q] * lddx + c);
            if (beta != 0.f) g += beta * *o;
            *o = g;
            if (dxp) store_planes4(dxp, C, pp[q], c, g);
        }
    }
}

// backward of a max pool fused into its conv's forward (dg_conv_fwd_pool): the
// window position and the sign of the pooled value were stored as one byte per
// element, so the full-size activation is not read.  The routed gradient is
// dy * act'(pooled) at the first maximum, 0 at the other three positions.
// dx (fp32) may be NULL when only its planes are consumed (a conv's backward
// on bf16x6 planes).
// (dxpC: C, or -C for the fp16x3 dy planes of an fp16x3 input gradient, scaled from (sm, sg))
__global__ void __launch_bounds__(256) k_maxpool_bwd_idx4(int N, int H, int W, int C, const unsigned char *idx,
                                                         const float *dy, int lddy, float *dx, int lddx, float beta,
                                                         float neg, unsigned short *dxp, int dxpC, const float *sm,
                                                         const float *sg) {
    const float xs = sm ? x3_grad_scale(sm, sg) : F16X3_XS;
    const int Ho = H / 2, Wo = W / 2, C4 = C >> 2;
    const int total = N * Ho * Wo * C4;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int op = e / C4;
        const int c = (e - op * C4) * 4;
        const int wo = op % Wo, t = op / Wo, ho = t % Ho, n = t / Ho;
        const long p0 = ((long)n * H + 2 * ho) * W + 2 * wo;
        const long pp[4] = {p0, p0 + 1, p0 + W, p0 + W + 1};
        const unsigned b = *reinterpret_cast<const unsigned *>(idx + (long)op * C + c);
        const f32x4 gy = *reinterpret_cast<const f32x4 *>(dy + (long)op * lddy + c);
        f32x4 gg;
#pragma unroll
        for (int k = 0; k < 4; ++k) gg[k] = gy[k] * (((b >> (8 * k)) & 4u) ? 1.f : neg);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 g;
#pragma unroll
            for (int k = 0; k < 4; ++k) g[k] = ((b >> (8 * k)) & 3u) == (unsigned)q ? gg[k] : 0.f;
            if (dx) {
                f32x4 *o = reinterpret_cast<f32x4 *>(dx + pp[q] * lddx + c);
                if (beta != 0.f) g += beta * *o;
                *o = g;
            }
            if (dxp) store_planes4(dxp, dxpC, pp[q], c, g, xs);
        }
    }
}

__global__ void __launch_bounds__(256) k_maxpool_bwd_tail(int N, int H, int W, int C, float *dx, int lddx,
                                                         float beta, unsigned short *dxp) {
    const int H2 = H / 2 * 2, W2 = W / 2 * 2;
    const long total = (long)N * H * W * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long ip = e / C;
        const int c = (int)(e - ip * C);
        const int w = (int)(ip % W);
        const int h = (int)((ip / W) % H);
        if (h < H2 && w < W2) continue;
        float *o = dx + ip * lddx + c;
        *o = beta != 0.f ? beta * *o : 0.f;
        if (dxp) store_planes1(dxp, C, ip, c, *o);
    }
}

// --------------------------------------------------------------------------
// UpSampling2D(2, nearest) followed by ReLU (autoencoder.py:117-131: the
// unpool's relu commutes with the replication).  x [N,H,W,C] -> z [N,2H,2W,C].
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_upsample_relu_fwd(int N, int H, int W, int C, const float *x, int ldx,
                                                          float *z, int ldz) {
    const int Ho = 2 * H, Wo = 2 * W;
    const long total = (long)N * Ho * Wo * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long op = e / C;
        const int c = (int)(e - op * C);
        const int wo = (int)(op % Wo);
        const long t = op / Wo;
        const int ho = (int)(t % Ho);
        const long n = t / Ho;
        const float v = x[((n * H + (ho >> 1)) * W + (wo >> 1)) * ldx + c];
        z[op * ldz + c] = v > 0.f ? v : 0.f;
    }
}

__global__ void __launch_bounds__(256) k_upsample_relu_bwd(int N, int H, int W, int C, const float *x, int ldx,
                                                          const float *dz, int lddz, float *dx, int lddx, float beta) {
    const int Wo = 2 * W;
    const long total = (long)N * H * W * C;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long ip = e / C;
        const int c = (int)(e - ip * C);
        const int w = (int)(ip % W);
        const long t = ip / W;
        const int h = (int)(t % H);
        const long n = t / H;
        float g = 0.f;
        if (x[ip * ldx + c] > 0.f) {
            const long o0 = (n * 2 * H + 2 * h) * (long)Wo + 2 * w;
            g = (dz[o0 * lddz + c] + dz[(o0 + 1) * lddz + c]) + (dz[(o0 + Wo) * lddz + c] + dz[(o0 + Wo + 1) * lddz + c]);
        }
        float *o = dx + ip * lddx + c;
        *o = beta != 0.f ? g + beta * *o : g;
    }
}

// --------------------------------------------------------------------------
// DepthwiseConv2D(3x3, stride 1, 'same' (pad 1/1), depth_multiplier 1, bias)
// kernel k[i][j][c] (Keras [3,3,C,1]).
//   y[n,h,w,c] = b[c] + sum_ij x[n,h+i-1,w+j-1,c] k[i,j,c]
// --------------------------------------------------------------------------
struct DwPlan {
    int RB, nrc, R;   // rows per chunk, row chunks per image, partial rows
};
static DwPlan dw_plan(int N, int H, int W, int C) {
    DwPlan p;
    const long cols = (long)dg_cdiv(C, 64) * dg_cdiv(W, 4) * N;
    int nrc = (int)std::max<long>(1, std::min<long>(H, dg_cdiv(2048, cols)));   // >= 2048 blocks
    p.RB = dg_cdiv(H, nrc);
    p.nrc = dg_cdiv(H, p.RB);
    p.R = N * p.nrc * dg_cdiv(W, 4);
    return p;
}

// Forward and input gradient: block (64 channels, 4 image columns, one image and a chunk
// of RB rows, the geometry of k_dw_bwd_filter below); wave v walks column w down the rows
// with the 3x3 input window in registers (three new loads per output, no index divisions).
// The taps are summed in the (i, j) order of the direct formula, padding taps as x * 0.
// (Thread per (pixel, channel) with nine loads and a div/mod chain per output: 184 /
// 165 us per call at FastSRGAN's 8 x 128 x 128 x 192, ~4.6x the HBM time.)
template <bool BWD>
__global__ void __launch_bounds__(256) k_dw_rows(int N, int H, int W, int C, const float *__restrict__ src, int lds,
                                                const float *__restrict__ k, const float *__restrict__ b,
                                                float *__restrict__ dst, int ldd, float beta, int RB, int nrc) {
    const int cl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int w = blockIdx.y * 4 + wv;
    if (c >= C || w >= W) return;
    const int n = blockIdx.z / nrc, rc = blockIdx.z - n * nrc;
    const int h0 = rc * RB, h1 = min(H, h0 + RB);
    float kk[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) kk[q] = k[q * C + c];
    const float bias = (!BWD && b) ? b[c] : 0.f;
    const bool okl = w > 0, okr = w + 1 < W;
    const float *sb = src + (long)n * H * W * lds + c;
    float *db = dst + (long)n * H * W * ldd + c;
    auto ld3 = [&](int h, float &v0, float &v1, float &v2) {
        const bool okh = h >= 0 && h < H;
        const float *r = sb + ((long)h * W + w) * lds;
        v0 = okh && okl ? r[-lds] : 0.f;
        v1 = okh ? r[0] : 0.f;
        v2 = okh && okr ? r[lds] : 0.f;
    };
    // window rows: u = row h-1, m = row h, d = row h+1 (columns w-1, w, w+1)
    float u0, u1, u2, m0, m1, m2;
    ld3(h0 - 1, u0, u1, u2);
    ld3(h0, m0, m1, m2);
    for (int h = h0; h < h1; ++h) {
        float d0, d1, d2;
        ld3(h + 1, d0, d1, d2);
        float s = 0.f;
        if (!BWD) {   // y[h][w] = sum_ij x[h+i-1][w+j-1] k[i][j]
            s = fmaf(u0, kk[0], s); s = fmaf(u1, kk[1], s); s = fmaf(u2, kk[2], s);
            s = fmaf(m0, kk[3], s); s = fmaf(m1, kk[4], s); s = fmaf(m2, kk[5], s);
            s = fmaf(d0, kk[6], s); s = fmaf(d1, kk[7], s); s = fmaf(d2, kk[8], s);
            db[((long)h * W + w) * ldd] = s + bias;
        } else {      // dx[h][w] = sum_ij dy[h-i+1][w-j+1] k[i][j]
            s = fmaf(d2, kk[0], s); s = fmaf(d1, kk[1], s); s = fmaf(d0, kk[2], s);
            s = fmaf(m2, kk[3], s); s = fmaf(m1, kk[4], s); s = fmaf(m0, kk[5], s);
            s = fmaf(u2, kk[6], s); s = fmaf(u1, kk[7], s); s = fmaf(u0, kk[8], s);
            float *o = db + ((long)h * W + w) * ldd;
            *o = beta != 0.f ? s + beta * *o : s;
        }
        u0 = m0; u1 = m1; u2 = m2;
        m0 = d0; m1 = d1; m2 = d2;
    }
}

// Filter gradient of the depthwise conv: partial sums of dk[i][j][c] (9 taps) and
// db[c] per block, part[r][10][C].  Block (64 channels, 4 image columns, one image and
// a chunk of RB rows): wave v walks column w down the rows, keeping the 3x3 window of x
// around (h, w) in registers -- per output pixel three new x loads (row h+1) and one dy
// load, 256 B per wave instruction, no index divisions -- and the four waves' sums are
// added in wave order.  (The row-chunk version -- one thread per (channel, pixel), nine
// x loads and a div/mod chain per pixel -- took 267 us per call at FastSRGAN's
// 8 x 128 x 128 x 192.)
__global__ void __launch_bounds__(256) k_dw_bwd_filter(int N, int H, int W, int C, const float *__restrict__ x,
                                                      int ldx, const float *__restrict__ dy, int lddy, int RB,
                                                      int nrc, float *__restrict__ part) {
    const int cl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int w = blockIdx.y * 4 + wv;
    const int n = blockIdx.z / nrc, rc = blockIdx.z - n * nrc;
    const int h0 = rc * RB, h1 = min(H, h0 + RB);
    float acc[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) acc[q] = 0.f;
    if (c < C && w < W) {
        const bool okl = w > 0, okr = w + 1 < W;
        const float *xb = x + (long)n * H * W * ldx + c;
        const float *gb = dy + (long)n * H * W * lddy + c;
        auto ldx3 = [&](int h, float &v0, float &v1, float &v2) {
            const bool okh = h >= 0 && h < H;
            const float *r = xb + ((long)h * W + w) * ldx;
            v0 = okh && okl ? r[-ldx] : 0.f;
            v1 = okh ? r[0] : 0.f;
            v2 = okh && okr ? r[ldx] : 0.f;
        };
        float a0, a1, a2, b0, b1, b2;
        ldx3(h0 - 1, a0, a1, a2);
        ldx3(h0, b0, b1, b2);
        for (int h = h0; h < h1; ++h) {
            float c0, c1, c2;
            ldx3(h + 1, c0, c1, c2);
            const float g = gb[((long)h * W + w) * lddy];
            acc[0] = fmaf(a0, g, acc[0]);
            acc[1] = fmaf(a1, g, acc[1]);
            acc[2] = fmaf(a2, g, acc[2]);
            acc[3] = fmaf(b0, g, acc[3]);
            acc[4] = fmaf(b1, g, acc[4]);
            acc[5] = fmaf(b2, g, acc[5]);
            acc[6] = fmaf(c0, g, acc[6]);
            acc[7] = fmaf(c1, g, acc[7]);
            acc[8] = fmaf(c2, g, acc[8]);
            acc[9] += g;
            a0 = b0; a1 = b1; a2 = b2;
            b0 = c0; b1 = c1; b2 = c2;
        }
    }
    __shared__ float red[4][10][64];
#pragma unroll
    for (int q = 0; q < 10; ++q) red[wv][q][cl] = acc[q];
    __syncthreads();
    if (c < C) {
        const long r = (long)blockIdx.z * gridDim.y + blockIdx.y;
        for (int q = wv; q < 10; q += 4) {
            const float s = red[0][q][cl] + red[1][q][cl] + red[2][q][cl] + red[3][q][cl];
            part[(r * 10 + q) * C + c] = s;
        }
    }
}

// --------------------------------------------------------------------------
// vgg19.preprocess_input (caffe mode) of (x + 1) * 255 / 2:
//   z[p, c'] = 127.5 * (x[p, 2 - c'] + 1) - mean[c'],  mean = (103.939, 116.779, 123.68) (BGR)
// ((x+1)*255)/2 and (x+1)*127.5 round identically in fp32: halving is exact.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_vgg_pre_fwd(long npix, const float *x, int ldx, float *z, int ldz) {
    const long total = npix * 3;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / 3;
        const int c = (int)(e - p * 3);
        const float mean = c == 0 ? 103.939f : (c == 1 ? 116.779f : 123.68f);
        z[p * ldz + c] = (x[p * ldx + (2 - c)] + 1.f) * 255.f / 2.f - mean;
    }
}

__global__ void __launch_bounds__(256) k_vgg_pre_bwd(long npix, const float *dz, int lddz, float *dx, int lddx,
                                                    float beta) {
    const long total = npix * 3;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / 3;
        const int c = (int)(e - p * 3);
        const float g = 127.5f * dz[p * lddz + (2 - c)];
        float *o = dx + p * lddx + c;
        *o = beta != 0.f ? g + beta * *o : g;
    }
}

// --------------------------------------------------------------------------
// scaled MSE: value = mean((s*a - s*b)^2) (Keras MeanSquaredError of
// features / 12.75); da = w * 2 s (s*a - s*b) / n.   Two-stage sum.
// --------------------------------------------------------------------------
constexpr int MSE_BLOCKS = 512;

__device__ __forceinline__ float block_sum256(float v, float *red) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) k_mse_partial(long npix, int C, const float *a, int lda, const float *b,
                                                    int ldb, float s, float wgrad, float inv_n, float *da, int ldda,
                                                    float *part) {
    __shared__ float red[4];
    const long total = npix * C;
    float acc = 0.f;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long p = e / C;
        const int c = (int)(e - p * C);
        const float d = a[p * lda + c] * s - b[p * ldb + c] * s;
        acc += d * d;
        if (da) da[p * ldda + c] = wgrad * 2.f * s * d * inv_n;
    }
    const float r = block_sum256(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
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

__global__ void __launch_bounds__(256) k_mse_final(const float *part, int nb, float inv_n, float *out) {
    __shared__ float sh[256];
    float v = 0.f;
    for (int i = threadIdx.x; i < nb; i += 256) v += part[i];
    const float s = tree_sum256(v, sh);
    if (threadIdx.x == 0) out[0] = s * inv_n;
}

// --------------------------------------------------------------------------
// SR-GAN loss set (train_srgan.py:84-96, train_fsrgan.py:86-96,
// train_autoencoder.py:84-100):
//   adv  = w_adv * BCE_logits(1, D(G(x)))         content = *content_value
//   mae  = mean|y - g|          mse = mean (y - g)^2
//   var  = w_var * mean_b total_variation(y - g)
//   disc = disc_scale * (BCE_logits(1, D(y)) + BCE_logits(0, D(G(x))))
//   gen_total = adv + t_mae*mae + t_mse*mse + t_content*content + t_var*var
// out[7] = {gen_total, adv, mae, mse, content, disc, var}; gradients of
// gen_total w.r.t. g (excluding the adv and content paths, which flow back
// through D and VGG) and of the two BCE sums w.r.t. the logits.
// --------------------------------------------------------------------------
struct GanLossArgs {
    int B, H, W, C;
    const float *gen; int ldgen;
    const float *tgt; int ldtgt;
    const float *zr; const float *zf; int nlog;
    float w_adv, w_var, disc_scale, t_mae, t_mse, t_content, t_var;
    const float *content;
    float *out;
    float *dgen; int lddgen;
    float *dzr_d, *dzf_d, *dzf_g;
    float *part_img;  // [LOSS_BLOCKS][3]
    float *part_log;  // [LOG_BLOCKS][3]
};
constexpr int GL_IMG_BLOCKS = 1024;
constexpr int GL_LOG_BLOCKS = 64;

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__device__ __forceinline__ float bce_logit(float z, float y) { return fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z))); }
__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + expf(-z)); }

__global__ void __launch_bounds__(256) k_ganloss_img(const GanLossArgs a) {
    __shared__ float red[4];
    const long npix = (long)a.B * a.H * a.W;
    const long total = npix * a.C;
    const float inv_n = 1.f / (float)total;
    const float tvs = a.t_var * a.w_var / (float)a.B;
    float s1 = 0.f, s2 = 0.f, stv = 0.f;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long pix = e / a.C;
        const int c = (int)(e - pix * a.C);
        const int w = (int)(pix % a.W);
        const int h = (int)((pix / a.W) % a.H);
        auto dv = [&](long px) { return a.tgt[px * a.ldtgt + c] - a.gen[px * a.ldgen + c]; };
        const float d = dv(pix);
        s1 += fabsf(d);
        s2 += d * d;
        float gtv = 0.f;
        if (h + 1 < a.H) { const float dd = dv(pix + a.W) - d; stv += fabsf(dd); gtv -= sgnf(dd); }
        if (w + 1 < a.W) { const float dd = dv(pix + 1) - d; stv += fabsf(dd); gtv -= sgnf(dd); }
        if (a.dgen) {
            if (h > 0) gtv += sgnf(d - dv(pix - a.W));
            if (w > 0) gtv += sgnf(d - dv(pix - 1));
            const float gd = a.t_mae * sgnf(d) * inv_n + a.t_mse * 2.f * d * inv_n + tvs * gtv;
            a.dgen[pix * a.lddgen + c] = -gd;  // d = y - g
        }
    }
    float r;
    r = block_sum256(s1, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 3 + 0] = r;
    r = block_sum256(s2, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 3 + 1] = r;
    r = block_sum256(stv, red); if (threadIdx.x == 0) a.part_img[blockIdx.x * 3 + 2] = r;
}

__global__ void __launch_bounds__(256) k_ganloss_logits(const GanLossArgs a) {
    __shared__ float red[4];
    const float inv_n = 1.f / (float)a.nlog;
    float r1 = 0.f, f0 = 0.f, f1 = 0.f;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < a.nlog; e += gridDim.x * blockDim.x) {
        const float zr = a.zr[e], zf = a.zf[e];
        r1 += bce_logit(zr, 1.f);
        f0 += bce_logit(zf, 0.f);
        f1 += bce_logit(zf, 1.f);
        if (a.dzr_d) a.dzr_d[e] = a.disc_scale * (sigm(zr) - 1.f) * inv_n;
        if (a.dzf_d) a.dzf_d[e] = a.disc_scale * sigm(zf) * inv_n;
        if (a.dzf_g) a.dzf_g[e] = a.w_adv * (sigm(zf) - 1.f) * inv_n;
    }
    float r;
    r = block_sum256(r1, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 0] = r;
    r = block_sum256(f0, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 1] = r;
    r = block_sum256(f1, red); if (threadIdx.x == 0) a.part_log[blockIdx.x * 3 + 2] = r;
}

__global__ void __launch_bounds__(256) k_ganloss_final(const GanLossArgs a) {
    __shared__ float sh[256];
    float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < GL_IMG_BLOCKS; b += 256)
        for (int q = 0; q < 3; ++q) v[q] += a.part_img[b * 3 + q];
    for (int b = threadIdx.x; b < GL_LOG_BLOCKS; b += 256)
        for (int q = 0; q < 3; ++q) v[3 + q] += a.part_log[b * 3 + q];
    float t[6];
    for (int q = 0; q < 6; ++q) t[q] = tree_sum256(v[q], sh);
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const float l1 = t[0], l2 = t[1], tv = t[2], r1 = t[3], f0 = t[4], f1 = t[5];
    const float n = (float)((long)a.B * a.H * a.W * a.C);
    const float nl = (float)a.nlog;
    const float adv = a.w_adv * (f1 / nl);
    const float mae = l1 / n, mse = l2 / n;
    const float var = a.w_var * (tv / (float)a.B);
    const float cont = a.content ? a.content[0] : 0.f;
    a.out[0] = adv + a.t_mae * mae + a.t_mse * mse + a.t_content * cont + a.t_var * var;
    a.out[1] = adv;
    a.out[2] = mae;
    a.out[3] = mse;
    a.out[4] = cont;
    a.out[5] = a.disc_scale * (r1 / nl + f0 / nl);
    a.out[6] = var;
}

}  // namespace dg

extern "C" {

int dg_prelu_workspace_size(int N, int H, int W, int C, int block, size_t *bytes) {
    DG_ARG(bytes, "NULL argument");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && (block == 1 || block == 2), "bad shape");
    dg::RedPlan rp = dg::red_plan((long)N * H * W);
    *bytes = (size_t)rp.R * C * block * block * sizeof(float) + 256;
    return DG_OK;
}

int dg_prelu_fwd(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha, float *z,
                 int ldz, dg_stream_t stream) {
    return dg_prelu_fwd_h(N, H, W, C, block, y, ldy, alpha, z, ldz, nullptr, stream);
}

int dg_prelu_fwd_h(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha, float *z,
                   int ldz, void *z_f16, dg_stream_t stream) {
    DG_ARG(y && alpha && z, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && (block == 1 || block == 2), "bad shape");
    DG_ARG(ldy >= C * block * block && ldz >= C, "bad strides");
    const long npix = (long)N * H * W;
    dg::ShufGeom g{H, W, C, block};
    if (dg::prelu_v4(C, {{y, ldy}, {z, ldz}, {alpha, 4}}) && (((uintptr_t)z_f16) & 7) == 0)
        hipLaunchKernelGGL(dg::k_prelu_fwd4, dim3(dg::lgrid(npix * C * block * block / 4)), dim3(256), 0,
                           (hipStream_t)stream, npix, g, y, ldy, alpha, z, ldz, (_Float16 *)z_f16);
    else
        hipLaunchKernelGGL(dg::k_prelu_fwd, dim3(dg::lgrid(npix * C * block * block)), dim3(256), 0,
                           (hipStream_t)stream, npix, g, y, ldy, alpha, z, ldz, (_Float16 *)z_f16);
    DG_LAUNCHED("prelu_fwd");
    return DG_OK;
}

int dg_prelu_bwd(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha, const float *dz,
                 int lddz, float *dy, int lddy, float beta, float *dalpha, float alpha_beta, void *ws,
                 size_t ws_bytes, dg_stream_t stream) {
    return dg_prelu_bwd_h(N, H, W, C, block, y, ldy, alpha, dz, lddz, dy, lddy, nullptr, beta, dalpha, alpha_beta, ws,
                          ws_bytes, stream);
}

int dg_prelu_bwd_h(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha,
                   const float *dz, int lddz, float *dy, int lddy, void *dy_f16, float beta, float *dalpha,
                   float alpha_beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(y && alpha && dz && dy && ws, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && (block == 1 || block == 2), "bad shape");
    DG_ARG(ldy >= C * block * block && lddy >= C * block * block && lddz >= C, "bad strides");
    size_t need;
    dg_prelu_workspace_size(N, H, W, C, block, &need);
    DG_ARG(ws_bytes >= need, "workspace too small");
    const long npix = (long)N * H * W;
    const int CB = C * block * block;
    dg::RedPlan rp = dg::red_plan(npix);
    dg::ShufGeom g{H, W, C, block};
    hipStream_t s = (hipStream_t)stream;
    if (dg::prelu_v4(C, {{y, ldy}, {dz, lddz}, {dy, lddy}, {alpha, 4}, {ws, 4}}) && (((uintptr_t)dy_f16) & 7) == 0)
        hipLaunchKernelGGL(dg::k_prelu_bwd4, dim3(dg_cdiv(CB, 64), rp.R), dim3(256), 0, s, npix, g, y, ldy, alpha, dz,
                           lddz, dy, lddy, beta, rp.rows, (float *)ws, (_Float16 *)dy_f16);
    else
        hipLaunchKernelGGL(dg::k_prelu_bwd, dim3(dg_cdiv(CB, 64), rp.R), dim3(256), 0, s, npix, g, y, ldy, alpha, dz,
                           lddz, dy, lddy, beta, rp.rows, (float *)ws, (_Float16 *)dy_f16);
    DG_LAUNCHED("prelu_bwd");
    if (dalpha) {
        hipLaunchKernelGGL(dg::k_prelu_alpha_final, dim3(dg_cdiv(C, 16)), dim3(256), 0, s, (const float *)ws, rp.R, C,
                           block * block, dalpha, alpha_beta);
        DG_LAUNCHED("prelu_alpha_final");
    }
    return DG_OK;
}

int dg_add(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float *out, int ldo,
           dg_stream_t stream) {
    return dg_add_h(npix, C, a, lda, b, ldb, out, ldo, nullptr, stream);
}

int dg_add_h(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float *out, int ldo,
             void *out_f16, dg_stream_t stream) {
    DG_ARG(a && b && out, "NULL tensor");
    DG_ARG(C > 0 && lda >= C && ldb >= C && ldo >= C, "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_add, dim3(dg::lgrid(npix * C)), dim3(256), 0, (hipStream_t)stream, (long)npix, C, a, lda,
                       b, ldb, out, ldo, (_Float16 *)out_f16);
    DG_LAUNCHED("add");
    return DG_OK;
}

int dg_accumulate(int64_t npix, int C, const float *src, int lds, float *dst, int ldd, float beta,
                  dg_stream_t stream) {
    DG_ARG(src && dst, "NULL tensor");
    DG_ARG(C > 0 && lds >= C && ldd >= C, "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_accumulate, dim3(dg::lgrid(npix * C)), dim3(256), 0, (hipStream_t)stream, (long)npix, C,
                       src, lds, dst, ldd, beta);
    DG_LAUNCHED("accumulate");
    return DG_OK;
}

int dg_act_fwd(int64_t npix, int C, const float *x, int ldx, int act, float alpha, float *z, int ldz,
               dg_stream_t stream) {
    DG_ARG(x && z, "NULL tensor");
    DG_ARG(C > 0 && ldx >= C && ldz >= C, "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_act_fwd, dim3(dg::lgrid(npix * C)), dim3(256), 0, (hipStream_t)stream, (long)npix, C, x,
                       ldx, act, alpha, z, ldz);
    DG_LAUNCHED("act_fwd");
    return DG_OK;
}

static bool pool_vec4(int C, const void *a, int lda, const void *b, int ldb, const void *c, int ldc) {
    return C % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 &&
           ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c)) & 15) == 0;
}

int dg_maxpool2_fwd_plf(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                        int y_planes_format, dg_stream_t stream) {
    return dg_maxpool2_fwd_x3(N, H, W, C, x, ldx, y, ldy, y_planes, y_planes_format, nullptr, nullptr, nullptr, stream);
}

int dg_maxpool2_fwd_x3(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                       int y_planes_format, const float *scale_m, const float *scale_g, const float *scale_c,
                       dg_stream_t stream) {
    DG_ARG(x && y, "NULL tensor");
    DG_ARG(scale_m || (!scale_g && !scale_c), "scale source: g / c without m");
    DG_ARG(N > 0 && H >= 2 && W >= 2 && C > 0 && ldx >= C && ldy >= C, "bad shape");
    DG_ARG(y_planes_format == DG_PLANES_BF16X6 || y_planes_format == DG_PLANES_F16X3, "bad plane format %d",
           y_planes_format);
    const long total = (long)N * (H / 2) * (W / 2) * C;
    DG_ARG(total < (1L << 31), "tensor too large");
    const bool v4 = pool_vec4(C, x, ldx, y, ldy, y, ldy);
    const int cm = y_planes_format == DG_PLANES_F16X3 ? 32 : 16;
    DG_ARG(!y_planes || (v4 && C % cm == 0 && (((uintptr_t)y_planes) & 15) == 0),
           "output planes need C %% %d == 0 and 16-byte aligned rows", cm);
    if (v4)
        hipLaunchKernelGGL(dg::k_maxpool_fwd4, dim3(dg::lgrid(total / 4)), dim3(256), 0, (hipStream_t)stream, N, H, W,
                           C, x, ldx, y, ldy, (unsigned short *)y_planes, y_planes_format == DG_PLANES_F16X3 ? -C : C,
                           scale_m, scale_g, scale_c);
    else
        hipLaunchKernelGGL(dg::k_maxpool_fwd, dim3(dg::lgrid(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C, x,
                           ldx, y, ldy);
    DG_LAUNCHED("maxpool_fwd");
    return DG_OK;
}

int dg_maxpool2_fwd_pl(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                       dg_stream_t stream) {
    return dg_maxpool2_fwd_plf(N, H, W, C, x, ldx, y, ldy, y_planes, DG_PLANES_BF16X6, stream);
}

int dg_maxpool2_fwd(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, dg_stream_t stream) {
    return dg_maxpool2_fwd_pl(N, H, W, C, x, ldx, y, ldy, nullptr, stream);
}

int dg_maxpool2_bwd_pl(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy, float *dx,
                       int lddx, float beta, int act, float alpha, void *dx_planes, dg_stream_t stream) {
    DG_ARG(x && dy && dx, "NULL tensor");
    DG_ARG(N > 0 && H >= 2 && W >= 2 && C > 0 && ldx >= C && lddy >= C && lddx >= C, "bad shape");
    DG_ARG(act >= DG_ACT_NONE && act <= DG_ACT_SIGMOID, "unknown activation %d", act);
    const long total = (long)N * (H / 2) * (W / 2) * C;
    DG_ARG((long)N * H * W * C < (1L << 31), "tensor too large");
    const bool v4 = pool_vec4(C, x, ldx, dy, lddy, dx, lddx);
    DG_ARG(!dx_planes || (v4 && C % 16 == 0 && (((uintptr_t)dx_planes) & 15) == 0),
           "gradient planes need C %% 16 == 0 and 16-byte aligned rows");
    unsigned short *dxp = (unsigned short *)dx_planes;
    if (v4)
        hipLaunchKernelGGL(dg::k_maxpool_bwd4, dim3(dg::lgrid(total / 4)), dim3(256), 0, (hipStream_t)stream, N, H, W,
                           C, x, ldx, dy, lddy, dx, lddx, beta, act, alpha, dxp);
    else
        hipLaunchKernelGGL(dg::k_maxpool_bwd, dim3(dg::lgrid(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C, x,
                           ldx, dy, lddy, dx, lddx, beta, act, alpha);
    DG_LAUNCHED("maxpool_bwd");
    if ((H & 1) || (W & 1)) {
        hipLaunchKernelGGL(dg::k_maxpool_bwd_tail, dim3(dg::lgrid((long)N * H * W * C)), dim3(256), 0,
                           (hipStream_t)stream, N, H, W, C, dx, lddx, beta, dxp);
        DG_LAUNCHED("maxpool_bwd_tail");
    }
    return DG_OK;
}

int dg_maxpool2_bwd(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy, float *dx,
                    int lddx, float beta, int act, float alpha, dg_stream_t stream) {
    return dg_maxpool2_bwd_pl(N, H, W, C, x, ldx, dy, lddy, dx, lddx, beta, act, alpha, nullptr, stream);
}

int dg_maxpool2_bwd_idx(int N, int H, int W, int C, const unsigned char *idx, const float *dy, int lddy,
                        float *dx, int lddx, float beta, int act, float alpha, void *dx_planes, dg_stream_t stream) {
    return dg_maxpool2_bwd_idx_x3(N, H, W, C, idx, dy, lddy, dx, lddx, beta, act, alpha, dx_planes, nullptr, nullptr,
                                  stream);
}

int dg_maxpool2_bwd_idx_x3(int N, int H, int W, int C, const unsigned char *idx, const float *dy, int lddy,
                           float *dx, int lddx, float beta, int act, float alpha, void *dx_planes,
                           const float *scale_m, const float *scale_g, dg_stream_t stream) {
    DG_ARG(idx && dy && (dx || dx_planes), "NULL tensor");
    DG_ARG(!scale_m || C % 32 == 0, "fp16x3 gradient planes need C %% 32 == 0");
    DG_ARG(N > 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0 && C > 0 && C % 16 == 0, "bad shape");
    DG_ARG(lddy >= C && lddy % 4 == 0 && (((uintptr_t)dy) & 15) == 0 && (((uintptr_t)idx) & 3) == 0,
           "dy needs a float4-aligned layout, idx 4-byte alignment");
    DG_ARG(!dx || (lddx >= C && lddx % 4 == 0 && (((uintptr_t)dx) & 15) == 0), "dx needs a float4-aligned layout");
    DG_ARG(dx || beta == 0.f, "accumulation (beta != 0) needs the fp32 dx");
    DG_ARG(!dx_planes || (((uintptr_t)dx_planes) & 15) == 0, "plane buffers must be 16-byte aligned");
    DG_ARG(act == DG_ACT_NONE || act == DG_ACT_RELU || act == DG_ACT_LRELU, "activation %d not sign-determined", act);
    DG_ARG((long)N * H * W * C < (1L << 31), "tensor too large");
    const float neg = act == DG_ACT_RELU ? 0.f : (act == DG_ACT_LRELU ? alpha : 1.f);
    const long total = (long)N * (H / 2) * (W / 2) * C;
    hipLaunchKernelGGL(dg::k_maxpool_bwd_idx4, dim3(dg::lgrid(total / 4)), dim3(256), 0, (hipStream_t)stream, N, H, W,
                       C, idx, dy, lddy, dx, lddx, beta, neg, (unsigned short *)dx_planes, scale_m ? -C : C, scale_m,
                       scale_g);
    DG_LAUNCHED("maxpool_bwd_idx");
    return DG_OK;
}

int dg_upsample2_relu_fwd(int N, int H, int W, int C, const float *x, int ldx, float *z, int ldz,
                          dg_stream_t stream) {
    DG_ARG(x && z, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && ldx >= C && ldz >= C, "bad shape");
    const long total = (long)N * 4 * H * W * C;
    hipLaunchKernelGGL(dg::k_upsample_relu_fwd, dim3(dg::lgrid(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C,
                       x, ldx, z, ldz);
    DG_LAUNCHED("upsample_relu_fwd");
    return DG_OK;
}

int dg_upsample2_relu_bwd(int N, int H, int W, int C, const float *x, int ldx, const float *dz, int lddz, float *dx,
                          int lddx, float beta, dg_stream_t stream) {
    DG_ARG(x && dz && dx, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && ldx >= C && lddz >= C && lddx >= C, "bad shape");
    const long total = (long)N * H * W * C;
    hipLaunchKernelGGL(dg::k_upsample_relu_bwd, dim3(dg::lgrid(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C,
                       x, ldx, dz, lddz, dx, lddx, beta);
    DG_LAUNCHED("upsample_relu_bwd");
    return DG_OK;
}

int dg_dwconv3_workspace_size(int N, int H, int W, int C, size_t *bytes) {
    DG_ARG(bytes, "NULL argument");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0, "bad shape");
    const dg::DwPlan dp = dg::dw_plan(N, H, W, C);
    *bytes = (size_t)dp.R * 10 * C * sizeof(float) + 256;
    return DG_OK;
}

int dg_dwconv3_fwd(int N, int H, int W, int C, const float *x, int ldx, const float *k, const float *bias, float *y,
                   int ldy, dg_stream_t stream) {
    DG_ARG(x && k && y, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && ldx >= C && ldy >= C, "bad shape");
    const dg::DwPlan dp = dg::dw_plan(N, H, W, C);
    hipLaunchKernelGGL(dg::k_dw_rows<false>, dim3(dg_cdiv(C, 64), dg_cdiv(W, 4), N * dp.nrc), dim3(256), 0,
                       (hipStream_t)stream, N, H, W, C, x, ldx, k, bias, y, ldy, 0.f, dp.RB, dp.nrc);
    DG_LAUNCHED("dwconv_fwd");
    return DG_OK;
}

int dg_dwconv3_bwd_data(int N, int H, int W, int C, const float *dy, int lddy, const float *k, float *dx, int lddx,
                        float beta, dg_stream_t stream) {
    DG_ARG(dy && k && dx, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && lddy >= C && lddx >= C, "bad shape");
    const dg::DwPlan dp = dg::dw_plan(N, H, W, C);
    hipLaunchKernelGGL(dg::k_dw_rows<true>, dim3(dg_cdiv(C, 64), dg_cdiv(W, 4), N * dp.nrc), dim3(256), 0,
                       (hipStream_t)stream, N, H, W, C, dy, lddy, k, (const float *)nullptr, dx, lddx, beta, dp.RB,
                       dp.nrc);
    DG_LAUNCHED("dwconv_bwd_data");
    return DG_OK;
}

int dg_dwconv3_bwd_filter(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy, float *dk,
                          float *dbias, float beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(x && dy && dk && ws, "NULL tensor");
    DG_ARG(N > 0 && H > 0 && W > 0 && C > 0 && ldx >= C && lddy >= C, "bad shape");
    size_t need;
    dg_dwconv3_workspace_size(N, H, W, C, &need);
    DG_ARG(ws_bytes >= need, "workspace too small");
    const dg::DwPlan dp = dg::dw_plan(N, H, W, C);
    hipStream_t s = (hipStream_t)stream;
    float *part = (float *)ws;
    hipLaunchKernelGGL(dg::k_dw_bwd_filter, dim3(dg_cdiv(C, 64), dg_cdiv(W, 4), N * dp.nrc), dim3(256), 0, s, N, H, W,
                       C, x, ldx, dy, lddy, dp.RB, dp.nrc, part);
    DG_LAUNCHED("dwconv_bwd_filter");
    // dk[q][c] (q = tap i*3+j) and dbias[c] (q = 9): ordered sums over the blocks' partials
    hipLaunchKernelGGL(dg::k_rows_final10, dim3(10, dg_cdiv(C, 16)), dim3(256), 0, s, (const float *)part, dp.R, C, dk,
                       dbias, beta);
    DG_LAUNCHED("dwconv_filter_final");
    return DG_OK;
}

int dg_vgg_preprocess_fwd(int64_t npix, const float *x, int ldx, float *z, int ldz, dg_stream_t stream) {
    DG_ARG(x && z, "NULL tensor");
    DG_ARG(ldx >= 3 && ldz >= 3, "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_vgg_pre_fwd, dim3(dg::lgrid(npix * 3)), dim3(256), 0, (hipStream_t)stream, (long)npix, x,
                       ldx, z, ldz);
    DG_LAUNCHED("vgg_preprocess_fwd");
    return DG_OK;
}

int dg_vgg_preprocess_bwd(int64_t npix, const float *dz, int lddz, float *dx, int lddx, float beta,
                          dg_stream_t stream) {
    DG_ARG(dz && dx, "NULL tensor");
    DG_ARG(lddz >= 3 && lddx >= 3, "bad strides");
    if (npix == 0) return DG_OK;
    hipLaunchKernelGGL(dg::k_vgg_pre_bwd, dim3(dg::lgrid(npix * 3)), dim3(256), 0, (hipStream_t)stream, (long)npix,
                       dz, lddz, dx, lddx, beta);
    DG_LAUNCHED("vgg_preprocess_bwd");
    return DG_OK;
}

int dg_mse_workspace_size(size_t *bytes) {
    DG_ARG(bytes, "NULL argument");
    *bytes = (size_t)dg::MSE_BLOCKS * sizeof(float) + 256;
    return DG_OK;
}

int dg_mse(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float scale, float *out,
           float *da, int ldda, float grad_weight, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(a && b && out && ws, "NULL tensor");
    DG_ARG(npix > 0 && C > 0 && lda >= C && ldb >= C && (!da || ldda >= C), "bad shape");
    DG_ARG(ws_bytes >= (size_t)dg::MSE_BLOCKS * sizeof(float), "workspace too small");
    const float inv_n = 1.f / (float)(npix * C);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(dg::k_mse_partial, dim3(dg::MSE_BLOCKS), dim3(256), 0, s, (long)npix, C, a, lda, b, ldb, scale,
                       grad_weight, inv_n, da, ldda, (float *)ws);
    DG_LAUNCHED("mse_partial");
    hipLaunchKernelGGL(dg::k_mse_final, dim3(1), dim3(256), 0, s, (const float *)ws, dg::MSE_BLOCKS, inv_n, out);
    DG_LAUNCHED("mse_final");
    return DG_OK;
}

int dg_gan_loss_workspace_size(size_t *bytes) {
    DG_ARG(bytes, "NULL argument");
    *bytes = (size_t)(dg::GL_IMG_BLOCKS * 3 + dg::GL_LOG_BLOCKS * 3 + 64) * sizeof(float);
    return DG_OK;
}

int dg_gan_loss(int B, int H, int W, int C, const float *gen, int ldgen, const float *tgt, int ldtgt,
                const float *logit_real, const float *logit_fake, int n_logits, const float *coef,
                const float *content_value, float *out, float *dgen, int lddgen, float *dlogit_real_d,
                float *dlogit_fake_d, float *dlogit_fake_g, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(gen && tgt && logit_real && logit_fake && coef && out && ws, "NULL tensor");
    DG_ARG(B > 0 && H > 0 && W > 0 && C > 0 && n_logits > 0, "bad shape");
    DG_ARG(ldgen >= C && ldtgt >= C && (!dgen || lddgen >= C), "bad strides");
    size_t need;
    dg_gan_loss_workspace_size(&need);
    DG_ARG(ws_bytes >= need, "workspace too small");
    dg::GanLossArgs a{};
    a.B = B; a.H = H; a.W = W; a.C = C;
    a.gen = gen; a.ldgen = ldgen; a.tgt = tgt; a.ldtgt = ldtgt;
    a.zr = logit_real; a.zf = logit_fake; a.nlog = n_logits;
    a.w_adv = coef[0]; a.w_var = coef[1]; a.disc_scale = coef[2];
    a.t_mae = coef[3]; a.t_mse = coef[4]; a.t_content = coef[5]; a.t_var = coef[6];
    a.content = content_value; a.out = out;
    a.dgen = dgen; a.lddgen = lddgen;
    a.dzr_d = dlogit_real_d; a.dzf_d = dlogit_fake_d; a.dzf_g = dlogit_fake_g;
    a.part_img = (float *)ws;
    a.part_log = a.part_img + dg::GL_IMG_BLOCKS * 3;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(dg::k_ganloss_img, dim3(dg::GL_IMG_BLOCKS), dim3(256), 0, s, a);
    DG_LAUNCHED("gan_loss_img");
    hipLaunchKernelGGL(dg::k_ganloss_logits, dim3(dg::GL_LOG_BLOCKS), dim3(256), 0, s, a);
    DG_LAUNCHED("gan_loss_logits");
    hipLaunchKernelGGL(dg::k_ganloss_final, dim3(1), dim3(256), 0, s, a);
    DG_LAUNCHED("gan_loss_final");
    return DG_OK;
}

}  // extern "C"
