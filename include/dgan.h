/*
 * dgan.h — C ABI of libdgan.so, the MI355X (gfx950) hot path of the
 * denoise-gan training step.
 *
 * The reference (pmcbride/denoise-gan) has no FFI: its hot path is the
 * tf.keras graph traced by `train_step` (train_pix2pix.py:33-71) and every
 * kernel below replaces a TensorFlow op that graph dispatches.  Each entry
 * point names the reference call site it stands in for.  Conventions:
 *
 *   - every tensor is caller-owned device memory, fp32, NHWC; activations
 *     carry an explicit pixel stride `ld*` (>= channels) so a layer can read
 *     or write one channel slice of a concatenated buffer in place
 *     (zero-copy skip concat, pix2pix.py:188 and :200);
 *   - weights keep the Keras layout: Conv2D HWIO [kh,kw,Cin,Cout]
 *     (pix2pix.py:115), Conv2DTranspose [kh,kw,Cout,Cin] (pix2pix.py:130);
 *   - the library never allocates on the hot path: scratch is queried with
 *     the *_workspace_size calls and handed in;
 *   - all work is enqueued on the caller's HIP stream (`dg_stream_t` is a
 *     hipStream_t); no call synchronises, so a whole step can be captured in
 *     a hipGraph;
 *   - every call returns DG_OK (0) or an error code; dg_last_error_string()
 *     explains the last failure of the calling thread.  No C++ exception
 *     crosses this boundary.
 */
#ifndef DGAN_H
#define DGAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *dg_stream_t;                 /* hipStream_t (NULL = legacy stream) */
typedef struct dg_conv_desc_s *dg_conv_t;  /* shapes immutable once created */

enum { DG_OK = 0, DG_ERR_ARG = 1, DG_ERR_HIP = 2, DG_ERR_WORKSPACE = 3, DG_ERR_UNSUPPORTED = 4 };

/* fused activations (Keras defaults: LeakyReLU alpha=0.3, pix2pix.py:121) */
enum { DG_ACT_NONE = 0, DG_ACT_LRELU = 1, DG_ACT_RELU = 2, DG_ACT_TANH = 3, DG_ACT_SIGMOID = 4 };

/* ops for dg_conv_workspace_size */
enum { DG_OP_FWD = 0, DG_OP_BWD_DATA = 1, DG_OP_BWD_FILTER = 2 };

const char *dg_last_error_string(void);
int dg_version(void);
/* "source_sha=<16 hex>;arch=gfx950;hip=<compiler>": the hash of the library sources
 * (csrc/*, include/dgan.h) this binary was compiled from -- provenance of a shipped .so */
const char *dg_build_info(void);
/* an empty kernel dispatch on `stream`: a mark in the dispatch sequence for profiling
 * (per-dispatch rocprofv3 PMC counters attributed to the calls between marks) */
int dg_mark(int id, dg_stream_t stream);
/* A measured max |value| (the fp16x3 scale sources below) is kept in a max slot of
 * DG_MAX_SLOT device floats: 8 per-workgroup shards of the producers' atomics, 32 floats (a
 * 128-byte line) apart, at slot[0], slot[32], ..., slot[224]; its value is their max and the
 * floats between them stay 0.  (Atomics to one line serialize: round 6 spread the shards.) */
#define DG_MAX_SLOT 256
int dg_max_slot_floats(void);

/* ------------------------------------------------------------------------
 * Convolution layers: Conv2D (pix2pix.py:115-116, :207-209, :217-218) and
 * Conv2DTranspose (pix2pix.py:130-133, :169-173).  Replaces TF's Conv2D,
 * Conv2DBackpropInput and Conv2DBackpropFilter kernels.
 *
 * Shapes are the LAYER's: input [N,H,W,Cin] -> output [N,Ho,Wo,Cout].
 * Padding is explicit (top/bottom/left/right) so TF 'same' asymmetry is
 * representable.  Conv2D:            Ho = (H + pt + pb - kh)/sh + 1.
 * Conv2DTranspose (transpose = 1):  Ho = (H - 1)*sh + kh - pt - pb, and the
 * pads are those of the equivalent forward conv (TF conv2d_backprop_input).
 * ---------------------------------------------------------------------- */
int dg_conv_desc_create(dg_conv_t *out, int N, int H, int W, int Cin, int Cout,
                        int kh, int kw, int sh, int sw,
                        int pad_t, int pad_b, int pad_l, int pad_r, int transpose);
int dg_conv_desc_destroy(dg_conv_t d);
int dg_conv_out_shape(dg_conv_t d, int *Ho, int *Wo);
int dg_conv_workspace_size(dg_conv_t d, int op, size_t *bytes);

/* Arithmetic of the conv GEMMs (TF runs them in fp32).
 *   DG_MATH_FP32   : v_mfma_f32_32x32x2_f32, exact fp32 FMA chains.
 *   DG_MATH_BF16X6 : each fp32 operand split exactly into bf16 hi+mid+lo, the
 *                    six piece products >= 2^-18 |ab| summed in the fp32 MFMA
 *                    accumulator (dropped terms < 2^-26 |ab|, below fp32
 *                    rounding) on the bf16 matrix cores, 2.7x the f32 MFMA rate.
 *   DG_MATH_FP16   : the reference's mixed_float16 policy (srgan.py:63-66,
 *                    train_srgan.py:312-318): both GEMM operands rounded to
 *                    fp16 (RNE), one v_mfma_f32_16x16x32_f16 per product,
 *                    fp32 accumulation and fp32 outputs; 6x the bf16x6 MFMA
 *                    rate.  Gradient operands need the caller's loss scale
 *                    (dg_loss_scale_*) to stay inside the fp16 range.
 *                    Eligible GEMMs: FWD Cin % 32 == 0, DGRAD Cout % 32 == 0,
 *                    WGRAD Cin, Cout % 16 == 0 (others keep fp32); no
 *                    caller-held planes (dg_conv_op_planes reports none).
 *   DG_MATH_F16X3  : fp16x3 wherever its kernels apply (the 3x3 stride-1 halo layers of the
 *                    frozen VGG19, pix2pix.py:53-67; every eligible pix2pix G / D GEMM,
 *                    pix2pix.py:110-142, :194-220), bf16x6 / fp32 tiles elsewhere: each fp32
 *                    operand, pre-scaled by a power of two s, is split into fp16 h + l (RNE,
 *                    |l| <= 2^-11 |s x|) and a product is h.h' + h.l' + l.h' -- three fp16 piece
 *                    products (dropped terms < 2^-21 |ab|) on three v_mfma_f32_16x16x32_f16 per
 *                    32 channels, half the bf16x6 MFMA count.  Scales: weights 2^8 (|w| < 255,
 *                    22 bits for |w| >= 2^-11); gradients and activations 2^(14 - e) from a
 *                    bound b < 2^e of the tensor (dg_conv_set_grad_scale, dg_conv_set_act_scale:
 *                    22 bits for every value >= 2^-17 b); an activation without a scale source
 *                    is measured by the op that splits it, or, in caller-held planes, keeps the
 *                    static 2^-4 (|x| < 2^20; 22 bits only for |x| >= 2).
 *                    A descriptor's x / dy planes are fp16x3 (4 B per element) when an fp16x3
 *                    op reads them, its w planes [fp16x3 | bf16x6] (dg_conv_planes_size).
 * New descriptors take $DG_CONV_MATH ("fp32" | "bf16x6" | "fp16" | "f16x3"; default bf16x6).
 * Changing the mode re-plans the descriptor: query workspace sizes after it. */
enum { DG_MATH_FP32 = 0, DG_MATH_BF16X6 = 1, DG_MATH_FP16 = 2, DG_MATH_F16X3 = 3 };
/* plane formats of dg_conv_planes_t buffers (dg_conv_planes_format) */
enum { DG_PLANES_BF16X6 = 0, DG_PLANES_F16X3 = 1 };
int dg_conv_set_math(dg_conv_t d, int math);
int dg_conv_get_math(dg_conv_t d, int *math);

/* y = act(conv(x, w) + bias) + beta * y            (bias may be NULL) */
int dg_conv_fwd(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias,
                float *y, int ldy, float beta, int act, float alpha,
                void *ws, size_t ws_bytes, dg_stream_t stream);
/* dx = dL/dx + beta * dx */
int dg_conv_bwd_data(dg_conv_t d, const float *dy, int lddy, const float *w,
                     float *dx, int lddx, float beta,
                     void *ws, size_t ws_bytes, dg_stream_t stream);
/* dx = (dL/dx) * act'(z) + beta * dx: the input gradient with the gradient of the
 * activation that PRODUCED the input (z = act(.), e.g. Conv2D(activation='relu')
 * feeding this conv, VGG19 / autoencoder.py:97-101) folded into the epilogue. */
int dg_conv_bwd_data_masked(dg_conv_t d, const float *dy, int lddy, const float *w,
                            float *dx, int lddx, float beta, const float *z, int ldz, int act, float alpha,
                            void *ws, size_t ws_bytes, dg_stream_t stream);
/* dw = dL/dw + beta * dw ; dbias = sum(dy) + beta * dbias  (dbias may be NULL) */
int dg_conv_bwd_filter(dg_conv_t d, const float *x, int ldx, const float *dy, int lddy,
                       float *dw, float *dbias, float beta,
                       void *ws, size_t ws_bytes, dg_stream_t stream);

/* Caller-held bf16x6 operand planes.  Under DG_MATH_BF16X6 every GEMM first
 * splits its two fp32 operands into bf16 hi/mid/lo planes (6 B per element);
 * the planes are a function of the tensor alone, so one split can serve every
 * op that reads the tensor: x by fwd and bwd_filter, dy by bwd_filter and
 * bwd_data, w by fwd and bwd_data.  A dg_conv_planes_t names a buffer
 * (dg_conv_planes_size bytes, 16-byte aligned) per tensor; an op that reads
 * a tensor as planes (dg_conv_op_planes) splits it into the given buffer, or,
 * when the tensor's bit is set in `ready`, reads the planes already there
 * without touching the fp32 tensor.  NULL buffers fall back to the workspace.
 * The caller owns validity: set a ready bit only after an op whose
 * dg_conv_op_planes mask holds that tensor has run on the same stream, and
 * clear it when the tensor changes.  Under DG_MATH_FP16 the same buffers hold
 * the tensor's fp16 copy ([rows][C], 2 B per element) that the fp16 GEMMs
 * read, converted once per tensor in the same way; `out` (producer-written
 * planes) is bf16x6-only. */
enum { DG_TENSOR_X = 1, DG_TENSOR_DY = 2, DG_TENSOR_W = 4 };
typedef struct dg_conv_planes {
    void *x, *dy, *w;  /* plane buffers (NULL: split into the workspace) */
    void *out;         /* if not NULL: the op also writes the planes of its output
                          (fwd: y, bwd_data: dx; channels % 16 == 0) -- the
                          consumer's x / dy planes, with no split pass */
    int ready;         /* DG_TENSOR_* bits whose buffer already holds the split */
    int out_format;    /* DG_PLANES_* of `out`: the consumer's x planes format (its
                          dg_conv_planes_format(DG_TENSOR_X)); DG_PLANES_F16X3 needs
                          channels % 32 == 0 (zero-initialised callers get bf16x6) */
} dg_conv_planes_t;
int dg_conv_planes_size(dg_conv_t d, int tensor, size_t *bytes);
/* DG_PLANES_F16X3 for the x / w planes of a descriptor whose forward runs fp16x3
 * (DG_MATH_F16X3), else DG_PLANES_BF16X6 */
int dg_conv_planes_format(dg_conv_t d, int tensor, int *format);
/* fp16x3 input gradients (DG_MATH_F16X3 bwd_data of a layer whose forward runs fp16x3;
 * VGG19's backward, pix2pix.py:45-51): a gradient has no static range, so its fp16x3 planes
 * are scaled by 2^(14 - e), bound = m * *g < 2^e (g NULL = 1) -- m a measured max |value|
 * kept in a max slot (DG_MAX_SLOT floats; m = the max of its shards), g a weight bound
 * max_ci sum_{taps, co} |w| -- which keeps every scaled value below 2^14.
 * dy_m / dy_g: the source of the dy planes' scale (the producer's: dx_m / dx_g of the
 * consuming layer, or dg_maxpool2_bwd_idx_x3's); NULL dy_m: bwd_data measures max |dy| of
 * its fp32 dy itself (dy planes must then not be ready).  dx_m / dx_g: the source of the
 * scale of the dx planes this op writes (planes->out with out_format DG_PLANES_F16X3),
 * normally (max |dy| of this layer, its weight bound).  dx_max: a max slot receiving max |dx|
 * by atomicMax (the caller zeroes them per step).  All device pointers, kept by the descriptor. */
int dg_conv_set_grad_scale(dg_conv_t d, const float *dy_m, const float *dy_g, const float *dx_m, const float *dx_g,
                           float *dx_max);
/* fp16x3 activation scale context (round 5).  An activation's fp16x3 planes are scaled by
 * 2^(14 - e) from a bound b = max(shards of m) * (g ? *g : 1) + (c ? *c : 0) < 2^e, like a gradient's,
 * so every |x| >= 2^-17 b keeps 22 bits (a static 2^-4 leaves |x| < 2 with a subnormal low piece).
 *   x_m / x_g / x_c: the source of the layer input's planes (the one their producer wrote them
 *     with: a BN forward's bound -- dg_bn_fwd_train_seg_x -- or a producing conv's output source
 *     below); a plain max slot (x_g, x_c NULL) is also measured into (max |x|) by any op of
 *     this descriptor that splits x itself.  NULL x_m: x planes in the workspace are measured per
 *     op; caller-held x planes keep the static 2^-4.
 *   y_m / y_g / y_c: the source of the output planes the forward writes for its consumer
 *     (planes->out, any arithmetic): normally (max |x| measured, max over output channels of
 *     sum |w| over taps and input channels, max |bias|) -- a bound of |y| after a ReLU /
 *     LeakyReLU / linear activation.  y_max: a max slot receiving max |y| of the forward (the
 *     16x16-tile, split-K reduce and small-Cin epilogues), the caller zeroes them.
 * All device pointers, kept by the descriptor. */
int dg_conv_set_act_scale(dg_conv_t d, const float *x_m, const float *x_g, const float *x_c, const float *y_m,
                          const float *y_g, const float *y_c, float *y_max);
/* max |x| over [rows][ld] (first C columns) into the max slot out by atomicMax (the caller
 * zeroes it): the measured max of a gradient entering an fp16x3 input
 * gradient from fp32 */
int dg_absmax(const float *x, int64_t rows, int C, int ld, float *out, dg_stream_t stream);
/* the same into the freshly zeroed max slot out (a measured max of one tensor) */
int dg_absmax_set(const float *x, int64_t rows, int C, int ld, float *out, dg_stream_t stream);
/* g_out[0] = max over output channels co of sum over k of |w[k][co]| (w as [K][Co]: an HWIO
 * kernel with K = kh*kw*Cin), c_out[0] (may be NULL) = max |bias| (0 for bias NULL): the
 * terms of a conv output's bound for dg_conv_set_act_scale (y_g, y_c).  zero8 (may be NULL):
 * a max slot zeroed on the way (the measured-max slot a following dg_absmax fills). */
int dg_weight_bound(const float *w, int64_t K, int Co, const float *bias, float *g_out, float *c_out,
                    float *zero8, dg_stream_t stream);
/* g_out[0] = max over input channels ci of sum over taps and output channels of |w[tap][ci][co]|
 * (an HWIO kernel, taps = kh*kw): the weight term of an fp16x3 input gradient's bound, |dx| <=
 * g_out[0] * max |dy| (dg_conv_set_grad_scale dx_g / dy_g of the graph executor's plans). */
int dg_weight_bound_in(const float *w, int taps, int Ci, int Co, float *g_out, dg_stream_t stream);
/* the arithmetic op's GEMM runs in (DG_MATH_*: fp32 for the exact direct kernels -- Co 1,
 * narrow, small-Cin -- and fp32 MFMA tiles; bf16x6, fp16 or fp16x3 for the split kernels):
 * per-op peaks for a roofline */
int dg_conv_op_arith(dg_conv_t d, int op, int *arith);
int dg_conv_op_planes(dg_conv_t d, int op, int *tensors);
int dg_conv_fwd_pl(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias,
                   float *y, int ldy, float beta, int act, float alpha,
                   const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream);
/* z == NULL: dg_conv_bwd_data; else dg_conv_bwd_data_masked */
int dg_conv_bwd_data_pl(dg_conv_t d, const float *dy, int lddy, const float *w,
                        float *dx, int lddx, float beta, const float *z, int ldz, int act, float alpha,
                        const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream);
int dg_conv_bwd_filter_pl(dg_conv_t d, const float *x, int ldx, const float *dy, int lddy,
                          float *dw, float *dbias, float beta,
                          const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_conv_bwd_data_pl masked by act'(x) taken from the sign of the hi plane of
 * x's bf16x6 planes (planes->x, ready: written by x's producer) instead of an
 * fp32 z, so a layer input that only exists as planes (a VGG19 conv -> conv
 * chain whose producer wrote no fp32 output: dg_conv_fwd_pl with y NULL) can
 * be masked (keras VGG19 ReLU, pix2pix.py:53-67).  act NONE / RELU / LRELU;
 * a positive fp32 value whose bf16 rounding underflows to 0 (|x| < 2^-133)
 * reads as <= 0.  dg_conv_fwd_pl accepts y == NULL when planes->out is set
 * and beta == 0: only the output's planes are written. */
int dg_conv_bwd_data_xmask(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx,
                           float beta, int act, float alpha, const dg_conv_planes_t *planes,
                           void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_conv_bwd_data_pl whose mask act'(z) multiplies the accumulated sum:
 * dx = act'(z) * (dL/dx + beta*dx) -- the last contribution of a gradient fan-in into an
 * activation without BN (the U-Net's down1 output reaches 'last' through the skip concat and
 * down2, pix2pix.py:115-121 / :180-190), so no separate act' pass over the summed gradient.
 * Split-precision plans only (DG_MATH_BF16X6 / F16X3 / FP16); others return DG_ERR_ARG. */
int dg_conv_bwd_data_masked_sum(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx,
                                float beta, const float *z, int ldz, int act, float alpha,
                                const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream);
/* Conv2D forward followed by MaxPool2D(2) on its activated output, fused into
 * the forward epilogue (VGG19 blockN_conv{2,4} -> blockN_pool, keras
 * applications VGG19 as built by pix2pix.py:53-67 / srgan.py:70-76; replaces
 * the conv + pool pair of dg_conv_fwd_pl + dg_maxpool2_fwd_pl).  Writes the
 * pooled output's bf16x6 planes (planes->out: the next conv's x planes) and/or
 * its fp32 values (pool_y, [N, Ho/2, Wo/2, Cout], may be NULL), and pool_idx
 * [N*Ho/2*Wo/2][Cout] bytes (bits 0-1: row-major window position of the first
 * maximum, bit 2: pooled value > 0) for dg_maxpool2_bwd_idx.  The conv's own
 * full-size output is not written.  DG_ERR_UNSUPPORTED unless
 * dg_conv_fwd_pool_ok: halo-tiled bf16x6 forward plan with one split,
 * Ho % 8 == 0, Wo % 16 == 0, act NONE / RELU / LRELU. */
int dg_conv_fwd_pool_ok(dg_conv_t d, int act, int *ok);
int dg_conv_fwd_pool(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias, int act, float alpha,
                     float *pool_y, int ldpy, unsigned char *pool_idx, const dg_conv_planes_t *planes,
                     void *ws, size_t ws_bytes, dg_stream_t stream);

/* ------------------------------------------------------------------------
 * BatchNormalization, training semantics of Keras' fused kernel
 * (pix2pix.py:119, :135, :211): batch statistics over the M = N*H*W rows,
 * biased variance for normalisation, moving stats updated with the
 * unbiased variance, eps 1e-3, momentum 0.99.  The activation that follows
 * in the reference block (LeakyReLU pix2pix.py:121/:213, Dropout+ReLU
 * :137-140) is fused into the apply pass.  Dropout uses a counter-based
 * hash keyed by (drop_seed, *step_dev, element) so results are reproducible
 * and restatable on the CPU; drop_rate 0 disables it.
 * ---------------------------------------------------------------------- */
int dg_bn_workspace_size(int M, int C, size_t *bytes);
int dg_bn_fwd_train(int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                    float *save_mean, float *save_invstd,
                    float *moving_mean, float *moving_var, float momentum, float eps,
                    float *z, int ldz, int act, float alpha,
                    float drop_rate, uint32_t drop_seed, const int32_t *step_dev,
                    void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_bn_fwd_train that also writes z's bf16x6 operand planes for up to two consuming
 * convs (zp0 / zp1, NULL = none): channel c of z lands at column col + c of a packed
 * [rows][3 * planesC] plane buffer (dg_conv_planes_t.x layout; a concat consumer gets
 * its slice), so those convs skip their x split pass (pass the planes as ready once
 * every slice is written).  planesC, col and C multiples of 16, 16-byte aligned. */
int dg_bn_fwd_train_pl(int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                       float *save_mean, float *save_invstd,
                       float *moving_mean, float *moving_var, float momentum, float eps,
                       float *z, int ldz, int act, float alpha,
                       float drop_rate, uint32_t drop_seed, const int32_t *step_dev,
                       void *zp0, int zp0C, int zp0col, void *zp1, int zp1C, int zp1col,
                       void *ws, size_t ws_bytes, dg_stream_t stream);
int dg_bn_fwd_infer(int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                    const float *moving_mean, const float *moving_var, float eps,
                    float *z, int ldz, int act, float alpha, dg_stream_t stream);
/* Backward of act(BN(y)) (+ dropout): reads dz (grad of the block output) and z (the
 * block output, for the activation mask), writes dy; dgamma/dbeta = grad + beta*old. */
int dg_bn_bwd(int M, int C, const float *dz, int lddz, const float *z, int ldz,
              const float *y, int ldy, const float *gamma,
              const float *save_mean, const float *save_invstd,
              int act, float alpha, float drop_rate,
              float *dy, int lddy, float *dgamma, float *dbeta, float beta,
              void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_bn_bwd that also writes dy's bf16x6 operand planes (dg_conv_planes_t.dy layout:
 * row r, channel c of plane p at r*3C + (c/16)*48 + 16p + c%16; C % 16 == 0, 16-byte
 * aligned) beside dy, so the consuming conv's bwd_data / bwd_filter skip their split
 * pass (pass those planes as ready).  dy_planes NULL == dg_bn_bwd. */
int dg_bn_bwd_pl(int M, int C, const float *dz, int lddz, const float *z, int ldz,
                 const float *y, int ldy, const float *gamma,
                 const float *save_mean, const float *save_invstd,
                 int act, float alpha, float drop_rate,
                 float *dy, int lddy, void *dy_planes, float *dgamma, float *dbeta, float beta,
                 void *ws, size_t ws_bytes, dg_stream_t stream);
/* Segmented forms: S independent BN calls over S consecutive row segments of M rows
 * each, in ONE launch set -- the reference's separate calls of one layer that the
 * step batches into one pass (G(x) / G(target), pix2pix.py:44 / :90; D(real) /
 * D(fake), train_pix2pix.py:47-48).  Segment s normalises with its own statistics
 * (save_mean / save_invstd are [S][C]); the moving averages take the segments'
 * updates in order; dropout on segment s uses seed drop_seed + s * drop_seed_stride
 * with the element index restarting per segment; backward: per-segment coefficients,
 * dgamma / dbeta summed over the segments.  S == 1 is the plain call. */
int dg_bn_workspace_size_seg(int S, int M, int C, size_t *bytes);
int dg_bn_fwd_train_seg(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                        float *save_mean, float *save_invstd,
                        float *moving_mean, float *moving_var, float momentum, float eps,
                        float *z, int ldz, int act, float alpha,
                        float drop_rate, uint32_t drop_seed, uint32_t drop_seed_stride, const int32_t *step_dev,
                        void *zp0, int zp0C, int zp0col, void *zp1, int zp1C, int zp1col,
                        void *ws, size_t ws_bytes, dg_stream_t stream);
int dg_bn_bwd_seg(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz,
                  const float *y, int ldy, const float *gamma,
                  const float *save_mean, const float *save_invstd,
                  int act, float alpha, float drop_rate,
                  float *dy, int lddy, void *dy_planes, float *dgamma, float *dbeta, float beta,
                  void *ws, size_t ws_bytes, dg_stream_t stream);
/* The same, also writing the consuming conv's DG_MATH_FP16 operand copy of z / dy
 * (z_f16 / dy_f16: [S*M rows][C] fp16, round-to-nearest-even -- the bytes the conv's own
 * conversion would write into its dg_conv_planes_t x / dy buffer, which the caller then
 * passes as ready; 8-byte aligned; NULL = none).  The SR family's mixed_float16 convs
 * (srgan.py:63-66) thus skip their per-call fp32 -> fp16 conversion of these operands.
 * res (may be NULL): a residual Add fused after the block, z = act(BN(y)) + res
 * ([S*M rows][C], pixel stride ldres; the residual blocks' keras.layers.Add,
 * srgan.py:165 / :180, fsrgan.py:176 / :214) -- the Add's own pass disappears.
 * Backward: z (the block output) is read only for act'; a linear BN without dropout
 * may pass z = NULL (the fused BN + Add above never writes its own z). */
int dg_bn_fwd_train_seg_h(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                          float *save_mean, float *save_invstd,
                          float *moving_mean, float *moving_var, float momentum, float eps,
                          float *z, int ldz, int act, float alpha,
                          float drop_rate, uint32_t drop_seed, uint32_t drop_seed_stride, const int32_t *step_dev,
                          void *zp0, int zp0C, int zp0col, void *zp1, int zp1C, int zp1col,
                          const float *res, int ldres, void *z_f16,
                          void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_bn_fwd_train_seg_h with bound-scaled fp16x3 z planes (round 5).  z_bound (a max slot,
 * zeroed and filled here; NULL: the static 2^-4): max over channels of (|gamma| invstd
 * max |y - mean| + |beta|) x the dropout keep scale >= max |z|, from per-chunk maxima of the
 * statistics pass -- the planes' scale source the consuming conv reads
 * (dg_conv_set_act_scale x_m = z_bound).  cp (may be NULL): cpC channels ([S*M rows], pixel
 * stride ldcp) of a second tensor whose planes go to zp0 at column cpcol with the same scale,
 * and cp_bound their bound (a max slot, merged into z_bound): the U-Net skip half of the
 * concatenation the next ConvT reads (pix2pix.py:188), so one scale covers its whole operand. */
int dg_bn_fwd_train_seg_x(int S, int M, int C, const float *y, int ldy, const float *gamma, const float *beta,
                          float *save_mean, float *save_invstd,
                          float *moving_mean, float *moving_var, float momentum, float eps,
                          float *z, int ldz, int act, float alpha,
                          float drop_rate, uint32_t drop_seed, uint32_t drop_seed_stride, const int32_t *step_dev,
                          void *zp0, int zp0C, int zp0col, void *zp1, int zp1C, int zp1col,
                          float *z_bound, const float *cp, int ldcp, int cpC, int cpcol, const float *cp_bound,
                          const float *res, int ldres, void *z_f16,
                          void *ws, size_t ws_bytes, dg_stream_t stream);
int dg_bn_bwd_seg_h(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz,
                    const float *y, int ldy, const float *gamma,
                    const float *save_mean, const float *save_invstd,
                    int act, float alpha, float drop_rate,
                    float *dy, int lddy, void *dy_planes, void *dy_f16, float *dgamma, float *dbeta, float beta,
                    void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_bn_bwd_seg_h with the format of the dy planes: DG_PLANES_F16X3 writes the consuming
 * DG_MATH_F16X3 conv's fp16x3 dy planes (C % 32 == 0), scaled by x3 scale 2^(14 - e) from
 * dy's bound b < 2^e -- b = max over channels of |A| max|dbn| + |B| max|y - mean| + |D|
 * >= max |dy| (dy = A dbn + B (y - mean) + D per channel), written into dy_bound (a max slot:
 * the bound's per-workgroup shards, their max is b) -- the buffer to pass that conv as its dy
 * scale source (dg_conv_set_grad_scale dy_m, dy_g NULL).  In the forward calls above a
 * NEGATIVE zp*C names the consumer's fp16x3 x planes of -zp*C channels (column and C
 * multiples of 32). */
int dg_bn_bwd_seg_x(int S, int M, int C, const float *dz, int lddz, const float *z, int ldz,
                    const float *y, int ldy, const float *gamma,
                    const float *save_mean, const float *save_invstd,
                    int act, float alpha, float drop_rate,
                    float *dy, int lddy, void *dy_planes, int dy_planes_format, float *dy_bound, void *dy_f16,
                    float *dgamma, float *dbeta, float beta, void *ws, size_t ws_bytes, dg_stream_t stream);
/* dg_bn_bwd_seg_x without z: act'(z) of a ReLU / LeakyReLU (or linear) BN block WITHOUT
 * dropout recomputed from y as the sign of t = y * scale + shift, the forward's per-channel
 * scale = gamma * invstd, shift = bn_beta - mean * scale (k_bn_stats_final's rounding, so t is
 * the forward's pre-activation bit for bit and sign(z) = sign(t)) -- one tensor fewer read in
 * both backward passes (pix2pix.py:119 / :135 / :211 BN sites, the down / up blocks' backward
 * of Pix2Pix.train_step train_pix2pix.py:27-34).  bn_beta (the BN offset, may be NULL = 0) is
 * the value the forward used (the gradients are taken before the optimizer step). */
int dg_bn_bwd_seg_r(int S, int M, int C, const float *dz, int lddz,
                    const float *y, int ldy, const float *gamma, const float *bn_beta,
                    const float *save_mean, const float *save_invstd, int act, float alpha,
                    float *dy, int lddy, void *dy_planes, int dy_planes_format, float *dy_bound, void *dy_f16,
                    float *dgamma, float *dbeta, float beta, void *ws, size_t ws_bytes, dg_stream_t stream);
/* dy = dz * act'(z)  for blocks without BN (pix2pix.py:118-121 with apply_batchnorm=False) */
int dg_act_bwd(int M, int C, const float *dz, int lddz, const float *z, int ldz,
               int act, float alpha, float *dy, int lddy, dg_stream_t stream);

/* ------------------------------------------------------------------------
 * pix2pix losses, forward values and gradients in one call
 * (Pix2Pix.generator_loss pix2pix.py:74-94, discriminator_loss :96-103).
 * gen/tgt/ident are [B,H,W,C] with pixel strides; ident (= G(target)) may be
 * NULL, then the identity term is 0.  weights[6] = {gan, l1, l2, tv, identity,
 * content} scales (reference: 1e-3, 1, 1, 1e-5, 1, 1).  out[8] (device) =
 * {gen_total, gan, l1, l2, content, disc, var, identity}: the tuple order of
 * train_step (train_pix2pix.py:71).  Gradient outputs may be NULL.
 * ---------------------------------------------------------------------- */
int dg_p2p_loss_workspace_size(int B, int H, int W, int C, int n_logits, size_t *bytes);
int dg_p2p_loss(int B, int H, int W, int C,
                const float *gen, int ldgen, const float *tgt, int ldtgt,
                const float *ident, int ldident,
                const float *logit_real, const float *logit_fake, int n_logits,
                const float *weights, const float *content_value, float *out,
                float *dgen, int lddgen, float *dident, int lddident,
                float *dlogit_real_d, float *dlogit_fake_d, float *dlogit_fake_g,
                void *ws, size_t ws_bytes, dg_stream_t stream);

/* ------------------------------------------------------------------------
 * Keras Adam (ResourceApplyAdam, train_pix2pix.py:68-69):
 *   t = *iter_dev + 1; lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
 *   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ; p -= lr_t m / (sqrt(v) + eps)
 * with g = grad_scale * grad (grad_scale folds the data-parallel 1/world).
 * Runs over one flat parameter arena.  dg_counter_add bumps the device
 * iteration counter afterwards (optimizer.iterations).
 * ---------------------------------------------------------------------- */
int dg_adam(float *p, const float *g, float *m, float *v, int64_t n,
            float lr, float beta1, float beta2, float eps, float grad_scale,
            const int32_t *iter_dev, dg_stream_t stream);
int dg_counter_add(int32_t *counter_dev, int32_t inc, dg_stream_t stream);
/* Dynamic loss scaling of the fp16 conv math (tf.keras mixed_precision
 * LossScaleOptimizer(loss_scale='dynamic'), srgan.py:64-67, used by
 * train_srgan.py:98-109): device state ls[4] = {scale, good steps, finite flag, 0},
 * initial {2^15, 0, 1, 0}.  Per step: dg_scale_by multiplies the loss-gradient
 * seeds by the scale, dg_check_finite clears the flag when a gradient is inf/nan,
 * dg_adam_ls unscales (grad_scale / scale) or skips the whole update when the flag
 * is clear (Keras skips apply_gradients), dg_counter_add_ls advances the optimizer's
 * iterations only on an applied step, and dg_loss_scale_update applies Keras'
 * rule (finite: after `period` (2000) good steps scale *= multiplier (2); not
 * finite: scale /= multiplier, at least 1) and re-arms the flag. */
int dg_scale_by(int64_t n, float *x, const float *loss_scale, dg_stream_t stream);
int dg_check_finite(int64_t n, const float *g, float *loss_scale, dg_stream_t stream);
int dg_adam_ls(float *p, const float *g, float *m, float *v, int64_t n, float lr, int64_t decay_steps,
               float decay_rate, int staircase, float beta1, float beta2, float eps, float grad_scale,
               const int32_t *iter_dev, const float *loss_scale, dg_stream_t stream);
int dg_counter_add_ls(int32_t *counter_dev, int32_t inc, const float *loss_scale, dg_stream_t stream);
int dg_loss_scale_update(float *loss_scale, int period, float multiplier, dg_stream_t stream);
/* Adam under keras.optimizers.schedules.ExponentialDecay (srgan.py:34-46,
 * fsrgan.py:30-43, autoencoder.py:26-37): the learning rate of the update
 * with iterations = *iter_dev is lr * decay_rate^(it / decay_steps) (floor
 * of the exponent when staircase).  decay_steps <= 0 means a constant lr. */
int dg_adam_sched(float *p, const float *g, float *m, float *v, int64_t n,
                  float lr, int64_t decay_steps, float decay_rate, int staircase,
                  float beta1, float beta2, float eps, float grad_scale,
                  const int32_t *iter_dev, dg_stream_t stream);

/* ------------------------------------------------------------------------
 * Data movement helpers.
 * dg_channel_concat: out[p, 0:ca] = a[p, 0:ca], out[p, ca:ca+cb] = b[p, 0:cb]
 *   (tf.keras.layers.concatenate([inp, tar]) at pix2pix.py:200).
 * dg_fill: p[0:n] = value.
 * ---------------------------------------------------------------------- */
int dg_channel_concat(int64_t npix, const float *a, int lda, int ca, const float *b, int ldb, int cb,
                      float *out, int ldo, dg_stream_t stream);
int dg_fill(float *p, int64_t n, float value, dg_stream_t stream);
/* dst[0:n] = fp16(src[0:n]) (round to nearest even; n % 8 == 0, 16-byte aligned): one launch
 * converting a whole parameter arena into the fp16 weight copies its DG_MATH_FP16 convs read
 * (dg_conv_planes_t.w views into dst, passed ready) instead of one conversion per conv */
int dg_to_f16(int64_t n, const float *src, void *dst, dg_stream_t stream);
int dg_strided_copy(int64_t npix, int C, const float *src, int lds, float *dst, int ldd, dg_stream_t stream);
/* dg_stage_pair: the pix2pix step's input staging in one launch -- cat[p, 0:C] = x[p],
 * cat[p, C:2C] = y[p] (concatenate([inp, tar]), pix2pix.py:200); catx[p, 0:C] = x[p] (D(fake)'s
 * input, its channels C..2C are G(x)); gx[p] = x[p], gy[p] = y[p] (dense: the G(x) / G(y) halves
 * of the identity pass's 2N-image batch, pix2pix.py:44,90).  x, y dense [npix, C], C <= 4;
 * catx, gx, gy may be NULL.  Replaces dg_channel_concat + three dg_strided_copy calls. */
int dg_stage_pair(int64_t npix, int C, const float *x, const float *y, float *cat, int ldcat, float *catx,
                  int ldcatx, float *gx, float *gy, dg_stream_t stream);

/* ------------------------------------------------------------------------
 * Layers of the SRGAN / FastSRGAN / Autoencoder models and of the frozen
 * VGG19 feature extractor.  Input-gradient outputs take `beta`
 * (dx = new + beta*dx) so a tensor with several consumers (residual
 * skips, concat members) accumulates its gradient in place.
 * ---------------------------------------------------------------------- */
/* PReLU(shared_axes=[1,2]) (srgan.py:139, :152), optionally preceded by
 * tf.nn.depth_to_space(., block=2) (srgan.py:138, fsrgan.py:198):
 * y [N,H,W,C*block^2] -> z [N,H*block,W*block,C]; alpha[C]. */
int dg_prelu_workspace_size(int N, int H, int W, int C, int block, size_t *bytes);
int dg_prelu_fwd(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha,
                 float *z, int ldz, dg_stream_t stream);
/* dy = dL/dy + beta*dy ; dalpha = dL/dalpha + alpha_beta*dalpha (dalpha may be NULL) */
int dg_prelu_bwd(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha,
                 const float *dz, int lddz, float *dy, int lddy, float beta,
                 float *dalpha, float alpha_beta, void *ws, size_t ws_bytes, dg_stream_t stream);
/* keras.layers.Add (srgan.py:165): out = a + b */
int dg_add(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float *out, int ldo,
           dg_stream_t stream);
/* _h forms: also the consuming / producing fp16 conv's operand copy (dg_bn_fwd_train_seg_h):
 * z_f16 [N*H*block*W*block][C], dy_f16 [N*H*W][C*block^2] (after beta), out_f16 [npix][C] */
int dg_prelu_fwd_h(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha,
                   float *z, int ldz, void *z_f16, dg_stream_t stream);
int dg_prelu_bwd_h(int N, int H, int W, int C, int block, const float *y, int ldy, const float *alpha,
                   const float *dz, int lddz, float *dy, int lddy, void *dy_f16, float beta,
                   float *dalpha, float alpha_beta, void *ws, size_t ws_bytes, dg_stream_t stream);
int dg_add_h(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float *out, int ldo,
             void *out_f16, dg_stream_t stream);
/* dst = src + beta*dst (gradient fan-in) */
int dg_accumulate(int64_t npix, int C, const float *src, int lds, float *dst, int ldd, float beta,
                  dg_stream_t stream);
/* z = act(x) (e.g. the sigmoid of the autoencoder discriminator's output, autoencoder.py:226) */
int dg_act_fwd(int64_t npix, int C, const float *x, int ldx, int act, float alpha, float *z, int ldz,
               dg_stream_t stream);
/* MaxPool2D(2, strides 2) (autoencoder.py:111-115, VGG19 block pools): [N,H,W,C] -> [N,H/2,W/2,C] */
int dg_maxpool2_fwd(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, dg_stream_t stream);
/* dx = routed dy * act'(x) + beta*dx; act (through x = the activation's output) folds the
 * gradient of the activation that produced the pool input (DG_ACT_NONE: plain MaxPoolGrad) */
int dg_maxpool2_bwd(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy,
                    float *dx, int lddx, float beta, int act, float alpha, dg_stream_t stream);
/* the same, also writing the bf16x6 planes (dg_conv_planes_t layout, C % 16 == 0) of y / dx for
 * the conv that reads them (VGG19: pool -> conv input, pool gradient -> the previous conv's dy) */
int dg_maxpool2_fwd_pl(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                       dg_stream_t stream);
/* the same with the consumer's plane format (DG_PLANES_*; fp16x3: C % 32 == 0) */
int dg_maxpool2_fwd_plf(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                        int y_planes_format, dg_stream_t stream);
/* the same with fp16x3 planes scaled from the source (scale_m, scale_g, scale_c) -- the
 * producing conv's output source (dg_conv_set_act_scale y_m / y_g / y_c), a bound of the pooled
 * values too; NULL scale_m: the static 2^-4 */
int dg_maxpool2_fwd_x3(int N, int H, int W, int C, const float *x, int ldx, float *y, int ldy, void *y_planes,
                       int y_planes_format, const float *scale_m, const float *scale_g, const float *scale_c,
                       dg_stream_t stream);
int dg_maxpool2_bwd_pl(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy,
                       float *dx, int lddx, float beta, int act, float alpha, void *dx_planes, dg_stream_t stream);
/* backward of a pool fused by dg_conv_fwd_pool, from its index bytes (the full-size
 * activation is not read): dx = dy * act'(pooled) at the first maximum, 0 elsewhere;
 * H, W even (the conv output), C % 16 == 0; dx may be NULL (beta 0) when only its
 * bf16x6 planes (dx_planes) are consumed */
int dg_maxpool2_bwd_idx(int N, int H, int W, int C, const unsigned char *idx, const float *dy, int lddy,
                        float *dx, int lddx, float beta, int act, float alpha, void *dx_planes, dg_stream_t stream);
/* the same writing the fp16x3 dy planes of an fp16x3 input gradient (C % 32 == 0), scaled
 * from (scale_m, scale_g) as dg_conv_set_grad_scale describes (NULL scale_m: bf16x6 planes) */
int dg_maxpool2_bwd_idx_x3(int N, int H, int W, int C, const unsigned char *idx, const float *dy, int lddy,
                           float *dx, int lddx, float beta, int act, float alpha, void *dx_planes,
                           const float *scale_m, const float *scale_g, dg_stream_t stream);
/* UpSampling2D(2, 'nearest') + relu (autoencoder.py:117-131): [N,H,W,C] -> [N,2H,2W,C] */
int dg_upsample2_relu_fwd(int N, int H, int W, int C, const float *x, int ldx, float *z, int ldz,
                          dg_stream_t stream);
int dg_upsample2_relu_bwd(int N, int H, int W, int C, const float *x, int ldx, const float *dz, int lddz,
                          float *dx, int lddx, float beta, dg_stream_t stream);
/* DepthwiseConv2D(3, strides 1, 'same', use_bias) (fsrgan.py:162-167); k [3,3,C] */
int dg_dwconv3_workspace_size(int N, int H, int W, int C, size_t *bytes);
int dg_dwconv3_fwd(int N, int H, int W, int C, const float *x, int ldx, const float *k, const float *bias,
                   float *y, int ldy, dg_stream_t stream);
int dg_dwconv3_bwd_data(int N, int H, int W, int C, const float *dy, int lddy, const float *k,
                        float *dx, int lddx, float beta, dg_stream_t stream);
int dg_dwconv3_bwd_filter(int N, int H, int W, int C, const float *x, int ldx, const float *dy, int lddy,
                          float *dk, float *dbias, float beta, void *ws, size_t ws_bytes, dg_stream_t stream);
/* vgg19.preprocess_input(((x + 1) * 255) / 2) (srgan.py:71-72): RGB->BGR, minus the caffe means */
int dg_vgg_preprocess_fwd(int64_t npix, const float *x, int ldx, float *z, int ldz, dg_stream_t stream);
int dg_vgg_preprocess_bwd(int64_t npix, const float *dz, int lddz, float *dx, int lddx, float beta,
                          dg_stream_t stream);
/* out[0] = mean((scale*a - scale*b)^2) (MeanSquaredError of VGG features / 12.75,
 * srgan.py:74-76); da = grad_weight * d out / d a (may be NULL) */
int dg_mse_workspace_size(size_t *bytes);
int dg_mse(int64_t npix, int C, const float *a, int lda, const float *b, int ldb, float scale, float *out,
           float *da, int ldda, float grad_weight, void *ws, size_t ws_bytes, dg_stream_t stream);
/* SR-GAN loss set (train_srgan.py:84-96, train_fsrgan.py:86-96, train_autoencoder.py:84-100).
 * coef[7] = {w_adv, w_var, disc_scale, t_mae, t_mse, t_content, t_var}:
 *   adv = w_adv*BCE_logits(1, fake); mae, mse raw; var = w_var*mean_b TV(y - g);
 *   disc = disc_scale*(BCE_logits(1, real) + BCE_logits(0, fake));
 *   gen_total = adv + t_mae*mae + t_mse*mse + t_content*content + t_var*var.
 * out[7] = {gen_total, adv, mae, mse, content, disc, var}.  dgen = d gen_total / d g
 * through the image terms only; the logit gradients are those of disc (d) and adv (g). */
int dg_gan_loss_workspace_size(size_t *bytes);
int dg_gan_loss(int B, int H, int W, int C, const float *gen, int ldgen, const float *tgt, int ldtgt,
                const float *logit_real, const float *logit_fake, int n_logits, const float *coef,
                const float *content_value, float *out, float *dgen, int lddgen,
                float *dlogit_real_d, float *dlogit_fake_d, float *dlogit_fake_g,
                void *ws, size_t ws_bytes, dg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DGAN_H */
