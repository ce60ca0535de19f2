// Single-output-channel convs (Co == 1 in the conv view): the PatchGAN's last
// layer, ZeroPadding2D() + Conv2D(1, 4, strides=1) over the 512-channel
// LeakyReLU output (pix2pix.py:210-212).  As a GEMM its input gradient has a
// K of kh*kw = 16 and its filter gradient an N of 1, so the MFMA tiles run
// almost empty; these two are direct kernels whose cost is the bytes of the
// wide tensor (dx written, x read) once.  (The forward stays on the GEMM
// recast, see co1_ok.)
//
// DGRAD dx[n,h,w,c] = sum over the taps (i,j) that reach (h,w) of dy[n,ho,wo] w[i,j,c]
//       Block = one input row; thread = (4 channels, pixel lane) with its filter
//       column w[:, :, c..c+3] in registers; the dy rows the strip reaches are
//       staged in LDS with zeros outside the output, so the 4x4 stride-1 tap
//       loop has no bounds tests (bs16 x2: 0.065 -> 0.027 ms per call).
// WGRAD dw[i,j,c] = sum_{n,ho,wo} x[n, ho*sh-pt+i, wo*sw-pl+j, c] dy[n,ho,wo]
//       Loop over INPUT pixels (each x float4 loaded once, four in flight, then
//       scattered into the kh x kw tap accumulators with staged dy values);
//       per-block partials [block][tap][c] go to the split-K slab and a second
//       kernel sums them in block order (deterministic).
#include "conv_impl.h"
#include <algorithm>

namespace dg {

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int CO1_KMAX = 4;        // kh, kw <= 4
constexpr int CO1_ROWS = 2;        // DGRAD / WGRAD: input rows per block
constexpr int CO1_LDC = 520;       // staged dy row (floats)

__host__ __device__ constexpr int co1_fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

bool co1_ok(const ConvGeom &g, int mode) {
    if (g.Co != 1 || g.kh > CO1_KMAX || g.kw > CO1_KMAX || g.Ci % 4) return false;
    // (the forward stays on the GEMM recast: a direct forward -- per output row, each
    // tap row's x . w dots for 8 pixels per wave, shift-added from LDS -- measured
    // 42-64 us against the recast's 54 us at bs32)
    if (mode == MODE_FWD) return false;
    // staged dy rows: the output columns input columns 0..W-1 reach
    const int ncol = co1_fdiv(g.W - 1 + g.pl, g.sw) - co1_fdiv(g.pl - (g.kw - 1), g.sw) + 1;
    return g.Ci <= 1024 && 256 % (g.Ci / 4) == 0 && ncol <= CO1_LDC;
}

int co1_wgrad_blocks(const ConvGeom &g) { return g.N * ((g.H + CO1_ROWS - 1) / CO1_ROWS); }

// A block's strip: image n, input rows [h0, h0 + rows); the dy rows / columns
// its pixels reach, staged in LDS with zeros outside the output (so that the
// stride-1 tap loops need no bounds tests: a padding tap adds x * 0)
struct Co1Strip {
    int n, h0, rows, ho_lo, wlo, nr, ncol;
};
__device__ __forceinline__ Co1Strip co1_strip(const ConvGeom &g, int rows) {
    Co1Strip s;
    const int nrb = (g.H + rows - 1) / rows;
    s.n = blockIdx.x / nrb;
    s.h0 = (blockIdx.x - s.n * nrb) * rows;
    s.rows = min(rows, g.H - s.h0);
    s.ho_lo = co1_fdiv(s.h0 + g.pt - (g.kh - 1), g.sh);
    s.nr = co1_fdiv(s.h0 + s.rows - 1 + g.pt, g.sh) - s.ho_lo + 1;
    s.wlo = co1_fdiv(g.pl - (g.kw - 1), g.sw);
    s.ncol = co1_fdiv(g.W - 1 + g.pl, g.sw) - s.wlo + 1;
    return s;
}
__device__ __forceinline__ void co1_stage(const float *dy, int ld, const ConvGeom &g, const Co1Strip &s,
                                          float (*dys)[CO1_LDC]) {
    for (int e = threadIdx.x; e < s.nr * s.ncol; e += 256) {
        const int r = e / s.ncol, cc = e - r * s.ncol;
        const int ho = s.ho_lo + r, wo = s.wlo + cc;
        dys[r][cc] = ((unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo)
                         ? dy[((long)(s.n * g.Ho + ho) * g.Wo + wo) * ld] : 0.f;
    }
}

// DGRAD: block = strip, thread = (4 channels c, pixel lane); the thread's
// filter column w[:, :, c..c+3] lives in registers, dy comes from LDS
template <bool K4>   // 4x4 stride 1 (the PatchGAN last layer): no per-tap tests
__global__ void __launch_bounds__(256)
k_co1_dgrad(const GemmArgs p) {
    __shared__ float dys[CO1_ROWS + CO1_KMAX][CO1_LDC];
    const ConvGeom &g = p.g;
    const Co1Strip st = co1_strip(g, 1);   // one input row per block: ~1000 blocks at bs16
    co1_stage(p.A, p.lda, g, st, dys);
    const int c4 = g.Ci / 4, P = 256 / c4;
    const int tid = threadIdx.x, c = (tid % c4) * 4, lanep = tid / c4;
    f32x4 wr[CO1_KMAX][CO1_KMAX];
    if constexpr (K4) {
#pragma unroll
        for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
            for (int j = 0; j < CO1_KMAX; ++j)
                wr[i][j] = *reinterpret_cast<const f32x4 *>(p.B + (long)(i * CO1_KMAX + j) * g.Ci + c);
    }
    __syncthreads();
    const bool cvec = (p.ldc & 3) == 0 && (((uintptr_t)p.C) & 15) == 0;
    const bool plain = p.C && cvec && !p.bias && p.act == DG_ACT_NONE && !p.mz && !p.mzp && p.beta == 0.f && !p.yp;
    for (int q = lanep; q < st.rows * g.W; q += P) {
        const int hr = q / g.W, w = q - hr * g.W, h = st.h0 + hr;
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        if constexpr (K4) {
            // 4x4 stride 1: tap (i, j) reads staged dy (hr + 3 - i, w + 3 - j); the 16 loads issue together
            float d[CO1_KMAX][CO1_KMAX];
#pragma unroll
            for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
                for (int j = 0; j < CO1_KMAX; ++j) d[i][j] = dys[hr + 3 - i][w + 3 - j];
            // packed FMAs (v_pk_fma_f32): channels (c, c+1) and (c+2, c+3)
            f32x2 lo = {0.f, 0.f}, hi = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
                for (int j = 0; j < CO1_KMAX; ++j) {
                    const f32x2 dd = {d[i][j], d[i][j]};
                    lo = __builtin_elementwise_fma(dd, f32x2{wr[i][j][0], wr[i][j][1]}, lo);
                    hi = __builtin_elementwise_fma(dd, f32x2{wr[i][j][2], wr[i][j][3]}, hi);
                }
            o = f32x4{lo[0], lo[1], hi[0], hi[1]};
        } else {
            for (int i = 0; i < g.kh; ++i) {
                const int th = h + g.pt - i;
                if (th % g.sh) continue;
                const float *dr = dys[co1_fdiv(th, g.sh) - st.ho_lo];
                for (int j = 0; j < g.kw; ++j) {
                    const int tw = w + g.pl - j;
                    if (tw % g.sw) continue;
                    const float dv = dr[co1_fdiv(tw, g.sw) - st.wlo];
                    const f32x4 wv = *reinterpret_cast<const f32x4 *>(p.B + (long)(i * g.kw + j) * g.Ci + c);
                    o[0] = fmaf(dv, wv[0], o[0]);
                    o[1] = fmaf(dv, wv[1], o[1]);
                    o[2] = fmaf(dv, wv[2], o[2]);
                    o[3] = fmaf(dv, wv[3], o[3]);
                }
            }
        }
        const long pix = (long)(st.n * g.H + h) * g.W + w;
        if (plain) {
            *reinterpret_cast<f32x4 *>(p.C + pix * p.ldc + c) = o;
            continue;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float v = o[u];
            if (p.bias) v += p.bias[c + u];
            o[u] = epi_mask(p, pix, c + u, act_fwd(v, p.act, p.alpha));
        }
        if (p.C) {
            float *dst = p.C + pix * p.ldc + c;
            if (cvec) {
                if (p.beta != 0.f) o += p.beta * *reinterpret_cast<const f32x4 *>(dst);
                *reinterpret_cast<f32x4 *>(dst) = o;
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = dst[u] = p.beta != 0.f ? o[u] + p.beta * dst[u] : o[u];
            }
        }
        if (p.yp) store_planes4(p.yp, p.ypC, pix, c, o, plane_scale(p));
    }
}

// WGRAD: block = strip, thread = (4 channels c, pixel lane); each x float4 is
// loaded once (four pixels' loads in flight) and feeds the kh x kw tap
// accumulators; the pixel lanes are summed through LDS in lane order and the
// block's partial [tap][c] goes to slab row blockIdx.x
template <bool K4>
__global__ void __launch_bounds__(256)
k_co1_wgrad(const GemmArgs p) {
    __shared__ __attribute__((aligned(16))) float dys[CO1_ROWS + CO1_KMAX][CO1_LDC];
    const ConvGeom &g = p.g;
    const Co1Strip st = co1_strip(g, CO1_ROWS);
    co1_stage(p.B, p.ldb, g, st, dys);
    const int c4 = g.Ci / 4, P = 256 / c4;
    const int tid = threadIdx.x, c = (tid % c4) * 4, lanep = tid / c4;
    f32x4 acc[CO1_KMAX][CO1_KMAX];
#pragma unroll
    for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
        for (int j = 0; j < CO1_KMAX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int npx = st.rows * g.W;
    const float *xb = p.A + (long)(st.n * g.H + st.h0) * g.W * p.lda + c;
    constexpr int PF = 4;
    for (int q0 = lanep; q0 < npx; q0 += PF * P) {
        f32x4 xs[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int q = q0 + u * P;
            xs[u] = q < npx ? *reinterpret_cast<const f32x4 *>(xb + (long)q * p.lda) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int q = q0 + u * P;
            if (q >= npx) break;
            const int hr = q / g.W, w = q - hr * g.W, h = st.h0 + hr;
            const f32x4 x = xs[u];
            if constexpr (K4) {
                float d[CO1_KMAX][CO1_KMAX];
#pragma unroll
                for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
                    for (int j = 0; j < CO1_KMAX; ++j) d[i][j] = dys[hr + 3 - i][w + 3 - j];
#pragma unroll
                for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
                    for (int j = 0; j < CO1_KMAX; ++j) {
                        acc[i][j][0] = fmaf(x[0], d[i][j], acc[i][j][0]);
                        acc[i][j][1] = fmaf(x[1], d[i][j], acc[i][j][1]);
                        acc[i][j][2] = fmaf(x[2], d[i][j], acc[i][j][2]);
                        acc[i][j][3] = fmaf(x[3], d[i][j], acc[i][j][3]);
                    }
            } else {
#pragma unroll
                for (int i = 0; i < CO1_KMAX; ++i) {
                    if (i >= g.kh) continue;
                    const int th = h + g.pt - i;
                    if (th % g.sh) continue;
                    const float *dr = dys[co1_fdiv(th, g.sh) - st.ho_lo];
#pragma unroll
                    for (int j = 0; j < CO1_KMAX; ++j) {
                        if (j >= g.kw) continue;
                        const int tw = w + g.pl - j;
                        if (tw % g.sw) continue;
                        const float dv = dr[co1_fdiv(tw, g.sw) - st.wlo];
                        acc[i][j][0] = fmaf(x[0], dv, acc[i][j][0]);
                        acc[i][j][1] = fmaf(x[1], dv, acc[i][j][1]);
                        acc[i][j][2] = fmaf(x[2], dv, acc[i][j][2]);
                        acc[i][j][3] = fmaf(x[3], dv, acc[i][j][3]);
                    }
                }
            }
        }
    }
    // sum the P pixel lanes through LDS (reusing dys: P * Ci = 1024 floats), in lane order
    float *red = &dys[0][0];
    float *part = p.slab + (long)blockIdx.x * g.kh * g.kw * g.Ci;
#pragma unroll
    for (int i = 0; i < CO1_KMAX; ++i)
#pragma unroll
        for (int j = 0; j < CO1_KMAX; ++j) {
            if (i >= g.kh || j >= g.kw) continue;   // block-uniform
            __syncthreads();
            *reinterpret_cast<f32x4 *>(red + lanep * g.Ci + c) = acc[i][j];
            __syncthreads();
            if (lanep == 0) {
                f32x4 s = *reinterpret_cast<const f32x4 *>(red + c);
                for (int r = 1; r < P; ++r) s += *reinterpret_cast<const f32x4 *>(red + r * g.Ci + c);
                *reinterpret_cast<f32x4 *>(part + (long)(i * g.kw + j) * g.Ci + c) = s;
            }
        }
}

// dw[k] = sum over blocks of partials[block][k] (+ beta dw): 16 k per block x 16
// interleaved block groups, each summed in block order, then the groups in order
constexpr int CO1_RG = 16;
__global__ void __launch_bounds__(256)
k_co1_wgrad_reduce(const GemmArgs p, int nblk) {
    __shared__ float red[CO1_RG][16];
    const ConvGeom &g = p.g;
    const long KT = (long)g.kh * g.kw * g.Ci;
    const int kl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const long k = (long)blockIdx.x * 16 + kl;
    float s = 0.f;
    if (k < KT) {
#pragma unroll 8
        for (int b = grp; b < nblk; b += CO1_RG) s += p.slab[(long)b * KT + k];
    }
    red[grp][kl] = s;
    __syncthreads();
    if (grp == 0 && k < KT) {
        float t = red[0][kl];
        for (int r = 1; r < CO1_RG; ++r) t += red[r][kl];
        float *dst = p.C + k * p.ldc;
        *dst = p.beta != 0.f ? t + p.beta * *dst : t;
    }
}

void launch_co1(int mode, const GemmArgs &a, hipStream_t s) {
    const ConvGeom &g = a.g;
    const bool s1 = g.sh == 1 && g.sw == 1 && g.kh == 4 && g.kw == 4;
    const int nblk = co1_wgrad_blocks(g);
    if (mode == MODE_DGRAD) {
        if (s1) hipLaunchKernelGGL(k_co1_dgrad<true>, dim3((unsigned)(g.N * g.H)), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_co1_dgrad<false>, dim3((unsigned)(g.N * g.H)), dim3(256), 0, s, a);
    } else {
        if (s1) hipLaunchKernelGGL(k_co1_wgrad<true>, dim3((unsigned)nblk), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_co1_wgrad<false>, dim3((unsigned)nblk), dim3(256), 0, s, a);
        const long KT = (long)g.kh * g.kw * g.Ci;
        hipLaunchKernelGGL(k_co1_wgrad_reduce, dim3((unsigned)dg_cdiv(KT, 16)), dim3(256), 0, s, a, nblk);
    }
}

}  // namespace dg
