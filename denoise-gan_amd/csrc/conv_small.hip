// Small-Cin stride-2 4x4 convs on the fp32 matrix cores (exact fp32 products,
// v_mfma_f32_32x32x2_f32): the layers whose input has 3 or 6 channels --
//   G.down1 Conv2D(64) on the 3-channel image      (pix2pix.py:115, first down block)
//   D.down1 Conv2D(64) on the 6-channel [inp, tar] (pix2pix.py:200-202)
//   G.last Conv2DTranspose(3) (pix2pix.py:169): its input gradient is a conv
//   view FWD over the 3-channel output gradient, its filter gradient a WGRAD
// -- forward (FWD) and filter gradient (WGRAD).  The generic GEMM kernels see
// a K of 48 / 96 here and gather im2col one float at a time.  These kernels
// work on one output row segment of P (32 or 64) pixels at a time: the 4
// input rows x (2P + 2) columns x CI channels under the segment ("strip") are
// loaded with coalesced reads into LDS, split by column parity so that a
// pixel's tap (i, j) sits at a fixed offset from the pixel's base
//   strip[i][j & 1][px + (j >> 1)][ci]
// and each MFMA operand is one ds_read_b32 at a compile-time offset from a
// per-lane base: no im2col image is materialised.  Bounds: at 256x256 bs16
// the D.down1 FWD is 6.4 GFLOP (41 us at the 157 TF/s fp32 MFMA peak)
// against 184 MB (29 us at 6.3 TB/s); G.down1 is 10 us of MFMA against
// 12.6 us of bytes -- near the ridge, so the strip loads are prefetched into
// registers one tile ahead and overlap the MFMAs.
//
// Geometry (conv view): kh = kw = 4, sh = sw = 2, CI in {3, 6}, Co % 64 == 0,
// Wo % 32 == 0 (P = 64 when Wo % 64 == 0).  The forward also runs VGG19's
// block1_conv1 (3x3 stride 1 'same' on the 3-channel preprocessed image,
// pix2pix.py:53-67): the strip is then 4 input rows x (P + 2) columns without
// the parity split, and the K of 27 is padded to two halves of rows {0, 1} and
// {2, 3} (row 3's weights are zero), so the same per-half constant offsets apply.
#include "conv_impl.h"
#include <algorithm>

namespace dg {

constexpr int SC_BN = 64;   // output channels per block
constexpr int SC_CH = 8;    // MFMA operands per register chunk

// x rounded up to the next value == r (mod 32): the strip strides keep the
// 16*CI taps of one pixel on distinct banks (ds_read_b32 banks are a/4 mod 32)
__host__ __device__ constexpr int sc_up(int x, int r) { return x + (((r - x) % 32) + 32) % 32; }

// KW x (up to 4 rows) filter, stride S in {1 (KW 3), 2 (KW 4)}
template <int CI, int P, int KW = 4, int S = 2>
struct Strip {
    static_assert((KW == 4 && S == 2) || (KW == 3 && S == 1), "4x4 stride 2 or 3x3 stride 1");
    static constexpr int COLS = S == 2 ? P + 1 : P + KW - 1;  // columns per parity
    static constexpr int PAR = S == 2 ? sc_up(COLS * CI, 2 * CI) : 0;   // parity stride (floats)
    static constexpr int ROW = S == 2 ? sc_up(2 * PAR, 4 * CI) : sc_up(COLS * CI, 4 * CI);  // input-row stride
    static constexpr int SIZE = 4 * ROW;
    static constexpr int WL = S * P + KW - S;                 // input columns loaded
    static constexpr int NLOAD = 4 * WL * CI;                 // elements loaded per tile
    static constexpr int KHALF = 2 * KW * CI;                 // k per MFMA half (filter rows 0-1 | 2-3)
    // offset of tap k = (i*KW + j)*CI + ci of pixel 0
    __host__ __device__ static constexpr int tap(int k) {
        return S == 2 ? ((k / CI) >> 2) * ROW + (((k / CI) & 3) & 1) * PAR + (((k / CI) & 3) >> 1) * CI + k % CI
                      : ((k / CI) / KW) * ROW + ((k / CI) % KW) * CI + k % CI;
    }
    // LDS position of loaded element (input row, input column wl, ci)
    __host__ __device__ static constexpr int pos(int row, int wl, int ci) {
        return S == 2 ? row * ROW + (wl & 1) * PAR + (wl >> 1) * CI + ci : row * ROW + wl * CI + ci;
    }
};

// Load the strip of segment (n, ho, wo0) into registers: element e = tid + q*NTHR of
// [row 0..3][input column 0..WL-1][ci], zero outside the image
template <int CI, int P, int NTHR, int KW = 4, int ST = 2>
__device__ __forceinline__ void strip_fetch(const GemmArgs &p, int n, int ho, int wo0, int tid,
                                            float (&r)[(Strip<CI, P, KW, ST>::NLOAD + NTHR - 1) / NTHR]) {
    using S = Strip<CI, P, KW, ST>;
    const ConvGeom &g = p.g;
    const int h0 = ST * ho - g.pt, w0 = ST * wo0 - g.pl;
#pragma unroll
    for (int q = 0; q < (S::NLOAD + NTHR - 1) / NTHR; ++q) {
        const int e = tid + q * NTHR;
        const int row = e / (S::WL * CI), rem = e - row * (S::WL * CI);
        const int wl = rem / CI, ci = rem - wl * CI;
        const int h = h0 + row, w = w0 + wl;
        const bool ok = ((S::NLOAD % NTHR) == 0 || e < S::NLOAD) && (unsigned)h < (unsigned)g.H &&
                        (unsigned)w < (unsigned)g.W;
        r[q] = ok ? p.A[((long)(n * g.H + h) * g.W + w) * p.lda + ci] : 0.f;
    }
}

template <int CI, int P, int NTHR, int KW = 4, int ST = 2>
__device__ __forceinline__ void strip_store(float *s, int tid,
                                            const float (&r)[(Strip<CI, P, KW, ST>::NLOAD + NTHR - 1) / NTHR]) {
    using S = Strip<CI, P, KW, ST>;
#pragma unroll
    for (int q = 0; q < (S::NLOAD + NTHR - 1) / NTHR; ++q) {
        const int e = tid + q * NTHR;
        if ((S::NLOAD % NTHR) != 0 && q == (S::NLOAD + NTHR - 1) / NTHR - 1 && e >= S::NLOAD) break;
        const int row = e / (S::WL * CI), rem = e - row * (S::WL * CI);
        const int wl = rem / CI, ci = rem - wl * CI;
        s[S::pos(row, wl, ci)] = r[q];
    }
}

// FWD epilogue of one wave's 32x32 tile (rows = pixels rbase.., columns cbase..): the
// accumulator goes through a wave-private LDS stage (32 x 36 floats) so that each lane
// finishes 4 runs of 4 consecutive columns (rows (lane >> 3) + 8i, columns 4 (lane & 7)..)
// -- 16-byte stores of y, 8-byte stores of its bf16x6 planes and one split per pair,
// instead of 16 scalar stores and splits per lane.  The global operands of the epilogue
// (gradient mask, beta * y) are loaded by small_epi_load at the top of the tile, ahead of
// the next tile's strip prefetch, so that waiting for them never waits for the prefetch.
constexpr int SC_STAGE = 32 * 36;
struct SmallEpi {
    f32x4 bias;
    f32x4 z[4], c[4];
};
__device__ __forceinline__ bool sc_vec(const void *ptr, int ld) { return ((ld & 3) == 0) && ((((uintptr_t)ptr) & 15) == 0); }
__device__ __forceinline__ f32x4 sc_ld4(const float *a, bool vec) {
    return vec ? *reinterpret_cast<const f32x4 *>(a) : f32x4{a[0], a[1], a[2], a[3]};
}
__device__ __forceinline__ void small_epi_load(const GemmArgs &p, int rbase, int cbase, int lane, SmallEpi &e) {
    const int col = cbase + (lane & 7) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const long pix = rbase + (lane >> 3) + 8 * i;
        const bool in = pix < p.M;
        if (p.mz) e.z[i] = in ? sc_ld4(p.mz + pix * p.ldmz + col, sc_vec(p.mz, p.ldmz)) : f32x4{0.f, 0.f, 0.f, 0.f};
        if (p.beta != 0.f) e.c[i] = in ? sc_ld4(p.C + pix * p.ldc + col, sc_vec(p.C, p.ldc)) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}
template <bool XL>
__device__ __forceinline__ void small_fwd_epilogue(const GemmArgs &p, const f32x16 &acc, int rbase, int cbase,
                                                   float *stage, int lane, const SmallEpi &e, float &vmax, float ys) {
    const int l32 = lane & 31, h2 = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h2) * 36 + l32] = acc[r];
    const bool cvec = sc_vec(p.C, p.ldc);
    const int col = cbase + (lane & 7) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = (lane >> 3) + 8 * i;
        f32x4 o = *reinterpret_cast<const f32x4 *>(stage + row * 36 + (lane & 7) * 4);
        const long pix = rbase + row;
        if (pix >= p.M) continue;
        if (p.bias) o += e.bias;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = act_fwd(o[q], p.act, p.alpha);
        if constexpr (XL) {
            if (p.mz) {
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] *= act_grad_from_out(e.z[i][q], p.mact, p.malpha);
            }
            if (p.beta != 0.f) o += p.beta * e.c[i];
        }
        float *dst = p.C + pix * p.ldc + col;
        if (!p.C) {
            // planes-only output (dg_conv_fwd_pl with y NULL)
        } else if (cvec) {
            *reinterpret_cast<f32x4 *>(dst) = o;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = o[q];
        }
        if (p.yp) store_planes4(p.yp, p.ypC, pix, col, o, ys);
        if (p.ymax) {   // (max |y|: the consumer's measured input, dg_conv_set_act_scale)
#pragma unroll
            for (int q = 0; q < 4; ++q) vmax = fmaxf(vmax, fabsf(o[q]));
        }
    }
}

// FWD: y[pix][co] = act(sum_k A[pix][k] w[k][co] + bias) (+ beta y, mask, planes).
// Block: 2*(P/32) waves over tiles of P pixels (one row segment) x 64 columns, grid-stride;
// wave (sub, nt) owns pixels sub*32.. and columns nt*32..; its w column lives in registers.
// K is split in halves over the MFMA's two k lanes (k = s + 8*CI*h2): taps i = 0,1 | 2,3.
// XL: the epilogue reads global operands (gradient mask or beta * y).  Without them the
// tile loop issues no loads besides the strip prefetch, and no wait ever covers the
// previous tile's stores.
template <int CI, int P, bool XL, int KW = 4, int ST = 2>
__global__ void __launch_bounds__(128 * (P / 32))
k_small_fwd(const GemmArgs p) {
    using S = Strip<CI, P, KW, ST>;
    constexpr int KH = S::KHALF;                  // k per half
    constexpr int KTOT = KW * KW * CI;            // real k (3x3: half 1's row 3 is padding)
    constexpr int CH = KH % SC_CH == 0 ? SC_CH : 6;
    static_assert(KH % CH == 0, "operand chunks");
    constexpr int NTHR = 128 * (P / 32);
    constexpr int NL = (S::NLOAD + NTHR - 1) / NTHR;
    __shared__ __attribute__((aligned(16))) float strip[2][S::SIZE];
    __shared__ __attribute__((aligned(16))) float stage[2 * (P / 32)][SC_STAGE];
    const ConvGeom &g = p.g;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int sub = wid >> 1, nt = wid & 1;
    const int l32 = lane & 31, h2 = lane >> 5;
    const int col0 = blockIdx.y * SC_BN + nt * 32;
    float wr[KH];
#pragma unroll
    for (int s = 0; s < KH; ++s) wr[s] = s + h2 * KH < KTOT ? p.B[(long)(s + h2 * KH) * p.ldb + col0 + l32] : 0.f;
    const int segs = g.Wo / P;
    const int ntiles = g.N * g.Ho * segs;
    const int abase = h2 * 2 * S::ROW + (sub * 32 + l32) * CI;
    SmallEpi epi;
    if (p.bias) epi.bias = sc_ld4(p.bias + col0 + (lane & 7) * 4, false);
    float pre[NL];
    float vmax = 0.f;   // max |y| of this lane's outputs (p.ymax)
    const X3Raw ysr = x3_raw(p.ys_m, p.ys_g, p.ys_c);   // (the output planes' scale source)
    int t = blockIdx.x;
    if (t >= ntiles) return;   // (the whole block: block_atomic_absmax below stays uniform)
    {
        const int row = t / segs, n = row / g.Ho;
        strip_fetch<CI, P, NTHR, KW, ST>(p, n, row - n * g.Ho, (t - row * segs) * P, tid, pre);
        strip_store<CI, P, NTHR, KW, ST>(strip[0], tid, pre);
    }
    __syncthreads();
    for (int it = 0; t < ntiles; t += gridDim.x, ++it) {
        const int tn = t + gridDim.x;
        const int row = t / segs;
        const int rbase = row * g.Wo + (t - row * segs) * P + sub * 32;
        if constexpr (XL) small_epi_load(p, rbase, col0, lane, epi);
        {   // (past the last tile: refetch this one -- straight-line code keeps the waits exact)
            const int tf = tn < ntiles ? tn : t;
            const int rown = tf / segs, n = rown / g.Ho;
            strip_fetch<CI, P, NTHR, KW, ST>(p, n, rown - n * g.Ho, (tf - rown * segs) * P, tid, pre);
        }
        const float *sb = strip[it & 1] + abase;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        // operands in chunks of CH, the next chunk's LDS reads in flight under this chunk's MFMAs
        float a[2][CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) a[0][u] = sb[S::tap(u)];
#pragma unroll
        for (int c = 0; c < KH / CH; ++c) {
            if (c + 1 < KH / CH) {
#pragma unroll
                for (int u = 0; u < CH; ++u) a[(c + 1) & 1][u] = sb[S::tap((c + 1) * CH + u)];
            }
#pragma unroll
            for (int u = 0; u < CH; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c & 1][u], wr[c * CH + u], acc, 0, 0, 0);
        }
        // the prefetched strip goes to LDS before this tile's stores are issued: waiting for the
        // loads then never waits for the stores (one vmcnt counts both)
        strip_store<CI, P, NTHR, KW, ST>(strip[(it + 1) & 1], tid, pre);
        small_fwd_epilogue<XL>(p, acc, rbase, col0, stage[wid], lane, epi, vmax, x3_raw_scale(ysr, F16X3_XS));
        __syncthreads();
    }
    if (p.ymax) block_atomic_absmax(p.ymax, vmax);
}

// WGRAD: dw[k][co] = sum over pixels of A[pix][k] dy[pix][co].  Block (split, column tile):
// conv-view output rows [split*rpb, ...) as K-tiles of one row segment of P pixels; wave
// (mt, nt) owns rows mt*32.. of the 16*CI filter rows and columns nt*32..; pixel 2s + h2 of
// the segment feeds MFMA step s.  Partials go to the split-K slab [split][M][N]
// (k_splitk_reduce sums them in split order) or, with one split, straight to C.
template <int CI, int P>
__global__ void __launch_bounds__(128 * ((16 * CI + 31) / 32))
k_small_wgrad(const GemmArgs p, int rows_per_block) {
    using S = Strip<CI, P>;
    constexpr int M = 16 * CI;
    constexpr int MT = (M + 31) / 32;
    constexpr int NTHR = 128 * MT;
    constexpr int NL = (S::NLOAD + NTHR - 1) / NTHR;
    constexpr int LDB = SC_BN + 4;                      // dy tile row stride (16-B rows)
    constexpr int NB = (P * SC_BN / 4 + NTHR - 1) / NTHR;   // float4 per thread
    __shared__ __attribute__((aligned(16))) float strip[2][S::SIZE];
    __shared__ __attribute__((aligned(16))) float Bs[2][P * LDB];
    const ConvGeom &g = p.g;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int mt = wid >> 1, nt = wid & 1;
    const int l32 = lane & 31, h2 = lane >> 5;
    const int split = blockIdx.x;
    const int n0 = blockIdx.y * SC_BN;
    const int segs = g.Wo / P;
    const int k0 = split * rows_per_block * segs;
    const int k1 = min(g.N * g.Ho, (split + 1) * rows_per_block) * segs;
    // filter row m = (i*4 + j)*CI + ci of this lane (rows past M read a valid slot; never stored)
    const int m = mt * 32 + l32;
    const int mm = m < M ? m : 0;
    const int tp = mm / CI, ci = mm - tp * CI;
    const int abase = (tp >> 2) * S::ROW + (tp & 1) * S::PAR + ((tp & 3) >> 1) * CI + ci + h2 * CI;
    const int bbase = h2 * LDB + nt * 32 + l32;
    const bool bvec = ((p.ldb & 3) == 0) && ((((uintptr_t)p.B) & 15) == 0);
    float pre[NL];
    f32x4 preb[NB];
    auto fetch = [&](int kt) {
        const int row = kt / segs, wo0 = (kt - row * segs) * P, n = row / g.Ho;
        strip_fetch<CI, P, NTHR>(p, n, row - n * g.Ho, wo0, tid, pre);
        const long pix0 = (long)row * g.Wo + wo0;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int e = tid + q * NTHR;
            const int k = e / (SC_BN / 4), c = (e - k * (SC_BN / 4)) * 4;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (e < P * SC_BN / 4) {
                const float *src = p.B + (pix0 + k) * p.ldb + n0 + c;
                if (bvec) v = *reinterpret_cast<const f32x4 *>(src);
                else v = f32x4{src[0], src[1], src[2], src[3]};
            }
            preb[q] = v;
        }
    };
    auto store = [&](int buf) {
        strip_store<CI, P, NTHR>(strip[buf], tid, pre);
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int e = tid + q * NTHR;
            if (e >= P * SC_BN / 4) break;
            const int k = e / (SC_BN / 4), c = (e - k * (SC_BN / 4)) * 4;
            *reinterpret_cast<f32x4 *>(&Bs[buf][k * LDB + c]) = preb[q];
        }
    };
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if (k0 < k1) {
        fetch(k0);
        store(0);
    }
    __syncthreads();
    for (int kt = k0, it = 0; kt < k1; ++kt, ++it) {
        if (kt + 1 < k1) fetch(kt + 1);
        const float *sa = strip[it & 1] + abase;
        const float *sb = Bs[it & 1] + bbase;
        float a[2][SC_CH], b[2][SC_CH];
#pragma unroll
        for (int u = 0; u < SC_CH; ++u) {
            a[0][u] = sa[2 * u * CI];
            b[0][u] = sb[2 * u * LDB];
        }
#pragma unroll
        for (int c = 0; c < P / 2 / SC_CH; ++c) {
            if (c + 1 < P / 2 / SC_CH) {
#pragma unroll
                for (int u = 0; u < SC_CH; ++u) {
                    const int st = (c + 1) * SC_CH + u;
                    a[(c + 1) & 1][u] = sa[2 * st * CI];
                    b[(c + 1) & 1][u] = sb[2 * st * LDB];
                }
            }
#pragma unroll
            for (int u = 0; u < SC_CH; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c & 1][u], b[c & 1][u], acc, 0, 0, 0);
        }
        if (kt + 1 < k1) store((it + 1) & 1);
        __syncthreads();
    }
    const int col = n0 + nt * 32 + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h2;
        if (row >= M) continue;
        if (p.splits > 1) {
            p.slab[((long)split * p.M + row) * p.N + col] = acc[r];
        } else {
            float *dst = p.C + (long)row * p.ldc + col;
            *dst = p.beta != 0.f ? acc[r] + p.beta * *dst : acc[r];
        }
    }
}

bool small_conv_ok(const ConvGeom &g, int mode, int lda) {
    (void)lda;
    if (mode != MODE_FWD && mode != MODE_WGRAD) return false;
    if (g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1)   // VGG19 block1_conv1 (forward only)
        return mode == MODE_FWD && g.Ci == 3 && g.Co % SC_BN == 0 && g.Wo % 32 == 0;
    return g.kh == 4 && g.kw == 4 && g.sh == 2 && g.sw == 2 && (g.Ci == 3 || g.Ci == 6) && g.Co % SC_BN == 0 &&
           g.Wo % 32 == 0;
}

// WGRAD splits: conv-view output rows per block so that ~2 blocks per CU run
int small_wgrad_rows_per_block(const ConvGeom &g) {
    const int rows = g.N * g.Ho, cols = g.Co / SC_BN;
    const int want = std::max(1, 512 / cols);
    return std::max(1, (rows + want - 1) / want);
}

template <int CI, int P, int KW = 4, int ST = 2>
static void launch_small(int mode, const GemmArgs &a, int rows_per_block, hipStream_t s) {
    const ConvGeom &g = a.g;
    if (mode == MODE_WGRAD) {
        if constexpr (KW == 4) {
            const int rows = g.N * g.Ho;
            const dim3 grid((unsigned)((rows + rows_per_block - 1) / rows_per_block), (unsigned)(g.Co / SC_BN));
            hipLaunchKernelGGL((k_small_wgrad<CI, P>), grid, dim3(128 * ((16 * CI + 31) / 32)), 0, s, a, rows_per_block);
        }
    } else {
        // persistent: as many blocks as are resident at once (a second partial round of
        // grid-stride blocks would leave most CUs idle at the tail)
        static int resident = 0;
        if (!resident) {
            int per_cu = 0, dev = 0, cus = 256;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_small_fwd<CI, P, true, KW, ST>, 128 * (P / 32),
                                                             0) != hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                cus = 256;
            resident = per_cu * cus;
        }
        const int ntiles = g.N * g.Ho * (g.Wo / P);
        const int cols = g.Co / SC_BN;
        const dim3 grid((unsigned)std::max(1, std::min(ntiles, resident / cols)), (unsigned)cols);
        if (a.mz || a.beta != 0.f) hipLaunchKernelGGL((k_small_fwd<CI, P, true, KW, ST>), grid, dim3(128 * (P / 32)), 0, s, a);
        else hipLaunchKernelGGL((k_small_fwd<CI, P, false, KW, ST>), grid, dim3(128 * (P / 32)), 0, s, a);
    }
}

void launch_small_conv(int mode, const GemmArgs &a, int rows_per_block, hipStream_t s) {
    const bool p64 = a.g.Wo % 64 == 0;
    if (a.g.kh == 3) {   // 3x3 stride 1, Ci 3 (small_conv_ok)
        if (p64) launch_small<3, 64, 3, 1>(mode, a, rows_per_block, s);
        else launch_small<3, 32, 3, 1>(mode, a, rows_per_block, s);
    } else if (a.g.Ci == 3) {
        if (p64) launch_small<3, 64>(mode, a, rows_per_block, s);
        else launch_small<3, 32>(mode, a, rows_per_block, s);
    } else {
        if (p64) launch_small<6, 64>(mode, a, rows_per_block, s);
        else launch_small<6, 32>(mode, a, rows_per_block, s);
    }
}

}  // namespace dg
