// bf16x6 split-precision implicit GEMM for the conv engine (gfx950).
//
// gfx950 runs v_mfma_f32_32x32x2_f32 at 1/16 of the bf16 matrix rate.  This
// kernel computes the same fp32 GEMMs as k_conv_gemm (conv.hip) on the bf16
// matrix cores: every fp32 operand is split exactly into three bf16 pieces,
//     x = hi + mid + lo          (RNE splits: |mid| <= 2^-9 |x|, |lo| <= 2^-18 |x|,
//                                  and the residual after lo is 0 for normal x)
// and each product a*b is formed from the six piece products whose magnitude
// is >= 2^-18 |a b|:
//     hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid
// The three dropped products (mid.lo, lo.mid, lo.lo) total < 2^-26 |a b|, below
// fp32's own rounding (2^-24); every bf16 x bf16 product is exact in the fp32
// MFMA accumulator.  So the result carries fp32 accuracy at 6/16 of the f32
// MFMA time per FLOP (tests/test_conv_gpu.py holds both paths to the same
// fp64-referenced tolerance).
//
// Tiling: WGM x WGN waves (4 or 8), block tile BM x BN x 16; each wave owns a
// (BM/WGM) x (BN/WGN) tile of 32x32 accumulators (v_mfma_f32_32x32x16_bf16).
// Operands are staged global -> registers and split into hi/mid/lo planes
// while being written to LDS:
//   KC operands (rows contiguous along k: FWD/DGRAD activations, DGRAD
//   weights): [plane][row][16 k] image, 32-byte rows whose two 16-byte halves
//   are XOR-swizzled by row bit 3; the 32x32x16 operand is one conflict-free
//   ds_read_b128 per lane.
//   RC operands (k-rows contiguous along the GEMM column: FWD weights, both
//   WGRAD operands): [plane][16 k][cols] image, stored as loaded (8-byte
//   writes of 4 columns) and transposed by the read -- two ds_read_b64_tr_b16
//   per operand (4 k-rows each); 16-dword blocks XOR-swizzled by k so the four
//   rows of one transposed read land on distinct banks.
// Double-buffered LDS, one barrier per K-tile, the MFMA chain split around
// the staging of the next tiles, as in k_conv_gemm.
#include "conv_impl.h"
#include <algorithm>

#ifndef DG_X6_SCHED
#define DG_X6_SCHED 1
#endif
#ifndef DG_X6_VPM
#define DG_X6_VPM 3
#endif

namespace dg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

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

// byte offset of bf16 element (row, kk) in a [rows][16] plane image
__device__ __forceinline__ int x6_off(int row, int kk) {
    return row * 32 + ((((kk >> 3) ^ (row >> 3)) & 1) << 4) + ((kk & 7) << 1);
}

// byte offset of bf16 element (k, col) in a [16][COLS] plane image (col even)
template <int COLS>
__device__ __forceinline__ int x6_rc_off(int k, int col) {
    constexpr int RW = COLS / 2;  // dwords per k-row
    const int swz = COLS >= 128 ? ((k & 3) << 4) : (((k >> 1) & 1) << 4);
    return 4 * (k * RW + ((col >> 1) ^ swz));
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 32x32x16 operand fragment (lane: column c0 + lane&31, k = 8(lane>>5) + 0..7)
// of an RC image, by two transposed reads
template <int COLS>
__device__ __forceinline__ bf16x8 x6_rc_frag(const char *plane, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int col = c0 + 16 * (g & 1) + 4 * pp;
    const int k = 8 * (g >> 1) + q;
    lds_s16x4 *p0 = (lds_s16x4 *)(plane + x6_rc_off<COLS>(k, col));
    lds_s16x4 *p1 = (lds_s16x4 *)(plane + x6_rc_off<COLS>(k + 4, col));
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Split pass: fp32 [rows][ld] (first C columns, C % 16 == 0) -> the packed
// bf16 plane layout of the bf16x6 GEMM: row r holds, per 16-column group j,
// hi[16] mid[16] lo[16] -- element (r, c) of plane p at r*3C + (c/16)*48 +
// 16p + c%16 -- so the three planes of one K-tile row are 96 contiguous bytes.
__global__ void __launch_bounds__(256)
k_split3(const float *__restrict__ src, int ld, long rows, int C, unsigned short *__restrict__ dst) {
    const int C8 = C >> 3;
    const long total = rows * C8;
    const bool vec = ((ld & 3) == 0) && ((((uintptr_t)src) & 15) == 0);
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const long r = e / C8;
        const int c = (int)(e - r * C8) * 8;
        const float *sp = src + r * ld + c;
        f32x4 v0, v1;
        if (vec) {
            v0 = *reinterpret_cast<const f32x4 *>(sp);
            v1 = *reinterpret_cast<const f32x4 *>(sp + 4);
        } else {
            v0 = f32x4{sp[0], sp[1], sp[2], sp[3]};
            v1 = f32x4{sp[4], sp[5], sp[6], sp[7]};
        }
        unsigned h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
        split3(v0[0], v0[1], h0, m0, l0);
        split3(v0[2], v0[3], h1, m1, l1);
        split3(v1[0], v1[1], h2, m2, l2);
        split3(v1[2], v1[3], h3, m3, l3);
        unsigned short *d = dst + r * 3 * C + (c >> 4) * 48 + (c & 8);
        *reinterpret_cast<u32x4 *>(d) = u32x4{h0, h1, h2, h3};
        *reinterpret_cast<u32x4 *>(d + 16) = u32x4{m0, m1, m2, m3};
        *reinterpret_cast<u32x4 *>(d + 32) = u32x4{l0, l1, l2, l3};
    }
}

// The GEMM.  A and B of GemmArgs point at the operands' packed bf16 planes
// (k_split3 output); lda / ldb are their column counts C (rows are 3C
// elements), a_bytes / b_bytes their extents.
template <int MODE, int BM, int BN, int WGM, int WGN, int MINW>
__global__ void __launch_bounds__(64 * WGM * WGN, MINW)
k_conv_gemm_x6(const GemmArgs p) {
    constexpr int BK = 16;
    constexpr bool A_KC = (MODE != MODE_WGRAD);
    constexpr bool B_KC = (MODE == MODE_DGRAD);
    constexpr int NT = 64 * WGM * WGN;  // threads
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    // bytes per plane tile; the 96-byte pad shifts plane p by 6p 16-byte bank
    // groups, so the 8 lanes of a ds_write_b128 group (chunks of 2 rows x 3
    // planes) land on distinct banks
    constexpr int APL = BM * 32 + 96, BPL = BN * 32 + 96;
    constexpr int BUF = 3 * (APL + BPL);            // bytes per buffer
    static_assert(WGM * WGN == 4 || WGM * WGN == 8, "4 or 8 waves");
    static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
    static_assert(BM % 32 == 0 && BN % 32 == 0 && BM <= 256 && BN <= 256, "tile");

    __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

    const ConvGeom &g = p.g;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid / WGN, wn = wid % WGN;
    const int l32 = lane & 31, h2 = lane >> 5;

    int zz, tile;
    xcd_remap(zz, tile);
    const int phase = zz / p.splits;
    const int split = zz - phase * p.splits;
    const int mt = tile / p.ntiles;
    const int nt = tile - mt * p.ntiles;
    const int m0 = mt * BM, n0 = nt * BN;

    int Mrows = p.M;
    PhaseInfo ph{};
    if constexpr (MODE == MODE_DGRAD) {
        ph = phase_info(g, phase, g.N);
        Mrows = ph.Mp;
        if (m0 >= Mrows) return;
    }
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    if (kbeg >= kend) return;
    const int nk = (kend - kbeg + BK - 1) / BK;

    // ---- loader geometry: 16-byte chunks (8 bf16 of one plane) ----
    // A row of a K-tile (KC) or 16 columns of a k-row (RC) is 6 chunks = 96
    // contiguous bytes: s = 2*plane + half.  KC tile: ROWS x 6 chunks; RC tile:
    // 16 k-rows x COLS/16 groups u x 6.  Either way 6*ROWS chunks, q = tid + NT*i.
    constexpr int A_CH = 6 * BM, B_CH = 6 * BN;
    constexpr int A_NI = (A_CH + NT - 1) / NT, B_NI = (B_CH + NT - 1) / NT;
    struct Chunk { int r, u, s; bool live; };
    auto kc_chunk = [](int q, int) { Chunk h; h.r = q / 6; h.u = 0; h.s = q - h.r * 6; return h; };
    auto rc_chunk = [](int q, int COLS) {
        Chunk h; const int per = 6 * (COLS / 16);
        h.r = q / per; int w = q - h.r * per; h.u = w / 6; h.s = w - h.u * 6; return h;
    };

    Chunk ach[A_NI], bch[B_NI];
#pragma unroll
    for (int i = 0; i < A_NI; ++i) {
        const int q = tid + NT * i;
        ach[i] = A_KC ? kc_chunk(q, BM) : rc_chunk(q, BM);
        ach[i].live = (A_CH % NT == 0) || q < A_CH;
    }
#pragma unroll
    for (int i = 0; i < B_NI; ++i) {
        const int q = tid + NT * i;
        bch[i] = B_KC ? kc_chunk(q, BN) : rc_chunk(q, BN);
        bch[i].live = (B_CH % NT == 0) || q < B_CH;
    }

    // KC A rows (FWD / DGRAD): output-pixel geometry of each chunk's row
    int arow_n[A_NI], arow_h[A_NI], arow_w[A_NI];
    // WGRAD A: (tap, ci) of each chunk's 8 columns
    int wg_i[A_NI], wg_j[A_NI], wg_ci[A_NI];
#pragma unroll
    for (int i = 0; i < A_NI; ++i) {
        arow_n[i] = -1; arow_h[i] = 0; arow_w[i] = 0; wg_i[i] = 0; wg_j[i] = 0; wg_ci[i] = 0;
        if constexpr (A_KC) {
            int m = m0 + ach[i].r;
            if (ach[i].live && m < Mrows) {
                if constexpr (MODE == MODE_FWD) {
                    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    arow_n[i] = n; arow_h[i] = ho * g.sh - g.pt; arow_w[i] = wo * g.sw - g.pl;
                } else {
                    // tap (a, b) of this phase reads dy[hh + ch - a][ww + cw - b]
                    // (exact: i = i0h + a*sh and ph + pt - i0h is a multiple of sh)
                    int ww = m % ph.Wp; int t = m / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                    arow_n[i] = n;
                    arow_h[i] = hh + (ph.ph + g.pt - ph.i0h) / g.sh;
                    arow_w[i] = ww + (ph.pw + g.pl - ph.i0w) / g.sw;
                }
            }
        } else {
            int mc = m0 + 16 * ach[i].u + 8 * (ach[i].s & 1);
            if (ach[i].live && mc < p.M) {
                arow_n[i] = 0;  // column valid
                int tap = mc / g.Ci; int ci = mc - tap * g.Ci; wg_i[i] = tap / g.kw; wg_j[i] = tap - wg_i[i] * g.kw;
                wg_ci[i] = (ci >> 4) * 48 + 16 * (ach[i].s >> 1) + (ci & 8);  // packed column offset
            }
        }
    }

    // K walk of FWD / DGRAD, channel-chunk-major: all taps (a, b) of one
    // 16-channel chunk, then the next chunk (see k_conv_gemm).  Kept as
    // wave-uniform counters advanced once per loaded K-tile.
    const int TA = MODE == MODE_FWD ? g.kh : g.Th, TB = MODE == MODE_FWD ? g.kw : g.Tw;
    int wk_a = 0, wk_b = 0, wk_chunk = 0;
    if constexpr (MODE != MODE_WGRAD) {
        int kk = kbeg / BK; wk_chunk = kk / (TA * TB); int t = kk - wk_chunk * TA * TB;
        wk_a = t / TB; wk_b = t - wk_a * TB;
    }
    auto walk_next = [&]() {
        if (++wk_b == TB) { wk_b = 0; if (++wk_a == TA) { wk_a = 0; ++wk_chunk; } }
    };

    const rsrc_t rA = make_rsrc((const float *)p.A, p.a_bytes);
    const rsrc_t rB = make_rsrc((const float *)p.B, p.b_bytes);
    auto bload16 = [](rsrc_t r, unsigned off) {
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    };

    u32x4 ra[A_NI], rb[B_NI];

    // WGRAD: output pixel -> (n, ho, wo) by multiply-shift division
    auto fdiv = [](unsigned n, unsigned mul, int shr) { return (__umulhi(n, mul) + n) >> shr; };

    auto load_tiles = [&](int k0) {
        // ----- A -----
        if constexpr (MODE == MODE_FWD) {
            const int i = wk_a, j = wk_b, ci0 = wk_chunk * BK;
#pragma unroll
            for (int q = 0; q < A_NI; ++q) {
                int hi = arow_h[q] + i, wi = arow_w[q] + j;
                bool ok = arow_n[q] >= 0 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                unsigned off = ((unsigned)((arow_n[q] * g.H + hi) * g.W + wi) * (3 * p.lda) + (ci0 >> 4) * 48 + 8 * ach[q].s) * 2u;
                ra[q] = bload16(rA, ok ? off : DG_OOB);
            }
        } else if constexpr (MODE == MODE_DGRAD) {
            const int i = ph.i0h + wk_a * g.sh, j = ph.i0w + wk_b * g.sw, co0 = wk_chunk * BK;
            const bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
            for (int q = 0; q < A_NI; ++q) {
                int ho = arow_h[q] - wk_a, wo = arow_w[q] - wk_b;
                bool ok = tapok && arow_n[q] >= 0 && (unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo;
                unsigned off = ((unsigned)((arow_n[q] * g.Ho + ho) * g.Wo + wo) * (3 * p.lda) + (co0 >> 4) * 48 + 8 * ach[q].s) * 2u;
                ra[q] = bload16(rA, ok ? off : DG_OOB);
            }
        } else {  // WGRAD: x gathered at each chunk's tap, k-rows are output pixels
#pragma unroll
            for (int q = 0; q < A_NI; ++q) {
                unsigned pix = (unsigned)(k0 + ach[q].r);
                unsigned t = fdiv(pix, p.mg_wo, p.sh_wo); int wo = (int)(pix - t * g.Wo);
                unsigned n = fdiv(t, p.mg_ho, p.sh_ho); int ho = (int)(t - n * g.Ho);
                int hi = ho * g.sh - g.pt + wg_i[q], wi = wo * g.sw - g.pl + wg_j[q];
                bool ok = arow_n[q] >= 0 && (int)pix < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                unsigned off = ((unsigned)(((int)n * g.H + hi) * g.W + wi) * (3 * p.lda) + wg_ci[q]) * 2u;
                ra[q] = bload16(rA, ok ? off : DG_OOB);
            }
        }
        // ----- B -----
        if constexpr (MODE == MODE_FWD) {  // w[k][co], k = (tap, ci)
            const int kr0 = (wk_a * g.kw + wk_b) * g.Ci + wk_chunk * BK;
#pragma unroll
            for (int q = 0; q < B_NI; ++q) {
                const int col = n0 + 16 * bch[q].u;
                const unsigned k = (unsigned)(kr0 + bch[q].r);
                const bool ok = bch[q].live && col < p.N;
                const unsigned off = (k * (3 * p.ldb) + (col >> 4) * 48 + 8 * bch[q].s) * 2u;
                rb[q] = bload16(rB, ok ? off : DG_OOB);
            }
        } else if constexpr (MODE == MODE_DGRAD) {  // w[i,j,ci,co]: rows ci contiguous along co
            const int i = ph.i0h + wk_a * g.sh, j = ph.i0w + wk_b * g.sw, co0 = wk_chunk * BK;
            const bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
            for (int q = 0; q < B_NI; ++q) {
                int ci = n0 + bch[q].r;
                bool ok = bch[q].live && tapok && ci < p.N;
                unsigned off = ((unsigned)((i * g.kw + j) * g.Ci + ci) * (3 * p.ldb) + (co0 >> 4) * 48 + 8 * bch[q].s) * 2u;
                rb[q] = bload16(rB, ok ? off : DG_OOB);
            }
        } else {  // WGRAD: dy rows (pixels) contiguous along co
#pragma unroll
            for (int q = 0; q < B_NI; ++q) {
                const int col = n0 + 16 * bch[q].u;
                const int pix = k0 + bch[q].r;
                const bool ok = bch[q].live && col < p.N && pix < kend;
                const unsigned off = ((unsigned)pix * (3 * p.ldb) + (col >> 4) * 48 + 8 * bch[q].s) * 2u;
                rb[q] = bload16(rB, ok ? off : DG_OOB);
            }
        }
        if constexpr (MODE != MODE_WGRAD) walk_next();
    };

    auto store_tiles = [&](int buf) {
        char *As = smem + buf * BUF;
        char *Bs = As + 3 * APL;
#pragma unroll
        for (int q = 0; q < A_NI; ++q) {
            if (!ach[q].live) continue;
            const int h = ach[q].s & 1;
            const int o = A_KC ? x6_off(ach[q].r, 8 * h) : x6_rc_off<BM>(ach[q].r, 16 * ach[q].u + 8 * h);
            *reinterpret_cast<u32x4 *>(As + (ach[q].s >> 1) * APL + o) = ra[q];
        }
#pragma unroll
        for (int q = 0; q < B_NI; ++q) {
            if (!bch[q].live) continue;
            const int h = bch[q].s & 1;
            const int o = B_KC ? x6_off(bch[q].r, 8 * h) : x6_rc_off<BN>(bch[q].r, 16 * bch[q].u + 8 * h);
            *reinterpret_cast<u32x4 *>(Bs + (bch[q].s >> 1) * BPL + o) = rb[q];
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    load_tiles(kbeg);
    store_tiles(0);
    if (nk > 1) load_tiles(kbeg + BK);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const char *As = smem + (kt & 1) * BUF;
        const char *Bs = As + 3 * APL;
        bf16x8 af[3][TM], bf[3][TN];
        // plane-major read order (hi, mid, lo), matching the MFMA order below,
        // so the first products wait only for the hi fragments
#pragma unroll
        for (int s = 0; s < 3; ++s) {
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                if constexpr (A_KC)
                    af[s][a] = *reinterpret_cast<const bf16x8 *>(As + s * APL + x6_off(wm * WTM + a * 32 + l32, 8 * h2));
                else
                    af[s][a] = x6_rc_frag<BM>(As + s * APL, wm * WTM + a * 32, lane);
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                if constexpr (B_KC)
                    bf[s][b] = *reinterpret_cast<const bf16x8 *>(Bs + s * BPL + x6_off(wn * WTN + b * 32 + l32, 8 * h2));
                else
                    bf[s][b] = x6_rc_frag<BN>(Bs + s * BPL, wn * WTN + b * 32, lane);
            }
        }
#if DG_X6_SCHED == 0
        __builtin_amdgcn_sched_barrier(0);
        // small products first, then the large ones
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][a], bf[0][b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[2][b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[1][b], acc[a][b], 0, 0, 0);
            }
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) store_tiles((kt & 1) ^ 1);
        if (kt + 2 < nk) load_tiles(kbeg + (kt + 2) * BK);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
            }
#else
        // One basic block: the staging of tiles kt+1 / kt+2 (buffer loads never
        // fault and the extra tiles past nk land in the idle LDS buffer, so it
        // runs unconditionally) is interleaved with the MFMA chain, a few
        // staging instructions in the shadow of each MFMA.
        store_tiles((kt & 1) ^ 1);
        load_tiles(kbeg + (kt + 2) * BK);
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            // hi.hi, mid.hi, hi.mid, mid.mid, lo.hi, hi.lo
            const int pa = s == 1 || s == 3 ? 1 : s == 4 ? 2 : 0;
            const int pb = s == 2 || s == 3 ? 1 : s == 5 ? 2 : 0;
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[pa][a], bf[pb][b], acc[a][b], 0, 0, 0);
        }
        constexpr int NMF = 6 * TM * TN;
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, DG_X6_VPM, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x004, 4, 0);  // SALU
            if (i % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
            if (i % 2 == 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
        }
#endif
        __syncthreads();
    }

    conv_epilogue<MODE, TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, Mrows, ph, phase, split, l32, h2);
}

void launch_split3(const float *src, int ld, long rows, int C, unsigned short *dst, hipStream_t s) {
    const long total = rows * (C / 8);
    if (total == 0) return;
    const unsigned blocks = (unsigned)std::min<long>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_split3, dim3(blocks), dim3(256), 0, s, src, ld, rows, C, dst);
}

// tile configs of the bf16x6 kernel (index = kX6Cfgs in conv.hip)
void launch_gemm_x6(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s) {
#define DG_X6(C, BM_, BN_, WM_, WN_, MW_)                                                                       \
    case C: {                                                                                                   \
        const dim3 blk(64 * WM_ * WN_);                                                                         \
        if (mode == MODE_FWD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_FWD, BM_, BN_, WM_, WN_, MW_>), grid, blk, 0, s, a); \
        else if (mode == MODE_DGRAD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_DGRAD, BM_, BN_, WM_, WN_, MW_>), grid, blk, 0, s, a); \
        else hipLaunchKernelGGL((k_conv_gemm_x6<MODE_WGRAD, BM_, BN_, WM_, WN_, MW_>), grid, blk, 0, s, a); \
        break;                                                                                                  \
    }
    switch (cfg) {
        DG_X6(0, 128, 128, 2, 2, 2)
        DG_X6(1, 128, 64, 2, 2, 2)
        DG_X6(2, 64, 128, 2, 2, 2)
        DG_X6(3, 64, 64, 2, 2, 3)
        DG_X6(4, 128, 128, 2, 2, 3)
        DG_X6(5, 256, 128, 4, 2, 2)
        DG_X6(6, 128, 256, 2, 4, 2)
        DG_X6(7, 256, 128, 2, 2, 2)
        DG_X6(8, 128, 256, 2, 2, 2)
    }
#undef DG_X6
}

}  // namespace dg
