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
// Operands arrive pre-split (k_split3 below, or caller-held planes): row r
// of a plane tensor holds, per 16-channel group, hi[16] mid[16] lo[16].
// Tiling: WGM x WGN waves (4 or 8), block tile BM x BN x 16 channels; each
// wave owns a (BM/WGM) x (BN/WGN) tile of 16x16 accumulators
// (v_mfma_f32_16x16x32_bf16, K = two 16-wide plane pieces).  K-tiles are
// staged global -> LDS by LDS-DMA (buffer_load ... lds, 1 KiB per wave
// instruction) into three buffers, two tiles in flight, one barrier per
// K-tile:
//   KC images (rows contiguous along k: FWD/DGRAD activations, DGRAD
//   weights): [plane][row][16 k], read as one ds_read_b128 per lane;
//   RC images (k-rows contiguous along the GEMM column: FWD weights, both
//   WGRAD operands): [plane][16 k][cols], XOR-swizzled by k and read
//   transposed (ds_read_b64_tr_b16).
// The epilogue is staged through LDS (conv_impl.h conv_epilogue16).
#include "conv_x6.h"
#include <algorithm>

namespace dg {

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

// Split pass of the fp16 conv math (DG_MATH_FP16, the reference's
// mixed_float16 policy): fp32 [rows][ld] -> fp16 [rows][C] (round to nearest
// even; beyond the fp16 range the value becomes inf, which the dynamic loss
// scale detects downstream).
__global__ void __launch_bounds__(256)
k_split_f16(const float *__restrict__ src, int ld, long rows, int C, _Float16 *__restrict__ dst) {
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
        f16x8 h;
#pragma unroll
        for (int q = 0; q < 4; ++q) { h[q] = (_Float16)v0[q]; h[4 + q] = (_Float16)v1[q]; }
        *reinterpret_cast<f16x8 *>(dst + r * C + c) = h;
    }
}

// The GEMM.  A and B of GemmArgs point at the operands' packed planes; lda /
// ldb are their column counts C, a_bytes / b_bytes their extents.
//   NI = 3 (DG_MATH_BF16X6): k_split3 planes, rows of 3C bf16, a K-tile is 16
//     channels whose three plane images feed three MFMAs (six piece products);
//   NI = 2 (DG_MATH_FP16): one fp16 plane, rows of C, a K-tile is 32 channels
//     (pixels for WGRAD) staged as two 16-wide images of one MFMA.
//   NI = 4 (DG_MATH_F16X3, common.h): fp16 h + l pieces of pre-scaled operands, a
//     K-tile is 32 channels (pixels) staged as four 16-wide images -- h and l of
//     k 0..15 and 16..31 -- feeding three MFMAs (h.h', l.h', h.l').  Activation /
//     gradient rows hold per 32-channel group h[32] l[32] (images 0,1 = h, 2,3 = l);
//     weight rows per 16-column group h[16] l[16]: as RC images (FWD) image i is
//     piece i>>1 of k-rows 16 (i&1) .., as KC images (DGRAD) images 0,2 = h, 1,3 = l.
// An operand row's K-chunk group holds 16 * NI elements in both layouts, so
// the KC images (k contiguous in memory) address identically; RC images
// (k-rows = GEMM rows of memory) take image i as plane i (NI = 3) or as the
// k-rows 16 i .. 16 i + 15 of the tile (NI = 2).
template <int MODE, int BM, int BN, int WGM, int WGN, int MINW, int NBUF = 3, int NI = 3>
__global__ void __launch_bounds__(64 * WGM * WGN, MINW)
k_conv_gemm_x6(const GemmArgs p) {
    static_assert(NBUF >= 2 && NBUF <= 4, "2 to 4 LDS buffers (1 to 3 K-tiles in flight)");
    static_assert(NI == 3 || NI == 2 || NI == 4, "bf16x6 (3 plane images), fp16 (2 chunk images), fp16x3 (4)");
    constexpr bool X6 = NI == 3;
    constexpr bool X3 = NI == 4;
    constexpr int BK = X6 ? 16 : 32;   // k per K-tile
    constexpr int GS = 16 * NI;        // elements of one K-chunk group in an operand row
    constexpr int RM = X6 ? 3 : (X3 ? 2 : 1);   // operand row = RM * C elements
    constexpr bool A_KC = (MODE != MODE_WGRAD);
    constexpr bool B_KC = (MODE == MODE_DGRAD);
    constexpr int NT = 64 * WGM * WGN;  // threads
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 16, TN = WTN / 16;  // 16x16 accumulator tiles per wave
    // bytes per plane tile; the 96-byte pad shifts plane p by 6p 16-byte bank
    // groups, so the 8 lanes of a ds_write_b128 group (chunks of 2 rows x 3
    // planes) land on distinct banks
    constexpr int APL = BM * 32 + 96, BPL = BN * 32 + 96;
    constexpr int BUF = NI * (APL + BPL);           // bytes per buffer
    constexpr int NW_ = WGM * WGN;
    static_assert(WGM * WGN == 4 || WGM * WGN == 8, "4 or 8 waves");
    static_assert(TM >= 1 && TN >= 1 && WTM % 16 == 0 && WTN % 16 == 0, "wave tile of 16x16 tiles");
    static_assert(BM % 32 == 0 && BN % 32 == 0 && BM <= 256 && BN <= 256, "tile");

    // three LDS buffers as separate objects: with the main loop unrolled by
    // three every DMA and every fragment read names its buffer statically, so
    // the compiler's LDS-DMA alias tracking does not drain the in-flight DMAs
    // of the other buffers before each read
    constexpr int STAGE = 16 * (WTN + 4);  // epilogue staging floats per wave (in smem0)
    constexpr int BUF0 = BUF > NW_ * STAGE * 4 ? BUF : NW_ * STAGE * 4;
    __shared__ __attribute__((aligned(16))) char smem0[BUF0];
    __shared__ __attribute__((aligned(16))) char smem1[BUF];
    __shared__ __attribute__((aligned(16))) char smem2[NBUF >= 3 ? BUF : 16];
    __shared__ __attribute__((aligned(16))) char smem3[NBUF == 4 ? BUF : 16];

    const ConvGeom &g = p.g;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WGN, wn = wid % WGN;
    const int l32 = lane & 31, h2 = lane >> 5;
    X3Pre x3s;   // (fp16x3: the scale sources, loaded here, combined in the epilogue)
    if constexpr (X3) x3s = x3_pre(p);

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

    // ---- LDS-DMA staging (buffer_load ... lds, 16 B per lane) ----
    // Each DMA instruction writes 1 KB of one plane image, lane L at byte 16L
    // (the destination is lane-linear); the swizzles of the images are
    // applied on the SOURCE side: lane L fetches the global 16-byte chunk that
    // belongs at its position.  Operand with X rows (KC) / X columns (RC) has
    // 3*X/32 such 1-KB slots per K-tile, dealt round-robin over the waves.
    constexpr int NW = WGM * WGN;
    constexpr int A_SL = NI * BM / 32, B_SL = NI * BN / 32;        // slots per tile
    constexpr int A_NJ = (A_SL + NW - 1) / NW, B_NJ = (B_SL + NW - 1) / NW;
    struct Slot { int plane, r, c; bool live; };  // KC: row r, half c; RC: k-row r, column c
    auto slot_of = [&](int d, bool kc, int X) __attribute__((always_inline)) {
        Slot sl; const int per = X / 32;  // 1-KB blocks per plane image
        sl.plane = d / per;
        const int pos = (d - sl.plane * per) * 1024 + 16 * lane;
        if (kc) {
            sl.r = pos >> 5;
            sl.c = (pos >> 4) & 1;
        } else {
            sl.r = pos / (2 * X);
            const int pdw = (pos - sl.r * 2 * X) >> 2;
            sl.c = 2 * (pdw ^ x6_rc_swz_cols(X, sl.r));
        }
        return sl;
    };
    Slot asl[A_NJ], bsl[B_NJ];
#pragma unroll
    for (int j = 0; j < A_NJ; ++j) {
        const int d = wid + NW * j;
        asl[j] = slot_of(d < A_SL ? d : 0, A_KC, BM);
        asl[j].live = d < A_SL;
    }
#pragma unroll
    for (int j = 0; j < B_NJ; ++j) {
        const int d = wid + NW * j;
        bsl[j] = slot_of(d < B_SL ? d : 0, B_KC, BN);
        bsl[j].live = d < B_SL;
    }
    // Every wave issues A_NJ + B_NJ DMAs per K-tile: when a slot count is not
    // a multiple of NW a wave's dead slots repeat slot 0's DMA (same source,
    // same LDS bytes, same data), so the DMA count and the s_waitcnt values
    // are compile-time, the K-tile body has no branches, and every DMA
    // provably targets the buffer being filled -- a DMA into some other LDS
    // object would make the compiler drain all DMAs (vmcnt(0)) before the
    // next fragment read.
    constexpr bool A_ALL = (A_SL % NW) == 0, B_ALL = (B_SL % NW) == 0;
    constexpr int NMINE = A_NJ + B_NJ;

    // A geometry per slot.  KC (FWD / DGRAD): the output pixel of row r.
    // WGRAD (RC): the (tap, ci) of columns c..c+7 and their packed offset.
    int arow_n[A_NJ], arow_h[A_NJ], arow_w[A_NJ];
    int wg_i[A_NJ], wg_j[A_NJ], wg_ci[A_NJ];
#pragma unroll
    for (int j = 0; j < A_NJ; ++j) {
        arow_n[j] = -1; arow_h[j] = 0; arow_w[j] = 0; wg_i[j] = 0; wg_j[j] = 0; wg_ci[j] = 0;
        if constexpr (A_KC) {
            int m = m0 + asl[j].r;
            if (m < Mrows) {
                if constexpr (MODE == MODE_FWD) {
                    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    arow_n[j] = n; arow_h[j] = ho * g.sh - g.pt; arow_w[j] = wo * g.sw - g.pl;
                } else {
                    // tap (a, b) of this phase reads dy[hh + ch - a][ww + cw - b]
                    // (exact: i = i0h + a*sh and ph + pt - i0h is a multiple of sh)
                    int ww = m % ph.Wp; int t = m / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                    arow_n[j] = n;
                    arow_h[j] = hh + (ph.ph + g.pt - ph.i0h) / g.sh;
                    arow_w[j] = ww + (ph.pw + g.pl - ph.i0w) / g.sw;
                }
            }
        } else {
            int mc = m0 + asl[j].c;
            if (mc < p.M) {
                arow_n[j] = 0;  // column valid
                int tap = mc / g.Ci; int ci = mc - tap * g.Ci; wg_i[j] = tap / g.kw; wg_j[j] = tap - wg_i[j] * g.kw;
                // packed column offset (fp16x3: piece plane>>1 of the 32-channel group)
                wg_ci[j] = X6 ? (ci >> 4) * 48 + 16 * asl[j].plane + (ci & 8)
                              : (X3 ? (ci >> 5) * 64 + 32 * (asl[j].plane >> 1) + (ci & 31) : ci);
            }
        }
    }

    // K walk of FWD / DGRAD, channel-chunk-major: all taps (a, b) of one
    // 16-channel chunk, then the next chunk (see k_conv_gemm).  Kept as
    // wave-uniform counters advanced once per issued K-tile.
    const int TA = MODE == MODE_FWD ? g.kh : g.Th, TB = MODE == MODE_FWD ? g.kw : g.Tw;
    int wk_a = 0, wk_b = 0, wk_chunk = 0;
    if constexpr (MODE != MODE_WGRAD) {
        int kk = kbeg / BK; wk_chunk = kk / (TA * TB); int t = kk - wk_chunk * TA * TB;
        wk_a = t / TB; wk_b = t - wk_a * TB;
    }
    // FWD / DGRAD: per-slot byte offsets at tap (0, 0) of chunk 0 plus a
    // bitmask of the taps whose source pixel lies inside the image, so the
    // K-tile issue is one add of a wave-uniform delta and one mask test per
    // slot (no per-tile index multiplies).
    int abase[A_NJ], amask[A_NJ], bbase[B_NJ];
    bool bok[B_NJ];
    if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
        for (int j = 0; j < A_NJ; ++j) {
            abase[j] = 0; amask[j] = 0;
            if (arow_n[j] < 0) continue;
            if constexpr (MODE == MODE_FWD) {
                abase[j] = (((arow_n[j] * g.H + arow_h[j]) * g.W + arow_w[j]) * (RM * p.lda) + 16 * asl[j].plane +
                            8 * asl[j].c) * 2;
                for (int a = 0; a < TA; ++a)
                    for (int b = 0; b < TB; ++b) {
                        const int hi = arow_h[j] + a, wi = arow_w[j] + b;
                        if ((unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W) amask[j] |= 1 << (a * TB + b);
                    }
            } else {
                abase[j] = (((arow_n[j] * g.Ho + arow_h[j]) * g.Wo + arow_w[j]) * (RM * p.lda) + 16 * asl[j].plane +
                            8 * asl[j].c) * 2;
                for (int a = 0; a < TA; ++a)
                    for (int b = 0; b < TB; ++b) {
                        const int i = ph.i0h + a * g.sh, jj = ph.i0w + b * g.sw;
                        const int ho = arow_h[j] - a, wo = arow_w[j] - b;
                        if (i < g.kh && jj < g.kw && (unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo)
                            amask[j] |= 1 << (a * TB + b);
                    }
            }
        }
#pragma unroll
        for (int j = 0; j < B_NJ; ++j) {
            if constexpr (MODE == MODE_FWD) {  // RC weights: k-row r, columns c..c+7
                const int col = n0 + bsl[j].c;
                bok[j] = col < p.N;
                bbase[j] = X6 ? (bsl[j].r * (3 * p.ldb) + (col >> 4) * 48 + 16 * bsl[j].plane + (col & 8)) * 2
                         : X3 ? ((bsl[j].r + 16 * (bsl[j].plane & 1)) * (2 * p.ldb) + (col >> 4) * 32 +
                                 16 * (bsl[j].plane >> 1) + (col & 8)) * 2
                              : ((bsl[j].r + 16 * bsl[j].plane) * p.ldb + col) * 2;
            } else {                           // KC weights: row ci
                const int ci = n0 + bsl[j].r;
                bok[j] = ci < p.N;
                bbase[j] = (ci * (RM * p.ldb) + 16 * bsl[j].plane + 8 * bsl[j].c) * 2;
            }
        }
    }
    auto walk_next = [&]() __attribute__((always_inline)) {  // branch-free (selects)
        const int nb = wk_b + 1;
        const bool wb = nb == TB;
        const int na = wk_a + (wb ? 1 : 0);
        const bool wa = na == TA;
        wk_b = wb ? 0 : nb;
        wk_a = wa ? 0 : na;
        wk_chunk += wa ? 1 : 0;
    };

    const rsrc4_t rA = make_rsrc4(p.A, p.a_bytes);
    const rsrc4_t rB = make_rsrc4(p.B, p.b_bytes);
    auto dma = [](rsrc4_t r, char *lds_base, unsigned off) __attribute__((always_inline)) { dma16(r, lds_base, off); };
    // WGRAD: output pixel -> (n, ho, wo) by multiply-shift division
    auto fdiv = [](unsigned n, unsigned mul, int shr) __attribute__((always_inline)) { return (__umulhi(n, mul) + n) >> shr; };

    // issue the DMA of the K-tile at k0 (the walker's tile) into LDS buffer sm
    auto issue_tile = [&](int k0, char *sm) __attribute__((always_inline)) {
        char *As = sm;
        char *Bs = As + NI * APL;
        // wave-uniform parts of this K-tile's offsets (tap (wk_a, wk_b) of chunk wk_chunk)
        int a_delta = 0, b_delta = 0, tap_bit = 0;
        bool b_tap_ok = true;
        if constexpr (MODE == MODE_FWD) {
            a_delta = ((wk_a * g.W + wk_b) * (RM * p.lda) + wk_chunk * GS) * 2;
            b_delta = (((wk_a * g.kw + wk_b) * g.Ci + wk_chunk * BK) * (RM * p.ldb)) * 2;
            tap_bit = wk_a * TB + wk_b;
        } else if constexpr (MODE == MODE_DGRAD) {
            a_delta = (wk_chunk * GS - (wk_a * g.Wo + wk_b) * (RM * p.lda)) * 2;
            const int i = ph.i0h + wk_a * g.sh, jj = ph.i0w + wk_b * g.sw;
            b_tap_ok = i < g.kh && jj < g.kw;
            b_delta = ((b_tap_ok ? (i * g.kw + jj) * g.Ci * (RM * p.ldb) : 0) + wk_chunk * GS) * 2;
            tap_bit = wk_a * TB + wk_b;
        }
        (void)a_delta; (void)b_delta; (void)tap_bit; (void)b_tap_ok;
        // a tile past this block's K range (the pipeline's tail) is issued out of range:
        // same DMA count, zeros, no memory traffic (WGRAD tests pix < kend per row)
        const bool live = MODE == MODE_WGRAD || k0 < kend;
#pragma unroll
        for (int j = 0; j < A_NJ; ++j) {
            const int d = asl[j].live ? wid + NW * j : 0, per = BM / 32;
            char *dst = As + asl[j].plane * APL + (d - asl[j].plane * per) * 1024;
            unsigned off;
            bool ok;
            if constexpr (MODE != MODE_WGRAD) {
                ok = (amask[j] >> tap_bit) & 1;
                off = (unsigned)(abase[j] + a_delta);
            } else {
                const unsigned pix = (unsigned)(k0 + asl[j].r + (X6 ? 0 : 16 * (X3 ? asl[j].plane & 1 : asl[j].plane)));
                const unsigned t = fdiv(pix, p.mg_wo, p.sh_wo); const int wo = (int)(pix - t * g.Wo);
                const unsigned n = fdiv(t, p.mg_ho, p.sh_ho); const int ho = (int)(t - n * g.Ho);
                const int hi = ho * g.sh - g.pt + wg_i[j], wi = wo * g.sw - g.pl + wg_j[j];
                ok = arow_n[j] >= 0 && (int)pix < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                off = ((unsigned)(((int)n * g.H + hi) * g.W + wi) * (RM * p.lda) + wg_ci[j]) * 2u;
            }
            dma(rA, dst, ok && live ? off : DG_OOB);
        }
#pragma unroll
        for (int j = 0; j < B_NJ; ++j) {
            const int d = bsl[j].live ? wid + NW * j : 0, per = BN / 32;
            char *dst = Bs + bsl[j].plane * BPL + (d - bsl[j].plane * per) * 1024;
            unsigned off;
            bool ok;
            if constexpr (MODE == MODE_FWD) {  // w[k][co], k = (tap, ci); RC: k-row r, columns c..c+7
                ok = bok[j];
                off = (unsigned)(bbase[j] + b_delta);
            } else if constexpr (MODE == MODE_DGRAD) {  // w[i,j,ci,co]: KC rows ci
                ok = bok[j] && b_tap_ok;
                off = (unsigned)(bbase[j] + b_delta);
            } else {  // WGRAD: dy rows (pixels) contiguous along co
                const int col = n0 + bsl[j].c;
                const int pix = k0 + bsl[j].r + (X6 ? 0 : 16 * (X3 ? bsl[j].plane & 1 : bsl[j].plane));
                ok = col < p.N && pix < kend;
                off = X6 ? ((unsigned)pix * (3 * p.ldb) + (col >> 4) * 48 + 16 * bsl[j].plane + (col & 8)) * 2u
                    : X3 ? ((unsigned)pix * (2 * p.ldb) + (col >> 5) * 64 + 32 * (bsl[j].plane >> 1) + (col & 31)) * 2u
                         : ((unsigned)pix * p.ldb + col) * 2u;
            }
            dma(rB, dst, ok && live ? off : DG_OOB);
        }
        if constexpr (MODE != MODE_WGRAD) walk_next();
    };
    // barrier without the vmcnt(0) drain of __syncthreads (DMAs stay in flight)
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Fragments of one K-tile for v_mfma_f32_16x16x32_bf16 with the 32-wide K
    // = two 16-wide plane pieces:  A [hi|mid], [hi|lo];  B [hi;mid], [mid;hi],
    // [lo;hi].  Per 16x16 tile three MFMAs then sum all six piece products:
    //   [hi|mid].[hi;mid] = hi.hi + mid.mid,  [hi|mid].[mid;hi] = hi.mid + mid.hi,
    //   [hi|lo].[lo;hi]   = hi.lo + lo.hi.
    // fp16 (NI = 2): A [k0..15 | k16..31], B [k0..15; k16..31], one
    // v_mfma_f32_16x16x32_f16 per 16x16 tile.
    auto frag = [&](const char *p0, const char *p1, int rc0, bool kc, bool is_a) __attribute__((always_inline)) {
        if (kc) return x6_kc_frag(p0, p1, rc0, lane);
        return is_a ? x6_rc_frag<BM>(p0, p1, rc0, lane) : x6_rc_frag<BN>(p0, p1, rc0, lane);
    };
    auto read_frags = [&](const char *sm, bf16x8 (&ahm)[TM], bf16x8 (&ahl)[TM], bf16x8 (&b1)[TN],
                          bf16x8 (&b2)[TN], bf16x8 (&b3)[TN]) __attribute__((always_inline)) {
        const char *A0 = sm, *A1 = sm + APL, *A2 = sm + (NI - 1) * APL;
        const char *B0 = sm + NI * APL, *B1 = B0 + BPL, *B2 = B0 + (NI - 1) * BPL;
#pragma unroll
        for (int a = 0; a < TM; ++a) {
            const int r0 = wm * WTM + a * 16;
            ahm[a] = frag(A0, A1, r0, A_KC, true);
            if constexpr (X6) ahl[a] = frag(A0, A2, r0, A_KC, true);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int c0 = wn * WTN + b * 16;
            b1[b] = frag(B0, B1, c0, B_KC, false);
            if constexpr (X6) {
                b2[b] = frag(B1, B0, c0, B_KC, false);
                b3[b] = frag(B2, B0, c0, B_KC, false);
            }
        }
    };

    // NBUF LDS buffers, AHEAD = NBUF-1 K-tiles in flight: iteration kt reads
    // the fragments of tile kt, issues the DMA of tile kt+AHEAD into the
    // buffer tile kt-1 used (every wave passed the barrier after reading it),
    // runs the MFMAs of tile kt, then waits until only the DMAs of tiles
    // kt+2 .. kt+AHEAD are outstanding and crosses the barrier.  DMAs past nk
    // fetch harmless data into idle buffers.
    constexpr int AHEAD = NBUF - 1;
    // MIDB: tile kt+NBUF goes into the buffer tile kt has just read into
    // registers (a second barrier per K-tile marks it free), so a DMA has NBUF
    // K-tiles of MFMAs to land instead of NBUF-1 (fp16x3 two-buffer tiles: 870
    // -> 919 img/s pix2pix; bf16x6 / fp16: SRGAN 4175 -> 4227).  DG_NO_MIDB
    // builds the plain pipeline, DG_MIDB_X3 the fp16x3-only form, for A/B runs
#if defined(DG_NO_MIDB)
    constexpr bool MIDB = false;
#elif defined(DG_MIDB_X3)
    constexpr bool MIDB = X3;
#else
    constexpr bool MIDB = true;
#endif
    constexpr int DIST = MIDB ? NBUF : AHEAD;
    auto ktile = [&](int kt, const char *cur, char *nxt) __attribute__((always_inline)) {
        if constexpr (X3) {
            // fp16x3: A [h | h'] / [l | l'] of k 0..15 | 16..31; B the same pairs (KC
            // weights of DGRAD: images 0,2 = h, 1,3 = l); h.h', l.h', h.l'
            f16x8 ah[TM], al[TM], bh[TN], bl[TN];
            const char *B0 = cur + 4 * APL;
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const int r0 = wm * WTM + a * 16;
                ah[a] = __builtin_bit_cast(f16x8, frag(cur, cur + APL, r0, A_KC, true));
                al[a] = __builtin_bit_cast(f16x8, frag(cur + 2 * APL, cur + 3 * APL, r0, A_KC, true));
            }
            constexpr int BH1 = B_KC ? 2 : 1, BL0 = B_KC ? 1 : 2;
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int c0 = wn * WTN + b * 16;
                bh[b] = __builtin_bit_cast(f16x8, frag(B0, B0 + BH1 * BPL, c0, B_KC, false));
                bl[b] = __builtin_bit_cast(f16x8, frag(B0 + BL0 * BPL, B0 + 3 * BPL, c0, B_KC, false));
            }
            if constexpr (MIDB) {
                barrier();
                issue_tile(kbeg + (kt + DIST) * BK, const_cast<char *>(cur));
            } else {
                issue_tile(kbeg + (kt + AHEAD) * BK, nxt);
            }
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
            wait_dma_c<(DIST - 1) * NMINE>();
            barrier();
            return;
        }
        bf16x8 ahm[TM], ahl[X6 ? TM : 1], b1[TN], b2[X6 ? TN : 1], b3[X6 ? TN : 1];
        if constexpr (X6) {
            read_frags(cur, ahm, ahl, b1, b2, b3);
        } else {
            bf16x8 dA[TM], dB[TN];
            read_frags(cur, ahm, dA, b1, dB, dB);
        }
        if constexpr (MIDB) {
            barrier();
            issue_tile(kbeg + (kt + DIST) * BK, const_cast<char *>(cur));
        } else {
            issue_tile(kbeg + (kt + AHEAD) * BK, nxt);
        }
        if constexpr (X6) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm[a], b1[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm[a], b2[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahl[a], b3[b], acc[a][b], 0, 0, 0);
        } else {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ahm[a]),
                                                                       __builtin_bit_cast(f16x8, b1[b]), acc[a][b],
                                                                       0, 0, 0);
        }
        wait_dma_c<(DIST - 1) * NMINE>();
        barrier();
    };
    auto pipeline = [&](char *L0, char *L1, char *L2, char *L3) __attribute__((always_inline)) {
        // the first DIST tiles (MIDB: one per buffer)
        issue_tile(kbeg, L0);
        if constexpr (DIST >= 2) issue_tile(kbeg + BK, L1);
        if constexpr (DIST >= 3) issue_tile(kbeg + 2 * BK, L2);
        if constexpr (DIST >= 4) issue_tile(kbeg + 3 * BK, L3);
        wait_dma_c<(DIST - 1) * NMINE>();
        barrier();
        int kt = 0;
        if constexpr (NBUF == 2) {
            // one K-tile ahead: tile kt+1 lands in the buffer tile kt-1 used while
            // the MFMAs of tile kt run
            for (; kt + 1 < nk; kt += 2) {
                ktile(kt, L0, L1);
                ktile(kt + 1, L1, L0);
            }
            if (kt < nk) ktile(kt, L0, L1);
        } else if constexpr (NBUF == 3) {
            for (; kt + 2 < nk; kt += 3) {
                ktile(kt, L0, L2);
                ktile(kt + 1, L1, L0);
                ktile(kt + 2, L2, L1);
            }
            if (kt < nk) ktile(kt, L0, L2);
            if (kt + 1 < nk) ktile(kt + 1, L1, L0);
        } else {
            for (; kt + 3 < nk; kt += 4) {
                ktile(kt, L0, L3);
                ktile(kt + 1, L1, L0);
                ktile(kt + 2, L2, L1);
                ktile(kt + 3, L3, L2);
            }
            if (kt < nk) ktile(kt, L0, L3);
            if (kt + 1 < nk) ktile(kt + 1, L1, L0);
            if (kt + 2 < nk) ktile(kt + 2, L2, L1);
        }
    };
    pipeline(smem0, smem1, smem2, smem3);

    // every wave's DMAs (including the harmless ones past nk) have landed
    // before smem0 becomes the epilogue's staging area
    wait_dma_c<0>();
    barrier();
    float ys_pre = 0.f;
    if constexpr (X3) {   // undo the operand scales (powers of two: exact)
        const float osc = x3_out_scale(p, x3s);
        ys_pre = p.yp ? x3_raw_scale(x3s.y, F16X3_XS) : 0.f;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) acc[a][b] *= osc;
    }
    static_assert(NW * STAGE * 4 <= BUF0, "epilogue staging fits in LDS buffer 0");
    // GEMM row -> output pixel (DGRAD: the phase's sub-grid; unit stride and
    // FWD / WGRAD rows are pixels / filter rows); slab rows are GEMM rows
    const bool ident = MODE != MODE_DGRAD || (g.sh == 1 && g.sw == 1);
    auto rowmap = [&](int row) __attribute__((always_inline)) -> RowPix {
        if (row >= Mrows) return RowPix{-1, -1};
        long pix = row;
        if constexpr (MODE == MODE_DGRAD) {
            if (!ident && p.splits == 1) {
                int ww = row % ph.Wp; int t = row / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                pix = (long)(n * g.H + hh * g.sh + ph.ph) * g.W + ww * g.sw + ph.pw;
            }
        }
        return RowPix{row, pix};
    };
    conv_epilogue16<MODE, TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, rowmap, phase, split, lane,
                                  reinterpret_cast<float *>(smem0) + wid * STAGE, ys_pre);
}

void launch_split3(const float *src, int ld, long rows, int C, unsigned short *dst, hipStream_t s) {
    const long total = rows * (C / 8);
    if (total == 0) return;
    const unsigned blocks = (unsigned)std::min<long>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_split3, dim3(blocks), dim3(256), 0, s, src, ld, rows, C, dst);
}

// Split pass of the fp16x3 forward operands (common.h): fp32 [rows][ld] (first C
// columns) -> per group of G columns h[G] l[G] of scale * value, 8 columns per lane
template <int G>
__global__ void __launch_bounds__(256)
k_split_x3(const float *__restrict__ src, int ld, long rows, int C, float scale, const float *sm, const float *sg,
           const float *sc, _Float16 *__restrict__ dst) {
    if (sm) scale = x3_grad_scale(sm, sg, sc);   // a bound-scaled operand: scale from its source
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
        f16x8 h, l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            _Float16 a, b;
            split_x3(v0[q], scale, a, b);
            h[q] = a; l[q] = b;
            split_x3(v1[q], scale, a, b);
            h[4 + q] = a; l[4 + q] = b;
        }
        _Float16 *d = dst + r * 2 * C + (c / G) * (2 * G) + (c % G);
        *reinterpret_cast<f16x8 *>(d) = h;
        *reinterpret_cast<f16x8 *>(d + G) = l;
    }
}

void launch_split_x3(const float *src, int ld, long rows, int C, void *dst, int group, float scale, hipStream_t s,
                     const float *sm, const float *sg, const float *sc) {
    const long total = rows * (C / 8);
    if (total == 0) return;
    const unsigned blocks = (unsigned)std::min<long>((total + 255) / 256, 8192);
    if (group == 32)
        hipLaunchKernelGGL(k_split_x3<32>, dim3(blocks), dim3(256), 0, s, src, ld, rows, C, scale, sm, sg, sc,
                           (_Float16 *)dst);
    else
        hipLaunchKernelGGL(k_split_x3<16>, dim3(blocks), dim3(256), 0, s, src, ld, rows, C, scale, sm, sg, sc,
                           (_Float16 *)dst);
}

// max |x| over [rows][ld] (first C columns) into *out (atomicMax; the caller zeroes it); a dense
// tensor (ld == C, 16-byte aligned) is read as one flat float4 array
__global__ void __launch_bounds__(256) k_absmax(const float *__restrict__ x, long rows, int C, int ld, float *out) {
    float m = 0.f;
    const long total = rows * C;
    if (ld == C && ((((uintptr_t)x) & 15) == 0)) {
        const long t4 = total >> 2;
        const long st = (long)gridDim.x * blockDim.x;
        long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
        auto m4 = [](f32x4 v) { return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))); };
        for (; e + 3 * st < t4; e += 4 * st) {   // (four loads in flight per lane)
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = reinterpret_cast<const f32x4 *>(x)[e + u * st];
#pragma unroll
            for (int u = 0; u < 4; ++u) m = fmaxf(m, m4(v[u]));
        }
        for (; e < t4; e += st) m = fmaxf(m, m4(reinterpret_cast<const f32x4 *>(x)[e]));
        for (long e = (t4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
             e += (long)gridDim.x * blockDim.x)
            m = fmaxf(m, fabsf(x[e]));
    } else {
        for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
            const long r = e / C;
            m = fmaxf(m, fabsf(x[r * ld + (e - r * C)]));
        }
    }
    block_atomic_absmax(out, m);
}

// forward bound of a conv's output (dg_conv_set_act_scale y_g / y_c): gout[0] = max over the
// Co columns of sum over the K rows of |w[k][co]| (HWIO kernels: K = kh*kw*Cin), cout[0] =
// max |bias| (0 without one); zero8 (may be NULL): 8 floats zeroed for a following absmax.
// One workgroup: 64 columns at a time, 4 row lanes per column, rows summed 8 loads at a time
// (the small-Cin layers per step -- K 48 / 96 -- and the frozen VGG19 once per weight version)
__global__ void __launch_bounds__(256) k_weight_bound(const float *__restrict__ w, long K, int Co,
                                                     const float *__restrict__ bias, float *gout, float *cout,
                                                     float *zero8) {
    __shared__ float red[256];
    if (zero8 && threadIdx.x < X3_SHARDS) zero8[threadIdx.x * X3_SHARD_STRIDE] = 0.f;
    const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
    float g = 0.f, c = 0.f;
    for (int c0 = 0; c0 < Co; c0 += 64) {
        const int co = c0 + cl;
        float sum = 0.f;
        if (co < Co) {
            long k = rl;
            for (; k + 28 < K; k += 32) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = w[(k + 4 * u) * Co + co];
#pragma unroll
                for (int u = 0; u < 8; ++u) sum += fabsf(v[u]);
            }
            for (; k < K; k += 4) sum += fabsf(w[k * Co + co]);
            if (bias && rl == 0) c = fmaxf(c, fabsf(bias[co]));
        }
        red[threadIdx.x] = sum;
        __syncthreads();
        if (rl == 0) g = fmaxf(g, red[cl] + red[64 + cl] + red[128 + cl] + red[192 + cl]);
        __syncthreads();
    }
    red[threadIdx.x] = g;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 64; ++i) g = fmaxf(g, red[i]);
        gout[0] = g;
    }
    __syncthreads();
    red[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x == 0 && cout) {
        for (int i = 1; i < 64; ++i) c = fmaxf(c, red[i]);
        cout[0] = c;
    }
}

// The same bound over a large kernel (the frozen VGG19's 3x3 layers, once per weight version:
// up to 627 us as one workgroup): workgroup b sums the 16 columns 16b.. over all K rows (16 row
// lanes per column, four loads in flight, the lanes combined in a fixed order), and its max goes
// to gout[0] by an integer atomicMax -- non-negative floats order as their bits, so the result is
// exact and independent of the order the workgroups finish in.  gout[0] is zeroed before the launch
// (launch_weight_bound); workgroup 0 also writes cout and zeroes zero8.
__global__ void __launch_bounds__(256) k_weight_bound_cols(const float *__restrict__ w, long K, int Co,
                                                          const float *__restrict__ bias, float *gout, float *cout,
                                                          float *zero8) {
    __shared__ float red[256];
    if (blockIdx.x == 0 && zero8 && threadIdx.x < X3_SHARDS) zero8[threadIdx.x * X3_SHARD_STRIDE] = 0.f;
    const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int co = blockIdx.x * 16 + cl;
    float sum = 0.f;
    if (co < Co) {
        long k = rl;
        for (; k + 48 < K; k += 64) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = w[(k + 16 * u) * Co + co];
#pragma unroll
            for (int u = 0; u < 4; ++u) sum += fabsf(v[u]);
        }
        for (; k < K; k += 16) sum += fabsf(w[k * Co + co]);
    }
    red[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x < 16) {
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += red[16 * r + threadIdx.x];
        red[threadIdx.x] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float g = 0.f;
        for (int i = 0; i < 16; ++i) g = fmaxf(g, red[i]);
        atomicMax(reinterpret_cast<unsigned *>(gout), __float_as_uint(g));
        if (blockIdx.x == 0 && cout) {
            float c = 0.f;
            if (bias)
                for (int i = 0; i < Co; ++i) c = fmaxf(c, fabsf(bias[i]));
            cout[0] = c;
        }
    }
}

// The input-gradient bound of a conv (dg_weight_bound_in): gout[0] = max over input channels ci of
// sum over taps and output channels of |w[tap][ci][co]| (HWIO), >= max |dx| / max |dy|.  One
// workgroup per ci, a fixed-order LDS tree per workgroup, the workgroups' maxima by integer
// atomicMax into gout[0] (zeroed before the launch).
__global__ void __launch_bounds__(256) k_weight_bound_in(const float *__restrict__ w, int taps, int Ci, int Co,
                                                        float *gout) {
    __shared__ float red[256];
    const int ci = blockIdx.x;
    float s = 0.f;
    for (int t = 0; t < taps; ++t) {
        const float *row = w + ((long)t * Ci + ci) * Co;
        for (int co = threadIdx.x; co < Co; co += 256) s += fabsf(row[co]);
    }
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned *>(gout), __float_as_uint(red[0]));
}

// one workgroup while the kernel is small (the trainable down1 layers' per-step bounds: K 48 / 96,
// Co 64 -- a memset node would cost more than the read), the column-parallel form beyond
constexpr long WBOUND_ONE_BLOCK_MAX = 1 << 16;

void launch_weight_bound(const float *w, long K, int Co, const float *bias, float *gout, float *cout, hipStream_t s,
                         float *zero8) {
    if (K * Co <= WBOUND_ONE_BLOCK_MAX) {
        hipLaunchKernelGGL(k_weight_bound, dim3(1), dim3(256), 0, s, w, K, Co, bias, gout, cout, zero8);
        return;
    }
    hipMemsetAsync(gout, 0, sizeof(float), s);
    hipLaunchKernelGGL(k_weight_bound_cols, dim3((Co + 15) / 16), dim3(256), 0, s, w, K, Co, bias, gout, cout, zero8);
}

void launch_weight_bound_in(const float *w, int taps, int Ci, int Co, float *gout, hipStream_t s) {
    hipMemsetAsync(gout, 0, sizeof(float), s);
    hipLaunchKernelGGL(k_weight_bound_in, dim3(Ci), dim3(256), 0, s, w, taps, Ci, Co, gout);
}

void launch_absmax(const float *x, long rows, int C, int ld, float *out, hipStream_t s) {
    const long total = rows * C;
    if (total == 0) return;
    const unsigned blocks = (unsigned)std::min<long>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(k_absmax, dim3(blocks), dim3(256), 0, s, x, rows, C, ld, out);
}

// both operands of one fp16 GEMM in one launch (blocks [0, nba) convert A, the rest B):
// the SR family's mixed_float16 steps run hundreds of small GEMMs, where each conversion
// launch costs about its launch latency (SRGAN: 368 per step, 17% of the step)
struct F16Split {
    const float *src;
    int ld;
    long rows;
    int C;
    _Float16 *dst;
};
__global__ void __launch_bounds__(256) k_split_f16_pair(F16Split a, F16Split b, unsigned nba) {
    const bool first = blockIdx.x < nba;
    const F16Split d = first ? a : b;
    const unsigned bid = first ? blockIdx.x : blockIdx.x - nba, nb = first ? nba : gridDim.x - nba;
    const int C8 = d.C >> 3;
    const long total = d.rows * C8;
    const bool vec = ((d.ld & 3) == 0) && ((((uintptr_t)d.src) & 15) == 0);
    for (long e = (long)bid * blockDim.x + threadIdx.x; e < total; e += (long)nb * blockDim.x) {
        const long r = e / C8;
        const int c = (int)(e - r * C8) * 8;
        const float *sp = d.src + r * d.ld + c;
        f32x4 v0, v1;
        if (vec) {
            v0 = *reinterpret_cast<const f32x4 *>(sp);
            v1 = *reinterpret_cast<const f32x4 *>(sp + 4);
        } else {
            v0 = f32x4{sp[0], sp[1], sp[2], sp[3]};
            v1 = f32x4{sp[4], sp[5], sp[6], sp[7]};
        }
        f16x8 h;
#pragma unroll
        for (int q = 0; q < 4; ++q) { h[q] = (_Float16)v0[q]; h[4 + q] = (_Float16)v1[q]; }
        *reinterpret_cast<f16x8 *>(d.dst + r * d.C + c) = h;
    }
}

void launch_split_f16_pair(const float *a, int lda, long ra, int ca, void *da, const float *b, int ldb, long rb,
                           int cb, void *db, hipStream_t s) {
    const long ta = ra * (ca / 8), tb = rb * (cb / 8);
    const unsigned nba = (unsigned)std::max<long>(1, std::min<long>((ta + 255) / 256, 4096));
    const unsigned nbb = (unsigned)std::max<long>(1, std::min<long>((tb + 255) / 256, 4096));
    hipLaunchKernelGGL(k_split_f16_pair, dim3(nba + nbb), dim3(256), 0, s, F16Split{a, lda, ra, ca, (_Float16 *)da},
                       F16Split{b, ldb, rb, cb, (_Float16 *)db}, nba);
}

void launch_split_f16(const float *src, int ld, long rows, int C, void *dst, hipStream_t s) {
    const long total = rows * (C / 8);
    if (total == 0) return;
    const unsigned blocks = (unsigned)std::min<long>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_split_f16, dim3(blocks), dim3(256), 0, s, src, ld, rows, C, (_Float16 *)dst);
}

// tile configs of the bf16x6 (ni 3) and fp16 (ni 2) kernels (index = kX6Cfgs / kF16Cfgs in conv.hip)
template <int NI>
static void launch_gemm_planes(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s) {
#define DG_X6(C, BM_, BN_, WM_, WN_, MW_, NB_)                                                                  \
    case C: {                                                                                                   \
        const dim3 blk(64 * WM_ * WN_);                                                                         \
        if (mode == MODE_FWD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_FWD, BM_, BN_, WM_, WN_, MW_, NB_, NI>), grid, blk, 0, s, a); \
        else if (mode == MODE_DGRAD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_DGRAD, BM_, BN_, WM_, WN_, MW_, NB_, NI>), grid, blk, 0, s, a); \
        else hipLaunchKernelGGL((k_conv_gemm_x6<MODE_WGRAD, BM_, BN_, WM_, WN_, MW_, NB_, NI>), grid, blk, 0, s, a); \
        break;                                                                                                  \
    }
    switch (cfg) {
        DG_X6(0, 128, 128, 2, 2, 2, 3)
        DG_X6(1, 128, 64, 2, 2, 2, 3)
        DG_X6(2, 64, 128, 2, 2, 2, 3)
        DG_X6(3, 64, 64, 2, 2, 3, 3)
        DG_X6(4, 256, 128, 4, 2, 2, 3)
        DG_X6(5, 128, 256, 2, 4, 2, 3)
        DG_X6(6, 128, 32, 4, 1, 3, 3)
    }
#undef DG_X6
}

void launch_gemm_x6(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s) {
    launch_gemm_planes<3>(mode, cfg, grid, a, s);
}

void launch_gemm_f16(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s) {
    launch_gemm_planes<2>(mode, cfg, grid, a, s);
}

// fp16x3 tile configs (index = kX3Cfgs in conv.hip): four 16-wide images per K-tile of
// 32, so the 128-wide tiles keep one K-tile ahead in two LDS buffers (67 KB at 128 x 128:
// two blocks per CU), the narrow ones two ahead in three
void launch_gemm_x3(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s) {
#define DG_X3(C, BM_, BN_, WM_, WN_, MW_, NB_)                                                                  \
    case C: {                                                                                                   \
        const dim3 blk(64 * WM_ * WN_);                                                                         \
        if (mode == MODE_FWD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_FWD, BM_, BN_, WM_, WN_, MW_, NB_, 4>), grid, blk, 0, s, a); \
        else if (mode == MODE_DGRAD) hipLaunchKernelGGL((k_conv_gemm_x6<MODE_DGRAD, BM_, BN_, WM_, WN_, MW_, NB_, 4>), grid, blk, 0, s, a); \
        else hipLaunchKernelGGL((k_conv_gemm_x6<MODE_WGRAD, BM_, BN_, WM_, WN_, MW_, NB_, 4>), grid, blk, 0, s, a); \
        break;                                                                                                  \
    }
#ifndef DG_X3_NB0
#define DG_X3_NB0 2
#endif
#ifndef DG_X3_NB12
#define DG_X3_NB12 2
#endif
    switch (cfg) {
        DG_X3(0, 128, 128, 2, 2, 2, DG_X3_NB0)
        DG_X3(1, 128, 64, 2, 2, 2, DG_X3_NB12)
        DG_X3(2, 64, 128, 2, 2, 2, DG_X3_NB12)
        DG_X3(3, 64, 64, 2, 2, 3, 3)
        DG_X3(4, 256, 128, 4, 2, 1, 2)
        DG_X3(5, 128, 256, 2, 4, 1, 2)
        DG_X3(6, 128, 32, 4, 1, 3, 3)
    }
#undef DG_X3
}

}  // namespace dg
