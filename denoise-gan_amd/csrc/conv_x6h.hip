// Halo-tiled bf16x6 implicit GEMM (gfx950) for
//   KT = 3: stride-1 3x3 convolutions, forward and input gradient -- every
//           VGG19 layer (pix2pix.py:53-67) and the 3x3 convs of the SR family;
//   KT = 4: stride-1 4x4 convolutions -- the input gradient of the PatchGAN's
//           ZeroPadding2D + Conv2D(512, 4) (pix2pix.py:206-208);
//   KT = 2: the input gradient of stride-2 4x4 convolutions, one sub-pixel
//           phase per grid slice (each phase is a stride-1 2x2 conv over dy)
//           -- the U-Net's Conv2DTranspose forwards (pix2pix.py:128-142) and
//           the down blocks' / PatchGAN's input gradients (:110-126, :194-211).
//
// The generic bf16x6 kernel (conv_x6.hip) stages each K-tile (one filter tap
// x 16 channels) as BM rows gathered from the activation planes, so each
// input pixel crosses L2 -> LDS once per tap that reads it.  Here a block
// owns a PH x PW = 8 x 16 output patch (its 128 GEMM rows) and stages, per
// 16-channel chunk, the (PH+KT-1) x (PW+KT-1) input halo ONCE; the KT*KT
// taps of the chunk read shifted windows of it.  A fragment of 16 GEMM rows
// is one patch row, i.e. 16 consecutive halo pixels, so a tap is a constant
// LDS offset (an immediate on the ds_read) and needs no per-row validity
// test: padding pixels are fetched out of range and land as zeros.
//
// Per block (4 waves, 2x2, wave tile 64 x BN/2 of 16x16 accumulators):
//   LDS: 2 halo buffers (3 planes x whole 1-KiB DMAs: 180 px -> 6 KiB for
//   KT 3, 153 px -> 5 KiB for KT 2) + NB weight K-tile buffers (3 for KT 3,
//   4 for KT 2 so a tap's buffer is fixed) = 74.6 / 79.1 KB for BN = 128, so
//   two blocks share a CU.
//   Pipeline: weight K-tiles two ahead; the halo of chunk c+1 is fetched
//   during the first K-tiles of chunk c, PPT 1-KiB pieces per wave per K-tile,
//   into the other halo buffer, and has landed by the chunk's last K-tile.
//   Every K-tile position within a chunk is unrolled, so the DMA count of
//   each position -- and so each s_waitcnt -- is a compile-time constant.
//   The epilogue maps patch rows to pixels (ragged patches at the image edge
//   are masked; a phase's pixels are scattered to (sh*hh + ph, sw*ww + pw))
//   and is shared with conv_x6.hip (staged through LDS).
//
// FWD (KT 3):  y[n,ho,wo]  = sum_{a,b} x [n, ho-pt+a, wo-pl+b] . w[a,b]      (halo origin (-pt, -pl))
// DGRAD:       dx[phase pixel (hh, ww)] = sum_{a,b} dy[n, hh+oh-a, ww+ow-b] . w[i0h+a*sh, i0w+b*sw]^T
//              (origin (oh-KT+1, ow-KT+1), taps mirrored; stride 1: oh = pt)
#include "conv_x6.h"
#include <algorithm>
#include <type_traits>
#include <utility>

namespace dg {

constexpr int HX_PH = 8, HX_PW = 16;
// tap positions column-major with A fragments kept across a filter column (the
// default); DG_X6H_TAPS_ROWMAJOR builds the row-major order that reloads all TM
// fragments per tap, for same-box A/B runs (scripts/build_variant.py)
#ifdef DG_X6H_TAPS_ROWMAJOR
constexpr bool kTapsColMajor = false;
#else
constexpr bool kTapsColMajor = true;
#endif
// Weight prefetch through a mid-K-tile barrier (as conv_x6.hip): once every wave
// holds K-tile T's fragments in registers, its buffer takes tile T+NB, so a DMA
// has NB K-tiles of MFMAs to land instead of NB-1.  DG_NO_MIDB builds the plain
// pipelines, DG_MIDB_X3 the fp16x3-only form, DG_MIDB_ALL every math, for same-box A/B runs.
// Default: fp16x3 and fp16 (SRGAN 4208 -> 4271 img/s, profiles/r4/ab_halo_midb_all.txt); the
// bf16x6 halo kernel keeps the plain pipeline (the autoencoder's 64^2 VGG19 forward ran 29 %
// slower with it, profiles/r5/ab_ae_r3_r5.txt)
#if defined(DG_NO_MIDB) || defined(DG_X6H_NOB)
constexpr int kMidb = 0;
#elif defined(DG_MIDB_X3)
constexpr int kMidb = 1;
#elif defined(DG_MIDB_ALL)
constexpr int kMidb = 2;
#else
constexpr int kMidb = 3;
#endif
// PACKED (fp16x3): the NPL plane images lie back to back (HPX * 32 bytes each) and
// only the whole halo is rounded up to KiB DMAs -- 23 KiB instead of 24 for KT 3,
// which keeps two fp16x3 blocks (two halo buffers, two weight buffers) per CU
template <int KT, int NPL = 3, bool PACKED = false, int PH = HX_PH>
struct HaloGeom {
    static constexpr int HH = PH + KT - 1, HW = HX_PW + KT - 1;
    static constexpr int HPX = HH * HW;
    static constexpr int HPL = PACKED ? HPX * 32 : (HPX * 32 + 1023) / 1024 * 1024;  // bytes per plane image
    static constexpr int BYTES = (NPL * HPL + 1023) / 1024 * 1024;                   // bytes per halo buffer
    static constexpr int HDMA = BYTES / 1024;                                         // one-KiB DMAs per halo
    static constexpr int NTAP = KT * KT;
};



// Forward epilogue fused with the 2x2 max pool that follows the conv (VGG19
// blockN_conv{2,4} -> blockN_pool, pix2pix.py:53-67 content features): a
// wave's 64 GEMM rows are 4 patch rows of 16 pixels, so every pool window
// (two patch rows a, a+1 of the same wave, two neighbouring pixels) lies in
// one wave's tile.  Rows are staged through LDS as in conv_epilogue16; the
// two pixels of a window row sit in lanes l and l ^ C4 (one swap), the
// window's row pair in registers across the a-loop.  The first maximum in
// row-major window order is kept (strict >: the pairwise and the sequential
// scan pick the same element), as k_maxpool_bwd4 routes.  Per pooled
// element: its bf16x6 planes (the next conv's x operand), optionally its
// fp32 value, and one byte {argmax, value > 0} for the backward -- the
// full-size activation is never written.
template <int TM, int TN, int PH = HX_PH>
__device__ __forceinline__ void conv_epilogue16_pool(const GemmArgs &p, f32x4 (&acc)[TM][TN], int prow0, int cbase,
                                                     int ty, int tx, int nimg, int lane, float *stage,
                                                     float ys_pre = 0.f, float *vacc = nullptr) {
    constexpr int WTN = 16 * TN;
    constexpr int LD = WTN + 4;
    constexpr int C4 = WTN / 4;
    constexpr int RPP = 64 / C4;
    constexpr int NP = 16 / RPP;
    static_assert(TM % 2 == 0 && 64 % C4 == 0 && 16 % RPP == 0 && RPP % 2 == 0, "window rows / pixel pairs in one wave");
    const ConvGeom &g = p.g;
    const int c4 = lane % C4, rsub = lane / C4;
    const int col = cbase + c4 * 4;
    const bool lead = (rsub & 1) == 0;          // holds the even pixel of its pair
    const bool colok = col < p.N;                // (N % 16 == 0: a float4 is all in or all out)
    const int Ho2 = g.Ho >> 1, Wo2 = g.Wo >> 1;
    f32x4 bias = {0.f, 0.f, 0.f, 0.f};
    if (p.bias && colok) bias = *reinterpret_cast<const f32x4 *>(p.bias + col);
    f32x4 hv[NP];
    unsigned hix[NP];
    float vmax = 0.f;   // max |pooled value| of this lane (p.ymax: the consumer's measured input)
    const float ys = p.yp ? (ys_pre > 0.f ? ys_pre : plane_scale(p)) : 0.f;
    // (row blocks in pairs -- a window's two rows -- with the pair loop not unrolled: the staging
    // takes compile-time acc indices in each case of a switch, as conv_epilogue16's, so one pair
    // body is the pool epilogue's code instead of TM / 2)
    auto stage_rows = [&](auto A) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                stage[(4 * (lane >> 4) + r) * LD + b * 16 + (lane & 15)] = acc[decltype(A)::value][b][r];
    };
    static_assert(TM == 2 || TM == 4, "row-block pairs");
#pragma clang loop unroll(disable)
    for (int a2 = 0; a2 < TM; a2 += 2)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int a = a2 + h;
        if (h == 0) {
            if (a2 == 0) stage_rows(std::integral_constant<int, 0>{});
            else stage_rows(std::integral_constant<int, (TM > 2 ? 2 : 0)>{});
        } else {
            if (a2 == 0) stage_rows(std::integral_constant<int, 1>{});
            else stage_rows(std::integral_constant<int, (TM > 2 ? 3 : 1)>{});
        }
#pragma unroll
        for (int pass = 0; pass < NP; ++pass) {
            const int rl = pass * RPP + rsub;
            f32x4 o = *reinterpret_cast<const f32x4 *>(stage + rl * LD + c4 * 4);
            o += bias;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = act_fwd(o[q], p.act, p.alpha);
            f32x4 po;
#pragma unroll
            for (int q = 0; q < 4; ++q) po[q] = __shfl_xor(o[q], C4);
            // window row: (this pixel, the next one) for the lead lane
            f32x4 hvv;
            unsigned hi = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool t = po[q] > o[q];
                hvv[q] = t ? po[q] : o[q];
                hi |= (t ? 1u : 0u) << (8 * q);
            }
            if (h == 0) {
                hv[pass] = hvv;
                hix[pass] = hi;
                continue;
            }
            f32x4 fv;
            unsigned fi = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool t = hvv[q] > hv[pass][q];   // the lower row only when strictly greater
                fv[q] = t ? hvv[q] : hv[pass][q];
                const unsigned id = t ? (((hi >> (8 * q)) & 1u) + 2u) : ((hix[pass] >> (8 * q)) & 1u);
                fi |= (id | (fv[q] > 0.f ? 4u : 0u)) << (8 * q);
            }
            if (!lead || !colok) continue;
            const int ho2 = (ty * PH + prow0 + a) >> 1, wo2 = (tx * HX_PW + rl) >> 1;
            const long pp = ((long)nimg * Ho2 + ho2) * Wo2 + wo2;
            *reinterpret_cast<unsigned *>(p.pidx + pp * p.N + col) = fi;
            if (p.pool_y) *reinterpret_cast<f32x4 *>(p.pool_y + pp * p.ldpy + col) = fv;
            if (p.yp) store_planes4(p.yp, p.ypC, pp, col, fv, ys);
#pragma unroll
            for (int q = 0; q < 4; ++q) vmax = fmaxf(vmax, fabsf(fv[q]));
        }
    }
    if (p.ymax) {
        if (vacc) *vacc = fmaxf(*vacc, vmax);
        else block_atomic_absmax(p.ymax, vmax);
    }
}

// f(integral_constant<T>) for T = 0 .. NTAP-1, unrolled at compile time
template <class F, int... T>
__device__ __forceinline__ void for_taps(F &&f, std::integer_sequence<int, T...>) {
    (f(std::integral_constant<int, T>{}), ...);
}

// NI = 3: bf16x6 (three bf16 plane images per 16-channel chunk, three MFMAs
// per fragment pair); NI = 2: fp16 (mixed_float16 policy): a chunk is 32
// channels, its two 16-channel halves are the two plane images and one
// v_mfma_f32_16x16x32_f16 covers them; NI = 4: fp16x3 (DG_MATH_F16X3 forward):
// a chunk is 32 channels as four plane images h0 h1 l0 l1 (h / l of channels
// 0-15 / 16-31), and three fp16 MFMAs over the 32 channels cover its three
// piece products: [h0|h1].[w_h0|w_h1] + [l0|l1].[w_h0|w_h1] + [h0|h1].[w_l0|w_l1]
// (= h.w_h + l.w_h + h.w_l) -- two A and two B fragment reads per K-tile.  Two
// weight buffers and packed halo images keep two blocks per CU; a K-tile's buffer
// takes tile T+2 once every wave holds its fragments (MIDB).
//
// PH = 16 (fp16x3 3x3 only): a 16 x 16 patch -- 256 GEMM rows -- on 8 waves (4 x 2), one block per
// CU: every weight K-tile staged in LDS feeds twice the rows, halving the weight traffic per MFMA
// that the 8 x 16 patch's two blocks per CU each stream (no weight DMAs ran the deep VGG19 layers
// 13-35 % faster, profiles/r5/pmc_x6h_waits.txt), and the halo overhead drops from 180 to 162
// pixels per 128 outputs.
template <int MODE, int BN, bool POOL, int KT, int NI = 3, int PH = HX_PH>
__global__ void __launch_bounds__(32 * PH, PH == HX_PH ? 2 : 1)
k_conv_gemm_x6h(const GemmArgs p, int tiles_x, int tiles_y) {
    static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "forward or input gradient");
    static_assert(!POOL || MODE == MODE_FWD, "the pool epilogue is a forward epilogue");
    static_assert(KT == 3 || MODE == MODE_DGRAD || (KT == 4 && NI == 4),
                  "3x3 stride 1, a stride-1 4x4 / stride-2 4x4-phase input gradient, or an fp16x3 4x4 stride-1 forward");
    static_assert(NI == 3 || (NI == 2 && KT == 3 && !POOL) || (NI == 4 && (KT == 3 || KT == 4 || (KT == 2 && MODE == MODE_DGRAD))),
                  "fp16: 3x3 stride 1, no pool epilogue; fp16x3: 3x3 stride 1, or the stride-2 4x4 input-gradient phases");
    constexpr bool X3 = NI == 4;
    static_assert(PH == HX_PH || (PH == 16 && X3 && KT == 3), "the 16 x 16 patch: fp16x3 3x3 only");
    constexpr int NPL = NI == 3 ? 3 : (X3 ? 4 : 2);   // plane images per chunk
    using HG = HaloGeom<KT, NPL, X3, PH>;
    constexpr int NTAP = HG::NTAP;
    // weight K-tile buffers: a tap position owns one (bf16x6 / fp16: two tiles in
    // flight); fp16x3: two buffers alternating by tap and chunk, one tile ahead
    // (fp16x3 3x3 BN 64: three -- 72.8 KB with the halos, still two blocks per CU -- so a weight
    // tile has two K-tiles of MFMAs to land; DG_X3H_NB2: two, for same-box A/B)
#ifdef DG_X3H_NB2
    constexpr int NB = X3 ? 2 : (NTAP % 3 == 0 ? 3 : 4);
#elif defined(DG_X3H16_NB)   // (the 16 x 16 patch's weight buffers, for same-box A/B)
    constexpr int NB = X3 ? (PH == 16 ? DG_X3H16_NB : ((KT == 3 && BN == 64) ? 3 : 2)) : (NTAP % 3 == 0 ? 3 : 4);
#else
    constexpr int NB = X3 ? ((KT == 3 && BN == 64) ? 3 : 2) : (NTAP % 3 == 0 ? 3 : 4);
#endif
    constexpr bool XPAR = X3 && NB == 2;   // buffers alternate by K-tile parity (NTAP odd: across chunks)
    static_assert(XPAR || NTAP % NB == 0, "tap positions line up with the weight buffers across chunks");
    constexpr int BK = NI == 3 ? 16 : 32, NW = PH / 2;   // channels per chunk; waves
    constexpr int WTM = 64, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
    constexpr bool B_KC = MODE == MODE_DGRAD;
    constexpr int BPL = BN * 32 + 96, BBUF = NPL * BPL;
    constexpr int B_SL = NPL * BN / 32, B_NJ = (B_SL + NW - 1) / NW;
    constexpr int H_NJ = (HG::HDMA + NW - 1) / NW;          // halo pieces per wave
    constexpr int PPT = (H_NJ + NTAP - 2) / (NTAP - 1);     // pieces per K-tile, none at the last tap
    static_assert((H_NJ - 1) / PPT < NTAP - 1, "the next chunk's halo lands by the chunk's last K-tile");
    constexpr int TL = (H_NJ - 1) / PPT;                    // the last tap position issuing halo pieces
    // mid-K-tile barrier form: needs the last NB-1 tap positions free of halo pieces
    // (the wait counts below), so not the KT 2 phases (4 taps, 4 buffers)
    constexpr bool MIDB = (kMidb == 2 || (kMidb == 1 && X3) || (kMidb == 3 && NI != 3)) && TL <= NTAP - NB;
    static_assert(XPAR || !X3 || MIDB, "fp16x3 with three weight buffers: the mid-K-tile barrier pipeline");
    // pipeline-tail DMAs (chunks past the split's range) out of range -- no traffic -- on the
    // fp16x3 / fp16 instances; the bf16x6 kernel issues them in range (the autoencoder's 64^2
    // VGG19 forward ran 23 % slower with the out-of-range form, profiles/r5/ab_ae_r3_r5.txt;
    // DG_TAIL_OOB_ALL: out of range everywhere, for A/B runs)
#if defined(DG_TAIL_OOB_ALL)
    constexpr bool kTailAll = false;
#else
    constexpr bool kTailAll = NI == 3;
#endif
    constexpr auto nh_of = [](int t) constexpr {   // halo pieces issued at tap position t (t < 0: t + NTAP)
        t = t < 0 ? t + NTAP : t;
        const int h0 = t * PPT, h1 = (t + 1) * PPT < H_NJ ? (t + 1) * PPT : H_NJ;
        return h1 > h0 ? h1 - h0 : 0;
    };
    constexpr auto midb_wait_v = [nh_of](int T) constexpr {
        int n = (NB - 1) * B_NJ;
        for (int j = 0; j < NB; ++j) n += nh_of(T - j);
        const int last = (NTAP - 1 - TL) * B_NJ;
        return T == NTAP - 1 && last < n ? last : n;
    };

    __shared__ __attribute__((aligned(16))) char hal[2][HG::BYTES];
    __shared__ __attribute__((aligned(16))) char bs0[BBUF];
    __shared__ __attribute__((aligned(16))) char bs1[BBUF];
    __shared__ __attribute__((aligned(16))) char bs2[NB >= 3 ? BBUF : 16];
    __shared__ __attribute__((aligned(16))) char bs3[NB == 4 ? BBUF : 16];
    char *const hal0 = hal[0], *const hal1 = hal[1];

    const ConvGeom &g = p.g;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    X3Pre x3s;   // (fp16x3: the scale sources, loaded here, combined in the epilogue)
    if constexpr (X3) x3s = x3_pre(p);

    int zz, tile;
    // (the 4 phases of a patch back to back on one XCD: down2 input gradient
    // 0.270 -> 0.257 ms, up7 forward 0.457 -> 0.446 at bs16 x2; the generic
    // kernel's deep-layer phases gained nothing)
    xcd_remap(zz, tile, MODE == MODE_DGRAD && p.nphase > 1 && !p.xcd_plain);
    const int phase = zz / p.splits;
    const int split = zz - phase * p.splits;
    int mt0 = tile / p.ntiles;
    int nt = tile - mt0 * p.ntiles;
    if (p.xcd_ng > 0) xcd_group_tile(p.xcd_ng, p.mtiles, p.ntiles, mt0, nt);
    const int n0 = nt * BN;
    // persistent blocks (fp16x3): patches mt0, mt0 + gm, ... (p.ptiles of them) of one n-tile,
    // phase and split run back to back -- the next patch's first halo and weight tiles are
    // fetched during the current patch's last chunk, so only the first patch waits for them.
    // The epilogue stages through the halo buffer just consumed (the other one is receiving).
    constexpr bool PERS = X3;
    const int PT = PERS ? max(1, p.ptiles) : 1;
    const int gm = gridDim.x / p.ntiles;
    // A source (FWD: x; DGRAD: dy) extents and the output grid of this block
    // (DGRAD: the phase's sub-grid; stride 1: the whole dx)
    const int Hin = MODE == MODE_FWD ? g.H : g.Ho, Win = MODE == MODE_FWD ? g.W : g.Wo;
    PhaseInfo ph{};
    int Hout, Wout, oh = 0, ow = 0;
    if constexpr (MODE == MODE_FWD) {
        Hout = g.Ho; Wout = g.Wo;
    } else {
        ph = phase_info(g, phase, g.N);
        Hout = ph.Hp; Wout = ph.Wp;
        // tap a of the phase reads dy row hh + oh - a (exact: ph + pt - i0h is a multiple of sh)
        oh = (ph.ph + g.pt - ph.i0h) / g.sh;
        ow = (ph.pw + g.pl - ph.i0w) / g.sw;
    }
    struct HTile {
        int tx, ty, nimg;
    };
    // the block's next patch from its j-th on (-1: none; a smaller phase grid skips patches)
    auto next_tile = [&](int j, HTile &t) __attribute__((always_inline)) -> int {
        for (; j < PT; ++j) {
            const int mt = mt0 + j * gm;
            if (mt >= p.mtiles) return -1;
            t.tx = mt % tiles_x;
            const int t_ = mt / tiles_x;
            t.ty = t_ % tiles_y;
            t.nimg = t_ / tiles_y;
            if (t.ty * PH < Hout && t.tx * HX_PW < Wout) return j;
        }
        return -1;
    };
    HTile cur, nxt;
    const int jc = next_tile(0, cur);
    if (jc < 0) return;   // block-uniform: a smaller phase grid
    int jn = next_tile(jc + 1, nxt);
    // channel chunks of this split (kchunk is a multiple of NTAP taps x BK channels)
    const int nch = p.K / (NTAP * BK);
    const int cbeg = split * (p.kchunk / (NTAP * BK));
    const int cend = min(nch, cbeg + p.kchunk / (NTAP * BK));
    if (cbeg >= cend) return;
    // filter tap (row-major in w) of tap position T.  Tap positions run
    // column-major (ta = T % KT fastest): the KT taps of one filter column read
    // halo windows one patch row apart, so each wave keeps its A fragments in
    // registers across them and reads one new patch row per tap instead of TM
    int tap_w[NTAP];
#pragma unroll
    for (int T = 0; T < NTAP; ++T) {
        const int ta = kTapsColMajor ? T % KT : T / KT, tb = kTapsColMajor ? T / KT : T % KT;
        if constexpr (MODE == MODE_FWD) {
            tap_w[T] = ta * g.kw + tb;
        } else {
            const int i = ph.i0h + ta * g.sh, j = ph.i0w + tb * g.sw;
            tap_w[T] = i * g.kw + j;
        }
    }

    const rsrc4_t rA = make_rsrc4(p.A, p.a_bytes);
    const rsrc4_t rB = make_rsrc4(p.B, p.b_bytes);
    auto dma = [](rsrc4_t r, char *lds_base, unsigned off) __attribute__((always_inline)) { dma16(r, lds_base, off); };
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // ---- halo pieces: wave piece s is DMA d = wid + NW*s of the HDMA (plane,
    // KiB) pieces (d >= HDMA repeats piece d - HDMA: same bytes, same data, and
    // every DMA provably targets the halo buffer); lane L of a piece fetches
    // the 16-byte half-row q = 64k + L of its plane image (halo pixel q/2,
    // channel half q&1).  hsrc: (halo row, halo column, element offset) of the
    // piece, or -1 past the halo's pixels; hoff: byte offset at chunk 0 in the
    // current patch (hoffn: the next one), or -1 outside the image.
    constexpr int PER = HG::HPL / 1024;
    int hsrc[H_NJ], hdst[H_NJ];
#pragma unroll
    for (int s = 0; s < H_NJ; ++s) {
        const int d = (wid + NW * s) % HG::HDMA;
        int pl, q;
        if constexpr (X3) {   // packed images: 16-byte unit q of the buffer -> (image, pixel, half)
            hdst[s] = d * 1024;
            const int u = d * 64 + lane;
            pl = u / (2 * HG::HPX);
            q = u - pl * 2 * HG::HPX;
        } else {
            pl = d / PER;
            const int kk = d - pl * PER;
            hdst[s] = pl * HG::HPL + kk * 1024;
            q = kk * 64 + lane;
        }
        hsrc[s] = -1;
        const int hp = q >> 1, hh = q & 1;
        if (hp < HG::HPX && pl < NPL) {
            const int hr = hp / HG::HW, hc = hp - hr * HG::HW;
            hsrc[s] = (hr << 16) | (hc << 8) | (16 * pl + 8 * hh);
        }
    }
    // (bf16x6 pixel rows: per 16 channels 3 x 16 plane values; fp16: the channel row
    // itself, plane image pl = channel half pl of the chunk; fp16x3: per 32 channels
    // h[32] l[32], image pl = 16 values at 16 pl)
    constexpr int PXS = NI == 3 ? 3 : (X3 ? 2 : 1);   // pixel stride in units of lda
    auto halo_offsets = [&](const HTile &t, int (&ho)[H_NJ]) __attribute__((always_inline)) {
        const int oy = MODE == MODE_FWD ? t.ty * PH - g.pt : t.ty * PH + oh - (KT - 1);
        const int ox = MODE == MODE_FWD ? t.tx * HX_PW - g.pl : t.tx * HX_PW + ow - (KT - 1);
#pragma unroll
        for (int s = 0; s < H_NJ; ++s) {
            ho[s] = -1;
            if (hsrc[s] < 0) continue;
            const int iy = oy + (hsrc[s] >> 16), ix = ox + ((hsrc[s] >> 8) & 255);
            if ((unsigned)iy < (unsigned)Hin && (unsigned)ix < (unsigned)Win)
                ho[s] = ((((t.nimg * Hin + iy) * Win + ix) * (PXS * p.lda)) + (hsrc[s] & 255)) * 2;
        }
    };
    int hoff[H_NJ], hoffn[H_NJ];
    halo_offsets(cur, hoff);
    // (no next patch: the pipeline tail reads the current patch's pixels at chunk cend, as
    // the one-patch kernel always did)
    if (jn >= 0) halo_offsets(nxt, hoffn);
    else {
#pragma unroll
        for (int s = 0; s < H_NJ; ++s) hoffn[s] = hoff[s];
    }
    // halo piece s of chunk `chunk` into hb; nxp: from the next patch's offsets
    auto issue_h = [&](int s, int chunk, char *hb, bool nxp) __attribute__((always_inline)) {
        // (chunks past the split's range -- the pipeline's tail -- out of range: no traffic)
        const int o = nxp ? hoffn[s] : hoff[s];
        dma(rA, hb + hdst[s],
            o >= 0 && (kTailAll || chunk < cend) ? (unsigned)(o + chunk * (NI == 3 ? 96 : (X3 ? 128 : 64)))
                                                 : DG_OOB);
    };

    // ---- weight K-tile slots (as conv_x6.hip): FWD RC image [16 k][BN],
    // DGRAD KC image [BN rows ci][16 k]
    int bbase[B_NJ];
    bool bok[B_NJ];
    int bdst[B_NJ];
#pragma unroll
    for (int j = 0; j < B_NJ; ++j) {
        const int d0 = wid + NW * j;
        const int d = d0 < B_SL ? d0 : 0;  // a dead slot repeats slot 0's DMA
        constexpr int per = BN / 32;
        const int plane = d / per;
        const int pos = (d - plane * per) * 1024 + 16 * lane;
        bdst[j] = plane * BPL + (d - plane * per) * 1024;
        if constexpr (!B_KC) {
            const int r = pos / (2 * BN);
            const int pdw = (pos - r * 2 * BN) >> 2;
            const int swz = BN >= 128 ? 8 * ((r & 3) | (((r >> 3) & 1) << 2))
                                      : (BN >= 64 ? 8 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) : 8 * ((r >> 1) & 1));
            const int col = n0 + 2 * (pdw ^ swz);
            bok[j] = col < p.N;
            if constexpr (NI == 3) bbase[j] = (r * (3 * p.ldb) + (col >> 4) * 48 + 16 * plane + (col & 8)) * 2;
            else if constexpr (X3)   // image = piece plane>>1 of k rows 16 (plane&1) ..
                bbase[j] = ((r + 16 * (plane & 1)) * (2 * p.ldb) + (col >> 4) * 32 + 16 * (plane >> 1) + (col & 8)) * 2;
            else bbase[j] = ((16 * plane + r) * p.ldb + col) * 2;   // image = k rows 16 plane ..
        } else {
            const int r = pos >> 5, c = (pos >> 4) & 1;
            const int ci = n0 + r;
            bok[j] = ci < p.N;
            if constexpr (X3)   // image = piece plane>>1 of co 16 (plane&1) .. of the chunk
                bbase[j] = (ci * (2 * p.ldb) + 32 * (plane & 1) + 16 * (plane >> 1) + 8 * c) * 2;
            else bbase[j] = (ci * (NI == 3 ? 3 * p.ldb : p.ldb) + 16 * plane + 8 * c) * 2;
        }
    }
    // tap position T of chunk c: FWD rows (tap*Ci + 16c) of w[(a,b,ci)][co];
    // DGRAD rows ci of w[i,j] at co-chunk c
    auto issue_b = [&](int T, int chunk, char *bs) __attribute__((always_inline)) {
#ifdef DG_X6H_NOB
        if constexpr (X3) return;   // (timing diagnostic only: no weight tiles move -- wrong results)
#endif
        int delta;
        constexpr int LW = NI == 3 ? 3 : (X3 ? 2 : 1);   // weight row stride in units of ldb
        if constexpr (!B_KC) delta = ((tap_w[T] * g.Ci + chunk * BK) * (LW * p.ldb)) * 2;
        else delta = (tap_w[T] * g.Ci * (LW * p.ldb) + chunk * (NI == 3 ? 48 : (X3 ? 64 : 32))) * 2;
#pragma unroll
        for (int j = 0; j < B_NJ; ++j) {
            dma(rB, bs + bdst[j], bok[j] && (kTailAll || chunk < cend) ? (unsigned)(bbase[j] + delta) : DG_OOB);
        }
    };
    auto bbuf = [&](int i) __attribute__((always_inline)) -> char * {
        return i == 0 ? bs0 : (i == 1 ? bs1 : (i == 2 ? bs2 : bs3));
    };
    constexpr int HIMG = HG::HPL;   // bytes between the plane images of a halo buffer

    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    // one K-tile: tap position T of chunk `chunk` from halo `hc`, weights in
    // bs[T % NB]; issues halo pieces PPT*T .. of chunk cn (the next one: chunk + 1, or the
    // next patch's first -- nxp) into `hn` and the weight tile two K-tiles ahead, then the
    // MFMAs, then waits for the next weight tile (and, at the chunk's last tap, the whole
    // next halo)
    // A fragments of patch rows wm*TM + r (r = a + da, 0 <= r < TM + KT - 1) of the
    // current filter column: {hi|mid} and {hi|lo} of 16 halo pixels
    // (fp16x3: fm = [h0|h1], fl = [l0|l1])
    bf16x8 fm[TM + KT - 1], fl[TM + KT - 1];
    auto ktile = [&](auto TT, auto PARc, int chunk, int cn, bool nxp, const char *hc, char *hn)
                     __attribute__((always_inline)) {
        constexpr int T = decltype(TT)::value;
        constexpr int PAR = decltype(PARc)::value;   // (fp16x3) parity of the chunk's first K-tile in this block's sequence (NTAP even: 0)
        constexpr int ta = kTapsColMajor ? T % KT : T / KT, tb = kTapsColMajor ? T / KT : T % KT;
        constexpr int da = MODE == MODE_FWD ? ta : KT - 1 - ta;
        constexpr int db = MODE == MODE_FWD ? tb : KT - 1 - tb;
        constexpr int H0P = T * PPT, H1P = (T + 1) * PPT < H_NJ ? (T + 1) * PPT : H_NJ;
        constexpr int NH = H1P > H0P ? H1P - H0P : 0;   // halo pieces issued in this K-tile
        const char *bc = XPAR ? bbuf((T + PAR) & 1) : bbuf(T % NB);
        char *bn = XPAR ? bbuf((T + PAR + 1) & 1) : bbuf((T + 2) % NB);
        bf16x8 b1[TN], b2[TN], b3[TN];
        const char *H0 = hc, *H1 = hc + HIMG, *H2 = hc + 2 * HIMG, *H3 = hc + 3 * HIMG;
        auto load_row = [&](int r) __attribute__((always_inline)) {
            const int r0 = (wm * TM + r) * HG::HW + db;
            if constexpr (X3) {
                fm[r] = x6_kc_frag(H0, H1, r0, lane);   // [h0|h1]
                fl[r] = x6_kc_frag(H2, H3, r0, lane);   // [l0|l1]
            } else {
                fm[r] = x6_kc_frag(H0, H1, r0, lane);
                if constexpr (NI == 3) fl[r] = x6_kc_frag(H0, H2, r0, lane);
            }
        };
        if constexpr (ta == 0 || !kTapsColMajor) {   // a new filter column: its first tap's TM rows
#pragma unroll
            for (int a = 0; a < TM; ++a) load_row(a + da);
        } else {                   // one row beyond the previous tap's window
            load_row(MODE == MODE_FWD ? da + TM - 1 : da);
        }
        const char *B0 = bc, *B1 = bc + BPL, *B2 = bc + 2 * BPL, *B3 = bc + 3 * BPL;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int c0 = wn * WTN + b * 16;
            if constexpr (X3 && B_KC) {
                b1[b] = x6_kc_frag(B0, B1, c0, lane);        // [w_h0|w_h1] (co halves of the chunk)
                b3[b] = x6_kc_frag(B2, B3, c0, lane);        // [w_l0|w_l1]
            } else if constexpr (X3) {
                b1[b] = x6_rc_frag<BN>(B0, B1, c0, lane);   // [w_h0|w_h1]
                b3[b] = x6_rc_frag<BN>(B2, B3, c0, lane);   // [w_l0|w_l1]
            } else if constexpr (B_KC) {
                b1[b] = x6_kc_frag(B0, B1, c0, lane);
                if constexpr (NI == 3) {
                    b2[b] = x6_kc_frag(B1, B0, c0, lane);
                    b3[b] = x6_kc_frag(B2, B0, c0, lane);
                }
            } else {
                b1[b] = x6_rc_frag<BN>(B0, B1, c0, lane);
                if constexpr (NI == 3) {
                    b2[b] = x6_rc_frag<BN>(B1, B0, c0, lane);
                    b3[b] = x6_rc_frag<BN>(B2, B0, c0, lane);
                }
            }
        }
        if constexpr (MIDB) {   // every wave holds this tile's fragments: its buffer takes tile T+NB
            barrier();
            if constexpr (T + NB < NTAP) issue_b(T + NB, chunk, const_cast<char *>(bc));
            else issue_b(T + NB - NTAP, cn, const_cast<char *>(bc));
        } else if constexpr (X3) {   // the next weight tile first: the wait below leaves only the halo pieces in flight
            if constexpr (T + 1 < NTAP) issue_b(T + 1, chunk, bn);
            else issue_b(0, cn, bn);
        }
#pragma unroll
        for (int s = H0P; s < H0P + NH; ++s) issue_h(s, cn, hn, nxp);
        if constexpr (!X3 && !MIDB) {
            if constexpr (T + 2 < NTAP) issue_b(T + 2, chunk, bn);
            else issue_b(T + 2 - NTAP, cn, bn);
        }
        if constexpr (X3) {   // h.w_h, l.w_h, h.w_l
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fm[a + da]),
                                                                      __builtin_bit_cast(f16x8, b1[b]), acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fl[a + da]),
                                                                      __builtin_bit_cast(f16x8, b1[b]), acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fm[a + da]),
                                                                      __builtin_bit_cast(f16x8, b3[b]), acc[a][b], 0, 0, 0);
        } else if constexpr (NI == 2) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fm[a + da]),
                                                                      __builtin_bit_cast(f16x8, b1[b]), acc[a][b], 0, 0, 0);
        } else {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[a + da], b1[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[a + da], b2[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[a + da], b3[b], acc[a][b], 0, 0, 0);
        }
        // DMAs issued in this K-tile may stay in flight; everything older
        // (the next weight tile, and at the last tap the whole next halo) has landed
        // (fp16x3: the weight tile issued in THIS K-tile, before its halo pieces, too)
        // (MIDB: the DMAs issued after tile T+1's weights -- tiles T+2 .. T+NB and the
        // halo pieces of K-tiles T+1-NB .. T -- may stay in flight; at the chunk's last
        // tap none issued before the last halo piece)
        wait_dma_c<MIDB ? midb_wait_v(T) : (X3 ? NH : B_NJ + NH)>();
        barrier();
    };
    auto chunk_tiles = [&](auto PARc, int chunk, int cn, bool nxp, const char *hc, char *hn)
                           __attribute__((always_inline)) {
        for_taps([&](auto TT) __attribute__((always_inline)) { ktile(TT, PARc, chunk, cn, nxp, hc, hn); },
                 std::make_integer_sequence<int, NTAP>{});
    };

    // prologue: the whole halo of the first chunk and its first two weight tiles
    // (fp16x3: its first one)
#pragma unroll
    for (int s = 0; s < H_NJ; ++s) issue_h(s, cbeg, hal0, false);
    issue_b(0, cbeg, bs0);
    if constexpr (MIDB) {   // one weight tile per buffer
        issue_b(1, cbeg, bs1);
        if constexpr (NB >= 3) issue_b(2, cbeg, bs2);
        if constexpr (NB >= 4) issue_b(3, cbeg, bs3);
        wait_dma_c<(NB - 1) * B_NJ>();
    } else if constexpr (X3) {
        wait_dma_c<0>();
    } else {
        issue_b(1, cbeg, bs1);
        wait_dma_c<B_NJ>();
    }
    barrier();

    constexpr int STAGE = 16 * (WTN + 4);
    static_assert(NW * STAGE * 4 <= (PERS ? 1 : 2) * HG::BYTES, "epilogue staging fits in the halo buffer(s)");
    float osc = 1.f, ys_pre = 0.f, vacc = 0.f;
    if constexpr (X3) {   // the operand scales to undo (powers of two: exact), the output planes' scale
        osc = x3_out_scale(p, x3s);
        ys_pre = p.yp ? x3_raw_scale(x3s.y, F16X3_XS) : 0.f;
    }
    // after a patch's last chunk (its K-tiles consumed halo buffer HB): the epilogue, then the
    // next patch (false: none)
    auto patch_end = [&](auto HB) __attribute__((always_inline)) -> bool {
        float *stage;
        if constexpr (PERS) {
            stage = reinterpret_cast<float *>(decltype(HB)::value ? hal1 : hal0) + wid * STAGE;
        } else {
            // every wave's DMAs (including the harmless ones past the last chunk)
            // have landed before the halo buffers become the epilogue's staging area
            wait_dma_c<0>();
            barrier();
            stage = reinterpret_cast<float *>(hal0) + wid * STAGE;
        }
        if constexpr (X3) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) acc[a][b] *= osc;
        }
        const int ty = cur.ty, tx = cur.tx, nimg = cur.nimg;
        // patch row -> output pixel; slab rows: FWD / stride-1 DGRAD pixels, a
        // phase's GEMM rows otherwise (as k_splitk_reduce maps them)
        auto rowmap = [&](int row) __attribute__((always_inline)) -> RowPix {
            const int ho = ty * PH + (row >> 4), wo = tx * HX_PW + (row & 15);
            if (ho >= Hout || wo >= Wout) return RowPix{-1, -1};
            if constexpr (MODE == MODE_DGRAD && KT == 2) {
                const long pix = ((long)nimg * g.H + ho * g.sh + ph.ph) * g.W + wo * g.sw + ph.pw;
                return RowPix{((long)nimg * Hout + ho) * Wout + wo, pix};
            } else {
                const long pix = ((long)nimg * Hout + ho) * Wout + wo;
                return RowPix{pix, pix};
            }
        };
        float *va = PERS ? &vacc : nullptr;
#ifdef DG_X6H_LAUNDER
        // the epilogue's arguments re-read from the kernarg segment here (scalar loads), instead of
        // held in SGPRs -- spilled to VGPR lanes -- across the whole patch loop
        const __attribute__((address_space(4))) GemmArgs *pq =
            (const __attribute__((address_space(4))) GemmArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(pq));
        const GemmArgs &pe = *(const GemmArgs *)pq;
#else
        const GemmArgs &pe = p;
#endif
        if constexpr (POOL)
            conv_epilogue16_pool<TM, TN, PH>(pe, acc, wm * TM, n0 + wn * WTN, ty, tx, nimg, lane, stage, ys_pre, va);
        else
            conv_epilogue16<MODE, TM, TN>(pe, acc, wm * WTM, n0 + wn * WTN, rowmap, phase, split, lane, stage, ys_pre,
                                          va);
        if (jn < 0) return false;
        // every wave has read its staging rows before the next patch's DMAs refill the buffer
        barrier();
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        cur = nxt;
#pragma unroll
        for (int s = 0; s < H_NJ; ++s) hoff[s] = hoffn[s];
        jn = next_tile(jn + 1, nxt);
        if (jn >= 0) halo_offsets(nxt, hoffn);
        return true;
    };
    if constexpr (PERS) {
        // chunk c of the current patch from halo buffer HB (the next chunk's halo into the other)
        int c = cbeg;
        auto step = [&](auto PARc, auto HB) __attribute__((always_inline)) -> bool {
            const bool lastc = c + 1 == cend;
            const int cn = lastc ? (jn >= 0 ? cbeg : cend) : c + 1;
            chunk_tiles(PARc, c, cn, lastc, decltype(HB)::value ? hal1 : hal0, decltype(HB)::value ? hal0 : hal1);
            c = lastc ? cbeg : cn;
            return !lastc || patch_end(HB);
        };
        while (step(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}) &&
               step(std::integral_constant<int, NTAP & 1>{}, std::integral_constant<int, 1>{})) {
        }
        if (p.ymax) block_atomic_absmax(p.ymax, vacc);
        wait_dma_c<0>();   // (the pipeline tail's DMAs have landed before the block's LDS is released)
    } else {
        // one patch: the chunk loop, then the epilogue outside it (in the loop body its registers
        // would be live beside the bf16x6 / fp16 fragments: 150-580 VGPRs of spills measured)
        int c = cbeg;
        for (; c + 1 < cend; c += 2) {
            chunk_tiles(std::integral_constant<int, 0>{}, c, c + 1, false, hal0, hal1);
            chunk_tiles(std::integral_constant<int, NTAP & 1>{}, c + 1, c + 2, false, hal1, hal0);
        }
        if (c < cend) chunk_tiles(std::integral_constant<int, 0>{}, c, c + 1, false, hal0, hal1);
        patch_end(std::integral_constant<int, 0>{});
    }
}

void launch_gemm_x6h(int mode, int bn, int kt, dim3 grid, const GemmArgs &a, int tiles_x, int tiles_y, hipStream_t s,
                     int ni, int ph) {
    const dim3 blk(256);
    if (ph == 16) {   // fp16x3 3x3 on the 16 x 16 patch (8 waves)
        const dim3 b16(512);
#define DG_X3H16(M_, B_, P_) hipLaunchKernelGGL((k_conv_gemm_x6h<M_, B_, P_, 3, 4, 16>), grid, b16, 0, s, a, tiles_x, tiles_y)
        if (mode == MODE_FWD && a.pidx) {
            if (bn == 128) DG_X3H16(MODE_FWD, 128, true);
            else DG_X3H16(MODE_FWD, 64, true);
        } else if (mode == MODE_FWD) {
            if (bn == 128) DG_X3H16(MODE_FWD, 128, false);
            else DG_X3H16(MODE_FWD, 64, false);
        } else {
            if (bn == 128) DG_X3H16(MODE_DGRAD, 128, false);
            else DG_X3H16(MODE_DGRAD, 64, false);
        }
#undef DG_X3H16
        return;
    }
#define DG_X6H(M_, B_, P_, K_) hipLaunchKernelGGL((k_conv_gemm_x6h<M_, B_, P_, K_>), grid, blk, 0, s, a, tiles_x, tiles_y)
#define DG_F16H(M_, B_) hipLaunchKernelGGL((k_conv_gemm_x6h<M_, B_, false, 3, 2>), grid, blk, 0, s, a, tiles_x, tiles_y)
#define DG_X3H(B_, P_) hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_FWD, B_, P_, 3, 4>), grid, blk, 0, s, a, tiles_x, tiles_y)
    // (bn 32: the SR discriminators' / FastSRGAN's 32-channel 3x3 layers, stride 1; a
    // 64-wide tile computes half zeros there)
    if (ni == 4 && kt == 4) {   // fp16x3 stride-1 4x4 forward / input gradient (BN 64)
        if (mode == MODE_FWD) hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_FWD, 64, false, 4, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
        else hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_DGRAD, 64, false, 4, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
    } else if (ni == 4 && mode == MODE_DGRAD && kt == 2) {   // fp16x3 stride-2 4x4 input-gradient phases (bn 64 | 128)
        if (bn == 128) hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_DGRAD, 128, false, 2, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
        else hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_DGRAD, 64, false, 2, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
    } else if (ni == 4 && mode == MODE_DGRAD) {   // fp16x3 input gradient (3x3 stride 1, bn 64 | 128)
        if (bn == 128) hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_DGRAD, 128, false, 3, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
        else hipLaunchKernelGGL((k_conv_gemm_x6h<MODE_DGRAD, 64, false, 3, 4>), grid, blk, 0, s, a, tiles_x, tiles_y);
    } else if (ni == 4) {   // fp16x3 forward (bn 64 | 128), optionally with the fused pool
        if (a.pidx) {
            if (bn == 128) DG_X3H(128, true);
            else DG_X3H(64, true);
        } else {
            if (bn == 128) DG_X3H(128, false);
            else DG_X3H(64, false);
        }
    } else if (ni == 2) {   // fp16: 3x3 stride 1, forward or input gradient
        if (mode == MODE_FWD) {
            if (bn == 128) DG_F16H(MODE_FWD, 128);
            else if (bn == 32) DG_F16H(MODE_FWD, 32);
            else DG_F16H(MODE_FWD, 64);
        } else {
            if (bn == 128) DG_F16H(MODE_DGRAD, 128);
            else if (bn == 32) DG_F16H(MODE_DGRAD, 32);
            else DG_F16H(MODE_DGRAD, 64);
        }
    } else if (mode == MODE_FWD && a.pidx) {
        if (bn == 128) DG_X6H(MODE_FWD, 128, true, 3);
        else DG_X6H(MODE_FWD, 64, true, 3);
    } else if (mode == MODE_FWD) {
        if (bn == 128) DG_X6H(MODE_FWD, 128, false, 3);
        else if (bn == 32) DG_X6H(MODE_FWD, 32, false, 3);
        else DG_X6H(MODE_FWD, 64, false, 3);
    } else if (kt == 2) {
        if (bn == 128) DG_X6H(MODE_DGRAD, 128, false, 2);
        else DG_X6H(MODE_DGRAD, 64, false, 2);
    } else if (kt == 4) {
        DG_X6H(MODE_DGRAD, 64, false, 4);
    } else {
        if (bn == 128) DG_X6H(MODE_DGRAD, 128, false, 3);
        else if (bn == 32) DG_X6H(MODE_DGRAD, 32, false, 3);
        else DG_X6H(MODE_DGRAD, 64, false, 3);
    }
#undef DG_X6H
#undef DG_F16H
#undef DG_X3H
}

}  // namespace dg
