// Convolution engine for the pix2pix training step on MI355X (gfx950).
//
// Replaces TF's Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter, which
// the reference dispatches for every Conv2D (pix2pix.py:115, :207, :217) and
// Conv2DTranspose (pix2pix.py:130, :169).  All three are written as one
// implicit GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32, exact fp32
// FMA chains), over the *conv view* of a layer:
//     x [N,H,W,Ci]  --conv(w HWIO [kh,kw,Ci,Co], stride, pad)-->  y [N,Ho,Wo,Co]
//   FWD   : C[m=(n,ho,wo)][co]  = sum_k im2col(x)[m][k=(i,j,ci)] * w[k][co]
//   DGRAD : per output phase (h%sh, w%sw) a dense GEMM over the Th*Tw taps
//           that hit that phase (sub-pixel decomposition, no zero-stuffing):
//           C[m=(n,hh,ww)][ci] = sum_{(a,b,co)} dy[n,ho,wo,co] * w[i,j,ci,co]
//   WGRAD : C[k=(i,j,ci)][co]   = sum_{m=(n,ho,wo)} im2col(x)[m][k] * dy[m][co]
//           split over m into fp32 partial slabs, reduced deterministically.
// Conv2DTranspose fwd is DGRAD, its input-grad is FWD and its filter grad is
// WGRAD with the roles of x and dy exchanged (Keras kernel [kh,kw,F,Cin] is
// exactly the HWIO kernel of the equivalent conv).
//
// Tiling: 256 threads = 4 waves; block tile BM x BN x BK(32); each wave owns
// a (BM/WGM) x (BN/WGN) sub-tile of 32x32 MFMA accumulators.  Operands are
// staged global -> registers -> LDS (double buffered, one barrier per
// K-tile), stored k-major ([k][m], [k][n]) so every MFMA operand fetch is a
// conflict-free ds_read_b32 of 32 consecutive floats per half-wave.
#include "conv_impl.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>

namespace dg {

// -------------------------------------------------------------------------
// The MFMA implicit-GEMM kernel
// -------------------------------------------------------------------------
template <int MODE, int BM, int BN, int WGM, int WGN, bool VEC, int BK, int MINW>
__global__ void __launch_bounds__(256, MINW)
k_conv_gemm(const GemmArgs p) {
    constexpr bool A_KC = (MODE != MODE_WGRAD);  // A rows contiguous along k
    constexpr bool B_KC = (MODE == MODE_DGRAD);  // B rows (n) contiguous along k
    constexpr int LDA = A_KC ? BM + 1 : BM + 4;
    constexpr int LDB = B_KC ? BN + 1 : BN + 4;
    constexpr int ASZ = BK * LDA;
    constexpr int BSZ = BK * LDB;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    static_assert(WGM * WGN == 4, "4 waves");
    static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
    static_assert(BK % 4 == 0 && BM >= 256 / (BK / 4) && BN >= 256 / (BK / 4), "KC loader geometry");
    static_assert(1024 / BM <= BK && 1024 / BN <= BK, "RC loader geometry");

    __shared__ __attribute__((aligned(16))) float smem[2 * (ASZ + BSZ)];

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

    // ---------------- A operand -----------------
    // KC (FWD / DGRAD): tile BM rows x BK, row r contiguous along k.
    constexpr int KC_TPR = BK / 4, KC_RPP = 256 / KC_TPR;  // KC vec: threads per row, rows per pass
    constexpr int KS_RPP = 256 / BK;                        // KC scalar: rows per pass
    constexpr int A_NPV = BM / KC_RPP;      // vec rows per thread
    constexpr int A_NES = BM * BK / 256;    // scalar elements per thread
    // RC (WGRAD): tile BK k-rows x BM, contiguous along m.
    constexpr int AR_TPR = BM / 4, AR_RPP = 256 / AR_TPR, AR_NP = BK / AR_RPP;
    constexpr int AR_NES = BM * BK / 256;

    // ---------------- B operand -----------------
    constexpr int B_NPV = BN / KC_RPP;      // KC vec rows per thread (DGRAD)
    constexpr int B_NES = BN * BK / 256;    // KC scalar elements per thread (DGRAD)
    constexpr int BR_TPR = BN / 4, BR_RPP = 256 / BR_TPR, BR_NP = BK / BR_RPP;  // RC vec

    // staging registers (sized for the largest variant used by this MODE)
    constexpr int A_REGS = A_KC ? (VEC ? A_NPV * 4 : A_NES) : (VEC ? AR_NP * 4 : AR_NES);
    constexpr int B_REGS = B_KC ? (VEC ? B_NPV * 4 : B_NES) : BR_NP * 4;
    float ra[A_REGS];
    float rb[B_REGS];

    // ---- per-thread precomputation ----
    // KC vec: thread -> (row rr + 32*ip, k-chunk c4)
    const int kc_c4 = tid % KC_TPR, kc_rr = tid / KC_TPR;
    // KC scalar: thread -> (kk = tid % 32, rows r0 + 8*e)
    const int ks_kk = tid % BK, ks_r0 = tid / BK;

    // row geometry for the A operand (FWD/DGRAD vec path), up to 4 rows
    int arow_n[A_NPV > 0 ? A_NPV : 1], arow_h[A_NPV > 0 ? A_NPV : 1], arow_w[A_NPV > 0 ? A_NPV : 1];
    if constexpr (A_KC && VEC) {
#pragma unroll
        for (int ip = 0; ip < A_NPV; ++ip) {
            int m = m0 + kc_rr + KC_RPP * ip;
            if (m < Mrows) {
                if constexpr (MODE == MODE_FWD) {
                    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    arow_n[ip] = n; arow_h[ip] = ho * g.sh - g.pt; arow_w[ip] = wo * g.sw - g.pl;
                } else {
                    int ww = m % ph.Wp; int t = m / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                    arow_n[ip] = n; arow_h[ip] = hh * g.sh + ph.ph; arow_w[ip] = ww * g.sw + ph.pw;
                }
            } else {
                arow_n[ip] = -1; arow_h[ip] = 0; arow_w[ip] = 0;
            }
        }
    }
    // WGRAD A (RC vec4): the thread's column chunk is fixed -> (i, j, ci) once
    const int ar_c4 = tid % AR_TPR, ar_kr = tid / AR_TPR;
    int wg_i = 0, wg_j = 0, wg_ci = 0; bool wg_colok = false;
    if constexpr (MODE == MODE_WGRAD && VEC) {
        int mc = m0 + 4 * ar_c4;
        wg_colok = mc < p.M;
        int tap = mc / g.Ci; wg_ci = mc - tap * g.Ci; wg_i = tap / g.kw; wg_j = tap - wg_i * g.kw;
    }
    // WGRAD A scalar: thread column c = tid % BM fixed
    const int as_c = tid % BM, as_kr = tid / BM;
    if constexpr (MODE == MODE_WGRAD && !VEC) {
        int mc = m0 + as_c;
        wg_colok = mc < p.M;
        int tap = mc / g.Ci; wg_ci = mc - tap * g.Ci; wg_i = tap / g.kw; wg_j = tap - wg_i * g.kw;
    }
    const int br_c4 = tid % BR_TPR, br_kr = tid / BR_TPR;

    // decode a DGRAD tap (k0 is a multiple of BK; VEC => whole tile inside one tap)
    auto dgrad_tap = [&](int k, int &i, int &j, int &co) {
        int tap = k / g.Co; co = k - tap * g.Co;
        int a = tap / g.Tw; int b = tap - a * g.Tw;
        i = ph.i0h + a * g.sh; j = ph.i0w + b * g.sw;
    };

    const rsrc_t rA = make_rsrc(p.A, p.a_bytes);
    const rsrc_t rB = make_rsrc(p.B, p.b_bytes);
    auto put4 = [](float *r, int ip, f32x4 v) {
        r[4 * ip + 0] = v[0]; r[4 * ip + 1] = v[1]; r[4 * ip + 2] = v[2]; r[4 * ip + 3] = v[3];
    };

    // VEC FWD/DGRAD walk the K-tiles channel-chunk-major (all taps of one
    // BK-channel chunk, then the next chunk): a block's input window for one
    // chunk (~30 KB) is re-read by the next kh*kw tiles while it is still in
    // L1/L2, instead of once per tap after the whole channel range streamed by.
    // k0 is the position in that walk; kr0 the real (tap, channel) K index.
    auto k_real = [&](int k0) -> int {
        if constexpr (VEC && MODE != MODE_WGRAD) {
            const int C = MODE == MODE_FWD ? g.Ci : g.Co;
            const int ntap = MODE == MODE_FWD ? g.kh * g.kw : g.Th * g.Tw;
            int kk = k0 / BK; int chunk = kk / ntap; int tap = kk - chunk * ntap;
            return tap * C + chunk * BK;
        } else {
            return k0;
        }
    };

    auto load_tiles = [&](int k0) {
        const int kr0 = k_real(k0);
        // ----- A -----
        if constexpr (MODE == MODE_FWD) {
            if constexpr (VEC) {
                int tap = kr0 / g.Ci; int ci0 = kr0 - tap * g.Ci;
                int i = tap / g.kw; int j = tap - i * g.kw;
#pragma unroll
                for (int ip = 0; ip < A_NPV; ++ip) {
                    int hi = arow_h[ip] + i, wi = arow_w[ip] + j;
                    bool ok = arow_n[ip] >= 0 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                    unsigned off = ((unsigned)((arow_n[ip] * g.H + hi) * g.W + wi) * p.lda + ci0 + 4 * kc_c4) * 4u;
                    put4(ra, ip, bload4(rA, ok ? off : DG_OOB));
                }
            } else {
                int k = k0 + ks_kk;
                int tap = k / g.Ci; int ci = k - tap * g.Ci;
                int i = tap / g.kw; int j = tap - i * g.kw;
                bool kok = k < kend;
#pragma unroll
                for (int e = 0; e < A_NES; ++e) {
                    int m = m0 + ks_r0 + KS_RPP * e;
                    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    int hi = ho * g.sh - g.pt + i, wi = wo * g.sw - g.pl + j;
                    bool ok = kok && m < Mrows && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                    unsigned off = ((unsigned)((n * g.H + hi) * g.W + wi) * p.lda + ci) * 4u;
                    ra[e] = bload1(rA, ok ? off : DG_OOB);
                }
            }
        } else if constexpr (MODE == MODE_DGRAD) {
            if constexpr (VEC) {
                int i, j, co0; dgrad_tap(kr0, i, j, co0);
                bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
                for (int ip = 0; ip < A_NPV; ++ip) {
                    int th = arow_h[ip] + g.pt - i, tw = arow_w[ip] + g.pl - j;
                    int ho = th / g.sh, wo = tw / g.sw;  // exact when th, tw >= 0 (phase-aligned taps)
                    bool ok = tapok && arow_n[ip] >= 0 && th >= 0 && tw >= 0 && ho < g.Ho && wo < g.Wo;
                    unsigned off = ((unsigned)((arow_n[ip] * g.Ho + ho) * g.Wo + wo) * p.lda + co0 + 4 * kc_c4) * 4u;
                    put4(ra, ip, bload4(rA, ok ? off : DG_OOB));
                }
            } else {
                int k = k0 + ks_kk;
                int i, j, co; dgrad_tap(k, i, j, co);
                bool kok = (k < kend) && (i < g.kh) && (j < g.kw);
#pragma unroll
                for (int e = 0; e < A_NES; ++e) {
                    int m = m0 + ks_r0 + KS_RPP * e;
                    int ww = m % ph.Wp; int t = m / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                    int th = hh * g.sh + ph.ph + g.pt - i, tw = ww * g.sw + ph.pw + g.pl - j;
                    int ho = th / g.sh, wo = tw / g.sw;
                    bool ok = kok && m < Mrows && th >= 0 && tw >= 0 && ho < g.Ho && wo < g.Wo;
                    unsigned off = ((unsigned)((n * g.Ho + ho) * g.Wo + wo) * p.lda + co) * 4u;
                    ra[e] = bload1(rA, ok ? off : DG_OOB);
                }
            }
        } else {  // WGRAD: A k-rows are pixels, columns are (tap, ci)
            if constexpr (VEC) {
#pragma unroll
                for (int ip = 0; ip < AR_NP; ++ip) {
                    int pix = k0 + ar_kr + AR_RPP * ip;
                    int wo = pix % g.Wo; int t = pix / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    int hi = ho * g.sh - g.pt + wg_i, wi = wo * g.sw - g.pl + wg_j;
                    bool ok = wg_colok && pix < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                    unsigned off = ((unsigned)((n * g.H + hi) * g.W + wi) * p.lda + wg_ci) * 4u;
                    put4(ra, ip, bload4(rA, ok ? off : DG_OOB));
                }
            } else {
#pragma unroll
                for (int e = 0; e < AR_NES; ++e) {
                    int pix = k0 + as_kr + (256 / BM) * e;
                    int wo = pix % g.Wo; int t = pix / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                    int hi = ho * g.sh - g.pt + wg_i, wi = wo * g.sw - g.pl + wg_j;
                    bool ok = wg_colok && pix < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                    unsigned off = ((unsigned)((n * g.H + hi) * g.W + wi) * p.lda + wg_ci) * 4u;
                    ra[e] = bload1(rA, ok ? off : DG_OOB);
                }
            }
        }
        // ----- B -----
        if constexpr (MODE == MODE_FWD) {  // w rows k contiguous along co
#pragma unroll
            for (int ip = 0; ip < BR_NP; ++ip) {
                int k = kr0 + br_kr + BR_RPP * ip;
                int col = n0 + 4 * br_c4;
                bool ok = (VEC || k < kend) && col < p.N;
                put4(rb, ip, bload4(rB, ok ? ((unsigned)k * p.ldb + col) * 4u : DG_OOB));
            }
        } else if constexpr (MODE == MODE_DGRAD) {  // w[i,j,ci,co]: rows ci contiguous along co
            if constexpr (VEC) {
                int i, j, co0; dgrad_tap(kr0, i, j, co0);
                bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
                for (int ip = 0; ip < B_NPV; ++ip) {
                    int ci = n0 + kc_rr + KC_RPP * ip;
                    bool ok = tapok && ci < p.N;
                    unsigned off = ((unsigned)((i * g.kw + j) * g.Ci + ci) * g.Co + co0 + 4 * kc_c4) * 4u;
                    put4(rb, ip, bload4(rB, ok ? off : DG_OOB));
                }
            } else {
                int k = k0 + ks_kk;
                int i, j, co; dgrad_tap(k, i, j, co);
                bool kok = (k < kend) && (i < g.kh) && (j < g.kw);
#pragma unroll
                for (int e = 0; e < B_NES; ++e) {
                    int ci = n0 + ks_r0 + KS_RPP * e;
                    bool ok = kok && ci < p.N;
                    unsigned off = ((unsigned)((i * g.kw + j) * g.Ci + ci) * g.Co + co) * 4u;
                    rb[e] = bload1(rB, ok ? off : DG_OOB);
                }
            }
        } else {  // WGRAD: dy rows (pixels) contiguous along co
#pragma unroll
            for (int ip = 0; ip < BR_NP; ++ip) {
                int pix = k0 + br_kr + BR_RPP * ip;
                int col = n0 + 4 * br_c4;
                bool ok = pix < kend && col < p.N;
                put4(rb, ip, bload4(rB, ok ? ((unsigned)pix * p.ldb + col) * 4u : DG_OOB));
            }
        }
    };

    auto store_tiles = [&](int buf) {
        float *As = smem + buf * (ASZ + BSZ);
        float *Bs = As + ASZ;
        if constexpr (A_KC) {
            if constexpr (VEC) {
#pragma unroll
                for (int ip = 0; ip < A_NPV; ++ip)
#pragma unroll
                    for (int q = 0; q < 4; ++q) As[(4 * kc_c4 + q) * LDA + kc_rr + KC_RPP * ip] = ra[4 * ip + q];
            } else {
#pragma unroll
                for (int e = 0; e < A_NES; ++e) As[ks_kk * LDA + ks_r0 + KS_RPP * e] = ra[e];
            }
        } else {
            if constexpr (VEC) {
#pragma unroll
                for (int ip = 0; ip < AR_NP; ++ip) {
                    f32x4 v = {ra[4 * ip], ra[4 * ip + 1], ra[4 * ip + 2], ra[4 * ip + 3]};
                    *reinterpret_cast<f32x4 *>(&As[(ar_kr + AR_RPP * ip) * LDA + 4 * ar_c4]) = v;
                }
            } else {
#pragma unroll
                for (int e = 0; e < AR_NES; ++e) As[(as_kr + (256 / BM) * e) * LDA + as_c] = ra[e];
            }
        }
        if constexpr (B_KC) {
            if constexpr (VEC) {
#pragma unroll
                for (int ip = 0; ip < B_NPV; ++ip)
#pragma unroll
                    for (int q = 0; q < 4; ++q) Bs[(4 * kc_c4 + q) * LDB + kc_rr + KC_RPP * ip] = rb[4 * ip + q];
            } else {
#pragma unroll
                for (int e = 0; e < B_NES; ++e) Bs[ks_kk * LDB + ks_r0 + KS_RPP * e] = rb[e];
            }
        } else {
#pragma unroll
            for (int ip = 0; ip < BR_NP; ++ip) {
                f32x4 v = {rb[4 * ip], rb[4 * ip + 1], rb[4 * ip + 2], rb[4 * ip + 3]};
                *reinterpret_cast<f32x4 *>(&Bs[(br_kr + BR_RPP * ip) * LDB + 4 * br_c4]) = v;
            }
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    // Pipeline (one barrier per K-tile): at the top of iteration kt, LDS buffer
    // kt%2 holds tile kt and the staging registers hold tile kt+1 (loads in
    // flight).  The MFMA chain of tile kt is split in two; between the halves
    // the wave writes tile kt+1 into the other buffer (free: every wave passed
    // the barrier after its last read of it) and issues the loads of tile kt+2,
    // so the matrix pipe keeps running across the staging work.
    load_tiles(kbeg);
    store_tiles(0);
    if (nk > 1) load_tiles(kbeg + BK);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        const float *As = smem + buf * (ASZ + BSZ) + h2 * LDA + wm * WTM + l32;
        const float *Bs = smem + buf * (ASZ + BSZ) + ASZ + h2 * LDB + wn * WTN + l32;
        // all fragments of the K-tile first (one LDS round trip), then the MFMA chain
        float af[BK / 2][TM], bf[BK / 2][TN];
#pragma unroll
        for (int s2 = 0; s2 < BK / 2; ++s2) {
#pragma unroll
            for (int a = 0; a < TM; ++a) af[s2][a] = As[2 * s2 * LDA + a * 32];
#pragma unroll
            for (int b = 0; b < TN; ++b) bf[s2][b] = Bs[2 * s2 * LDB + b * 32];
        }
        // keep the whole read block ahead of the MFMA chain (the scheduler would
        // otherwise sink each read next to its MFMA and expose LDS latency per k-step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s2 = 0; s2 < BK / 4; ++s2)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s2][a], bf[s2][b], acc[a][b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) store_tiles(buf ^ 1);
        if (kt + 2 < nk) load_tiles(kbeg + (kt + 2) * BK);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s2 = BK / 4; s2 < BK / 2; ++s2)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s2][a], bf[s2][b], acc[a][b], 0, 0, 0);
        __syncthreads();
    }

    // (the loop's last barrier: every wave is done with smem, which now stages the epilogue)
    static_assert(4 * 32 * 36 <= 2 * (ASZ + BSZ), "epilogue staging fits in the operand tiles");
    auto rowmap = [&](int row) __attribute__((always_inline)) -> RowPix {
        if (row >= Mrows) return RowPix{-1, -1};
        if constexpr (MODE == MODE_DGRAD) {
            int ww = row % ph.Wp; int t = row / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
            return RowPix{row, (long)(n * g.H + hh * g.sh + ph.ph) * g.W + ww * g.sw + ph.pw};
        } else {
            return RowPix{row, row};
        }
    };
    conv_epilogue32<MODE, TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, rowmap, phase, split, lane, smem + wid * 32 * 36);
}

// split-K reduction + epilogue (deterministic: slabs summed in split order)
template <int MODE>
__global__ void __launch_bounds__(256)
k_splitk_reduce(const GemmArgs p, int V4) {
    const ConvGeom &g = p.g;
    const int phase = blockIdx.y;
    int Mrows = p.M;
    PhaseInfo ph{};
    if constexpr (MODE == MODE_DGRAD) {
        ph = phase_info(g, phase, g.N);
        Mrows = ph.Mp;
    }
    const long plane = (long)p.M * p.N;
    const float *base = p.slab + (long)phase * p.splits * plane;
    const float ys = p.yp ? plane_scale(p) : 0.f;
    float vmax = 0.f;   // max |output| of this lane (p.ymax)
    if (V4) {  // N % 4 == 0, ldc % 4 == 0, 16-byte aligned C: float4 outputs, V4 lanes per output
        // tpo = V4 (a power of two <= 64) lanes per output: the block's 256 threads are opb = 256 / tpo
        // consecutive outputs x tpo split lanes, lane j summing slabs j, j + tpo, ... in order (four
        // loads in flight) -- a wave's 64 lanes read opb consecutive float4 of one slab -- then lane 0
        // adds the lanes' sums in lane order through LDS.  (Round 5 interleaved the tpo lanes of one
        // output inside a wave: 16 scattered 64-byte pieces per load, one load in flight per lane --
        // 2.3 TB/s on the filter gradients' 32 MB of partials, profiles/r6/reduce_args.txt.)
        const int tpo = V4, opb = 256 / tpo;
        const int o = threadIdx.x % opb, j = threadIdx.x / opb;
        __shared__ f32x4 red[256];
        const int N4 = p.N >> 2;
        const long total = (long)Mrows * N4;
        const long step = (long)tpo * plane;
        for (long e0 = (long)blockIdx.x * opb; e0 < total; e0 += (long)gridDim.x * opb) {   // (block-uniform)
            const long e = e0 + o;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            int row = 0, col = 0;
            if (e < total) {
                row = (int)(e / N4);
                col = (int)(e - (long)row * N4) * 4;
                const float *src = base + (long)row * p.N + col + (long)j * plane;
                int s = j;
                for (; s + 3 * tpo < p.splits; s += 4 * tpo, src += 4 * step) {
                    const f32x4 a0 = *reinterpret_cast<const f32x4 *>(src);
                    const f32x4 a1 = *reinterpret_cast<const f32x4 *>(src + step);
                    const f32x4 a2 = *reinterpret_cast<const f32x4 *>(src + 2 * step);
                    const f32x4 a3 = *reinterpret_cast<const f32x4 *>(src + 3 * step);
                    v += a0;
                    v += a1;
                    v += a2;
                    v += a3;
                }
                for (; s < p.splits; s += tpo, src += step) v += *reinterpret_cast<const f32x4 *>(src);
            }
            if (tpo > 1) {
                red[threadIdx.x] = v;
                __syncthreads();
                if (j == 0)
                    for (int k = 1; k < tpo; ++k) v += red[k * opb + o];
                __syncthreads();
            }
            if (j != 0 || e >= total) continue;
            long pix;
            if constexpr (MODE == MODE_DGRAD) {
                int ww = row % ph.Wp; int t = row / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
                pix = (long)(n * g.H + hh * g.sh + ph.ph) * g.W + ww * g.sw + ph.pw;
            } else {
                pix = row;
            }
            const long off = pix * p.ldc;
            f32x4 ov, mf;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float x = v[q];
                if (p.bias) x += p.bias[col + q];
                mf[q] = epi_mask_factor(p, pix, col + q);
                ov[q] = act_fwd(x, p.act, p.alpha) * mf[q];
            }
            if (p.C) {
                f32x4 *dst = reinterpret_cast<f32x4 *>(p.C + off + col);
                if (p.beta != 0.f) ov += p.beta * (p.mask_acc ? (*dst) * mf : (*dst));
                *dst = ov;
            }
            if (p.yp) store_planes4(p.yp, p.ypC, pix, col, ov, ys);
#pragma unroll
            for (int q = 0; q < 4; ++q) vmax = fmaxf(vmax, fabsf(ov[q]));
        }
        if (p.ymax) block_atomic_absmax(p.ymax, vmax);
        return;
    }
    const long total = (long)Mrows * p.N;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        int row = (int)(e / p.N);
        int col = (int)(e - (long)row * p.N);
        float v = 0.f;
        for (int s = 0; s < p.splits; ++s) v += base[s * plane + (long)row * p.N + col];
        long pix;
        if constexpr (MODE == MODE_DGRAD) {
            int ww = row % ph.Wp; int t = row / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
            pix = (long)(n * g.H + hh * g.sh + ph.ph) * g.W + ww * g.sw + ph.pw;
        } else {
            pix = row;
        }
        const long off = pix * p.ldc;
        if (p.bias) v += p.bias[col];
        const float mf = epi_mask_factor(p, pix, col);
        v = act_fwd(v, p.act, p.alpha) * mf;
        if (p.C) {
            if (p.beta != 0.f) v += p.beta * (p.mask_acc ? p.C[off + col] * mf : p.C[off + col]);
            p.C[off + col] = v;
        }
        if (p.yp) store_planes1(p.yp, p.ypC, pix, col, v, ys);
        vmax = fmaxf(vmax, fabsf(v));
    }
    if (p.ymax) block_atomic_absmax(p.ymax, vmax);
}

// -------------------------------------------------------------------------
// Narrow kernels (GEMM N <= 4): D.last Conv2D(1) (pix2pix.py:217) and the
// G.last Conv2DTranspose(3) (pix2pix.py:169).  MFMA tiles would waste >= 8x
// here; these are VALU dot-product kernels with coalesced activation reads.
// -------------------------------------------------------------------------
constexpr int NARROW_MAX = 8;

// FWD with Co <= 4: one wave per output pixel, lanes over (tap, ci).
__global__ void __launch_bounds__(256)
k_narrow_fwd(const GemmArgs p) {
    const ConvGeom &g = p.g;
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= p.M) return;
    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
    float acc[NARROW_MAX] = {};
    const int Co = g.Co;
    for (int i = 0; i < g.kh; ++i) {
        int hi = ho * g.sh - g.pt + i;
        if (hi < 0 || hi >= g.H) continue;
        for (int j = 0; j < g.kw; ++j) {
            int wi = wo * g.sw - g.pl + j;
            if (wi < 0 || wi >= g.W) continue;
            const float *xp = p.A + ((long)(n * g.H + hi) * g.W + wi) * p.lda;
            const float *wp = p.B + (long)(i * g.kw + j) * g.Ci * Co;
            for (int ci = lane; ci < g.Ci; ci += 64) {
                float xv = xp[ci];
#pragma unroll
                for (int co = 0; co < NARROW_MAX; ++co)
                    if (co < Co) acc[co] += xv * wp[(long)ci * Co + co];
            }
        }
    }
#pragma unroll
    for (int co = 0; co < NARROW_MAX; ++co) {
        float v = acc[co];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        acc[co] = v;
    }
    if (lane == 0) {
        for (int co = 0; co < Co; ++co) {
            float v = acc[co];
            if (p.bias) v += p.bias[co];
            v = epi_mask(p, m, co, act_fwd(v, p.act, p.alpha));
            long off = (long)m * p.ldc + co;
            if (p.beta != 0.f) v += p.beta * p.C[off];
            p.C[off] = v;
        }
    }
}

// DGRAD with Ci <= 4: one thread per output pixel of one phase; w staged in LDS.
__global__ void __launch_bounds__(256)
k_narrow_dgrad(const GemmArgs p, int w_in_lds) {
    extern __shared__ __attribute__((aligned(16))) float wl[];
    const ConvGeom &g = p.g;
    const int phase = blockIdx.y;
    PhaseInfo ph = phase_info(g, phase, g.N);
    const long wsz = (long)g.kh * g.kw * g.Ci * g.Co;
    const float *wsrc = p.B;
    if (w_in_lds) {
        for (long e = threadIdx.x; e < wsz; e += blockDim.x) wl[e] = p.B[e];
        __syncthreads();
        wsrc = wl;
    }
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= ph.Mp) return;
    int ww = m % ph.Wp; int t = m / ph.Wp; int hh = t % ph.Hp; int n = t / ph.Hp;
    const int h = hh * g.sh + ph.ph, w = ww * g.sw + ph.pw;
    const int Ci = g.Ci, Co = g.Co;
    float acc[NARROW_MAX] = {};
    for (int a = 0; a < g.Th; ++a) {
        int i = ph.i0h + a * g.sh;
        int th = h + g.pt - i;
        if (i >= g.kh || th < 0) continue;
        int ho = th / g.sh;
        if (ho >= g.Ho) continue;
        for (int b = 0; b < g.Tw; ++b) {
            int j = ph.i0w + b * g.sw;
            int tw = w + g.pl - j;
            if (j >= g.kw || tw < 0) continue;
            int wo = tw / g.sw;
            if (wo >= g.Wo) continue;
            const float *dyp = p.A + ((long)(n * g.Ho + ho) * g.Wo + wo) * p.lda;
            const float *wp = wsrc + (long)(i * g.kw + j) * Ci * Co;
            if ((Co & 3) == 0 && (p.lda & 3) == 0) {
                for (int co = 0; co < Co; co += 4) {
                    f32x4 d = *reinterpret_cast<const f32x4 *>(dyp + co);
#pragma unroll
                    for (int ci = 0; ci < NARROW_MAX; ++ci) {
                        if (ci < Ci) {
                            const float *wr = wp + (long)ci * Co + co;
                            acc[ci] += d[0] * wr[0] + d[1] * wr[1] + d[2] * wr[2] + d[3] * wr[3];
                        }
                    }
                }
            } else {
                for (int co = 0; co < Co; ++co) {
                    float d = dyp[co];
#pragma unroll
                    for (int ci = 0; ci < NARROW_MAX; ++ci)
                        if (ci < Ci) acc[ci] += d * wp[(long)ci * Co + co];
                }
            }
        }
    }
    const long pix = (long)(n * g.H + h) * g.W + w;
    long off = pix * p.ldc;
    for (int ci = 0; ci < Ci; ++ci) {
        float v = acc[ci];
        if (p.bias) v += p.bias[ci];
        v = epi_mask(p, pix, ci, act_fwd(v, p.act, p.alpha));
        if (p.beta != 0.f) v += p.beta * p.C[off + ci];
        p.C[off + ci] = v;
    }
}

// DGRAD with a few input channels (Ci = CI <= 8, Co 32 or 64): VGG19
// block1_conv1's input gradient (3x3 s1, Ci 3) and D.down1's (4x4 s2, Ci 6).  One thread per output
// pixel of one phase, a block = an 8 x 32 tile of the phase grid; per
// 32-channel chunk the block stages the dy halo its taps read
// ((8+TH-1) x (32+TW-1) pixels, 16-byte loads, pixel stride 36 floats so the
// per-lane ds_read_b128 are conflict-free) and the chunk's weights of the
// phase's TH x TW taps (read as LDS broadcasts), then runs fp32 FMA chains.
// dy is read from HBM once (the GEMM recast writes and re-reads a
// pixels x (taps*Ci) matrix instead).
constexpr int DIR_PH = 8, DIR_PW = 32, DIR_CC = 32, DIR_CS = DIR_CC + 4;

template <int CI, int TH, int TW>
__global__ void __launch_bounds__(256)
k_direct_dgrad(const GemmArgs p, int tiles_x, int tiles_y) {
    constexpr int HH = DIR_PH + TH - 1, HW = DIR_PW + TW - 1;
    __shared__ __attribute__((aligned(16))) float hal[HH * HW * DIR_CS];
    __shared__ __attribute__((aligned(16))) float wl[TH * TW * CI * DIR_CC];
    const ConvGeom &g = p.g;
    // the phases of one tile are adjacent blocks, so they share the tile's dy
    // rows through L2 (phase-major order would re-read dy from HBM per phase)
    const int nph = g.sh * g.sw;
    const PhaseInfo ph = phase_info(g, blockIdx.x % nph, g.N);
    int t = blockIdx.x / nph;
    const int tx = t % tiles_x;
    t /= tiles_x;
    const int ty = t % tiles_y;
    const int n = t / tiles_y;
    const int hh0 = ty * DIR_PH, ww0 = tx * DIR_PW;
    if (hh0 >= ph.Hp || ww0 >= ph.Wp) return;  // block-uniform: this phase's grid is smaller
    // phase pixel (hh, ww) = output pixel (hh*sh + ph, ww*sw + pw); tap a of
    // the phase is filter row i0h + a*sh and reads dy row hh + oh - a
    const int oh = (ph.ph + g.pt - ph.i0h) / g.sh, ow = (ph.pw + g.pl - ph.i0w) / g.sw;
    const int ho0 = hh0 + oh - (TH - 1), wo0 = ww0 + ow - (TW - 1);
    const int lr = threadIdx.x / DIR_PW, lc = threadIdx.x % DIR_PW;
    float acc[CI];
#pragma unroll
    for (int ci = 0; ci < CI; ++ci) acc[ci] = 0.f;
    // dy halo of a chunk: NL 16-byte loads per thread, all issued before any
    // is stored; the next chunk's are issued before this chunk's FMAs
    constexpr int NE = HH * HW * (DIR_CC / 4), NL = (NE + 255) / 256;
    f32x4 hv[NL];
    auto load_halo = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int e = threadIdx.x + 256 * k;
            hv[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (e < NE) {
                const int q = e % (DIR_CC / 4), px = e / (DIR_CC / 4);
                const int r = px / HW, c = px - r * HW;
                const int ho = ho0 + r, wo = wo0 + c;
                if ((unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo)
                    hv[k] = *reinterpret_cast<const f32x4 *>(p.A + ((long)(n * g.Ho + ho) * g.Wo + wo) * p.lda + c0 +
                                                             4 * q);
            }
        }
    };
    load_halo(0);
    for (int c0 = 0; c0 < g.Co; c0 += DIR_CC) {
        __syncthreads();  // every thread is done with the previous chunk
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int e = threadIdx.x + 256 * k;
            if (e < NE) {
                const int q = e % (DIR_CC / 4), px = e / (DIR_CC / 4);
                *reinterpret_cast<f32x4 *>(&hal[px * DIR_CS + 4 * q]) = hv[k];
            }
        }
        for (int e = threadIdx.x; e < TH * TW * CI * DIR_CC; e += 256) {
            const int cc = e % DIR_CC, k = e / DIR_CC;
            const int ci = k % CI, tap = k / CI;
            const int i = ph.i0h + (tap / TW) * g.sh, j = ph.i0w + (tap % TW) * g.sw;
            wl[e] = (i < g.kh && j < g.kw) ? p.B[((long)(i * g.kw + j) * g.Ci + ci) * g.Co + c0 + cc] : 0.f;
        }
        __syncthreads();
        if (c0 + DIR_CC < g.Co) load_halo(c0 + DIR_CC);
#pragma unroll
        for (int a = 0; a < TH; ++a)
#pragma unroll
            for (int b = 0; b < TW; ++b) {
                const float *hp = &hal[((lr + TH - 1 - a) * HW + (lc + TW - 1 - b)) * DIR_CS];
                const float *wp = &wl[(a * TW + b) * CI * DIR_CC];
#pragma unroll
                for (int q = 0; q < DIR_CC / 4; ++q) {
                    const f32x4 d = *reinterpret_cast<const f32x4 *>(hp + 4 * q);
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) {
                        const f32x4 w = *reinterpret_cast<const f32x4 *>(wp + ci * DIR_CC + 4 * q);
                        float v = acc[ci];
                        v = fmaf(d[0], w[0], v);
                        v = fmaf(d[1], w[1], v);
                        v = fmaf(d[2], w[2], v);
                        v = fmaf(d[3], w[3], v);
                        acc[ci] = v;
                    }
                }
            }
    }
    const int hh = hh0 + lr, ww = ww0 + lc;
    if (hh >= ph.Hp || ww >= ph.Wp) return;
    const long pix = (long)(n * g.H + hh * g.sh + ph.ph) * g.W + ww * g.sw + ph.pw;
    const long off = pix * p.ldc;
#pragma unroll
    for (int ci = 0; ci < CI; ++ci) {
        float v = acc[ci];
        if (p.bias) v += p.bias[ci];
        v = epi_mask(p, pix, ci, act_fwd(v, p.act, p.alpha));
        if (p.beta != 0.f) v += p.beta * p.C[off + ci];
        p.C[off + ci] = v;
    }
}

// direct DGRAD kernels instantiated: (Ci, taps per phase) of the layers above
// (measured per layer in the training step: VGG block1_conv1 dgrad 0.210 ->
// 0.172 ms (0.132 with the batched, prefetched halo loads), D.down1 dgrad
// 0.208 -> 0.122 ms; G.last forward with Co 128 ran 0.239 -> 0.38 ms, so
// Co > 64 stays on the GEMM recast)
static bool direct_dgrad_ok(const ConvGeom &g) {
    if (g.Co % DIR_CC || g.Co > 64) return false;
    const bool t33 = g.Th == 3 && g.Tw == 3, t22 = g.Th == 2 && g.Tw == 2;
    return (g.Ci == 3 && (t33 || t22)) || (g.Ci == 6 && t22);
}

static void launch_direct_dgrad(const GemmArgs &a, hipStream_t s) {
    const ConvGeom &g = a.g;
    const int Hp = (g.H + g.sh - 1) / g.sh, Wp = (g.W + g.sw - 1) / g.sw;
    const int tx = (Wp + DIR_PW - 1) / DIR_PW, ty = (Hp + DIR_PH - 1) / DIR_PH;
    const dim3 grid((unsigned)(g.N * tx * ty * g.sh * g.sw));
    if (g.Ci == 3 && g.Th == 3) hipLaunchKernelGGL((k_direct_dgrad<3, 3, 3>), grid, dim3(256), 0, s, a, tx, ty);
    else if (g.Ci == 3) hipLaunchKernelGGL((k_direct_dgrad<3, 2, 2>), grid, dim3(256), 0, s, a, tx, ty);
    else hipLaunchKernelGGL((k_direct_dgrad<6, 2, 2>), grid, dim3(256), 0, s, a, tx, ty);
}

// FWD with Co <= 4 and Ci % 4 == 0: one thread per output pixel, the filter in
// LDS as [tap][ci/4][co][4] (16-byte broadcast reads), 16-byte x loads.
// (The wave-per-pixel kernel above leaves half the lanes idle at Ci 32 and
// spends a 6-step shuffle reduction per output: 0.86 ms for FastSRGAN's
// 3-channel output conv at bs8 512x512.)
constexpr int NFWD_WMAX = 8192;   // filter floats in LDS
// Smallest output (pixels) the thread-per-pixel kernel takes; below it the
// wave-per-pixel k_narrow_fwd runs.  Set from a same-box A/B of the two
// kernels over the SR family's narrow layers (scripts/diag/narrow_ab.py,
// profiles/r3/narrow_ab.txt): px is 8.5x faster at M 2.1M (FastSRGAN's output
// conv), 5.5x at 295K, 1.3x at 16K, 1.1x at 8K; the two tie at the launch
// floor below (M 1152: 14.0 vs 13.8 us, M 64: 16.0 vs 14.3 us).
constexpr long NFWD_PX_MIN_M = 4096;
template <int CO>
__global__ void __launch_bounds__(256)
k_narrow_fwd_px(const GemmArgs p) {
    __shared__ __attribute__((aligned(16))) float wl[NFWD_WMAX];
    const ConvGeom &g = p.g;
    const int ci4 = g.Ci / 4, ntap = g.kh * g.kw;
    for (int e = threadIdx.x; e < ntap * g.Ci * CO; e += 256) {
        // e = ((tap * ci4 + c4) * CO + co) * 4 + q  <-  w[tap][c4*4 + q][co]
        const int q = e & 3, co = (e >> 2) % CO, rest = (e >> 2) / CO;
        const int c4 = rest % ci4, tap = rest / ci4;
        wl[e] = p.B[((long)tap * g.Ci + c4 * 4 + q) * CO + co];
    }
    __syncthreads();
    for (int m = blockIdx.x * 256 + threadIdx.x; m < p.M; m += gridDim.x * 256) {
        const int wo = m % g.Wo, t = m / g.Wo, ho = t % g.Ho, n = t / g.Ho;
        float acc[CO];
#pragma unroll
        for (int co = 0; co < CO; ++co) acc[co] = 0.f;
        for (int i = 0; i < g.kh; ++i) {
            const int hi = ho * g.sh - g.pt + i;
            if (hi < 0 || hi >= g.H) continue;
            for (int j = 0; j < g.kw; ++j) {
                const int wi = wo * g.sw - g.pl + j;
                if (wi < 0 || wi >= g.W) continue;
                const f32x4 *xp = reinterpret_cast<const f32x4 *>(p.A + ((long)(n * g.H + hi) * g.W + wi) * p.lda);
                const f32x4 *wp = reinterpret_cast<const f32x4 *>(wl) + (long)(i * g.kw + j) * ci4 * CO;
#pragma unroll 4
                for (int c = 0; c < ci4; ++c) {
                    const f32x4 x = xp[c];
#pragma unroll
                    for (int co = 0; co < CO; ++co) {
                        const f32x4 w = wp[c * CO + co];
                        acc[co] = fmaf(x[0], w[0], fmaf(x[1], w[1], fmaf(x[2], w[2], fmaf(x[3], w[3], acc[co]))));
                    }
                }
            }
        }
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            float v = acc[co];
            if (p.bias) v += p.bias[co];
            v = epi_mask(p, m, co, act_fwd(v, p.act, p.alpha));
            const long off = (long)m * p.ldc + co;
            if (p.beta != 0.f) v += p.beta * p.C[off];
            p.C[off] = v;
        }
    }
}

// WGRAD with Co < 8: partial[split][k=(tap,ci)][co].  Block (tap, 256-channel
// chunk, pixel split): 256 threads = CL channels x PL = 256/CL pixel lanes
// (CL = Ci rounded up to a power of two, at most 256), four pixels' loads in
// flight per lane; the PL lanes' sums are added through LDS in lane order.
// (One thread per channel left 7/8 of a block idle at Ci 32 and ran FastSRGAN's
// 3-channel output conv's filter gradient at 11.3 ms per step.)
__global__ void __launch_bounds__(256)
k_narrow_wgrad(const GemmArgs p) {
    __shared__ float red[256 * NARROW_MAX];
    const ConvGeom &g = p.g;
    const int nchunk = (g.Ci + 255) / 256;
    const int tap = blockIdx.x / nchunk;
    const int cchunk = blockIdx.x - tap * nchunk;
    int CL = 1;
    while (CL < g.Ci - cchunk * 256 && CL < 256) CL <<= 1;
    const int PL = 256 / CL;
    const int cl = threadIdx.x % CL, pl = threadIdx.x / CL;
    const int ci = cchunk * 256 + cl;
    const bool cok = ci < g.Ci;
    const int split = blockIdx.y;
    const int i = tap / g.kw, j = tap - (tap / g.kw) * g.kw;
    const int Co = g.Co;
    const int pb = split * p.kchunk, pe = min(p.K, pb + p.kchunk);
    float acc[NARROW_MAX] = {};
    constexpr int U = 4;
    // (wo, ho, n) of this lane's next pixel, advanced by PL per pixel (no divisions in the loop)
    int wo = (pb + pl) % g.Wo, ho = ((pb + pl) / g.Wo) % g.Ho, n = (pb + pl) / (g.Wo * g.Ho);
    auto advance = [&]() __attribute__((always_inline)) {
        wo += PL;
        if (wo >= g.Wo) {   // divisions only on a row wrap
            const int q = wo / g.Wo;
            wo -= q * g.Wo;
            ho += q;
            if (ho >= g.Ho) {
                const int q2 = ho / g.Ho;
                ho -= q2 * g.Ho;
                n += q2;
            }
        }
    };
    for (int pix0 = pb + pl; pix0 < pe; pix0 += U * PL) {
        float xv[U], dv[U][NARROW_MAX];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int pix = pix0 + u * PL;
            xv[u] = 0.f;
#pragma unroll
            for (int co = 0; co < NARROW_MAX; ++co) dv[u][co] = 0.f;
            const int hi = ho * g.sh - g.pt + i, wi = wo * g.sw - g.pl + j, nn = n;
            advance();
            if (pix >= pe) continue;
            if (!cok || hi < 0 || hi >= g.H || wi < 0 || wi >= g.W) continue;
            xv[u] = p.A[((long)(nn * g.H + hi) * g.W + wi) * p.lda + ci];
            const float *dyp = p.B + (long)pix * p.ldb;
#pragma unroll
            for (int co = 0; co < NARROW_MAX; ++co)
                if (co < Co) dv[u][co] = dyp[co];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int co = 0; co < NARROW_MAX; ++co) acc[co] += xv[u] * dv[u][co];
    }
#pragma unroll
    for (int co = 0; co < NARROW_MAX; ++co) red[threadIdx.x * NARROW_MAX + co] = acc[co];
    __syncthreads();
    if (pl != 0 || !cok) return;
    for (int l = 1; l < PL; ++l)
#pragma unroll
        for (int co = 0; co < NARROW_MAX; ++co) acc[co] += red[(threadIdx.x + l * CL) * NARROW_MAX + co];
    const int krow = tap * g.Ci + ci;
    for (int co = 0; co < Co; ++co)
        p.slab[((long)split * p.M + krow) * p.N + co] = acc[co];
}

// WGRAD at stride 1 with few filter rows x output channels: the SR family's
// 3-channel output convs (e.g. FastSRGAN's 3x3 32 -> 3 at 512x512) and the
// 3-channel input convs of the SR discriminators (3x3 3 -> 32 at 512x512):
// dW[(tap, ci)][co] = sum over output pixels of x[pixel + tap][ci] * dy[pixel][co].
// A block walks output row segments of NWT_TP pixels: it stages the
// kh x (NWT_TP + kw - 1) x Ci input window and the segment's dy (CG groups of
// 4 channels per pixel) in LDS once; thread t owns slots s = t, t + 256, ...,
// slot s = (filter row q = s / CG, channel group s % CG) with 4 sums in
// registers -- per pixel one ds_read_b32 of x (shared by the CG lanes of a
// row) and one float4 of dy, every x element staged once per segment instead
// of once per tap.  Partials per block [block][Q * CG][4] are summed in block
// order by k_narrow_wgrad_final.  (k_narrow_wgrad above -- one block per tap,
// each lane a chain of 4 pixels' loads in flight -- took 1.04 ms for
// FastSRGAN's output conv at bs8; the 3 -> 32 input conv's filter gradient ran
// 455 us per call on 64 x 64 fp32 tiles, 27 of whose 64 rows exist.)
constexpr int NWT_TP = 64;
constexpr int NWT_QMAX = 4;    // slots per thread: Q * CG <= 1024
static int narrow_tile_groups(const ConvGeom &g) { return (g.Co + 3) / 4; }
static size_t narrow_tile_lds(const ConvGeom &g) {
    return ((size_t)g.kh * (NWT_TP + g.kw - 1) * g.Ci + 4 * NWT_TP * (size_t)narrow_tile_groups(g)) * sizeof(float);
}
static bool narrow_tile_ok(const ConvGeom &g) {
    const long S = (long)g.kh * g.kw * g.Ci * narrow_tile_groups(g);
    return g.sh == 1 && g.sw == 1 && S <= 256L * NWT_QMAX && narrow_tile_lds(g) <= 64 * 1024;
}
static int narrow_tile_segments(const ConvGeom &g) {
    return g.N * g.Ho * ((g.Wo + NWT_TP - 1) / NWT_TP);
}

__global__ void __launch_bounds__(256)
k_narrow_wgrad_tile(const GemmArgs p, int nseg, float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const ConvGeom &g = p.g;
    const int Ci = g.Ci, KW = g.kw, KH = g.kh, Co = g.Co;
    const int CG = (Co + 3) >> 2;
    const int XW = NWT_TP + KW - 1;
    const int XE = KH * XW * Ci;                             // staged x floats
    float *xs = sm;                                          // [KH][XW][Ci]
    f32x4 *ds = reinterpret_cast<f32x4 *>(sm + ((XE + 3) & ~3));   // [NWT_TP][CG] dy
    const bool xv4 = (Ci & 3) == 0 && (p.lda & 3) == 0 && (((uintptr_t)p.A) & 15) == 0;
    const bool dv4 = (Co & 3) == 0 && (p.ldb & 3) == 0 && (((uintptr_t)p.B) & 15) == 0;
    const int S = KH * KW * Ci * CG;
    const int segw = (g.Wo + NWT_TP - 1) / NWT_TP;
    f32x4 acc[NWT_QMAX];
#pragma unroll
    for (int u = 0; u < NWT_QMAX; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const int sx = seg % segw, t = seg / segw;
        const int ho = t % g.Ho, n = t / g.Ho;
        const int wo0 = sx * NWT_TP;
        if (xv4) {
            const int ci4 = Ci >> 2;
            for (int e = threadIdx.x; e < XE / 4; e += 256) {
                const int c4 = e % ci4, r = e / ci4;
                const int col = r % XW, i = r / XW;
                const int hi = ho - g.pt + i, wi = wo0 - g.pl + col;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if ((unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W)
                    v = *reinterpret_cast<const f32x4 *>(p.A + ((long)(n * g.H + hi) * g.W + wi) * p.lda + 4 * c4);
                reinterpret_cast<f32x4 *>(xs)[e] = v;
            }
        } else {
            for (int e = threadIdx.x; e < XE; e += 256) {
                const int c = e % Ci, r = e / Ci;
                const int col = r % XW, i = r / XW;
                const int hi = ho - g.pt + i, wi = wo0 - g.pl + col;
                xs[e] = ((unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W)
                            ? p.A[((long)(n * g.H + hi) * g.W + wi) * p.lda + c] : 0.f;
            }
        }
        for (int e = threadIdx.x; e < NWT_TP * CG; e += 256) {
            const int px = e / CG, cg = e - px * CG;
            const int wo = wo0 + px;
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
            if (wo < g.Wo) {
                const float *dp = p.B + ((long)(n * g.Ho + ho) * g.Wo + wo) * p.ldb + 4 * cg;
                if (dv4) {
                    d = *reinterpret_cast<const f32x4 *>(dp);
                } else {
#pragma unroll
                    for (int co = 0; co < 4; ++co)
                        if (4 * cg + co < Co) d[co] = dp[co];
                }
            }
            ds[e] = d;
        }
        __syncthreads();
        const int npx = min(NWT_TP, g.Wo - wo0);
#pragma unroll
        for (int u = 0; u < NWT_QMAX; ++u) {
            const int sl = threadIdx.x + 256 * u;
            if (sl < S) {
                const int q = sl / CG, cg = sl - q * CG;
                const int tap = q / Ci, c = q - tap * Ci;
                const int i = tap / KW, j = tap - i * KW;
                const float *xr = xs + (i * XW + j) * Ci + c;
                const f32x4 *dr = ds + cg;
                f32x4 a = acc[u];
                for (int px = 0; px < npx; ++px) {
                    const float xv = xr[px * Ci];
                    const f32x4 d = dr[px * CG];
#pragma unroll
                    for (int co = 0; co < 4; ++co) a[co] = fmaf(xv, d[co], a[co]);
                }
                acc[u] = a;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < NWT_QMAX; ++u) {
        const int sl = threadIdx.x + 256 * u;
        if (sl < S) reinterpret_cast<f32x4 *>(part)[(long)blockIdx.x * S + sl] = acc[u];
    }
}

// dW[q][co] = sum over the R partial blocks of part[r][q][co] (+ beta dW), with
// part rows of 4 * CG floats per filter row q: block = 16 outputs x 16 row lanes
// summing rows r = lane, lane + 16, ... in order, then the lanes in lane order
__global__ void __launch_bounds__(256)
k_narrow_wgrad_final(const GemmArgs p, int R, const float *__restrict__ part) {
    __shared__ float red[256];
    const int CG4 = 4 * ((p.N + 3) >> 2);
    const int T = p.M * CG4;
    const int ol = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int o = blockIdx.x * 16 + ol;
    float sacc = 0.f;
    if (o < T) {
#pragma unroll 8
        for (int r = rl; r < R; r += 16) sacc += part[(long)r * T + o];
    }
    red[threadIdx.x] = sacc;
    __syncthreads();
    if (rl == 0 && o < T) {
        const int q = o / CG4, co = o - q * CG4;
        if (co < p.N) {
            float t = red[ol];
            for (int l = 1; l < 16; ++l) t += red[l * 16 + ol];
            float *dst = p.C + (long)q * p.ldc + co;
            *dst = p.beta != 0.f ? t + p.beta * *dst : t;
        }
    }
}

// column sum for bias gradients: out[c] = sum_r dy[r*ld + c] + beta*out[c].
// Block (row chunk, channel chunk): 256 threads = CC channels (adjacent lanes
// read adjacent channels of one row) x RL = 256/CC row lanes, each summing its
// rows in order, then the row lanes in lane order -> partial[c][blockIdx.x].
// (One channel per block with the threads down the rows read one float per
// row: 107 us per call, 3.6 ms of FastSRGAN's step.)
__global__ void __launch_bounds__(256)
k_colsum_partial(const float *dy, int ld, long M, int C, long rows_per_block, float *partial) {
    __shared__ float red[256];
    int CC = 1;
    while (CC < C && CC < 64) CC <<= 1;
    const int RL = 256 / CC;
    const int cl = threadIdx.x % CC, rl = threadIdx.x / CC;
    const int c = blockIdx.y * CC + cl;
    long r0 = (long)blockIdx.x * rows_per_block;
    long r1 = min(M, r0 + rows_per_block);
    float s = 0.f;
    if (c < C) {
#pragma unroll 4
        for (long r = r0 + rl; r < r1; r += RL) s += dy[r * ld + c];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (rl != 0 || c >= C) return;
    for (int l = 1; l < RL; ++l) s += red[l * CC + cl];
    partial[(long)c * gridDim.x + blockIdx.x] = s;
}
// one block per channel: thread t sums partials t, t + 256, ... in order, then a
// fixed-shape LDS tree
__global__ void __launch_bounds__(256) k_colsum_final(const float *partial, int nblk, int C, float *out, float beta) {
    __shared__ float red[256];
    const int c = blockIdx.x;
    float s = 0.f;
    for (int b = threadIdx.x; b < nblk; b += 256) s += partial[(long)c * nblk + b];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = red[0] + (beta != 0.f ? beta * out[c] : 0.f);
}

// ---- recast helpers (see Recast) -------------------------------------------
__global__ void __launch_bounds__(256)
k_transpose(const float *__restrict__ src, int R, int Cc, float *__restrict__ dst, int Rp) {
    // dst[c][r] = src[r][c] for r < R, 0 for R <= r < Rp (row stride Rp)
    const long total = (long)Rp * Cc;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        int c = (int)(e / Rp);
        int r = (int)(e - (long)c * Rp);
        dst[e] = r < R ? src[(long)r * Cc + c] : 0.f;
    }
}

// y[m] = sum over taps of V[input pixel of tap][tap] (+bias, act, beta)   (FWD, Co == 1)
__global__ void __launch_bounds__(256)
k_recast_fwd_gather(const GemmArgs p, const float *__restrict__ V, int nv) {
    const ConvGeom &g = p.g;
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= g.N * g.Ho * g.Wo) return;
    int wo = m % g.Wo; int t = m / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
    float v = 0.f;
    for (int i = 0; i < g.kh; ++i) {
        int hi = ho * g.sh - g.pt + i;
        if (hi < 0 || hi >= g.H) continue;
        for (int j = 0; j < g.kw; ++j) {
            int wi = wo * g.sw - g.pl + j;
            if (wi < 0 || wi >= g.W) continue;
            v += V[((long)(n * g.H + hi) * g.W + wi) * nv + i * g.kw + j];
        }
    }
    if (p.bias) v += p.bias[0];
    v = epi_mask(p, m, 0, act_fwd(v, p.act, p.alpha));
    long off = (long)m * p.ldc;
    if (p.beta != 0.f) v += p.beta * p.C[off];
    p.C[off] = v;
}

// dx[n,h,w,ci] = sum over taps hitting (h,w) of V[(n,ho,wo)][(i,j,ci)]   (DGRAD col2im)
__global__ void __launch_bounds__(256)
k_recast_col2im(const GemmArgs p, const float *__restrict__ V, int nv) {
    const ConvGeom &g = p.g;
    const long total = (long)g.N * g.H * g.W * g.Ci;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int ci = (int)(e % g.Ci);
        const long pix = e / g.Ci;
        const int w = (int)(pix % g.W);
        const int h = (int)((pix / g.W) % g.H);
        const int n = (int)(pix / ((long)g.W * g.H));
        float v = 0.f;
        if (g.Th <= 4 && g.Tw <= 4) {
            // the taps hitting (h, w) are i = i0 + a*sh, j = j0 + b*sw: all their
            // loads issue before the sum, which adds them in the same (i, j)
            // order as the loop below (absent taps add +0: the same bits)
            const int i0 = (h + g.pt) % g.sh, j0 = (w + g.pl) % g.sw;
            float t[4][4];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int i = i0 + a * g.sh, j = j0 + b * g.sw;
                    const int ho = (h + g.pt - i) / g.sh, wo = (w + g.pl - j) / g.sw;
                    const bool ok = a < g.Th && b < g.Tw && i < g.kh && j < g.kw && h + g.pt - i >= 0 &&
                                    w + g.pl - j >= 0 && ho < g.Ho && wo < g.Wo;
                    t[a][b] = ok ? V[((long)(n * g.Ho + ho) * g.Wo + wo) * nv + (i * g.kw + j) * g.Ci + ci] : 0.f;
                }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) v += t[a][b];
        } else {
            for (int i = 0; i < g.kh; ++i) {
                int th = h + g.pt - i;
                if (th < 0 || th % g.sh) continue;
                int ho = th / g.sh;
                if (ho >= g.Ho) continue;
                for (int j = 0; j < g.kw; ++j) {
                    int tw = w + g.pl - j;
                    if (tw < 0 || tw % g.sw) continue;
                    int wo = tw / g.sw;
                    if (wo >= g.Wo) continue;
                    v += V[((long)(n * g.Ho + ho) * g.Wo + wo) * nv + (i * g.kw + j) * g.Ci + ci];
                }
            }
        }
        if (p.bias) v += p.bias[ci];
        v = epi_mask(p, pix, ci, act_fwd(v, p.act, p.alpha));
        long off = pix * p.ldc + ci;
        if (p.beta != 0.f) v += p.beta * p.C[off];
        p.C[off] = v;
    }
}

// G[p_in][(i,j)] = dy[output pixel that reads p_in through tap (i,j)] or 0   (WGRAD, Co == 1)
__global__ void __launch_bounds__(256)
k_recast_wgrad_gather(const GemmArgs p, const float *__restrict__ dy, int lddy, float *__restrict__ G) {
    const ConvGeom &g = p.g;
    const int nt = g.kh * g.kw;
    const long total = (long)g.N * g.H * g.W * nt;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int tap = (int)(e % nt);
        const long pix = e / nt;
        const int w = (int)(pix % g.W);
        const int h = (int)((pix / g.W) % g.H);
        const int n = (int)(pix / ((long)g.W * g.H));
        const int i = tap / g.kw, j = tap - (tap / g.kw) * g.kw;
        float v = 0.f;
        int th = h + g.pt - i, tw = w + g.pl - j;
        if (th >= 0 && tw >= 0 && th % g.sh == 0 && tw % g.sw == 0) {
            int ho = th / g.sh, wo = tw / g.sw;
            if (ho < g.Ho && wo < g.Wo) v = dy[((long)(n * g.Ho + ho) * g.Wo + wo) * lddy];
        }
        G[e] = v;
    }
}

// -------------------------------------------------------------------------
// Host side: descriptor, planner, launch
// -------------------------------------------------------------------------
// tile configs: block tile, wave grid, K-tile depth, min waves/SIMD (register budget),
// resident blocks per CU (LDS / registers), relative cost per FLOP (measured on MI355X)
struct TileCfg {
    int bm, bn, wgm, wgn, bk, minw, bpc;
    double eff;
};
static const TileCfg kCfgs[] = {
    {128, 128, 2, 2, 32, 2, 2, 1.00}, {128, 64, 2, 2, 32, 2, 2, 1.12}, {64, 128, 2, 2, 32, 2, 2, 1.12},
    {64, 64, 2, 2, 32, 2, 3, 1.35},   {32, 128, 1, 4, 32, 2, 3, 1.50}, {128, 128, 2, 2, 16, 3, 3, 1.00},
    {128, 64, 2, 2, 16, 3, 3, 1.12},
    // 32-wide tiles for the 32-channel layers of the SR discriminators (srgan.py:232-272):
    // a 64-wide tile computes half zeros there
    {128, 32, 4, 1, 32, 2, 3, 1.40}, {256, 32, 4, 1, 32, 2, 2, 1.30},
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);
// bf16x6 kernel configs (conv_x6.hip launch_gemm_x6), K-tile 16
static const TileCfg kX6Cfgs[] = {
    {128, 128, 2, 2, 16, 2, 2, 1.00}, {128, 64, 2, 2, 16, 2, 2, 1.15}, {64, 128, 2, 2, 16, 2, 2, 1.15},
    {64, 64, 2, 2, 16, 3, 4, 1.40},   {256, 128, 4, 2, 16, 2, 1, 1.00}, {128, 256, 2, 4, 16, 2, 1, 0.90},
    {128, 32, 4, 1, 16, 3, 4, 1.45},   // 32-wide (SR discriminators' 32-channel layers)
};
constexpr int kNumX6Cfgs = sizeof(kX6Cfgs) / sizeof(kX6Cfgs[0]);
// fp16 kernel configs (conv_x6.hip launch_gemm_f16: the same tiles, K-tile 32)
static const TileCfg kF16Cfgs[] = {
    {128, 128, 2, 2, 32, 2, 2, 1.00}, {128, 64, 2, 2, 32, 2, 2, 1.15}, {64, 128, 2, 2, 32, 2, 2, 1.15},
    {64, 64, 2, 2, 32, 3, 4, 1.40},   {256, 128, 4, 2, 32, 2, 1, 1.00}, {128, 256, 2, 4, 32, 2, 1, 0.90},
    {128, 32, 4, 1, 32, 3, 4, 1.45},   // 32-wide (SR discriminators' 32-channel layers)
};
constexpr int kNumF16Cfgs = sizeof(kF16Cfgs) / sizeof(kF16Cfgs[0]);
// fp16x3 kernel configs (conv_x6.hip launch_gemm_x3: four images per K-tile of 32, the
// 128-wide tiles one K-tile ahead in two LDS buffers)
static const TileCfg kX3Cfgs[] = {
    {128, 128, 2, 2, 32, 2, 2, 1.00}, {128, 64, 2, 2, 32, 2, 3, 1.15}, {64, 128, 2, 2, 32, 2, 3, 1.15},
    {64, 64, 2, 2, 32, 3, 3, 1.40},   {256, 128, 4, 2, 32, 2, 1, 1.00}, {128, 256, 2, 4, 32, 2, 1, 0.90},
    {128, 32, 4, 1, 32, 3, 2, 1.45},
};
constexpr int kNumX3Cfgs = sizeof(kX3Cfgs) / sizeof(kX3Cfgs[0]);

struct OpPlan {
    int narrow;      // 1 => VALU narrow kernel
    int direct;      // narrow DGRAD on k_direct_dgrad (dy halo staged in LDS)
    int x6;          // 1 => bf16x6 split-precision kernel (kX6Cfgs), 2 => fp16 (kF16Cfgs), 3 => fp16x3 halo
                     // forward (DG_MATH_F16X3), else fp32 MFMA (kCfgs)
    int cfg;         // tile config index
    int vec;
    int splits, kchunk;
    int M, N, K, nphase;
    int mtiles, ntiles;
    size_t slab_bytes;  // split-K partial slabs
    size_t gemm_bytes;  // workspace of the GEMM (split-K slabs + bf16x6 planes)
    size_t ws_bytes;    // total workspace of the layer op (GEMM + bias partials)
    size_t colsum_off;  // bwd_filter: offset of the bias column-sum partials
    // bf16x6: operand plane dims (rows x C for A and B) and workspace offsets
    long x6_ra, x6_rb;
    int x6_ca, x6_cb;
    size_t x6_a_off, x6_b_off;
    // halo-tiled bf16x6 kernel (conv_x6h.hip): 1 = stride-1 3x3 FWD / DGRAD,
    // 2 = stride-2 4x4 DGRAD phases; cfg = its BN, tiles of hph x 16 output pixels
    // (hph 8, or 16: the fp16x3 3x3 16 x 16 patch on 8 waves)
    int halo, htx, hty, hph;
    // fp16x3 halo plans without split-K: patches per block (persistent blocks, conv_x6h.hip)
    int ptiles;
    // small-Cin 4x4 stride-2 kernels (conv_small.hip); WGRAD: conv-view output rows per block
    int small, small_rows;
    // single-output-channel direct kernels (conv_co1.hip)
    int co1;
    // ConvT(3) forward on the fused MFMA + col2im kernel (conv_tlast.hip)
    int tlast;
    // narrow stride-1 filter gradient on row segments (k_narrow_wgrad_tile): partial blocks
    int ntile;
    // fp16x3 input gradient: workspace offset of the max |dy| float (no scale source set)
    size_t x3_max_off;   // (+X3_SLOT floats: max |x| when the x operand has no scale source)
};

// A narrow op (GEMM N <= 8) recast as a 1x1-geometry MFMA GEMM plus a gather:
//   FWD,   Co == 1 : V[p_in][(i,j)]      = x[p_in][:] . w[(i,j)][:]   ; y = shift-and-add of V
//   DGRAD, Ci <= 8 : V[p_out][(i,j,ci)]  = dy[p_out][:] . w[(i,j,ci)][:] ; dx = col2im(V)
//   WGRAD, Co == 1 : dw[(i,j)][ci]       = sum_p G[p][(i,j)] x[p][ci], G = dy gathered per tap
struct Recast {
    int on;
    int mode1;          // engine mode of the 1x1 GEMM
    ConvGeom g1;        // its geometry (N=1, H=1, W=pixels)
    OpPlan p1;          // its plan
    int nv;             // columns of V / G
    int nvp;            // row stride of V (nv rounded up so the 1x1 GEMM stays on the bf16x6 path)
    size_t wt_off, v_off, slab_off, bytes;
};

}  // namespace dg

struct dg_conv_desc_s {
    int transpose;
    int math;                        // DG_MATH_*
    // fp16x3 input gradient scale context (dg_conv_set_grad_scale): sources (m, g) of the dy
    // and dx planes' scales, and where max |dx| goes (device pointers; NULL = unset)
    const float *gs_dy_m, *gs_dy_g, *gs_dx_m, *gs_dx_g;
    float *gs_dx_max;
    // fp16x3 activation scale context (dg_conv_set_act_scale): source (m, g, c) of the x planes'
    // scale, of the forward's output planes' scale, and where max |y| of the forward goes
    const float *as_x_m, *as_x_g, *as_x_c, *as_y_m, *as_y_g, *as_y_c;
    float *as_y_max;
    int N, H, W, Cin, Cout, Ho, Wo;  // layer view
    dg::ConvGeom g;                  // conv view
    dg::OpPlan plan[3];              // indexed by DG_OP_*
    dg::Recast rc[3];
};

namespace dg {

static int engine_mode(const dg_conv_desc_s *d, int op) {
    // layer op -> conv-view engine
    if (!d->transpose) return op == DG_OP_FWD ? MODE_FWD : (op == DG_OP_BWD_DATA ? MODE_DGRAD : MODE_WGRAD);
    return op == DG_OP_FWD ? MODE_DGRAD : (op == DG_OP_BWD_DATA ? MODE_FWD : MODE_WGRAD);
}

static bool cfg_vec(const ConvGeom &g, int mode, int bk) {
    if (mode == MODE_FWD) return g.Ci % bk == 0;
    if (mode == MODE_DGRAD) return g.Co % bk == 0;
    return g.Ci % 4 == 0;
}

// Tile config + split-K count for plan pl (M, N, K, nphase set) from a config
// table; returns the modelled time.  Modelled time of a candidate:
//   rounds x (blocks per CU x per-block MFMA work) / (CU peak x occupancy efficiency)
// + split-K slab traffic, where blocks per CU = min(resident limit, blocks / 256).
// Plan features switched off for same-box A/B runs: DG_PLAN_DISABLE is a
// comma-separated list of {shortk, small, co1, tlast, direct, halo, halo2, halo4, halo_f16, xcd_phase, narrow_px, ntile,
// tile32, f16planes, halo32}
// (read when a descriptor is planned; unset in production runs)
static bool plan_off(const char *feature) {
    const char *list = getenv("DG_PLAN_DISABLE");
    if (!list) return false;
    const size_t n = strlen(feature);
    for (const char *q = list; *q;) {
        const char *e = strchr(q, ',');
        const size_t len = e ? (size_t)(e - q) : strlen(q);
        if (len == n && !strncmp(q, feature, n)) return true;
        if (!e) break;
        q = e + 1;
    }
    return false;
}

static double choose_tiles(OpPlan &pl, const TileCfg *cfgs, int ncfg, double peak, const char *force_env,
                           int rule = -1) {
    const double cu_flops = peak / 256.0;
    static const double occ_eff[] = {0.0, 0.62, 0.80, 0.88, 0.92};
    int forced = rule;   // (a measured per-shape rule of the caller; the environment overrides it)
    if (const char *f = getenv(force_env)) forced = atoi(f);
    // DG_FORCE_SPLITS: split-K count for sweeps (scripts/diag/deep_sweep.py); unset in production
    long fsplits = 0;
    if (const char *f = getenv("DG_FORCE_SPLITS")) fsplits = atol(f);
    // fp32 GEMMs with a short K over many rows (the Cin 3/6 layers and the
    // G.last recast: K 27..128, M >= 64K): per-layer sweep on MI355X (bs32)
    // has the 128x64 BK-16 three-blocks-per-CU tile fastest on every one
    // (D.down1 fwd 0.159 -> 0.117 ms, G.last bwd_data 0.188 -> 0.166, G.last
    // recast 0.241 -> 0.219); the MFMA-time model misses their prologue /
    // epilogue weight
    if (forced < 0 && cfgs == kCfgs && pl.K <= 256 && pl.N <= 128 && (long)pl.M * pl.nphase >= 65536 &&
        !plan_off("shortk"))
        forced = (pl.N <= 32 && !plan_off("tile32")) ? 7 : 6;   // (32 columns: the 128 x 32 tile)
    int best = -1; double best_t = 1e30; long best_splits = 1;
    for (int c = 0; c < ncfg; ++c) {
        const TileCfg &t = cfgs[c];
        if (forced >= 0 && c != forced) continue;
        if (forced < 0 && pl.N <= 64 && t.bn > 64) continue;
        if (forced < 0 && t.bn == 32 && plan_off("tile32")) continue;
        long mt = (pl.M + t.bm - 1) / t.bm, nt = (pl.N + t.bn - 1) / t.bn;
        long tiles = mt * nt * pl.nphase;
        long ktiles = (pl.K + t.bk - 1) / t.bk;
        for (long splits = 1; splits <= std::max<long>(1, fsplits > 0 ? ktiles : ktiles / 4); splits *= 2) {
            if (fsplits > 0 && splits != fsplits) continue;
            long kt_per = (ktiles + splits - 1) / splits;
            long blocks = tiles * splits;
            long bpc = std::min<long>(t.bpc, (blocks + 255) / 256);
            double rounds = std::ceil((double)blocks / (256.0 * bpc));
            // occupancy in 4-wave units: an 8-wave block counts as two
            const long occ = std::min<long>(4, bpc * (t.wgm * t.wgn) / 4);
            const double eff = t.eff;
            double tc = rounds * bpc * 2.0 * t.bm * t.bn * kt_per * t.bk * eff / (cu_flops * occ_eff[occ]);
            double ts = splits > 1 ? (double)splits * pl.nphase * pl.M * pl.N * 8.0 / 5.0e12 + 2e-6 : 0.0;
            if (tc + ts < best_t) { best_t = tc + ts; best = c; best_splits = splits; }
            if (blocks >= 1024 && fsplits <= 0) break;
        }
    }
    if (best < 0) best = 0;
    pl.cfg = best;

    const TileCfg &t = cfgs[best];
    long ktiles = (pl.K + t.bk - 1) / t.bk;
    long kt_per = (ktiles + best_splits - 1) / best_splits;
    pl.kchunk = (int)(kt_per * t.bk);
    pl.splits = (int)((ktiles + kt_per - 1) / kt_per);
    pl.mtiles = (pl.M + t.bm - 1) / t.bm;
    pl.ntiles = (pl.N + t.bn - 1) / t.bn;
    return best_t;
}

// x6_extra: seconds the split-precision path costs beyond its GEMM and split passes (plan_all:
// a filter gradient whose operands no other op of the layer splits measures and splits both)
static OpPlan make_plan(const ConvGeom &g, int mode, int math, double x6_extra = 0.0) {
    OpPlan pl{};
    if (mode == MODE_FWD) {
        pl.M = g.N * g.Ho * g.Wo; pl.N = g.Co; pl.K = g.kh * g.kw * g.Ci; pl.nphase = 1;
        pl.narrow = g.Co < 8;
    } else if (mode == MODE_DGRAD) {
        pl.nphase = g.sh * g.sw;
        int Hp = (g.H + g.sh - 1) / g.sh, Wp = (g.W + g.sw - 1) / g.sw;
        pl.M = g.N * Hp * Wp; pl.N = g.Ci; pl.K = g.Th * g.Tw * g.Co;
        pl.narrow = g.Ci < 8;
    } else {
        pl.M = g.kh * g.kw * g.Ci; pl.N = g.Co; pl.K = g.N * g.Ho * g.Wo; pl.nphase = 1;
        pl.narrow = g.Co < 8;
    }
    pl.vec = cfg_vec(g, mode, 32);
    if (co1_ok(g, mode) && math != DG_MATH_FP16 && !plan_off("co1")) {
        // Co == 1 (PatchGAN last layer): direct kernels, exact fp32 FMA chains
        pl.co1 = 1; pl.narrow = 0;
        pl.splits = 1; pl.kchunk = pl.K; pl.mtiles = pl.ntiles = 1;
        pl.slab_bytes = mode == MODE_WGRAD ? (size_t)co1_wgrad_blocks(g) * g.kh * g.kw * g.Ci * sizeof(float) : 0;
        pl.ws_bytes = pl.gemm_bytes = pl.slab_bytes;
        if (getenv("DG_PLAN_DEBUG"))
            fprintf(stderr, "[dg plan] mode %d M=%d N=%d K=%d -> co1\n", mode, pl.M, pl.N, pl.K);
        return pl;
    }
    if (pl.narrow) {
        pl.splits = 1; pl.kchunk = pl.K; pl.ws_bytes = 0; pl.slab_bytes = 0;
        if (mode == MODE_WGRAD && narrow_tile_ok(g) && !plan_off("ntile")) {
            pl.ntile = 1;
            pl.splits = std::min(1024, narrow_tile_segments(g));   // partial blocks
            pl.slab_bytes = (size_t)pl.splits * pl.M * 4 * narrow_tile_groups(g) * sizeof(float);
            pl.ws_bytes = pl.slab_bytes;
        } else if (mode == MODE_WGRAD) {
            // pixels split so that taps*ci_chunks*splits ~ 1024 blocks
            long blocks = (long)g.kh * g.kw * ((g.Ci + 255) / 256);
            int s = (int)std::max<long>(1, std::min<long>(1024 / std::max<long>(blocks, 1), pl.K / 64));
            pl.splits = std::max(1, s);
            pl.kchunk = (pl.K + pl.splits - 1) / pl.splits;
            pl.slab_bytes = (size_t)pl.splits * pl.M * pl.N * sizeof(float);
            pl.ws_bytes = pl.slab_bytes;
        }
        pl.gemm_bytes = pl.ws_bytes;
        return pl;
    }
    if (mode == MODE_WGRAD && g.Ci < 8 && narrow_tile_ok(g) && !plan_off("ntile")) {
        // 1-7 input channels at stride 1 (the SR discriminators' 3 -> 32 input conv): the
        // filter-gradient GEMM has Q = kh*kw*Ci <= 63 rows; the row-segment kernel instead
        pl.ntile = 1;
        pl.splits = std::min(1024, narrow_tile_segments(g));
        pl.kchunk = pl.K; pl.mtiles = pl.ntiles = 1;
        pl.slab_bytes = (size_t)pl.splits * pl.M * 4 * narrow_tile_groups(g) * sizeof(float);
        pl.ws_bytes = pl.gemm_bytes = pl.slab_bytes;
        if (getenv("DG_PLAN_DEBUG"))
            fprintf(stderr, "[dg plan] mode %d M=%d N=%d K=%d -> ntile blocks %d\n", mode, pl.M, pl.N, pl.K, pl.splits);
        return pl;
    }
    if (small_conv_ok(g, mode, 0) && !plan_off("small")) {
        // 3 / 6 input channels, 4x4 stride 2 (G.down1, D.down1, G.last's gradients): exact fp32
        // on the 32x32x2 MFMA whatever the math mode (neither low-precision path takes Cin 3 / 6)
        pl.small = 1;
        pl.splits = 1; pl.kchunk = pl.K; pl.mtiles = pl.ntiles = 1;
        if (mode == MODE_WGRAD) {
            pl.small_rows = small_wgrad_rows_per_block(g);
            const int rows = g.N * g.Ho;
            pl.splits = (rows + pl.small_rows - 1) / pl.small_rows;
        }
        pl.slab_bytes = pl.splits > 1 ? (size_t)pl.splits * pl.M * pl.N * sizeof(float) : 0;
        pl.ws_bytes = pl.gemm_bytes = pl.slab_bytes;
        if (getenv("DG_PLAN_DEBUG"))
            fprintf(stderr, "[dg plan] mode %d M=%d N=%d K=%d -> small splits %d\n", mode, pl.M, pl.N, pl.K, pl.splits);
        return pl;
    }
    // Tile + split-K choice: the cheaper of the fp32 kernel and (math mode
    // BF16X6, eligible shapes) the bf16x6 kernel plus its two split passes.
    double t32 = choose_tiles(pl, kCfgs, kNumCfgs, 157.3e12, "DG_FORCE_CFG");
    int x6_ok = 0;
    long ra = 0, ca = 0, rb = 0, cb = 0;
    if (mode == MODE_FWD) {
        x6_ok = g.Ci % 16 == 0 && g.Co % 16 == 0;
        ra = (long)g.N * g.H * g.W; ca = g.Ci; rb = (long)g.kh * g.kw * g.Ci; cb = g.Co;
    } else if (mode == MODE_DGRAD) {
        x6_ok = g.Co % 16 == 0;
        ra = (long)g.N * g.Ho * g.Wo; ca = g.Co; rb = (long)g.kh * g.kw * g.Ci; cb = g.Co;
    } else {
        x6_ok = g.Ci % 16 == 0 && g.Co % 16 == 0;
        ra = (long)g.N * g.H * g.W; ca = g.Ci; rb = (long)g.N * g.Ho * g.Wo; cb = g.Co;
    }
    // (the bf16x6 kernel keeps a per-row bitmask of valid taps: at most 32 taps; DG_MATH_F16X3
    // is bf16x6 wherever its fp16x3 forward does not apply)
    x6_ok = x6_ok && (math == DG_MATH_BF16X6 || math == DG_MATH_F16X3) && 6.0 * ra * ca < 2.0e9 &&
            6.0 * rb * cb < 2.0e9 && g.kh * g.kw <= 32;
    // (DG_MATH_F16X3: the halo kernel's fp16x3 form for 3x3 stride-1 forwards (Cin % 32 == 0,
    // Cout % 16 == 0, Cout > 32) and input gradients (Cout % 32 == 0 chunks the reduction over
    // output channels, Cin % 16 == 0 and Cin > 32 the BN 64 / 128 tiles), see hx3 below)
    const bool x3_geom = math == DG_MATH_F16X3 && g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1 &&
                         !plan_off("x3") && !plan_off("halo") &&
                         ((mode == MODE_FWD && g.Ci % 32 == 0 && g.Co % 16 == 0 && g.Co > 32) ||
                          (mode == MODE_DGRAD && g.Co % 32 == 0 && g.Ci % 16 == 0 && g.Ci > 32 &&
                           !plan_off("x3dgrad")));
    // fp16x3 on the implicit-GEMM kernel (conv_x6.hip NI 4) for every other eligible op of a
    // DG_MATH_F16X3 descriptor: 32-channel chunks of the activation / gradient operand,
    // 16-column weight groups
    const bool x3_gen = math == DG_MATH_F16X3 && !plan_off("x3") && !plan_off("x3gen") && g.kh * g.kw <= 32 &&
                        ((mode == MODE_FWD && g.Ci % 32 == 0 && g.Co % 16 == 0) ||
                         (mode == MODE_DGRAD && g.Co % 32 == 0 && g.Ci % 16 == 0) ||
                         (mode == MODE_WGRAD && g.Ci % 32 == 0 && g.Co % 32 == 0));
    if (x6_ok) {
        OpPlan p6 = pl;
        double t6 = choose_tiles(p6, kX6Cfgs, kNumX6Cfgs, 2516.6e12 / 6.0, "DG_FORCE_X6CFG");
        t6 += (double)(ra * ca + rb * cb) * 10.0 / 4.0e12 + 4e-6 + x6_extra;  // split passes: read 4 B, write 6 B
        // (the implicit-GEMM fp16x3 ops where the split path beats the fp32 tiles at all: on
        // pix2pix's deepest layers (M 32..128 rows) the fp32 tiles win; DG_FORCE_X3: every
        // eligible op, for the kernel tests at small sizes.  The halo kernel's fp16x3 3x3 layers
        // stay forced: the network picks its math by image size, sr_trainer.VGGNetwork.  Plans
        // of one network in different arithmetics are safe: the host keeps weight planes per
        // layout (dg_conv_planes_format / _size), dgan/graph.py, tests/test_mixed_math_gpu.py)
        if (t6 < t32 || getenv("DG_FORCE_X6CFG") || x3_geom || (x3_gen && getenv("DG_FORCE_X3"))) {
            pl = p6;
            pl.x6 = 1;
            pl.x6_ra = ra; pl.x6_ca = (int)ca; pl.x6_rb = rb; pl.x6_cb = (int)cb;
        }
    }
    if (math == DG_MATH_FP16) {
        // the reference's mixed_float16 policy: one fp16 plane per operand, K-tiles of 32
        int ok = 0;
        if (mode == MODE_FWD) ok = g.Ci % 32 == 0 && g.Co % 16 == 0;
        else if (mode == MODE_DGRAD) ok = g.Co % 32 == 0;
        else ok = g.Ci % 16 == 0 && g.Co % 16 == 0;
        ok = ok && 2.0 * ra * ca < 2.0e9 && 2.0 * rb * cb < 2.0e9 && g.kh * g.kw <= 32;
        if (ok) {
            pl.x6 = 0;
            choose_tiles(pl, kF16Cfgs, kNumF16Cfgs, 2516.6e12, "DG_FORCE_F16CFG");
            pl.x6 = 2;
            pl.x6_ra = ra; pl.x6_ca = (int)ca; pl.x6_rb = rb; pl.x6_cb = (int)cb;
        }
    }
    if (!pl.x6) choose_tiles(pl, kCfgs, kNumCfgs, 157.3e12, "DG_FORCE_CFG");
    // halo-tiled kernel: 3x3 stride-1 FWD / DGRAD (kt 3), and the sub-pixel
    // phases of a 4x4 stride-2 DGRAD (kt 2: ConvT forwards, down-block input gradients)
    const bool h33 = (mode == MODE_FWD || mode == MODE_DGRAD) && g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1 &&
                     pl.K % 144 == 0;
    // (phase grids that fill at least 3/4 of their 8 x 16 patches: on the deep
    // U-Net layers -- 8x8 and smaller phase grids -- the generic tiles win,
    // e.g. up3's forward 0.086 vs 0.243 ms per step)
    const int hp2 = (g.H + 1) / 2, wp2 = (g.W + 1) / 2;
    const bool h22 = mode == MODE_DGRAD && g.kh == 4 && g.kw == 4 && g.sh == 2 && g.sw == 2 && g.Th == 2 &&
                     g.Tw == 2 && pl.K % 64 == 0 &&
                     4L * hp2 * wp2 >= 3L * ((hp2 + 7) / 8 * 8) * ((wp2 + 15) / 16 * 16) && !plan_off("halo2");
    // (stride-1 4x4: the PatchGAN's 512-channel conv, input gradient only: its
    // forward measured 0.709 vs 0.668 ms on the generic 128 x 256 tiles at bs16 x2,
    // the input gradient 0.666 vs 0.690)
    const bool h44 = mode == MODE_DGRAD && g.kh == 4 && g.kw == 4 && g.sh == 1 && g.sw == 1 &&
                     pl.K % 256 == 0 && !plan_off("halo4");
    // (fp16: 3x3 only, 32-channel chunks; the forward's pool epilogue stays bf16x6)
    const bool hf16 = pl.x6 == 2 && h33 && pl.K % 288 == 0 && pl.N % 16 == 0 && !plan_off("halo_f16");
    // fp16x3 forward (DG_MATH_F16X3): 3x3 stride-1 layers with 32-channel chunks and at
    // least 48 output columns (BN 64 / 128 tiles) -- VGG19's layers after block1_conv1
    const bool hx3 = x3_geom && pl.x6 == 1 && h33 && pl.K % 288 == 0 && 4.0 * ra * ca < 2.0e9 &&
                     4.0 * rb * cb < 2.0e9;
    // fp16x3 stride-2 4x4 input-gradient phases on the halo kernel (ConvT forwards, down-block
    // input gradients of G / D) where the implicit-GEMM fp16x3 plan applies (32-channel chunks)
    const bool hx3p = x3_gen && pl.x6 == 1 && h22 && pl.K % 128 == 0 && 4.0 * ra * ca < 2.0e9 &&
                      4.0 * rb * cb < 2.0e9 && !plan_off("x3h2");
    // fp16x3 stride-1 4x4 (the PatchGAN's 512-channel conv, forward and input gradient) on the
    // halo kernel: 11 x 19 halo, BN 64 (72.4 KB, two blocks per CU) -- full step 982 vs 972 img/s
    // on the implicit-GEMM fp16x3 tiles (profiles/r5/ab_x3h_kt4.txt; DG_PLAN_DISABLE=x3h4)
    const bool f44 = mode == MODE_FWD && g.kh == 4 && g.kw == 4 && g.sh == 1 && g.sw == 1;
    const bool hx3q = x3_gen && pl.x6 == 1 && (h44 || f44) && pl.K % 512 == 0 && 4.0 * ra * ca < 2.0e9 &&
                      4.0 * rb * cb < 2.0e9 && !plan_off("x3h4");
    if ((pl.x6 == 1 && (h33 || h22 || h44 || hx3q) || hf16) && !plan_off("halo")) {
        // each input pixel staged once per channel chunk instead of once per tap
        const int ntap = h33 ? 9 : (h44 || f44 ? 16 : 4);
        const int bkc = (pl.x6 == 2 || hx3 || hx3p || hx3q) ? 32 : 16;   // channels per chunk
        int Hout, Wout;
        if (mode == MODE_FWD) { Hout = g.Ho; Wout = g.Wo; }
        else if (h33 || h44) { Hout = g.H; Wout = g.W; }
        else { Hout = (g.H + 1) / 2; Wout = (g.W + 1) / 2; }   // phase 0's grid, the largest
        pl.halo = h33 ? 1 : (h44 || f44 ? 4 : 2);
        // fp16x3 3x3 on 16 x 16 patches (8 waves, one block per CU): the K >= 4096 layers (512
        // reduction channels: VGG19 block4_conv2-4 forward and input gradient, 4-6 % faster, one
        // stream) where the grid still fills the chip at one block per CU; the shorter-K layers ran
        // 2-11 % slower on it (profiles/r6/ab_x3h_ph16.txt).  DG_X3H_PH=8|16 forces,
        // DG_PLAN_DISABLE=x3h16: 8 x 16 everywhere
        pl.hph = 8;
        if (hx3 && Hout >= 16 && pl.K >= 4096 && !plan_off("x3h16")) {
            const long t16 = (long)g.N * ((Wout + 15) / 16) * ((Hout + 15) / 16) * ((pl.N + 127) / 128);
            pl.hph = t16 >= 256 ? 16 : 8;
        }
        if (hx3)
            if (const char *e = getenv("DG_X3H_PH")) pl.hph = atoi(e) == 16 && Hout >= 16 ? 16 : 8;
        pl.htx = (Wout + 15) / 16;
        pl.hty = (Hout + pl.hph - 1) / pl.hph;
        // (4x4: BN 128 needs 93 KB of LDS -- one block per CU -- and measured 0.685 vs
        // 0.666 ms for BN 64, which keeps two)
        // (32 output columns, 3x3: BN 32 -- the SR family's 32-channel layers; a 64-wide tile
        // spends half its MFMAs on zero columns there)
        pl.cfg = pl.N > 64 && !h44 && !f44 ? 128 : (h33 && pl.N <= 32 && !plan_off("halo32") ? 32 : 64);
        pl.mtiles = g.N * pl.htx * pl.hty;
        // (same-box A/B of the target: 256 -0.2%, 1024 -0.8% full step vs 512)
        long target = 512;
        // (diagnostic: DG_X3_TARGET sets the fp16x3 plans' block target for same-box sweeps)
        if (hx3 && getenv("DG_X3_TARGET")) target = atol(getenv("DG_X3_TARGET"));
        // fp16x3 3x3 grids short of the target at BN 128: BN 64 tiles, twice the blocks, instead
        // of (twice the) split-K, whose partial slabs and reduce launch cost more than the halved
        // tile -- VGG19 block5 at bs32 0.148 -> 0.140 ms fwd, 0.152 -> 0.142 bwd_data, block4_conv1
        // bwd_data 0.261 -> 0.255 (profiles/r5/ab_x3h_bn64.txt; DG_PLAN_DISABLE=x3h_bn64: BN 128)
        if (pl.hph == 16) target /= 2;   // (one block per CU)
        if (hx3 && pl.cfg == 128 && (long)pl.mtiles * ((pl.N + 127) / 128) * pl.nphase < target &&
            !plan_off("x3h_bn64"))
            pl.cfg = 64;
        pl.ntiles = (pl.N + pl.cfg - 1) / pl.cfg;
        // split-K over channel chunks (at least two per split) until ~2 blocks per CU
        const long nch = pl.K / (bkc * ntap), blocks = (long)pl.mtiles * pl.ntiles * pl.nphase;
        long splits = 1;
        while (blocks * splits < target && splits * 4 <= nch) splits *= 2;
        const long cps = (nch + splits - 1) / splits;
        pl.kchunk = (int)(cps * bkc * ntap);
        pl.splits = (int)((nch + cps - 1) / cps);
        if (hx3 || hx3p || hx3q) pl.x6 = 3;
        // fp16x3 plans with more patches than resident blocks (2 per CU): each block runs
        // several patches back to back, the next patch's halo and weights fetched under the
        // current patch's MFMAs, so a block waits for HBM once instead of once per patch.
        // ~512 blocks (one per slot) for the stride-2 phases and for 3x3 layers of <= 4
        // channel chunks per patch (VGG19 block1_conv2 fwd 0.959 -> 0.832 ms, bwd_data 1.000
        // -> 0.830, G up7 fwd 0.351 -> 0.304, down2 bwd_data 0.220 -> 0.191 at bs32); deeper
        // 3x3 layers amortise their prologue over >= 72 K-tiles and measured 1-2 % slower at
        // 512, so ~2048 there (profiles/r5/ab_x3h_persistent.txt)
        // (DG_X3H_PTILES: patches per block, DG_X3H_PDIV: the block target, for same-box A/B)
        pl.ptiles = 1;
        if ((hx3 || hx3p || hx3q) && pl.splits == 1) {
            const long tot = (long)pl.mtiles * pl.ntiles * pl.nphase;
            long pdiv = hx3p || nch <= 4 ? 512 : 2048;
            if (pl.hph == 16) pdiv /= 2;   // (one block per CU)
            if (const char *e = getenv("DG_X3H_PDIV")) pdiv = std::max(1L, atol(e));
            long pt = tot / pdiv;
            if (const char *e = getenv("DG_X3H_PTILES")) pt = atol(e);
            pl.ptiles = (int)std::max(1L, std::min(pt, 64L));
        }
    }
    if (x3_gen && pl.x6 == 1 && 4.0 * ra * ca < 2.0e9 && 4.0 * rb * cb < 2.0e9) {
        pl.halo = 0; pl.htx = pl.hty = 0;
        // short-K forward / input-gradient GEMMs (K = 16 taps x 64..128 channels: G / D down2-3
        // forwards, the up6 / up7 input gradients): the 64 x 128 tile at K 1024 and 128 x 128 at
        // K 2048 -- the MFMA-time model's 128 x 256 pick loses there to its prologue / epilogue
        // share (bs32 sweep: up7 bwd_data 0.406 -> 0.323 ms, D down2 fwd 0.238 -> 0.210, G down3
        // fwd 0.182 -> 0.167, up6 bwd_data 0.282 -> 0.263; profiles/r5/x3cfg_sweep.txt;
        // DG_PLAN_DISABLE=x3shortk: the model's pick)
        const int rule = mode == MODE_WGRAD || pl.N <= 64 || plan_off("x3shortk") ? -1
                         : (pl.K <= 1024 ? 2 : (pl.K <= 2048 ? 0 : -1));
        choose_tiles(pl, kX3Cfgs, kNumX3Cfgs, 2516.6e12 / 3.0, "DG_FORCE_X3CFG", rule);
        pl.x6 = 3;
    }
    pl.vec = pl.x6 ? 1 : cfg_vec(g, mode, kCfgs[pl.cfg].bk);
    pl.slab_bytes = pl.splits > 1 ? (size_t)pl.nphase * pl.splits * pl.M * pl.N * sizeof(float) : 0;
    pl.ws_bytes = pl.slab_bytes;
    if (pl.x6) {
        // workspace: [split-K slabs][A planes][B planes] (6 B per element bf16x6, 2 B fp16, 4 B fp16x3)
        // (+ fp16x3: 8 floats for max |dy| when no scale source is set)
        const size_t eb = pl.x6 == 2 ? 2 : (pl.x6 == 3 ? 4 : 6);
        pl.x6_a_off = (pl.ws_bytes + 255) & ~(size_t)255;
        pl.x6_b_off = (pl.x6_a_off + eb * ra * ca + 255) & ~(size_t)255;
        pl.ws_bytes = pl.x6_b_off + eb * rb * cb;
        if (pl.x6 == 3) {   // (max |dy| and max |x| when no scale source is set: any mode may read dy / x)
            pl.x3_max_off = (pl.ws_bytes + 255) & ~(size_t)255;
            pl.ws_bytes = pl.x3_max_off + 2 * X3_SLOT * sizeof(float);
        }
    }
    pl.gemm_bytes = pl.ws_bytes;
    if (getenv("DG_PLAN_DEBUG"))
        fprintf(stderr, "[dg plan] mode %d M=%d N=%d K=%d -> %s cfg %d splits %d ph %d ptiles %d\n", mode, pl.M, pl.N, pl.K,
                pl.halo == 2 ? (pl.x6 == 3 ? "x3h2" : "x6h2") : pl.halo == 4 ? "x6h4" : pl.halo ? (pl.x6 == 2 ? "f16h" : (pl.x6 == 3 ? "x3h" : "x6h")) : (pl.x6 == 2 ? "f16" : (pl.x6 == 3 ? "x3" : (pl.x6 ? "x6" : "fp32"))),
                pl.cfg, pl.splits, pl.halo ? std::max(8, pl.hph) : 0, pl.ptiles);
    return pl;
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
// bytes of the fp16x3 weight planes of a forward plan (x6 3), 256-aligned
static size_t x3_w_bytes(const OpPlan &pl) { return al256((size_t)4 * pl.x6_rb * pl.x6_cb); }

static ConvGeom geom_1x1(long pixels, int ci, int co) {
    ConvGeom q{};
    q.N = 1; q.H = 1; q.W = (int)pixels; q.Ci = ci; q.Ho = 1; q.Wo = (int)pixels; q.Co = co;
    q.kh = q.kw = q.sh = q.sw = 1; q.pt = q.pl = 0; q.Th = q.Tw = 1;
    return q;
}

// (a recast GEMM's operands are gathered / transposed fp32 scratch, not a layer's tensors:
// DG_MATH_F16X3 descriptors run them bf16x6)
static int recast_math(const dg_conv_desc_s *d) { return d->math == DG_MATH_F16X3 ? DG_MATH_BF16X6 : d->math; }

// decide whether a narrow op runs as a recast 1x1 MFMA GEMM (+ gather), and size its workspace
static void plan_recast(dg_conv_desc_s *d, int op) {
    Recast &rc = d->rc[op];
    rc = Recast{};
    if (!d->plan[op].narrow) return;
    const ConvGeom &g = d->g;
    const int mode = engine_mode(d, op);
    const int ntap = g.kh * g.kw;
    if (mode == MODE_FWD) {
        if (g.Co != 1 || g.Ci % 32 || ntap % 4 || ntap < 8) return;
        long P = (long)g.N * g.H * g.W;
        rc.nv = ntap; rc.nvp = ntap; rc.mode1 = MODE_FWD;
        rc.g1 = geom_1x1(P, g.Ci, ntap);
        rc.p1 = make_plan(rc.g1, MODE_FWD, recast_math(d));
        rc.wt_off = 0;
        rc.v_off = al256((size_t)g.Ci * ntap * 4);
        rc.slab_off = al256(rc.v_off + (size_t)P * ntap * 4);
    } else if (mode == MODE_DGRAD) {
        const int nv = ntap * g.Ci;
        if (tlast_ok(g) && !plan_off("tlast")) {
            d->plan[op].tlast = 1;
            if (getenv("DG_PLAN_DEBUG")) fprintf(stderr, "[dg plan] mode %d -> tlast\n", mode);
            return;
        }
        if (direct_dgrad_ok(g) && !plan_off("direct")) {
            d->plan[op].direct = 1;
            return;
        }
        if (g.Co % 32 || nv < 8) return;
        const int nvp = (nv + 15) & ~15;  // zero-padded columns (e.g. VGG block1_conv1: 3x3x3 = 27 -> 32)
        long P = (long)g.N * g.Ho * g.Wo;
        rc.nv = nv; rc.nvp = nvp; rc.mode1 = MODE_FWD;
        rc.g1 = geom_1x1(P, g.Co, nvp);
        rc.p1 = make_plan(rc.g1, MODE_FWD, recast_math(d));
        rc.wt_off = 0;
        rc.v_off = al256((size_t)g.Co * nvp * 4);
        rc.slab_off = al256(rc.v_off + (size_t)P * nvp * 4);
    } else {
        if (g.Co != 1 || g.Ci % 4 || g.Ci < 8 || ntap % 4) return;
        long P = (long)g.N * g.H * g.W;
        rc.nv = ntap; rc.nvp = ntap; rc.mode1 = MODE_WGRAD;
        rc.g1 = geom_1x1(P, ntap, g.Ci);
        rc.p1 = make_plan(rc.g1, MODE_WGRAD, recast_math(d));
        rc.wt_off = 0;
        rc.v_off = 0;
        rc.slab_off = al256((size_t)P * ntap * 4);
    }
    if (rc.p1.narrow) return;
    rc.bytes = rc.slab_off + rc.p1.gemm_bytes;
    rc.on = 1;
}

static size_t colsum_ws(long M, int C);

// (re)plan the three ops of a descriptor for its math mode
static void plan_all(dg_conv_desc_s *d) {
    for (int op = 0; op < 3; ++op) {
        // (DG_MATH_F16X3: fp16x3 wherever make_plan finds the op eligible, bf16x6 elsewhere)
        // A filter gradient reads the layer's input and output gradient, whose fp16x3 planes exist
        // only where the forward / input gradient of the layer runs fp16x3 (the producers write
        // them for those ops); otherwise its split path also zeroes a max slot and measures the
        // operand (memset + absmax launches and a read) before splitting it -- G down7 / up2
        // filter gradients: 37 us of passes around a 27-42 us GEMM (round 6, profiles/r6/calls.txt)
        double extra = 0.0;
        if (op == DG_OP_BWD_FILTER && d->math == DG_MATH_F16X3) {
            const double xin = (double)d->N * d->H * d->W * d->Cin, gout = (double)d->N * d->Ho * d->Wo * d->Cout;
            if (d->plan[DG_OP_FWD].x6 != 3) extra += 8e-6 + xin * 4.0 / 4.0e12;
            if (d->plan[DG_OP_BWD_DATA].x6 != 3) extra += 8e-6 + gout * 4.0 / 4.0e12;
        }
        d->plan[op] = make_plan(d->g, engine_mode(d, op), d->math, plan_off("wgrad_extra") ? 0.0 : extra);
        plan_recast(d, op);
        if (d->rc[op].on) d->plan[op].ws_bytes = d->rc[op].bytes;
        if (op == DG_OP_BWD_FILTER) {
            // room for the bias column sum partials after the split-K slabs
            size_t extra = colsum_ws(1, d->Cout);
            size_t base = d->rc[op].on ? d->rc[op].bytes : d->plan[op].gemm_bytes;
            d->plan[op].colsum_off = (base + 255) & ~(size_t)255;
            d->plan[op].ws_bytes = d->plan[op].colsum_off + extra;
        }
    }
}

static int default_math() {
    const char *m = getenv("DG_CONV_MATH");
    if (m && (!strcmp(m, "fp32") || !strcmp(m, "0"))) return DG_MATH_FP32;
    if (m && (!strcmp(m, "fp16") || !strcmp(m, "2"))) return DG_MATH_FP16;
    if (m && (!strcmp(m, "f16x3") || !strcmp(m, "3"))) return DG_MATH_F16X3;
    (void)m;
    return DG_MATH_BF16X6;
}


template <int MODE>
static void launch_gemm(int cfg, int vec, dim3 grid, const GemmArgs &a, hipStream_t s) {
#define DG_L(C, BM_, BN_, WM_, WN_, BK_, MW_)                                                           \
    case C:                                                                                             \
        if (vec) hipLaunchKernelGGL((k_conv_gemm<MODE, BM_, BN_, WM_, WN_, true, BK_, MW_>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((k_conv_gemm<MODE, BM_, BN_, WM_, WN_, false, BK_, MW_>), grid, dim3(256), 0, s, a); \
        break;
    switch (cfg) {
        DG_L(0, 128, 128, 2, 2, 32, 2)
        DG_L(1, 128, 64, 2, 2, 32, 2)
        DG_L(2, 64, 128, 2, 2, 32, 2)
        DG_L(3, 64, 64, 2, 2, 32, 2)
        DG_L(4, 32, 128, 1, 4, 32, 2)
        DG_L(5, 128, 128, 2, 2, 16, 3)
        DG_L(6, 128, 64, 2, 2, 16, 3)
        DG_L(7, 128, 32, 4, 1, 32, 2)
        DG_L(8, 256, 32, 4, 1, 32, 2)
    }
#undef DG_L
}

static GemmArgs make_args(const ConvGeom &g, const OpPlan &pl, const float *A, int lda, const float *B, int ldb,
                          float *C, int ldc, const float *bias, float beta, int act, float alpha, void *slab) {
    GemmArgs a{};
    a.g = g; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
    a.bias = bias; a.beta = beta; a.act = act; a.alpha = alpha;
    a.M = pl.M; a.N = pl.N; a.K = pl.K; a.kchunk = pl.kchunk; a.splits = pl.splits;
    a.mtiles = pl.mtiles; a.ntiles = pl.ntiles; a.nphase = pl.nphase;
    a.slab = (float *)slab;
    a.xcd_plain = plan_off("xcd_phase");
    a.ptiles = pl.halo ? std::max(1, pl.ptiles) : 1;
    // n-grouped XCD raster (xcd_group_tile) for the stride-1 4x4 halo plans (the PatchGAN's conv:
    // 8 n-tiles of 64 columns over 256 patches at bs16 x 2): with every XCD running all 8 n-tiles
    // its L2 streams the whole 8.4 MB fp16x3 filter per round of patches -- the forward read 562 MB
    // for 105 MB of operands (profiles/r5/r5_final_pmc_layers.md); in groups of NG the XCD keeps
    // ntiles / NG column blocks.  DG_XCD_NG: the group count (0: off), for same-box A/B
    if (pl.halo == 4 && pl.ptiles <= 1 && pl.splits == 1 && pl.nphase == 1) {
        int ng = 4;
        if (const char *e = getenv("DG_XCD_NG")) ng = atoi(e);
        const long tot = (long)pl.mtiles * pl.ntiles;
        if ((ng == 1 || ng == 2 || ng == 4 || ng == 8) && tot % 8 == 0 && pl.ntiles % ng == 0 &&
            pl.mtiles % (8 / ng) == 0)
            a.xcd_ng = ng;
    }
    return a;
}

// caller-held bf16x6 planes of the two engine operands (dg_conv_planes_t mapped
// onto A / B of one op): NULL = split into the workspace; ready = already split
struct PlaneRefs {
    void *a, *b;
    int a_ready, b_ready;
    int b_x6;   // (fp16x3 op, B = w) the weight buffer also holds bf16x6 planes behind the fp16x3 part
};

static int run_gemm(int mode, const OpPlan &pl, const GemmArgs &a, hipStream_t s, const PlaneRefs *pr = nullptr);
static bool tensor_x3(const dg_conv_desc_s *d, int t);
static int finish_splitk(int mode, const OpPlan &pl, const GemmArgs &a, hipStream_t s);

// narrow op through its recast (1x1 MFMA GEMM + gather)
static int run_recast(const dg_conv_desc_s *d, int op, const GemmArgs &a0, char *ws, hipStream_t s) {
    const Recast &rc = d->rc[op];
    const ConvGeom &g = d->g;
    float *wt = (float *)(ws + rc.wt_off);
    float *V = (float *)(ws + rc.v_off);
    void *slab = ws + rc.slab_off;
    if (rc.mode1 == MODE_FWD && engine_mode(d, op) == MODE_FWD) {
        // Co == 1: V = x . wt, wt[ci][(i,j)] = w[(i,j)][ci]
        hipLaunchKernelGGL(k_transpose, dim3(std::min<unsigned>(dg_cdiv((long)rc.nv * g.Ci, 256), 1024)), dim3(256), 0, s,
                           a0.B, rc.nv, g.Ci, wt, rc.nv);
        DG_LAUNCHED("recast_transpose");
        GemmArgs a = make_args(rc.g1, rc.p1, a0.A, a0.lda, wt, rc.nv, V, rc.nv, nullptr, 0.f, DG_ACT_NONE, 0.f, slab);
        int r = run_gemm(MODE_FWD, rc.p1, a, s);
        if (r != DG_OK) return r;
        hipLaunchKernelGGL(k_recast_fwd_gather, dim3(dg_cdiv((long)g.N * g.Ho * g.Wo, 256)), dim3(256), 0, s, a0, V, rc.nv);
        DG_LAUNCHED("recast_fwd_gather");
        return DG_OK;
    }
    if (rc.mode1 == MODE_FWD) {
        // DGRAD, Ci <= 8: V = dy . wt, wt[co][(i,j,ci)] = w[(i,j,ci)][co]; dx = col2im(V)
        hipLaunchKernelGGL(k_transpose, dim3(std::min<unsigned>(dg_cdiv((long)rc.nvp * g.Co, 256), 1024)), dim3(256), 0, s,
                           a0.B, rc.nv, g.Co, wt, rc.nvp);
        DG_LAUNCHED("recast_transpose");
        GemmArgs a = make_args(rc.g1, rc.p1, a0.A, a0.lda, wt, rc.nvp, V, rc.nvp, nullptr, 0.f, DG_ACT_NONE, 0.f, slab);
        int r = run_gemm(MODE_FWD, rc.p1, a, s);
        if (r != DG_OK) return r;
        long total = (long)g.N * g.H * g.W * g.Ci;
        hipLaunchKernelGGL(k_recast_col2im, dim3((unsigned)std::min<long>(dg_cdiv(total, 256), 8192)), dim3(256), 0, s,
                           a0, V, rc.nvp);
        DG_LAUNCHED("recast_col2im");
        return DG_OK;
    }
    // WGRAD, Co == 1: G gathered from dy, dw[(i,j)][ci] = G^T . x (a WGRAD GEMM of 1x1 geometry)
    long total = (long)g.N * g.H * g.W * rc.nv;
    hipLaunchKernelGGL(k_recast_wgrad_gather, dim3((unsigned)std::min<long>(dg_cdiv(total, 256), 8192)), dim3(256), 0, s,
                       a0, a0.B, a0.ldb, V);
    DG_LAUNCHED("recast_wgrad_gather");
    GemmArgs a = make_args(rc.g1, rc.p1, V, rc.nv, a0.A, a0.lda, a0.C, g.Ci, nullptr, a0.beta, DG_ACT_NONE, 0.f, slab);
    return run_gemm(MODE_WGRAD, rc.p1, a, s);
}

// outputs of the max pool fused into a forward epilogue (dg_conv_fwd_pool)
struct PoolOut {
    unsigned char *idx;
    float *y;
    int ldy;
    unsigned short *planes;
    int planes_fmt;   // DG_PLANES_*: the consuming conv's x plane format
};

// the forward plan of d can run MaxPool2D(2) in its epilogue: the halo-tiled
// bf16x6 kernel with one split over whole 8 x 16 patches, and an activation
// whose derivative is a function of the output's sign
static bool pool_fusable(const dg_conv_desc_s *d, int act) {
    const OpPlan &pl = d->plan[DG_OP_FWD];
    return !d->transpose && (pl.x6 == 1 || pl.x6 == 3) && pl.halo == 1 && pl.cfg != 32 && pl.splits == 1 &&
           !d->rc[DG_OP_FWD].on &&
           d->g.Ho % (pl.hph == 16 ? 16 : 8) == 0 &&
           d->g.Wo % 16 == 0 && d->g.Co % 16 == 0 &&
           (act == DG_ACT_NONE || act == DG_ACT_RELU || act == DG_ACT_LRELU);
}

static int run_engine(const dg_conv_desc_s *d, int op, const float *A, int lda, const float *B, int ldb,
                      float *C, int ldc, const float *bias, float beta, int act, float alpha,
                      void *ws, size_t ws_bytes, hipStream_t s, const float *mz = nullptr, int ldmz = 0,
                      int mact = DG_ACT_NONE, float malpha = 0.f, const PlaneRefs *pr = nullptr,
                      unsigned short *yp = nullptr, const PoolOut *po = nullptr,
                      const unsigned short *mzp = nullptr, int yp_fmt = DG_PLANES_BF16X6) {
    const int mode = engine_mode(d, op);
    const OpPlan &pl = d->plan[op];
    const size_t need = d->rc[op].on ? d->rc[op].bytes : pl.gemm_bytes;
    DG_ARG(ws_bytes >= need, "workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    DG_ARG(need == 0 || ws != nullptr, "workspace pointer is NULL");
    GemmArgs a = make_args(d->g, pl, A, lda, B, ldb, C, ldc, bias, beta, act, alpha, ws);
    // (mact | DG_MASK_SUM: the mask also multiplies beta*C -- the conv_epilogue16 / split-K reduce
    // epilogues of the x6 / fp16x3 / fp16 plans implement it)
    a.mask_acc = (mact & DG_MASK_SUM) ? 1 : 0;
    mact &= ~DG_MASK_SUM;
    DG_ARG(!a.mask_acc || (pl.x6 && !d->rc[op].on && (mz || mzp)),
           "mask of the accumulated sum: only on the split-precision plans, with a mask");
    a.mz = mz; a.ldmz = ldmz; a.mact = mact; a.malpha = malpha;
    if (pl.x6 == 3) {
        // fp16x3 operand roles (op_tensors): A is x or dy, B is w, or, in a filter gradient,
        // dy or x; dy is scaled from its bound (dg_conv_set_grad_scale's dy source, else
        // measured by run_gemm), x from its source (dg_conv_set_act_scale; else measured by
        // run_gemm when it splits x into the workspace), w by F16X3_WS
        a.x3_sa = F16X3_XS;
        a.x3_sb = op == DG_OP_BWD_FILTER ? F16X3_XS : F16X3_WS;
        a.x3_dyn = op == DG_OP_FWD ? 0 : ((op == DG_OP_BWD_DATA || d->transpose) ? 1 : 2);
        const int xo = op == DG_OP_BWD_DATA ? 0 : ((op == DG_OP_FWD || !d->transpose) ? 1 : 2);   // x: A 1, B 2
        if (a.x3_dyn == 1) { a.as_m = d->gs_dy_m; a.as_g = d->gs_dy_g; }
        if (a.x3_dyn == 2) { a.bs_m = d->gs_dy_m; a.bs_g = d->gs_dy_g; }
        if (xo == 1) { a.as_m = d->as_x_m; a.as_g = d->as_x_g; a.as_c = d->as_x_c; }
        if (xo == 2) { a.bs_m = d->as_x_m; a.bs_g = d->as_x_g; a.bs_c = d->as_x_c; }
    }
    if (op == DG_OP_FWD) {
        // the activation scale context: the output planes' source and max |y| (any arithmetic:
        // a forward writes the planes of its consumer)
        a.ys_m = d->as_y_m; a.ys_g = d->as_y_g; a.ys_c = d->as_y_c; a.ymax = d->as_y_max;
        DG_ARG(!a.ymax || !(pl.narrow || pl.co1 || d->rc[op].on),
               "max |y| is measured by the GEMM epilogues, the split-K reduce and the small-Cin kernels only (this "
               "forward runs a narrow / Co-1 / recast kernel)");
    }
    if (op == DG_OP_BWD_DATA) {
        // the gradient scale context (dg_conv_set_grad_scale): dx planes' scale source, max |dx|
        a.ys_m = d->gs_dx_m; a.ys_g = d->gs_dx_g; a.ymax = d->gs_dx_max;
        DG_ARG(!a.ymax || pl.x6 || pl.splits > 1,
               "max |dx| is measured by the 16x16-tile epilogues and the split-K reduce only (plan of this input "
               "gradient: neither)");
        DG_ARG(yp_fmt != DG_PLANES_F16X3 || a.ys_m,
               "fp16x3 gradient planes need a scale source (dg_conv_set_grad_scale)");
    }
    if (po) {
        DG_ARG(op == DG_OP_FWD && pool_fusable(d, act), "this forward plan cannot fuse the max pool");
        DG_ARG(po->idx && (((uintptr_t)po->idx) & 3) == 0, "pool index buffer NULL or not 4-byte aligned");
        DG_ARG(po->y || po->planes, "fused pool writes neither values nor planes");
        DG_ARG(!po->y || (po->ldy % 4 == 0 && po->ldy >= d->g.Co && (((uintptr_t)po->y) & 15) == 0),
               "pooled output needs ldy %% 4 == 0 and 16-byte alignment");
        DG_ARG(!po->planes || (((uintptr_t)po->planes) & 15) == 0, "plane buffers must be 16-byte aligned");
        DG_ARG(beta == 0.f, "the fused pool overwrites its output (beta must be 0)");
        a.pidx = po->idx; a.pool_y = po->y; a.ldpy = po->ldy;
        a.yp = po->planes; a.ypC = d->g.Co;
        if (po->planes && po->planes_fmt == DG_PLANES_F16X3) {
            DG_ARG(d->g.Co % 32 == 0, "fp16x3 output planes need channels %% 32 == 0");
            a.ypC = -d->g.Co;
        }
    }
    if (mzp) {
        // mask from the hi plane's sign: the small-Cin kernels read fp32 masks only
        DG_ARG(!mz && !pl.small, "plane mask: not with an fp32 mask, nor on the small-Cin kernels");
        DG_ARG(mact == DG_ACT_NONE || mact == DG_ACT_RELU || mact == DG_ACT_LRELU,
               "plane mask needs a sign-determined activation (got %d)", mact);
        a.mzp = mzp; a.mzpC = mode == MODE_FWD ? d->g.Co : d->g.Ci;
        // (the layer input's planes: fp16x3 when this descriptor's ops read them so)
        if (tensor_x3(d, DG_TENSOR_X)) a.mzpC = -a.mzpC;
    }
    if (!C && !po) {
        // planes-only output: the GEMM epilogues skip the fp32 store
        DG_ARG(yp && beta == 0.f && mode != MODE_WGRAD && !pl.narrow && (!pl.small || mode == MODE_FWD) &&
                   !d->rc[op].on,
               "output NULL: only a GEMM-path op writing its output planes (beta 0) may omit it");
    }
    if (pl.M == 0 || pl.N == 0) return DG_OK;
    if (yp) {
        // planes of the output beside it: the GEMM epilogues (fp32, bf16x6,
        // split-K reduce) write them; the narrow / recast paths (output
        // channels < 16, never plane-eligible) are refused
        const int oc = mode == MODE_WGRAD ? 0 : (mode == MODE_FWD ? d->g.Co : d->g.Ci);
        DG_ARG(oc % 16 == 0 && !pl.narrow && !d->rc[op].on, "output planes need a GEMM path and channels %% 16 == 0");
        DG_ARG((((uintptr_t)yp) & 15) == 0, "plane buffers must be 16-byte aligned");
        a.yp = yp; a.ypC = oc;
        if (yp_fmt == DG_PLANES_F16X3) {
            DG_ARG(oc % 32 == 0, "fp16x3 output planes need channels %% 32 == 0");
            a.ypC = -oc;
        }
    }
    if (d->rc[op].on) {
        DG_ARG(lda % 4 == 0 && ((uintptr_t)A & 15) == 0, "recast path needs lda%%4==0 and 16B-aligned A");
        return run_recast(d, op, a, (char *)ws, s);
    }
    if (pl.co1) {
        const ConvGeom &g = d->g;
        if (mode == MODE_WGRAD) {
            DG_ARG(lda % 4 == 0 && ((uintptr_t)A & 15) == 0, "Co == 1 filter gradient needs ldx %% 4 == 0 and 16B-aligned x");
        } else {
            DG_ARG(ldb <= 1 && ((uintptr_t)B & 15) == 0, "Co == 1 kernels need a dense 16B-aligned filter");
            if (mode == MODE_FWD)
                DG_ARG(lda % 4 == 0 && ((uintptr_t)A & 15) == 0, "Co == 1 forward needs ldx %% 4 == 0 and 16B-aligned x");
            else
                DG_ARG((long)g.N * g.H * g.W * g.Ci < (1L << 31), "operand larger than 2^31 elements");
        }
        launch_co1(mode, a, s);
        DG_LAUNCHED("co1");
        return DG_OK;
    }
    if (pl.ntile) {   // (mode == MODE_WGRAD)
        float *part = a.slab;
        DG_ARG(part != nullptr, "workspace pointer is NULL");
        hipLaunchKernelGGL(k_narrow_wgrad_tile, dim3(pl.splits), dim3(256), narrow_tile_lds(d->g), s, a,
                           narrow_tile_segments(d->g), part);
        DG_LAUNCHED("narrow_wgrad_tile");
        hipLaunchKernelGGL(k_narrow_wgrad_final, dim3(dg_cdiv(pl.M * 4 * narrow_tile_groups(d->g), 16)), dim3(256), 0,
                           s, a, pl.splits, (const float *)part);
        DG_LAUNCHED("narrow_wgrad_final");
        return DG_OK;
    }
    if (pl.narrow) {
        const ConvGeom &gg = d->g;
        const bool px = mode == MODE_FWD && gg.Ci % 4 == 0 && a.lda % 4 == 0 && (((uintptr_t)a.A) & 15) == 0 &&
                        (gg.Co == 1 || gg.Co == 3) && (long)gg.kh * gg.kw * gg.Ci * gg.Co <= NFWD_WMAX &&
                        pl.M >= NFWD_PX_MIN_M && !plan_off("narrow_px");
        if (px) {
            const unsigned grid = (unsigned)std::min<long>(dg_cdiv(pl.M, 256), 8192);
            if (gg.Co == 1) hipLaunchKernelGGL(k_narrow_fwd_px<1>, dim3(grid), dim3(256), 0, s, a);
            else hipLaunchKernelGGL(k_narrow_fwd_px<3>, dim3(grid), dim3(256), 0, s, a);
            DG_LAUNCHED("narrow_fwd_px");
        } else if (mode == MODE_FWD) {
            hipLaunchKernelGGL(k_narrow_fwd, dim3(dg_cdiv(pl.M, 4)), dim3(256), 0, s, a);
            DG_LAUNCHED("narrow_fwd");
        } else if (mode == MODE_DGRAD && pl.tlast && !a.mz && !a.mzp && a.lda % 4 == 0 &&
                   ((((uintptr_t)a.A) | ((uintptr_t)a.B)) & 15) == 0) {
            launch_tlast_fwd(a, s);
            DG_LAUNCHED("tlast_fwd");
        } else if (mode == MODE_DGRAD && pl.direct && a.lda % 4 == 0 && ((uintptr_t)a.A & 15) == 0) {
            launch_direct_dgrad(a, s);
            DG_LAUNCHED("direct_dgrad");
        } else if (mode == MODE_DGRAD) {
            size_t wbytes = (size_t)d->g.kh * d->g.kw * d->g.Ci * d->g.Co * sizeof(float);
            int in_lds = wbytes <= 64 * 1024;
            hipLaunchKernelGGL(k_narrow_dgrad, dim3(dg_cdiv(pl.M, 256), pl.nphase), dim3(256), in_lds ? wbytes : 0, s, a, in_lds);
            DG_LAUNCHED("narrow_dgrad");
        } else {
            a.splits = pl.splits; a.kchunk = pl.kchunk;
            hipLaunchKernelGGL(k_narrow_wgrad, dim3(d->g.kh * d->g.kw * ((d->g.Ci + 255) / 256), pl.splits), dim3(256), 0, s, a);
            DG_LAUNCHED("narrow_wgrad");
            long total = (long)pl.M * pl.N;
            hipLaunchKernelGGL(k_splitk_reduce<MODE_WGRAD>, dim3((unsigned)std::min<long>(dg_cdiv(total, 256), 2048), 1), dim3(256), 0, s, a, 0);
            DG_LAUNCHED("narrow_wgrad_reduce");
        }
        return DG_OK;
    }
    if (pl.small) {
        const ConvGeom &g = d->g;
        const long xin = (long)g.N * g.H * g.W, xout = (long)g.N * g.Ho * g.Wo;
        DG_ARG((xin - 1) * lda + g.Ci < (1L << 31) && xout * ldb < (1L << 31) && xout * ldc < (1L << 31),
               "operand larger than 2^31 elements");
        launch_small_conv(mode, a, pl.small_rows, s);
        DG_LAUNCHED(mode == MODE_WGRAD ? "small_wgrad" : "small_fwd");
        return finish_splitk(mode, pl, a, s);
    }
    return run_gemm(mode, pl, a, s, pr);
}

static int run_gemm(int mode, const OpPlan &pl, const GemmArgs &a_in, hipStream_t s, const PlaneRefs *pr) {
    GemmArgs a = a_in;
    const float *A = a.A, *B = a.B;
    const int lda = a.lda, ldb = a.ldb;
    {   // operand extents for the buffer-resource range checks
        const ConvGeom &g = a.g;
        const long xin = (long)g.N * g.H * g.W, xout = (long)g.N * g.Ho * g.Wo;
        long ab, bb;
        if (mode == MODE_FWD) {
            ab = ((xin - 1) * lda + g.Ci) * 4;
            bb = ((long)(pl.K - 1) * ldb + pl.N) * 4;
        } else if (mode == MODE_DGRAD) {
            ab = ((xout - 1) * lda + g.Co) * 4;
            bb = (long)g.kh * g.kw * g.Ci * g.Co * 4;
        } else {
            ab = ((xin - 1) * lda + g.Ci) * 4;
            bb = ((xout - 1) * ldb + g.Co) * 4;
        }
        DG_ARG(ab < (1L << 31) && bb < (1L << 31), "operand larger than 2 GiB (buffer-resource offsets are 32-bit)");
        a.a_bytes = (unsigned)ab;
        a.b_bytes = (unsigned)bb;
    }
    if (pl.x6 == 3) {
        // fp16x3: activations / gradients -> fp16x3 planes in 32-channel groups, weights in
        // 16-column groups (common.h); a caller-held weight buffer also receives the
        // weights' bf16x6 planes behind them when a bf16x6 op of the layer reads them
        // (tensor_plane_bytes).  The gradient operand (a.x3_dyn) is scaled from its bound:
        // a.as_m / as_g, the caller's scale source, else max |dy| measured here
        char *ws = (char *)a.slab;
        DG_ARG(ws != nullptr, "workspace pointer is NULL");
        DG_ARG(a.x3_sa > 0.f && a.x3_sb > 0.f, "fp16x3 GEMM without its operand roles (run_engine)");
        void *pa = ws + pl.x6_a_off, *pb = ws + pl.x6_b_off;
        const bool b_w = mode != MODE_WGRAD;                    // B is the weight tensor
        const int ldbw = (mode == MODE_DGRAD) ? a.g.Co : ldb;   // DGRAD B is the dense weight tensor
        if (pr && pr->a) pa = pr->a;
        if (pr && pr->b) pb = pr->b;
        const bool a_ready = pr && pr->a && pr->a_ready;
        const bool b_ready = pr && pr->b && pr->b_ready;
        // an operand without a scale source is measured before its split: max |value| into the
        // workspace -- a gradient always (its planes must not be ready), an activation whose
        // planes live in the workspace (caller-held activation planes without a source keep the
        // static F16X3_XS, the producers' default); an activation source that is a plain max
        // slot (g, c unset) is measured into by the op that splits x
        for (int o = 1; o <= 2; ++o) {
            const bool is_a = o == 1;
            if (!is_a && b_w) continue;
            const float *&m = is_a ? a.as_m : a.bs_m;
            const bool ready = is_a ? a_ready : b_ready;
            const bool held = is_a ? (pr && pr->a) : (pr && pr->b);
            const bool grad = a.x3_dyn == o;
            float *meas = nullptr;
            if (!m) {
                DG_ARG(!grad || !ready, "fp16x3 dy planes given without their scale source (dg_conv_set_grad_scale)");
                if (!grad && held) continue;
                meas = (float *)(ws + pl.x3_max_off + (grad ? 0 : X3_SLOT * sizeof(float)));
            } else if (!ready && (is_a ? !a.as_g && !a.as_c : !a.bs_g && !a.bs_c) && !grad) {
                meas = const_cast<float *>(m);   // an x source that is a plain max slot: measured by this split
            }
            if (!meas) continue;
            if (hipMemsetAsync(meas, 0, X3_SLOT * sizeof(float), s) != hipSuccess) {
                dg::set_error("hipMemsetAsync failed");
                return DG_ERR_HIP;
            }
            if (is_a) launch_absmax(A, pl.x6_ra, pl.x6_ca, lda, meas, s);
            else launch_absmax(B, pl.x6_rb, pl.x6_cb, ldb, meas, s);
            DG_LAUNCHED("absmax_operand");
            if (is_a) { a.as_m = meas; a.as_g = nullptr; a.as_c = nullptr; }
            else { a.bs_m = meas; a.bs_g = nullptr; a.bs_c = nullptr; }
        }
        if (!a_ready) {
            launch_split_x3(A, lda, pl.x6_ra, pl.x6_ca, pa, 32, a.x3_sa, s, a.as_m, a.as_g, a.as_c);
            DG_LAUNCHED("split_x3_a");
        }
        if (!b_ready) {
            if (!b_w) {
                launch_split_x3(B, ldb, pl.x6_rb, pl.x6_cb, pb, 32, a.x3_sb, s, a.bs_m, a.bs_g, a.bs_c);
                DG_LAUNCHED("split_x3_b");
            } else {
                launch_split_x3(B, ldbw, pl.x6_rb, pl.x6_cb, pb, 16, F16X3_WS, s);
                DG_LAUNCHED("split_x3_w");
                if (pr && pr->b && pr->b_x6) {
                    launch_split3(B, ldbw, pl.x6_rb, pl.x6_cb, (unsigned short *)((char *)pb + x3_w_bytes(pl)), s);
                    DG_LAUNCHED("split3_w");
                }
            }
        }
        a.A = (const float *)pa; a.lda = pl.x6_ca; a.a_bytes = (unsigned)(4 * pl.x6_ra * pl.x6_ca);
        a.B = (const float *)pb; a.ldb = pl.x6_cb; a.b_bytes = (unsigned)(4 * pl.x6_rb * pl.x6_cb);
        dim3 grid(pl.mtiles * pl.ntiles, pl.nphase * pl.splits);
        if (pl.halo) {
            // (persistent blocks: patch row mt0 + j * gm, j < ptiles, of each of the gm * ntiles blocks)
            grid.x = (unsigned)((pl.mtiles + a.ptiles - 1) / a.ptiles * pl.ntiles);
            launch_gemm_x6h(mode, pl.cfg, pl.halo == 2 ? 2 : (pl.halo == 4 ? 4 : 3), grid, a, pl.htx, pl.hty, s, 4,
                            pl.hph == 16 ? 16 : 8);
            DG_LAUNCHED("conv_gemm_x3h");
        } else {
            fastdiv_magic((unsigned)a.g.Wo, a.mg_wo, a.sh_wo);
            fastdiv_magic((unsigned)a.g.Ho, a.mg_ho, a.sh_ho);
            launch_gemm_x3(mode, pl.cfg, grid, a, s);
            DG_LAUNCHED("conv_gemm_x3");
        }
        return finish_splitk(mode, pl, a, s);
    }
    if (pl.x6 == 2) {
        // fp16: round the operands into one fp16 plane each -- the caller-held
        // copies (dg_conv_planes_t: a layer's x, dy and w are converted once
        // and shared by the ops that read them) or the workspace
        char *ws = (char *)a.slab;
        DG_ARG(ws != nullptr, "workspace pointer is NULL");
        void *pa = ws + pl.x6_a_off, *pb = ws + pl.x6_b_off;
        const int ldbw = (mode == MODE_DGRAD) ? a.g.Co : ldb;
        if (pr && pr->a) pa = pr->a;
        if (pr && pr->b) pb = pr->b;
        const bool need_a = !(pr && pr->a && pr->a_ready), need_b = !(pr && pr->b && pr->b_ready);
        if (need_a && need_b) {
            launch_split_f16_pair(A, lda, pl.x6_ra, pl.x6_ca, pa, B, ldbw, pl.x6_rb, pl.x6_cb, pb, s);
            DG_LAUNCHED("split_f16");
        } else if (need_a) {
            launch_split_f16(A, lda, pl.x6_ra, pl.x6_ca, pa, s);
            DG_LAUNCHED("split_f16_a");
        } else if (need_b) {
            launch_split_f16(B, ldbw, pl.x6_rb, pl.x6_cb, pb, s);
            DG_LAUNCHED("split_f16_b");
        }
        a.A = (const float *)pa; a.lda = pl.x6_ca; a.a_bytes = (unsigned)(2 * pl.x6_ra * pl.x6_ca);
        a.B = (const float *)pb; a.ldb = pl.x6_cb; a.b_bytes = (unsigned)(2 * pl.x6_rb * pl.x6_cb);
        fastdiv_magic((unsigned)a.g.Wo, a.mg_wo, a.sh_wo);
        fastdiv_magic((unsigned)a.g.Ho, a.mg_ho, a.sh_ho);
        DG_ARG(a.yp == nullptr, "fp16 conv math writes no bf16x6 output planes");
        dim3 grid(pl.mtiles * pl.ntiles, pl.nphase * pl.splits);
        if (pl.halo) launch_gemm_x6h(mode, pl.cfg, 3, grid, a, pl.htx, pl.hty, s, 2);
        else launch_gemm_f16(mode, pl.cfg, grid, a, s);
        DG_LAUNCHED("conv_gemm_f16");
        return finish_splitk(mode, pl, a, s);
    }
    if (pl.x6) {
        // split both operands into bf16 hi/mid/lo planes in the workspace, then
        // point the GEMM at plane 0 of each (dense rows of x6_ca / x6_cb)
        char *ws = (char *)a.slab;
        DG_ARG(ws != nullptr, "workspace pointer is NULL");
        unsigned short *pa = (unsigned short *)(ws + pl.x6_a_off);
        unsigned short *pb = (unsigned short *)(ws + pl.x6_b_off);
        const long pas = pl.x6_ra * pl.x6_ca, pbs = pl.x6_rb * pl.x6_cb;
        const int ldbw = (mode == MODE_DGRAD) ? a.g.Co : ldb;  // DGRAD B is the dense weight tensor
        if (pr && pr->a) pa = (unsigned short *)pr->a;
        if (pr && pr->b) pb = (unsigned short *)pr->b;
        if (!(pr && pr->a && pr->a_ready)) {
            launch_split3(A, lda, pl.x6_ra, pl.x6_ca, pa, s);
            DG_LAUNCHED("split3_a");
        }
        if (!(pr && pr->b && pr->b_ready)) {
            launch_split3(B, ldbw, pl.x6_rb, pl.x6_cb, pb, s);
            DG_LAUNCHED("split3_b");
        }
        a.A = (const float *)pa; a.lda = pl.x6_ca; a.a_bytes = (unsigned)(3 * pas * 2);
        fastdiv_magic((unsigned)a.g.Wo, a.mg_wo, a.sh_wo);
        fastdiv_magic((unsigned)a.g.Ho, a.mg_ho, a.sh_ho);
        a.B = (const float *)pb; a.ldb = pl.x6_cb; a.b_bytes = (unsigned)(3 * pbs * 2);
        dim3 grid(pl.mtiles * pl.ntiles, pl.nphase * pl.splits);
        if (pl.halo) launch_gemm_x6h(mode, pl.cfg, pl.halo == 2 ? 2 : (pl.halo == 4 ? 4 : 3), grid, a, pl.htx, pl.hty, s);
        else launch_gemm_x6(mode, pl.cfg, grid, a, s);
        DG_LAUNCHED("conv_gemm_x6");
        return finish_splitk(mode, pl, a, s);
    }
    if (mode == MODE_FWD || mode == MODE_WGRAD) {
        DG_ARG(pl.N % 4 == 0 && ldb % 4 == 0, "GEMM N (%d) and ldb (%d) must be multiples of 4", pl.N, ldb);
    }
    if (pl.vec) {
        DG_ARG(lda % 4 == 0 && ((uintptr_t)A & 15) == 0, "vector path needs lda%%4==0 and 16B-aligned A");
    }
    DG_ARG(((uintptr_t)B & 15) == 0 || mode == MODE_DGRAD, "B must be 16B aligned");
    dim3 grid(pl.mtiles * pl.ntiles, pl.nphase * pl.splits);
    switch (mode) {
    case MODE_FWD: launch_gemm<MODE_FWD>(pl.cfg, pl.vec, grid, a, s); break;
    case MODE_DGRAD: launch_gemm<MODE_DGRAD>(pl.cfg, pl.vec, grid, a, s); break;
    default: launch_gemm<MODE_WGRAD>(pl.cfg, pl.vec, grid, a, s); break;
    }
    DG_LAUNCHED("conv_gemm");
    return finish_splitk(mode, pl, a, s);
}

// split-K reduction + epilogue of a GEMM whose kernel wrote partial slabs
static int finish_splitk(int mode, const OpPlan &pl, const GemmArgs &a, hipStream_t s) {
    if (pl.splits > 1) {
        // float4 outputs with tpo lanes per output (tpo = 0 -> scalar path)
        // (tpo lanes per float4 output until ~256K threads read the slabs, each lane summing >= 4)
        int tpo = 0;
        if ((pl.N % 4 == 0) && (a.ldc % 4 == 0) && ((((uintptr_t)a.C) | ((uintptr_t)a.slab)) & 15) == 0) {
            tpo = 1;
            const long E = (long)pl.M * pl.N / 4 * pl.nphase;
            while (tpo < 64 && tpo * 4 <= pl.splits && E * tpo < 262144) tpo <<= 1;
        }
        const int v4 = tpo;
        long total = tpo ? (long)pl.M * pl.N / 4 * tpo : (long)pl.M * pl.N;
        dim3 rg((unsigned)std::min<long>(dg_cdiv(total, 256), 4096), pl.nphase);
        static const bool trace = getenv("DG_TRACE_REDUCE") != nullptr;
        if (trace)
            fprintf(stderr, "[reduce] mode %d M %ld N %d splits %d nphase %d tpo %d grid %u C %d beta %g bias %d yp %d ymax %d mz %d mzp %d ys_m %d\n",
                    mode, (long)pl.M, pl.N, pl.splits, pl.nphase, tpo, rg.x, a.C != nullptr, a.beta, a.bias != nullptr,
                    a.yp != nullptr, a.ymax != nullptr, a.mz != nullptr, a.mzp != nullptr, a.ys_m != nullptr);
        switch (mode) {
        case MODE_FWD: hipLaunchKernelGGL(k_splitk_reduce<MODE_FWD>, rg, dim3(256), 0, s, a, v4); break;
        case MODE_DGRAD: hipLaunchKernelGGL(k_splitk_reduce<MODE_DGRAD>, rg, dim3(256), 0, s, a, v4); break;
        default: hipLaunchKernelGGL(k_splitk_reduce<MODE_WGRAD>, rg, dim3(256), 0, s, a, v4); break;
        }
        DG_LAUNCHED("splitk_reduce");
    }
    return DG_OK;
}

static size_t colsum_ws(long M, int C) {
    (void)M;
    return (size_t)C * 1024 * sizeof(float);
}

static int run_colsum(const float *dy, int ld, long M, int C, float *out, float beta, float *ws, hipStream_t s) {
    // row chunks of >= 256 rows (<= 64 loads per lane), at most 1024 (colsum_ws)
    int nblk = (int)std::min<long>(1024, std::max<long>(1, dg_cdiv(M, 256)));
    long rpb = (M + nblk - 1) / nblk;
    int cc = 1;
    while (cc < C && cc < 64) cc <<= 1;
    hipLaunchKernelGGL(k_colsum_partial, dim3(nblk, dg_cdiv(C, cc)), dim3(256), 0, s, dy, ld, M, C, rpb, ws);
    DG_LAUNCHED("colsum_partial");
    hipLaunchKernelGGL(k_colsum_final, dim3(C), dim3(256), 0, s, ws, nblk, C, out, beta);
    DG_LAUNCHED("colsum_final");
    return DG_OK;
}

// layer tensors (DG_TENSOR_*) read as engine operands A and B by op
static void op_tensors(const dg_conv_desc_s *d, int op, int &ta, int &tb) {
    if (op == DG_OP_FWD) { ta = DG_TENSOR_X; tb = DG_TENSOR_W; }
    else if (op == DG_OP_BWD_DATA) { ta = DG_TENSOR_DY; tb = DG_TENSOR_W; }
    else if (!d->transpose) { ta = DG_TENSOR_X; tb = DG_TENSOR_DY; }
    else { ta = DG_TENSOR_DY; tb = DG_TENSOR_X; }  // conv view of a transposed layer: A = its output grad
}

// an op that reads operand planes at all: bf16x6 (x6 1), the fp16 copy (x6 2,
// DG_MATH_FP16: [rows][C] fp16, the same for every op that reads the tensor) or fp16x3
// (x6 3); fp32 / narrow / recast plans read fp32
static bool op_reads_planes(const dg_conv_desc_s *d, int op) {
    const OpPlan &pl = d->plan[op];
    if ((pl.x6 != 1 && pl.x6 != 2 && pl.x6 != 3) || pl.narrow || d->rc[op].on || pl.M == 0 || pl.N == 0) return false;
    return !(pl.x6 == 2 && plan_off("f16planes"));
}
// tensor t's planes are fp16x3 when an fp16x3 op reads them; a bf16x6 op of the same
// layer then splits that tensor itself, except w, whose buffer holds [fp16x3 | bf16x6]
static bool tensor_reader(const dg_conv_desc_s *d, int t, int x6) {
    for (int op = 0; op < 3; ++op) {
        int ta, tb;
        op_tensors(d, op, ta, tb);
        if (((ta | tb) & t) && op_reads_planes(d, op) && d->plan[op].x6 == x6) return true;
    }
    return false;
}
static bool tensor_x3(const dg_conv_desc_s *d, int t) { return tensor_reader(d, t, 3); }
static size_t x3_wbytes(const dg_conv_desc_s *d) {
    return al256((size_t)4 * d->g.kh * d->g.kw * d->Cin * d->Cout);
}
static size_t tensor_plane_bytes(const dg_conv_desc_s *d, int t) {
    const size_t nw = (size_t)d->g.kh * d->g.kw * d->Cin * d->Cout;
    if (t == DG_TENSOR_X) return (size_t)(tensor_x3(d, t) ? 4 : 6) * d->N * d->H * d->W * d->Cin;
    if (t == DG_TENSOR_DY) return (size_t)(tensor_x3(d, t) ? 4 : 6) * d->N * d->Ho * d->Wo * d->Cout;
    if (!tensor_x3(d, t)) return 6 * nw;
    return x3_wbytes(d) + (tensor_reader(d, t, 1) ? 6 * nw : 0);
}

// tensors op reads as operand planes (op_reads_planes); x and dy only in the format
// tensor_x3 gives them
static int op_plane_mask(const dg_conv_desc_s *d, int op) {
    if (!op_reads_planes(d, op)) return 0;
    int ta, tb;
    op_tensors(d, op, ta, tb);
    const bool x3 = d->plan[op].x6 == 3;
    int m = ta | tb;
    for (int t : {DG_TENSOR_X, DG_TENSOR_DY})
        if ((m & t) && tensor_x3(d, t) != x3) m &= ~t;
    return m;
}

// dg_conv_planes_t -> the op's PlaneRefs (out = nullptr when the op takes no planes)
static int plane_refs(const dg_conv_desc_s *d, int op, const dg_conv_planes_t *p, PlaneRefs &r,
                      const PlaneRefs *&out) {
    out = nullptr;
    if (!p || !op_plane_mask(d, op)) return DG_OK;
    int ta, tb;
    op_tensors(d, op, ta, tb);
    auto buf = [&](int t) -> void * { return t == DG_TENSOR_X ? p->x : (t == DG_TENSOR_DY ? p->dy : p->w); };
    const int mask = op_plane_mask(d, op);
    r.a = (mask & ta) ? buf(ta) : nullptr; r.b = (mask & tb) ? buf(tb) : nullptr;
    r.a_ready = (p->ready & ta) != 0; r.b_ready = (p->ready & tb) != 0;
    // a bf16x6 op of a layer with fp16x3 weight planes: the weights' bf16x6 part of the buffer
    if (tb == DG_TENSOR_W && r.b) {
        if (d->plan[op].x6 == 1 && tensor_x3(d, DG_TENSOR_W)) r.b = (char *)r.b + x3_wbytes(d);
        r.b_x6 = d->plan[op].x6 == 3 && tensor_reader(d, DG_TENSOR_W, 1);
    }
    DG_ARG(((((uintptr_t)r.a) | ((uintptr_t)r.b)) & 15) == 0, "plane buffers must be 16-byte aligned");
    out = &r;
    return DG_OK;
}

}  // namespace dg

// -------------------------------------------------------------------------
// C ABI
// -------------------------------------------------------------------------
extern "C" {

int dg_conv_desc_create(dg_conv_t *out, int N, int H, int W, int Cin, int Cout, int kh, int kw, int sh, int sw,
                        int pad_t, int pad_b, int pad_l, int pad_r, int transpose) {
    DG_ARG(out != nullptr, "out is NULL");
    DG_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "bad shape N=%d H=%d W=%d Cin=%d Cout=%d", N, H, W, Cin, Cout);
    DG_ARG(kh > 0 && kw > 0 && sh > 0 && sw > 0, "bad kernel/stride");
    DG_ARG(pad_t >= 0 && pad_b >= 0 && pad_l >= 0 && pad_r >= 0, "negative padding");
    dg_conv_desc_s *d = new (std::nothrow) dg_conv_desc_s();
    if (!d) { dg::set_error("out of host memory"); return DG_ERR_ARG; }
    d->transpose = transpose ? 1 : 0;
    d->N = N; d->H = H; d->W = W; d->Cin = Cin; d->Cout = Cout;
    dg::ConvGeom &g = d->g;
    g.kh = kh; g.kw = kw; g.sh = sh; g.sw = sw; g.pt = pad_t; g.pl = pad_l;
    g.N = N;
    if (!transpose) {
        d->Ho = (H + pad_t + pad_b - kh) / sh + 1;
        d->Wo = (W + pad_l + pad_r - kw) / sw + 1;
        g.H = H; g.W = W; g.Ci = Cin; g.Ho = d->Ho; g.Wo = d->Wo; g.Co = Cout;
    } else {
        d->Ho = (H - 1) * sh + kh - pad_t - pad_b;
        d->Wo = (W - 1) * sw + kw - pad_l - pad_r;
        g.H = d->Ho; g.W = d->Wo; g.Ci = Cout; g.Ho = H; g.Wo = W; g.Co = Cin;
        if ((g.H + pad_t + pad_b - kh) / sh + 1 != H || (g.W + pad_l + pad_r - kw) / sw + 1 != W) {
            delete d;
            dg::set_error("transposed conv: inconsistent output size");
            return DG_ERR_ARG;
        }
    }
    if (d->Ho <= 0 || d->Wo <= 0) {
        delete d;
        dg::set_error("empty output (Ho=%d Wo=%d)", d->Ho, d->Wo);
        return DG_ERR_ARG;
    }
    g.Th = (kh + sh - 1) / sh;
    g.Tw = (kw + sw - 1) / sw;
    d->math = dg::default_math();
    dg::plan_all(d);
    *out = d;
    return DG_OK;
}

int dg_conv_set_math(dg_conv_t d, int math) {
    DG_ARG(d != nullptr, "descriptor is NULL");
    DG_ARG(math == DG_MATH_FP32 || math == DG_MATH_BF16X6 || math == DG_MATH_FP16 || math == DG_MATH_F16X3,
           "unknown conv math mode %d", math);
    d->math = math;
    dg::plan_all(d);
    return DG_OK;
}

int dg_conv_get_math(dg_conv_t d, int *math) {
    DG_ARG(d != nullptr && math != nullptr, "NULL argument");
    *math = d->math;
    return DG_OK;
}

int dg_conv_desc_destroy(dg_conv_t d) {
    delete d;
    return DG_OK;
}

int dg_conv_out_shape(dg_conv_t d, int *Ho, int *Wo) {
    DG_ARG(d && Ho && Wo, "NULL argument");
    *Ho = d->Ho; *Wo = d->Wo;
    return DG_OK;
}

int dg_conv_workspace_size(dg_conv_t d, int op, size_t *bytes) {
    DG_ARG(d && bytes, "NULL argument");
    DG_ARG(op >= 0 && op < 3, "bad op %d", op);
    *bytes = d->plan[op].ws_bytes;
    return DG_OK;
}

int dg_conv_planes_size(dg_conv_t d, int tensor, size_t *bytes) {
    DG_ARG(d && bytes, "NULL argument");
    DG_ARG(tensor == DG_TENSOR_X || tensor == DG_TENSOR_DY || tensor == DG_TENSOR_W, "bad tensor id %d", tensor);
    *bytes = dg::tensor_plane_bytes(d, tensor);
    return DG_OK;
}

int dg_conv_planes_format(dg_conv_t d, int tensor, int *format) {
    DG_ARG(d && format, "NULL argument");
    DG_ARG(tensor == DG_TENSOR_X || tensor == DG_TENSOR_DY || tensor == DG_TENSOR_W, "bad tensor id %d", tensor);
    *format = dg::tensor_x3(d, tensor) ? DG_PLANES_F16X3 : DG_PLANES_BF16X6;
    return DG_OK;
}

int dg_absmax(const float *x, int64_t rows, int C, int ld, float *out, dg_stream_t stream) {
    DG_ARG(x && out, "NULL tensor");
    DG_ARG(rows >= 0 && C > 0 && ld >= C, "bad shape");
    dg::launch_absmax(x, rows, C, ld, out, (hipStream_t)stream);
    DG_LAUNCHED("absmax");
    return DG_OK;
}

int dg_absmax_set(const float *x, int64_t rows, int C, int ld, float *out, dg_stream_t stream) {
    DG_ARG(out, "NULL tensor");
    if (hipMemsetAsync(out, 0, dg::X3_SLOT * sizeof(float), (hipStream_t)stream) != hipSuccess) {
        dg::set_error("hipMemsetAsync failed");
        return DG_ERR_HIP;
    }
    return dg_absmax(x, rows, C, ld, out, stream);
}

int dg_weight_bound(const float *w, int64_t K, int Co, const float *bias, float *g_out, float *c_out,
                    float *zero8, dg_stream_t stream) {
    DG_ARG(w && g_out, "NULL tensor");
    DG_ARG(K > 0 && Co > 0, "bad shape");
    dg::launch_weight_bound(w, K, Co, bias, g_out, c_out, (hipStream_t)stream, zero8);
    DG_LAUNCHED("weight_bound");
    return DG_OK;
}

int dg_weight_bound_in(const float *w, int taps, int Ci, int Co, float *g_out, dg_stream_t stream) {
    DG_ARG(w && g_out, "NULL tensor");
    DG_ARG(taps > 0 && Ci > 0 && Co > 0, "bad shape");
    dg::launch_weight_bound_in(w, taps, Ci, Co, g_out, (hipStream_t)stream);
    DG_LAUNCHED("weight_bound_in");
    return DG_OK;
}

int dg_conv_set_grad_scale(dg_conv_t d, const float *dy_m, const float *dy_g, const float *dx_m, const float *dx_g,
                           float *dx_max) {
    DG_ARG(d != nullptr, "descriptor is NULL");
    d->gs_dy_m = dy_m; d->gs_dy_g = dy_g; d->gs_dx_m = dx_m; d->gs_dx_g = dx_g; d->gs_dx_max = dx_max;
    return DG_OK;
}

int dg_conv_set_act_scale(dg_conv_t d, const float *x_m, const float *x_g, const float *x_c, const float *y_m,
                          const float *y_g, const float *y_c, float *y_max) {
    DG_ARG(d != nullptr, "descriptor is NULL");
    DG_ARG(x_m || (!x_g && !x_c), "x scale source: g / c without m");
    DG_ARG(y_m || (!y_g && !y_c), "output scale source: g / c without m");
    d->as_x_m = x_m; d->as_x_g = x_g; d->as_x_c = x_c;
    d->as_y_m = y_m; d->as_y_g = y_g; d->as_y_c = y_c; d->as_y_max = y_max;
    return DG_OK;
}

int dg_conv_op_arith(dg_conv_t d, int op, int *arith) {
    DG_ARG(d && arith, "NULL argument");
    DG_ARG(op >= 0 && op < 3, "bad op %d", op);
    const dg::OpPlan &pl = d->rc[op].on ? d->rc[op].p1 : d->plan[op];
    *arith = (pl.narrow || pl.co1 || pl.small || pl.ntile) ? DG_MATH_FP32 : pl.x6;
    return DG_OK;
}

int dg_conv_op_planes(dg_conv_t d, int op, int *tensors) {
    DG_ARG(d && tensors, "NULL argument");
    DG_ARG(op >= 0 && op < 3, "bad op %d", op);
    *tensors = dg::op_plane_mask(d, op);
    return DG_OK;
}

int dg_conv_fwd_pl(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias, float *y, int ldy,
                   float beta, int act, float alpha, const dg_conv_planes_t *planes, void *ws, size_t ws_bytes,
                   dg_stream_t stream) {
    DG_ARG(d && x && w && (y || (planes && planes->out)), "NULL tensor");
    DG_ARG(ldx >= d->Cin && (!y || ldy >= d->Cout), "pixel stride smaller than channels");
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int e = dg::plane_refs(d, DG_OP_FWD, planes, r, pr);
    if (e != DG_OK) return e;
    return dg::run_engine(d, DG_OP_FWD, x, ldx, w, d->transpose ? 0 : d->Cout, y, ldy, bias, beta, act, alpha, ws,
                          ws_bytes, (hipStream_t)stream, nullptr, 0, DG_ACT_NONE, 0.f, pr,
                          planes ? (unsigned short *)planes->out : nullptr, nullptr, nullptr,
                          planes ? planes->out_format : DG_PLANES_BF16X6);
}

int dg_conv_fwd_pool_ok(dg_conv_t d, int act, int *ok) {
    DG_ARG(d && ok, "NULL argument");
    *ok = dg::pool_fusable(d, act) ? 1 : 0;
    return DG_OK;
}

int dg_conv_fwd_pool(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias, int act, float alpha,
                     float *pool_y, int ldpy, unsigned char *pool_idx, const dg_conv_planes_t *planes, void *ws,
                     size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(d && x && w && pool_idx, "NULL tensor");
    DG_ARG(ldx >= d->Cin, "pixel stride smaller than channels");
    DG_ARG(act >= DG_ACT_NONE && act <= DG_ACT_SIGMOID, "unknown activation %d", act);
    if (!dg::pool_fusable(d, act)) {
        dg::set_error("forward plan cannot fuse the max pool (dg_conv_fwd_pool_ok)");
        return DG_ERR_UNSUPPORTED;
    }
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int e = dg::plane_refs(d, DG_OP_FWD, planes, r, pr);
    if (e != DG_OK) return e;
    dg::PoolOut po{pool_idx, pool_y, ldpy, planes ? (unsigned short *)planes->out : nullptr,
                   planes ? planes->out_format : DG_PLANES_BF16X6};
    return dg::run_engine(d, DG_OP_FWD, x, ldx, w, d->Cout, nullptr, d->Cout, bias, 0.f, act, alpha, ws, ws_bytes,
                          (hipStream_t)stream, nullptr, 0, DG_ACT_NONE, 0.f, pr, nullptr, &po);
}

int dg_conv_fwd(dg_conv_t d, const float *x, int ldx, const float *w, const float *bias, float *y, int ldy,
                float beta, int act, float alpha, void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_conv_fwd_pl(d, x, ldx, w, bias, y, ldy, beta, act, alpha, nullptr, ws, ws_bytes, stream);
}

int dg_conv_bwd_data_pl(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx, float beta,
                        const float *z, int ldz, int act, float alpha, const dg_conv_planes_t *planes, void *ws,
                        size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(d && dy && w && dx, "NULL tensor");
    DG_ARG(lddy >= d->Cout && lddx >= d->Cin, "pixel stride smaller than channels");
    DG_ARG(!z || ldz >= d->Cin, "pixel stride smaller than channels");
    DG_ARG(act >= DG_ACT_NONE && act <= DG_ACT_SIGMOID, "unknown activation %d", act);
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int e = dg::plane_refs(d, DG_OP_BWD_DATA, planes, r, pr);
    if (e != DG_OK) return e;
    return dg::run_engine(d, DG_OP_BWD_DATA, dy, lddy, w, d->transpose ? d->g.Co : 0, dx, lddx, nullptr, beta,
                          DG_ACT_NONE, 0.f, ws, ws_bytes, (hipStream_t)stream, z, z ? ldz : 0,
                          z ? act : DG_ACT_NONE, alpha, pr, planes ? (unsigned short *)planes->out : nullptr, nullptr,
                          nullptr, planes ? planes->out_format : DG_PLANES_BF16X6);
}

int dg_conv_bwd_data_masked_sum(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx,
                                float beta, const float *z, int ldz, int act, float alpha,
                                const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(d && dy && w && dx && z, "NULL tensor");
    DG_ARG(lddy >= d->Cout && lddx >= d->Cin && ldz >= d->Cin, "pixel stride smaller than channels");
    DG_ARG(act >= DG_ACT_NONE && act <= DG_ACT_SIGMOID, "unknown activation %d", act);
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int e = dg::plane_refs(d, DG_OP_BWD_DATA, planes, r, pr);
    if (e != DG_OK) return e;
    return dg::run_engine(d, DG_OP_BWD_DATA, dy, lddy, w, d->transpose ? d->g.Co : 0, dx, lddx, nullptr, beta,
                          DG_ACT_NONE, 0.f, ws, ws_bytes, (hipStream_t)stream, z, ldz, act | dg::DG_MASK_SUM, alpha,
                          pr, planes ? (unsigned short *)planes->out : nullptr, nullptr, nullptr,
                          planes ? planes->out_format : DG_PLANES_BF16X6);
}

int dg_conv_bwd_data_xmask(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx, float beta,
                           int act, float alpha, const dg_conv_planes_t *planes, void *ws, size_t ws_bytes,
                           dg_stream_t stream) {
    DG_ARG(d && dy && w && dx && planes && planes->x, "NULL tensor or x planes");
    DG_ARG((planes->ready & DG_TENSOR_X) != 0, "x planes not ready (written by x's producer or a split)");
    DG_ARG((((uintptr_t)planes->x) & 7) == 0, "x planes must be 8-byte aligned");
    DG_ARG(lddy >= d->Cout && lddx >= d->Cin, "pixel stride smaller than channels");
    DG_ARG(d->Cin % 16 == 0, "x planes need Cin %% 16 == 0");
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int e = dg::plane_refs(d, DG_OP_BWD_DATA, planes, r, pr);
    if (e != DG_OK) return e;
    return dg::run_engine(d, DG_OP_BWD_DATA, dy, lddy, w, d->transpose ? d->g.Co : 0, dx, lddx, nullptr, beta,
                          DG_ACT_NONE, 0.f, ws, ws_bytes, (hipStream_t)stream, nullptr, 0, act, alpha, pr,
                          (unsigned short *)planes->out, nullptr, (const unsigned short *)planes->x,
                          planes->out_format);
}

int dg_conv_bwd_data(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx, float beta,
                     void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_conv_bwd_data_pl(d, dy, lddy, w, dx, lddx, beta, nullptr, 0, DG_ACT_NONE, 0.f, nullptr, ws, ws_bytes,
                               stream);
}

int dg_conv_bwd_data_masked(dg_conv_t d, const float *dy, int lddy, const float *w, float *dx, int lddx,
                            float beta, const float *z, int ldz, int act, float alpha, void *ws, size_t ws_bytes,
                            dg_stream_t stream) {
    DG_ARG(z, "NULL tensor");
    return dg_conv_bwd_data_pl(d, dy, lddy, w, dx, lddx, beta, z, ldz, act, alpha, nullptr, ws, ws_bytes, stream);
}

int dg_conv_bwd_filter(dg_conv_t d, const float *x, int ldx, const float *dy, int lddy, float *dw, float *dbias,
                       float beta, void *ws, size_t ws_bytes, dg_stream_t stream) {
    return dg_conv_bwd_filter_pl(d, x, ldx, dy, lddy, dw, dbias, beta, nullptr, ws, ws_bytes, stream);
}

int dg_conv_bwd_filter_pl(dg_conv_t d, const float *x, int ldx, const float *dy, int lddy, float *dw, float *dbias,
                          float beta, const dg_conv_planes_t *planes, void *ws, size_t ws_bytes, dg_stream_t stream) {
    DG_ARG(d && x && dy && dw, "NULL tensor");
    DG_ARG(ldx >= d->Cin && lddy >= d->Cout, "pixel stride smaller than channels");
    const dg::OpPlan &pl = d->plan[DG_OP_BWD_FILTER];
    DG_ARG(ws_bytes >= pl.ws_bytes && ws != nullptr, "workspace too small: need %zu bytes", pl.ws_bytes);
    size_t slab_bytes = pl.colsum_off;
    dg::PlaneRefs r{};
    const dg::PlaneRefs *pr;
    int rc = dg::plane_refs(d, DG_OP_BWD_FILTER, planes, r, pr);
    if (rc != DG_OK) return rc;
    // conv view: A = conv input, B = conv output grad
    if (!d->transpose)
        rc = dg::run_engine(d, DG_OP_BWD_FILTER, x, ldx, dy, lddy, dw, d->g.Co, nullptr, beta, DG_ACT_NONE, 0.f, ws,
                            slab_bytes, (hipStream_t)stream, nullptr, 0, DG_ACT_NONE, 0.f, pr);
    else
        rc = dg::run_engine(d, DG_OP_BWD_FILTER, dy, lddy, x, ldx, dw, d->g.Co, nullptr, beta, DG_ACT_NONE, 0.f, ws,
                            slab_bytes, (hipStream_t)stream, nullptr, 0, DG_ACT_NONE, 0.f, pr);
    if (rc != DG_OK) return rc;
    if (dbias) {
        long M = (long)d->N * d->Ho * d->Wo;
        float *cws = (float *)((char *)ws + pl.colsum_off);
        return dg::run_colsum(dy, lddy, M, d->Cout, dbias, beta, cws, (hipStream_t)stream);
    }
    return DG_OK;
}

}  // extern "C"
