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

template <int MODE, int BM, int BN, int WGM, int WGN, int MINW>
__global__ void __launch_bounds__(64 * WGM * WGN, MINW)
k_conv_gemm_x6(const GemmArgs p) {
    constexpr int BK = 16;
    constexpr bool A_KC = (MODE != MODE_WGRAD);
    constexpr bool B_KC = (MODE == MODE_DGRAD);
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int APL = BM * 32, BPL = BN * 32;     // bytes per plane
    constexpr int BUF = 3 * (APL + BPL);            // bytes per buffer
    constexpr int NT = 64 * WGM * WGN;  // threads
    static_assert(WGM * WGN == 4 || WGM * WGN == 8, "4 or 8 waves");
    static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
    static_assert(BM % (NT / 4) == 0 && BN % (NT / 4) == 0 && (4 * BM) % NT == 0 && (4 * BN) % NT == 0 &&
                  BM <= 256 && BN <= 256, "loader geometry");

    __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

    const ConvGeom &g = p.g;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid / WGN, wn = wid % WGN;
    const int l32 = lane & 31, h2 = lane >> 5;

    const int zz = blockIdx.y;
    const int phase = zz / p.splits;
    const int split = zz - phase * p.splits;
    const int tile = blockIdx.x;
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

    // ---- loader geometry ----
    // KC: rows x 16 k, one float4 (4 k) per (row, c4); NT/4 rows per pass
    const int kc_c4 = tid & 3, kc_r = tid >> 2;
    constexpr int KRP = NT / 4;
    constexpr int A_KCP = BM / KRP, B_KCP = BN / KRP;
    // RC: 16 k-rows x COLS, one float4 (4 columns) per (k-row, column quad)
    constexpr int A_RCQ = BM / 4, B_RCQ = BN / 4;    // column quads per k-row
    constexpr int A_RCP = 4 * BM / NT, B_RCP = 4 * BN / NT;  // passes (k-rows per thread)
    const int ar_cq = tid % A_RCQ, ar_r = tid / A_RCQ;
    const int br_cq = tid % B_RCQ, br_r = tid / B_RCQ;

    // KC A rows (FWD / DGRAD)
    int arow_n[A_KCP], arow_h[A_KCP], arow_w[A_KCP];
    if constexpr (A_KC) {
#pragma unroll
        for (int ip = 0; ip < A_KCP; ++ip) {
            int m = m0 + kc_r + KRP * ip;
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
    // WGRAD A: the thread's column quad is 4 consecutive ci of one tap
    int wg_i = 0, wg_j = 0, wg_ci = 0; bool wg_ok = false;
    if constexpr (MODE == MODE_WGRAD) {
        int mc = m0 + 4 * ar_cq;
        wg_ok = mc < p.M;
        int tap = mc / g.Ci; wg_ci = mc - tap * g.Ci; wg_i = tap / g.kw; wg_j = tap - wg_i * g.kw;
    }

    auto dgrad_tap = [&](int k, int &i, int &j, int &co) {
        int tap = k / g.Co; co = k - tap * g.Co;
        int a = tap / g.Tw; int b = tap - a * g.Tw;
        i = ph.i0h + a * g.sh; j = ph.i0w + b * g.sw;
    };
    // channel-chunk-major K walk for FWD / DGRAD (see k_conv_gemm)
    auto k_real = [&](int k0) -> int {
        if constexpr (MODE != MODE_WGRAD) {
            const int C = MODE == MODE_FWD ? g.Ci : g.Co;
            const int ntap = MODE == MODE_FWD ? g.kh * g.kw : g.Th * g.Tw;
            int kk = k0 / BK; int chunk = kk / ntap; int tap = kk - chunk * ntap;
            return tap * C + chunk * BK;
        } else {
            return k0;
        }
    };

    const rsrc_t rA = make_rsrc(p.A, p.a_bytes);
    const rsrc_t rB = make_rsrc(p.B, p.b_bytes);

    // staging registers
    constexpr int A_REGS = A_KC ? A_KCP : A_RCP;
    constexpr int B_REGS = B_KC ? B_KCP : B_RCP;
    f32x4 ra[A_REGS], rb[B_REGS];

    auto load_tiles = [&](int k0) {
        const int kr0 = k_real(k0);
        // ----- A -----
        if constexpr (MODE == MODE_FWD) {
            int tap = kr0 / g.Ci; int ci0 = kr0 - tap * g.Ci;
            int i = tap / g.kw; int j = tap - i * g.kw;
#pragma unroll
            for (int ip = 0; ip < A_KCP; ++ip) {
                int hi = arow_h[ip] + i, wi = arow_w[ip] + j;
                bool ok = arow_n[ip] >= 0 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                unsigned off = ((unsigned)((arow_n[ip] * g.H + hi) * g.W + wi) * p.lda + ci0 + 4 * kc_c4) * 4u;
                ra[ip] = bload4(rA, ok ? off : DG_OOB);
            }
        } else if constexpr (MODE == MODE_DGRAD) {
            int i, j, co0; dgrad_tap(kr0, i, j, co0);
            bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
            for (int ip = 0; ip < A_KCP; ++ip) {
                int th = arow_h[ip] + g.pt - i, tw = arow_w[ip] + g.pl - j;
                int ho = th / g.sh, wo = tw / g.sw;
                bool ok = tapok && arow_n[ip] >= 0 && th >= 0 && tw >= 0 && ho < g.Ho && wo < g.Wo;
                unsigned off = ((unsigned)((arow_n[ip] * g.Ho + ho) * g.Wo + wo) * p.lda + co0 + 4 * kc_c4) * 4u;
                ra[ip] = bload4(rA, ok ? off : DG_OOB);
            }
        } else {  // WGRAD: x gathered at the thread's tap, k-rows are output pixels
#pragma unroll
            for (int ip = 0; ip < A_RCP; ++ip) {
                int pix = k0 + ar_r + (NT / A_RCQ) * ip;
                int wo = pix % g.Wo; int t = pix / g.Wo; int ho = t % g.Ho; int n = t / g.Ho;
                int hi = ho * g.sh - g.pt + wg_i, wi = wo * g.sw - g.pl + wg_j;
                bool ok = wg_ok && pix < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                unsigned off = ((unsigned)((n * g.H + hi) * g.W + wi) * p.lda + wg_ci) * 4u;
                ra[ip] = bload4(rA, ok ? off : DG_OOB);
            }
        }
        // ----- B -----
        if constexpr (MODE == MODE_FWD) {  // w[k][co]
            const int col = n0 + 4 * br_cq;
#pragma unroll
            for (int ip = 0; ip < B_RCP; ++ip) {
                unsigned k = (unsigned)(kr0 + br_r + (NT / B_RCQ) * ip);
                rb[ip] = bload4(rB, col < p.N ? (k * p.ldb + col) * 4u : DG_OOB);
            }
        } else if constexpr (MODE == MODE_DGRAD) {  // w[i,j,ci,co]: rows ci contiguous along co
            int i, j, co0; dgrad_tap(kr0, i, j, co0);
            bool tapok = (i < g.kh) && (j < g.kw);
#pragma unroll
            for (int ip = 0; ip < B_KCP; ++ip) {
                int ci = n0 + kc_r + KRP * ip;
                bool ok = tapok && ci < p.N;
                unsigned off = ((unsigned)((i * g.kw + j) * g.Ci + ci) * g.Co + co0 + 4 * kc_c4) * 4u;
                rb[ip] = bload4(rB, ok ? off : DG_OOB);
            }
        } else {  // WGRAD: dy rows (pixels) contiguous along co
            const int col = n0 + 4 * br_cq;
#pragma unroll
            for (int ip = 0; ip < B_RCP; ++ip) {
                int pix = k0 + br_r + (NT / B_RCQ) * ip;
                bool ok = col < p.N && pix < kend;
                rb[ip] = bload4(rB, ok ? ((unsigned)pix * p.ldb + col) * 4u : DG_OOB);
            }
        }
    };

    // one float4 -> three 8-byte plane writes at byte offset o
    auto store4 = [&](char *base, int plane_bytes, int o, const f32x4 &v) {
        unsigned h0, m0_, l0, h1, m1, l1;
        split3(v[0], v[1], h0, m0_, l0);
        split3(v[2], v[3], h1, m1, l1);
        *reinterpret_cast<u32x2 *>(base + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2 *>(base + plane_bytes + o) = u32x2{m0_, m1};
        *reinterpret_cast<u32x2 *>(base + 2 * plane_bytes + o) = u32x2{l0, l1};
    };

    auto store_tiles = [&](int buf) {
        char *As = smem + buf * BUF;
        char *Bs = As + 3 * APL;
        if constexpr (A_KC) {
#pragma unroll
            for (int ip = 0; ip < A_KCP; ++ip) store4(As, APL, x6_off(kc_r + KRP * ip, 4 * kc_c4), ra[ip]);
        } else {
#pragma unroll
            for (int ip = 0; ip < A_RCP; ++ip)
                store4(As, APL, x6_rc_off<BM>(ar_r + (NT / A_RCQ) * ip, 4 * ar_cq), ra[ip]);
        }
        if constexpr (B_KC) {
#pragma unroll
            for (int ip = 0; ip < B_KCP; ++ip) store4(Bs, BPL, x6_off(kc_r + KRP * ip, 4 * kc_c4), rb[ip]);
        } else {
#pragma unroll
            for (int ip = 0; ip < B_RCP; ++ip)
                store4(Bs, BPL, x6_rc_off<BN>(br_r + (NT / B_RCQ) * ip, 4 * br_cq), rb[ip]);
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
#pragma unroll
        for (int a = 0; a < TM; ++a) {
            if constexpr (A_KC) {
                const int o = x6_off(wm * WTM + a * 32 + l32, 8 * h2);
#pragma unroll
                for (int s = 0; s < 3; ++s) af[s][a] = *reinterpret_cast<const bf16x8 *>(As + s * APL + o);
            } else {
#pragma unroll
                for (int s = 0; s < 3; ++s) af[s][a] = x6_rc_frag<BM>(As + s * APL, wm * WTM + a * 32, lane);
            }
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            if constexpr (B_KC) {
                const int o = x6_off(wn * WTN + b * 32 + l32, 8 * h2);
#pragma unroll
                for (int s = 0; s < 3; ++s) bf[s][b] = *reinterpret_cast<const bf16x8 *>(Bs + s * BPL + o);
            } else {
#pragma unroll
                for (int s = 0; s < 3; ++s) bf[s][b] = x6_rc_frag<BN>(Bs + s * BPL, wn * WTN + b * 32, lane);
            }
        }
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
        __syncthreads();
    }

    conv_epilogue<MODE, TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, Mrows, ph, phase, split, l32, h2);
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
    }
#undef DG_X6
}

}  // namespace dg
