// Shared device-side definitions of the conv engine (conv.hip: fp32 MFMA
// kernels, planner and C ABI; conv_x6.hip: the bf16x6 split-precision kernel).
#pragma once
#include "common.h"

namespace dg {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
// run_engine's mask activation flag: the mask multiplies the accumulated sum (GemmArgs.mask_acc)
constexpr int DG_MASK_SUM = 0x100;

struct ConvGeom {
    int N, H, W, Ci;  // conv-view input
    int Ho, Wo, Co;   // conv-view output
    int kh, kw, sh, sw, pt, pl;
    int Th, Tw;       // DGRAD taps per phase
};

struct GemmArgs {
    ConvGeom g;
    const float *A; int lda;
    const float *B; int ldb;
    float *C; int ldc;
    const float *bias;
    float beta; int act; float alpha;
    int M, N, K;       // GEMM dims; DGRAD: M = max rows over phases
    int kchunk;        // K per split (multiple of BK)
    int splits;
    int mtiles, ntiles;
    int nphase;
    float *slab;       // split-K partials [nphase*splits][M][N]
    unsigned a_bytes, b_bytes;  // extents of A and B for the buffer-resource range check
    unsigned mg_wo, mg_ho;      // multiply-shift division by g.Wo / g.Ho (bf16x6 WGRAD)
    int sh_wo, sh_ho;
    // optional gradient mask of the output (dg_conv_bwd_data_masked):
    // C = (result * act'(mz)) + beta*C, act' expressed through the activation's output mz
    const float *mz; int ldmz; int mact; float malpha;
    // optional planes of the final output (dg_conv_planes_t.out), written beside C:
    // ypC > 0 bf16x6 [pixel][3 * ypC] in the packed layout of k_split3; ypC < 0 the
    // consumer's fp16x3 planes [pixel][2 * -ypC] (common.h store_planes4)
    unsigned short *yp; int ypC;
    // optional MaxPool2D(2) of the activated output, fused into the forward
    // epilogue of the halo kernel (dg_conv_fwd_pool): the pooled output's
    // planes go to yp (pooled pixel index), its fp32 values to pool_y (may be
    // NULL), and per element one byte to pidx: bits 0-1 the window position
    // of the first maximum (row-major), bit 2 set when the pooled value > 0.
    // C (the full-size output) is not written.
    unsigned char *pidx; float *pool_y; int ldpy;
    // fp16x3 scale sources (x3_grad_scale: bound = max(m) * g + c) of the A and B operand
    // planes (m NULL: the static scale x3_sa / x3_sb -- F16X3_XS, F16X3_WS for weights) and of
    // the output planes (ys_m NULL: F16X3_XS); ymax receives max |output|
    const float *as_m, *as_g, *as_c, *bs_m, *bs_g, *bs_c, *ys_m, *ys_g, *ys_c;
    float *ymax;
    // fp16x3 GEMMs: which operand is the gradient (0 none, 1 A, 2 B) -- measured here when it
    // arrives without a scale source -- and the static scales
    int x3_dyn; float x3_sa, x3_sb;
    // optional gradient mask from the planes of the activation output instead of
    // its fp32 values (dg_conv_bwd_data_xmask): act' of a sign-determined
    // activation from the sign of the hi plane, [pixel][3 mzpC] (mzpC < 0: fp16x3)
    const unsigned short *mzp; int mzpC;
    // 1: DGRAD phase blocks in the plain XCD order (A/B switch DG_PLAN_DISABLE=xcd_phase)
    int xcd_plain;
    // fp16x3 halo kernel: patches per block (blocks gm = gridDim.x / ntiles; block's patches
    // mt0 + j * gm, j < ptiles); other kernels 1
    int ptiles;
    // 1: the gradient mask also multiplies the accumulated beta*C (dg_conv_bwd_data_masked_sum:
    // C = act'(mz) * (result + beta*C), a fan-in whose other contribution arrived unmasked)
    int mask_acc;
    // halo kernel, one patch per block, one phase, no split: > 0 = the n-tiles are dealt to the
    // XCDs in xcd_ng groups (XCD x runs the n-tiles of group x % xcd_ng over patches of part
    // x / xcd_ng), so an XCD's L2 keeps its weight columns instead of streaming every column of
    // the filter (xcd_group_tile); 0: the plain XCD order
    int xcd_ng;
};

// (mt, nt) of this block under the n-grouped XCD raster (GemmArgs.xcd_ng = NG > 0): blocks are
// dealt round-robin to the 8 XCDs (lin & 7 labels the XCD, lin >> 3 the dispatch order on it);
// XCD x takes n-tiles [g TPG, (g+1) TPG) of group g = x % NG and patches [h MPH, (h+1) MPH) of
// part h = x / NG, TPG = ntiles / NG, MPH = mtiles / (8 / NG).  A bijection when the grid is
// mtiles x ntiles with both divisible as stated (the planner checks); speed only, any placement
// is correct.
__device__ __forceinline__ void xcd_group_tile(int ng, int mtiles, int ntiles, int &mt, int &nt) {
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int x = lin & 7, idx = lin >> 3;
    const int tpg = ntiles / ng, mph = mtiles / (8 / ng);
    nt = (x % ng) * tpg + idx % tpg;
    mt = (x / ng) * mph + idx / tpg;
}

// the factor that undoes an fp16x3 GEMM's operand scales (powers of two: exact)
__device__ __forceinline__ float x3_out_scale(const GemmArgs &p) {
    const float sa = p.as_m ? x3_grad_scale(p.as_m, p.as_g, p.as_c) : p.x3_sa;
    const float sb = p.bs_m ? x3_grad_scale(p.bs_m, p.bs_g, p.bs_c) : p.x3_sb;
    return 1.f / (sa * sb);
}

// the scale sources of an fp16x3 GEMM (operands A, B and the output planes), loaded at kernel entry
struct X3Pre {
    X3Raw a, b, y;
};
__device__ __forceinline__ X3Pre x3_pre(const GemmArgs &p) {
    return X3Pre{x3_raw(p.as_m, p.as_g, p.as_c), x3_raw(p.bs_m, p.bs_g, p.bs_c), x3_raw(p.ys_m, p.ys_g, p.ys_c)};
}
__device__ __forceinline__ float x3_out_scale(const GemmArgs &p, const X3Pre &r) {
    return 1.f / (x3_raw_scale(r.a, p.x3_sa) * x3_raw_scale(r.b, p.x3_sb));
}

// hi plane of element (pix, col) of a packed plane tensor, as a float (its sign is
// the element's; C < 0: fp16x3 planes of -C channels, the value times F16X3_XS)
__device__ __forceinline__ float hi_plane(const unsigned short *zp, int C, long pix, int col) {
    if (C < 0)
        return (float)reinterpret_cast<const _Float16 *>(zp)[pix * 2 * (-C) + (col >> 5) * 64 + (col & 31)];
    return __uint_as_float((unsigned)zp[pix * 3 * C + (col >> 4) * 48 + (col & 15)] << 16);
}
// the same for columns col..col+3 (col % 4 == 0): one 8-byte load
__device__ __forceinline__ f32x4 hi_plane4(const unsigned short *zp, int C, long pix, int col) {
    if (C < 0) {
        const f16x4_t h = *reinterpret_cast<const f16x4_t *>(reinterpret_cast<const _Float16 *>(zp) +
                                                           pix * 2 * (-C) + (col >> 5) * 64 + (col & 31));
        return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    }
    const u32x2_t h = *reinterpret_cast<const u32x2_t *>(zp + pix * 3 * C + (col >> 4) * 48 + (col & 15));
    return f32x4{__uint_as_float(h[0] << 16), __uint_as_float(h[0] & 0xffff0000u), __uint_as_float(h[1] << 16),
                 __uint_as_float(h[1] & 0xffff0000u)};
}

// the fp16x3 scale of the output planes (static activation scale unless a gradient source is set)
__device__ __forceinline__ float plane_scale(const GemmArgs &p) {
    return p.ys_m ? x3_grad_scale(p.ys_m, p.ys_g, p.ys_c) : F16X3_XS;
}

__device__ __forceinline__ float epi_mask_factor(const GemmArgs &p, long pix, int col) {
    if (p.mz) return act_grad_from_out(p.mz[pix * p.ldmz + col], p.mact, p.malpha);
    if (p.mzp) return act_grad_from_out(hi_plane(p.mzp, p.mzpC, pix, col), p.mact, p.malpha);
    return 1.f;
}
__device__ __forceinline__ float epi_mask(const GemmArgs &p, long pix, int col, float v) {
    if (p.mz) return v * act_grad_from_out(p.mz[pix * p.ldmz + col], p.mact, p.malpha);
    if (p.mzp) return v * act_grad_from_out(hi_plane(p.mzp, p.mzpC, pix, col), p.mact, p.malpha);
    return v;
}

// Branch-free operand loads: raw buffer loads through a resource whose range
// check returns 0 for an out-of-range offset, so padding taps and ragged tile
// edges need no exec-masked branches (an invalid element is given DG_OOB).
constexpr unsigned DG_OOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const float *base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, unsigned byte_off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
__device__ __forceinline__ float bload1(rsrc_t r, unsigned byte_off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8
// XCDs (linear id % 8), each with its own 4 MiB L2.  Renumber the linear id
// so that each XCD receives a contiguous range of (split, tile) ids: with the
// n-tile fastest in the tile id, the n-tiles of one m-tile (which read the
// same A rows) and neighbouring m-tiles (which share halo rows) then run on
// one XCD and hit its L2 instead of each XCD fetching them.
// y_fast: decode the contiguous ids with y fastest instead -- for a DGRAD
// whose grid y runs over sub-pixel phases, the phases of one tile read the
// same dy rows, so they then run back to back on one XCD (its L2 serves the
// later ones) instead of on different XCDs that each fetch dy from HBM.
__device__ __forceinline__ void xcd_remap(int &y, int &x, bool y_fast = false) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int total = nx * ny;
    const int lin = blockIdx.y * nx + blockIdx.x;
    const int q = total >> 3, r = total & 7, xcd = lin & 7, idx = lin >> 3;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    if (y_fast) {
        x = id / ny;
        y = id - x * ny;
    } else {
        y = id / nx;
        x = id - y * nx;
    }
}

// n / d = (umulhi(n, mul) + n) >> shr for 0 <= n < 2^31 (round-up magic number)
inline void fastdiv_magic(unsigned d, unsigned &mul, int &shr) {
    int s = 0;
    while ((1ull << s) < d) ++s;
    mul = (unsigned)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    shr = s;
}

struct PhaseInfo {
    int ph, pw, Hp, Wp, Mp, i0h, i0w;
};

__device__ __forceinline__ PhaseInfo phase_info(const ConvGeom &g, int phase, int N) {
    PhaseInfo q;
    q.ph = phase / g.sw;
    q.pw = phase - q.ph * g.sw;
    q.Hp = (g.H - q.ph + g.sh - 1) / g.sh;
    q.Wp = (g.W - q.pw + g.sw - 1) / g.sw;
    if (q.Hp < 0) q.Hp = 0;
    if (q.Wp < 0) q.Wp = 0;
    q.Mp = N * q.Hp * q.Wp;
    q.i0h = ((q.ph + g.pt) % g.sh + g.sh) % g.sh;
    q.i0w = ((q.pw + g.pl) % g.sw + g.sw) % g.sw;
    return q;
}

// Row of a GEMM tile -> (row of the split-K slab, output pixel); slab < 0
// marks a row outside the output.
struct RowPix {
    long slab, pix;
};

// The same for 16x16 accumulator tiles (v_mfma_f32_16x16x32_bf16 C layout:
// col = lane&15, row = 4(lane>>4) + r), staged through LDS: the wave writes
// 16 rows of its tile at a time into `stage` (16 x (16*TN + 4) floats, its
// own region) and reads them back row-contiguous, so every global access is
// 16 bytes per lane (C, the split-K slab, beta*C and the gradient mask) and
// the row -> pixel map (`rowmap(rbase + local row)` -> RowPix) is evaluated
// once per row per lane.
// What the GEMM epilogues hoist per call (epi_out4)
struct EpiCtx {
    bool cvec, mvec, svec;   // 16-byte C / gradient mask / split-K slab access possible
    float ys;                // the output planes' scale
};
__device__ __forceinline__ EpiCtx epi_ctx(const GemmArgs &p, float ys_pre) {
    EpiCtx e;
    e.cvec = ((p.ldc & 3) == 0) && ((((uintptr_t)p.C) & 15) == 0);
    e.mvec = ((p.ldmz & 3) == 0) && ((((uintptr_t)p.mz) & 15) == 0);
    e.svec = ((p.N & 3) == 0) && ((((uintptr_t)p.slab) & 15) == 0);
    e.ys = p.yp ? (ys_pre > 0.f ? ys_pre : plane_scale(p)) : 0.f;
    return e;
}

// Output columns col .. col+3 of GEMM row rp (staged accumulators v): the split-K slab, or bias +
// activation + gradient mask + beta*C into C, the consumer's planes and the max |output|.
__device__ __forceinline__ void epi_out4(const GemmArgs &p, const EpiCtx &e, const RowPix &rp, int col, const f32x4 &v,
                                         int phase, int split, float &vmax) {
    if (rp.slab < 0 || col >= p.N) return;
    const bool full = col + 3 < p.N;
    if (p.splits > 1) {
        float *dst = p.slab + ((long)(phase * p.splits + split) * p.M + rp.slab) * p.N + col;
        if (e.svec && full) {
            *reinterpret_cast<f32x4 *>(dst) = v;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (col + q < p.N) dst[q] = v[q];
        }
        return;
    }
    const long pix = rp.pix;
    float *dst = p.C + pix * p.ldc + col;
    f32x4 o = v;
    if (p.bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] += (col + q < p.N) ? p.bias[col + q] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = act_fwd(o[q], p.act, p.alpha);
    f32x4 mf = {1.f, 1.f, 1.f, 1.f};   // the mask factors (p.mask_acc: beta*C's too)
    if (p.mz) {
        const float *mz = p.mz + pix * p.ldmz + col;
        f32x4 z;
        if (e.mvec && full) {
            z = *reinterpret_cast<const f32x4 *>(mz);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = (col + q < p.N) ? mz[q] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) mf[q] = act_grad_from_out(z[q], p.mact, p.malpha);
        o *= mf;
    } else if (p.mzp) {
        f32x4 z;
        if (full) {
            z = hi_plane4(p.mzp, p.mzpC, pix, col);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = (col + q < p.N) ? hi_plane(p.mzp, p.mzpC, pix, col + q) : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) mf[q] = act_grad_from_out(z[q], p.mact, p.malpha);
        o *= mf;
    }
    if (!p.C) {
        // planes-only output (dg_conv_fwd_pl with y == NULL, beta 0)
    } else if (e.cvec && full) {
        if (p.beta != 0.f) {
            const f32x4 c = *reinterpret_cast<const f32x4 *>(dst);
            o += p.beta * (p.mask_acc ? c * mf : c);
        }
        *reinterpret_cast<f32x4 *>(dst) = o;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (col + q < p.N)
                o[q] = dst[q] = p.beta != 0.f ? o[q] + p.beta * (p.mask_acc ? dst[q] * mf[q] : dst[q]) : o[q];
    }
    if (p.yp) {
        if (full) {
            store_planes4(p.yp, p.ypC, pix, col, o, e.ys);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (col + q < p.N) store_planes1(p.yp, p.ypC, pix, col + q, o[q], e.ys);
        }
    }
    if (p.ymax) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (col + q < p.N) vmax = fmaxf(vmax, fabsf(o[q]));
    }
}

// The same for 16x16 accumulator tiles (v_mfma_f32_16x16x32_bf16 C layout:
// col = lane&15, row = 4(lane>>4) + r), staged through LDS: the wave writes
// 16 rows of its tile at a time into `stage` (16 x (16*TN + 4) floats, its
// own region) and reads them back row-contiguous, so every global access is
// 16 bytes per lane (C, the split-K slab, beta*C and the gradient mask) and
// the row -> pixel map (`rowmap(rbase + local row)` -> RowPix) is evaluated
// once per row per lane.
template <int MODE, int TM, int TN, class RowMap>
__device__ __forceinline__ void conv_epilogue16(const GemmArgs &p, f32x4 (&acc)[TM][TN], int rbase, int cbase,
                                                RowMap rowmap, int phase, int split, int lane, float *stage,
                                                float ys_pre = 0.f, float *vacc = nullptr) {
    // (vacc != NULL: max |output| folded into *vacc -- a persistent block's later atomic -- instead)
    // (ys_pre > 0: the output planes' scale, computed by the caller from loads issued at entry)
    constexpr int WTN = 16 * TN;
    constexpr int LD = WTN + 4;   // padded staging row (floats): conflict-free writes
    constexpr int C4 = WTN / 4;   // float4 per row
    constexpr int RPP = 64 / C4;  // rows per pass of the wave
    static_assert(64 % C4 == 0 && 16 % RPP == 0, "wave tile width");
    const EpiCtx e = epi_ctx(p, ys_pre);
    const int c4 = lane % C4;
    const int col = cbase + c4 * 4;
    float vmax = 0.f;   // max |output| of this lane (p.ymax)
    // accumulator row block a into the stage: compile-time indices into acc in each case of a
    // switch, so the row-block loop itself need not unroll (one epi_out4 body per epilogue)
    auto stage_rows = [&](auto A) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                stage[(4 * (lane >> 4) + r) * LD + b * 16 + (lane & 15)] = acc[decltype(A)::value][b][r];
    };
#ifdef DG_EPI_UNROLL_ROWS
#pragma clang loop unroll(full)
#else
#pragma clang loop unroll(disable)
#endif
    for (int a = 0; a < TM; ++a) {
        static_assert(TM <= 4, "row blocks");
        switch (a) {
        case 0: stage_rows(std::integral_constant<int, 0>{}); break;
        case 1: if constexpr (TM > 1) stage_rows(std::integral_constant<int, (TM > 1 ? 1 : 0)>{}); break;
        case 2: if constexpr (TM > 2) stage_rows(std::integral_constant<int, (TM > 2 ? 2 : 0)>{}); break;
        default: if constexpr (TM > 3) stage_rows(std::integral_constant<int, (TM > 3 ? 3 : 0)>{}); break;
        }
        // (the passes read the staged rows back from LDS, so they need no unrolling: one pass body
        // per accumulator row block keeps the epilogue's code -- inlined once or twice per kernel,
        // executed once per tile -- a quarter of the fully unrolled form's, which ran to ~100 KB of the
        // 250 KB fp16x3 halo kernels against a 64 KB instruction cache.  DG_EPI_UNROLL_PASSES: the
        // unrolled form, for same-box A/B)
#ifdef DG_EPI_UNROLL_PASSES
#pragma clang loop unroll(full)
#else
#pragma clang loop unroll(disable)
#endif
        for (int pass = 0; pass < 16 / RPP; ++pass) {
            const int rl = pass * RPP + lane / C4;
            const f32x4 v = *reinterpret_cast<const f32x4 *>(stage + rl * LD + c4 * 4);
            epi_out4(p, e, rowmap(rbase + a * 16 + rl), col, v, phase, split, vmax);
        }
    }
    if (p.ymax) {
        if (vacc) *vacc = fmaxf(*vacc, vmax);
        else block_atomic_absmax(p.ymax, vmax);
    }
}

// The fp32 kernel's epilogue (k_conv_gemm: 32x32 accumulator tiles, MFMA C layout col = lane&31,
// row = (r&3) + 8(r>>2) + 4(lane>>5)) staged through LDS the same way: a wave writes one 32x32
// tile into `stage` (32 x 36 floats, its own region) and reads it back as 8 float4 per row, 8 rows
// per pass of the wave (epi_out4).  Round 5 wrote each of the TM x TN x 16 accumulators with its own
// runtime-branched store -- a fully unrolled epilogue of up to ~150 KB of code in a ~200 KB kernel.
template <int MODE, int TM, int TN, class RowMap>
__device__ __forceinline__ void conv_epilogue32(const GemmArgs &p, f32x16 (&acc)[TM][TN], int rbase, int cbase,
                                                RowMap rowmap, int phase, int split, int lane, float *stage) {
    constexpr int LD = 36;
    const EpiCtx e = epi_ctx(p, 0.f);
    const int l32 = lane & 31, h2 = lane >> 5, c4 = lane & 7;
    float vmax = 0.f;
#pragma clang loop unroll(full)
    for (int a = 0; a < TM; ++a) {
#pragma clang loop unroll(full)
        for (int b = 0; b < TN; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h2) * LD + l32] = acc[a][b][r];
#pragma clang loop unroll(disable)
            for (int pass = 0; pass < 4; ++pass) {
                const int rl = pass * 8 + (lane >> 3);
                const f32x4 v = *reinterpret_cast<const f32x4 *>(stage + rl * LD + c4 * 4);
                epi_out4(p, e, rowmap(rbase + a * 32 + rl), cbase + b * 32 + c4 * 4, v, phase, split, vmax);
            }
        }
    }
    if (p.ymax) block_atomic_absmax(p.ymax, vmax);
}

// launcher of the bf16x6 kernels (conv_x6.hip); cfg indexes kX6Cfgs
void launch_gemm_x6(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s);
// the halo-tiled bf16x6 kernel (conv_x6h.hip): kt 3 = stride-1 3x3 FWD / DGRAD, kt 2 = the
// sub-pixel phases of a stride-2 4x4 DGRAD (grid y = phase * splits + split); bn = 64 | 128.
// ni 3 bf16x6, 2 fp16 (DG_MATH_FP16), 4 fp16x3 (kt 3, bn 64 | 128; kt 2 phases; kt 4 stride-1 4x4
// forward / input gradient, bn 64).
// a.pidx != NULL selects the fused max-pool epilogue (FWD, one split, output Ho % 8 == 0, Wo % 16 == 0)
// ph 16: the 16 x 16 patch on 8 waves (fp16x3 kt 3, bn 64 | 128)
void launch_gemm_x6h(int mode, int bn, int kt, dim3 grid, const GemmArgs &a, int tiles_x, int tiles_y, hipStream_t s,
                     int ni = 3, int ph = 8);
// fp32 [rows][ld] (first C columns, C % 8 == 0) -> bf16 hi/mid/lo planes [rows][C]
void launch_split3(const float *src, int ld, long rows, int C, unsigned short *dst, hipStream_t s);
// fp32 [rows][ld] -> fp16x3 planes (common.h): per group of G columns (32: activations,
// 16: weights) h[G] l[G] of scale * value; C % G == 0
// (sm != NULL: a bound-scaled operand, scale = x3_grad_scale(sm, sg, sc) instead of `scale`)
void launch_split_x3(const float *src, int ld, long rows, int C, void *dst, int group, float scale, hipStream_t s,
                     const float *sm = nullptr, const float *sg = nullptr, const float *sc = nullptr);
// max |x| of [rows][ld] (first C columns) into *out by atomicMax (zeroed by the caller)
void launch_absmax(const float *x, long rows, int C, int ld, float *out, hipStream_t s);
// max over columns of sum_k |w[k][co]| into gout[0], max |bias| into cout[0] (dg_weight_bound)
void launch_weight_bound(const float *w, long K, int Co, const float *bias, float *gout, float *cout, hipStream_t s,
                         float *zero8 = nullptr);
// max over input channels of sum over taps and output channels of |w[tap][ci][co]| into gout[0]
// (dg_weight_bound_in)
void launch_weight_bound_in(const float *w, int taps, int Ci, int Co, float *gout, hipStream_t s);
// the fp16 conv math (DG_MATH_FP16): one fp16 plane [rows][C] and its GEMM (kF16Cfgs)
void launch_split_f16(const float *src, int ld, long rows, int C, void *dst, hipStream_t s);
void launch_split_f16_pair(const float *a, int lda, long ra, int ca, void *da, const float *b, int ldb, long rb,
                           int cb, void *db, hipStream_t s);
void launch_gemm_f16(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s);
// fp16x3 (DG_MATH_F16X3) generic GEMM: kX3Cfgs tiles, NI = 4 images per K-tile of 32
void launch_gemm_x3(int mode, int cfg, dim3 grid, const GemmArgs &a, hipStream_t s);
// small-Cin 4x4 stride-2 FWD / WGRAD on fp32 MFMA (conv_small.hip)
bool small_conv_ok(const ConvGeom &g, int mode, int lda);
int small_wgrad_rows_per_block(const ConvGeom &g);
void launch_small_conv(int mode, const GemmArgs &a, int rows_per_block, hipStream_t s);

// single-output-channel FWD / DGRAD / WGRAD direct kernels (conv_co1.hip)
bool co1_ok(const ConvGeom &g, int mode);
int co1_wgrad_blocks(const ConvGeom &g);
void launch_co1(int mode, const GemmArgs &a, hipStream_t s);
// Conv2DTranspose(3) forward, 4x4 stride 2, conv-view Co 128: fused MFMA + col2im (conv_tlast.hip)
bool tlast_ok(const ConvGeom &g);
void launch_tlast_fwd(const GemmArgs &a, hipStream_t s);

}  // namespace dg
