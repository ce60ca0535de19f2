// The generator's last layer, Conv2DTranspose(3, 4, strides=2, 'same') + tanh
// (pix2pix.py:169-173), forward.  In the conv view it is the input gradient
// (DGRAD) of a 4x4 stride-2 conv with Ci = 3 and Co = 128:
//   out[n,h,w,c] = sum over the 2x2 taps (i,j) that reach (h,w) of
//                  sum_co x[n,ho,wo,co] W[i,j,c,co],  ho = (h+pt-i)/2, wo = (w+pl-j)/2
// As a GEMM its N is 3, so the planner used to recast it: a 1x1 GEMM
// V = x . W^T (N = 48 = 16 taps x 3 channels) into a 100 MB workspace at bs16,
// then a col2im pass re-reading V (0.215 ms per step).  This kernel does both
// in one block: per 16 x 32 output tile it forms V for the 10 x 18 input
// pixels the tile reaches on the fp32 matrix cores (v_mfma_f32_16x16x4_f32,
// exact fp32 products), keeps V in LDS and shift-adds it into the tile with
// bias and activation.  x is read once per tile (1.4x halo overlap, L2 hits),
// V never leaves the CU.
//
// Operand layout of the MFMA (16x16x4 f32): A lane l holds A[l%16][k = l/16],
// B lane l holds B[k = l/16][l%16].  The K slots are permuted so that each
// lane loads 16 bytes: for channel group kg (16 channels) lane slot s holds
// channels kg*16 + 4s .. +3, and K-step t of the group uses element t of that
// float4 for both operands (slot s <-> channel kg*16 + 4s + t).
#include "conv_impl.h"
#include <algorithm>

namespace dg {

constexpr int TL_TH = 16, TL_TW = 32;          // output tile (conv-view input pixels)
constexpr int TL_RI = TL_TH / 2 + 2;           // input rows a tile reaches (k4 s2): 10
constexpr int TL_CW = TL_TW / 2 + 2;           // input columns: 18
constexpr int TL_P = TL_RI * TL_CW;            // 180 input pixels
constexpr int TL_MT = (TL_P + 15) / 16;        // 12 M-tiles of 16 pixels
constexpr int TL_CO = 128;                     // conv-view Co = the GEMM K
constexpr int TL_KG = TL_CO / 16;              // channel groups of 16
constexpr int TL_VS = 49;                      // V row stride (floats, odd: conflict-free)

bool tlast_ok(const ConvGeom &g) {
    return g.kh == 4 && g.kw == 4 && g.sh == 2 && g.sw == 2 && g.Ci == 3 && g.Co == TL_CO;
}

// persistent: each block walks tiles blockIdx.x, + gridDim.x, ...; the filter
// fragments are loaded once per wave, and each wave's first x loads of the
// next tile are in flight under the current tile's col2im
template <int CI>
__global__ void __launch_bounds__(256, 2)
k_tlast_fwd(const GemmArgs p, int tiles_x, int tiles_y) {
    constexpr int NT = CI;                     // N-tiles: 16*CI V columns (tap, channel)
    constexpr int MW = TL_MT / 4;              // M-tiles per wave
    __shared__ float Vs[TL_MT * 16 * TL_VS];
    const ConvGeom &g = p.g;
    const int ntiles = g.N * tiles_x * tiles_y;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int l16 = lane & 15, s = lane >> 4;
    // B: every (N-tile, channel group) float4 of this lane
    f32x4 b[NT][TL_KG];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int kg = 0; kg < TL_KG; ++kg)
            b[nt][kg] = *reinterpret_cast<const f32x4 *>(p.B + (long)(nt * 16 + l16) * TL_CO + kg * 16 + 4 * s);
    struct Tile {
        int n, H0, W0, ho_lo, wo_lo;
    };
    auto tile_of = [&](int t) __attribute__((always_inline)) {
        Tile q;
        const int tx = t % tiles_x;
        t /= tiles_x;
        const int ty = t % tiles_y;
        q.n = t / tiles_y;
        q.H0 = ty * TL_TH;
        q.W0 = tx * TL_TW;
        // input rows ho >= ceil((H0 + pt - 3) / 2): arithmetic shifts floor negative values
        q.ho_lo = (q.H0 + g.pt - 2) >> 1;
        q.wo_lo = (q.W0 + g.pl - 2) >> 1;
        return q;
    };
    auto load_a = [&](const Tile &q, int mt, f32x4 (&a)[TL_KG]) __attribute__((always_inline)) {
        const int m = mt * 16 + l16;
        const int r = m / TL_CW, c = m - r * TL_CW;
        const int ho = q.ho_lo + r, wo = q.wo_lo + c;
        const bool ok = m < TL_P && (unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo;
        const float *src = p.A + ((long)(q.n * g.Ho + (ok ? ho : 0)) * g.Wo + (ok ? wo : 0)) * p.lda + 4 * s;
#pragma unroll
        for (int kg = 0; kg < TL_KG; ++kg)
            a[kg] = ok ? *reinterpret_cast<const f32x4 *>(src + kg * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    int t = blockIdx.x;
    if (t >= ntiles) return;
    Tile cur = tile_of(t);
    f32x4 an[TL_KG];
    load_a(cur, wid, an);
    for (; t < ntiles; t += gridDim.x) {
        const int tn = t + gridDim.x;
        const Tile nxt = tile_of(tn < ntiles ? tn : t);
#pragma unroll
        for (int k = 0; k < MW; ++k) {
            const int mt = wid + 4 * k;
            f32x4 a[TL_KG];
#pragma unroll
            for (int kg = 0; kg < TL_KG; ++kg) a[kg] = an[kg];
            if (k + 1 < MW) load_a(cur, mt + 4, an);
            else if (tn < ntiles) load_a(nxt, wid, an);
            f32x4 acc[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kg = 0; kg < TL_KG; ++kg)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kg][e], b[nt][kg][e], acc[nt], 0, 0, 0);
            // D layout: lane holds rows 4*(lane/16) + r, column lane%16
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) Vs[(mt * 16 + 4 * s + r) * TL_VS + nt * 16 + l16] = acc[nt][r];
        }
        __syncthreads();
        // col2im: output pixel (h, w) sums its 2x2 taps in (i, j) order
        for (int q = threadIdx.x; q < TL_TH * TL_TW; q += 256) {
            const int h = cur.H0 + q / TL_TW, w = cur.W0 + q % TL_TW;
            if (h >= g.H || w >= g.W) continue;
            const int i0 = (h + g.pt) & 1, j0 = (w + g.pl) & 1;
            float v[CI];
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) v[ci] = 0.f;
#pragma unroll
            for (int ai = 0; ai < 2; ++ai) {
                const int i = i0 + 2 * ai;
                const int r = ((h + g.pt - i) >> 1) - cur.ho_lo;
#pragma unroll
                for (int bj = 0; bj < 2; ++bj) {
                    const int j = j0 + 2 * bj;
                    const int c = ((w + g.pl - j) >> 1) - cur.wo_lo;
                    const float *vp = Vs + (r * TL_CW + c) * TL_VS + (i * 4 + j) * CI;
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) v[ci] += vp[ci];
                }
            }
            const long pix = (long)(cur.n * g.H + h) * g.W + w;
            float *dst = p.C + pix * p.ldc;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) {
                float o = v[ci];
                if (p.bias) o += p.bias[ci];
                o = act_fwd(o, p.act, p.alpha);
                if (p.beta != 0.f) o += p.beta * dst[ci];
                dst[ci] = o;
            }
        }
        __syncthreads();   // V is rewritten by the next tile
        cur = nxt;
    }
}

void launch_tlast_fwd(const GemmArgs &a, hipStream_t s) {
    const ConvGeom &g = a.g;
    const int tx = (g.W + TL_TW - 1) / TL_TW, ty = (g.H + TL_TH - 1) / TL_TH;
    // two resident blocks per CU (212 VGPRs); 256 CUs
    const int grid = std::min(g.N * tx * ty, 512);
    hipLaunchKernelGGL(k_tlast_fwd<3>, dim3((unsigned)grid), dim3(256), 0, s, a, tx, ty);
}

}  // namespace dg
