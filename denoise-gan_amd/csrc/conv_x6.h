// Device helpers shared by the bf16x6 GEMM kernels (conv_x6.hip: the
// implicit GEMM over any conv geometry; conv_x6h.hip: the halo-tiled kernel
// for stride-1 3x3 convs): the bf16 plane split, the LDS plane images and
// their MFMA fragment reads, and the compile-time DMA wait.
#pragma once
#include "conv_impl.h"

namespace dg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// LDS plane images (bf16), read by v_mfma_f32_16x16x32_bf16 fragments whose
// 32-wide K is two 16-wide plane pieces side by side (see the kernel):
//   KC image [rows][16 k], 32-byte rows: lane l of a read takes row l&15 and
//   the 8-k half (l>>4)&1 of plane (l>>5 ? P1 : P0) -- conflict-free as is.
//   RC image [16 k][COLS], read transposed (ds_read_b64_tr_b16): the 8-dword
//   blocks of k-row k are XOR-swizzled by f(k) so the eight k-rows one 32-lane
//   half touches (k and k+8 for 4 consecutive k) land on distinct banks.
// (Both verified exhaustively against the gfx950 bank model for 64/128/256;
// the 32-column images of the 32-wide tiles keep a row-local swap.)
__device__ __forceinline__ int x6_off(int row, int half) { return row * 32 + 16 * half; }

// (a 32-column image has 16 dwords per k-row: only the 0 / 8 swap stays inside it)
__device__ __forceinline__ int x6_rc_swz_cols(int cols, int k) {  // in dwords
    return cols >= 128 ? 8 * ((k & 3) | (((k >> 3) & 1) << 2))
                       : (cols >= 64 ? 8 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) : 8 * ((k >> 1) & 1));
}
template <int COLS>
__device__ __forceinline__ int x6_rc_swz(int k) {  // in dwords
    return x6_rc_swz_cols(COLS, k);
}
// byte offset of bf16 element (k, col) in a [16][COLS] plane image (col even)
template <int COLS>
__device__ __forceinline__ int x6_rc_off(int k, int col) {
    return 4 * (k * (COLS / 2) + ((col >> 1) ^ x6_rc_swz<COLS>(k)));
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16x16x32 operand fragment of an RC image pair: lane l gets column
// c0 + (l&15) at k = 8(l>>4) + 0..7 of the concatenated K, i.e. k-rows
// 8((l>>4)&1) + 0..7 of plane P0 (l < 32) or P1 (l >= 32); two transposed reads
template <int COLS>
__device__ __forceinline__ bf16x8 x6_rc_frag(const char *p0, const char *p1, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const char *pl = g < 2 ? p0 : p1;
    const int col = c0 + 4 * pp, k = 8 * (g & 1) + q;
    lds_s16x4 *a0 = (lds_s16x4 *)(pl + x6_rc_off<COLS>(k, col));
    lds_s16x4 *a1 = (lds_s16x4 *)(pl + x6_rc_off<COLS>(k + 4, col));
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(a1);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// the same from a KC image pair: one 16-byte read per lane
__device__ __forceinline__ bf16x8 x6_kc_frag(const char *p0, const char *p1, int r0, int lane) {
    const int g = lane >> 4;
    return *reinterpret_cast<const bf16x8 *>((g < 2 ? p0 : p1) + x6_off(r0 + (lane & 15), g & 1));
}

// wait until at most N of this wave's DMAs are in flight (compile-time N: no
// runtime switch in the K-tile body)
template <int N>
__device__ __forceinline__ void wait_dma_c() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA of 16 bytes per lane (buffer_load_dwordx4 ... lds: lane L's bytes
// land at M0 + 16 L), issued from inline asm.  Through the compiler builtin
// the wait-count pass cannot tell LDS buffers apart (it would need alias
// scope metadata) and puts an s_waitcnt vmcnt(0) in front of the first
// fragment read of every K-tile, draining the DMAs meant to stay in flight.
// Invisible to it, the DMAs are ordered only by the kernels' own
// wait_dma_c<> + barrier (asm with a memory clobber, so no LDS access moves
// across them); the compiler's own vmcnt waits can only over-wait because of
// them (in-order completion), never under-wait.
typedef rsrc_t rsrc4_t;
__device__ __forceinline__ rsrc4_t make_rsrc4(const void *base, unsigned bytes) {
    // scalar operands: the asm takes the descriptor in SGPRs ("s")
    const unsigned long long a = (unsigned long long)(uintptr_t)base;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
    const unsigned n = (unsigned)__builtin_amdgcn_readfirstlane((int)bytes);
    return make_rsrc((const float *)(uintptr_t)(((unsigned long long)hi << 32) | lo), n);
}
// The asm opens with `s_nop 4`: hipcc pads no hazard into an asm statement
// (cdna_hip_programming.md §5.7 item 2), and two reach this one -- a VALU write of
// a descriptor SGPR (the spill restore `v_readlane_b32 s7, ...` hipcc places
// among the DMAs of these SGPR-spilling kernels) needs 5 wait states before a
// VMEM instruction reads it, and the compiler's `s_mov_b32 m0` one before an
// LDS-DMA.  Without the pad (round 5 and before) a regalloc change put such a
// restore 1-3 instructions ahead of a DMA in k_conv_gemm_x6h<DGRAD, 128, .., 2, 4>
// (G up5 / up6 forward): run-to-run different outputs, one memory-access fault
// (round 6, scripts/diag/determinism.py; profiles/r6/dma_hazard.txt).
__device__ __forceinline__ void dma16(rsrc4_t r, char *lds, unsigned off) {
    const unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char *)lds;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(off), "s"(r), "{m0}"(la) : "memory");
}

}  // namespace dg
