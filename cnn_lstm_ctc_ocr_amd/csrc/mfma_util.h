// Register/LDS staging helpers shared by the MFMA kernels (gemm.hip, lstm.hip).
#pragma once
#include "common.h"

namespace ocrk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 8 consecutive elements of the compute type held in registers. Plain
// ext-vector members (no unions, no struct copies from memory): loads become
// vector loads and SROA keeps every staging set in VGPRs.
template <typename CT> struct V8;
template <> struct V8<bf16> {
    u32x4 q;
    __device__ __forceinline__ unsigned short e(int i) const {
        return (unsigned short)(q[i >> 1] >> (16 * (i & 1)));
    }
};
template <> struct V8<float> {
    f32x4 q0, q1;
    __device__ __forceinline__ float e(int i) const { return i < 4 ? q0[i] : q1[i - 4]; }
};
template <typename CT> struct RawT;
template <> struct RawT<bf16> { using T = unsigned short; };
template <> struct RawT<float> { using T = float; };

__device__ __forceinline__ void vzero(V8<bf16>& x) { x.q = u32x4{0u, 0u, 0u, 0u}; }
__device__ __forceinline__ void vzero(V8<float>& x) { x.q0 = x.q1 = f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ void vload(V8<bf16>& x, const bf16* p) { x.q = *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void vload(V8<float>& x, const float* p) {
    x.q0 = reinterpret_cast<const f32x4*>(p)[0];
    x.q1 = reinterpret_cast<const f32x4*>(p)[1];
}
__device__ __forceinline__ void vload_lds(V8<bf16>& x, const unsigned short* p) { x.q = *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void vload_lds(V8<float>& x, const float* p) {
    x.q0 = reinterpret_cast<const f32x4*>(p)[0];
    x.q1 = reinterpret_cast<const f32x4*>(p)[1];
}
__device__ __forceinline__ void vstore_lds(unsigned short* d, const V8<bf16>& x) { *reinterpret_cast<u32x4*>(d) = x.q; }
__device__ __forceinline__ void vstore_lds(float* d, const V8<float>& x) {
    reinterpret_cast<f32x4*>(d)[0] = x.q0;
    reinterpret_cast<f32x4*>(d)[1] = x.q1;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// bf16 MFMA fragment from a row-contiguous [k][row] LDS image: two
// ds_read_b64_tr_b16, the second `second` elements (16 k-rows) further on.
__device__ __forceinline__ bf16x8 frag_tr(const unsigned short* p, int second) {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + second));
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}
// the same permuted k order from a k-contiguous row: k = 4g..4g+3 and 16+4g..16+4g+3
__device__ __forceinline__ bf16x8 frag_perm(const unsigned short* row, int g) {
    s16x4 lo = *reinterpret_cast<const s16x4*>(row + 4 * g);
    s16x4 hi = *reinterpret_cast<const s16x4*>(row + 16 + 4 * g);
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

// fp32 operands on the bf16 MFMA ("bf16x3"): x = hi + lo with hi = bf16(x) and
// lo = bf16(x - hi) (both round-to-nearest-even), so |x - hi - lo| <= 2^-17 |x|
// (2^-9 from hi, times 2^-8 from lo); a product a.b is taken as
// ah.bh + ah.bl + al.bh (the dropped al.bl is <= 2^-18 |a.b|) with f32
// accumulation: ~2^-16 relative per product, against fp32's 2^-24 -- 3
// v_mfma_f32_16x16x32_bf16 (16 cycles each, 2.5 PF dense) instead of the f32
// MFMA (v_mfma_f32_16x16x4_f32, 157 TF): 5.3x the rate per product.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2_bf16(float x0, float x1, unsigned& hi, unsigned& lo) {
    const bf16x2_t h = __builtin_convertvector(f32x2_t{x0, x1}, bf16x2_t);
    const f32x2_t hf = __builtin_convertvector(h, f32x2_t);
    const bf16x2_t l = __builtin_convertvector(f32x2_t{x0 - hf[0], x1 - hf[1]}, bf16x2_t);
    hi = __builtin_bit_cast(unsigned, h);
    lo = __builtin_bit_cast(unsigned, l);
}
__device__ __forceinline__ void split8_bf16(const V8<float>& x, u32x4& hi, u32x4& lo) {
    unsigned h[4], l[4];
    split2_bf16(x.q0[0], x.q0[1], h[0], l[0]);
    split2_bf16(x.q0[2], x.q0[3], h[1], l[1]);
    split2_bf16(x.q1[0], x.q1[1], h[2], l[2]);
    split2_bf16(x.q1[2], x.q1[3], h[3], l[3]);
    hi = u32x4{h[0], h[1], h[2], h[3]};
    lo = u32x4{l[0], l[1], l[2], l[3]};
}
// x = hi + mid + lo exactly (three RNE bf16 roundings of the running residual:
// each residual is exact in fp32, the last one has <= 8 significant bits), for
// products to fp32 precision on the bf16 MFMA: the six terms down to 2^-16
// relative (hh, hm, mh, hl, mm, lh), the dropped ones <= 2^-25.
__device__ __forceinline__ void split3_bf16(float x0, float x1, unsigned& hi, unsigned& mid, unsigned& lo) {
    const bf16x2_t h = __builtin_convertvector(f32x2_t{x0, x1}, bf16x2_t);
    const f32x2_t r = f32x2_t{x0, x1} - __builtin_convertvector(h, f32x2_t);
    const bf16x2_t m = __builtin_convertvector(r, bf16x2_t);
    const bf16x2_t l = __builtin_convertvector(r - __builtin_convertvector(m, f32x2_t), bf16x2_t);
    hi = __builtin_bit_cast(unsigned, h);
    mid = __builtin_bit_cast(unsigned, m);
    lo = __builtin_bit_cast(unsigned, l);
}
__device__ __forceinline__ void split8_bf16x3(const V8<float>& x, u32x4& hi, u32x4& mid, u32x4& lo) {
    unsigned h[4], m[4], l[4];
    split3_bf16(x.q0[0], x.q0[1], h[0], m[0], l[0]);
    split3_bf16(x.q0[2], x.q0[3], h[1], m[1], l[1]);
    split3_bf16(x.q1[0], x.q1[1], h[2], m[2], l[2]);
    split3_bf16(x.q1[2], x.q1[3], h[3], m[3], l[3]);
    hi = u32x4{h[0], h[1], h[2], h[3]};
    mid = u32x4{m[0], m[1], m[2], m[3]};
    lo = u32x4{l[0], l[1], l[2], l[3]};
}

// Buffer resource from provably wave-uniform words (readfirstlane; the byte
// count clamped with integer ops -- HIP's min<int64_t> lowers to v_min_f64, a
// VALU value). A descriptor the compiler cannot prove uniform is kept in VGPRs
// and every buffer op on it is wrapped in a waterfall loop
// (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
    const uint64_t b = (uint64_t)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(bytes > 0x7fffffff ? 0x7fffffff : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// The same descriptor as four SGPR words, for inline-asm buffer operations.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t uniform_rsrc_words(const void* base, int64_t bytes) {
    const uint64_t b = (uint64_t)base;
    const int lo = (int)__builtin_amdgcn_readfirstlane((unsigned)b);
    const int hi = (int)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32) & 0xffffu);   // stride 0
    const int nb = __builtin_amdgcn_readfirstlane(bytes > 0x7fffffff ? 0x7fffffff : (int)bytes);
    return i32x4_t{lo, hi, nb, 0x00020000};
}

// LDS-DMA (buffer_load_dwordx4 ... lds, 16 B per lane, lane-linear at `lds`) as
// inline asm. The compiler's waitcnt pass cannot tell one LDS buffer of a kernel's
// single __shared__ array from another, so after the builtin form it drains every
// pending DMA (s_waitcnt vmcnt(0)) in front of each ds_read -- which defeats a
// schedule that keeps DMAs in flight across phases. Hidden from it, the caller's
// counted vm_wait<N> + barriers are the only ordering (RAW and WAR as the
// schedule states), and the compiler's own vmcnt waits only over-count.
// The LDS address is an operand bound to m0 itself ("{m0}"): the compiler writes
// m0 and knows it is live, so no reserved-register clobber is needed (a clobber
// list naming m0 "may not be preserved"); the s_nop covers the m0 -> LDS-DMA
// hazard, which the compiler cannot see inside the asm.
__device__ __forceinline__ void lds_dma16_asm(const i32x4_t& r, void* lds, unsigned voff) {
    const unsigned a = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :: "v"(voff), "s"(r), "{m0}"(a) : "memory");
}

}  // namespace ocrk
