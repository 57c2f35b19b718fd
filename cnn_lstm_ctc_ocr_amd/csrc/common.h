// Shared device/host helpers for libocrk (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <mutex>
#include "ocrk.h"

typedef __bf16 bf16;

namespace ocrk {

// Thread-local last error message (read through ocrk_last_error()).
void set_error(const char* fmt, ...);
// Turn a pending hipGetLastError() into an ocrk status (+ message).
int launch_status(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Launch configuration that depends on the device -- kernel attributes set
// with hipFuncSetAttribute, CU counts, occupancy -- is cached PER DEVICE and
// set up thread-safely: one process may drive several GPUs, one thread each
// ("a per-device kernel-module cache (thread-safe)").
constexpr int kMaxDevices = 64;
constexpr int kMaxCuWords = 32;                       // CU-mask words (1024 CUs)
inline int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d < 0 ? 0 : (d >= kMaxDevices ? kMaxDevices - 1 : d);
}
struct DeviceOnce {
    std::once_flag f[kMaxDevices];
};
template <typename Fn>
inline void once_per_device(DeviceOnce& o, Fn&& fn) {
    std::call_once(o.f[current_device()], fn);
}
// CUs of the current device.
inline int cu_count() {
    static DeviceOnce o;
    static int n[kMaxDevices];
    const int d = current_device();
    std::call_once(o.f[d], [d] {
        int v = 0;
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d);
        n[d] = v > 0 ? v : 256;
    });
    return n[d];
}
// Raise a kernel's dynamic-LDS limit to `bytes`, once per device (call with a
// function-local `static DeviceOnce`, one per kernel instantiation).
inline void set_dyn_lds(DeviceOnce& o, const void* kern, int bytes) {
    once_per_device(o, [kern, bytes] {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    });
}

// Engine options (route and schedule switches kept for A/B measurement and for
// the parity tests of alternative routes). Each starts from its OCRK_<NAME>
// environment variable, read ONCE for the process (the first opt() call);
// afterwards only ocrk_set_option changes it. A lookup is one relaxed atomic
// load: no getenv on a launch path.
enum Option : int {
    OPT_CONV_DIRECT = 0,      // 0 implicit GEMM only, 1 (default) the Cin 32 shapes, 2 every covered shape
    OPT_CONV_ROWS,            // 1 (default) row-walking conv kernels, 0 the chunked direct / TN engines
    OPT_CONV_ROWS_WIDE,       // 1 (default) conv3-conv6 on the row kernels too, 0 GEMM / direct engines
    OPT_CONV_WGRAD_BLOCKS,    // 1 (default) conv5/6 weight gradients as channel blocks, 2 conv7/8 too, 0 TN
    OPT_LSTM_SPIN_LIMIT,      // polls before a persistent hand-off wait gives up (<= 0: 1 << 22)
    OPT_PERSIST_LATE,         // 1 (default) late epilogue loads behind the staging DMA, 0 at the step top
    OPT_LSTM_BWD_KSPLIT,      // 1: the K-split persistent BPTT (opt-in)
    OPT_LSTM_BWD_PB16,        // 1: K-split partial products exchanged in bf16
    OPT_LSTM_BWD_R16,         // 1 (default) 16-row / 64-unit BPTT members at H = 512, 0 the 32-row gather
    OPT_CTC_LDS,              // 1 (default) CTC lattices in LDS when they fit, 0 in the global workspace
    OPT_PP_PERSIST_NK,        // ping-pong GEMM: persistent workgroups when K-tiles per item <= this (8)
    OPT_PP_DEEP,              // 1: the deep-lead ping-pong schedule for the plain (A_ROWK) GEMMs
    OPT_NT_F32_EXACT,         // 1 (default): exact-mode fp32 convolutions on the NT ring (0: generic engine)
    OPT_NT_F32_MASK,          // 1 (default): the masked fp32 data gradients on the NT ring too (0: generic engine)
    OPT_NT_F32_X6,            // 1: exact-mode NT convolutions as six bf16 products (fp32-precision split; opt-in)
    OPT_BEAM_WAVE,            // 1 (default): the one-wave beam search for K <= 16, 0 the block kernel
    OPT_BN_BWD_BLOCKS,        // BN backward pass-1 workgroup cap (2048; 64 .. 8192)
    OPT_BN_ROUTE,             // 1 (default): window-walk BN backward for the non-overlapping pools
    OPT_BN_ROUTE_SEG,         // pooled columns per thread of the window walk (8; 4, 8 or 16)
    OPT_BN_ROUTE_NCH,         // channels per thread of the window walk (4; or 8)
    OPT_CONV_TN_ITEMS,        // workgroup cap of the conv weight-gradient TN launches beside the backward (192)
    OPT_CONV_TN4_ITEMS,       // split-K target items of the 4-wave TN conv weight gradients (512)
    OPT_CONV_WGRAD_CUS,       // CUs the channel-block conv weight gradients take (192; 0 = every CU)
    OPT_F32_MFMA,             // 1: exact f32 products for every fp32 GEMM of the process (else per ocrk_set_f32_gemm_mode)
    OPT_GEMM_NT,              // 1 (default): the NT LDS-DMA ring, 0 the generic engine only
    OPT_GEMM_NT_STAGED,       // 1 (default): the NT ring's LDS-staged bf16 epilogue, 0 direct 2-B stores
    OPT_GEMM_PP,              // 1 (default): the ping-pong NT engine for the large plain GEMMs
    OPT_GEMM_PPTN,            // 1 (default): the ping-pong TN engine for the wide weight gradients
    OPT_PP_MIN_N,             // narrowest plain GEMM (N) on the ping-pong engine (512)
    OPT_GEMM_TN,              // 1 (default): the 4-wave TN engine, 0 the generic engine
    OPT_LSTM_DMA,             // 1 (default): LDS-DMA staging in the per-step LSTM forward kernels
    OPT_LSTM_BWD_DMA,         // 1 (default): LDS-DMA staging in the per-step LSTM backward kernels
    OPT_LSTM_FWD_R16,         // 1 (default): 16-row / 64-unit members for the bf16 forward loop at H = 512
    OPT_NT_TAP_UNIFORM,       // 1 (default): the NT ring's tap-uniform im2col addressing where C % BK == 0
    OPT_COUNT
};
int64_t opt(Option o);

}  // namespace ocrk

#define OCRK_REQUIRE(cond, ...)                       \
    do {                                                \
        if (!(cond)) {                                  \
            ocrk::set_error(__VA_ARGS__);               \
            return OCRK_ERR_INVALID_ARG;                \
        }                                               \
    } while (0)

// ---------------------------------------------------------------- device math
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// 8 consecutive elements as fp32 (16-B / 32-B vector access).
struct F8 { float v[8]; };

template <typename T> __device__ __forceinline__ F8 load8(const T* p);
template <> __device__ __forceinline__ F8 load8<float>(const float* p) {
    F8 r;
    float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
}
template <> __device__ __forceinline__ F8 load8<bf16>(const bf16* p) {
    union { uint4 q; bf16 e[8]; } u;
    u.q = *reinterpret_cast<const uint4*>(p);
    F8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (float)u.e[i];
    return r;
}
// The raw bytes of 8 elements, converted to fp32 only at use (cvt8): a prefetch
// kept raw does not make the compiler wait for its load where it is issued (a
// load8 converts at once, so its wait lands right behind the load).
template <typename T> struct Pend8;
template <> struct Pend8<float> { float4 a, b; };
template <> struct Pend8<bf16> { uint4 q; };
template <typename T> __device__ __forceinline__ Pend8<T> load_pend8(const T* p);
template <> __device__ __forceinline__ Pend8<float> load_pend8<float>(const float* p) {
    return Pend8<float>{reinterpret_cast<const float4*>(p)[0], reinterpret_cast<const float4*>(p)[1]};
}
template <> __device__ __forceinline__ Pend8<bf16> load_pend8<bf16>(const bf16* p) {
    return Pend8<bf16>{*reinterpret_cast<const uint4*>(p)};
}
__device__ __forceinline__ F8 cvt8(const Pend8<float>& r) {
    return F8{{r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w}};
}
__device__ __forceinline__ F8 cvt8(const Pend8<bf16>& r) {
    union { uint4 q; bf16 e[8]; } u;
    u.q = r.q;
    F8 f;
#pragma unroll
    for (int i = 0; i < 8; ++i) f.v[i] = (float)u.e[i];
    return f;
}

template <typename T> __device__ __forceinline__ void store8(T* p, const F8& x);
template <> __device__ __forceinline__ void store8<float>(float* p, const F8& x) {
    reinterpret_cast<float4*>(p)[0] = make_float4(x.v[0], x.v[1], x.v[2], x.v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(x.v[4], x.v[5], x.v[6], x.v[7]);
}
template <> __device__ __forceinline__ void store8<bf16>(bf16* p, const F8& x) {
    union { uint4 q; bf16 e[8]; } u;
#pragma unroll
    for (int i = 0; i < 8; ++i) u.e[i] = (bf16)x.v[i];
    *reinterpret_cast<uint4*>(p) = u.q;
}

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at bits 15:14;
// expcnt and lgkmcnt left at their maxima). Counted waits let LDS-DMA stages
// land one at a time while later stages stay in flight.
template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | (7 << 4) | (15 << 8));
}

// A lane's value combined with its partner lane l ^ 16 / l ^ 32 without the LDS crossbar
// (__shfl_xor is a ds_bpermute): gfx950's v_permlane16_swap / v_permlane32_swap with both
// operands v return, per lane, v of the lane and of its partner (in either order; + and | are
// commutative, so the bits equal the shuffle forms').
__device__ __forceinline__ unsigned or_xor16(unsigned v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return r[0] | r[1];
}
__device__ __forceinline__ unsigned or_xor32(unsigned v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r[0] | r[1];
}
__device__ __forceinline__ float add_xor16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// 64-lane wave reductions.
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The same through DPP: row_ror 8/4/2/1 gives every lane its 16-lane row's
// result (no LDS crossbar round trips), the four rows are then combined from
// v_readlane in a fixed order -- ~4x fewer cycles on a serial chain than the
// ds_bpermute butterfly above (different summation order).
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_of(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    v = fmaxf(v, dpp_row<0x128>(v));
    v = fmaxf(v, dpp_row<0x124>(v));
    v = fmaxf(v, dpp_row<0x122>(v));
    v = fmaxf(v, dpp_row<0x121>(v));
    return fmaxf(fmaxf(lane_of(v, 0), lane_of(v, 16)), fmaxf(lane_of(v, 32), lane_of(v, 48)));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_row<0x128>(v);
    v += dpp_row<0x124>(v);
    v += dpp_row<0x122>(v);
    v += dpp_row<0x121>(v);
    return (lane_of(v, 0) + lane_of(v, 16)) + (lane_of(v, 32) + lane_of(v, 48));
}
