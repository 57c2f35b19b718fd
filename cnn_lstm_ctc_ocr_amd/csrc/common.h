// Shared device/host helpers for libocrk (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include "ocrk.h"

typedef __bf16 bf16;

namespace ocrk {

// Thread-local last error message (read through ocrk_last_error()).
void set_error(const char* fmt, ...);
// Turn a pending hipGetLastError() into an ocrk status (+ message).
int launch_status(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace ocrk

#define OCRK_REQUIRE(cond, ...)                         \
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
