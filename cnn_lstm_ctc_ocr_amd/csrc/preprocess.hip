// a1: image preprocess, uint8 -> float in [-0.5, 0.5].
// Mirrors validate._preprocess_image (src/weinman/validate.py:56-68) and the
// TF1 convert_image_dtype(uint8->f32) it calls: cast, multiply by
// float32(1/255), then subtract 0.5 -- two separately rounded ops (no FMA).
#include "common.h"

__device__ __forceinline__ float preprocess_px(uint8_t v) {
#pragma clang fp contract(off)
    return (float)v * (1.0f / 255.0f) - 0.5f;
}

template <typename T>
__global__ void __launch_bounds__(256) preprocess_kernel(const uint8_t* __restrict__ in,
                                                         T* __restrict__ out, int64_t n) {
    int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 3 < n) {
        uchar4 v = *reinterpret_cast<const uchar4*>(in + i);
        out[i + 0] = from_f32<T>(preprocess_px(v.x));
        out[i + 1] = from_f32<T>(preprocess_px(v.y));
        out[i + 2] = from_f32<T>(preprocess_px(v.z));
        out[i + 3] = from_f32<T>(preprocess_px(v.w));
    } else {
        for (; i < n; ++i) out[i] = from_f32<T>(preprocess_px(in[i]));
    }
}

extern "C" int ocrk_preprocess(const uint8_t* in, int64_t n, void* out, int dtype, void* stream) {
    OCRK_REQUIRE(n >= 0 && (n == 0 || (in && out)), "ocrk_preprocess: bad arguments");
    OCRK_REQUIRE((reinterpret_cast<uintptr_t>(in) & 3) == 0, "ocrk_preprocess: input not 4-byte aligned");
    if (n == 0) return OCRK_OK;
    dim3 grid((unsigned)ocrk::cdiv(n, 1024));
    if (dtype == OCRK_F32)
        preprocess_kernel<float><<<grid, 256, 0, ocrk::as_stream(stream)>>>(in, (float*)out, n);
    else if (dtype == OCRK_BF16)
        preprocess_kernel<bf16><<<grid, 256, 0, ocrk::as_stream(stream)>>>(in, (bf16*)out, n);
    else
        OCRK_REQUIRE(false, "ocrk_preprocess: unsupported dtype %d", dtype);
    return ocrk::launch_status("ocrk_preprocess");
}
