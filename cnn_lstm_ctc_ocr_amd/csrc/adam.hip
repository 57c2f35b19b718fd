// a13: the train op's Adam update (src/weinman/train.py:128-137 AdamOptimizer
// + optimize_loss; [TF1] ApplyAdam) over the flat fp32 parameter buffer:
//   m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2); p -= lr_t m / (sqrt(v) + eps)
// with lr_t = lr sqrt(1 - b2^t) / (1 - b1^t) precomputed by the caller.
// One pass, 16 B per lane per stream: HBM-bound (4 reads + 3 writes of fp32).
// ZERO (ocrk_adam_ex, OCRK_ADAM_ZERO_GRAD): the gradient is cleared as it is
// read -- the next step's zero_grad pass (a separate 4-byte-per-parameter
// fill at the top of the step) folded into this one (+1 write stream).
#include "common.h"

template <bool ZERO>
__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
            int64_t n, float lr_t, float b1, float b2, float eps, float grad_scale) {
    const int64_t n4 = n / 4;
    const float c1 = 1.f - b1, c2 = 1.f - b2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 pp = reinterpret_cast<float4*>(p)[i], gg = reinterpret_cast<const float4*>(g)[i];
        float4 mm = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
        float* pe = &pp.x; float* ge = &gg.x; float* me = &mm.x; float* ve = &vv.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float gk = ge[k] * grad_scale;
            me[k] += (gk - me[k]) * c1;
            ve[k] += (gk * gk - ve[k]) * c2;
            pe[k] -= lr_t * me[k] / (sqrtf(ve[k]) + eps);
        }
        reinterpret_cast<float4*>(p)[i] = pp;
        reinterpret_cast<float4*>(m)[i] = mm;
        reinterpret_cast<float4*>(v)[i] = vv;
        if constexpr (ZERO) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float gk = g[i] * grad_scale;
        m[i] += (gk - m[i]) * c1;
        v[i] += (gk * gk - v[i]) * c2;
        p[i] -= lr_t * m[i] / (sqrtf(v[i]) + eps);
        if constexpr (ZERO) g[i] = 0.f;
    }
}

extern "C" int ocrk_adam_ex(float* p, float* g, float* m, float* v, int64_t n, float lr_t, float beta1,
                            float beta2, float eps, float grad_scale, unsigned flags, void* stream) {
    if (n == 0) return OCRK_OK;
    OCRK_REQUIRE(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0, "ocrk_adam: buffers must be 16-B aligned");
    OCRK_REQUIRE((flags & ~(unsigned)OCRK_ADAM_ZERO_GRAD) == 0, "ocrk_adam_ex: unknown flags 0x%x", flags);
    unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ocrk::cdiv(n / 4 + 1, 256), 4096));
    hipStream_t s = ocrk::as_stream(stream);
    if (flags & OCRK_ADAM_ZERO_GRAD)
        adam_kernel<true><<<grid, 256, 0, s>>>(p, g, m, v, n, lr_t, beta1, beta2, eps, grad_scale);
    else
        adam_kernel<false><<<grid, 256, 0, s>>>(p, g, m, v, n, lr_t, beta1, beta2, eps, grad_scale);
    return ocrk::launch_status("ocrk_adam");
}

extern "C" int ocrk_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr_t, float beta1,
                         float beta2, float eps, float grad_scale, void* stream) {
    return ocrk_adam_ex(p, const_cast<float*>(g), m, v, n, lr_t, beta1, beta2, eps, grad_scale, 0u, stream);
}
