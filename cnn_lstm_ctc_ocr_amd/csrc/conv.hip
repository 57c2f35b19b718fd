// a1+a2: the conv tower's convolutions (src/weinman/model.py:84-109, :126-146).
//
//   conv1   3x3 'valid', Cin = 1: a direct stencil fused with the uint8 ->
//           float preprocess (validate.py:56-68) and bias + ReLU. Cout/8 lanes
//           per output pixel, 8 channels each, from 9 cached pixels;
//           HBM-bound on the Cout-wide output write.
//   conv2-8 3x3 'same', Cin >= 32: implicit GEMM on MFMA (gemm.hip) --
//           M = B*H*W pixels, N = Cout, K = 9*Cin ordered (kh, kw, cin) so one
//           16-B staging load is 8 consecutive channels of one tap (NHWC).
//           Forward epilogue: bias, ReLU (odd layers) or per-tile BatchNorm
//           partial statistics (even layers, consumed by bn.hip).
//   backward: data = implicit GEMM over dy with mirrored taps against the
//           [Cin][kh][kw][Cout] weight image (+ the previous layer's ReLU mask);
//           weight = split-K GEMM im2col(x)^T . dy; bias = column sums of dy.
#include "common.h"
#include "gemm.h"
#include "reduce.h"

// ----------------------------------------------------------------- conv1 fwd
// G = COUT/8 lanes per output pixel, 8 channels each: a wave's 16-B stores
// cover 64/G consecutive pixels' whole channel rows (contiguous NHWC bytes)
// instead of one 16-B piece of 64 different pixels; the G lanes of a pixel
// read the same 9 input bytes (one cache line). Same fma order per channel.
template <typename TIn, typename TOut, int COUT>
__global__ void __launch_bounds__(256)
conv1_fwd_kernel(const TIn* __restrict__ x, int B, int H, int W, const float* __restrict__ w,
                 const float* __restrict__ bias, TOut* __restrict__ y) {
    constexpr int G = COUT / 8, PPB = 256 / G;
    static_assert(COUT % 8 == 0 && 256 % G == 0, "channel groups");
    __shared__ float sw[9 * COUT];
    __shared__ float sb[COUT];
    for (int i = threadIdx.x; i < 9 * COUT; i += 256) sw[i] = w[i];
    for (int i = threadIdx.x; i < COUT; i += 256) sb[i] = bias[i];
    __syncthreads();
    const int Ho = H - 2, Wo = W - 2;
    const int64_t npix = (int64_t)B * Ho * Wo;
    const int c0 = 8 * (threadIdx.x % G);
    for (int64_t pix = (int64_t)blockIdx.x * PPB + threadIdx.x / G; pix < npix; pix += (int64_t)gridDim.x * PPB) {
        int wo = (int)(pix % Wo);
        int64_t t = pix / Wo;
        int ho = (int)(t % Ho);
        int b = (int)(t / Ho);
        float px[9];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                TIn v = x[((int64_t)b * H + ho + kh) * W + wo + kw];
                if constexpr (sizeof(TIn) == 1) {
#pragma clang fp contract(off)
                    px[kh * 3 + kw] = (float)v * (1.0f / 255.0f) - 0.5f;   // validate.py:61-62
                } else {
                    px[kh * 3 + kw] = to_f32(v);
                }
            }
        F8 o;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float acc = sb[c0 + c];
#pragma unroll
            for (int k = 0; k < 9; ++k) acc = fmaf(px[k], sw[k * COUT + c0 + c], acc);
            o.v[c] = fmaxf(acc, 0.f);
        }
        store8(y + pix * COUT + c0, o);
    }
}

// ------------------------------------------------------- conv1 weight grad
// dw[k][c] = sum_pix x(pix + tap k) * dz[pix][c]; db[c] = sum_pix dz[pix][c].
// Each block reduces a pixel range into a [10][COUT] partial (slab); a second
// kernel sums the slabs in a fixed order (deterministic). A thread (8
// channels) keeps U pixels' loads in flight per pass; the lanes of a wave
// that share a channel group are combined with a fixed xor-shuffle tree, so
// the block needs only a [waves][groups][80] scratch and several blocks fit
// on a CU (the former [256][81] scratch allowed one: one wave per SIMD,
// latency-bound).
template <typename TIn, typename TG, int COUT>
__global__ void __launch_bounds__(256)
conv1_wgrad_partial(const TIn* __restrict__ x, const TG* __restrict__ dz, int B, int H, int W,
                    int64_t pix_per_block, float* __restrict__ slab) {
    constexpr int G = COUT / 8;              // channel groups of 8
    constexpr int P = 256 / G;               // pixels processed in parallel
    constexpr int U = 4;                     // pixels per thread per pass
    static_assert(64 % G == 0, "groups within a wave");
    __shared__ float red[4][G][10 * 8 + 1];
    const int Ho = H - 2, Wo = W - 2;
    const int64_t npix = (int64_t)B * Ho * Wo;
    const int cg = threadIdx.x % G, pl = threadIdx.x / G;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc[10][8];
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[k][c] = 0.f;
    const int64_t p0 = (int64_t)blockIdx.x * pix_per_block;
    const int64_t p1 = p0 + pix_per_block < npix ? p0 + pix_per_block : npix;
    for (int64_t q0 = p0 + pl; q0 < p1; q0 += (int64_t)P * U) {
        F8 g[U];
        float xv[U][9];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t pix = q0 + (int64_t)u * P;
            if (pix < p1) {
                const int wo = (int)(pix % Wo);
                const int64_t t = pix / Wo;
                const int ho = (int)(t % Ho);
                const int b = (int)(t / Ho);
                g[u] = load8(dz + pix * COUT + cg * 8);
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        const TIn v = x[((int64_t)b * H + ho + kh) * W + wo + kw];
                        if constexpr (sizeof(TIn) == 1) {
#pragma clang fp contract(off)
                            xv[u][kh * 3 + kw] = (float)v * (1.0f / 255.0f) - 0.5f;
                        } else {
                            xv[u][kh * 3 + kw] = to_f32(v);
                        }
                    }
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) g[u].v[c] = 0.f;
#pragma unroll
                for (int k = 0; k < 9; ++k) xv[u][k] = 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < 9; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[k][c] = fmaf(xv[u][k], g[u].v[c], acc[k][c]);
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[9][c] += g[u].v[c];
        }
    }
    // lanes l, l ^ G, l ^ 2G, ... of a wave hold the same channel group
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float v = acc[k][c];
#pragma unroll
            for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
            if (lane < G) red[wave][lane][k * 8 + c] = v;
        }
    __syncthreads();
    for (int o = threadIdx.x; o < 10 * COUT; o += 256) {
        const int k = o / COUT, c = o % COUT, gg = c / 8, ci = c % 8;
        slab[(int64_t)blockIdx.x * 10 * COUT + o] =
            ((red[0][gg][k * 8 + ci] + red[1][gg][k * 8 + ci]) + red[2][gg][k * 8 + ci]) + red[3][gg][k * 8 + ci];
    }
}

// out0 <- first n0 columns of sum_i slab[i][:], out1 <- the rest (fixed order)
__global__ void __launch_bounds__(256)
sum_slabs_kernel(const float* __restrict__ slab, int nslab, int width, float* __restrict__ out0,
                 int n0, float* __restrict__ out1, int accumulate) {
    __shared__ double part[4][64];
    const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int o = blockIdx.x * 64 + cl;
    double s = 0.0;
    if (o < width) {
#pragma unroll 8
        for (int i = q; i < nslab; i += 4) s += slab[(int64_t)i * width + o];
    }
    part[q][cl] = s;
    __syncthreads();
    if (q == 0 && o < width) {
        float t = (float)(part[0][cl] + part[1][cl] + part[2][cl] + part[3][cl]);
        if (o < n0) out0[o] = accumulate ? out0[o] + t : t;
        else if (out1) out1[o - n0] = accumulate ? out1[o - n0] + t : t;
    }
}

// ------------------------------------------------------------------ C ABI
extern "C" int ocrk_conv1_fwd(const void* x, int x_is_u8, int B, int H, int W, const float* w,
                              const float* bias, int cout, void* y, int dtype, void* stream) {
    OCRK_REQUIRE(B >= 0 && H >= 3 && W >= 3, "ocrk_conv1_fwd: bad shape B=%d H=%d W=%d", B, H, W);
    OCRK_REQUIRE(cout == 32, "ocrk_conv1_fwd: Cout=%d (this build carries the model.py:47 Cout=32)", cout);
    if (B == 0) return OCRK_OK;
    int64_t npix = (int64_t)B * (H - 2) * (W - 2);
    dim3 grid((unsigned)std::min<int64_t>(ocrk::cdiv(npix, 256 / (32 / 8)), 65535));   // 64 pixels per block pass
    hipStream_t s = ocrk::as_stream(stream);
    if (x_is_u8) {
        if (dtype == OCRK_BF16) conv1_fwd_kernel<uint8_t, bf16, 32><<<grid, 256, 0, s>>>((const uint8_t*)x, B, H, W, w, bias, (bf16*)y);
        else conv1_fwd_kernel<uint8_t, float, 32><<<grid, 256, 0, s>>>((const uint8_t*)x, B, H, W, w, bias, (float*)y);
    } else {
        if (dtype == OCRK_BF16) conv1_fwd_kernel<bf16, bf16, 32><<<grid, 256, 0, s>>>((const bf16*)x, B, H, W, w, bias, (bf16*)y);
        else conv1_fwd_kernel<float, float, 32><<<grid, 256, 0, s>>>((const float*)x, B, H, W, w, bias, (float*)y);
    }
    return ocrk::launch_status("ocrk_conv1_fwd");
}

static int64_t conv1_blocks(int64_t npix) { return std::max<int64_t>(1, std::min<int64_t>(1024, ocrk::cdiv(npix, 2048))); }

extern "C" size_t ocrk_conv1_wgrad_workspace_size(int B, int H, int W, int cout) {
    int64_t npix = (int64_t)B * (H - 2) * (W - 2);
    return (size_t)conv1_blocks(npix) * 10 * cout * sizeof(float);
}

extern "C" int ocrk_conv1_bwd_weight(const void* x, int x_is_u8, const void* dz, int B, int H, int W,
                                     int cout, float* dw, float* db, int accumulate, void* ws,
                                     size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(cout == 32, "ocrk_conv1_bwd_weight: Cout=%d unsupported", cout);
    OCRK_REQUIRE(ws_bytes >= ocrk_conv1_wgrad_workspace_size(B, H, W, cout), "ocrk_conv1_bwd_weight: workspace too small");
    int64_t npix = (int64_t)B * (H - 2) * (W - 2);
    int64_t nb = conv1_blocks(npix);
    int64_t per = ocrk::cdiv(npix, nb);
    hipStream_t s = ocrk::as_stream(stream);
    float* slab = (float*)ws;
    if (x_is_u8) {
        if (dtype == OCRK_BF16) conv1_wgrad_partial<uint8_t, bf16, 32><<<nb, 256, 0, s>>>((const uint8_t*)x, (const bf16*)dz, B, H, W, per, slab);
        else conv1_wgrad_partial<uint8_t, float, 32><<<nb, 256, 0, s>>>((const uint8_t*)x, (const float*)dz, B, H, W, per, slab);
    } else {
        if (dtype == OCRK_BF16) conv1_wgrad_partial<bf16, bf16, 32><<<nb, 256, 0, s>>>((const bf16*)x, (const bf16*)dz, B, H, W, per, slab);
        else conv1_wgrad_partial<float, float, 32><<<nb, 256, 0, s>>>((const float*)x, (const float*)dz, B, H, W, per, slab);
    }
    int st = ocrk::launch_status("ocrk_conv1_bwd_weight");
    if (st) return st;
    sum_slabs_kernel<<<(10 * cout + 63) / 64, 256, 0, s>>>(slab, (int)nb, 10 * cout, dw, 9 * cout, db, accumulate);
    return ocrk::launch_status("ocrk_conv1_bwd_weight reduce");
}

extern "C" size_t ocrk_conv_stats_tiles(int64_t M) { return (size_t)ocrk::cdiv(M, 128); }

namespace ocrk {   // conv_direct.hip: the narrow-channel layers (returns -1 when the shape is not covered)
int conv_direct_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout,
                    void* y, int relu, float* stats, hipStream_t s);
int conv_direct_bwd_data(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                         const void* relu_mask, float* stats, hipStream_t s);
size_t conv_direct_wgrad_ws_bytes(int B, int H, int W, int cin, int cout);
int conv_direct_wgrad(const void* x, const void* dy, int B, int H, int W, int cin, int cout, float* dw,
                      int accumulate, void* ws, size_t ws_bytes, hipStream_t s);
}

extern "C" int ocrk_conv3x3_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk,
                                const float* bias, int cout, void* y, int y_dtype, int relu,
                                float* stats, int dtype, void* stream) {
    ocrk::GemmParams p = {};
    p.M = B * H * W; p.N = cout; p.K = 9 * cin; p.batch = 1;
    p.A = x; p.B = w_nk; p.ldb = 9 * cin;
    p.C = y; p.ldc = cout; p.c_bf16 = y_dtype == OCRK_BF16;
    p.bias = bias; p.relu = relu; p.alpha = 1.f; p.stats = stats;
    p.splits = 1; p.k_chunk = (int)ocrk::cdiv(p.K, 32) * 32;
    p.convH = H; p.convW = W; p.convC = cin;
    if (dtype == OCRK_BF16 && y_dtype == OCRK_BF16) {
        const int st = ocrk::conv_direct_fwd(x, B, H, W, cin, w_nk, bias, cout, y, relu, stats, ocrk::as_stream(stream));
        if (st >= 0) return st;
    }
    return ocrk::gemm(p, ocrk::A_IM2COL, ocrk::B_NK, dtype, ocrk::as_stream(stream));
}

// Optional fused bias gradient of the producing (odd) conv: the GEMM's
// per-128-row-tile column statistics are taken after the ReLU mask, so their
// sums are the column sums of dx; slab_sum reduces them in a fixed order.
// workspace: stats [tiles][2 cin] f32 | part [SLAB_P][cin] double
static int64_t bwd_data_tiles(int B, int H, int W) { return ocrk::cdiv((int64_t)B * H * W, 128); }

extern "C" size_t ocrk_conv3x3_bwd_data_workspace_size(int B, int H, int W, int cin) {
    return ((size_t)bwd_data_tiles(B, H, W) * 2 * cin * sizeof(float) + 7) / 8 * 8 +
           (size_t)ocrk::SLAB_P * cin * sizeof(double);
}

extern "C" int ocrk_conv3x3_bwd_data(const void* dy, int B, int H, int W, int cout, const void* w_bwd,
                                     int cin, void* dx, const void* relu_mask, float* dbias, int accumulate,
                                     void* ws, size_t ws_bytes, int dtype, void* stream) {
    ocrk::GemmParams p = {};
    p.M = B * H * W; p.N = cin; p.K = 9 * cout; p.batch = 1;
    p.A = dy; p.B = w_bwd; p.ldb = 9 * cout;
    p.C = dx; p.ldc = cin; p.c_bf16 = dtype == OCRK_BF16;
    p.mask = relu_mask; p.ldmask = cin; p.alpha = 1.f;
    p.splits = 1; p.k_chunk = (int)ocrk::cdiv(p.K, 32) * 32;
    p.convH = H; p.convW = W; p.convC = cout;
    if (dbias) {
        OCRK_REQUIRE(ws && ws_bytes >= ocrk_conv3x3_bwd_data_workspace_size(B, H, W, cin),
                     "ocrk_conv3x3_bwd_data: workspace too small for the bias gradient");
        p.stats = (float*)ws;
    }
    hipStream_t s = ocrk::as_stream(stream);
    int st = dtype == OCRK_BF16 ? ocrk::conv_direct_bwd_data(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, p.stats, s) : -1;
    if (st < 0) st = ocrk::gemm(p, ocrk::A_IM2COL_FLIP, ocrk::B_NK, dtype, s);
    if (st || !dbias) return st;
    const int tiles = (int)bwd_data_tiles(B, H, W);
    double* part = (double*)((char*)ws + ((size_t)tiles * 2 * cin * sizeof(float) + 7) / 8 * 8);
    return ocrk::slab_sum((const float*)ws, tiles, cin, part, nullptr, dbias, nullptr, cin, accumulate, s, 2 * cin);
}

static int wgrad_splits(int64_t M, int cin, int cout) {
    // enough partial tiles to cover the chip ~2x (the 256 x 256 ping-pong
    // engine: ~1x, one item per CU); each split >= 4096 pixels
    if (ocrk::gemm_pptn_covers(ocrk::A_IM2COL_T, 9 * cin, cout, cin)) {
        const int64_t tiles = ocrk::cdiv(9 * cin, 256) * ocrk::cdiv(cout, 256);
        return (int)std::max<int64_t>(1, std::min<int64_t>(256 / tiles, M / 2048));   // items <= 256: one round
    }
    int64_t tiles = ocrk::cdiv(9 * cin, 128) * ocrk::cdiv(cout, cout <= 32 ? 32 : (cout <= 64 ? 64 : 128));
    int64_t want = ocrk::cdiv(512, tiles);
    int64_t maxs = std::max<int64_t>(1, M / 4096);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, maxs));
}

extern "C" size_t ocrk_conv3x3_wgrad_workspace_size(int B, int H, int W, int cin, int cout) {
    int64_t M = (int64_t)B * H * W;
    return std::max(ocrk::gemm_splitk_ws_bytes(9 * cin, cout, 1, wgrad_splits(M, cin, cout)),
                    ocrk::conv_direct_wgrad_ws_bytes(B, H, W, cin, cout));
}

extern "C" int ocrk_conv3x3_bwd_weight(const void* x, const void* dy, int B, int H, int W, int cin,
                                       int cout, float* dw, int accumulate, void* ws, size_t ws_bytes,
                                       int dtype, void* stream) {
    int64_t M = (int64_t)B * H * W;
    ocrk::GemmParams p = {};
    p.M = 9 * cin; p.N = cout; p.K = (int)M; p.batch = 1;
    p.A = x; p.B = dy; p.ldb = cout;
    p.C = dw; p.ldc = cout; p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
    int splits = wgrad_splits(M, cin, cout);
    p.k_chunk = (int)(ocrk::cdiv(ocrk::cdiv(M, splits), 32) * 32);
    p.splits = (int)ocrk::cdiv(M, p.k_chunk);
    p.splitk_ws = (float*)ws;
    OCRK_REQUIRE(p.splits == 1 || ws_bytes >= ocrk::gemm_splitk_ws_bytes(p.M, p.N, 1, p.splits),
                 "ocrk_conv3x3_bwd_weight: workspace too small");
    p.convH = H; p.convW = W; p.convC = cin;
    if (dtype == OCRK_BF16) {
        const int st = ocrk::conv_direct_wgrad(x, dy, B, H, W, cin, cout, dw, accumulate, ws, ws_bytes,
                                               ocrk::as_stream(stream));
        if (st >= 0) return st;
    }
    return ocrk::gemm(p, ocrk::A_IM2COL_T, ocrk::B_KN, dtype, ocrk::as_stream(stream));
}
