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
#include "mfma_util.h"

// ----------------------------------------------------------------- conv1 fwd
// A workgroup owns one output strip: (image b, C1_WR rows, C1_PX consecutive
// output columns). The C1_WR + 2 input rows it needs (C1_PX + 2 values each)
// are preprocessed once into LDS; a thread keeps the 72 weights + 8 biases of its
// channel group (c0 = 8 (tid % G)) in registers and produces G (pixel, group)
// items, item = tid + 256 j -> pixel item / G: a wave's 16-B stores cover
// 64/G consecutive pixels' whole channel rows (1 KB contiguous). No per-pixel
// 64-bit index arithmetic, one byte load per input value per workgroup.
// Same fma order per channel as the oracle's sum (bias, then taps row-major).
constexpr int C1_PX = 256;   // output columns per strip
constexpr int C1_WR = 8;     // output rows per strip (4 strips per 32-row crop: one round at 4 per CU)

template <typename TIn>
__device__ __forceinline__ float conv1_in(TIn v) {
    if constexpr (sizeof(TIn) == 1) {
#pragma clang fp contract(off)
        return (float)v * (1.0f / 255.0f) - 0.5f;                        // validate.py:61-62
    } else {
        return to_f32(v);
    }
}

// the ROWS input rows of a strip into LDS (preprocessed): every load of the
// workgroup's share is issued before the first is used (fixed trip count)
template <typename TIn, int ROWS>
__device__ __forceinline__ void conv1_stage(const TIn* __restrict__ x, int H, int W, int b, int h0, int wo0,
                                            float (*sx)[C1_PX + 2]) {
    constexpr int N = ROWS * (C1_PX + 2), IT = (N + 255) / 256;
    TIn v[IT];
    bool ok[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int i = threadIdx.x + 256 * q;
        const int r = i / (C1_PX + 2), col = i - r * (C1_PX + 2);
        const int xc = wo0 + col, h = h0 + r;
        ok[q] = i < N && xc < W && h < H;
        v[q] = ok[q] ? x[((int64_t)b * H + h) * W + xc] : TIn(0);
    }
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int i = threadIdx.x + 256 * q;
        if (i < N) {
            const int r = i / (C1_PX + 2), col = i - r * (C1_PX + 2);
            sx[r][col] = ok[q] ? conv1_in(v[q]) : 0.f;
        }
    }
}

template <typename TIn, typename TOut, int COUT>
__global__ void __launch_bounds__(256)
conv1_fwd_kernel(const TIn* __restrict__ x, int B, int H, int W, const float* __restrict__ w,
                 const float* __restrict__ bias, TOut* __restrict__ y, uint8_t* __restrict__ bits) {
    constexpr int G = COUT / 8;
    static_assert(COUT % 8 == 0 && 256 % G == 0, "channel groups");
    __shared__ float sx[C1_WR + 2][C1_PX + 2];
    const int Ho = H - 2, Wo = W - 2;
    const int nch = (Wo + C1_PX - 1) / C1_PX, nrg = (Ho + C1_WR - 1) / C1_WR;
    const int chunk = blockIdx.x % nch;
    const int t = blockIdx.x / nch;
    const int rg = t % nrg, b = t / nrg;
    const int ho0 = rg * C1_WR, wo0 = chunk * C1_PX;
    const int nrows = min(C1_WR, Ho - ho0);
    const int c0 = 8 * (threadIdx.x % G);
    float wr[9][8], br[8];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) wr[k][c] = w[k * COUT + c0 + c];
#pragma unroll
    for (int c = 0; c < 8; ++c) br[c] = bias[c0 + c];
    conv1_stage<TIn, C1_WR + 2>(x, H, W, b, ho0, wo0, sx);
    __syncthreads();
    for (int r = 0; r < nrows; ++r) {
        TOut* yrow = y + (((int64_t)b * Ho + ho0 + r) * Wo + wo0) * COUT + c0;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int p = (threadIdx.x + 256 * j) / G;
            if (wo0 + p >= Wo) break;
            float px[9];
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) px[kh * 3 + kw] = sx[r + kh][p + kw];
            F8 o;
            unsigned on = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                float acc = br[c];
#pragma unroll
                for (int k = 0; k < 9; ++k) acc = fmaf(px[k], wr[k][c], acc);
                o.v[c] = fmaxf(acc, 0.f);
                on |= (o.v[c] > 0.f ? 1u : 0u) << c;
            }
            store8(yrow + (int64_t)p * COUT, o);
            // the ReLU's bit mask (bit c of byte g: channel 8 g + c of the pixel), the
            // backward's mask at 1/16 of the bf16 output's bytes
            if (bits) bits[(((int64_t)b * Ho + ho0 + r) * Wo + wo0 + p) * (COUT / 8) + c0 / 8] = (uint8_t)on;
        }
    }
}

// ------------------------------------------------------- conv1 weight grad
// dw[k][c] = sum_pix x(pix + tap k) * dz[pix][c]; db[c] = sum_pix dz[pix][c].
// A workgroup owns C1_GR output rows x C1_PX columns of one image: the
// C1_GR + 2 input rows are preprocessed into LDS once, then per row every
// thread accumulates its G items' dz pieces into [10][8] partials for its
// fixed channel group while the raw pieces of the next two rows are in flight
// (kept as loaded -- 16 B per item for bf16 -- and widened at use). Lanes of a
// wave that share a group are combined with a reduce-scatter butterfly, the 4
// waves in a fixed order -> one [10][COUT] slab row per workgroup; slab_sum
// adds the rows in a fixed order (deterministic).
constexpr int C1_GR = 15;    // output rows per weight-gradient strip (2 strips per 32-row crop: one round at 2 per CU)

template <typename T> struct Raw8;
template <> struct Raw8<bf16> {
    ocrk::u32x4 q;
    __device__ __forceinline__ void load(const bf16* p) { q = *reinterpret_cast<const ocrk::u32x4*>(p); }
    __device__ __forceinline__ void zero() { q = ocrk::u32x4{0u, 0u, 0u, 0u}; }
    __device__ __forceinline__ float at(int i) const { return __uint_as_float((q[i >> 1] >> (16 * (i & 1))) << 16); }
};
template <> struct Raw8<float> {
    F8 f;
    __device__ __forceinline__ void load(const float* p) { f = load8(p); }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int i = 0; i < 8; ++i) f.v[i] = 0.f;
    }
    __device__ __forceinline__ float at(int i) const { return f.v[i]; }
};

template <typename TIn, typename TG, int COUT>
__global__ void __launch_bounds__(256)
conv1_wgrad_partial(const TIn* __restrict__ x, const TG* __restrict__ dz, int B, int H, int W,
                    float* __restrict__ slab) {
    constexpr int G = COUT / 8;              // channel groups of 8
    static_assert(64 % G == 0, "groups within a wave");
    __shared__ float sx[C1_GR + 2][C1_PX + 2];
    __shared__ float red[4][G][10 * 8 + 1];
    const int Ho = H - 2, Wo = W - 2;
    const int nch = (Wo + C1_PX - 1) / C1_PX, nrg = (Ho + C1_GR - 1) / C1_GR;
    const int chunk = blockIdx.x % nch;
    const int t = blockIdx.x / nch;
    const int rg = t % nrg, b = t / nrg;
    const int ho0 = rg * C1_GR, wo0 = chunk * C1_PX;
    const int nrows = min(C1_GR, Ho - ho0);
    const int cg = threadIdx.x % G;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    auto load_row = [&](Raw8<TG> (&g)[G], int r) {
        const TG* drow = dz + (((int64_t)b * Ho + ho0 + r) * Wo + wo0) * COUT + cg * 8;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int p = (threadIdx.x + 256 * j) / G;
            if (r < nrows && wo0 + p < Wo) g[j].load(drow + (int64_t)p * COUT);
            else g[j].zero();
        }
    };
    // rows 0 and 1 in flight with the input staging
    Raw8<TG> g0[G], g1[G];
    load_row(g0, 0);
    load_row(g1, 1);
    conv1_stage<TIn, C1_GR + 2>(x, H, W, b, ho0, wo0, sx);
    float acc[10][8];
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[k][c] = 0.f;
    __syncthreads();
    for (int r = 0; r < nrows; ++r) {
        Raw8<TG> g[G];
#pragma unroll
        for (int j = 0; j < G; ++j) { g[j] = g0[j]; g0[j] = g1[j]; }
        load_row(g1, r + 2);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int p = (threadIdx.x + 256 * j) / G;
            float px[9], gv[8];
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) px[kh * 3 + kw] = sx[r + kh][p + kw];
#pragma unroll
            for (int c = 0; c < 8; ++c) gv[c] = g[j].at(c);
#pragma unroll
            for (int k = 0; k < 9; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[k][c] = fmaf(px[k], gv[c], acc[k][c]);
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[9][c] += gv[c];
        }
    }
    // lanes l, l ^ G, l ^ 2G, ... of a wave hold the same channel group: a
    // reduce-scatter butterfly over those lanes (each level keeps half of the
    // values and trades the other half: 40 + 20 + 10 + 5 independent shuffles
    // instead of 4 x 80 dependent ones); a lane ends with 5 sums, values
    // base .. base + 4 of its group
    static_assert(G == 4, "the butterfly below is laid out for 4 groups (COUT = 32)");
    float a[80];
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) a[k * 8 + c] = acc[k][c];
    int base = 0;
#pragma unroll
    for (int lvl = 0, half = 40; lvl < 4; ++lvl, half >>= 1) {
        const int m = G << lvl;
        const bool hi = lane & m;
        float t[40];
#pragma unroll
        for (int i = 0; i < half; ++i) t[i] = __shfl_xor(hi ? a[i] : a[i + half], m, 64);
#pragma unroll
        for (int i = 0; i < half; ++i) a[i] = (hi ? a[i + half] : a[i]) + t[i];
        base += hi ? half : 0;
    }
    // lanes with (lane & (G - 1)) == group hold disjoint 5-value pieces of its 80 sums
#pragma unroll
    for (int i = 0; i < 5; ++i) red[wave][lane & (G - 1)][base + i] = a[i];
    __syncthreads();
    for (int o = threadIdx.x; o < 10 * COUT; o += 256) {
        const int k = o / COUT, c = o % COUT, gg = c / 8, ci = c % 8;
        slab[(int64_t)blockIdx.x * 10 * COUT + o] =
            ((red[0][gg][k * 8 + ci] + red[1][gg][k * 8 + ci]) + red[2][gg][k * 8 + ci]) + red[3][gg][k * 8 + ci];
    }
}

// ------------------------------------------------------------------ C ABI
static int conv1_fwd_run(const void* x, int x_is_u8, int B, int H, int W, const float* w, const float* bias,
                         int cout, void* y, uint8_t* bits, int dtype, void* stream) {
    OCRK_REQUIRE(B >= 0 && H >= 3 && W >= 3, "ocrk_conv1_fwd: bad shape B=%d H=%d W=%d", B, H, W);
    OCRK_REQUIRE(cout == 32, "ocrk_conv1_fwd: Cout=%d (this build carries the model.py:47 Cout=32)", cout);
    if (B == 0) return OCRK_OK;
    const int64_t blocks = (int64_t)B * ocrk::cdiv(H - 2, C1_WR) * ocrk::cdiv(W - 2, C1_PX);
    OCRK_REQUIRE(blocks < (1ll << 31), "ocrk_conv1_fwd: too many rows");
    dim3 grid((unsigned)blocks);
    hipStream_t s = ocrk::as_stream(stream);
    if (x_is_u8) {
        if (dtype == OCRK_BF16) conv1_fwd_kernel<uint8_t, bf16, 32><<<grid, 256, 0, s>>>((const uint8_t*)x, B, H, W, w, bias, (bf16*)y, bits);
        else conv1_fwd_kernel<uint8_t, float, 32><<<grid, 256, 0, s>>>((const uint8_t*)x, B, H, W, w, bias, (float*)y, bits);
    } else {
        if (dtype == OCRK_BF16) conv1_fwd_kernel<bf16, bf16, 32><<<grid, 256, 0, s>>>((const bf16*)x, B, H, W, w, bias, (bf16*)y, bits);
        else conv1_fwd_kernel<float, float, 32><<<grid, 256, 0, s>>>((const float*)x, B, H, W, w, bias, (float*)y, bits);
    }
    return ocrk::launch_status("ocrk_conv1_fwd");
}

extern "C" int ocrk_conv1_fwd(const void* x, int x_is_u8, int B, int H, int W, const float* w,
                              const float* bias, int cout, void* y, int dtype, void* stream) {
    return conv1_fwd_run(x, x_is_u8, B, H, W, w, bias, cout, y, nullptr, dtype, stream);
}

// the same with the ReLU's bit mask: relu_bits u8 [B,H-2,W-2][cout/8], bit c of byte g
// = (y[..][8 g + c] > 0) -- the mask ocrk_conv2_bwd_data_conv1_wgrad reads
extern "C" int ocrk_conv1_fwd_relu_bits(const void* x, int x_is_u8, int B, int H, int W, const float* w,
                                        const float* bias, int cout, void* y, void* relu_bits, int dtype,
                                        void* stream) {
    OCRK_REQUIRE(relu_bits, "ocrk_conv1_fwd_relu_bits: null mask");
    return conv1_fwd_run(x, x_is_u8, B, H, W, w, bias, cout, y, (uint8_t*)relu_bits, dtype, stream);
}

static int64_t conv1_blocks(int B, int H, int W) {
    return std::max<int64_t>(1, (int64_t)B * ocrk::cdiv(H - 2, C1_GR) * ocrk::cdiv(W - 2, C1_PX));
}

extern "C" size_t ocrk_conv1_wgrad_workspace_size(int B, int H, int W, int cout) {
    // slab [blocks][10 cout] f32 | part [SLAB_P][10 cout] double (slab_sum's two-stage form)
    return ((size_t)conv1_blocks(B, H, W) * 10 * cout * sizeof(float) + 15) / 16 * 16 +
           (size_t)ocrk::SLAB_P * 10 * cout * sizeof(double);
}

extern "C" int ocrk_conv1_bwd_weight(const void* x, int x_is_u8, const void* dz, int B, int H, int W,
                                     int cout, float* dw, float* db, int accumulate, void* ws,
                                     size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(cout == 32, "ocrk_conv1_bwd_weight: Cout=%d unsupported", cout);
    OCRK_REQUIRE(ws_bytes >= ocrk_conv1_wgrad_workspace_size(B, H, W, cout), "ocrk_conv1_bwd_weight: workspace too small");
    OCRK_REQUIRE(B >= 1 && H >= 3 && W >= 3, "ocrk_conv1_bwd_weight: bad shape B=%d H=%d W=%d", B, H, W);
    const int64_t nb = conv1_blocks(B, H, W);
    OCRK_REQUIRE(nb < (1ll << 31), "ocrk_conv1_bwd_weight: too many rows");
    hipStream_t s = ocrk::as_stream(stream);
    float* slab = (float*)ws;
    if (x_is_u8) {
        if (dtype == OCRK_BF16) conv1_wgrad_partial<uint8_t, bf16, 32><<<nb, 256, 0, s>>>((const uint8_t*)x, (const bf16*)dz, B, H, W, slab);
        else conv1_wgrad_partial<uint8_t, float, 32><<<nb, 256, 0, s>>>((const uint8_t*)x, (const float*)dz, B, H, W, slab);
    } else {
        if (dtype == OCRK_BF16) conv1_wgrad_partial<bf16, bf16, 32><<<nb, 256, 0, s>>>((const bf16*)x, (const bf16*)dz, B, H, W, slab);
        else conv1_wgrad_partial<float, float, 32><<<nb, 256, 0, s>>>((const float*)x, (const float*)dz, B, H, W, slab);
    }
    int st = ocrk::launch_status("ocrk_conv1_bwd_weight");
    if (st) return st;
    double* part = (double*)((char*)ws + ((size_t)nb * 10 * cout * sizeof(float) + 15) / 16 * 16);
    return ocrk::slab_sum(slab, (int)nb, 10 * cout, part, nullptr, dw, db, 9 * cout, accumulate, s);
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
size_t conv_rows_wgrad_ws_bytes(int B, int cin, int cout);
bool conv_rows_fwd_covers(int B, int H, int W, int cin, int cout);
int conv_rows_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout, void* y,
                  int relu, float* stats, hipStream_t s);
int conv_rows_dgrad(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                    const void* relu_mask, float* stats, hipStream_t s);
int conv_rows_wgrad(const void* x, const void* dy, int B, int H, int W, int cin, int cout, float* dw, int accumulate,
                    void* ws, size_t ws_bytes, hipStream_t s);
bool conv_rows_dgrad_c1_covers(int B, int H, int W, int cin, int cout);
bool conv_rows_fwd_bits_covers(int B, int H, int W, int cin, int cout);
bool conv12_fwd_covers(int B, int H, int W);
int conv12_fwd(const void* img, int x_is_u8, int B, int H, int W, const float* w1, const float* b1,
               const void* w_nk2, const float* b2, void* y1, void* bits, void* z, float* stats, hipStream_t s);
int conv_rows_wgrad_c1x(const void* img, int x_is_u8, const float* w1, const float* b1, const void* dy, int B, int H,
                        int W, float* dw, int accumulate, void* ws, size_t ws_bytes, hipStream_t s);
int conv_rows_fwd_bits(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout,
                       void* y, void* bits, hipStream_t s);
bool conv_rows_dgrad_bits_covers(int B, int H, int W, int cin, int cout);
int conv_rows_dgrad_bits(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                         const void* bits, float* stats, hipStream_t s);
bool gemm_nt_enabled();
bool nt_staged_enabled();
int64_t conv_rows_dgrad_c1_parts(int B);
int conv_rows_dgrad_c1(const void* dy, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                       const void* relu_bits, const void* x, int x_is_u8, float* part, hipStream_t s);
int64_t conv_rows_bwd_w2_parts(int B);
int conv_rows_bwd_w2(const void* dy, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                     const void* relu_bits, const void* x, int x_is_u8, const float* w1, const float* b1,
                     float* c1part, float* w2part, float* dw2, int accumulate, hipStream_t s);
}

// conv1 -> conv2 forward as one row walk (bf16 training): conv1's output rows are produced
// into conv2's ring from the image (conv1 on the MFMA, hi + lo split operands) instead of
// being written and re-read. x [B,IH,IW] u8 (x_is_u8: the fused preprocess) or bf16; w1 f32
// [3][3][1][32], b1 [32]; w_nk2 bf16 [32][3][3][32], b2 [32]; outputs y1 [B,IH-2,IW-2,32]
// bf16 (conv1's ReLU output), relu_bits u8 [B,IH-2,IW-2][4] (its bit mask), z (conv2's
// pre-BN output, same shape) and stats [B*(IH-2)][2][32] (conv2's per-row BN partials,
// ocrk_bn_finalize_tiles with tile_rows = IW-2). y1 may be NULL: not written
// (ocrk_conv12_bwd recomputes it).
extern "C" int ocrk_conv12_fwd_supported(int B, int IH, int IW, int dtype) {
    return dtype == OCRK_BF16 && IH >= 3 && IW >= 3 && ocrk::conv12_fwd_covers(B, IH - 2, IW - 2) ? 1 : 0;
}

extern "C" int ocrk_conv12_fwd(const void* x, int x_is_u8, int B, int IH, int IW, const float* w1, const float* b1,
                               const void* w_nk2, const float* b2, void* y1, void* relu_bits, void* z, float* stats,
                               int dtype, void* stream) {
    OCRK_REQUIRE(ocrk_conv12_fwd_supported(B, IH, IW, dtype), "ocrk_conv12_fwd: B=%d IH=%d IW=%d dtype=%d not covered",
                 B, IH, IW, dtype);
    OCRK_REQUIRE(x && w1 && b1 && w_nk2 && relu_bits && z && stats, "ocrk_conv12_fwd: null pointer");
    return ocrk::conv12_fwd(x, x_is_u8, B, IH - 2, IW - 2, w1, b1, w_nk2, b2, y1, relu_bits, z, stats,
                            ocrk::as_stream(stream));
}

#ifdef OCRK_EXPERIMENTS
// (tools build, include/ocrk_debug.h: measured +55 us in the step, it lands on the tail)
// conv2's weight gradient with its input y1 = relu(conv1(x)) recomputed per row from the
// image instead of read (bf16): dw [3][3][32][32] f32 (+)= sum y1 (x) dz over the batch,
// y1 bit-identical to ocrk_conv12_fwd's. x, w1, b1 as ocrk_conv12_fwd; dz [B,IH-2,IW-2,32]
// bf16; ws per ocrk_conv3x3_wgrad_workspace_size(B, IH-2, IW-2, 32, 32).
extern "C" int ocrk_conv2_bwd_weight_c1x_supported(int B, int IH, int IW, int dtype) {
    return ocrk_conv12_fwd_supported(B, IH, IW, dtype);
}

extern "C" int ocrk_conv2_bwd_weight_c1x(const void* x, int x_is_u8, int B, int IH, int IW, const float* w1,
                                         const float* b1, const void* dz, float* dw, int accumulate, void* ws,
                                         size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(ocrk_conv2_bwd_weight_c1x_supported(B, IH, IW, dtype),
                 "ocrk_conv2_bwd_weight_c1x: B=%d IH=%d IW=%d dtype=%d not covered", B, IH, IW, dtype);
    OCRK_REQUIRE(x && w1 && b1 && dz && dw && ws, "ocrk_conv2_bwd_weight_c1x: null pointer");
    int st = ocrk::conv_rows_wgrad_c1x(x, x_is_u8, w1, b1, dz, B, IH - 2, IW - 2, dw, accumulate, ws, ws_bytes,
                                       ocrk::as_stream(stream));
    OCRK_REQUIRE(st >= 0, "ocrk_conv2_bwd_weight_c1x: workspace too small or path disabled");
    return st;
}
#endif  // OCRK_EXPERIMENTS

// conv2's backward-data and conv1's weight gradient as one pass (bf16): the data
// gradient dy1 = relu'(y1) . conv2^T(dz2) is contracted against conv1's input as
// it is produced and never stored (its only consumer is conv1's weight gradient:
// conv1 is the first layer). dz2 [B,H,W,32], x [B,H+2,W+2] u8 or bf16, y1 the
// ReLU mask [B,H,W,32] -- or relu_bits, its bit mask from ocrk_conv1_fwd_relu_bits (u8
// [B,H,W][4], 1/16 of the bytes; exactly one of the two); dw1 [3,3,1,32] / db1 [32] (+)= the sums.
// workspace: part [B * bands][10 * 32] f32 | slab_sum's [SLAB_P][320] double
extern "C" int ocrk_conv2_bwd_data_conv1_wgrad_supported(int B, int H, int W, int cin, int cout, int dtype) {
    return dtype == OCRK_BF16 && ocrk::conv_rows_dgrad_c1_covers(B, H, W, cin, cout) ? 1 : 0;
}

extern "C" size_t ocrk_conv2_bwd_data_conv1_wgrad_workspace_size(int B, int H, int W) {
    (void)H; (void)W;
    return ((size_t)ocrk::conv_rows_dgrad_c1_parts(std::max(B, 1)) * 10 * 32 * sizeof(float) + 15) / 16 * 16 +
           (size_t)ocrk::SLAB_P * 10 * 32 * sizeof(double);
}

extern "C" int ocrk_conv2_bwd_data_conv1_wgrad(const void* dz, int B, int H, int W, const void* w_bwd,
                                               const void* relu_mask, const void* relu_bits, const void* x,
                                               int x_is_u8, float* dw, float* db, int accumulate, void* ws,
                                               size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(ocrk_conv2_bwd_data_conv1_wgrad_supported(B, H, W, 32, 32, dtype),
                 "ocrk_conv2_bwd_data_conv1_wgrad: B=%d H=%d W=%d dtype=%d not covered", B, H, W, dtype);
    OCRK_REQUIRE(dz && w_bwd && x && dw && db && ws, "ocrk_conv2_bwd_data_conv1_wgrad: null pointer");
    OCRK_REQUIRE(!relu_mask != !relu_bits, "ocrk_conv2_bwd_data_conv1_wgrad: give exactly one of relu_mask / relu_bits");
    OCRK_REQUIRE(ws_bytes >= ocrk_conv2_bwd_data_conv1_wgrad_workspace_size(B, H, W) && (uintptr_t)ws % 16 == 0,
                 "ocrk_conv2_bwd_data_conv1_wgrad: workspace too small or misaligned");
    const int64_t nb = ocrk::conv_rows_dgrad_c1_parts(B);
    OCRK_REQUIRE(nb < (1ll << 31), "ocrk_conv2_bwd_data_conv1_wgrad: too many rows");
    hipStream_t s = ocrk::as_stream(stream);
    float* part = (float*)ws;
    int st = ocrk::conv_rows_dgrad_c1(dz, B, H, W, w_bwd, relu_mask, relu_bits, x, x_is_u8, part, s);
    if (st) return st;
    double* part2 = (double*)((char*)ws + ((size_t)nb * 10 * 32 * sizeof(float) + 15) / 16 * 16);
    return ocrk::slab_sum(part, (int)nb, 10 * 32, part2, nullptr, dw, db, 9 * 32, accumulate, s);
}

// conv1 -> conv2 backward as one row walk (bf16 training; the backward of ocrk_conv12_fwd,
// src/weinman/model.py:84-123): conv2's data gradient (dy1 = relu'(y1) . conv2^T(dz2),
// contracted into conv1's weight gradient as it is produced, as
// ocrk_conv2_bwd_data_conv1_wgrad) AND conv2's weight gradient, whose input y1 =
// relu(conv1(x)) is recomputed per row from the image (the bits ocrk_conv12_fwd produced)
// instead of read -- so the forward need not write y1. dz2 [B,H,W,32] bf16, w_bwd conv2's
// backward image, relu_mask / relu_bits as ocrk_conv2_bwd_data_conv1_wgrad, x [B,H+2,W+2]
// u8 or bf16, w1 [3][3][1][32] / b1 [32] f32 conv1's variables; dw2 [3][3][32][32],
// dw1 [3][3][1][32], db1 [32] f32 (+)= the sums.
// workspace: conv1 partials | slab_sum's doubles | conv2 partials [max(2, B)][9216] f32
static size_t conv12_bwd_c1_bytes(int B) {
    return ((size_t)ocrk::conv_rows_bwd_w2_parts(std::max(B, 1)) * 10 * 32 * sizeof(float) + 15) / 16 * 16;
}

extern "C" int ocrk_conv12_bwd_supported(int B, int H, int W, int dtype) {
    return dtype == OCRK_BF16 && ocrk::conv_rows_dgrad_c1_covers(B, H, W, 32, 32) ? 1 : 0;
}

extern "C" size_t ocrk_conv12_bwd_workspace_size(int B, int H, int W) {
    (void)H; (void)W;
    return conv12_bwd_c1_bytes(B) + (size_t)ocrk::SLAB_P * 10 * 32 * sizeof(double) +
           (size_t)std::max<int64_t>(2, ocrk::conv_rows_bwd_w2_parts(std::max(B, 1))) * 9 * 32 * 32 * sizeof(float);
}

extern "C" int ocrk_conv12_bwd(const void* dz, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                               const void* relu_bits, const void* x, int x_is_u8, const float* w1, const float* b1,
                               float* dw2, float* dw1, float* db1, int accumulate, void* ws, size_t ws_bytes,
                               int dtype, void* stream) {
    OCRK_REQUIRE(ocrk_conv12_bwd_supported(B, H, W, dtype), "ocrk_conv12_bwd: B=%d H=%d W=%d dtype=%d not covered",
                 B, H, W, dtype);
    OCRK_REQUIRE(dz && w_bwd && x && w1 && b1 && dw2 && dw1 && db1 && ws, "ocrk_conv12_bwd: null pointer");
    OCRK_REQUIRE(!relu_mask != !relu_bits, "ocrk_conv12_bwd: give exactly one of relu_mask / relu_bits");
    OCRK_REQUIRE(ws_bytes >= ocrk_conv12_bwd_workspace_size(B, H, W) && (uintptr_t)ws % 16 == 0,
                 "ocrk_conv12_bwd: workspace too small or misaligned");
    const int64_t nb = ocrk::conv_rows_bwd_w2_parts(B);
    OCRK_REQUIRE(nb < (1ll << 31), "ocrk_conv12_bwd: too many rows");
    hipStream_t s = ocrk::as_stream(stream);
    float* c1part = (float*)ws;
    double* c1sum = (double*)((char*)ws + conv12_bwd_c1_bytes(B));
    float* w2part = (float*)((char*)c1sum + (size_t)ocrk::SLAB_P * 10 * 32 * sizeof(double));
    int st = ocrk::conv_rows_bwd_w2(dz, B, H, W, w_bwd, relu_mask, relu_bits, x, x_is_u8, w1, b1, c1part, w2part, dw2,
                                    accumulate, s);
    if (st) return st;
    return ocrk::slab_sum(c1part, (int)nb, 10 * 32, c1sum, nullptr, dw1, db1, 9 * 32, accumulate, s);
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
        int st = stats ? -1 : ocrk::conv_rows_fwd(x, B, H, W, cin, w_nk, bias, cout, y, relu, nullptr, ocrk::as_stream(stream));
        if (st >= 0) return st;
        st = ocrk::conv_direct_fwd(x, B, H, W, cin, w_nk, bias, cout, y, relu, stats, ocrk::as_stream(stream));
        if (st >= 0) return st;
    }
    return ocrk::gemm(p, ocrk::A_IM2COL, ocrk::B_NK, dtype, ocrk::as_stream(stream));
}

// The forward with the BatchNorm partials per OUTPUT ROW (conv2's shape on the
// row-walking kernel): stats [B*H][2][cout], finalized with tile_rows = W.
extern "C" int ocrk_conv3x3_fwd_rowstats_supported(int B, int H, int W, int cin, int cout) {
    return ocrk::conv_rows_fwd_covers(B, H, W, cin, cout) ? 1 : 0;
}

extern "C" int ocrk_conv3x3_fwd_rowstats(const void* x, int B, int H, int W, int cin, const void* w_nk,
                                         const float* bias, int cout, void* y, int relu, float* stats, void* stream) {
    OCRK_REQUIRE(stats && ocrk::conv_rows_fwd_covers(B, H, W, cin, cout),
                 "ocrk_conv3x3_fwd_rowstats: shape B=%d H=%d W=%d %d->%d not covered", B, H, W, cin, cout);
    return ocrk::conv_rows_fwd(x, B, H, W, cin, w_nk, bias, cout, y, relu, stats, ocrk::as_stream(stream));
}

// Optional fused bias gradient of the producing (odd) conv: the GEMM's
// per-128-row-tile column statistics are taken after the ReLU mask, so their
// sums are the column sums of dx; slab_sum reduces them in a fixed order.
// workspace: stats [tiles][2 cin] f32 | part [SLAB_P][cin] double
static int64_t bwd_data_tiles(int B, int H, int W) { return ocrk::cdiv((int64_t)B * H * W, 128); }

// dx (and, with stats, the per-tile column statistics of the masked dx)
static int bwd_data_run(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                        const void* relu_mask, float* stats, int dtype, hipStream_t s, const void* relu_bits = nullptr) {
    ocrk::GemmParams p = {};
    p.M = B * H * W; p.N = cin; p.K = 9 * cout; p.batch = 1;
    p.A = dy; p.B = w_bwd; p.ldb = 9 * cout;
    p.C = dx; p.ldc = cin; p.c_bf16 = dtype == OCRK_BF16;
    p.mask = relu_mask; p.ldmask = cin; p.alpha = 1.f;
    p.splits = 1; p.k_chunk = (int)ocrk::cdiv(p.K, 32) * 32;
    p.convH = H; p.convW = W; p.convC = cout;
    p.stats = stats;
    if (relu_bits) {                         // the bit-mask routes only (rows kernel, else the NT engine)
        const int sb = ocrk::conv_rows_dgrad_bits(dy, B, H, W, cout, w_bwd, cin, dx, relu_bits, stats, s);
        if (sb >= 0) return sb;
        p.mask = nullptr;
        p.mask_bits = relu_bits;
        return ocrk::gemm(p, ocrk::A_IM2COL_FLIP, ocrk::B_NK, dtype, s);
    }
    int st = dtype == OCRK_BF16 ? ocrk::conv_rows_dgrad(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, stats, s) : -1;
    if (st < 0 && dtype == OCRK_BF16) st = ocrk::conv_direct_bwd_data(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, stats, s);
    if (st < 0) st = ocrk::gemm(p, ocrk::A_IM2COL_FLIP, ocrk::B_NK, dtype, s);
    return st;
}

// ReLU bit masks between an odd conv's forward and the next even conv's backward-data
// (conv3 -> conv4, conv5 -> conv6, conv7 -> conv8 in the path): the forward writes
// relu_bits [B*H*W][cout/8] (bit c of byte c/8: y[..][c] > 0) beside y, the data gradient
// reads them instead of the bf16 y -- 1/16 of the mask bytes. Covered: bf16 on the wide
// row kernels (forward 32->64, 64->64, 64->128; backward-data 64<-64) or the NT engine's
// staged epilogue (channels a multiple of 8, K = 9 Cin >= 512 or Cout <= 64).
static bool nt_bits_ok(int cin, int cout) {
    return ocrk::gemm_nt_enabled() && ocrk::nt_staged_enabled() && cin % 8 == 0 && cout % 8 == 0 &&
           (9 * cin >= 512 || cout <= 64);
}

extern "C" int ocrk_conv3x3_fwd_relu_bits_supported(int B, int H, int W, int cin, int cout, int dtype) {
    if (dtype != OCRK_BF16 || B < 1 || H < 1 || W < 1 || (int64_t)B * H * W >= (1ll << 31)) return 0;
    return ocrk::conv_rows_fwd_bits_covers(B, H, W, cin, cout) || nt_bits_ok(cin, cout) ? 1 : 0;
}

extern "C" int ocrk_conv3x3_fwd_relu_bits(const void* x, int B, int H, int W, int cin, const void* w_nk,
                                          const float* bias, int cout, void* y, void* relu_bits, int dtype,
                                          void* stream) {
    OCRK_REQUIRE(relu_bits && ocrk_conv3x3_fwd_relu_bits_supported(B, H, W, cin, cout, dtype),
                 "ocrk_conv3x3_fwd_relu_bits: B=%d H=%d W=%d %d->%d dtype=%d not covered", B, H, W, cin, cout, dtype);
    hipStream_t s = ocrk::as_stream(stream);
    const int st = ocrk::conv_rows_fwd_bits(x, B, H, W, cin, w_nk, bias, cout, y, relu_bits, s);
    if (st >= 0) return st;
    ocrk::GemmParams p = {};
    p.M = B * H * W; p.N = cout; p.K = 9 * cin; p.batch = 1;
    p.A = x; p.B = w_nk; p.ldb = 9 * cin;
    p.C = y; p.ldc = cout; p.c_bf16 = 1;
    p.bias = bias; p.relu = 1; p.alpha = 1.f;
    p.splits = 1; p.k_chunk = (int)ocrk::cdiv(p.K, 32) * 32;
    p.convH = H; p.convW = W; p.convC = cin;
    p.relu_bits = relu_bits;
    return ocrk::gemm(p, ocrk::A_IM2COL, ocrk::B_NK, dtype, s);
}

extern "C" int ocrk_conv3x3_bwd_data_bits_supported(int B, int H, int W, int cout, int cin, int dtype) {
    if (dtype != OCRK_BF16 || B < 1 || H < 1 || W < 1 || (int64_t)B * H * W >= (1ll << 31)) return 0;
    return ocrk::conv_rows_dgrad_bits_covers(B, H, W, cin, cout) || nt_bits_ok(cout, cin) ? 1 : 0;
}

extern "C" size_t ocrk_conv3x3_bwd_data_workspace_size(int B, int H, int W, int cin) {
    return ((size_t)bwd_data_tiles(B, H, W) * 2 * cin * sizeof(float) + 7) / 8 * 8 +
           (size_t)ocrk::SLAB_P * cin * sizeof(double);
}

// ocrk_conv3x3_bwd_data with the mask as the producer's bit mask (ocrk_conv3x3_fwd_relu_bits)
extern "C" int ocrk_conv3x3_bwd_data_bits(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin,
                                          void* dx, const void* relu_bits, float* dbias, int accumulate, void* ws,
                                          size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(relu_bits && ocrk_conv3x3_bwd_data_bits_supported(B, H, W, cout, cin, dtype),
                 "ocrk_conv3x3_bwd_data_bits: B=%d H=%d W=%d %d<-%d dtype=%d not covered", B, H, W, cin, cout, dtype);
    hipStream_t s = ocrk::as_stream(stream);
    if (!dbias) return bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, nullptr, nullptr, dtype, s, relu_bits);
    OCRK_REQUIRE(ws && ws_bytes >= ocrk_conv3x3_bwd_data_workspace_size(B, H, W, cin),
                 "ocrk_conv3x3_bwd_data_bits: workspace too small for the bias gradient");
    int st = bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, nullptr, (float*)ws, dtype, s, relu_bits);
    if (st) return st;
    const int tiles = (int)bwd_data_tiles(B, H, W);
    double* part = (double*)((char*)ws + ((size_t)tiles * 2 * cin * sizeof(float) + 7) / 8 * 8);
    return ocrk::slab_sum((const float*)ws, tiles, cin, part, nullptr, dbias, nullptr, cin, accumulate, s, 2 * cin);
}

extern "C" int ocrk_conv3x3_bwd_data(const void* dy, int B, int H, int W, int cout, const void* w_bwd,
                                     int cin, void* dx, const void* relu_mask, float* dbias, int accumulate,
                                     void* ws, size_t ws_bytes, int dtype, void* stream) {
    hipStream_t s = ocrk::as_stream(stream);
    if (!dbias) return bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, nullptr, dtype, s);
    OCRK_REQUIRE(ws && ws_bytes >= ocrk_conv3x3_bwd_data_workspace_size(B, H, W, cin),
                 "ocrk_conv3x3_bwd_data: workspace too small for the bias gradient");
    int st = bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, (float*)ws, dtype, s);
    if (st) return st;
    const int tiles = (int)bwd_data_tiles(B, H, W);
    double* part = (double*)((char*)ws + ((size_t)tiles * 2 * cin * sizeof(float) + 7) / 8 * 8);
    return ocrk::slab_sum((const float*)ws, tiles, cin, part, nullptr, dbias, nullptr, cin, accumulate, s, 2 * cin);
}

// The same with the bias-gradient partials left to the caller: `slab` gets the
// per-128-row-tile column (sum, M2) of the masked dx, [ocrk_conv_stats_tiles(B*H*W)]
// rows of 2*cin floats (sums in the first cin); ocrk_slab_sum(slab, tiles, cin,
// 2*cin, dbias, ...) on any stream ordered after this call gives the dbias of
// ocrk_conv3x3_bwd_data -- the same bits, off the data-gradient critical path.
// ocrk_conv3x3_bwd_data_bits with the bias-gradient reduction left to the caller (as _slab)
extern "C" int ocrk_conv3x3_bwd_data_bits_slab(const void* dy, int B, int H, int W, int cout, const void* w_bwd,
                                               int cin, void* dx, const void* relu_bits, float* slab, int dtype,
                                               void* stream) {
    OCRK_REQUIRE(slab && relu_bits && ocrk_conv3x3_bwd_data_bits_supported(B, H, W, cout, cin, dtype),
                 "ocrk_conv3x3_bwd_data_bits_slab: B=%d H=%d W=%d %d<-%d dtype=%d not covered (or no slab)", B, H, W,
                 cin, cout, dtype);
    return bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, nullptr, slab, dtype, ocrk::as_stream(stream), relu_bits);
}

extern "C" int ocrk_conv3x3_bwd_data_slab(const void* dy, int B, int H, int W, int cout, const void* w_bwd,
                                          int cin, void* dx, const void* relu_mask, float* slab, int dtype,
                                          void* stream) {
    OCRK_REQUIRE(slab, "ocrk_conv3x3_bwd_data_slab: slab is required");
    return bwd_data_run(dy, B, H, W, cout, w_bwd, cin, dx, relu_mask, slab, dtype, ocrk::as_stream(stream));
}

// Item cap of the 256 x 256 weight-gradient launches (OCRK_CONV_TN_ITEMS):
// they run on the side stream beside the main stream's BN backward and data
// gradients, whose kernels cannot share a CU with an item (VGPRs), so 192
// items (of 256 CUs) leave those 64 CUs. Same-box A/B of the step: 5.241-5.248
// ms vs 5.266-5.281 at 256 (one round on the chip); 224: 5.27, 160: 5.24-5.27.
static int conv_tn_items() {
    const int64_t v = ocrk::opt(ocrk::OPT_CONV_TN_ITEMS);
    return v >= 16 ? (int)v : 192;
}

static int wgrad_splits(int64_t M, int cin, int cout) {
    // enough partial tiles to cover the chip ~2x (the 256 x 256 ping-pong
    // engine: ~1x, one item per CU); each split >= 4096 pixels
    if (ocrk::gemm_pptn_covers(ocrk::A_IM2COL_T, 9 * cin, cout, cin)) {
        const int64_t tiles = ocrk::cdiv(9 * cin, 256) * ocrk::cdiv(cout, 256);
        return (int)std::max<int64_t>(1, std::min<int64_t>(conv_tn_items() / tiles, M / 2048));
    }
    int64_t tiles = ocrk::cdiv(9 * cin, 128) * ocrk::cdiv(cout, cout <= 32 ? 32 : (cout <= 64 ? 64 : 128));
    const int64_t iv = ocrk::opt(ocrk::OPT_CONV_TN4_ITEMS);
    const int items = iv >= 16 ? (int)iv : 512;
    int64_t want = ocrk::cdiv(items, tiles);
    int64_t maxs = std::max<int64_t>(1, M / 4096);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, maxs));
}

extern "C" size_t ocrk_conv3x3_wgrad_workspace_size(int B, int H, int W, int cin, int cout) {
    int64_t M = (int64_t)B * H * W;
    size_t ws = std::max(ocrk::gemm_splitk_ws_bytes(9 * cin, cout, 1, wgrad_splits(M, cin, cout)),
                         ocrk::conv_direct_wgrad_ws_bytes(B, H, W, cin, cout));
    if ((cin == 32 && cout == 32) || (cout == 64 && (cin == 32 || cin == 64)) ||
        (cout == 128 && (cin == 64 || cin == 128)) || (cout == 256 && (cin == 128 || cin == 256)))
        ws = std::max(ws, ocrk::conv_rows_wgrad_ws_bytes(B, cin, cout));
    return ws;
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
        int st = ocrk::conv_rows_wgrad(x, dy, B, H, W, cin, cout, dw, accumulate, ws, ws_bytes, ocrk::as_stream(stream));
        if (st >= 0) return st;
        st = ocrk::conv_direct_wgrad(x, dy, B, H, W, cin, cout, dw, accumulate, ws, ws_bytes, ocrk::as_stream(stream));
        if (st >= 0) return st;
    }
    return ocrk::gemm(p, ocrk::A_IM2COL_T, ocrk::B_KN, dtype, ocrk::as_stream(stream));
}
