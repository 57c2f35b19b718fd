// a3+a4: BatchNorm -> ReLU -> max-pool of the even conv layers
// (norm_layer src/weinman/model.py:118-123, conv_layer :105-107, pool_layer
// :111-116, pool8 :145-146).
//
// Forward (train): the conv epilogue leaves per-128-row-tile (sum, M2)
// partials; bn_finalize merges them (Chan, in double) into batch mean/invstd
// and the moving averages ([TF1] momentum 0.99, moving variance from the
// unbiased batch variance). bn_relu_pool applies BN + ReLU + pool in one pass
// (thread = one pooled pixel x 8 channels) and can write the last pool
// (pool8) straight into the time-major [T, B, C] feature layout the RNN reads
// (model.py:147 squeeze + :212 transpose folded away).
// Backward: the routed gradient ([TF1] MaxPoolGrad: first max of the
// window, ReLU mask) is re-derived from z, never stored as an argmax; a
// deterministic two-pass BN backward (partials -> ordered sum -> apply). For
// the path's pools both passes walk the pooling windows (bn_bwd_route_kernel;
// the apply pass repeats the walk instead of reading a staged gradient image).
#include <type_traits>

#include "common.h"
#include "reduce.h"

using ocrk::slab_sum;
using ocrk::SLAB_P;

// --------------------------------------------------------------- finalize
// Merge the per-tile (sum, M2) partials of the [tiles][2C] table in double:
// M2 of the union = sum(M2_b) + sum(s_b^2 / n_b) - S^2 / N (the between-tile
// term; exact in double at these magnitudes). Every row of the table holds
// all channels, so a block per channel would drag every cache line of the
// table through each of C CUs; instead pass 1 (bn_stats_partial_kernel)
// sums row ranges across all columns with row-contiguous loads, pass 2
// (bn_finalize_kernel, a block per channel) adds the ranges in a fixed tree
// order (deterministic) and finalizes.
constexpr int BN_PARTS = 256;
__global__ void __launch_bounds__(256)
bn_stats_partial_kernel(const float* __restrict__ stats, int tiles, int64_t M, int tile_rows, int C, int rpb,
                        double* __restrict__ part) {
    __shared__ double sacc[3 * 256];                    // [lanes][3][C] with lanes * C <= 256 ... see below
    const int NC = 2 * C;
    const int lanes = NC <= 256 ? 256 / NC : 1;         // table rows read at once
    const int full = (int)(M / tile_rows);
    const double inv_full = 1.0 / (double)tile_rows;
    const int t0 = blockIdx.x * rpb, t1 = min(tiles, t0 + rpb);
    double a[2] = {0, 0}, q[2] = {0, 0};
    const int lr = NC <= 256 ? threadIdx.x / NC : 0;
    const int j0 = NC <= 256 ? threadIdx.x % NC : threadIdx.x;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = j0 + 256 * h;
        if (j >= NC || (h == 1 && NC <= 256)) continue;
        for (int t = t0 + lr; t < t1; t += lanes) {
            const double v = stats[(int64_t)t * NC + j];
            a[h] += v;
            if (j < C) q[h] += v * v * (t < full ? inv_full : 1.0 / (double)(M - (int64_t)t * tile_rows));
        }
    }
    // lane partials -> shared [3][C] in lane order (lanes * NC == 256 when NC <= 256)
    for (int l = 0; l < lanes; ++l) {
        if (lr == l) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = j0 + 256 * h;
                if (j >= NC || (h == 1 && NC <= 256)) continue;
                if (j < C) {
                    sacc[j] = (l == 0 ? 0.0 : sacc[j]) + a[h];
                    sacc[C + j] = (l == 0 ? 0.0 : sacc[C + j]) + q[h];
                } else {
                    sacc[2 * C + (j - C)] = (l == 0 ? 0.0 : sacc[2 * C + (j - C)]) + a[h];
                }
            }
        }
        __syncthreads();
    }
    for (int k = threadIdx.x; k < 3 * C; k += 256) part[(int64_t)blockIdx.x * 3 * C + k] = sacc[k];
}

// mean / invstd (and the moving averages) of channel c from the merged sums:
// S = sum x, Q = sum_t s_t^2 / n_t, W2 = sum_t M2_t over nt values
__device__ __forceinline__ void bn_final_channel(int c, double S, double Q, double W2, double nt, float eps,
                                                 float momentum, float* __restrict__ mean_out,
                                                 float* __restrict__ invstd_out, float* __restrict__ moving_mean,
                                                 float* __restrict__ moving_var) {
    const double mu = S / nt;
    const double m2 = fmax(W2 + Q - S * mu, 0.0);
    const double var = m2 / nt;
    mean_out[c] = (float)mu;
    invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (moving_mean) {
        float dec = 1.f - momentum;
        double var_u = nt > 1 ? m2 / (nt - 1) : var;
        moving_mean[c] = moving_mean[c] - (moving_mean[c] - (float)mu) * dec;
        moving_var[c] = moving_var[c] - (moving_var[c] - (float)var_u) * dec;
    }
}

// MOMENTS: write the merged (S, Q, W2) and the count M to moments [3C + 1]
// instead of finalizing (the cross-rank form: the three sums and the count are
// additive over ranks, so one SUM all-reduce of the vector then
// bn_finalize_moments_kernel gives the statistics of the union of the batches)
template <bool MOMENTS>
__global__ void __launch_bounds__(256)
bn_finalize_kernel(const double* __restrict__ part, int nparts, int64_t M, int C, float eps, float momentum,
                   float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ moving_mean,
                   float* __restrict__ moving_var, double* __restrict__ moments) {
    __shared__ double ss[256], sq[256], sw[256];
    const int c = blockIdx.x;
    double S = 0, Q = 0, W2 = 0;
    for (int b = threadIdx.x; b < nparts; b += 256) {
        S += part[(int64_t)b * 3 * C + c];
        Q += part[(int64_t)b * 3 * C + C + c];
        W2 += part[(int64_t)b * 3 * C + 2 * C + c];
    }
    ss[threadIdx.x] = S; sq[threadIdx.x] = Q; sw[threadIdx.x] = W2;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            ss[threadIdx.x] += ss[threadIdx.x + s];
            sq[threadIdx.x] += sq[threadIdx.x + s];
            sw[threadIdx.x] += sw[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if constexpr (MOMENTS) {
            moments[c] = ss[0];
            moments[C + c] = sq[0];
            moments[2 * C + c] = sw[0];
            if (c == 0) moments[3 * C] = (double)M;
        } else {
            bn_final_channel(c, ss[0], sq[0], sw[0], (double)M, eps, momentum, mean_out, invstd_out, moving_mean,
                             moving_var);
        }
    }
}

__global__ void __launch_bounds__(256)
bn_finalize_moments_kernel(const double* __restrict__ moments, int C, float eps, float momentum,
                           float* __restrict__ mean_out, float* __restrict__ invstd_out,
                           float* __restrict__ moving_mean, float* __restrict__ moving_var) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < C)
        bn_final_channel(c, moments[c], moments[C + c], moments[2 * C + c], moments[3 * C], eps, momentum, mean_out,
                         invstd_out, moving_mean, moving_var);
}

// the apply pass's dsum from the cross-rank sums: the kernels scale dsum by
// 1 / (this launch's pixels), so dsum_ws = dsum * pixels / (all ranks' pixels)
__global__ void bn_dsum_scale_kernel(const float* __restrict__ dsum, const double* __restrict__ count, int64_t npix,
                                     int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)((double)dsum[i] * (double)npix / count[0]);
}

__global__ void bn_infer_params_kernel(const float* mm, const float* mv, int C, float eps,
                                       float* mean, float* invstd) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) {
        mean[c] = mm[c];
        invstd[c] = (float)(1.0 / sqrt((double)mv[c] + (double)eps));
    }
}

// ---------------------------------------------------- BN + ReLU + pool fwd
template <typename T>
__global__ void __launch_bounds__(256)
bn_relu_pool_fwd_kernel(const T* __restrict__ z, int B, int H, int W, int C,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        const float* __restrict__ gamma, const float* __restrict__ beta, int kh, int kw,
                        int sh, int sw, T* __restrict__ out, int time_major) {
    const int Ho = (H - kh) / sh + 1, Wo = (W - kw) / sw + 1, G = C / 8;
    const int64_t items = (int64_t)B * Ho * Wo * G;
    for (int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x; it < items; it += (int64_t)gridDim.x * 256) {
        int g = (int)(it % G);
        int64_t op = it / G;
        int wo = (int)(op % Wo);
        int64_t t = op / Wo;
        int ho = (int)(t % Ho), b = (int)(t / Ho);
        int c0 = g * 8;
        float sc[8], sf[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            sc[i] = gamma[c0 + i] * invstd[c0 + i];
            sf[i] = beta[c0 + i] - mean[c0 + i] * sc[i];
        }
        F8 best;
#pragma unroll
        for (int i = 0; i < 8; ++i) best.v[i] = -INFINITY;
        for (int dh = 0; dh < kh; ++dh)
            for (int dw = 0; dw < kw; ++dw) {
                F8 v = load8(z + (((int64_t)b * H + ho * sh + dh) * W + wo * sw + dw) * C + c0);
#pragma unroll
                for (int i = 0; i < 8; ++i) best.v[i] = fmaxf(best.v[i], fmaxf(fmaf(v.v[i], sc[i], sf[i]), 0.f));
            }
        int64_t o = time_major ? (((int64_t)wo * B + b) * Ho + ho) * C + c0
                               : (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
        store8(out + o, best);
    }
}

// ----------------------------------------------------------- backward
// Gradient arriving at pre-pool pixel (h, w) for 8 channels: sum of dp over
// the windows whose first maximum is (h, w), masked by ReLU.
template <typename T>
__device__ __forceinline__ void routed_grad(const T* __restrict__ z, const T* __restrict__ dp, int B, int H,
                                            int W, int C, int b, int h, int w, int c0, int kh, int kw,
                                            int sh, int sw, int dp_time_major, const float* sc, const float* sf,
                                            float* da, float* zc) {
    const int Ho = (H - kh) / sh + 1, Wo = (W - kw) / sw + 1;
    F8 me = load8(z + (((int64_t)b * H + h) * W + w) * C + c0);
    float a_me[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        zc[i] = me.v[i];
        a_me[i] = fmaf(me.v[i], sc[i], sf[i]);
        da[i] = 0.f;
    }
    int ho_lo = max(0, (h - kh + sh) / sh), ho_hi = min(Ho - 1, h / sh);
    int wo_lo = max(0, (w - kw + sw) / sw), wo_hi = min(Wo - 1, w / sw);
    if (h - kh + 1 < 0) ho_lo = 0;
    if (w - kw + 1 < 0) wo_lo = 0;
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
        for (int wo = wo_lo; wo <= wo_hi; ++wo) {
            if (ho * sh > h || ho * sh + kh <= h || wo * sw > w || wo * sw + kw <= w) continue;
            // first max over the window (row-major scan) of relu(bn(z))
            float best[8];
            int arg[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; arg[i] = -1; }
            for (int dh = 0; dh < kh; ++dh)
                for (int dw = 0; dw < kw; ++dw) {
                    F8 v = load8(z + (((int64_t)b * H + ho * sh + dh) * W + wo * sw + dw) * C + c0);
                    int pos = dh * kw + dw;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        float y = fmaxf(fmaf(v.v[i], sc[i], sf[i]), 0.f);
                        if (y > best[i]) { best[i] = y; arg[i] = pos; }
                    }
                }
            int mypos = (h - ho * sh) * kw + (w - wo * sw);
            int64_t o = dp_time_major ? (((int64_t)wo * B + b) * Ho + ho) * C + c0
                                      : (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
            F8 g = load8(dp + o);
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (arg[i] == mypos) da[i] += g.v[i];
        }
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (!(a_me[i] > 0.f)) da[i] = 0.f;
}

// pass 1: route the pooled gradient (first max of each window, ReLU mask) to
// the pre-pool pixels ONCE, store it (da is dp's value or 0: exact in the
// compute dtype) for pass 2, and reduce per-block partial sums of da and
// da*xhat per channel.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_kernel(const T* __restrict__ z, const T* __restrict__ dp, int B, int H, int W, int C,
                     const float* __restrict__ mean, const float* __restrict__ invstd,
                     const float* __restrict__ gamma, const float* __restrict__ beta, int kh, int kw,
                     int sh, int sw, int dp_time_major, int items_per_block, float* __restrict__ slab,
                     T* __restrict__ da_out) {
    __shared__ float red[256][17];
    const int G = C / 8;
    const int items = B * H * W * G;                    // < 2^31 (checked by the caller)
    const int g = threadIdx.x % G;       // fixed: items_per_block % 256 == 0 and 256 % G == 0
    const int c0 = g * 8;
    float sc[8], sf[8], mu[8], is[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        is[i] = invstd[c0 + i];
        mu[i] = mean[c0 + i];
        sc[i] = gamma[c0 + i] * is[i];
        sf[i] = beta[c0 + i] - mu[i] * sc[i];
    }
    float s1[8], s2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s1[i] = s2[i] = 0.f;
    const int i0 = blockIdx.x * items_per_block;
    const int i1 = min(items, i0 + items_per_block);
    for (int it = i0 + threadIdx.x; it < i1; it += 256) {
        const int px = it / G;
        const int w = px % W, t = px / W;
        const int h = t % H, b = t / H;
        float da[8], zc[8];
        routed_grad(z, dp, B, H, W, C, b, h, w, c0, kh, kw, sh, sw, dp_time_major, sc, sf, da, zc);
        F8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s1[i] += da[i];
            s2[i] += da[i] * ((zc[i] - mu[i]) * is[i]);
            o.v[i] = da[i];
        }
        store8(da_out + (int64_t)px * C + c0, o);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) { red[threadIdx.x][i] = s1[i]; red[threadIdx.x][8 + i] = s2[i]; }
    __syncthreads();
    for (int o = threadIdx.x; o < 2 * C; o += 256) {
        int which = o / C, c = o % C, gg = c / 8, ci = c % 8;
        float s = 0.f;
        for (int q = gg; q < 256; q += G) s += red[q][which * 8 + ci];
        slab[(int64_t)blockIdx.x * 2 * C + o] = s;
    }
}

// N consecutive channels of one pixel (N = 4 or 8): raw bits as loaded, widened at use
template <typename T, int N> struct RawN;
template <> struct RawN<bf16, 8> { uint4 q; };
template <> struct RawN<bf16, 4> { uint2 q; };
template <> struct RawN<float, 8> { float4 a, b; };
template <> struct RawN<float, 4> { float4 a; };
template <typename T, int N>
__device__ __forceinline__ RawN<T, N> load_raw(const T* p) {
    RawN<T, N> r;
    if constexpr (std::is_same<T, bf16>::value) {
        if constexpr (N == 8) r.q = *reinterpret_cast<const uint4*>(p);
        else r.q = *reinterpret_cast<const uint2*>(p);
    } else {
        r.a = reinterpret_cast<const float4*>(p)[0];
        if constexpr (N == 8) r.b = reinterpret_cast<const float4*>(p)[1];
    }
    return r;
}
template <typename T, int N>
__device__ __forceinline__ void widen(const RawN<T, N>& r, float (&f)[N]) {
    if constexpr (std::is_same<T, bf16>::value) {
        const unsigned* w = reinterpret_cast<const unsigned*>(&r.q);
#pragma unroll
        for (int i = 0; i < N / 2; ++i) {
            f[2 * i] = __uint_as_float(w[i] << 16);
            f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    } else {
        f[0] = r.a.x; f[1] = r.a.y; f[2] = r.a.z; f[3] = r.a.w;
        if constexpr (N == 8) { f[4] = r.b.x; f[5] = r.b.y; f[6] = r.b.z; f[7] = r.b.w; }
    }
}
template <typename T, int N>
__device__ __forceinline__ void load_n(const T* p, float (&f)[N]) { widen<T, N>(load_raw<T, N>(p), f); }
template <typename T, int N>
__device__ __forceinline__ void store_n(T* p, const float (&f)[N]) {
    if constexpr (std::is_same<T, bf16>::value) {
        unsigned w[N / 2];
#pragma unroll
        for (int i = 0; i < N / 2; ++i) {
            union { bf16 e[2]; unsigned u; } c;
            c.e[0] = (bf16)f[2 * i];
            c.e[1] = (bf16)f[2 * i + 1];
            w[i] = c.u;
        }
        if constexpr (N == 8) *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
        else *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
    } else {
        reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
        if constexpr (N == 8) reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
    }
}

// pass 1, window-centric (the pools of the path: KH == stride_h, SW <= KW).
// Thread = (image b, pooled row ho, SEG consecutive pooled columns, NCH
// channels). It streams the KH pre-pool rows of its column range left to
// right through a KW-column register window, evaluates each pooling window
// ONCE ([TF1] first max, row-major scan of relu(bn(z))), adds dp to the
// winner's register accumulator and retires a column (ReLU mask, store, sums)
// as it leaves the window: every z element is read once, instead of once per
// covering window plus once for itself as in bn_bwd_reduce_kernel. The
// PRE = (KW-1)/SW windows left of the range that still reach into it are
// re-evaluated (their own columns are not retired here). Rows below the last
// pooling window, and columns right of it, receive no gradient: zeros.
// NCH = 4 halves the thread's registers (~110 instead of ~205 VGPRs at 8: two
// waves per SIMD made the serial walk latency-bound) at 8-B accesses.
//
// APPLY = pass 2 of the same window walk: instead of staging the routed
// gradient da for a streaming apply pass (2 x |z| more bytes), the walk is
// repeated and each retired column goes straight to
// dz = gamma*invstd*(da - sum(da)/n - xhat*sum(da*xhat)/n), its per-block
// column sums (the conv bias gradient) into `slab` (C per block). Pixels no
// window covers (rows below the last window) have da = 0 but a non-zero dz.
// DG (with APPLY): also the dgamma partials sum da * xhat from z (slab rows of 2C:
// [bias | dgamma]) -- the pooled-output pass 1 recovers xhat only to the stored
// output's precision, so dgamma itself is summed here, from z as the walk's pass 1 does.
template <typename T, int KH, int KW, int SW, int SEG, bool APPLY = false, int NCH = 8, bool DG = false>
__global__ void __launch_bounds__(256)
bn_bwd_route_kernel(const T* __restrict__ z, const T* __restrict__ dp, int B, int H, int W, int C,
                    const float* __restrict__ mean, const float* __restrict__ invstd,
                    const float* __restrict__ gamma, const float* __restrict__ beta, int dp_time_major,
                    int nseg, int tasks_per_block, float* __restrict__ slab, T* __restrict__ da_out,
                    const float* __restrict__ dsum = nullptr) {
    static_assert(SW >= 1 && SW <= KW, "stride <= window");
    static_assert(NCH == 4 || NCH == 8, "4 or 8 channels per thread");
    constexpr int PRE = (KW - 1) / SW;
    __shared__ float red[256][2 * NCH + 1];
    const int G = C / NCH;
    const int Ho = (H - KH) / KH + 1, Wo = (W - KW) / SW + 1;
    const int tasks = B * Ho * nseg * G;
    const int g = threadIdx.x % G;
    const int c0 = g * NCH;
    float sc[NCH], sf[NCH], mu[NCH], is[NCH], am[NCH], bm[NCH];
    const float inv_n = 1.f / (float)((int64_t)B * H * W);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        is[i] = invstd[c0 + i];
        mu[i] = mean[c0 + i];
        sc[i] = gamma[c0 + i] * is[i];
        sf[i] = beta[c0 + i] - mu[i] * sc[i];
        am[i] = APPLY ? dsum[c0 + i] * inv_n : 0.f;
        bm[i] = APPLY ? dsum[C + c0 + i] * inv_n : 0.f;
    }
    float s1[NCH], s2[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) s1[i] = s2[i] = 0.f;
    const int t0 = blockIdx.x * tasks_per_block;
    const int t1 = min(tasks, t0 + tasks_per_block);
    for (int task = t0 + threadIdx.x; task < t1; task += 256) {
        int rest = task / G;
        const int seg = rest % nseg;
        rest /= nseg;
        const int ho = rest % Ho, b = rest / Ho;
        const int wa = seg * SEG, wb = min(Wo, wa + SEG);
        const int own0 = wa * SW, own1 = (seg == nseg - 1) ? W : wb * SW;
        const bool tail_rows = (ho == Ho - 1) && (Ho * KH < H);
        const T* zrow = z + (((int64_t)b * H + ho * KH) * W) * C + c0;
        T* drow = da_out + (((int64_t)b * H + ho * KH) * W) * C + c0;

        float zr[KW][KH][NCH], dr[KW][KH][NCH];
        auto retire = [&](int x, const float (&zc)[KH][NCH], const float (&dc)[KH][NCH]) {
            if (x < own0 || x >= own1) return;
#pragma unroll
            for (int dh = 0; dh < KH; ++dh) {
                float o[NCH];
#pragma unroll
                for (int i = 0; i < NCH; ++i) {
                    const float d = fmaf(zc[dh][i], sc[i], sf[i]) > 0.f ? dc[dh][i] : 0.f;
                    const float xh = (zc[dh][i] - mu[i]) * is[i];
                    if constexpr (APPLY) {
                        o[i] = sc[i] * (d - am[i] - xh * bm[i]);
                        s1[i] += o[i];
                        if constexpr (DG) s2[i] += d * xh;
                    } else {
                        s1[i] += d;
                        s2[i] += d * xh;
                        o[i] = d;
                    }
                }
                if (APPLY || da_out) store_n<T, NCH>(drow + ((int64_t)dh * W + x) * C, o);
            }
            if (tail_rows && (APPLY || da_out)) {
                for (int h = Ho * KH; h < H; ++h) {
                    float o[NCH];
                    if constexpr (APPLY) {
                        float zt[NCH];
                        load_n<T, NCH>(z + (((int64_t)b * H + h) * W + x) * C + c0, zt);
#pragma unroll
                        for (int i = 0; i < NCH; ++i) {
                            o[i] = sc[i] * (-am[i] - (zt[i] - mu[i]) * is[i] * bm[i]);
                            s1[i] += o[i];
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < NCH; ++i) o[i] = 0.f;
                    }
                    store_n<T, NCH>(da_out + (((int64_t)b * H + h) * W + x) * C + c0, o);
                }
            }
        };
        const int wfirst = max(0, wa - PRE);
#pragma unroll
        for (int j = 0; j < KW; ++j)
#pragma unroll
            for (int dh = 0; dh < KH; ++dh) {
                load_n<T, NCH>(zrow + ((int64_t)dh * W + wfirst * SW + j) * C, zr[j][dh]);
#pragma unroll
                for (int i = 0; i < NCH; ++i) dr[j][dh][i] = 0.f;
            }
        auto dp_off = [&](int wo) {
            return dp_time_major ? (((int64_t)wo * B + b) * Ho + ho) * C + c0
                                 : (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
        };
        // the pooled gradient is prefetched a window ahead like the z columns: the
        // window's compute then waits only for loads issued a window earlier (in-order
        // vmcnt), not for the loads just issued (a same-window dp load behind the
        // prefetch made every window wait vmcnt(0))
        float gp[NCH];
        load_n<T, NCH>(dp + dp_off(wfirst), gp);
        for (int wo = wfirst; wo < wb; ++wo) {
            const int x0 = wo * SW;
            // next window's pooled gradient and new columns in flight first, kept raw
            // (converted when they enter the window, after this window's work)
            RawN<T, NCH> nz[SW][KH];
            RawN<T, NCH> gpn;
            const bool more = wo + 1 < wb;
            if (more) {
                gpn = load_raw<T, NCH>(dp + dp_off(wo + 1));
#pragma unroll
                for (int j = 0; j < SW; ++j)
#pragma unroll
                    for (int dh = 0; dh < KH; ++dh)
                        nz[j][dh] = load_raw<T, NCH>(zrow + ((int64_t)dh * W + x0 + KW + j) * C);
            }
#pragma unroll
            for (int i = 0; i < NCH; ++i) {
                float best = -INFINITY;
                int arg = -1;
#pragma unroll
                for (int dh = 0; dh < KH; ++dh)
#pragma unroll
                    for (int j = 0; j < KW; ++j) {
                        const float y = fmaxf(fmaf(zr[j][dh][i], sc[i], sf[i]), 0.f);
                        if (y > best) { best = y; arg = dh * KW + j; }
                    }
#pragma unroll
                for (int dh = 0; dh < KH; ++dh)
#pragma unroll
                    for (int j = 0; j < KW; ++j)
                        if (arg == dh * KW + j) dr[j][dh][i] += gp[i];
            }
            // the first SW columns leave the window
#pragma unroll
            for (int j = 0; j < SW; ++j) retire(x0 + j, zr[j], dr[j]);
            if (!more) break;
            widen<T, NCH>(gpn, gp);
#pragma unroll
            for (int j = 0; j + SW < KW; ++j)
#pragma unroll
                for (int dh = 0; dh < KH; ++dh)
#pragma unroll
                    for (int i = 0; i < NCH; ++i) { zr[j][dh][i] = zr[j + SW][dh][i]; dr[j][dh][i] = dr[j + SW][dh][i]; }
#pragma unroll
            for (int j = 0; j < SW; ++j)
#pragma unroll
                for (int dh = 0; dh < KH; ++dh) {
                    widen<T, NCH>(nz[j][dh], zr[KW - SW + j][dh]);
#pragma unroll
                    for (int i = 0; i < NCH; ++i) dr[KW - SW + j][dh][i] = 0.f;
                }
        }
        // columns still in the last window, then the uncovered ones on the right
        const int xl = (wb - 1) * SW;
#pragma unroll
        for (int j = SW; j < KW; ++j) retire(xl + j, zr[j], dr[j]);
        for (int x = max(xl + KW, own0); x < own1; ++x) {
            float zc[KH][NCH], dc[KH][NCH];                 // no gradient (z matters only for APPLY's dz)
#pragma unroll
            for (int dh = 0; dh < KH; ++dh) {
                if constexpr (APPLY) {
                    load_n<T, NCH>(zrow + ((int64_t)dh * W + x) * C, zc[dh]);
                } else {
#pragma unroll
                    for (int i = 0; i < NCH; ++i) zc[dh][i] = 0.f;
                }
#pragma unroll
                for (int i = 0; i < NCH; ++i) dc[dh][i] = 0.f;
            }
            retire(x, zc, dc);
        }
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) { red[threadIdx.x][i] = s1[i]; red[threadIdx.x][NCH + i] = s2[i]; }
    __syncthreads();
    const int nout = (APPLY && !DG) ? C : 2 * C;
    for (int o = threadIdx.x; o < nout; o += 256) {
        int which = o / C, c = o % C, gg = c / NCH, ci = c % NCH;
        float s = 0.f;
        for (int q = gg; q < 256; q += G) s += red[q][which * NCH + ci];
        slab[(int64_t)blockIdx.x * nout + o] = s;
    }
}


// pass 1 from the forward's pooled output p (its saved result, the next layer's
// input) instead of z: the routed gradient da is dp at each window's first max when
// that max is ReLU-active (p > 0), and there xhat = (p - beta) / gamma, so
//   sum da = sum_{p > 0} dp,   sum da * xhat = sum_{p > 0} dp * (p - beta) / gamma
// over the POOLED elements -- a stream over p and dp (1/4 of z's bytes for the 2x2
// pools, 1/2 and 1/3 for the others) instead of the window walk over z. xhat is
// recovered from the stored p to |p| ulp / |gamma| ~ (|beta| / |gamma| + |xhat|) ulp,
// where the walk's (z - mean) * invstd carries (|mean| * invstd + |xhat|) ulp: a
// channel whose |beta| / |gamma| exceeds max(4, |mean| * invstd) (gamma = 0 included)
// is ill-conditioned for the recovery, and the 8-channel group holding it evaluates its
// windows from z instead ([TF1] first max of relu(bn(z)), row-major scan, exactly the
// walk's per-window terms) -- decided per channel on the device, no host sync.
// Per-block [s1 | s2] rows of 2C, the window walk's slab format. Thread = 8
// channels, 4 items in flight.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_pooled_sums_kernel(const T* __restrict__ p, const T* __restrict__ dp, int64_t items, int C,
                          const float* __restrict__ gamma, const float* __restrict__ beta,
                          const float* __restrict__ mean, const float* __restrict__ invstd, const T* __restrict__ z,
                          int B, int H, int W, int kh, int kw, int sh, int sw, int time_major, int items_per_block,
                          float* __restrict__ slab) {
    __shared__ float red[256][17];
    const int G = C / 8;
    const int g = threadIdx.x % G, c0 = 8 * g;     // fixed: items_per_block % 256 == 0, 256 % G == 0
    float rg[8], bt[8], s1[8], s2[8];
    bool from_z = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float ga = gamma[c0 + i], be = beta[c0 + i];
        const float cz = fabsf(mean[c0 + i]) * invstd[c0 + i];
        from_z |= !(fabsf(be) <= fmaxf(4.f, cz) * fabsf(ga));       // gamma = 0 or NaN: z
        rg[i] = ga != 0.f ? 1.f / ga : 0.f;
        bt[i] = be;
        s1[i] = s2[i] = 0.f;
    }
    const int64_t i0 = (int64_t)blockIdx.x * items_per_block;
    const int64_t i1 = min(items, i0 + items_per_block);
    if (from_z) {
        // the z form for this channel group: each pooled element's window re-evaluated
        const int Ho = (H - kh) / sh + 1, Wo = (W - kw) / sw + 1;
        float sc[8], sf[8], mu[8], is[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            is[i] = invstd[c0 + i];
            mu[i] = mean[c0 + i];
            sc[i] = gamma[c0 + i] * is[i];
            sf[i] = beta[c0 + i] - mu[i] * sc[i];
        }
        for (int64_t it = i0 + threadIdx.x; it < i1; it += 256) {
            const int64_t pix = it / G;
            int b, ho, wo;
            if (time_major) {                       // [Wo][B][Ho][C]
                ho = (int)(pix % Ho);
                const int64_t r = pix / Ho;
                b = (int)(r % B);
                wo = (int)(r / B);
            } else {                                // [B][Ho][Wo][C]
                wo = (int)(pix % Wo);
                const int64_t r = pix / Wo;
                ho = (int)(r % Ho);
                b = (int)(r / Ho);
            }
            float best[8], zb[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; zb[i] = 0.f; }
            for (int dh = 0; dh < kh; ++dh)
                for (int dw = 0; dw < kw; ++dw) {
                    const F8 v = load8(z + (((int64_t)b * H + ho * sh + dh) * W + wo * sw + dw) * C + c0);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float y = fmaxf(fmaf(v.v[i], sc[i], sf[i]), 0.f);
                        if (y > best[i]) { best[i] = y; zb[i] = v.v[i]; }
                    }
                }
            const F8 dv = load8(dp + it * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float d = best[i] > 0.f ? dv.v[i] : 0.f;
                s1[i] += d;
                s2[i] += d * ((zb[i] - mu[i]) * is[i]);
            }
        }
    } else {
        constexpr int U = 4;
        for (int64_t it = i0 + threadIdx.x; it < i1; it += 256 * U) {
            Pend8<T> pr[U], dr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = min(it + 256 * u, i1 - 1);       // clamped (a fixed load count)
                pr[u] = load_pend8(p + q * 8);
                dr[u] = load_pend8(dp + q * 8);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (it + 256 * u >= i1) break;
                const F8 pv = cvt8(pr[u]), dv = cvt8(dr[u]);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float d = pv.v[i] > 0.f ? dv.v[i] : 0.f;
                    s1[i] += d;
                    s2[i] += d * ((pv.v[i] - bt[i]) * rg[i]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) { red[threadIdx.x][i] = s1[i]; red[threadIdx.x][8 + i] = s2[i]; }
    __syncthreads();
    for (int o = threadIdx.x; o < 2 * C; o += 256) {
        const int which = o / C, c = o % C, gg = c / 8, ci = c % 8;
        float s = 0.f;
        for (int q = gg; q < 256; q += G) s += red[q][which * 8 + ci];
        slab[(int64_t)blockIdx.x * 2 * C + o] = s;
    }
}

// pass 2 (streaming): dz = gamma*invstd*(da - sum(da)/n - xhat*sum(da*xhat)/n),
// plus per-block partial column sums of dz -- the gradient of the conv bias
// in front of the BN (fused here instead of a separate pass over dz).
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(const T* __restrict__ z, const T* __restrict__ da_in, int npix, int C,
                    const float* __restrict__ mean, const float* __restrict__ invstd,
                    const float* __restrict__ gamma, const float* __restrict__ dsum, int items_per_block,
                    T* __restrict__ dz, float* __restrict__ bslab) {
    __shared__ float red[256][9];
    const int G = C / 8;
    const int items = npix * G;
    const int g = threadIdx.x % G, c0 = g * 8;
    const float inv_n = 1.f / (float)npix;
    float sc[8], mu[8], is[8], a[8], bb[8], cs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = c0 + i;
        is[i] = invstd[c];
        mu[i] = mean[c];
        sc[i] = gamma[c] * is[i];
        a[i] = dsum[c] * inv_n;
        bb[i] = dsum[C + c] * inv_n;
        cs[i] = 0.f;
    }
    const int i0 = blockIdx.x * items_per_block;
    const int i1 = min(items, i0 + items_per_block);
    for (int it = i0 + threadIdx.x; it < i1; it += 256) {
        const int64_t off = (int64_t)(it / G) * C + c0;
        const F8 zz = load8(z + off), dd = load8(da_in + off);
        F8 out;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float xhat = (zz.v[i] - mu[i]) * is[i];
            out.v[i] = sc[i] * (dd.v[i] - a[i] - xhat * bb[i]);
            cs[i] += out.v[i];
        }
        store8(dz + off, out);
    }
    if (!bslab) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) red[threadIdx.x][i] = cs[i];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        const int gg = c / 8, ci = c % 8;
        float s = 0.f;
        for (int q = gg; q < 256; q += G) s += red[q][ci];
        bslab[(int64_t)blockIdx.x * C + c] = s;
    }
}

// ------------------------------------------------------------------ C ABI
extern "C" size_t ocrk_bn_finalize_workspace_size(int tiles, int C) {
    return (size_t)std::min(BN_PARTS, std::max(1, tiles)) * 3 * C * sizeof(double);
}

extern "C" int ocrk_bn_finalize_tiles(const float* stats, int tiles, int tile_rows, int64_t M, int C, float eps,
                                      float momentum, float* mean, float* invstd, float* moving_mean,
                                      float* moving_var, void* ws, size_t ws_bytes, void* stream);

extern "C" int ocrk_bn_finalize(const float* stats, int tiles, int64_t M, int C, float eps, float momentum,
                                float* mean, float* invstd, float* moving_mean, float* moving_var, void* ws,
                                size_t ws_bytes, void* stream) {
    return ocrk_bn_finalize_tiles(stats, tiles, 128, M, C, eps, momentum, mean, invstd, moving_mean, moving_var, ws,
                                  ws_bytes, stream);
}

extern "C" int ocrk_bn_finalize_tiles(const float* stats, int tiles, int tile_rows, int64_t M, int C, float eps,
                                      float momentum, float* mean, float* invstd, float* moving_mean,
                                      float* moving_var, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(tiles >= 1 && C >= 1 && C <= 256 && M >= 1 && tile_rows >= 1 &&
                 (int64_t)(tiles - 1) * tile_rows < M && (int64_t)tiles * tile_rows >= M,
                 "ocrk_bn_finalize: bad sizes");
    OCRK_REQUIRE(ws && ws_bytes >= ocrk_bn_finalize_workspace_size(tiles, C), "ocrk_bn_finalize: workspace too small");
    hipStream_t s = ocrk::as_stream(stream);
    const int np0 = std::min(BN_PARTS, tiles);
    const int rpb = (tiles + np0 - 1) / np0;
    const int np = (tiles + rpb - 1) / rpb;
    bn_stats_partial_kernel<<<np, 256, 0, s>>>(stats, tiles, M, tile_rows, C, rpb, (double*)ws);
    int st = ocrk::launch_status("ocrk_bn_finalize partial sums");
    if (st) return st;
    bn_finalize_kernel<false><<<C, 256, 0, s>>>((const double*)ws, np, M, C, eps, momentum, mean, invstd,
                                                moving_mean, moving_var, nullptr);
    return ocrk::launch_status("ocrk_bn_finalize");
}

extern "C" int ocrk_bn_moments(const float* stats, int tiles, int tile_rows, int64_t M, int C, double* moments,
                               void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(tiles >= 1 && C >= 1 && C <= 256 && M >= 1 && tile_rows >= 1 &&
                 (int64_t)(tiles - 1) * tile_rows < M && (int64_t)tiles * tile_rows >= M,
                 "ocrk_bn_moments: bad sizes");
    OCRK_REQUIRE(moments, "ocrk_bn_moments: moments is required");
    OCRK_REQUIRE(ws && ws_bytes >= ocrk_bn_finalize_workspace_size(tiles, C), "ocrk_bn_moments: workspace too small");
    hipStream_t s = ocrk::as_stream(stream);
    const int np0 = std::min(BN_PARTS, tiles);
    const int rpb = (tiles + np0 - 1) / np0;
    const int np = (tiles + rpb - 1) / rpb;
    bn_stats_partial_kernel<<<np, 256, 0, s>>>(stats, tiles, M, tile_rows, C, rpb, (double*)ws);
    int st = ocrk::launch_status("ocrk_bn_moments partial sums");
    if (st) return st;
    bn_finalize_kernel<true><<<C, 256, 0, s>>>((const double*)ws, np, M, C, 0.f, 0.f, nullptr, nullptr, nullptr,
                                               nullptr, moments);
    return ocrk::launch_status("ocrk_bn_moments");
}

extern "C" int ocrk_bn_finalize_moments(const double* moments, int C, float eps, float momentum, float* mean,
                                        float* invstd, float* moving_mean, float* moving_var, void* stream) {
    OCRK_REQUIRE(moments && C >= 1 && C <= 256, "ocrk_bn_finalize_moments: bad arguments");
    bn_finalize_moments_kernel<<<(C + 255) / 256, 256, 0, ocrk::as_stream(stream)>>>(moments, C, eps, momentum, mean,
                                                                                    invstd, moving_mean, moving_var);
    return ocrk::launch_status("ocrk_bn_finalize_moments");
}

extern "C" int ocrk_bn_infer_params(const float* moving_mean, const float* moving_var, int C, float eps,
                                    float* mean, float* invstd, void* stream) {
    bn_infer_params_kernel<<<(C + 255) / 256, 256, 0, ocrk::as_stream(stream)>>>(moving_mean, moving_var, C,
                                                                               eps, mean, invstd);
    return ocrk::launch_status("ocrk_bn_infer_params");
}

static unsigned grid_for(int64_t items) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ocrk::cdiv(items, 256), 8192)); }

extern "C" int ocrk_bn_relu_pool_fwd(const void* z, int B, int H, int W, int C, const float* mean,
                                     const float* invstd, const float* gamma, const float* beta, int kh,
                                     int kw, int sh, int sw, void* out, int time_major, int dtype,
                                     void* stream) {
    OCRK_REQUIRE(C % 8 == 0 && H >= kh && W >= kw, "ocrk_bn_relu_pool_fwd: bad shape");
    OCRK_REQUIRE(!time_major || (H - kh) / sh + 1 == 1, "ocrk_bn_relu_pool_fwd: time-major output needs Ho == 1");
    int64_t items = (int64_t)B * ((H - kh) / sh + 1) * ((W - kw) / sw + 1) * (C / 8);
    if (items == 0) return OCRK_OK;
    hipStream_t s = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16)
        bn_relu_pool_fwd_kernel<bf16><<<grid_for(items), 256, 0, s>>>((const bf16*)z, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, (bf16*)out, time_major);
    else
        bn_relu_pool_fwd_kernel<float><<<grid_for(items), 256, 0, s>>>((const float*)z, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, (float*)out, time_major);
    return ocrk::launch_status("ocrk_bn_relu_pool_fwd");
}

// pass-1 blocks (= rows of the partial-sum slab the ordered column sums walk on the
// critical path): at most OCRK_BN_BWD_BLOCKS (default 2048)
static int64_t bn_bwd_blocks(int64_t items) {
    const int64_t v = ocrk::opt(ocrk::OPT_BN_BWD_BLOCKS);
    const int64_t cap = v >= 64 && v <= 8192 ? v : 2048;
    return std::max<int64_t>(1, std::min<int64_t>(cap, ocrk::cdiv(items, 256 * 8)));
}
static int64_t bn_bwd_ipb(int64_t items, int64_t nb) { return ocrk::cdiv(ocrk::cdiv(items, nb), 256) * 256; }

// Window-centric pass 1 covers the path's pools (2x2/[2,2], 2x2/[2,1],
// [3,1]/[3,1]); 0 = use the pixel-centric kernel. OCRK_BN_ROUTE=0 disables it.
// pooled columns per thread of the window walk (option BN_ROUTE_SEG: 4, 8 or 16) and
// channels per thread (BN_ROUTE_NCH: 4 or 8)
static int bn_route_seg() {
    const int64_t v = ocrk::opt(ocrk::OPT_BN_ROUTE_SEG);
    return (v == 4 || v == 16) ? (int)v : 8;
}
static int bn_route_nch() { return ocrk::opt(ocrk::OPT_BN_ROUTE_NCH) == 8 ? 8 : 4; }

template <typename T, int KH, int KW, int SW, bool APPLY, int NCH, bool DG, typename... A>
static void launch_route_n(int seg, int nr, hipStream_t s, A... args) {
    switch (seg) {
    case 4: bn_bwd_route_kernel<T, KH, KW, SW, 4, APPLY, NCH, DG><<<nr, 256, 0, s>>>(args...); break;
    case 16: bn_bwd_route_kernel<T, KH, KW, SW, 16, APPLY, NCH, DG><<<nr, 256, 0, s>>>(args...); break;
    default: bn_bwd_route_kernel<T, KH, KW, SW, 8, APPLY, NCH, DG><<<nr, 256, 0, s>>>(args...); break;
    }
}
template <typename T, int KH, int KW, int SW, bool APPLY, bool DG = false, typename... A>
static void launch_route(int seg, int nr, hipStream_t s, A... args) {
    if (bn_route_nch() == 8) launch_route_n<T, KH, KW, SW, APPLY, 8, DG>(seg, nr, s, args...);
    else launch_route_n<T, KH, KW, SW, APPLY, 4, DG>(seg, nr, s, args...);
}
template <typename T, int KH, int KW, int SW, typename... A>
static void launch_apply(bool dg, int seg, int nr, hipStream_t s, A... args) {
    if (dg) launch_route<T, KH, KW, SW, true, true>(seg, nr, s, args...);
    else launch_route<T, KH, KW, SW, true, false>(seg, nr, s, args...);
}

static int bn_route_variant(int kh, int kw, int sh, int sw, int H, int W) {
    if (!ocrk::opt(ocrk::OPT_BN_ROUTE) || sh != kh || H < kh || W < kw) return 0;
    if (kh == 2 && kw == 2 && sw == 2) return 1;
    if (kh == 2 && kw == 2 && sw == 1) return 2;
    if (kh == 3 && kw == 1 && sw == 1) return 3;
    return 0;
}

// part [SLAB_P][2C] doubles | slab [nb][2C] | dsum [2C] | bias slab [nb][2C] | routed da [B*H*W*C]
// (4 B per element: any dtype; the bias slab's rows are [bias | dgamma] in the pooled form)
static size_t bn_ws_floats(int64_t nb, int C) {
    size_t f = (size_t)SLAB_P * 2 * C * 2 + (size_t)(nb * 2 * C + 2 * C + nb * 2 * C);
    return (f + 3) / 4 * 4;                                           // 16-B align the da image
}

extern "C" size_t ocrk_bn_bwd_workspace_size(int B, int H, int W, int C) {
    int64_t items = (int64_t)B * H * W * (C / 8);
    int64_t nb = bn_bwd_blocks(items);
    nb = ocrk::cdiv(items, bn_bwd_ipb(items, nb));
    return bn_ws_floats(nb, C) * sizeof(float) + (size_t)B * H * W * C * sizeof(float);
}

// The window walk's launch: tasks (b, pooled row, column segment, channel group),
// tasks per block (a multiple of 256) and blocks, at most nb of them.
struct WalkGrid { int nseg, tpb, blocks; };
static WalkGrid walk_grid(int B, int H, int W, int C, int kh, int kw, int sw, int64_t nb) {
    const int Ho = (H - kh) / kh + 1, Wo = (W - kw) / sw + 1;
    const int nseg = (int)ocrk::cdiv(Wo, bn_route_seg());
    const int64_t tasks = (int64_t)B * Ho * nseg * (C / bn_route_nch());
    const int64_t nbr = std::max<int64_t>(1, std::min<int64_t>(nb, ocrk::cdiv(tasks, 256)));
    const int64_t tpb = ocrk::cdiv(ocrk::cdiv(tasks, nbr), 256) * 256;
    return WalkGrid{nseg, (int)tpb, (int)ocrk::cdiv(tasks, tpb)};
}

// Rows of the conv-bias partial-sum slab the apply pass writes (one per block);
// pooled: the pass-1-from-pooled-output form (every route variant applies by walking).
static int64_t bn_bwd_bias_rows(int B, int H, int W, int C, int kh, int kw, int sh, int sw, bool pooled = false) {
    const int64_t items = (int64_t)B * H * W * (C / 8);
    int64_t nb = bn_bwd_blocks(items);
    nb = ocrk::cdiv(items, bn_bwd_ipb(items, nb));
    const int rk = bn_route_variant(kh, kw, sh, sw, H, W);
    if (rk == 1 || rk == 3 || (rk == 2 && pooled)) return walk_grid(B, H, W, C, kh, kw, sw, nb).blocks;
    return nb;
}

extern "C" size_t ocrk_bn_bwd_bias_slab_rows(int B, int H, int W, int C, int kh, int kw, int sh, int sw) {
    if (C < 8 || C % 8 != 0 || (int64_t)B * H * W == 0) return 1;
    return (size_t)bn_bwd_bias_rows(B, H, W, C, kh, kw, sh, sw);
}

// 0 = the pooled-output form is not taken for this shape / pool (or option BN_ROUTE=0):
// ocrk_bn_relu_pool_bwd_pooled then refuses a bias_slab (callers take the z form)
extern "C" size_t ocrk_bn_bwd_pooled_bias_slab_rows(int B, int H, int W, int C, int kh, int kw, int sh, int sw) {
    if (!bn_route_variant(kh, kw, sh, sw, H, W)) return 0;
    if (C < 8 || C % 8 != 0 || (int64_t)B * H * W == 0) return 1;
    return (size_t)bn_bwd_bias_rows(B, H, W, C, kh, kw, sh, sw, true);
}

static int bn_bwd_impl(const void* z, const void* dp, int B, int H, int W, int C, const float* mean,
                       const float* invstd, const float* gamma, const float* beta, int kh, int kw, int sh, int sw,
                       int dp_time_major, void* dz, float* dgamma, float* dbeta, float* dbias, int accumulate,
                       float* bias_slab_out, void* ws, size_t ws_bytes, int dtype, void* stream, int phase = 0,
                       float* dsum_out = nullptr, const float* dsum_in = nullptr, const double* count = nullptr,
                       const void* pooled = nullptr) {
    // phase 0: both passes; 1: pass 1 + the ordered sums only (dsum_out gets them); 2: the
    // apply pass from cross-rank sums dsum_in over count pixels (ws as left by phase 1)
    OCRK_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "ocrk_bn_relu_pool_bwd: C=%d unsupported", C);
    OCRK_REQUIRE(ws_bytes >= ocrk_bn_bwd_workspace_size(B, H, W, C), "ocrk_bn_relu_pool_bwd: workspace too small");
    const int64_t items = (int64_t)B * H * W * (C / 8);
    OCRK_REQUIRE(items < (1ll << 31) && (int64_t)B * H * W < (1ll << 31), "ocrk_bn_relu_pool_bwd: tensor too large");
    if (items == 0) return OCRK_OK;
    int64_t nb = bn_bwd_blocks(items);
    const int64_t ipb = bn_bwd_ipb(items, nb);
    nb = ocrk::cdiv(items, ipb);
    double* part = (double*)ws;
    float* slab = (float*)(part + (size_t)SLAB_P * 2 * C);
    float* dsum = slab + nb * 2 * C;
    float* bslab = bias_slab_out ? bias_slab_out : dsum + 2 * C;
    void* da = (float*)ws + bn_ws_floats(nb, C);
    const int npix = B * H * W;
    hipStream_t s = ocrk::as_stream(stream);
    int nr = (int)nb;                                   // slab rows of pass 1
    const int rk = bn_route_variant(kh, kw, sh, sw, H, W);
    const int seg = bn_route_seg();
    // pass 1 from the pooled output (window-walk pools only: pass 2 then walks for all three)
    const bool from_pooled = pooled && rk;
    const int64_t pitems = from_pooled ? (int64_t)B * ((H - kh) / sh + 1) * ((W - kw) / sw + 1) * (C / 8) : 0;
    if (from_pooled) {
        nr = (int)std::max<int64_t>(1, std::min<int64_t>(nb, ocrk::cdiv(pitems, 256 * 4)));
    } else if (rk) {
        const int Ho = (H - kh) / kh + 1, Wo = (W - kw) / sw + 1;
        const int64_t tasks = (int64_t)B * Ho * ocrk::cdiv(Wo, seg) * (C / bn_route_nch());
        const int64_t nbr = std::min<int64_t>(nb, ocrk::cdiv(tasks, 256));
        nr = (int)ocrk::cdiv(tasks, ocrk::cdiv(ocrk::cdiv(tasks, nbr), 256) * 256);
    }
    int st = OCRK_OK;
    if (phase == 2) {
        bn_dsum_scale_kernel<<<ocrk::cdiv(2 * C, 256), 256, 0, s>>>(dsum_in, count, npix, 2 * C, dsum);
        st = ocrk::launch_status("ocrk_bn_relu_pool_bwd_apply scale");
        if (st) return st;
    } else if (from_pooled) {
        const int ipb2 = (int)(ocrk::cdiv(ocrk::cdiv(pitems, nr), 256) * 256);
        nr = (int)ocrk::cdiv(pitems, ipb2);
        if (dtype == OCRK_BF16)
            bn_bwd_pooled_sums_kernel<bf16><<<nr, 256, 0, s>>>((const bf16*)pooled, (const bf16*)dp, pitems, C, gamma,
                                                               beta, mean, invstd, (const bf16*)z, B, H, W, kh, kw,
                                                               sh, sw, dp_time_major, ipb2, slab);
        else
            bn_bwd_pooled_sums_kernel<float><<<nr, 256, 0, s>>>((const float*)pooled, (const float*)dp, pitems, C,
                                                                gamma, beta, mean, invstd, (const float*)z, B, H, W,
                                                                kh, kw, sh, sw, dp_time_major, ipb2, slab);
    } else if (rk) {
        const int Ho = (H - kh) / kh + 1, Wo = (W - kw) / sw + 1;
        const int nseg = (int)ocrk::cdiv(Wo, seg);
        const int64_t tasks = (int64_t)B * Ho * nseg * (C / bn_route_nch());
        const int64_t nbr = std::min<int64_t>(nb, ocrk::cdiv(tasks, 256));
        const int tpb = (int)(ocrk::cdiv(ocrk::cdiv(tasks, nbr), 256) * 256);
#define ROUTE_ARGS B, H, W, C, mean, invstd, gamma, beta, dp_time_major, nseg, tpb, slab
        if (dtype == OCRK_BF16) {
            const bf16 *zz = (const bf16*)z, *pp = (const bf16*)dp;
            bf16* dd = (bf16*)da;
            // pass 1 stages da only for the overlapping 2x2/[2,1] pools (their pass 2
            // streams it: measured faster than re-walking the windows); else pass 2 re-walks
            if (rk == 1) launch_route<bf16, 2, 2, 2, false>(seg, nr, s, zz, pp, ROUTE_ARGS, (bf16*)nullptr, (const float*)nullptr);
            else if (rk == 2) launch_route<bf16, 2, 2, 1, false>(seg, nr, s, zz, pp, ROUTE_ARGS, dd, (const float*)nullptr);
            else launch_route<bf16, 3, 1, 1, false>(seg, nr, s, zz, pp, ROUTE_ARGS, (bf16*)nullptr, (const float*)nullptr);
        } else {
            const float *zz = (const float*)z, *pp = (const float*)dp;
            float* dd = (float*)da;
            if (rk == 1) launch_route<float, 2, 2, 2, false>(seg, nr, s, zz, pp, ROUTE_ARGS, (float*)nullptr, (const float*)nullptr);
            else if (rk == 2) launch_route<float, 2, 2, 1, false>(seg, nr, s, zz, pp, ROUTE_ARGS, dd, (const float*)nullptr);
            else launch_route<float, 3, 1, 1, false>(seg, nr, s, zz, pp, ROUTE_ARGS, (float*)nullptr, (const float*)nullptr);
        }
#undef ROUTE_ARGS
    } else if (dtype == OCRK_BF16) {
        bn_bwd_reduce_kernel<bf16><<<nb, 256, 0, s>>>((const bf16*)z, (const bf16*)dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, (int)ipb, slab, (bf16*)da);
    } else {
        bn_bwd_reduce_kernel<float><<<nb, 256, 0, s>>>((const float*)z, (const float*)dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, (int)ipb, slab, (float*)da);
    }
    if (phase != 2) {
        st = ocrk::launch_status("ocrk_bn_relu_pool_bwd reduce");
        if (st) return st;
        st = slab_sum(slab, nr, 2 * C, part, phase == 1 ? dsum_out : dsum, dbeta, from_pooled ? nullptr : dgamma, C,
                      accumulate, s);   // dbeta | dgamma (pooled: dgamma from the apply walk)
        if (st || phase == 1) return st;
    }
    if (rk == 1 || rk == 3 || (rk == 2 && from_pooled)) {
        // pass 2 repeats the window walk (no staged da image): dz and the conv-bias partial sums
        const WalkGrid wg = walk_grid(B, H, W, C, kh, kw, sw, nb);
        const int nseg = wg.nseg, tpb = wg.tpb;
        nr = wg.blocks;
#define APPLY_ARGS B, H, W, C, mean, invstd, gamma, beta, dp_time_major, nseg, tpb, bslab
        const bool dg = from_pooled;                  // [bias | dgamma] rows: dgamma summed from z here
        if (dtype == OCRK_BF16) {
            const bf16 *zz = (const bf16*)z, *pp = (const bf16*)dp;
            bf16* dd = (bf16*)dz;
            const float* ds = dsum;
            if (rk == 1) launch_apply<bf16, 2, 2, 2>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
            else if (rk == 2) launch_apply<bf16, 2, 2, 1>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
            else launch_apply<bf16, 3, 1, 1>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
        } else {
            const float *zz = (const float*)z, *pp = (const float*)dp;
            float* dd = (float*)dz;
            const float* ds = dsum;
            if (rk == 1) launch_apply<float, 2, 2, 2>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
            else if (rk == 2) launch_apply<float, 2, 2, 1>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
            else launch_apply<float, 3, 1, 1>(dg, seg, nr, s, zz, pp, APPLY_ARGS, dd, ds);
        }
#undef APPLY_ARGS
        st = ocrk::launch_status("ocrk_bn_relu_pool_bwd apply (window walk)");
        if (st || bias_slab_out) return st;
        if (dg) return slab_sum(bslab, nr, 2 * C, part, nullptr, dbias, dgamma, C, accumulate, s);
        if (!dbias) return st;
        return slab_sum(bslab, nr, C, part, nullptr, dbias, nullptr, C, accumulate, s);
    }
    float* bs = (dbias || bias_slab_out) ? bslab : nullptr;
    if (dtype == OCRK_BF16)
        bn_bwd_apply_kernel<bf16><<<nb, 256, 0, s>>>((const bf16*)z, (const bf16*)da, npix, C, mean, invstd, gamma, dsum, (int)ipb, (bf16*)dz, bs);
    else
        bn_bwd_apply_kernel<float><<<nb, 256, 0, s>>>((const float*)z, (const float*)da, npix, C, mean, invstd, gamma, dsum, (int)ipb, (float*)dz, bs);
    st = ocrk::launch_status("ocrk_bn_relu_pool_bwd apply");
    if (st || !dbias || bias_slab_out) return st;
    return slab_sum(bslab, (int)nb, C, part, nullptr, dbias, nullptr, C, accumulate, s);
}

extern "C" int ocrk_bn_relu_pool_bwd(const void* z, const void* dp, int B, int H, int W, int C,
                                     const float* mean, const float* invstd, const float* gamma,
                                     const float* beta, int kh, int kw, int sh, int sw, int dp_time_major,
                                     void* dz, float* dgamma, float* dbeta, float* dbias, int accumulate,
                                     void* ws, size_t ws_bytes, int dtype, void* stream) {
    return bn_bwd_impl(z, dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, dz, dgamma,
                       dbeta, dbias, accumulate, nullptr, ws, ws_bytes, dtype, stream);
}

// The same with the conv-bias partials left to the caller: bias_slab gets
// ocrk_bn_bwd_bias_slab_rows(...) rows of C floats; ocrk_slab_sum(bias_slab,
// rows, C, C, dbias, ...) on any stream ordered after this call gives the dbias
// of ocrk_bn_relu_pool_bwd (same bits), off the critical path.
extern "C" int ocrk_bn_relu_pool_bwd_slab(const void* z, const void* dp, int B, int H, int W, int C,
                                          const float* mean, const float* invstd, const float* gamma,
                                          const float* beta, int kh, int kw, int sh, int sw, int dp_time_major,
                                          void* dz, float* dgamma, float* dbeta, int accumulate, float* bias_slab,
                                          void* ws, size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(bias_slab, "ocrk_bn_relu_pool_bwd_slab: bias_slab is required");
    return bn_bwd_impl(z, dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, dz, dgamma,
                       dbeta, nullptr, accumulate, bias_slab, ws, ws_bytes, dtype, stream);
}

// The same with pass 1 read from the forward's pooled output `pooled` (the
// ocrk_bn_relu_pool_fwd result: same layout as dp) instead of walking z -- see
// bn_bwd_pooled_sums_kernel (dgamma from xhat = (pooled - beta) / gamma; gamma = 0
// drops a channel's xhat terms). The window-walk pools only (2x2/[2,2], 2x2/[2,1],
// [3,1]/[3,1]; other pools take the z form). dgamma is summed from z in the apply
// walk. bias_slab (or NULL: dbias and dgamma (+)= their sums directly) gets
// ocrk_bn_bwd_pooled_bias_slab_rows(...) rows of 2C, [bias | dgamma] partials.
extern "C" int ocrk_bn_relu_pool_bwd_pooled(const void* z, const void* pooled, const void* dp, int B, int H, int W,
                                            int C, const float* mean, const float* invstd, const float* gamma,
                                            const float* beta, int kh, int kw, int sh, int sw, int dp_time_major,
                                            void* dz, float* dgamma, float* dbeta, float* dbias, int accumulate,
                                            float* bias_slab, void* ws, size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(pooled, "ocrk_bn_relu_pool_bwd_pooled: pooled is required");
    // a [bias | dgamma] slab exists only for the pooled form; the z form would write C-wide rows
    OCRK_REQUIRE(!bias_slab || bn_route_variant(kh, kw, sh, sw, H, W),
                 "ocrk_bn_relu_pool_bwd_pooled: bias_slab given but the pooled form is off for this pool "
                 "(ocrk_bn_bwd_pooled_bias_slab_rows() == 0)");
    return bn_bwd_impl(z, dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, dz, dgamma,
                       dbeta, bias_slab ? nullptr : dbias, accumulate, bias_slab, ws, ws_bytes, dtype, stream, 0,
                       nullptr, nullptr, nullptr, pooled);
}

// The two passes apart, for BatchNorm statistics over several ranks' batches:
// _reduce accumulates this batch's dgamma / dbeta and writes its ordered sums
// dsum [2C] (sum dy | sum dy * xhat, routed through ReLU + pool); the caller
// SUM-reduces dsum over the ranks; _apply then forms dz with the cross-rank sums
// over `count` (device double: all ranks' pixels, ocrk_bn_moments' last entry
// after the same all-reduce). ws is shared by the two calls and must be left
// untouched between them. One rank with dsum unchanged and count = B*H*W
// reproduces ocrk_bn_relu_pool_bwd[_slab] up to the rounding of the scale.
extern "C" int ocrk_bn_relu_pool_bwd_reduce(const void* z, const void* dp, int B, int H, int W, int C,
                                            const float* mean, const float* invstd, const float* gamma,
                                            const float* beta, int kh, int kw, int sh, int sw, int dp_time_major,
                                            float* dgamma, float* dbeta, int accumulate, float* dsum, void* ws,
                                            size_t ws_bytes, int dtype, void* stream) {
    OCRK_REQUIRE(dsum, "ocrk_bn_relu_pool_bwd_reduce: dsum is required");
    return bn_bwd_impl(z, dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, nullptr, dgamma,
                       dbeta, nullptr, accumulate, nullptr, ws, ws_bytes, dtype, stream, 1, dsum);
}

extern "C" int ocrk_bn_relu_pool_bwd_apply(const void* z, const void* dp, int B, int H, int W, int C,
                                           const float* mean, const float* invstd, const float* gamma,
                                           const float* beta, int kh, int kw, int sh, int sw, int dp_time_major,
                                           const float* dsum, const double* count, void* dz, float* dbias,
                                           int accumulate, float* bias_slab, void* ws, size_t ws_bytes, int dtype,
                                           void* stream) {
    OCRK_REQUIRE(dsum && count && dz, "ocrk_bn_relu_pool_bwd_apply: dsum, count and dz are required");
    return bn_bwd_impl(z, dp, B, H, W, C, mean, invstd, gamma, beta, kh, kw, sh, sw, dp_time_major, dz, nullptr,
                       nullptr, dbias, accumulate, bias_slab, ws, ws_bytes, dtype, stream, 2, nullptr, dsum, count);
}
