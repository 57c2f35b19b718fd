// Small byte-moving kernels around the hot ops: dtype casts, the weight-image
// permutes (HWIO -> [Cout][kh][kw][Cin] for the forward conv GEMM and
// [Cin][kh][kw][Cout] for backward-data), deterministic column sums (bias
// gradients) and the ReLU-mask product of the logits layer backward.
#include "common.h"
#include "reduce.h"
#include "mfma_util.h"

template <typename TI, typename TO>
__global__ void __launch_bounds__(256) cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = from_f32<TO>(to_f32(in[i]));
}

// out[i1][i0][i2] = in[i0][i1][i2]
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) permute3_kernel(const TI* __restrict__ in, int d0, int d1, int d2,
                                                       TO* __restrict__ out) {
    const int64_t n = (int64_t)d0 * d1 * d2;
    for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < n; o += (int64_t)gridDim.x * 256) {
        int i2 = (int)(o % d2);
        int64_t t = o / d2;
        int i0 = (int)(t % d0);
        int i1 = (int)(t / d0);
        out[o] = from_f32<TO>(to_f32(in[((int64_t)i0 * d1 + i1) * d2 + i2]));
    }
}

namespace ocrk {
namespace {

// Column sums of a [nslab][NC] f32 slab matrix in a fixed order, double
// accumulation. One launch: a 256-thread workgroup per 16 columns, 4 column
// quads x 64 row groups; a thread's rows are loaded 16 at a time (16-B loads,
// all in flight) and added in row order, then the 64 row groups meet in LDS in a
// fixed order. The slab tables here are <= ~2k rows x a few hundred columns (a
// few hundred KB) and sit on the step's critical path between a BN backward's
// passes: the previous 64-column / 16-row-group form walked a 2048-row slab in 16
// dependent rounds on one or two CUs (8-17 us per call in the step); this one in
// 2 rounds on 4+ CUs. One launch still beats the two-stage form's two, and a
// 4-wave workgroup finds a CU slot beside the other stream's GEMMs. Rows not a
// multiple of 4 columns wide (or unaligned) take the two-stage form below.
__global__ void __launch_bounds__(256)
slab_sum_fused(const float* __restrict__ slab, int nslab, int NC, int ld, float* __restrict__ res,
               float* __restrict__ dst_lo, float* __restrict__ dst_hi, int split, int accumulate) {
    constexpr int RG = 64, CQ = 4, U = 16;
    __shared__ double red[RG][4 * CQ + 1];
    const int cq = threadIdx.x % CQ, rg = threadIdx.x / CQ;
    const int c0 = blockIdx.x * 4 * CQ + 4 * cq;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    if (c0 < NC) {
        const float* col = slab + c0;
        int i = rg;
        for (; i + (U - 1) * RG < nslab; i += U * RG) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const f32x4*>(col + (int64_t)(i + u * RG) * ld);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) s[e] += v[u][e];
        }
        for (; i < nslab; i += RG) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(col + (int64_t)i * ld);
#pragma unroll
            for (int e = 0; e < 4; ++e) s[e] += v[e];
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rg][4 * cq + e] = s[e];
    __syncthreads();
    if (threadIdx.x < 4 * CQ) {
        const int c = blockIdx.x * 4 * CQ + threadIdx.x;
        if (c >= NC) return;
        double t = 0.0;
        for (int y = 0; y < RG; ++y) t += red[y][threadIdx.x];
        const float v = (float)t;
        if (res) res[c] = v;
        float* d = c < split ? (dst_lo ? dst_lo + c : nullptr) : (dst_hi ? dst_hi + (c - split) : nullptr);
        if (d) *d = accumulate ? *d + v : v;
    }
}

// Two-stage form (any NC / ld): stage 1 -> part [SLAB_P][NC] doubles, stage 2 -> the result.
__global__ void __launch_bounds__(256)
slab_sum_stage1(const float* __restrict__ slab, int nslab, int NC, int ld, double* __restrict__ part) {
    __shared__ double red[4][64];
    const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int rows = (nslab + SLAB_P - 1) / SLAB_P;
    const int r0 = blockIdx.y * rows, r1 = min(nslab, r0 + rows);
    double s = 0.0;
    if (c < NC)
        for (int i = r0 + q; i < r1; i += 4) s += slab[(int64_t)i * ld + c];
    red[q][cl] = s;
    __syncthreads();
    if (q == 0 && c < NC) part[(int64_t)blockIdx.y * NC + c] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// res[o] = sum; then (accumulate ? += : =) into dst_lo[o] for o < split, dst_hi[o - split] above
__global__ void __launch_bounds__(64)
slab_sum_stage2(const double* __restrict__ part, int NC, float* __restrict__ res, float* __restrict__ dst_lo,
                float* __restrict__ dst_hi, int split, int accumulate) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= NC) return;
    double t = 0.0;
    for (int y = 0; y < SLAB_P; ++y) t += part[(int64_t)y * NC + c];
    const float v = (float)t;
    if (res) res[c] = v;
    float* d = c < split ? (dst_lo ? dst_lo + c : nullptr) : (dst_hi ? dst_hi + (c - split) : nullptr);
    if (d) *d = accumulate ? *d + v : v;
}

}  // namespace

int slab_sum(const float* slab, int nslab, int NC, double* part, float* res, float* dst_lo, float* dst_hi,
             int split, int accumulate, hipStream_t s, int ld) {
    const int l = ld > 0 ? ld : NC;
    if (NC % 4 == 0 && l % 4 == 0 && ((uintptr_t)slab & 15) == 0) {
        slab_sum_fused<<<(NC + 15) / 16, 256, 0, s>>>(slab, nslab, NC, l, res, dst_lo, dst_hi, split, accumulate);
        return ocrk::launch_status("slab sum");
    }
    slab_sum_stage1<<<dim3((NC + 63) / 64, SLAB_P), 256, 0, s>>>(slab, nslab, NC, ld > 0 ? ld : NC, part);
    int st = ocrk::launch_status("slab sum 1");
    if (st) return st;
    slab_sum_stage2<<<(NC + 63) / 64, 64, 0, s>>>(part, NC, res, dst_lo, dst_hi, split, accumulate);
    return ocrk::launch_status("slab sum 2");
}

}  // namespace ocrk

// column sums of [M][N]: block (x, y) reduces column block x (TPR groups of 8
// columns, one 16-B vector per thread per row; a wave reads 64 consecutive
// chunks of a row when N >= 512) over row range y, combines its threads in a
// fixed order and writes slab row y; slab_sum then sums the slabs in a
// fixed order (deterministic for a given shape).
template <typename T>
__global__ void __launch_bounds__(256) colsum_partial_kernel(const T* __restrict__ in, int64_t M, int N,
                                                             int64_t rows_per_block, float* __restrict__ slab) {
    __shared__ float red[256 * 9];
    const int G = N / 8;                       // column groups of 8
    const int TPR = G < 64 ? G : 64;           // threads per row
    const int RPP = 256 / TPR;                 // rows per pass
    const int tg = threadIdx.x % TPR, tr = threadIdx.x / TPR;
    const int g = blockIdx.x * TPR + tg;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (tr < RPP && g < G) {
#pragma unroll 4
        for (int64_t r = r0 + tr; r < r1; r += RPP) {
            const F8 v = load8(in + r * N + g * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] += v.v[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) red[threadIdx.x * 9 + i] = acc[i];
    __syncthreads();
    for (int o = threadIdx.x; o < TPR * 8; o += 256) {
        int gg = o / 8, i = o % 8;
        float sum = 0.f;
        for (int q = 0; q < RPP; ++q) sum += red[(q * TPR + gg) * 9 + i];
        if (blockIdx.x * TPR + gg < G) slab[(int64_t)blockIdx.y * N + (blockIdx.x * TPR + gg) * 8 + i] = sum;
    }
}

template <typename TO>
__global__ void __launch_bounds__(256) relu_mask_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                        int64_t n, float scale, TO* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = from_f32<TO>(y[i] > 0.f ? dy[i] * scale : 0.f);
}

static unsigned grid1d(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ocrk::cdiv(n, 256), 16384)); }

extern "C" int ocrk_cast(const void* in, int in_dtype, void* out, int out_dtype, int64_t n, void* stream) {
    if (n == 0) return OCRK_OK;
    hipStream_t s = ocrk::as_stream(stream);
    if (in_dtype == OCRK_F32 && out_dtype == OCRK_BF16) cast_kernel<float, bf16><<<grid1d(n), 256, 0, s>>>((const float*)in, (bf16*)out, n);
    else if (in_dtype == OCRK_BF16 && out_dtype == OCRK_F32) cast_kernel<bf16, float><<<grid1d(n), 256, 0, s>>>((const bf16*)in, (float*)out, n);
    else if (in_dtype == OCRK_F32 && out_dtype == OCRK_F32) cast_kernel<float, float><<<grid1d(n), 256, 0, s>>>((const float*)in, (float*)out, n);
    else cast_kernel<bf16, bf16><<<grid1d(n), 256, 0, s>>>((const bf16*)in, (bf16*)out, n);
    return ocrk::launch_status("ocrk_cast");
}

// x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (RNE; |x - hi - lo| <= 2^-17 |x|):
// the bf16x3 split as two bf16 planes, so a bf16 GEMM engine can form
// ah.bh + ah.bl + al.bh in three accumulating calls. 8 elements per thread.
__global__ void split_bf16_kernel(const float* __restrict__ x, unsigned* __restrict__ hi, unsigned* __restrict__ lo,
                                  int64_t n8) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
        unsigned h[4], l[4];
        ocrk::split2_bf16(a.x, a.y, h[0], l[0]);
        ocrk::split2_bf16(a.z, a.w, h[1], l[1]);
        ocrk::split2_bf16(b.x, b.y, h[2], l[2]);
        ocrk::split2_bf16(b.z, b.w, h[3], l[3]);
        reinterpret_cast<uint4*>(hi)[i] = make_uint4(h[0], h[1], h[2], h[3]);
        reinterpret_cast<uint4*>(lo)[i] = make_uint4(l[0], l[1], l[2], l[3]);
    }
}

extern "C" int ocrk_split_bf16(const float* x, int64_t n, void* hi, void* lo, void* stream) {
    OCRK_REQUIRE(n % 8 == 0 && ((uintptr_t)x | (uintptr_t)hi | (uintptr_t)lo) % 16 == 0,
                 "ocrk_split_bf16: n=%lld must be a multiple of 8 and the buffers 16-B aligned", (long long)n);
    if (n == 0) return OCRK_OK;
    split_bf16_kernel<<<grid1d(n / 8), 256, 0, ocrk::as_stream(stream)>>>(x, (unsigned*)hi, (unsigned*)lo, n / 8);
    return ocrk::launch_status("ocrk_split_bf16");
}

extern "C" int ocrk_permute3(const void* in, int in_dtype, int d0, int d1, int d2, void* out, int out_dtype,
                             void* stream) {
    int64_t n = (int64_t)d0 * d1 * d2;
    if (n == 0) return OCRK_OK;
    hipStream_t s = ocrk::as_stream(stream);
    OCRK_REQUIRE(in_dtype == OCRK_F32, "ocrk_permute3: f32 input only");
    if (out_dtype == OCRK_BF16) permute3_kernel<float, bf16><<<grid1d(n), 256, 0, s>>>((const float*)in, d0, d1, d2, (bf16*)out);
    else permute3_kernel<float, float><<<grid1d(n), 256, 0, s>>>((const float*)in, d0, d1, d2, (float*)out);
    return ocrk::launch_status("ocrk_permute3");
}

// Row blocks: enough (column block x row block) workgroups to fill the chip
// (~2048), at least 64 rows each.
static int colsum_col_blocks(int N) { return (int)ocrk::cdiv(N / 8, 64); }
static int64_t colsum_blocks(int64_t M, int N) {
    const int64_t want = std::max<int64_t>(1, 2048 / colsum_col_blocks(std::max(N, 8)));
    return std::max<int64_t>(1, std::min<int64_t>(want, ocrk::cdiv(M, 64)));
}

// slab [nb][N] f32 | part [SLAB_P][N] double
extern "C" size_t ocrk_colsum_workspace_size(int64_t M, int N) {
    return ((size_t)colsum_blocks(M, N) * N * sizeof(float) + 7) / 8 * 8 + (size_t)ocrk::SLAB_P * N * sizeof(double);
}

extern "C" int ocrk_colsum(const void* in, int64_t M, int N, int dtype, float* out, int accumulate, void* ws,
                           size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ws_bytes >= ocrk_colsum_workspace_size(M, N), "ocrk_colsum: workspace too small");
    OCRK_REQUIRE(N % 8 == 0, "ocrk_colsum: N=%d must be a multiple of 8", N);
    if (N == 0) return OCRK_OK;
    int64_t nb = colsum_blocks(M, N);
    int64_t rpb = ocrk::cdiv(M, nb);
    nb = std::max<int64_t>(1, ocrk::cdiv(M, rpb));
    hipStream_t s = ocrk::as_stream(stream);
    dim3 grid(colsum_col_blocks(N), (unsigned)nb);
    if (dtype == OCRK_BF16) colsum_partial_kernel<bf16><<<grid, 256, 0, s>>>((const bf16*)in, M, N, rpb, (float*)ws);
    else colsum_partial_kernel<float><<<grid, 256, 0, s>>>((const float*)in, M, N, rpb, (float*)ws);
    int st = ocrk::launch_status("ocrk_colsum");
    if (st) return st;
    double* part = (double*)((char*)ws + ((size_t)nb * N * sizeof(float) + 7) / 8 * 8);
    return ocrk::slab_sum((const float*)ws, (int)nb, N, part, nullptr, out, nullptr, N, accumulate, s);
}

extern "C" size_t ocrk_slab_sum_workspace_size(int nc) { return (size_t)ocrk::SLAB_P * std::max(nc, 1) * sizeof(double); }

extern "C" int ocrk_slab_sum(const float* slab, int nslab, int nc, int ld, float* out, int accumulate, void* ws,
                             size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(nslab >= 0 && nc >= 0 && ld >= nc, "ocrk_slab_sum: bad sizes");
    OCRK_REQUIRE(ws_bytes >= ocrk_slab_sum_workspace_size(nc), "ocrk_slab_sum: workspace too small");
    if (nc == 0) return OCRK_OK;
    return ocrk::slab_sum(slab, nslab, nc, (double*)ws, nullptr, out, nullptr, nc, accumulate, ocrk::as_stream(stream),
                          ld);
}

extern "C" int ocrk_relu_mask(const float* dy, const float* y, int64_t n, float scale, void* out, int out_dtype,
                              void* stream) {
    if (n == 0) return OCRK_OK;
    hipStream_t s = ocrk::as_stream(stream);
    if (out_dtype == OCRK_BF16) relu_mask_kernel<bf16><<<grid1d(n), 256, 0, s>>>(dy, y, n, scale, (bf16*)out);
    else relu_mask_kernel<float><<<grid1d(n), 256, 0, s>>>(dy, y, n, scale, (float*)out);
    return ocrk::launch_status("ocrk_relu_mask");
}

// out[r*out_rs + c*out_cs] = in[r*in_rs + c*in_cs]  (weight images for the GEMMs)
template <typename TO>
__global__ void __launch_bounds__(256) strided_copy_kernel(const float* __restrict__ in, int64_t rows, int64_t cols,
                                                           int64_t in_rs, int64_t in_cs, TO* __restrict__ out,
                                                           int64_t out_rs, int64_t out_cs) {
    const int64_t n = rows * cols;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        int64_t r = i / cols, c = i - r * cols;
        out[r * out_rs + c * out_cs] = from_f32<TO>(in[r * in_rs + c * in_cs]);
    }
}

extern "C" int ocrk_strided_copy(const float* in, int64_t rows, int64_t cols, int64_t in_rs, int64_t in_cs,
                                 void* out, int out_dtype, int64_t out_rs, int64_t out_cs, void* stream) {
    int64_t n = rows * cols;
    if (n == 0) return OCRK_OK;
    hipStream_t s = ocrk::as_stream(stream);
    if (out_dtype == OCRK_BF16)
        strided_copy_kernel<bf16><<<grid1d(n), 256, 0, s>>>(in, rows, cols, in_rs, in_cs, (bf16*)out, out_rs, out_cs);
    else
        strided_copy_kernel<float><<<grid1d(n), 256, 0, s>>>(in, rows, cols, in_rs, in_cs, (float*)out, out_rs, out_cs);
    return ocrk::launch_status("ocrk_strided_copy");
}

// All weight images of a parameter version in ONE launch: a table of 2-D
// copies out[r*out_rs + c] = in[r*in_rs + c] (plain) or out[c*out_rs + r] =
// in[r*in_rs + c] (transposed), f32 -> dtype, cut into 32 x 32 tiles. A
// workgroup finds its job by binary search over the tiles' prefix offsets,
// stages the tile in LDS and writes it back row-contiguous either way (the
// per-image strided copies wrote one side 2 bytes at a time).
struct CopyJob {
    const float* src;
    void* dst;
    int64_t rows, cols, in_rs, out_rs, tile0;
    int transpose, dtype;
};
static_assert(sizeof(CopyJob) == 8 * 8, "job layout (include/ocrk.h)");

// The job search runs over the tables' first tiles staged in LDS (one load
// round trip instead of a chain of dependent global loads per workgroup: the
// ~21k single-tile workgroups of a parameter version were latency-bound on it).
// Jobs whose sizes, strides and addresses are 4-element aligned (all but the
// 95-column logits) move 16-B float4 reads and 4-element packed writes (one
// each per thread); the rest keep the scalar form.
constexpr int COPY_JOBS_LDS = 256;
__global__ void __launch_bounds__(256) copy_batch_kernel(const CopyJob* __restrict__ jobs, int njobs) {
    __shared__ float tile[32][33];
    __shared__ int64_t first[COPY_JOBS_LDS];
    const int64_t t = blockIdx.x;
    int lo = 0, hi = njobs - 1;
    if (njobs <= COPY_JOBS_LDS) {
        if ((int)threadIdx.x < njobs) first[threadIdx.x] = jobs[threadIdx.x].tile0;
        __syncthreads();
        while (lo < hi) {                               // last job with tile0 <= t
            const int mid = (lo + hi + 1) >> 1;
            if (first[mid] <= t) lo = mid; else hi = mid - 1;
        }
    } else {
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (jobs[mid].tile0 <= t) lo = mid; else hi = mid - 1;
        }
    }
    const CopyJob j = jobs[lo];
    const int64_t lt = t - j.tile0, tc = (j.cols + 31) / 32;
    const int64_t r0 = (lt / tc) * 32, c0 = (lt % tc) * 32;
    const bool bf = j.dtype == OCRK_BF16;
    const bool vec = ((j.rows | j.cols | j.in_rs | j.out_rs) & 3) == 0 && ((uintptr_t)j.src & 15) == 0 &&
                     ((uintptr_t)j.dst & (bf ? 7 : 15)) == 0;
    if (vec) {
        const int q = threadIdx.x >> 3, c4 = (threadIdx.x & 7) * 4;      // tile row / first of 4 columns
        if (r0 + q < j.rows && c0 + c4 < j.cols) {
            const float4 v = *reinterpret_cast<const float4*>(j.src + (r0 + q) * j.in_rs + c0 + c4);
            tile[q][c4] = v.x; tile[q][c4 + 1] = v.y; tile[q][c4 + 2] = v.z; tile[q][c4 + 3] = v.w;
        }
        __syncthreads();
        float o[4];
        int64_t orow, ocol;
        if (j.transpose) {                              // out row = input column q, 4 input rows
            orow = c0 + q; ocol = r0 + c4;
            if (orow >= j.cols || ocol >= j.rows) return;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = tile[c4 + e][q];
        } else {
            orow = r0 + q; ocol = c0 + c4;
            if (orow >= j.rows || ocol >= j.cols) return;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = tile[q][c4 + e];
        }
        const int64_t off = orow * j.out_rs + ocol;
        if (bf) {
            typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
            u32x2_t w;
            w[0] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)o[0]) |
                   ((unsigned)__builtin_bit_cast(unsigned short, (bf16)o[1]) << 16);
            w[1] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)o[2]) |
                   ((unsigned)__builtin_bit_cast(unsigned short, (bf16)o[3]) << 16);
            *reinterpret_cast<u32x2_t*>(reinterpret_cast<bf16*>(j.dst) + off) = w;
        } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(j.dst) + off) = make_float4(o[0], o[1], o[2], o[3]);
        }
        return;
    }
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;      // 32 x 8
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t r = r0 + ty + 8 * k, c = c0 + tx;
        tile[ty + 8 * k][tx] = (r < j.rows && c < j.cols) ? j.src[r * j.in_rs + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int64_t orow, ocol;
        float v;
        if (j.transpose) {                              // out row = input column
            orow = c0 + ty + 8 * k; ocol = r0 + tx;
            v = tile[tx][ty + 8 * k];
            if (orow >= j.cols || ocol >= j.rows) continue;
        } else {
            orow = r0 + ty + 8 * k; ocol = c0 + tx;
            v = tile[ty + 8 * k][tx];
            if (orow >= j.rows || ocol >= j.cols) continue;
        }
        const int64_t o = orow * j.out_rs + ocol;
        if (bf) reinterpret_cast<bf16*>(j.dst)[o] = (bf16)v;
        else reinterpret_cast<float*>(j.dst)[o] = v;
    }
}

extern "C" int ocrk_copy_batch(const void* jobs, int njobs, int64_t total_tiles, void* stream) {
    OCRK_REQUIRE(njobs >= 1 && total_tiles >= 1 && total_tiles < (1ll << 31), "ocrk_copy_batch: njobs=%d tiles=%lld",
                 njobs, (long long)total_tiles);
    copy_batch_kernel<<<(unsigned)total_tiles, 256, 0, ocrk::as_stream(stream)>>>((const CopyJob*)jobs, njobs);
    return ocrk::launch_status("ocrk_copy_batch");
}

// x[i] *= s[0]  (upstream scalar gradient applied on device, no host sync)
__global__ void __launch_bounds__(256) mul_scalar_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ s) {
    const float v = s[0];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] *= v;
}

extern "C" int ocrk_mul_scalar(float* x, int64_t n, const float* s, void* stream) {
    if (n == 0) return OCRK_OK;
    mul_scalar_kernel<<<grid1d(n), 256, 0, ocrk::as_stream(stream)>>>(x, n, s);
    return ocrk::launch_status("ocrk_mul_scalar");
}

// out[0] = mean(x[0:n]) in a fixed order (reduce_mean of the CTC losses, model.py:228)
__global__ void __launch_bounds__(256) mean_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
    __shared__ double s[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) acc += x[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = n > 0 ? (float)(s[0] / n) : 0.f;
}

extern "C" int ocrk_mean(const float* x, int n, float* out, void* stream) {
    mean_kernel<<<1, 256, 0, ocrk::as_stream(stream)>>>(x, n, out);
    return ocrk::launch_status("ocrk_mean");
}

// convnet_layers tail (src/weinman/model.py:152-163): seq_len = floor((w - 2) / 2) - 2
__global__ void seq_len_kernel(const int* __restrict__ widths, int n, int* __restrict__ out) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        int a = widths[i] - 2;
        int q = a >= 0 ? a / 2 : -((-a + 1) / 2);   // floor division
        out[i] = q - 1 - 1;
    }
}

extern "C" int ocrk_seq_len(const int* widths, int n, int* out, void* stream) {
    if (n == 0) return OCRK_OK;
    seq_len_kernel<<<(n + 255) / 256, 256, 0, ocrk::as_stream(stream)>>>(widths, n, out);
    return ocrk::launch_status("ocrk_seq_len");
}

// ------------------------------------------------------------ status word
__global__ void status_clear_kernel(unsigned* word, unsigned bits) {
    if (threadIdx.x == 0) atomicAnd(word, ~bits);
}

extern "C" int ocrk_status_clear(unsigned* status_word, uint32_t bits, void* stream) {
    OCRK_REQUIRE(status_word != nullptr, "ocrk_status_clear: null status word");
    if (!bits) return OCRK_OK;
    status_clear_kernel<<<1, 64, 0, ocrk::as_stream(stream)>>>(status_word, bits);
    return ocrk::launch_status("ocrk_status_clear");
}
