// Pipelined MFMA engine for the k-contiguous ("NT") operand modes, bf16:
//   A: A_ROWK (activations [M][lda]), A_IM2COL / A_IM2COL_FLIP (3x3 conv,
//      NHWC source, 8-channel chunks never cross a tap because C % 8 == 0)
//   B: B_NK (weights [N][ldb])
// which covers the conv forward / backward-data, the recurrent input
// projections and the dx GEMMs (gemm.h lists the modes).
//
// Structure (cdna_hip_programming.md section 5, "pipelining across
// barriers"): 256 threads, BM x BN x 64 tiles, a 3-stage LDS ring filled by
// LDS-DMA (buffer_load_dwordx4 ... lds) so loads for stages k+1 and k+2 are in
// flight while stage k is on MFMA; one raw s_barrier per k-step, counted
// s_waitcnt vmcnt (never __syncthreads inside the loop: its fence would drain
// the DMA queue).
// LDS images are lane-linear: one wave instruction writes 8 rows x 128 B.
// The 16-B chunk index of each row is XOR-swizzled with (row & 7) on the
// GLOBAL side (lane L of a row loads chunk (L & 7) ^ (L >> 3)), so the MFMA
// fragment reads (16 rows, one chunk each) hit 8 distinct chunk slots per
// 8 lanes: conflict-free ds_read_b128.
// Zero fill (im2col padding taps, rows >= M / N, k >= K): the lane's buffer
// offset is pushed past the resource's num_records, which returns 0.
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr int NT_BK = 64;            // k per stage (128 B per row)
constexpr int NT_STAGES = 3;
constexpr unsigned NT_OOB = 0x80000000u;

template <int AM>
struct ARow {                         // per-lane precomputed row geometry of one A instruction
    int64_t base;                     // ROWK: element offset of the row; IM2COL: of pixel (b,h,w) channel 0
    int h, w;                         // IM2COL only
    bool ok;
};

__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <int BM, int BN, int WAVES_M, int AM>
__global__ void __launch_bounds__(256) gemm_nt_kernel(const GemmParams p) {
    constexpr int WAVES_N = 4 / WAVES_M;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ROWB = NT_BK * 2;                       // 128 B per row
    constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
    constexpr int NA = BM / 32, NB = BN / 32;             // DMA instructions per thread per stage
    static_assert(BM % 32 == 0 && BN % 32 == 0 && TM >= 1 && TN >= 1, "tile");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int zb = blockIdx.z / p.splits, zs = blockIdx.z - zb * p.splits;
    const bf16* A = reinterpret_cast<const bf16*>(p.A) + zb * p.strideA;
    const bf16* B = reinterpret_cast<const bf16*>(p.B) + zb * p.strideB;
    const int kbeg = zs * p.k_chunk;
    const int kend = min(p.K, kbeg + p.k_chunk);
    const int nk = max(0, (kend - kbeg + NT_BK - 1) / NT_BK);

    // buffer resources (num_records = bytes; anything beyond reads as 0)
    int64_t a_elems, b_elems = (int64_t)p.N * p.ldb;
    if constexpr (AM == A_ROWK) a_elems = (int64_t)p.M * p.lda;
    else a_elems = (int64_t)p.M * p.convC;               // NHWC source with M = B*H*W pixels
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)min<int64_t>(a_elems * 2, 0x7fffffff), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, (int)min<int64_t>(b_elems * 2, 0x7fffffff), 0x00020000);

    // this lane's chunk within its row (global side of the swizzle)
    const int lrow = lane >> 3;                           // row within the 8-row instruction
    const int chunk = (lane & 7) ^ lrow;                  // row & 7 == lrow (instruction rows start at multiples of 8)

    ARow<AM> arow[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int r = (i * 4 + wave) * 8 + lrow;
        const int m = m0 + r;
        arow[i].ok = m < p.M;
        const int mm = arow[i].ok ? m : 0;
        if constexpr (AM == A_ROWK) {
            arow[i].base = (int64_t)mm * p.lda;
            arow[i].h = arow[i].w = 0;
        } else {
            const int W = p.convW, H = p.convH;
            const int w = mm % W, t2 = mm / W, h = t2 % H;
            arow[i].h = h;
            arow[i].w = w;
            arow[i].base = (int64_t)mm * p.convC;
        }
    }
    int64_t brow[NB];
    bool bok[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int n = n0 + (i * 4 + wave) * 8 + lrow;
        bok[i] = n < p.N;
        brow[i] = (int64_t)(bok[i] ? n : 0) * p.ldb;
    }

    auto issue = [&](int kt, int stage) {
        const int k = kbeg + kt * NT_BK + 8 * chunk;
        const bool kok = k < kend;
        char* sa = smem + stage * STAGE;
        char* sb = sa + A_BYTES;
        int tap_off = 0, dh = 0, dw = 0, cch = 0;
        if constexpr (AM != A_ROWK) {
            const int C = p.convC;
            const int tap = kok ? k / C : 0;
            cch = k - tap * C;
            const int kh = tap / 3, kw = tap - kh * 3;
            if constexpr (AM == A_IM2COL_FLIP) { dh = 1 - kh; dw = 1 - kw; }
            else { dh = kh - 1; dw = kw - 1; }
            tap_off = (dh * p.convW + dw) * C + cch;
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            bool ok = kok && arow[i].ok;
            int64_t e;
            if constexpr (AM == A_ROWK) {
                e = arow[i].base + k;
            } else {
                const int hh = arow[i].h + dh, ww = arow[i].w + dw;
                ok = ok && hh >= 0 && hh < p.convH && ww >= 0 && ww < p.convW;
                e = arow[i].base + tap_off;
            }
            const unsigned voff = ok ? (unsigned)(e * 2) : NT_OOB;
            lds_dma16(ra, sa + ((i * 4 + wave) * 8) * ROWB, voff);
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const unsigned voff = (kok && bok[i]) ? (unsigned)((brow[i] + k) * 2) : NT_OOB;
            lds_dma16(rb, sb + ((i * 4 + wave) * 8) * ROWB, voff);
        }
    };

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
    const int i16 = lane & 15, g = lane >> 4, sw = lane & 7;
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed (stage kt+1 may still be in flight), then everyone is past stage kt-1
        if (kt + 1 < nk) {
            if constexpr (NA + NB == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if constexpr (NA + NB == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else if constexpr (NA + NB == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            else if constexpr (NA + NB == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else if constexpr (NA + NB == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if constexpr (NA + NB == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if constexpr (NA + NB == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else if constexpr (NA + NB == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if constexpr (NA + NB == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else if constexpr (NA + NB == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 2 < nk) issue(kt + 2, (kt + 2) % NT_STAGES);
        const char* sa = smem + (kt % NT_STAGES) * STAGE;
        const char* sb = sa + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < NT_BK / 32; ++kk) {
            const int slot = ((kk * 4 + g) ^ sw) * 16;
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(sa + (wm * WM + i * 16 + i16) * ROWB + slot);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (wn * WN + j * 16 + i16) * ROWB + slot);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();                                      // LDS is reused by the stats epilogue

    // ------------------------------------------------------------ epilogue
    const int row_base = m0 + wm * WM + (lane >> 4) * 4;
    const int col_base = n0 + wn * WN + (lane & 15);
    if (p.splits > 1) {
        float* ws = p.splitk_ws + ((int64_t)zb * p.splits + zs) * (int64_t)p.M * p.N;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = row_base + i * 16 + r, col = col_base + j * 16;
                    if (row < p.M && col < p.N) ws[(int64_t)row * p.N + col] = acc[i][j][r];
                }
        return;
    }
    const float* bias = p.bias ? p.bias + zb * p.strideBias : nullptr;
    const bf16* mask = reinterpret_cast<const bf16*>(p.mask);
    float* Cf = reinterpret_cast<float*>(p.C) + zb * p.strideC;
    bf16* Cb = reinterpret_cast<bf16*>(p.C) + zb * p.strideC;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = col_base + j * 16;
        const float bcol = (bias && col < p.N) ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row_base + i * 16 + r;
                float v = p.alpha * acc[i][j][r] + bcol;
                if (row < p.M && col < p.N) {
                    if (mask && !((float)mask[(int64_t)row * p.ldmask + col] > 0.f)) v = 0.f;
                    if (p.relu) v = fmaxf(v, 0.f);
                    const int64_t off = (int64_t)row * p.ldc + col;
                    if (p.c_bf16) {
                        Cb[off] = (bf16)v;
                    } else {
                        if (p.accumulate) v += Cf[off];
                        Cf[off] = v;
                    }
                }
                acc[i][j][r] = v;
            }
    }
    if (!p.stats) return;

    // per-column (sum, M2) over the tile's valid rows (see gemm.hip)
    float* s_red = reinterpret_cast<float*>(smem);         // [WAVES_M][BN]
    const int valid_rows = min(BM, p.M - m0);
    float tsum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (row_base + i * 16 + r < p.M) s += acc[i][j][r];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        tsum[j] = s;
    }
    if (lane < 16)
#pragma unroll
        for (int j = 0; j < TN; ++j) s_red[wm * BN + wn * WN + j * 16 + lane] = tsum[j];
    __syncthreads();
    float tmean[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int c = wn * WN + j * 16 + (lane & 15);
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < WAVES_M; ++q) s += s_red[q * BN + c];
        tsum[j] = s;
        tmean[j] = s / (float)valid_rows;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (row_base + i * 16 + r < p.M) {
                    const float d = acc[i][j][r] - tmean[j];
                    s += d * d;
                }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (lane < 16) s_red[wm * BN + wn * WN + j * 16 + lane] = s;
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int c = wn * WN + j * 16 + lane;
            if (n0 + c < p.N) {
                float m2 = 0.f;
#pragma unroll
                for (int q = 0; q < WAVES_M; ++q) m2 += s_red[q * BN + c];
                float* st = p.stats + (int64_t)blockIdx.x * 2 * p.N;
                st[n0 + c] = tsum[j];
                st[p.N + n0 + c] = m2;
            }
        }
    }
}

template <int BM, int BN, int WAVES_M, int AM>
int launch_nt(const GemmParams& p, hipStream_t stream) {
    constexpr int LDS = NT_STAGES * (BM + BN) * NT_BK * 2;
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<BM, BN, WAVES_M, AM>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        configured = true;
    }
    dim3 grid((unsigned)cdiv(p.M, BM), (unsigned)cdiv(p.N, BN), (unsigned)(p.batch * p.splits));
    gemm_nt_kernel<BM, BN, WAVES_M, AM><<<grid, 256, LDS, stream>>>(p);
    return launch_status("gemm_nt");
}

template <int AM>
int dispatch_nt(const GemmParams& p, hipStream_t s) {
    // BM is the pixel / row dimension (large on every caller); BN follows N.
    if (p.N <= 32) return launch_nt<256, 32, 4, AM>(p, s);
    if (p.N <= 64) return launch_nt<256, 64, 4, AM>(p, s);
    return launch_nt<256, 128, 2, AM>(p, s);
}

}  // namespace

bool gemm_nt_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("OCRK_GEMM_NT");      // opt-in: not yet faster than gemm.hip
        on = (e && e[0] == '1') ? 1 : 0;
    }
    return on == 1;
}

// Runs the NT engine when it covers (mode, dtype); returns -1 when it does not.
int gemm_nt(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    if (!gemm_nt_enabled() || dtype != OCRK_BF16 || bmode != B_NK) return -1;
    if (p.K % 8 != 0) return -1;
    if (amode == A_ROWK) {
        if (p.lda % 8 != 0 || p.ldb % 8 != 0) return -1;          // 16-B aligned rows
        return dispatch_nt<A_ROWK>(p, stream);
    }
    if (amode == A_IM2COL) return dispatch_nt<A_IM2COL>(p, stream);
    if (amode == A_IM2COL_FLIP) return dispatch_nt<A_IM2COL_FLIP>(p, stream);
    return -1;
}

}  // namespace ocrk
