// Pipelined MFMA engine for the k-major ("TN") operand modes, bf16:
//   A: A_COLK (A(m,k) = A[k*lda + m]: activations [K][M], the recurrent and
//      logits weight gradients) or A_IM2COL_T (3x3 conv weight gradient:
//      A((tap,c), pixel) = x[pixel shifted by tap][c])
//   B: B_KN (B(k,n) = B[k*ldb + n]: gradients [K][N])
// Both operands are contiguous along m / n, so each stage is staged as
// [BK][rows] images (rows contiguous) by LDS-DMA and read into MFMA fragments
// with ds_read_b64_tr_b16 (frag_tr; A and B share its permuted k-slot order,
// so the products pair up exactly). Pipeline, zero fill and epilogue as in
// gemm_nt.hip. The 16-B chunks of each k-row are XOR-swizzled on the global
// side (f(r) = r mod chunks-per-row, or (r >> 2) mod 4 for 64-B rows) so the
// 16 k-rows a wave's transposed read touches spread over the bank groups.
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr unsigned TN_OOB = 0x80000000u;

__device__ __forceinline__ void tn_dma16(const i32x4_t& r, void* lds, unsigned voff) {
    lds_dma16_asm(r, lds, voff);                          // asm: see mfma_util.h
}

template <int CPR>
__device__ __forceinline__ int tn_swz(int r) { return CPR >= 8 ? (r & (CPR - 1)) : ((r >> 2) & (CPR - 1)); }

template <int BM, int BN, int BK, int S, int WAVES_M, int AM, int NW = 4>
__global__ void __launch_bounds__(NW * 64) gemm_tn_kernel(const GemmParams p) {
    constexpr int WAVES_N = NW / WAVES_M;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ROWA = BM * 2, ROWB = BN * 2;                    // bytes per k-row
    constexpr int CPRA = ROWA / 16, CPRB = ROWB / 16;              // 16-B chunks per k-row
    constexpr int RPIA = 1024 / ROWA, RPIB = 1024 / ROWB;          // k-rows per wave instruction
    constexpr int A_BYTES = BK * ROWA, B_BYTES = BK * ROWB, STAGE = A_BYTES + B_BYTES;
    constexpr int NA = BK / (NW * RPIA), NB = BK / (NW * RPIB);    // DMA instructions per thread per stage
    constexpr int NPS = NA + NB;
    static_assert(BK % 32 == 0 && S >= 2 && NA >= 1 && NB >= 1, "stage shape");
    static_assert(CPRA >= 4 && CPRB >= 4 && TM >= 1 && TN >= 1, "tile");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int zb = blockIdx.z / p.splits, zs = blockIdx.z - zb * p.splits;
    const bf16* A = reinterpret_cast<const bf16*>(p.A) + zb * p.strideA;
    const bf16* B = reinterpret_cast<const bf16*>(p.B) + zb * p.strideB;
    const int kbeg = zs * p.k_chunk;
    const int kend = min(p.K, kbeg + p.k_chunk);
    const int nk = max(0, (kend - kbeg + BK - 1) / BK);

    int64_t a_elems;
    if constexpr (AM == A_COLK) a_elems = (int64_t)p.K * p.lda;
    else a_elems = (int64_t)p.K * p.convC;                        // NHWC source, K = B*H*W pixels
    const int64_t b_elems = (int64_t)p.K * p.ldb;
    const i32x4_t ra = uniform_rsrc_words(A, a_elems * 2);
    const i32x4_t rb = uniform_rsrc_words(B, b_elems * 2);

    // ---- per-lane geometry of each A instruction (stage-invariant parts)
    const int qa = lane / CPRA, sa_slot = lane % CPRA;
    int a_r[NA];                  // k-row within the stage
    int a_m[NA];                  // first m of the lane's chunk (or -1: past M)
    int a_tap[NA];                // IM2COL_T: (dh+1)*3+(dw+1) packed as dh, dw below; COLK unused
    int a_ch[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int r = (i * NW + wave) * RPIA + qa;
        a_r[i] = r;
        const int c = sa_slot ^ tn_swz<CPRA>(r);
        const int m = m0 + 8 * c;
        a_m[i] = m < p.M ? m : -1;
        a_tap[i] = 0;
        a_ch[i] = 0;
        if constexpr (AM == A_IM2COL_T) {
            const int mm = m < p.M ? m : 0;
            const int tap = mm / p.convC;
            a_ch[i] = mm - tap * p.convC;
            a_tap[i] = tap;
        }
    }
    // pixel coordinates of each A instruction's k-row, advanced by BK per stage
    int a_w[NA], a_h[NA], a_b[NA];
    if constexpr (AM == A_IM2COL_T) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int k = kbeg + a_r[i];
            const int kk = k < p.K ? k : 0;
            a_w[i] = kk % p.convW;
            const int t = kk / p.convW;
            a_h[i] = t % p.convH;
            a_b[i] = t / p.convH;
        }
    }
    // ---- B instructions
    const int qb = lane / CPRB, sb_slot = lane % CPRB;
    int b_r[NB], b_n[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int r = (i * NW + wave) * RPIB + qb;
        b_r[i] = r;
        const int n = n0 + 8 * (sb_slot ^ tn_swz<CPRB>(r));
        b_n[i] = n < p.N ? n : -1;
    }

    auto issue = [&](int kt, int stage) {
        char* sa = smem + stage * STAGE;
        char* sb = sa + A_BYTES;
        const int kbase = kbeg + kt * BK;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int k = kbase + a_r[i];
            bool ok = k < kend && a_m[i] >= 0;
            unsigned voff;
            if constexpr (AM == A_COLK) {
                voff = (unsigned)(((int64_t)k * p.lda + a_m[i]) * 2);
            } else {
                const int kh = a_tap[i] / 3, kw = a_tap[i] - 3 * kh;
                const int hh = a_h[i] + kh - 1, ww = a_w[i] + kw - 1;
                ok = ok && hh >= 0 && hh < p.convH && ww >= 0 && ww < p.convW;
                voff = (unsigned)(((((int64_t)a_b[i] * p.convH + hh) * p.convW + ww) * p.convC + a_ch[i]) * 2);
                // next stage: k-row + BK
                int w = a_w[i] + BK, h = a_h[i], b = a_b[i];
                while (w >= p.convW) {
                    w -= p.convW;
                    if (++h == p.convH) { h = 0; ++b; }
                }
                a_w[i] = w; a_h[i] = h; a_b[i] = b;
            }
            tn_dma16(ra, sa + ((i * NW + wave) * RPIA) * ROWA, ok ? voff : TN_OOB);
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = kbase + b_r[i];
            const bool ok = k < kend && b_n[i] >= 0;
            const unsigned voff = (unsigned)(((int64_t)k * p.ldb + b_n[i]) * 2);
            tn_dma16(rb, sb + ((i * NW + wave) * RPIB) * ROWB, ok ? voff : TN_OOB);
        }
    };

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // stages are issued strictly in order, so the pixel advance above stays in step
#pragma unroll
    for (int st = 0; st < S - 1; ++st)
        if (st < nk) issue(st, st);
    const int i16 = lane & 15, g = lane >> 4;
    const int kr0 = 4 * g + (i16 >> 2);                 // k-row of this lane's tr read (first half)
    const int mq = 4 * (i16 & 3);                       // m offset within the 16-wide block
    for (int kt = 0; kt < nk; ++kt) {
        const int ahead = min(S - 2, nk - 1 - kt);
        if constexpr (S >= 3) {
            if (ahead >= 1) vm_wait<NPS>();
            else vm_wait<0>();
        } else {
            vm_wait<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
        const char* sa = smem + (kt % S) * STAGE;
        const char* sb = sa + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
            const int r = kk * 32 + kr0;                // second read at r + 16: same swizzle
            bf16x8 bfr[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = wn * WN + j * 16 + mq;
                const int off = r * ROWB + (((n >> 3) ^ tn_swz<CPRB>(r)) << 4) + (n & 7) * 2;
                bfr[j] = frag_tr(reinterpret_cast<const unsigned short*>(sb + off), 16 * BN);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int m = wm * WM + i * 16 + mq;
                const int off = r * ROWA + (((m >> 3) ^ tn_swz<CPRA>(r)) << 4) + (m & 7) * 2;
                const bf16x8 af = frag_tr(reinterpret_cast<const unsigned short*>(sa + off), 16 * BM);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    }

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
                if (row < p.M && col < p.N) {
                    float v = p.alpha * acc[i][j][r] + bcol;
                    if (p.relu) v = fmaxf(v, 0.f);
                    const int64_t off = (int64_t)row * p.ldc + col;
                    if (p.c_bf16) {
                        Cb[off] = (bf16)v;
                    } else {
                        if (p.accumulate) v += Cf[off];
                        Cf[off] = v;
                    }
                }
            }
    }
}

template <int BM, int BN, int BK, int S, int WAVES_M, int AM>
int launch_tn(const GemmParams& p, hipStream_t stream) {
    constexpr int LDS = S * BK * (BM + BN) * 2;
    static DeviceOnce configured;
    set_dyn_lds(configured, reinterpret_cast<const void*>(&gemm_tn_kernel<BM, BN, BK, S, WAVES_M, AM>), LDS);
    dim3 grid((unsigned)cdiv(p.M, BM), (unsigned)cdiv(p.N, BN), (unsigned)(p.batch * p.splits));
    gemm_tn_kernel<BM, BN, BK, S, WAVES_M, AM><<<grid, 256, LDS, stream>>>(p);
    return launch_status("gemm_tn");
}

#ifdef OCRK_EXPERIMENTS
int tn_stages() {                                    // OCRK_GEMM_TN_STAGES=3: 3-stage ring (experiments)
    static const int st = [] {                 // thread-safe once
        const char* e = getenv("OCRK_GEMM_TN_STAGES");
        return (e && e[0] == '3') ? 3 : 2;
    }();
    return st;
}
#endif

template <int AM>
int dispatch_tn(const GemmParams& p, hipStream_t s) {
#ifdef OCRK_EXPERIMENTS
    if (tn_stages() == 3) {
        if (p.N <= 32) return launch_tn<128, 32, 64, 3, 4, AM>(p, s);
        if (p.N <= 64) return launch_tn<128, 64, 64, 3, 2, AM>(p, s);
        return launch_tn<128, 128, 64, 3, 2, AM>(p, s);
    }
#endif
    if (p.N <= 32) return launch_tn<128, 32, 64, 2, 4, AM>(p, s);
    if (p.N <= 64) return launch_tn<128, 64, 64, 2, 2, AM>(p, s);
    return launch_tn<128, 128, 64, 2, 2, AM>(p, s);
}

}  // namespace

bool gemm_tn_enabled() {
    return opt(OPT_GEMM_TN) != 0;
}

int gemm_tn(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    if (!gemm_tn_enabled() || dtype != OCRK_BF16 || bmode != B_KN || p.stats) return -1;
    if (p.M % 8 != 0 || p.N % 8 != 0) return -1;
    if (amode == A_COLK) {
        if (p.lda % 8 != 0 || p.ldb % 8 != 0) return -1;
        return dispatch_tn<A_COLK>(p, stream);
    }
    if (amode == A_IM2COL_T) {
        if (p.convC % 8 != 0 || p.ldb % 8 != 0) return -1;
        if (p.N > 128) return -1;          // 2304 x 256 (conv8): the generic engine measured faster
        return dispatch_tn<A_IM2COL_T>(p, stream);
    }
    return -1;
}

}  // namespace ocrk
