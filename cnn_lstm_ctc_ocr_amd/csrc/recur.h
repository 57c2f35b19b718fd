// Shared pieces of the recurrent step kernels (lstm.hip, gru.hip): the
// streaming MFMA core that computes one step's h . W tile, 4-wide epilogue
// loads/stores and the exp-based gate nonlinearities.
#pragma once
#include "common.h"
#include "mfma_util.h"

namespace ocrk {

// X3 (CT = float): each fp32 fragment pair is split at the read into bf16 hi / lo
// (split8_bf16) and multiplied as al.bh + ah.bl + ah.bh on the bf16 MFMA (the
// fp32 loops outside exact mode, kernels.f32_exact); else exact f32 MFMA.
template <typename CT, int BR, int NC, int KC, bool X3 = false>
struct RecurCore {
    static_assert(!X3 || sizeof(CT) == 4, "the split is of fp32 operands");
    using RT = typename RawT<CT>::T;
    static constexpr int LDK = KC + 8;
    static constexpr int NVA = (BR * KC / 8 + 255) / 256;
    static constexpr int NVB = (NC * KC / 8 + 255) / 256;
    static constexpr int TILES = (BR / 16) * (NC / 16);
    static constexpr int TPW = TILES >= 4 ? TILES / 4 : 1;
    static constexpr int STAGE_BYTES = 2 * (BR + NC) * LDK * (int)sizeof(RT);
    static constexpr int EPI_BYTES = BR * (NC + 1) * 4;
    static constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
    static_assert(TILES % 4 == 0 || TILES < 4, "tile split");
    static constexpr bool FULL_A = (BR * KC / 8) % 256 == 0;
    static constexpr bool FULL_B = (NC * KC / 8) % 256 == 0;

    template <typename BCol>
    __device__ __forceinline__ static void load(V8<CT> (&ra)[NVA], V8<CT> (&rb)[NVB], const CT* __restrict__ a_rows,
                                                int64_t lda, const BCol& bcol, int k0) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            if (FULL_A || idx < BR * KC / 8) {
                int r = idx / (KC / 8), kq = idx % (KC / 8);
                vload(ra[v], a_rows + (int64_t)r * lda + k0 + 8 * kq);
            }
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            if (FULL_B || idx < NC * KC / 8) {
                int n = idx / (KC / 8), kq = idx % (KC / 8);
                vload(rb[v], bcol(n) + k0 + 8 * kq);
            }
        }
    }
    __device__ __forceinline__ static void store(const V8<CT> (&ra)[NVA], const V8<CT> (&rb)[NVB], RT* sA, RT* sB,
                                                 int buf) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            if (FULL_A || idx < BR * KC / 8)
                vstore_lds(sA + buf * BR * LDK + (idx / (KC / 8)) * LDK + 8 * (idx % (KC / 8)), ra[v]);
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            if (FULL_B || idx < NC * KC / 8)
                vstore_lds(sB + buf * NC * LDK + (idx / (KC / 8)) * LDK + 8 * (idx % (KC / 8)), rb[v]);
        }
    }
    __device__ __forceinline__ static void compute(floatx4 (&acc)[TPW], const RT* sA, const RT* sB, int buf) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            int q = wave + 4 * i;
            if (q >= TILES) break;
            int tm = q / (NC / 16), tn = q % (NC / 16);
            const RT* a = sA + buf * BR * LDK + (tm * 16 + (lane & 15)) * LDK + 8 * (lane >> 4);
            const RT* b = sB + buf * NC * LDK + (tn * 16 + (lane & 15)) * LDK + 8 * (lane >> 4);
#pragma unroll
            for (int ks = 0; ks < KC / 32; ++ks) {
                if constexpr (sizeof(CT) == 2) {
                    bf16x8 af = *reinterpret_cast<const bf16x8*>(a + ks * 32);
                    bf16x8 bfr = *reinterpret_cast<const bf16x8*>(b + ks * 32);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i], 0, 0, 0);
                } else if constexpr (X3) {
                    // the bf16 MFMA's operand layout is this staging's: lane group g holds
                    // k = 32 ks + 8 g .. + 7 of its row
                    V8<float> af, bfr;
                    vload_lds(af, a + ks * 32);
                    vload_lds(bfr, b + ks * 32);
                    u32x4 ah, al, bh, bl;
                    split8_bf16(af, ah, al);
                    split8_bf16(bfr, bh, bl);
                    const bf16x8 ahb = __builtin_bit_cast(bf16x8, ah), alb = __builtin_bit_cast(bf16x8, al);
                    const bf16x8 bhb = __builtin_bit_cast(bf16x8, bh), blb = __builtin_bit_cast(bf16x8, bl);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alb, bhb, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahb, blb, acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahb, bhb, acc[i], 0, 0, 0);
                } else {
                    V8<float> af, bfr;
                    vload_lds(af, a + ks * 32);
                    vload_lds(bfr, b + ks * 32);
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af.e(kk), bfr.e(kk), acc[i], 0, 0, 0);
                }
            }
        }
    }

    // acc <- A[BR, K] . Bcols[NC, K]^T ; A rows at a_rows + r*lda, B col n at bcol(n).
    // begin() issues the loads of chunks 0 and 1 (so the caller can overlap
    // other loads with them); finish() runs the pipeline: two register sets
    // in flight while one chunk is on MFMA.
    V8<CT> ra0[NVA], rb0[NVB], ra1[NVA], rb1[NVB];

    template <typename BCol>
    __device__ __forceinline__ void begin(const CT* __restrict__ a_rows, int64_t lda, const BCol& bcol, int K) {
        load(ra0, rb0, a_rows, lda, bcol, 0);
        if (K / KC > 1) load(ra1, rb1, a_rows, lda, bcol, KC);
    }

    template <typename BCol>
    __device__ __forceinline__ void finish(const CT* __restrict__ a_rows, int64_t lda, const BCol& bcol, int K,
                                           char* lds, floatx4 (&acc)[TPW]) {
        RT* sA = reinterpret_cast<RT*>(lds);
        RT* sB = sA + 2 * BR * LDK;
#pragma unroll
        for (int i = 0; i < TPW; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        const int nch = K / KC;
        store(ra0, rb0, sA, sB, 0);
        __syncthreads();
        for (int c = 0; c < nch; c += 2) {
            if (c + 2 < nch) load(ra0, rb0, a_rows, lda, bcol, (c + 2) * KC);
            compute(acc, sA, sB, 0);
            if (c + 1 < nch) store(ra1, rb1, sA, sB, 1);
            __syncthreads();
            if (c + 1 >= nch) break;
            if (c + 3 < nch) load(ra1, rb1, a_rows, lda, bcol, (c + 3) * KC);
            compute(acc, sA, sB, 1);
            if (c + 2 < nch) store(ra0, rb0, sA, sB, 0);
            __syncthreads();
        }
    }

    // accumulators -> LDS [BR][NC+1] f32 (call after run(); ends with a barrier)
    __device__ __forceinline__ static void spill(const floatx4 (&acc)[TPW], char* lds) {
        float* sG = reinterpret_cast<float*>(lds);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            int q = wave + 4 * i;
            if (q >= TILES) break;
            int tm = q / (NC / 16), tn = q % (NC / 16);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sG[(tm * 16 + (lane >> 4) * 4 + r) * (NC + 1) + tn * 16 + (lane & 15)] = acc[i][r];
        }
        __syncthreads();
    }
};

// 4 consecutive elements of CT (8 B for bf16, 16 B for f32)
template <typename CT> struct V4;
template <> struct V4<bf16> { typedef unsigned int u32x2 __attribute__((ext_vector_type(2))); u32x2 q; };
template <> struct V4<float> { f32x4 q; };
__device__ __forceinline__ void ld4(float (&v)[4], const bf16* p) {
    V4<bf16>::u32x2 q = *reinterpret_cast<const V4<bf16>::u32x2*>(p);
    v[0] = __builtin_bit_cast(float, q[0] << 16); v[1] = __builtin_bit_cast(float, q[0] & 0xffff0000u);
    v[2] = __builtin_bit_cast(float, q[1] << 16); v[3] = __builtin_bit_cast(float, q[1] & 0xffff0000u);
}
__device__ __forceinline__ void ld4(float (&v)[4], const float* p) {
    f32x4 q = *reinterpret_cast<const f32x4*>(p);
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
}
__device__ __forceinline__ void st4(bf16* p, const float (&v)[4]) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 q = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *reinterpret_cast<bf16x4*>(p) = q;
}
__device__ __forceinline__ void st4(float* p, const float (&v)[4]) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
}
// exp-based gate nonlinearities: one v_exp + one v_rcp each (1-ulp hardware
// reciprocal instead of the ~10-instruction IEEE division sequence, which
// made up ~40 % of the step epilogue's VALU work). Saturate correctly:
// exp -> inf gives rcp(inf) = 0.
__device__ __forceinline__ float sig_fast(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

__device__ __forceinline__ int step_time(int dir, int s, int len) {
    return (dir == 0 || s >= len) ? s : len - 1 - s;
}

// acc[i][j] += A_i . B_j over NKS 32-deep k-steps, both operands resident in
// LDS as lane-linear rows whose 16-B chunks are XOR-swizzled by (row & 15):
// arow[i] / brow[j] point at this lane's row (16-row fragment i16 = lane&15),
// g = lane >> 4 picks the 8-element k group, sw = row & 15. Fully unrolled
// with the fragment reads PF k-steps ahead of the MFMAs that use them (left
// to itself the scheduler sinks every read next to its MFMA and waits on
// it; a sched_barrier per k-step pins the order), and the chunk offsets
// precomputed so each read is one ds_read_b128 with an immediate offset.
// KSTRIDE: bytes between consecutive 128-element k blocks of a row (256 for
// row-contiguous images, the block size for k-block-major images).
template <int NKS, int TM, int TN, int PF = 2, int KSTRIDE = 256>
__device__ __forceinline__ void lds_mma_16x16x32(const char* const (&arow)[TM], const char* const (&brow)[TN],
                                                 int g, int sw, floatx4 (&acc)[TM][TN]) {
    const int gs = g ^ sw;                              // (4 ks + g) ^ sw == 4 ks ^ (g ^ sw)
    const char* pa[TM][4];
    const char* pb[TN][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int off = ((4 * q) ^ gs) * 16;
#pragma unroll
        for (int i = 0; i < TM; ++i) pa[i][q] = arow[i] + off;
#pragma unroll
        for (int j = 0; j < TN; ++j) pb[j][q] = brow[j] + off;
    }
    constexpr int R = PF + 1;
    bf16x8 fa[R][TM], fb[R][TN];
    auto load = [&](int ks, int slot) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[slot][i] = *reinterpret_cast<const bf16x8*>(pa[i][ks & 3] + (ks >> 2) * KSTRIDE);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[slot][j] = *reinterpret_cast<const bf16x8*>(pb[j][ks & 3] + (ks >> 2) * KSTRIDE);
    };
#pragma unroll
    for (int ks = 0; ks < PF && ks < NKS; ++ks) load(ks, ks);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        if (ks + PF < NKS) load(ks + PF, (ks + PF) % R);
        // keep the scheduler from sinking the reads next to their MFMAs
        __builtin_amdgcn_sched_barrier(0);
        const int c = ks % R;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[c][i], fb[c][j], acc[i][j], 0, 0, 0);
    }
}

// Workgroup -> (unit block, batch block, direction) of a recurrent step
// launch on a 1-D grid of nU * nB * 2 workgroups. Dispatch hands consecutive
// block ids round-robin to the 8 XCDs; the map gives each XCD a contiguous
// range of (direction, unit block, batch block) with the batch block
// fastest, i.e. a 1/8 slice of the direction's units for every batch block.
// An XCD then reads only its own W_h slice (1/8 of W_h, each row slice
// shared by the nB workgroups of that unit block) plus the direction's h,
// instead of the whole W_h[dir] -- measured: the previous map, all unit
// blocks of one (batch block, direction) on an XCD, re-fetched all of W_h
// from beyond L2 every step (FETCH_SIZE ~20 MB per step at B=256, H=512;
// L2 does not keep it across launches). Placement is a speed choice only:
// nothing depends on it for correctness.
struct StepTile { int u, b, dir; };
__device__ __forceinline__ StepTile step_tile(int nU, int nB) {
    const int id = blockIdx.x, total = 2 * nU * nB;
    int j = id;
    if (total % 8 == 0) j = (id & 7) * (total >> 3) + (id >> 3);
    const int b = j % nB, rest = j / nB;
    return {rest % nU, b, rest / nU};
}

}  // namespace ocrk
