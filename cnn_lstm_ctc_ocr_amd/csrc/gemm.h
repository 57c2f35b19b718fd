// MFMA GEMM engine shared by the conv, recurrent-projection and logits ops.
//
//   C[M,N] (+)= A[M,K] . B[K,N]  (+ bias[N]) (ReLU) (* mask>0)    fp32 accumulate
//
// Operands are staged global -> registers -> LDS (double buffered, one barrier
// per 32-deep k-step) into a canonical k-contiguous image [rows][32+8]; the
// staging layer is what makes one kernel serve every op on the path:
//   A_ROWK         A(m,k) = A[m*lda + k]                 (activations, row major)
//   A_COLK         A(m,k) = A[k*lda + m]                 (activations, transposed: weight grads)
//   A_IM2COL       A(m,k) = x[b, h+kh-1, w+kw-1, c]      (3x3 'same' conv forward)
//   A_IM2COL_FLIP  A(m,k) = dy[b, h-kh+1, w-kw+1, c]     (conv backward-data)
//   A_IM2COL_T     A(i,k) = x[b, h+kh-1, w+kw-1, c], i=(kh,kw,c), k=(b,h,w)  (conv weight grad)
//   B_NK           B(k,n) = B[n*ldb + k]                 (weights stored [N][K])
//   B_KN           B(k,n) = B[k*ldb + n]                 (activations / grads stored [K][N])
// compute types: bf16 (v_mfma_f32_16x16x32_bf16) and f32 (v_mfma_f32_16x16x4_f32,
// exact fp32 products).
#pragma once
#include "common.h"

namespace ocrk {

enum AMode { A_ROWK = 0, A_COLK = 1, A_IM2COL = 2, A_IM2COL_FLIP = 3, A_IM2COL_T = 4 };
enum BMode { B_NK = 0, B_KN = 1 };

struct GemmParams {
    int M, N, K;
    int batch;                     // independent problems along grid.z (with strides)
    const void* A; int64_t lda; int64_t strideA;
    const void* B; int64_t ldb; int64_t strideB;
    void* C; int64_t ldc; int64_t strideC;
    int c_bf16;                    // C element type: 0 f32, 1 bf16
    const float* bias; int64_t strideBias;   // [N] per problem or NULL
    const void* mask; int64_t ldmask;        // C *= (mask[m,n] > 0); mask has the compute type; or NULL
    int accumulate;                // C += result (f32 C only)
    int relu;
    float alpha;
    float* stats;                  // per (m-tile, column): [gridDim.x][2][N] sum and M2 of the tile's rows, or NULL
    float* splitk_ws;              // [batch][splits][M][N] f32 partials when splits > 1
    int splits;
    int k_chunk;                   // k-range per split (multiple of 32)
    int convH, convW, convC;       // im2col source geometry (NHWC) for the A_IM2COL* modes
    int epi_staged;                // gemm_nt (set by it): bf16 C (and the mask) move through an LDS tile
    // ReLU bit masks (bit c of byte c/8 of row m: column c > 0; rows of N/8 bytes), NT engine,
    // staged bf16 epilogue only: mask_bits replaces `mask` as C's mask; relu_bits receives
    // the bit mask of the (ReLU) output C
    const void* mask_bits;
    void* relu_bits;
};

// XCD-aware tile order for a 1-D grid of 8 * ceil(tm * tn / 8) workgroups.
// Dispatch deals consecutive workgroup ids round-robin to the 8 XCDs (each
// with its own L2); this gives XCD x the contiguous tile range
// [x * per, (x + 1) * per) of a grouped order (GM m-tiles x all n-tiles, m
// fastest), so the ~32 tiles an XCD runs at once share A rows and B columns
// in its L2 (and conv tiles share their im2col halo rows) instead of every
// XCD fetching every operand block from beyond L2. Speed only: any order is
// correct. valid = false for the padding workgroups past tm * tn.
struct TileIdx { int bm, bn; bool valid; };
__device__ __forceinline__ TileIdx xcd_tile(int tm, int tn) {
    const int nT = tm * tn, per = (nT + 7) >> 3;
    const int t = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (t >= nT) return {0, 0, false};
    constexpr int GM = 4;
    const int gsz = GM * tn, grp = t / gsz, first = grp * GM;
    const int gm = min(GM, tm - first), w = t - grp * gsz;
    return {first + w % gm, w / gm, true};
}
__host__ __forceinline__ unsigned xcd_grid(int tm, int tn) { return 8u * (unsigned)((tm * tn + 7) / 8); }

// Launch C = A.B with the given operand modes. dtype: OCRK_F32 / OCRK_BF16
// (type of A and B). Picks the tile shape from M, N.
int gemm(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream);

// Split-K GEMM: partials into p.splitk_ws, then a reduce applying the epilogue.
size_t gemm_splitk_ws_bytes(int M, int N, int batch, int splits);
// Sum p.splits f32 partials [splits][M][N] (p.splitk_ws) into C with the epilogue
// (alpha, bias, relu, accumulate) -- also used by kernels that leave their own partials.
int splitk_finish(const GemmParams& p, hipStream_t stream);

// Pipelined LDS-DMA engine for bf16 A_ROWK / A_IM2COL / A_IM2COL_FLIP x B_NK
// (gemm_nt.hip). Returns -1 when it does not cover the call (the caller then
// uses the generic engine), else a status. OCRK_GEMM_NT=0 disables it.
int gemm_nt(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream);
// fp32 operands: exact f32 MFMA (OCRK_F32_MFMA=1) instead of the bf16x3 split
bool f32_exact_mfma();

// 8-wave ping-pong engine (gemm_pp.hip): 256 x {256,128} x 64 tiles for the
// large bf16 A_ROWK / A_IM2COL / A_IM2COL_FLIP x B_NK GEMMs (N >= 96). Returns
// -1 when it does not cover the call. OCRK_GEMM_PP=0 disables it.
int gemm_pp(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream);

// 8-wave ping-pong engine for A_COLK x B_KN weight gradients (gemm_pptn.hip),
// f32 C or split-K partials, M, N >= 256. -1 when not covered (OCRK_GEMM_PPTN=0).
bool gemm_pptn_covers(int amode, int M, int N, int convC);   // shape test of gemm_pptn (wgrad split choice)
int gemm_pptn(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream);

// The same pipeline for the k-major modes A_COLK / A_IM2COL_T x B_KN (conv
// weight gradients, recurrent / logits weight gradients), gemm_tn.hip.
// Returns -1 when not covered. OCRK_GEMM_TN=0 disables it.
int gemm_tn(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream);

}  // namespace ocrk
