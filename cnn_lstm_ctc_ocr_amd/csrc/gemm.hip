// MFMA GEMM engine (see gemm.h for the operand modes).
//
// Tile: TBM x TBN x 32, 256 threads = 4 waves in a 2 x 2 grid, each wave owns a
// (TBM/2) x (TBN/2) block of 16 x 16 MFMA accumulators. Global -> register
// staging of tile k+1 is issued before the MFMAs of tile k and written to the
// other LDS buffer after them (one barrier per k-step). LDS rows are padded by
// 8 elements (16 B for bf16) so the per-lane 16-B fragment reads of a 16-row
// group fall on distinct bank groups.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

// Element (row, k) address for the A operand; ok=false -> zero.
template <int AM, typename CT>
__device__ __forceinline__ const CT* a_addr(const GemmParams& p, const CT* A, int m, int k, bool& ok) {
    if constexpr (AM == A_ROWK) {
        ok = m < p.M && k < p.K;
        return A + (int64_t)m * p.lda + k;
    } else if constexpr (AM == A_COLK) {
        ok = m < p.M && k < p.K;
        return A + (int64_t)k * p.lda + m;
    } else {
        // pixel index and (tap, channel) index
        int pix, kidx;
        if constexpr (AM == A_IM2COL_T) { pix = k; kidx = m; ok = k < p.K && m < p.M; }
        else { pix = m; kidx = k; ok = m < p.M && k < p.K; }
        const int C = p.convC, W = p.convW, H = p.convH;
        int tap = kidx / C, c = kidx - tap * C;
        int kh = tap / 3, kw = tap - kh * 3;
        int w = pix % W, t2 = pix / W, h = t2 % H, b = t2 / H;
        int hh, ww;
        if constexpr (AM == A_IM2COL_FLIP) { hh = h - kh + 1; ww = w - kw + 1; }
        else { hh = h + kh - 1; ww = w + kw - 1; }
        ok = ok && hh >= 0 && hh < H && ww >= 0 && ww < W;
        return A + (((int64_t)b * H + hh) * W + ww) * C + c;
    }
}

template <int BMD, typename CT>
__device__ __forceinline__ const CT* b_addr(const GemmParams& p, const CT* B, int n, int k, bool& ok) {
    ok = n < p.N && k < p.K;
    if constexpr (BMD == B_NK) return B + (int64_t)n * p.ldb + k;
    else return B + (int64_t)k * p.ldb + n;
}

// X3 (CT = float): fp32 operands split at staging into bf16 hi / lo LDS images
// ([row][k], k-contiguous, the hi image at [0, ELEMS), lo at [ELEMS, 2 ELEMS))
// and multiplied as ah.bh + ah.bl + al.bh on v_mfma_f32_16x16x32_bf16
// (mfma_util.h split2_bf16): the fp32 serving path at 3/16 of the bf16 MFMA
// cost per product instead of the f32 MFMA's 16/1 (X3 = false: exact fp32
// products on v_mfma_f32_16x16x4_f32, OCRK_F32_MFMA=1).
template <typename CT, int AM, int BMD, int TBM, int TBN, bool X3 = false>
__global__ void __launch_bounds__(256) gemm_kernel(const GemmParams p) {
    static_assert(!X3 || sizeof(CT) == 4, "bf16x3 splits fp32 operands");
    using RT = typename std::conditional<X3, unsigned short, typename RawT<CT>::T>::type;
    constexpr int BK = 32, LDK = BK + 8;
    constexpr int WM = TBM / 2, WN = TBN / 2, TM = WM / 16, TN = WN / 16;
    constexpr bool A_K = (AM == A_ROWK || AM == A_IM2COL || AM == A_IM2COL_FLIP);
    constexpr bool B_K = (BMD == B_NK);
    constexpr bool BF = sizeof(CT) == 2;
    // bf16 operands whose source is contiguous along the row (m or n) are kept
    // row-contiguous in LDS ([k][row], written with 16-B stores) and read as
    // MFMA fragments with ds_read_b64_tr_b16. Row stride T+16 elements puts
    // the 8 rows of a 32-lane half on 8 distinct 32-B bank slots.
    constexpr bool A_TR = BF && !A_K, B_TR = BF && !B_K;
    // With a transposed image the MFMA k-slot order is permuted (same for A
    // and B): lane group g, element j holds k = (j < 4 ? 4g + j : 16 + 4g + j - 4).
    constexpr bool PERM = A_TR || B_TR;
    constexpr int LDA_R = TBM + 16, LDB_R = TBN + 16;
    constexpr int A_ELEMS = A_TR ? BK * LDA_R : TBM * LDK;
    constexpr int B_ELEMS = B_TR ? BK * LDB_R : TBN * LDK;
    constexpr int NVA = (TBM * BK / 8 + 255) / 256;
    constexpr int NVB = (TBN * BK / 8 + 255) / 256;
    __shared__ __attribute__((aligned(16))) RT sA[2][X3 ? 2 * A_ELEMS : A_ELEMS];
    __shared__ __attribute__((aligned(16))) RT sB[2][X3 ? 2 * B_ELEMS : B_ELEMS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * TBM, n0 = blockIdx.y * TBN;
    const int zb = blockIdx.z / p.splits, zs = blockIdx.z - zb * p.splits;
    const CT* A = reinterpret_cast<const CT*>(p.A) + zb * p.strideA;
    const CT* B = reinterpret_cast<const CT*>(p.B) + zb * p.strideB;
    const int kbeg = zs * p.k_chunk;
    const int kend = min(p.K, kbeg + p.k_chunk);
    const int nk = max(0, (kend - kbeg + BK - 1) / BK);

    V8<CT> ra[NVA], rb[NVB];
    auto load_tiles = [&](int k0) {
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            vzero(ra[v]);
            if (idx < TBM * BK / 8) {
                int m, k;
                if constexpr (A_K) { m = m0 + (idx >> 2); k = k0 + 8 * (idx & 3); }
                else { k = k0 + idx / (TBM / 8); m = m0 + 8 * (idx % (TBM / 8)); }
                bool ok;
                const CT* src = a_addr<AM, CT>(p, A, m, k, ok);
                if (ok && k < kend) vload(ra[v], src);
            }
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            vzero(rb[v]);
            if (idx < TBN * BK / 8) {
                int n, k;
                if constexpr (B_K) { n = n0 + (idx >> 2); k = k0 + 8 * (idx & 3); }
                else { k = k0 + idx / (TBN / 8); n = n0 + 8 * (idx % (TBN / 8)); }
                bool ok;
                const CT* src = b_addr<BMD, CT>(p, B, n, k, ok);
                if (ok && k < kend) vload(rb[v], src);
            }
        }
    };
    auto store_tiles_x3 = [&](int buf) {
        if constexpr (X3) {
#pragma unroll
            for (int v = 0; v < NVA; ++v) {
                int idx = tid + 256 * v;
                if (idx < TBM * BK / 8) {
                    u32x4 hi, lo;
                    split8_bf16(ra[v], hi, lo);
                    if constexpr (A_K) {
                        const int o = (idx >> 2) * LDK + 8 * (idx & 3);
                        *reinterpret_cast<u32x4*>(&sA[buf][o]) = hi;
                        *reinterpret_cast<u32x4*>(&sA[buf][A_ELEMS + o]) = lo;
                    } else {
                        int kk = idx / (TBM / 8), r0 = 8 * (idx % (TBM / 8));
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            sA[buf][(r0 + i) * LDK + kk] = (unsigned short)(hi[i >> 1] >> (16 * (i & 1)));
                            sA[buf][A_ELEMS + (r0 + i) * LDK + kk] = (unsigned short)(lo[i >> 1] >> (16 * (i & 1)));
                        }
                    }
                }
            }
#pragma unroll
            for (int v = 0; v < NVB; ++v) {
                int idx = tid + 256 * v;
                if (idx < TBN * BK / 8) {
                    u32x4 hi, lo;
                    split8_bf16(rb[v], hi, lo);
                    if constexpr (B_K) {
                        const int o = (idx >> 2) * LDK + 8 * (idx & 3);
                        *reinterpret_cast<u32x4*>(&sB[buf][o]) = hi;
                        *reinterpret_cast<u32x4*>(&sB[buf][B_ELEMS + o]) = lo;
                    } else {
                        int kk = idx / (TBN / 8), r0 = 8 * (idx % (TBN / 8));
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            sB[buf][(r0 + i) * LDK + kk] = (unsigned short)(hi[i >> 1] >> (16 * (i & 1)));
                            sB[buf][B_ELEMS + (r0 + i) * LDK + kk] = (unsigned short)(lo[i >> 1] >> (16 * (i & 1)));
                        }
                    }
                }
            }
        }
    };
    auto store_tiles = [&](int buf) {
        if constexpr (X3) {
            store_tiles_x3(buf);
        } else {
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            if (idx < TBM * BK / 8) {
                if constexpr (A_K) {
                    vstore_lds(&sA[buf][(idx >> 2) * LDK + 8 * (idx & 3)], ra[v]);
                } else {
                    int kk = idx / (TBM / 8), r0 = 8 * (idx % (TBM / 8));
                    if constexpr (A_TR) {
                        vstore_lds(&sA[buf][kk * LDA_R + r0], ra[v]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) sA[buf][(r0 + i) * LDK + kk] = ra[v].e(i);
                    }
                }
            }
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            if (idx < TBN * BK / 8) {
                if constexpr (B_K) {
                    vstore_lds(&sB[buf][(idx >> 2) * LDK + 8 * (idx & 3)], rb[v]);
                } else {
                    int kk = idx / (TBN / 8), r0 = 8 * (idx % (TBN / 8));
                    if constexpr (B_TR) {
                        vstore_lds(&sB[buf][kk * LDB_R + r0], rb[v]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) sB[buf][(r0 + i) * LDK + kk] = rb[v].e(i);
                    }
                }
            }
        }
        }
    };

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) {
        load_tiles(kbeg);
        store_tiles(0);
        __syncthreads();
    }
    const int g = lane >> 4, i16 = lane & 15;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
        if constexpr (X3) {
            // k-contiguous hi / lo images, lane (i16, g) holds k = 8g .. 8g + 7 of its row
            bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const RT* ap = &sA[buf][(wm * WM + i * 16 + i16) * LDK + 8 * g];
                ah[i] = *reinterpret_cast<const bf16x8*>(ap);
                al[i] = *reinterpret_cast<const bf16x8*>(ap + A_ELEMS);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const RT* bp = &sB[buf][(wn * WN + j * 16 + i16) * LDK + 8 * g];
                bh[j] = *reinterpret_cast<const bf16x8*>(bp);
                bl[j] = *reinterpret_cast<const bf16x8*>(bp + B_ELEMS);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        } else if constexpr (BF) {
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (A_TR) {
                    const RT* ap = &sA[buf][(4 * g + (i16 >> 2)) * LDA_R + wm * WM + i * 16 + 4 * (i16 & 3)];
                    af[i] = frag_tr(ap, 16 * LDA_R);
                } else {
                    const RT* ap = &sA[buf][(wm * WM + i * 16 + i16) * LDK];
                    af[i] = PERM ? frag_perm(ap, g) : *reinterpret_cast<const bf16x8*>(ap + 8 * g);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (B_TR) {
                    const RT* bp = &sB[buf][(4 * g + (i16 >> 2)) * LDB_R + wn * WN + j * 16 + 4 * (i16 & 3)];
                    bfr[j] = frag_tr(bp, 16 * LDB_R);
                } else {
                    const RT* bp = &sB[buf][(wn * WN + j * 16 + i16) * LDK];
                    bfr[j] = PERM ? frag_perm(bp, g) : *reinterpret_cast<const bf16x8*>(bp + 8 * g);
                }
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        } else {
            // f32: lane group g feeds k-slot g with k = 8g + kk (same map for A and B)
            const RT* a_base = &sA[buf][(wm * WM + i16) * LDK + 8 * g];
            const RT* b_base = &sB[buf][(wn * WN + i16) * LDK + 8 * g];
            V8<float> af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) vload_lds(af[i], a_base + i * 16 * LDK);
#pragma unroll
            for (int j = 0; j < TN; ++j) vload_lds(bfr[j], b_base + j * 16 * LDK);
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].e(kk), bfr[j].e(kk), acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_tiles(buf ^ 1);
        __syncthreads();
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
                    int row = row_base + i * 16 + r, col = col_base + j * 16;
                    if (row < p.M && col < p.N) ws[(int64_t)row * p.N + col] = acc[i][j][r];
                }
        return;
    }
    const float* bias = p.bias ? p.bias + zb * p.strideBias : nullptr;
    const CT* mask = reinterpret_cast<const CT*>(p.mask);
    float* Cf = reinterpret_cast<float*>(p.C) + zb * p.strideC;
    bf16* Cb = reinterpret_cast<bf16*>(p.C) + zb * p.strideC;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            int col = col_base + j * 16;
            float bcol = (bias && col < p.N) ? bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = row_base + i * 16 + r;
                float v = p.alpha * acc[i][j][r] + bcol;
                if (row < p.M && col < p.N) {
                    if (mask && !(to_f32(mask[(int64_t)row * p.ldmask + col]) > 0.f)) v = 0.f;
                    if (p.relu) v = fmaxf(v, 0.f);
                    int64_t off = (int64_t)row * p.ldc + col;
                    if (p.c_bf16) {
                        Cb[off] = (bf16)v;
                    } else {
                        if (p.accumulate) v += Cf[off];
                        Cf[off] = v;
                    }
                }
                acc[i][j][r] = v;   // keep the epilogue value for the statistics below
            }
        }
    if (!p.stats) return;

    // Per-column (sum, M2) of this tile's valid rows, pre-activation values.
    // Two register passes (tile mean first) keep the later Chan merge stable.
    __shared__ float s_red[2][TBN];
    const int valid_rows = min(TBM, p.M - m0);
    float tsum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (row_base + i * 16 + r < p.M) s += acc[i][j][r];
        s = add_xor32(add_xor16(s));
        tsum[j] = s;
    }
    if (lane < 16)
#pragma unroll
        for (int j = 0; j < TN; ++j) s_red[wm][wn * WN + j * 16 + lane] = tsum[j];
    __syncthreads();
    float tmean[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        int c = wn * WN + j * 16 + (lane & 15);
        tsum[j] = s_red[0][c] + s_red[1][c];
        tmean[j] = tsum[j] / (float)valid_rows;
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
                    float d = acc[i][j][r] - tmean[j];
                    s += d * d;
                }
        s = add_xor32(add_xor16(s));
        if (lane < 16) s_red[wm][wn * WN + j * 16 + lane] = s;
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            int c = wn * WN + j * 16 + lane;
            if (n0 + c < p.N) {
                float* st = p.stats + (int64_t)blockIdx.x * 2 * p.N;
                st[n0 + c] = tsum[j];
                st[p.N + n0 + c] = s_red[0][c] + s_red[1][c];
            }
        }
    }
}

// Sum the split-K partials and apply the epilogue (bias / relu / accumulate).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const GemmParams p) {
    const int64_t MN = (int64_t)p.M * p.N;
    const int zb = blockIdx.y;
    const float* ws = p.splitk_ws + (int64_t)zb * p.splits * MN;
    const float* bias = p.bias ? p.bias + zb * p.strideBias : nullptr;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < MN; e += (int64_t)gridDim.x * 256) {
        float v = 0.f;
        for (int s = 0; s < p.splits; ++s) v += ws[s * MN + e];
        int row = (int)(e / p.N), col = (int)(e - (int64_t)row * p.N);
        v = p.alpha * v + (bias ? bias[col] : 0.f);
        if (p.relu) v = fmaxf(v, 0.f);
        int64_t off = zb * p.strideC + (int64_t)row * p.ldc + col;
        if (p.c_bf16) {
            reinterpret_cast<bf16*>(p.C)[off] = (bf16)v;
        } else {
            float* C = reinterpret_cast<float*>(p.C);
            C[off] = p.accumulate ? C[off] + v : v;
        }
    }
}

// The same with 4 columns per thread (16-B partial loads, one vector store)
// when N, ldc and strideC are multiples of 4 and C / the partials are 16-B
// aligned; per element the partials are summed in the same order.
__global__ void __launch_bounds__(256) splitk_reduce4_kernel(const GemmParams p) {
    const int64_t MN = (int64_t)p.M * p.N, n4 = MN / 4;
    const int zb = blockIdx.y;
    const float4* ws = reinterpret_cast<const float4*>(p.splitk_ws + (int64_t)zb * p.splits * MN);
    const float* bias = p.bias ? p.bias + zb * p.strideBias : nullptr;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < p.splits; ++s) {
            const float4 u = ws[s * n4 + e];
            v[0] += u.x; v[1] += u.y; v[2] += u.z; v[3] += u.w;
        }
        const int64_t e0 = e * 4;
        const int row = (int)(e0 / p.N), col = (int)(e0 - (int64_t)row * p.N);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = p.alpha * v[j] + (bias ? bias[col + j] : 0.f);
            if (p.relu) v[j] = fmaxf(v[j], 0.f);
        }
        const int64_t off = zb * p.strideC + (int64_t)row * p.ldc + col;
        if (p.c_bf16) {
            union { uint2 q; bf16 h[4]; } o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o.h[j] = (bf16)v[j];
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(p.C) + off) = o.q;
        } else {
            float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + off);
            float4 c = make_float4(v[0], v[1], v[2], v[3]);
            if (p.accumulate) {
                const float4 o = *C;
                c = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
            }
            *C = c;
        }
    }
}

// Many splits over a small output (the conv weight gradients: 100+ slices of
// a 288 x 32 .. 2304 x 256 tile set): 16 output quads x 16 split-parts per
// workgroup. Part q sums splits q, q + 16, ... (two 16-B loads in flight),
// then the 16 part sums of a quad are added in part order -- a fixed order,
// so the result is reproducible run to run (it differs from the serial
// order in rounding only).
__global__ void __launch_bounds__(256) splitk_reduce4p_kernel(const GemmParams p) {
    const int64_t MN = (int64_t)p.M * p.N, n4 = MN / 4;
    const int zb = blockIdx.y;
    const float4* ws = reinterpret_cast<const float4*>(p.splitk_ws + (int64_t)zb * p.splits * MN);
    const int part = threadIdx.x >> 4, ql = threadIdx.x & 15;
    const int64_t e = (int64_t)blockIdx.x * 16 + ql;
    __shared__ float4 red[16][16];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < n4) {
        int s = part;
        for (; s + 16 < p.splits; s += 32) {
            const float4 u0 = ws[s * n4 + e], u1 = ws[(s + 16) * n4 + e];
            v.x += u0.x; v.y += u0.y; v.z += u0.z; v.w += u0.w;
            v.x += u1.x; v.y += u1.y; v.z += u1.z; v.w += u1.w;
        }
        if (s < p.splits) {
            const float4 u = ws[s * n4 + e];
            v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
    }
    red[part][ql] = v;
    __syncthreads();
    if (part != 0 || e >= n4) return;
    float r[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const float4 u = red[q][ql];
        r[0] += u.x; r[1] += u.y; r[2] += u.z; r[3] += u.w;
    }
    const float* bias = p.bias ? p.bias + zb * p.strideBias : nullptr;
    const int64_t e0 = e * 4;
    const int row = (int)(e0 / p.N), col = (int)(e0 - (int64_t)row * p.N);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = p.alpha * r[j] + (bias ? bias[col + j] : 0.f);
        if (p.relu) r[j] = fmaxf(r[j], 0.f);
    }
    const int64_t off = zb * p.strideC + (int64_t)row * p.ldc + col;
    if (p.c_bf16) {
        union { uint2 q; bf16 h[4]; } o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.h[j] = (bf16)r[j];
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(p.C) + off) = o.q;
    } else {
        float4* C = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + off);
        float4 c = make_float4(r[0], r[1], r[2], r[3]);
        if (p.accumulate) {
            const float4 o = *C;
            c = make_float4(o.x + r[0], o.y + r[1], o.z + r[2], o.w + r[3]);
        }
        *C = c;
    }
}

int splitk_finish(const GemmParams& p, hipStream_t stream) {
    if (p.splits <= 1) return OCRK_OK;
    int64_t MN = (int64_t)p.M * p.N;
    const bool v4 = p.N % 4 == 0 && p.ldc % 4 == 0 && p.strideC % 4 == 0 &&
                    (uintptr_t)p.C % 16 == 0 && (uintptr_t)p.splitk_ws % 16 == 0;
    // many slices of a small output: split the slices over the threads; a
    // few slices of a large output (the recurrent dW, 8-31 slices of 0.5-2 M
    // values): one thread per quad keeps the grid small (it shares the CUs
    // with the persistent BPTT)
    if (v4 && (p.splits >= 32 || (p.splits >= 8 && MN / 4 < 65536))) {
        dim3 rg((unsigned)cdiv(MN / 4, 16), (unsigned)p.batch);
        splitk_reduce4p_kernel<<<rg, 256, 0, stream>>>(p);
        return launch_status("gemm splitk reduce");
    }
    if (v4) {
        dim3 rg((unsigned)std::min<int64_t>(cdiv(MN / 4, 256), 4096), (unsigned)p.batch);
        splitk_reduce4_kernel<<<rg, 256, 0, stream>>>(p);
        return launch_status("gemm splitk reduce");
    }
    dim3 rg((unsigned)std::min<int64_t>(cdiv(MN, 256), 4096), (unsigned)p.batch);
    splitk_reduce_kernel<<<rg, 256, 0, stream>>>(p);
    return launch_status("gemm splitk reduce");
}

size_t gemm_splitk_ws_bytes(int M, int N, int batch, int splits) {
    return splits > 1 ? (size_t)batch * splits * M * N * sizeof(float) : 0;
}

// fp32 GEMMs on the bf16x3 split (mode 0, the default) or the exact f32 MFMA
// (mode 1: ocrk_set_f32_gemm_mode, or OCRK_F32_MFMA=1 for the whole process).
// Process-wide, not per thread: torch's autograd runs a backward's launches on
// its own device thread, which must see the mode the training step set.
static std::atomic<int> g_f32_mode{0};

bool f32_exact_mfma() {
    return opt(OPT_F32_MFMA) == 1 || g_f32_mode.load(std::memory_order_relaxed) == 1;
}

template <typename CT, int AM, int BMD>
static int launch_tiles(const GemmParams& p0, hipStream_t stream) {
    GemmParams p = p0;
    int TBM = 128, TBN = p.N <= 32 ? 32 : (p.N <= 64 ? 64 : 128);
    dim3 grid((unsigned)cdiv(p.M, TBM), (unsigned)cdiv(p.N, TBN), (unsigned)(p.batch * p.splits));
    constexpr bool F32 = sizeof(CT) == 4;
    if (F32 && !f32_exact_mfma()) {
        if (TBN == 32) gemm_kernel<CT, AM, BMD, 128, 32, F32><<<grid, 256, 0, stream>>>(p);
        else if (TBN == 64) gemm_kernel<CT, AM, BMD, 128, 64, F32><<<grid, 256, 0, stream>>>(p);
        else gemm_kernel<CT, AM, BMD, 128, 128, F32><<<grid, 256, 0, stream>>>(p);
    } else if (TBN == 32) gemm_kernel<CT, AM, BMD, 128, 32><<<grid, 256, 0, stream>>>(p);
    else if (TBN == 64) gemm_kernel<CT, AM, BMD, 128, 64><<<grid, 256, 0, stream>>>(p);
    else gemm_kernel<CT, AM, BMD, 128, 128><<<grid, 256, 0, stream>>>(p);
    int st = launch_status("gemm");
    if (st != OCRK_OK) return st;
    return splitk_finish(p, stream);
}

template <typename CT>
static int dispatch_modes(const GemmParams& p, int amode, int bmode, hipStream_t s) {
#define GM(AMx, BMx) if (amode == AMx && bmode == BMx) return launch_tiles<CT, AMx, BMx>(p, s)
    GM(A_ROWK, B_NK);
    GM(A_ROWK, B_KN);
    GM(A_COLK, B_KN);
    GM(A_IM2COL, B_NK);
    GM(A_IM2COL_FLIP, B_NK);
    GM(A_IM2COL_T, B_KN);
#undef GM
    set_error("gemm: unsupported operand modes A=%d B=%d", amode, bmode);
    return OCRK_ERR_INVALID_ARG;
}

int gemm(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    if (p.M <= 0 || p.N <= 0 || p.batch <= 0) return OCRK_OK;
    OCRK_REQUIRE(p.K >= 0 && p.splits >= 1 && p.k_chunk > 0 && p.k_chunk % 32 == 0,
                 "gemm: bad K=%d splits=%d k_chunk=%d", p.K, p.splits, p.k_chunk);
    bool a_rows = (amode == A_COLK || amode == A_IM2COL_T);
    OCRK_REQUIRE(p.K % 8 == 0 || (a_rows && bmode == B_KN),
                 "gemm: K=%d must be a multiple of 8 for k-contiguous operands", p.K);
    OCRK_REQUIRE(!a_rows || p.M % 8 == 0, "gemm: M=%d must be a multiple of 8 for this A mode", p.M);
    OCRK_REQUIRE(bmode != B_KN || p.N % 8 == 0, "gemm: N=%d must be a multiple of 8 for B_KN", p.N);
    OCRK_REQUIRE(amode < A_IM2COL || p.convC % 8 == 0, "gemm: conv channels must be a multiple of 8");
    OCRK_REQUIRE(!(p.stats && (p.splits > 1 || p.batch > 1)), "gemm: stats need splits=1, batch=1");
    OCRK_REQUIRE(!(p.accumulate && p.c_bf16), "gemm: accumulate needs an f32 C");
    if (p.mask_bits || p.relu_bits) {                   // bit masks: the NT engine's staged epilogue only
        const int st = gemm_nt(p, amode, bmode, dtype, stream);
        OCRK_REQUIRE(st >= 0, "gemm: ReLU bit masks need the NT engine (bf16 C, staged epilogue) for this shape");
        return st;
    }
    int nt = gemm_pp(p, amode, bmode, dtype, stream);
    if (nt >= 0) return nt != OCRK_OK ? nt : splitk_finish(p, stream);
    nt = gemm_nt(p, amode, bmode, dtype, stream);
    if (nt < 0) nt = gemm_pptn(p, amode, bmode, dtype, stream);
    if (nt < 0) nt = gemm_tn(p, amode, bmode, dtype, stream);
    if (nt >= 0) return nt != OCRK_OK ? nt : splitk_finish(p, stream);
    if (dtype == OCRK_BF16) return dispatch_modes<bf16>(p, amode, bmode, stream);
    if (dtype == OCRK_F32) return dispatch_modes<float>(p, amode, bmode, stream);
    set_error("gemm: unsupported dtype %d", dtype);
    return OCRK_ERR_INVALID_ARG;
}

}  // namespace ocrk

// ------------------------------------------------------------------- C ABI
// Generic dense GEMM used by the recurrent projections and the logits layer:
// C[b] = alpha * op(A[b]) . op(B[b]) + bias (ReLU), op per trans flags:
//   trans_a = 0: A is [M][K] (lda), 1: A is [K][M];  trans_b = 0: B is [K][N], 1: B is [N][K].
extern "C" int ocrk_set_f32_gemm_mode(int mode) {
    OCRK_REQUIRE(mode == 0 || mode == 1, "ocrk_set_f32_gemm_mode: mode %d not 0 (bf16x3) or 1 (exact)", mode);
    return ocrk::g_f32_mode.exchange(mode);
}

extern "C" int ocrk_f32_gemm_exact(void) { return ocrk::f32_exact_mfma() ? 1 : 0; }

extern "C" size_t ocrk_gemm_workspace_size(int M, int N, int batch, int splits) {
    return ocrk::gemm_splitk_ws_bytes(M, N, batch, splits);
}

extern "C" int ocrk_gemm(int trans_a, int trans_b, int M, int N, int K, float alpha, const void* A,
                         int64_t lda, int64_t stride_a, const void* B, int64_t ldb, int64_t stride_b,
                         void* C, int64_t ldc, int64_t stride_c, int c_dtype, const float* bias,
                         int relu, int accumulate, int batch, int dtype, int splits, void* ws,
                         size_t ws_bytes, void* stream) {
    ocrk::GemmParams p = {};
    p.M = M; p.N = N; p.K = K; p.batch = batch < 1 ? 1 : batch;
    p.A = A; p.lda = lda; p.strideA = stride_a;
    p.B = B; p.ldb = ldb; p.strideB = stride_b;
    p.C = C; p.ldc = ldc; p.strideC = stride_c;
    p.c_bf16 = c_dtype == OCRK_BF16;
    p.bias = bias; p.strideBias = 0;
    p.relu = relu; p.accumulate = accumulate; p.alpha = alpha;
    p.splits = splits < 1 ? 1 : splits;
    int kc = (int)ocrk::cdiv(K, p.splits);
    p.k_chunk = (int)ocrk::cdiv(kc < 32 ? 32 : kc, 32) * 32;
    p.splits = (int)ocrk::cdiv(K > 0 ? K : 1, p.k_chunk);
    p.splitk_ws = (float*)ws;
    OCRK_REQUIRE(p.splits == 1 || ws_bytes >= ocrk::gemm_splitk_ws_bytes(M, N, p.batch, p.splits),
                 "ocrk_gemm: split-K workspace too small");
    int amode = trans_a ? ocrk::A_COLK : ocrk::A_ROWK;
    int bmode = trans_b ? ocrk::B_NK : ocrk::B_KN;
    return ocrk::gemm(p, amode, bmode, dtype, ocrk::as_stream(stream));
}
