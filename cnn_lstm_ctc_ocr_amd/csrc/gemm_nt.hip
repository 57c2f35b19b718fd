// Pipelined MFMA engine for the k-contiguous ("NT") operand modes, bf16:
//   A: A_ROWK (activations [M][lda]), A_IM2COL / A_IM2COL_FLIP (3x3 conv,
//      NHWC source, 8-channel chunks never cross a tap because C % 8 == 0)
//   B: B_NK (weights [N][ldb])
// which covers the conv forward / backward-data, the recurrent input
// projections and the dx GEMMs (gemm.h lists the modes).
//
// Structure (cdna_hip_programming.md section 5, "pipelining across
// barriers"): 256 threads, BM x BN x BK tiles, an S-stage LDS ring filled by
// LDS-DMA (buffer_load_dwordx4 ... lds) so the loads of the next S-1 stages
// are in flight while one stage is on MFMA; one raw s_barrier per k-step,
// counted s_waitcnt vmcnt (never __syncthreads inside the loop: its fence
// would drain the DMA queue).
// LDS images are lane-linear: one wave instruction writes 1 KB = 8 rows of
// 128 B (BK = 64) or 16 rows of 64 B (BK = 32). The 16-B chunk index of each
// row is XOR-swizzled on the GLOBAL side (BK=64: slot = chunk ^ (row & 7);
// BK=32: slot = chunk ^ ((row >> 2) & 3)) so every 8 lanes of an MFMA
// fragment read (16 rows, one chunk each) hit 8 distinct 16-B bank groups.
// Zero fill (im2col padding taps, rows >= M / N, k >= K): the lane's buffer
// offset is pushed past the resource's num_records, which returns 0.
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr unsigned NT_OOB = 0x80000000u;

constexpr unsigned NT_BADROW = 0xFFFFFFFFu;        // row outside the matrix

__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

// F32 (the fp32 serving / parity path): A and B are fp32, staged by the same
// LDS-DMA ring (BK = 32 -> 128-B rows, the bf16 BK = 64 geometry), and every
// MFMA fragment is split at the read into bf16 hi / lo (mfma_util.h
// split8_bf16) for the three bf16 products ah.bh + ah.bl + al.bh.
// EXACT (with F32): exact fp32 products on v_mfma_f32_16x16x4_f32 instead of the split --
// the fp32 Trainer's conv tower (kernels.f32_exact); lane group g supplies k = 8g + e to
// the e-th of 8 MFMAs per 32-deep step (any k order sums the same products).
// TU (tap-uniform im2col, C % BK == 0 and every K slice a multiple of BK): a k-tile of
// BK channels never crosses a 3x3 tap, so the tap, its (dh, dw) shift and the channel
// offset are wave-uniform per k-step -- carried as scalars from one k-step to the next
// instead of a per-lane k / C division -- and each A row's border test is one bit of a
// 9-bit valid-tap mask built in the prologue (the generic path spent ~85 VALU per
// 32 MFMAs on this address arithmetic; profiles/r6_nt_sq.txt).
template <int BM, int BN, int BK, int S, int WAVES_M, int AM, int NW = 4, bool F32 = false, bool EXACT = false,
          bool X6 = false, bool TU = false>
__global__ void __launch_bounds__(NW * 64) gemm_nt_kernel(const GemmParams p) {
    // 8-wave tiles hold 128 accumulators per lane: no BN-statistics epilogue
    // (its second pass over the accumulators would spill); launch_nt routes
    // calls with stats to a 4-wave tile.
    constexpr bool ST = NW == 4;
    constexpr int WAVES_N = NW / WAVES_M;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ESZ = F32 ? 4 : 2;                      // operand element bytes
    constexpr int EPC = 16 / ESZ;                         // elements per 16-B chunk
    constexpr int ROWB = BK * ESZ;                        // bytes per LDS row
    constexpr int RPI = 1024 / ROWB;                      // rows per wave instruction
    constexpr int CPR = ROWB / 16;                        // 16-B chunks per row
    constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
    // DMA instructions per thread per stage. Every wave issues the same count
    // (the vmcnt arithmetic relies on it): when BN < 4 * RPI the spare waves
    // repeat another wave's B instruction (same bytes to the same LDS rows).
    constexpr int NA = BM / (NW * RPI), NB = BN >= NW * RPI ? BN / (NW * RPI) : 1;
    constexpr int BBLK = BN / RPI;                        // B row blocks per stage
    constexpr int NPS = NA + NB;
    static_assert((BK == 32 || BK == 64) && S >= 2, "BK 32 or 64, >= 2 stages");
    static_assert(!F32 || BK == 32, "fp32 operands: BK = 32 (128-B rows)");
    static_assert(BM % (NW * RPI) == 0 && BN % RPI == 0 && (BN < NW * RPI || BN % (NW * RPI) == 0), "tile");
    static_assert(TM >= 1 && TN >= 1, "wave tile");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const TileIdx tix = xcd_tile((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
    if (!tix.valid) return;
    const int m0 = tix.bm * BM, n0 = tix.bn * BN;
    const int zb = blockIdx.z / p.splits, zs = blockIdx.z - zb * p.splits;
    const char* A = reinterpret_cast<const char*>(p.A) + zb * p.strideA * ESZ;
    const char* B = reinterpret_cast<const char*>(p.B) + zb * p.strideB * ESZ;
    const int kbeg = zs * p.k_chunk;
    const int kend = min(p.K, kbeg + p.k_chunk);
    const int nk = max(0, (kend - kbeg + BK - 1) / BK);

    // buffer resources (num_records = bytes; anything beyond reads as 0)
    int64_t a_elems, b_elems = (int64_t)p.N * p.ldb;
    if constexpr (AM == A_ROWK) a_elems = (int64_t)p.M * p.lda;
    else a_elems = (int64_t)p.M * p.convC;               // NHWC source with M = B*H*W pixels
    const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(A, a_elems * ESZ);
    const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(B, b_elems * ESZ);

    // this lane's row within its instruction and the chunk it fetches (global side of the swizzle);
    // instruction rows start at multiples of RPI, so row & (RPI-1) == lrow
    const int lrow = lane / CPR;
    const int chunk = ROWB == 128 ? ((lane & 7) ^ lrow) : ((lane & 3) ^ ((lrow >> 2) & 3));

    // per-lane row geometry of each DMA instruction, as 32-bit byte offsets
    // (every operand here is < 2 GB) with NT_BADROW for rows past M / N
    unsigned aoff[NA], ahw[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int m = m0 + (i * NW + wave) * RPI + lrow;
        ahw[i] = 0;
        if constexpr (AM == A_ROWK) {
            aoff[i] = m < p.M ? (unsigned)((int64_t)m * p.lda * ESZ) : NT_BADROW;
        } else {
            const int W = p.convW, H = p.convH;
            const int mm = m < p.M ? m : 0;
            const int w = mm % W, h = (mm / W) % H;
            ahw[i] = ((unsigned)h << 16) | (unsigned)w;
            aoff[i] = m < p.M ? (unsigned)((int64_t)mm * p.convC * ESZ) : NT_BADROW;
        }
    }
    unsigned boff[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int n = n0 + ((i * NW + wave) % BBLK) * RPI + lrow;
        boff[i] = n < p.N ? (unsigned)((int64_t)n * p.ldb * ESZ) : NT_BADROW;
    }

    // TU: valid-tap masks of this lane's A rows (bit t: tap t = 3 kh + kw keeps the
    // shifted pixel inside the image) and the k-step's tap / channel offset as scalars
    unsigned tmask[NA];
    int tu_tap = 0, tu_cc = 0;
    if constexpr (TU) {
        static_assert(AM != A_ROWK, "TU is the im2col form");
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            tmask[i] = 0;
            if (aoff[i] == NT_BADROW) continue;
            const int h = (int)(ahw[i] >> 16), w = (int)(ahw[i] & 0xffff);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int kh = t / 3, kw = t % 3;
                const int dh = AM == A_IM2COL_FLIP ? 1 - kh : kh - 1, dw = AM == A_IM2COL_FLIP ? 1 - kw : kw - 1;
                const int hh = h + dh, ww = w + dw;
                if (hh >= 0 && hh < p.convH && ww >= 0 && ww < p.convW) tmask[i] |= 1u << t;
            }
        }
        tu_tap = __builtin_amdgcn_readfirstlane(kbeg / p.convC);
        tu_cc = __builtin_amdgcn_readfirstlane(kbeg - tu_tap * p.convC);
    }
    const unsigned lane_koff = (unsigned)(EPC * chunk * ESZ);

    // TU: k-steps are issued in order (kt = 0, 1, 2, ...), each advancing the tap state by BK
    auto issue_tu = [&](int kt, int stage) {
        const int kg = kbeg + kt * BK;                    // wave-uniform
        const bool kok = kg < kend;
        char* sa = smem + stage * STAGE;
        char* sb = sa + A_BYTES;
        const int kh = tu_tap / 3, kw = tu_tap - 3 * (tu_tap / 3);
        const int dh = AM == A_IM2COL_FLIP ? 1 - kh : kh - 1, dw = AM == A_IM2COL_FLIP ? 1 - kw : kw - 1;
        const unsigned toff = (unsigned)(((dh * p.convW + dw) * p.convC + tu_cc) * ESZ) + lane_koff;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const bool ok = kok && ((tmask[i] >> tu_tap) & 1u);
            lds_dma16(ra, sa + ((i * NW + wave) * RPI) * ROWB, ok ? aoff[i] + toff : NT_OOB);
        }
        const unsigned kb = (unsigned)(kg * ESZ) + lane_koff;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const bool ok = kok && boff[i] != NT_BADROW;
            lds_dma16(rb, sb + (((i * NW + wave) % BBLK) * RPI) * ROWB, ok ? boff[i] + kb : NT_OOB);
        }
        tu_cc += BK;
        if (tu_cc >= p.convC) { tu_cc = 0; ++tu_tap; }
    };

    auto issue = [&](int kt, int stage) {
        if constexpr (TU) {
            issue_tu(kt, stage);
            return;
        }
        const int k = kbeg + kt * BK + EPC * chunk;
        const bool kok = k < kend;
        char* sa = smem + stage * STAGE;
        char* sb = sa + A_BYTES;
        int tap_off = 0, dh = 0, dw = 0;
        if constexpr (AM != A_ROWK) {
            const int C = p.convC;
            const int tap = kok ? k / C : 0;
            const int cch = k - tap * C;
            const int kh = tap / 3, kw = tap - kh * 3;
            if constexpr (AM == A_IM2COL_FLIP) { dh = 1 - kh; dw = 1 - kw; }
            else { dh = kh - 1; dw = kw - 1; }
            tap_off = ((dh * p.convW + dw) * C + cch) * ESZ;
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            bool ok = kok && aoff[i] != NT_BADROW;
            unsigned voff;
            if constexpr (AM == A_ROWK) {
                voff = aoff[i] + (unsigned)(k * ESZ);
            } else {
                const int hh = (int)(ahw[i] >> 16) + dh, ww = (int)(ahw[i] & 0xffff) + dw;
                ok = ok && hh >= 0 && hh < p.convH && ww >= 0 && ww < p.convW;
                voff = aoff[i] + (unsigned)tap_off;
            }
            lds_dma16(ra, sa + ((i * NW + wave) * RPI) * ROWB, ok ? voff : NT_OOB);
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const bool ok = kok && boff[i] != NT_BADROW;
            lds_dma16(rb, sb + (((i * NW + wave) % BBLK) * RPI) * ROWB, ok ? boff[i] + (unsigned)(k * ESZ) : NT_OOB);
        }
    };

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int st = 0; st < S - 1; ++st)
        if (st < nk) issue(st, st);
    const int i16 = lane & 15, g = lane >> 4;
    const int swz = ROWB == 128 ? (lane & 7) : ((i16 >> 2) & 3);
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed: the stages issued after it (up to S-2 of them) may stay in flight
        const int ahead = min(S - 2, nk - 1 - kt);
        if constexpr (S >= 5) {
            if (ahead >= 4) vm_wait<4 * NPS>();
            else if (ahead == 3) vm_wait<3 * NPS>();
            else if (ahead == 2) vm_wait<2 * NPS>();
            else if (ahead == 1) vm_wait<NPS>();
            else vm_wait<0>();
        } else if constexpr (S >= 4) {
            if (ahead >= 2) vm_wait<2 * NPS>();
            else if (ahead == 1) vm_wait<NPS>();
            else vm_wait<0>();
        } else if constexpr (S == 3) {
            if (ahead >= 1) vm_wait<NPS>();
            else vm_wait<0>();
        } else {
            vm_wait<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                     // everyone's stage kt is in, stage kt-1 is free
        asm volatile("" ::: "memory");
        if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
        const char* sa = smem + (kt % S) * STAGE;
        const char* sb = sa + A_BYTES;
        if constexpr (F32 && EXACT && X6) {
            // products to fp32 precision on the bf16 MFMA: each fragment split into
            // hi / mid / lo at the read, six products per tile pair, smallest first
            const int s0 = ((2 * g) ^ swz) * 16, s1 = ((2 * g + 1) ^ swz) * 16;
            auto frag = [&](const char* row, bf16x8& h, bf16x8& m, bf16x8& l) {
                V8<float> v;
                v.q0 = *reinterpret_cast<const f32x4*>(row + s0);
                v.q1 = *reinterpret_cast<const f32x4*>(row + s1);
                u32x4 a, b, c;
                split8_bf16x3(v, a, b, c);
                h = __builtin_bit_cast(bf16x8, a);
                m = __builtin_bit_cast(bf16x8, b);
                l = __builtin_bit_cast(bf16x8, c);
            };
            bf16x8 bh[TN], bm[TN], bl[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) frag(sb + (wn * WN + j * 16 + i16) * ROWB, bh[j], bm[j], bl[j]);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 ah, am, al;
                frag(sa + (wm * WM + i * 16 + i16) * ROWB, ah, am, al);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
                }
            }
            continue;
        }
        if constexpr (F32 && EXACT) {
            const int s0 = ((2 * g) ^ swz) * 16, s1 = ((2 * g + 1) ^ swz) * 16;
            auto frag = [&](const char* row) {
                V8<float> v;
                v.q0 = *reinterpret_cast<const f32x4*>(row + s0);
                v.q1 = *reinterpret_cast<const f32x4*>(row + s1);
                return v;
            };
            V8<float> bv[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = frag(sb + (wn * WN + j * 16 + i16) * ROWB);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const V8<float> av = frag(sa + (wm * WM + i * 16 + i16) * ROWB);
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.e(e), bv[j].e(e), acc[i][j], 0, 0, 0);
            }
            continue;
        }
        if constexpr (F32) {
            // lane group g holds k = 8g .. 8g + 7 = fp32 chunks 2g, 2g + 1 of its row
            const int s0 = ((2 * g) ^ swz) * 16, s1 = ((2 * g + 1) ^ swz) * 16;
            auto frag = [&](const char* row, bf16x8& hi, bf16x8& lo) {
                V8<float> v;
                v.q0 = *reinterpret_cast<const f32x4*>(row + s0);
                v.q1 = *reinterpret_cast<const f32x4*>(row + s1);
                u32x4 h, l;
                split8_bf16(v, h, l);
                hi = __builtin_bit_cast(bf16x8, h);
                lo = __builtin_bit_cast(bf16x8, l);
            };
            bf16x8 bh[TN], bl[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) frag(sb + (wn * WN + j * 16 + i16) * ROWB, bh[j], bl[j]);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 ah, al;
                frag(sa + (wm * WM + i * 16 + i16) * ROWB, ah, al);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
                }
            }
            continue;
        }
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
            const int slot = ((kk * 4 + g) ^ swz) * 16;
            bf16x8 bfr[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (wn * WN + j * 16 + i16) * ROWB + slot);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(sa + (wm * WM + i * 16 + i16) * ROWB + slot);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
            }
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
    const bf16* mask = reinterpret_cast<const bf16*>(p.mask);   // the C type's ReLU mask (F32: fp32, unstaged)
    const float* maskf = reinterpret_cast<const float*>(p.mask);
    float* Cf = reinterpret_cast<float*>(p.C) + zb * p.strideC;
    bf16* Cb = reinterpret_cast<bf16*>(p.C) + zb * p.strideC;
    // Staged epilogue (bf16 C): the tile goes through LDS (pitch TP bytes, after
    // the statistics scratch) and leaves as 16-B row chunks, so a wave's store
    // covers whole output rows instead of 16 two-byte columns x 4 rows; the
    // ReLU mask comes in the same way. Values are bit-identical to the direct path.
    constexpr int TP = BN * 2 + 16, T_OFF = 4096, CPT = BN / 8;
    constexpr bool TILE_FITS = T_OFF + BM * TP <= S * STAGE;
    const bool staged = TILE_FITS && p.epi_staged;
    char* tile = smem + T_OFF;
    const uint8_t* mbits = reinterpret_cast<const uint8_t*>(p.mask_bits);
    if (staged && (mask || mbits)) {
        for (int q = tid; q < BM * CPT; q += NW * 64) {
            const int r = q / CPT, cc = q - r * CPT;
            const int row = m0 + r, col = n0 + 8 * cc;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (row < p.M && col < p.N) {
                if (mbits) {                               // one byte of bits -> 8 bf16 (1.0 or 0)
                    const unsigned m = mbits[(int64_t)row * (p.N >> 3) + (col >> 3)];
                    unsigned w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        w[i] = ((m >> (2 * i)) & 1u ? 0x3f80u : 0u) | ((m >> (2 * i + 1)) & 1u ? 0x3f800000u : 0u);
                    v = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
                    v = *reinterpret_cast<const uint4*>(mask + (int64_t)row * p.ldmask + col);
                }
            }
            *reinterpret_cast<uint4*>(tile + r * TP + cc * 16) = v;
        }
        __syncthreads();
    }
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
                    if (staged) {
                        bf16* e = reinterpret_cast<bf16*>(tile + (row - m0) * TP + (col - n0) * 2);
                        if ((mask || mbits) && !((float)*e > 0.f)) v = 0.f;
                        if (p.relu) v = fmaxf(v, 0.f);
                        *e = (bf16)v;
                    } else {
                        if constexpr (F32) {
                            if (maskf && !(maskf[(int64_t)row * p.ldmask + col] > 0.f)) v = 0.f;
                        } else {
                            if (mask && !((float)mask[(int64_t)row * p.ldmask + col] > 0.f)) v = 0.f;
                        }
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
                acc[i][j][r] = v;
            }
    }
    if (staged) {
        __syncthreads();
        uint8_t* rbits = reinterpret_cast<uint8_t*>(p.relu_bits);
        for (int q = tid; q < BM * CPT; q += NW * 64) {
            const int r = q / CPT, cc = q - r * CPT;
            const int row = m0 + r, col = n0 + 8 * cc;
            if (row < p.M && col < p.N) {
                const uint4 v = *reinterpret_cast<const uint4*>(tile + r * TP + cc * 16);
                *reinterpret_cast<uint4*>(Cb + (int64_t)row * p.ldc + col) = v;
                if (rbits) {                               // the 8 values' (> 0) bits: one byte
                    const unsigned w[4] = {v.x, v.y, v.z, v.w};
                    unsigned m = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        m |= (__uint_as_float(w[i] << 16) > 0.f ? 1u : 0u) << (2 * i);
                        m |= (__uint_as_float(w[i] & 0xffff0000u) > 0.f ? 1u : 0u) << (2 * i + 1);
                    }
                    rbits[(int64_t)row * (p.N >> 3) + (col >> 3)] = (uint8_t)m;
                }
            }
        }
    }
    if constexpr (!ST) return;
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
        s = add_xor32(add_xor16(s));
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
        s = add_xor32(add_xor16(s));
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
                float* st = p.stats + (int64_t)tix.bm * 2 * p.N;
                st[n0 + c] = tsum[j];
                st[p.N + n0 + c] = m2;
            }
        }
    }
}

template <int BM, int BN, int BK, int S, int WAVES_M, int AM, int NW, bool F32, bool EXACT, bool X6, bool TU>
int launch_nt_k(const GemmParams& p, hipStream_t stream) {
    constexpr int LDS = S * (BM + BN) * BK * (F32 ? 4 : 2);
    static DeviceOnce configured;
    set_dyn_lds(configured,
                reinterpret_cast<const void*>(&gemm_nt_kernel<BM, BN, BK, S, WAVES_M, AM, NW, F32, EXACT, X6, TU>),
                LDS);
    dim3 grid(xcd_grid((int)cdiv(p.M, BM), (int)cdiv(p.N, BN)), 1u, (unsigned)(p.batch * p.splits));
    gemm_nt_kernel<BM, BN, BK, S, WAVES_M, AM, NW, F32, EXACT, X6, TU><<<grid, NW * 64, LDS, stream>>>(p);
    return launch_status("gemm_nt");
}

// the tap-uniform im2col form where it applies (option NT_TAP_UNIFORM, default on)
template <int BK, int AM>
bool nt_tap_uniform(const GemmParams& p) {
    return AM != A_ROWK && opt(OPT_NT_TAP_UNIFORM) != 0 && p.convC % BK == 0 &&
           (p.splits == 1 || p.k_chunk % BK == 0);
}

template <int BM, int BN, int BK, int S, int WAVES_M, int AM, int NW = 4, bool F32 = false, bool EXACT = false,
          bool X6 = false>
int launch_nt(const GemmParams& p, hipStream_t stream) {
    if constexpr (NW == 8 && !F32) {
        if (p.stats) return launch_nt<128, 128, 64, 2, 2, AM, 4>(p, stream);
    }
    if constexpr (AM != A_ROWK) {
        if (nt_tap_uniform<BK, AM>(p))
            return launch_nt_k<BM, BN, BK, S, WAVES_M, AM, NW, F32, EXACT, X6, true>(p, stream);
    }
    return launch_nt_k<BM, BN, BK, S, WAVES_M, AM, NW, F32, EXACT, X6, false>(p, stream);
}

// fp32 operands (BK = 32: 128-B fp32 rows) on the bf16x3 split, or with EXACT products
// (X6: to fp32 precision as six bf16 products, else the f32 MFMA)
template <int AM, bool EXACT = false, bool X6 = false>
int dispatch_nt_f32(const GemmParams& p, hipStream_t s) {
    if (p.N <= 32) return launch_nt<128, 32, 32, 3, 4, AM, 4, true, EXACT, X6>(p, s);
    if (p.N <= 64) return launch_nt<128, 64, 32, 3, 2, AM, 4, true, EXACT, X6>(p, s);
    return launch_nt<128, 128, 32, 2, 2, AM, 4, true, EXACT, X6>(p, s);
}

// Tile configurations (OCRK_GEMM_NT_CFG picks one for experiments; by default
// the shape decides). BM x BN x BK / stages -> LDS -> workgroups per CU:
//   0: 256 x 128 x 64 / 3 -> 144 KB -> 1     1: 128 x 128 x 64 / 2 -> 64 KB -> 2
//   2: 128 x 128 x 32 / 3 ->  48 KB -> 3     3: 128 x 128 x 64 / 3 -> 96 KB -> 1
//   4: 256 x 128 x 32 / 4 ->  96 KB -> 1     5: 128 x 128 x 32 / 4 -> 64 KB -> 2
//   6: 256 x 256 x 64 / 2, 8 waves -> 128 KB -> 1 (2 waves per SIMD)
//   7: 256 x 128 x 64 / 2, 8 waves ->  96 KB -> 1   8: 256 x 256 x 32 / 3, 8 waves -> 96 KB
//   9: 256 x 256 x 32 / 4, 8 waves -> 128 KB       10: 256 x 128 x 32 / 4, 8 waves -> 64 KB -> 2
//  11: 128 x 128 x 32 / 6 -> 96 KB -> 1           12: 128 x 128 x 32 / 5 -> 80 KB -> 2
//  13: 128 x 128 x 64 / 4 -> 128 KB -> 1          14: 128 x 64 x 64 / 3 -> 72 KB -> 2
#ifdef OCRK_EXPERIMENTS
int nt_cfg() {                                       // tools-only build (make exp)
    static const int c = [] {
        const char* e = getenv("OCRK_GEMM_NT_CFG");
        return e ? atoi(e) : -1;
    }();
    return c;
}
#endif

template <int AM>
int dispatch_nt(const GemmParams& p, hipStream_t s) {
#ifdef OCRK_EXPERIMENTS
    switch (nt_cfg()) {                                  // experiments (tools/gemm_sweep.sh, make exp)
        case 0: return launch_nt<256, 128, 64, 3, 2, AM>(p, s);
        case 1: return launch_nt<128, 128, 64, 2, 2, AM>(p, s);
        case 2: return launch_nt<128, 128, 32, 3, 2, AM>(p, s);
        case 3: return launch_nt<128, 128, 64, 3, 2, AM>(p, s);
        case 4: return launch_nt<256, 128, 32, 4, 2, AM>(p, s);
        case 5: return launch_nt<128, 128, 32, 4, 2, AM>(p, s);
        case 6: return launch_nt<256, 256, 64, 2, 2, AM, 8>(p, s);
        case 7: return launch_nt<256, 128, 64, 2, 4, AM, 8>(p, s);
        case 8: return launch_nt<256, 256, 32, 3, 2, AM, 8>(p, s);
        case 9: return launch_nt<256, 256, 32, 4, 2, AM, 8>(p, s);
        case 10: return launch_nt<256, 128, 32, 4, 4, AM, 8>(p, s);
        case 11: return launch_nt<128, 128, 32, 6, 2, AM>(p, s);
        case 12: return launch_nt<128, 128, 32, 5, 2, AM>(p, s);
        case 13: return launch_nt<128, 128, 64, 4, 2, AM>(p, s);
        case 14: return launch_nt<128, 64, 64, 3, 2, AM>(p, s);
        case 15: return launch_nt<64, 96, 64, 3, 2, AM>(p, s);
        case 16: return launch_nt<64, 128, 32, 4, 2, AM>(p, s);
        case 17: return launch_nt<128, 96, 64, 3, 2, AM>(p, s);
        case 18: return launch_nt<64, 128, 64, 3, 2, AM>(p, s);
        default: break;
    }
#endif
    // measured on MI355X (tools/bench_gemm.py): narrow N -> BK=32, 3 stages;
    // wide N with enough row tiles -> 256 x 256 (8 waves); else 128 x 128 x 64, 2 stages
    if (p.N <= 32) return launch_nt<128, 32, 32, 3, 4, AM>(p, s);
    if (p.N <= 64) return launch_nt<128, 64, 32, 3, 2, AM>(p, s);
    // N in (64, 96] (the logits, 96 classes): 64 x 96 tiles, three stages -- twice the
    // workgroups of a 128 x 128 tile with no idle columns (19.9 vs 29.9 us at 32000 x 96 x 1024)
    if (p.N <= 96) return launch_nt<64, 96, 64, 3, 2, AM>(p, s);
    // (the 256 x 256 tile's C does not fit the staged epilogue: bit masks stay on 128 x 128)
    if (p.N >= 512 && p.M >= 16384 && !p.mask_bits && !p.relu_bits) return launch_nt<256, 256, 64, 2, 2, AM, 8>(p, s);
    return launch_nt<128, 128, 64, 2, 2, AM>(p, s);
}

}  // namespace

bool gemm_nt_enabled() {
    return opt(OPT_GEMM_NT) != 0;              // 0: the generic engine only
}

bool nt_staged_enabled() {
    return opt(OPT_GEMM_NT_STAGED) != 0;       // 0: direct 2-B stores
}

// Runs the NT engine when it covers (mode, dtype); returns -1 when it does not.
int gemm_nt(const GemmParams& p0, int amode, int bmode, int dtype, hipStream_t stream) {
    if (!gemm_nt_enabled() || bmode != B_NK) return -1;
    if (dtype == OCRK_F32) {
        // fp32: the bf16x3 split on this ring (the generic engine keeps the short-K
        // shapes and OCRK_F32_MFMA=1)
        // (K >= 256 here: the first recurrent layer's input projection, K = 256, ran 3x
        // slower on the generic engine's bf16x3 staging -- 463 vs ~150 us per C5 bucket)
        // exact mode (the fp32 Trainer's conv tower): the implicit-GEMM convolutions on this
        // ring with exact f32 products (option NT_F32_EXACT=0: the generic engine)
        const bool exact = f32_exact_mfma();
        if (exact && (amode == A_ROWK || !opt(OPT_NT_F32_EXACT))) return -1;
        // (a ReLU mask -- the masked data gradients -- is fp32 here and read unstaged)
        if (p0.c_bf16 || (p0.mask && !opt(OPT_NT_F32_MASK)) || p0.K % 4 != 0 || (p0.k_chunk < 256 && p0.N > 64))
            return -1;
        GemmParams p = p0;
        p.epi_staged = 0;
        if (amode == A_ROWK) {
            if (p.lda % 4 != 0 || p.ldb % 4 != 0) return -1;
            return dispatch_nt_f32<A_ROWK>(p, stream);
        }
        if (p.convC % 4 != 0 || p.ldb % 4 != 0) return -1;
        const bool x6 = exact && opt(OPT_NT_F32_X6);
        if (amode == A_IM2COL) return x6 ? dispatch_nt_f32<A_IM2COL, true, true>(p, stream)
                                      : exact ? dispatch_nt_f32<A_IM2COL, true>(p, stream)
                                              : dispatch_nt_f32<A_IM2COL>(p, stream);
        if (amode == A_IM2COL_FLIP) return x6 ? dispatch_nt_f32<A_IM2COL_FLIP, true, true>(p, stream)
                                           : exact ? dispatch_nt_f32<A_IM2COL_FLIP, true>(p, stream)
                                                   : dispatch_nt_f32<A_IM2COL_FLIP>(p, stream);
        return -1;
    }
    if (dtype != OCRK_BF16) return -1;
    GemmParams p = p0;
    // 16-B row chunks of C (and of the mask) must be aligned and never straddle N
    p.epi_staged = nt_staged_enabled() && p.c_bf16 && p.splits == 1 && p.N % 8 == 0 && p.ldc % 8 == 0 &&
                   p.strideC % 8 == 0 && (uintptr_t)p.C % 16 == 0 &&
                   (!p.mask || (p.ldmask % 8 == 0 && (uintptr_t)p.mask % 16 == 0));
    // wide N with short K (a few k-steps: store-bound) runs better on the
    // generic engine's three resident workgroups per CU (measured)
    if (p.K % 8 != 0 || (p.k_chunk < 512 && p.N > 64)) return -1;
    // bit masks (mask_bits / relu_bits) live in the staged epilogue only
    if ((p.mask_bits || p.relu_bits) && (!p.epi_staged || p.batch != 1 || p.ldc != p.N)) return -1;
    if (amode == A_ROWK) {
        if (p.lda % 8 != 0 || p.ldb % 8 != 0) return -1;          // 16-B aligned rows
        return dispatch_nt<A_ROWK>(p, stream);
    }
    if (amode == A_IM2COL) return dispatch_nt<A_IM2COL>(p, stream);
    if (amode == A_IM2COL_FLIP) return dispatch_nt<A_IM2COL_FLIP>(p, stream);
    return -1;
}

}  // namespace ocrk
