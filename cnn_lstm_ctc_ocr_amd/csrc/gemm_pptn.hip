// 8-wave ping-pong MFMA engine for the k-major ("TN") weight gradients, bf16
// operands, f32 C:
//   C[M,N] (+)= A^T . B,  A stored [K][lda] (A(m,k) = A[k*lda + m]),
//                         B stored [K][ldb] (B(k,n) = B[k*ldb + n])
// -- the recurrent and logits weight gradients dW = x^T dG, h_prev^T dG over
// the T*B time-major rows (model_bu.py:167-199 / model.py:216-220, the
// gradient of the input projection and of the recurrent product), K = T*B.
//
// Same schedule as gemm_pp.hip (read it first): 256 x 256 x 64 tiles, 512
// threads as 2 (rows) x 4 (columns) waves, four phases per K-tile over the
// output quadrants, four 16-KB LDS-DMA units per K-tile issued one per phase
// for the next K-tile, waves 4-7 one barrier behind waves 0-3, the same RAW /
// WAR barrier arithmetic and counted vmcnt waits. Only the operand images
// differ: both operands are k-major, so each unit is two [64 k][64 columns]
// bf16 blocks (128-B rows, 16-B chunk slot = chunk ^ (k & 7), swizzled on
// the global side) and the MFMA fragments come out of them with
// ds_read_b64_tr_b16 (frag_tr: 8 k-values of one column per lane, the same
// k order for A and B).
//   A blocks b = 0..3 hold columns m0 + 64b .. +64: U0 = {0, 2} (row
//   quadrant 0 of both row halves), U3 = {1, 3};
//   B blocks hold the column halves two waves read in one phase:
//   U1 = {[wn0 q0 | wn1 q0], [wn2 q0 | wn3 q0]}, U2 = the q1 halves.
// Work items = output tiles x K slices, one per workgroup; split K writes f32
// partials (reduced by gemm.hip's splitk_finish), else C (+)= in place.
//
// AM = A_IM2COL_T: the conv weight gradient dW[(kh,kw,c)][cout] = im2col(x)^T
// . dy over the B*H*W pixels (model.py:84-109 backward). A k-row of a
// 64-column A block is then 64 channels of ONE tap at the shifted pixel --
// 128 contiguous bytes of the NHWC input (Cin % 64 == 0) -- or zeros where
// the tap leaves the image, so the same LDS-DMA unit layout applies with a
// per-lane source offset.
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr unsigned TT_OOB = 0x80000000u;

__device__ __forceinline__ void tt_dma16(const i32x4_t& r, void* lds, unsigned voff) {
    lds_dma16_asm(r, lds, voff);
}

__device__ __forceinline__ void tt_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int AM>
__global__ void __launch_bounds__(512) gemm_pptn_kernel(const GemmParams p) {
    constexpr int BM = 256, BN = 256, BK = 64, ROWB = 128, BLK = BK * ROWB;   // 8-KB [64 k][64 col] block
    constexpr int A_BYTES = 4 * BLK, BUF = 8 * BLK;
    constexpr int NUA = 2, NUB = 2;                       // DMA instructions per wave per unit
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int i16 = lane & 15, g = lane >> 4;

    // ---- the item: XCD-contiguous ranges as in gemm_pp (one item per workgroup)
    const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
    const int nT = tm * tn;
    const int nitems = nT * p.batch * p.splits;
    const int per = (nitems + 7) >> 3;
    const int w = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (w >= nitems || (int)(blockIdx.x >> 3) >= per) return;
    const int z = w / nT, t = w - z * nT;
    constexpr int GM = 4;
    const int gsz = GM * tn, grp = t / gsz, first = grp * GM;
    const int gm = min(GM, tm - first), rr = t - grp * gsz;
    const int m0 = (first + rr % gm) * BM, n0 = (rr / gm) * BN;
    const int zb = z / p.splits, zs = z - zb * p.splits;
    const bf16* A = reinterpret_cast<const bf16*>(p.A) + zb * p.strideA;
    const bf16* B = reinterpret_cast<const bf16*>(p.B) + zb * p.strideB;
    const int kbeg = zs * p.k_chunk;
    const int kend = min(p.K, kbeg + p.k_chunk);
    const int nk = max(1, (kend - kbeg + BK - 1) / BK);
    const i32x4_t ra = uniform_rsrc_words(A, (int64_t)p.K * (AM == A_IM2COL_T ? p.convC : p.lda) * 2);
    const i32x4_t rb = uniform_rsrc_words(B, (int64_t)p.K * p.ldb * 2);

    // ---- per-lane DMA geometry: instruction idx = i*8 + wave (i = 0, 1) of a
    // unit covers block idx >> 3, k-rows (idx & 7)*8 + lane/8, slot lane & 7
    const int krow_l = (wave & 7) * 8 + (lane >> 3);       // k-row within the K-tile (same for i = 0, 1)
    const int chunk = (lane & 7) ^ (krow_l & 7);           // global 16-B chunk of the row this lane fetches
    // A: unit 0 blocks {0, 2}, unit 3 blocks {1, 3} -> column offsets (i = 0, 1)
    const int acol[4] = {0, 128, 64, 192};                 // [U0 i0, U0 i1, U3 i0, U3 i1]
    // B: block [wnA q | wnB q]: chunk c < 4 from wave 2*pair, else 2*pair + 1
    auto bcol = [&](int q, int pair) { return (2 * pair + (chunk >> 2)) * 64 + q * 32 + (chunk & 3) * 8; };
    const int bcols[4] = {bcol(0, 0), bcol(0, 1), bcol(1, 0), bcol(1, 1)};   // [U1 i0, U1 i1, U2 i0, U2 i1]
    const unsigned a_lane = (unsigned)(((int64_t)krow_l * p.lda + m0 + 8 * chunk) * 2);
    const unsigned b_lane = (unsigned)(((int64_t)krow_l * p.ldb + n0) * 2);
    // IM2COL_T: the tap (dh, dw) and first channel of each A sub-block (uniform per item),
    // and this lane's pixel (row h, column w) of the K-tile being issued
    int t_dh[4] = {0, 0, 0, 0}, t_dw[4] = {0, 0, 0, 0}, t_c0[4] = {0, 0, 0, 0};
    if constexpr (AM == A_IM2COL_T) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int col = min(m0 + acol[s], p.M - 1);
            const int tap = col / p.convC;
            t_dh[s] = tap / 3 - 1;
            t_dw[s] = tap % 3 - 1;
            t_c0[s] = col - tap * p.convC;
        }
    }

    auto issue = [&](auto U_, int kt, char* buf) {
        constexpr int U = decltype(U_)::value;
        const int k = kbeg + kt * BK + krow_l;
        const bool kok = k < kend;
        const unsigned kst = (unsigned)((int64_t)(kt * BK + kbeg) * (U == 0 || U == 3 ? p.lda : p.ldb) * 2);
        if constexpr ((U == 0 || U == 3) && AM == A_IM2COL_T) {
            const int pix_w = k % p.convW, pix_h = (k / p.convW) % p.convH;   // this lane's pixel
#pragma unroll
            for (int i = 0; i < NUA; ++i) {
                const int s = (U == 0 ? 0 : 2) + i;
                const int hh = pix_h + t_dh[s], ww = pix_w + t_dw[s];
                const bool ok = kok && m0 + acol[s] + 8 * chunk < p.M && hh >= 0 && hh < p.convH && ww >= 0 &&
                                ww < p.convW;
                const int64_t off = ((int64_t)(k + t_dh[s] * p.convW + t_dw[s]) * p.convC + t_c0[s] + 8 * chunk) * 2;
                tt_dma16(ra, buf + (acol[s] / 64) * BLK + (wave & 7) * 1024, ok ? (unsigned)off : TT_OOB);
            }
        } else if constexpr (U == 0 || U == 3) {
#pragma unroll
            for (int i = 0; i < NUA; ++i) {
                const int s = (U == 0 ? 0 : 2) + i;
                const bool ok = kok && m0 + acol[s] + 8 * chunk < p.M;
                tt_dma16(ra, buf + (acol[s] / 64) * BLK + (wave & 7) * 1024, ok ? a_lane + kst + acol[s] * 2 : TT_OOB);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NUB; ++i) {
                const int s = (U == 1 ? 0 : 2) + i;
                const int blk = (U == 1 ? 0 : 2) + i;          // B block index 0..3
                const bool ok = kok && n0 + bcols[s] < p.N;
                tt_dma16(rb, buf + A_BYTES + blk * BLK + (wave & 7) * 1024,
                         ok ? b_lane + kst + (unsigned)(bcols[s] * 2) : TT_OOB);
            }
        }
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;

    // Staging schedule: every unit is issued as soon as the reads of its slot
    // (two K-tiles back, same buffer) allow, so it has 4-5 phases to land
    // before the wait that retires it (a K-tile ahead left it 2, and the waits
    // stalled on DMA latency). Per K-tile k, in issue order:
    //   phase 0: U3(k+1)    phase 2: U1(k+2)    phase 3: U0(k+2), U2(k+2)
    // (U1 and U0 / U2 of K-tile k are read in phases 0 / 0 / 1, U3 in phase 2;
    // a slot is rewritten >= 2 phases after its last read). B q0 stays in
    // registers from phase 0 to phase 3, so phase 3 reads nothing. Waits, each
    // before a phase's first barrier for the next phase's reads, count the DMAs
    // issued after the retired one: phase 0 (U2(k)) 10, phase 1 (U3(k)) 8,
    // phase 3 (U0, U1 of k+1) 10 instructions; the last two K-tiles drain to 0.
    issue(I0{}, 0, smem);
    issue(I1{}, 0, smem);
    issue(I2{}, 0, smem);
    issue(I3{}, 0, smem);
    if (nk > 1) {
        issue(I1{}, 1, smem + BUF);
        issue(I0{}, 1, smem + BUF);
        issue(I2{}, 1, smem + BUF);
        vm_wait<NUB + NUA + NUB>();                       // K-tile 0 landed
    } else {
        vm_wait<0>();
    }
    tt_barrier();
    if (wm == 1) tt_barrier();                            // stagger: waves 4-7 one barrier behind

    // transposed fragment reads (frag_tr): lane reads k-row kr0 (+16) of the
    // 32-deep kk block, 4 consecutive columns at cq within a 16-column group
    const int kr0 = 4 * g + (i16 >> 2), cq = 4 * (i16 & 3);
    bf16x8 afr[4][2], bq0[2][2], bq1[2][2];
    auto tr_addr = [&](int blk_off, int col, int kk) {   // byte offset of (k-row kk*32 + kr0, col) in a block
        const int r = kk * 32 + kr0;
        return blk_off + r * ROWB + ((((col >> 3) ^ (r & 7))) << 4) + (col & 7) * 2;
    };
    auto read_a = [&](const char* cur, int qa) {
        const int blk = (2 * wm + qa) * BLK;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                afr[i][kk] = frag_tr(reinterpret_cast<const unsigned short*>(cur + tr_addr(blk, i * 16 + cq, kk)),
                                     16 * (ROWB / 2));
    };
    auto read_b = [&](const char* cur, int qb, bf16x8 (&bfr)[2][2]) {
        const int blk = A_BYTES + (2 * qb + (wn >> 1)) * BLK;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                bfr[j][kk] = frag_tr(reinterpret_cast<const unsigned short*>(
                                         cur + tr_addr(blk, (wn & 1) * 32 + j * 16 + cq, kk)),
                                     16 * (ROWB / 2));
    };
    auto mfma_q = [&](auto QA_, auto QB_, const bf16x8 (&bfr)[2][2]) {
        constexpr int QA = decltype(QA_)::value, QB = decltype(QB_)::value;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[QA * 4 + i][QB * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        bfr[j][kk], afr[i][kk], acc[QA * 4 + i][QB * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    for (int kt = 0; kt < nk; ++kt) {
        char* cur = smem + (kt & 1) * BUF;
        char* nxt = smem + ((kt + 1) & 1) * BUF;
        const bool full = kt + 2 < nk;
        // phase 0: A q0, B q0; U3 of the next K-tile
        read_a(cur, 0);
        read_b(cur, 0, bq0);
        if (kt + 1 < nk) issue(I3{}, kt + 1, nxt);
        if (full) vm_wait<NUA + NUB + NUA + NUB + NUA>(); else vm_wait<0>();
        tt_barrier();
        mfma_q(I0{}, I0{}, bq0);
        tt_barrier();
        // phase 1: B q1
        read_b(cur, 1, bq1);
        if (full) vm_wait<NUB + NUA + NUB + NUA>(); else vm_wait<0>();
        tt_barrier();
        mfma_q(I0{}, I1{}, bq1);
        tt_barrier();
        // phase 2: A q1; U1 of K-tile kt+2 into this buffer (no wait: phase 3 reads nothing)
        read_a(cur, 1);
        if (full) issue(I1{}, kt + 2, cur);
        tt_barrier();
        mfma_q(I1{}, I1{}, bq1);
        tt_barrier();
        // phase 3: U0, U2 of K-tile kt+2
        if (full) {
            issue(I0{}, kt + 2, cur);
            issue(I2{}, kt + 2, cur);
            vm_wait<NUB + NUA + NUB + NUA + NUB>();
        } else {
            vm_wait<0>();
        }
        tt_barrier();
        mfma_q(I1{}, I0{}, bq0);
        tt_barrier();
    }
    if (wm == 0) tt_barrier();                            // balance the stagger

    // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + wm*128 + i*16 + i16,
    // n = n0 + wn*64 + j*16 + 4g; f32 (+)= or split-K partials
    const int mrow0 = m0 + wm * 128 + i16, ncol0 = n0 + wn * 64 + 4 * g;
    float* C;
    int64_t ldc;
    bool acc_c;
    if (p.splits > 1) {
        C = p.splitk_ws + ((int64_t)zb * p.splits + zs) * (int64_t)p.M * p.N;
        ldc = p.N;
        acc_c = false;
    } else {
        C = reinterpret_cast<float*>(p.C) + zb * p.strideC;
        ldc = p.ldc;
        acc_c = p.accumulate != 0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = mrow0 + i * 16;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = ncol0 + j * 16;
            if (n >= p.N) continue;
            floatx4* dst = reinterpret_cast<floatx4*>(C + (int64_t)m * ldc + n);
            floatx4 v = acc[i][j] * p.alpha;
            if (acc_c) v += *dst;
            *dst = v;
        }
    }
}

}  // namespace

bool gemm_pptn_enabled() {
    return opt(OPT_GEMM_PPTN) != 0;            // 0: the 4-wave TN engine
}

// Runs the ping-pong TN engine when it covers the call; -1 otherwise.
bool gemm_pptn_covers(int amode, int M, int N, int convC) {
#ifdef OCRK_EXPERIMENTS
    static const int nmin = [] { const char* e = getenv("OCRK_PPTN_NMIN"); return e ? atoi(e) : 256; }();
#else
    constexpr int nmin = 256;
#endif
    if (!gemm_pptn_enabled() || M < 256 || N < nmin || M % 8 != 0 || N % 8 != 0) return false;
    if (amode == A_COLK) return true;
    return amode == A_IM2COL_T && convC % 64 == 0;        // a 64-column A block = one tap's channels
}

// Runs the ping-pong TN engine when it covers the call; -1 otherwise.
int gemm_pptn(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    if (dtype != OCRK_BF16 || bmode != B_KN || !gemm_pptn_covers(amode, p.M, p.N, p.convC)) return -1;
    if (p.c_bf16 || p.bias || p.relu || p.mask || p.stats) return -1;
    if (p.ldb % 8 != 0 || (amode == A_COLK && p.lda % 8 != 0)) return -1;
    if (p.splits == 1 && (p.ldc % 4 != 0 || (uintptr_t)p.C % 16 != 0 || p.strideC % 4 != 0)) return -1;
    if (p.splits > 1 && (uintptr_t)p.splitk_ws % 16 != 0) return -1;
    const int64_t a_bytes = (int64_t)p.K * (amode == A_COLK ? p.lda : p.convC) * 2;
    if (a_bytes >= (1ll << 31) || (int64_t)p.K * p.ldb * 2 >= (1ll << 31)) return -1;
    if (amode == A_IM2COL_T && p.batch != 1) return -1;
    constexpr int LDS = 2 * 8 * 64 * 128;
    const void* kern = amode == A_COLK ? reinterpret_cast<const void*>(&gemm_pptn_kernel<A_COLK>)
                                       : reinterpret_cast<const void*>(&gemm_pptn_kernel<A_IM2COL_T>);
    static DeviceOnce configured[2];
    set_dyn_lds(configured[amode == A_COLK ? 0 : 1], kern, LDS);
    const int64_t items = cdiv(p.M, 256) * cdiv(p.N, 256) * (int64_t)p.batch * p.splits;
    const dim3 grid((unsigned)(cdiv(items, 8) * 8));
    if (amode == A_COLK) gemm_pptn_kernel<A_COLK><<<grid, 512, LDS, stream>>>(p);
    else gemm_pptn_kernel<A_IM2COL_T><<<grid, 512, LDS, stream>>>(p);
    return launch_status("gemm_pptn");
}

}  // namespace ocrk
