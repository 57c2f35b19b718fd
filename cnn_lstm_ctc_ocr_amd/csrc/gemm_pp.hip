// 8-wave ping-pong MFMA engine for the k-contiguous ("NT") operand modes, bf16:
//   A: A_ROWK (activations [M][lda]) or A_IM2COL / A_IM2COL_FLIP (3x3 conv,
//      NHWC source, 8-channel chunks never cross a tap because C % 8 == 0)
//   B: B_NK (weights [N][ldb])
// It carries the large GEMMs of the step: the recurrent input projections
// gx = x . W_x^T + b (model_bu.py:186-192), their data gradients
// dx = dG . W_x, the logits data gradient (model.py:216-220) and the wide
// convolutions (forward and backward-data, model.py:84-109) with their fused
// epilogues (bias, ReLU, producer ReLU mask, BN column statistics).
//
// Geometry: a 256 x BN x 64 tile (BN = 256 or 128) per 512-thread workgroup,
// 8 waves as 2 (rows) x 4 (columns); wave (wm, wn) owns rows wm*128 .. +128
// and BN/4 columns. Each K-tile ("step") is consumed in four phases, one
// output quadrant (64 rows x BN/8 columns) each:
//     phase 0: A rows q0, B cols q0      phase 2: A rows q1, B cols q1
//     phase 1: A rows q0, B cols q1      phase 3: A rows q1, B cols q0
// and staged in four DMA units whose order matches that consumption:
//     U0 = A rows q0 (of both row halves), U1 = B cols q0, U2 = B cols q1,
//     U3 = A rows q1,
// unit u of step s+1 being issued (LDS-DMA, buffer_load ... lds) in phase u
// of step s into the other of two LDS buffers.
//
// Persistent: one workgroup per CU walks its work items (output tile x K
// slice) as ONE stream of steps, so the first K-tile of the next item is
// prefetched during the last K-tile of the current one; between the two the
// epilogue runs through the LDS buffer the last step just freed.
//
// Every phase is {fragment reads (ds_read_b128) + the phase's DMA issue +
// a counted vmcnt} -> s_barrier -> {16 or 8 MFMAs} -> s_barrier. Waves 4-7
// (the second row half; one per SIMD beside waves 0-3) run one barrier behind
// waves 0-3, so on every SIMD one wave's MFMAs overlap its partner's reads and
// DMA issue (cdna_hip_programming.md, "The 256^2 8-phase template").
// Ordering, in barriers (G0 = waves 0-3 pass phase n's barriers 2n and 2n+1,
// G1 = waves 4-7 pass 2n+1 and 2n+2):
//  * RAW: each wave waits (vmcnt) in phase n for its DMAs of phase n-2 and
//    earlier, before its first barrier of phase n, so a unit issued in phase
//    m has landed for every wave by barrier 2m+5; G0 reads phase n's
//    fragments after barrier 2n-1, G1 after 2n, so a unit is read no earlier
//    than phase m+3 -- units 0..3 of step s+1 (phases 4s..4s+3) are first read
//    in phases 4s+4, 4s+4, 4s+5, 4s+6.
//  * WAR: the reads of phase n are complete (lgkmcnt) in the waves' MFMA
//    segments, i.e. by barrier 2n+2; a DMA into the same bytes is issued
//    after barrier 2m-1 (G0) / 2m (G1), so m >= n+2 is required: unit u's
//    bytes of step s-1 were last read in phases 4s-4, 4s-1, 4s-3, 4s-2 and
//    are rewritten in phases 4s, 4s+1, 4s+2, 4s+3.
//  * Item boundary: G0 passes one extra barrier (the groups meet), every wave
//    stages its output in the freed buffer and stores it, all meet again
//    (the staging is complete before the next DMA into that buffer), and G1
//    re-enters one barrier behind. The epilogue's PP_EPI_STORES buffer stores
//    are the youngest VMEM ops at the next item's first two waits, whose
//    counts include them, so those waits do not drain the stores.
//
// LDS images are lane-linear (one DMA instruction = 8 rows x 128 B); the 16-B
// chunk index of each row is XOR-swizzled by (row & 7) on the GLOBAL side, so
// each 16-lane group of a ds_read_b128 fragment read hits 16 distinct bank
// groups (conflict-free).
// The MFMA operands are passed as (B fragment, A fragment): each lane then
// holds 4 consecutive OUTPUT COLUMNS of one output row (C^T fragment layout),
// so the bias and the ReLU mask are read as vectors and the bf16 staging
// image is written with 8-B LDS stores.
// Zero fill (im2col padding taps, rows >= M / N, k >= K): the lane's buffer
// offset is pushed past the resource's num_records, which returns 0 (and
// drops a store).
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr unsigned PP_OOB = 0x80000000u;

__device__ __forceinline__ void pp_dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ void pp_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N> __device__ __forceinline__ void vm_wait_nop() {}

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

// work item w -> (output tile, z = batch * splits + slice); tiles in groups
// of 4 row-tiles x all column-tiles (row-tile fastest) so the items an XCD
// runs at once share A rows and B columns in its L2
struct PPItem { int m0, n0, zb, zs; };
__device__ __forceinline__ PPItem pp_item(int w, int tm, int tn, int splits, int BM, int BN) {
    const int nT = tm * tn;
    const int z = w / nT, t = w - z * nT;
    constexpr int GM = 4;
    const int gsz = GM * tn, grp = t / gsz, first = grp * GM;
    const int gm = min(GM, tm - first), r = t - grp * gsz;
    PPItem it;
    it.m0 = (first + r % gm) * BM;
    it.n0 = (r / gm) * BN;
    it.zb = z / splits;
    it.zs = z - it.zb * splits;
    return it;
}

template <int AM, int BN, bool STATS, bool MASK>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const GemmParams p) {
    constexpr int BM = 256, BK = 64, ROWB = 128;          // 64 bf16 = 128 B per LDS row
    constexpr int WCOLS = BN / 4;                         // columns per wave (64 / 32)
    constexpr int QN = WCOLS / 32;                        // 16-column fragments per quadrant (2 / 1)
    constexpr int A_BYTES = BM * ROWB, BUF = (BM + BN) * ROWB;
    constexpr int NUA = 2;                                // DMA instructions per wave, A unit (128 rows)
    constexpr int NUB = BN / 128;                         // ... B unit (BN/2 rows)
    constexpr int HBLK = WCOLS / 16;                      // 8-row blocks per wave column-half
    constexpr int NU0 = NUA, NU1 = NUB, NU2 = NUB, NU3 = NUA;
    // epilogue staging: per wave CR rows x PITCH bytes inside the freed buffer
    constexpr int PITCH = WCOLS * 2 + 16, CPRW = WCOLS / 8;
    constexpr int CR = BN == 256 ? 32 : 64;
    constexpr int NST = 128 * CPRW / 64;                  // 16-B stores per lane per item (bf16 C)
    static_assert(BN == 256 || BN == 128, "BN");
    static_assert(8 * CR * PITCH <= BUF, "staging fits the freed buffer");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const bf16* mask = reinterpret_cast<const bf16*>(p.mask);

    // the wave index is made provably uniform: it feeds the LDS-DMA
    // destinations (M0), which would otherwise be wrapped in waterfall loops
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int i16 = lane & 15, g = lane >> 4, sw = lane & 7;

    // ---- this workgroup's items: XCD x (= blockIdx % 8 under round-robin
    // dispatch) owns the contiguous item range [x*per, (x+1)*per)
    const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
    const int nitems = tm * tn * p.batch * p.splits;
    const int per = (nitems + 7) >> 3;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, sp = gridDim.x >> 3;
    const int wend = min(nitems, (xcd + 1) * per);
    int w_issue = xcd * per + slot;                       // item being prefetched
    if (w_issue >= wend) return;

    const int lrow = lane >> 3;
    const int cs = (lane & 7) ^ lrow;                     // global 16-B chunk this lane fetches
    int arow[4];                                          // [U0 i0, U0 i1, U3 i0, U3 i1] tile rows
    arow[0] = wave * 8;
    arow[1] = 128 + wave * 8;
    arow[2] = 64 + wave * 8;
    arow[3] = 192 + wave * 8;
    int bcol[2 * NUB];                                    // [U1 i.., U2 i..] tile columns
#pragma unroll
    for (int i = 0; i < NUB; ++i) {
        const int b = i * 8 + wave;
        bcol[i] = (b / HBLK) * WCOLS + (b % HBLK) * 8;
        bcol[NUB + i] = bcol[i] + WCOLS / 2;
    }

    // ---- issue side: the item whose K-tiles are being prefetched. Per-lane
    // state is one byte offset per operand (row lrow of an 8-row block) plus,
    // for im2col, the (h, w) of the lane's pixel in each A block; the block
    // parts are uniform (SGPRs).
    __amdgpu_buffer_rsrc_t ra, rb;
    unsigned ahw[4];
    int i_m0 = 0, i_n0 = 0, i_kbeg = 0, i_kend = 0, i_nk = 0, i_kt = 0;
    const int64_t a_ld = AM == A_ROWK ? p.lda : p.convC;  // elements per A row (pixel)
    const unsigned a_lane = (unsigned)(lrow * a_ld * 2), b_lane = (unsigned)(lrow * p.ldb * 2);
    auto setup_issue = [&](int w) {
        const PPItem it = pp_item(w, tm, tn, p.splits, BM, BN);
        const bf16* A = reinterpret_cast<const bf16*>(p.A) + it.zb * p.strideA;
        const bf16* B = reinterpret_cast<const bf16*>(p.B) + it.zb * p.strideB;
        ra = uniform_rsrc(A, (int64_t)p.M * a_ld * 2);
        rb = uniform_rsrc(B, (int64_t)p.N * p.ldb * 2);
        i_m0 = it.m0;
        i_n0 = it.n0;
        i_kbeg = it.zs * p.k_chunk;
        i_kend = min(p.K, i_kbeg + p.k_chunk);
        i_nk = max(1, (i_kend - i_kbeg + BK - 1) / BK);   // >= 1 step per item (K = 0: zero tile)
        i_kt = 0;
        if constexpr (AM != A_ROWK) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = it.m0 + arow[i] + lrow;
                const int mm = m < p.M ? m : 0;
                const int wq = mm % p.convW, h = (mm / p.convW) % p.convH;
                ahw[i] = ((unsigned)h << 16) | (unsigned)wq;
            }
        }
    };

    // issue DMA unit U of the issue side's current K-tile into `buf`
    auto issue = [&](auto U_, char* buf) {
        constexpr int U = decltype(U_)::value;
        const int k = i_kbeg + i_kt * BK + 8 * cs;
        const bool kok = k < i_kend;
        if constexpr (U == 0 || U == 3) {
            int tap_off = 0, dh = 0, dw = 0;
            if constexpr (AM != A_ROWK) {
                const int C = p.convC;
                const int tap = kok ? k / C : 0;
                const int cch = k - tap * C;
                const int kh = tap / 3, kw = tap - kh * 3;
                if constexpr (AM == A_IM2COL_FLIP) { dh = 1 - kh; dw = 1 - kw; }
                else { dh = kh - 1; dw = kw - 1; }
                tap_off = ((dh * p.convW + dw) * C + cch) * 2;
            }
#pragma unroll
            for (int i = 0; i < NUA; ++i) {
                const int s = (U == 0 ? 0 : 2) + i;
                const int mrow = i_m0 + arow[s];            // uniform first row of the block
                bool ok = kok && lrow < p.M - mrow;
                unsigned voff = a_lane + (unsigned)(mrow * a_ld * 2);
                if constexpr (AM == A_ROWK) {
                    voff += (unsigned)(k * 2);
                } else {
                    const int hh = (int)(ahw[s] >> 16) + dh, ww = (int)(ahw[s] & 0xffff) + dw;
                    ok = ok && hh >= 0 && hh < p.convH && ww >= 0 && ww < p.convW;
                    voff += (unsigned)tap_off;
                }
                pp_dma16(ra, buf + arow[s] * ROWB, ok ? voff : PP_OOB);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NUB; ++i) {
                const int s = (U == 1 ? 0 : NUB) + i;
                const int ncol = i_n0 + bcol[s];
                const bool ok = kok && lrow < p.N - ncol;
                const unsigned voff = b_lane + (unsigned)(ncol * p.ldb * 2) + (unsigned)(k * 2);
                pp_dma16(rb, buf + A_BYTES + bcol[s] * ROWB, ok ? voff : PP_OOB);
            }
        }
    };
    // after the 4 units of a K-tile: the next K-tile, or the next item's first
    auto advance_issue = [&]() -> bool {
        if (++i_kt < i_nk) return true;
        w_issue += sp;
        if (w_issue >= wend) return false;
        setup_issue(w_issue);
        return true;
    };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;

    // ---- compute side
    int w_comp = w_issue;
    PPItem cur_it = pp_item(w_comp, tm, tn, p.splits, BM, BN);
    int c_nk, c_kt = 0;

    // prologue: the first item's K-tile 0 into buffer 0
    setup_issue(w_issue);
    c_nk = i_nk;
    issue(I0{}, smem);
    issue(I1{}, smem);
    issue(I2{}, smem);
    issue(I3{}, smem);
    bool more = advance_issue();
    vm_wait<0>();
    pp_barrier();
    if (wm == 1) pp_barrier();                            // stagger: waves 4-7 one barrier behind

    floatx4 acc[8][2 * QN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2 * QN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    bf16x8 afr[4][2], bfr[QN][2];
    // ds_read_b128 base addresses: (chunk kk*4 + g) ^ sw = (g ^ sw) ^ 4kk
    const int a_base = (wm * 128 + i16) * ROWB, b_base = A_BYTES + (wn * WCOLS + i16) * ROWB;
    auto read_a = [&](const char* cur, int qa) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                afr[i][kk] = *reinterpret_cast<const bf16x8*>(
                    cur + a_base + (qa * 64 + i * 16) * ROWB + (((kk * 4 + g) ^ sw) << 4));
    };
    auto read_b = [&](const char* cur, int qb) {
#pragma unroll
        for (int j = 0; j < QN; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                bfr[j][kk] = *reinterpret_cast<const bf16x8*>(
                    cur + b_base + (qb * (WCOLS / 2) + j * 16) * ROWB + (((kk * 4 + g) ^ sw) << 4));
    };
    auto mfma_q = [&](auto QA_, auto QB_) {
        constexpr int QA = decltype(QA_)::value, QB = decltype(QB_)::value;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < QN; ++j)
                    acc[QA * 4 + i][QB * QN + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        bfr[j][kk], afr[i][kk], acc[QA * 4 + i][QB * QN + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

#ifdef PP_NOWAIT
#define vm_wait vm_wait_nop
#endif
    int s = 0;                                            // step counter (buffer = s & 1)
    bool prev_issued = false;                             // phase 3 of the previous step issued a unit
    bool after_epi = false;                               // the epilogue's stores sit between the units
    for (;;) {
        const char* cur = smem + (s & 1) * BUF;
        char* nxt = smem + ((s + 1) & 1) * BUF;
        // ---- phase 0: A q0 + B q0; retire phase n-2 (unit 2 of this step)
        read_a(cur, 0);
        read_b(cur, 0);
        if (more) issue(I0{}, nxt);
        if (after_epi) {
            // [U2 U3 | stores | U0']: keep U3, the stores and U0' in flight
            if (more) vm_wait<NU3 + NST + NU0>(); else vm_wait<NU3 + NST>();
        } else if (more) {
            if (prev_issued) vm_wait<NU0 + NU3>(); else vm_wait<NU0>();
        } else {
            if (prev_issued) vm_wait<NU3>(); else vm_wait<0>();
        }
        pp_barrier();
        mfma_q(I0{}, I0{});
        pp_barrier();
        // ---- phase 1: B q1; retire unit 3 of this step
        read_b(cur, 1);
        if (more) issue(I1{}, nxt);
        if (after_epi) {
            if (more) vm_wait<NST + NU0 + NU1>(); else vm_wait<NST>();
        } else {
            if (more) vm_wait<NU1 + NU0>(); else vm_wait<0>();
        }
        pp_barrier();
        mfma_q(I0{}, I1{});
        pp_barrier();
        // ---- phase 2: A q1 (B q1 kept); retire unit 0 of the next step
        read_a(cur, 1);
        if (more) { issue(I2{}, nxt); vm_wait<NU2 + NU1>(); }
        else vm_wait<0>();
        pp_barrier();
        mfma_q(I1{}, I1{});
        pp_barrier();
        // ---- phase 3: B q0 (A q1 kept); retire unit 1 of the next step
        read_b(cur, 0);
        if (more) { issue(I3{}, nxt); vm_wait<NU3 + NU2>(); }
        else vm_wait<0>();
        pp_barrier();
        mfma_q(I1{}, I0{});
        pp_barrier();
        prev_issued = more;
        after_epi = false;
        if (more) more = advance_issue();
        ++s;
        if (++c_kt < c_nk) continue;

#ifdef PP_NOWAIT
#undef vm_wait
#endif
        // ================================================= item epilogue
        if (wm == 0) pp_barrier();                        // groups meet: every read of `cur` is done
        const int mrow0 = cur_it.m0 + wm * 128 + i16;
        const int ncol0 = cur_it.n0 + wn * WCOLS + 4 * g;
        char* stg = const_cast<char*>(cur) + wave * (CR * PITCH);
        {
            // bias (buffer load: 0 past N or without bias), producer ReLU mask,
            // ReLU -- in place in the accumulators
            const __amdgpu_buffer_rsrc_t rbias =
                uniform_rsrc(p.bias ? p.bias + cur_it.zb * p.strideBias : p.bias, p.bias ? (int64_t)p.N * 4 : 0);
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) {
                const int n = ncol0 + j * 16;
                const floatx4 bv = __builtin_bit_cast(
                    floatx4, __builtin_amdgcn_raw_buffer_load_b128(rbias, n < p.N ? (unsigned)(n * 4) : PP_OOB, 0, 0));
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    floatx4 v = acc[i][j] * p.alpha + bv;
                    if constexpr (MASK) {
                        const int m = mrow0 + i * 16;
                        if (m < p.M && n < p.N) {
                            // the 4 mask values as two 32-bit words, each bf16 widened by a shift
                            // (comparing the u16x4 elements as bf16 kept only element 0's verdict
                            // for all four: tools/pp_mask_probe.py)
                            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                            const u32x2 mw = *reinterpret_cast<const u32x2*>(mask + (int64_t)m * p.ldmask + n);
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const unsigned bits = (r & 1) ? (mw[r >> 1] & 0xffff0000u) : (mw[r >> 1] << 16);
                                if (!(__uint_as_float(bits) > 0.f)) v[r] = 0.f;
                            }
                        }
                    }
                    if (p.relu) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
                    }
                    acc[i][j] = v;
                }
            }
            if constexpr (STATS) {
                // per-column (sum, M2) over this wave's 128 rows = one
                // 128-row stats tile (gemm.h): shifted sums about the
                // column's first row, reduced over the 16 lanes that share
                // the columns, M2 = q - s^2 / n
                const int mbase = cur_it.m0 + wm * 128;
                if (mbase < p.M) {
                    const int valid = min(128, p.M - mbase);
                    float* st = p.stats + (int64_t)(mbase / 128) * 2 * p.N;
#pragma unroll
                    for (int j = 0; j < 2 * QN; ++j) {
                        const int n = ncol0 + j * 16;
                        floatx4 sh;
#pragma unroll
                        for (int r = 0; r < 4; ++r) sh[r] = __shfl(acc[0][j][r], lane & 48, 64);
                        floatx4 s1 = floatx4{0.f, 0.f, 0.f, 0.f}, q = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            if (mrow0 + i * 16 < p.M) {
                                const floatx4 d = acc[i][j] - sh;
                                s1 += d;
                                q += d * d;
                            }
                        }
#pragma unroll
                        for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                s1[r] += __shfl_xor(s1[r], o, 64);
                                q[r] += __shfl_xor(q[r], o, 64);
                            }
                        }
                        if (i16 == 0 && n < p.N) {
                            const float cnt = (float)valid;
                            floatx4 sum, m2;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                sum[r] = cnt * sh[r] + s1[r];
                                m2[r] = fmaxf(q[r] - s1[r] * s1[r] / cnt, 0.f);
                            }
                            *reinterpret_cast<floatx4*>(st + n) = sum;
                            *reinterpret_cast<floatx4*>(st + p.N + n) = m2;
                        }
                    }
                }
            }
            // bf16 C through a per-wave LDS image (CR rows x BN/4 columns,
            // pitch +16 B) in the freed buffer: each store instruction then
            // writes whole rows at 16 B per lane, not 16 rows x 8 B pieces
            // (partial lines, measured ~1.6 TB/s chip-wide)
            bf16* Cb = reinterpret_cast<bf16*>(p.C) + cur_it.zb * p.strideC;
            const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(Cb, ((int64_t)(p.M - 1) * p.ldc + p.N) * 2);
            const int c8 = lane % CPRW, r0 = lane / CPRW;
            const int n = cur_it.n0 + wn * WCOLS + 8 * c8;
#pragma unroll
            for (int h = 0; h < 128 / CR; ++h) {
#pragma unroll
                for (int i = 0; i < CR / 16; ++i)
#pragma unroll
                    for (int j = 0; j < 2 * QN; ++j) {
                        u16x4 o;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            o[r] = __builtin_bit_cast(unsigned short, (bf16)acc[h * (CR / 16) + i][j][r]);
                        *reinterpret_cast<u16x4*>(stg + (i * 16 + i16) * PITCH + (j * 16 + 4 * g) * 2) = o;
                    }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int q = 0; q < CR * CPRW / 64; ++q) {
                    const int r = r0 + q * (64 / CPRW);
                    const int m = cur_it.m0 + wm * 128 + h * CR + r;
                    const u32x4 v = *reinterpret_cast<const u32x4*>(stg + r * PITCH + c8 * 16);
                    const unsigned off = (m < p.M && n < p.N) ? (unsigned)(((int64_t)m * p.ldc + n) * 2) : PP_OOB;
                    __builtin_amdgcn_raw_buffer_store_b128(v, rc, off, 0, 0);
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();                                     // staging done before the next DMA into `cur`
        w_comp += sp;
        if (w_comp >= wend) break;
        cur_it = pp_item(w_comp, tm, tn, p.splits, BM, BN);
        c_nk = max(1, (min(p.K, cur_it.zs * p.k_chunk + p.k_chunk) - cur_it.zs * p.k_chunk + BK - 1) / BK);
        c_kt = 0;
        after_epi = true;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (wm == 1) pp_barrier();                        // re-stagger
    }
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime count (the in-flight VMEM ops a
// schedule allows): a scalar jump table over the immediate forms; n > 63 waits
// for vmcnt(63), which is stricter and so still correct.
__device__ __forceinline__ void vm_wait_n(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    n = n > 63 ? 63 : n;
    switch (n) {
#define VW1(i) case i: vm_wait<i>(); break;
#define VW8(b) VW1(b) VW1(b + 1) VW1(b + 2) VW1(b + 3) VW1(b + 4) VW1(b + 5) VW1(b + 6) VW1(b + 7)
        VW8(0) VW8(8) VW8(16) VW8(24) VW8(32) VW8(40) VW8(48) VW8(56)
#undef VW8
#undef VW1
    default: vm_wait<0>();
    }
}

// vm_wait_n with the schedule's steady-state count as a one-compare fast path
template <int FAST>
__device__ __forceinline__ void vm_wait_fast(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    if (n == FAST) vm_wait<FAST>();
    else vm_wait_n(n);
}

// ---------------------------------------------------------------------------
// Deep-lead form of the ping-pong engine (A_ROWK, bf16 C, bias / ReLU
// epilogue): the same 256 x BN x 64 tile, 8 waves, 4 phases per K-tile and
// the same two 64-KB LDS buffers, but each DMA unit is issued as soon as the
// slot it overwrites is free, not a whole K-tile ahead into the other buffer,
// so a unit lands 5-6 phases (1.25-1.5 K-tiles) after its issue instead of 3.
// What frees the slots early: the B q0 fragments are kept in registers from
// phase 0 to phase 3 (phase 3 reads no LDS), so in step s (buffer s & 1):
//     last reads  U0, U1: phase 0   U2: phase 1   U3: phase 2
// and a slot may be re-filled two phases after its last read (the stagger:
// G1 reads one barrier behind G0). The unit stream, one unit per phase:
//     phase 0: U2(s+1)   phase 1: U3(s+1)   phase 2: U0(s+2)   phase 3: U1(s+2)
// into the buffer of the step it belongs to. Waits (counted from a uniform
// tally of the VMEM ops this wave issued, so item boundaries, epilogue stores
// and the end of the stream need no special cases), each two phases before
// the read they protect:
//     phase 0: U3(s)        phase 2: U0 + U1(s+1)        phase 3: U2(s+1)
// Item epilogue (persistent workgroups, items prefetched across): when item i
// ends in step s, U3(s+1) and U0, U1(s+2) are in flight, but the U2 and U3
// slots of step s's buffer are free until phase 0 of step s+1, so each wave
// stages its C rows there, 16 rows at a time (per-wave areas of 2.3 / 1.3 KB:
// waves 0-3 in the four U2 pieces, waves 4-7 in the two U3 row blocks), and
// the next item's first step starts only after a barrier behind those reads.
// The bias (projections only) is loaded at the top of the epilogue, which
// drains the three units then in flight (in-order vmcnt) -- at most ~1 us per
// item; holding it in registers through the last step instead costs 16 VGPRs
// the schedule does not have (256 with spills).
template <int BN>
__global__ void __launch_bounds__(512) gemm_pp_deep_kernel(const GemmParams p) {
    constexpr int BM = 256, BK = 64, ROWB = 128;
    constexpr int WCOLS = BN / 4;
    constexpr int QN = WCOLS / 32;
    constexpr int A_BYTES = BM * ROWB, BUF = (BM + BN) * ROWB;
    constexpr int NUA = 2, NUB = BN / 128;
    constexpr int HBLK = WCOLS / 16;
    constexpr int PITCH = WCOLS * 2 + 16, CPRW = WCOLS / 8;
    constexpr int CR = 16;                                // staged rows per round
    constexpr int NST = 128 * CPRW / 64;                  // 16-B C stores per lane per item
    static_assert(BN == 256 || BN == 128, "BN");
    static_assert(CR * PITCH <= (BN == 256 ? 4096 : 2048), "a wave's staging fits its slot piece");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int i16 = lane & 15, g = lane >> 4, sw = lane & 7;

    const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
    const int nitems = tm * tn * p.batch * p.splits;
    const int per = (nitems + 7) >> 3;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, sp = gridDim.x >> 3;
    const int wend = min(nitems, (xcd + 1) * per);
    int w_issue = xcd * per + slot;
    if (w_issue >= wend) return;

    const int lrow = lane >> 3;
    const int cs = (lane & 7) ^ lrow;
    int arow[4];
    arow[0] = wave * 8;
    arow[1] = 128 + wave * 8;
    arow[2] = 64 + wave * 8;
    arow[3] = 192 + wave * 8;
    int bcol[2 * NUB];
#pragma unroll
    for (int i = 0; i < NUB; ++i) {
        const int b = i * 8 + wave;
        bcol[i] = (b / HBLK) * WCOLS + (b % HBLK) * 8;
        bcol[NUB + i] = bcol[i] + WCOLS / 2;
    }

    i32x4_t ra, rb;
    int i_m0 = 0, i_n0 = 0, i_kbeg = 0, i_kend = 0, i_nk = 0, i_kt = 0;
    const unsigned a_lane = (unsigned)(lrow * p.lda * 2), b_lane = (unsigned)(lrow * p.ldb * 2);
    auto setup_issue = [&](int w) {
        const PPItem it = pp_item(w, tm, tn, p.splits, BM, BN);
        const bf16* A = reinterpret_cast<const bf16*>(p.A) + it.zb * p.strideA;
        const bf16* B = reinterpret_cast<const bf16*>(p.B) + it.zb * p.strideB;
        ra = uniform_rsrc_words(A, (int64_t)p.M * p.lda * 2);
        rb = uniform_rsrc_words(B, (int64_t)p.N * p.ldb * 2);
        i_m0 = it.m0;
        i_n0 = it.n0;
        i_kbeg = it.zs * p.k_chunk;
        i_kend = min(p.K, i_kbeg + p.k_chunk);
        i_nk = max(1, (i_kend - i_kbeg + BK - 1) / BK);
        i_kt = 0;
    };
    int ops = 0;                                          // VMEM ops this wave has issued (uniform)
    // unit U of the issue side's current K-tile into `buf` (inline asm: the
    // compiler's waitcnt pass does not see these, the counted waits order them)
    auto issue = [&](auto U_, char* buf) {
        constexpr int U = decltype(U_)::value;
        const int k = i_kbeg + i_kt * BK + 8 * cs;
        const bool kok = k < i_kend;
        if constexpr (U == 0 || U == 3) {
#pragma unroll
            for (int i = 0; i < NUA; ++i) {
                const int s = (U == 0 ? 0 : 2) + i;
                const int mrow = i_m0 + arow[s];
                const bool ok = kok && lrow < p.M - mrow;
                const unsigned voff = a_lane + (unsigned)(mrow * p.lda * 2) + (unsigned)(k * 2);
                lds_dma16_asm(ra, buf + arow[s] * ROWB, ok ? voff : PP_OOB);
            }
            ops += NUA;
        } else {
#pragma unroll
            for (int i = 0; i < NUB; ++i) {
                const int s = (U == 1 ? 0 : NUB) + i;
                const int ncol = i_n0 + bcol[s];
                const bool ok = kok && lrow < p.N - ncol;
                const unsigned voff = b_lane + (unsigned)(ncol * p.ldb * 2) + (unsigned)(k * 2);
                lds_dma16_asm(rb, buf + A_BYTES + bcol[s] * ROWB, ok ? voff : PP_OOB);
            }
            ops += NUB;
        }
    };
    int is = 0;                                           // step the issue side is on
    auto advance_issue = [&]() -> bool {
        ++is;
        if (++i_kt < i_nk) return true;
        w_issue += sp;
        if (w_issue >= wend) return false;
        setup_issue(w_issue);
        return true;
    };
    auto ibuf = [&]() { return smem + (is & 1) * BUF; };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;

    int w_comp = w_issue;
    PPItem cur_it = pp_item(w_comp, tm, tn, p.splits, BM, BN);
    int c_nk, c_kt = 0;

    // prologue: step 0 whole, then U0 / U1 of step 1
    int m3_cur = 0, m3_next = 0, m2_next = 0, m1_next = 0, m1_next2 = 0;
    setup_issue(w_issue);
    c_nk = i_nk;
    issue(I0{}, ibuf());
    issue(I1{}, ibuf());
    issue(I2{}, ibuf());
    issue(I3{}, ibuf());
    m3_cur = ops;
    bool more = advance_issue();
    if (more) {
        issue(I0{}, ibuf());
        issue(I1{}, ibuf());
        m1_next = ops;
    }
    vm_wait_n(ops - m3_cur);
    pp_barrier();
    if (wm == 1) pp_barrier();

    floatx4 acc[8][2 * QN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2 * QN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    bf16x8 afr[4][2], bq0[QN][2], bq1[QN][2];
    const int a_base = (wm * 128 + i16) * ROWB, b_base = A_BYTES + (wn * WCOLS + i16) * ROWB;
    auto read_a = [&](const char* cur, int qa) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                afr[i][kk] = *reinterpret_cast<const bf16x8*>(
                    cur + a_base + (qa * 64 + i * 16) * ROWB + (((kk * 4 + g) ^ sw) << 4));
    };
    auto read_b = [&](const char* cur, int qb, bf16x8 (&bf)[QN][2]) {
#pragma unroll
        for (int j = 0; j < QN; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                bf[j][kk] = *reinterpret_cast<const bf16x8*>(
                    cur + b_base + (qb * (WCOLS / 2) + j * 16) * ROWB + (((kk * 4 + g) ^ sw) << 4));
    };
    auto mfma_q = [&](auto QA_, auto QB_, const bf16x8 (&bf)[QN][2]) {
        constexpr int QA = decltype(QA_)::value, QB = decltype(QB_)::value;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < QN; ++j)
                    acc[QA * 4 + i][QB * QN + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        bf[j][kk], afr[i][kk], acc[QA * 4 + i][QB * QN + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    int s = 0;
    for (;;) {
        const char* cur = smem + (s & 1) * BUF;
        // ---- phase 0: A q0 + B q0 (B q0 kept to phase 3); U2(s+1); retire U3(s)
        read_a(cur, 0);
        read_b(cur, 0, bq0);
        if (more) { issue(I2{}, ibuf()); m2_next = ops; }
        vm_wait_fast<NUA + 2 * NUB>(ops - m3_cur);                 // U0, U1, U2(s+1) stay in flight
        pp_barrier();
        mfma_q(I0{}, I0{}, bq0);
        pp_barrier();
        // ---- phase 1: B q1; U3(s+1)
        read_b(cur, 1, bq1);
        if (more) {
            issue(I3{}, ibuf());
            m3_next = ops;
            more = advance_issue();
        }
        pp_barrier();
        mfma_q(I0{}, I1{}, bq1);
        pp_barrier();
        // ---- phase 2: A q1 (B q1 kept); U0(s+2); retire U0 + U1(s+1)
        read_a(cur, 1);
        if (more) issue(I0{}, ibuf());
        vm_wait_fast<NUB + 2 * NUA>(ops - m1_next);                // U2, U3(s+1), U0(s+2) stay
        pp_barrier();
        mfma_q(I1{}, I1{}, bq1);
        pp_barrier();
        // ---- phase 3: no LDS reads (B q0 from phase 0); U1(s+2); retire U2(s+1)
        if (more) { issue(I1{}, ibuf()); m1_next2 = ops; }
        vm_wait_fast<2 * NUA + NUB>(ops - m2_next);                // U3(s+1), U0, U1(s+2) stay
        pp_barrier();
        mfma_q(I1{}, I0{}, bq0);
        pp_barrier();
        m3_cur = m3_next;
        m1_next = m1_next2;
        ++s;
        if (++c_kt < c_nk) continue;

        // ================================================= item epilogue
        if (wm == 0) pp_barrier();                        // groups meet: step s's reads are done
        // staging: the U2 (waves 0-3) / U3 (waves 4-7) slots of step s's buffer
        char* stg = const_cast<char*>(cur) +
                    (wm == 0 ? A_BYTES + (wn * WCOLS + WCOLS / 2) * ROWB : (wn < 2 ? 64 : 192) * ROWB + (wn & 1) * 4096);
        floatx4 bv[2 * QN];
        if (p.bias) {
            const __amdgpu_buffer_rsrc_t rbias = uniform_rsrc(p.bias + cur_it.zb * p.strideBias, (int64_t)p.N * 4);
            const int ncol0 = cur_it.n0 + wn * WCOLS + 4 * g;
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) {
                const int n = ncol0 + j * 16;
                bv[j] = __builtin_bit_cast(
                    floatx4, __builtin_amdgcn_raw_buffer_load_b128(rbias, n < p.N ? (unsigned)(n * 4) : PP_OOB, 0, 0));
            }
            ops += 2 * QN;
        } else {
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) bv[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < 2 * QN; ++j) {
            const floatx4 b = bv[j];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                floatx4 v = acc[i][j] * p.alpha + b;
                if (p.relu) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
                }
                acc[i][j] = v;
            }
        }
        bf16* Cb = reinterpret_cast<bf16*>(p.C) + cur_it.zb * p.strideC;
        const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(Cb, ((int64_t)(p.M - 1) * p.ldc + p.N) * 2);
        const int c8 = lane % CPRW, r0 = lane / CPRW;
        const int n = cur_it.n0 + wn * WCOLS + 8 * c8;
#pragma unroll
        for (int h = 0; h < 128 / CR; ++h) {
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) {
                u16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = __builtin_bit_cast(unsigned short, (bf16)acc[h][j][r]);
                *reinterpret_cast<u16x4*>(stg + i16 * PITCH + (j * 16 + 4 * g) * 2) = o;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int q = 0; q < CR * CPRW / 64; ++q) {
                const int r = r0 + q * (64 / CPRW);
                const int m = cur_it.m0 + wm * 128 + h * CR + r;
                const u32x4 v = *reinterpret_cast<const u32x4*>(stg + r * PITCH + c8 * 16);
                const unsigned off = (m < p.M && n < p.N) ? (unsigned)(((int64_t)m * p.ldc + n) * 2) : PP_OOB;
                __builtin_amdgcn_raw_buffer_store_b128(v, rc, off, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        ops += NST;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();                                     // staging reads done before U2 / U3(s+1) refill them
        w_comp += sp;
        if (w_comp >= wend) break;
        cur_it = pp_item(w_comp, tm, tn, p.splits, BM, BN);
        c_nk = max(1, (min(p.K, cur_it.zs * p.k_chunk + p.k_chunk) - cur_it.zs * p.k_chunk + BK - 1) / BK);
        c_kt = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 2 * QN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (wm == 1) pp_barrier();                        // re-stagger
    }
}

template <int BN>
int launch_pp_deep(const GemmParams& p, hipStream_t stream) {
    constexpr int LDS = 2 * (256 + BN) * 128;
    static DeviceOnce configured;
    set_dyn_lds(configured, reinterpret_cast<const void*>(&gemm_pp_deep_kernel<BN>), LDS);
    const int ncu = cu_count();
    const int64_t items = cdiv(p.M, 256) * cdiv(p.N, BN) * (int64_t)p.batch * p.splits;
    // persistent: one workgroup per CU, items prefetched across
    const int64_t grid = std::min<int64_t>(cdiv(items, 8) * 8, (int64_t)(ncu / 8) * 8);
    gemm_pp_deep_kernel<BN><<<dim3((unsigned)grid), 512, LDS, stream>>>(p);
    return launch_status("gemm_pp_deep");
}

template <int AM, int BN, bool STATS, bool MASK>
int launch_pp_k(const GemmParams& p, hipStream_t stream) {
    constexpr int LDS = 2 * (256 + BN) * 128;
    static DeviceOnce configured;
    set_dyn_lds(configured, reinterpret_cast<const void*>(&gemm_pp_kernel<AM, BN, STATS, MASK>), LDS);
    const int ncu = cu_count();
    const int64_t items = cdiv(p.M, 256) * cdiv(p.N, BN) * (int64_t)p.batch * p.splits;
    // Short K (a few steps per item): persistent, one workgroup per CU, the
    // next item's first K-tile prefetched under the current one. Long K: one
    // item per workgroup -- the epilogue's stores then never sit in front of
    // the next item's DMA waits (vmcnt is in order), measured faster for K >= 1024.
    const int64_t nk = cdiv(p.K, 64);
    const int64_t grid = nk <= opt(OPT_PP_PERSIST_NK) ? std::min<int64_t>(cdiv(items, 8) * 8, (int64_t)(ncu / 8) * 8)
                                 : cdiv(items, 8) * 8;
    gemm_pp_kernel<AM, BN, STATS, MASK><<<dim3((unsigned)grid), 512, LDS, stream>>>(p);
    return launch_status("gemm_pp");
}

template <int AM, int BN>
int launch_pp(const GemmParams& p, hipStream_t stream) {
    if (AM == A_IM2COL_FLIP && p.mask) {
        if (p.stats) return launch_pp_k<AM, BN, true, true>(p, stream);
        return launch_pp_k<AM, BN, false, true>(p, stream);
    }
    if (p.mask) return -1;
#ifdef OCRK_EXPERIMENTS
    // the deep-lead schedule (tools build: measured no gain, its wait fraction 0.404 vs 0.415,
    // profiles/r6_pp_deep_counters.txt)
    if (AM == A_ROWK && !p.stats && opt(OPT_PP_DEEP)) return launch_pp_deep<BN>(p, stream);
#endif
    if (p.stats) return launch_pp_k<AM, BN, true, false>(p, stream);
    return launch_pp_k<AM, BN, false, false>(p, stream);
}

template <int AM>
int dispatch_pp(const GemmParams& p, hipStream_t s) {
    // 256-wide tiles when they still give every CU an item, else 128
    if (p.N >= 192 && cdiv(p.M, 256) * cdiv(p.N, 256) * p.batch * p.splits >= 256) return launch_pp<AM, 256>(p, s);
    return launch_pp<AM, 128>(p, s);
}

}  // namespace

bool gemm_pp_enabled() {
    return opt(OPT_GEMM_PP) != 0;              // 0: the previous engines only
}

// Runs the ping-pong engine when it covers (mode, dtype, shape); -1 otherwise.
// Routed: plain A_ROWK GEMMs with N >= 512 (the recurrent input projections,
// the recurrent and logits data gradients); the convolutions and the narrow
// data gradient measured faster on the NT engine (tools/bench_pp.py).
int gemm_pp(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    if (!gemm_pp_enabled() || dtype != OCRK_BF16 || bmode != B_NK) return -1;
    // bf16 C, whole K per item (no split-K partials, no f32 accumulation)
    if (!p.c_bf16 || p.accumulate || p.splits != 1) return -1;
    if (p.N % 8 != 0 || p.K % 8 != 0) return -1;
    if ((int64_t)p.M < 4096) return -1;
#ifdef OCRK_EXPERIMENTS
    static const int all = [] { const char* e = getenv("OCRK_GEMM_PP"); return e && e[0] == '2'; }();
#else
    constexpr int all = 0;
#endif
    // the convolutions stay on the NT / row engines: routed here (N >= 128) they measured
    // 1.4-2.1x slower per layer and 5.23-5.51 vs 5.08-5.11 ms per step (round 4)
    // plain GEMMs from N >= PP_MIN_N (512: the narrow L1 data gradient, N = 256, stays on NT)
    if (!all && (amode != A_ROWK || p.N < opt(OPT_PP_MIN_N))) return -1;   // OCRK_GEMM_PP=2: every shape (make exp)
    if (p.N < 96) return -1;
    // 32-bit buffer offsets
    const int64_t a_bytes = (amode == A_ROWK ? (int64_t)p.M * p.lda : (int64_t)p.M * p.convC) * 2;
    const int64_t c_bytes = (int64_t)p.M * p.ldc * 2;
    if (a_bytes >= (1ll << 31) || (int64_t)p.N * p.ldb * 2 >= (1ll << 31) || c_bytes >= (1ll << 31)) return -1;
    // 16-B (staged bf16) / 8-B epilogue vectors: C, the mask and the bias rows aligned
    if (p.ldc % 8 != 0 || p.strideC % 8 != 0 || (uintptr_t)p.C % 16 != 0) return -1;
    if (p.bias && (uintptr_t)p.bias % 16 != 0) return -1;
    if (p.mask && (p.ldmask % 8 != 0 || (uintptr_t)p.mask % 16 != 0)) return -1;
    if (amode == A_ROWK) {
        if (p.lda % 8 != 0 || p.ldb % 8 != 0) return -1;
        return dispatch_pp<A_ROWK>(p, stream);
    }
    if (p.ldb % 8 != 0) return -1;
    if (amode == A_IM2COL) return dispatch_pp<A_IM2COL>(p, stream);
    if (amode == A_IM2COL_FLIP) return dispatch_pp<A_IM2COL_FLIP>(p, stream);
    return -1;
}

}  // namespace ocrk
