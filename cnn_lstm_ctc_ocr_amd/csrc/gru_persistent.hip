// a7': the BiGRU time loop as ONE persistent launch per layer and direction
// pair (rnn_layer with tf.contrib.rnn.GRUCell, src/weinman/model.py:167-199,
// the cell model.py:213-214 selects; bidirectional_dynamic_rnn with
// sequence_length). [TF1] GRUCell: [r, u] = sig([x, h] Wg + bg);
// c = tanh([x, r*h] Wc + bc); h' = u h + (1 - u) c.
//
// Groups, members, placement and the hand-off protocol are the LSTM's
// (persist.h): a group is (direction, 32 batch rows), a member owns 32 hidden
// units, 2 * B/32 * H/32 co-resident workgroups (256 at B = 256, H = 512).
// The reset gate multiplies h BEFORE the candidate matmul, so a GRU step has
// TWO group-wide exchanges where the LSTM has one:
//   forward step s:  h_{s-1}  -> gates r, u of own units -> publish r*h_{s-1}
//                    r*h      -> candidate c of own units -> publish h_s
//   backward step s: dz_c     -> d(r*h) of own units -> dz_r, dz_u -> publish
//                    dz_r,u   -> dh_{s-1} of own units (carried in registers)
// One flag word per member counts exchanges (2 per step), so every wait is
// "all flags >= n". Each exchanged row block is [32 rows x N] bf16, double
// buffered by step parity (a member cannot lap the slowest one by two
// exchanges: every publish waits for the exchange before it).
//
// MFMA split: every GEMM of the step is split over the 4 waves by K (wave w
// owns a quarter of the k-range, both 16-row M tiles and all N tiles); each
// wave stages only its k-range of the exchanged rows in its own LDS region
// (whole-row sc1/nt loads, no workgroup barrier) and the 4 partial products
// meet in LDS. The member's weight slices stay in VGPRs for the whole
// sequence: forward Wg_h^T (64 gate columns) + Wc_h^T (32 columns), backward
// Wc_h + Wg_h rows of the member's 32 units -- 96 x H bf16 = 96 VGPRs per
// lane at H = 512.
#include "persist.h"
#include "recur.h"

using namespace ocrk;

namespace {

// acc[mt][j] += rows[16 mt + i][k] . bw[j][k] over this wave's k-range: the
// group's published rows (row stride ld elements, from rbase) are staged by
// LDS-DMA straight into the wave's LDS block (rows of KR elements, 16-B
// pieces XOR-swizzled per row so the 16 rows of an operand read hit distinct
// bank groups), all 32 rows in flight at once; M tile 0 multiplies as soon as
// its 16 rows have landed (counted vmcnt: nothing else is issued in between).
__device__ __forceinline__ int stage_swz(int r, int lpr) { return lpr >= 8 ? (r & 7) : ((r >> 2) & 3); }

struct NoExtra {
    __device__ void operator()() const {}
};

// `extra` issues exactly NX vector-memory loads BEHIND the DMAs (operands of a
// later phase): the counted waits below then leave them in flight, so they
// never delay a hand-off poll or this staging (vmcnt completes in order).
template <int KR, int NT, int NX = 0, typename F = NoExtra>
__device__ __forceinline__ void stage_mma(__amdgpu_buffer_rsrc_t rs, int64_t rbase, int ld, bool local,
                                          unsigned short* sA, int wstride, const bf16x8 (&bw)[NT][KR / 32],
                                          floatx4 (&acc)[2][NT], F extra = F()) {
    constexpr int LPR = KR / 8, RPI = 64 / LPR, NI = PBR / RPI;     // NI 1-KB DMA instructions per wave
    static_assert(LPR >= 4 && 64 % LPR == 0 && NI % 2 == 0 && NI / 2 < 16, "row staging");
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned short* sa = sA + wu * wstride;                          // wave-uniform LDS base (M0)
    const int lr = lane / LPR, slot = lane % LPR;
    if (local) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int r = q * RPI + lr;
            const unsigned off = (unsigned)((rbase + (int64_t)r * ld + 8 * (slot ^ stage_swz(r, LPR))) * 2);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(sa + q * 512), 16,
                                                     off, 0, 0, 2);           // nt
        }
    } else {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int r = q * RPI + lr;
            const unsigned off = (unsigned)((rbase + (int64_t)r * ld + 8 * (slot ^ stage_swz(r, LPR))) * 2);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(sa + q * 512), 16,
                                                     off, 0, 0, 16);          // sc1
        }
    }
    auto mma_tile = [&](int mt) {
        const int R = 16 * mt + c;
#pragma unroll
        for (int kk = 0; kk < KR / 32; ++kk) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(&sa[R * KR + 8 * ((4 * kk + g) ^ stage_swz(R, LPR))]);
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][kk], acc[mt][j], 0, 0, 0);
        }
    };
    if constexpr (NX > 0) {
        asm volatile("" ::: "memory");
        extra();
    }
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI / 2 + NX) : "memory");
    mma_tile(0);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NX) : "memory");
    mma_tile(1);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 ld8(__amdgpu_buffer_rsrc_t r, int64_t byte_off) {
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)byte_off, 0, 0));
}
__device__ __forceinline__ void unpack4(u32x2 q, float (&v)[4]) {
    v[0] = __uint_as_float(q[0] << 16); v[1] = __uint_as_float(q[0] & 0xffff0000u);
    v[2] = __uint_as_float(q[1] << 16); v[3] = __uint_as_float(q[1] & 0xffff0000u);
}

// wave w's accumulators -> its partial block sP[w][32 rows][ld]
template <int NT>
__device__ __forceinline__ void spill_partial(const floatx4 (&acc)[2][NT], float* sP, int ld) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) sP[(w * PBR + 16 * mt + 4 * g + r) * ld + 16 * j + c] = acc[mt][j][r];
}

// sum of the 4 waves' partials at (row, col..col+3)
__device__ __forceinline__ void sum_partials(const float* sP, int ld, int row, int col, float (&z)[4]) {
    f32x4 p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = *reinterpret_cast<const f32x4*>(&sP[(q * PBR + row) * ld + col]);
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = (p[0][e] + p[1][e]) + (p[2][e] + p[3][e]);
}

__device__ __forceinline__ float bf16r(float x) { return (float)(bf16)x; }

}  // namespace

// ---------------------------------------------------------------- forward
// KS = H / 32. gx [T][B][2][3H] = x . [Wg_x | Wc_x] + [bg | bc] (r | u | c per
// direction, one GEMM before the loop); whgT [2][2H][H] (row = gate*H + unit),
// whcT [2][H][H] (row = unit). Saves hprev_t, rh_t [T][B][2][H] and acts_t
// [T][B][2][3H] = (r, u, c) in time order, zeros at steps >= len.
template <int KS>
__global__ void __launch_bounds__(256, 1)
gru_fwd_persistent_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whgT, const bf16* __restrict__ whcT,
                          bf16* __restrict__ hx, bf16* __restrict__ rhx, const int* __restrict__ seq_len, int T,
                          int B, bf16* __restrict__ out, bf16* __restrict__ hprev_t, bf16* __restrict__ rh_t,
                          bf16* __restrict__ acts_t, unsigned* __restrict__ flags, unsigned* __restrict__ err,
                          unsigned spin_limit) {
    constexpr int H = KS * 32, G3 = 3 * H, NU = H / PHU, KR = H / 4, KW = KR / 32;
    constexpr int LDA = KR + 8, LDG = 2 * PHU + 4, LDC = PHU + 4;
    static_assert(NU <= 64 && KW >= 1, "one poll lane per member; k-range per wave");
    __shared__ __attribute__((aligned(16))) unsigned short sA[4 * PBR * LDA];   // [wave][row][k of its range]
    __shared__ __attribute__((aligned(16))) float sPg[4 * PBR * LDG];          // [wave][row][r units | u units]
    __shared__ __attribute__((aligned(16))) float sPc[4 * PBR * LDC];          // [wave][row][c units]

    int group, member;
    persistent_role(2 * (B / PBR), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);
    bool dead = false;

    // resident B fragments, k = w KR + 32 kk + 8 g: gate N-tile j col c is
    // gate (16 j + c) >> 5 of unit u0 + ((16 j + c) & 31); candidate N-tile j col c is unit u0 + 16 j + c
    bf16x8 bg[4][KW], bc[2][KW];
    {
        const bf16* wg = whgT + (size_t)dir * 2 * H * H;
        const bf16* wc = whcT + (size_t)dir * H * H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = 16 * j + c;
            const bf16* row = wg + (size_t)((n >> 5) * H + u0 + (n & 31)) * H + w * KR + 8 * g;
#pragma unroll
            for (int kk = 0; kk < KW; ++kk) bg[j][kk] = *reinterpret_cast<const bf16x8*>(row + 32 * kk);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bf16* row = wc + (size_t)(u0 + 16 * j + c) * H + w * KR + 8 * g;
#pragma unroll
            for (int kk = 0; kk < KW; ++kk) bc[j][kk] = *reinterpret_cast<const bf16x8*>(row + 32 * kk);
        }
    }

    // the epilogue item of this thread: row er, units eu..eu+3
    const int er = tid >> 3, eu = 4 * (tid & 7);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));                       // settled before the loop (lstm_persistent.hip)
    float hst[4] = {0.f, 0.f, 0.f, 0.f};
    const int xbytes = 2 * 2 * B * H * 2;
    const auto hx_rsrc = __builtin_amdgcn_make_buffer_rsrc(hx, 0, xbytes, 0x00020000);
    const auto rhx_rsrc = __builtin_amdgcn_make_buffer_rsrc(rhx, 0, xbytes, 0x00020000);

    // gx as one buffer: its loads are issued behind the first staging DMA as
    // exactly 3 buffer instructions (stage_mma's counted waits rely on that)
    const __amdgpu_buffer_rsrc_t gx_rsrc = uniform_rsrc(gx, (int64_t)T * B * 2 * G3 * 2);

    for (int s = 0; s < T; ++s) {
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        // 0. this step's input projections (independent of h), issued behind the
        //    h_{s-1} staging DMA so that neither the hand-off poll nor the staging
        //    waits for their HBM latency (vmcnt completes in order)
        float pr[4], pu[4], pc[4];
        u32x2 gq[3];
        auto load_gx = [&]() {
            const int64_t e = (tb * G3 + u0 + eu) * 2;
            gq[0] = ld8(gx_rsrc, e);
            gq[1] = ld8(gx_rsrc, e + 2 * H);
            gq[2] = ld8(gx_rsrc, e + 4 * H);
        };
        float zr[4] = {0.f, 0.f, 0.f, 0.f}, zu[4] = {0.f, 0.f, 0.f, 0.f}, zc[4] = {0.f, 0.f, 0.f, 0.f};
        if (s == 0) load_gx();
        if (s > 0) {
            // 1. gates: h_{s-1} . Wg_h over this wave's k-range (h_{-1} = 0: nothing at s = 0)
            group_wait(gflags, NU, base + 2u * s, local, err, OCRK_STATUS_LSTM_FWD_TIMEOUT, spin_limit, dead);
            floatx4 acc[2][4];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            stage_mma<KR, 4, 3>(hx_rsrc, ((int64_t)(((s - 1) & 1) * 2 + dir) * B + b0) * H + w * KR, H, local, sA,
                                PBR * LDA, bg, acc, load_gx);
            spill_partial<4>(acc, sPg, LDG);
            __syncthreads();
            sum_partials(sPg, LDG, er, eu, zr);
            sum_partials(sPg, LDG, er, PHU + eu, zu);
        }
        unpack4(gq[0], pr);
        unpack4(gq[1], pu);
        unpack4(gq[2], pc);
        float ar[4], au[4], rh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            ar[e] = sig_fast(zr[e] + pr[e]);
            au[e] = sig_fast(zu[e] + pu[e]);
            rh[e] = valid ? bf16r(ar[e] * hst[e]) : 0.f;
        }
        if (s > 0) {
            // 2. publish r*h of own units, then the candidate: (r*h) . Wc_h
            put8((gu64*)(rhx + ((int64_t)((s & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu), pack4(rh), local);
            group_post(gflags + member, base + 2u * s + 1u, local);
            group_wait(gflags, NU, base + 2u * s + 1u, local, err, OCRK_STATUS_LSTM_FWD_TIMEOUT, spin_limit, dead);
            floatx4 acc[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            stage_mma<KR, 2>(rhx_rsrc, ((int64_t)((s & 1) * 2 + dir) * B + b0) * H + w * KR, H, local, sA, PBR * LDA,
                             bc, acc);
            spill_partial<2>(acc, sPc, LDC);
            __syncthreads();
            sum_partials(sPc, LDC, er, eu, zc);
        }
        // 3. the new state of own units; publish h_s
        float ac[4], hp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            ac[e] = tanh_fast(zc[e] + pc[e]);
            const float hn = au[e] * hst[e] + (1.f - au[e]) * ac[e];
            hp[e] = valid ? hst[e] : 0.f;
            if (valid) hst[e] = bf16r(hn);
            if (!valid) { ar[e] = 0.f; au[e] = 0.f; ac[e] = 0.f; }
        }
        put8((gu64*)(hx + ((int64_t)((s & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu), pack4(hst), local);
        group_post(gflags + member, base + 2u * s + 2u, local);
        // 4. layer output and the tensors saved for the backward pass (drain behind the next step)
        {
            // padded positions (t = s >= len) get this direction's zeros: the caller need not clear out
            float ov[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = valid ? hst[e] : 0.f;
            st4(out + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu, ov);
        }
        st4(hprev_t + tb * H + u0 + eu, hp);
        st4(rh_t + tb * H + u0 + eu, rh);
        bf16* a = acts_t + tb * G3 + u0 + eu;
        st4(a, ar);
        st4(a + H, au);
        st4(a + 2 * H, ac);
    }
}

// ---------------------------------------------------------------- backward
// whg [2][H][2H] = Wg_h, whc [2][H][H] = Wc_h (row = the member's unit as k of
// dh / d(r*h)). Reverse step i (s = T-1-i), own units, dh carried in registers:
//   dh_tot = dh + dout;  dz_c = dh_tot (1-u)(1-c^2)             -> publish dz_c
//   d(rh)  = dz_c . Wc_h^T (K = H, all units)
//   dz_r = d(rh) h r(1-r);  dz_u = dh_tot (h-c) u(1-u)          -> publish dz_r, dz_u
//   dh     = dh_tot u + d(rh) r + [dz_r, dz_u] . Wg_h^T (K = 2H)
// dG_t [T][B][2][3H] = (dz_r, dz_u, dz_c) in time order for the weight-gradient GEMMs.
template <int KS>
__global__ void __launch_bounds__(256, 1)
gru_bwd_persistent_kernel(const bf16* __restrict__ whg, const bf16* __restrict__ whc, bf16* __restrict__ zxc,
                          bf16* __restrict__ zxg, const int* __restrict__ seq_len, int T, int B,
                          const bf16* __restrict__ dout, const bf16* __restrict__ hprev_t,
                          const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t, unsigned* __restrict__ flags,
                          unsigned* __restrict__ err, unsigned spin_limit, float* __restrict__ bpart) {
    constexpr int H = KS * 32, G3 = 3 * H, NU = H / PHU;
    constexpr int KRC = H / 4, KWC = KRC / 32, KRG = H / 2, KWG = KRG / 32;
    constexpr int LDA = KRG + 8, LDP = PHU + 4;
    static_assert(NU <= 64 && KWC >= 1, "one poll lane per member; k-range per wave");
    __shared__ __attribute__((aligned(16))) unsigned short sA[4 * PBR * LDA];
    __shared__ __attribute__((aligned(16))) float sP1[4 * PBR * LDP];
    __shared__ __attribute__((aligned(16))) float sP2[4 * PBR * LDP];

    int group, member;
    persistent_role(2 * (B / PBR), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);
    bool dead = false;

    // resident B fragments: N-tile j col c = unit u0 + 16 j + c; k = w KR + 32 kk + 8 g
    bf16x8 bc[2][KWC], bg[2][KWG];
    {
        const bf16* wc = whc + (size_t)dir * H * H;
        const bf16* wg = whg + (size_t)dir * H * 2 * H;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bf16* rc = wc + (size_t)(u0 + 16 * j + c) * H + w * KRC + 8 * g;
            const bf16* rg = wg + (size_t)(u0 + 16 * j + c) * 2 * H + w * KRG + 8 * g;
#pragma unroll
            for (int kk = 0; kk < KWC; ++kk) bc[j][kk] = *reinterpret_cast<const bf16x8*>(rc + 32 * kk);
#pragma unroll
            for (int kk = 0; kk < KWG; ++kk) bg[j][kk] = *reinterpret_cast<const bf16x8*>(rg + 32 * kk);
        }
    }

    const int er = tid >> 3, eu = 4 * (tid & 7);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));                       // settled before the loop (lstm_persistent.hip)
    float dh[4] = {0.f, 0.f, 0.f, 0.f};
    float bsum[3][4] = {};                              // the bias gradients: (dz_r, dz_u, dz_c) summed over steps
    const auto zxc_rsrc = __builtin_amdgcn_make_buffer_rsrc(zxc, 0, 2 * 2 * B * H * 2, 0x00020000);
    const auto zxg_rsrc = __builtin_amdgcn_make_buffer_rsrc(zxg, 0, 2 * 2 * B * 2 * H * 2, 0x00020000);

    // the step's epilogue operands are prefetched one step ahead, issued behind
    // the previous step's second staging DMA as exactly 5 buffer loads: loaded at
    // the top of the step they sat in front of its first hand-off drain and poll
    const __amdgpu_buffer_rsrc_t act_rsrc = uniform_rsrc(acts_t, (int64_t)T * B * 2 * G3 * 2);
    const __amdgpu_buffer_rsrc_t hp_rsrc = uniform_rsrc(hprev_t, (int64_t)T * B * 2 * H * 2);
    const __amdgpu_buffer_rsrc_t do_rsrc = uniform_rsrc(dout, (int64_t)T * B * 2 * H * 2);
    u32x2 pq[5];
    auto load_step = [&](int ii) {
        const int ts = step_time(dir, T - 1 - ii, elen);
        const int64_t tbb = ((int64_t)ts * B + b0 + er) * 2 + dir;
        const int64_t a = (tbb * G3 + u0 + eu) * 2;
        pq[0] = ld8(act_rsrc, a);
        pq[1] = ld8(act_rsrc, a + 2 * H);
        pq[2] = ld8(act_rsrc, a + 4 * H);
        pq[3] = ld8(hp_rsrc, (tbb * H + u0 + eu) * 2);
        pq[4] = ld8(do_rsrc, (((int64_t)ts * B + b0 + er) * 2 * H + dir * H + u0 + eu) * 2);
    };
    load_step(0);

    for (int i = 0; i < T; ++i) {
        const int s = T - 1 - i;
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        float ar[4], au[4], ac[4], hp[4], go[4];
        unpack4(pq[0], ar);
        unpack4(pq[1], au);
        unpack4(pq[2], ac);
        unpack4(pq[3], hp);
        unpack4(pq[4], go);
        // 1. dh_tot and dz_c of own units; publish dz_c
        float dt[4], dzc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            dt[e] = valid ? dh[e] + go[e] : 0.f;
            dzc[e] = bf16r(dt[e] * (1.f - au[e]) * (1.f - ac[e] * ac[e]));
        }
        put8((gu64*)(zxc + ((int64_t)((i & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu), pack4(dzc), local);
        group_post(gflags + member, base + 2u * i + 1u, local);
        group_wait(gflags, NU, base + 2u * i + 1u, local, err, OCRK_STATUS_LSTM_BWD_TIMEOUT, spin_limit, dead);
        // 2. d(r*h) of own units = dz_c . Wc_h^T
        float drh[4];
        {
            floatx4 acc[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            stage_mma<KRC, 2>(zxc_rsrc, ((int64_t)((i & 1) * 2 + dir) * B + b0) * H + w * KRC, H, local, sA, PBR * LDA, bc,
                              acc);
            spill_partial<2>(acc, sP1, LDP);
            __syncthreads();
            sum_partials(sP1, LDP, er, eu, drh);
        }
        float dzr[4], dzu[4], direct[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            dzr[e] = bf16r(drh[e] * hp[e] * ar[e] * (1.f - ar[e]));
            dzu[e] = bf16r(dt[e] * (hp[e] - ac[e]) * au[e] * (1.f - au[e]));
            direct[e] = dt[e] * au[e] + drh[e] * ar[e];
        }
        if (i + 1 < T) {
            // 3. publish dz_r, dz_u; dh_{s-1} of own units = [dz_r, dz_u] . Wg_h^T + direct terms
            gu64* zg = (gu64*)(zxg + ((int64_t)((i & 1) * 2 + dir) * B + b0 + er) * 2 * H + u0 + eu);
            put8(zg, pack4(dzr), local);
            put8(zg + H / 4, pack4(dzu), local);
            group_post(gflags + member, base + 2u * i + 2u, local);
            group_wait(gflags, NU, base + 2u * i + 2u, local, err, OCRK_STATUS_LSTM_BWD_TIMEOUT, spin_limit, dead);
            floatx4 acc[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            stage_mma<KRG, 2, 5>(zxg_rsrc, ((int64_t)((i & 1) * 2 + dir) * B + b0) * 2 * H + w * KRG, 2 * H, local, sA,
                                 PBR * LDA, bg, acc, [&]() { load_step(i + 1); });
            spill_partial<2>(acc, sP2, LDP);
            __syncthreads();
            float rec[4];
            sum_partials(sP2, LDP, er, eu, rec);
#pragma unroll
            for (int e = 0; e < 4; ++e) dh[e] = valid ? rec[e] + direct[e] : 0.f;
        }
        // 4. time-order gate gradients for the weight-gradient GEMMs
        bf16* gt = dG_t + tb * G3 + u0 + eu;
        st4(gt, dzr);
        st4(gt + H, dzu);
        st4(gt + 2 * H, dzc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bsum[0][e] += valid ? dzr[e] : 0.f;
            bsum[1][e] += valid ? dzu[e] : 0.f;
            bsum[2][e] += valid ? dzc[e] : 0.f;
        }
    }
    if (bpart) {
        // the layer's bias gradients (model.py:170-180 gates / candidate biases),
        // fused: the member's 32 rows meet in LDS, one thread per gate column
        // writes the member's partial; the caller sums the B/32 slices
        constexpr int LDR = 3 * PHU + 4;
        float* red = reinterpret_cast<float*>(sA);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[er * LDR + k * PHU + eu + e] = bsum[k][e];
        __syncthreads();
        if (tid < 3 * PHU) {
            float sum = 0.f;
            for (int r = 0; r < PBR; ++r) sum += red[r * LDR + tid];
            bpart[(int64_t)(bs * 2 + dir) * G3 + (tid / PHU) * H + u0 + (tid % PHU)] = sum;
        }
    }
}

// ------------------------------------------------------------------ C ABI
template <typename Kern>
static int co_resident(Kern k, int B, int H) {
    if (B <= 0 || B % PBR || !(H == 256 || H == 512)) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess) return 0;
    return 2L * (B / PBR) * (H / PHU) <= (long)cus * per_cu ? 1 : 0;
}

extern "C" size_t ocrk_gru_fwd_persistent_workspace_size(int B, int H) {
    // counters, then the h and r*h exchange buffers [2 parity][2 dir][B][H] bf16
    return persistent_counter_bytes(B, H) + (size_t)2 * 2 * 2 * B * H * sizeof(bf16);
}

extern "C" int ocrk_gru_fwd_persistent_supported(int B, int H) {
    return H == 512 ? co_resident(gru_fwd_persistent_kernel<16>, B, H) : co_resident(gru_fwd_persistent_kernel<8>, B, H);
}

extern "C" int ocrk_gru_fwd_persistent(const void* gx, const void* whgT, const void* whcT, const int* seq_len, int T,
                                       int B, int H, void* out, void* hprev_t, void* rh_t, void* acts_t,
                                       unsigned* err, unsigned* flags, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_gru_fwd_persistent_supported(B, H), "ocrk_gru_fwd_persistent: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_gru_fwd_persistent_workspace_size(B, H), "ocrk_gru_fwd_persistent: workspace too small");
    OCRK_REQUIRE(err != nullptr, "ocrk_gru_fwd_persistent: status word required");
    if (T <= 0) return OCRK_OK;
    hipStream_t st = ocrk::as_stream(stream);
    const size_t counters = persistent_counter_bytes(B, H);
    bf16* hx = (bf16*)((char*)ws + counters);
    bf16* rhx = hx + (size_t)2 * 2 * B * H;
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    if (!flags && hipMemsetAsync(ws, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_gru_fwd_persistent memset");
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
    if (H == 512)
        gru_fwd_persistent_kernel<16><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whgT, (const bf16*)whcT, hx, rhx,
                                                            seq_len, T, B, (bf16*)out, (bf16*)hprev_t, (bf16*)rh_t,
                                                            (bf16*)acts_t, cnt, err, recur_spin_limit());
    else
        gru_fwd_persistent_kernel<8><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whgT, (const bf16*)whcT, hx, rhx,
                                                           seq_len, T, B, (bf16*)out, (bf16*)hprev_t, (bf16*)rh_t,
                                                           (bf16*)acts_t, cnt, err, recur_spin_limit());
    return ocrk::launch_status("ocrk_gru_fwd_persistent");
}

extern "C" size_t ocrk_gru_bwd_persistent_workspace_size(int B, int H) {
    // counters, then the dz_c [2][2][B][H] and dz_(r,u) [2][2][B][2H] exchange buffers (bf16)
    return persistent_counter_bytes(B, H) + (size_t)2 * 2 * 3 * B * H * sizeof(bf16);
}

extern "C" int ocrk_gru_bwd_persistent_supported(int B, int H) {
    return H == 512 ? co_resident(gru_bwd_persistent_kernel<16>, B, H) : co_resident(gru_bwd_persistent_kernel<8>, B, H);
}

extern "C" int ocrk_gru_bwd_persistent(const void* whg, const void* whc, const int* seq_len, int T, int B, int H,
                                       const void* dout, const void* hprev_t, const void* acts_t, void* dG_t,
                                       unsigned* err, unsigned* flags, float* dbias_part, void* ws, size_t ws_bytes,
                                       void* stream) {
    OCRK_REQUIRE(ocrk_gru_bwd_persistent_supported(B, H), "ocrk_gru_bwd_persistent: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_gru_bwd_persistent_workspace_size(B, H), "ocrk_gru_bwd_persistent: workspace too small");
    OCRK_REQUIRE(err != nullptr, "ocrk_gru_bwd_persistent: status word required");
    if (T <= 0) return OCRK_OK;
    hipStream_t st = ocrk::as_stream(stream);
    const size_t counters = persistent_counter_bytes(B, H);
    bf16* zxc = (bf16*)((char*)ws + counters);
    bf16* zxg = zxc + (size_t)2 * 2 * B * H;
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    if (!flags && hipMemsetAsync(ws, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_gru_bwd_persistent memset");
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
    if (H == 512)
        gru_bwd_persistent_kernel<16><<<grid, 256, 0, st>>>((const bf16*)whg, (const bf16*)whc, zxc, zxg, seq_len, T, B,
                                                            (const bf16*)dout, (const bf16*)hprev_t, (const bf16*)acts_t,
                                                            (bf16*)dG_t, cnt, err, recur_spin_limit(), dbias_part);
    else
        gru_bwd_persistent_kernel<8><<<grid, 256, 0, st>>>((const bf16*)whg, (const bf16*)whc, zxc, zxg, seq_len, T, B,
                                                           (const bf16*)dout, (const bf16*)hprev_t, (const bf16*)acts_t,
                                                           (bf16*)dG_t, cnt, err, recur_spin_limit(), dbias_part);
    return ocrk::launch_status("ocrk_gru_bwd_persistent");
}
