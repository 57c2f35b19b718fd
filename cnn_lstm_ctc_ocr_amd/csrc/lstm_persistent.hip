// a7': the BiLSTM forward time loop as ONE persistent launch per layer
// (rnn_layer, src/weinman/model_bu.py:167-199; [TF1] LSTMCell i, j, f, o,
// forget_bias 1; bidirectional_dynamic_rnn with sequence_length).
//
// Work split (bf16, H = 32 KS): 2 directions x B/32 batch slices = groups, each
// of H/32 member workgroups (16 at H = 512, B = 256: 256 workgroups, one per
// CU, all co-resident). A member owns 32 hidden units (x 4 gates = 128 gate
// columns) of one direction for 32 batch rows; its W_h^T slice [128 x H] stays
// in VGPRs for the whole sequence as MFMA B fragments (wave w: units
// 8w..8w+7, 4 gates = two 16-column tiles, all H/32 k-steps: 128 VGPRs) and
// its cell state c in registers. Per step a member
//   0. issues the loads of its gx tile (independent of h) first;
//   1. waits until the 16 members of its group have published h_{s-1}: one
//      flag word per member (sharded), polled by 16 lanes of wave 0;
//   2. stages h_{s-1}[32 x H] into LDS with sc1 (L1-bypassing) loads;
//   3. runs 2 x 2 tiles x H/32 k-steps of v_mfma_f32_16x16x32_bf16 per wave;
//   4. finishes the gates wave-locally (lanes l and l^8 hold the i/f and j/o
//      halves of one unit: two shuffles), keeping c in registers;
//   5. publishes h_s with sc1 stores, drains (vmcnt 0), barriers, and one lane
//      stores its flag = s + 1 (sc1);
//   6. only then stores the layer output and the tensors saved for the
//      backward pass (they drain behind the next step).
// Hand-off form: MI355X_MICROARCH.md "Valid forms", table row 1 (sc1 payload
// stores drained by every storing wave before the barrier, one lane's sc1 flag
// store per workgroup; consumer: sc1 poll of every shard, barrier, every
// payload load sc1) -- correct under any placement. Placement is used for
// speed only: the members of a group are the workgroups with equal
// blockIdx % 8 (dealt to one XCD by the dispatcher), so the group's hand-off
// traffic and its W_h^T slices stay on one XCD. Spins are bounded: on timeout
// the kernel records an error word and runs to completion (no hang).
#include "common.h"
#include "mfma_util.h"
#include "persist.h"
#include "recur.h"

using namespace ocrk;

namespace {

// diagnostics (ocrk_lstm_debug_stamps): thread 0 stamps step 64 (slots 0-5) and the top of step 65 (slot 6)
__device__ __forceinline__ void pstamp(long long* dbg, int s, int i) {
    if (dbg && threadIdx.x == 0 && (s == 64 || (s == 65 && i == 0)))
        dbg[(int64_t)blockIdx.x * 8 + (s == 65 ? 6 : i)] = __builtin_amdgcn_s_memrealtime();
}

// The layer's bias gradient, fused into the BPTT: each thread summed dz of its
// (row, 4 units, NG gates) over every step in f32 registers; the 32 rows of the
// member meet in LDS (`red`, >= 32 x (32 NG + 4) floats, free after the loop)
// and one thread per gate column writes the member's partial
// part[slice_off + gate H + u0 + unit]; the caller sums the B/32 slices
// (ocrk_colsum). Fixed order throughout: deterministic. part == NULL: skipped.
template <int NG>
__device__ __forceinline__ void bias_partials(float* part, const float (&bsum)[NG][4], float* red, int64_t slice_off,
                                              int H, int u0) {
    if (!part) return;
    constexpr int LDR = NG * PHU + 4;
    const int tid = threadIdx.x, er = tid >> 3, eu = 4 * (tid & 7);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NG; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[er * LDR + k * PHU + eu + e] = bsum[k][e];
    __syncthreads();
    if (tid < NG * PHU) {
        float sum = 0.f;
        for (int r = 0; r < PBR; ++r) sum += red[r * LDR + tid];
        part[slice_off + (tid / PHU) * H + u0 + (tid % PHU)] = sum;
    }
}

}  // namespace

extern long long* g_lstm_dbg;

static unsigned lstm_spin_limit() { return recur_spin_limit(); }

// KS = H / 32 k-steps. LATE (H = 512): the step's gx loads are issued AFTER the
// hand-off poll, behind the h_{s-1} LDS-DMA, and written to LDS after the MFMAs:
// vmcnt is in-order, so gx loads issued before the poll made every poll (and
// the staging wait) wait for their HBM latency as well.
// NIN > 0 (H = 512, LATE; the first layer, In = NIN = 256): the input projection
// x_t . W_x + b is FUSED into the loop instead of read as gx. The member's
// W_x^T slice (its 128 gate columns x NIN) stays in registers like W_h's; the
// 32 rows x_t of the step (each row's own t: reverse direction, ragged lengths)
// are staged by LDS-DMA one step ahead into a 2-deep ring (16-B pieces
// XOR-swizzled by row, so a fragment read of 16 rows hits 16 bank groups) --
// issued right behind the h_{s-1} staging DMA, landed by that step's publish
// drain; the x . W_x MFMAs of step s run at its top, before the hand-off poll
// (they do not depend on h), the bias is added in the cell. No gx tensor: the
// [T*B, 8H] projection GEMM and its 2 x 262 MB of HBM traffic (B = 256) go away.
template <int KS, bool LATE = false, int NIN = 0>
__global__ void __launch_bounds__(256, 1)
lstm_fwd_persistent_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whT, bf16* __restrict__ hx,
                           const int* __restrict__ seq_len, int T, int B, bf16* __restrict__ out,
                           bf16* __restrict__ hprev_t, float* __restrict__ cprev_t, bf16* __restrict__ acts_t,
                           unsigned* __restrict__ flags, unsigned* __restrict__ err, unsigned spin_limit,
                           long long* __restrict__ dbg, const bf16* __restrict__ xin = nullptr,
                           const bf16* __restrict__ wxT = nullptr, const float* __restrict__ bias = nullptr) {
    constexpr int H = KS * 32;
    constexpr int G4 = 4 * H;
    constexpr int NU = H / PHU;                         // members per group
    constexpr int LDH = H + 8;                          // padded LDS row (bf16 elements)
    static_assert(NU <= 64, "one poll lane per member");
    constexpr int LDG = 4 * PHU + 4;                    // padded gate row (floats)
    constexpr bool fx = NIN > 0;
    static_assert(!fx || (LATE && KS == 16 && NIN == 256), "fused input projection: H = 512, In = 256, late loads");
    constexpr int KX = fx ? NIN / 32 : 1;               // k-steps of the input projection
    __shared__ __attribute__((aligned(16))) unsigned short sh[PBR * LDH];
    __shared__ __attribute__((aligned(16))) unsigned short sgx[fx ? 8 : PBR * 4 * PHU];   // [row][gate][unit] bf16
    __shared__ __attribute__((aligned(16))) float sG[PBR * LDG];                 // [row][gate][unit] f32
    __shared__ __attribute__((aligned(16))) unsigned short sx[fx ? 2 * PBR * NIN : 8];    // x ring [2][row][NIN]
    __shared__ int s_len[PBR];

    int group, member;
    persistent_role(2 * (B / PBR), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int lu = 8 * w + (c & 7);                     // the unit (within the slice) this lane finishes
    const int my_unit = u0 + lu;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);
    if (dbg && threadIdx.x == 0) dbg[(int64_t)blockIdx.x * 8 + 7] = local ? 1 : 0;     // diagnostics: hand-off form

    // ---- resident B fragments: N-tile j holds gates 2j + (c >> 3) of unit my_unit
    bf16x8 bw[2][KS];
    const bf16* wdir = whT + (size_t)dir * G4 * H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bf16* row = wdir + (size_t)((2 * j + (c >> 3)) * H + my_unit) * H + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + ks * 32);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(bw[j][ks]));   // see the BPTT kernel

    // ---- fused input projection: resident W_x^T fragments (same N-tile / lane map as W_h)
    bf16x8 bx[fx ? 2 : 1][KX];
    if constexpr (fx) {
        const bf16* xdir = wxT + (size_t)dir * G4 * NIN;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bf16* row = xdir + (size_t)((2 * j + (c >> 3)) * H + my_unit) * NIN + 8 * g;
#pragma unroll
            for (int kx = 0; kx < KX; ++kx) bx[j][kx] = *reinterpret_cast<const bf16x8*>(row + kx * 32);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kx = 0; kx < KX; ++kx) asm volatile("" ::"v"(bx[j][kx]));
    }

    // ---- the epilogue item of this thread: row er, units eu..eu+3 (all 4 gates)
    const int er = tid >> 3, eu = 4 * (tid & 7);
    const int elen = seq_len[b0 + er];
    // settle the load before the loop: its first use inside the loop otherwise made
    // the waitcnt pass drain every outstanding load there, every step (vmcnt(0));
    // measured 2.74 -> 2.64 us/step forward, 3.51 -> 3.39 BPTT (the same below)
    asm volatile("" ::"v"(elen));
    float cst[4] = {0.f, 0.f, 0.f, 0.f}, hst[4] = {0.f, 0.f, 0.f, 0.f};
    float bsr[fx ? 4 : 1][4];                           // fused: the projection bias of the thread's 16 gate columns
    if constexpr (fx) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) bsr[k][e] = bias[dir * G4 + k * H + u0 + eu + e];
    }
    if (tid < PBR) s_len[tid] = seq_len[b0 + tid];
    __syncthreads();

    // fused: x_t rows of step `step` into ring slot `buf` -- 4 LDS-DMA wave instructions
    // of 2 rows x 512 B; lane l fetches logical piece (l & 31) ^ (row & 15) into slot l & 31
    const __amdgpu_buffer_rsrc_t x_rsrc = uniform_rsrc(fx ? (const void*)xin : (const void*)whT,
                                                       fx ? (int64_t)T * B * NIN * 2 : 16);
    // the x rows this lane fetches (fixed over the steps): their lengths and fixed byte parts
    int xlen[fx ? 4 : 1], xfix[fx ? 4 : 1];
    if constexpr (fx) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = 2 * (w * 4 + q) + (lane >> 5);
            xlen[q] = s_len[r];
            xfix[q] = (b0 + r) * NIN * 2 + 16 * ((lane & 31) ^ (r & 15));
        }
    }
    auto issue_x = [&](int step, int buf) {
        if constexpr (fx) {
            const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned off = step < T
                    ? (unsigned)step_time(dir, step, xlen[q]) * (unsigned)(B * NIN * 2) + (unsigned)xfix[q]
                    : 0x80000000u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    x_rsrc, (__attribute__((address_space(3))) void*)(sx + (buf * PBR + 2 * (wu * 4 + q)) * NIN), 16,
                    off, 0, 0, 0);
            }
        }
    };
    if constexpr (fx) {
        issue_x(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // gx tile loader: 32 rows x 4 gates x 4 chunks of 8 units = 512 16-B pieces, 2 per thread
    int gx_lr[2], gx_gate[2], gx_q[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        const int id = tid + 256 * v;
        gx_lr[v] = id >> 4;
        gx_gate[v] = (id >> 2) & 3;
        gx_q[v] = id & 3;
    }

    // buffer resources for the sc1 hand-off traffic
    const int64_t hx_elems = (int64_t)2 * 2 * B * H;
    auto hx_rsrc = __builtin_amdgcn_make_buffer_rsrc(hx, 0, (int)(hx_elems * 2), 0x00020000);
    constexpr bool late = LATE && KS == 16;
    // gx as one buffer (the late path's loads are single buffer instructions, so the
    // counted vmcnt wait below can rely on their number)
    const __amdgpu_buffer_rsrc_t gx_rsrc = uniform_rsrc(gx, (int64_t)T * B * 2 * G4 * 2);

    for (int s = 0; s < T; ++s) {
        pstamp(dbg, s, 0);
        // 0. the step's gx tile (independent of h): loads in flight across the wait
        //    (late: issued behind the staging DMA instead)
        u32x4 gxv[2];
        auto load_gx = [&]() {
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int lr = gx_lr[v];
                const int t = step_time(dir, s, s_len[lr]);
                const int64_t e = (((int64_t)t * B + b0 + lr) * 2 + dir) * G4 + gx_gate[v] * H + u0 + 8 * gx_q[v];
                if constexpr (late)
                    gxv[v] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(gx_rsrc, (int)(e * 2), 0, 0));
                else
                    gxv[v] = *reinterpret_cast<const u32x4*>(gx + e);
            }
        };
        if constexpr (!late) load_gx();

        floatx4 acc[2][2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // fused: gates = x_t . W_x (independent of h) -- run in the shadow of the
        // h_{s-1} staging DMA (at s = 0 there is none)
        auto x_mma = [&]() {
            if constexpr (fx) {
                const unsigned short* xs = sx + (s & 1) * PBR * NIN;
#pragma unroll
                for (int kx = 0; kx < KX; ++kx) {
                    const int sl = (4 * kx + g) ^ c;             // rows c and 16 + c share the swizzle
                    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&xs[c * NIN + 8 * sl]);
                    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&xs[(16 + c) * NIN + 8 * sl]);
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bx[j][kx], acc[0][j], 0, 0, 0);
                        acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bx[j][kx], acc[1][j], 0, 0, 0);
                    }
                }
            }
        };

        if (s > 0) {
            // 1. wait until every member of the group published h_{s-1} (flag >= s)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)s;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)s))) break;
                    poll_pause();
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_FWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            pstamp(dbg, s, 1);
            // 2. stage h_{s-1} rows (sc1 loads: the bytes were written through by other CUs)
            const int64_t hbase = ((int64_t)(((s - 1) & 1) * 2 + dir) * B + b0) * H;
            if constexpr (KS == 16) {
                // H = 512: one 1-KB row per LDS-DMA wave instruction, 8 rows per wave,
                // straight into the padded LDS rows (drained before the barrier below)
                const int wu = __builtin_amdgcn_readfirstlane(w);
                const unsigned lo = (unsigned)(lane * 16);
                if (local) {
#pragma unroll
                    for (int q = 0; q < PBR / 4; ++q) {
                        const int r = wu * (PBR / 4) + q;
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            hx_rsrc, (__attribute__((address_space(3))) void*)(sh + r * LDH), 16,
                            (unsigned)((hbase + (int64_t)r * H) * 2) + lo, 0, 0, 2);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < PBR / 4; ++q) {
                        const int r = wu * (PBR / 4) + q;
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            hx_rsrc, (__attribute__((address_space(3))) void*)(sh + r * LDH), 16,
                            (unsigned)((hbase + (int64_t)r * H) * 2) + lo, 0, 0, 16);
                    }
                }
                if constexpr (fx) {
                    asm volatile("" ::: "memory");
                    issue_x(s + 1, (s + 1) & 1);                 // next step's x rows behind the 8 DMAs
                    x_mma();                                     // while the h rows land
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                } else if constexpr (late) {
                    asm volatile("" ::: "memory");
                    load_gx();                                   // 2 loads behind the 8 DMAs
                    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            } else {
            u32x4 hv[PBR * H / 8 / 256];
#pragma unroll
            for (int v = 0; v < PBR * H / 8 / 256; ++v) {
                const int idx = tid + 256 * v;
                const int row = idx / (H / 8), kq = idx % (H / 8);
                const int off = (int)((hbase + (int64_t)row * H + 8 * kq) * 2);
                hv[v] = get16(hx_rsrc, off, local);
            }
#pragma unroll
            for (int v = 0; v < PBR * H / 8 / 256; ++v) {
                const int idx = tid + 256 * v;
                const int row = idx / (H / 8), kq = idx % (H / 8);
                *reinterpret_cast<u32x4*>(&sh[row * LDH + 8 * kq]) = hv[v];
            }
            }
        } else if constexpr (fx) {
            issue_x(1, 1);
            x_mma();
        } else if constexpr (late) {
            load_gx();
        }
        if constexpr (!late) {
#pragma unroll
            for (int v = 0; v < 2; ++v)
                *reinterpret_cast<u32x4*>(&sgx[(gx_lr[v] * 4 + gx_gate[v]) * PHU + 8 * gx_q[v]]) = gxv[v];
        }
        __syncthreads();
        pstamp(dbg, s, 2);
        if (s > 0) {
            // 3. gates += h_{s-1} . W_h
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&sh[c * LDH + ks * 32 + 8 * g]);
                bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&sh[(16 + c) * LDH + ks * 32 + 8 * g]);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[j][ks], acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[j][ks], acc[1][j], 0, 0, 0);
                }
            }
        }

        if constexpr (late && !fx) {
            // the gx tile, landed during the MFMAs (read after the barrier below; the
            // previous step's reads of sgx ended before its flag barrier)
#pragma unroll
            for (int v = 0; v < 2; ++v)
                *reinterpret_cast<u32x4*>(&sgx[(gx_lr[v] * 4 + gx_gate[v]) * PHU + 8 * gx_q[v]]) = gxv[v];
        }
        // 4. spill the gate pre-activations: lane (c, g) of wave w holds, for N-tile j,
        //    gate 2j + (c >> 3) of unit 8w + (c & 7), rows 16 mt + 4 g + r
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    sG[(16 * mt + 4 * g + r) * LDG + (2 * j + (c >> 3)) * PHU + lu] = acc[mt][j][r];
        __syncthreads();
        pstamp(dbg, s, 3);

        // 5. the cell update of (row er, units eu..eu+3), all lanes busy
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        float a4[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4 z = *reinterpret_cast<const f32x4*>(&sG[er * LDG + k * PHU + eu]);
            if constexpr (fx) {
#pragma unroll
                for (int e = 0; e < 4; ++e) a4[k][e] = z[e] + bsr[k][e];
            } else {
                typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
                const u16x4 xg = *reinterpret_cast<const u16x4*>(&sgx[(er * 4 + k) * PHU + eu]);
#pragma unroll
                for (int e = 0; e < 4; ++e) a4[k][e] = z[e] + bits_f(xg[e]);
            }
        }
        float hn[4], cp[4], hp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float ai = sig_fast(a4[0][e]);
            const float aj = tanh_fast(a4[1][e]);
            const float af = sig_fast(a4[2][e] + 1.0f);       // forget_bias = 1
            const float ao = sig_fast(a4[3][e]);
            const float cn = af * cst[e] + ai * aj;
            const float h = ao * tanh_fast(cn);
            a4[0][e] = valid ? ai : 0.f; a4[1][e] = valid ? aj : 0.f;
            a4[2][e] = valid ? af : 0.f; a4[3][e] = valid ? ao : 0.f;
            cp[e] = valid ? cst[e] : 0.f;
            hp[e] = valid ? hst[e] : 0.f;
            if (valid) { cst[e] = cn; hst[e] = (float)(bf16)h; }
            hn[e] = hst[e];                                   // published state (carried when invalid)
        }

        // 6. publish h_s (8-B sc1 stores), drain, barrier, one lane raises the flag
        {
            const int64_t obase = ((int64_t)((s & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu;
            const unsigned long long v =
                (unsigned long long)((unsigned)bf16_bits(hn[0]) | ((unsigned)bf16_bits(hn[1]) << 16)) |
                ((unsigned long long)((unsigned)bf16_bits(hn[2]) | ((unsigned)bf16_bits(hn[3]) << 16)) << 32);
            put8((gu64*)(hx + obase), v, local);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(s + 1), local);
        pstamp(dbg, s, 4);

        // 7. the layer output and the tensors saved for the backward pass
        //    (time order; they drain behind the next step)
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        {
            // padded positions (t = s >= len) get this direction's zeros: the caller need not clear out
            float ov[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = valid ? hn[e] : 0.f;
            st4(out + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu, ov);
        }
        st4(hprev_t + tb * H + u0 + eu, hp);
        st4(cprev_t + tb * H + u0 + eu, cp);
#pragma unroll
        for (int k = 0; k < 4; ++k) st4(acts_t + tb * G4 + k * H + u0 + eu, a4[k]);
        pstamp(dbg, s, 5);
    }
}

// ------------------------------------------- forward, 16-row / 64-unit members
// The forward loop above stages, per member and step, the group's h_{s-1} rows
// of its 32 batch rows (32 KB at H = 512) and runs 64 MFMAs per wave on 4 waves.
// Here a member owns 16 batch rows and 64 hidden units, as the 16-row BPTT
// (groups = 2 x B/16 of 8 members: the same B workgroups, one per CU at B =
// 256): 16 KB staged per step (two 1-KB row DMAs per wave into padded LDS rows),
// 8 waves, wave w owning units 8w .. 8w+7 of all 4 gates = two 16-column N-tiles
// over the full K = H with its W_h^T slice resident (2 x 16 k-steps x 4 VGPRs =
// 128), 32 MFMAs per wave per step on the one 16-row M-tile. Cell: 2 units of one
// row per thread, the step's gx read straight into registers behind the staging
// DMA (4 buffer loads). Hand-off form, census, counting flags and the saved
// tensors as the kernel above.
constexpr int R16_ROWS = 16, R16_UNITS = 64;

__global__ void __launch_bounds__(512, 1)
lstm_fwd_r16_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whT, bf16* __restrict__ hx,
                    const int* __restrict__ seq_len, int T, int B, bf16* __restrict__ out, bf16* __restrict__ hprev_t,
                    float* __restrict__ cprev_t, bf16* __restrict__ acts_t, unsigned* __restrict__ flags,
                    unsigned* __restrict__ err, unsigned spin_limit) {
    constexpr int KS = 16, H = 512, G4 = 4 * H;
    constexpr int RB = R16_ROWS, UM = R16_UNITS;
    constexpr int NU = H / UM;                          // members per group (8)
    constexpr int LDH = H + 8;                          // padded LDS row (bf16 elements)
    constexpr int LDG = 4 * UM + 4;                     // padded gate row (floats)
    __shared__ __attribute__((aligned(16))) unsigned short sh[RB * LDH];
    __shared__ __attribute__((aligned(16))) float sG[RB * LDG];             // [row][gate][unit]

    int group, member;
    persistent_role(2 * (B / RB), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * UM, b0 = bs * RB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int lu = 8 * w + (c & 7);                     // the unit (within the slice) of this lane's columns
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);

    // resident B fragments: N-tile j holds gates 2j + (c >> 3) of unit u0 + lu
    bf16x8 bw[2][KS];
    const bf16* wdir = whT + (size_t)dir * G4 * H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bf16* row = wdir + (size_t)((2 * j + (c >> 3)) * H + u0 + lu) * H + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + ks * 32);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(bw[j][ks]));   // settled before the loop

    // the cell item: row er, units eu, eu + 1 (all 4 gates)
    const int er = tid >> 5, eu = 2 * (tid & 31);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));
    float cst[2] = {0.f, 0.f}, hst[2] = {0.f, 0.f};

    const int64_t hx_elems = (int64_t)2 * 2 * B * H;
    auto hx_rsrc = __builtin_amdgcn_make_buffer_rsrc(hx, 0, (int)(hx_elems * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t gx_rsrc = uniform_rsrc(gx, (int64_t)T * B * 2 * G4 * 2);
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const unsigned lo16 = (unsigned)(lane * 16);

    for (int s = 0; s < T; ++s) {
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        unsigned lg[4];
        auto load_gx = [&]() {                           // 4 buffer loads: 2 units x 4 gates
#pragma unroll
            for (int k = 0; k < 4; ++k)
                lg[k] = __builtin_amdgcn_raw_buffer_load_b32(gx_rsrc, (int)((tb * G4 + k * H + u0 + eu) * 2), 0, 0);
        };
        floatx4 acc[2];
        acc[0] = acc[1] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (s > 0) {
            // 1. wait until every member of the group published h_{s-1} (flag >= s)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)s;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)s))) break;
                    poll_pause();
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_FWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            // 2. stage the group's 16 h_{s-1} rows: rows 2w, 2w + 1, one 1-KB LDS-DMA each
            const int64_t hbase = ((int64_t)(((s - 1) & 1) * 2 + dir) * B + b0) * H;
            if (local) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = 2 * wu + q;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        hx_rsrc, (__attribute__((address_space(3))) void*)(sh + r * LDH), 16,
                        (unsigned)((hbase + (int64_t)r * H) * 2) + lo16, 0, 0, 2);      // nt
                }
            } else {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = 2 * wu + q;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        hx_rsrc, (__attribute__((address_space(3))) void*)(sh + r * LDH), 16,
                        (unsigned)((hbase + (int64_t)r * H) * 2) + lo16, 0, 0, 16);     // sc1
                }
            }
            asm volatile("" ::: "memory");
            load_gx();                                   // 4 loads behind the 2 DMAs
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            __syncthreads();
            // 3. gates += h_{s-1} . W_h over the full K
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sh[c * LDH + ks * 32 + 8 * g]);
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[j][ks], acc[j], 0, 0, 0);
            }
        } else {
            load_gx();
        }
        // 4. spill the gate pre-activations: lane (c, g) holds rows 4 g + r of N-tile j,
        //    gate 2j + (c >> 3) of unit lu
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) sG[(4 * g + r) * LDG + (2 * j + (c >> 3)) * UM + lu] = acc[j][r];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // gx landed
        __syncthreads();

        // 5. the cell update of (row er, units eu, eu + 1)
        float a4[4][2];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x2_t z = *reinterpret_cast<const f32x2_t*>(&sG[er * LDG + k * UM + eu]);
            a4[k][0] = z[0] + __uint_as_float(lg[k] << 16);
            a4[k][1] = z[1] + __uint_as_float(lg[k] & 0xffff0000u);
        }
        float hn[2], cp[2], hp[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float ai = sig_fast(a4[0][e]);
            const float aj = tanh_fast(a4[1][e]);
            const float af = sig_fast(a4[2][e] + 1.0f);       // forget_bias = 1
            const float ao = sig_fast(a4[3][e]);
            const float cn = af * cst[e] + ai * aj;
            const float h = ao * tanh_fast(cn);
            a4[0][e] = valid ? ai : 0.f; a4[1][e] = valid ? aj : 0.f;
            a4[2][e] = valid ? af : 0.f; a4[3][e] = valid ? ao : 0.f;
            cp[e] = valid ? cst[e] : 0.f;
            hp[e] = valid ? hst[e] : 0.f;
            if (valid) { cst[e] = cn; hst[e] = (float)(bf16)h; }
            hn[e] = hst[e];                                   // published state (carried when invalid)
        }
        auto pack2 = [](float x0, float x1) {
            return (unsigned)bf16_bits(x0) | ((unsigned)bf16_bits(x1) << 16);
        };

        // 6. publish h_s (4-B stores), drain, barrier, one lane raises the flag
        {
            gu32* ph = (gu32*)(hx + ((int64_t)((s & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu);
            const unsigned v = pack2(hn[0], hn[1]);
            if (local) *ph = v;
            else __hip_atomic_store(ph, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(s + 1), local);

        // 7. the layer output (zeros past the length) and the tensors saved for the
        //    backward pass (time order; they drain behind the next step)
        *reinterpret_cast<unsigned*>(out + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu) =
            valid ? pack2(hn[0], hn[1]) : 0u;
        *reinterpret_cast<unsigned*>(hprev_t + tb * H + u0 + eu) = pack2(hp[0], hp[1]);
        *reinterpret_cast<f32x2_t*>(cprev_t + tb * H + u0 + eu) = f32x2_t{cp[0], cp[1]};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            *reinterpret_cast<unsigned*>(acts_t + tb * G4 + k * H + u0 + eu) = pack2(a4[k][0], a4[k][1]);
    }
}

// ---------------------------------------------------------------- backward
// BPTT of the same layer as ONE persistent launch (groups, members and the
// hand-off form of the forward). Member (group, unit slice) owns units
// u0..u0+31 of one direction for 32 batch rows. Reverse step i (s = T-1-i):
//   dh_rec[rows, own units] = dz_{i-1}[rows, 4H] . W_h[own units, 4H]^T
// with K = 4H split over the 4 waves by gate (wave w: the H columns of gate
// w; its W_h slice [32 units x H] stays in VGPRs as B fragments), the A
// operand being the group's published dz rows, which each wave stages for its
// own k-range in LDS with full-row sc1 loads (each byte once per workgroup). The 4 partial products meet
// in LDS; the cell's gradient (dc kept in registers across steps) gives dz
// for (row, 4 units, 4 gates) per thread, published (sc1) for step i+1 and
// stored in time order for the weight-gradient GEMMs.
// LATE (H = 512): the epilogue operands are loaded AFTER the hand-off poll,
// behind the dz LDS-DMA (single buffer loads; counted vmcnt), so neither the
// poll nor the staging wait also waits for their HBM latency.
template <int KS, bool LATE = false>
__global__ void __launch_bounds__(256, 1)
lstm_bwd_persistent_kernel(const bf16* __restrict__ wh, bf16* __restrict__ dzx, const int* __restrict__ seq_len,
                           int T, int B, const bf16* __restrict__ dout, const float* __restrict__ cprev_t,
                           const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t, unsigned* __restrict__ flags,
                           unsigned* __restrict__ err, unsigned spin_limit, long long* __restrict__ dbg,
                           float* __restrict__ bpart) {
    constexpr int H = KS * 32;
    constexpr int G4 = 4 * H;
    constexpr int NU = H / PHU;
    constexpr int LDP = PHU + 4;                        // padded partial row (floats)
    constexpr int LDA = H + 8;                          // padded staged dz row (bf16)
    static_assert(NU <= 64 && (H == 256 || H == 512), "one poll lane per member; whole-row wave loads");
    __shared__ __attribute__((aligned(16))) float sP[4 * PBR * LDP];   // [wave][row][unit]
    __shared__ __attribute__((aligned(16))) unsigned short sA[4 * PBR * LDA];   // [wave][row][k of gate w]

    int group, member;
    persistent_role(2 * (B / PBR), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);
    if (dbg && threadIdx.x == 0) dbg[(int64_t)blockIdx.x * 8 + 7] = local ? 1 : 0;     // diagnostics: hand-off form

    // resident B fragments: N-tile j = units u0 + 16 j + c; k = w H + 32 ks + 8 g
    bf16x8 bw[2][KS];
    const bf16* wdir = wh + (size_t)dir * H * G4;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bf16* row = wdir + (size_t)(u0 + 16 * j + c) * G4 + w * H + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + ks * 32);
    }
    // the resident fragments are in before the loop: an empty asm that reads every
    // fragment makes the waitcnt pass wait for them HERE, after which it knows they
    // landed -- instead of re-waiting in every step for loads it still counts as
    // outstanding (which made the tile-0 MFMAs wait for the tile-1 rows' DMA)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(bw[j][ks]));

    const int er = tid >> 3, eu = 4 * (tid & 7);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));                       // settled before the loop (see the forward)
    float dcs[4] = {0.f, 0.f, 0.f, 0.f};
    float bsum[4][4] = {};                              // the bias gradient: sum of dz over this row's steps
    const int64_t zx_elems = (int64_t)2 * 2 * B * G4;
    auto zx_rsrc = __builtin_amdgcn_make_buffer_rsrc(dzx, 0, (int)(zx_elems * 2), 0x00020000);
    constexpr bool late = LATE && KS == 16;
    const __amdgpu_buffer_rsrc_t act_rsrc = uniform_rsrc(acts_t, (int64_t)T * B * 2 * G4 * 2);
    const __amdgpu_buffer_rsrc_t cp_rsrc = uniform_rsrc(cprev_t, (int64_t)T * B * 2 * H * 4);
    const __amdgpu_buffer_rsrc_t do_rsrc = uniform_rsrc(dout, (int64_t)T * B * 2 * H * 2);

    for (int i = 0; i < T; ++i) {
        const int s = T - 1 - i;
        pstamp(dbg, i, 0);
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        // 0. epilogue operands (independent of the recurrence) in flight first
        //    (late: behind the staging DMA, as exactly 6 buffer loads)
        float pa[4][4], pcp[4], pdo[4];
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        u32x2 la[4], ldo;
        u32x4 lcp;
        auto load_late = [&]() {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                la[k] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                    act_rsrc, (int)((tb * G4 + k * H + u0 + eu) * 2), 0, 0));
            lcp = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(cp_rsrc, (int)((tb * H + u0 + eu) * 4), 0, 0));
            ldo = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                do_rsrc, (int)((((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu) * 2), 0, 0));
        };
        if constexpr (!late) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ld4(pa[k], acts_t + tb * G4 + k * H + u0 + eu);
            ld4(pcp, cprev_t + tb * H + u0 + eu);
            ld4(pdo, dout + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu);
        }

        floatx4 acc[2][2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (i > 0) {
            // 1. wait until every member of the group published dz_{i-1} (flag >= i)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)i;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)i))) break;
                    poll_pause();
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_BWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            pstamp(dbg, i, 1);
            // 2. wave w stages the 32 dz rows of gate w's k-range (32 x H bf16) in
            //    its own LDS region: full rows per wave instruction (16 B per lane,
            //    sc1), 8 rows per batch, two batches in flight; M-tile mt's MFMAs
            //    start once its 16 rows are in (wave-local: no workgroup barrier)
            const int64_t rbase = ((int64_t)(((i - 1) & 1) * 2 + dir) * B + b0) * G4 + w * H;
            unsigned short* sa = sA + w * PBR * LDA;
            constexpr int LPR = H / 8, RPI = 64 / LPR, NI = 8 / RPI;     // lanes per row, rows per instruction
            const int lrow = lane / LPR, lcol = 8 * (lane % LPR);
            auto load_rows = [&](u32x4 (&v)[NI], int r0) {
#pragma unroll
                for (int q = 0; q < NI; ++q) {
                    const int off = (int)((rbase + (int64_t)(r0 + q * RPI + lrow) * G4 + lcol) * 2);
                    v[q] = get16(zx_rsrc, off, local);
                }
            };
            auto store_rows = [&](const u32x4 (&v)[NI], int r0) {
#pragma unroll
                for (int q = 0; q < NI; ++q)
                    *reinterpret_cast<u32x4*>(&sa[(r0 + q * RPI + lrow) * LDA + lcol]) = v[q];
            };
            auto mma_tile = [&](int mt) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const bf16x8 af = *reinterpret_cast<const bf16x8*>(&sa[(16 * mt + c) * LDA + ks * 32 + 8 * g]);
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][ks], acc[mt][j], 0, 0, 0);
                }
            };
            if constexpr (KS == 16) {
                // H = 512: a dz row of the wave's k-range is 1 KB = one LDS-DMA wave
                // instruction (16 B per lane) straight into its padded LDS row -- all
                // 32 rows in flight at once, no VGPR round trip; M-tile 0 multiplies
                // as soon as its 16 rows have landed (counted vmcnt: everything issued
                // before the DMAs is older, so vmcnt(16) covers rows 0-15)
                const int wu = __builtin_amdgcn_readfirstlane(w);
                unsigned short* sau = sA + wu * PBR * LDA;
                const int64_t rb = ((int64_t)(((i - 1) & 1) * 2 + dir) * B + b0) * G4 + wu * H;
                const unsigned lo = (unsigned)(lane * 16);
                if (local) {
#pragma unroll
                    for (int r = 0; r < PBR; ++r)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            zx_rsrc, (__attribute__((address_space(3))) void*)(sau + r * LDA), 16,
                            (unsigned)((rb + (int64_t)r * G4) * 2) + lo, 0, 0, 2);      // nt
                } else {
#pragma unroll
                    for (int r = 0; r < PBR; ++r)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            zx_rsrc, (__attribute__((address_space(3))) void*)(sau + r * LDA), 16,
                            (unsigned)((rb + (int64_t)r * G4) * 2) + lo, 0, 0, 16);     // sc1
                }
                if constexpr (late) {
                    asm volatile("" ::: "memory");
                    load_late();                                 // 6 loads behind the 32 DMAs
                    asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
                    mma_tile(0);
                    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                    mma_tile(1);
                } else {
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    mma_tile(0);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    mma_tile(1);
                }
            } else {
                u32x4 v0[NI], v1[NI];
                load_rows(v0, 0);
                load_rows(v1, 8);
                store_rows(v0, 0);
                load_rows(v0, 16);
                store_rows(v1, 8);
                load_rows(v1, 24);
                mma_tile(0);
                store_rows(v0, 16);
                store_rows(v1, 24);
                mma_tile(1);
            }
        } else if constexpr (late) {
            load_late();
        }
        if constexpr (late) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pa[k][0] = __uint_as_float(la[k][0] << 16); pa[k][1] = __uint_as_float(la[k][0] & 0xffff0000u);
                pa[k][2] = __uint_as_float(la[k][1] << 16); pa[k][3] = __uint_as_float(la[k][1] & 0xffff0000u);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) pcp[e] = __uint_as_float(lcp[e]);
            pdo[0] = __uint_as_float(ldo[0] << 16); pdo[1] = __uint_as_float(ldo[0] & 0xffff0000u);
            pdo[2] = __uint_as_float(ldo[1] << 16); pdo[3] = __uint_as_float(ldo[1] & 0xffff0000u);
        }
        // 3. the four partial products (one per gate's k-range) meet in LDS
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    sP[(w * PBR + 16 * mt + 4 * g + r) * LDP + 16 * j + c] = acc[mt][j][r];
        __syncthreads();
        pstamp(dbg, i, 2);

        // 4. the cell's gradient for (row er, units eu..eu+3)
        float dz[4][4];
        {
            f32x4 p[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) p[q] = *reinterpret_cast<const f32x4*>(&sP[(q * PBR + er) * LDP + eu]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float dh = ((p[0][e] + p[1][e]) + (p[2][e] + p[3][e])) + pdo[e];
                const float ai = pa[0][e], aj = pa[1][e], af = pa[2][e], ao = pa[3][e];
                const float cp = pcp[e];
                const float cc = af * cp + ai * aj;
                const float tc = tanh_fast(cc);
                const float dc = dcs[e] + dh * ao * (1.f - tc * tc);
                dz[3][e] = valid ? dh * tc * ao * (1.f - ao) : 0.f;
                dz[0][e] = valid ? dc * aj * ai * (1.f - ai) : 0.f;
                dz[1][e] = valid ? dc * ai * (1.f - aj * aj) : 0.f;
                dz[2][e] = valid ? dc * cp * af * (1.f - af) : 0.f;
                dcs[e] = valid ? dc * af : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) bsum[k][e] += dz[k][e];
        }
        // 5. publish dz (8-B sc1 stores, one per gate), drain, barrier, one lane raises the flag
        {
            const int64_t zbase = ((int64_t)((i & 1) * 2 + dir) * B + b0 + er) * G4 + u0 + eu;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const unsigned long long v =
                    (unsigned long long)((unsigned)bf16_bits(dz[k][0]) | ((unsigned)bf16_bits(dz[k][1]) << 16)) |
                    ((unsigned long long)((unsigned)bf16_bits(dz[k][2]) | ((unsigned)bf16_bits(dz[k][3]) << 16)) << 32);
                put8((gu64*)(dzx + zbase + k * H), v, local);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(i + 1), local);
        pstamp(dbg, i, 3);
        // 6. time-order copy for the weight-gradient GEMMs (drains behind the next step)
#pragma unroll
        for (int k = 0; k < 4; ++k) st4(dG_t + tb * G4 + k * H + u0 + eu, dz[k]);
        pstamp(dbg, i, 4);
    }
    bias_partials<4>(bpart, bsum, reinterpret_cast<float*>(sA), (bs * 2 + dir) * G4, H, u0);
}

// ------------------------------------------ backward, 16-row / 64-unit members
// The gather BPTT above stages, per member and step, the group's dz rows of its
// 32 batch rows: 32 x 4H bf16 = 128 KB per CU per step at H = 512 -- the step's
// floor (~100 GB/s per CU from L2 into LDS, MI355X_MICROARCH.md handoff-payload).
// That volume is rows x 4H whatever the unit slice, so here a member owns 16
// batch rows and 64 hidden units (groups = 2 x B/16 of 8 members: the same B
// workgroups, one per CU at B = 256) and stages 64 KB. 8 waves: wave w takes
// gate q = w >> 1, k-half kh = w & 1 (256 of the gate's 512 columns): its W_h
// slice [64 units][256 k] is resident (4 N-tiles x 8 k-steps = 128 VGPRs), it
// stages ITS 16 dz rows x 256 columns (8 KB, 8 LDS-DMA wave instructions of two
// 512-B rows, unpadded, 16-B pieces XOR-swizzled by row on the global side so a
// fragment read of 16 rows hits 16 distinct bank groups) and multiplies them
// wave-locally (32 MFMAs); the eight K-slice partials meet in LDS in a fixed
// order. Cell: 2 units of one row per thread. Hand-off form, census, counting
// flags, late epilogue loads and bias partials as the gather kernel.
__global__ void __launch_bounds__(512, 1)
lstm_bwd_r16_kernel(const bf16* __restrict__ wh, bf16* __restrict__ dzx, const int* __restrict__ seq_len, int T,
                    int B, const bf16* __restrict__ dout, const float* __restrict__ cprev_t,
                    const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t, unsigned* __restrict__ flags,
                    unsigned* __restrict__ err, unsigned spin_limit, float* __restrict__ bpart) {
    constexpr int H = 512, G4 = 4 * H;
    constexpr int RB = R16_ROWS, UM = R16_UNITS;
    constexpr int NU = H / UM;                          // members per group (8)
    constexpr int KW = 256;                             // k columns per wave
    constexpr int KSW = KW / 32;                        // k-steps per wave (8)
    constexpr int LDP = UM + 4;                         // partial row pitch (floats)
    __shared__ __attribute__((aligned(16))) unsigned short sA[8 * RB * KW];   // [wave][row][swizzled 16-B slots]
    __shared__ __attribute__((aligned(16))) float sP[8 * RB * LDP];           // [wave][row][unit]

    int group, member;
    persistent_role(2 * (B / RB), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * UM, b0 = bs * RB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int kbase = (w >> 1) * H + (w & 1) * KW;      // this wave's dz / W_h columns
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);

    // resident B fragments: N-tile j = units u0 + 16 j + c; k = kbase + 32 ks + 8 g
    bf16x8 bw[4][KSW];
    const bf16* wdir = wh + (size_t)dir * H * G4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bf16* row = wdir + (size_t)(u0 + 16 * j + c) * G4 + kbase + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KSW; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + ks * 32);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < KSW; ++ks) asm volatile("" ::"v"(bw[j][ks]));   // settled before the loop

    // the cell item: row er, units eu, eu + 1 (all 4 gates)
    const int er = tid >> 5, eu = 2 * (tid & 31);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));
    float dcs[2] = {0.f, 0.f};
    float bsum[4][2] = {};
    const int64_t zx_elems = (int64_t)2 * 2 * B * G4;
    auto zx_rsrc = __builtin_amdgcn_make_buffer_rsrc(dzx, 0, (int)(zx_elems * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t act_rsrc = uniform_rsrc(acts_t, (int64_t)T * B * 2 * G4 * 2);
    const __amdgpu_buffer_rsrc_t cp_rsrc = uniform_rsrc(cprev_t, (int64_t)T * B * 2 * H * 4);
    const __amdgpu_buffer_rsrc_t do_rsrc = uniform_rsrc(dout, (int64_t)T * B * 2 * H * 2);
    // DMA lane geometry (fixed over the steps): instruction d covers rows 2d, 2d + 1;
    // lane l writes row 2d + (l >> 5), slot l & 31, fetching the global 16-B piece
    // (l & 31) ^ row of that row's wave columns
    const int wu = __builtin_amdgcn_readfirstlane(w);
    unsigned short* sa = sA + wu * RB * KW;
    unsigned dma_off[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const int r = 2 * d + (lane >> 5);
        dma_off[d] = (unsigned)((r * G4 + kbase + 8 * ((lane & 31) ^ (r & 15))) * 2);
    }

    for (int i = 0; i < T; ++i) {
        const int s = T - 1 - i;
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        unsigned la[4], ldo;
        u32x2 lcp;
        auto load_late = [&]() {                        // 6 buffer loads
#pragma unroll
            for (int k = 0; k < 4; ++k)
                la[k] = __builtin_amdgcn_raw_buffer_load_b32(act_rsrc, (int)((tb * G4 + k * H + u0 + eu) * 2), 0, 0);
            lcp = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(cp_rsrc, (int)((tb * H + u0 + eu) * 4), 0, 0));
            ldo = __builtin_amdgcn_raw_buffer_load_b32(
                do_rsrc, (int)((((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu) * 2), 0, 0);
        };
        floatx4 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (i > 0) {
            // 1. wait until every member of the group published dz_{i-1} (flag >= i)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)i;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)i))) break;
                    poll_pause();
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_BWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            // 2. this wave's 16 rows x 256 columns of dz_{i-1}, wave-local (8 LDS-DMA)
            const unsigned rb = (unsigned)(((int64_t)(((i - 1) & 1) * 2 + dir) * B + b0) * G4 * 2);
            if (local) {
#pragma unroll
                for (int d = 0; d < 8; ++d)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        zx_rsrc, (__attribute__((address_space(3))) void*)(sa + d * 2 * KW), 16, rb + dma_off[d], 0, 0, 2);
            } else {
#pragma unroll
                for (int d = 0; d < 8; ++d)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        zx_rsrc, (__attribute__((address_space(3))) void*)(sa + d * 2 * KW), 16, rb + dma_off[d], 0, 0, 16);
            }
            asm volatile("" ::: "memory");
            load_late();                                 // 6 loads behind the 8 DMAs
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            // 3. dh partial of this wave's K slice: [16 rows] x [64 units]
#pragma unroll
            for (int ks = 0; ks < KSW; ++ks) {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(&sa[c * KW + 8 * ((4 * ks + g) ^ c)]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][ks], acc[j], 0, 0, 0);
            }
        } else {
            load_late();
        }
        // 4. the eight partials meet in LDS: lane (c, g) holds rows 4 g + r of units 16 j + c
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) sP[(w * RB + 4 * g + r) * LDP + 16 * j + c] = acc[j][r];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the epilogue operands landed
        __syncthreads();
        float pa[4][2], pcp[2], pdo[2];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pa[k][0] = __uint_as_float(la[k] << 16);
            pa[k][1] = __uint_as_float(la[k] & 0xffff0000u);
        }
        pcp[0] = __uint_as_float(lcp[0]);
        pcp[1] = __uint_as_float(lcp[1]);
        pdo[0] = __uint_as_float(ldo << 16);
        pdo[1] = __uint_as_float(ldo & 0xffff0000u);

        // 5. the cell's gradient for (row er, units eu, eu + 1)
        float dz[4][2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float p[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) p[q] = sP[(q * RB + er) * LDP + eu + e];
            const float dh = (((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]))) + pdo[e];
            const float ai = pa[0][e], aj = pa[1][e], af = pa[2][e], ao = pa[3][e];
            const float cp = pcp[e];
            const float cc = af * cp + ai * aj;
            const float tc = tanh_fast(cc);
            const float dc = dcs[e] + dh * ao * (1.f - tc * tc);
            dz[3][e] = valid ? dh * tc * ao * (1.f - ao) : 0.f;
            dz[0][e] = valid ? dc * aj * ai * (1.f - ai) : 0.f;
            dz[1][e] = valid ? dc * ai * (1.f - aj * aj) : 0.f;
            dz[2][e] = valid ? dc * cp * af * (1.f - af) : 0.f;
            dcs[e] = valid ? dc * af : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bsum[k][0] += dz[k][0];
            bsum[k][1] += dz[k][1];
        }
        // 6. publish dz (4-B stores, one per gate), drain, barrier, one lane raises the flag
        unsigned zv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) zv[k] = (unsigned)bf16_bits(dz[k][0]) | ((unsigned)bf16_bits(dz[k][1]) << 16);
        {
            const int64_t zbase = ((int64_t)((i & 1) * 2 + dir) * B + b0 + er) * G4 + u0 + eu;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                gu32* pz = (gu32*)(dzx + zbase + k * H);
                if (local) *pz = zv[k];
                else __hip_atomic_store(pz, zv[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(i + 1), local);
        // 7. time-order copy for the weight-gradient GEMMs (drains behind the next step)
#pragma unroll
        for (int k = 0; k < 4; ++k) *reinterpret_cast<unsigned*>(dG_t + tb * G4 + k * H + u0 + eu) = zv[k];
    }
    // bias partials of this 16-row slice: the 16 rows of every (gate, unit) meet in LDS
    if (bpart) {
        __syncthreads();
        float* red = sP;                                 // [row][4 gates x 64 units], free after the loop
        constexpr int LDR = 4 * UM + 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            red[er * LDR + k * UM + eu] = bsum[k][0];
            red[er * LDR + k * UM + eu + 1] = bsum[k][1];
        }
        __syncthreads();
        if (tid < 4 * UM) {
            float sum = 0.f;
            for (int r = 0; r < RB; ++r) sum += red[r * LDR + tid];
            bpart[(int64_t)(bs * 2 + dir) * G4 + (tid / UM) * H + u0 + (tid % UM)] = sum;
        }
    }
}

// ---------------------------------------------------- backward, K-split form
// The same BPTT with the recurrent product split over the members by K
// instead of by output unit (opt-in, OCRK_LSTM_BWD_KSPLIT=1; the default is the
// gather form above). Member m computes, from ITS OWN dz (the 4 gates x 32
// units it just produced, never exchanged), the partial product
//   P_m[32 rows, H units] = dz_m[32 rows, 128 gate cols] . W_h[H units, own 128 gate cols]^T
// (K = 128: one 32-deep k-step per gate; wave w: units w H/4 .. +H/4, its W_h
// slice resident in VGPRs as B fragments), and publishes it as NU f32 blocks
// of 32 rows x 32 units, block m' for the member that owns those units. A
// member's dh_rec is then the fixed-order sum of the NU blocks addressed to it
// (one 16-B load per block per thread, all in flight at once, summed in
// registers -- deterministic). Per step and member this moves 64 KB in and
// 64 KB out (f32) instead of gathering every member's dz rows (128 KB bf16 in),
// keeps no staged rows in LDS (8.5 KB instead of 149 KB), and takes dz out of
// the exchange, so dh is formed from f32 partial sums of the UNROUNDED-in-
// exchange products (dz enters the MFMA in bf16 as before).
// Thread mapping of the cell's gradient = the MFMA output layout: wave w
// handles M-tile w >> 1 and the 16-unit half w & 1 of the member's units;
// lane (c, g) holds rows 16 (w >> 1) + 4 g + r (r = 0..3) of unit 16 (w & 1) + c.
template <int KS, bool PB16>
__global__ void __launch_bounds__(256, 1)
lstm_bwd_ksplit_kernel(const bf16* __restrict__ wh, void* __restrict__ px, const int* __restrict__ seq_len, int T,
                       int B, const bf16* __restrict__ dout, const float* __restrict__ cprev_t,
                       const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t, unsigned* __restrict__ flags,
                       unsigned* __restrict__ err, unsigned spin_limit, long long* __restrict__ dbg,
                       float* __restrict__ bpart) {
    constexpr int H = KS * 32;
    constexpr int G4 = 4 * H;
    constexpr int NU = H / PHU;                          // members per group
    constexpr int NT = H / 64;                           // 16-unit N-tiles per wave (H/4 units)
    constexpr int LDA = 4 * PHU + 8;                     // padded dz row: 128 gate cols + 8 (bf16)
    constexpr int BLK = PBR * PHU;                       // elements per (dst, src) block
    constexpr int EB = PB16 ? 2 : 4;                     // bytes per exchanged element
    static_assert(NU <= 64 && (H == 256 || H == 512), "one poll lane per member");
    __shared__ __attribute__((aligned(16))) unsigned short sA[PBR * LDA];
    // the step's epilogue operands, staged row-wise (vector loads) and read per element
    __shared__ __attribute__((aligned(16))) unsigned short sAct[PBR * LDA];      // [row][gate][unit] bf16
    __shared__ __attribute__((aligned(16))) float sCp[PBR * (PHU + 4)];           // [row][unit]
    __shared__ __attribute__((aligned(16))) float sDo[PBR * (PHU + 4)];
    __shared__ int s_len[PBR];

    int group, member;
    const int ngroups = 2 * (B / PBR);
    persistent_role(ngroups, NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);
    if (dbg && threadIdx.x == 0) dbg[(int64_t)blockIdx.x * 8 + 7] = local ? 1 : 0;

    // resident B fragments: bw[nt][k] = W_h[unit w H/4 + 16 nt + c][k H + u0 + 8 g .. + 7]
    bf16x8 bw[NT][4];
    {
        const bf16* wdir = wh + (size_t)dir * H * G4;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bw[nt][k] = *reinterpret_cast<const bf16x8*>(
                    wdir + (size_t)(w * (H / 4) + 16 * nt + c) * G4 + k * H + u0 + 8 * g);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("" ::"v"(bw[nt][k]));     // see the gather BPTT
    }
    if (tid < PBR) s_len[tid] = seq_len[b0 + tid];
    __syncthreads();

    const int emt = w >> 1, entl = w & 1;
    const int ul = 16 * entl + c;                        // the unit (in the slice) of this thread's elements
    const int rb = 16 * emt + 4 * g;                     // its 4 rows rb .. rb + 3
    int len[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) len[r] = s_len[rb + r];
    // row-wise loader item of the epilogue operands: row er, units eu .. eu + 3
    const int er = tid >> 3, eu = 4 * (tid & 7);
    const int elen = s_len[er];
    float dcs[4] = {0.f, 0.f, 0.f, 0.f};
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};               // the bias gradient: dz of (this unit, gate k), own rows
    // exchange X[parity][group][dst][src][BLK]; a block's element order is the MFMA
    // output order [mt][n-tile half][lane][r], so producer and consumer lanes move
    // 4 contiguous elements each
    const int64_t par_stride = (int64_t)ngroups * NU * NU * BLK;
    auto x_rsrc = __builtin_amdgcn_make_buffer_rsrc(px, 0, (int)(2 * par_stride * EB), 0x00020000);
    const int my_off = ((emt * 2 + entl) * 64 + lane) * 4;          // elements, inside a block

    for (int i = 0; i < T; ++i) {
        const int s = T - 1 - i;
        pstamp(dbg, i, 0);
        // 0. epilogue operands (independent of the recurrence): vector loads of row er
        {
            const int t = step_time(dir, s, elen);
            const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            u32x2 av[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) av[k] = *reinterpret_cast<const u32x2*>(acts_t + tb * G4 + k * H + u0 + eu);
            const f32x4 cv = *reinterpret_cast<const f32x4*>(cprev_t + tb * H + u0 + eu);
            const u32x2 dv = *reinterpret_cast<const u32x2*>(dout + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu);
#pragma unroll
            for (int k = 0; k < 4; ++k) *reinterpret_cast<u32x2*>(&sAct[er * LDA + k * PHU + eu]) = av[k];
            *reinterpret_cast<f32x4*>(&sCp[er * (PHU + 4) + eu]) = cv;
            f32x4 dvf;
            dvf[0] = __uint_as_float(dv[0] << 16); dvf[1] = __uint_as_float(dv[0] & 0xffff0000u);
            dvf[2] = __uint_as_float(dv[1] << 16); dvf[3] = __uint_as_float(dv[1] & 0xffff0000u);
            *reinterpret_cast<f32x4*>(&sDo[er * (PHU + 4) + eu]) = dvf;
        }
        float dh[4] = {0.f, 0.f, 0.f, 0.f};
        if (i > 0) {
            // 1. every member published its partial products of step i-1 (flag >= i)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)i;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)i))) break;
                    poll_pause();
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_BWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            pstamp(dbg, i, 1);
            // 2. dh_rec = sum over the NU source members of their block for this member (fixed order)
            const int64_t boff = ((int64_t)((i - 1) & 1) * par_stride +
                                  ((int64_t)group * NU + member) * NU * BLK + my_off) * EB;
            if constexpr (PB16) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                u32x2 pv[NU];
#pragma unroll
                for (int src = 0; src < NU; ++src)
                    pv[src] = local ? __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(x_rsrc, (int)(boff + (int64_t)src * BLK * EB), 0, 2))
                                    : __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(x_rsrc, (int)(boff + (int64_t)src * BLK * EB), 0, 16));
#pragma unroll
                for (int src = 0; src < NU; ++src) {
                    dh[0] += __uint_as_float(pv[src][0] << 16); dh[1] += __uint_as_float(pv[src][0] & 0xffff0000u);
                    dh[2] += __uint_as_float(pv[src][1] << 16); dh[3] += __uint_as_float(pv[src][1] & 0xffff0000u);
                }
            } else {
                u32x4 pv[NU];
#pragma unroll
                for (int src = 0; src < NU; ++src) pv[src] = get16(x_rsrc, (int)(boff + (int64_t)src * BLK * EB), local);
#pragma unroll
                for (int src = 0; src < NU; ++src)
#pragma unroll
                    for (int r = 0; r < 4; ++r) dh[r] += __uint_as_float(pv[src][r]);
            }
        } else {
            __syncthreads();                                 // the staged epilogue operands
        }
        // 3. the cell's gradient for (rows rb..rb+3, unit ul); dz to LDS as the MFMA A operand
        float dz[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = rb + r;
            const bool valid = s < len[r];
            const float dhr = dh[r] + sDo[row * (PHU + 4) + ul];
            const float ai = bits_f(sAct[row * LDA + 0 * PHU + ul]), aj = bits_f(sAct[row * LDA + 1 * PHU + ul]);
            const float af = bits_f(sAct[row * LDA + 2 * PHU + ul]), ao = bits_f(sAct[row * LDA + 3 * PHU + ul]);
            const float cp = sCp[row * (PHU + 4) + ul];
            const float cc = af * cp + ai * aj;
            const float tc = tanh_fast(cc);
            const float dc = dcs[r] + dhr * ao * (1.f - tc * tc);
            dz[3][r] = valid ? dhr * tc * ao * (1.f - ao) : 0.f;
            dz[0][r] = valid ? dc * aj * ai * (1.f - ai) : 0.f;
            dz[1][r] = valid ? dc * ai * (1.f - aj * aj) : 0.f;
            dz[2][r] = valid ? dc * cp * af * (1.f - af) : 0.f;
            dcs[r] = valid ? dc * af : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            bsum[k] += (dz[k][0] + dz[k][1]) + (dz[k][2] + dz[k][3]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) sA[(rb + r) * LDA + k * PHU + ul] = bf16_bits(dz[k][r]);
        __syncthreads();
        pstamp(dbg, i, 2);
        if (i + 1 < T) {
            // 4. P = dz_own . W_h(own gate cols)^T over this wave's H/4 units
            floatx4 acc[2][NT];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&sA[c * LDA + k * PHU + 8 * g]);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&sA[(16 + c) * LDA + k * PHU + 8 * g]);
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[nt][k], acc[0][nt], 0, 0, 0);
                    acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[nt][k], acc[1][nt], 0, 0, 0);
                }
            }
            // 5. publish the blocks (plain stores stay in the XCD's L2 when the group is
            //    on one XCD, else write-through), drain, barrier, flag
            const int64_t pbase = (int64_t)(i & 1) * par_stride + (int64_t)group * NU * NU * BLK;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int dst = (w * (H / 4) + 16 * nt) / PHU;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const int64_t off = (pbase + ((int64_t)dst * NU + member) * BLK +
                                         ((mt * 2 + (nt & 1)) * 64 + lane) * 4) * EB;
                    if constexpr (PB16) {
                        const float (&v)[4] = *reinterpret_cast<const float(*)[4]>(&acc[mt][nt]);
                        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                        const unsigned long long q = pack4(v);
                        const u32x2 qq = __builtin_bit_cast(u32x2, q);
                        if (local) __builtin_amdgcn_raw_buffer_store_b64(qq, x_rsrc, (int)off, 0, 0);
                        else __builtin_amdgcn_raw_buffer_store_b64(qq, x_rsrc, (int)off, 0, 16);
                    } else {
                        const u32x4 v = __builtin_bit_cast(u32x4, acc[mt][nt]);
                        if (local) __builtin_amdgcn_raw_buffer_store_b128(v, x_rsrc, (int)off, 0, 0);
                        else __builtin_amdgcn_raw_buffer_store_b128(v, x_rsrc, (int)off, 0, 16);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) raise_flag(gflags + member, base + (unsigned)(i + 1), local);
        }
        pstamp(dbg, i, 3);
        // 6. time-order copy of dz for the weight-gradient GEMMs, 16 B per piece from
        //    the LDS tile (drains behind the next step; sA is rewritten only after
        //    the next step's wait barrier)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int p = tid + 256 * v;
            const int row = p >> 4, k = (p >> 2) & 3, q = p & 3;
            const int t = step_time(dir, s, s_len[row]);
            const u32x4 val = *reinterpret_cast<const u32x4*>(&sA[row * LDA + k * PHU + 8 * q]);
            *reinterpret_cast<u32x4*>(dG_t + (((int64_t)t * B + b0 + row) * 2 + dir) * G4 + k * H + u0 + 8 * q) = val;
        }
        pstamp(dbg, i, 4);
    }
    if (bpart) {
        // the bias partial of (unit ul, gate k) over the member's 32 rows: the
        // 8 threads holding that unit (4 g x 2 M tiles) meet in LDS, fixed order
        __syncthreads();
        float* red = reinterpret_cast<float*>(sAct);                    // [8 row groups][128 gate cols]
#pragma unroll
        for (int k = 0; k < 4; ++k) red[(emt * 4 + g) * (4 * PHU) + k * PHU + ul] = bsum[k];
        __syncthreads();
        if (tid < 4 * PHU) {
            float sum = 0.f;
            for (int q = 0; q < 8; ++q) sum += red[q * (4 * PHU) + tid];
            bpart[(int64_t)(bs * 2 + dir) * G4 + (tid / PHU) * H + u0 + (tid % PHU)] = sum;
        }
    }
}

// The late-load forms (option PERSIST_LATE=0 disables them); their buffer loads
// address the largest operand (`bytes`) with 32-bit offsets.
static bool persist_late(int64_t bytes) { return opt(OPT_PERSIST_LATE) != 0 && bytes < 0x7fffffffll; }

// ------------------------------------------------------------------ C ABI
extern "C" size_t ocrk_lstm_fwd_persistent_workspace_size(int B, int H) {
    // flag word + XCC word per workgroup (128-B aligned block), then the h exchange buffer
    size_t counters = ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    return counters + (size_t)2 * 2 * B * H * sizeof(bf16);
}

// Can the whole grid be co-resident? (every group must run at once)
extern "C" int ocrk_lstm_fwd_persistent_supported(int B, int H) {
    if (B % PBR || H % PHU || !(H == 256 || H == 512)) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    hipError_t e = H == 512
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_fwd_persistent_kernel<16>, 256, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_fwd_persistent_kernel<8>, 256, 0);
    if (e != hipSuccess) return 0;
    const long grid = 2L * (B / PBR) * (H / PHU);
    return grid <= (long)cus * per_cu ? 1 : 0;
}

extern "C" size_t ocrk_persistent_flags_size(int B, int H) {
    return (B > 0 && B % PBR == 0 && H > 0 && H % PHU == 0) ? persistent_counter_bytes(B, H) : 0;
}

// the 16-row / 64-unit forward (H = 512): default where its grid (B workgroups) is co-resident;
// option LSTM_FWD_R16=0 keeps the 32-row kernel (A/B and tests)
static bool lstm_fwd_r16(int B, int H) {
    if (opt(OPT_LSTM_FWD_R16) == 0 || H != 512 || B % PBR) return false;         // flag words as the 32-row form
    static ocrk::DeviceOnce once;
    static int per_cu[ocrk::kMaxDevices];
    const int dev = ocrk::current_device();
    ocrk::once_per_device(once, [dev] {
        int n = 0;
        per_cu[dev] = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, lstm_fwd_r16_kernel, 512, 0) == hipSuccess ? n : 0;
    });
    return 2L * (B / R16_ROWS) * (H / R16_UNITS) <= (long)ocrk::cu_count() * per_cu[dev];
}

extern "C" int ocrk_lstm_fwd_persistent(const void* gx, const void* whT, const int* seq_len, int T, int B, int H,
                                        void* out, void* hprev_t, float* cprev_t, void* acts_t, unsigned* err,
                                        unsigned* flags, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_fwd_persistent_supported(B, H), "ocrk_lstm_fwd_persistent: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_fwd_persistent_workspace_size(B, H), "ocrk_lstm_fwd_persistent: workspace too small");
    hipStream_t st = ocrk::as_stream(stream);
    size_t counters = ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    bf16* hx = (bf16*)((char*)ws + counters);
    if (!flags && hipMemsetAsync(cnt, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_lstm_fwd_persistent memset");
    if (lstm_fwd_r16(B, H) && (int64_t)T * B * 8 * H * 2 < 0x7fffffffll) {
        // counters: 2 (B/16) x 8 members = the same count as 2 (B/32) x 16
        lstm_fwd_r16_kernel<<<2u * (unsigned)(B / R16_ROWS) * (unsigned)(H / R16_UNITS), 512, 0, st>>>(
            (const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t,
            (bf16*)acts_t, cnt, err, lstm_spin_limit());
        return ocrk::launch_status("ocrk_lstm_fwd_persistent");
    }
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
    if (H == 512 && persist_late((int64_t)T * B * 8 * H * 2))
        lstm_fwd_persistent_kernel<16, true><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out,
                                                                   (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err, lstm_spin_limit(), g_lstm_dbg);
    else if (H == 512)
        lstm_fwd_persistent_kernel<16><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out,
                                                             (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err, lstm_spin_limit(), g_lstm_dbg);
    else
        lstm_fwd_persistent_kernel<8><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out,
                                                            (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err, lstm_spin_limit(), g_lstm_dbg);
    return ocrk::launch_status("ocrk_lstm_fwd_persistent");
}

#ifdef OCRK_EXPERIMENTS
// (tools build, include/ocrk_debug.h: measured no gain -- every step 0.7 us longer,
// profiles/r3_fused_projection.txt)
// Fused first layer: x [T][B][n_in] (time-major features), wxT [2][4H][n_in] (per
// direction W_x^T, gate-major rows), bias f32 [2][4H]; everything else as above.
extern "C" int ocrk_lstm_fwd_persistent_x_supported(int B, int H, int n_in) {
    if (H != 512 || n_in != 256 || B % PBR) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_fwd_persistent_kernel<16, true, 256>, 256, 0) != hipSuccess)
        return 0;
    const long grid = 2L * (B / PBR) * (H / PHU);
    return grid <= (long)cus * per_cu ? 1 : 0;
}

extern "C" int ocrk_lstm_fwd_persistent_x(const void* x, int n_in, const void* wxT, const float* bias, const void* whT,
                                          const int* seq_len, int T, int B, int H, void* out, void* hprev_t,
                                          float* cprev_t, void* acts_t, unsigned* err, unsigned* flags, void* ws,
                                          size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_fwd_persistent_x_supported(B, H, n_in),
                 "ocrk_lstm_fwd_persistent_x: B=%d H=%d n_in=%d unsupported or not co-resident", B, H, n_in);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_fwd_persistent_workspace_size(B, H), "ocrk_lstm_fwd_persistent_x: workspace too small");
    OCRK_REQUIRE(x && wxT && bias && err, "ocrk_lstm_fwd_persistent_x: null operand");
    OCRK_REQUIRE((int64_t)T * B * n_in * 2 < 0x7fffffffll, "ocrk_lstm_fwd_persistent_x: x exceeds 2 GB");
    if (T <= 0) return OCRK_OK;
    hipStream_t st = ocrk::as_stream(stream);
    size_t counters = ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    bf16* hx = (bf16*)((char*)ws + counters);
    if (!flags && hipMemsetAsync(cnt, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_lstm_fwd_persistent_x memset");
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
    lstm_fwd_persistent_kernel<16, true, 256><<<grid, 256, 0, st>>>(
        nullptr, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err,
        lstm_spin_limit(), g_lstm_dbg, (const bf16*)x, (const bf16*)wxT, bias);
    return ocrk::launch_status("ocrk_lstm_fwd_persistent_x");
}
#endif  // OCRK_EXPERIMENTS

// ---------------------------------------------------------- backward C ABI
// OCRK_LSTM_BWD_KSPLIT=1: the K-split form (read per launch). Off by default:
// measured 5.2 (bf16 partials) / 7.0 (f32) against 4.2 us per step for the
// gather form at B=256, H=512 -- its exchange buffer (NU x NU blocks per group,
// 2-4 MB per XCD) does not stay in the XCD's L2 between steps.
static bool lstm_bwd_ksplit() { return opt(OPT_LSTM_BWD_KSPLIT) == 1; }

extern "C" size_t ocrk_lstm_bwd_persistent_workspace_size(int B, int H) {
    // flag word + XCC word per workgroup (128-B aligned block), then the exchange buffer:
    // K-split: [2 parities][groups][NU dst][NU src][32 x 32] f32; gather: [2][2][B][4H] bf16
    size_t counters = ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    const size_t nu = (size_t)(H / PHU);
    const size_t ksplit = (size_t)2 * 2 * (B / PBR) * nu * nu * PBR * PHU * sizeof(float);
    const size_t gather = (size_t)2 * 2 * B * 4 * H * sizeof(bf16);
    return counters + (ksplit > gather ? ksplit : gather);
}

// the 16-row / 64-unit BPTT (H = 512): default where its grid (B workgroups) is co-resident;
// option LSTM_BWD_R16=0 keeps the 32-row gather kernel (A/B and tests)
static bool lstm_bwd_r16(int B, int H) {
    if (opt(OPT_LSTM_BWD_R16) == 0 || H != 512 || B % PBR || lstm_bwd_ksplit()) return false;   // flag words as the gather form
    static ocrk::DeviceOnce once;
    static int per_cu[ocrk::kMaxDevices];
    const int dev = ocrk::current_device();
    ocrk::once_per_device(once, [dev] {
        int n = 0;
        per_cu[dev] = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, lstm_bwd_r16_kernel, 512, 0) == hipSuccess ? n : 0;
    });
    return 2L * (B / R16_ROWS) * (H / R16_UNITS) <= (long)ocrk::cu_count() * per_cu[dev];
}

extern "C" int ocrk_lstm_bwd_persistent_slices(int B, int H) {
    if (lstm_bwd_r16(B, H)) return B / R16_ROWS;
    return B % PBR == 0 ? B / PBR : 0;
}

extern "C" int ocrk_lstm_bwd_persistent_supported(int B, int H) {
    if (lstm_bwd_r16(B, H)) return 1;
    if (B % PBR || H % PHU || !(H == 256 || H == 512)) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
#ifdef OCRK_EXPERIMENTS
    hipError_t e = lstm_bwd_ksplit()
        ? (H == 512 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_ksplit_kernel<16, false>, 256, 0)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_ksplit_kernel<8, false>, 256, 0))
        : (H == 512 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_persistent_kernel<16>, 256, 0)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_persistent_kernel<8>, 256, 0));
#else
    hipError_t e = H == 512 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_persistent_kernel<16>, 256, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_persistent_kernel<8>, 256, 0);
#endif
    if (e != hipSuccess) return 0;
    const long grid = 2L * (B / PBR) * (H / PHU);
    return grid <= (long)cus * per_cu ? 1 : 0;
}

extern "C" int ocrk_lstm_bwd_persistent(const void* wh, const int* seq_len, int T, int B, int H, const void* dout,
                                        const float* cprev_t, const void* acts_t, void* dG_t, unsigned* err,
                                        unsigned* flags, float* dbias_part, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_bwd_persistent_supported(B, H), "ocrk_lstm_bwd_persistent: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_bwd_persistent_workspace_size(B, H), "ocrk_lstm_bwd_persistent: workspace too small");
    hipStream_t st = ocrk::as_stream(stream);
    size_t counters = ((size_t)2 * 2 * (B / PBR) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    bf16* zx = (bf16*)((char*)ws + counters);
    if (!flags && hipMemsetAsync(cnt, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_lstm_bwd_persistent memset");
    if (lstm_bwd_r16(B, H)) {
        // counters: 2 (B/16) x 8 members = the same count as 2 (B/32) x 16
        lstm_bwd_r16_kernel<<<2u * (unsigned)(B / R16_ROWS) * (unsigned)(H / R16_UNITS), 512, 0, st>>>(
            (const bf16*)wh, zx, seq_len, T, B, (const bf16*)dout, cprev_t, (const bf16*)acts_t, (bf16*)dG_t, cnt, err,
            lstm_spin_limit(), dbias_part);
        return ocrk::launch_status("ocrk_lstm_bwd_persistent");
    }
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
#ifdef OCRK_EXPERIMENTS
    if (lstm_bwd_ksplit()) {
        const bool pb16 = opt(OPT_LSTM_BWD_PB16) == 1;            // partial products exchanged in bf16
#define KSPLIT_LAUNCH(KSV, PB)                                                                                   \
        lstm_bwd_ksplit_kernel<KSV, PB><<<grid, 256, 0, st>>>((const bf16*)wh, zx, seq_len, T, B, (const bf16*)dout,  \
                                                             cprev_t, (const bf16*)acts_t, (bf16*)dG_t, cnt, err,     \
                                                             lstm_spin_limit(), g_lstm_dbg, dbias_part)
        if (H == 512) { if (pb16) KSPLIT_LAUNCH(16, true); else KSPLIT_LAUNCH(16, false); }
        else { if (pb16) KSPLIT_LAUNCH(8, true); else KSPLIT_LAUNCH(8, false); }
#undef KSPLIT_LAUNCH
        return ocrk::launch_status("ocrk_lstm_bwd_persistent");
    }
#endif
    if (H == 512 && persist_late((int64_t)T * B * 8 * H * 2))
        lstm_bwd_persistent_kernel<16, true><<<grid, 256, 0, st>>>((const bf16*)wh, zx, seq_len, T, B, (const bf16*)dout, cprev_t,
                                                                   (const bf16*)acts_t, (bf16*)dG_t, cnt, err, lstm_spin_limit(), g_lstm_dbg,
                                                             dbias_part);
    else if (H == 512)
        lstm_bwd_persistent_kernel<16><<<grid, 256, 0, st>>>((const bf16*)wh, zx, seq_len, T, B, (const bf16*)dout, cprev_t,
                                                             (const bf16*)acts_t, (bf16*)dG_t, cnt, err, lstm_spin_limit(), g_lstm_dbg,
                                                             dbias_part);
    else
        lstm_bwd_persistent_kernel<8><<<grid, 256, 0, st>>>((const bf16*)wh, zx, seq_len, T, B, (const bf16*)dout, cprev_t,
                                                            (const bf16*)acts_t, (bf16*)dG_t, cnt, err, lstm_spin_limit(), g_lstm_dbg,
                                                             dbias_part);
    return ocrk::launch_status("ocrk_lstm_bwd_persistent");
}
