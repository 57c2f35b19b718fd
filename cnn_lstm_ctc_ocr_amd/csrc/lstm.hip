// a7': the bidirectional LSTM time loop (rnn_layer, src/weinman/model_bu.py:167-199;
// [TF1] LSTMCell gate order i, j, f, o, forget_bias 1.0, no peepholes;
// bidirectional_dynamic_rnn(time_major, sequence_length)).
//
// Split of the work: the input projection x_t . W_x + b for every t and both
// directions is ONE MFMA GEMM before the loop (gemm.hip, N = 8H). What stays
// sequential is h_{s-1} . W_h: per step one launch covers both directions.
// A workgroup owns HU hidden units x all 4 gates (4*HU gate columns) of one
// direction for BR batch rows; it streams h_{s-1}[BR, H] and its W_h^T slice
// [4*HU, H] through LDS in KC-deep chunks (two register sets in flight),
// accumulates on MFMA, then runs the cell update for its (row, unit) pairs
// with the gate pre-activations exchanged through LDS, so c stays with its
// owner and only h is published for the next step.
//
// Sequence lengths: step s of the backward direction reads time
// t = len-1-s ([TF1] reverse_sequence); steps s >= len carry the state and
// emit zeros. Everything saved for the backward pass is stored in TIME order
// ([T][B][2][*]) so the weight-gradient GEMMs afterwards are plain GEMMs.
//
// Backward step (reverse s): dh = dout + dG_{s+1} . W_h^T (K = 4H, same
// streaming core), then the gate gradients; dG is published for the next
// step and scattered into time order for the dW_x / dW_h / dX GEMMs.
#include "recur.h"

using namespace ocrk;

// Diagnostic stamps (tools/bench_lstm.py --stamps): thread 0 of every
// workgroup writes s_memrealtime (100 MHz) at fixed points into dbg.
__device__ __forceinline__ void stamp(long long* dbg, int i) {
    if (dbg && threadIdx.x == 0) {
        long long t = __builtin_amdgcn_s_memrealtime();
        dbg[(((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + i] = t;
    }
}

// --------------------------------------------------------------- forward
// The forward cell update for the (row, 4 units) pairs of this thread, from
// the step's gate pre-activations in LDS (sG [BR][4*HU+1] f32) and the
// operands preloaded at kernel entry.
template <typename CT, int BR, int HU>
__device__ __forceinline__ void lstm_fwd_epilogue(const float* __restrict__ sG, const int (&plen)[(BR * HU / 4 + 255) / 256],
                                                  const float (&pg)[(BR * HU / 4 + 255) / 256][4][4],
                                                  const float (&pc)[(BR * HU / 4 + 255) / 256][4],
                                                  const float (&ph)[(BR * HU / 4 + 255) / 256][4], int s, int B, int H,
                                                  int b0, int u0, int dir, float* __restrict__ c_state,
                                                  CT* __restrict__ h_out, CT* __restrict__ out,
                                                  CT* __restrict__ hprev_t, float* __restrict__ cprev_t,
                                                  CT* __restrict__ acts_t) {
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    constexpr bool EFULL = (BR * UQ) % 256 == 0;
    const int G4 = 4 * H;
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int len = plen[q];
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;          // state index
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;           // time-order row
        CT* a = acts_t + tb * G4 + uu;
        if (s < len) {
            const float* gl = sG + r * (4 * HU + 1) + u;
            float ai[4], aj[4], af[4], ao[4], c[4], h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                ai[e] = sig_fast(gl[0 * HU + e] + pg[q][0][e]);
                aj[e] = tanh_fast(gl[1 * HU + e] + pg[q][1][e]);
                af[e] = sig_fast(gl[2 * HU + e] + pg[q][2][e] + 1.0f);   // forget_bias = 1
                ao[e] = sig_fast(gl[3 * HU + e] + pg[q][3][e]);
                c[e] = af[e] * pc[q][e] + ai[e] * aj[e];
                h[e] = ao[e] * tanh_fast(c[e]);
            }
            st4(c_state + st, c);
            st4(h_out + st, h);
            st4(out + ((int64_t)t * B + b) * 2 * H + dir * H + uu, h);
            st4(hprev_t + tb * H + uu, ph[q]);
            st4(cprev_t + tb * H + uu, pc[q]);
            st4(a + 0 * H, ai); st4(a + 1 * H, aj); st4(a + 2 * H, af); st4(a + 3 * H, ao);
        } else {
            const float z[4] = {0.f, 0.f, 0.f, 0.f};
            st4(h_out + st, ph[q]);
            st4(hprev_t + tb * H + uu, z);
            st4(cprev_t + tb * H + uu, z);
            st4(a + 0 * H, z); st4(a + 1 * H, z); st4(a + 2 * H, z); st4(a + 3 * H, z);
        }
    }
}

// Epilogue operands (gx, c, h, len) do not depend on the GEMM: they are loaded
// into registers at kernel entry so their HBM latency hides under the GEMM.
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
lstm_fwd_step_kernel(const CT* __restrict__ gx, const CT* __restrict__ whT, const CT* __restrict__ h_in,
                     CT* __restrict__ h_out, float* __restrict__ c_state, const int* __restrict__ seq_len,
                     int s, int T, int B, int H, CT* __restrict__ out, CT* __restrict__ hprev_t,
                     float* __restrict__ cprev_t, CT* __restrict__ acts_t, long long* __restrict__ dbg) {
    using Core = RecurCore<CT, BR, 4 * HU, KC>;
    stamp(dbg, 0);
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G4 = 4 * H;

    // thread <-> (row r, 4 consecutive units u..u+3) of the epilogue
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    static_assert(HU % 4 == 0, "4-unit epilogue vectors");
    constexpr bool EFULL = (BR * UQ) % 256 == 0;     // whole passes: no lane guard (bf16 tiles)
    // 1. sequence lengths; 2. the GEMM's first chunks; 3. the epilogue
    // operands (t depends on len) -- all loads unconditional, no lane branches.
    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
    const CT* a_rows = h_in + ((int64_t)dir * B + b0) * H;
    const CT* wdir = whT + (int64_t)dir * 4 * H * H;
    auto bcol = [&](int n) { return wdir + (int64_t)((n / HU) * H + u0 + (n % HU)) * H; };
    Core core;
    core.begin(a_rows, H, bcol, H);
    stamp(dbg, 1);
    float pg[EPQ4][4][4], pc[EPQ4][4], ph[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        ld4(pc[q], c_state + st);
        ld4(ph[q], h_in + st);
        const int t = step_time(dir, s, plen[q]);
        const CT* g = gx + (((int64_t)t * B + b) * 2 + dir) * G4 + uu;
#pragma unroll
        for (int k = 0; k < 4; ++k) ld4(pg[q][k], g + k * H);
    }
    stamp(dbg, 2);
    floatx4 acc[Core::TPW];
    core.finish(a_rows, H, bcol, H, lds, acc);
    stamp(dbg, 3);
    Core::spill(acc, lds);
    stamp(dbg, 4);
    lstm_fwd_epilogue<CT, BR, HU>(reinterpret_cast<const float*>(lds), plen, pg, pc, ph, s, B, H, b0, u0, dir, c_state,
                                  h_out, out, hprev_t, cprev_t, acts_t);
    stamp(dbg, 5);
}

// Forward step with the whole GEMM operand set in LDS (bf16, K = H <= 512):
// 64 h rows and the 64 W_h^T rows of this tile's 16 units x 4 gates, 2H bytes
// each, fetched in ONE burst of LDS-DMA (global_load_lds_dwordx4: no VGPR
// round trip, every load in flight at once) while the epilogue operands load
// into registers; then the 64 x 64 x H product on MFMA straight from LDS.
// Rows are lane-linear with the 16-B chunk index XOR-swizzled by (row & 15) on
// the global side, so each 16-lane group of a ds_read_b128 fragment read covers
// all 64 banks (conflict-free; row starts are 256-B aligned).
template <int H_>
__global__ void __launch_bounds__(256)
lstm_fwd_step_dma_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whT, const bf16* __restrict__ h_in,
                         bf16* __restrict__ h_out, float* __restrict__ c_state, const int* __restrict__ seq_len,
                         int s, int T, int B, bf16* __restrict__ out, bf16* __restrict__ hprev_t,
                         float* __restrict__ cprev_t, bf16* __restrict__ acts_t, long long* __restrict__ dbg) {
    constexpr int BR = 64, HU = 16, NC = 4 * HU, H = H_;
    stamp(dbg, 0);
    constexpr int ROWB = 2 * H, CPR = ROWB / 16, RPI = 64 / CPR;     // 16-B chunks per row, rows per wave instr
    constexpr int NI = BR / (4 * RPI);                              // instructions per wave per operand
    static_assert(CPR % 16 == 0 && 64 % CPR == 0, "H = 256 or 512");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char* sA = lds;
    char* sB = lds + BR * ROWB;
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G4 = 4 * H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;

    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min(tid + 256 * q, BR * UQ - 1) / UQ];

    // 1. the operand burst
    const bf16* a_rows = h_in + ((int64_t)dir * B + b0) * H;
    const bf16* wdir = whT + (int64_t)dir * 4 * H * H;
    const int lrow = lane / CPR, chunk = (lane % CPR) ^ 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int r = (i * 4 + wave) * RPI + lrow;
        const int c = (lane % CPR) ^ (r & 15);
        __builtin_amdgcn_global_load_lds((const void*)(a_rows + (int64_t)r * H + 8 * c),
                                         (__attribute__((address_space(3))) void*)(sA + (i * 4 + wave) * RPI * ROWB),
                                         16, 0, 0);
        const bf16* brow = wdir + (int64_t)((r / HU) * H + u0 + (r % HU)) * H;
        __builtin_amdgcn_global_load_lds((const void*)(brow + 8 * c),
                                         (__attribute__((address_space(3))) void*)(sB + (i * 4 + wave) * RPI * ROWB),
                                         16, 0, 0);
    }
    (void)chunk;
    stamp(dbg, 1);
    // 2. epilogue operands (do not depend on the product)
    float pg[EPQ4][4][4], pc[EPQ4][4], ph[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = tid + 256 * q;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        ld4(pc[q], c_state + st);
        ld4(ph[q], h_in + st);
        const int t = step_time(dir, s, plen[q]);
        const bf16* g = gx + (((int64_t)t * B + b) * 2 + dir) * G4 + uu;
#pragma unroll
        for (int k = 0; k < 4; ++k) ld4(pg[q][k], g + k * H);
    }
    stamp(dbg, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(dbg, 3);

    // 3. 64 x 64 x H on MFMA, 2 x 2 waves of 32 x 32
    const int wm = wave >> 1, wn = wave & 1, i16 = lane & 15, g = lane >> 4, sw = lane & 15;
    floatx4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    {
        const char* ar[2] = {sA + (wm * 32 + i16) * ROWB, sA + (wm * 32 + 16 + i16) * ROWB};
        const char* br[2] = {sB + (wn * 32 + i16) * ROWB, sB + (wn * 32 + 16 + i16) * ROWB};
        lds_mma_16x16x32<H / 32, 2, 2>(ar, br, g, sw, acc);
    }
    __syncthreads();
    float* sG = reinterpret_cast<float*>(lds);                      // [BR][NC+1]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sG[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * (NC + 1) + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    stamp(dbg, 4);
    lstm_fwd_epilogue<bf16, BR, HU>(sG, plen, pg, pc, ph, s, B, H, b0, u0, dir, c_state, h_out, out, hprev_t,
                                    cprev_t, acts_t);
    stamp(dbg, 5);
}

// -------------------------------------------------------------- backward
// Per-thread epilogue operands of a backward step (independent of the
// recurrent product, so they are fetched before / while it is computed).
template <int BR, int HU>
struct LstmBwdOps {
    static constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    static constexpr bool EFULL = (BR * UQ) % 256 == 0;   // whole passes: no lane guard
    int plen[EPQ4];
    float pa[EPQ4][4][4], pcp[EPQ4][4], pdc[EPQ4][4], pdo[EPQ4][4];

    template <typename CT>
    __device__ __forceinline__ void load(const int* __restrict__ seq_len, const float* __restrict__ dc_state,
                                         const CT* __restrict__ acts_t, const float* __restrict__ cprev_t,
                                         const CT* __restrict__ dout, int s, int B, int H, int b0, int u0,
                                         int dir) {
#pragma unroll
        for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
        const int G4 = 4 * H;
#pragma unroll
        for (int q = 0; q < EPQ4; ++q) {
            const int idx = threadIdx.x + 256 * q;
            if (!EFULL && idx >= BR * UQ) continue;
            const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
            ld4(pdc[q], dc_state + ((int64_t)dir * B + b) * H + uu);
            const int t = step_time(dir, s, plen[q]);
            const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
            const CT* a = acts_t + tb * G4 + uu;
#pragma unroll
            for (int k = 0; k < 4; ++k) ld4(pa[q][k], a + k * H);
            ld4(pcp[q], cprev_t + tb * H + uu);
            ld4(pdo[q], dout + ((int64_t)t * B + b) * 2 * H + dir * H + uu);
        }
    }

    // sG: the recurrent product dh_rec as [BR][HU + 1] fp32.
    template <typename CT>
    __device__ __forceinline__ void epilogue(const float* __restrict__ sG, int s, int B, int H, int b0, int u0,
                                             int dir, float* __restrict__ dc_state, CT* __restrict__ dg_out,
                                             CT* __restrict__ dG_t) const {
        const int G4 = 4 * H;
#pragma unroll
        for (int q = 0; q < EPQ4; ++q) {
            const int idx = threadIdx.x + 256 * q;
            if (!EFULL && idx >= BR * UQ) continue;
            const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
            const int len = plen[q];
            const int t = step_time(dir, s, len);
            const int64_t st = ((int64_t)dir * B + b) * H + uu;
            const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
            CT* dgo = dg_out + ((int64_t)dir * B + b) * G4 + uu;
            CT* dgt = dG_t + tb * G4 + uu;
            if (s < len) {
                float di[4], dj[4], df[4], dO[4], dcn[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float dh = sG[r * (HU + 1) + u + e] + pdo[q][e];
                    float ai = pa[q][0][e], aj = pa[q][1][e], af = pa[q][2][e], ao = pa[q][3][e];
                    float cp = pcp[q][e];
                    float c = af * cp + ai * aj;
                    float tc = tanh_fast(c);
                    float dc = pdc[q][e] + dh * ao * (1.f - tc * tc);
                    dO[e] = dh * tc * ao * (1.f - ao);
                    di[e] = dc * aj * ai * (1.f - ai);
                    dj[e] = dc * ai * (1.f - aj * aj);
                    df[e] = dc * cp * af * (1.f - af);
                    dcn[e] = dc * af;
                }
                st4(dc_state + st, dcn);
                st4(dgo + 0 * H, di); st4(dgo + 1 * H, dj); st4(dgo + 2 * H, df); st4(dgo + 3 * H, dO);
                st4(dgt + 0 * H, di); st4(dgt + 1 * H, dj); st4(dgt + 2 * H, df); st4(dgt + 3 * H, dO);
            } else {
                const float z[4] = {0.f, 0.f, 0.f, 0.f};
                st4(dc_state + st, z);
                st4(dgo + 0 * H, z); st4(dgo + 1 * H, z); st4(dgo + 2 * H, z); st4(dgo + 3 * H, z);
                st4(dgt + 0 * H, z); st4(dgt + 1 * H, z); st4(dgt + 2 * H, z); st4(dgt + 3 * H, z);
            }
        }
    }
};

template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
lstm_bwd_step_kernel(const CT* __restrict__ wh, const CT* __restrict__ dg_in, CT* __restrict__ dg_out,
                     float* __restrict__ dc_state, const int* __restrict__ seq_len, int s, int T, int B, int H,
                     const CT* __restrict__ dout, const float* __restrict__ cprev_t,
                     const CT* __restrict__ acts_t, CT* __restrict__ dG_t) {
    using Core = RecurCore<CT, BR, HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G4 = 4 * H;
    static_assert(HU % 4 == 0, "4-unit epilogue vectors");
    const CT* a_rows = dg_in + ((int64_t)dir * B + b0) * G4;
    const CT* wdir = wh + (int64_t)dir * H * G4;
    auto bcol = [&](int n) { return wdir + (int64_t)(u0 + n) * G4; };
    Core core;
    core.begin(a_rows, G4, bcol, G4);
    LstmBwdOps<BR, HU> ops;
    ops.load(seq_len, dc_state, acts_t, cprev_t, dout, s, B, H, b0, u0, dir);
    floatx4 acc[Core::TPW];
    core.finish(a_rows, G4, bcol, G4, lds, acc);
    Core::spill(acc, lds);
    ops.epilogue(reinterpret_cast<const float*>(lds), s, B, H, b0, u0, dir, dc_state, dg_out, dG_t);
}

// bf16 backward step with the operands streamed by LDS-DMA: the 64 dG rows
// and the 16 W_h rows (K = 4H) pass through a two-buffer ring of 512-deep
// k-chunks (80 KB each, 1 KB per row, 16-B chunks XOR-swizzled by row), so
// chunk c+1 is in flight while chunk c is on MFMA. Wave w owns batch rows
// 16w..16w+15 of the 64 x 16 product.
template <int H_>
__global__ void __launch_bounds__(256)
lstm_bwd_step_dma_kernel(const bf16* __restrict__ wh, const bf16* __restrict__ dg_in, bf16* __restrict__ dg_out,
                         float* __restrict__ dc_state, const int* __restrict__ seq_len, int s, int T, int B,
                         const bf16* __restrict__ dout, const float* __restrict__ cprev_t,
                         const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t) {
    constexpr int BR = 64, HU = 16, H = H_, G4 = 4 * H;
    constexpr int KCH = 512, NCH = G4 / KCH, ROWB = 2 * KCH;     // one wave instruction per 1-KB row
    constexpr int BUFB = (BR + HU) * ROWB, NPS = (BR + HU) / 4;  // DMA instructions per wave per chunk
    static_assert(G4 % KCH == 0 && NCH >= 2, "H = 256 or 512");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    // epilogue operands first: vmcnt retires in order, so the counted waits
    // below also cover them
    LstmBwdOps<BR, HU> ops;
    ops.load(seq_len, dc_state, acts_t, cprev_t, dout, s, B, H, b0, u0, dir);

    const bf16* a_rows = dg_in + ((int64_t)dir * B + b0) * G4;
    const bf16* wdir = wh + ((int64_t)dir * H + u0) * G4;
    auto issue = [&](int c) {
        char* sA = lds + (c & 1) * BUFB;
        char* sB = sA + BR * ROWB;
#pragma unroll
        for (int i = 0; i < BR / 4; ++i) {
            const int r = i * 4 + wave;
            __builtin_amdgcn_global_load_lds((const void*)(a_rows + (int64_t)r * G4 + c * KCH + 8 * (lane ^ (r & 15))),
                                             (__attribute__((address_space(3))) void*)(sA + r * ROWB), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < HU / 4; ++i) {
            const int n = i * 4 + wave;
            __builtin_amdgcn_global_load_lds((const void*)(wdir + (int64_t)n * G4 + c * KCH + 8 * (lane ^ (n & 15))),
                                             (__attribute__((address_space(3))) void*)(sB + n * ROWB), 16, 0, 0);
        }
    };
    issue(0);
    issue(1);

    const int i16 = lane & 15, g = lane >> 4, sw = lane & 15;
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) vm_wait<NPS>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();                       // everyone's chunk c has landed
        const char* sA = lds + (c & 1) * BUFB + (wave * 16 + i16) * ROWB;
        const char* sB = lds + (c & 1) * BUFB + BR * ROWB + i16 * ROWB;
        {
            const char* ar[1] = {sA};
            const char* br[1] = {sB};
            floatx4 (&acc11)[1][1] = reinterpret_cast<floatx4 (&)[1][1]>(acc);
            lds_mma_16x16x32<KCH / 32, 1, 1, 4>(ar, br, g, sw, acc11);
        }
        if (c + 2 < NCH) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();                   // buffer c & 1 is free again
            issue(c + 2);
        }
    }
    __syncthreads();
    float* sG = reinterpret_cast<float*>(lds);              // [BR][HU + 1]
#pragma unroll
    for (int r = 0; r < 4; ++r) sG[(wave * 16 + g * 4 + r) * (HU + 1) + i16] = acc[r];
    __syncthreads();
    ops.epilogue(sG, s, B, H, b0, u0, dir, dc_state, dg_out, dG_t);
}

// ------------------------------------------------------------------ C ABI
long long* g_lstm_dbg = nullptr;   // diagnostics only (ocrk_lstm_debug_stamps)

extern "C" int ocrk_lstm_debug_stamps(long long* buf) { g_lstm_dbg = buf; return OCRK_OK; }

static bool lstm_dma_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("OCRK_LSTM_DMA");
        on = (e && e[0] == '0') ? 0 : 1;
        if (on) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_fwd_step_dma_kernel<512>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 256 * 512);
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_fwd_step_dma_kernel<256>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 256 * 256);
        }
    }
    return on == 1;
}

// Backward ring: 2 x 80 KB of dynamic LDS. OCRK_LSTM_BWD_DMA=0 disables it.
constexpr int LSTM_BWD_DMA_LDS = 2 * (64 + 16) * 1024;
static bool lstm_bwd_dma_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("OCRK_LSTM_BWD_DMA");
        on = (e && e[0] == '0') ? 0 : 1;
        if (on) {
            hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_step_dma_kernel<512>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, LSTM_BWD_DMA_LDS);
            hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_step_dma_kernel<256>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, LSTM_BWD_DMA_LDS);
            if (e1 != hipSuccess || e2 != hipSuccess) on = 0;
        }
    }
    return on == 1;
}

// Tile shapes: bf16 BR=64 x HU=16 (fwd K-chunk 128, bwd 256); f32 BR=32 x HU=8/16.
#define FWD_BF16 bf16, 64, 16, 256
#define FWD_F32 float, 32, 8, 64
#define BWD_BF16 bf16, 64, 16, 256
#define BWD_F32 float, 32, 16, 128

extern "C" int ocrk_lstm_fwd_step(const void* gx, const void* whT, const void* h_in, void* h_out,
                                  float* c_state, const int* seq_len, int s, int T, int B, int H, void* out,
                                  void* hprev_t, float* cprev_t, void* acts_t, int dtype, void* stream) {
    hipStream_t st = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16) {
        OCRK_REQUIRE(H % 256 == 0 && B % 64 == 0, "ocrk_lstm_fwd_step: bf16 needs H %% 256 == 0 and B %% 64 == 0 (H=%d B=%d)", H, B);
        dim3 grid(H / 16 * (B / 64) * 2);
        if (lstm_dma_enabled() && (H == 512 || H == 256)) {
            if (H == 512)
                lstm_fwd_step_dma_kernel<512><<<grid, 256, 256 * 512, st>>>((const bf16*)gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, g_lstm_dbg);
            else
                lstm_fwd_step_dma_kernel<256><<<grid, 256, 256 * 256, st>>>((const bf16*)gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, g_lstm_dbg);
            return ocrk::launch_status("ocrk_lstm_fwd_step");
        }
        lstm_fwd_step_kernel<FWD_BF16><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, H, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, g_lstm_dbg);
    } else {
        OCRK_REQUIRE(H % 64 == 0 && B % 32 == 0, "ocrk_lstm_fwd_step: f32 needs H %% 64 == 0 and B %% 32 == 0 (H=%d B=%d)", H, B);
        dim3 grid(H / 8 * (B / 32) * 2);
        lstm_fwd_step_kernel<FWD_F32><<<grid, 256, 0, st>>>((const float*)gx, (const float*)whT, (const float*)h_in, (float*)h_out, c_state, seq_len, s, T, B, H, (float*)out, (float*)hprev_t, cprev_t, (float*)acts_t, g_lstm_dbg);
    }
    return ocrk::launch_status("ocrk_lstm_fwd_step");
}

extern "C" int ocrk_lstm_bwd_step(const void* wh, const void* dg_in, void* dg_out, float* dc_state,
                                  const int* seq_len, int s, int T, int B, int H, const void* dout,
                                  const float* cprev_t, const void* acts_t, void* dG_t, int dtype,
                                  void* stream) {
    hipStream_t st = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16) {
        OCRK_REQUIRE(H % 64 == 0 && B % 64 == 0, "ocrk_lstm_bwd_step: bf16 needs H %% 64 == 0 and B %% 64 == 0");
        dim3 grid(H / 16 * (B / 64) * 2);
        if (lstm_bwd_dma_enabled() && !g_lstm_dbg && (H == 512 || H == 256)) {
            if (H == 512)
                lstm_bwd_step_dma_kernel<512><<<grid, 256, LSTM_BWD_DMA_LDS, st>>>((const bf16*)wh, (const bf16*)dg_in, (bf16*)dg_out, dc_state, seq_len, s, T, B, (const bf16*)dout, cprev_t, (const bf16*)acts_t, (bf16*)dG_t);
            else
                lstm_bwd_step_dma_kernel<256><<<grid, 256, LSTM_BWD_DMA_LDS, st>>>((const bf16*)wh, (const bf16*)dg_in, (bf16*)dg_out, dc_state, seq_len, s, T, B, (const bf16*)dout, cprev_t, (const bf16*)acts_t, (bf16*)dG_t);
            return ocrk::launch_status("ocrk_lstm_bwd_step");
        }
        lstm_bwd_step_kernel<BWD_BF16><<<grid, 256, 0, st>>>((const bf16*)wh, (const bf16*)dg_in, (bf16*)dg_out, dc_state, seq_len, s, T, B, H, (const bf16*)dout, cprev_t, (const bf16*)acts_t, (bf16*)dG_t);
    } else {
        OCRK_REQUIRE(H % 32 == 0 && B % 32 == 0, "ocrk_lstm_bwd_step: f32 needs H %% 32 == 0 and B %% 32 == 0");
        dim3 grid(H / 16 * (B / 32) * 2);
        lstm_bwd_step_kernel<BWD_F32><<<grid, 256, 0, st>>>((const float*)wh, (const float*)dg_in, (float*)dg_out, dc_state, seq_len, s, T, B, H, (const float*)dout, cprev_t, (const float*)acts_t, (float*)dG_t);
    }
    return ocrk::launch_status("ocrk_lstm_bwd_step");
}

// Whole time loops (T launches each) so a binding makes one call per layer.
extern "C" int ocrk_lstm_fwd(const void* gx, const void* whT, void* h_state /*[2 bufs][2][B][H]*/,
                             float* c_state, const int* seq_len, int T, int B, int H, void* out, void* hprev_t,
                             float* cprev_t, void* acts_t, int dtype, void* stream) {
    size_t esz = dtype == OCRK_BF16 ? 2 : 4;
    char* hs = (char*)h_state;
    size_t hbytes = (size_t)2 * B * H * esz;
    for (int s = 0; s < T; ++s) {
        int st = ocrk_lstm_fwd_step(gx, whT, hs + (s & 1) * hbytes, hs + ((s + 1) & 1) * hbytes, c_state, seq_len,
                                    s, T, B, H, out, hprev_t, cprev_t, acts_t, dtype, stream);
        if (st) return st;
    }
    return OCRK_OK;
}

extern "C" int ocrk_lstm_bwd(const void* wh, void* dg_state /*[2 bufs][2][B][4H]*/, float* dc_state,
                             const int* seq_len, int T, int B, int H, const void* dout, const float* cprev_t,
                             const void* acts_t, void* dG_t, int dtype, void* stream) {
    size_t esz = dtype == OCRK_BF16 ? 2 : 4;
    char* ds = (char*)dg_state;
    size_t gbytes = (size_t)2 * B * 4 * H * esz;
    for (int i = 0; i < T; ++i) {
        int s = T - 1 - i;
        int st = ocrk_lstm_bwd_step(wh, ds + (i & 1) * gbytes, ds + ((i + 1) & 1) * gbytes, dc_state, seq_len, s,
                                    T, B, H, dout, cprev_t, acts_t, dG_t, dtype, stream);
        if (st) return st;
    }
    return OCRK_OK;
}
