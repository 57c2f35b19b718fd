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
#include "gemm.h"
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

// Forward step with the whole operand set in LDS (bf16, K = H <= 512), moved
// by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, all in flight at
// once) in k-block-major order: block kc = k in [128 kc, 128 kc + 128) of the
// 64 h rows and the 64 W_h^T rows of this tile's 16 units x 4 gates, 256 B
// per row, 16-B chunks XOR-swizzled by (row & 15) on the global side (each
// 16-lane group of a ds_read_b128 fragment read covers all 64 banks). The
// MFMAs of block kc start as soon as it has landed (counted vmcnt, raw
// s_barrier) while later blocks are in flight. The epilogue operands (gx
// tile, c tile) ride the same DMA queue behind the GEMM blocks; h_{s-1} of
// the tile's own units is read back from the A image.
template <int H_>
__global__ void __launch_bounds__(256)
lstm_fwd_step_dma_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whT, const bf16* __restrict__ h_in,
                         bf16* __restrict__ h_out, float* __restrict__ c_state, const int* __restrict__ seq_len,
                         int s, int T, int B, bf16* __restrict__ out, bf16* __restrict__ hprev_t,
                         float* __restrict__ cprev_t, bf16* __restrict__ acts_t, long long* __restrict__ dbg) {
    constexpr int BR = 64, HU = 16, NC = 4 * HU, H = H_;
    constexpr int NCH = H / 128, ROWB = 256, BLK = 2 * BR * ROWB;   // k blocks, bytes per row per block, block bytes
    constexpr int GX_OFF = NCH * BLK, C_OFF = GX_OFF + BR * 4 * HU * 2;
    static_assert(H % 128 == 0 && NCH >= 1 && NCH <= 4, "H = 128, 256, 384 or 512");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    stamp(dbg, 0);
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G4 = 4 * H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int UQ = HU / 4;
    static_assert(BR * UQ == 256, "one epilogue item per thread");

    // sequence lengths: SCALAR loads of the wave's row groups, issued now and
    // waited for only after the DMA burst is out (a vector load here would
    // be waited for with vmcnt(0) behind the whole burst: the compiler does
    // not count LDS-DMA), then picked per lane with selects. Inline asm
    // because the compiler turns the select chain back into a vector gather.
    typedef int int8v __attribute__((ext_vector_type(8)));
    typedef int int16v __attribute__((ext_vector_type(16)));
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int gr0 = (0 * 4 + wv) * 8 + (lane >> 3), gr1 = (1 * 4 + wv) * 8 + (lane >> 3);
    int8v sl0, sl1;
    int16v sle;
    {
        // byte offsets made explicitly uniform: the pointer must sit in SGPRs
        const unsigned o0 = __builtin_amdgcn_readfirstlane((b0 + (0 * 4 + wv) * 8) * 4);
        const unsigned o1 = __builtin_amdgcn_readfirstlane((b0 + (1 * 4 + wv) * 8) * 4);
        const unsigned oe = __builtin_amdgcn_readfirstlane((b0 + wv * 16) * 4);
        asm volatile("s_load_dwordx8 %0, %1, %2" : "=&s"(sl0) : "s"(seq_len), "s"(o0));
        asm volatile("s_load_dwordx8 %0, %1, %2" : "=&s"(sl1) : "s"(seq_len), "s"(o1));
        asm volatile("s_load_dwordx16 %0, %1, %2" : "=&s"(sle) : "s"(seq_len), "s"(oe));
    }

    // 1. GEMM operand blocks, k-block-major; 8 wave instructions per block
    const bf16* a_rows = h_in + ((int64_t)dir * B + b0) * H;
    const bf16* wdir = whT + (int64_t)dir * 4 * H * H + (int64_t)u0 * H;
    const int c16 = lane & 15;
#pragma unroll
    for (int kc = 0; kc < NCH; ++kc)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int ii = i * 4 + wave, r = 4 * ii + (lane >> 4);     // r < 64: h row; else W^T row r - 64
            const int n = r - BR;
            const bf16* src = r < BR ? a_rows + (int64_t)r * H : wdir + (int64_t)((n / HU) * H + (n % HU)) * H;
            __builtin_amdgcn_global_load_lds((const void*)(src + kc * 128 + 8 * (c16 ^ (r & 15))),
                                             (__attribute__((address_space(3))) void*)(lds + kc * BLK + 4 * ii * ROWB),
                                             16, 0, 0);
        }
    // 2. epilogue operands: gx [64 rows][4 gates][16 units] bf16 (2 instructions
    //    per wave), c [64 rows][16] f32 (1 per wave)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(sl0), "+s"(sl1), "+s"(sle));
    int plen[1], len0 = sl0[0], len1 = sl1[0];
    plen[0] = sle[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        len0 = (lane >> 3) == k ? sl0[k] : len0;
        len1 = (lane >> 3) == k ? sl1[k] : len1;
    }
#pragma unroll
    for (int k = 1; k < 16; ++k) plen[0] = (lane >> 2) == k ? sle[k] : plen[0];
    {
        const int gate = (lane & 7) >> 1, half = lane & 1;
        const int t0 = step_time(dir, s, len0), t1 = step_time(dir, s, len1);
        const bf16* g0 = gx + (((int64_t)t0 * B + b0 + gr0) * 2 + dir) * G4 + gate * H + u0 + half * 8;
        const bf16* g1 = gx + (((int64_t)t1 * B + b0 + gr1) * 2 + dir) * G4 + gate * H + u0 + half * 8;
        __builtin_amdgcn_global_load_lds((const void*)g0,
                                         (__attribute__((address_space(3))) void*)(lds + GX_OFF + (0 * 4 + wave) * 1024),
                                         16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)g1,
                                         (__attribute__((address_space(3))) void*)(lds + GX_OFF + (1 * 4 + wave) * 1024),
                                         16, 0, 0);
        const float* cs = c_state + ((int64_t)dir * B + b0 + wave * 16 + (lane >> 2)) * H + u0 + (lane & 3) * 4;
        __builtin_amdgcn_global_load_lds((const void*)cs,
                                         (__attribute__((address_space(3))) void*)(lds + C_OFF + wave * 1024),
                                         16, 0, 0);
    }
    stamp(dbg, 1);

    // 3. 64 x 64 x H on MFMA, 2 x 2 waves of 32 x 32, block by block as they land
    const int wm = wave >> 1, wn = wave & 1, i16 = lane & 15, g = lane >> 4, sw = lane & 15;
    floatx4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NCH; ++kc) {
        // block kc landed: the blocks after it and the 3 epilogue moves are younger
        const int younger = 8 * (NCH - 1 - kc) + 3;     // folds under the unrolled loop
        if (younger == 27) vm_wait<27>();
        else if (younger == 19) vm_wait<19>();
        else if (younger == 11) vm_wait<11>();
        else vm_wait<3>();
        __builtin_amdgcn_s_barrier();
        if (kc == 0) stamp(dbg, 2);
        const char* base = lds + kc * BLK;
        const char* ar[2] = {base + (wm * 32 + i16) * ROWB, base + (wm * 32 + 16 + i16) * ROWB};
        const char* br[2] = {base + (BR + wn * 32 + i16) * ROWB, base + (BR + wn * 32 + 16 + i16) * ROWB};
        lds_mma_16x16x32<4, 2, 2, 2>(ar, br, g, sw, acc);
    }
    stamp(dbg, 3);
    // h_{s-1} of this thread's 4 units, from the A image (before the spill overwrites block 0)
    const int er = tid / UQ, eu = 4 * (tid % UQ);
    float pg[1][4][4], pc[1][4], ph[1][4];
    {
        const int k = u0 + eu;
        const char* p = lds + (k / 128) * BLK + er * ROWB + ((((k % 128) / 8) ^ (er & 15)) * 16) + (k % 8) * 2;
        ld4(ph[0], reinterpret_cast<const bf16*>(p));
    }
    vm_wait<0>();
    __syncthreads();                                      // gx / c tiles in; every wave is done with block 0
    float* sG = reinterpret_cast<float*>(lds);            // [BR][NC+1]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sG[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * (NC + 1) + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        ld4(pg[0][k], reinterpret_cast<const bf16*>(lds + GX_OFF + er * 128 + k * 32 + eu * 2));
    ld4(pc[0], reinterpret_cast<const float*>(lds + C_OFF + er * 64 + eu * 4));
    __syncthreads();
    stamp(dbg, 4);
    lstm_fwd_epilogue<bf16, BR, HU>(sG, plen, pg, pc, ph, s, B, H, b0, u0, dir, c_state, h_out, out, hprev_t,
                                    cprev_t, acts_t);
    stamp(dbg, 5);
}

// Sequence lengths of the 16 rows b0 + 16 w .. +15 of wave w by ONE scalar
// load (inline asm: issued early and waited for late, after the LDS-DMA burst
// is out -- a vector load would be waited for with vmcnt(0), i.e. behind
// every DMA issued before its use, and the compiler folds a select chain on
// plain loads back into a vector gather), then picked per lane.
typedef int int16v_t __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int16v_t wave_rows_len16_issue(const int* __restrict__ seq_len, int b0, int wave) {
    const unsigned off = __builtin_amdgcn_readfirstlane((b0 + wave * 16) * 4);
    int16v_t v;
    asm volatile("s_load_dwordx16 %0, %1, %2" : "=&s"(v) : "s"(seq_len), "s"(off));
    return v;
}
// row 16 w + (lane >> 2): the epilogue row when 4 threads share a row
__device__ __forceinline__ int wave_rows_len16_pick(int16v_t v, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v));
    int len = v[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) len = (lane >> 2) == k ? v[k] : len;
    return len;
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
        load_operands(dc_state, acts_t, cprev_t, dout, s, B, H, b0, u0, dir);
    }

    // the same with plen[] already set
    template <typename CT>
    __device__ __forceinline__ void load_operands(const float* __restrict__ dc_state, const CT* __restrict__ acts_t,
                                                  const float* __restrict__ cprev_t, const CT* __restrict__ dout,
                                                  int s, int B, int H, int b0, int u0, int dir) {
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

template <typename CT, int BR, int HU, int KC, bool X3 = false>
__global__ void __launch_bounds__(256)
lstm_bwd_step_kernel(const CT* __restrict__ wh, const CT* __restrict__ dg_in, CT* __restrict__ dg_out,
                     float* __restrict__ dc_state, const int* __restrict__ seq_len, int s, int T, int B, int H,
                     const CT* __restrict__ dout, const float* __restrict__ cprev_t,
                     const CT* __restrict__ acts_t, CT* __restrict__ dG_t) {
    using Core = RecurCore<CT, BR, HU, KC, X3>;
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

// bf16 backward step with every operand moved by LDS-DMA. The 64 dG rows and
// the 16 W_h rows (K = 4H) stream through a three-buffer ring of 256-deep
// k-chunks (40 KB each, 512 B per row, 16-B chunks XOR-swizzled by row & 15),
// two chunks in flight while one is on MFMA; the epilogue operands (dc,
// c_prev, gate activations and dout of the step's time rows) ride the same
// queue behind the first two chunks into a region of their own. Counted
// vmcnt waits + raw s_barrier per chunk. Wave w owns batch rows 16w..16w+15
// of the 64 x 16 product and moves the epilogue operands of those rows.
constexpr int LSTM_BWD_KCH = 256, LSTM_BWD_RING = 3;
constexpr int LSTM_BWD_BUFB = (64 + 16) * 2 * LSTM_BWD_KCH;
constexpr int LSTM_BWD_EPI = 64 * 128 + 64 * 64 + 64 * 64 + 64 * 32;   // acts | c_prev | dc | dout
constexpr int LSTM_BWD_DMA_LDS = LSTM_BWD_RING * LSTM_BWD_BUFB + LSTM_BWD_EPI;
template <int H_>
__global__ void __launch_bounds__(256)
lstm_bwd_step_dma_kernel(const bf16* __restrict__ wh, const bf16* __restrict__ dg_in, bf16* __restrict__ dg_out,
                         float* __restrict__ dc_state, const int* __restrict__ seq_len, int s, int T, int B,
                         const bf16* __restrict__ dout, const float* __restrict__ cprev_t,
                         const bf16* __restrict__ acts_t, bf16* __restrict__ dG_t) {
    constexpr int BR = 64, HU = 16, H = H_, G4 = 4 * H;
    constexpr int KCH = LSTM_BWD_KCH, NCH = G4 / KCH, ROWB = 2 * KCH, RING = LSTM_BWD_RING;
    constexpr int BUFB = LSTM_BWD_BUFB, NPS = (BR + HU) / 2 / 4;  // DMA instructions per wave per chunk (2 rows each)
    constexpr int EPI = RING * BUFB, A_OFF = EPI, CP_OFF = A_OFF + 64 * 128, DC_OFF = CP_OFF + 64 * 64,
                  DO_OFF = DC_OFF + 64 * 64, NEPI = 5;            // epilogue DMA instructions per wave
    static_assert(G4 % KCH == 0 && NCH >= 2 && NPS == 10, "H = 256 or 512");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    typedef __attribute__((address_space(3))) void* lds_p;

    const int16v_t lens = wave_rows_len16_issue(seq_len, b0, wave);   // rows 16w .. 16w+15

    const bf16* a_rows = dg_in + ((int64_t)dir * B + b0) * G4;
    const bf16* wdir = wh + ((int64_t)dir * H + u0) * G4;
    auto issue = [&](int c) {
        char* buf = lds + (c % RING) * BUFB;
#pragma unroll
        for (int i = 0; i < NPS; ++i) {
            const int ii = i * 4 + wave, r = 2 * ii + (lane >> 5);       // r < 64: dG row; else W_h row r - 64
            const bf16* src = r < BR ? a_rows + (int64_t)r * G4 : wdir + (int64_t)(r - BR) * G4;
            __builtin_amdgcn_global_load_lds((const void*)(src + c * KCH + 8 * ((lane & 31) ^ (r & 15))),
                                             (lds_p)(buf + 2 * ii * ROWB), 16, 0, 0);
        }
    };
    issue(0);
    issue(1);
    // epilogue operands of rows 16w.. (time row per sequence length)
    int plen;
    {
        int16v_t v = lens;
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v));
        auto pick = [&](int k) {
            int x = v[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) x = k == q ? v[q] : x;
            return x;
        };
        const int rb = b0 + wave * 16;
        // gate activations: 2 x 8 rows x 4 gates x 32 B
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int rr = i * 8 + (lane >> 3), t = step_time(dir, s, pick(rr));
            const bf16* src = acts_t + (((int64_t)t * B + rb + rr) * 2 + dir) * G4 + ((lane & 7) >> 1) * H + u0 +
                              (lane & 1) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_p)(lds + A_OFF + (wave * 16 + i * 8) * 128), 16,
                                             0, 0);
        }
        {   // c_prev (f32, 64 B per row) and the dc state
            const int rr = lane >> 2, t = step_time(dir, s, pick(rr));
            const float* src = cprev_t + (((int64_t)t * B + rb + rr) * 2 + dir) * H + u0 + (lane & 3) * 4;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_p)(lds + CP_OFF + wave * 16 * 64), 16, 0, 0);
            const float* dsrc = dc_state + ((int64_t)dir * B + rb + rr) * H + u0 + (lane & 3) * 4;
            __builtin_amdgcn_global_load_lds((const void*)dsrc, (lds_p)(lds + DC_OFF + wave * 16 * 64), 16, 0, 0);
        }
        {   // dout (bf16, 32 B per row): half a wave
            const int rr = (lane & 31) >> 1, t = step_time(dir, s, pick(rr));
            const bf16* src = dout + ((int64_t)t * B + rb + rr) * 2 * H + dir * H + u0 + (lane & 1) * 8;
            if (lane < 32)
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_p)(lds + DO_OFF + wave * 16 * 32), 16, 0, 0);
        }
        plen = pick(lane >> 2);                         // this thread's epilogue row 16w + lane/4
    }

    const int i16 = lane & 15, g = lane >> 4, sw = lane & 15;
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        // chunk c landed; younger: chunk c+1 (if any) and, for c <= 1, the epilogue moves
        const int younger = (c + 1 < NCH ? NPS : 0) + (c <= 1 ? NEPI : 0);
        if (younger == NPS + NEPI) vm_wait<NPS + NEPI>();
        else if (younger == NPS) vm_wait<NPS>();
        else if (younger == NEPI) vm_wait<NEPI>();
        else vm_wait<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                   // chunk c in for every wave; buffer (c+2)%3 is free
        if (c + 2 < NCH) issue(c + 2);
        const char* buf = lds + (c % RING) * BUFB;
        const char* ar[1] = {buf + (wave * 16 + i16) * ROWB};
        const char* br[1] = {buf + (BR + i16) * ROWB};
        floatx4 (&acc11)[1][1] = reinterpret_cast<floatx4 (&)[1][1]>(acc);
        lds_mma_16x16x32<KCH / 32, 1, 1, 4>(ar, br, g, sw, acc11);
    }
    vm_wait<0>();
    __syncthreads();                                    // epilogue operands in; every wave done with the ring
    LstmBwdOps<BR, HU> ops;
    static_assert(LstmBwdOps<BR, HU>::EPQ4 == 1 && LstmBwdOps<BR, HU>::UQ == 4, "one item per thread");
    {
        const int r = threadIdx.x / 4, u = 4 * (threadIdx.x % 4);
        ops.plen[0] = plen;
#pragma unroll
        for (int k = 0; k < 4; ++k) ld4(ops.pa[0][k], reinterpret_cast<const bf16*>(lds + A_OFF + r * 128 + k * 32 + u * 2));
        ld4(ops.pcp[0], reinterpret_cast<const float*>(lds + CP_OFF + r * 64 + u * 4));
        ld4(ops.pdc[0], reinterpret_cast<const float*>(lds + DC_OFF + r * 64 + u * 4));
        ld4(ops.pdo[0], reinterpret_cast<const bf16*>(lds + DO_OFF + r * 32 + u * 2));
    }
    float* sG = reinterpret_cast<float*>(lds);              // [BR][HU + 1], in ring buffer 0
#pragma unroll
    for (int r = 0; r < 4; ++r) sG[(wave * 16 + g * 4 + r) * (HU + 1) + i16] = acc[r];
    __syncthreads();
    ops.epilogue(sG, s, B, H, b0, u0, dir, dc_state, dg_out, dG_t);
}

// ------------------------------------------------------------------ C ABI
long long* g_lstm_dbg = nullptr;   // diagnostics only (ocrk_lstm_debug_stamps)

#ifdef OCRK_EXPERIMENTS
// include/ocrk_debug.h: exported by the tools-only build (make exp) alone
extern "C" int ocrk_lstm_debug_stamps(long long* buf) { g_lstm_dbg = buf; return OCRK_OK; }
#endif

// GEMM blocks (2 x 64 rows x 2H bytes) + gx tile (8 KB) + c tile (4 KB)
static constexpr int lstm_fwd_dma_lds(int H) { return 2 * 64 * 2 * H + 64 * 64 * 2 + 64 * 16 * 4; }
static bool lstm_dma_enabled() {
    const bool on = ocrk::opt(ocrk::OPT_LSTM_DMA) != 0;
    if (on) {
        static DeviceOnce a512, a256;
        set_dyn_lds(a512, reinterpret_cast<const void*>(&lstm_fwd_step_dma_kernel<512>), lstm_fwd_dma_lds(512));
        set_dyn_lds(a256, reinterpret_cast<const void*>(&lstm_fwd_step_dma_kernel<256>), lstm_fwd_dma_lds(256));
    }
    return on;
}

// Backward ring + epilogue operands: 138 KB of dynamic LDS. OCRK_LSTM_BWD_DMA=0 disables it
// (and a device that refuses the LDS limit falls back to the VGPR-staged kernel).
static bool lstm_bwd_dma_enabled() {
    if (!ocrk::opt(ocrk::OPT_LSTM_BWD_DMA)) return false;
    static DeviceOnce once;
    static bool ok[kMaxDevices];
    once_per_device(once, [] {
        hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_step_dma_kernel<512>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, LSTM_BWD_DMA_LDS);
        hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_step_dma_kernel<256>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, LSTM_BWD_DMA_LDS);
        ok[current_device()] = e1 == hipSuccess && e2 == hipSuccess;
    });
    return ok[current_device()];
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
                lstm_fwd_step_dma_kernel<512><<<grid, 256, lstm_fwd_dma_lds(512), st>>>((const bf16*)gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, g_lstm_dbg);
            else
                lstm_fwd_step_dma_kernel<256><<<grid, 256, lstm_fwd_dma_lds(256), st>>>((const bf16*)gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, (bf16*)out, (bf16*)hprev_t, cprev_t, (bf16*)acts_t, g_lstm_dbg);
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
        // fp32 BPTT: exact f32 MFMA in exact mode, else the bf16x3 split (the fp32 Trainer's
        // recurrent layers outside its conv tower, kernels.f32_exact)
        if (ocrk::f32_exact_mfma())
            lstm_bwd_step_kernel<BWD_F32><<<grid, 256, 0, st>>>((const float*)wh, (const float*)dg_in, (float*)dg_out, dc_state, seq_len, s, T, B, H, (const float*)dout, cprev_t, (const float*)acts_t, (float*)dG_t);
        else
            lstm_bwd_step_kernel<BWD_F32, true><<<grid, 256, 0, st>>>((const float*)wh, (const float*)dg_in, (float*)dg_out, dc_state, seq_len, s, T, B, H, (const float*)dout, cprev_t, (const float*)acts_t, (float*)dG_t);
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
