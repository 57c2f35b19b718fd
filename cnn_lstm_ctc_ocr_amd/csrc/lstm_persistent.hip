// a7': the BiLSTM forward time loop as ONE persistent launch per layer
// (rnn_layer, src/weinman/model_bu.py:167-199; [TF1] LSTMCell i, j, f, o,
// forget_bias 1; bidirectional_dynamic_rnn with sequence_length).
//
// Work split (bf16, B = 256, H = 512): 256 workgroups = 2 directions x B/32
// batch slices x H/32 unit slices, one per CU, all co-resident. A workgroup
// owns 32 hidden units (x 4 gates = 128 gate columns) of one direction for 32
// batch rows. Its W_h^T slice [128 x H] stays in VGPRs for the whole
// sequence as MFMA B fragments (wave w: units 8w..8w+7, 4 gates = two 16-col
// tiles, all H/32 k-steps: 128 VGPRs). Per step the workgroup
//   1. waits until the 16 workgroups of its (direction, batch slice) group
//      published h_{s-1} (one agent-scope counter per group, polled by one lane),
//   2. stages h_{s-1}[32 x H] into LDS with write-through (sc1) loads,
//   3. runs 2 x 2 tiles x H/32 k-steps of v_mfma_f32_16x16x32_bf16 per wave,
//   4. finishes the gates wave-locally (lane l and l^8 hold the i/j and f/o
//      halves of the same unit: two shuffles), keeps c in registers,
//   5. writes h_s as sc1 stores (4-B pairs), the layer output and the saved
//      tensors for the backward pass, drains, barriers, and one lane adds 1 to
//      the group counter.
// Hand-off form: MI355X_MICROARCH.md "Valid forms" row 1 (sc1 payload stores,
// every storing wave drained before the barrier, one lane's agent atomic add;
// consumer: sc1 poll, barrier, every payload load sc1). Spins are bounded: on
// timeout the kernel records an error word and finishes (no hang).
#include "common.h"
#include "mfma_util.h"

using namespace ocrk;

namespace {

constexpr int PBR = 32, PHU = 32;          // batch rows, hidden units per workgroup
constexpr unsigned SPIN_LIMIT = 1u << 22;  // polls (with s_sleep) before giving up

__device__ __forceinline__ int step_time_p(int dir, int s, int len) {
    return (dir == 0 || s >= len) ? s : len - 1 - s;
}
__device__ __forceinline__ float sigf(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) { return 2.f / (1.f + __expf(-2.f * x)) - 1.f; }

__device__ __forceinline__ unsigned short bf16_bits(float x) {
    bf16 b = (bf16)x;
    return __builtin_bit_cast(unsigned short, b);
}

// diagnostics (ocrk_lstm_debug_stamps): thread 0 stamps step S_DBG
__device__ __forceinline__ void pstamp(long long* dbg, int s, int i) {
    if (dbg && threadIdx.x == 0 && s == 64) {
        dbg[(((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + i] =
            __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace

extern long long* g_lstm_dbg;

// KS = H / 32 k-steps
template <int KS>
__global__ void __launch_bounds__(256, 1)
lstm_fwd_persistent_kernel(const bf16* __restrict__ gx, const bf16* __restrict__ whT, bf16* __restrict__ hx,
                           const int* __restrict__ seq_len, int T, int B, bf16* __restrict__ out,
                           bf16* __restrict__ hprev_t, float* __restrict__ cprev_t, bf16* __restrict__ acts_t,
                           unsigned* __restrict__ cnt, unsigned* __restrict__ err, long long* __restrict__ dbg) {
    constexpr int H = KS * 32;
    constexpr int G4 = 4 * H;
    constexpr int LDH = H + 8;                          // padded LDS row (bf16 elements)
    __shared__ __attribute__((aligned(16))) unsigned short sh[PBR * LDH];
    // per-step output staging (row-contiguous 32-unit pieces)
    __shared__ __attribute__((aligned(16))) unsigned short so_h[PBR * PHU], so_out[PBR * PHU], so_hp[PBR * PHU];
    __shared__ __attribute__((aligned(16))) float so_cp[PBR * PHU];
    __shared__ __attribute__((aligned(16))) unsigned short so_a[PBR * 4 * PHU];
    __shared__ int s_t[PBR], s_valid[PBR], s_len[PBR];

    const int us = blockIdx.x, bs = blockIdx.y, dir = blockIdx.z;
    const int nu = gridDim.x;                           // workgroups per group
    const int u0 = us * PHU, b0 = bs * PBR;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int my_unit = u0 + 8 * w + (c & 7);           // the unit this lane finishes
    unsigned* my_cnt = cnt + dir * gridDim.y + bs;

    // ---- resident B fragments: N-tile j holds gates 2j + (c >> 3) of unit my_unit
    bf16x8 bw[2][KS];
    const bf16* wdir = whT + (size_t)dir * G4 * H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bf16* row = wdir + (size_t)((2 * j + (c >> 3)) * H + my_unit) * H + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + ks * 32);
    }

    // ---- the 4 (row, unit) pairs this lane finishes: M-tile mt, register r
    // lanes c < 8 take registers r = 0,1; lanes c >= 8 take r = 2,3
    const int rbase = (c >= 8) ? 2 : 0;
    int prow[4], plen[4];
    float cst[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int mt = p >> 1, r = rbase + (p & 1);
        prow[p] = b0 + 16 * mt + 4 * g + r;
        plen[p] = seq_len[prow[p]];
        cst[p] = 0.f;
    }
    float hst[4] = {0.f, 0.f, 0.f, 0.f};
    if (tid < PBR) s_len[tid] = seq_len[b0 + tid];
    static_assert(PHU == 32 && PBR == 32, "staging index math assumes 32 x 32 tiles");

    // buffer resources for the sc1 hand-off traffic
    const int64_t hx_elems = (int64_t)2 * 2 * B * H;
    auto hx_rsrc = __builtin_amdgcn_make_buffer_rsrc(hx, 0, (int)(hx_elems * 2), 0x00020000);

    for (int s = 0; s < T; ++s) {
        pstamp(dbg, s, 0);
        // epilogue operands first: they do not depend on h
        float pg[4][4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int t = step_time_p(dir, s, plen[p]);
            const bf16* gp = gx + (((int64_t)t * B + prow[p]) * 2 + dir) * G4 + my_unit;
#pragma unroll
            for (int k = 0; k < 4; ++k) pg[p][k] = (float)gp[k * H];
        }

        floatx4 acc[2][2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};

        if (s > 0) {
            // 1. wait for the group's h_{s-1}
            if (tid == 0) {
                const unsigned target = (unsigned)nu * (unsigned)s;
                unsigned spins = 0;
                while (__hip_atomic_load(my_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > SPIN_LIMIT) {
                        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            pstamp(dbg, s, 1);
            // 2. stage h_{s-1} rows (sc1 loads: the bytes were written through by other CUs)
            const int64_t base = ((int64_t)(((s - 1) & 1) * 2 + dir) * B + b0) * H;
#pragma unroll
            for (int v = 0; v < PBR * H / 8 / 256; ++v) {
                const int idx = tid + 256 * v;
                const int row = idx / (H / 8), kq = idx % (H / 8);
                const int off = (int)((base + (int64_t)row * H + 8 * kq) * 2);
                u32x4 q = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(hx_rsrc, off, 0, 16));
                *reinterpret_cast<u32x4*>(&sh[row * LDH + 8 * kq]) = q;
            }
            __syncthreads();
            pstamp(dbg, s, 2);
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

        pstamp(dbg, s, 3);
        // 4. gates for (row, unit): lane c < 8 holds i (tile 0) and f (tile 1),
        //    lane c ^ 8 holds j and o of the same unit and rows. Results go to
        //    LDS staging rows [32 rows][32 units] so the stores leave as 16-B pieces.
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float x0 = __shfl_xor(acc[mt][0][r], 8, 64);
                const float x1 = __shfl_xor(acc[mt][1][r], 8, 64);
                if ((r >> 1) == (rbase >> 1)) {          // this lane's register pair
                    const int p = mt * 2 + (r & 1);
                    const float gi = (c < 8) ? acc[mt][0][r] : x0;
                    const float gj = (c < 8) ? x0 : acc[mt][0][r];
                    const float gf = (c < 8) ? acc[mt][1][r] : x1;
                    const float go = (c < 8) ? x1 : acc[mt][1][r];
                    const bool valid = s < plen[p];
                    const float ai = sigf(gi + pg[p][0]);
                    const float aj = tanhf_(gj + pg[p][1]);
                    const float af = sigf(gf + pg[p][2] + 1.0f);      // forget_bias = 1
                    const float ao = sigf(go + pg[p][3]);
                    const float cn = af * cst[p] + ai * aj;
                    const float hn = ao * tanhf_(cn);
                    const int lr = prow[p] - b0, lu = my_unit - u0;
                    so_h[lr * PHU + lu] = bf16_bits(valid ? hn : hst[p]);      // published state
                    so_out[lr * PHU + lu] = bf16_bits(valid ? hn : 0.f);
                    so_hp[lr * PHU + lu] = bf16_bits(valid ? hst[p] : 0.f);
                    so_cp[lr * PHU + lu] = valid ? cst[p] : 0.f;
                    so_a[(lr * 4 + 0) * PHU + lu] = bf16_bits(valid ? ai : 0.f);
                    so_a[(lr * 4 + 1) * PHU + lu] = bf16_bits(valid ? aj : 0.f);
                    so_a[(lr * 4 + 2) * PHU + lu] = bf16_bits(valid ? af : 0.f);
                    so_a[(lr * 4 + 3) * PHU + lu] = bf16_bits(valid ? ao : 0.f);
                    if (valid) { cst[p] = cn; hst[p] = hn; }
                }
            }
        if (tid < PBR) {
            const int len = s_len[tid];
            s_t[tid] = step_time_p(dir, s, len);
            s_valid[tid] = s < len;
        }
        __syncthreads();
        pstamp(dbg, s, 4);

        // 5. publish h_s (32 rows x 64 B, sc1), drain, barrier, one lane signals
        const int64_t obase = (int64_t)((s & 1) * 2 + dir) * B * H;
        if (tid < PBR * PHU / 8) {
            const int lr = tid / (PHU / 8), q = tid % (PHU / 8);
            const u32x4 v = *reinterpret_cast<const u32x4*>(&so_h[lr * PHU + 8 * q]);
            const int off = (int)((obase + (int64_t)(b0 + lr) * H + u0 + 8 * q) * 2);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), hx_rsrc, off, 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pstamp(dbg, s, 5);
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pstamp(dbg, s, 6);

        // 6. the rest (layer output + saved tensors) drains behind the next step
        //    pieces: out 128, hprev 128, cprev 256, acts 512 (16 B each) = 4 per thread
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int id = tid + 256 * v;
            if (id < 128) {                                           // out [t][b][2H]
                const int lr = id / 4, q = id % 4;
                const int64_t o = ((int64_t)s_t[lr] * B + b0 + lr) * 2 * H + dir * H + u0 + 8 * q;
                if (s_valid[lr]) *reinterpret_cast<u32x4*>(out + o) = *reinterpret_cast<const u32x4*>(&so_out[lr * PHU + 8 * q]);
            } else if (id < 256) {                                    // hprev [t][b][2][H]
                const int lr = (id - 128) / 4, q = (id - 128) % 4;
                const int64_t o = (((int64_t)s_t[lr] * B + b0 + lr) * 2 + dir) * H + u0 + 8 * q;
                *reinterpret_cast<u32x4*>(hprev_t + o) = *reinterpret_cast<const u32x4*>(&so_hp[lr * PHU + 8 * q]);
            } else if (id < 512) {                                    // cprev [t][b][2][H] f32
                const int lr = (id - 256) / 8, q = (id - 256) % 8;
                const int64_t o = (((int64_t)s_t[lr] * B + b0 + lr) * 2 + dir) * H + u0 + 4 * q;
                *reinterpret_cast<f32x4*>(cprev_t + o) = *reinterpret_cast<const f32x4*>(&so_cp[lr * PHU + 4 * q]);
            } else {                                                  // acts [t][b][2][4H]
                const int k = id - 512, lr = k / 16, gq = k % 16, gate = gq / 4, q = gq % 4;
                const int64_t o = (((int64_t)s_t[lr] * B + b0 + lr) * 2 + dir) * G4 + gate * H + u0 + 8 * q;
                *reinterpret_cast<u32x4*>(acts_t + o) = *reinterpret_cast<const u32x4*>(&so_a[(lr * 4 + gate) * PHU + 8 * q]);
            }
        }
    }
}

// ------------------------------------------------------------------ C ABI
extern "C" size_t ocrk_lstm_fwd_persistent_workspace_size(int B, int H) {
    // group counters (16-B aligned block) + error word, then the h exchange buffer
    size_t counters = ((size_t)2 * (B / PBR) * sizeof(unsigned) + 16 + 15) / 16 * 16;
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

extern "C" int ocrk_lstm_fwd_persistent(const void* gx, const void* whT, const int* seq_len, int T, int B, int H,
                                        void* out, void* hprev_t, float* cprev_t, void* acts_t, unsigned* err,
                                        void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_fwd_persistent_supported(B, H), "ocrk_lstm_fwd_persistent: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_fwd_persistent_workspace_size(B, H), "ocrk_lstm_fwd_persistent: workspace too small");
    hipStream_t st = ocrk::as_stream(stream);
    size_t counters = ((size_t)2 * (B / PBR) * sizeof(unsigned) + 16 + 15) / 16 * 16;
    unsigned* cnt = (unsigned*)ws;
    bf16* hx = (bf16*)((char*)ws + counters);
    if (hipMemsetAsync(cnt, 0, counters, st) != hipSuccess) return ocrk::launch_status("ocrk_lstm_fwd_persistent memset");
    dim3 grid(H / PHU, B / PBR, 2);
    if (H == 512)
        lstm_fwd_persistent_kernel<16><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out,
                                                             (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err, g_lstm_dbg);
    else
        lstm_fwd_persistent_kernel<8><<<grid, 256, 0, st>>>((const bf16*)gx, (const bf16*)whT, hx, seq_len, T, B, (bf16*)out,
                                                            (bf16*)hprev_t, cprev_t, (bf16*)acts_t, cnt, err, g_lstm_dbg);
    return ocrk::launch_status("ocrk_lstm_fwd_persistent");
}
