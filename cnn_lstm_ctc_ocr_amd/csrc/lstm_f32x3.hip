// a7' in fp32 (the reference's precision, src/weinman/model_bu.py:187-192; the
// serving path src/processing/server.py:78-145 runs the graph in float32): the
// BiLSTM forward time loop as ONE persistent launch per layer, with the
// recurrent product h_{s-1} . W_h on the bf16 MFMA through the bf16x3 split
// (mfma_util.h split2_bf16: ah.bh + ah.bl + al.bh, ~2^-16 relative per product,
// f32 accumulation) -- the per-step fp32 kernels (csrc/lstm.hip) took 8.3 us
// per step on the f32 MFMA plus a launch each.
//
// Work split (H = 512): 2 directions x B/RB batch slices = groups (RB = 16 rows
// when that grid is co-resident, B <= 128, else 32), each of 16 member
// workgroups owning 32 hidden units (as lstm_persistent.hip), but 8 waves: wave w owns units 4w..4w+3 x 4 gates = one 16-column MFMA N-tile, its
// W_h^T slice split once into hi / lo bf16 B fragments resident in VGPRs (2 x 16
// k-steps x 4 VGPRs = 128). Per step a member
//   1. waits until the group published h_{s-1} (flag words, bounded spin);
//   2. stages the group's h_{s-1} rows as TWO bf16 planes (hi, lo: each
//      producer split its own h once) -- 64 rows of 1 KB, one LDS-DMA wave
//      instruction each, 8 per wave -- and behind them its gx loads (fp32, the
//      bias is in gx: the projection GEMM's epilogue);
//   3. runs 16 k-steps x 2 M-tiles x 3 v_mfma_f32_16x16x32_bf16 per wave;
//   4. the cell update in fp32 (2 units of one row per thread), c and h kept
//      in fp32 registers;
//   5. publishes h_s as its hi / lo split (4-B stores per plane), drains,
//      barriers, one lane raises the member flag;
//   6. writes the fp32 layer output (zeros past the row's length) and, when
//      asked (training), the tensors the BPTT reads.
// The hand-off form, the XCC census and the counting flag words are
// persist.h's, exactly as the bf16 loop uses them.
#include "common.h"
#include "mfma_util.h"
#include "persist.h"
#include "recur.h"

using namespace ocrk;

namespace {

__device__ __forceinline__ void put4(gu32* p, unsigned v, bool local) {
    if (local) *p = v;
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int X3_KS = 16;                       // H = 512
constexpr int X3_THREADS = 512;

}  // namespace

// RB = batch rows per group slice: 32, or 16 when the grid 2 (B/16) (H/32) still
// fits one workgroup per CU (B <= 128 at H = 512) -- half the staged rows and half
// the MFMAs per member per step (one M-tile), on twice the CUs.
template <int RB>
__global__ void __launch_bounds__(X3_THREADS, 1)
lstm_fwd_persistent_f32x3_kernel(const float* __restrict__ gx, const float* __restrict__ whT,
                                 unsigned short* __restrict__ hx, const int* __restrict__ seq_len, int T, int B,
                                 float* __restrict__ out, float* __restrict__ hprev_t, float* __restrict__ cprev_t,
                                 float* __restrict__ acts_t, unsigned* __restrict__ flags,
                                 unsigned* __restrict__ err, unsigned spin_limit) {
    static_assert(RB == 16 || RB == 32, "row slices of 16 or 32");
    constexpr int KS = X3_KS;
    constexpr int H = KS * 32;
    constexpr int G4 = 4 * H;
    constexpr int NU = H / PHU;                         // members per group (16)
    constexpr int MT = RB / 16;                         // MFMA M-tiles per member
    constexpr int LDH = H + 8;                          // padded staged row (bf16 elements)
    constexpr int LDG = 4 * PHU + 4;                    // padded gate row (floats)
    constexpr int CELLS = RB * 16;                      // cell threads: (row, 2 units) each
    constexpr int DPW = 2 * RB / 8;                     // staging DMAs per wave (both planes)
    __shared__ __attribute__((aligned(16))) unsigned short sh[2 * RB * LDH];     // [hi | lo][row][k]
    __shared__ __attribute__((aligned(16))) float sG[RB * LDG];                  // [row][gate][unit]

    int group, member;
    persistent_role(2 * (B / RB), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * PHU, b0 = bs * RB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);

    // ---- resident B fragments, split once: N-tile column c = gate (c >> 2) of unit 4w + (c & 3)
    bf16x8 bh[KS], bl[KS];
    {
        const float* row = whT + (size_t)dir * G4 * H + (size_t)((c >> 2) * H + u0 + 4 * w + (c & 3)) * H + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            V8<float> v;
            vload(v, row + ks * 32);
            u32x4 hi, lo;
            split8_bf16(v, hi, lo);
            bh[ks] = __builtin_bit_cast(bf16x8, hi);
            bl[ks] = __builtin_bit_cast(bf16x8, lo);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(bh[ks]), "v"(bl[ks]));   // settled before the loop
    }

    // ---- the cell item of this thread (tid < CELLS): row er, units eu, eu + 1 (all 4 gates)
    const bool cell = tid < CELLS;
    const int er = cell ? tid >> 4 : 0, eu = 2 * (tid & 15);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));
    float cst[2] = {0.f, 0.f}, hst[2] = {0.f, 0.f};

    const int64_t hx_plane = (int64_t)2 * 2 * B * H;    // elements per plane ([parity][dir][B][H])
    auto hx_rsrc = __builtin_amdgcn_make_buffer_rsrc(hx, 0, (int)(2 * hx_plane * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t gx_rsrc = uniform_rsrc(gx, (int64_t)T * B * 2 * G4 * 4);
    const bool save = hprev_t != nullptr;

    for (int s = 0; s < T; ++s) {
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        float gxv[4][2];
        auto load_gx = [&]() {                           // 4 buffer loads (out of range reads 0 when idle)
            const int64_t e = (((int64_t)t * B + b0 + er) * 2 + dir) * G4 + u0 + eu;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x2_t v = __builtin_bit_cast(
                    f32x2_t, __builtin_amdgcn_raw_buffer_load_b64(gx_rsrc, (int)((e + q * H) * 4), 0, 0));
                gxv[q][0] = v[0];
                gxv[q][1] = v[1];
            }
        };
        floatx4 acc[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (s > 0) {
            // 1. wait until every member of the group published h_{s-1} (flag >= base + s)
            if (w == 0) {
                unsigned spins = 0;
                while (true) {
                    unsigned f = base + (unsigned)s;
                    if (lane < NU) f = poll_word(gflags + lane, local);
                    if (__all(reached(f, base + (unsigned)s))) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > spin_limit) {
                        if (lane == 0) __hip_atomic_fetch_or(err, (unsigned)OCRK_STATUS_LSTM_FWD_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            // 2. stage both planes of h_{s-1}: row r of plane p is one 1-KB LDS-DMA wave instruction
            const int64_t hbase = ((int64_t)(((s - 1) & 1) * 2 + dir) * B + b0) * H;
            const int wu = __builtin_amdgcn_readfirstlane(w);
            const unsigned lo16 = (unsigned)(lane * 16);
#define X3_STAGE(AUX)                                                                                  \
    _Pragma("unroll") for (int q = 0; q < DPW; ++q) {                                                 \
        const int pr = wu * DPW + q, plane = pr / RB, r = pr % RB;                                    \
        const unsigned off = (unsigned)(((int64_t)plane * hx_plane + hbase + (int64_t)r * H) * 2) + lo16; \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                     \
            hx_rsrc, (__attribute__((address_space(3))) void*)(sh + (plane * RB + r) * LDH), 16, off, 0, 0, AUX); \
    }
            if (local) { X3_STAGE(2) }                           // nt: the group's XCD L2
            else { X3_STAGE(16) }                                // sc1: any placement
#undef X3_STAGE
            asm volatile("" ::: "memory");
            load_gx();                                          // 4 loads behind the staging DMAs
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            __syncthreads();
            // 3. gates += h_{s-1} . W_h on the bf16x3 split
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const unsigned short* ap = &sh[(16 * mt + c) * LDH + ks * 32 + 8 * g];
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ap);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(ap + RB * LDH);
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[ks], acc[mt], 0, 0, 0);
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[ks], acc[mt], 0, 0, 0);
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[ks], acc[mt], 0, 0, 0);
                }
            }
        } else {
            load_gx();
        }
        // 4. gate pre-activations through LDS: lane (c, g) holds rows 16 mt + 4 g + r of column c
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sG[(16 * mt + 4 * g + r) * LDG + (c >> 2) * PHU + 4 * w + (c & 3)] = acc[mt][r];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // gx landed
        __syncthreads();

        // 5. the cell update of (row er, units eu, eu + 1)
        float a4[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x2_t z = *reinterpret_cast<const f32x2_t*>(&sG[er * LDG + q * PHU + eu]);
            a4[q][0] = z[0] + gxv[q][0];
            a4[q][1] = z[1] + gxv[q][1];
        }
        float hn[2], cp[2], hp[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float ai = sig_fast(a4[0][e]);
            const float aj = tanh_fast(a4[1][e]);
            const float af = sig_fast(a4[2][e] + 1.0f);         // forget_bias = 1
            const float ao = sig_fast(a4[3][e]);
            const float cn = af * cst[e] + ai * aj;
            const float h = ao * tanh_fast(cn);
            a4[0][e] = valid ? ai : 0.f; a4[1][e] = valid ? aj : 0.f;
            a4[2][e] = valid ? af : 0.f; a4[3][e] = valid ? ao : 0.f;
            cp[e] = valid ? cst[e] : 0.f;
            hp[e] = valid ? hst[e] : 0.f;
            if (valid) { cst[e] = cn; hst[e] = h; }
            hn[e] = hst[e];                                     // published state (carried when invalid)
        }

        // 6. publish h_s as its hi / lo split (one 4-B store per plane), drain, barrier, flag
        if (cell) {
            unsigned hi, lo;
            split2_bf16(hn[0], hn[1], hi, lo);
            const int64_t o = ((int64_t)((s & 1) * 2 + dir) * B + b0 + er) * H + u0 + eu;
            put4((gu32*)(hx + o), hi, local);
            put4((gu32*)(hx + hx_plane + o), lo, local);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(s + 1), local);

        // 7. the layer output (zeros past the length) and, for the BPTT, the saved tensors
        if (cell) {
            const f32x2_t ov = {valid ? hn[0] : 0.f, valid ? hn[1] : 0.f};
            *reinterpret_cast<f32x2_t*>(out + ((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu) = ov;
            if (save) {
                const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
                *reinterpret_cast<f32x2_t*>(hprev_t + tb * H + u0 + eu) = f32x2_t{hp[0], hp[1]};
                *reinterpret_cast<f32x2_t*>(cprev_t + tb * H + u0 + eu) = f32x2_t{cp[0], cp[1]};
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<f32x2_t*>(acts_t + tb * G4 + q * H + u0 + eu) = f32x2_t{a4[q][0], a4[q][1]};
            }
        }
    }
}

// rows per member for batch B: 16 when that grid is co-resident, else 32
template <int RB>
static bool x3_fits(int B, int H, int cus) {
    int per_cu = 0;
    if (B % RB ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_fwd_persistent_f32x3_kernel<RB>, X3_THREADS, 0) !=
            hipSuccess)
        return false;
    return 2L * (B / RB) * (H / PHU) <= (long)cus * per_cu;
}

static int x3_rows(int B, int H) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (x3_fits<16>(B, H, cus)) return 16;
    if (x3_fits<32>(B, H, cus)) return 32;
    return 0;
}

// ------------------------------------------------------------------ C ABI
extern "C" size_t ocrk_lstm_fwd_persistent_f32_workspace_size(int B, int H) {
    // flag word + XCC word per workgroup at 16-row slices (the larger count; 128-B block),
    // then the hi / lo h exchange planes
    const size_t counters = ((size_t)2 * 2 * (B / 16) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128;
    return counters + (size_t)2 * 2 * 2 * B * H * sizeof(unsigned short);
}

// the counting hand-off words of this loop (sized for 16-row slices)
extern "C" size_t ocrk_lstm_fwd_persistent_f32_flags_size(int B, int H) {
    return (B > 0 && B % 16 == 0 && H > 0 && H % PHU == 0)
               ? ((size_t)2 * 2 * (B / 16) * (H / PHU) * sizeof(unsigned) + 127) / 128 * 128 : 0;
}

extern "C" int ocrk_lstm_fwd_persistent_f32_supported(int B, int H) {
    if (B <= 0 || H != 32 * X3_KS) return 0;
    return x3_rows(B, H) ? 1 : 0;
}

extern "C" int ocrk_lstm_fwd_persistent_f32(const float* gx, const float* whT, const int* seq_len, int T, int B,
                                            int H, float* out, float* hprev_t, float* cprev_t, float* acts_t,
                                            unsigned* err, unsigned* flags, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_fwd_persistent_f32_supported(B, H),
                 "ocrk_lstm_fwd_persistent_f32: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_fwd_persistent_f32_workspace_size(B, H),
                 "ocrk_lstm_fwd_persistent_f32: workspace too small");
    OCRK_REQUIRE(gx && whT && seq_len && out && err, "ocrk_lstm_fwd_persistent_f32: null operand");
    OCRK_REQUIRE(!hprev_t == !cprev_t && !hprev_t == !acts_t,
                 "ocrk_lstm_fwd_persistent_f32: hprev_t, cprev_t, acts_t all or none");
    OCRK_REQUIRE((int64_t)T * B * 8 * H * 4 < 0x7fffffffll, "ocrk_lstm_fwd_persistent_f32: gx exceeds 2 GB");
    OCRK_REQUIRE(T >= 1, "ocrk_lstm_fwd_persistent_f32: T=%d", T);
    hipStream_t st = ocrk::as_stream(stream);
    const size_t counters = ocrk_lstm_fwd_persistent_f32_flags_size(B, H);
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    unsigned short* hx = (unsigned short*)((char*)ws + counters);
    if (!flags && hipMemsetAsync(cnt, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_lstm_fwd_persistent_f32 memset");
    const int rb = x3_rows(B, H);
    const unsigned grid = 2u * (unsigned)(B / rb) * (unsigned)(H / PHU);
    if (rb == 16)
        lstm_fwd_persistent_f32x3_kernel<16><<<grid, X3_THREADS, 0, st>>>(gx, whT, hx, seq_len, T, B, out, hprev_t,
                                                                         cprev_t, acts_t, cnt, err, recur_spin_limit());
    else
        lstm_fwd_persistent_f32x3_kernel<32><<<grid, X3_THREADS, 0, st>>>(gx, whT, hx, seq_len, T, B, out, hprev_t,
                                                                         cprev_t, acts_t, cnt, err, recur_spin_limit());
    return ocrk::launch_status("ocrk_lstm_fwd_persistent_f32");
}
