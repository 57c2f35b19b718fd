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

// ---------------------------------------------------------------- backward
// The fp32 BPTT as ONE persistent launch per layer on the same split: member
// (direction, 32-row batch slice, 32 units) of the gather form (grid B), 8 waves:
// wave w takes gate w >> 1 and k-half w & 1 (256 of the gate's 512 dz columns),
// its W_h slice [32 units][256 k] split once into resident hi / lo B fragments
// (2 N-tiles x 8 k-steps x 2 planes = 128 VGPRs). Per reverse step a member
//   1. waits until the group published dz_{i-1} (flag words, bounded spin);
//   2. stages ITS 16 rows x 256 columns of dz_{i-1} hi and lo (16 LDS-DMA wave
//      instructions of two unpadded 512-B rows, 16-B pieces XOR-swizzled by row
//      on the global side) for M-tile 0, multiplies them (3 bf16 MFMAs per
//      product), then the same rows 16-31 into the same 16 KB for M-tile 1:
//      the two planes of 32 rows (32 KB per wave) do not fit beside each other
//      in LDS, so the tiles are staged in turn; the cell's operands (acts,
//      c_prev, dout: fp32) ride behind the first tile's DMA;
//   3. the eight K-slice partials meet in LDS (each wave's own staging region,
//      free after its MFMAs) and are summed in a fixed order;
//   4. the cell's gradient in fp32 (2 units of one row per thread), dc kept in
//      registers, bias partials summed over the steps;
//   5. publishes dz as its hi / lo split (4-B stores per plane), drains,
//      barriers, one lane raises the member flag; writes dz (fp32) in time order.
// Hand-off form, census and counting flags: persist.h's, as every loop here.
__global__ void __launch_bounds__(512, 1)
lstm_bwd_persistent_f32x3_kernel(const float* __restrict__ wh, unsigned short* __restrict__ dzx,
                                 const int* __restrict__ seq_len, int T, int B, const float* __restrict__ dout,
                                 const float* __restrict__ cprev_t, const float* __restrict__ acts_t,
                                 float* __restrict__ dG_t, unsigned* __restrict__ flags, unsigned* __restrict__ err,
                                 unsigned spin_limit, float* __restrict__ bpart) {
    constexpr int H = 32 * X3_KS, G4 = 4 * H;
    constexpr int RB = PBR, UM = PHU;                   // 32 rows x 32 units per member
    constexpr int NU = H / UM;                          // members per group (16)
    constexpr int KW = 256, KSW = KW / 32;              // k columns / k-steps per wave
    constexpr int REG = 2 * 16 * KW;                    // elements per wave region: [plane][16 rows][256]
    constexpr int LDP = UM + 4;                         // partial row pitch (floats)
    static_assert(RB * LDP * 4 <= REG * 2, "the partials fit the wave's staging region");
    __shared__ __attribute__((aligned(16))) unsigned short sA[8 * REG];

    int group, member;
    persistent_role(2 * (B / RB), NU, group, member);
    const int dir = group & 1, bs = group >> 1;
    const int u0 = member * UM, b0 = bs * RB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int kbase = (w >> 1) * H + (w & 1) * KW;
    gu32* gflags = (gu32*)(flags) + group * NU;
    unsigned base;
    const bool local = persistent_setup((gu32*)flags, group, NU, member, err, spin_limit, base);

    // resident B fragments, split once: N-tile j = units u0 + 16 j + c; k = kbase + 32 ks + 8 g
    bf16x8 bh[2][KSW], bl[2][KSW];
    const float* wdir = wh + (size_t)dir * H * G4;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float* row = wdir + (size_t)(u0 + 16 * j + c) * G4 + kbase + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KSW; ++ks) {
            V8<float> v;
            vload(v, row + ks * 32);
            u32x4 hi, lo;
            split8_bf16(v, hi, lo);
            bh[j][ks] = __builtin_bit_cast(bf16x8, hi);
            bl[j][ks] = __builtin_bit_cast(bf16x8, lo);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < KSW; ++ks) asm volatile("" ::"v"(bh[j][ks]), "v"(bl[j][ks]));   // settled before the loop

    // the cell item: row er, units eu, eu + 1 (all 4 gates)
    const int er = tid >> 4, eu = 2 * (tid & 15);
    const int elen = seq_len[b0 + er];
    asm volatile("" ::"v"(elen));
    float dcs[2] = {0.f, 0.f};
    float bsum[4][2] = {};
    const int64_t plane = (int64_t)2 * 2 * B * G4;      // elements per exchange plane ([parity][dir][B][4H])
    auto zx_rsrc = __builtin_amdgcn_make_buffer_rsrc(dzx, 0, (int)(2 * plane * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t act_rsrc = uniform_rsrc(acts_t, (int64_t)T * B * 2 * G4 * 4);
    const __amdgpu_buffer_rsrc_t cp_rsrc = uniform_rsrc(cprev_t, (int64_t)T * B * 2 * H * 4);
    const __amdgpu_buffer_rsrc_t do_rsrc = uniform_rsrc(dout, (int64_t)T * B * 2 * H * 4);
    // DMA lane geometry: instruction d covers rows 2d, 2d + 1 of a 16-row tile;
    // lane l writes row 2d + (l >> 5), slot l & 31, fetching the global 16-B piece
    // (l & 31) ^ (row & 15) of that row's wave columns
    const int wu = __builtin_amdgcn_readfirstlane(w);
    unsigned short* sa = sA + wu * REG;
    unsigned dma_off[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const int r = 2 * d + (lane >> 5);
        dma_off[d] = (unsigned)((r * G4 + kbase + 8 * ((lane & 31) ^ (r & 15))) * 2);
    }
    typedef __attribute__((address_space(3))) void* lds_p;

    for (int i = 0; i < T; ++i) {
        const int s = T - 1 - i;
        const bool valid = s < elen;
        const int t = step_time(dir, s, elen);
        const int64_t tb = ((int64_t)t * B + b0 + er) * 2 + dir;
        f32x2_t la[4], lcp, ldo;
        auto load_late = [&]() {                        // 6 buffer loads
#pragma unroll
            for (int k = 0; k < 4; ++k)
                la[k] = __builtin_bit_cast(
                    f32x2_t, __builtin_amdgcn_raw_buffer_load_b64(act_rsrc, (int)((tb * G4 + k * H + u0 + eu) * 4), 0, 0));
            lcp = __builtin_bit_cast(f32x2_t, __builtin_amdgcn_raw_buffer_load_b64(cp_rsrc, (int)((tb * H + u0 + eu) * 4), 0, 0));
            ldo = __builtin_bit_cast(f32x2_t, __builtin_amdgcn_raw_buffer_load_b64(
                do_rsrc, (int)((((int64_t)t * B + b0 + er) * 2 * H + dir * H + u0 + eu) * 4), 0, 0));
        };
        floatx4 acc[2][2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[m][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (i > 0) {
            // 1. wait until every member of the group published dz_{i-1} (flag >= base + i)
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
            const unsigned rb0 = (unsigned)(((int64_t)(((i - 1) & 1) * 2 + dir) * B + b0) * G4 * 2);
            // 2. the two 16-row M-tiles of this wave's 256 columns, hi and lo planes, in turn
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const unsigned rbm = rb0 + (unsigned)(16 * m * G4 * 2);
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) {
                    const unsigned poff = rbm + (unsigned)(pl * plane * 2);
                    if (local) {
#pragma unroll
                        for (int d = 0; d < 8; ++d)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(zx_rsrc, (lds_p)(sa + pl * 16 * KW + d * 2 * KW), 16,
                                                                     poff + dma_off[d], 0, 0, 2);
                    } else {
#pragma unroll
                        for (int d = 0; d < 8; ++d)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(zx_rsrc, (lds_p)(sa + pl * 16 * KW + d * 2 * KW), 16,
                                                                     poff + dma_off[d], 0, 0, 16);
                    }
                }
                asm volatile("" ::: "memory");
                if (m == 0) {
                    load_late();                                 // 6 loads behind the first tile's 16 DMAs
                    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int ks = 0; ks < KSW; ++ks) {
                    const int so = c * KW + 8 * ((4 * ks + g) ^ c);
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&sa[so]);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(&sa[16 * KW + so]);
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j][ks], acc[m][j], 0, 0, 0);
                        acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j][ks], acc[m][j], 0, 0, 0);
                        acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j][ks], acc[m][j], 0, 0, 0);
                    }
                }
                // the tile's reads are in registers before the next tile's DMA into the same bytes
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
        } else {
            load_late();
        }
        // 3. the eight partials meet in LDS (each wave's own region): lane (c, g) holds
        //    rows 16 m + 4 g + r of units 16 j + c
        float* sP = reinterpret_cast<float*>(sa);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) sP[(16 * m + 4 * g + r) * LDP + 16 * j + c] = acc[m][j][r];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the cell's operands landed
        __syncthreads();

        // 4. the cell's gradient for (row er, units eu, eu + 1)
        float dz[4][2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float p[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) p[q] = reinterpret_cast<const float*>(sA + q * REG)[er * LDP + eu + e];
            const float dh = (((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]))) + ldo[e];
            const float ai = la[0][e], aj = la[1][e], af = la[2][e], ao = la[3][e];
            const float cp = lcp[e];
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
        // 5. publish dz as hi / lo (4-B stores per plane and gate), drain, barrier, flag
        {
            const int64_t zbase = ((int64_t)((i & 1) * 2 + dir) * B + b0 + er) * G4 + u0 + eu;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                unsigned hi, lo;
                split2_bf16(dz[k][0], dz[k][1], hi, lo);
                put4((gu32*)(dzx + zbase + k * H), hi, local);
                put4((gu32*)(dzx + plane + zbase + k * H), lo, local);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                                 // every wave's partial reads done before the next DMA
        if (tid == 0) raise_flag(gflags + member, base + (unsigned)(i + 1), local);
        // the time-order copy for the weight-gradient and data-gradient GEMMs (drains behind the next step)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            *reinterpret_cast<f32x2_t*>(dG_t + tb * G4 + k * H + u0 + eu) = f32x2_t{dz[k][0], dz[k][1]};
    }
    // bias partials of this 32-row slice: the rows of every (gate, unit) meet in LDS
    if (bpart) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(sA);       // [row][4 gates x 32 units], free after the loop
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

static bool x3_bwd_fits(int B, int H) {
    int dev = 0, cus = 0, per_cu = 0;
    if (B % PBR || H != 32 * X3_KS) return false;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_persistent_f32x3_kernel, X3_THREADS, 0) !=
        hipSuccess)
        return false;
    return 2L * (B / PBR) * (H / PHU) <= (long)cus * per_cu;
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

// the fp32 BPTT on the split (exact mode keeps the per-step exact kernels)
extern "C" int ocrk_lstm_bwd_persistent_f32_supported(int B, int H) {
    if (B <= 0 || H != 32 * X3_KS) return 0;
    return x3_bwd_fits(B, H) ? 1 : 0;
}

extern "C" size_t ocrk_lstm_bwd_persistent_f32_workspace_size(int B, int H) {
    // the gather form's counters (persist.h), then the hi / lo dz exchange planes [2 planes][2 parities][2 dirs][B][4H] bf16
    if (B <= 0 || B % PBR || H != 32 * X3_KS) return 0;
    return persistent_counter_bytes(B, H) + (size_t)2 * 2 * 2 * B * 4 * H * sizeof(unsigned short);
}

extern "C" int ocrk_lstm_bwd_persistent_f32(const float* wh, const int* seq_len, int T, int B, int H,
                                            const float* dout, const float* cprev_t, const float* acts_t, float* dG_t,
                                            unsigned* err, unsigned* flags, float* dbias_part, void* ws,
                                            size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(ocrk_lstm_bwd_persistent_f32_supported(B, H),
                 "ocrk_lstm_bwd_persistent_f32: B=%d H=%d unsupported or not co-resident", B, H);
    OCRK_REQUIRE(ws_bytes >= ocrk_lstm_bwd_persistent_f32_workspace_size(B, H),
                 "ocrk_lstm_bwd_persistent_f32: workspace too small");
    OCRK_REQUIRE(wh && seq_len && dout && cprev_t && acts_t && dG_t && err, "ocrk_lstm_bwd_persistent_f32: null operand");
    OCRK_REQUIRE((int64_t)T * B * 8 * H * 4 < 0x7fffffffll, "ocrk_lstm_bwd_persistent_f32: acts exceed 2 GB");
    OCRK_REQUIRE(T >= 1, "ocrk_lstm_bwd_persistent_f32: T=%d", T);
    hipStream_t st = ocrk::as_stream(stream);
    const size_t counters = persistent_counter_bytes(B, H);      // flags: ocrk_persistent_flags_size's buffer
    unsigned* cnt = flags ? flags : (unsigned*)ws;
    unsigned short* zx = (unsigned short*)((char*)ws + counters);
    if (!flags && hipMemsetAsync(cnt, 0, counters, st) != hipSuccess)
        return ocrk::launch_status("ocrk_lstm_bwd_persistent_f32 memset");
    const unsigned grid = 2u * (unsigned)(B / PBR) * (unsigned)(H / PHU);
    lstm_bwd_persistent_f32x3_kernel<<<grid, X3_THREADS, 0, st>>>(wh, zx, seq_len, T, B, dout, cprev_t, acts_t, dG_t,
                                                                  cnt, err, recur_spin_limit(), dbias_part);
    return ocrk::launch_status("ocrk_lstm_bwd_persistent_f32");
}
