// a1+a2: direct 3x3 'same' convolution for the narrow-channel layers
// (src/weinman/model.py:84-109; conv2-conv5 forward, conv2-conv4 backward-data).
//
// Why not the implicit GEMM (gemm_nt.hip) here: with Cin = 32/64 a K = 9 Cin
// reduction is 9-18 MFMA k-steps per 128-pixel tile, so every workgroup
// pays its prologue, B-tile load and pipeline fill for a few dozen MFMAs,
// and every input pixel is gathered 9 times through L2.
//
// This kernel is persistent: a workgroup keeps the layer's weights in VGPRs
// (B fragments, loaded once) and walks a contiguous range of 128-pixel chunks
// of the flattened NHWC pixel index m = (b H + h) W + w. For a chunk it stages,
// per tap row dh in {-1, 0, +1}, the CONTIGUOUS run of input pixels
// [m0 + dh W - 1, m0 + dh W + 129) -- 3 x 130 pixels, each byte once, with
// LDS-DMA (buffer_load ... lds; out-of-range pixels come back as 0) -- and
// forms all 9 taps from LDS: tap (dh, dw) of output pixel m is staged pixel
// (m - m0) + dw + 1 of row dh. A tap that crosses the image's left/right edge
// or top/bottom row (where the flat shift wraps into a neighbouring row or
// image) is zeroed per lane by a select on the A fragment. The next chunk's
// DMA is in flight while the current one multiplies.
//
// Same arithmetic contract as the GEMM path: f32 accumulation of bf16
// products over k = (kh, kw, cin), bias / ReLU / ReLU-mask epilogue, bf16
// output, and the BatchNorm partial statistics (sum, M2 about the tile mean)
// of each 128-pixel tile -- identical tile boundaries, so bn_finalize and
// slab_sum read them unchanged. FLIP = backward-data: dy taps mirrored
// (dh = 1 - kh, dw = 1 - kw) against the [cin][kh][kw][cout] weight image.
#include <climits>

#include "common.h"
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr int CM = 128;                    // output pixels per chunk = BN statistics tile
constexpr unsigned DOOB = 0x80000000u;     // buffer offset past every range: loads 0, stores dropped

__device__ __forceinline__ unsigned short bf16_u16(float v) { return __builtin_bit_cast(unsigned short, (bf16)v); }

// sum over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1): every lane gets it
__device__ __forceinline__ float row_sum16(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xf, 0xf, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xf, 0xf, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xf, 0xf, false));
    return v;
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

// Workgroup barrier that waits only for this wave's LDS traffic: __syncthreads
// also drains vmcnt, which would wait for the chunks still being prefetched
// (their LDS-DMA completion is awaited explicitly with counted vmcnt waits).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int CI, int NO, int WN>
struct DirectCfg {
    static constexpr int KS = 9 * CI / 32;          // 32-deep k-steps, tap-major
    static constexpr int KB = CI / 32;              // k-steps per tap
    static constexpr int WM = 4 / WN;               // waves along M
    static constexpr int MTW = 8 / WM;              // 16-pixel M tiles per wave
    static constexpr int NTW = NO / 16 / WN;        // 16-channel N tiles per wave
    static constexpr int PXB = CI * 2;              // bytes per staged pixel
    static constexpr int PP = CI / 8;               // 16-B pieces per pixel
    static constexpr int PPB = 16 / PP;             // pixels per 256-B bank row
    static constexpr int RB = (CM + 2) * PXB;       // bytes per staged tap row
    static constexpr int NCH = 3 * RB / 16;         // 16-B DMA pieces per stage
    static constexpr int NBLK = (NCH + 63) / 64;    // 1-KB wave DMA blocks per stage
    static constexpr int NDW = (NBLK + 3) / 4;      // DMA instructions per wave per stage (padded: uniform count)
    static constexpr int NBUF = 3;                  // stages: chunk i computes while i+1, i+2 land
    static constexpr int SBA = NBLK * 1024;
    static constexpr int TRASH_OFF = NBUF * SBA;    // 1-KB sink of the padding DMA blocks
    static constexpr int ZERO_OFF = TRASH_OFF + 1024;   // 256 B of zeros: the A operand of an off-image tap
    static constexpr int RED_OFF = ZERO_OFF + 256;
    static constexpr int LDS = RED_OFF + 2 * WM * NO * 4;
    static constexpr int NSTO = MTW * NTW;          // 8-B output stores per lane per chunk
    static constexpr int NMSK = MTW * NTW;          // 8-B mask loads per lane per chunk
    static constexpr int NSS = 2 * NTW;             // statistics stores per lane per chunk (STATS)
    static_assert(NTW >= 1 && MTW * WM == 8 && NTW * KS * 4 <= 160, "direct conv tiling / register budget");
};

// Accumulator layout: the MFMA runs with the weights as its A operand and
// the pixels as its B operand, so lane (p, g) ends up holding output channels
// 16 j + 4 g + 0..3 of pixel 16 i + p -- four consecutive channels of one
// pixel, stored (and masked) as one 8-B access without an LDS transpose.
template <int CI, int NO, int WN, bool FLIP, bool STATS, bool MASK>
__global__ void __launch_bounds__(256)
conv3x3_direct_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, const float* __restrict__ bias,
                      const bf16* __restrict__ mask, bf16* __restrict__ y, float* __restrict__ stats, int relu,
                      int M, int H, int W, int nchunks, int cpw) {
    using C = DirectCfg<CI, NO, WN>;
    extern __shared__ __attribute__((aligned(1024))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % C::WM, wn = wave / C::WM;
    const int p = lane & 15, g = lane >> 4;

    // XCD-aware contiguous chunk ranges: the workgroups one XCD runs at once
    // walk neighbouring chunks, whose tap rows overlap in that XCD's L2
    const int nb = gridDim.x;
    const int bid = (nb % 8 == 0) ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
    const int c_begin = bid * cpw;
    const int c_end = min(nchunks, c_begin + cpw);
    if (c_begin >= c_end) return;

    const int xbytes = M * C::PXB;
    const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(x, (int64_t)xbytes);
    const __amdgpu_buffer_rsrc_t ry = uniform_rsrc(y, (int64_t)M * NO * 2);
    const __amdgpu_buffer_rsrc_t rst = uniform_rsrc(STATS ? (const void*)stats : (const void*)y,
                                                    (int64_t)nchunks * 2 * NO * 4);
    const __amdgpu_buffer_rsrc_t rmk = uniform_rsrc(MASK ? (const void*)mask : (const void*)y, (int64_t)M * NO * 2);

    // resident A fragments (weights): N tile j -> output channels (wn NTW + j) 16 + p, k = 32 ks + 8 g
    bf16x8 bw[C::NTW][C::KS];
#pragma unroll
    for (int j = 0; j < C::NTW; ++j) {
        const bf16* row = w + (size_t)((wn * C::NTW + j) * 16 + p) * (9 * CI) + 8 * g;
#pragma unroll
        for (int ks = 0; ks < C::KS; ++ks) bw[j][ks] = *reinterpret_cast<const bf16x8*>(row + 32 * ks);
    }
    float bcol[C::NTW][4];
#pragma unroll
    for (int j = 0; j < C::NTW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) bcol[j][r] = bias ? bias[(wn * C::NTW + j) * 16 + 4 * g + r] : 0.f;
    if (tid < 16) *reinterpret_cast<u32x4*>(smem + C::ZERO_OFF + 16 * tid) = u32x4{0u, 0u, 0u, 0u};

    // DMA pieces: LDS piece q (16 B, lane-linear per 1-KB block) of tap row r
    // holds staged pixel P = within / PP, logical piece (within % PP) ^
    // ((P / PPB) % PP) -- the XOR makes the 16 lanes of an operand read (16
    // consecutive pixels, one piece) hit 16 different 16-B bank groups. The
    // source offset relative to the chunk's first pixel is fixed per lane.
    int doff[C::NDW];
#pragma unroll
    for (int i = 0; i < C::NDW; ++i) {
        const int blk = i * 4 + wave;
        const int q = blk * 64 + lane;
        const int r = q / (C::RB / 16), within = q - r * (C::RB / 16);
        const int P = within / C::PP, piece = (within % C::PP) ^ ((P / C::PPB) % C::PP);
        doff[i] = (blk < C::NBLK && q < C::NCH) ? ((r - 1) * W - 1 + P) * C::PXB + piece * 16 : INT_MIN;
    }
    // Every wave issues NDW blocks (padding blocks and chunks past the range
    // load nothing into a sink block), so the vmcnt arithmetic is uniform.
    auto issue = [&](int chunk, int buf) {
        const bool live = chunk < c_end;
        const int base_off = chunk * CM * C::PXB;
        char* base = smem + buf * C::SBA;
#pragma unroll
        for (int i = 0; i < C::NDW; ++i) {
            const int blk = i * 4 + wave;
            const int off = base_off + doff[i];
            const bool ok = live && doff[i] != INT_MIN && (unsigned)off < (unsigned)xbytes;
            dma16(rx, blk < C::NBLK ? base + blk * 1024 : smem + C::TRASH_OFF, ok ? (unsigned)off : DOOB);
        }
    };

    // this lane's pixel in each M tile: position in the image, walked incrementally
    int pcol[C::MTW], prow[C::MTW];
#pragma unroll
    for (int i = 0; i < C::MTW; ++i) {
        const int m = c_begin * CM + 16 * (wm * C::MTW + i) + p;
        pcol[i] = m % W;
        prow[i] = (m / W) % H;
    }
    // swizzled byte offset of (pixel 16 i' + p + d, piece g) within a tap row, d = dw + 1
    int sx[C::MTW][3];
#pragma unroll
    for (int i = 0; i < C::MTW; ++i)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int P = 16 * (wm * C::MTW + i) + p + d;
            sx[i][d] = P * C::PXB + 16 * (((P / C::PPB) % C::PP) ^ g);
        }

    float* red = reinterpret_cast<float*>(smem + C::RED_OFF);   // [2][WM][NO]
    constexpr int NMK = MASK ? C::NMSK : 0;

    issue(c_begin, 0);
    issue(c_begin + 1, 1);
    for (int ch = c_begin; ch < c_end; ++ch) {
        const int k = ch - c_begin;
        const int buf = k % C::NBUF;
        const int m0 = ch * CM;
        // this chunk's DMA has landed (counted: the newer DMA, stores and mask
        // loads stay in flight); every wave is done with the buffer the next DMA overwrites
        constexpr int PER = C::NSTO + (STATS ? C::NSS : 0) + NMK;   // non-DMA VMEM ops per chunk
        static_assert(C::NDW + 2 * PER < 64, "vmcnt immediate");
        if (k == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::NDW) : "memory");
        else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::NDW + PER) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::NDW + 2 * PER) : "memory");
        lds_barrier();
        // MASK: the producer's activations at this lane's (pixel, 4 channels); the
        // next-but-one DMA goes out after they are consumed (vmcnt completes in
        // order: a wait for these loads would also wait for a DMA issued before them)
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        u32x2 mk[MASK ? C::MTW : 1][MASK ? C::NTW : 1];
        if constexpr (MASK) {
#pragma unroll
            for (int i = 0; i < C::MTW; ++i)
#pragma unroll
                for (int j = 0; j < C::NTW; ++j) {
                    const int m = m0 + 16 * (wm * C::MTW + i) + p;
                    const unsigned off = m < M ? (unsigned)((m * NO + (wn * C::NTW + j) * 16 + 4 * g) * 2) : DOOB;
                    mk[i][j] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rmk, off, 0, 0));
                }
        } else {
            issue(ch + 2, (k + 2) % C::NBUF);
        }

        // operand addresses: tap (dh, dw) of M tile i, or the zero block when
        // the tap leaves the image (left/right column, top/bottom row)
        const char* st = smem + buf * C::SBA;
        const char* zero = smem + C::ZERO_OFF;
        floatx4 acc[C::MTW][C::NTW];
#pragma unroll
        for (int i = 0; i < C::MTW; ++i)
#pragma unroll
            for (int j = 0; j < C::NTW; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // the A fragments of a tap row (3 taps) are read ahead of its MFMAs, so the
        // LDS latency is paid once per tap row instead of once per fragment
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            bf16x8 af[3][C::MTW][C::KB];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int dh = FLIP ? 1 - kh : kh - 1, dw = FLIP ? 1 - kw : kw - 1;
#pragma unroll
                for (int i = 0; i < C::MTW; ++i) {
                    const bool ok = (dh < 0 ? prow[i] != 0 : (dh > 0 ? prow[i] != H - 1 : true)) &&
                                    (dw < 0 ? pcol[i] != 0 : (dw > 0 ? pcol[i] != W - 1 : true));
                    const char* a = ok ? st + (dh + 1) * C::RB + sx[i][dw + 1] : zero + 16 * g;
#pragma unroll
                    for (int kb = 0; kb < C::KB; ++kb) {
                        // logical piece 4 kb + g: ((P / PPB) % PP ^ g) ^ 4 kb  ->  byte offset ^ 64 kb
                        const char* ak = ok ? (const char*)((uintptr_t)a ^ (uintptr_t)(64 * kb)) : a;
                        af[kw][i][kb] = *reinterpret_cast<const bf16x8*>(ak);
                    }
                }
            }
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                for (int i = 0; i < C::MTW; ++i)
#pragma unroll
                    for (int kb = 0; kb < C::KB; ++kb)
#pragma unroll
                        for (int j = 0; j < C::NTW; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][(kh * 3 + kw) * C::KB + kb],
                                                                                 af[kw][i][kb], acc[i][j], 0, 0, 0);
        }

        // ------------------------------------------------ epilogue
        const int valid = min(CM, M - m0);
#pragma unroll
        for (int i = 0; i < C::MTW; ++i)
#pragma unroll
            for (int j = 0; j < C::NTW; ++j) {
                const int ml = 16 * (wm * C::MTW + i) + p;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r] + bcol[j][r];
                    if constexpr (MASK) {
                        const unsigned h = mk[i][j][r >> 1] >> (16 * (r & 1));
                        if (!(__uint_as_float(h << 16) > 0.f)) v[r] = 0.f;
                    }
                    if (relu) v[r] = fmaxf(v[r], 0.f);
                    acc[i][j][r] = ml < valid ? v[r] : 0.f;
                }
                const u32x2 pk = {(unsigned)bf16_u16(v[0]) | ((unsigned)bf16_u16(v[1]) << 16),
                                  (unsigned)bf16_u16(v[2]) | ((unsigned)bf16_u16(v[3]) << 16)};
                const unsigned off = ml < valid ? (unsigned)(((m0 + ml) * NO + (wn * C::NTW + j) * 16 + 4 * g) * 2) : DOOB;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pk), ry, off, 0, 0);
            }
        if constexpr (MASK) issue(ch + 2, (k + 2) % C::NBUF);
        if constexpr (STATS) {
            // per-column (sum, M2 about the tile mean) over the tile's valid
            // pixels: lanes with equal g hold the same 4 columns -> reduce over p
            float ts[C::NTW][4];
#pragma unroll
            for (int j = 0; j < C::NTW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float s = 0.f;
#pragma unroll
                    for (int i = 0; i < C::MTW; ++i) s += acc[i][j][r];
                    ts[j][r] = row_sum16(s);
                }
            if (p == 0)
#pragma unroll
                for (int j = 0; j < C::NTW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) red[wm * NO + (wn * C::NTW + j) * 16 + 4 * g + r] = ts[j][r];
            lds_barrier();
            float* red2 = red + C::WM * NO;
            const float inv_valid = 1.f / (float)valid;     // exact for full tiles (128 = 2^7)
#pragma unroll
            for (int j = 0; j < C::NTW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int col = (wn * C::NTW + j) * 16 + 4 * g + r;
                    float s = 0.f;
#pragma unroll
                    for (int q = 0; q < C::WM; ++q) s += red[q * NO + col];
                    ts[j][r] = s;
                    const float mean = s * inv_valid;
                    float d2 = 0.f;
#pragma unroll
                    for (int i = 0; i < C::MTW; ++i) {
                        const float d = acc[i][j][r] - mean;
                        if (16 * (wm * C::MTW + i) + p < valid) d2 += d * d;
                    }
                    d2 = row_sum16(d2);
                    if (p == 0) red2[wm * NO + col] = d2;
                }
            lds_barrier();
            // lane (p, g) of a wm == 0 wave writes column (wn NTW + j) 16 + 4 g + (p & 3) for p < 4
            const bool writer = wm == 0 && p < 4;
#pragma unroll
            for (int j = 0; j < C::NTW; ++j) {
                const int col = (wn * C::NTW + j) * 16 + 4 * g + (p & 3);
                float m2 = 0.f;
#pragma unroll
                for (int q = 0; q < C::WM; ++q) m2 += red2[q * NO + col];
                const float sum = (p & 3) == 0 ? ts[j][0] : (p & 3) == 1 ? ts[j][1] : (p & 3) == 2 ? ts[j][2] : ts[j][3];
                const unsigned o = writer ? (unsigned)((ch * 2 * NO + col) * 4) : DOOB;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, sum), rst, o, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m2), rst, writer ? o + NO * 4 : DOOB, 0, 0);
            }
        }
        // advance this lane's pixels by one chunk
#pragma unroll
        for (int i = 0; i < C::MTW; ++i) {
            pcol[i] += CM;
            while (pcol[i] >= W) {
                pcol[i] -= W;
                prow[i] = prow[i] == H - 1 ? 0 : prow[i] + 1;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------ weight gradient
// dW[kh][kw][ci][co] = sum over pixels of x[px + (dh, dw)][ci] * dy[px][co],
// Cin = 32 (conv2, conv3). Same persistent chunk walk as the forward: per
// 128-pixel chunk the 3 tap-row runs of x (3 x 130 pixels) and the dy chunk
// are staged by LDS-DMA, and the k = pixel reduction runs on MFMA with both
// operands read k-transposed (ds_read_b64_tr_b16: a lane gets pixels
// 4g..4g+3 and 16+4g..16+4g+3 of a 32-pixel k-step, one channel). Off-image
// taps: the x run of tap row dh = -1 (+1) drops pixels of the image's last
// (first) row AT THE DMA (every product such a pixel enters belongs to an
// output pixel in the first (last) row); the dy fragment of tap column
// dw = -1 (+1) is masked in registers where its pixel is in the first (last)
// column. The workgroup keeps its dW partial in registers over its chunk
// range and writes it once; the split-K reduce sums the partials.
template <int CO>
struct WgCfg {
    static constexpr int CI = 32, PXB = 64;
    static constexpr int NTN = CO / 16;             // N tiles (16 output channels)
    static constexpr int WN = NTN;                  // waves along N: one N tile each
    static constexpr int WM = 4 / WN;               // waves along M
    static constexpr int MT = 9 * CI / 16;          // 18 M tiles of (tap, 16 ci)
    static constexpr int MTW = MT / WM;             // M tiles per wave (9 or 18)
    static constexpr int XRB = (CM + 2) * PXB;      // x tap-row run
    static constexpr int DYB = CM * CO * 2;         // the dy chunk
    static constexpr int NXP = 3 * XRB / 16;        // x pieces
    static constexpr int NDP = DYB / 16;            // dy pieces
    static constexpr int XBLK = (NXP + 63) / 64;    // x blocks: a wave's DMA block is all x or all dy
    static constexpr int NBLK = XBLK + (NDP + 63) / 64;   // (a uniform buffer descriptor per instruction)
    static constexpr int NDW = (NBLK + 3) / 4;
    static constexpr int SBA = NBLK * 1024;
    // two stages when two workgroups then fit a CU, else three when they fit
    static constexpr int NBUF = 2 * SBA + 1024 <= 80 * 1024 ? 2 : (3 * SBA + 1024 <= 160 * 1024 ? 3 : 2);
    static constexpr int PD = NBUF - 1;             // prefetch distance
    static constexpr int TRASH_OFF = NBUF * SBA;
    static constexpr int LDS = TRASH_OFF + 1024;
    static constexpr int PER_CU = LDS <= 80 * 1024 ? 2 : 1;
    static_assert(MT % WM == 0 && 4 % WN == 0, "wave split");
    static_assert(NDW * (PD - 1) < 64 && LDS <= 160 * 1024, "vmcnt immediate / LDS");
};

template <int CO>
__global__ void __launch_bounds__(256)
conv3x3_wgrad_direct_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ part,
                            int M, int H, int W, int nchunks, int cpw) {
    using C = WgCfg<CO>;
    extern __shared__ __attribute__((aligned(1024))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % C::WM, wn = wave / C::WM;
    const int i16 = lane & 15, g = lane >> 4;

    const int nb = gridDim.x;
    const int bid = (nb % 8 == 0) ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
    const int c_begin = bid * cpw;
    const int c_end = min(nchunks, c_begin + cpw);
    float* out = part + (size_t)blockIdx.x * 9 * C::CI * CO;

    floatx4 acc[C::MTW];
#pragma unroll
    for (int t = 0; t < C::MTW; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};

    if (c_begin < c_end) {
        const int xbytes = M * C::PXB, ybytes = M * CO * 2;
        const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(x, (int64_t)xbytes);
        const __amdgpu_buffer_rsrc_t rd = uniform_rsrc(dy, (int64_t)ybytes);
        const int HW = H * W;
        // per DMA slot: pixel offset from the chunk's first pixel, byte offset
        // within the pixel, the tap row (x slots) and the pixel's (row, col), walked per chunk
        int s_dpx[C::NDW], s_boff[C::NDW], s_kind[C::NDW], s_row[C::NDW], s_col[C::NDW];
#pragma unroll
        for (int i = 0; i < C::NDW; ++i) {
            const int blk = i * 4 + wave;
            const int q = blk * 64 + lane;
            int dpx = 0, boff = 0, kind = -1;                 // kind: 0..2 x tap row, 3 dy, -1 none
            if (blk < C::XBLK && q < C::NXP) {
                const int r = q / (C::XRB / 16), w16 = q - r * (C::XRB / 16);
                dpx = (r - 1) * W - 1 + w16 / (C::PXB / 16);
                boff = (w16 % (C::PXB / 16)) * 16;
                kind = r;
            } else if (blk >= C::XBLK && blk < C::NBLK && q - C::XBLK * 64 < C::NDP) {
                const int w16 = q - C::XBLK * 64;
                dpx = w16 / (CO * 2 / 16);
                boff = (w16 % (CO * 2 / 16)) * 16;
                kind = 3;
            }
            s_dpx[i] = dpx; s_boff[i] = boff; s_kind[i] = kind;
            const int pp = (((c_begin * CM + dpx) % HW) + HW) % HW;   // periodic in the image: negatives too
            s_row[i] = pp / W;
            s_col[i] = pp % W;
        }
        // the slots' (row, col) advance by one chunk per issue: issue chunks in order from c_begin
        auto issue = [&](int chunk, int buf) {
            const bool live = chunk < c_end;
            char* base = smem + buf * C::SBA;
#pragma unroll
            for (int i = 0; i < C::NDW; ++i) {
                const int blk = i * 4 + wave;
                const int k = s_kind[i];
                const int pix = chunk * CM + s_dpx[i];
                bool ok = live && k >= 0 && pix >= 0 && pix < M;
                if (k == 0) ok = ok && s_row[i] != H - 1;          // tap row -1: not the last row
                if (k == 2) ok = ok && s_row[i] != 0;              // tap row +1: not the first row
                const bool isx = blk < C::XBLK;                   // wave-uniform: one descriptor per instruction
                const unsigned off = (unsigned)(isx ? pix * C::PXB : pix * CO * 2) + (unsigned)s_boff[i];
                dma16(isx ? rx : rd, blk < C::NBLK ? base + blk * 1024 : smem + C::TRASH_OFF, ok ? off : DOOB);
                s_col[i] += CM;
                while (s_col[i] >= W) {
                    s_col[i] -= W;
                    s_row[i] = s_row[i] == H - 1 ? 0 : s_row[i] + 1;
                }
            }
        };
#pragma unroll
        for (int d = 0; d < C::PD; ++d) issue(c_begin + d, d);
        for (int ch = c_begin; ch < c_end; ++ch) {
            const int k = ch - c_begin;
            const int buf = k % C::NBUF;
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::NDW * (C::PD - 1)) : "memory");
            lds_barrier();
            issue(ch + C::PD, (k + C::PD) % C::NBUF);
            const char* st = smem + buf * C::SBA;
            const char* xs = st;                                 // [3][130 px][32 ci]
            const char* ds = st + C::XBLK * 1024;                // [128 px][CO]
            const int cq = 4 * (i16 & 3);
            const int colbase = (ch * CM) % W;                   // column of the chunk's first pixel
#pragma unroll
            for (int kk = 0; kk < CM / 32; ++kk) {
                const int pr = kk * 32 + 4 * g + (i16 >> 2);     // this lane's k-row (pixel) of the read
                // dy fragment: elements e hold pixels 32 kk + 4 g + (e & 3) + 16 (e >> 2); masked
                // copies for the tap columns -1 (first column dropped) and +1 (last column dropped)
                const bf16x8 bv = frag_tr(reinterpret_cast<const unsigned short*>(ds + pr * CO * 2 + (wn * 16 + cq) * 2),
                                          16 * CO);
                u32x4 mlo, mhi;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    unsigned lo = 0u, hi = 0u;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int e = 2 * d + h;
                        int c = colbase + kk * 32 + 4 * g + (e & 3) + 16 * (e >> 2);
                        while (c >= W) c -= W;
                        const unsigned half = 0xffffu << (16 * h);
                        if (c != 0) lo |= half;
                        if (c != W - 1) hi |= half;
                    }
                    mlo[d] = lo;
                    mhi[d] = hi;
                }
                const u32x4 bq = __builtin_bit_cast(u32x4, bv);
                const bf16x8 bfr[3] = {__builtin_bit_cast(bf16x8, bq & mlo), bv, __builtin_bit_cast(bf16x8, bq & mhi)};
#pragma unroll
                for (int t = 0; t < C::MTW; ++t) {
                    // M tile t of this wave: tap compile-time (WM = 2: the wave's ci tile is wm)
                    const int tap = C::WM == 2 ? t : t / 2, ct = C::WM == 2 ? wm : t % 2;
                    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
                    const bf16x8 afr = frag_tr(reinterpret_cast<const unsigned short*>(
                                                   xs + (dh + 1) * C::XRB + (pr + dw + 1) * C::PXB + (ct * 16 + cq) * 2),
                                               16 * C::PXB / 2);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[dw + 1], afr, acc[t], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // lane holds dW[tap][ci = ct*16 + i16][co = wn*16 + 4g .. +3]
#pragma unroll
    for (int t = 0; t < C::MTW; ++t) {
        const int tap = C::WM == 2 ? t : t / 2, ct = C::WM == 2 ? wm : t % 2;
        float* o = out + ((size_t)tap * C::CI + ct * 16 + i16) * CO + wn * 16 + 4 * g;
        *reinterpret_cast<floatx4*>(o) = acc[t];
    }
}

template <int CI, int NO, int WN, bool FLIP, bool STATS, bool MASK>
int launch_direct(const bf16* x, const bf16* w, const float* bias, const bf16* mask, bf16* y, float* stats,
                  int relu, int B, int H, int W, hipStream_t s) {
    using C = DirectCfg<CI, NO, WN>;
    auto kern = conv3x3_direct_kernel<CI, NO, WN, FLIP, STATS, MASK>;
    static DeviceOnce once;
    static int per_cu_dev[kMaxDevices];
    once_per_device(once, [&] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  C::LDS);
        int pc = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, 256, C::LDS) != hipSuccess || pc < 1) pc = 1;
        per_cu_dev[current_device()] = pc;
    });
    const int per_cu = per_cu_dev[current_device()], ncu = cu_count();
    const int M = B * H * W;
    const int nchunks = (int)cdiv(M, CM);
    int grid = ncu * per_cu;
    if (grid > nchunks) grid = nchunks;
    const int cpw = (int)cdiv(nchunks, grid);
    grid = (int)cdiv(nchunks, cpw);
    kern<<<grid, 256, C::LDS, s>>>(x, w, bias, mask, y, stats, relu, M, H, W, nchunks, cpw);
    return launch_status("conv3x3_direct");
}

}  // namespace

// OCRK_CONV_DIRECT=0: implicit GEMM only; 2: every shape the kernel covers
// (default: the Cin = 32 / Cout = 32 shapes it was measured faster on,
// tools/bench_conv.py -> profiles/r2_conv_layers.txt)
int conv_direct_mode() { return (int)opt(OPT_CONV_DIRECT); }

// forward: y = conv(x) + bias (ReLU if relu), optional per-128-pixel-tile (sum, M2)
int conv_direct_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout,
                    void* y, int relu, float* stats, hipStream_t s) {
    const int mode = conv_direct_mode();
    if (mode == 0 || (int64_t)B * H * W * (cin > cout ? cin : cout) * 2 > 0x7fffffffLL) return -1;
    if (mode == 1 && cin != 32) return -1;
    const bf16* xb = (const bf16*)x;
    const bf16* wb = (const bf16*)w_nk;
    bf16* yb = (bf16*)y;
#define OCRK_DF(CI, NO, WN)                                                                                  \
    if (cin == CI && cout == NO)                                                                           \
        return stats ? launch_direct<CI, NO, WN, false, true, false>(xb, wb, bias, nullptr, yb, stats, relu, B, H, W, s) \
                     : launch_direct<CI, NO, WN, false, false, false>(xb, wb, bias, nullptr, yb, nullptr, relu, B, H, W, s);
    OCRK_DF(32, 32, 1)
    OCRK_DF(32, 64, 1)
    OCRK_DF(64, 64, 2)
    OCRK_DF(64, 128, 4)
#undef OCRK_DF
    return -1;
}

// weight gradient for Cin = 32: per-workgroup partials [grid][9][32][cout] in ws, then the split-K reduce
size_t conv_direct_wgrad_ws_bytes(int B, int H, int W, int cin, int cout) {
    if (cin != 32 || (cout != 32 && cout != 64)) return 0;
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int per_cu = cout == 32 ? WgCfg<32>::PER_CU : WgCfg<64>::PER_CU;
    return (size_t)per_cu * (ncu > 0 ? ncu : 256) * 9 * cin * cout * sizeof(float);
}

int conv_direct_wgrad(const void* x, const void* dy, int B, int H, int W, int cin, int cout, float* dw,
                      int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
    const int mode = conv_direct_mode();
    if (mode == 0 || cin != 32 || (cout != 32 && cout != 64)) return -1;
    if (mode == 1 && cout != 32) return -1;           // conv3 (32 -> 64): the TN engine measured faster
    if ((int64_t)B * H * W * (cout > cin ? cout : cin) * 2 > 0x7fffffffLL) return -1;
    if (ws_bytes < conv_direct_wgrad_ws_bytes(B, H, W, cin, cout) || (uintptr_t)ws % 16 != 0) return -1;
    const int M = B * H * W;
    const int nchunks = (int)cdiv(M, CM);
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    int grid = (cout == 32 ? WgCfg<32>::PER_CU : WgCfg<64>::PER_CU) * ncu;   // co-resident
    if (grid > nchunks) grid = nchunks;
    const int cpw = (int)cdiv(nchunks, grid);
    grid = (int)cdiv(nchunks, cpw);
    if (cout == 32) {
        static DeviceOnce cfg;
        set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_wgrad_direct_kernel<32>), WgCfg<32>::LDS);
        conv3x3_wgrad_direct_kernel<32><<<grid, 256, WgCfg<32>::LDS, s>>>((const bf16*)x, (const bf16*)dy, (float*)ws, M, H, W, nchunks, cpw);
    } else {
        static DeviceOnce cfg;
        set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_wgrad_direct_kernel<64>), WgCfg<64>::LDS);
        conv3x3_wgrad_direct_kernel<64><<<grid, 256, WgCfg<64>::LDS, s>>>((const bf16*)x, (const bf16*)dy, (float*)ws, M, H, W, nchunks, cpw);
    }
    int st = launch_status("conv3x3_wgrad_direct");
    if (st) return st;
    GemmParams p = {};
    p.M = 9 * cin; p.N = cout; p.K = M; p.batch = 1;
    p.C = dw; p.ldc = cout; p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
    p.splits = grid; p.splitk_ws = (float*)ws;
    return splitk_finish(p, s);
}

// backward-data: dx = conv_flip(dy) (x ReLU mask of the producer), optional tile column statistics
int conv_direct_bwd_data(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                         const void* relu_mask, float* stats, hipStream_t s) {
    const int mode = conv_direct_mode();
    if (mode == 0 || (int64_t)B * H * W * (cin > cout ? cin : cout) * 2 > 0x7fffffffLL) return -1;
    if (mode == 1 && cin != 32) return -1;
    const bf16* a = (const bf16*)dy;
    const bf16* wb = (const bf16*)w_bwd;
    const bf16* mk = (const bf16*)relu_mask;
    bf16* o = (bf16*)dx;
#define OCRK_DB(CI, NO, WN)                                                                                   \
    if (cout == CI && cin == NO) {                                                                          \
        if (mk) return stats ? launch_direct<CI, NO, WN, true, true, true>(a, wb, nullptr, mk, o, stats, 0, B, H, W, s)   \
                             : launch_direct<CI, NO, WN, true, false, true>(a, wb, nullptr, mk, o, nullptr, 0, B, H, W, s); \
        return stats ? launch_direct<CI, NO, WN, true, true, false>(a, wb, nullptr, nullptr, o, stats, 0, B, H, W, s)     \
                     : launch_direct<CI, NO, WN, true, false, false>(a, wb, nullptr, nullptr, o, nullptr, 0, B, H, W, s); \
    }
    OCRK_DB(32, 32, 1)
    OCRK_DB(64, 32, 1)
    OCRK_DB(64, 64, 2)
#undef OCRK_DB
    return -1;
}

}  // namespace ocrk
