// a1 backward: the weight gradient of conv2 (3x3 'same', 32 -> 32 channels at
// 30 x 254, src/weinman/model.py:84-109 backward) by walking image ROWS.
//
//   dW[kh][kw][ci][co] = sum_{b,h,w} x[b][h+kh-1][w+kw-1][ci] * dy[b][h][w][co]
//
// Why rows: the chunked direct kernel (conv_direct.hip) stages, per 128-pixel
// chunk of the flat pixel index, three tap rows of x (3 x 130 pixels) plus the
// chunk's dy by LDS-DMA -- every x byte is staged three times, and the per-chunk
// DMA issue, wait and barrier dominate (137 us for 36 GFLOP / 250 MB). Here a
// workgroup owns whole images and walks their rows: output row h needs x rows
// h-1, h, h+1 (a 4-slot LDS ring, each x row loaded ONCE and used by three
// output rows) and dy row h (2-slot ring). The next rows are loaded into
// registers while the current row multiplies and written to the ring after it.
//
// MFMA mapping (16x16x32 bf16, f32 accumulate): per output row and tap
// (kh, kw), C[ci][co] += A[ci][w] . B[w][co] over the row's pixels w (K = 256:
// the 254 pixels + 2 zero columns), A = x row h+kh-1 shifted by kw-1 pixels.
// Both ring images are [pixel][channel] (channels contiguous, the NHWC rows
// as loaded), i.e. k-major, and the fragments come out of them with
// ds_read_b64_tr_b16 (frag_tr, the TN engine's reads): a kw shift is a shift
// of the k-row. A zero pixel on each side of every x row is the 'same'
// padding along w; an x row outside the image skips its three taps.
// Wave q multiplies the k-steps {2q, 2q+1} (pixels 64q .. 64q+63) for all 9
// taps: 9 x 2 x 2 accumulator tiles (144 VGPRs) held across all rows; at the
// end the 4 waves' partials are added in wave order in LDS and the workgroup
// writes one [9][32][32] f32 slab row; the split-K reduce sums the slab rows
// in a fixed order (deterministic).
#include <type_traits>

#include "common.h"
#include "gemm.h"
#include "mfma_util.h"

namespace ocrk {

namespace {

constexpr int RW_CI = 32, RW_CO = 32;
constexpr int RW_ROWB = RW_CI * 2;                 // 64 B per pixel (ci or co)
constexpr int RW_XROWS = 258;                      // pixels -1 .. 256 of an x row
constexpr int RW_DROWS = 256;                      // pixels 0 .. 255 of a dy row
constexpr int RW_XSLOT = RW_XROWS * RW_ROWB;       // 16.1 KB
constexpr int RW_DSLOT = RW_DROWS * RW_ROWB;       // 16 KB
constexpr int RW_XOFF = 0, RW_DOFF = 4 * RW_XSLOT;
constexpr int RW_RING = RW_DOFF + 2 * RW_DSLOT;    // 96.5 KB
constexpr int RW_PART = 9 * RW_CI * RW_CO;         // floats per partial
constexpr int RW_LDS = 4 * RW_PART * 4 > RW_RING ? 4 * RW_PART * 4 : RW_RING;   // 144 KB (end: wave partials)
constexpr int RW_MAXW = 254;

// The XOR swizzle of a 4-chunk (64-B) row r: v = (r >> 2) & 3 with its two bits swapped
// (0, 2, 1, 3). Any 16 consecutive rows then have distinct (r mod 4, swizzle) pairs (a
// ds_read_b128 of one chunk per row, 16 lanes a clock: no bank conflict), and rows r and r + 4
// use the other chunk PAIR (a ds_read_b64_tr_b16 of a chunk pair over 8 rows, 32 lanes a
// clock: with v itself rows r and r + 4 hit the same pair -- 2-way conflicts, 0.41-0.45 of
// the row kernels' LDS cycles; profiles/r6_conv12_bwd.txt)
__device__ __forceinline__ int swz4(int r) {
    const int v = (r >> 2) & 3;
    return ((v & 1) << 1) | (v >> 1);
}

// LDS byte offset of 16-B chunk c of image row r (4 chunks per row, swz4-swizzled)
__device__ __forceinline__ int rw_off(int r, int c) { return r * RW_ROWB + ((c ^ swz4(r)) << 4); }

// two fp32 values -> one word of two RNE bf16 (a single v_cvt_pk_bf16_f32; the
// per-value casts + shift / or took three VALU instructions per pair)
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}

// workgroup barrier over LDS traffic only (the row prefetch loads stay in flight)
__device__ __forceinline__ void rw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

constexpr int RD_XROW = 260;                       // floats per image ring row (pixels 0 .. 257, zero past W + 1)
constexpr int C12_XSLOTS = 8;                      // image ring rows of the conv1 producers

// validate.py:61-62 (the preprocess conv.hip's conv1 kernels apply, same rounding)
__device__ __forceinline__ float conv1_pre_u8(unsigned v) {
#pragma clang fp contract(off)
    return (float)v * (1.0f / 255.0f) - 0.5f;
}

// conv1's weights as MFMA A fragments (hi, lo) and its bias in the D layout: channel
// tile j, lane row = channel 16 j + i16, k = taps 8 g .. 8 g + 7 (taps >= 9: zero)
struct C1Frags {
    u32x4 wh[2], wl[2];
    const float* b1;              // read at use (4 floats per tile: fewer live registers)
};
__device__ __forceinline__ void c1_frags(C1Frags& f, const float* __restrict__ w1, const float* __restrict__ b1,
                                         int i16, int g) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int t0 = 8 * g + 2 * p, t1 = t0 + 1;
            const float v0 = t0 < 9 ? w1[t0 * RW_CO + 16 * j + i16] : 0.f;
            const float v1 = t1 < 9 ? w1[t1 * RW_CO + 16 * j + i16] : 0.f;
            unsigned hh, ll;
            split2_bf16(v0, v1, hh, ll);
            f.wh[j][p] = hh;
            f.wl[j][p] = ll;
        }
    }
    f.b1 = b1;
}

// conv1's output at one 16-pixel tile of row r (relu(b1 + 3x3 'valid' conv of image rows
// r .. r + 2, held preprocessed in the XS-row f32 image ring `ximg`) on the MFMA: per
// 16-channel tile D[ch][px] = b1 + W1^T[ch][tap] . X[tap][px], K = 9 taps padded to 32,
// hi + lo bf16 operands (3 products; XIN 2 = a bf16 image, exact in hi: 2). The lane's
// pixel is px (its i16); o[j] = the bf16 pairs of channels 16 j + 4 g .. + 3, mword |=
// their ReLU bits (bit c = channel c). The same bits wherever it runs.
typedef unsigned int c1_u32x2 __attribute__((ext_vector_type(2)));
template <int XIN, int XS>
__device__ __forceinline__ void c1_px16(const float* ximg, int r, int px, int g, const C1Frags& f, c1_u32x2 (&o)[2],
                                        unsigned& mword) {
    // B operand, k = tap t = 8 g + e (K padded to 32): lane group g = 0 holds taps 0-7
    // (kh = e / 3, kw = e % 3, compile-time), g = 1 tap 8 in slot 0, the rest zero -- so all
    // lanes gather the nine taps from three wave-uniform row bases and select (no per-lane
    // tap division: ~50 VALU fewer per 16-pixel tile, the same values)
    const float* x0 = ximg + (r & (XS - 1)) * RD_XROW + px;
    const float* x1 = ximg + ((r + 1) & (XS - 1)) * RD_XROW + px;
    const float* x2 = ximg + ((r + 2) & (XS - 1)) * RD_XROW + px;
    const float tp[9] = {x0[0], x0[1], x0[2], x1[0], x1[1], x1[2], x2[0], x2[1], x2[2]};
    float xv[8];
    xv[0] = g == 0 ? tp[0] : (g == 1 ? tp[8] : 0.f);
#pragma unroll
    for (int e = 1; e < 8; ++e) xv[e] = g == 0 ? tp[e] : 0.f;
    u32x4 bh, bl;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        unsigned hh, ll;
        split2_bf16(xv[2 * p], xv[2 * p + 1], hh, ll);
        bh[p] = hh;
        bl[p] = ll;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        floatx4 d = *reinterpret_cast<const floatx4*>(f.b1 + 16 * j + 4 * g);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.wh[j]),
                                                    __builtin_bit_cast(bf16x8, bh), d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.wl[j]),
                                                    __builtin_bit_cast(bf16x8, bh), d, 0, 0, 0);
        if constexpr (XIN == 1)
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.wh[j]),
                                                        __builtin_bit_cast(bf16x8, bl), d, 0, 0, 0);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[e] = fmaxf(d[e], 0.f);
            mword |= (v[e] > 0.f ? 1u : 0u) << (16 * j + 4 * g + e);
        }
        o[j][0] = pack_bf16x2(v[0], v[1]);
        o[j][1] = pack_bf16x2(v[2], v[3]);
    }
}

// conv1's output row r into a conv row ring slot ([pixel + 1][32 channels], rw_off
// layout; pixels past W untouched). Wave w covers pixels 64 w .. 64 w + 63. y1row /
// bitsrow (or NULL): the row's bf16 values and its ReLU bit mask (u32 per pixel) to
// global memory.
template <int XIN, int XS = C12_XSLOTS>
__device__ __forceinline__ void c1_make_row(char* slot, const float* ximg, int r, int W, int wave, int i16, int g,
                                            const C1Frags& f, bf16* y1row, unsigned* bitsrow) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int px = 64 * wave + 16 * n + i16;
        c1_u32x2 o[2];
        unsigned mword = 0;
        c1_px16<XIN, XS>(ximg, r, px, g, f, o, mword);
        if (px < W) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                *reinterpret_cast<c1_u32x2*>(slot + rw_off(px + 1, 2 * j + (g >> 1)) + (g & 1) * 8) = o[j];
                if (y1row) *reinterpret_cast<c1_u32x2*>(y1row + (size_t)px * RW_CI + 16 * j + 4 * g) = o[j];
            }
        }
        if (bitsrow) {
            mword = or_xor32(or_xor16(mword));
            if (g == 0 && px < W) bitsrow[px] = mword;
        }
    }
}

// C1X (1: u8, 2: bf16 image): conv2's x = y1 is not read but recomputed per row from the
// image (c1_make_row: the same bits conv12_fwd_rows_kernel produced), so the fused forward
// need not write y1 at all -- 125 MB written and 125 MB read less per step at C3
template <int C1X = 0>
__global__ void __launch_bounds__(256, 1)
conv3x3_wgrad_rows_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ part,
                          int B, int H, int W, const void* __restrict__ img = nullptr,
                          const float* __restrict__ w1 = nullptr, const float* __restrict__ b1 = nullptr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, g = lane >> 4;
    const int kr0 = 4 * g + (i16 >> 2);            // k-row of this lane's transposed read
    const int mq = 4 * (i16 & 3);                   // channel offset within a 16-wide tile

    // zero both rings once: the pad pixels (x rows 0 and W+1.., dy rows W..255) stay zero
    for (int i = tid; i < RW_RING / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};
    float* ximg = reinterpret_cast<float*>(smem + RW_LDS);           // C1X: [8][RD_XROW] image rows
    if constexpr (C1X != 0)
        for (int i = tid; i < C12_XSLOTS * RD_XROW; i += 256) ximg[i] = 0.f;
    C1Frags f1;
    if constexpr (C1X != 0) c1_frags(f1, w1, b1, i16, g);
    const int XW = W + 2;
    unsigned xraw = 0;
    auto x_fetch = [&](int bb, int r) {
        const size_t o = ((size_t)bb * (H + 2) + min(max(r, 0), H + 1)) * XW + min(tid, XW - 1);
        if constexpr (C1X == 1) xraw = reinterpret_cast<const uint8_t*>(img)[o];
        else if constexpr (C1X == 2) xraw = reinterpret_cast<const unsigned short*>(img)[o];
    };
    auto x_put = [&](int r) {
        if (tid < XW) ximg[(r & (C12_XSLOTS - 1)) * RD_XROW + tid] = C1X == 1 ? conv1_pre_u8(xraw) : __uint_as_float(xraw << 16);
    };

    floatx4 acc[9][2][2];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[t][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // a row = W pixels x 4 chunks <= 1016 chunks: 4 per thread. Two register
    // sets: the rows written to the ring at the end of step h were loaded during
    // step h-1, so a whole step of MFMAs covers their latency.
    constexpr int PER = 4;
    u32x4 sx[2][PER], sd[2][PER];
    // every lane loads (lanes past the row re-read its last chunk, never stored):
    // branch-free loads keep a fixed count in flight, so the compiler's waits
    // before the ring stores are counted (vmcnt(N)) instead of vmcnt(0)
    const int qmax = W * 4 - 1;
    auto load_row = [&](const bf16* base, u32x4 (&v)[PER]) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = min(tid + 256 * i, qmax);
            v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)q * 8);
        }
    };
    auto store_row = [&](int slot_off, int rshift, const u32x4 (&v)[PER]) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = tid + 256 * i;
            if (q < W * 4) {
                const int px = q >> 2, c = q & 3;
                *reinterpret_cast<u32x4*>(smem + slot_off + rw_off(px + rshift, c)) = v[i];
            }
        }
    };
    auto xslot = [&](int row) { return RW_XOFF + (row & 3) * RW_XSLOT; };
    auto dslot = [&](int row) { return RW_DOFF + (row & 1) * RW_DSLOT; };

    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const bf16* xb = x + (size_t)b * H * W * RW_CI;
        const bf16* db = dy + (size_t)b * H * W * RW_CO;
        auto xrow = [&](int r) { return xb + (size_t)r * W * RW_CI; };
        auto drow = [&](int r) { return db + (size_t)r * W * RW_CO; };
        __syncthreads();                            // the previous image's last reads are done
        if constexpr (C1X != 0) {
            // prologue: image rows 0 .. 4 into the image ring, then x rows 0, 1 produced
            for (int r = 0; r <= 4 && r < H + 2; ++r) {
                x_fetch(b, r);
                x_put(r);
            }
            __syncthreads();
            c1_make_row<C1X>(smem + xslot(0), ximg, 0, W, wave, i16, g, f1, nullptr, nullptr);
            if (H > 1) c1_make_row<C1X>(smem + xslot(1), ximg, 1, W, wave, i16, g, f1, nullptr, nullptr);
            load_row(drow(0), sd[1]);
            store_row(dslot(0), 0, sd[1]);
            if (H > 1) load_row(drow(1), sd[0]);
        } else {
            // prologue: x rows 0, 1 and dy row 0 into the ring; x row 2 / dy row 1 into set 0
            load_row(xrow(0), sx[1]);
            load_row(drow(0), sd[1]);
            store_row(xslot(0), 1, sx[1]);
            store_row(dslot(0), 0, sd[1]);
            if (H > 1) {
                load_row(xrow(1), sx[1]);
                store_row(xslot(1), 1, sx[1]);
                load_row(drow(1), sd[0]);
            }
            if (H > 2) load_row(xrow(2), sx[0]);
        }
        // step h: rows h-1..h+1 of x and row h of dy are in the ring; set P holds
        // x row h+2 / dy row h+1 (loaded during step h-1); set 1-P receives x row
        // h+3 / dy row h+2 now
        auto step = [&](int h, auto P_) {
            constexpr int P = decltype(P_)::value;
            __syncthreads();
            // unconditional (a clamped row past the image): a fixed count of loads in
            // flight lets the stores below wait for the older set only
            if constexpr (C1X != 0) x_fetch(b, h + 5);
            else load_row(xrow(min(h + 3, H - 1)), sx[1 - P]);
            load_row(drow(min(h + 2, H - 1)), sd[1 - P]);
            const char* dsl = smem + dslot(h);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int r = (2 * wave + kk) * 32 + kr0;      // dy k-row (pixel); the second read at r + 16
                bf16x8 bfr[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int n = 16 * j + mq;
                    bfr[j] = frag_tr(reinterpret_cast<const unsigned short*>(dsl + rw_off(r, n >> 3) + (n & 7) * 2),
                                     16 * RW_CO);
                }
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    const int hr = h + kh - 1;
                    if (hr < 0 || hr >= H) continue;           // wave-uniform
                    const char* xsl = smem + xslot(hr);
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        const int rx = r + kw;                 // x pixel w + kw - 1 at image row w + kw
#pragma unroll
                        for (int i = 0; i < 2; ++i) {
                            const int m = 16 * i + mq;
                            const bf16x8 af = frag_tr(
                                reinterpret_cast<const unsigned short*>(xsl + rw_off(rx, m >> 3) + (m & 7) * 2),
                                16 * RW_CI);
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                acc[kh * 3 + kw][i][j] =
                                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[kh * 3 + kw][i][j], 0, 0, 0);
                        }
                    }
                }
            }
            // rows h+2 / h+1 into the slots nobody reads this step (x row h-2's, dy row h-1's)
            if constexpr (C1X != 0) {
                // x row h+2 produced from image rows h+2 .. h+4; image row h+5 into the slot of h-3
                if (h + 2 < H) c1_make_row<C1X>(smem + xslot(h + 2), ximg, h + 2, W, wave, i16, g, f1, nullptr, nullptr);
                if (h + 5 < H + 2) x_put(h + 5);
            } else {
                if (h + 2 < H) store_row(xslot(h + 2), 1, sx[P]);
            }
            if (h + 1 < H) store_row(dslot(h + 1), 0, sd[P]);
        };
        for (int h = 0; h < H; h += 2) {
            step(h, std::integral_constant<int, 0>{});
            if (h + 1 < H) step(h + 1, std::integral_constant<int, 1>{});
        }
    }

    // the four waves' partials, added in wave order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem) + wave * RW_PART;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ci = 16 * i + 4 * g + e, co = 16 * j + i16;
                    red[(t * RW_CI + ci) * RW_CO + co] = acc[t][i][j][e];
                }
    __syncthreads();
    const float* r0 = reinterpret_cast<const float*>(smem);
    float* out = part + (size_t)blockIdx.x * RW_PART;
    for (int o = tid * 4; o < RW_PART; o += 256 * 4) {
        f32x4 s = *reinterpret_cast<const f32x4*>(r0 + o);
#pragma unroll
        for (int q = 1; q < 4; ++q) s += *reinterpret_cast<const f32x4*>(r0 + q * RW_PART + o);
        *reinterpret_cast<f32x4*>(out + o) = s;
    }
}

// Backward-data of conv2 by rows: dx[h][w][ci] = (y1[h][w][ci] > 0) *
//   sum_{kh,kw,co} dy[h+1-kh][w+1-kw][co] . Wb[ci][kh][kw][co]
// (w_bwd image [cin][3][3][cout], the mirrored taps of ocrk_conv3x3_bwd_data).
// A workgroup owns a band of output rows of one image and walks it: dy rows
// h-1 .. h+1 sit in a 4-slot LDS ring ([pixel][co], one zero pixel each side),
// each loaded once (the next one into registers a step ahead). The weights are
// the MFMA A operand, resident in VGPRs (9 taps x 2 ci tiles); the dy pixels
// the B operand (ds_read_b128 of 8 co of one pixel), so a lane ends up with 4
// consecutive ci of one pixel: the ReLU mask is one 8-B load and dx one 8-B
// store. Wave q covers pixels 64q .. 64q+63 of each row (4 x 2 tiles x 9 taps).
constexpr int RD_BANDS = 2;                        // row bands per image: 2 workgroups per CU
constexpr int RD_LDS = 4 * RW_XSLOT;               // 64.5 KB

// conv1 weight gradient fused into conv2's backward-data (XIN != 0): dx = dy1, the
// gradient at conv1's ReLU output, feeds only conv1's weight gradient
//   dW1[kh][kw][ci] = sum_{h,w} x[h+kh][w+kw] . dy1[h][w][ci],  db1[ci] = sum dy1[h][w][ci]
// (conv1 is 'valid' on the [H+2][W+2] single-channel image), so it is contracted
// here as it is produced instead of written (125 MB at C3) and re-read by
// conv1_wgrad_partial. Per row a wave multiplies A = X[tap][pixel] (taps 0-8, tap
// row 9 = ones for db1) by B = dy1[pixel][ci] on the 16x16x32 bf16 MFMA, K = its
// 64 pixels as two 32-pixel blocks: the dy1 block goes through a 2 KB per-wave
// LDS tile ([pixel][ci], read back transposed with frag_tr), the x rows sit in a
// 4-row f32 ring (preprocessed once per row), split hi + lo into bf16 (the u8
// path's x = v/255 - 0.5 is not a bf16 value; |x - hi - lo| <= 2^-17 |x|).
// 8 MFMAs per row beside the data gradient's 72; one [10][32] partial per workgroup.
constexpr int RD_XRING = 4 * RD_XROW * 4;          // 4.1 KB
constexpr int RD_TSLOT = 32 * RW_ROWB;             // 2 KB: one wave's 32-pixel block of dy1
constexpr int RD_LDS_C1 = RD_LDS + RD_XRING + 4 * RD_TSLOT;   // 76.6 KB (2 workgroups per CU)
constexpr int RD_C1_PART = 10 * RW_CI;             // floats per workgroup partial: [tap 0-8 | bias][ci]

// BITS: the ReLU mask as conv1's bit mask (u32 per pixel, bit c = channel c: ocrk_conv1_fwd_relu_bits)
// instead of its bf16 output -- 4 B per pixel read instead of 64
template <int XIN, bool BITS = false>   // XIN 0: dx out; 1 / 2: conv1's u8 / bf16 input -> conv1 dW partials, no dx
__global__ void __launch_bounds__(256, 2)
conv3x3_dgrad_rows_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ wb, const bf16* __restrict__ mask,
                          bf16* __restrict__ dx, int B, int H, int W, const void* __restrict__ xin,
                          float* __restrict__ c1part) {
    constexpr bool C1 = XIN != 0;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, g = lane >> 4;
    const int b = blockIdx.x / RD_BANDS, band = blockIdx.x - b * RD_BANDS;
    const int rows = (H + RD_BANDS - 1) / RD_BANDS;
    const int h0 = band * rows, h1 = min(H, h0 + rows);
    if (h0 >= h1) {
        if constexpr (C1)
            for (int o = tid; o < RD_C1_PART; o += 256) c1part[(size_t)blockIdx.x * RD_C1_PART + o] = 0.f;
        return;
    }

    for (int i = tid; i < (C1 ? RD_LDS_C1 : RD_LDS) / 16; i += 256)
        reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};

    // conv1 weight-gradient state (XIN != 0): x ring, this wave's dy1 tile, accumulators
    float* xring = reinterpret_cast<float*>(smem + RD_LDS);
    char* tile = smem + RD_LDS + RD_XRING + wave * RD_TSLOT;
    const int XW = W + 2;
    unsigned xraw = 0;
    auto x_fetch = [&](int r) {                      // this thread's pixel of x row r (clamped: a fixed load count)
        const size_t o = ((size_t)b * (H + 2) + r) * XW + min(tid, XW - 1);
        if constexpr (XIN == 1) xraw = reinterpret_cast<const uint8_t*>(xin)[o];
        else if constexpr (XIN == 2) xraw = reinterpret_cast<const unsigned short*>(xin)[o];
    };
    auto x_put = [&](int r) {
        if (tid < XW)
            xring[(r & 3) * RD_XROW + tid] = XIN == 1 ? conv1_pre_u8(xraw) : __uint_as_float(xraw << 16);
    };
    floatx4 c1acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    const int kr0 = 4 * g + (i16 >> 2), mq = 4 * (i16 & 3);   // frag_tr lane geometry (k-row, ci offset)
    const int tap = min(i16, 8), tkh = tap / 3, tkw = tap - 3 * tkh;

    // resident A fragments: ci tile i, tap t -> w_bwd[16 i + i16][t][8 g .. 8 g + 7]
    bf16x8 wa[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
            wa[t][i] = *reinterpret_cast<const bf16x8*>(wb + ((size_t)(16 * i + i16) * 9 + t) * RW_CO + 8 * g);

    constexpr int PER = 4;
    const int qmax = W * 4 - 1;
    u32x4 sd[2][PER];
    const bf16* dyb = dy + (size_t)b * H * W * RW_CO;
    auto drow = [&](int r) { return dyb + (size_t)r * W * RW_CO; };
    auto load_row = [&](const bf16* base, u32x4 (&v)[PER]) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = min(tid + 256 * i, qmax);
            v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)q * 8);
        }
    };
    auto store_row = [&](int row, const u32x4 (&v)[PER]) {
        char* slot = smem + (row & 3) * RW_XSLOT;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = tid + 256 * i;
            if (q < W * 4) *reinterpret_cast<u32x4*>(slot + rw_off((q >> 2) + 1, q & 3)) = v[i];
        }
    };
    auto zero_row = [&](int row) {                   // a dy row outside the image
        char* slot = smem + (row & 3) * RW_XSLOT;
        for (int i = tid; i < RW_XSLOT / 16; i += 256) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
    };
    __syncthreads();
    // prologue: dy rows h0-1, h0, h0+1 into the ring (zero rows past the image), h0+2 into set 0
    for (int r = h0 - 1; r <= h0 + 1; ++r) {
        if (r < 0 || r >= H) {
            zero_row(r);
        } else {
            load_row(drow(r), sd[1]);
            store_row(r, sd[1]);
        }
    }
    if constexpr (C1) {                              // x rows h0 .. h0+2 (conv1 is 'valid': all inside)
        for (int r = h0; r <= h0 + 2; ++r) {
            x_fetch(r);
            x_put(r);
        }
    }
    load_row(drow(min(h0 + 2, H - 1)), sd[0]);

    auto step = [&](int h, auto P_) {
        constexpr int P = decltype(P_)::value;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        load_row(drow(min(h + 3, H - 1)), sd[1 - P]);
        if constexpr (C1) x_fetch(min(h + 3, H + 1));
        // the ReLU mask of this row's outputs, in flight during the MFMAs
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        u32x2 mk[4][2];
        unsigned mb[4];
        if constexpr (BITS) {
            const unsigned* mrow = reinterpret_cast<const unsigned*>(mask) + ((size_t)b * H + h) * W;
#pragma unroll
            for (int n = 0; n < 4; ++n) mb[n] = mrow[min(64 * wave + 16 * n + i16, W - 1)];
        } else {
            const bf16* mrow = mask + ((size_t)b * H + h) * W * RW_CI;
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int px = min(64 * wave + 16 * n + i16, W - 1);
                    mk[n][i] = *reinterpret_cast<const u32x2*>(mrow + (size_t)px * RW_CI + 16 * i + 4 * g);
                }
        }
        floatx4 acc[4][2];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 2; ++i) acc[n][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const char* slot = smem + ((h + 1 - kh) & 3) * RW_XSLOT;   // zero rows past the image
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    // output pixel w = 64 q + 16 n + i16 reads dy pixel w + 1 - kw = image row w + 2 - kw
                    const int r = 64 * wave + 16 * n + i16 + 2 - kw;
                    const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rw_off(r, g));
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        acc[n][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][i], bf, acc[n][i], 0, 0, 0);
                }
            }
        }
        // lane: ci 16 i + 4 g .. +3 of pixel 64 q + 16 n + i16
        auto dx_bits = [&](int n, int i) {
            u32x2 o;
#pragma unroll
            for (int e2 = 0; e2 < 2; ++e2) {
                bool k0, k1;
                if constexpr (BITS) {
                    const unsigned sh = mb[n] >> (16 * i + 4 * g + 2 * e2);
                    k0 = sh & 1u;
                    k1 = sh & 2u;
                } else {
                    const unsigned m = mk[n][i][e2];
                    k0 = __uint_as_float(m << 16) > 0.f;
                    k1 = __uint_as_float(m & 0xffff0000u) > 0.f;
                }
                o[e2] = pack_bf16x2(k0 ? acc[n][i][2 * e2] : 0.f, k1 ? acc[n][i][2 * e2 + 1] : 0.f);
            }
            return o;
        };
        if constexpr (!C1) {
            bf16* orow = dx + ((size_t)b * H + h) * W * RW_CI;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int px = 64 * wave + 16 * n + i16;
                if (px >= W) continue;
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    *reinterpret_cast<u32x2*>(orow + (size_t)px * RW_CI + 16 * i + 4 * g) = dx_bits(n, i);
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {             // the wave's pixel blocks 64 q + 32 kb .. +31
#pragma unroll
                for (int nn = 0; nn < 2; ++nn) {
                    const int n = 2 * kb + nn;
                    const bool in = 64 * wave + 16 * n + i16 < W;   // pixels past the row contribute zero
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        u32x2 o = dx_bits(n, i);
                        if (!in) o = u32x2{0u, 0u};
                        *reinterpret_cast<u32x2*>(tile + rw_off(16 * nn + i16, 2 * i + (g >> 1)) + (g & 1) * 8) = o;
                    }
                }
                // the wave's own tile writes land before its transposed reads
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bf16x8 bfr[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int c = 16 * j + mq;
                    bfr[j] = frag_tr(reinterpret_cast<const unsigned short*>(tile + rw_off(kr0, c >> 3) + (c & 7) * 2),
                                     16 * RW_CO);
                }
                // A: lane row = tap (i16; 9 = the ones row of db1, 10-15 unused), k-slots of frag_tr's order
                const float* xs = xring + ((h + tkh) & 3) * RD_XROW + 64 * wave + 32 * kb + 4 * g + tkw;
                u32x4 ah, al;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int q = (p & 1) * 2 + (p >> 1) * 16;
                    unsigned hi2, lo2;
                    split2_bf16(xs[q], xs[q + 1], hi2, lo2);
                    ah[p] = i16 < 9 ? hi2 : (i16 == 9 ? 0x3f803f80u : 0u);
                    al[p] = i16 < 9 ? lo2 : 0u;
                }
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c1acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), bfr[j], c1acc[j],
                                                                       0, 0, 0);
                if constexpr (XIN == 1) {                // a bf16 input is exact in hi
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        c1acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al), bfr[j],
                                                                           c1acc[j], 0, 0, 0);
                }
            }
        }
        // dy row h+2 into the slot of row h-2 (or zeros past the image)
        if (h + 2 < H) store_row(h + 2, sd[P]);
        else if (h + 2 == H) zero_row(h + 2);
        if constexpr (C1)                                // x row h+3 into the slot of row h-1
            if (h + 3 < H + 2) x_put(h + 3);
    };
    for (int h = h0; h < h1; h += 2) {
        step(h, std::integral_constant<int, 0>{});
        if (h + 1 < h1) step(h + 1, std::integral_constant<int, 1>{});
    }
    if constexpr (C1) {
        // the four waves' [10][32] partials (lane: taps 4 g .. 4 g + 3 of ci 16 j + i16), added in wave order
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (4 * g + e < 10) red[wave * RD_C1_PART + (4 * g + e) * RW_CI + 16 * j + i16] = c1acc[j][e];
        __syncthreads();
        for (int o = tid; o < RD_C1_PART; o += 256)
            c1part[(size_t)blockIdx.x * RD_C1_PART + o] =
                ((red[o] + red[RD_C1_PART + o]) + red[2 * RD_C1_PART + o]) + red[3 * RD_C1_PART + o];
    }
}

// conv1 -> conv2's whole backward as one row walk, two wave roles per CU: waves 0-3 run
// conv2's backward-data with conv1's weight gradient contracted in (the loop of
// conv3x3_dgrad_rows_kernel<XIN, BITS>, unchanged), waves 4-7 conv2's weight gradient
//   dW[kh][kw][ci][co] += sum_w y1[h][w][ci] . dz[h+1-kh][w+1-kw][co]
// on the same dz ring rows (h-1 .. h+1 at step h), y1's row h recomputed from the image ring
// (c1_px16: the bits ocrk_conv12_fwd produced, so the forward writes no y1), 32 pixels at a
// time through the wave's own 2 KB tile (A = y1^T by frag_tr, B = the ring rows shifted by
// 1 - kw; the wgrad row kernel's 9 x 2 x 2 accumulator tiles). Wave q of each role sits on
// SIMD q: a dgrad wave and a wgrad wave share each MFMA pipe, and neither role's registers
// (resident weights + data-gradient tiles; 144 accumulator registers) are live in the
// other's loop, so two waves of <= 256 registers fit a SIMD. The roles meet at one barrier
// per row: the dgrad waves load the ring rows and image rows for both, into slots neither
// reads in that step. One band per image (one workgroup per CU, 86.6 KB of ring + tiles, the
// end's wave partials 149 KB). Partials: c1part [B][10][32] as the dgrad kernel's,
// w2part [B][9][32][32] (the four wgrad waves summed in wave order).
constexpr int C12B_TILES = RD_LDS + RD_XRING;                           // 4 dy1 tiles (2 KB), then 4 y1 tiles (4 KB)
constexpr int C12B_LDS_WALK = C12B_TILES + 12 * RD_TSLOT;               // 94.6 KB
constexpr int C12B_C1RED = 4 * RW_PART * 4;                             // the wgrad partials end here
constexpr int C12B_LDS = C12B_C1RED + 4 * RD_C1_PART * 4;               // 149 KB
static_assert(C12B_LDS >= C12B_LDS_WALK, "end partials overlay the walk's LDS");

template <int XIN, bool BITS>
__global__ void __launch_bounds__(512, 1)
conv12_bwd_rows_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ wb, const bf16* __restrict__ mask,
                       int B, int H, int W, const void* __restrict__ xin, const float* __restrict__ w1,
                       const float* __restrict__ b1, float* __restrict__ c1part, float* __restrict__ w2part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = wave & 3;                                  // SIMD / pixel quarter
    const bool wgrad_role = wave >= 4;
    const int i16 = lane & 15, g = lane >> 4;
    const int b = blockIdx.x;
    const int kr0 = 4 * g + (i16 >> 2), mq = 4 * (i16 & 3);   // frag_tr lane geometry
    const int XW = W + 2;
    float* xring = reinterpret_cast<float*>(smem + RD_LDS);

    for (int i = tid; i < C12B_LDS_WALK / 16; i += 512) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();

    if (!wgrad_role) {
        // ---- waves 0-3: conv2's backward-data + conv1's weight gradient (tid 0 .. 255)
        char* tile = smem + C12B_TILES + q * RD_TSLOT;
        unsigned xraw = 0;
        auto x_fetch = [&](int r) {
            const size_t o = ((size_t)b * (H + 2) + r) * XW + min(tid, XW - 1);
            if constexpr (XIN == 1) xraw = reinterpret_cast<const uint8_t*>(xin)[o];
            else xraw = reinterpret_cast<const unsigned short*>(xin)[o];
        };
        auto x_put = [&](int r) {
            if (tid < XW) xring[(r & 3) * RD_XROW + tid] = XIN == 1 ? conv1_pre_u8(xraw) : __uint_as_float(xraw << 16);
        };
        floatx4 c1acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
        const int tap = min(i16, 8), tkh = tap / 3, tkw = tap - 3 * tkh;
        bf16x8 wa[9][2];
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i)
                wa[t][i] = *reinterpret_cast<const bf16x8*>(wb + ((size_t)(16 * i + i16) * 9 + t) * RW_CO + 8 * g);
        constexpr int PER = 4;
        const int qmax = W * 4 - 1;
        u32x4 sd[2][PER];
        const bf16* dyb = dy + (size_t)b * H * W * RW_CO;
        auto drow = [&](int r) { return dyb + (size_t)r * W * RW_CO; };
        auto load_row = [&](const bf16* base, u32x4 (&v)[PER]) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int qq = min(tid + 256 * i, qmax);
                v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)qq * 8);
            }
        };
        auto store_row = [&](int row, const u32x4 (&v)[PER]) {
            char* slot = smem + (row & 3) * RW_XSLOT;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int qq = tid + 256 * i;
                if (qq < W * 4) *reinterpret_cast<u32x4*>(slot + rw_off((qq >> 2) + 1, qq & 3)) = v[i];
            }
        };
        auto zero_row = [&](int row) {
            char* slot = smem + (row & 3) * RW_XSLOT;
            for (int i = tid; i < RW_XSLOT / 16; i += 256) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
        };
        // prologue: dy rows -1, 0, 1 (zero rows past the image), x rows 0 .. 2, dy row 2 into set 0
        for (int r = -1; r <= 1; ++r) {
            if (r < 0 || r >= H) {
                zero_row(r);
            } else {
                load_row(drow(r), sd[1]);
                store_row(r, sd[1]);
            }
        }
        for (int r = 0; r <= 2; ++r) {
            x_fetch(r);
            x_put(r);
        }
        load_row(drow(min(2, H - 1)), sd[0]);

        auto step = [&](int h, auto P_) {
            constexpr int P = decltype(P_)::value;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            load_row(drow(min(h + 3, H - 1)), sd[1 - P]);
            x_fetch(min(h + 3, H + 1));
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            u32x2 mk[4][2];
            unsigned mb[4];
            if constexpr (BITS) {
                const unsigned* mrow = reinterpret_cast<const unsigned*>(mask) + ((size_t)b * H + h) * W;
#pragma unroll
                for (int n = 0; n < 4; ++n) mb[n] = mrow[min(64 * q + 16 * n + i16, W - 1)];
            } else {
                const bf16* mrow = mask + ((size_t)b * H + h) * W * RW_CI;
#pragma unroll
                for (int n = 0; n < 4; ++n)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int px = min(64 * q + 16 * n + i16, W - 1);
                        mk[n][i] = *reinterpret_cast<const u32x2*>(mrow + (size_t)px * RW_CI + 16 * i + 4 * g);
                    }
            }
            floatx4 acc[4][2];
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[n][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const char* slot = smem + ((h + 1 - kh) & 3) * RW_XSLOT;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
                    for (int n = 0; n < 4; ++n) {
                        const int r = 64 * q + 16 * n + i16 + 2 - kw;
                        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rw_off(r, g));
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            acc[n][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][i], bf, acc[n][i], 0, 0, 0);
                    }
                }
            }
            auto dx_bits = [&](int n, int i) {
                u32x2 o;
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2) {
                    bool k0, k1;
                    if constexpr (BITS) {
                        const unsigned sh = mb[n] >> (16 * i + 4 * g + 2 * e2);
                        k0 = sh & 1u;
                        k1 = sh & 2u;
                    } else {
                        const unsigned m = mk[n][i][e2];
                        k0 = __uint_as_float(m << 16) > 0.f;
                        k1 = __uint_as_float(m & 0xffff0000u) > 0.f;
                    }
                    o[e2] = pack_bf16x2(k0 ? acc[n][i][2 * e2] : 0.f, k1 ? acc[n][i][2 * e2 + 1] : 0.f);
                }
                return o;
            };
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
                for (int nn = 0; nn < 2; ++nn) {
                    const int n = 2 * kb + nn;
                    const bool in = 64 * q + 16 * n + i16 < W;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        u32x2 o = dx_bits(n, i);
                        if (!in) o = u32x2{0u, 0u};
                        *reinterpret_cast<u32x2*>(tile + rw_off(16 * nn + i16, 2 * i + (g >> 1)) + (g & 1) * 8) = o;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bf16x8 bfr[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int c = 16 * j + mq;
                    bfr[j] = frag_tr(reinterpret_cast<const unsigned short*>(tile + rw_off(kr0, c >> 3) + (c & 7) * 2),
                                     16 * RW_CO);
                }
                const float* xs = xring + ((h + tkh) & 3) * RD_XROW + 64 * q + 32 * kb + 4 * g + tkw;
                u32x4 ah, al;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int qq = (p & 1) * 2 + (p >> 1) * 16;
                    unsigned hi2, lo2;
                    split2_bf16(xs[qq], xs[qq + 1], hi2, lo2);
                    ah[p] = i16 < 9 ? hi2 : (i16 == 9 ? 0x3f803f80u : 0u);
                    al[p] = i16 < 9 ? lo2 : 0u;
                }
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c1acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), bfr[j], c1acc[j],
                                                                       0, 0, 0);
                if constexpr (XIN == 1) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        c1acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al), bfr[j],
                                                                           c1acc[j], 0, 0, 0);
                }
            }
            // dy row h+2 into the slot of row h-2 (or zeros past the image); x row h+3 into
            // the slot of row h-1 (the wgrad waves read rows h-1 .. h+1 / h .. h+2 this step)
            if (h + 2 < H) store_row(h + 2, sd[P]);
            else if (h + 2 == H) zero_row(h + 2);
            if (h + 3 < H + 2) x_put(h + 3);
        };
        for (int h = 0; h < H; h += 2) {
            step(h, std::integral_constant<int, 0>{});
            if (h + 1 < H) step(h + 1, std::integral_constant<int, 1>{});
        }
        __syncthreads();                                     // the walk is over: LDS is free
        float* red = reinterpret_cast<float*>(smem + C12B_C1RED);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (4 * g + e < 10) red[q * RD_C1_PART + (4 * g + e) * RW_CI + 16 * j + i16] = c1acc[j][e];
    } else {
        // ---- waves 4-7: conv2's weight gradient over pixels 64 q .. 64 q + 63
        char* tile = smem + C12B_TILES + (4 + 2 * q) * RD_TSLOT;      // 64 pixel rows
        C1Frags f1;
        c1_frags(f1, w1, b1, i16, g);
        floatx4 wacc[9][2][2];
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) wacc[t][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int h = 0; h < H; ++h) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            // y1's pixels 64 q .. 64 q + 63 of row h (zero past W) into the wave's tile (the
            // previous row's reads of it are done: the barrier's lgkmcnt wait)
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int px = 64 * q + 16 * n + i16;
                c1_u32x2 o[2];
                unsigned mword = 0;
                c1_px16<XIN, 4>(xring, h, px, g, f1, o, mword);
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    *reinterpret_cast<c1_u32x2*>(tile + rw_off(16 * n + i16, 2 * i + (g >> 1)) + (g & 1) * 8) =
                        px < W ? o[i] : c1_u32x2{0u, 0u};
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                bf16x8 ya[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int m = 16 * i + mq;
                    ya[i] = frag_tr(reinterpret_cast<const unsigned short*>(tile + rw_off(32 * kb + kr0, m >> 3) + (m & 7) * 2),
                                    16 * RW_CI);
                }
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    const char* dsl = smem + ((h + 1 - kh) & 3) * RW_XSLOT;   // zero rows past the image
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        const int rd = 64 * q + 32 * kb + kr0 + 2 - kw;
                        bf16x8 zb[2];
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int n = 16 * j + mq;
                            zb[j] = frag_tr(reinterpret_cast<const unsigned short*>(dsl + rw_off(rd, n >> 3) + (n & 7) * 2),
                                            16 * RW_CO);
                        }
#pragma unroll
                        for (int i = 0; i < 2; ++i)
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                wacc[kh * 3 + kw][i][j] =
                                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(ya[i], zb[j], wacc[kh * 3 + kw][i][j], 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();                                     // the walk is over: LDS is free
        float* red = reinterpret_cast<float*>(smem) + q * RW_PART;
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        red[(t * RW_CI + 16 * i + 4 * g + e) * RW_CO + 16 * j + i16] = wacc[t][i][j][e];
    }
    __syncthreads();
    // both roles' partials, the waves added in wave order
    const float* c1r = reinterpret_cast<const float*>(smem + C12B_C1RED);
    for (int o = tid; o < RD_C1_PART; o += 512)
        c1part[(size_t)b * RD_C1_PART + o] = ((c1r[o] + c1r[RD_C1_PART + o]) + c1r[2 * RD_C1_PART + o]) +
                                             c1r[3 * RD_C1_PART + o];
    const float* r0 = reinterpret_cast<const float*>(smem);
    float* out = w2part + (size_t)b * RW_PART;
    for (int o = tid * 4; o < RW_PART; o += 512 * 4) {
        f32x4 v = *reinterpret_cast<const f32x4*>(r0 + o);
#pragma unroll
        for (int qq = 1; qq < 4; ++qq) v += *reinterpret_cast<const f32x4*>(r0 + qq * RW_PART + o);
        *reinterpret_cast<f32x4*>(out + o) = v;
    }
}

// Forward of conv2 by rows: z[h][w][co] = bias[co] + sum_{kh,kw,ci}
// x[h+kh-1][w+kw-1][ci] . Wn[co][kh][kw][ci] (w_nk image), optional ReLU, and
// the BatchNorm partial statistics of each OUTPUT ROW (tile = one image row of
// W pixels: [B*H][2][cout] (sum, M2 about the row mean), finalized with
// tile_rows = W). Same ring / band walk as the backward-data kernel above,
// with x rows in the ring and the w_nk fragments resident.
// RELU a template flag: a runtime flag compiled to a max and a select per output value
// in the unrolled epilogue (the kernel's VALU count sets its row step)
template <bool RELU>
__global__ void __launch_bounds__(256, 2)
conv3x3_fwd_rows_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wn, const float* __restrict__ bias,
                        bf16* __restrict__ y, float* __restrict__ stats, int B, int H, int W) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float s_red[2][4][RW_CO];           // [sum | M2][wave][channel]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, g = lane >> 4;
    const int b = blockIdx.x / RD_BANDS, band = blockIdx.x - b * RD_BANDS;
    const int rows = (H + RD_BANDS - 1) / RD_BANDS;
    const int h0 = band * rows, h1 = min(H, h0 + rows);
    if (h0 >= h1) return;

    for (int i = tid; i < RD_LDS / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};

    // resident A fragments: co tile j, tap t -> w_nk[16 j + i16][t][8 g .. 8 g + 7]
    bf16x8 wa[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            wa[t][j] = *reinterpret_cast<const bf16x8*>(wn + ((size_t)(16 * j + i16) * 9 + t) * RW_CI + 8 * g);
    float bco[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) bco[j][e] = bias ? bias[16 * j + 4 * g + e] : 0.f;

    constexpr int PER = 4;
    const int qmax = W * 4 - 1;
    u32x4 sd[2][PER];
    const bf16* xb = x + (size_t)b * H * W * RW_CI;
    auto xrow = [&](int r) { return xb + (size_t)r * W * RW_CI; };
    auto load_row = [&](const bf16* base, u32x4 (&v)[PER]) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = min(tid + 256 * i, qmax);
            v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)q * 8);
        }
    };
    auto store_row = [&](int row, const u32x4 (&v)[PER]) {
        char* slot = smem + (row & 3) * RW_XSLOT;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = tid + 256 * i;
            if (q < W * 4) *reinterpret_cast<u32x4*>(slot + rw_off((q >> 2) + 1, q & 3)) = v[i];
        }
    };
    auto zero_row = [&](int row) {
        char* slot = smem + (row & 3) * RW_XSLOT;
        for (int i = tid; i < RW_XSLOT / 16; i += 256) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
    };
    __syncthreads();
    for (int r = h0 - 1; r <= h0 + 1; ++r) {
        if (r < 0 || r >= H) {
            zero_row(r);
        } else {
            load_row(xrow(r), sd[1]);
            store_row(r, sd[1]);
        }
    }
    load_row(xrow(min(h0 + 2, H - 1)), sd[0]);
    const float inv_w = 1.f / (float)W;
    // pixels past the row (the last tile): weight 0 in the row statistics -- an FMA per
    // value instead of an add and a select (exact: x * 1 and x * 0 of finite values)
    float inrow[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) inrow[n] = 64 * wave + 16 * n + i16 < W ? 1.f : 0.f;

    auto step = [&](int h, auto P_) {
        constexpr int P = decltype(P_)::value;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        load_row(xrow(min(h + 3, H - 1)), sd[1 - P]);
        floatx4 acc[4][2];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[n][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const char* slot = smem + ((h + kh - 1) & 3) * RW_XSLOT;   // zero rows past the image
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    // output pixel w = 64 q + 16 n + i16 reads x pixel w + kw - 1 = image row w + kw
                    const int r = 64 * wave + 16 * n + i16 + kw;
                    const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rw_off(r, g));
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[n][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][j], bf, acc[n][j], 0, 0, 0);
                }
            }
        }
        // lane: co 16 j + 4 g .. +3 of pixel 64 q + 16 n + i16
        float sum[2][4] = {};
#pragma unroll
        for (int n = 0; n < 4; ++n) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = acc[n][j][e] + bco[j][e];
                    if constexpr (RELU) v = fmaxf(v, 0.f);
                    acc[n][j][e] = v;
                    sum[j][e] = __builtin_fmaf(v, inrow[n], sum[j][e]);
                }
        }
        bf16* orow = y + ((size_t)b * H + h) * W * RW_CO;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int px = 64 * wave + 16 * n + i16;
            if (px >= W) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                u32x2 o;
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2)         // one v_cvt_pk_bf16_f32 per pair
                    o[e2] = __builtin_bit_cast(unsigned, __builtin_convertvector(
                        (f32x2_t{acc[n][j][2 * e2], acc[n][j][2 * e2 + 1]}), bf16x2_t));
                *reinterpret_cast<u32x2*>(orow + (size_t)px * RW_CO + 16 * j + 4 * g) = o;
            }
        }
        if (stats) {
            // the row's (sum, M2): lanes of a 16-lane row share channels -> DPP row sums,
            // waves in wave order through LDS; M2 about the row mean in a second pass
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = sum[j][e];
                    v += dpp_row<0x128>(v);
                    v += dpp_row<0x124>(v);
                    v += dpp_row<0x122>(v);
                    v += dpp_row<0x121>(v);
                    sum[j][e] = v;
                }
            if (i16 == 0)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) s_red[0][wave][16 * j + 4 * g + e] = sum[j][e];
            rw_barrier();
            float mean[2][4], q2[2][4];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int c = 16 * j + 4 * g + e;
                    mean[j][e] = (((s_red[0][0][c] + s_red[0][1][c]) + s_red[0][2][c]) + s_red[0][3][c]) * inv_w;
                    q2[j][e] = 0.f;
                }
#pragma unroll
            for (int n = 0; n < 4; ++n) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = (acc[n][j][e] - mean[j][e]) * inrow[n];
                        q2[j][e] = __builtin_fmaf(d, d, q2[j][e]);
                    }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = q2[j][e];
                    v += dpp_row<0x128>(v);
                    v += dpp_row<0x124>(v);
                    v += dpp_row<0x122>(v);
                    v += dpp_row<0x121>(v);
                    q2[j][e] = v;
                }
            if (i16 == 0)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) s_red[1][wave][16 * j + 4 * g + e] = q2[j][e];
            rw_barrier();
            if (tid < 2 * RW_CO) {
                const int k = tid / RW_CO, c = tid - k * RW_CO;
                stats[((size_t)b * H + h) * 2 * RW_CO + tid] =
                    ((s_red[k][0][c] + s_red[k][1][c]) + s_red[k][2][c]) + s_red[k][3][c];
            }
        }
        if (h + 2 < H) store_row(h + 2, sd[P]);
        else if (h + 2 == H) zero_row(h + 2);
    };
    for (int h = h0; h < h1; h += 2) {
        step(h, std::integral_constant<int, 0>{});
        if (h + 1 < h1) step(h + 1, std::integral_constant<int, 1>{});
    }
}

// The weight gradient by rows for Cout = 64 (conv3: 32 -> 64, conv4: 64 -> 64 at
// 15 x 127): the same ring walk, but wave q owns output channels 16q .. 16q+15
// over the WHOLE row (K = KPX pixels, KPX/32 k-steps), so no cross-wave sum:
// acc [9 taps][CI/16 tiles] (18 / 36 f32x4). x rows are CI*2 bytes, dy rows 128 B,
// 16-B chunks XOR-swizzled per row (rows of >= 8 chunks by r mod 8, of 4 chunks by swz4).
template <int CPR>
__device__ __forceinline__ int rc_off(int r, int c) {
    const int sw = CPR >= 8 ? (r & 7) : swz4(r);
    return r * CPR * 16 + ((c ^ sw) << 4);
}

template <int CI, int KPX, int CO_ = 64>
struct RcCfg {
    static constexpr int CO = CO_, NW = CO / 16, NT = NW * 64;
    static constexpr int XCPR = CI / 8, DCPR = CO / 8;       // 16-B chunks per pixel
    static constexpr int XSLOT = (KPX + 2) * CI * 2, DSLOT = KPX * CO * 2;
    static constexpr int DOFF = 4 * XSLOT;
    static constexpr int LDS = DOFF + 2 * DSLOT;
    static constexpr int XPER = (KPX * XCPR + NT - 1) / NT, DPER = (KPX * DCPR + NT - 1) / NT;   // chunks per thread
    static constexpr int PART = 9 * CI * CO;
};

// Wider layers as channel blocks (round 4): blockIdx.y = (ci block, co block) of a
// CI x CO sub-problem of an XCT -> DCT channel layer (conv5 64 -> 128: two co halves;
// conv6 128 -> 128: four quadrants), x and dy read with their full channel strides;
// each workgroup writes its [9][CI][CO] partial as [tap][split] slabs of the block
// ([y][tap][gridDim.x][CI][CO]), so one ordered split reduce per block lands the
// taps at their [9][XCT][DCT] rows. Every x / dy byte of the block is read once per
// workgroup (the 4-wave TN engine re-read the im2col rows per tap: ~700 MB of HBM
// traffic per conv6 launch).
template <int CI, int KPX, int CO_>
__global__ void __launch_bounds__((RcCfg<CI, KPX, CO_>::NT), 1)
conv3x3_wgrad_rows_co_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ part,
                             int B, int H, int W, int xct, int dct, int nco) {
    using C = RcCfg<CI, KPX, CO_>;
    constexpr int CO = C::CO, TI = CI / 16, NT = C::NT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, g = lane >> 4;
    const int kr0 = 4 * g + (i16 >> 2);
    const int mq = 4 * (i16 & 3);

    for (int i = tid; i < C::LDS / 16; i += NT) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};

    floatx4 acc[9][TI];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[t][i] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int xq = W * C::XCPR - 1, dq = W * C::DCPR - 1;
    const int xc0 = (blockIdx.y / nco) * CI, dc0 = (blockIdx.y % nco) * CO;
    u32x4 sx[2][C::XPER], sd[2][C::DPER];
    // chunk q of a row = pixel q / (CPR) , 8-channel piece q % CPR of the block's channels
    auto load_x = [&](const bf16* base, u32x4 (&v)[C::XPER]) {
#pragma unroll
        for (int i = 0; i < C::XPER; ++i) {
            const int q = min(tid + NT * i, xq);
            v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)(q / C::XCPR) * xct + xc0 + (q % C::XCPR) * 8);
        }
    };
    auto load_d = [&](const bf16* base, u32x4 (&v)[C::DPER]) {
#pragma unroll
        for (int i = 0; i < C::DPER; ++i) {
            const int q = min(tid + NT * i, dq);
            v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)(q / C::DCPR) * dct + dc0 + (q % C::DCPR) * 8);
        }
    };
    auto store_x = [&](int row, const u32x4 (&v)[C::XPER]) {
        char* slot = smem + (row & 3) * C::XSLOT;
#pragma unroll
        for (int i = 0; i < C::XPER; ++i) {
            const int q = tid + NT * i;
            if (q <= xq) *reinterpret_cast<u32x4*>(slot + rc_off<C::XCPR>(q / C::XCPR + 1, q % C::XCPR)) = v[i];
        }
    };
    auto store_d = [&](int row, const u32x4 (&v)[C::DPER]) {
        char* slot = smem + C::DOFF + (row & 1) * C::DSLOT;
#pragma unroll
        for (int i = 0; i < C::DPER; ++i) {
            const int q = tid + NT * i;
            if (q <= dq) *reinterpret_cast<u32x4*>(slot + rc_off<C::DCPR>(q / C::DCPR, q % C::DCPR)) = v[i];
        }
    };

    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const bf16* xb = x + (size_t)b * H * W * xct;
        const bf16* db = dy + (size_t)b * H * W * dct;
        auto xrow = [&](int r) { return xb + (size_t)r * W * xct; };
        auto drow = [&](int r) { return db + (size_t)r * W * dct; };
        __syncthreads();
        load_x(xrow(0), sx[1]);
        load_d(drow(0), sd[1]);
        store_x(0, sx[1]);
        store_d(0, sd[1]);
        if (H > 1) {
            load_x(xrow(1), sx[1]);
            store_x(1, sx[1]);
            load_d(drow(1), sd[0]);
        }
        if (H > 2) load_x(xrow(2), sx[0]);
        auto step = [&](int h, auto P_) {
            constexpr int P = decltype(P_)::value;
            rw_barrier();
            load_x(xrow(min(h + 3, H - 1)), sx[1 - P]);
            load_d(drow(min(h + 2, H - 1)), sd[1 - P]);
            const char* dsl = smem + C::DOFF + (h & 1) * C::DSLOT;
#pragma unroll
            for (int kk = 0; kk < KPX / 32; ++kk) {
                const int r = kk * 32 + kr0;
                const int n = 16 * wave + mq;
                const bf16x8 bfr = frag_tr(
                    reinterpret_cast<const unsigned short*>(dsl + rc_off<C::DCPR>(r, n >> 3) + (n & 7) * 2), 16 * CO);
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    const int hr = h + kh - 1;
                    if (hr < 0 || hr >= H) continue;
                    const char* xsl = smem + (hr & 3) * C::XSLOT;
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
                        for (int i = 0; i < TI; ++i) {
                            const int m = 16 * i + mq;
                            const bf16x8 af = frag_tr(reinterpret_cast<const unsigned short*>(
                                                          xsl + rc_off<C::XCPR>(r + kw, m >> 3) + (m & 7) * 2),
                                                      16 * CI);
                            acc[kh * 3 + kw][i] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[kh * 3 + kw][i], 0, 0, 0);
                        }
                    }
                }
            }
            if (h + 2 < H) store_x(h + 2, sx[P]);
            if (h + 1 < H) store_d(h + 1, sd[P]);
        };
        for (int h = 0; h < H; h += 2) {
            step(h, std::integral_constant<int, 0>{});
            if (h + 1 < H) step(h + 1, std::integral_constant<int, 1>{});
        }
    }
    // this wave's 16 output channels of the [9][CI][CO] partial, tap t into slab
    // [blockIdx.y][t][blockIdx.x]
    float* out = part + (size_t)blockIdx.y * 9 * gridDim.x * (CI * CO) + (size_t)blockIdx.x * (CI * CO);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                out[(size_t)t * gridDim.x * (CI * CO) + (16 * i + 4 * g + e) * CO + 16 * wave + i16] = acc[t][i][e];
}

// Generic forward by rows for the wider layers (conv3-conv6, W <= KPX):
// NW waves, wave w owns output channels 16w .. 16w+15 (CO = 16 NW) with its
// 9 x CI/32 weight fragments resident (the MFMA A operand); every wave runs
// over all KPX/16 pixel tiles of the row, B fragments from the x ring (one
// ds_read_b128 = 8 ci of one pixel). Per-row BatchNorm partials are wave-local
// (a wave owns its channels): DPP row sums over the 16 pixels of a tile, the
// tiles in order, M2 about the row mean in a second pass.
// conv1 -> conv2 forward in one row walk (bf16 training, conv2's 32 -> 32 with the BN row
// statistics): conv2's x ring rows (conv1's output y1 = relu(conv1(image)), 'valid' on the
// [H+2][W+2] single-channel image) are PRODUCED here from an 8-row f32 ring of preprocessed
// image rows instead of being loaded -- conv1's separate pass and conv2's re-read of y1
// (125 MB at C3) are gone. conv1 itself runs on the MFMA: per 16-pixel tile and 16-channel
// tile, D[ch][px] = b1 + W1^T[ch][tap] . X[tap][px] over K = 9 taps (padded to 32), the
// operands split hi + lo in bf16 (3 products: ~2^-16 per product against fp32's conv1,
// whose output is rounded to bf16 anyway). The produced rows also leave as y1 (the
// weight gradient's operand) and as the ReLU bit mask (the backward-data's mask), owned
// rows only. y1 row r is produced at the end of step r - 2 (the ring slot of row r - 4),
// image row r + 3 put at the end of step r - 2 (the ring slot of row r - 5).
constexpr int C12_LDS = RD_LDS + C12_XSLOTS * RD_XROW * 4;

template <int XIN, bool WY1>   // XIN 1: u8 image (the fused preprocess), 2: bf16 preprocessed image; WY1: y1 out
__global__ void __launch_bounds__(256, 2)
conv12_fwd_rows_kernel(const void* __restrict__ img, const float* __restrict__ w1, const float* __restrict__ b1,
                       const bf16* __restrict__ wn, const float* __restrict__ bias, bf16* __restrict__ y1,
                       unsigned* __restrict__ bits, bf16* __restrict__ y, float* __restrict__ stats, int B, int H,
                       int W) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float s_red[2][4][RW_CO];           // [sum | M2][wave][channel]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, g = lane >> 4;
    const int b = blockIdx.x / RD_BANDS, band = blockIdx.x - b * RD_BANDS;
    const int rows = (H + RD_BANDS - 1) / RD_BANDS;
    const int h0 = band * rows, h1 = min(H, h0 + rows);
    if (h0 >= h1) return;

    for (int i = tid; i < C12_LDS / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};
    float* ximg = reinterpret_cast<float*>(smem + RD_LDS);          // [8][RD_XROW] preprocessed image rows

    // conv2's resident A fragments: co tile j, tap t -> w_nk[16 j + i16][t][8 g .. 8 g + 7]
    bf16x8 wa[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            wa[t][j] = *reinterpret_cast<const bf16x8*>(wn + ((size_t)(16 * j + i16) * 9 + t) * RW_CI + 8 * g);
    float bco[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) bco[j][e] = bias ? bias[16 * j + 4 * g + e] : 0.f;
    // conv1's A fragments (hi, lo) and bias (c1_frags: the layout every conv1 producer uses)
    C1Frags f1;
    c1_frags(f1, w1, b1, i16, g);
    const int XW = W + 2;
    unsigned xraw = 0;
    auto x_fetch = [&](int r) {                      // this thread's pixel of image row r (clamped)
        const size_t o = ((size_t)b * (H + 2) + min(max(r, 0), H + 1)) * XW + min(tid, XW - 1);
        if constexpr (XIN == 1) xraw = reinterpret_cast<const uint8_t*>(img)[o];
        else xraw = reinterpret_cast<const unsigned short*>(img)[o];
    };
    auto x_put = [&](int r) {
        if (tid < XW) ximg[(r & (C12_XSLOTS - 1)) * RD_XROW + tid] = XIN == 1 ? conv1_pre_u8(xraw) : __uint_as_float(xraw << 16);
    };
    auto zero_row = [&](int row) {                   // a y1 row outside the image ('same' padding of conv2)
        char* slot = smem + (row & 3) * RW_XSLOT;
        for (int i = tid; i < RW_XSLOT / 16; i += 256) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
    };
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    // y1 row r (0 <= r < H) into conv2's ring slot r & 3 (pixels past W stay zero), and to
    // y1 (WY1) / bits when the band owns row r. Image rows r .. r + 2 are in the image ring.
    auto make_y1 = [&](int r) {
        char* slot = smem + (r & 3) * RW_XSLOT;
        const bool own = r >= h0 && r < h1;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int px = 64 * wave + 16 * n + i16;
            c1_u32x2 o[2];
            unsigned mword = 0;
            c1_px16<XIN, C12_XSLOTS>(ximg, r, px, g, f1, o, mword);
            if (px < W) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    *reinterpret_cast<c1_u32x2*>(slot + rw_off(px + 1, 2 * j + (g >> 1)) + (g & 1) * 8) = o[j];
                    if (WY1 && own)
                        *reinterpret_cast<c1_u32x2*>(y1 + (((size_t)b * H + r) * W + px) * RW_CI + 16 * j + 4 * g) = o[j];
                }
            }
            mword = or_xor32(or_xor16(mword));
            if (own && g == 0 && px < W) bits[((size_t)b * H + r) * W + px] = mword;
        }
    };

    __syncthreads();
    // prologue: image rows h0-1 .. h0+4 into the image ring, then y1 rows h0-1 .. h0+1 into the ring
    for (int r = h0 - 1; r <= h0 + 4; ++r) {
        if (r >= 0 && r < H + 2) {
            x_fetch(r);
            x_put(r);
        }
    }
    __syncthreads();
    for (int r = h0 - 1; r <= h0 + 1; ++r) {
        if (r < 0 || r >= H) zero_row(r);
        else make_y1(r);
    }
    const float inv_w = 1.f / (float)W;
    float inrow[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) inrow[n] = 64 * wave + 16 * n + i16 < W ? 1.f : 0.f;

    for (int h = h0; h < h1; ++h) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        x_fetch(h + 5);                              // image row h + 5, put at the end of this step
        floatx4 acc[4][2];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[n][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const char* slot = smem + ((h + kh - 1) & 3) * RW_XSLOT;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int r = 64 * wave + 16 * n + i16 + kw;
                    const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rw_off(r, g));
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[n][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][j], bf, acc[n][j], 0, 0, 0);
                }
            }
        }
        float sum[2][4] = {};
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = acc[n][j][e] + bco[j][e];
                    acc[n][j][e] = v;
                    sum[j][e] = __builtin_fmaf(v, inrow[n], sum[j][e]);
                }
        bf16* orow = y + ((size_t)b * H + h) * W * RW_CO;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int px = 64 * wave + 16 * n + i16;
            if (px >= W) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                u32x2 o;
                o[0] = pack_bf16x2(acc[n][j][0], acc[n][j][1]);
                o[1] = pack_bf16x2(acc[n][j][2], acc[n][j][3]);
                *reinterpret_cast<u32x2*>(orow + (size_t)px * RW_CO + 16 * j + 4 * g) = o;
            }
        }
        // the row's (sum, M2) as conv3x3_fwd_rows_kernel
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = sum[j][e];
                v += dpp_row<0x128>(v);
                v += dpp_row<0x124>(v);
                v += dpp_row<0x122>(v);
                v += dpp_row<0x121>(v);
                sum[j][e] = v;
            }
        if (i16 == 0)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) s_red[0][wave][16 * j + 4 * g + e] = sum[j][e];
        rw_barrier();
        float mean[2][4], q2[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 16 * j + 4 * g + e;
                mean[j][e] = (((s_red[0][0][c] + s_red[0][1][c]) + s_red[0][2][c]) + s_red[0][3][c]) * inv_w;
                q2[j][e] = 0.f;
            }
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = (acc[n][j][e] - mean[j][e]) * inrow[n];
                    q2[j][e] = __builtin_fmaf(d, d, q2[j][e]);
                }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = q2[j][e];
                v += dpp_row<0x128>(v);
                v += dpp_row<0x124>(v);
                v += dpp_row<0x122>(v);
                v += dpp_row<0x121>(v);
                q2[j][e] = v;
            }
        if (i16 == 0)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) s_red[1][wave][16 * j + 4 * g + e] = q2[j][e];
        rw_barrier();
        if (tid < 2 * RW_CO) {
            const int k = tid / RW_CO, c = tid - k * RW_CO;
            stats[((size_t)b * H + h) * 2 * RW_CO + tid] =
                ((s_red[k][0][c] + s_red[k][1][c]) + s_red[k][2][c]) + s_red[k][3][c];
        }
        // y1 row h+2 into the slot of row h-2 (zeros past the image); image row h+5 into the
        // image slot of row h-3 (rows h+2 .. h+4, read by make_y1, are in other slots)
        if (h + 2 < H) make_y1(h + 2);
        else if (h + 2 == H) zero_row(h + 2);
        if (h + 5 < H + 2) x_put(h + 5);
    }
}

template <int CI, int CO, int KPX, int CS = 1>
struct RfCfg {
    // CS workgroups split the output channels of a row band (CO / CS per workgroup)
    static constexpr int NW = CO / 16 / CS, NT = NW * 64, KS = CI / 32, PT = KPX / 16;
    static constexpr int CPR = CI / 8;
    static constexpr int XSLOT = (KPX + 2) * CI * 2;
    static constexpr int LDS = 4 * XSLOT;
    static constexpr int PER = (KPX * CPR + NT - 1) / NT;
    static constexpr int PER_CU = LDS <= 80 * 1024 && NW <= 4 ? 2 : 1;
    static constexpr int BANDS = PER_CU;
    static constexpr int PH = KS >= 4 && NW > 4 ? 2 : 1;    // pixel parts per row (register budget)
};

// bits (RELU only, or NULL): the output's ReLU bit mask, [B*H*W][CO/8] bytes, bit c = channel c > 0
template <int CI, int CO, int KPX, int CS, bool RELU>
__global__ void __launch_bounds__((RfCfg<CI, CO, KPX, CS>::NT), (RfCfg<CI, CO, KPX, CS>::PER_CU))
conv3x3_fwd_rows_co_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wn, const float* __restrict__ bias,
                           bf16* __restrict__ y, float* __restrict__ stats, int B, int H, int W,
                           uint16_t* __restrict__ bits) {
    using C = RfCfg<CI, CO, KPX, CS>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int cs = blockIdx.x % CS;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6) + cs * C::NW;     // the wave's output-channel tile
    const int i16 = lane & 15, g = lane >> 4;
    const int bid = blockIdx.x / CS;
    const int b = bid / C::BANDS, band = bid - b * C::BANDS;
    const int rows = (H + C::BANDS - 1) / C::BANDS;
    const int h0 = band * rows, h1 = min(H, h0 + rows);
    if (h0 >= h1) return;
    for (int i = tid; i < C::LDS / 16; i += C::NT) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};

    bf16x8 wa[9][C::KS];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int k = 0; k < C::KS; ++k)
            wa[t][k] = *reinterpret_cast<const bf16x8*>(wn + ((size_t)(16 * wave + i16) * 9 + t) * CI + 32 * k + 8 * g);
    float bco[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bco[e] = bias ? bias[16 * wave + 4 * g + e] : 0.f;

    const int qmax = W * C::CPR - 1;
    u32x4 sx[2][C::PER];
    const bf16* xb = x + (size_t)b * H * W * CI;
    auto xrow = [&](int r) { return xb + (size_t)r * W * CI; };
    auto load_row = [&](const bf16* base, u32x4 (&v)[C::PER]) {
#pragma unroll
        for (int i = 0; i < C::PER; ++i) v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)min(tid + C::NT * i, qmax) * 8);
    };
    auto store_row = [&](int row, const u32x4 (&v)[C::PER]) {
        char* slot = smem + (row & 3) * C::XSLOT;
#pragma unroll
        for (int i = 0; i < C::PER; ++i) {
            const int q = tid + C::NT * i;
            if (q <= qmax) *reinterpret_cast<u32x4*>(slot + rc_off<C::CPR>(q / C::CPR + 1, q % C::CPR)) = v[i];
        }
    };
    auto zero_row = [&](int row) {
        char* slot = smem + (row & 3) * C::XSLOT;
        for (int i = tid; i < C::XSLOT / 16; i += C::NT) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
    };
    __syncthreads();
    for (int r = h0 - 1; r <= h0 + 1; ++r) {
        if (r < 0 || r >= H) {
            zero_row(r);
        } else {
            load_row(xrow(r), sx[1]);
            store_row(r, sx[1]);
        }
    }
    load_row(xrow(min(h0 + 2, H - 1)), sx[0]);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

    auto step = [&](int h, auto P_) {
        constexpr int P = decltype(P_)::value;
        rw_barrier();
        load_row(xrow(min(h + 3, H - 1)), sx[1 - P]);
        // the row in PH pixel parts (PT/PH tiles each: fewer live accumulators for
        // the 8-wave configs); each part's (n, sum, M2 about its mean) merged into the
        // row's by Chan's formula
        constexpr int PP = C::PT / C::PH;
        float rs[4] = {0.f, 0.f, 0.f, 0.f}, rm2[4] = {0.f, 0.f, 0.f, 0.f};
        float rn = 0.f;
        bf16* orow = y + ((size_t)b * H + h) * W * CO;
#pragma unroll
        for (int ph = 0; ph < C::PH; ++ph) {
            floatx4 acc[PP];
#pragma unroll
            for (int n = 0; n < PP; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const char* slot = smem + ((h + kh - 1) & 3) * C::XSLOT;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                    for (int k = 0; k < C::KS; ++k)
#pragma unroll
                        for (int n = 0; n < PP; ++n) {
                            const int pt = ph * PP + n;
                            const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rc_off<C::CPR>(16 * pt + i16 + kw, 4 * k + g));
                            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][k], bf, acc[n], 0, 0, 0);
                        }
            }
            float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int n = 0; n < PP; ++n) {
                const int px = 16 * (ph * PP + n) + i16;
                const float inrow = px < W ? 1.f : 0.f;      // FMA weight instead of a select per value
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = acc[n][e] + bco[e];
                    if constexpr (RELU) v = fmaxf(v, 0.f);
                    acc[n][e] = v;
                    sum[e] = __builtin_fmaf(v, inrow, sum[e]);
                }
                if (px < W) {
                    u32x2 o;
                    o[0] = pack_bf16x2(acc[n][0], acc[n][1]);
                    o[1] = pack_bf16x2(acc[n][2], acc[n][3]);
                    *reinterpret_cast<u32x2*>(orow + (size_t)px * CO + 16 * wave + 4 * g) = o;
                }
                if constexpr (RELU) {
                    if (bits) {                            // the 4 lanes of a pixel: 16 channels -> one u16
                        unsigned m = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e) m |= (acc[n][e] > 0.f ? 1u : 0u) << (4 * g + e);
                        m = or_xor32(or_xor16(m));
                        if (g == 0 && px < W) bits[((size_t)b * H + h) * W * (CO / 16) + (size_t)px * (CO / 16) + wave] =
                            (uint16_t)m;
                    }
                }
            }
            if (stats) {
                const int p0 = 16 * PP * ph;
                const float np = (float)max(0, min(W - p0, 16 * PP));
                if (np > 0.f) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float v = sum[e];
                        v += dpp_row<0x128>(v);
                        v += dpp_row<0x124>(v);
                        v += dpp_row<0x122>(v);
                        v += dpp_row<0x121>(v);
                        const float mean = v / np;
                        float q = 0.f;
#pragma unroll
                        for (int n = 0; n < PP; ++n) {
                            const float d = (acc[n][e] - mean) * (16 * (ph * PP + n) + i16 < W ? 1.f : 0.f);
                            q = __builtin_fmaf(d, d, q);
                        }
                        q += dpp_row<0x128>(q);
                        q += dpp_row<0x124>(q);
                        q += dpp_row<0x122>(q);
                        q += dpp_row<0x121>(q);
                        if (ph == 0) {
                            rs[e] = v;
                            rm2[e] = q;
                        } else {                                   // Chan: merge (rn, rs, rm2) with (np, v, q)
                            const float dm = v / np - rs[e] / rn;
                            rm2[e] += q + dm * dm * rn * np / (rn + np);
                            rs[e] += v;
                        }
                    }
                    rn += np;
                }
            }
        }
        if (stats && i16 == 0) {
            float* st = stats + ((size_t)b * H + h) * 2 * CO + 16 * wave + 4 * g;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                st[e] = rs[e];
                st[CO + e] = rm2[e];
            }
        }
        if (h + 2 < H) store_row(h + 2, sx[P]);
        else if (h + 2 == H) zero_row(h + 2);
    };
    for (int h = h0; h < h1; h += 2) {
        step(h, std::integral_constant<int, 0>{});
        if (h + 1 < h1) step(h + 1, std::integral_constant<int, 1>{});
    }
}

template <int CI, int CO, int KPX, int CS = 1>
static int launch_fwd_co(const void* x, int B, int H, int W, const void* w_nk, const float* bias, void* y, int relu,
                         float* stats, hipStream_t s, void* relu_bits = nullptr) {
    using C = RfCfg<CI, CO, KPX, CS>;
    static DeviceOnce cfg, cfg_r;
    if (relu) {
        set_dyn_lds(cfg_r, reinterpret_cast<const void*>(&conv3x3_fwd_rows_co_kernel<CI, CO, KPX, CS, true>), C::LDS);
        conv3x3_fwd_rows_co_kernel<CI, CO, KPX, CS, true><<<B * C::BANDS * CS, C::NT, C::LDS, s>>>(
            (const bf16*)x, (const bf16*)w_nk, bias, (bf16*)y, stats, B, H, W, (uint16_t*)relu_bits);
    } else {
        set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_fwd_rows_co_kernel<CI, CO, KPX, CS, false>), C::LDS);
        conv3x3_fwd_rows_co_kernel<CI, CO, KPX, CS, false><<<B * C::BANDS * CS, C::NT, C::LDS, s>>>(
            (const bf16*)x, (const bf16*)w_nk, bias, (bf16*)y, stats, B, H, W, nullptr);
    }
    return launch_status("conv3x3_fwd_rows_co");
}

// Generic backward-data by rows (routed for conv4's 64 <- 64; conv5's 64 <- 128
// measured slower here at one workgroup per CU: 78 vs 68 us): dx[h][w][ci] =
// mask * sum_{kh,kw,co} dy[h+1-kh][w+1-kw][co] . Wb[ci][kh][kw][co]. NW = CI/16
// waves, wave w owns input channels 16w .. 16w+15 with its 9 x CO/32 w_bwd
// fragments resident; dy rows in the 4-slot ring. With `stats` (the bias
// gradient of the producing layer) each workgroup writes the column sums of
// its masked dx as ONE row of the [tiles][2][CI] table (sums in the first CI)
// and the rows past the grid are zeroed, so summing every table row gives
// the same total as the 128-pixel tiles of the GEMM path.
template <int CI, int CO, int KPX, int CS = 1>
struct RbCfg {
    // CS workgroups split the input channels (the outputs here) of a row band
    static constexpr int NW = CI / 16 / CS, NT = NW * 64, KS = CO / 32, PT = KPX / 16;
    static constexpr int CPR = CO / 8;
    static constexpr int XSLOT = (KPX + 2) * CO * 2;
    static constexpr int LDS = 4 * XSLOT;
    static constexpr int PER = (KPX * CPR + NT - 1) / NT;
    static constexpr int PER_CU = LDS <= 80 * 1024 && NW <= 4 ? 2 : 1;
    static constexpr int BANDS = PER_CU;
};

// MB: `mask` is the producer's ReLU bit mask ([B*H*W][CI/8] bytes, bit c = channel c), 2 B per
// (pixel, wave) instead of the bf16 output's 8 B per lane
template <int CI, int CO, int KPX, int CS, bool MB = false>
__global__ void __launch_bounds__((RbCfg<CI, CO, KPX, CS>::NT), (RbCfg<CI, CO, KPX, CS>::PER_CU))
conv3x3_dgrad_rows_co_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ wb,
                             const bf16* __restrict__ mask, bf16* __restrict__ dx, float* __restrict__ stats,
                             int stat_rows, int B, int H, int W) {
    using C = RbCfg<CI, CO, KPX, CS>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int cs = blockIdx.x % CS;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6) + cs * C::NW;     // the wave's channel tile
    const int i16 = lane & 15, g = lane >> 4;
    const int bid = blockIdx.x / CS;
    const int b = bid / C::BANDS, band = bid - b * C::BANDS;
    const int rows = (H + C::BANDS - 1) / C::BANDS;
    const int h0 = band * rows, h1 = min(H, h0 + rows);
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    const int nbid = gridDim.x / CS;               // table rows written: one per band workgroup
    if (stats && cs == 0)                          // table rows past them: zero
        for (int r = nbid + bid; r < stat_rows; r += nbid)
            for (int i = tid; i < 2 * CI; i += C::NT) stats[(size_t)r * 2 * CI + i] = 0.f;
    if (h0 < h1) {
        for (int i = tid; i < C::LDS / 16; i += C::NT) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0u, 0u, 0u, 0u};
        bf16x8 wa[9][C::KS];
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int k = 0; k < C::KS; ++k)
                wa[t][k] = *reinterpret_cast<const bf16x8*>(wb + ((size_t)(16 * wave + i16) * 9 + t) * CO + 32 * k + 8 * g);
        const int qmax = W * C::CPR - 1;
        u32x4 sx[2][C::PER];
        const bf16* db = dy + (size_t)b * H * W * CO;
        auto drow = [&](int r) { return db + (size_t)r * W * CO; };
        auto load_row = [&](const bf16* base, u32x4 (&v)[C::PER]) {
#pragma unroll
            for (int i = 0; i < C::PER; ++i)
                v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)min(tid + C::NT * i, qmax) * 8);
        };
        auto store_row = [&](int row, const u32x4 (&v)[C::PER]) {
            char* slot = smem + (row & 3) * C::XSLOT;
#pragma unroll
            for (int i = 0; i < C::PER; ++i) {
                const int q = tid + C::NT * i;
                if (q <= qmax) *reinterpret_cast<u32x4*>(slot + rc_off<C::CPR>(q / C::CPR + 1, q % C::CPR)) = v[i];
            }
        };
        auto zero_row = [&](int row) {
            char* slot = smem + (row & 3) * C::XSLOT;
            for (int i = tid; i < C::XSLOT / 16; i += C::NT) reinterpret_cast<u32x4*>(slot)[i] = u32x4{0u, 0u, 0u, 0u};
        };
        __syncthreads();
        for (int r = h0 - 1; r <= h0 + 1; ++r) {
            if (r < 0 || r >= H) {
                zero_row(r);
            } else {
                load_row(drow(r), sx[1]);
                store_row(r, sx[1]);
            }
        }
        load_row(drow(min(h0 + 2, H - 1)), sx[0]);
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

        auto step = [&](int h, auto P_) {
            constexpr int P = decltype(P_)::value;
            rw_barrier();
            load_row(drow(min(h + 3, H - 1)), sx[1 - P]);
            u32x2 mk[C::PT];
            unsigned mbv[C::PT];
            if constexpr (MB) {
                const uint16_t* mrow = reinterpret_cast<const uint16_t*>(mask) + ((size_t)b * H + h) * W * (CI / 16);
#pragma unroll
                for (int n = 0; n < C::PT; ++n) mbv[n] = mrow[(size_t)min(16 * n + i16, W - 1) * (CI / 16) + wave];
            } else {
                const bf16* mrow = mask ? mask + ((size_t)b * H + h) * W * CI : nullptr;
                if (mask) {
#pragma unroll
                    for (int n = 0; n < C::PT; ++n)
                        mk[n] = *reinterpret_cast<const u32x2*>(mrow + (size_t)min(16 * n + i16, W - 1) * CI + 16 * wave + 4 * g);
                }
            }
            floatx4 acc[C::PT];
#pragma unroll
            for (int n = 0; n < C::PT; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const char* slot = smem + ((h + 1 - kh) & 3) * C::XSLOT;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                    for (int k = 0; k < C::KS; ++k)
#pragma unroll
                        for (int n = 0; n < C::PT; ++n) {
                            const bf16x8 bf = *reinterpret_cast<const bf16x8*>(slot + rc_off<C::CPR>(16 * n + i16 + 2 - kw, 4 * k + g));
                            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kh * 3 + kw][k], bf, acc[n], 0, 0, 0);
                        }
            }
            bf16* orow = dx + ((size_t)b * H + h) * W * CI;
#pragma unroll
            for (int n = 0; n < C::PT; ++n) {
                const int px = 16 * n + i16;
                if (px >= W) continue;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[n][e];
                if constexpr (MB) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (!((mbv[n] >> (4 * g + e)) & 1u)) v[e] = 0.f;
                } else if (mask) {
#pragma unroll
                    for (int e2 = 0; e2 < 2; ++e2) {
                        const unsigned m = mk[n][e2];
                        if (!(__uint_as_float(m << 16) > 0.f)) v[2 * e2] = 0.f;
                        if (!(__uint_as_float(m & 0xffff0000u) > 0.f)) v[2 * e2 + 1] = 0.f;
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) bsum[e] += v[e];
                u32x2 o;
                o[0] = pack_bf16x2(v[0], v[1]);
                o[1] = pack_bf16x2(v[2], v[3]);
                *reinterpret_cast<u32x2*>(orow + (size_t)px * CI + 16 * wave + 4 * g) = o;
            }
            if (h + 2 < H) store_row(h + 2, sx[P]);
            else if (h + 2 == H) zero_row(h + 2);
        };
        for (int h = h0; h < h1; h += 2) {
            step(h, std::integral_constant<int, 0>{});
            if (h + 1 < h1) step(h + 1, std::integral_constant<int, 1>{});
        }
    }
    if (stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = bsum[e];
            v += dpp_row<0x128>(v);
            v += dpp_row<0x124>(v);
            v += dpp_row<0x122>(v);
            v += dpp_row<0x121>(v);
            bsum[e] = v;
        }
        if (i16 == 0) {
            float* st = stats + (size_t)bid * 2 * CI + 16 * wave + 4 * g;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                st[e] = bsum[e];
                st[CI + e] = 0.f;
            }
        }
    }
}

template <int CI, int CO, int KPX, int CS = 1, bool MB = false>
static int launch_dgrad_co(const void* dy, int B, int H, int W, const void* w_bwd, void* dx, const void* mask,
                           float* stats, hipStream_t s) {
    using C = RbCfg<CI, CO, KPX, CS>;
    const int grid = B * C::BANDS * CS;
    const int64_t trows = cdiv((int64_t)B * H * W, 128);
    if (stats && trows < B * C::BANDS) return -1;  // the table has fewer rows than band workgroups
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_dgrad_rows_co_kernel<CI, CO, KPX, CS, MB>), C::LDS);
    conv3x3_dgrad_rows_co_kernel<CI, CO, KPX, CS, MB><<<grid, C::NT, C::LDS, s>>>(
        (const bf16*)dy, (const bf16*)w_bwd, (const bf16*)mask, (bf16*)dx, stats, (int)trows, B, H, W);
    return launch_status("conv3x3_dgrad_rows_co");
}

}  // namespace

// OCRK_CONV_ROWS=0: the chunked direct kernel instead
static bool rows_enabled() { return opt(OPT_CONV_ROWS) != 0; }

// OCRK_CONV_WGRAD_BLOCKS=0: conv5 / conv6 weight gradients stay on the 4-wave TN engine
static bool rows_wgrad_blocks() { return opt(OPT_CONV_WGRAD_BLOCKS) != 0; }

// OCRK_CONV_WGRAD_BLOCKS=2: conv7 / conv8 as channel blocks too (else the ping-pong TN engine)
static bool rows_wgrad_blocks_wide() { return opt(OPT_CONV_WGRAD_BLOCKS) == 2; }

// (at least two partials: splitk_finish sums two or more, a single one is paired with zeros)
size_t conv_rows_wgrad_ws_bytes(int B, int cin, int cout) {
    return (size_t)std::max(2, std::min(B, std::max(cu_count(), 1))) * 9 * cin * cout * sizeof(float);
}

// one partial slab: the reduce that turns partials into dw needs two, so the second is zero
static int single_partial_pad(GemmParams& p, float* ws, size_t slab_floats, hipStream_t s) {
    if (p.splits > 1) return OCRK_OK;
    p.splits = 2;
    return hipMemsetAsync(ws + slab_floats, 0, slab_floats * sizeof(float), s) == hipSuccess ? OCRK_OK : OCRK_ERR_HIP;
}

// OCRK_CONV_ROWS_WIDE=0: the wider layers (conv3-conv6) stay on the GEMM / direct engines
static bool rows_wide_enabled() { return opt(OPT_CONV_ROWS_WIDE) != 0; }

static bool rows_fwd_wide(int cin, int cout) {
    // conv6's 128 -> 128 stays on the GEMM engine: one 8-wave workgroup spills
    // (146 vs 110 us), two 4-wave workgroups per band (CS = 2, one wave per SIMD at
    // 133 KB of ring) are latency-bound (158 us forward, 172 us backward-data)
    return (cin == 32 && cout == 64) || (cin == 64 && cout == 64) || (cin == 64 && cout == 128);
}

// forward with per-row BatchNorm partials (stats [B*H][2][cout], tile_rows = W)
bool conv_rows_fwd_covers(int B, int H, int W, int cin, int cout) {
    if (!rows_enabled() || W < 1 || H < 1 || B < 1) return false;
    if (cin == RW_CI && cout == RW_CO) return W <= RW_MAXW;
    return rows_wide_enabled() && rows_fwd_wide(cin, cout) && W <= 128;
}

int conv_rows_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout, void* y,
                  int relu, float* stats, hipStream_t s) {
    if (!conv_rows_fwd_covers(B, H, W, cin, cout)) return -1;
    if (cin != RW_CI || cout != RW_CO) {
        if (cin == 32) return launch_fwd_co<32, 64, 128>(x, B, H, W, w_nk, bias, y, relu, stats, s);
        if (cout == 64) return launch_fwd_co<64, 64, 128>(x, B, H, W, w_nk, bias, y, relu, stats, s);
        return launch_fwd_co<64, 128, 128>(x, B, H, W, w_nk, bias, y, relu, stats, s);
    }
    static DeviceOnce cfg, cfg_r;
    if (relu) {
        set_dyn_lds(cfg_r, reinterpret_cast<const void*>(&conv3x3_fwd_rows_kernel<true>), RD_LDS);
        conv3x3_fwd_rows_kernel<true><<<B * RD_BANDS, 256, RD_LDS, s>>>((const bf16*)x, (const bf16*)w_nk, bias, (bf16*)y,
                                                                        stats, B, H, W);
    } else {
        set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_fwd_rows_kernel<false>), RD_LDS);
        conv3x3_fwd_rows_kernel<false><<<B * RD_BANDS, 256, RD_LDS, s>>>((const bf16*)x, (const bf16*)w_nk, bias, (bf16*)y,
                                                                         stats, B, H, W);
    }
    return launch_status("conv3x3_fwd_rows");
}

// backward-data with the producer's ReLU mask, conv2's shape only (-1 otherwise)
int conv_rows_dgrad(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                    const void* relu_mask, float* stats, hipStream_t s) {
    if (!rows_enabled() || W < 1 || H < 1 || B < 1) return -1;
    if (rows_wide_enabled() && W <= 128) {
        if (cin == 64 && cout == 64) return launch_dgrad_co<64, 64, 128>(dy, B, H, W, w_bwd, dx, relu_mask, stats, s);
    }
    if (cin != RW_CI || cout != RW_CO || W > RW_MAXW) return -1;
    if (!relu_mask || stats) return -1;
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_dgrad_rows_kernel<0>), RD_LDS);
    conv3x3_dgrad_rows_kernel<0><<<B * RD_BANDS, 256, RD_LDS, s>>>((const bf16*)dy, (const bf16*)w_bwd,
                                                                   (const bf16*)relu_mask, (bf16*)dx, B, H, W,
                                                                   nullptr, nullptr);
    return launch_status("conv3x3_dgrad_rows");
}

// ReLU bit masks on the wide row kernels: the forward of conv3 / conv5 (32 -> 64, 64 -> 128;
// 64 -> 64 too) writes its output's bits, conv4's backward-data (64 <- 64) reads them
bool conv_rows_fwd_bits_covers(int B, int H, int W, int cin, int cout) {
    return conv_rows_fwd_covers(B, H, W, cin, cout) && !(cin == RW_CI && cout == RW_CO);
}

int conv_rows_fwd_bits(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias, int cout,
                       void* y, void* bits, hipStream_t s) {
    if (!conv_rows_fwd_bits_covers(B, H, W, cin, cout)) return -1;
    if (cin == 32) return launch_fwd_co<32, 64, 128>(x, B, H, W, w_nk, bias, y, 1, nullptr, s, bits);
    if (cout == 64) return launch_fwd_co<64, 64, 128>(x, B, H, W, w_nk, bias, y, 1, nullptr, s, bits);
    return launch_fwd_co<64, 128, 128>(x, B, H, W, w_nk, bias, y, 1, nullptr, s, bits);
}

bool conv_rows_dgrad_bits_covers(int B, int H, int W, int cin, int cout) {
    return rows_enabled() && rows_wide_enabled() && B >= 1 && H >= 1 && W >= 1 && W <= 128 && cin == 64 && cout == 64;
}

int conv_rows_dgrad_bits(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin, void* dx,
                         const void* bits, float* stats, hipStream_t s) {
    if (!conv_rows_dgrad_bits_covers(B, H, W, cin, cout)) return -1;
    return launch_dgrad_co<64, 64, 128, 1, true>(dy, B, H, W, w_bwd, dx, bits, stats, s);
}

#ifdef OCRK_EXPERIMENTS
// conv2's weight gradient with conv1's output recomputed from the image (no y1 tensor):
// dw [3][3][32][32] (+)= sum y1 (x) dz, y1 = relu(conv1(img)) produced per row by
// c1_make_row -- the bits conv12_fwd_rows_kernel made in the forward
constexpr int RW_LDS_C1X = RW_LDS + C12_XSLOTS * RD_XROW * 4;     // 155.6 KB (one workgroup per CU)

int conv_rows_wgrad_c1x(const void* img, int x_is_u8, const float* w1, const float* b1, const void* dy, int B, int H,
                        int W, float* dw, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
    if (!rows_enabled() || W < 1 || H < 1 || B < 1 || W > RW_MAXW) return -1;
    if (ws_bytes < conv_rows_wgrad_ws_bytes(B, RW_CI, RW_CO) || (uintptr_t)ws % 16 != 0) return -1;
    const int grid = std::min(B, std::max(cu_count(), 1));
    static DeviceOnce cfg_u8, cfg_bf;
    if (x_is_u8) {
        set_dyn_lds(cfg_u8, reinterpret_cast<const void*>(&conv3x3_wgrad_rows_kernel<1>), RW_LDS_C1X);
        conv3x3_wgrad_rows_kernel<1><<<grid, 256, RW_LDS_C1X, s>>>(nullptr, (const bf16*)dy, (float*)ws, B, H, W, img,
                                                                   w1, b1);
    } else {
        set_dyn_lds(cfg_bf, reinterpret_cast<const void*>(&conv3x3_wgrad_rows_kernel<2>), RW_LDS_C1X);
        conv3x3_wgrad_rows_kernel<2><<<grid, 256, RW_LDS_C1X, s>>>(nullptr, (const bf16*)dy, (float*)ws, B, H, W, img,
                                                                   w1, b1);
    }
    int st = launch_status("conv3x3_wgrad_rows_c1x");
    if (st) return st;
    GemmParams p = {};
    p.M = 9 * RW_CI; p.N = RW_CO; p.K = B * H * W; p.batch = 1;
    p.C = dw; p.ldc = RW_CO; p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
    p.splits = grid; p.splitk_ws = (float*)ws;
    return splitk_finish(p, s);
}
#endif  // OCRK_EXPERIMENTS

bool conv12_fwd_covers(int B, int H, int W) {
    return rows_enabled() && B >= 1 && H >= 1 && W >= 1 && W <= RW_MAXW;
}

// conv1 -> conv2 forward (conv12_fwd_rows_kernel): y1 [B,H,W,32] bf16 (or NULL: not written), bits [B,H,W] u32, z [B,H,W,32]
// bf16, stats [B*H][2][32] (conv2's per-row BN partials, tile_rows = W)
int conv12_fwd(const void* img, int x_is_u8, int B, int H, int W, const float* w1, const float* b1,
               const void* w_nk2, const float* b2, void* y1, void* bits, void* z, float* stats, hipStream_t s) {
    if (!conv12_fwd_covers(B, H, W)) return -1;
    auto go = [&](auto kern, DeviceOnce& cfg) {
        set_dyn_lds(cfg, reinterpret_cast<const void*>(kern), C12_LDS);
        kern<<<B * RD_BANDS, 256, C12_LDS, s>>>(img, w1, b1, (const bf16*)w_nk2, b2, (bf16*)y1, (unsigned*)bits,
                                                (bf16*)z, stats, B, H, W);
    };
    static DeviceOnce cfg[4];
    if (x_is_u8) {
        if (y1) go(conv12_fwd_rows_kernel<1, true>, cfg[0]);
        else go(conv12_fwd_rows_kernel<1, false>, cfg[1]);
    } else {
        if (y1) go(conv12_fwd_rows_kernel<2, true>, cfg[2]);
        else go(conv12_fwd_rows_kernel<2, false>, cfg[3]);
    }
    return launch_status("conv12_fwd_rows");
}

bool conv_rows_dgrad_c1_covers(int B, int H, int W, int cin, int cout) {
    return rows_enabled() && B >= 1 && H >= 1 && W >= 1 && W <= RW_MAXW && cin == RW_CI && cout == RW_CO;
}

int64_t conv_rows_dgrad_c1_parts(int B) { return (int64_t)B * RD_BANDS; }

// conv2's backward-data with conv1's weight gradient contracted in (no dx): one
// [10][32] f32 partial per workgroup into `part` ([B * RD_BANDS][10][32])
template <int XIN, bool BITS>
static void launch_dgrad_c1(const void* dy, int B, int H, int W, const void* w_bwd, const void* mask, const void* x,
                            float* part, hipStream_t s) {
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_dgrad_rows_kernel<XIN, BITS>), RD_LDS_C1);
    conv3x3_dgrad_rows_kernel<XIN, BITS><<<B * RD_BANDS, 256, RD_LDS_C1, s>>>(
        (const bf16*)dy, (const bf16*)w_bwd, (const bf16*)mask, nullptr, B, H, W, x, part);
}

int conv_rows_dgrad_c1(const void* dy, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                       const void* relu_bits, const void* x, int x_is_u8, float* part, hipStream_t s) {
    if (relu_bits) {
        if (x_is_u8) launch_dgrad_c1<1, true>(dy, B, H, W, w_bwd, relu_bits, x, part, s);
        else launch_dgrad_c1<2, true>(dy, B, H, W, w_bwd, relu_bits, x, part, s);
    } else {
        if (x_is_u8) launch_dgrad_c1<1, false>(dy, B, H, W, w_bwd, relu_mask, x, part, s);
        else launch_dgrad_c1<2, false>(dy, B, H, W, w_bwd, relu_mask, x, part, s);
    }
    return launch_status("conv3x3_dgrad_rows_c1");
}

int64_t conv_rows_bwd_w2_parts(int B) { return (int64_t)B; }

// conv2's whole backward with conv1's weight gradient as one row walk
// (conv12_bwd_rows_kernel): c1part [B][10 * 32] as conv_rows_dgrad_c1, and conv2's weight
// gradient dw2 [3][3][32][32] (+)= the sum of w2part [B][9216] in a fixed order (splitk_finish)
template <int XIN, bool BITS>
static void launch_bwd_w2(const void* dy, int B, int H, int W, const void* w_bwd, const void* mask, const void* x,
                          const float* w1, const float* b1, float* c1part, float* w2part, hipStream_t s) {
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv12_bwd_rows_kernel<XIN, BITS>), C12B_LDS);
    conv12_bwd_rows_kernel<XIN, BITS><<<B, 512, C12B_LDS, s>>>((const bf16*)dy, (const bf16*)w_bwd, (const bf16*)mask,
                                                               B, H, W, x, w1, b1, c1part, w2part);
}

int conv_rows_bwd_w2(const void* dy, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                     const void* relu_bits, const void* x, int x_is_u8, const float* w1, const float* b1,
                     float* c1part, float* w2part, float* dw2, int accumulate, hipStream_t s) {
    if (relu_bits) {
        if (x_is_u8) launch_bwd_w2<1, true>(dy, B, H, W, w_bwd, relu_bits, x, w1, b1, c1part, w2part, s);
        else launch_bwd_w2<2, true>(dy, B, H, W, w_bwd, relu_bits, x, w1, b1, c1part, w2part, s);
    } else {
        if (x_is_u8) launch_bwd_w2<1, false>(dy, B, H, W, w_bwd, relu_mask, x, w1, b1, c1part, w2part, s);
        else launch_bwd_w2<2, false>(dy, B, H, W, w_bwd, relu_mask, x, w1, b1, c1part, w2part, s);
    }
    int st = launch_status("conv12_bwd_rows");
    if (st) return st;
    GemmParams p = {};
    p.M = 9 * RW_CI; p.N = RW_CO; p.K = B * H * W; p.batch = 1;
    p.C = dw2; p.ldc = RW_CO; p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
    p.splits = (int)conv_rows_bwd_w2_parts(B); p.splitk_ws = w2part;
    st = single_partial_pad(p, w2part, RW_PART, s);
    return st ? st : splitk_finish(p, s);
}

// an XCT -> DCT layer as (XCT / CI) x (DCT / CO) channel blocks of CI x CO
template <int CI, int KPX, int CO = 64>
static int launch_rows_co(const void* x, const void* dy, int B, int H, int W, int xct, int dct, float* dw,
                          int accumulate, void* ws, hipStream_t s) {
    using C = RcCfg<CI, KPX, CO>;
    const int nci = xct / CI, nco = dct / CO, nb = nci * nco;
    // one round of workgroups over the blocks (one per CU: ~99 KB of LDS each). The
    // channel-block launches run on the side stream beside the conv backward's main
    // stream, so they take at most 192 CUs (the other weight-gradient launches' cap):
    // same box 5.096-5.100 vs 5.097-5.113 ms with all 256, 5.106-5.123 at 128
    // (OCRK_CONV_WGRAD_CUS overrides; 0 = every CU)
    const int cap = (int)opt(OPT_CONV_WGRAD_CUS);
    const int cus = (nb > 1 && cap > 0) ? std::min(cap, cu_count()) : cu_count();
    // (at least two: the split-K reduce sums two or more partials; a workgroup past the
    // batch writes zeros)
    const int grid = std::max(2, std::min(B, std::max(cus, 1) / nb));
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_wgrad_rows_co_kernel<CI, KPX, CO>), C::LDS);
    conv3x3_wgrad_rows_co_kernel<CI, KPX, CO><<<dim3(grid, nb), C::NT, C::LDS, s>>>(
        (const bf16*)x, (const bf16*)dy, (float*)ws, B, H, W, xct, dct, nco);
    int st = launch_status("conv3x3_wgrad_rows_co");
    if (st) return st;
    for (int q = 0; q < nb; ++q) {
        // block q: taps as the batch ([9][grid] slabs of CI x CO), each tap's rows at t * XCT
        GemmParams p = {};
        p.M = CI; p.N = CO; p.K = B * H * W; p.batch = 9;
        p.C = dw + (size_t)(q / nco) * CI * dct + (q % nco) * CO; p.ldc = dct; p.strideC = (int64_t)xct * dct;
        p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
        p.splits = grid; p.splitk_ws = (float*)ws + (size_t)q * 9 * grid * CI * CO;
        st = splitk_finish(p, s);
        if (st) return st;
    }
    return OCRK_OK;
}

// -1 when the shape is not conv2's (Cin = Cout = 32, W <= 254) or the path is off
int conv_rows_wgrad(const void* x, const void* dy, int B, int H, int W, int cin, int cout, float* dw, int accumulate,
                    void* ws, size_t ws_bytes, hipStream_t s) {
    if (!rows_enabled() || W < 1 || H < 1 || B < 1) return -1;
    if (ws_bytes < conv_rows_wgrad_ws_bytes(B, cin, cout) || (uintptr_t)ws % 16 != 0) return -1;
    if (cout == 64 && W <= 128) {                    // conv3 / conv4
        if (cin == 32) return launch_rows_co<32, 128>(x, dy, B, H, W, 32, 64, dw, accumulate, ws, s);
        if (cin == 64) return launch_rows_co<64, 128>(x, dy, B, H, W, 64, 64, dw, accumulate, ws, s);
        return -1;
    }
    // conv5 (64 -> 128) and conv6 (128 -> 128) as 64 x 64 channel blocks (one block as
    // one 8-wave workgroup would spill its 144-288 accumulator registers)
    if (cout == 128 && W <= 128 && (cin == 64 || cin == 128) && rows_wgrad_blocks())
        return launch_rows_co<64, 128>(x, dy, B, H, W, cin, 128, dw, accumulate, ws, s);
    if (cout == 256 && W <= 128 && (cin == 128 || cin == 256) && rows_wgrad_blocks_wide())
        return launch_rows_co<64, 128>(x, dy, B, H, W, cin, 256, dw, accumulate, ws, s);
    if (cin != RW_CI || cout != RW_CO || W > RW_MAXW) return -1;
    const int grid = std::max(2, std::min(B, std::max(cu_count(), 1)));   // (>= 2: as launch_rows_co)
    static DeviceOnce cfg;
    set_dyn_lds(cfg, reinterpret_cast<const void*>(&conv3x3_wgrad_rows_kernel<0>), RW_LDS);
    conv3x3_wgrad_rows_kernel<0><<<grid, 256, RW_LDS, s>>>((const bf16*)x, (const bf16*)dy, (float*)ws, B, H, W);
    int st = launch_status("conv3x3_wgrad_rows");
    if (st) return st;
    GemmParams p = {};
    p.M = 9 * cin; p.N = cout; p.K = B * H * W; p.batch = 1;
    p.C = dw; p.ldc = cout; p.c_bf16 = 0; p.accumulate = accumulate; p.alpha = 1.f;
    p.splits = grid; p.splitk_ws = (float*)ws;
    return splitk_finish(p, s);
}

}  // namespace ocrk
