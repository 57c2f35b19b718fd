// a7: the bidirectional GRU time loop of rnn_layer (src/weinman/model.py:167-199,
// tf.contrib.rnn.GRUCell, bidirectional_dynamic_rnn(time_major, sequence_length)).
// [TF1] GRUCell: [r, u] = sig([x, h] Wg + bg); c = tanh([x, r*h] Wc + bc);
// h' = u h + (1 - u) c -- the reset gate multiplies h BEFORE the candidate
// matmul, so each step is two dependent GEMMs.
//
// As for the LSTM (lstm.hip) the input projections x_t . [Wg_x | Wc_x] + b of
// every t and both directions are ONE GEMM before the loop (N = 6H, per
// direction [r | u | c]). Per step and for both directions at once:
//   gate kernel : h . Wg_h (N = 2H) -> r, u; publishes r*h for
//   cand kernel : (r*h) . Wc_h (N = H) -> c, h'.
// Backward per reverse step s:
//   cand kernel : d(rh) = dz_c . Wc_h^T (K = H) -> dz_r, dz_u, and the direct
//                 terms dh_tot*u + d(rh)*r of dh_prev;
//   gate kernel : dh_prev = [dz_r, dz_u] . Wg_h^T (K = 2H) + direct terms,
//                 then dh_tot and dz_c of step s-1 (fused, so the next
//                 launch's GEMM operand is ready).
// All saved tensors are in time order [T][B][2][*] so the weight gradients
// are plain GEMMs afterwards. Steps s >= len carry h and emit zeros.
#include "recur.h"

using namespace ocrk;

namespace {

// ------------------------------------------------------------ forward gate
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
gru_fwd_gate_kernel(const CT* __restrict__ gx, const CT* __restrict__ whgT, const CT* __restrict__ h,
                    CT* __restrict__ rh, const int* __restrict__ seq_len, int s, int B, int H,
                    CT* __restrict__ rh_t, CT* __restrict__ acts_t) {
    using Core = RecurCore<CT, BR, 2 * HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G3 = 3 * H;
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    constexpr bool EFULL = (BR * UQ) % 256 == 0;
    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
    const CT* a_rows = h + ((int64_t)dir * B + b0) * H;
    const CT* wdir = whgT + (int64_t)dir * 2 * H * H;
    auto bcol = [&](int n) { return wdir + (int64_t)((n / HU) * H + u0 + (n % HU)) * H; };
    Core core;
    core.begin(a_rows, H, bcol, H);
    float pg[EPQ4][2][4], ph[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        ld4(ph[q], h + ((int64_t)dir * B + b) * H + uu);
        const int t = step_time(dir, s, plen[q]);
        const CT* g = gx + (((int64_t)t * B + b) * 2 + dir) * G3 + uu;
        ld4(pg[q][0], g);
        ld4(pg[q][1], g + H);
    }
    floatx4 acc[Core::TPW];
    core.finish(a_rows, H, bcol, H, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int len = plen[q];
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
        CT* a = acts_t + tb * G3 + uu;
        if (s < len) {
            const float* gl = sG + r * (2 * HU + 1) + u;
            float ar[4], au[4], v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                ar[e] = sig_fast(gl[e] + pg[q][0][e]);
                au[e] = sig_fast(gl[HU + e] + pg[q][1][e]);
                v[e] = ar[e] * ph[q][e];
            }
            st4(rh + st, v);
            st4(rh_t + tb * H + uu, v);
            st4(a, ar);
            st4(a + H, au);
        } else {
            const float z[4] = {0.f, 0.f, 0.f, 0.f};
            st4(rh + st, z);
            st4(rh_t + tb * H + uu, z);
            st4(a, z);
            st4(a + H, z);
        }
    }
}

// ------------------------------------------------------- forward candidate
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
gru_fwd_cand_kernel(const CT* __restrict__ gx, const CT* __restrict__ whcT, const CT* __restrict__ rh,
                    CT* __restrict__ h, const int* __restrict__ seq_len, int s, int B, int H,
                    CT* __restrict__ out, CT* __restrict__ hprev_t, CT* __restrict__ acts_t) {
    using Core = RecurCore<CT, BR, HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G3 = 3 * H;
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    constexpr bool EFULL = (BR * UQ) % 256 == 0;
    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
    const CT* a_rows = rh + ((int64_t)dir * B + b0) * H;
    const CT* wdir = whcT + (int64_t)dir * H * H;
    auto bcol = [&](int n) { return wdir + (int64_t)(u0 + n) * H; };
    Core core;
    core.begin(a_rows, H, bcol, H);
    float pgc[EPQ4][4], ph[EPQ4][4], pu[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        ld4(ph[q], h + ((int64_t)dir * B + b) * H + uu);
        const int t = step_time(dir, s, plen[q]);
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
        ld4(pgc[q], gx + tb * G3 + 2 * H + uu);
        ld4(pu[q], acts_t + tb * G3 + H + uu);
    }
    floatx4 acc[Core::TPW];
    core.finish(a_rows, H, bcol, H, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int len = plen[q];
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
        if (s < len) {
            const float* gl = sG + r * (HU + 1) + u;
            float c[4], hn[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                c[e] = tanh_fast(gl[e] + pgc[q][e]);
                hn[e] = pu[q][e] * ph[q][e] + (1.f - pu[q][e]) * c[e];
            }
            st4(h + st, hn);
            st4(out + ((int64_t)t * B + b) * 2 * H + dir * H + uu, hn);
            st4(hprev_t + tb * H + uu, ph[q]);
            st4(acts_t + tb * G3 + 2 * H + uu, c);
        } else {
            const float z[4] = {0.f, 0.f, 0.f, 0.f};
            st4(hprev_t + tb * H + uu, z);
            st4(acts_t + tb * G3 + 2 * H + uu, z);
        }
    }
}

// dh_tot and dz_c of step s for one (row, 4 units), given the carried dh.
template <typename CT>
__device__ __forceinline__ void gru_bwd_head(int dir, int s, int len, int b, int uu, int B, int H,
                                             const float (&dh)[4], const CT* __restrict__ dout,
                                             const CT* __restrict__ acts_t, float* __restrict__ dh_tot,
                                             CT* __restrict__ dzc, CT* __restrict__ dG_t) {
    const int t = step_time(dir, s, len);
    const int64_t st = ((int64_t)dir * B + b) * H + uu;
    const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
    float d[4], z[4];
    if (s < len) {
        float go[4], au[4], ac[4];
        ld4(go, dout + ((int64_t)t * B + b) * 2 * H + dir * H + uu);
        ld4(au, acts_t + tb * 3 * H + H + uu);
        ld4(ac, acts_t + tb * 3 * H + 2 * H + uu);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            d[e] = dh[e] + go[e];
            z[e] = d[e] * (1.f - au[e]) * (1.f - ac[e] * ac[e]);
        }
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = z[e] = 0.f;
    }
    st4(dh_tot + st, d);
    st4(dzc + st, z);
    st4(dG_t + tb * 3 * H + 2 * H + uu, z);
}

template <typename CT>
__global__ void __launch_bounds__(256)
gru_bwd_prep_kernel(const int* __restrict__ seq_len, int s, int B, int H, const CT* __restrict__ dout,
                    const CT* __restrict__ acts_t, float* __restrict__ dh_tot, CT* __restrict__ dzc,
                    CT* __restrict__ dG_t) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;      // (dir, b, unit quad)
    const int UQ = H / 4;
    if (i >= (int64_t)2 * B * UQ) return;
    const int dir = (int)(i / ((int64_t)B * UQ)), rem = (int)(i % ((int64_t)B * UQ));
    const int b = rem / UQ, uu = 4 * (rem % UQ);
    const float zero[4] = {0.f, 0.f, 0.f, 0.f};
    gru_bwd_head<CT>(dir, s, seq_len[b], b, uu, B, H, zero, dout, acts_t, dh_tot, dzc, dG_t);
}

// ------------------------------------------------------ backward candidate
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
gru_bwd_cand_kernel(const CT* __restrict__ whc, const CT* __restrict__ dzc, const float* __restrict__ dh_tot,
                    CT* __restrict__ dzg, float* __restrict__ direct, const int* __restrict__ seq_len, int s,
                    int B, int H, const CT* __restrict__ hprev_t, const CT* __restrict__ acts_t,
                    CT* __restrict__ dG_t) {
    using Core = RecurCore<CT, BR, HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    const int G3 = 3 * H;
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    constexpr bool EFULL = (BR * UQ) % 256 == 0;
    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
    const CT* a_rows = dzc + ((int64_t)dir * B + b0) * H;
    const CT* wdir = whc + (int64_t)dir * H * H;
    auto bcol = [&](int n) { return wdir + (int64_t)(u0 + n) * H; };
    Core core;
    core.begin(a_rows, H, bcol, H);
    float pa[EPQ4][3][4], php[EPQ4][4], pd[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int t = step_time(dir, s, plen[q]);
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
#pragma unroll
        for (int k = 0; k < 3; ++k) ld4(pa[q][k], acts_t + tb * G3 + k * H + uu);
        ld4(php[q], hprev_t + tb * H + uu);
        ld4(pd[q], dh_tot + ((int64_t)dir * B + b) * H + uu);
    }
    floatx4 acc[Core::TPW];
    core.finish(a_rows, H, bcol, H, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int len = plen[q];
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
        CT* g = dzg + ((int64_t)dir * B + b) * 2 * H + uu;
        CT* gt = dG_t + tb * G3 + uu;
        if (s < len) {
            const float* gl = sG + r * (HU + 1) + u;
            float dzr[4], dzu[4], dd[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float drh = gl[e];
                const float ar = pa[q][0][e], au = pa[q][1][e], ac = pa[q][2][e], hp = php[q][e];
                const float dt = pd[q][e];
                dzr[e] = drh * hp * ar * (1.f - ar);
                dzu[e] = dt * (hp - ac) * au * (1.f - au);
                dd[e] = dt * au + drh * ar;
            }
            st4(g, dzr); st4(g + H, dzu);
            st4(gt, dzr); st4(gt + H, dzu);
            st4(direct + st, dd);
        } else {
            const float z[4] = {0.f, 0.f, 0.f, 0.f};
            st4(g, z); st4(g + H, z);
            st4(gt, z); st4(gt + H, z);
            st4(direct + st, z);
        }
    }
}

// ----------------------------------------------------------- backward gate
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
gru_bwd_gate_kernel(const CT* __restrict__ whg, const CT* __restrict__ dzg, const float* __restrict__ direct,
                    float* __restrict__ dh_tot, CT* __restrict__ dzc, const int* __restrict__ seq_len, int s,
                    int B, int H, const CT* __restrict__ dout, const CT* __restrict__ acts_t,
                    CT* __restrict__ dG_t) {
    using Core = RecurCore<CT, BR, HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const StepTile tl = step_tile(H / HU, B / BR);
    const int u0 = tl.u * HU, b0 = tl.b * BR, dir = tl.dir;
    constexpr int UQ = HU / 4, EPQ4 = (BR * UQ + 255) / 256;
    constexpr bool EFULL = (BR * UQ) % 256 == 0;
    int plen[EPQ4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) plen[q] = seq_len[b0 + min((int)threadIdx.x + 256 * q, BR * UQ - 1) / UQ];
    const CT* a_rows = dzg + ((int64_t)dir * B + b0) * 2 * H;
    const CT* wdir = whg + (int64_t)dir * H * 2 * H;
    auto bcol = [&](int n) { return wdir + (int64_t)(u0 + n) * 2 * H; };
    Core core;
    core.begin(a_rows, 2 * H, bcol, 2 * H);
    float pdd[EPQ4][4];
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        ld4(pdd[q], direct + ((int64_t)dir * B + b) * H + uu);
    }
    floatx4 acc[Core::TPW];
    core.finish(a_rows, 2 * H, bcol, 2 * H, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
#pragma unroll
    for (int q = 0; q < EPQ4; ++q) {
        const int idx = threadIdx.x + 256 * q;
        if (!EFULL && idx >= BR * UQ) continue;
        const int r = idx / UQ, u = 4 * (idx % UQ), b = b0 + r, uu = u0 + u;
        const int len = plen[q];
        float dh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dh[e] = s < len ? sG[r * (HU + 1) + u + e] + pdd[q][e] : 0.f;
        if (s > 0) gru_bwd_head<CT>(dir, s - 1, len, b, uu, B, H, dh, dout, acts_t, dh_tot, dzc, dG_t);
    }
}

}  // namespace

// ------------------------------------------------------------------ C ABI
// Tile shapes: bf16 BR=64 x HU=16, K chunk 256 (H % 256 == 0); f32 BR=32, K chunk 64.
#define GATE_BF16 bf16, 64, 16, 256
#define CAND_BF16 bf16, 64, 16, 256
#define GATE_F32 float, 32, 8, 64
#define CAND_F32 float, 32, 16, 64

static int gru_check(const char* what, int B, int H, int dtype) {
    if (dtype == OCRK_BF16) {
        OCRK_REQUIRE(H % 256 == 0 && B % 64 == 0, "%s: bf16 needs H %% 256 == 0 and B %% 64 == 0 (H=%d B=%d)", what,
                     H, B);
    } else {
        OCRK_REQUIRE(dtype == OCRK_F32, "%s: dtype", what);
        OCRK_REQUIRE(H % 64 == 0 && B % 32 == 0, "%s: f32 needs H %% 64 == 0 and B %% 32 == 0 (H=%d B=%d)", what, H,
                     B);
    }
    return OCRK_OK;
}

extern "C" int ocrk_gru_fwd_step(const void* gx, const void* whgT, const void* whcT, void* h, void* rh,
                                 const int* seq_len, int s, int T, int B, int H, void* out, void* hprev_t,
                                 void* rh_t, void* acts_t, int dtype, void* stream) {
    if (int e = gru_check("ocrk_gru_fwd_step", B, H, dtype)) return e;
    OCRK_REQUIRE(s >= 0 && s < T, "ocrk_gru_fwd_step: step %d not in [0, %d)", s, T);
    hipStream_t st = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16) {
        gru_fwd_gate_kernel<GATE_BF16><<<dim3(H / 16 * (B / 64) * 2), 256, 0, st>>>(
            (const bf16*)gx, (const bf16*)whgT, (const bf16*)h, (bf16*)rh, seq_len, s, B, H, (bf16*)rh_t, (bf16*)acts_t);
        gru_fwd_cand_kernel<CAND_BF16><<<dim3(H / 16 * (B / 64) * 2), 256, 0, st>>>(
            (const bf16*)gx, (const bf16*)whcT, (const bf16*)rh, (bf16*)h, seq_len, s, B, H, (bf16*)out, (bf16*)hprev_t,
            (bf16*)acts_t);
    } else {
        gru_fwd_gate_kernel<GATE_F32><<<dim3(H / 8 * (B / 32) * 2), 256, 0, st>>>(
            (const float*)gx, (const float*)whgT, (const float*)h, (float*)rh, seq_len, s, B, H, (float*)rh_t, (float*)acts_t);
        gru_fwd_cand_kernel<CAND_F32><<<dim3(H / 16 * (B / 32) * 2), 256, 0, st>>>(
            (const float*)gx, (const float*)whcT, (const float*)rh, (float*)h, seq_len, s, B, H, (float*)out, (float*)hprev_t,
            (float*)acts_t);
    }
    return ocrk::launch_status("ocrk_gru_fwd_step");
}

extern "C" int ocrk_gru_fwd(const void* gx, const void* whgT, const void* whcT, void* h, void* rh,
                            const int* seq_len, int T, int B, int H, void* out, void* hprev_t, void* rh_t,
                            void* acts_t, int dtype, void* stream) {
    for (int s = 0; s < T; ++s) {
        int e = ocrk_gru_fwd_step(gx, whgT, whcT, h, rh, seq_len, s, T, B, H, out, hprev_t, rh_t, acts_t, dtype,
                                  stream);
        if (e) return e;
    }
    return OCRK_OK;
}

extern "C" int ocrk_gru_bwd(const void* whg, const void* whc, void* dzg, void* dzc, float* dh_tot, float* direct,
                            const int* seq_len, int T, int B, int H, const void* dout, const void* hprev_t,
                            const void* acts_t, void* dG_t, int dtype, void* stream) {
    if (int e = gru_check("ocrk_gru_bwd", B, H, dtype)) return e;
    if (T <= 0) return OCRK_OK;
    hipStream_t st = ocrk::as_stream(stream);
    const int prep_blocks = (int)ocrk::cdiv((int64_t)2 * B * (H / 4), 256);
    if (dtype == OCRK_BF16) {
        gru_bwd_prep_kernel<bf16><<<prep_blocks, 256, 0, st>>>(seq_len, T - 1, B, H, (const bf16*)dout,
                                                               (const bf16*)acts_t, dh_tot, (bf16*)dzc,
                                                               (bf16*)dG_t);
        for (int s = T - 1; s >= 0; --s) {
            gru_bwd_cand_kernel<CAND_BF16><<<dim3(H / 16 * (B / 64) * 2), 256, 0, st>>>(
                (const bf16*)whc, (const bf16*)dzc, dh_tot, (bf16*)dzg, direct, seq_len, s, B, H,
                (const bf16*)hprev_t, (const bf16*)acts_t, (bf16*)dG_t);
            gru_bwd_gate_kernel<GATE_BF16><<<dim3(H / 16 * (B / 64) * 2), 256, 0, st>>>(
                (const bf16*)whg, (const bf16*)dzg, direct, dh_tot, (bf16*)dzc, seq_len, s, B, H,
                (const bf16*)dout, (const bf16*)acts_t, (bf16*)dG_t);
        }
    } else {
        gru_bwd_prep_kernel<float><<<prep_blocks, 256, 0, st>>>(seq_len, T - 1, B, H, (const float*)dout,
                                                                (const float*)acts_t, dh_tot, (float*)dzc,
                                                                (float*)dG_t);
        for (int s = T - 1; s >= 0; --s) {
            gru_bwd_cand_kernel<CAND_F32><<<dim3(H / 16 * (B / 32) * 2), 256, 0, st>>>(
                (const float*)whc, (const float*)dzc, dh_tot, (float*)dzg, direct, seq_len, s, B, H,
                (const float*)hprev_t, (const float*)acts_t, (float*)dG_t);
            gru_bwd_gate_kernel<CAND_F32><<<dim3(H / 16 * (B / 32) * 2), 256, 0, st>>>(
                (const float*)whg, (const float*)dzg, direct, dh_tot, (float*)dzc, seq_len, s, B, H,
                (const float*)dout, (const float*)acts_t, (float*)dG_t);
        }
    }
    return ocrk::launch_status("ocrk_gru_bwd");
}
