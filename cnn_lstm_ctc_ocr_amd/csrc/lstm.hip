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
#include "common.h"
#include "mfma_util.h"

using namespace ocrk;

template <typename CT, int BR, int NC, int KC>
struct RecurCore {
    using RT = typename RawT<CT>::T;
    static constexpr int LDK = KC + 8;
    static constexpr int NVA = (BR * KC / 8 + 255) / 256;
    static constexpr int NVB = (NC * KC / 8 + 255) / 256;
    static constexpr int TILES = (BR / 16) * (NC / 16);
    static constexpr int TPW = TILES >= 4 ? TILES / 4 : 1;
    static constexpr int STAGE_BYTES = 2 * (BR + NC) * LDK * (int)sizeof(RT);
    static constexpr int EPI_BYTES = BR * (NC + 1) * 4;
    static constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
    static_assert(TILES % 4 == 0 || TILES < 4, "tile split");

    template <typename BCol>
    __device__ __forceinline__ static void load(V8<CT> (&ra)[NVA], V8<CT> (&rb)[NVB], const CT* __restrict__ a_rows,
                                                int64_t lda, const BCol& bcol, int k0) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            if (idx < BR * KC / 8) {
                int r = idx / (KC / 8), kq = idx % (KC / 8);
                vload(ra[v], a_rows + (int64_t)r * lda + k0 + 8 * kq);
            }
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            if (idx < NC * KC / 8) {
                int n = idx / (KC / 8), kq = idx % (KC / 8);
                vload(rb[v], bcol(n) + k0 + 8 * kq);
            }
        }
    }
    __device__ __forceinline__ static void store(const V8<CT> (&ra)[NVA], const V8<CT> (&rb)[NVB], RT* sA, RT* sB,
                                                 int buf) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int v = 0; v < NVA; ++v) {
            int idx = tid + 256 * v;
            if (idx < BR * KC / 8)
                vstore_lds(sA + buf * BR * LDK + (idx / (KC / 8)) * LDK + 8 * (idx % (KC / 8)), ra[v]);
        }
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
            int idx = tid + 256 * v;
            if (idx < NC * KC / 8)
                vstore_lds(sB + buf * NC * LDK + (idx / (KC / 8)) * LDK + 8 * (idx % (KC / 8)), rb[v]);
        }
    }
    __device__ __forceinline__ static void compute(floatx4 (&acc)[TPW], const RT* sA, const RT* sB, int buf) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            int q = wave + 4 * i;
            if (q >= TILES) break;
            int tm = q / (NC / 16), tn = q % (NC / 16);
            const RT* a = sA + buf * BR * LDK + (tm * 16 + (lane & 15)) * LDK + 8 * (lane >> 4);
            const RT* b = sB + buf * NC * LDK + (tn * 16 + (lane & 15)) * LDK + 8 * (lane >> 4);
#pragma unroll
            for (int ks = 0; ks < KC / 32; ++ks) {
                if constexpr (sizeof(CT) == 2) {
                    bf16x8 af = *reinterpret_cast<const bf16x8*>(a + ks * 32);
                    bf16x8 bfr = *reinterpret_cast<const bf16x8*>(b + ks * 32);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i], 0, 0, 0);
                } else {
                    V8<float> af, bfr;
                    vload_lds(af, a + ks * 32);
                    vload_lds(bfr, b + ks * 32);
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af.e(kk), bfr.e(kk), acc[i], 0, 0, 0);
                }
            }
        }
    }

    // acc <- A[BR, K] . Bcols[NC, K]^T ; A rows at a_rows + r*lda, B col n at bcol(n).
    // Two register sets (chunks c+1, c+2) in flight while chunk c is on MFMA.
    template <typename BCol>
    __device__ __forceinline__ static void run(const CT* __restrict__ a_rows, int64_t lda, const BCol& bcol, int K,
                                               char* lds, floatx4 (&acc)[TPW]) {
        RT* sA = reinterpret_cast<RT*>(lds);
        RT* sB = sA + 2 * BR * LDK;
#pragma unroll
        for (int i = 0; i < TPW; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        V8<CT> ra0[NVA], rb0[NVB], ra1[NVA], rb1[NVB];
        const int nch = K / KC;
        load(ra0, rb0, a_rows, lda, bcol, 0);
        if (nch > 1) load(ra1, rb1, a_rows, lda, bcol, KC);
        store(ra0, rb0, sA, sB, 0);
        __syncthreads();
        for (int c = 0; c < nch; c += 2) {
            if (c + 2 < nch) load(ra0, rb0, a_rows, lda, bcol, (c + 2) * KC);
            compute(acc, sA, sB, 0);
            if (c + 1 < nch) store(ra1, rb1, sA, sB, 1);
            __syncthreads();
            if (c + 1 >= nch) break;
            if (c + 3 < nch) load(ra1, rb1, a_rows, lda, bcol, (c + 3) * KC);
            compute(acc, sA, sB, 1);
            if (c + 2 < nch) store(ra0, rb0, sA, sB, 0);
            __syncthreads();
        }
    }

    // accumulators -> LDS [BR][NC+1] f32 (call after run(); ends with a barrier)
    __device__ static void spill(const floatx4 (&acc)[TPW], char* lds) {
        float* sG = reinterpret_cast<float*>(lds);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            int q = wave + 4 * i;
            if (q >= TILES) break;
            int tm = q / (NC / 16), tn = q % (NC / 16);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sG[(tm * 16 + (lane >> 4) * 4 + r) * (NC + 1) + tn * 16 + (lane & 15)] = acc[i][r];
        }
        __syncthreads();
    }
};

__device__ __forceinline__ int step_time(int dir, int s, int len) {
    return (dir == 0 || s >= len) ? s : len - 1 - s;
}

// --------------------------------------------------------------- forward
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
lstm_fwd_step_kernel(const float* __restrict__ gx, const CT* __restrict__ whT, const CT* __restrict__ h_in,
                     CT* __restrict__ h_out, float* __restrict__ c_state, const int* __restrict__ seq_len,
                     int s, int T, int B, int H, CT* __restrict__ out, CT* __restrict__ hprev_t,
                     float* __restrict__ cprev_t, float* __restrict__ acts_t) {
    using Core = RecurCore<CT, BR, 4 * HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const int u0 = blockIdx.x * HU, b0 = blockIdx.y * BR, dir = blockIdx.z;
    const CT* a_rows = h_in + ((int64_t)dir * B + b0) * H;
    const CT* wdir = whT + (int64_t)dir * 4 * H * H;
    auto bcol = [&](int n) { return wdir + (int64_t)((n / HU) * H + u0 + (n % HU)) * H; };
    floatx4 acc[Core::TPW];
    Core::run(a_rows, H, bcol, H, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
    const int G4 = 4 * H;
    for (int idx = threadIdx.x; idx < BR * HU; idx += 256) {
        const int r = idx / HU, u = idx % HU, b = b0 + r, uu = u0 + u;
        const int len = seq_len[b];
        const bool valid = s < len;
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;          // state index
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;           // time-order row
        const float hp = to_f32(h_in[st]);
        const float cp = c_state[st];
        if (valid) {
            const float* g = gx + tb * G4;
            float pi = sG[r * (4 * HU + 1) + 0 * HU + u] + g[0 * H + uu];
            float pj = sG[r * (4 * HU + 1) + 1 * HU + u] + g[1 * H + uu];
            float pf = sG[r * (4 * HU + 1) + 2 * HU + u] + g[2 * H + uu];
            float po = sG[r * (4 * HU + 1) + 3 * HU + u] + g[3 * H + uu];
            float ai = sigmoidf_(pi), aj = tanhf(pj), af = sigmoidf_(pf + 1.0f), ao = sigmoidf_(po);
            float c = af * cp + ai * aj;
            float h = ao * tanhf(c);
            c_state[st] = c;
            h_out[st] = from_f32<CT>(h);
            out[((int64_t)t * B + b) * 2 * H + dir * H + uu] = from_f32<CT>(h);
            hprev_t[tb * H + uu] = from_f32<CT>(hp);
            cprev_t[tb * H + uu] = cp;
            float* a = acts_t + tb * G4;
            a[0 * H + uu] = ai; a[1 * H + uu] = aj; a[2 * H + uu] = af; a[3 * H + uu] = ao;
        } else {
            h_out[st] = h_in[st];
            hprev_t[tb * H + uu] = from_f32<CT>(0.f);
            cprev_t[tb * H + uu] = 0.f;
            float* a = acts_t + tb * G4;
            a[0 * H + uu] = 0.f; a[1 * H + uu] = 0.f; a[2 * H + uu] = 0.f; a[3 * H + uu] = 0.f;
        }
    }
}

// -------------------------------------------------------------- backward
template <typename CT, int BR, int HU, int KC>
__global__ void __launch_bounds__(256)
lstm_bwd_step_kernel(const CT* __restrict__ wh, const CT* __restrict__ dg_in, CT* __restrict__ dg_out,
                     float* __restrict__ dc_state, const int* __restrict__ seq_len, int s, int T, int B, int H,
                     const CT* __restrict__ dout, const float* __restrict__ cprev_t,
                     const float* __restrict__ acts_t, CT* __restrict__ dG_t) {
    using Core = RecurCore<CT, BR, HU, KC>;
    __shared__ __attribute__((aligned(16))) char lds[Core::LDS_BYTES];
    const int u0 = blockIdx.x * HU, b0 = blockIdx.y * BR, dir = blockIdx.z;
    const int G4 = 4 * H;
    const CT* a_rows = dg_in + ((int64_t)dir * B + b0) * G4;
    const CT* wdir = wh + (int64_t)dir * H * G4;
    auto bcol = [&](int n) { return wdir + (int64_t)(u0 + n) * G4; };
    floatx4 acc[Core::TPW];
    Core::run(a_rows, G4, bcol, G4, lds, acc);
    Core::spill(acc, lds);
    const float* sG = reinterpret_cast<const float*>(lds);
    for (int idx = threadIdx.x; idx < BR * HU; idx += 256) {
        const int r = idx / HU, u = idx % HU, b = b0 + r, uu = u0 + u;
        const int len = seq_len[b];
        const bool valid = s < len;
        const int t = step_time(dir, s, len);
        const int64_t st = ((int64_t)dir * B + b) * H + uu;
        const int64_t tb = ((int64_t)t * B + b) * 2 + dir;
        CT* dgo = dg_out + ((int64_t)dir * B + b) * G4;
        CT* dgt = dG_t + tb * G4;
        if (valid) {
            float dh = sG[r * (HU + 1) + u] + to_f32(dout[((int64_t)t * B + b) * 2 * H + dir * H + uu]);
            const float* a = acts_t + tb * G4;
            float ai = a[0 * H + uu], aj = a[1 * H + uu], af = a[2 * H + uu], ao = a[3 * H + uu];
            float cp = cprev_t[tb * H + uu];
            float c = af * cp + ai * aj;
            float tc = tanhf(c);
            float dc = dc_state[st] + dh * ao * (1.f - tc * tc);
            float d_o = dh * tc * ao * (1.f - ao);
            float d_i = dc * aj * ai * (1.f - ai);
            float d_j = dc * ai * (1.f - aj * aj);
            float d_f = dc * cp * af * (1.f - af);
            dc_state[st] = dc * af;
            CT vi = from_f32<CT>(d_i), vj = from_f32<CT>(d_j), vf = from_f32<CT>(d_f), vo = from_f32<CT>(d_o);
            dgo[0 * H + uu] = vi; dgo[1 * H + uu] = vj; dgo[2 * H + uu] = vf; dgo[3 * H + uu] = vo;
            dgt[0 * H + uu] = vi; dgt[1 * H + uu] = vj; dgt[2 * H + uu] = vf; dgt[3 * H + uu] = vo;
        } else {
            CT z = from_f32<CT>(0.f);
            dc_state[st] = 0.f;
            dgo[0 * H + uu] = z; dgo[1 * H + uu] = z; dgo[2 * H + uu] = z; dgo[3 * H + uu] = z;
            dgt[0 * H + uu] = z; dgt[1 * H + uu] = z; dgt[2 * H + uu] = z; dgt[3 * H + uu] = z;
        }
    }
}

// ------------------------------------------------------------------ C ABI
// Tile shapes: bf16 BR=64 x HU=16 (fwd K-chunk 128, bwd 256); f32 BR=32 x HU=8/16.
#define FWD_BF16 bf16, 64, 16, 128
#define FWD_F32 float, 32, 8, 64
#define BWD_BF16 bf16, 64, 16, 256
#define BWD_F32 float, 32, 16, 128

extern "C" int ocrk_lstm_fwd_step(const float* gx, const void* whT, const void* h_in, void* h_out,
                                  float* c_state, const int* seq_len, int s, int T, int B, int H, void* out,
                                  void* hprev_t, float* cprev_t, float* acts_t, int dtype, void* stream) {
    hipStream_t st = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16) {
        OCRK_REQUIRE(H % 128 == 0 && B % 64 == 0, "ocrk_lstm_fwd_step: bf16 needs H %% 128 == 0 and B %% 64 == 0 (H=%d B=%d)", H, B);
        dim3 grid(H / 16, B / 64, 2);
        lstm_fwd_step_kernel<FWD_BF16><<<grid, 256, 0, st>>>(gx, (const bf16*)whT, (const bf16*)h_in, (bf16*)h_out, c_state, seq_len, s, T, B, H, (bf16*)out, (bf16*)hprev_t, cprev_t, acts_t);
    } else {
        OCRK_REQUIRE(H % 64 == 0 && B % 32 == 0, "ocrk_lstm_fwd_step: f32 needs H %% 64 == 0 and B %% 32 == 0 (H=%d B=%d)", H, B);
        dim3 grid(H / 8, B / 32, 2);
        lstm_fwd_step_kernel<FWD_F32><<<grid, 256, 0, st>>>(gx, (const float*)whT, (const float*)h_in, (float*)h_out, c_state, seq_len, s, T, B, H, (float*)out, (float*)hprev_t, cprev_t, acts_t);
    }
    return ocrk::launch_status("ocrk_lstm_fwd_step");
}

extern "C" int ocrk_lstm_bwd_step(const void* wh, const void* dg_in, void* dg_out, float* dc_state,
                                  const int* seq_len, int s, int T, int B, int H, const void* dout,
                                  const float* cprev_t, const float* acts_t, void* dG_t, int dtype,
                                  void* stream) {
    hipStream_t st = ocrk::as_stream(stream);
    if (dtype == OCRK_BF16) {
        OCRK_REQUIRE(H % 64 == 0 && B % 64 == 0, "ocrk_lstm_bwd_step: bf16 needs H %% 64 == 0 and B %% 64 == 0");
        dim3 grid(H / 16, B / 64, 2);
        lstm_bwd_step_kernel<BWD_BF16><<<grid, 256, 0, st>>>((const bf16*)wh, (const bf16*)dg_in, (bf16*)dg_out, dc_state, seq_len, s, T, B, H, (const bf16*)dout, cprev_t, acts_t, (bf16*)dG_t);
    } else {
        OCRK_REQUIRE(H % 32 == 0 && B % 32 == 0, "ocrk_lstm_bwd_step: f32 needs H %% 32 == 0 and B %% 32 == 0");
        dim3 grid(H / 16, B / 32, 2);
        lstm_bwd_step_kernel<BWD_F32><<<grid, 256, 0, st>>>((const float*)wh, (const float*)dg_in, (float*)dg_out, dc_state, seq_len, s, T, B, H, (const float*)dout, cprev_t, acts_t, (float*)dG_t);
    }
    return ocrk::launch_status("ocrk_lstm_bwd_step");
}

// Whole time loops (T launches each) so a binding makes one call per layer.
extern "C" int ocrk_lstm_fwd(const float* gx, const void* whT, void* h_state /*[2 bufs][2][B][H]*/,
                             float* c_state, const int* seq_len, int T, int B, int H, void* out, void* hprev_t,
                             float* cprev_t, float* acts_t, int dtype, void* stream) {
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
                             const float* acts_t, void* dG_t, int dtype, void* stream) {
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
