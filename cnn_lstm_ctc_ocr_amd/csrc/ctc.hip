// a9/a10: CTC loss + gradient w.r.t. logits, and the greedy decoder.
//
// ctc_loss_layer (src/weinman/model.py:224-229) calls tf.nn.ctc_loss with
// time_major logits [T, B, C], preprocess_collapse_repeated=False,
// ctc_merge_repeated=True; blank = C - 1. validate._get_output
// (src/weinman/validate.py:81-92) calls tf.nn.ctc_greedy_decoder(merge_repeated=True).
//
// Layout / work split: one 1024-thread workgroup per sequence b. The extended
// label l' = [blank, l1, blank, l2, ..., blank] (S = 2L+1 states) lives in
// registers of a single wave: lane j holds states j, j+64, ... (R registers).
// The frame log-sum-exps (DPP wave reductions) and the emission log-probs of
// the extended label are gathered first with many loads in flight, the frame
// softmax cached in LDS when it fits; then wave 0 runs the alpha recursion
// while wave 1 runs the beta recursion (wave-synchronous, shuffles only, no
// barriers inside the time loop, the next step's emissions read one step
// ahead) on emissions and lattices held in LDS (a global workspace when
// [T, S] is too large), in log2 units so each log-sum-exp is two hardware
// transcendentals; finally a wave per frame writes the gradient row.
// The 16 waves serve the per-frame passes, which are latency chains
// (measured at T=125, B=256, C=96: 43 us with the gradient vs 96 us for the
// 256-thread, natural-log, global-reread form).
#include <cfloat>

#include "common.h"

#define CTC_THREADS 1024            // 16 waves: the per-frame passes (log-sum-exp, occupations, gradient) are latency chains; measured 43 vs 75 us at 256
#define CTC_MAX_R 8                 // S <= 512  (labels up to 255 symbols)
#define CTC_MAX_T 4096
#define CTC_MAX_C 256

// The lattices and emissions hold log2 probabilities: the log-sum-exps are
// then v_exp_f32 / v_log_f32 (base-2 hardware transcendentals, one
// instruction each) instead of the libm expf / logf sequences, on the
// recursion's serial chain. The -FLT_MAX floor keeps an all -inf argument
// list NaN-free without a branch (2^-inf = 0, log2 0 = -inf).
constexpr float LOG2E_F = 1.4426950408889634f, LN2_F = 0.6931471805599453f;
__device__ __forceinline__ float lse2b(float a, float b) {
    const float m = fmaxf(fmaxf(a, b), -FLT_MAX);
    return m + __builtin_amdgcn_logf(__builtin_amdgcn_exp2f(a - m) + __builtin_amdgcn_exp2f(b - m));
}
__device__ __forceinline__ float lse3b(float a, float b, float c) {
    const float m = fmaxf(fmaxf(fmaxf(a, b), c), -FLT_MAX);
    return m + __builtin_amdgcn_logf(__builtin_amdgcn_exp2f(a - m) + __builtin_amdgcn_exp2f(b - m) +
                                     __builtin_amdgcn_exp2f(c - m));
}

// value of register r at lane-1 (state s-1), across the register boundary.
__device__ __forceinline__ float shift_up1(const float* a, int r, int lane) {
    float v = __shfl_up(a[r], 1, 64);
    float w = __shfl(a[r > 0 ? r - 1 : 0], 63, 64);
    return lane == 0 ? (r > 0 ? w : -INFINITY) : v;
}
__device__ __forceinline__ float shift_up2(const float* a, int r, int lane) {
    float v = __shfl_up(a[r], 2, 64);
    float w = __shfl(a[r > 0 ? r - 1 : 0], 62 + lane, 64);
    return lane < 2 ? (r > 0 ? w : -INFINITY) : v;
}
__device__ __forceinline__ float shift_dn1(const float* a, int r, int R, int lane) {
    float v = __shfl_down(a[r], 1, 64);
    float w = __shfl(a[r + 1 < R ? r + 1 : r], 0, 64);
    return lane == 63 ? (r + 1 < R ? w : -INFINITY) : v;
}
__device__ __forceinline__ float shift_dn2(const float* a, int r, int R, int lane) {
    float v = __shfl_down(a[r], 2, 64);
    float w = __shfl(a[r + 1 < R ? r + 1 : r], lane - 62, 64);
    return lane >= 62 ? (r + 1 < R ? w : -INFINITY) : v;
}

// Emission log-probabilities of the extended label, em[t*S + s] =
// logit(t, l'_s) - lse(t): with LAT they are precomputed into LDS (every
// gather issued up front, in parallel), so the serial recursions below read
// LDS instead of waiting on a global load per step; without LAT (lattices too
// large for LDS) they are read from the logits in the loop, as before. The
// values are the same fp32 expressions either way.
// Whole-wave DPP shifts (GFX9 wave_shr:1 / wave_shl:1): lane i takes lane i-1
// (resp. i+1); the lane shifted in gets -inf. Used when the lattice fits one
// register (S <= 64) instead of ds_bpermute shuffles on the recursion's
// critical path.
__device__ __forceinline__ float wave_shr1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -INFINITY),
                                                                 __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_shl1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -INFINITY),
                                                                 __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

// Emission of state slot r at frame t, log2 units: from the LDS table (LAT)
// or from the logits.
template <bool LAT>
__device__ __forceinline__ float ctc_em(const float* __restrict__ logits, const float* lse, const float* em, int t,
                                        int S, int es, int cls, int B, int C, int b) {
    if constexpr (LAT) return em[(size_t)t * S + es];
    else return (logits[((size_t)t * B + b) * C + cls] - lse[t]) * LOG2E_F;
}

// The emissions of step t + 1 are read while step t computes (one step
// ahead), so the LDS / global latency is off the recursion's serial chain.
template <int R, bool LAT>
__device__ void ctc_alpha(const float* __restrict__ logits, const float* lse, const float* em, const int* lab,
                          int S, int L, int B, int C, int b, int blank, float* alpha) {
    const int lane = threadIdx.x & 63;
    int cls[R], es[R];
    bool skip[R];
    float a[R], en[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int s = lane + 64 * r;
        cls[r] = (s < S) ? ((s & 1) ? lab[s >> 1] : blank) : blank;
        es[r] = s < S ? s : S - 1;
        skip[r] = (s < S) && (s & 1) && s >= 3 && lab[s >> 1] != lab[(s >> 1) - 1];
        const float lp = ctc_em<LAT>(logits, lse, em, 0, S, es[r], cls[r], B, C, b);
        a[r] = (s < 2 && s < S) ? lp : -INFINITY;
        if (s < S) alpha[s] = a[r];
        en[r] = 1 < L ? ctc_em<LAT>(logits, lse, em, 1, S, es[r], cls[r], B, C, b) : 0.f;
    }
    for (int t = 1; t < L; ++t) {
        float e[R], nxt[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            e[r] = en[r];
            if (t + 1 < L) en[r] = ctc_em<LAT>(logits, lse, em, t + 1, S, es[r], cls[r], B, C, b);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // shuffles run in every lane (convergent); select afterwards
            float a1, a2;
            if constexpr (R == 1) {
                a1 = wave_shr1(a[0]);
                a2 = wave_shr1(a1);
            } else {
                a1 = shift_up1(a, r, lane);
                a2 = shift_up2(a, r, lane);
            }
            a2 = skip[r] ? a2 : -INFINITY;
            nxt[r] = lse3b(a[r], a1, a2) + e[r];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            int s = lane + 64 * r;
            a[r] = s < S ? nxt[r] : -INFINITY;
            if (s < S) alpha[(size_t)t * S + s] = a[r];
        }
    }
}

template <int R, bool LAT>
__device__ void ctc_beta(const float* __restrict__ logits, const float* lse, const float* em, const int* lab,
                         int S, int L, int B, int C, int b, int blank, float* beta) {
    const int lane = threadIdx.x & 63;
    int cls[R], es[R];
    bool skipn[R];   // transition s -> s+2 allowed
    float bt[R], en[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int s = lane + 64 * r;
        cls[r] = (s < S) ? ((s & 1) ? lab[s >> 1] : blank) : blank;
        es[r] = s < S ? s : S - 1;
        int s2 = s + 2;
        skipn[r] = (s2 < S) && (s2 & 1) && s2 >= 3 && lab[s2 >> 1] != lab[(s2 >> 1) - 1];
        bt[r] = (s < S && s >= S - 2) ? 0.f : -INFINITY;
        if (s < S) beta[(size_t)(L - 1) * S + s] = bt[r];
        en[r] = L >= 2 ? ctc_em<LAT>(logits, lse, em, L - 1, S, es[r], cls[r], B, C, b) : 0.f;
    }
    for (int t = L - 2; t >= 0; --t) {
        float nb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            int s = lane + 64 * r;
            nb[r] = s < S ? bt[r] + en[r] : -INFINITY;
            if (t >= 1) en[r] = ctc_em<LAT>(logits, lse, em, t, S, es[r], cls[r], B, C, b);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float b1, b2;
            if constexpr (R == 1) {
                b1 = wave_shl1(nb[0]);
                b2 = wave_shl1(b1);
            } else {
                b1 = shift_dn1(nb, r, R, lane);
                b2 = shift_dn2(nb, r, R, lane);
            }
            b2 = skipn[r] ? b2 : -INFINITY;
            bt[r] = lse3b(nb[r], b1, b2);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            int s = lane + 64 * r;
            if (s < S) beta[(size_t)t * S + s] = bt[r];
            else bt[r] = -INFINITY;
        }
    }
}

// LAT: the emissions and both lattices live in dynamic LDS ([T][Smax] each,
// CTC_LAT_MAX bytes at most); otherwise the lattices go to the global workspace.
#define CTC_LAT_MAX (112 * 1024)

template <int R, bool LAT>
__global__ void __launch_bounds__(CTC_THREADS)
ctc_loss_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                const int* __restrict__ label_len, const int* __restrict__ seq_len, int T, int B,
                int C, int max_label, float grad_scale, float* __restrict__ loss,
                float* __restrict__ grad, int* __restrict__ status, unsigned* __restrict__ status_word,
                float* __restrict__ ws, int pcache) {
    extern __shared__ float s_lat[];
    __shared__ float s_lse[CTC_MAX_T];
    __shared__ float s_logp;
    __shared__ int s_req;
    __shared__ int s_lab[CTC_MAX_R * 32];
    __shared__ int s_next[CTC_MAX_R * 32];          // next label index with the same class, or -1
    __shared__ int s_first[CTC_MAX_C];              // first label index of each class, or -1
    __shared__ float s_bocc[CTC_MAX_T];             // blank occupation per frame

    const int b = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int blank = C - 1;
    const int L = min(max(seq_len[b], 0), T);
    const int Lab = label_len[b];
    const int S = 2 * Lab + 1;
    const int Smax = 2 * max_label + 1;
    const size_t TS = (size_t)T * Smax;
    float* em = s_lat;
    float* alpha = LAT ? s_lat + TS : ws + (size_t)b * 2 * TS;
    float* beta = alpha + TS;
    // pcache (LAT only): the frame softmax p[t][k] kept in LDS behind the lattices
    // by the log-sum-exp pass, so the gradient pass reads neither the logits
    // from global memory again nor recomputes the exponentials
    float* sp = (LAT && pcache && grad) ? s_lat + 3 * TS : nullptr;

    // validation (TF1 raises InvalidArgumentError for every case flagged here):
    // a label_len outside [0, max_label] never indexes the label row or the
    // lattice; label values must lie in [0, C-1) (C-1 is the blank)
    __shared__ int s_code;
    if (threadIdx.x == 0) s_code = (Lab < 0 || Lab > max_label) ? 2 : 0;
    __syncthreads();
    if (s_code == 0) {
        bool bad = false;
        for (int i = threadIdx.x; i < Lab; i += CTC_THREADS) {
            const int v = labels[(size_t)b * max_label + i];
            bad |= v < 0 || v >= blank;
            s_lab[i] = v;
        }
        if (__syncthreads_or(bad) && threadIdx.x == 0) s_code = 3;
    }
    __syncthreads();
    // feasibility: L + #repeats <= seq_len  ([TF1] ctc_loss_calculator)
    if (threadIdx.x == 0 && s_code == 0) {
        int reps = 0;
        for (int i = 1; i < Lab; ++i) reps += s_lab[i] == s_lab[i - 1];
        s_req = Lab + reps;
        if (s_req > L || L == 0) s_code = 1;
    }
    __syncthreads();
    if (s_code != 0) {
        if (threadIdx.x == 0) {
            loss[b] = INFINITY;
            if (status) status[b] = s_code;
            if (status_word)
                __hip_atomic_fetch_or(status_word, 1u << s_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (grad)
            for (int i = threadIdx.x; i < T * C; i += CTC_THREADS) {
                int t = i / C, k = i % C;
                grad[((size_t)t * B + b) * C + k] = 0.f;
            }
        return;
    }
    if (status && threadIdx.x == 0) status[b] = 0;

    // log-sum-exp of every valid frame: a wave takes U frames at a time with all
    // of their loads in flight, then reduces them one by one
    constexpr int NW = CTC_THREADS / 64, NQ = CTC_MAX_C / 64, U = 8;
    for (int t0 = wave; t0 < L; t0 += U * NW) {
        float v[U][NQ];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + u * NW;
            const float* row = logits + ((size_t)t * B + b) * C;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int k = lane + 64 * q;
                v[u][q] = (t < L && k < C) ? row[k] : -INFINITY;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + u * NW;                   // wave-uniform
            if (t >= L) continue;
            float m = -INFINITY;
#pragma unroll
            for (int q = 0; q < NQ; ++q) m = fmaxf(m, v[u][q]);
            m = wave_max_dpp(m);
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                if (lane + 64 * q < C) sum += expf(v[u][q] - m);
            sum = wave_sum_dpp(sum);
            const float lse_t = m + logf(sum);           // the same value in every lane
            if (lane == 0) s_lse[t] = lse_t;
            if (sp) {
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    if (lane + 64 * q < C) sp[t * C + lane + 64 * q] = expf(v[u][q] - lse_t);
            }
            if constexpr (LAT) {
                // the frame's emissions from the registers already loaded (lane k % 64, slot k / 64)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int s = lane + 64 * r;
                    const int k = s < S ? ((s & 1) ? s_lab[s >> 1] : blank) : blank;
                    float val = 0.f;
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const float w = __shfl(v[u][q], k & 63, 64);
                        if ((k >> 6) == q) val = w;
                    }
                    if (s < S) em[(size_t)t * S + s] = (val - lse_t) * LOG2E_F;
                }
            }
        }
    }
    __syncthreads();

    if (wave == 0)
        ctc_alpha<R, LAT>(logits, s_lse, em, s_lab, S, L, B, C, b, blank, alpha);
    else if (wave == 1)
        ctc_beta<R, LAT>(logits, s_lse, em, s_lab, S, L, B, C, b, blank, beta);
    __syncthreads();
    if (threadIdx.x == 0) {
        const float* last = alpha + (size_t)(L - 1) * S;
        s_logp = S >= 2 ? lse2b(last[S - 1], last[S - 2]) : last[0];
    }
    __syncthreads();
    const float logp = s_logp;                          // log2 p(label | x)
    if (threadIdx.x == 0) loss[b] = -logp * LN2_F;
    if (!grad) return;

    // grad[t,k] = softmax - sum_{s: l'_s = k} exp(alpha + beta - logp).
    // (1) occupations E = exp(alpha + beta - logp) of every (t, s), in place of
    // alpha; the class -> label-index chains (first / next) for (3)
    const int ns = L * S;
    for (int i = threadIdx.x; i < ns; i += CTC_THREADS) alpha[i] = __builtin_amdgcn_exp2f(alpha[i] + beta[i] - logp);
    for (int k = threadIdx.x; k < C; k += CTC_THREADS) {
        int f = -1;
        for (int j = Lab - 1; j >= 0; --j) f = s_lab[j] == k ? j : f;
        s_first[k] = f;
    }
    for (int j = threadIdx.x; j < Lab; j += CTC_THREADS) {
        int nx = -1;
        for (int q = Lab - 1; q > j; --q) nx = s_lab[q] == s_lab[j] ? q : nx;
        s_next[j] = nx;
    }
    __syncthreads();
    // (2) blank occupation of each frame: a wave per frame, lanes over the even states
    for (int t = wave; t < L; t += CTC_THREADS / 64) {
        const float* et = alpha + (size_t)t * S;
        float o = 0.f;
        for (int s2 = 2 * lane; s2 < S; s2 += 128) o += et[s2];
        o = wave_sum_dpp(o);
        if (lane == 0) s_bocc[t] = o;
    }
    __syncthreads();
    // (3) the gradient, a wave per frame, lanes along the C classes (one row of
    // C contiguous floats per frame); a label class walks its (usually 0 or 1)
    // states. The softmax comes from the LDS cache (pcache) or the logits.
    for (int t = wave; t < T; t += CTC_THREADS / 64) {
        float* grow = grad + ((size_t)t * B + b) * C;
        if (t >= L) {
            for (int k = lane; k < C; k += 64) grow[k] = 0.f;
            continue;
        }
        const float* lrow = logits + ((size_t)t * B + b) * C;
        const float* et = alpha + (size_t)t * S;
        const float lse_t = s_lse[t], bocc = s_bocc[t];
        for (int k = lane; k < C; k += 64) {
            const float p = sp ? sp[t * C + k] : expf(lrow[k] - lse_t);
            float occ;
            if (k == blank) {
                occ = bocc;
            } else {
                occ = 0.f;
                for (int j = s_first[k]; j >= 0; j = s_next[j]) occ += et[2 * j + 1];
            }
            grow[k] = grad_scale * (p - occ);
        }
    }
}

// ------------------------------------------------------------- greedy decode
// One 256-thread workgroup per sequence, one frame per thread (frames t, t+256,
// ...): the thread's whole logits row (C floats, contiguous) is loaded with all
// its 16-B loads in flight, then reduced in register order -- first max on
// ties, [TF1] Eigen maxCoeff -- into LDS. Wave 0 then compacts the frames 64 at
// a time (merge repeats against the previous frame's argmax, drop blanks; a
// ballot prefix places each lane's label), while lane 0 sums the maxima in frame
// order (neg_sum_logits, the decoder's log_probability output, in TF's order).
// The previous form walked a sequence's frames one dependent load + shuffle
// reduction at a time with one wave: 110 us for B = 64, T = 125.
#define GREEDY_MAX_T 4096
#define GREEDY_VEC 32                                   // rows of up to 4 * 32 = 128 floats in registers
__global__ void __launch_bounds__(256)
ctc_greedy_kernel(const float* __restrict__ logits, const int* __restrict__ seq_len, int T, int B,
                  int C, int merge_repeated, int64_t* __restrict__ out, int* __restrict__ out_len,
                  float* __restrict__ neg_sum) {
    __shared__ int s_arg[GREEDY_MAX_T];
    __shared__ float s_max[GREEDY_MAX_T];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int L = min(max(seq_len[b], 0), T);
    const int blank = C - 1;
    const bool vec = (C % 4) == 0 && C <= 4 * GREEDY_VEC;
    for (int t = tid; t < L; t += 256) {
        const float* row = logits + ((size_t)t * B + b) * C;
        float best = -INFINITY;
        int arg = 0;
        if (vec) {
            float4 v[GREEDY_VEC];
            const int n4 = C >> 2;
#pragma unroll
            for (int q = 0; q < GREEDY_VEC; ++q)
                if (q < n4) v[q] = reinterpret_cast<const float4*>(row)[q];
#pragma unroll
            for (int q = 0; q < GREEDY_VEC; ++q)
                if (q < n4) {
                    if (v[q].x > best) { best = v[q].x; arg = 4 * q; }
                    if (v[q].y > best) { best = v[q].y; arg = 4 * q + 1; }
                    if (v[q].z > best) { best = v[q].z; arg = 4 * q + 2; }
                    if (v[q].w > best) { best = v[q].w; arg = 4 * q + 3; }
                }
        } else {
            for (int k = 0; k < C; ++k) {
                const float x = row[k];
                if (x > best) { best = x; arg = k; }
            }
        }
        s_arg[t] = arg;
        s_max[t] = best;
    }
    __syncthreads();
    if (tid >= 64) return;
    // wave 0: compaction in chunks of 64 frames; lane 0 also sums in frame order
    int n = 0;
    for (int t0 = 0; t0 < L; t0 += 64) {
        const int t = t0 + lane;
        bool emit = false;
        int k = 0;
        if (t < L) {
            k = s_arg[t];
            const int prev = t > 0 ? s_arg[t - 1] : -1;
            emit = k != blank && !(merge_repeated && k == prev);
        }
        const unsigned long long m = __ballot(emit);
        if (emit) out[(size_t)b * T + n + __popcll(m & ((1ull << lane) - 1ull))] = k;
        n += __popcll(m);
    }
    if (lane == 0) {
        float acc = 0.f;
        for (int t = 0; t < L; ++t) acc -= s_max[t];
        out_len[b] = n;
        if (neg_sum) neg_sum[b] = acc;
    }
    for (int i = n + lane; i < T; i += 64) out[(size_t)b * T + i] = -1;
}

// ------------------------------------------------------------------- C ABI
extern "C" size_t ocrk_ctc_workspace_size(int T, int B, int max_label_len) {
    return (size_t)B * 2 * T * (2 * (size_t)max_label_len + 1) * sizeof(float);
}

extern "C" int ocrk_ctc_loss(const float* logits, const int* labels, const int* label_len,
                             const int* seq_len, int T, int B, int C, int max_label_len,
                             float grad_scale, float* loss, float* grad, int* status,
                             unsigned* status_word, void* ws, size_t ws_bytes, void* stream) {
    OCRK_REQUIRE(T > 0 && T <= CTC_MAX_T, "ocrk_ctc_loss: T=%d out of range (1..%d)", T, CTC_MAX_T);
    OCRK_REQUIRE(B >= 0 && C >= 2 && C <= CTC_MAX_C, "ocrk_ctc_loss: bad B=%d / C=%d", B, C);
    OCRK_REQUIRE(max_label_len >= 0 && 2 * max_label_len + 1 <= 64 * CTC_MAX_R,
                 "ocrk_ctc_loss: max_label_len=%d too long (<= %d)", max_label_len, (64 * CTC_MAX_R - 1) / 2);
    OCRK_REQUIRE(ws_bytes >= ocrk_ctc_workspace_size(T, B, max_label_len),
                 "ocrk_ctc_loss: workspace too small");
    if (B == 0) return OCRK_OK;
    OCRK_REQUIRE(logits && labels && label_len && seq_len && loss && ws, "ocrk_ctc_loss: null pointer");
    int R = (2 * max_label_len + 1 + 63) / 64;
    hipStream_t s = ocrk::as_stream(stream);
    const size_t lat = 3 * (size_t)T * (2 * (size_t)max_label_len + 1) * sizeof(float);
    const bool in_lds = lat <= CTC_LAT_MAX && ocrk::opt(ocrk::OPT_CTC_LDS) != 0;   // 0: lattices in the workspace
    // the softmax cache behind the lattices when it fits as well
    const size_t pbytes = (size_t)T * C * sizeof(float);
    const int pcache = in_lds && grad && lat + pbytes <= CTC_LAT_MAX;
    const size_t dyn = lat + (pcache ? pbytes : 0);
#define CTC_ARGS logits, labels, label_len, seq_len, T, B, C, max_label_len, grad_scale, loss, grad, status, status_word, (float*)ws, pcache
#define CTC_LAUNCH(RR)                                                                                      \
    do {                                                                                                    \
        if (in_lds) {                                                                                       \
            static ocrk::DeviceOnce attr;                                                                   \
            ocrk::set_dyn_lds(attr, reinterpret_cast<const void*>(&ctc_loss_kernel<RR, true>), CTC_LAT_MAX); \
            ctc_loss_kernel<RR, true><<<B, CTC_THREADS, dyn, s>>>(CTC_ARGS);                                \
        } else {                                                                                            \
            ctc_loss_kernel<RR, false><<<B, CTC_THREADS, 0, s>>>(CTC_ARGS);                                 \
        }                                                                                                   \
    } while (0)
    if (R <= 1) CTC_LAUNCH(1);
    else if (R <= 2) CTC_LAUNCH(2);
    else if (R <= 4) CTC_LAUNCH(4);
    else CTC_LAUNCH(8);
#undef CTC_LAUNCH
#undef CTC_ARGS
    return ocrk::launch_status("ocrk_ctc_loss");
}

extern "C" int ocrk_ctc_greedy_decode(const float* logits, const int* seq_len, int T, int B, int C,
                                      int merge_repeated, int64_t* out, int* out_len,
                                      float* neg_sum_logits, void* stream) {
    OCRK_REQUIRE(T > 0 && T <= GREEDY_MAX_T && B >= 0 && C >= 1,
                 "ocrk_ctc_greedy_decode: bad sizes T=%d B=%d C=%d", T, B, C);
    if (B == 0) return OCRK_OK;
    OCRK_REQUIRE(logits && seq_len && out && out_len, "ocrk_ctc_greedy_decode: null pointer");
    ctc_greedy_kernel<<<B, 256, 0, ocrk::as_stream(stream)>>>(logits, seq_len, T, B, C, merge_repeated,
                                                             out, out_len, neg_sum_logits);
    return ocrk::launch_status("ocrk_ctc_greedy_decode");
}
