// a11 -- CTC prefix beam search, tf.nn.ctc_beam_search_decoder with the
// default scorer (src/weinman/test.py:84-88 beam 128 merge_repeated=True;
// src/weinman/client.py:227-231 merge_repeated=False). [TF1]
// ctc_beam_search.h Step()/TopPaths() semantics, restated in
// oracle/ref_graph.py:ctc_beam_search_single.
//
// One 256-thread workgroup per sequence; the beam lives in LDS.
//   * A prefix is identified by a 64-bit hash of its label sequence (TF keeps
//     one tree node per prefix; "parent active" and "child already in the
//     beam" are hash lookups against the current beam).
//   * TF's bounded top-N with strict '>' against the bottom is "top-K of
//     {beams with updated probabilities} U {new children}, ordered by total
//     desc, ties by TF's insertion order (beams in rank order, then children
//     by parent rank and label)" -- except for one order-dependent effect:
//     when beam j has been pushed out of the top-N before its parent p (ranked
//     above j) reaches label(j) in its child loop, TF re-offers j as a new
//     child, rejects it and resets j.oldp, so j's own children are never
//     expanded this step ("wiped"). A wave-0 pass over parent ranks decides
//     the wiped beams by counting, for each such (p, j), the items offered
//     before that moment that beat j (sorted-logit binary searches per
//     branch); the gate "p.oldp.total > bottom" is the same count.
//   * The selection itself gives each item a 47-bit key (total desc :
//     insertion order) and a block radix-select finds the K-th smallest key;
//     no candidate list is materialised.
//   * Emitted prefixes are appended to a per-sequence arena (parent id,
//     label) in global memory; TopPaths walks it back with LabelSeq's merge.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int BEAM_MAX_K = 128;
constexpr int BEAM_MAX_C = 128;
constexpr int BEAM_THREADS = 256;
constexpr int ORDER_BITS = 15;          // insertion order < n + n*C <= 16512
constexpr uint64_t ROOT_HASH = 0x6a09e667f3bcc909ull;

__device__ __forceinline__ uint64_t child_hash(uint64_t parent, int label) {
    uint64_t z = parent ^ ((uint64_t)(label + 1) * 0x9E3779B97F4A7C15ull);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// [TF1] ctc_loss_util.h LogSumExp.
__device__ __forceinline__ float log_sum_exp(float a, float b) {
    if (a == -INFINITY) return b;
    if (b == -INFINITY) return a;
    return a > b ? a + log1pf(expf(b - a)) : b + log1pf(expf(a - b));
}

// Larger float -> smaller key.
__device__ __forceinline__ uint64_t desc_bits(float f) {
    uint32_t u = __float_as_uint(f);
    uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return (uint64_t)(~ord);
}

struct BeamLds {
    float x[BEAM_MAX_C];                 // log-softmax row
    float xs[BEAM_MAX_C];                // non-blank x sorted desc (wipe-pass counts)
    // current beam (sorted by total desc); o* = newp of the previous step
    uint64_t h[BEAM_MAX_K], ph[BEAM_MAX_K];
    int lab[BEAM_MAX_K], id[BEAM_MAX_K], pidx[BEAM_MAX_K];
    int has_kid[BEAM_MAX_K], wiped[BEAM_MAX_K];
    float ot[BEAM_MAX_K], ob[BEAM_MAX_K], ol[BEAM_MAX_K];
    float nt[BEAM_MAX_K], nb[BEAM_MAX_K], nl[BEAM_MAX_K];   // loop-1 updates
    uint32_t act[BEAM_MAX_K][BEAM_MAX_C / 32];             // child label already a beam
    // next beam staging
    uint64_t h2[BEAM_MAX_K], ph2[BEAM_MAX_K];
    int lab2[BEAM_MAX_K], id2[BEAM_MAX_K];
    float t2[BEAM_MAX_K], b2[BEAM_MAX_K], l2[BEAM_MAX_K];
    uint64_t sel[BEAM_MAX_K];
    uint32_t hist[BEAM_THREADS / 64][256];
    uint32_t wsum[BEAM_THREADS / 64];
    float red[BEAM_THREADS / 64];
    uint64_t prefix;
    uint32_t kk, n_sel, n_valid;
    int n, next_id;
    float tau;
};

__device__ __forceinline__ int block_sync_max_f(BeamLds& s, float v, float* out) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s.red[w] = v;
    __syncthreads();
    float m = s.red[0];
#pragma unroll
    for (int i = 1; i < BEAM_THREADS / 64; ++i) m = fmaxf(m, s.red[i]);
    *out = m;
    __syncthreads();
    return 0;
}

// Item i of the candidate set: beams [0, n), then n*(C-1) children
// (parent r, label l) -- skipped when l is already a beam, r was wiped, or
// the total cannot beat tau.
__device__ __forceinline__ bool beam_item(const BeamLds& s, int i, int n, int C, uint64_t* key) {
    if (i < n) {
        *key = (desc_bits(s.nt[i]) << ORDER_BITS) | (uint64_t)i;
        return true;
    }
    const int q = i - n;
    const int r = q / (C - 1), l = q - r * (C - 1);
    if (s.wiped[r]) return false;
    if ((s.act[r][l >> 5] >> (l & 31)) & 1u) return false;
    const float v = s.x[l] + (l == s.lab[r] ? s.ob[r] : s.ot[r]);
    if (!(v > s.tau)) return false;
    *key = (desc_bits(v) << ORDER_BITS) | (uint64_t)(n + r * C + l);
    return true;
}

// Wave-0 helper: number of offered items that beat `thr` (total >= thr when
// ge, else > thr; beams i < j_rank win a tie at equal totals) among: every
// beam's updated entry, all children of the unwiped branches ranked before
// p, and p's children with label < l_lim.
__device__ int count_better(const BeamLds& s, float thr, bool ge, int j_rank, int p, int l_lim, int n,
                            int C, int lane) {
    const int nl = C - 1;
    int c = 0;
    for (int i = lane; i < n; i += 64) {
        const float v = s.nt[i];
        c += ge ? (v >= thr) : (v > thr || (v == thr && i < j_rank));
        // active child i of an earlier branch is counted above as a beam, not as a child
        const int r = s.pidx[i];
        if (r >= 0 && r < p && !s.wiped[r] && s.lab[i] != s.lab[r]) {
            const float cv = s.x[s.lab[i]] + s.ot[r];
            c -= ge ? (cv >= thr) : (cv > thr);
        }
    }
    for (int r = lane; r < p; r += 64) {
        if (s.wiped[r]) continue;
        const float o = s.ot[r];
        int lo = 0, hi = nl;                               // first slot failing the predicate
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const float v = s.xs[mid] + o;
            if (ge ? (v >= thr) : (v > thr)) lo = mid + 1; else hi = mid;
        }
        c += lo;
        const int pl = s.lab[r];
        if (pl >= 0) {                                     // own label extends from the blank-ending prob
            const float vo = s.x[pl] + o;
            c -= ge ? (vo >= thr) : (vo > thr);
            if (!((s.act[r][pl >> 5] >> (pl & 31)) & 1u)) {
                const float vb = s.x[pl] + s.ob[r];
                c += ge ? (vb >= thr) : (vb > thr);
            }
        }
    }
    for (int l = lane; l < l_lim; l += 64) {
        if ((s.act[p][l >> 5] >> (l & 31)) & 1u) continue;
        const float v = s.x[l] + (l == s.lab[p] ? s.ob[p] : s.ot[p]);
        c += ge ? (v >= thr) : (v > thr);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    return c;
}

__global__ void __launch_bounds__(BEAM_THREADS)
ctc_beam_kernel(const float* __restrict__ logits, const int* __restrict__ seq_len, int T, int B, int C,
                int K, int top_paths, int merge_repeated, int64_t* __restrict__ out,
                int* __restrict__ out_len, float* __restrict__ log_probs, int2* __restrict__ arena_all) {
    __shared__ BeamLds s;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int L = min(max(seq_len[b], 0), T);
    const int blank = C - 1;
    int2* arena = arena_all + (size_t)b * (1 + (size_t)T * K);

    if (tid == 0) {
        s.h[0] = ROOT_HASH; s.ph[0] = 0; s.lab[0] = -1; s.id[0] = 0;
        s.ot[0] = 0.f; s.ob[0] = 0.f; s.ol[0] = -INFINITY;
        s.n = 1; s.next_id = 1;
        arena[0] = make_int2(-1, -1);
    }
    __syncthreads();

    for (int t = 0; t < L; ++t) {
        // ---- input row -> log-softmax (Step(): max removed, then norm_offset)
        const float* row = logits + ((size_t)t * B + b) * C;
        float v = tid < C ? row[tid] : -INFINITY;
        float m;
        block_sync_max_f(s, v, &m);
        float e = tid < C ? expf(v - m) : 0.f;
        e = wave_sum(e);
        if (lane == 0) s.red[w] = e;
        __syncthreads();
        float z = 0.f;
#pragma unroll
        for (int i = 0; i < BEAM_THREADS / 64; ++i) z += s.red[i];
        const float norm = logf(z);
        if (tid < C) s.x[tid] = (v - m) - norm;
        const int n = s.n;
        __syncthreads();

        // ---- sorted logits, parent lookup, clear per-step flags
        if (tid < C && tid != blank) {
            const float xl = s.x[tid];
            int rank = 0;
            for (int j = 0; j < C; ++j) {
                if (j == blank) continue;
                const float xj = s.x[j];
                rank += (xj > xl) || (xj == xl && j < tid);
            }
            s.xs[rank] = xl;
        }
        if (tid < n) {
            int p = -1;
            if (s.lab[tid] >= 0) {
                const uint64_t want = s.ph[tid];
                for (int j = 0; j < n; ++j)
                    if (s.h[j] == want) { p = j; break; }
            }
            s.pidx[tid] = p;
            s.has_kid[tid] = 0;
            s.wiped[tid] = 0;
#pragma unroll
            for (int q = 0; q < BEAM_MAX_C / 32; ++q) s.act[tid][q] = 0u;
        }
        __syncthreads();

        // ---- loop 1: extend every beam by blank / its own label
        float my_nt = INFINITY;
        if (tid < n) {
            const int l = s.lab[tid], p = s.pidx[tid];
            float nl = s.ol[tid];
            if (l >= 0) {
                if (p >= 0) {
                    const float prev = (l == s.lab[p]) ? s.ob[p] : s.ot[p];
                    nl = log_sum_exp(nl, prev);
                }
                nl += s.x[l];
                if (p >= 0) atomicOr(&s.act[p][l >> 5], 1u << (l & 31));
                if (p >= 0 && p < tid) s.has_kid[p] = 1;
            }
            const float nb = s.ot[tid] + s.x[blank];
            my_nt = log_sum_exp(nb, nl);
            s.nl[tid] = nl; s.nb[tid] = nb; s.nt[tid] = my_nt;
        }
        // tau: with a full beam no child at or below the weakest updated beam
        // can enter (the beam wins the tie on insertion order).
        float mn = -wave_max(-my_nt);
        if (lane == 0) s.red[w] = mn;
        __syncthreads();
        if (tid == 0) {
            float q = s.red[0];
#pragma unroll
            for (int i = 1; i < BEAM_THREADS / 64; ++i) q = fminf(q, s.red[i]);
            s.tau = (n == K) ? q : -INFINITY;
            s.prefix = 0; s.kk = 0; s.n_sel = 0;
        }
        __syncthreads();

        // ---- wipe pass (wave 0), in parent rank order
        if (w == 0) {
            for (int p = 0; p < n; ++p) {
                if (!s.has_kid[p] || s.wiped[p]) continue;
                if (count_better(s, s.ot[p], true, 0, p, 0, n, C, lane) >= K) continue;   // p gated
                for (int j0 = p + 1; j0 < n; j0 += 64) {
                    const int jj = j0 + lane;
                    uint64_t kids = __ballot(jj < n && s.pidx[jj] == p);
                    while (kids) {
                        const int j = j0 + __builtin_ctzll(kids);
                        kids &= kids - 1;
                        const int c = count_better(s, s.nt[j], false, j, p, s.lab[j], n, C, lane);
                        if (lane == 0 && c >= K) s.wiped[j] = 1;
                    }
                }
            }
        }
        __syncthreads();

        // ---- radix select of the K-th smallest key (47 bits, 8-bit digits)
        const int n_items = n + n * (C - 1);
        uint64_t pmask = 0;
        bool take_all = false;
        for (int shift = 40; shift >= 0; shift -= 8) {
            for (int i = tid; i < (BEAM_THREADS / 64) * 256; i += BEAM_THREADS) (&s.hist[0][0])[i] = 0u;
            __syncthreads();
            const uint64_t prefix = s.prefix;
            for (int i = tid; i < n_items; i += BEAM_THREADS) {
                uint64_t key;
                if (beam_item(s, i, n, C, &key) && (key & pmask) == prefix)
                    atomicAdd(&s.hist[w][(key >> shift) & 255u], 1u);
            }
            __syncthreads();
            uint32_t c = 0;
#pragma unroll
            for (int q = 0; q < BEAM_THREADS / 64; ++q) c += s.hist[q][tid];
            // block inclusive scan over the 256 digits
            uint32_t incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                uint32_t u = __shfl_up(incl, o, 64);
                if (lane >= o) incl += u;
            }
            if (lane == 63) s.wsum[w] = incl;
            __syncthreads();
            uint32_t base = 0;
            for (int q = 0; q < w; ++q) base += s.wsum[q];
            incl += base;
            const uint32_t excl = incl - c;
            uint32_t total = 0;
#pragma unroll
            for (int q = 0; q < BEAM_THREADS / 64; ++q) total += s.wsum[q];
            if (shift == 40) {
                if (total <= (uint32_t)K) take_all = true;   // uniform across the block
                if (tid == 0) { s.n_valid = total; s.kk = min(total, (uint32_t)K); }
                __syncthreads();
            }
            if (take_all) break;
            const uint32_t kk = s.kk;
            __syncthreads();
            if (c > 0 && excl < kk && kk <= incl) {
                s.prefix = prefix | ((uint64_t)tid << shift);
                s.kk = kk - excl;
            }
            pmask |= (uint64_t)255u << shift;
            __syncthreads();
        }
        const uint64_t theta = take_all ? ~0ull : s.prefix;

        // ---- gather the selected keys and rank them
        for (int i = tid; i < n_items; i += BEAM_THREADS) {
            uint64_t key;
            if (beam_item(s, i, n, C, &key) && key <= theta) {
                uint32_t pos = atomicAdd(&s.n_sel, 1u);
                if (pos < (uint32_t)BEAM_MAX_K) s.sel[pos] = key;
            }
        }
        __syncthreads();
        const int n_sel = min((int)s.n_sel, K);
        uint64_t my_key = ~0ull;
        int my_rank = 0;
        if (tid < n_sel) {
            my_key = s.sel[tid];
            for (int j = 0; j < n_sel; ++j) my_rank += s.sel[j] < my_key;
        }
        // new prefixes get arena ids in rank order
        const int order = tid < n_sel ? (int)(my_key & ((1u << ORDER_BITS) - 1)) : 0;
        const bool is_new = tid < n_sel && order >= n;
        __syncthreads();
        if (tid < n_sel) s.sel[my_rank] = my_key;
        __syncthreads();
        {
            const uint64_t k2 = tid < n_sel ? s.sel[tid] : 0;
            const int o2 = (int)(k2 & ((1u << ORDER_BITS) - 1));
            const bool new2 = tid < n_sel && o2 >= n;
            const uint64_t bal = __ballot(new2);
            const int before = __popcll(bal & ((1ull << lane) - 1ull));
            if (lane == 0) s.wsum[w] = __popcll(bal);
            __syncthreads();
            int off = s.next_id;
            for (int q = 0; q < w; ++q) off += s.wsum[q];
            if (tid < n_sel) {
                if (!new2) {
                    const int j = o2;
                    s.h2[tid] = s.h[j]; s.ph2[tid] = s.ph[j]; s.lab2[tid] = s.lab[j]; s.id2[tid] = s.id[j];
                    s.t2[tid] = s.nt[j]; s.b2[tid] = s.nb[j]; s.l2[tid] = s.nl[j];
                } else {
                    const int q = o2 - n, r = q / C, l = q - r * C;
                    const int nid = off + before;
                    const float val = s.x[l] + (l == s.lab[r] ? s.ob[r] : s.ot[r]);
                    s.h2[tid] = child_hash(s.h[r], l); s.ph2[tid] = s.h[r]; s.lab2[tid] = l;
                    s.id2[tid] = nid;
                    s.t2[tid] = val; s.b2[tid] = -INFINITY; s.l2[tid] = val;
                    arena[nid] = make_int2(s.id[r], l);
                }
            }
            (void)is_new;
            __syncthreads();
            if (tid == 0) {
                int nn = 0;
#pragma unroll
                for (int q = 0; q < BEAM_THREADS / 64; ++q) nn += s.wsum[q];
                s.next_id += nn;
                s.n = n_sel;
            }
            if (tid < n_sel) {
                s.h[tid] = s.h2[tid]; s.ph[tid] = s.ph2[tid]; s.lab[tid] = s.lab2[tid]; s.id[tid] = s.id2[tid];
                s.ot[tid] = s.t2[tid]; s.ob[tid] = s.b2[tid]; s.ol[tid] = s.l2[tid];
            }
            __syncthreads();
        }
    }

    // ---- TopPaths: walk the arena back, LabelSeq(merge_repeated)
    const int n = s.n;
    for (int k = tid; k < top_paths; k += BEAM_THREADS) {
        int64_t* o = out + ((size_t)k * B + b) * T;
        int len = 0;
        if (k < n) {
            int e = s.id[k], prev = -1;
            while (e > 0) {
                const int2 a = arena[e];
                if (!merge_repeated || a.y != prev) ++len;
                prev = a.y;
                e = a.x;
            }
            e = s.id[k]; prev = -1;
            int pos = len;
            while (e > 0) {
                const int2 a = arena[e];
                if (!merge_repeated || a.y != prev) o[--pos] = a.y;
                prev = a.y;
                e = a.x;
            }
            log_probs[(size_t)b * top_paths + k] = s.ot[k];
        } else {
            log_probs[(size_t)b * top_paths + k] = -INFINITY;
        }
        for (int i = len; i < T; ++i) o[i] = -1;
        out_len[(size_t)k * B + b] = len;
    }
}

// ---------------------------------------------------------------------------
// K <= 16, C <= 128 (BASELINE configs[4]'s beam 16): ONE WAVE per sequence,
// four sequences per workgroup, no workgroup barrier and no LDS. The same
// semantics as ctc_beam_kernel (which stays the form for K > 16), restated for
// 64 lanes:
//   * beam j lives in lane j's registers (hash, parent hash, label, arena id,
//     total / blank / label log-probs); per-index reads are v_readlane (uniform
//     index) or ds_bpermute (per-lane index);
//   * lane l holds the log-softmax of labels l and l + 64, and for each of them
//     16-bit parent masks: act (child (r, l) already a beam), own (l == lab[r]);
//   * the wipe pass's counts (count_better above) are per-label-lane sums over
//     the branch masks plus a wave sum;
//   * the selection is a 16-round extraction: the candidates of one label over
//     the parents ranked in beam order (totals non-increasing, so a label's
//     children come in key order -- own-label children, which use the blank-
//     ending probability, are a separate head on their parent's lane) and the
//     updated beams are sorted heads; each round takes the wave-minimum 64-bit
//     key (total desc : TF insertion order) and advances that head. The keys
//     come out in rank order, so the next beam needs no sort.
// The block form spent ~20 workgroup barriers and a 6-digit radix select per
// frame: 4.08 ms per C5 launch, ~16 us per frame.
constexpr int WB_K = 16;
constexpr int WB_WAVES = 4;

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int rli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rlf(float v, int l) {
    return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), l));
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const unsigned lo = (unsigned)__shfl((int)(unsigned)v, src, 64);
    const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
// DPP row rotations (8, 4, 2, 1 within each 16-lane row: no LDS crossbar round
// trip) give every lane its row's result; the four rows meet through v_readlane.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_step(uint64_t v) {
    const uint64_t u = ((uint64_t)dpp_u<CTRL>((unsigned)(v >> 32)) << 32) | dpp_u<CTRL>((unsigned)v);
    return u < v ? u : v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    v = dpp_min_step<0x128>(v);
    v = dpp_min_step<0x124>(v);
    v = dpp_min_step<0x122>(v);
    v = dpp_min_step<0x121>(v);
    const uint64_t a = rl64(v, 0), b = rl64(v, 16), c = rl64(v, 32), d = rl64(v, 48);
    const uint64_t ab = a < b ? a : b, cd = c < d ? c : d;
    return ab < cd ? ab : cd;
}
__device__ __forceinline__ int wave_sum_i(int v) {
    v += (int)dpp_u<0x128>((unsigned)v);
    v += (int)dpp_u<0x124>((unsigned)v);
    v += (int)dpp_u<0x122>((unsigned)v);
    v += (int)dpp_u<0x121>((unsigned)v);
    return (rli(v, 0) + rli(v, 16)) + (rli(v, 32) + rli(v, 48));
}

__global__ void __launch_bounds__(64 * WB_WAVES)
ctc_beam_wave_kernel(const float* __restrict__ logits, const int* __restrict__ seq_len, int T, int B, int C,
                     int K, int top_paths, int merge_repeated, int64_t* __restrict__ out,
                     int* __restrict__ out_len, float* __restrict__ log_probs, int2* __restrict__ arena_all) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * WB_WAVES + (threadIdx.x >> 6);
    if (b >= B) return;                                  // whole waves only: no workgroup barrier below
    const int L = min(max(seq_len[b], 0), T);
    const int blank = C - 1;
    int2* arena = arena_all + (size_t)b * (1 + (size_t)T * K);
    const int L0 = lane, L1 = lane + 64;
    const bool ok0 = L0 < blank, ok1 = L1 < blank;       // the non-blank labels this lane holds

    // beam j in lane j (j < n)
    uint64_t bh = ROOT_HASH, bph = 0;
    int blab = -1, bid = 0;
    float bot = 0.f, bob = 0.f, bol = -INFINITY;
    int n = 1, next_id = 1;
    if (lane == 0) arena[0] = make_int2(-1, -1);

    auto load_row = [&](int t, float& a0, float& a1) {
        const float* row = logits + ((size_t)t * B + b) * C;
        a0 = L0 < C ? row[L0] : -INFINITY;
        a1 = L1 < C ? row[L1] : -INFINITY;
    };
    float n0 = -INFINITY, n1 = -INFINITY;
    if (L > 0) load_row(0, n0, n1);

    for (int t = 0; t < L; ++t) {
        const float v0 = n0, v1 = n1;
        if (t + 1 < L) load_row(t + 1, n0, n1);          // the next frame's loads in flight over this one
        // ---- log-softmax of the frame (Step(): max removed, then norm_offset), the block form's order
        const float m = wave_max_dpp(fmaxf(v0, v1));
        const float e0 = L0 < C ? expf(v0 - m) : 0.f;
        const float e1 = L1 < C ? expf(v1 - m) : 0.f;
        const float z = wave_sum_dpp(e0) + wave_sum_dpp(e1);
        const float norm = logf(z);
        const float x0 = (v0 - m) - norm, x1 = (v1 - m) - norm;
        const float xb = blank < 64 ? rlf(x0, blank) : rlf(x1, blank - 64);
        auto xval = [&](int l) {                         // x[l] for a per-lane label (all lanes call)
            const float a = __shfl(x0, l & 63, 64), c2 = __shfl(x1, l & 63, 64);
            return l < 64 ? a : c2;
        };

        // ---- parent of each beam: the beam whose hash is its parent hash
        int p = -1;
        for (int j = 0; j < n; ++j)
            if (p < 0 && blab >= 0 && rl64(bh, j) == bph) p = j;
        if (lane >= n) p = -1;

        // ---- loop 1: every beam extended by blank / its own label
        const int ps = p < 0 ? 0 : p;
        const int plab = __shfl(blab, ps, 64);
        const float pob = __shfl(bob, ps, 64), pot = __shfl(bot, ps, 64);
        const float xl = xval(blab < 0 ? 0 : blab);
        float nl = bol, nb = -INFINITY, nt = INFINITY;
        if (lane < n) {
            if (blab >= 0) {
                if (p >= 0) nl = log_sum_exp(nl, blab == plab ? pob : pot);
                nl += xl;
            }
            nb = bot + xb;
            nt = log_sum_exp(nb, nl);
        }

        // ---- per-label parent masks, has-kid mask, own-label-child-active mask
        unsigned act0 = 0u, act1 = 0u, own0 = 0u, own1 = 0u, hk = 0u, ownact = 0u;
        for (int j = 0; j < n; ++j) {
            const int lj = rli(blab, j), pj = rli(p, j);
            if (lj < 0) continue;
            if (pj >= 0) {
                if (lj == L0) act0 |= 1u << pj;
                if (lj == L1) act1 |= 1u << pj;
                if (pj < j) hk |= 1u << pj;
                if (lj == rli(blab, pj)) ownact |= 1u << pj;
            }
            if (lj == L0) own0 |= 1u << j;
            if (lj == L1) own1 |= 1u << j;
        }
        const unsigned all_n = n >= 32 ? ~0u : ((1u << n) - 1u);
        // with a full beam no child at or below the weakest updated beam can enter
        const float tau = n == K ? -rlf(wave_max(lane < n ? -nt : -INFINITY), 0) : -INFINITY;

        // ---- wipe pass (count_better, per label lane), parents in rank order
        unsigned W = 0u;
        auto count_better = [&](float thr, bool ge, int jr, int pp, int llim) {
            int c = 0;
            if (lane < n) c += ge ? (nt >= thr) : (nt > thr || (nt == thr && lane < jr));
            const unsigned R = ((1u << pp) - 1u) & ~W;
            for (unsigned m2 = R; m2; m2 &= m2 - 1u) {
                const int r = __builtin_ctz(m2);
                const float otr = rlf(bot, r), obr = rlf(bob, r);
                if (ok0 && !((act0 >> r) & 1u)) {
                    const float v = x0 + (((own0 >> r) & 1u) ? obr : otr);
                    c += ge ? (v >= thr) : (v > thr);
                }
                if (ok1 && !((act1 >> r) & 1u)) {
                    const float v = x1 + (((own1 >> r) & 1u) ? obr : otr);
                    c += ge ? (v >= thr) : (v > thr);
                }
            }
            const float otp = rlf(bot, pp), obp = rlf(bob, pp);
            if (ok0 && L0 < llim && !((act0 >> pp) & 1u)) {
                const float v = x0 + (((own0 >> pp) & 1u) ? obp : otp);
                c += ge ? (v >= thr) : (v > thr);
            }
            if (ok1 && L1 < llim && !((act1 >> pp) & 1u)) {
                const float v = x1 + (((own1 >> pp) & 1u) ? obp : otp);
                c += ge ? (v >= thr) : (v > thr);
            }
            return wave_sum_i(c);
        };
        for (unsigned hm = hk; hm; hm &= hm - 1u) {
            const int pp = __builtin_ctz(hm);
            if ((W >> pp) & 1u) continue;
            if (count_better(rlf(bot, pp), true, 0, pp, 0) >= K) continue;   // p gated
            for (int j = pp + 1; j < n; ++j) {
                if (rli(p, j) != pp) continue;
                if (count_better(rlf(nt, j), false, j, pp, rli(blab, j)) >= K) W |= 1u << j;
            }
        }

        // ---- selection: K rounds of the wave-minimum key over the sorted heads. Each
        //      round only the winning lane advances one head; its next key's parent total
        //      is a v_readlane at the (uniform) winner's pointer -- no LDS round trip.
        const unsigned avail0 = ok0 ? (all_n & ~(act0 | own0 | W)) : 0u;
        const unsigned avail1 = ok1 ? (all_n & ~(act1 | own1 | W)) : 0u;
        int ptr0 = avail0 ? __builtin_ctz(avail0) : 32, ptr1 = avail1 ? __builtin_ctz(avail1) : 32;
        auto label_key = [&](float xv, int ptr, int lab, float o) {
            if (ptr >= n) return ~0ull;
            const float v = xv + o;
            // the rest of this label's parents rank lower: nothing further can beat tau either
            return v > tau ? ((desc_bits(v) << ORDER_BITS) | (uint64_t)(n + ptr * C + lab)) : ~0ull;
        };
        uint64_t key0 = label_key(x0, ptr0, L0, __shfl(bot, ptr0 & 63, 64));
        uint64_t key1 = label_key(x1, ptr1, L1, __shfl(bot, ptr1 & 63, 64));
        // own-label child of the beam in this lane, and the beam itself
        const float vo = xl + bob;
        uint64_t keyo = (lane < n && blab >= 0 && !((W >> lane) & 1u) && !((ownact >> lane) & 1u) && vo > tau)
                            ? ((desc_bits(vo) << ORDER_BITS) | (uint64_t)(n + lane * C + blab)) : ~0ull;
        uint64_t keyb = lane < n ? ((desc_bits(nt) << ORDER_BITS) | (uint64_t)lane) : ~0ull;
        uint64_t selk = ~0ull;
        int ns = 0;
        for (int k = 0; k < K; ++k) {
            uint64_t mine = key0 < key1 ? key0 : key1;
            mine = mine < keyo ? mine : keyo;
            mine = mine < keyb ? mine : keyb;
            const uint64_t kmin = wave_min_u64(mine);
            if (kmin == ~0ull) break;
            if (lane == k) selk = kmin;
            ++ns;
            const int win = __builtin_ctzll(__ballot(mine == kmin));          // the one lane holding it
            if (lane == win) {
                if (key0 == kmin) {
                    const unsigned rest = avail0 & ~((2u << ptr0) - 1u);
                    ptr0 = rest ? __builtin_ctz(rest) : 32;
                } else if (key1 == kmin) {
                    const unsigned rest = avail1 & ~((2u << ptr1) - 1u);
                    ptr1 = rest ? __builtin_ctz(rest) : 32;
                } else if (keyo == kmin) {
                    keyo = ~0ull;
                } else {
                    keyb = ~0ull;
                }
            }
            const int p0w = rli(ptr0, win), p1w = rli(ptr1, win);
            const float o0w = rlf(bot, p0w & 63), o1w = rlf(bot, p1w & 63);
            if (lane == win) {
                key0 = label_key(x0, ptr0, L0, o0w);
                key1 = label_key(x1, ptr1, L1, o1w);
            }
        }

        // ---- the next beam, in rank order (the extraction order)
        const int o = (int)(selk & ((1u << ORDER_BITS) - 1));
        const bool sel = lane < ns;
        const bool isnew = sel && o >= n;
        const int q = o - n, r = isnew ? q / C : 0, l = isnew ? q - r * C : 0;
        const int src = isnew ? r : (sel ? o : 0);
        const uint64_t sh_ = shfl64(bh, src), sph = shfl64(bph, src);
        const int slab = __shfl(blab, src, 64), sid = __shfl(bid, src, 64);
        const float sot = __shfl(bot, src, 64), sob = __shfl(bob, src, 64);
        const float snt = __shfl(nt, src, 64), snb = __shfl(nb, src, 64), snl = __shfl(nl, src, 64);
        const float xnew = xval(l);
        const uint64_t newmask = __ballot(isnew);
        const int nid = next_id + __popcll(newmask & ((1ull << lane) - 1ull));
        if (isnew) {
            const float val = xnew + (l == slab ? sob : sot);
            bh = child_hash(sh_, l); bph = sh_; blab = l; bid = nid;
            bot = val; bob = -INFINITY; bol = val;
            arena[nid] = make_int2(sid, l);
        } else if (sel) {
            bh = sh_; bph = sph; blab = slab; bid = sid;
            bot = snt; bob = snb; bol = snl;
        }
        next_id += __popcll(newmask);
        n = ns;
    }

    // ---- TopPaths: walk the arena back, LabelSeq(merge_repeated); -1 fill by the whole wave
    int len = 0;
    if (lane < top_paths) {
        int64_t* ov = out + ((size_t)lane * B + b) * T;
        if (lane < n) {
            int e = bid, prev = -1;
            while (e > 0) {
                const int2 a = arena[e];
                if (!merge_repeated || a.y != prev) ++len;
                prev = a.y;
                e = a.x;
            }
            e = bid; prev = -1;
            int pos = len;
            while (e > 0) {
                const int2 a = arena[e];
                if (!merge_repeated || a.y != prev) ov[--pos] = a.y;
                prev = a.y;
                e = a.x;
            }
            log_probs[(size_t)b * top_paths + lane] = bot;
        } else {
            log_probs[(size_t)b * top_paths + lane] = -INFINITY;
        }
        out_len[(size_t)lane * B + b] = len;
    }
    for (int k = 0; k < top_paths; ++k) {
        const int lk = rli(len, k);
        int64_t* ov = out + ((size_t)k * B + b) * T;
        for (int i = lk + lane; i < T; i += 64) ov[i] = -1;
    }
}

}  // namespace

// OCRK_BEAM_WAVE=0: the block form for every beam width (A/B)
static bool wave_beam_enabled() { return ocrk::opt(ocrk::OPT_BEAM_WAVE) != 0; }

extern "C" size_t ocrk_ctc_beam_workspace_size(int T, int B, int beam_width) {
    if (T < 0 || B < 0 || beam_width < 1) return 0;
    return (size_t)B * (1 + (size_t)T * beam_width) * sizeof(int2);
}

extern "C" int ocrk_ctc_beam_decode(const float* logits, const int* seq_len, int T, int B, int C,
                                    int beam_width, int top_paths, int merge_repeated, int64_t* out,
                                    int* out_len, float* log_probs, void* ws, size_t ws_bytes,
                                    void* stream) {
    OCRK_REQUIRE(T > 0 && B >= 0 && C >= 2 && C <= BEAM_MAX_C,
                 "ocrk_ctc_beam_decode: bad sizes T=%d B=%d C=%d (C <= %d)", T, B, C, BEAM_MAX_C);
    OCRK_REQUIRE(beam_width >= 1 && beam_width <= BEAM_MAX_K,
                 "ocrk_ctc_beam_decode: beam_width %d not in [1, %d]", beam_width, BEAM_MAX_K);
    OCRK_REQUIRE(top_paths >= 1 && top_paths <= beam_width,
                 "ocrk_ctc_beam_decode: top_paths %d not in [1, beam_width]", top_paths);
    if (B == 0) return OCRK_OK;
    OCRK_REQUIRE(logits && seq_len && out && out_len && log_probs && ws,
                 "ocrk_ctc_beam_decode: null pointer");
    OCRK_REQUIRE(ws_bytes >= ocrk_ctc_beam_workspace_size(T, B, beam_width),
                 "ocrk_ctc_beam_decode: workspace too small");
    if (beam_width <= WB_K && wave_beam_enabled())
        ctc_beam_wave_kernel<<<(unsigned)ocrk::cdiv(B, WB_WAVES), 64 * WB_WAVES, 0, ocrk::as_stream(stream)>>>(
            logits, seq_len, T, B, C, beam_width, top_paths, merge_repeated, out, out_len, log_probs,
            reinterpret_cast<int2*>(ws));
    else
        ctc_beam_kernel<<<B, BEAM_THREADS, 0, ocrk::as_stream(stream)>>>(
            logits, seq_len, T, B, C, beam_width, top_paths, merge_repeated, out, out_len, log_probs,
            reinterpret_cast<int2*>(ws));
    return ocrk::launch_status("ocrk_ctc_beam_decode");
}
