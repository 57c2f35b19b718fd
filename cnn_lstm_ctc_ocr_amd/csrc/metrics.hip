// a14 -- tf.edit_distance(hypothesis, label, normalize=False) and the
// CER / sequence-error totals of src/weinman/test.py:89-99.
//
// One wave per (hypothesis, label) pair. Lane j of chunk c holds column
// 1 + 64c + j of the Levenshtein row. Row i is
//   A_j = min(D[i-1][j] + 1, D[i-1][j-1] + (h_i != l_j)),   A_0 = i
//   D[i][j] = min_{k<=j} (A_k + j - k)
// i.e. j + a prefix-min of (A_k - k) across lanes, carried between chunks.
#include "common.h"

namespace {

constexpr int ED_MAX_LABEL = 256;
constexpr int ED_CHUNKS = ED_MAX_LABEL / 64;

__device__ __forceinline__ int wave_prefix_min(int v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int u = __shfl_up(v, o, 64);
        if (lane >= o) v = min(v, u);
    }
    return v;
}

__global__ void __launch_bounds__(256)
edit_distance_kernel(const int64_t* __restrict__ hyp, const int* __restrict__ hyp_len, int hyp_stride,
                     const int* __restrict__ label, const int* __restrict__ label_len, int label_stride,
                     int B, float* __restrict__ dist, int* __restrict__ totals) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;                                  // whole wave exits together
    const int Lh = min(max(hyp_len[b], 0), hyp_stride);
    const int Ll = min(max(label_len[b], 0), label_stride);
    const int64_t* h = hyp + (size_t)b * hyp_stride;
    const int* l = label + (size_t)b * label_stride;

    int lab[ED_CHUNKS], row[ED_CHUNKS];
#pragma unroll
    for (int c = 0; c < ED_CHUNKS; ++c) {
        const int j = 1 + c * 64 + lane;
        lab[c] = j <= Ll ? l[j - 1] : -2;
        row[c] = j;                                      // D[0][j] = j
    }
    const int nchunks = (Ll + 63) >> 6;
    for (int i = 1; i <= Lh; ++i) {
        const int hi = (int)h[i - 1];
        int carry_old = i - 1;                           // D[i-1][0]
        int carry_min = i;                               // min_{k<j}(A_k - k), k = 0 term
#pragma unroll
        for (int c = 0; c < ED_CHUNKS; ++c) {
            if (c < nchunks) {
                const int j = 1 + c * 64 + lane;
                int left_old = __shfl_up(row[c], 1, 64);
                if (lane == 0) left_old = carry_old;
                const int a = min(row[c] + 1, left_old + (hi != lab[c] ? 1 : 0));
                int pm = wave_prefix_min(a - j, lane);
                pm = min(pm, carry_min);
                carry_old = __shfl(row[c], 63, 64);
                row[c] = j + pm;
                carry_min = __shfl(pm, 63, 64);
            }
        }
    }
    int d;
    if (Ll == 0) {
        d = Lh;
    } else {
        const int c = (Ll - 1) >> 6, src = (Ll - 1) & 63;
        int v = 0;
#pragma unroll
        for (int q = 0; q < ED_CHUNKS; ++q)
            if (q == c) v = row[q];
        d = __shfl(v, src, 64);
    }
    if (lane == 0) {
        if (dist) dist[b] = (float)d;
        if (totals) {
            atomicAdd(&totals[0], d);
            atomicAdd(&totals[1], d > 0 ? 1 : 0);
            atomicAdd(&totals[2], Ll);
        }
    }
}

}  // namespace

extern "C" int ocrk_edit_distance(const int64_t* hyp, const int* hyp_len, int hyp_stride, const int* label,
                                  const int* label_len, int label_stride, int B, float* dist, int* totals,
                                  void* stream) {
    OCRK_REQUIRE(B >= 0 && hyp_stride >= 0 && label_stride >= 0 && label_stride <= ED_MAX_LABEL,
                 "ocrk_edit_distance: bad sizes B=%d hyp_stride=%d label_stride=%d (<= %d)", B, hyp_stride,
                 label_stride, ED_MAX_LABEL);
    if (B == 0) return OCRK_OK;
    OCRK_REQUIRE(hyp && hyp_len && label && label_len && (dist || totals), "ocrk_edit_distance: null pointer");
    edit_distance_kernel<<<(B + 3) / 4, 256, 0, ocrk::as_stream(stream)>>>(hyp, hyp_len, hyp_stride, label,
                                                                           label_len, label_stride, B, dist,
                                                                           totals);
    return ocrk::launch_status("ocrk_edit_distance");
}
