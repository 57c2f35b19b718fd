// Plain GEMMs on hipBLASLt: C[M,N] (bf16) = A[M,K] . B[N,K]^T (+ bias[N], f32)
// with A row-major and B stored [N][K] -- the recurrent input projections
// (gx = x . W_x^T + b, model.py:180-199 / rnn_layer) and the data gradients
// dx = dG . W_x of the recurrent and logits layers. These are plain library
// GEMMs (no im2col, no fused BN statistics / masks): on these shapes hipBLASLt
// measured ~2x the hand-written NT engine (tools/bench_vendor.py vs
// tools/bench_gemm.py), so gemm() routes them here; everything with a fused
// epilogue or an implicit-GEMM operand stays on the hand-written engines.
// OCRK_BLASLT=0 disables the route.
//
// Also the weight gradients (TN): C[M,N] f32 (+= when accumulating) =
// A[K,M]^T . B[K,N] with both operands stored k-major (dW = x^T dG,
// h_prev^T dG, logits x^T dpre): hipBLASLt sees A' = B as N x K (ld = ldb,
// op N) and B' = A as M x K (ld = lda, op T); beta = 1 accumulates into the
// f32 gradient, and one call covers all of K (no split-K partials).
// Opt-in (OCRK_BLASLT_TN=1): on the step's shapes (M = 256..1024, N = 2048,
// K = 32000) the library's heuristic pick measured 200-394 TFLOP/s
// (tools/bench_gemm.py), and the train step 8.25 ms against 8.03 ms with the
// split-K gemm_tn engine, so gemm_tn stays the default.
//
// Row-major C[M][N] is column-major C^T (N x M, ld = ldc) = B . A^T: hipBLASLt
// sees A' = B as a K x N column-major matrix (ld = ldb) with op T, B' = A as
// K x M (ld = lda) with op N, m = N, n = M; the bias (one value per n of our
// C) is then per row of D, which is what HIPBLASLT_EPILOGUE_BIAS adds.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <tuple>

#include "gemm.h"

namespace ocrk {
namespace {

struct LtPlan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo;
    size_t ws = 0;
    bool ok = false;
};

typedef std::tuple<int, int, int, int64_t, int64_t, int64_t, bool, bool> PlanKey;   // ..., bias, tn

constexpr size_t LT_WS_BYTES = 32u << 20;

struct LtState {
    hipblasLtHandle_t h = nullptr;
    bool tried = false, ok = false;
    std::map<PlanKey, LtPlan> plans;
    std::map<hipStream_t, void*> ws;                  // one workspace per stream (main / side run concurrently)
};

LtState& lt() {
    static LtState s;
    if (!s.tried) {
        s.tried = true;
        const char* e = getenv("OCRK_BLASLT");   // opt-in A/B reference only (OCRK_BLASLT=1)
        if (!(e && e[0] == '1')) return s;
        s.ok = hipblasLtCreate(&s.h) == HIPBLAS_STATUS_SUCCESS;
    }
    return s;
}

void* lt_ws(LtState& s, hipStream_t st) {
    auto it = s.ws.find(st);
    if (it != s.ws.end()) return it->second;
    // a stream's workspace is allocated on its first eager use; a stream being
    // captured into a hipGraph must not allocate (the caller then falls back
    // to the in-house engine)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, LT_WS_BYTES) != hipSuccess) p = nullptr;
    s.ws[st] = p;
    return p;
}

LtPlan* lt_plan(LtState& s, const GemmParams& p, bool bias, bool tn) {
    PlanKey key{p.M, p.N, p.K, p.lda, p.ldb, p.ldc, bias, tn};
    auto it = s.plans.find(key);
    if (it != s.plans.end()) return it->second.ok ? &it->second : nullptr;
    LtPlan& pl = s.plans[key];
    bool good = hipblasLtMatmulDescCreate(&pl.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
    const hipblasOperation_t opA = tn ? HIPBLAS_OP_N : HIPBLAS_OP_T, opB = tn ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)) ==
                       HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)) ==
                       HIPBLAS_STATUS_SUCCESS;
    if (bias) {
        const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
        const int32_t bt = HIP_R_32F;
        good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) ==
                           HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt,
                                                       sizeof(bt)) == HIPBLAS_STATUS_SUCCESS;
    }
    if (tn) {
        good = good && hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, p.N, p.K, p.ldb) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, p.M, p.K, p.lda) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lc, HIP_R_32F, p.N, p.M, p.ldc) == HIPBLAS_STATUS_SUCCESS;
    } else {
        good = good && hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, p.K, p.N, p.ldb) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, p.K, p.M, p.lda) == HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatrixLayoutCreate(&pl.lc, HIP_R_16BF, p.N, p.M, p.ldc) == HIPBLAS_STATUS_SUCCESS;
    }
    if (good) {
        hipblasLtMatmulPreference_t pref;
        good = hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
        const uint64_t wsb = LT_WS_BYTES;
        good = good && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                             sizeof(wsb)) == HIPBLAS_STATUS_SUCCESS;
        hipblasLtMatmulHeuristicResult_t res[1];
        int n = 0;
        good = good && hipblasLtMatmulAlgoGetHeuristic(s.h, pl.desc, pl.la, pl.lb, pl.lc, pl.lc, pref, 1, res, &n) ==
                           HIPBLAS_STATUS_SUCCESS && n > 0;
        if (good) {
            pl.algo = res[0].algo;
            pl.ws = res[0].workspaceSize;
        }
        hipblasLtMatmulPreferenceDestroy(pref);
    }
    pl.ok = good && pl.ws <= LT_WS_BYTES;
    return pl.ok ? &pl : nullptr;
}

}  // namespace

bool blaslt_tn_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("OCRK_BLASLT_TN");      // OCRK_BLASLT_TN=1: weight gradients on hipBLASLt
        on = (e && e[0] == '1') ? 1 : 0;
    }
    return on == 1;
}

int gemm_blaslt(const GemmParams& p, int amode, int bmode, int dtype, hipStream_t stream) {
    const bool nt = amode == A_ROWK && bmode == B_NK && p.c_bf16 && !p.accumulate;
    const bool tn = amode == A_COLK && bmode == B_KN && !p.c_bf16 && !p.bias && blaslt_tn_enabled();
    if (!(nt || tn) || dtype != OCRK_BF16) return -1;
    if (p.batch != 1 || p.stats || p.mask || p.relu || p.alpha != 1.f) return -1;
    if (nt && p.splits != 1) return -1;
    if (tn && (((uintptr_t)p.A | (uintptr_t)p.B | (uintptr_t)p.C) % 16 != 0 || p.lda % 8 || p.ldb % 8 || p.ldc % 4))
        return -1;
    LtState& s = lt();
    if (!s.ok) return -1;
    LtPlan* pl = lt_plan(s, p, p.bias != nullptr, tn);
    if (!pl) return -1;
    void* ws = pl->ws ? lt_ws(s, stream) : nullptr;
    if (pl->ws && !ws) return -1;
    if (p.bias) {
        const void* bp = p.bias;
        if (hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)) !=
            HIPBLAS_STATUS_SUCCESS)
            return -1;
    }
    const float alpha = 1.f, beta = p.accumulate ? 1.f : 0.f;
    hipblasStatus_t st = hipblasLtMatmul(s.h, pl->desc, &alpha, p.B, pl->la, p.A, pl->lb, &beta, p.C, pl->lc, p.C,
                                         pl->lc, &pl->algo, ws, pl->ws, stream);
    if (st != HIPBLAS_STATUS_SUCCESS) {
        set_error("gemm_blaslt: hipblasLtMatmul failed (%d) for M=%d N=%d K=%d", (int)st, p.M, p.N, p.K);
        return OCRK_ERR_HIP;
    }
    return launch_status("gemm_blaslt");
}

}  // namespace ocrk
