/* Diagnostics of the tools-only build (`make exp` -> tools/libocrk_exp.so,
 * compiled with -DOCRK_EXPERIMENTS; load it with OCRK_LIB=tools/libocrk_exp.so).
 * NOT part of the product ABI (include/ocrk.h): libocrk.so does not export
 * these, and the experiment toggles they accompany (OCRK_GEMM_NT_CFG,
 * OCRK_GEMM_TN_STAGES=3, OCRK_GEMM_PP=2) are inert in it. */
#pragma once
#ifdef __cplusplus
extern "C" {
#endif

/* When buf != NULL the persistent / per-step LSTM forward kernels' workgroups
 * write s_memrealtime stamps ([grid][8] int64) into buf (tools/bench_lstm.py,
 * tools/bench_persist.py). */
int ocrk_lstm_debug_stamps(long long* buf);

#ifdef __cplusplus
}
#endif
