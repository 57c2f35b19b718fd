/* Diagnostics of the tools-only build (`make exp` -> tools/libocrk_exp.so,
 * compiled with -DOCRK_EXPERIMENTS; load it with OCRK_LIB=tools/libocrk_exp.so).
 * NOT part of the product ABI (include/ocrk.h): libocrk.so does not export
 * these, and the experiment toggles they accompany (OCRK_GEMM_NT_CFG,
 * OCRK_GEMM_TN_STAGES=3, OCRK_GEMM_PP=2) are inert in it. */
#pragma once
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Routes measured slower or no better in the train step and kept only here (round 6
 * pruning): the product library does not build them.
 *
 * A stream on the current device whose kernels run on only n_cus of its CUs
 * (hipExtStreamCreateWithCUMask; the CUs left out are evenly spaced over the CU
 * order). NOTE: a BLOCKING stream (the call takes no flags) -- beside work on the
 * legacy NULL stream it serialises with it (the round-5 "+2 ms" A/B); beside a
 * non-blocking step stream masks of 96-192 CUs measured no change at all.
 * Released with ocrk_stream_destroy. */
int ocrk_stream_create_cu_limited(int n_cus, void** stream);
int ocrk_stream_destroy(void* stream);

/* Stream ordering through a ring of events created with hipEventDisableSystemFence
 * (mode 1) or hipEventReleaseToDevice (mode 2) instead of a default event record
 * (mode 0): box-dependent, -35 to +25 us per step. */
int ocrk_stream_wait(void* waiter, void* signaller, int mode);

/* conv2's weight gradient with y1 = relu(conv1(x)) recomputed per row from the image
 * (the partner of ocrk_conv12_fwd with y1 = NULL; +55 us in the step: it lands on the
 * tail). dz bf16 [B,IH-2,IW-2,32]; dw f32 [3][3][32][32] (+)=. */
int ocrk_conv2_bwd_weight_c1x_supported(int B, int IH, int IW, int dtype);
int ocrk_conv2_bwd_weight_c1x(const void* x, int x_is_u8, int B, int IH, int IW, const float* w1, const float* b1,
                              const void* dz, float* dw, int accumulate, void* ws, size_t ws_bytes, int dtype,
                              void* stream);

/* The first layer's forward loop with its input projection fused (no gx): every step
 * 0.7 us longer, no gain (profiles/r3_fused_projection.txt). */
int ocrk_lstm_fwd_persistent_x_supported(int B, int H, int n_in);
int ocrk_lstm_fwd_persistent_x(const void* x, int n_in, const void* wxT, const float* bias, const void* whT,
                               const int* seq_len, int T, int B, int H, void* out, void* hprev_t, float* cprev_t,
                               void* acts_t, unsigned* err, unsigned* flags, void* ws, size_t ws_bytes,
                               void* stream);

/* When buf != NULL the persistent / per-step LSTM forward kernels' workgroups
 * write s_memrealtime stamps ([grid][8] int64) into buf (tools/bench_lstm.py,
 * tools/bench_persist.py). */
int ocrk_lstm_debug_stamps(long long* buf);

#ifdef __cplusplus
}
#endif
