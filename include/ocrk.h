/*
 * ocrk.h -- C ABI of libocrk.so, the MI355X (gfx950) kernels behind the
 * CNN -> BiLSTM -> CTC line-OCR hot path.
 *
 * The reference (tgialoimtr/cnn_lstm_ctc_ocr) has no FFI: its hot path is the
 * TensorFlow-1 graph built by src/weinman/model.py and run by sess.run in
 * src/processing/server.py:132 / src/weinman/train.py:199. Each entry point
 * below names the reference graph op it replaces (file:line). A binding
 * (ctypes here) calls these with device pointers owned by
 * the caller (PyTorch allocations), plain sizes, and the caller's HIP stream.
 *
 * Conventions
 *   - every compute entry returns OCRK_OK (0) or an error code; the message is
 *     available from ocrk_last_error() (thread-local);
 *   - every launch is stream-ordered on `stream` (a hipStream_t, NULL = legacy
 *     default stream); no entry synchronises, allocates or frees device memory,
 *     so all of them are hipGraph-capturable;
 *   - tensors are dense row-major; images/activations are NHWC; the recurrent
 *     and CTC tensors are time-major [T, B, ...] as in the reference
 *     (model.py:212, model.py:226 `time_major=True`);
 *   - `dtype` selects the storage/compute type of activations and weights
 *     (OCRK_F32 or OCRK_BF16); accumulation is always fp32.
 */
#ifndef OCRK_H_
#define OCRK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCRK_ABI_VERSION 7   /* 7: ocrk_conv12_bwd (+ _supported, _workspace_size) */

enum ocrk_status {
    OCRK_OK = 0,
    OCRK_ERR_INVALID_ARG = 1,
    OCRK_ERR_HIP = 2,
    OCRK_ERR_INFEASIBLE = 3 /* CTC: label longer than the input sequence allows */
};

enum ocrk_dtype { OCRK_F32 = 0, OCRK_BF16 = 1 };

/* How OCRK_F32 operands are multiplied by every GEMM / implicit-GEMM conv entry point
 * (process-wide -- torch's autograd issues a backward's launches from its own device
 * thread, so a per-thread mode would miss them; a process that trains in fp32 and
 * serves at the same time must serialise the two; returns the previous
 * mode or an error code):
 *   0 (default) "bf16x3": each fp32 operand split into bf16 hi + lo and a product taken
 *     as ah.bh + ah.bl + al.bh on the bf16 MFMA, f32 accumulation (~2^-16 relative per
 *     product): the fp32 serving path (server.py:78-145 runs float32), logits within
 *     1e-4 of the float64 graph;
 *   1 "exact": v_mfma_f32_16x16x4_f32, exact fp32 products -- fp32 training
 *     (train.Trainer on a float32 store), whose conv-tower gradients amplify product
 *     errors through the BN backward. Also forced by OCRK_F32_MFMA=1.
 * No reference counterpart (TF1 computes float32 on the CPU). */
int ocrk_set_f32_gemm_mode(int mode);
int ocrk_f32_gemm_exact(void);

/* Device status word: a caller-owned, zero-initialised u32 in device memory.
 * Kernels OR these bits into it (agent-scope atomics) when a sequence cannot
 * be processed or a bounded device wait gives up, and still run to completion
 * (no hang, no trap). The library never synchronises: the caller reads the word
 * at a sync point it already has and raises (the Python layer does this;
 * model.py:224-229's tf.nn.ctc_loss raises InvalidArgumentError for the CTC
 * cases with ignore_longer_outputs_than_inputs=False). */
enum ocrk_device_status {
    OCRK_STATUS_CTC_INFEASIBLE = 1 << 1,   /* label + repeats > seq_len, or seq_len == 0 */
    OCRK_STATUS_CTC_BAD_LENGTH = 1 << 2,   /* label_len < 0 or > max_label_len */
    OCRK_STATUS_CTC_BAD_LABEL = 1 << 3,    /* a label value outside [0, C-1) (C-1 is the blank) */
    OCRK_STATUS_LSTM_FWD_TIMEOUT = 1 << 4, /* persistent recurrent forward: a hand-off wait gave up */
    OCRK_STATUS_LSTM_BWD_TIMEOUT = 1 << 5, /* persistent BPTT: a hand-off wait gave up */
    OCRK_STATUS_LSTM_CENSUS = 1 << 6       /* persistent launch: a group's placement census gave up */
};

/* Clear `bits` of the device status word with a device-side atomic AND-NOT,
 * stream-ordered: only the bits the caller has read are cleared, so a bit that
 * a later, still in-flight launch sets is kept (a plain memset would erase it).
 * No reference counterpart (TF raises synchronously at sess.run). */
int ocrk_status_clear(unsigned* status_word, uint32_t bits, void* stream);

int ocrk_version(void);
const char* ocrk_last_error(void);

/* Engine options: route / schedule switches kept for A/B measurement and for the
 * parity tests of alternative routes (no reference counterpart). Each starts from
 * its OCRK_<NAME> environment variable, read once per process; afterwards only
 * ocrk_set_option changes it (process-wide, takes effect at the next launch; the
 * "OCRK_" prefix is optional in `name`). Names: CONV_DIRECT, CONV_ROWS,
 * CONV_ROWS_WIDE, CONV_WGRAD_BLOCKS, LSTM_SPIN_LIMIT, PERSIST_LATE,
 * LSTM_BWD_R16, CTC_LDS, PP_PERSIST_NK, NT_F32_EXACT,
 * NT_F32_MASK, NT_F32_X6, BEAM_WAVE, BN_BWD_BLOCKS, BN_ROUTE, BN_ROUTE_SEG,
 * BN_ROUTE_NCH, CONV_TN_ITEMS, CONV_TN4_ITEMS,
 * CONV_WGRAD_CUS, F32_MFMA, GEMM_NT, GEMM_NT_STAGED, GEMM_PP, GEMM_PPTN, PP_MIN_N, GEMM_TN, LSTM_DMA,
 * LSTM_BWD_DMA, LSTM_FWD_R16, NT_TAP_UNIFORM (meanings in csrc/common.h). Unknown name: OCRK_ERR_INVALID_ARG.
 * `prev` may be NULL. (LSTM_BWD_KSPLIT, LSTM_BWD_PB16 and PP_DEEP: the tools build
 * only -- routes measured slower, not compiled into this library.) */
int ocrk_set_option(const char* name, int64_t value, int64_t* prev);

/* x = hi + lo, hi = bf16(x), lo = bf16(x - hi) (round to nearest even; |x - hi - lo| <=
 * 2^-17 |x|): the bf16x3 split as two bf16 planes [n], so the bf16 GEMM engines form an
 * fp32 product as hi.hi + hi.lo + lo.hi in three accumulating calls (the fp32 training
 * step's weight gradients, train.Trainer). n % 8 == 0, 16-B aligned buffers.
 * No reference counterpart (TF1 multiplies float32 directly). */
int ocrk_split_bf16(const float* x, int64_t n, void* hi, void* lo, void* stream);
int ocrk_get_option(const char* name, int64_t* value);

/* a1 -- validate._preprocess_image (src/weinman/validate.py:56-68):
 * out[i] = float32(in[i]) * float32(1/255) - 0.5, n elements. */
int ocrk_preprocess(const uint8_t* in, int64_t n, void* out, int dtype, void* stream);

/* a9 -- ctc_loss_layer (src/weinman/model.py:224-229) = tf.nn.ctc_loss(labels,
 * logits, seq_len, time_major=True), preprocess_collapse_repeated=False,
 * ctc_merge_repeated=True, blank = C-1, softmax taken inside.
 *   logits  f32 [T, B, C]           labels   i32 [B, max_label_len] (dense, padded)
 *   label_len i32 [B]               seq_len  i32 [B] (frames used per sequence)
 *   loss    f32 [B]  (-log p; +inf for a sequence that cannot be scored)
 *   grad    f32 [T, B, C] or NULL: grad_scale * d loss_b / d logits (0 for t >= seq_len,
 *           all 0 for a sequence that cannot be scored)
 *   status  i32 [B] or NULL: 0 scored, 1 infeasible, 2 bad label_len, 3 bad label value
 *   status_word u32* or NULL: the device status word (OCRK_STATUS_CTC_* bits)
 *   ws: >= ocrk_ctc_workspace_size(T, B, max_label_len) bytes */
size_t ocrk_ctc_workspace_size(int T, int B, int max_label_len);
int ocrk_ctc_loss(const float* logits, const int* labels, const int* label_len, const int* seq_len,
                  int T, int B, int C, int max_label_len, float grad_scale, float* loss, float* grad,
                  int* status, unsigned* status_word, void* ws, size_t ws_bytes, void* stream);

/* a10 -- validate._get_output (src/weinman/validate.py:81-92) =
 * tf.nn.ctc_greedy_decoder(logits, seq_len, merge_repeated) + sparse_to_dense(-1):
 *   out i64 [B, T] (labels then -1), out_len i32 [B], neg_sum_logits f32 [B] or NULL. */
int ocrk_ctc_greedy_decode(const float* logits, const int* seq_len, int T, int B, int C,
                           int merge_repeated, int64_t* out, int* out_len, float* neg_sum_logits,
                           void* stream);


/* a11 -- tf.nn.ctc_beam_search_decoder(logits, seq_len, beam_width, top_paths, merge_repeated)
 * with the default scorer (src/weinman/test.py:84-88 beam 128, merge_repeated=1;
 * src/weinman/client.py:227-231 merge_repeated=0). logits f32 [T, B, C] (blank = C-1, C <= 128),
 * beam_width <= 128, top_paths <= beam_width. out i64 [top_paths][B][T] (labels then -1),
 * out_len i32 [top_paths][B], log_probs f32 [B][top_paths] (log-softmax path scores).
 * ws >= ocrk_ctc_beam_workspace_size(T, B, beam_width) bytes. */
size_t ocrk_ctc_beam_workspace_size(int T, int B, int beam_width);
int ocrk_ctc_beam_decode(const float* logits, const int* seq_len, int T, int B, int C, int beam_width,
                         int top_paths, int merge_repeated, int64_t* out, int* out_len, float* log_probs,
                         void* ws, size_t ws_bytes, void* stream);

/* a14 -- tf.edit_distance(hypothesis, label, normalize=False) (src/weinman/test.py:90) per row:
 * hyp i64 [B][hyp_stride] with hyp_len i32 [B]; label i32 [B][label_stride] (<= 256) with
 * label_len i32 [B]. dist f32 [B] (or NULL); totals i32[3] (or NULL) accumulates
 * {sum edit, count(edit > 0), sum label_len} -- label_error / sequence_error of test.py:91-99. */
int ocrk_edit_distance(const int64_t* hyp, const int* hyp_len, int hyp_stride, const int* label,
                       const int* label_len, int label_stride, int B, float* dist, int* totals,
                       void* stream);

/* ------------------------------------------------------------- conv tower
 * a1+a2 conv1 -- conv_layer(layer_params[0]) (src/weinman/model.py:84-109,134):
 * 3x3 'valid', Cin = 1, bias + ReLU, fused with the uint8 preprocess of
 * validate._preprocess_image when x_is_u8 (x: u8 or dtype [B,H,W]); w f32 HWIO
 * [3][3][1][cout], bias f32 [cout]; y dtype [B,H-2,W-2,cout]. */
int ocrk_conv1_fwd(const void* x, int x_is_u8, int B, int H, int W, const float* w, const float* bias,
                   int cout, void* y, int dtype, void* stream);
/* The same, also writing the ReLU's bit mask relu_bits u8 [B,H-2,W-2][cout/8]: bit c of
 * byte g = (y[...][8 g + c] > 0) -- the training forward's mask for conv2's fused
 * backward (ocrk_conv2_bwd_data_conv1_wgrad), 1/16 of y's bf16 bytes. */
int ocrk_conv1_fwd_relu_bits(const void* x, int x_is_u8, int B, int H, int W, const float* w, const float* bias,
                             int cout, void* y, void* relu_bits, int dtype, void* stream);
/* conv1 -> conv2 forward as one row walk (bf16 training; conv_layer 1 and 2, model.py:84-109,
 * 134-137): conv1's output rows are produced into conv2's LDS ring from the image (conv1 on
 * the MFMA with hi + lo bf16 operands) instead of being written and re-read by conv2. Replaces
 * ocrk_conv1_fwd_relu_bits + ocrk_conv3x3_fwd_rowstats of the first block. x [B,IH,IW] u8
 * (x_is_u8) or bf16; w1 f32 [3][3][1][32], b1 [32]; w_nk2 bf16 [32][3][3][32], b2 [32];
 * y1, z bf16 [B,IH-2,IW-2,32] (y1 may be NULL: not written -- ocrk_conv12_bwd recomputes it);
 * relu_bits u8 [B,IH-2,IW-2][4];
 * stats [B*(IH-2)][2][32] (tile_rows = IW-2). */
int ocrk_conv12_fwd_supported(int B, int IH, int IW, int dtype);
int ocrk_conv12_fwd(const void* x, int x_is_u8, int B, int IH, int IW, const float* w1, const float* b1,
                    const void* w_nk2, const float* b2, void* y1, void* relu_bits, void* z, float* stats, int dtype,
                    void* stream);
/* conv1 weight/bias gradient from dz = dL/d(pre-ReLU conv1), f32 outputs. */
size_t ocrk_conv1_wgrad_workspace_size(int B, int H, int W, int cout);
int ocrk_conv1_bwd_weight(const void* x, int x_is_u8, const void* dz, int B, int H, int W, int cout,
                          float* dw, float* db, int accumulate, void* ws, size_t ws_bytes, int dtype,
                          void* stream);
/* conv2's backward-data and conv1's weight gradient in one pass (bf16; conv2's
 * Cin = Cout = 32, W <= 254): replaces ocrk_conv3x3_bwd_data(dz2, ..., relu_mask = y1)
 * followed by ocrk_conv1_bwd_weight(x, dy1) -- the backprop of conv_layer 2 and 1
 * (model.py:84-109,134-137; TF1's Conv2DBackpropInput of conv2 + Conv2DBackpropFilter
 * and the bias gradient of conv1). dy1 is contracted against x as it is produced and
 * never stored. dz [B,H,W,32] (H, W: conv1's output size), w_bwd [32][3][3][32],
 * the ReLU mask: relu_mask = y1 [B,H,W,32] or relu_bits = its bit mask from
 * ocrk_conv1_fwd_relu_bits (exactly one non-NULL); x [B,H+2,W+2] u8 (x_is_u8: the
 * fused preprocess) or bf16; dw [3][3][1][32] / db [32] f32 (+)= the gradients
 * (fixed-order reduction). */
int ocrk_conv2_bwd_data_conv1_wgrad_supported(int B, int H, int W, int cin, int cout, int dtype);
size_t ocrk_conv2_bwd_data_conv1_wgrad_workspace_size(int B, int H, int W);
int ocrk_conv2_bwd_data_conv1_wgrad(const void* dz, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                                    const void* relu_bits, const void* x, int x_is_u8, float* dw, float* db,
                                    int accumulate, void* ws, size_t ws_bytes, int dtype, void* stream);

/* conv1 -> conv2 backward as one row walk (round 6; the backward of ocrk_conv12_fwd,
 * src/weinman/model.py:84-123 -- TF's conv2d backprop-input / backprop-filter of conv2 and
 * backprop-filter of conv1): conv2's data gradient contracted into conv1's weight gradient
 * as above, plus conv2's weight gradient, its input y1 = relu(conv1(x)) recomputed per row
 * from the image (the bits ocrk_conv12_fwd made), so the forward may pass y1 = NULL.
 * dz [B,H,W,32] bf16; w_bwd conv2's backward image; relu_mask [B,H,W,32] bf16 or relu_bits
 * [B,H,W] u32 (exactly one); x [B,H+2,W+2] u8 (x_is_u8) or bf16; w1 [3][3][1][32] / b1 [32]
 * f32; dw2 [3][3][32][32], dw1 [3][3][1][32], db1 [32] f32 (+)= the batch sums (fixed-order
 * reductions: deterministic). */
int ocrk_conv12_bwd_supported(int B, int H, int W, int dtype);
size_t ocrk_conv12_bwd_workspace_size(int B, int H, int W);
int ocrk_conv12_bwd(const void* dz, int B, int H, int W, const void* w_bwd, const void* relu_mask,
                    const void* relu_bits, const void* x, int x_is_u8, const float* w1, const float* b1, float* dw2,
                    float* dw1, float* db1, int accumulate, void* ws, size_t ws_bytes, int dtype, void* stream);

/* a2 conv2..conv8 -- conv_layer (model.py:84-109) with 'same' padding as an
 * implicit GEMM on MFMA. x [B,H,W,cin]; w_nk [cout][3][3][cin] (dtype);
 * y [B,H,W,cout] in y_dtype; bias f32 or NULL; relu 0/1. stats (or NULL):
 * [ocrk_conv_stats_tiles(B*H*W)][2][cout] per-tile (sum, M2) of the output,
 * the BatchNorm statistics input of ocrk_bn_finalize. */
size_t ocrk_conv_stats_tiles(int64_t M);
/* conv2's forward on the row-walking kernel (conv_rows.hip: Cin = Cout = 32, W <= 254,
 * bf16): stats [B*H][2][cout] = (sum, M2) of each OUTPUT ROW of W pixels, for
 * ocrk_bn_finalize_tiles(..., tile_rows = W, ...). The same z bits as ocrk_conv3x3_fwd. */
int ocrk_conv3x3_fwd_rowstats_supported(int B, int H, int W, int cin, int cout);
int ocrk_conv3x3_fwd_rowstats(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias,
                              int cout, void* y, int relu, float* stats, void* stream);
int ocrk_conv3x3_fwd(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias,
                     int cout, void* y, int y_dtype, int relu, float* stats, int dtype, void* stream);
/* dx [B,H,W,cin] = conv3x3 backward-data of dy [B,H,W,cout] with w_bwd
 * [cin][3][3][cout]; if relu_mask != NULL, dx *= (relu_mask > 0) (the ReLU of
 * the layer that produced x). If dbias != NULL, dbias [cin] f32 (+)= the
 * column sums of dx (the bias gradient of that layer, conv_layer bias
 * model.py:97-104), from the GEMM's per-tile column statistics; needs ws of
 * ocrk_conv3x3_bwd_data_workspace_size bytes (else ws may be NULL). */
size_t ocrk_conv3x3_bwd_data_workspace_size(int B, int H, int W, int cin);
int ocrk_conv3x3_bwd_data(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin,
                          void* dx, const void* relu_mask, float* dbias, int accumulate, void* ws,
                          size_t ws_bytes, int dtype, void* stream);
/* ReLU bit masks between an odd conv's forward and the next even conv's backward-data
 * (conv3 -> conv4, conv5 -> conv6, conv7 -> conv8): _fwd_relu_bits is ocrk_conv3x3_fwd with
 * relu = 1 that also writes relu_bits u8 [B*H*W][cout/8] (bit c of byte c/8: y[..][c] > 0);
 * _bwd_data_bits is ocrk_conv3x3_bwd_data with that bit mask as the ReLU mask (1/16 of the
 * bf16 mask's bytes). bf16 only; *_supported says whether a shape is covered (the wide row
 * kernels or the NT engine's staged epilogue). */
int ocrk_conv3x3_fwd_relu_bits_supported(int B, int H, int W, int cin, int cout, int dtype);
int ocrk_conv3x3_fwd_relu_bits(const void* x, int B, int H, int W, int cin, const void* w_nk, const float* bias,
                               int cout, void* y, void* relu_bits, int dtype, void* stream);
int ocrk_conv3x3_bwd_data_bits_supported(int B, int H, int W, int cout, int cin, int dtype);
int ocrk_conv3x3_bwd_data_bits(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin,
                               void* dx, const void* relu_bits, float* dbias, int accumulate, void* ws,
                               size_t ws_bytes, int dtype, void* stream);
/* The same with the bias-gradient partials left to the caller (as ocrk_conv3x3_bwd_data_slab). */
int ocrk_conv3x3_bwd_data_bits_slab(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin,
                                    void* dx, const void* relu_bits, float* slab, int dtype, void* stream);
/* The same with the bias-gradient reduction left to the caller (e.g. on a side
 * stream, off the data-gradient critical path): slab [ocrk_conv_stats_tiles(B*H*W)]
 * [2*cin] f32 gets the per-tile column (sum, M2) of the masked dx; then
 * ocrk_slab_sum(slab, tiles, cin, 2*cin, dbias, ...) = ocrk_conv3x3_bwd_data's dbias. */
int ocrk_conv3x3_bwd_data_slab(const void* dy, int B, int H, int W, int cout, const void* w_bwd, int cin,
                               void* dx, const void* relu_mask, float* slab, int dtype, void* stream);
/* dw f32 HWIO [3][3][cin][cout] (+)= im2col(x)^T . dy (split-K). */
size_t ocrk_conv3x3_wgrad_workspace_size(int B, int H, int W, int cin, int cout);
int ocrk_conv3x3_bwd_weight(const void* x, const void* dy, int B, int H, int W, int cin, int cout,
                            float* dw, int accumulate, void* ws, size_t ws_bytes, int dtype, void* stream);

/* a3+a4 -- norm_layer (model.py:118-123) + ReLU (:107) + pool_layer / pool8
 * (:111-116, :145-146). bn_finalize: TRAIN-mode batch statistics from the conv
 * epilogue partials (mean, 1/sqrt(var+eps)) and the [TF1] moving averages
 * (moving_mean/var may be NULL = no update). bn_infer_params: INFER mode. */
size_t ocrk_bn_finalize_workspace_size(int tiles, int C);
/* ocrk_bn_finalize for partials of tile_rows rows per tile (the last may be short) */
int ocrk_bn_finalize_tiles(const float* stats, int tiles, int tile_rows, int64_t M, int C, float eps,
                           float momentum, float* mean, float* invstd, float* moving_mean, float* moving_var,
                           void* ws, size_t ws_bytes, void* stream);
int ocrk_bn_finalize(const float* stats, int tiles, int64_t M, int C, float eps, float momentum,
                     float* mean, float* invstd, float* moving_mean, float* moving_var, void* ws, size_t ws_bytes,
                     void* stream);   /* ws: ocrk_bn_finalize_workspace_size bytes (row-range partial sums) */
/* Batch statistics over several data-parallel ranks' batches (SyncBN; the
 * reference is one device, so N ranks with these match its statistics over the
 * union of their batches). ocrk_bn_moments: this rank's merged sums of the same
 * partials, moments f64 [3C + 1] = (sum x | sum_t s_t^2/n_t | sum_t M2_t | M),
 * all additive over ranks; SUM-all-reduce the vector, then
 * ocrk_bn_finalize_moments = ocrk_bn_finalize of the union (the moving averages
 * with the union's unbiased variance). ws: ocrk_bn_finalize_workspace_size. */
int ocrk_bn_moments(const float* stats, int tiles, int tile_rows, int64_t M, int C, double* moments, void* ws,
                    size_t ws_bytes, void* stream);
int ocrk_bn_finalize_moments(const double* moments, int C, float eps, float momentum, float* mean, float* invstd,
                             float* moving_mean, float* moving_var, void* stream);
int ocrk_bn_infer_params(const float* moving_mean, const float* moving_var, int C, float eps,
                         float* mean, float* invstd, void* stream);
/* out = maxpool(relu(gamma (z-mean) invstd + beta)), window kh x kw, stride
 * sh x sw, 'valid'. time_major (requires Ho == 1): out is [Wo, B, C], the
 * features tensor of model.py:147 already transposed as at model.py:212. */
int ocrk_bn_relu_pool_fwd(const void* z, int B, int H, int W, int C, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, int kh, int kw,
                          int sh, int sw, void* out, int time_major, int dtype, void* stream);
/* Backward of the above: dz [B,H,W,C] from dp (pooled gradient, time-major if
 * dp_time_major); dgamma/dbeta f32; dbias f32 or NULL = column sums of dz, the gradient
 * of the conv bias in front of the BN (accumulate 0/1 for all three). */
size_t ocrk_bn_bwd_workspace_size(int B, int H, int W, int C);
int ocrk_bn_relu_pool_bwd(const void* z, const void* dp, int B, int H, int W, int C, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, int kh, int kw,
                          int sh, int sw, int dp_time_major, void* dz, float* dgamma, float* dbeta,
                          float* dbias, int accumulate, void* ws, size_t ws_bytes, int dtype, void* stream);
/* The same with the conv-bias reduction left to the caller: bias_slab f32
 * [ocrk_bn_bwd_bias_slab_rows(...)][C] gets the apply pass's per-block column sums
 * of dz; ocrk_slab_sum(bias_slab, rows, C, C, dbias, ...) = the dbias above. */
size_t ocrk_bn_bwd_bias_slab_rows(int B, int H, int W, int C, int kh, int kw, int sh, int sw);
int ocrk_bn_relu_pool_bwd_slab(const void* z, const void* dp, int B, int H, int W, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* beta, int kh, int kw,
                               int sh, int sw, int dp_time_major, void* dz, float* dgamma, float* dbeta,
                               int accumulate, float* bias_slab, void* ws, size_t ws_bytes, int dtype,
                               void* stream);
/* The same with pass 1 (the dgamma / dbeta sums) read from the forward's pooled
 * output `pooled` (ocrk_bn_relu_pool_fwd's result, laid out as dp) instead of walking
 * z: sum dy = sum_{pooled > 0} dp, sum dy * xhat = sum_{pooled > 0} dp (pooled - beta) / gamma
 * (xhat recovered at each window's max). A channel where |beta| / |gamma| exceeds
 * max(4, |mean| * invstd) (gamma = 0 included) is ill-conditioned for that recovery:
 * its 8-channel group re-evaluates its windows from z instead (decided on the device).
 * Window-walk pools only (2x2/[2,2], 2x2/[2,1], [3,1]/[3,1]); others take the z form.
 * dgamma itself is summed from z in the apply walk (xhat as the z form computes it).
 * bias_slab: NULL (dbias (+)= the conv-bias gradient) or the caller's
 * [ocrk_bn_bwd_pooled_bias_slab_rows(...)][2C] partial rows [bias | dgamma] -- both
 * reductions are then the caller's (ocrk_slab_sum over each half; dbias ignored).
 * ocrk_bn_bwd_pooled_bias_slab_rows() == 0: this pool takes the z form (or option
 * BN_ROUTE is 0), and a bias_slab is refused (OCRK_ERR_INVALID_ARG). */
size_t ocrk_bn_bwd_pooled_bias_slab_rows(int B, int H, int W, int C, int kh, int kw, int sh, int sw);
int ocrk_bn_relu_pool_bwd_pooled(const void* z, const void* pooled, const void* dp, int B, int H, int W, int C,
                                 const float* mean, const float* invstd, const float* gamma, const float* beta,
                                 int kh, int kw, int sh, int sw, int dp_time_major, void* dz, float* dgamma,
                                 float* dbeta, float* dbias, int accumulate, float* bias_slab, void* ws,
                                 size_t ws_bytes, int dtype, void* stream);
/* The backward's two passes apart, for SyncBN: _reduce accumulates this rank's
 * dgamma / dbeta and writes dsum f32 [2C] (sum dy | sum dy*xhat through the ReLU
 * and pool routing); SUM-all-reduce dsum over the ranks; _apply forms dz from
 * those sums over `count` (device f64: all ranks' pixels, ocrk_bn_moments' last
 * entry after its all-reduce), with dbias / bias_slab as above. The same ws
 * serves both calls and must be left untouched between them. */
int ocrk_bn_relu_pool_bwd_reduce(const void* z, const void* dp, int B, int H, int W, int C, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, int kh, int kw,
                                 int sh, int sw, int dp_time_major, float* dgamma, float* dbeta, int accumulate,
                                 float* dsum, void* ws, size_t ws_bytes, int dtype, void* stream);
int ocrk_bn_relu_pool_bwd_apply(const void* z, const void* dp, int B, int H, int W, int C, const float* mean,
                                const float* invstd, const float* gamma, const float* beta, int kh, int kw,
                                int sh, int sw, int dp_time_major, const float* dsum, const double* count,
                                void* dz, float* dbias, int accumulate, float* bias_slab, void* ws,
                                size_t ws_bytes, int dtype, void* stream);

/* ------------------------------------------------------------- recurrent
 * a7' -- rnn_layer with LSTMCell (src/weinman/model_bu.py:167-199), both
 * directions, one launch per time step. Layouts (time order, d = direction):
 *   gx      dtype [T][B][2][4H] = x . W_x + b  (ocrk_gemm, N = 8H; bf16 in bf16 mode)
 *   whT     dtype [2][4H][H]   (recurrent kernel rows of [In+H][4H], transposed)
 *   wh      dtype [2][H][4H]   (recurrent kernel rows as stored)
 *   h_state dtype [2 bufs][2][B][H], c_state f32 [2][B][H] (zero before s = 0)
 *   out     dtype [T][B][2H]   (layer output, must be zeroed: t >= len stays 0)
 *   hprev_t dtype [T][B][2][H], cprev_t f32 [T][B][2][H], acts_t dtype [T][B][2][4H] (gate activations)
 *   dout    dtype [T][B][2H]   dG_t dtype [T][B][2][4H]
 *   dg_state dtype [2 bufs][2][B][4H], dc_state f32 [2][B][H] (zero before the loop) */
int ocrk_lstm_fwd_step(const void* gx, const void* whT, const void* h_in, void* h_out, float* c_state,
                       const int* seq_len, int s, int T, int B, int H, void* out, void* hprev_t,
                       float* cprev_t, void* acts_t, int dtype, void* stream);
int ocrk_lstm_bwd_step(const void* wh, const void* dg_in, void* dg_out, float* dc_state, const int* seq_len,
                       int s, int T, int B, int H, const void* dout, const float* cprev_t,
                       const void* acts_t, void* dG_t, int dtype, void* stream);
/* Persistent forward time loop (bf16, H in {256, 512}, B % 32 == 0): ONE launch
 * runs all T steps of both directions; W_h stays in registers, h is exchanged
 * between co-resident workgroups through write-through stores and per-member
 * flags (model_bu.py:167-199). Same outputs as ocrk_lstm_fwd (h_state/c_state not needed).
 * _supported() says whether the grid fits co-resident on this device; err is
 * the device status word (OCRK_STATUS_LSTM_FWD_TIMEOUT / _CENSUS bits OR-ed in
 * when a bounded hand-off wait gives up; OCRK_LSTM_SPIN_LIMIT sets the bound). */
int ocrk_lstm_fwd_persistent_supported(int B, int H);
size_t ocrk_lstm_fwd_persistent_workspace_size(int B, int H);
int ocrk_lstm_fwd_persistent(const void* gx, const void* whT, const int* seq_len, int T, int B, int H,
                             void* out, void* hprev_t, float* cprev_t, void* acts_t, unsigned* err,
                             unsigned* flags, void* ws, size_t ws_bytes, void* stream);
/* Persistent backward time loop (BPTT of the same layer, bf16): ONE launch runs
 * all T reverse steps of both directions with W_h slices in registers, the
 * gate gradients dz exchanged between the co-resident workgroups of a
 * (direction, 32-row batch slice) group, dc kept in registers. Same dG_t as
 * ocrk_lstm_bwd (dg_state/dc_state not needed); err: the device status word
 * (OCRK_STATUS_LSTM_BWD_TIMEOUT / _CENSUS). */
/* a7' in fp32 (model_bu.py:187-192 in the reference's float32; the serving path
 * server.py:78-145): the forward time loop as one persistent launch, h . W_h on the
 * bf16 MFMA through the bf16x3 split (hi/lo bf16 operands, ah.bh + ah.bl + al.bh,
 * f32 accumulate; ~2^-16 relative per product). gx f32 [T][B][2][4H] (bias included),
 * whT f32 [2][4H][H]; out f32 [T][B][2H] (zeros past each row's length);
 * hprev_t / cprev_t f32 [T][B][2][H] and acts_t f32 [T][B][2][4H] for the BPTT, or
 * all three NULL (inference). H = 512, B % 16 == 0, grid 2 (B/RB) (H/32) co-resident
 * (RB = 16 or 32 rows per member); flags: ocrk_lstm_fwd_persistent_f32_flags_size(B, H)
 * zeroed words kept by the caller (or NULL: cleared per launch); status bits
 * OCRK_STATUS_LSTM_FWD_TIMEOUT / _CENSUS. */
int ocrk_lstm_fwd_persistent_f32_supported(int B, int H);
size_t ocrk_lstm_fwd_persistent_f32_workspace_size(int B, int H);
/* The caller-kept counting hand-off words of this loop (it slices the batch by 16 rows
 * when that grid is co-resident, B <= 128 at H = 512, else by 32). */
size_t ocrk_lstm_fwd_persistent_f32_flags_size(int B, int H);
int ocrk_lstm_fwd_persistent_f32(const float* gx, const float* whT, const int* seq_len, int T, int B, int H,
                                 float* out, float* hprev_t, float* cprev_t, float* acts_t, unsigned* err,
                                 unsigned* flags, void* ws, size_t ws_bytes, void* stream);
/* a7' BPTT in fp32 on the same split: one persistent launch per layer, members
 * (direction, 32-row slice, 32 units) of 8 waves (gate x k-half), W_h hi / lo resident,
 * dz exchanged as hi / lo bf16 planes. wh f32 [2][H][4H]; dout / cprev_t f32
 * [T][B][2][H] (dout as [T][B][2H]); acts_t / dG_t f32 [T][B][2][4H]; dbias_part f32
 * [B/32][2][4H] (or NULL). H = 512, B % 32 == 0, the B-workgroup grid co-resident;
 * flags: ocrk_persistent_flags_size(B, H). Not used in exact fp32 mode (the per-step
 * exact kernels of ocrk_lstm_bwd_step). */
int ocrk_lstm_bwd_persistent_f32_supported(int B, int H);
size_t ocrk_lstm_bwd_persistent_f32_workspace_size(int B, int H);
int ocrk_lstm_bwd_persistent_f32(const float* wh, const int* seq_len, int T, int B, int H, const float* dout,
                                 const float* cprev_t, const float* acts_t, float* dG_t, unsigned* err,
                                 unsigned* flags, float* dbias_part, void* ws, size_t ws_bytes, void* stream);
int ocrk_lstm_bwd_persistent_supported(int B, int H);
/* Rows of dbias_part the BPTT launch writes: B/16 when it runs the 16-row / 64-unit
 * member form (H = 512, its B-workgroup grid co-resident; 64 KB of dz gathered per CU
 * per step instead of 128 KB), else B/32. */
int ocrk_lstm_bwd_persistent_slices(int B, int H);
size_t ocrk_lstm_bwd_persistent_workspace_size(int B, int H);
int ocrk_lstm_bwd_persistent(const void* wh, const int* seq_len, int T, int B, int H, const void* dout,
                             const float* cprev_t, const void* acts_t, void* dG_t, unsigned* err,
                             unsigned* flags, float* dbias_part, void* ws, size_t ws_bytes, void* stream);
/* a7 -- rnn_layer with tf.contrib.rnn.GRUCell (src/weinman/model.py:167-199; [TF1] GRUCell:
 * [r, u] = sig([x, h] Wg + bg), c = tanh([x, r*h] Wc + bc), h' = u h + (1 - u) c) under
 * bidirectional_dynamic_rnn(time_major, sequence_length). gx dtype [T][B][2][3H] = x . [Wg_x | Wc_x]
 * + [bg | bc] per direction (one GEMM). whgT dtype [2][2H][H], whcT [2][H][H] (h-parts,
 * transposed). State h [2][B][H] and rh [2][B][H] (zeroed h). Outputs: out [T][B][2H] (zeroed by
 * the caller; rows past seq_len stay 0), time-order hprev_t, rh_t [T][B][2][H], acts_t
 * [T][B][2][3H] = (r, u, c). One step = two launches (gate, candidate) for both directions. */
int ocrk_gru_fwd_step(const void* gx, const void* whgT, const void* whcT, void* h, void* rh,
                      const int* seq_len, int s, int T, int B, int H, void* out, void* hprev_t, void* rh_t,
                      void* acts_t, int dtype, void* stream);
int ocrk_gru_fwd(const void* gx, const void* whgT, const void* whcT, void* h, void* rh, const int* seq_len,
                 int T, int B, int H, void* out, void* hprev_t, void* rh_t, void* acts_t, int dtype,
                 void* stream);
/* GRU BPTT: whg dtype [2][H][2H], whc [2][H][H] (h-parts, untransposed); scratch dzg [2][B][2H],
 * dzc [2][B][H] (dtype), dh_tot, direct f32 [2][B][H]; dout dtype [T][B][2H]. dG_t dtype
 * [T][B][2][3H] = (dz_r, dz_u, dz_c) in time order, for the dW / dx GEMMs. */
int ocrk_gru_bwd(const void* whg, const void* whc, void* dzg, void* dzc, float* dh_tot, float* direct,
                 const int* seq_len, int T, int B, int H, const void* dout, const void* hprev_t,
                 const void* acts_t, void* dG_t, int dtype, void* stream);
/* Persistent GRU time loops (bf16, H in {256, 512}, B % 32 == 0): ONE launch runs
 * all T steps of both directions (forward) or all T reverse steps (BPTT), the
 * member's W_h slices in registers. The reset gate multiplies h before the
 * candidate matmul, so a step has two group-wide exchanges (r*h, then h; in
 * BPTT dz_c, then dz_r/dz_u). Same outputs as ocrk_gru_fwd / ocrk_gru_bwd
 * without the state/scratch buffers; err: the device status word
 * (OCRK_STATUS_LSTM_FWD_TIMEOUT / _BWD_TIMEOUT / _CENSUS, bounded by
 * OCRK_LSTM_SPIN_LIMIT as for the LSTM loops). */
int ocrk_gru_fwd_persistent_supported(int B, int H);
size_t ocrk_gru_fwd_persistent_workspace_size(int B, int H);
int ocrk_gru_fwd_persistent(const void* gx, const void* whgT, const void* whcT, const int* seq_len, int T, int B,
                            int H, void* out, void* hprev_t, void* rh_t, void* acts_t, unsigned* err,
                            unsigned* flags, void* ws, size_t ws_bytes, void* stream);
int ocrk_gru_bwd_persistent_supported(int B, int H);
size_t ocrk_gru_bwd_persistent_workspace_size(int B, int H);
int ocrk_gru_bwd_persistent(const void* whg, const void* whc, const int* seq_len, int T, int B, int H,
                            const void* dout, const void* hprev_t, const void* acts_t, void* dG_t, unsigned* err,
                            unsigned* flags, float* dbias_part, void* ws, size_t ws_bytes, void* stream);
/* dbias_part (the two BPTT entry points; NULL = skipped): f32 [S][2][G] with
 * S = ocrk_lstm_bwd_persistent_slices(B, H) for the LSTM (B/16 or B/32), B/32 for the GRU,
 * G = 4H (LSTM) / 3H (GRU): per batch slice and direction, the sum of the
 * gate gradients dG_t over its rows and steps -- the layer's bias gradient
 * (model_bu.py:173-180 / model.py:170-180, tf.gradients of the [x,h].W + b
 * sums) fused into the loop; the caller sums the S rows (ocrk_slab_sum)
 * instead of reading dG_t again. */
/* Hand-off words of the persistent loops (the `flags` argument of the four
 * *_persistent entry points above): NULL = they live in the workspace and are
 * cleared by a memset before every launch; else a caller-kept buffer of
 * ocrk_persistent_flags_size(B, H) bytes, zeroed ONCE, that the loops count on
 * from (no clearing launch in front of every loop). Keep one buffer per
 * (entry point, B, H, stream): launches sharing a buffer must not overlap. */
size_t ocrk_persistent_flags_size(int B, int H);
int ocrk_lstm_fwd(const void* gx, const void* whT, void* h_state, float* c_state, const int* seq_len,
                  int T, int B, int H, void* out, void* hprev_t, float* cprev_t, void* acts_t, int dtype,
                  void* stream);
int ocrk_lstm_bwd(const void* wh, void* dg_state, float* dc_state, const int* seq_len, int T, int B, int H,
                  const void* dout, const float* cprev_t, const void* acts_t, void* dG_t, int dtype,
                  void* stream);

/* ------------------------------------------------------- dense / generic
 * MFMA GEMM: C[b] = alpha op(A[b]) op(B[b]) + bias (ReLU) (+= C if accumulate).
 * trans_a: 0 A=[M][K] (lda), 1 A=[K][M]; trans_b: 0 B=[K][N] (ldb), 1 B=[N][K].
 * A/B in dtype, C in c_dtype (accumulate needs f32). Used for the recurrent
 * input projections (model.py:187-192), the logits layer (model.py:216-220)
 * and their gradients. splits > 1 = split-K through ws. */
size_t ocrk_gemm_workspace_size(int M, int N, int batch, int splits);
int ocrk_gemm(int trans_a, int trans_b, int M, int N, int K, float alpha, const void* A, int64_t lda,
              int64_t stride_a, const void* B, int64_t ldb, int64_t stride_b, void* C, int64_t ldc,
              int64_t stride_c, int c_dtype, const float* bias, int relu, int accumulate, int batch,
              int dtype, int splits, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- train op
 * a13 -- Adam of train.py:128-137 ([TF1] ApplyAdam) on a flat f32 buffer;
 * lr_t = lr sqrt(1-b2^t)/(1-b1^t) computed by the caller; g is scaled by
 * grad_scale (e.g. 1/world_size after a summing all-reduce). */
int ocrk_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr_t, float beta1,
              float beta2, float eps, float grad_scale, void* stream);
/* The same update with flags: OCRK_ADAM_ZERO_GRAD clears g as it is read (the
 * next step's zero-gradient pass folded into the optimizer's; Trainer uses it
 * and skips its own fill). */
#define OCRK_ADAM_ZERO_GRAD 1u
int ocrk_adam_ex(float* p, float* g, float* m, float* v, int64_t n, float lr_t, float beta1,
                 float beta2, float eps, float grad_scale, unsigned flags, void* stream);

/* Batched weight images: ONE launch for a table of 2-D copies (device array of
 * `njobs` records of 8 x 8 bytes: {const float* src; void* dst; int64 rows, cols,
 * in_rs, out_rs, tile0; int32 transpose, dtype}), tile0 = the job's first 32x32
 * tile (prefix sum, ascending), total_tiles = all jobs' tiles. Plain:
 * dst[r*out_rs + c] = src[r*in_rs + c]; transposed: dst[c*out_rs + r] =
 * src[r*in_rs + c]; f32 -> dtype. Replaces the per-image ocrk_strided_copy /
 * ocrk_permute3 launches of a parameter version (ParamStore.refresh_images). */
int ocrk_copy_batch(const void* jobs, int njobs, int64_t total_tiles, void* stream);
/* -------------------------------------------------------------- utilities */
int ocrk_cast(const void* in, int in_dtype, void* out, int out_dtype, int64_t n, void* stream);
int ocrk_permute3(const void* in, int in_dtype, int d0, int d1, int d2, void* out, int out_dtype,
                  void* stream);  /* out[i1][i0][i2] = in[i0][i1][i2] */
int ocrk_strided_copy(const float* in, int64_t rows, int64_t cols, int64_t in_rs, int64_t in_cs, void* out,
                      int out_dtype, int64_t out_rs, int64_t out_cs, void* stream);
size_t ocrk_colsum_workspace_size(int64_t M, int N);
int ocrk_colsum(const void* in, int64_t M, int N, int dtype, float* out, int accumulate, void* ws,
                size_t ws_bytes, void* stream);
/* out [nc] f32 (+)= the column sums of a [nslab][ld] f32 slab of partial rows, in
 * a fixed order with double accumulation (deterministic): the reduction step
 * of the *_slab entry points and of the persistent loops' dbias_part. */
size_t ocrk_slab_sum_workspace_size(int nc);
int ocrk_slab_sum(const float* slab, int nslab, int nc, int ld, float* out, int accumulate, void* ws,
                  size_t ws_bytes, void* stream);
/* out = (y > 0) ? dy * scale : 0 (ReLU backward of the logits, model.py:216) */
int ocrk_relu_mask(const float* dy, const float* y, int64_t n, float scale, void* out, int out_dtype,
                   void* stream);
int ocrk_mul_scalar(float* x, int64_t n, const float* s, void* stream);
int ocrk_mean(const float* x, int n, float* out, void* stream);
/* model.py:152-163: seq_len = floor((width - 2) / 2) - 2 */
int ocrk_seq_len(const int* widths, int n, int* out, void* stream);

/* Launch-probe timers (bench.py's roofline leg; no reference counterpart).
 * A hipEvent_t behind an opaque handle; ocrk_timer_record on a stream that is
 * being captured into a hipGraph adds an event-record node at the capture
 * frontier, so graph replays keep timing the bracketed work.
 * ocrk_timer_elapsed = milliseconds between two completed records. */
int ocrk_timer_create(void** ev);
int ocrk_timer_record(void* ev, void* stream);
int ocrk_timer_elapsed(void* ev0, void* ev1, float* ms);
int ocrk_timer_destroy(void* ev);

/* Host-side CRC32C (Castagnoli) of n bytes continuing from `crc` (0 to start):
 * TFRecord framing and TensorBundle checksums for the input pipeline and the
 * checkpoint reader/writer (src/weinman/mjsynth.py:148-172, train.py:152-165). */
uint32_t ocrk_crc32c(const void* data, size_t n, uint32_t crc);

#ifdef __cplusplus
}
#endif
#endif /* OCRK_H_ */
