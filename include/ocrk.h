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

#define OCRK_ABI_VERSION 1

enum ocrk_status {
    OCRK_OK = 0,
    OCRK_ERR_INVALID_ARG = 1,
    OCRK_ERR_HIP = 2,
    OCRK_ERR_INFEASIBLE = 3 /* CTC: label longer than the input sequence allows */
};

enum ocrk_dtype { OCRK_F32 = 0, OCRK_BF16 = 1 };

int ocrk_version(void);
const char* ocrk_last_error(void);

/* a1 -- validate._preprocess_image (src/weinman/validate.py:56-68):
 * out[i] = float32(in[i]) * float32(1/255) - 0.5, n elements. */
int ocrk_preprocess(const uint8_t* in, int64_t n, void* out, int dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OCRK_H_ */
