/* ocrk_comm: the optional gradient all-reduce of the data-parallel train step
 * (SURVEY.md §8b "optional allreduce (RCCL)", §8e) as a C ABI beside libocrk.so.
 *
 * The reference has no multi-device path (src/weinman/train.py:128-137 builds one
 * tower); C4 (B = 2048 over 8 MI355X) adds one RCCL sum of the flat fp32 gradient
 * buffer per step. The Python trainer exchanges it through torch.distributed
 * (backend "nccl" = RCCL; train.GradBuckets); this library is the same collective
 * for a host that binds the kernels through the C ABI instead of PyTorch (a TF
 * custom-op build). It is a separate shared object so libocrk.so
 * itself does not depend on RCCL.
 *
 * One communicator per process and GPU (one process per GPU over xGMI):
 *   rank 0: ocrk_comm_unique_id(id)  -> send the OCRK_COMM_ID_BYTES bytes to every rank
 *   every rank: ocrk_comm_init(&comm, world, rank, id, device)
 *   per step:   ocrk_allreduce_sum(flat_grad, n, OCRK_COMM_F32, comm, stream)  (in place, stream-ordered)
 *   end:        ocrk_comm_destroy(comm)
 * Every call returns OCRK_COMM_OK (0) or an error code; ocrk_comm_last_error() holds
 * the calling thread's last message. */
#ifndef OCRK_COMM_H_
#define OCRK_COMM_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCRK_COMM_ABI_VERSION 1
#define OCRK_COMM_ID_BYTES 128

enum ocrk_comm_status { OCRK_COMM_OK = 0, OCRK_COMM_ERR_INVALID_ARG = 1, OCRK_COMM_ERR_RCCL = 2, OCRK_COMM_ERR_HIP = 3 };
/* element types of ocrk_allreduce_sum (0 / 1 are include/ocrk.h's OCRK_F32 / OCRK_BF16) */
enum ocrk_comm_dtype { OCRK_COMM_F32 = 0, OCRK_COMM_BF16 = 1, OCRK_COMM_F64 = 2, OCRK_COMM_I32 = 3 };

int ocrk_comm_version(void);
/* rank 0's rendezvous token (ncclGetUniqueId), OCRK_COMM_ID_BYTES bytes into id_out */
int ocrk_comm_unique_id(void* id_out);
/* this rank's communicator on HIP device `device` (ncclCommInitRank; blocks until all
 * `world` ranks have called it with the same id) */
int ocrk_comm_init(void** comm, int world, int rank, const void* id, int device);
int ocrk_comm_info(void* comm, int* world, int* rank);
/* buf[0 .. count) = the element-wise sum over the ranks, in place, on `stream` (NULL:
 * the default stream). The gradient exchange of train.py's GradBuckets: the caller
 * scales by 1 / world (the optimizer's grad_scale) */
int ocrk_allreduce_sum(void* buf, size_t count, int dtype, void* comm, void* stream);
int ocrk_comm_destroy(void* comm);
const char* ocrk_comm_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* OCRK_COMM_H_ */
