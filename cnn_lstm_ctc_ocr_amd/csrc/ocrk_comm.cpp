// RCCL all-reduce behind include/ocrk_comm.h: the data-parallel gradient exchange of the
// C4 train step for hosts that bind the C ABI instead of PyTorch.
// Host code only; every collective is enqueued on the caller's HIP stream, in place.
#include "ocrk_comm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int rccl_status(ncclResult_t r, const char* what) {
    return r == ncclSuccess ? OCRK_COMM_OK : fail(OCRK_COMM_ERR_RCCL, "%s: %s", what, ncclGetErrorString(r));
}

static_assert(sizeof(ncclUniqueId) == OCRK_COMM_ID_BYTES, "RCCL's unique id is not OCRK_COMM_ID_BYTES bytes");

}  // namespace

extern "C" {

int ocrk_comm_version(void) { return OCRK_COMM_ABI_VERSION; }

int ocrk_comm_unique_id(void* id_out) {
    if (!id_out) return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_comm_unique_id: null id buffer");
    ncclUniqueId id;
    const int st = rccl_status(ncclGetUniqueId(&id), "ocrk_comm_unique_id");
    if (st == OCRK_COMM_OK) std::memcpy(id_out, &id, sizeof id);
    return st;
}

int ocrk_comm_init(void** comm, int world, int rank, const void* id, int device) {
    if (!comm || !id) return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_comm_init: null comm slot or id");
    *comm = nullptr;
    if (world < 1 || rank < 0 || rank >= world)
        return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_comm_init: rank %d outside world %d", rank, world);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_comm_init: device %d of %d", device, ndev);
    // the communicator binds the CURRENT device: switch to `device` for the init and
    // give the calling thread its previous device back afterwards
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return fail(OCRK_COMM_ERR_HIP, "ocrk_comm_init: hipGetDevice");
    if (hipSetDevice(device) != hipSuccess) return fail(OCRK_COMM_ERR_HIP, "ocrk_comm_init: hipSetDevice(%d)", device);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclComm_t c = nullptr;
    const int st = rccl_status(ncclCommInitRank(&c, world, uid, rank), "ocrk_comm_init");
    if (st == OCRK_COMM_OK) *comm = c;
    if (prev != device && hipSetDevice(prev) != hipSuccess) {
        if (c) ncclCommDestroy(c);
        *comm = nullptr;
        return fail(OCRK_COMM_ERR_HIP, "ocrk_comm_init: restoring device %d", prev);
    }
    return st;
}

int ocrk_comm_info(void* comm, int* world, int* rank) {
    if (!comm || !world || !rank) return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_comm_info: null argument");
    int st = rccl_status(ncclCommCount((ncclComm_t)comm, world), "ocrk_comm_info (count)");
    if (st != OCRK_COMM_OK) return st;
    return rccl_status(ncclCommUserRank((ncclComm_t)comm, rank), "ocrk_comm_info (rank)");
}

int ocrk_allreduce_sum(void* buf, size_t count, int dtype, void* comm, void* stream) {
    if (!comm) return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_allreduce_sum: null communicator");
    if (count == 0) return OCRK_COMM_OK;
    if (!buf) return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_allreduce_sum: null buffer for %zu elements", count);
    ncclDataType_t t;
    switch (dtype) {
        case OCRK_COMM_F32: t = ncclFloat32; break;
        case OCRK_COMM_BF16: t = ncclBfloat16; break;
        case OCRK_COMM_F64: t = ncclFloat64; break;
        case OCRK_COMM_I32: t = ncclInt32; break;
        default: return fail(OCRK_COMM_ERR_INVALID_ARG, "ocrk_allreduce_sum: dtype %d", dtype);
    }
    return rccl_status(ncclAllReduce(buf, buf, count, t, ncclSum, (ncclComm_t)comm, (hipStream_t)stream),
                       "ocrk_allreduce_sum");
}

int ocrk_comm_destroy(void* comm) {
    if (!comm) return OCRK_COMM_OK;
    return rccl_status(ncclCommDestroy((ncclComm_t)comm), "ocrk_comm_destroy");
}

const char* ocrk_comm_last_error(void) { return g_err; }

}  // extern "C"
