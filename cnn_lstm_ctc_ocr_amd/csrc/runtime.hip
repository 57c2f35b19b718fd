// libocrk runtime plumbing: version, thread-local error string, launch status.
#include <cstdarg>
#include <cstdio>
#include "common.h"

namespace ocrk {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return OCRK_ERR_HIP;
    }
    return OCRK_OK;
}

}  // namespace ocrk

extern "C" {

int ocrk_version(void) { return OCRK_ABI_VERSION; }

const char* ocrk_last_error(void) { return ocrk::g_err; }

}  // extern "C"
