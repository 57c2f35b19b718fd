// libocrk runtime plumbing: version, thread-local error string, launch status.
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
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

// ---------------------------------------------------------------- options
namespace {
struct OptDef {
    const char* name;
    int64_t def;
    bool exp = false;       // measured-slower route: only the tools build (make exp) reads / sets it
};
constexpr OptDef kOptDefs[OPT_COUNT] = {
    {"CONV_DIRECT", 1}, {"CONV_ROWS", 1}, {"CONV_ROWS_WIDE", 1}, {"CONV_WGRAD_BLOCKS", 1},
    {"LSTM_SPIN_LIMIT", 0}, {"PERSIST_LATE", 1}, {"LSTM_BWD_KSPLIT", 0, true}, {"LSTM_BWD_PB16", 0, true},
    {"LSTM_BWD_R16", 1}, {"CTC_LDS", 1}, {"PP_PERSIST_NK", 8}, {"PP_DEEP", 0, true}, {"NT_F32_EXACT", 1},
    {"NT_F32_MASK", 1},
    {"NT_F32_X6", 0}, {"BEAM_WAVE", 1}, {"BN_BWD_BLOCKS", 2048}, {"BN_ROUTE", 1}, {"BN_ROUTE_SEG", 8}, {"BN_ROUTE_NCH", 4},
    {"CONV_TN_ITEMS", 192},
    {"CONV_TN4_ITEMS", 512}, {"CONV_WGRAD_CUS", 192}, {"F32_MFMA", 0}, {"GEMM_NT", 1}, {"GEMM_NT_STAGED", 1},
    {"GEMM_PP", 1}, {"GEMM_PPTN", 1}, {"PP_MIN_N", 512}, {"GEMM_TN", 1}, {"LSTM_DMA", 1}, {"LSTM_BWD_DMA", 1},
    {"LSTM_FWD_R16", 1}, {"NT_TAP_UNIFORM", 1},
};
std::atomic<int64_t> g_opts[OPT_COUNT];
std::once_flag g_opts_once;

#ifdef OCRK_EXPERIMENTS
constexpr bool kExperiments = true;
#else
constexpr bool kExperiments = false;
#endif

void init_opts() {
    for (int i = 0; i < OPT_COUNT; ++i) {
        if (kOptDefs[i].exp && !kExperiments) {          // the product library: the default, always
            g_opts[i].store(kOptDefs[i].def, std::memory_order_relaxed);
            continue;
        }
        char env[64];
        snprintf(env, sizeof(env), "OCRK_%s", kOptDefs[i].name);
        const char* e = getenv(env);
        g_opts[i].store(e && *e ? atoll(e) : kOptDefs[i].def, std::memory_order_relaxed);
    }
}

int find_opt(const char* name) {
    if (!name) return -1;
    if (!strncmp(name, "OCRK_", 5)) name += 5;
    for (int i = 0; i < OPT_COUNT; ++i)
        if (!strcmp(name, kOptDefs[i].name)) return kOptDefs[i].exp && !kExperiments ? -1 : i;
    return -1;
}
}  // namespace

int64_t opt(Option o) {
    std::call_once(g_opts_once, init_opts);
    return g_opts[o].load(std::memory_order_relaxed);
}

}  // namespace ocrk

extern "C" {

int ocrk_version(void) { return OCRK_ABI_VERSION; }

int ocrk_set_option(const char* name, int64_t value, int64_t* prev) {
    const int i = ocrk::find_opt(name);
    OCRK_REQUIRE(i >= 0, "ocrk_set_option: unknown option '%s'", name ? name : "(null)");
    ocrk::opt((ocrk::Option)i);                         // defaults from the environment first
    const int64_t old = ocrk::g_opts[i].exchange(value, std::memory_order_relaxed);
    if (prev) *prev = old;
    return OCRK_OK;
}

int ocrk_get_option(const char* name, int64_t* value) {
    const int i = ocrk::find_opt(name);
    OCRK_REQUIRE(i >= 0 && value, "ocrk_get_option: unknown option '%s' or null slot", name ? name : "(null)");
    *value = ocrk::opt((ocrk::Option)i);
    return OCRK_OK;
}

const char* ocrk_last_error(void) { return ocrk::g_err; }

// Event timers for launch probes. Recorded on a capturing stream they become
// event-record nodes of the hipGraph (appended at the capture frontier), so a
// replayed graph still timestamps the launches it brackets.
int ocrk_timer_create(void** ev) {
    OCRK_REQUIRE(ev != nullptr, "ocrk_timer_create: null handle slot");
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return ocrk::launch_status("ocrk_timer_create");
    *ev = e;
    return OCRK_OK;
}

int ocrk_timer_record(void* ev, void* stream) {
    OCRK_REQUIRE(ev != nullptr, "ocrk_timer_record: null event");
    hipStream_t st = ocrk::as_stream(stream);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return ocrk::launch_status("ocrk_timer_record");
    hipError_t e = hipSuccess;
    if (cs == hipStreamCaptureStatusActive) {
        // append an event-record node after the capture's current frontier and
        // make it the new frontier (the stream-ordered equivalent of a record)
        unsigned long long id = 0;
        hipGraph_t g = nullptr;
        const hipGraphNode_t* deps = nullptr;
        size_t nd = 0;
        hipGraphNode_t node = nullptr;
        e = hipStreamGetCaptureInfo_v2(st, &cs, &id, &g, &deps, &nd);
        if (e == hipSuccess) e = hipGraphAddEventRecordNode(&node, g, deps, nd, (hipEvent_t)ev);
        if (e == hipSuccess) e = hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
    } else {
        e = hipEventRecord((hipEvent_t)ev, st);
    }
    if (e != hipSuccess) {
        ocrk::set_error("ocrk_timer_record: %s", hipGetErrorString(e));
        return OCRK_ERR_HIP;
    }
    return OCRK_OK;
}

#ifdef OCRK_EXPERIMENTS
// include/ocrk_debug.h (tools build): fence-less stream forks and CU-masked streams.
// Both measured no gain in the train step; a CU-masked stream is a
// BLOCKING stream (hipExtStreamCreateWithCUMask takes no flags), so beside work on the
// legacy NULL stream it serialises with it.
int ocrk_stream_wait(void* waiter, void* signaller, int mode) {
    OCRK_REQUIRE(mode >= 0 && mode <= 2, "ocrk_stream_wait: mode %d", mode);
    constexpr int RING = 64, MAXDEV = 64;
    static std::mutex mu;
    static hipEvent_t ring[MAXDEV][3][RING] = {};
    static int next[MAXDEV][3] = {};
    int dev = 0;
    // the events live on the signaller's device (a ring per device and mode)
    if (hipStreamGetDevice(ocrk::as_stream(signaller), &dev) != hipSuccess || dev < 0 || dev >= MAXDEV)
        return ocrk::launch_status("ocrk_stream_wait");
    std::lock_guard<std::mutex> lk(mu);
    const int i = next[dev][mode];
    hipEvent_t& ev = ring[dev][mode][i];
    if (!ev) {
        const unsigned fl = hipEventDisableTiming |
                            (mode == 1 ? hipEventDisableSystemFence : mode == 2 ? hipEventReleaseToDevice : 0u);
        int cur = 0;
        hipError_t ce = hipGetDevice(&cur);
        if (ce == hipSuccess && cur != dev) ce = hipSetDevice(dev);   // created on the signaller's device
        if (ce == hipSuccess) ce = hipEventCreateWithFlags(&ev, fl);
        if (cur != dev) {
            const hipError_t re = hipSetDevice(cur);
            if (ce == hipSuccess) ce = re;
        }
        if (ce != hipSuccess) {
            ocrk::set_error("ocrk_stream_wait create: %s", hipGetErrorString(ce));
            return OCRK_ERR_HIP;
        }
    }
    next[dev][mode] = (i + 1) % RING;
    hipError_t e = hipEventRecord(ev, ocrk::as_stream(signaller));
    if (e == hipSuccess) e = hipStreamWaitEvent(ocrk::as_stream(waiter), ev, 0);
    if (e != hipSuccess) {
        ocrk::set_error("ocrk_stream_wait: %s", hipGetErrorString(e));
        return OCRK_ERR_HIP;
    }
    return OCRK_OK;
}

int ocrk_stream_create_cu_limited(int n_cus, void** stream) {
    OCRK_REQUIRE(stream != nullptr && n_cus > 0, "ocrk_stream_create_cu_limited: n_cus %d / null slot", n_cus);
    const int total = ocrk::cu_count();
    uint32_t mask[ocrk::kMaxCuWords] = {};
    OCRK_REQUIRE(total <= 32 * ocrk::kMaxCuWords, "ocrk_stream_create_cu_limited: %d CUs", total);
    // keep n of every `total` CUs, the left-out ones evenly spaced over the CU
    // order (so every XCD / shader engine keeps some for other streams)
    const int keep = n_cus < total ? n_cus : total;
    for (int i = 0; i < total; ++i) {
        const bool on = (int64_t)(i + 1) * keep / total != (int64_t)i * keep / total;
        if (on) mask[i / 32] |= 1u << (i % 32);
    }
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)((total + 31) / 32), mask);
    if (e != hipSuccess) {
        ocrk::set_error("ocrk_stream_create_cu_limited: %s", hipGetErrorString(e));
        return OCRK_ERR_HIP;
    }
    *stream = s;
    return OCRK_OK;
}

int ocrk_stream_destroy(void* stream) {
    if (stream) (void)hipStreamDestroy(ocrk::as_stream(stream));
    return OCRK_OK;
}
#endif  // OCRK_EXPERIMENTS

int ocrk_timer_elapsed(void* ev0, void* ev1, float* ms) {
    OCRK_REQUIRE(ev0 && ev1 && ms, "ocrk_timer_elapsed: null argument");
    hipError_t e = hipEventElapsedTime(ms, (hipEvent_t)ev0, (hipEvent_t)ev1);
    if (e != hipSuccess) {
        ocrk::set_error("ocrk_timer_elapsed: %s", hipGetErrorString(e));
        return OCRK_ERR_HIP;
    }
    return OCRK_OK;
}

int ocrk_timer_destroy(void* ev) {
    if (ev) (void)hipEventDestroy((hipEvent_t)ev);
    return OCRK_OK;
}

}  // extern "C"

// ------------------------------------------------------------ host CRC32C
// Castagnoli CRC (TFRecord framing, TensorBundle checksums): SSE4.2 crc32
// instruction when the host has it, else a byte table.
namespace {
uint32_t crc_table[256];
bool crc_table_ready = false;

void build_crc_table() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_table[i] = c;
    }
    crc_table_ready = true;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t c, const unsigned char* p, size_t n) {
    uint64_t c64 = c;
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c64 = __builtin_ia32_crc32di(c64, v);
        p += 8;
        n -= 8;
    }
    c = (uint32_t)c64;
    while (n--) c = __builtin_ia32_crc32qi(c, *p++);
    return c;
}
}  // namespace

extern "C" uint32_t ocrk_crc32c(const void* data, size_t n, uint32_t crc) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    uint32_t c = ~crc;
    if (__builtin_cpu_supports("sse4.2")) {
        c = crc32c_hw(c, p, n);
    } else {
        if (!crc_table_ready) build_crc_table();
        for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    }
    return ~c;
}
