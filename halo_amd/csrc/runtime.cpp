// Runtime: error state, device selection, per-device state, buffers.
#include "runtime.hpp"
#include "msm.hpp"

#include <atomic>
#include <cstdio>
#include <cstring>

namespace halo {

static thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

void clear_error() { g_last_error.clear(); }

int DevBuf::reserve(size_t n) {
    if (n <= bytes && ptr) return HALO_OK;
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    if (n == 0) n = 16;
    hipError_t e = hipMalloc(&ptr, n);
    if (e != hipSuccess) {
        ptr = nullptr;
        return set_error(HALO_ENOMEM, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    }
    bytes = n;
    return HALO_OK;
}

ScratchUse::ScratchUse(DeviceState* st_, hipStream_t s_) : st(st_), s(s_) {
    if (st && st->scratch_used && st->scratch_last != s) (void)hipStreamWaitEvent(s, st->scratch_ev, 0);
}

ScratchUse::~ScratchUse() {
    if (!st) return;
    if (!st->scratch_ev && hipEventCreateWithFlags(&st->scratch_ev, hipEventDisableTiming) != hipSuccess) return;
    if (hipEventRecord(st->scratch_ev, s) == hipSuccess) {
        st->scratch_last = s;
        st->scratch_used = true;
    }
}

void DevBuf::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

DevBuf::~DevBuf() {
    // Device state lives for the process; freeing at exit can race the HIP runtime teardown.
}

static std::mutex g_states_mu;
static std::vector<DeviceState*> g_states;

DeviceState* current_state() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        set_error(HALO_EDEVICE, "no HIP device available: %s", hipGetErrorString(e));
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_states_mu);
    if ((int)g_states.size() <= dev) g_states.resize(dev + 1, nullptr);
    if (!g_states[dev]) {
        g_states[dev] = new DeviceState();
        g_states[dev]->device = dev;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            g_states[dev]->num_cu = cus;
    }
    return g_states[dev];
}

int copy_h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return HALO_OK;
    HALO_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return HALO_OK;
}

int copy_d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return HALO_OK;
    HALO_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    HALO_HIP(hipStreamSynchronize(s));
    return HALO_OK;
}

// ---- profiling ------------------------------------------------------------------------------
struct ProfEntry {
    std::string name;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    size_t launches = 0;
    double total_ms = 0;
};
static std::mutex g_prof_mu;
static std::vector<ProfEntry> g_prof;
static bool g_prof_on = false;

bool prof_enabled() { return g_prof_on; }

ProfScope::ProfScope(const char* name, hipStream_t stream) {
    if (!g_prof_on) return;
    s = stream;
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (size_t i = 0; i < g_prof.size(); i++)
        if (g_prof[i].name == name) slot = (int)i;
    if (slot < 0) {
        g_prof.push_back(ProfEntry{name, {}, 0, 0.0});
        slot = (int)g_prof.size() - 1;
    }
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        slot = -1;
        return;
    }
}

ProfScope::~ProfScope() {
    if (slot < 0) return;
    std::lock_guard<std::mutex> g(g_prof_mu);
    g_prof[slot].pending.emplace_back(a, b);
}

static void prof_drain() {
    for (auto& e : g_prof) {
        for (auto& p : e.pending) {
            (void)hipEventSynchronize(p.second);
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
                e.total_ms += ms;
                e.launches++;
            }
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
        e.pending.clear();
    }
}

// ---- tuning ----------------------------------------------------------------------------------
static const char* const kTuneNames[TUNE_COUNT] = {"ipa_weighted", "ipa_tail",           "ipa_srs_tail_n", "ipa_mat_n",
                                                   "msm_multi_max", "ipa_pool_keep_bytes", "ntt_big_max_log",
                                                   "ntt_even_split", "ipa_pair_max"};
// ntt_big_max_log: the largest transform split into two passes on 2048-element blocks (2^17..2^this);
// larger ones, and any below 2^17, take passes of <= 8 bits on 1024-element blocks (ntt.hip ntt_radices)
// ntt_even_split: passes of <= 8 bits split into even radices where possible (ntt_radices)
// ipa_pair_max: weighted IPA rounds up to this many terms per side run L and R as one MSM (2^19: every
// weighted round of a 2^20 opening; the pair's 17-bit keys sort in a 9-bit and an 8-bit pass)
static const long long kTuneDefault[TUNE_COUNT] = {1, 1, 4096, 2048, 1ll << 18, 1ll << 30, 22, 0, 1ll << 19};
static std::atomic<long long> g_tune[TUNE_COUNT] = {{1},  {1},  {4096}, {2048}, {1ll << 18},
                                                    {1ll << 30}, {22}, {0},  {1ll << 19}};
long long tuning(TuneKey k) { return g_tune[k].load(std::memory_order_relaxed); }
static int tune_index(const char* key) {
    if (!key) return -1;
    for (int k = 0; k < TUNE_COUNT; k++)
        if (!strcmp(key, kTuneNames[k])) return k;
    return -1;
}

}  // namespace halo

using namespace halo;

extern "C" int halo_profile_enable(int on) {
    std::lock_guard<std::mutex> g(g_prof_mu);
    g_prof_on = on != 0;
    return HALO_OK;
}

extern "C" int halo_profile_reset(void) {
    std::lock_guard<std::mutex> g(g_prof_mu);
    prof_drain();
    g_prof.clear();
    return HALO_OK;
}

extern "C" int halo_profile_read(const char* name, size_t* launches, double* total_ms) {
    clear_error();
    if (!name) return set_error(HALO_EINVAL, "null name");
    std::lock_guard<std::mutex> g(g_prof_mu);
    prof_drain();
    for (auto& e : g_prof)
        if (e.name == name) {
            if (launches) *launches = e.launches;
            if (total_ms) *total_ms = e.total_ms;
            return HALO_OK;
        }
    if (launches) *launches = 0;
    if (total_ms) *total_ms = 0;
    return HALO_OK;
}

extern "C" {

int halo_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int halo_init(int device) {
    clear_error();
    int n = halo_device_count();
    if (n <= 0) return set_error(HALO_EDEVICE, "no HIP device available");
    if (device < 0 || device >= n) return set_error(HALO_EINVAL, "device %d out of range (%d devices)", device, n);
    HALO_HIP(hipSetDevice(device));
    HALO_HIP(hipFree(nullptr));  // create context
    return current_state() ? HALO_OK : HALO_EDEVICE;
}

const char* halo_last_error(void) { return g_last_error.c_str(); }

int halo_abi_version(void) { return 100; }

// Releases the library's HIP objects while the runtime is alive: pending profiling events, the MSM
// pipeline's streams and events, the scratch fence events.  Python registers it with atexit
// (halo_amd/_lib.py), which runs before the HIP runtime's own teardown; after it no static
// destructor of this library touches HIP.  The library stays usable (objects are recreated).
int halo_shutdown(void) {
    (void)hipDeviceSynchronize();
    {
        std::lock_guard<std::mutex> g(g_prof_mu);
        prof_drain();
        g_prof.clear();
        g_prof_on = false;
    }
    msm_shutdown();
    ipa_shutdown();
    std::lock_guard<std::mutex> g(g_states_mu);
    for (DeviceState* st : g_states) {
        if (!st) continue;
        std::lock_guard<std::mutex> g2(st->mu);
        if (st->scratch_ev) (void)hipEventDestroy(st->scratch_ev);
        st->scratch_ev = nullptr;
        for (SrsState& srs : st->srs) {
            if (srs.small_ev) (void)hipEventDestroy(srs.small_ev);
            if (srs.small_tab_ev) (void)hipEventDestroy(srs.small_tab_ev);
            srs.small_ev = srs.small_tab_ev = nullptr;
        }
        st->scratch_used = false;
        st->scratch_last = nullptr;
    }
    return HALO_OK;
}

int halo_set_tuning(const char* key, long long value) {
    clear_error();
    const int k = tune_index(key);
    if (k < 0) return set_error(HALO_EINVAL, "unknown tuning key '%s'", key ? key : "(null)");
    g_tune[k].store(value < 0 ? kTuneDefault[k] : value);
    return HALO_OK;
}

int halo_get_tuning(const char* key, long long* value) {
    clear_error();
    const int k = tune_index(key);
    if (k < 0) return set_error(HALO_EINVAL, "unknown tuning key '%s'", key ? key : "(null)");
    if (!value) return set_error(HALO_EINVAL, "halo_get_tuning: null value");
    *value = g_tune[k].load();
    return HALO_OK;
}

int halo_stream_sync(void* stream) {
    HALO_HIP(hipStreamSynchronize((hipStream_t)stream));
    return HALO_OK;
}

}  // extern "C"
