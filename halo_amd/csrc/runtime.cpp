// Runtime: error state, device selection, per-device state, buffers.
#include "runtime.hpp"

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

}  // namespace halo

using namespace halo;

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

int halo_stream_sync(void* stream) {
    HALO_HIP(hipStreamSynchronize((hipStream_t)stream));
    return HALO_OK;
}

}  // extern "C"
