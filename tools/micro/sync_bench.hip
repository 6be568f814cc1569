// Host round-trip latency of a short kernel (launch -> host sees completion) by wait method:
//   0 hipStreamSynchronize   1 spin on hipStreamQuery   2 hipEventRecord + spin on hipEventQuery
//   3 hipEventRecord + hipEventSynchronize   4 kernel writes a flag to pinned host memory, host spins on it
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_tiny(unsigned* flag, unsigned v) {
    if (threadIdx.x == 0 && flag) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    unsigned* flag;
    CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
    *flag = 0;
    const int N = 2000;
    for (int mode = 0; mode < 5; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 1; i <= N; i++) {
                hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, mode == 4 ? flag : nullptr, (unsigned)(i + rep * N));
                if (mode == 0) CK(hipStreamSynchronize(s));
                if (mode == 1) while (hipStreamQuery(s) == hipErrorNotReady) {}
                if (mode == 2) { CK(hipEventRecord(e, s)); while (hipEventQuery(e) == hipErrorNotReady) {} }
                if (mode == 3) { CK(hipEventRecord(e, s)); CK(hipEventSynchronize(e)); }
                if (mode == 4) while (__atomic_load_n((volatile unsigned*)flag, __ATOMIC_ACQUIRE) != (unsigned)(i + rep * N)) {}
            }
            auto t1 = std::chrono::steady_clock::now();
            if (rep) printf("mode %d: %7.2f us per round trip\n", mode, std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
        }
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
