// Cost of stream-ordering packets between dependent kernels on one queue (MI355X):
// N iterations of a short kernel (about 20 us of work on every CU) with, between launches,
//   0: nothing            1: hipEventRecord (no timing)      2: hipStreamWaitEvent on an event
//   recorded (and completed) long ago on another stream    3: both    4: event record on s + wait on s2
// Prints the mean time per iteration; the difference to case 0 is the packets' cost.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_work(float* p, int iters) {
    float v = p[blockIdx.x * blockDim.x + threadIdx.x];
    for (int i = 0; i < iters; i++) v = v * 1.0000001f + 0.5f;
    p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

int main() {
    const int blocks = 256 * 8, threads = 256, N = 200;
    float* d;
    CK(hipMalloc(&d, (size_t)blocks * threads * 4));
    CK(hipMemset(d, 0, (size_t)blocks * threads * 4));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t old, e, t0, t1;
    CK(hipEventCreateWithFlags(&old, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventRecord(old, s2));
    CK(hipStreamSynchronize(s2));
    for (int iters : {2000, 20000}) {
        for (int mode = 0; mode < 5; mode++) {
            for (int rep = 0; rep < 2; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(t0, s));
                for (int i = 0; i < N; i++) {
                    hipLaunchKernelGGL(k_work, dim3(blocks), dim3(threads), 0, s, d, iters);
                    if (mode == 1 || mode == 3) CK(hipEventRecord(e, s));
                    if (mode == 2 || mode == 3) CK(hipStreamWaitEvent(s, old, 0));
                    if (mode == 4) {
                        CK(hipEventRecord(e, s));
                        CK(hipStreamWaitEvent(s2, e, 0));
                    }
                }
                CK(hipEventRecord(t1, s));
                CK(hipEventSynchronize(t1));
                float ms;
                CK(hipEventElapsedTime(&ms, t0, t1));
                if (rep) printf("iters %6d mode %d: %8.2f us per iteration\n", iters, mode, 1e3 * ms / N);
            }
        }
    }
    return 0;
}
