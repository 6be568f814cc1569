// Microbenchmark (gfx950): field-multiplication throughput of one dependent product chain per lane
// (fe_mul) against two independent chains interleaved mad by mad (fe_mul_x2), at 1-8 waves per SIMD.
// Question it answers: is the single-chain product latency-bound at the 4 waves/SIMD k_acc runs at?
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../halo_amd/csrc mul_ilp_bench.hip -o mul_ilp_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "fields.hpp"
using namespace halo;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// V0: two products per iteration, each one chain (fe_mul then fe_mul); V1: the same two products
// through fe_mul_x2.  Both do 2 modmul per iteration on 2 independent values.
template <int V, int MINW>
__global__ __launch_bounds__(256, MINW) void bench(uint4* d, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<FqCfg> a = fe_load<FqCfg>(d + 8 * i), b = fe_load<FqCfg>(d + 8 * i + 2);
    Fe<FqCfg> c = fe_load<FqCfg>(d + 8 * i + 4), e = fe_load<FqCfg>(d + 8 * i + 6);
    for (int k = 0; k < iters; k++) {
        Fe<FqCfg> x, y;
        if (V == 0) {
            x = fe_mul(a, b);
            y = fe_mul(c, e);
        } else {
            fe_mul_x2(a, b, c, e, x, y);
        }
        b = a;
        a = x;
        e = c;
        c = y;
    }
    fe_store(d + 8 * i, a);
    fe_store(d + 8 * i + 4, c);
}

template <typename K>
double timeit(K kern, uint4* d, int blocks, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main() {
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;
        const size_t n = (size_t)256 * blocks;
        uint4* d;
        CHECK(hipMalloc(&d, n * 8 * sizeof(uint4)));
        std::vector<uint32_t> h(n * 32);
        for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u + 12345) & 0x1fffffffu;
        const int iters = 256;
        double t[2];
        std::vector<uint32_t> o[2];
        for (int v = 0; v < 2; v++) {
            CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            t[v] = timeit(v == 0 ? bench<0, 2> : bench<1, 2>, d, blocks, iters);
            CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            hipLaunchKernelGGL((v == 0 ? bench<0, 2> : bench<1, 2>), dim3(blocks), dim3(256), 0, 0, d, 5);
            o[v].resize(h.size());
            CHECK(hipMemcpy(o[v].data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        }
        printf("waves/SIMD %d: fe_mul x2 %.3e, fe_mul_x2 %.3e modmul/s, same=%d\n", wps,
               2.0 * n * iters / (t[0] * 1e-3), 2.0 * n * iters / (t[1] * 1e-3), (int)(o[0] == o[1]));
        CHECK(hipFree(d));
    }
    return 0;
}
