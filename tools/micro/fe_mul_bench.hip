// Microbenchmark: throughput of halo::fe_mul (round 3: one inline-asm v_mad_u64_u32 chain per column,
// mad_chain.hpp) against one asm statement per product (round 2), two interleaved chains, and the
// compiler-scheduled C expression (split column sums), on gfx950; plus single-wave latency.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "fields.hpp"
using namespace halo;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while(0)

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t d; uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint64_t mad64s(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t d; uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "s"(b), "v"(c));
    return d;
}

template <class C>
__device__ __forceinline__ Fe<C> fe_mul_asm(const Fe<C>& a, const Fe<C>& b) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            acc = mad64(a.v[i], b.v[j], acc);
        }
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (i >= k || j < 1 || j >= NLIMB || C::P[j] == 0) continue;
            acc = mad64s(m[i], C::P[j], acc);
        }
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}

// two interleaved chains per column (independent neighbours: no dependent-mad hazard nop)
template <class C>
__device__ __forceinline__ Fe<C> fe_mul_asm2(const Fe<C>& a, const Fe<C>& b) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
        uint64_t acc2 = 0;
        int par = 0;
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            if (par++ & 1) acc2 = mad64(a.v[i], b.v[j], acc2); else acc = mad64(a.v[i], b.v[j], acc);
        }
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (i >= k || j < 1 || j >= NLIMB || C::P[j] == 0) continue;
            if (par++ & 1) acc2 = mad64s(m[i], C::P[j], acc2); else acc = mad64s(m[i], C::P[j], acc);
        }
        acc += acc2;
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}


template <typename K>
double timeit(K kern, uint4* d, int blocks, int threads, int iters) {
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, iters);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, iters);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

// compiler-scheduled column sums (split chains, more ILP)
template <class C>
__device__ __forceinline__ Fe<C> fe_mul_c(const Fe<C>& a, const Fe<C>& b) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            acc += (uint64_t)a.v[i] * b.v[j];
        }
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (i >= k || j < 1 || j >= NLIMB || C::P[j] == 0) continue;
            acc += (uint64_t)m[i] * C::P[j];
        }
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}
template <int V>
__global__ void bench(uint4* d, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<FqCfg> a = fe_load<FqCfg>(d + 4 * i), b = fe_load<FqCfg>(d + 4 * i + 2);
    for (int k = 0; k < iters; k++) {
        Fe<FqCfg> c = V == 0 ? fe_mul(a, b) : (V == 1 ? fe_mul_asm(a, b) : (V == 2 ? fe_mul_asm2(a, b) : fe_mul_c(a, b)));
        b = a;
        a = c;
    }
    fe_store(d + 4 * i, a);
}

template <int V>
__global__ void lat(uint4* d, int iters) {
    const int i = threadIdx.x;
    Fe<FqCfg> a = fe_load<FqCfg>(d + 4 * i), b = fe_load<FqCfg>(d + 4 * i + 2);
    for (int k = 0; k < iters; k++) a = V == 0 ? fe_mul_c(a, b) : (V == 1 ? fe_mul_asm(a, b) : fe_mul(a, b));
    fe_store(d + 4 * i, a);
}

int main() {
    {
        uint4* d; CHECK(hipMalloc(&d, 64 * 4 * sizeof(uint4)));
        CHECK(hipMemset(d, 1, 64 * 4 * sizeof(uint4)));
        for (int v = 0; v < 3; v++) {
            double t = timeit(v == 0 ? lat<0> : (v == 1 ? lat<1> : lat<2>), d, 1, 64, 4096);
            printf("single-wave dependent chain: %s %.1f ns per modmul\n",
                   v == 0 ? "compiler-split" : (v == 1 ? "asm per product" : "fields.hpp fe_mul"), t * 1e6 / 4096);
        }
        CHECK(hipFree(d));
    }
    const int threads = 256;
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;  // wps waves per SIMD
        size_t n = (size_t)threads * blocks;
        uint4* d; CHECK(hipMalloc(&d, n * 4 * sizeof(uint4)));
        std::vector<uint32_t> h(n * 16);
        for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u + 12345) & 0x3fffffffu;
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        const int iters = 512;
        double t0 = timeit(bench<0>, d, blocks, threads, iters);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        double t1 = timeit(bench<1>, d, blocks, threads, iters);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        double t2 = timeit(bench<2>, d, blocks, threads, iters);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        double t3 = timeit(bench<3>, d, blocks, threads, iters);
        std::vector<uint32_t> o0(n * 16), o1(n * 16);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(threads), 0, 0, d, 7);
        CHECK(hipMemcpy(o0.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(threads), 0, 0, d, 7);
        CHECK(hipMemcpy(o1.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> o2(n * 16);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(threads), 0, 0, d, 7);
        CHECK(hipMemcpy(o2.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> o3(n * 16);
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(bench<3>, dim3(blocks), dim3(threads), 0, 0, d, 7);
        CHECK(hipMemcpy(o3.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        printf("waves/SIMD %d: fe_mul (fields.hpp, one asm statement per multiplication) %.3e, asm per product %.3e, asm-2chain %.3e, compiler-split %.3e modmul/s, same=%d%d%d\n", wps,
               n * (double)iters / (t0 * 1e-3), n * (double)iters / (t1 * 1e-3), n * (double)iters / (t2 * 1e-3),
               n * (double)iters / (t3 * 1e-3), (int)(o0 == o1), (int)(o0 == o2), (int)(o0 == o3));
        CHECK(hipFree(d));
    }
    return 0;
}
