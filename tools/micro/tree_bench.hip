// Single-wave / single-block latency of the XYZZ tree sums (tree.hpp) on gfx950: one block runs
// ITER dependent group sums (the sum re-enters lane 0), so the time per call is the critical path of
// one tree:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../halo_amd/csrc -o tb tree_bench.hip
// (round 5: the levels that leave their sums in place measured 20.9 us per isolated 64-lane tree
// against 19.6 us for the round-3 levels that moved every sum to its list position, yet the library's
// tail rounds and small MSMs ran faster with them: pcdl::open 2^10 1.54 -> 1.48 ms, interleaved)
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "tree.hpp"
using namespace halo;
using F = FqCfg;  // Pallas base field
#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                        \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int ITER = 200;

template <class Cv>
__global__ void k_points(uint4* out, uint32_t n) {
    using Fb = typename Cv::Base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<Fb> g;
    g.x = fe_neg(fe_one<Fb>());
    g.y = fe_add(fe_one<Fb>(), fe_one<Fb>());
    XYZZ<Fb> acc = xyzz_id<Fb>();
    uint32_t k = (i * 2654435761u + 17) | 1u;
    for (int b = 31; b >= 0; b--) {
        acc = xyzz_dbl(acc);
        if ((k >> b) & 1u) acc = xyzz_madd(acc, g);
    }
    xyzz_store(out + 8 * i, acc);
}

// G: group size; block = 64 (wave) or 256 threads
// live: lanes (of each wave) holding points, the others the identity
__global__ __launch_bounds__(256) void k_tree(const uint4* pts, uint32_t G, uint4* out, uint32_t live) {
    __shared__ uint4 red[256 / 2 * 8];
    XYZZ<F> v = (threadIdx.x & 63u) < live ? xyzz_load<F>(pts + 8 * threadIdx.x) : xyzz_id<F>();
    for (int it = 0; it < ITER; it++) {
        const XYZZ<F> s = G <= 64 ? wave_group_sum<F>(v, G) : block_group_sum<F>(v, G, red);
        if (threadIdx.x == 0) v = s;  // the next tree depends on this one
        __syncthreads();
    }
    if (threadIdx.x == 0) xyzz_store(out, v);
}

int main() {
    uint4 *pts, *out;
    CHECK(hipMalloc(&pts, 256 * 128));
    CHECK(hipMalloc(&out, 128));
    hipLaunchKernelGGL(k_points<PallasCurve>, dim3(1), dim3(256), 0, 0, pts, 256);
    CHECK(hipDeviceSynchronize());
    const struct { int block; uint32_t G, live; } cfg[] = {{64, 64, 64}, {64, 8, 64}, {256, 256, 64}, {256, 64, 64},
                                                           {256, 256, 16}, {64, 64, 16}, {64, 64, 1}};
    for (auto c : cfg) {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        hipLaunchKernelGGL(k_tree, dim3(1), dim3(c.block), 0, 0, pts, c.G, out, c.live);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_tree, dim3(1), dim3(c.block), 0, 0, pts, c.G, out, c.live);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        uint32_t h[32];
        CHECK(hipMemcpy(h, out, 128, hipMemcpyDeviceToHost));
        uint32_t x = 0;
        for (int i = 0; i < 32; i++) x = x * 31 + h[i];
        printf("block %3d G %3u live %2u: %.2f us per tree (check %08x)\n", c.block, c.G, c.live,
               ms * 1e3 / ITER, x);
    }
    return 0;
}
