// Prototype A/B: bucket accumulation with batch-affine additions against the
// XYZZ mixed additions of k_acc, on gfx950.  Each thread sums chunks of K = 16 points gathered at
// random from a 2^20-point table (as k_acc gathers the window-shifted SRS):
//   xyzz  : one XYZZ accumulator per chunk, xyzz_madd_acc per point (k_acc's inner loop, 8M + 2S);
//   affJ  : J chunks per thread advanced in lockstep, affine accumulators; each step adds one point to
//           each of the J accumulators with ONE inversion (Montgomery's trick over the J differences:
//           3 (J - 1) / J multiplications + fe_inv / J, then 2M + 1S per addition).
// Reports additions per second and checks that both give the same chunk sums (affine).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../halo_amd/csrc -o batch_affine_bench batch_affine_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

#include "curve.hpp"
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

constexpr int K = 16;
constexpr uint32_t NPTS = 1u << 20;

__device__ __forceinline__ uint32_t rnd(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// random points: 2^i-style multiples are not needed, any curve points do -- k G by double-and-add
template <class Cv>
__global__ void k_points(uint4* out, uint32_t n) {
    using Fb = typename Cv::Base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<Fb> g;
    g.x = fe_neg(fe_one<Fb>());  // (-1, 2): the Pasta generator
    g.y = fe_add(fe_one<Fb>(), fe_one<Fb>());
    XYZZ<Fb> acc = xyzz_id<Fb>();
    uint32_t k = rnd(i * 2654435761u + 17) | 1u;
    for (int b = 31; b >= 0; b--) {
        acc = xyzz_dbl(acc);
        if ((k >> b) & 1u) acc = xyzz_madd(acc, g);
    }
    aff_store(out + 4 * i, xyzz_to_aff(acc));
}

__device__ __forceinline__ void store_canon(uint4* p, const Affine<F>& a) {
    Affine<F> c;
    c.x = fe_canon(a.x);
    c.y = fe_canon(a.y);
    aff_store(p, c);
}

__device__ __forceinline__ uint32_t pidx(uint32_t chunk, int e) { return rnd(chunk * 977u + (uint32_t)e * 31337u) & (NPTS - 1); }

__global__ __launch_bounds__(256) void k_xyzz(const uint4* pts, uint32_t nchunks, uint4* out) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    XYZZ<F> acc = xyzz_id<F>();
    for (int e = 0; e < K; e++) acc = xyzz_madd_acc(acc, aff_load<F>(pts + 4 * pidx(c, e)), 0u);
    store_canon(out + 4 * c, xyzz_to_aff(xyzz_settle(acc)));
}

__global__ __launch_bounds__(256) void k_xyzz_plain(const uint4* pts, uint32_t nchunks, uint4* out) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    XYZZ<F> acc = xyzz_id<F>();
    for (int e = 0; e < K; e++) acc = xyzz_madd(acc, aff_load<F>(pts + 4 * pidx(c, e)));
    store_canon(out + 4 * c, xyzz_to_aff(acc));
}

// J chunks per thread: chunks t * J + j
template <int J>
__global__ __launch_bounds__(256) void k_aff(const uint4* pts, uint32_t nchunks, uint4* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if ((size_t)t * J >= nchunks) return;
    Affine<F> A[J];
#pragma unroll
    for (int j = 0; j < J; j++) A[j] = aff_load<F>(pts + 4 * pidx(t * J + j, 0));
    for (int e = 1; e < K; e++) {
        Fe<F> pre[J];
        Fe<F> run = fe_one<F>();
#pragma unroll
        for (int j = 0; j < J; j++) {
            const Affine<F> P = aff_load<F>(pts + 4 * pidx(t * J + j, e));
            run = fe_mul(run, fe_sub(P.x, A[j].x));  // (random points: x_P != x_A)
            pre[j] = run;
        }
        Fe<F> inv = fe_inv(run);
#pragma unroll
        for (int j = J - 1; j >= 0; j--) {
            const Affine<F> P = aff_load<F>(pts + 4 * pidx(t * J + j, e));  // L1/L2 hit
            const Fe<F> dx = fe_sub(P.x, A[j].x);
            const Fe<F> ij = j ? fe_mul(inv, pre[j - 1]) : inv;
            if (j) inv = fe_mul(inv, dx);
            const Fe<F> lam = fe_mul(fe_sub(P.y, A[j].y), ij);
            Affine<F> R;
            R.x = fe_sub(fe_sub(fe_sqr(lam), A[j].x), P.x);
            R.y = fe_sub(fe_mul(lam, fe_sub(A[j].x, R.x)), A[j].y);
            A[j] = R;
        }
    }
#pragma unroll
    for (int j = 0; j < J; j++) store_canon(out + 4 * ((size_t)t * J + j), A[j]);
}

template <typename Kern>
float timeit(Kern k, dim3 g, const uint4* pts, uint32_t nchunks, uint4* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k, g, dim3(256), 0, 0, pts, nchunks, out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k, g, dim3(256), 0, 0, pts, nchunks, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main() {
    uint4 *pts, *o1, *o2;
    const uint32_t nchunks = 1u << 20;  // 16 M additions, the k_acc launch of a 2^20 MSM
    CHECK(hipMalloc(&pts, (size_t)NPTS * 64));
    CHECK(hipMalloc(&o1, (size_t)nchunks * 64));
    CHECK(hipMalloc(&o2, (size_t)nchunks * 64));
    hipLaunchKernelGGL(k_points<PallasCurve>, dim3(NPTS / 256), dim3(256), 0, 0, pts, NPTS);
    CHECK(hipDeviceSynchronize());
    const double adds = (double)nchunks * (K - 1);
    const float tx = timeit(k_xyzz, dim3(nchunks / 256), pts, nchunks, o1);
    printf("xyzz madd (k_acc inner loop): %.3f ms, %.3e additions/s\n", tx, adds / (tx * 1e-3));
    std::vector<uint4> h1((size_t)nchunks * 4), h2((size_t)nchunks * 4);
    CHECK(hipMemcpy(h1.data(), o1, (size_t)nchunks * 64, hipMemcpyDeviceToHost));
    auto run = [&](auto kern, int J, const char* name) {
        const float t = timeit(kern, dim3((nchunks / J + 255) / 256), pts, nchunks, o2);
        CHECK(hipMemcpy(h2.data(), o2, (size_t)nchunks * 64, hipMemcpyDeviceToHost));
        size_t same = 0;
        for (size_t i = 0; i < (size_t)nchunks * 4; i++)
            same += h1[i].x == h2[i].x && h1[i].y == h2[i].y && h1[i].z == h2[i].z && h1[i].w == h2[i].w;
        size_t first = 0;
        while (first < (size_t)nchunks * 4 && h1[first].x == h2[first].x && h1[first].y == h2[first].y) first++;
        printf("%s (J = %d): %.3f ms, %.3e additions/s, %.2fx of xyzz, same chunk sums %s (%zu of %zu words; first diff %zu)\n",
               name, J, t, adds / (t * 1e-3), tx / t, same == (size_t)nchunks * 4 ? "yes" : "NO", same,
               (size_t)nchunks * 4, first);
    };
    run(k_xyzz_plain, 1, "xyzz madd (complete formula, check)");
    run(k_aff<1>, 1, "affine (one inversion per addition)");
    run(k_aff<4>, 4, "batch affine");
    run(k_aff<8>, 8, "batch affine");
    run(k_aff<16>, 16, "batch affine");
    return 0;
}
