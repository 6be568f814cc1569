// Calibration microbenchmark (gfx950): rocPRIM's radix_sort_pairs on the MSM's sort shape -- 15.7 M
// (16-bit bucket key, 32-bit point reference) pairs, 2^20 points x 15 windows -- as the yardstick for
// the hand-written LSD passes in halo_amd/csrc/sort.hip (not linked into the library).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 sort_bench.hip -o sort_bench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdio.h>
#include <vector>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main() {
    const size_t n = (size_t)15 << 20;
    std::vector<uint32_t> hk(n), hv(n);
    uint64_t x = 0x48414c4f;
    for (size_t i = 0; i < n; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        hk[i] = (uint32_t)(x >> 48);
        hv[i] = (uint32_t)i;
    }
    uint32_t *k0, *k1, *v0, *v1;
    CHECK(hipMalloc(&k0, n * 4)); CHECK(hipMalloc(&k1, n * 4)); CHECK(hipMalloc(&v0, n * 4)); CHECK(hipMalloc(&v1, n * 4));
    CHECK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
    size_t tmp_bytes = 0;
    CHECK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 0, 16));
    void* tmp;
    CHECK(hipMalloc(&tmp, tmp_bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int it = 0; it < 3; it++) CHECK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, 16));
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < reps; it++) CHECK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, 16));
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint32_t> ok(n);
    CHECK(hipMemcpy(ok.data(), k1, n * 4, hipMemcpyDeviceToHost));
    bool sorted = true;
    for (size_t i = 1; i < n; i++) sorted &= ok[i - 1] <= ok[i];
    printf("rocprim radix_sort_pairs 16-bit keys, %zu pairs: %.1f us per sort (%.2f G pairs/s), sorted=%d\n", n,
           ms * 1e3 / reps, n / (ms * 1e-3 / reps) * 1e-9, (int)sorted);
    return 0;
}
