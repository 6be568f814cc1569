// VALU issue ceilings by instruction class on one MI355X (round 5; the compute roofline of bench.py).
//
// Each kernel runs 8 independent chains of one instruction (or of a fixed mix) per lane, 64 per loop
// iteration, at 8 waves per SIMD, so the rate is the SIMD's issue rate for that class, not a latency.
// The mixes test whether class costs ADD on a SIMD (MI355X_MICROARCH.md: "costs add") -- if a 1:1 mix
// of a VOP3 and a VOP2 instruction took less than the sum of their costs, a ceiling built by adding
// per-class costs would not be a ceiling.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/issue_bench.hip -o tools/micro/issue_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// I64: the chain variable is 64-bit; I32: 32-bit.  BODY(x) expands one instruction on chain x.
#define KERNEL(NAME, T, INSTR)                                                                 \
    __global__ void NAME(uint4* data, int iters) {                                              \
        int i = blockIdx.x * blockDim.x + threadIdx.x;                                          \
        uint4 x = data[i];                                                                      \
        T a0 = x.x, a1 = x.y, a2 = x.z, a3 = x.w, a4 = x.x ^ 1, a5 = x.y ^ 2, a6 = x.z ^ 3, a7 = x.w ^ 4; \
        uint32_t m = x.x | 1;                                                                   \
        for (int k = 0; k < iters; k++) {                                                       \
            _Pragma("unroll") for (int u = 0; u < 8; u++) {                                     \
                asm volatile(INSTR : "+v"(a0) : "v"(m)); asm volatile(INSTR : "+v"(a1) : "v"(m)); \
                asm volatile(INSTR : "+v"(a2) : "v"(m)); asm volatile(INSTR : "+v"(a3) : "v"(m)); \
                asm volatile(INSTR : "+v"(a4) : "v"(m)); asm volatile(INSTR : "+v"(a5) : "v"(m)); \
                asm volatile(INSTR : "+v"(a6) : "v"(m)); asm volatile(INSTR : "+v"(a7) : "v"(m)); \
            }                                                                                   \
        }                                                                                       \
        data[i] = make_uint4((uint32_t)(a0 ^ a1 ^ a2 ^ a3), (uint32_t)(a4 ^ a5 ^ a6 ^ a7), (uint32_t)a0, (uint32_t)a7); \
    }

KERNEL(k_mad_u64, uint64_t, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
KERNEL(k_mad_i64, uint64_t, "v_mad_i64_i32 %0, vcc, %1, %1, %0")
KERNEL(k_ashr64, uint64_t, "v_ashrrev_i64 %0, 29, %0")
KERNEL(k_lshladd64, uint64_t, "v_lshl_add_u64 %0, %0, 0, %0")
KERNEL(k_add3, uint32_t, "v_add3_u32 %0, %0, %1, %0")
KERNEL(k_alignbit, uint32_t, "v_alignbit_b32 %0, %0, %1, 29")
KERNEL(k_and_lit, uint32_t, "v_and_b32_e32 %0, 0x1fffffff, %0")
KERNEL(k_and, uint32_t, "v_and_b32_e32 %0, %0, %1")
KERNEL(k_add, uint32_t, "v_add_u32_e32 %0, %0, %1")
KERNEL(k_sub, uint32_t, "v_sub_u32_e32 %0, %0, %1")
KERNEL(k_ashr32, uint32_t, "v_ashrrev_i32_e32 %0, 29, %0")
KERNEL(k_mov, uint32_t, "v_mov_b32_e32 %0, %1")
KERNEL(k_cndmask, uint32_t, "v_cndmask_b32_e32 %0, %0, %1, vcc")
// 1:1 mixes: a 64-bit chain and a 32-bit chain advanced alternately (two instructions per step)
#define MIX(NAME, I64, I32)                                                                     \
    __global__ void NAME(uint4* data, int iters) {                                              \
        int i = blockIdx.x * blockDim.x + threadIdx.x;                                          \
        uint4 x = data[i];                                                                      \
        uint64_t a0 = x.x, a1 = x.y, a2 = x.z, a3 = x.w;                                        \
        uint32_t b0 = x.x ^ 1, b1 = x.y ^ 2, b2 = x.z ^ 3, b3 = x.w ^ 4;                        \
        uint32_t m = x.x | 1;                                                                   \
        for (int k = 0; k < iters; k++) {                                                       \
            _Pragma("unroll") for (int u = 0; u < 8; u++) {                                     \
                asm volatile(I64 : "+v"(a0) : "v"(m)); asm volatile(I32 : "+v"(b0) : "v"(m));   \
                asm volatile(I64 : "+v"(a1) : "v"(m)); asm volatile(I32 : "+v"(b1) : "v"(m));   \
                asm volatile(I64 : "+v"(a2) : "v"(m)); asm volatile(I32 : "+v"(b2) : "v"(m));   \
                asm volatile(I64 : "+v"(a3) : "v"(m)); asm volatile(I32 : "+v"(b3) : "v"(m));   \
            }                                                                                   \
        }                                                                                       \
        data[i] = make_uint4((uint32_t)(a0 ^ a1), (uint32_t)(a2 ^ a3), b0 ^ b1, b2 ^ b3);      \
    }
MIX(k_mix_mad_and, "v_mad_u64_u32 %0, vcc, %1, %1, %0", "v_and_b32_e32 %0, 0x1fffffff, %0")
MIX(k_mix_mad_ashr, "v_mad_i64_i32 %0, vcc, %1, %1, %0", "v_ashrrev_i32_e32 %0, 29, %0")
MIX(k_mix_mad_shr64, "v_mad_i64_i32 %0, vcc, %1, %1, %0", "v_add_u32_e32 %0, %0, %1")
KERNEL(k_mix_add3_add, uint32_t, "v_add3_u32 %0, %0, %1, %0\n v_add_u32_e32 %0, %0, %1")

template <typename K>
static float timeit(K kern, uint4* d, int blocks, int threads, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, iters);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const int threads = 256, blocks = 256 * 8;  // 8 waves per SIMD
    const size_t n = (size_t)threads * blocks;
    uint4* d;
    CHECK(hipMalloc(&d, n * sizeof(uint4)));
    std::vector<uint32_t> h(n * 4);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u + 12345);
    CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const int iters = 512;
    struct R { const char* name; void (*k)(uint4*, int); int per_step; };
    R rs[] = {{"v_mad_u64_u32", k_mad_u64, 1},     {"v_mad_i64_i32", k_mad_i64, 1},   {"v_ashrrev_i64", k_ashr64, 1},
              {"v_lshl_add_u64", k_lshladd64, 1},  {"v_add3_u32", k_add3, 1},         {"v_alignbit_b32", k_alignbit, 1},
              {"v_and_b32_e32 lit", k_and_lit, 1}, {"v_and_b32_e32", k_and, 1},        {"v_add_u32_e32", k_add, 1},
              {"v_sub_u32_e32", k_sub, 1},         {"v_ashrrev_i32_e32", k_ashr32, 1}, {"v_mov_b32_e32", k_mov, 1},
              {"v_cndmask_b32_e32", k_cndmask, 1}, {"mix mad_u64 + and lit", k_mix_mad_and, 1},
              {"mix mad_i64 + ashr_i32", k_mix_mad_ashr, 1},
              {"mix mad_i64 + add_u32", k_mix_mad_shr64, 1}, {"mix add3 + add_u32", k_mix_add3_add, 2}};
    // (mixes: 64 instructions per iteration of 4 + 4 chains x 8 = per_step 1, i.e. counted once each)
    printf("# class  ms  lane-instr/s  wave-instr per CU per clk at 2.4 GHz  SIMD cycles per wave-instr\n");
    for (auto& r : rs) {
        float ms = timeit(r.k, d, blocks, threads, iters);
        const double li = (double)n * iters * 64 * r.per_step;  // lane-instructions
        const double rate = li / (ms * 1e-3);
        printf("%-26s %.3f ms %.3e lane-instr/s %.2f wave/clk/CU %.2f cyc/SIMD\n", r.name, ms, rate,
               rate / 64 / 256 / 2.4e9, 4.0 / (rate / 64 / 256 / 2.4e9));
    }
    return 0;
}
