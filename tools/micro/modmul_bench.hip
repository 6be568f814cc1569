// Microbenchmark: modular-multiplication throughput variants on gfx950 (design exploration).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while(0)

// ---- V1: 32-bit CIOS (compiler)
namespace v1 {
#define P1 0x992d30edu
#define P2 0x094cf91bu
#define P3 0x224698fcu
#define P7 0x40000000u
__device__ __forceinline__ void mont_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[10];
#pragma unroll
  for (int j=0;j<10;j++) t[j]=0;
#pragma unroll
  for (int i=0;i<8;i++) {
    uint64_t acc = 0;
#pragma unroll
    for (int j=0;j<8;j++) { acc = (uint64_t)a[j]*b[i] + (uint64_t)t[j] + (acc>>32); t[j]=(uint32_t)acc; }
    acc = (uint64_t)t[8] + (acc>>32); t[8]=(uint32_t)acc; t[9]=(uint32_t)(acc>>32);
    uint32_t m = 0u - t[0];
    acc = (uint64_t)m + t[0];
    acc = (uint64_t)m*P1 + t[1] + (acc>>32); t[0]=(uint32_t)acc;
    acc = (uint64_t)m*P2 + t[2] + (acc>>32); t[1]=(uint32_t)acc;
    acc = (uint64_t)m*P3 + t[3] + (acc>>32); t[2]=(uint32_t)acc;
    acc = (uint64_t)t[4] + (acc>>32); t[3]=(uint32_t)acc;
    acc = (uint64_t)t[5] + (acc>>32); t[4]=(uint32_t)acc;
    acc = (uint64_t)t[6] + (acc>>32); t[5]=(uint32_t)acc;
    acc = (uint64_t)m*P7 + t[7] + (acc>>32); t[6]=(uint32_t)acc;
    acc = (uint64_t)t[8] + (acc>>32); t[7]=(uint32_t)acc;
    t[8] = t[9] + (uint32_t)(acc>>32);
  }
  uint32_t s[8]; uint32_t borrow=0;
  const uint32_t pp[8]={1u,P1,P2,P3,0,0,0,P7};
#pragma unroll
  for (int j=0;j<8;j++){ uint64_t d=(uint64_t)t[j]-pp[j]-borrow; s[j]=(uint32_t)d; borrow=(uint32_t)(d>>32)&1; }
  bool ge = t[8] || !borrow;
#pragma unroll
  for (int j=0;j<8;j++) r[j]= ge? s[j]:t[j];
}
__global__ void bench(uint4* data, int iters) {
  int i = blockIdx.x*blockDim.x+threadIdx.x;
  uint32_t a[8], b[8];
  uint4 x=data[3*i], y=data[3*i+1];
  a[0]=x.x;a[1]=x.y;a[2]=x.z;a[3]=x.w;a[4]=y.x;a[5]=y.y;a[6]=y.z;a[7]=y.w; a[7]&=0x3fffffff;
  for(int j=0;j<8;j++) b[j]=a[j]^0x12345;
  for (int k=0;k<iters;k++){ uint32_t c[8]; mont_mul(c,a,b); for(int j=0;j<8;j++){b[j]=a[j];a[j]=c[j];} }
  data[3*i]=make_uint4(a[0],a[1],a[2],a[3]); data[3*i+1]=make_uint4(a[4],a[5],a[6],a[7]);
}
}

// ---- V2: 29-bit radix FIPS (compiler)
namespace v2 {
constexpr int NL=9; constexpr int W=29; constexpr uint32_t MASK=(1u<<W)-1;
constexpr uint32_t PL[9]={0x1,0x9698768,0x133e46e6,0xd31f812,0x224,0,0,0,0x400000};
__device__ __forceinline__ void mont_mul(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k=0;k<2*NL-1;k++) {
#pragma unroll
    for (int i=0;i<NL;i++) { int j=k-i; if (j<0||j>=NL) continue; acc += (uint64_t)a[i]*b[j]; }
#pragma unroll
    for (int i=0;i<NL;i++) { int j=k-i; if (i>=k || i>=NL || j<1 || j>=NL || PL[j]==0) continue; acc += (uint64_t)m[i]*PL[j]; }
    if (k<NL) { uint32_t mk = (0u - (uint32_t)acc) & MASK; m[k]=mk; acc += mk; acc >>= W; }
    else { r[k-NL] = (uint32_t)acc & MASK; acc >>= W; }
  }
  r[NL-1]=(uint32_t)acc;
}
__global__ void bench(uint4* data, int iters) {
  int i = blockIdx.x*blockDim.x+threadIdx.x;
  uint32_t a[9], b[9];
  uint4 x=data[3*i], y=data[3*i+1], z=data[3*i+2];
  a[0]=x.x;a[1]=x.y;a[2]=x.z;a[3]=x.w;a[4]=y.x;a[5]=y.y;a[6]=y.z;a[7]=y.w;a[8]=z.x;
  for(int j=0;j<9;j++) {a[j]&=MASK; b[j]=a[j]^0x12345;}
  a[8]&=0x3fffff; b[8]&=0x3fffff;
  for (int k=0;k<iters;k++){ uint32_t c[9]; mont_mul(c,a,b); for(int j=0;j<9;j++){b[j]=a[j];a[j]=c[j];} }
  data[3*i]=make_uint4(a[0],a[1],a[2],a[3]); data[3*i+1]=make_uint4(a[4],a[5],a[6],a[7]); data[3*i+2]=make_uint4(a[8],0,0,0);
}
}

// ---- raw instruction throughput (inline asm, 8 independent chains, 8 instrs per block)
#define RAW_KERNEL(NAME, INSTR) \
__global__ void NAME(uint4* data, int iters) { \
  int i = blockIdx.x*blockDim.x+threadIdx.x; \
  uint4 x = data[3*i]; \
  uint64_t a0=x.x, a1=x.y, a2=x.z, a3=x.w, a4=x.x^1, a5=x.y^2, a6=x.z^3, a7=x.w^4; \
  uint32_t m = x.x | 1; \
  for (int k=0;k<iters;k++) { \
    _Pragma("unroll") for (int u=0;u<8;u++) { \
      asm volatile(INSTR : "+v"(a0) : "v"(m)); asm volatile(INSTR : "+v"(a1) : "v"(m)); \
      asm volatile(INSTR : "+v"(a2) : "v"(m)); asm volatile(INSTR : "+v"(a3) : "v"(m)); \
      asm volatile(INSTR : "+v"(a4) : "v"(m)); asm volatile(INSTR : "+v"(a5) : "v"(m)); \
      asm volatile(INSTR : "+v"(a6) : "v"(m)); asm volatile(INSTR : "+v"(a7) : "v"(m)); \
    } \
  } \
  data[3*i] = make_uint4((uint32_t)(a0^a1^a2^a3), (uint32_t)((a4^a5^a6^a7)>>32), (uint32_t)(a0>>32), (uint32_t)a7); \
}
#define RAW32(NAME, INSTR) \
__global__ void NAME(uint4* data, int iters) { \
  int i = blockIdx.x*blockDim.x+threadIdx.x; \
  uint4 x = data[3*i]; \
  uint32_t a0=x.x, a1=x.y, a2=x.z, a3=x.w, a4=x.x^1, a5=x.y^2, a6=x.z^3, a7=x.w^4; \
  uint32_t m = x.x | 1; \
  for (int k=0;k<iters;k++) { \
    _Pragma("unroll") for (int u=0;u<8;u++) { \
      asm volatile(INSTR : "+v"(a0) : "v"(m)); asm volatile(INSTR : "+v"(a1) : "v"(m)); \
      asm volatile(INSTR : "+v"(a2) : "v"(m)); asm volatile(INSTR : "+v"(a3) : "v"(m)); \
      asm volatile(INSTR : "+v"(a4) : "v"(m)); asm volatile(INSTR : "+v"(a5) : "v"(m)); \
      asm volatile(INSTR : "+v"(a6) : "v"(m)); asm volatile(INSTR : "+v"(a7) : "v"(m)); \
    } \
  } \
  data[3*i] = make_uint4((uint32_t)(a0^a1^a2^a3), (uint32_t)((a4^a5^a6^a7)>>32), (uint32_t)(a0>>32), (uint32_t)a7); \
}
RAW_KERNEL(raw_mad, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
RAW_KERNEL(raw_add64, "v_lshl_add_u64 %0, %0, 0, %0")
RAW32(raw_add32, "v_add_co_u32 %0, vcc, %0, %1")
RAW32(raw_mullo, "v_mul_lo_u32 %0, %0, %1")
RAW32(raw_mulhi, "v_mul_hi_u32 %0, %0, %1")
RAW_KERNEL(raw_shr64, "v_lshrrev_b64 %0, 29, %0")
RAW32(raw_addu32, "v_add_u32 %0, %0, %1")
RAW32(raw_add3, "v_add3_u32 %0, %0, %1, %0")
RAW32(raw_and, "v_and_b32 %0, %0, %1")
RAW32(raw_fma, "v_fma_f32 %0, %0, %1, %0")
RAW32(raw_addc, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
RAW32(raw_mad24, "v_mad_u32_u24 %0, %0, %1, %0")
RAW32(raw_bfe, "v_bfe_u32 %0, %0, 3, 29")
RAW32(raw_alignbit, "v_alignbit_b32 %0, %0, %1, 29")

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

int main() {
  const int threads = 256, blocks = 256 * 16;
  size_t n = (size_t)threads * blocks;
  uint4* d; CHECK(hipMalloc(&d, n * 3 * sizeof(uint4)));
  std::vector<uint32_t> h(n * 12);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u + 12345);
  CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  int iters = 256;
  double ms;
  ms = timeit(v1::bench, d, blocks, threads, iters);
  printf("v1 32-bit CIOS : %.3f ms  %.3e modmul/s\n", ms, n * (double)iters / (ms * 1e-3));
  ms = timeit(v2::bench, d, blocks, threads, iters);
  printf("v2 29-bit FIPS : %.3f ms  %.3e modmul/s\n", ms, n * (double)iters / (ms * 1e-3));
  {
    // latency: one wave per SIMD (1024 waves of 64 lanes), dependent chain
    int it2 = 64;
    for (int wpc : {1, 2, 4, 8}) {
      double t = timeit(v2::bench, d, 256 * wpc, 256, it2);
      printf("v2 latency-bound %d wave/SIMD: %.3f ms -> %.0f ns per dependent modmul\n", wpc, t, t * 1e6 / it2);
    }
  }
  auto rawrep=[&](const char* nm, void(*k)(uint4*,int)){ double t=timeit(k,d,blocks,threads,iters); double ips=n*(double)iters*64/(t*1e-3); printf("%-12s %.3f ms %.3e inst/s = %.1f wave-inst/clk/CU @2.4GHz\n", nm, t, ips, ips/64/256/2.4e9);};
  rawrep("mad_u64_u32", raw_mad); rawrep("lshl_add_u64", raw_add64); rawrep("add_co_u32", raw_add32); rawrep("mul_lo_u32", raw_mullo); rawrep("mul_hi_u32", raw_mulhi); rawrep("lshrrev_b64", raw_shr64);
  rawrep("add_u32", raw_addu32); rawrep("add3_u32", raw_add3); rawrep("and_b32", raw_and); rawrep("fma_f32", raw_fma);
  rawrep("addc_co_u32", raw_addc); rawrep("mad_u32_u24", raw_mad24); rawrep("bfe_u32", raw_bfe); rawrep("alignbit", raw_alignbit);
  return 0;
  ms = timeit(raw_mad, d, blocks, threads, iters);
  printf("raw v_mad_u64_u32 : %.3f ms  %.3e inst/s (%.2f per CU per clk @2.4GHz)\n", ms, n * (double)iters * 64 / (ms * 1e-3), n*(double)iters*64/(ms*1e-3)/256/2.4e9);
  ms = timeit(raw_add64, d, blocks, threads, iters);
  printf("raw add64 : %.3f ms  %.3e inst/s (%.2f per CU per clk)\n", ms, n * (double)iters * 64 / (ms * 1e-3), n*(double)iters*64/(ms*1e-3)/256/2.4e9);
  ms = timeit(raw_add32, d, blocks, threads, iters);
  printf("raw add32+xor : %.3f ms  %.3e inst/s (%.2f per CU per clk)\n", ms, n * (double)iters * 128 / (ms * 1e-3), n*(double)iters*128/(ms*1e-3)/256/2.4e9);
  return 0;
}
