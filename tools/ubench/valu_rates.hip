// VALU issue-cost probe for the CGR step's instruction mix on gfx950:
// each kernel runs 8 independent chains of one instruction, kIters times,
// on every CU; cycles per wave-instruction per SIMD = elapsed cycles * SIMDs
// / (waves * instructions).  hipcc --offload-arch=gfx950 -O3 valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

#define CHAIN8(INSN)                                                            \
  for (int i = 0; i < kIters; ++i) {                                            \
    asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c));                              \
    asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));                              \
  }

__global__ void k_fma_f64(double *out, double b, double c) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  CHAIN8("v_fma_f64 %0, %0, %1, %2")
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ void k_fma_f32(double *out, float b, float c) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  CHAIN8("v_fma_f32 %0, %0, %1, %2")
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ void k_and_b32(double *out, unsigned b, unsigned c) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  CHAIN8("v_and_or_b32 %0, %0, %1, %2")
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ void k_bfe(double *out, unsigned b, unsigned c) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  CHAIN8("v_bfe_u32 %0, %0, %1, %2")
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// cvt_i32_f64: chain through an int->double round trip is 2 insns; use a
// separate destination and feed back via the b operand dependency-free
__global__ void k_cvt_i32_f64(double *out, double b, double c) {
  int r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
  double x = b + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r0) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r1) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r2) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r3) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r4) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r5) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r6) : "v"(x));
    asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(r7) : "v"(x));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}
// dependent f64 fma chain (latency): one chain
__global__ void k_fma_f64_dep(double *out, double b, double c) {
  double a0 = threadIdx.x;
  for (int i = 0; i < kIters * 8; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
// LDS 64-bit atomics at random cells of a 16K-cell table
__global__ void k_ds_add_u64(double *out, double b, double c) {
  extern __shared__ unsigned long long t[];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) t[i] = 0;
  __syncthreads();
  uint32_t h = threadIdx.x * 2654435761u + blockIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      h = h * 1664525u + 1013904223u;
      atomicAdd(&t[h >> 18], 1ull);
    }
  }
  __syncthreads();
  out[blockIdx.x * blockDim.x + threadIdx.x] = (double)t[threadIdx.x];
}

template <typename F>
void run(const char *name, F kfn, int waves_per_simd, size_t lds, double *out, int vinsn_per_iter) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
  const int threads = 256 * waves_per_simd;   // 4 SIMDs
  if (lds) hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kfn, dim3(cus), dim3(threads), lds, 0, out, 1.0000001, 0.5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double cycles = ms * 1e-3 * clk * 1e3;
  const double insn = (double)kIters * vinsn_per_iter * waves_per_simd;   // per SIMD
  printf("%-16s waves/SIMD %d  %.3f ms  %.2f cycles per wave-insn per SIMD (clock %d MHz)\n", name,
         waves_per_simd, ms, cycles / insn, clk / 1000);
}

int main() {
  double *out;
  hipMalloc(&out, 256 * 1024 * 8 * 4);
  for (int w : {1, 4}) {
    run("fma_f64", k_fma_f64, w, 0, out, 8);
    run("fma_f32", k_fma_f32, w, 0, out, 8);
    run("and_or_b32", k_and_b32, w, 0, out, 8);
    run("bfe_u32", k_bfe, w, 0, out, 8);
    run("cvt_i32_f64", k_cvt_i32_f64, w, 0, out, 8);
    run("fma_f64 dep", k_fma_f64_dep, w, 0, out, 8);
    run("ds_add_u64", k_ds_add_u64, w, 16384 * 8, out, 8);
  }
  hipFree(out);
  return 0;
}
