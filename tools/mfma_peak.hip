// Microbenchmark: sustained v_mfma_f32_32x32x2_f32 rate with every SIMD busy
// (4 independent accumulators per wave, one wave per SIMD), and the clock the
// chip holds meanwhile (s_memtime / s_memrealtime at 100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x16 = __attribute__((ext_vector_type(16))) float;

__global__ __launch_bounds__(256) void mfma_loop(float* out, unsigned long long* clk, int iters) {
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f + blockIdx.x * 1e-4f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
  int nblk = 256 * 2, iters = 20000;
  float* out; unsigned long long* clk;
  hipMalloc(&out, nblk * 256 * 4); hipMalloc(&clk, nblk * 16);
  hipLaunchKernelGGL(mfma_loop, dim3(nblk), dim3(256), 0, 0, out, clk, 100);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop, dim3(nblk), dim3(256), 0, 0, out, clk, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  double flops = (double)nblk * 4 /*waves*/ * iters * 4 * 32 * 32 * 2 * 2;
  printf("mfma_f32_32x32x2: %.1f TFLOP/s over %.3f ms; block0 clock %.3f GHz (%llu cycles / %llu ticks@100MHz)\n",
         flops / ms / 1e9, ms, (double)h[0] / (double)h[1] * 0.1, h[0], h[1]);
  return 0;
}
