// f64_issue_probe.hip — diagnostic microbenchmark (not part of the product): cycles per
// v_fma_f64 / v_mul_f64 wave-instruction for ONE wave per SIMD vs TWO, independent chains
// (throughput) and one dependent chain (latency).  Decides whether the lane kernel is
// issue-bound at one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o f64_issue_probe tools/f64_issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int CHAINS>
__global__ void __launch_bounds__(64) fma_kernel(double* out, long long* cyc, int iters, double a) {
  double acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = threadIdx.x + c;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_fma(acc[c], a, 1.0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += acc[c];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
void run(int waves, double* out, long long* cyc) {
  const int iters = 2000;
  hipLaunchKernelGGL(fma_kernel<CHAINS>, dim3(waves), dim3(64), 0, 0, out, cyc, iters, 0.999);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(fma_kernel<CHAINS>, dim3(waves), dim3(64), 0, 0, out, cyc, iters, 0.999);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[8192];
  hipMemcpy(h, cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < waves; i++) mean += h[i];
  mean /= waves;
  const double instr = (double)iters * 16 * CHAINS;
  printf("chains %2d waves %5d (%.1f/SIMD): %.2f memtime-cycles per wave-instr, kernel %.3f ms -> %.2f ns per instr per wave\n",
         CHAINS, waves, waves / 1024.0, mean / instr, ms, ms * 1e6 / instr);
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 8192 * 64 * 8);
  hipMalloc(&cyc, 8192 * 8);
  for (int w : {1024, 2048, 4096}) {
    run<1>(w, out, cyc);
    run<8>(w, out, cyc);
  }
  return 0;
}
