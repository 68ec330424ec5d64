// Dependent-chain latency and independent-stream issue cost of the binary64 operations the
// lane kernel is built from (one wave per SIMD, s_memtime cycles), to price its critical paths.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/f64_latency.hip -o tools/f64_latency
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 256;

template <int OP>
__device__ __forceinline__ double step(double x, double y) {
  if constexpr (OP == 0) return x * y;
  if constexpr (OP == 1) return x + y;
  if constexpr (OP == 2) return __builtin_fma(x, y, 0.5);
  if constexpr (OP == 3) return y / x;
  if constexpr (OP == 4) return __builtin_sqrt(x) + y;
  return x;
}

// DEP: one chain of kN dependent ops; else 8 independent chains of kN/8 ops
template <int OP, bool DEP>
__global__ __launch_bounds__(64, 1) void probe(const double* in, double* out, long long* cyc) {
  double y = in[threadIdx.x];
  double x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = in[64 + threadIdx.x] + k;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  // opaque register dependences pin the chain between the two stamps
#pragma unroll
  for (int k = 0; k < 8; k++) asm volatile("" : "+v"(x[k]));
  asm volatile("" : "+v"(y));
  if constexpr (DEP) {
#pragma unroll
    for (int i = 0; i < kN; i++) x[0] = step<OP>(x[0], y);
  } else {
#pragma unroll
    for (int i = 0; i < kN / 8; i++)
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = step<OP>(x[k], y);
  }
  __builtin_amdgcn_s_waitcnt(0);
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s += x[k];
  asm volatile("s_nop 0" : "+v"(s));
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, bool DEP>
double run(const char* name, const double* din, double* dout, long long* dcyc) {
  probe<OP, DEP><<<1, 64>>>(din, dout, dcyc);  // warm
  probe<OP, DEP><<<1, 64>>>(din, dout, dcyc);
  long long c = 0;
  hipMemcpy(&c, dcyc, sizeof(c), hipMemcpyDeviceToHost);
  const double per = (double)c / kN;
  printf("%-6s %-5s %7.2f cycles per op (%lld for %d)\n", name, DEP ? "dep" : "indep", per, c, kN);
  return per;
}

int main() {
  double h[128];
  for (int i = 0; i < 128; i++) h[i] = 1.0 + 1e-3 * i;
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&dout, 64 * sizeof(double));
  hipMalloc(&dcyc, sizeof(long long));
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  run<0, true>("mul", din, dout, dcyc);
  run<0, false>("mul", din, dout, dcyc);
  run<1, true>("add", din, dout, dcyc);
  run<1, false>("add", din, dout, dcyc);
  run<2, true>("fma", din, dout, dcyc);
  run<2, false>("fma", din, dout, dcyc);
  run<3, true>("div", din, dout, dcyc);
  run<3, false>("div", din, dout, dcyc);
  run<4, true>("sqrt", din, dout, dcyc);
  run<4, false>("sqrt", din, dout, dcyc);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
