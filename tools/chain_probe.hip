// chain_probe.hip — diagnostic microbenchmark (not part of the product): s_memtime cycles per
// link of a dependent f64 chain, one wave per SIMD, for the operations that make up the solver's
// serial chains: add, IEEE division, sqrt, and the reference's distance() (qp_common.h).  Also
// an LDS store -> load round trip (the lead-lane hand-off).  Tells how far a serial chain in the
// kernels is from its latency floor.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../motion-generation-using-quadratic-programs_amd/csrc/qp_common.h"

enum { OP_ADD, OP_DIV, OP_SQRT, OP_DIST, OP_LDS, OP_DIST2 };

template <int OP>
__global__ void __launch_bounds__(64) chain_kernel(double* out, long long* cyc, int iters, double a) {
  __shared__ double buf[64];
  double x = 1.0 + threadIdx.x * 1e-3, y = 0.75 + threadIdx.x * 1e-4;
  buf[threadIdx.x] = x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      if constexpr (OP == OP_ADD) x = x + a;
      if constexpr (OP == OP_DIV) x = a / x;
      if constexpr (OP == OP_SQRT) x = sqrt(x) + a;
      if constexpr (OP == OP_DIST) x = qpk::qp_distance(a, x) * 0.5;
      if constexpr (OP == OP_DIST2) {  // two independent chains interleaved
        x = qpk::qp_distance(a, x) * 0.5;
        y = qpk::qp_distance(a, y) * 0.5;
      }
      if constexpr (OP == OP_LDS) {
        buf[(threadIdx.x + 1) & 63] = x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        x = buf[threadIdx.x] + a;
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x + y;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int waves, double* out, long long* cyc, double a) {
  const int iters = 500;
  hipLaunchKernelGGL(chain_kernel<OP>, dim3(waves), dim3(64), 0, 0, out, cyc, iters, a);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(chain_kernel<OP>, dim3(waves), dim3(64), 0, 0, out, cyc, iters, a);
  hipDeviceSynchronize();
  static long long h[8192];
  hipMemcpy(h, cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < waves; i++) mean += h[i];
  mean /= waves;
  printf("%-26s waves %5d (%.0f/SIMD): %7.1f cycles per chain link\n", name, waves, waves / 1024.0,
         mean / (iters * 8.0));
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 8192 * 64 * 8);
  hipMalloc(&cyc, 8192 * 8);
  for (int w : {1024, 2048}) {
    run<OP_ADD>("add", w, out, cyc, 1e-9);
    run<OP_DIV>("div", w, out, cyc, 1.0000001);
    run<OP_SQRT>("sqrt + add", w, out, cyc, 0.5);
    run<OP_DIST>("distance * 0.5", w, out, cyc, 0.3);
    run<OP_DIST2>("2 x distance (interleaved)", w, out, cyc, 0.3);
    run<OP_LDS>("LDS store->load + add", w, out, cyc, 1e-9);
  }
  return 0;
}
