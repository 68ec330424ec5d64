// launch_probe.hip — per-launch overhead of a qp_lane-shaped grid (diagnostic, not product code).
//
// 1 024 workgroups of one wave (one per SIMD) or 256 of four, 40 KiB of LDS per wave and the lane kernel's register
// budget (launch_bounds(64, 1)); every wave spins on the 100 MHz constant clock for D us, then
// writes 64 B per lane (the lane kernel's x / f / status stores).  20 launches back to back on
// one stream between one event pair: (time / 20) - D is what a launch costs beyond its waves.
//   usage: ./launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES, 1) spin_kernel(double* out, int ticks, int lds_touch) {
  __shared__ double sbuf[5120 * WAVES];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (lds_touch) sbuf[threadIdx.x] = (double)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(2);
  const size_t i = (size_t)blockIdx.x * 64 * WAVES + threadIdx.x;
  double v = lds_touch ? sbuf[threadIdx.x ^ 1] : 1.0;
#pragma unroll
  for (int k = 0; k < 8; k++) out[i * 8 + k] = v + k;
}

int main() {
  const int blocks = 1024, reps = 20;
  double* out;
  CK(hipMalloc(&out, (size_t)blocks * 64 * 8 * sizeof(double)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int durs_us[] = {0, 5, 20, 35};
  for (int wv : {1, 4})
  for (int lds = 0; lds < 2; lds++)
    for (int d : durs_us) {
      const int ticks = d * 100;  // 100 MHz
      auto launch = [&]() {
        if (wv == 1)
          hipLaunchKernelGGL(spin_kernel<1>, dim3(blocks), dim3(64), 0, 0, out, ticks, lds);
        else
          hipLaunchKernelGGL(spin_kernel<4>, dim3(blocks / 4), dim3(256), 0, 0, out, ticks, lds);
      };
      for (int w = 0; w < 3; w++) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; r++) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms * 1000.0 / reps;
      printf("waves/WG %d lds_touch %d spin %2d us: %.2f us per launch, overhead %.2f us\n", wv, lds, d, per, per - d);
    }
  return 0;
}
