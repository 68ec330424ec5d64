// sqrt_probe.hip — diagnostic (not part of the product): checks qpk::sqrt_1to2 against the
// compiler's sqrt() bit for bit on the GPU, for every x in [1, 2) on a stride of binary64
// patterns (plus both ends and random mantissas), and qp_distance (sqrt_1to2) against qp_distance_libm (sqrt()) on
// random operand pairs including zeros, equal magnitudes, infinities, NaN and denormals.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/sqrt_probe tools/sqrt_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../motion-generation-using-quadratic-programs_amd/csrc/qp_common.h"

__global__ void sqrt_kernel(unsigned long long* bad, unsigned long long n, unsigned long long stride) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // binary64 patterns of [1, 2): exponent 0x3ff, 52-bit mantissa; pattern i * stride + i % 977
  const unsigned long long mant = (i * stride + (i % 977)) & ((1ull << 52) - 1);
  double x = __builtin_bit_cast(double, (0x3ffull << 52) | mant);
  if (i == n - 1) x = 2.0;
  const double a = sqrt(x), b = qpk::sqrt_1to2(x);
  if (__builtin_bit_cast(unsigned long long, a) != __builtin_bit_cast(unsigned long long, b))
    atomicAdd(bad, 1ull);
}

__device__ double pick(unsigned long long h) {
  const unsigned k = h % 16;
  const double m = (double)((h >> 8) & 0xfffff) / 1048576.0 + 0.5;
  switch (k) {
    case 0: return 0.0;
    case 1: return -0.0;
    case 2: return __builtin_inf();
    case 3: return __builtin_nan("");
    case 4: return 4.9e-324 * (double)((h >> 20) & 0xff);
    case 5: return m * 1e300;
    case 6: return -m * 1e-300;
    default: return ((h >> 40) & 1 ? -m : m) * __builtin_ldexp(1.0, (int)((h >> 41) & 0x3f) - 32);
  }
}

__global__ void dist_kernel(unsigned long long* bad, unsigned long long n) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long h1 = i * 0x9e3779b97f4a7c15ull, h2 = (i + 7) * 0xc2b2ae3d27d4eb4full;
  h1 ^= h1 >> 29;
  h2 ^= h2 >> 31;
  const double a = pick(h1);
  const double b = (i % 5 == 0) ? -a : pick(h2);
  const double r1 = qpk::qp_distance_libm(a, b), r2 = qpk::qp_distance(a, b);
  const bool n1 = r1 != r1, n2 = r2 != r2;
  if (n1 != n2 || (!n1 && __builtin_bit_cast(unsigned long long, r1) != __builtin_bit_cast(unsigned long long, r2)))
    atomicAdd(bad, 1ull);
}

int main() {
  unsigned long long* bad;
  hipMalloc(&bad, 16);
  hipMemset(bad, 0, 16);
  const unsigned long long n = 1ull << 30, stride = ((1ull << 52) / n) | 1;
  hipLaunchKernelGGL(sqrt_kernel, dim3((unsigned)(n / 256)), dim3(256), 0, 0, bad, n, stride);
  const unsigned long long nd = 1ull << 28;
  hipLaunchKernelGGL(dist_kernel, dim3((unsigned)(nd / 256)), dim3(256), 0, 0, bad + 1, nd);
  unsigned long long h[2];
  hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
  printf("sqrt_1to2 vs sqrt: %llu mismatches of %llu\n", h[0], n);
  printf("qp_distance vs qp_distance_libm: %llu mismatches of %llu\n", h[1], nd);
  return (h[0] || h[1]) ? 1 : 0;
}
