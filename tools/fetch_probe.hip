// fetch_probe.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns the qp_lane kernel uses (MI355X_MICROARCH.md §HBM: only 16-B coalesced streaming reads
// are calibrated there; "calibrate on a known byte count in your own access pattern").
//
// Every probe kernel moves a known number of bytes exactly once from (or to) a buffer far larger
// than the 256 MiB Infinity Cache, so each byte is an HBM transfer.  Run it under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_probe      (and a separate pass with WRITE_SIZE)
// and divide the counter (KiB) by the bytes printed for each kernel.
//   coalesced_x4   lane t reads 16 B at base + 16 t (+1 KiB per step): the guide's calibrated case
//   coalesced_lds  the same bytes by global_load_lds_dwordx4 (G / CE staging)
//   coalesced_x2   lane t reads 8 B at base + 8 t (+512 B per step): qp_wave's CI rows (lane =
//                  constraint) and the workspace variant's column-major J
//   lane_x4        lane t reads its own 1792-B QP record with dwordx4 (per-lane blocks, stride 1792)
//   lane_x2        the same records with 8-B loads (dwordx2)
//   lane_lds       the same records by per-lane global_load_lds_dwordx4 (the CI-row copy)
//   lane_touch4    lane t loads ONE dword per 128-B line of its record (the lane kernel's CI /
//                  ci0 warm-up): the lines move, 4 B per line reach a register
//   store_lane_x2  lane t writes its own 56-B x record with 8-B stores (x, stride 56)
//   store_x2       lane t writes 8 B at base + 8 t (f)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(e)                                                                   \
  do {                                                                             \
    hipError_t err_ = (e);                                                         \
    if (err_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int kRec = 1792;  // bytes per QP record (C1's algorithmic bytes per QP)

__global__ void __launch_bounds__(64) coalesced_x4(const double2* __restrict__ src, int64_t n16, double* out) {
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 64) {
    const double2 v = src[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;  // keeps the loads; never true for the zero-filled buffer
}

__global__ void __launch_bounds__(64) coalesced_x2(const double* __restrict__ src, int64_t n8, double* out) {
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 64) acc += src[i];
  if (acc == 12345.678) out[0] = acc;
}

__global__ void __launch_bounds__(64) coalesced_lds(const double* __restrict__ src, int64_t n16, double* out) {
  __shared__ double buf[2048];
  for (int64_t c = (int64_t)blockIdx.x * 64 * 8; c < n16; c += (int64_t)gridDim.x * 64 * 8) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int64_t e = (c + k * 64 + threadIdx.x) * 2;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + (e < n16 * 2 ? e : 0)),
                                       (__attribute__((address_space(3))) void*)(buf + k * 128), 16, 0, 0);
    }
    __syncthreads();
    if (buf[threadIdx.x] == 12345.678) out[0] = buf[threadIdx.x];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(64) lane_x4(const char* __restrict__ src, int64_t nrec, double* out) {
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= nrec) return;
  const double2* p = reinterpret_cast<const double2*>(src + r * kRec);
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < kRec / 16; k++) {
    const double2 v = p[k];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;
}

__global__ void __launch_bounds__(64) lane_x2(const char* __restrict__ src, int64_t nrec, double* out) {
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= nrec) return;
  const double* p = reinterpret_cast<const double*>(src + r * kRec);
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < kRec / 8; k++) acc += p[k];
  if (acc == 12345.678) out[0] = acc;
}

__global__ void __launch_bounds__(64) lane_lds(const char* __restrict__ src, int64_t nrec, double* out) {
  __shared__ double buf[kRec / 8 * 64];  // 112 KiB
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const double* p = reinterpret_cast<const double*>(src + (r < nrec ? r : 0) * kRec);
#pragma unroll 8
  for (int k = 0; k < kRec / 16; k++)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + 2 * k),
                                     (__attribute__((address_space(3))) void*)(buf + k * 128), 16, 0, 0);
  __syncthreads();
  if (buf[threadIdx.x * 2] == 12345.678) out[0] = buf[threadIdx.x];
}

__global__ void __launch_bounds__(64) lane_touch4(const char* __restrict__ src, int64_t nrec, double* out) {
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= nrec) return;
  const char* p = src + r * kRec;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kRec / 128; k++) acc += *reinterpret_cast<const uint32_t*>(p + k * 128);
  if (acc == 12345u) out[0] = acc;
}

__global__ void __launch_bounds__(64) store_lane_x2(double* __restrict__ dst, int64_t nrec) {
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= nrec) return;
#pragma unroll
  for (int k = 0; k < 7; k++) dst[r * 7 + k] = (double)k;
}

__global__ void __launch_bounds__(64) store_x2(double* __restrict__ dst, int64_t n) {
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r < n) dst[r] = 1.0;
}

int main() {
  const int64_t nrec = 1 << 18;                  // 262 144 records
  const int64_t bytes = nrec * kRec;             // 448 MiB: beyond the Infinity Cache
  char *a = nullptr, *b = nullptr;
  double* out = nullptr;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipMemset(b, 0, bytes));
  CHECK(hipDeviceSynchronize());
  const unsigned blocks = (unsigned)(nrec / 64);
  // consecutive kernels alternate between the two 448-MiB buffers, so no kernel finds the
  // previous one's bytes in the Infinity Cache
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(coalesced_x4, dim3(4096), dim3(64), 0, 0, (const double2*)a, bytes / 16, out);
    hipLaunchKernelGGL(coalesced_lds, dim3(4096), dim3(64), 0, 0, (const double*)b, bytes / 16, out);
    hipLaunchKernelGGL(coalesced_x2, dim3(4096), dim3(64), 0, 0, (const double*)a, bytes / 8, out);
    hipLaunchKernelGGL(lane_x4, dim3(blocks), dim3(64), 0, 0, b, nrec, out);
    hipLaunchKernelGGL(lane_x2, dim3(blocks), dim3(64), 0, 0, a, nrec, out);
    hipLaunchKernelGGL(lane_lds, dim3(blocks), dim3(64), 0, 0, b, nrec, out);
    hipLaunchKernelGGL(lane_touch4, dim3(blocks), dim3(64), 0, 0, a, nrec, out);
    hipLaunchKernelGGL(store_lane_x2, dim3(blocks), dim3(64), 0, 0, (double*)a, nrec);
    hipLaunchKernelGGL(store_x2, dim3(blocks), dim3(64), 0, 0, (double*)b, nrec);
    CHECK(hipDeviceSynchronize());
  }
  printf("read kernels: %lld bytes each (coalesced_x4, coalesced_lds, coalesced_x2, lane_x4, lane_x2, lane_lds, lane_touch4 (lines))\n",
         (long long)bytes);
  printf("store_lane_x2: %lld bytes; store_x2: %lld bytes\n", (long long)(nrec * 56), (long long)(nrec * 8));
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(out));
  return 0;
}
