// qp_layout.hip — device conversion between the two batch layouts of include/qpgpu.h.
//
// A tile of 64 QPs occupies the same contiguous 64*E doubles in both layouts (QP-major:
// [t][e]; TILED64: [e][t]), so the conversion is a 64 x E transpose per tile, staged through
// LDS in 64 x 32 chunks so both the HBM read and the HBM write are whole contiguous rows.
#include "qp_common.h"

namespace qpk {

constexpr int kChunk = 32;

__global__ void __launch_bounds__(256) relayout_kernel(int64_t batch, int E, const double* src,
                                                       double* dst, int to_tiled) {
  __shared__ double tile[64][kChunk + 1];
  const int64_t k = blockIdx.x;  // tile index
  const int e0 = blockIdx.y * kChunk;
  const int ec = min(kChunk, E - e0);
  const int valid = (int)min<int64_t>(64, batch - k * 64);
  const double* s = src + k * 64 * (int64_t)E;
  double* d = dst + k * 64 * (int64_t)E;
  for (int idx = threadIdx.x; idx < 64 * kChunk; idx += blockDim.x) {
    if (to_tiled) {  // read [t][e0 + c] runs, write [e0 + c][t] rows
      const int t = idx / kChunk, c = idx % kChunk;
      if (t < valid && c < ec) tile[t][c] = s[(int64_t)t * E + e0 + c];
    } else {
      const int c = idx / 64, t = idx % 64;
      if (t < valid && c < ec) tile[t][c] = s[(int64_t)(e0 + c) * 64 + t];
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * kChunk; idx += blockDim.x) {
    if (to_tiled) {
      const int c = idx / 64, t = idx % 64;
      if (t < valid && c < ec) d[(int64_t)(e0 + c) * 64 + t] = tile[t][c];
    } else {
      const int t = idx / kChunk, c = idx % kChunk;
      if (t < valid && c < ec) d[(int64_t)t * E + e0 + c] = tile[t][c];
    }
  }
}

}  // namespace qpk

extern "C" hipError_t qpk_relayout(int64_t batch, int E, const double* src, double* dst,
                                   int to_tiled, hipStream_t stream) {
  const int64_t tiles = (batch + 63) / 64;
  const int chunks = (E + qpk::kChunk - 1) / qpk::kChunk;
  hipLaunchKernelGGL(qpk::relayout_kernel, dim3((unsigned)tiles, (unsigned)chunks), dim3(256), 0,
                     stream, batch, E, src, dst, to_tiled);
  return hipGetLastError();
}
