// qp_panel.hip — MFMA panel setup for the large dense QPs (64 < n <= 256; BASELINE config C5).
//
// The setup of solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; SURVEY.md
// §8(a) rows a2-a4: cholesky_decomposition, J = L^{-T} with c2 = trace(J), cholesky_solve for the
// unconstrained start x0 = -G^{-1} g0, f0 = 1/2 g0.x0, c1 = trace(G)) is O(n^3): ~14 M FMA per QP
// at n = 256.  Here it runs as BLAS-3 on the f64 matrix cores (v_mfma_f64_16x16x4_f64), one QP
// per 256-thread workgroup, blocked in 16 x 16 tiles:
//   * right-looking blocked Cholesky: wave 0 factors the 16 x 16 diagonal block in LDS and
//     inverts it (W_k = L_kk^{-1}); the panel L_ik = A_ik W_k^T and the trailing update
//     A_ij -= L_ik L_jk^T are MFMA tiles spread over the 4 waves, the panel kept in LDS;
//   * X = L^{-1} by block columns: X_jj = W_j, X_ij = -W_i sum_k L_ik X_kj; every block of a
//     column stays in registers in the MFMA C/D layout, which is exactly the B-operand layout
//     of the next product (k index = row), so no tile is ever transposed;
//   * X is written row-major, which IS J = L^{-T} column-major (J[k][j] = X[j][k]) — the layout
//     the active-set loop of qp_wave.hip (GJR) reads coalesced in its Givens sweeps and update_z;
//   * x0 = -X^T (X g0), f0, c1, c2 and the status go to a per-QP header in the workspace.
// The blocked sums reorder the reference's floating-point operations, so this path matches the
// reference within north_star's 1e-10 relative tolerance rather than bitwise; QPGPU_FLAG_EXACT
// (and QPGPU_FLAG_WRITE_FACTOR, whose factor must be the reference's bits) select the serial
// restatement in qp_wave.hip instead.  A non-positive pivot reports NOT_POSITIVE_DEFINITE with
// that pivot as f, like the reference's "sum" (same index; the value within rounding).
#include "qp_common.h"

namespace qpk {

using d4 = __attribute__((ext_vector_type(4))) double;

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// v_mfma_f64_16x16x4_f64 lane maps (cdna_hip_programming.md §Fragment layout): lane l supplies
// A[row l&15][k l>>4] and B[k l>>4][col l&15]; result register g of lane l is C[(l>>4)+4g][l&15].
template <int NMAX>
__global__ void __launch_bounds__(256) qp_panel_setup_kernel(const QpArgs a, double* __restrict__ ws) {
  using WS = BigWs<NMAX>;
  constexpr int JS = WS::JS;
  constexpr int NBMAX = NMAX / 16;
  __shared__ double W[NBMAX][16][17];  // W_k = L_kk^{-1}
  __shared__ double P[NMAX][17];       // panel: block column k of L (rows below the diagonal)
  __shared__ double D[16][17];         // diagonal block being factored
  __shared__ double shd[4];
  __shared__ int shi[4];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t b = blockIdx.x;
  if (b >= a.batch) return;  // uniform per block
  const int n = a.n, T = a.tile;
  const int npad = (n + 15) & ~15, NB = npad >> 4;
  double* const Jc = ws + b * WS::PER_QP;  // X = L^{-1} row-major == J column-major
  double* const A = Jc + WS::OFF_R;        // scratch: G -> L (row-major)
  double* const H = Jc + WS::OFF_H;        // header
  const double* Gb = a.G + qbase_rt(b, n * n, T);
  const double* g0b = a.g0 + qbase_rt(b, n, T);
  const int r16 = lane & 15, q4 = lane >> 4;

  // ---- G -> A (lower triangle, padded to a multiple of 16 with an identity block), c1
  for (int e = tid; e < npad * npad; e += 256) {
    const int i = e / npad, j = e - i * npad;
    if (j > i) continue;  // the factorization reads the lower triangle only
    A[i * JS + j] = (i < n && j < n) ? Gb[(int64_t)(i * n + j) * T] : (i == j ? 1.0 : 0.0);
  }
  if (tid == 0) {
    double c1 = 0.0;
    for (int i = 0; i < n; i++) c1 += Gb[(int64_t)(i * n + i) * T];
    shd[0] = c1;
    shd[2] = __builtin_inf();  // smallest / largest pivot (certification of the loop, H[4])
    shd[3] = 0.0;
    shi[0] = 0;
  }
  __syncthreads();

  // ---- right-looking blocked Cholesky
  for (int k = 0; k < NB; k++) {
    if (wave == 0) {
      for (int e = lane; e < 256; e += 64) {
        const int r = e >> 4, c = e & 15;
        D[r][c] = c <= r ? A[(k * 16 + r) * JS + k * 16 + c] : 0.0;
      }
      sg_sync();
      bool fail = false;
      for (int c = 0; c < 16; c++) {
        const double piv = D[c][c];
        if (piv <= 0.0) {  // the reference's "sum <= 0" (NaN passes, as there)
          if (lane == 0) {
            shi[0] = 1;
            shd[1] = piv;
          }
          fail = true;
          break;
        }
        const double dg = sqrt(piv);
        if (lane == 0 && k * 16 + c < n) {  // (the padding's identity pivots excluded)
          shd[2] = fmin(shd[2], piv);
          shd[3] = fmax(shd[3], piv);
        }
        sg_sync();
        if (lane < 16) {
          if (lane > c)
            D[lane][c] = D[lane][c] / dg;
          else if (lane == c)
            D[c][c] = dg;
        }
        sg_sync();
        for (int e = lane; e < 256; e += 64) {
          const int r = e >> 4, s = e & 15;
          if (r > c && s > c && s <= r) D[r][s] -= D[r][c] * D[s][c];
        }
        sg_sync();
      }
      if (!fail) {
        // W_k = L_kk^{-1}: lane c runs the forward substitution for column c
        if (lane < 16) {
          const int c = lane;
          for (int i = 0; i < 16; i++) {
            double v = 0.0;
            if (i >= c) {
              v = (i == c) ? 1.0 : 0.0;
              for (int t = c; t < i; t++) v -= D[i][t] * W[k][t][c];
              v = v / D[i][i];
            }
            W[k][i][c] = v;
          }
        }
        for (int e = lane; e < 256; e += 64) {
          const int r = e >> 4, c = e & 15;
          A[(k * 16 + r) * JS + k * 16 + c] = c <= r ? D[r][c] : 0.0;
        }
      }
    }
    __syncthreads();
    if (shi[0]) break;
    // panel: L_ik = A_ik W_k^T   (B[t][c] = W_k[c][t])
    for (int ib = k + 1 + wave; ib < NB; ib += 4) {
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int t = 4 * q + q4;
        acc = mfma4(A[(ib * 16 + r16) * JS + k * 16 + t], W[k][r16][t], acc);
      }
#pragma unroll
      for (int g = 0; g < 4; g++) {
        const int row = q4 + 4 * g;
        A[(ib * 16 + row) * JS + k * 16 + r16] = acc[g];
        P[ib * 16 + row][r16] = acc[g];
      }
    }
    __syncthreads();
    // trailing update of the lower block triangle: A_ij -= L_ik L_jk^T, k < j <= i
    {
      const int Tn = NB - 1 - k;
      const int pairs = Tn * (Tn + 1) / 2;
      for (int pi = wave; pi < pairs; pi += 4) {
        int ib = k + 1, rem = pi;
        while (rem >= ib - k) {
          rem -= ib - k;
          ib++;
        }
        const int jb = k + 1 + rem;
        d4 acc;
#pragma unroll
        for (int g = 0; g < 4; g++) acc[g] = A[(ib * 16 + q4 + 4 * g) * JS + jb * 16 + r16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int t = 4 * q + q4;
          acc = mfma4(-P[ib * 16 + r16][t], P[jb * 16 + r16][t], acc);
        }
#pragma unroll
        for (int g = 0; g < 4; g++) A[(ib * 16 + q4 + 4 * g) * JS + jb * 16 + r16] = acc[g];
      }
    }
    __syncthreads();
  }
  if (shi[0]) {
    if (tid == 0) {
      H[0] = (double)QPGPU_QP_NOT_POSITIVE_DEFINITE;
      H[1] = shd[1];
    }
    return;
  }

  // ---- X = L^{-1} by block columns (snake-assigned to the 4 waves for balance)
  for (int jb = 0; jb < NB; jb++) {
    const int pos = jb & 7;
    if ((pos < 4 ? pos : 7 - pos) != wave) continue;
    d4 X[NBMAX];
#pragma unroll
    for (int t = 0; t < NBMAX; t++) X[t] = d4{0.0, 0.0, 0.0, 0.0};
    // blocks above the diagonal are zero
    for (int ib = 0; ib < jb; ib++)
#pragma unroll
      for (int g = 0; g < 4; g++) Jc[(ib * 16 + q4 + 4 * g) * JS + jb * 16 + r16] = 0.0;
#pragma unroll
    for (int t = 0; t < NBMAX; t++)
      if (t == jb) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
          X[t][g] = W[jb][q4 + 4 * g][r16];
          Jc[(jb * 16 + q4 + 4 * g) * JS + jb * 16 + r16] = X[t][g];
        }
      }
    for (int ib = jb + 1; ib < NB; ib++) {
      d4 S = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kb = 0; kb < NBMAX; kb++) {
        if (kb >= jb && kb < ib) {
          double av[4];
#pragma unroll
          for (int q = 0; q < 4; q++) av[q] = A[(ib * 16 + r16) * JS + kb * 16 + 4 * q + q4];
#pragma unroll
          for (int q = 0; q < 4; q++) S = mfma4(av[q], X[kb][q], S);
        }
      }
      d4 Xn = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; q++) Xn = mfma4(-W[ib][r16][4 * q + q4], S[q], Xn);
#pragma unroll
      for (int t = 0; t < NBMAX; t++)
        if (t == ib) X[t] = Xn;
#pragma unroll
      for (int g = 0; g < 4; g++) Jc[(ib * 16 + q4 + 4 * g) * JS + jb * 16 + r16] = Xn[g];
    }
  }
  __syncthreads();

  // ---- x0 = -X^T (X g0), f0 = 1/2 g0.x0 (reference cholesky_solve, @.text+0x31a2), c2
  double* const yv = &P[0][0];  // reuse the panel buffer: y at [0, NMAX), g0 at [NMAX, 2 NMAX)
  double* const gv = &P[0][0] + NMAX;
  for (int i = tid; i < npad; i += 256) gv[i] = i < n ? g0b[(int64_t)i * T] : 0.0;
  __syncthreads();
  for (int i = tid; i < n; i += 256) {
    double s = 0.0;
    for (int j = 0; j <= i; j++) s += Jc[i * JS + j] * gv[j];
    yv[i] = s;
  }
  __syncthreads();
  for (int j = tid; j < n; j += 256) {
    double s = 0.0;
    for (int i = j; i < n; i++) s += Jc[i * JS + j] * yv[i];
    H[WS::HX + j] = -s;
  }
  __syncthreads();
  if (tid == 0) {
    double f = 0.0, c2 = 0.0;
    for (int i = 0; i < n; i++) {
      f += gv[i] * H[WS::HX + i];
      c2 += Jc[i * JS + i];
    }
    H[0] = (double)QPGPU_QP_OK;
    H[1] = 0.5 * f;
    H[2] = shd[0];
    H[3] = c2;
    H[4] = shd[3] / shd[2];  // pivot spread: the loop marks QPs beyond 1e8 for the EXACT re-solve
  }
}

}  // namespace qpk

extern "C" hipError_t qpk_launch_panel_setup(const qpk::QpArgs* a, hipStream_t stream, double* ws) {
  if (a->n > qpk::kBigN) return hipErrorInvalidValue;
  hipLaunchKernelGGL((qpk::qp_panel_setup_kernel<qpk::kBigN>), dim3((unsigned)a->batch), dim3(256), 0,
                     stream, *a, ws);
  return hipGetLastError();
}
