// mgqp_device.hip — the batched controller cycle on the GPU (see mgqp_device.h).
//
// One lane per robot.  Per-robot workspace is robot-minor ("SoA": element e of robot r at
// [e * count + r]) so a wave's accesses to one element are one coalesced 256-byte load; the QP
// arrays handed to the solver are QP-major doubles (the solver's default layout).  Float and
// double expressions are evaluated in exactly the host controller's order (no contraction:
// built with -ffp-contract=off), so the device cycle equals the host-orchestrated batched path
// bit for bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <map>
#include <mutex>
#include <string>

#include "mgqp_device.h"
#include "qpgpu.h"

namespace mgqp_dev {

namespace {

__device__ __forceinline__ float ld(const float* a, int64_t e, int64_t count, int64_t r) {
  return a[e * count + r];
}

// ------------------------------------------------------------------ builder (:912-1143)
__global__ void build_tasks_kernel(Plan P, Work W) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  const int D = P.dof, dim = P.dim, ws = P.ws;
  const float* ang = P.angles + r * P.status_len;
  const float* vel = P.velocities + r * P.status_len;
  for (int g = 0; g < P.ngen; ++g) {
    const RowGen G = P.gen[g];
    const int j = G.joint;
    if (G.type == GEN_TASK) {
      const int jc = P.jac_cols[j], L = P.ts_len[j];
      const float* J = P.jac[j] + r * (int64_t)ws * jc;
      const float* Jd = P.jacd[j] + r * (int64_t)ws * jc;
      for (int rr = 0; rr < ws; ++rr) {
        const int row = G.row0 + rr;
        for (int c = 0; c < dim; ++c)
          W.cond[((int64_t)row * dim + c) * K + r] = c < jc ? J[rr * jc + c] : 0.f;
        float jq = 0.f;
        for (int c = 0; c < jc; ++c) jq += Jd[rr * jc + c] * vel[c];
        const bool fp = G.flags & F_POS, fv = G.flags & F_VEL, fa = G.flags & F_ACC;
        const float dP = fp ? P.ts[j][0][r * L + rr] : 0.f, cP = fp ? P.ts[j][3][r * L + rr] : 0.f;
        const float dV = fv ? P.ts[j][1][r * L + rr] : 0.f, cV = fv ? P.ts[j][4][r * L + rr] : 0.f;
        const float dA = fa ? P.ts[j][2][r * L + rr] : 0.f, cA = fa ? P.ts[j][5][r * L + rr] : 0.f;
        float t = P.kTP * (dP - cP);
        t = t + P.kTD * (dV - cV);
        t = t - jq;
        t = t + dA;
        t = t - cA;
        W.goal[(int64_t)row * K + r] = -t;
      }
    } else if (G.type == GEN_JOINT) {
      const int row = G.row0;
      for (int c = 0; c < dim; ++c) W.cond[((int64_t)row * dim + c) * K + r] = c == j ? 1.f : 0.f;
      const float qd = (G.flags & F_POS) ? P.js[j][0][r] : ang[j];
      const float qdd = (G.flags & F_VEL) ? P.js[j][1][r] : vel[j];
      W.goal[(int64_t)row * K + r] = -(P.kJP * (qd - ang[j]) + P.kJD * (qdd - vel[j]));
    } else {  // GEN_DYN: [M -I], goal 0
      const float* M = P.inertia + r * (int64_t)D * D;
      for (int rr = 0; rr < D; ++rr) {
        const int row = G.row0 + rr;
        for (int c = 0; c < dim; ++c) {
          const float v = c < D ? M[rr * D + c] : (c == D + rr ? -1.f : 0.f);
          W.cond[((int64_t)row * dim + c) * K + r] = v;
        }
        W.goal[(int64_t)row * K + r] = 0.f;
      }
    }
  }
  // limits (:1113-1130): [accP'; tauP; -accN'; -tauN]
  for (int i = 0; i < D; ++i) {
    const double lp = log((double)(float)(P.sup[i] - ang[i]));
    const double ln = -log((double)(float)(ang[i] - P.inf[i]));
    const double ap = (double)P.accP[i], an = (double)P.accN[i];
    const float accP = (float)(lp < ap ? lp : ap);  // std::min(ap, lp)
    const float accN = (float)(an < ln ? ln : an);  // std::max(an, ln)
    W.limits[(int64_t)i * K + r] = accP;
    W.limits[(int64_t)(D + i) * K + r] = P.tP[i];
    W.limits[(int64_t)(2 * D + i) * K + r] = -accN;
    W.limits[(int64_t)(3 * D + i) * K + r] = -P.tN[i];
  }
}

__global__ void init_kernel(Plan P, Work W, double* G, double* g0, int init_qp) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  const int dim = P.dim;
  for (int i = 0; i < dim; ++i) {
    for (int j = 0; j < dim; ++j) W.Z[((int64_t)i * dim + j) * K + r] = i == j ? 1.f : 0.f;
    W.res[(int64_t)i * K + r] = 0.f;
    W.u[(int64_t)i * K + r] = 0.f;
  }
  W.state[r] = 0;
  if (init_qp) {
    for (int i = 0; i < dim * dim; ++i) G[r * dim * dim + i] = (i / dim == i % dim) ? 1.0 : 0.0;
    for (int i = 0; i < dim; ++i) g0[r * dim + i] = 0.0;
  }
}

// ------------------------------------------------------------------ level QP (:783-793, :655-708)
__global__ void build_level_kernel(Plan P, Work W, int row0, int p, double* CE, double* ce0,
                                   double* CI, double* ci0) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  const int n = P.dim, m = P.nineq;
  // A = cond_l * Z (p x n) -> CE (n x p), CE[j][i] = A(i, j)
  for (int i = 0; i < p; ++i) {
    const int64_t crow = (int64_t)(row0 + i) * n;
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
      for (int k = 0; k < n; ++k) s += ld(W.cond, crow + k, K, r) * ld(W.Z, (int64_t)k * n + j, K, r);
      CE[r * n * p + j * p + i] = (double)s;
    }
    float cl = 0.f;
    for (int k = 0; k < n; ++k) cl += ld(W.cond, crow + k, K, r) * ld(W.res, k, K, r);
    ce0[r * p + i] = (double)(ld(W.goal, row0 + i, K, r) - cl);
  }
  // B = Bcumul * Z (m x n) -> CI (n x m)
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
      for (int k = 0; k < n; ++k) s += W.Bcumul[i * n + k] * ld(W.Z, (int64_t)k * n + j, K, r);
      CI[r * n * m + j * m + i] = (double)s;
    }
    ci0[r * m + i] = (double)ld(W.limits, i, K, r);
  }
}

// ------------------------------------------------------------------ finish level (:814-862)
__device__ __forceinline__ bool bad_f(double f) { return isnan(f) || f == INFINITY; }

// One-sided Jacobi, same rotation sequence and arithmetic as hestenes() in mgqp_controller.cpp.
// X: rows x k at lds[(i*k + c) * BS + t]; W (k x k) follows X when present.
__device__ void hestenes_lds(double* X, int rows, int k, double* Wm, int BS, int t) {
  for (int sweep = 0; sweep < 80; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < k - 1; ++p)
      for (int q = p + 1; q < k; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int i = 0; i < rows; ++i) {
          const double xp = X[(i * k + p) * BS + t], xq = X[(i * k + q) * BS + t];
          al += xp * xp;
          be += xq * xq;
          ga += xp * xq;
        }
        if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
        rotated = true;
        const double zeta = (be - al) / (2.0 * ga);
        const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
        for (int i = 0; i < rows; ++i) {
          double& xp = X[(i * k + p) * BS + t];
          double& xq = X[(i * k + q) * BS + t];
          const double a0 = xp, b0 = xq;
          xp = c * a0 - s * b0;
          xq = s * a0 + c * b0;
        }
        if (Wm)
          for (int i = 0; i < k; ++i) {
            double& wp = Wm[(i * k + p) * BS + t];
            double& wq = Wm[(i * k + q) * BS + t];
            const double a0 = wp, b0 = wq;
            wp = c * a0 - s * b0;
            wq = s * a0 + c * b0;
          }
      }
    if (!rotated) break;
  }
}

__global__ void finish_level_kernel(Plan P, Work W, const double* x1, const double* f1,
                                    const int32_t* st1, const double* x2, const double* f2,
                                    const int32_t* st2, int acc_rows) {
  extern __shared__ double lds[];
  const int BS = blockDim.x, t = threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * BS + t;
  const int64_t K = W.count;
  const bool live = r < K && W.state[r] == 0;
  const int n = P.dim;
  if (live) {
    // solveNextStep's decision (:708-744); DEPENDENT / step cap = the reference's throw
    bool ok = true, exc = false;
    const int s1 = st1[r];
    if (s1 == QPGPU_QP_DEPENDENT || s1 == QPGPU_QP_MAX_ITER) {
      exc = true;
    } else if (!bad_f(f1[r])) {
      for (int i = 0; i < n; ++i) W.u[(int64_t)i * K + r] = (float)x1[r * n + i];
    } else {
      const int s2 = st2[r];
      if (s2 == QPGPU_QP_DEPENDENT || s2 == QPGPU_QP_MAX_ITER) {
        exc = true;
      } else if (!bad_f(f2[r])) {
        for (int i = 0; i < n; ++i) W.u[(int64_t)i * K + r] = (float)x2[r * n + i];
      } else {
        for (int i = 0; i < n; ++i) W.u[(int64_t)i * K + r] = 0.f;
        ok = false;
      }
    }
    if (exc) {
      W.state[r] = 2;
    } else if (!ok) {
      W.state[r] = 1;  // stops here; the result is last_res (== res)
    } else {
      // res = last_res + Z u   (mulv then add, :818)
      float zu[64];
      for (int i = 0; i < n; ++i) {
        float s = 0.f;
        for (int k = 0; k < n; ++k)
          s += ld(W.Z, (int64_t)i * n + k, K, r) * ld(W.u, k, K, r);
        zu[i] = s;
      }
      for (int i = 0; i < n; ++i) W.res[(int64_t)i * K + r] = ld(W.res, i, K, r) + zu[i];
    }
  }
  if (acc_rows <= 0) return;
  const bool proj = live && W.state[r] == 0;
  // Z = I - V A V^T of Acumul = cond rows [0, acc_rows) (nullspace_projector in the host code)
  const int rr = acc_rows, c = n, k = rr < c ? rr : c;
  double* X = lds;
  double* Wm = rr >= c ? lds + (int64_t)rr * c * BS : nullptr;
  if (proj) {
    if (rr >= c) {
      for (int i = 0; i < rr; ++i)
        for (int j = 0; j < c; ++j) X[(i * c + j) * BS + t] = ld(W.cond, (int64_t)i * n + j, K, r);
      for (int i = 0; i < c; ++i)
        for (int j = 0; j < c; ++j) Wm[(i * c + j) * BS + t] = i == j ? 1.0 : 0.0;
      hestenes_lds(X, rr, c, Wm, BS, t);
    } else {
      for (int i = 0; i < rr; ++i)
        for (int j = 0; j < c; ++j) X[(j * rr + i) * BS + t] = ld(W.cond, (int64_t)i * n + j, K, r);
      hestenes_lds(X, c, rr, nullptr, BS, t);
    }
    // singular values, thin V (in place: V[:, j] = W[:, j] or X[:, j] / sigma_j)
    bool keep[64];
    for (int j = 0; j < k; ++j) {
      double nrm = 0;
      if (rr >= c) {
        for (int i = 0; i < rr; ++i) nrm += X[(i * c + j) * BS + t] * X[(i * c + j) * BS + t];
        keep[j] = !((double)(float)sqrt(nrm) < 0.0000000000000001);
      } else {
        for (int i = 0; i < c; ++i) nrm += X[(i * rr + j) * BS + t] * X[(i * rr + j) * BS + t];
        const double sg = sqrt(nrm);
        keep[j] = !((double)(float)sg < 0.0000000000000001);
        for (int i = 0; i < c; ++i)
          X[(i * rr + j) * BS + t] = sg > 0 ? X[(i * rr + j) * BS + t] / sg : 0.0;
      }
    }
    const double* V = rr >= c ? Wm : X;
    const int vs = rr >= c ? c : rr;  // row stride of V
    for (int i = 0; i < c; ++i)
      for (int j = 0; j < c; ++j) {
        double s = 0;
        for (int l = 0; l < k; ++l)
          if (keep[l]) s += V[(i * vs + l) * BS + t] * V[(j * vs + l) * BS + t];
        W.Z[((int64_t)i * n + j) * K + r] = (i == j ? 1.f : 0.f) - (float)s;
      }
  }
}

// ------------------------------------------------------------------ register-resident versions
// For dim N <= 14 (DOF <= 7): Z lives in registers (N*N floats) and the Jacobi operand of the
// common r < N case (X = Acumul^T, N x r, r <= N-1) too, fully unrolled over N and RMAX = N-1
// with wave-uniform guards on the runtime row count.  Same operation order as the generic
// kernels (and the host), so the results are bit-identical.
template <int N>
__global__ __launch_bounds__(64) void build_level_reg_kernel(Plan P, Work W, int row0, int p,
                                                             double* CE, double* ce0, double* CI,
                                                             double* ci0) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  const int m = P.nineq;
  float Z[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) Z[i][j] = ld(W.Z, i * N + j, K, r);
  float res[N];
#pragma unroll
  for (int i = 0; i < N; ++i) res[i] = ld(W.res, i, K, r);
  double* CEr = CE + r * N * p;
  for (int i = 0; i < p; ++i) {
    const int64_t crow = (int64_t)(row0 + i) * N;
    float c[N];
#pragma unroll
    for (int k = 0; k < N; ++k) c[k] = ld(W.cond, crow + k, K, r);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < N; ++k) sum += c[k] * Z[k][j];
      CEr[j * p + i] = (double)sum;
    }
    float cl = 0.f;
#pragma unroll
    for (int k = 0; k < N; ++k) cl += c[k] * res[k];
    ce0[r * p + i] = (double)(ld(W.goal, row0 + i, K, r) - cl);
  }
  double* CIr = CI + r * N * m;
#pragma unroll
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < m; ++i) {
      const float* b = W.Bcumul + i * N;
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < N; ++k) sum += b[k] * Z[k][j];
      CIr[j * m + i] = (double)sum;
    }
  for (int i = 0; i < m; ++i) ci0[r * m + i] = (double)ld(W.limits, i, K, r);
}

template <int N, int R>
__global__ __launch_bounds__(64) void finish_level_reg_kernel(Plan P, Work W, const double* x1,
                                                              const double* f1, const int32_t* st1,
                                                              const double* x2, const double* f2,
                                                              const int32_t* st2, int acc_rows) {
  constexpr int RM = R;  // exact stacked row count (< N): X = Acumul^T is N x R
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  if (W.state[r] != 0) return;
  bool ok = true, exc = false;
  const int s1 = st1[r];
  const double* xs = x1;
  if (s1 == QPGPU_QP_DEPENDENT || s1 == QPGPU_QP_MAX_ITER) {
    exc = true;
  } else if (bad_f(f1[r])) {
    const int s2 = st2[r];
    if (s2 == QPGPU_QP_DEPENDENT || s2 == QPGPU_QP_MAX_ITER) exc = true;
    else if (!bad_f(f2[r])) xs = x2;
    else ok = false;
  }
  if (exc) {
    W.state[r] = 2;
    return;
  }
  float u[N];
#pragma unroll
  for (int i = 0; i < N; ++i) u[i] = ok ? (float)xs[r * N + i] : 0.f;
#pragma unroll
  for (int i = 0; i < N; ++i) W.u[(int64_t)i * K + r] = u[i];
  if (!ok) {
    W.state[r] = 1;
    return;
  }
  {
    float zu[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < N; ++k) sum += ld(W.Z, i * N + k, K, r) * u[k];
      zu[i] = sum;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) W.res[(int64_t)i * K + r] = ld(W.res, i, K, r) + zu[i];
  }
  if (acc_rows <= 0) return;
  (void)acc_rows;  // == R (checked by the launcher)
  constexpr int rr = R;
  double X[N][RM];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j) X[i][j] = j < rr ? (double)ld(W.cond, (int64_t)j * N + i, K, r) : 0.0;
  for (int sweep = 0; sweep < 80; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < RM - 1; ++p)
#pragma unroll
      for (int q = p + 1; q < RM; ++q) {
        double al = 0, be = 0, ga = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          al += X[i][p] * X[i][p];
          be += X[i][q] * X[i][q];
          ga += X[i][p] * X[i][q];
        }
        if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
        rotated = true;
        const double zeta = (be - al) / (2.0 * ga);
        const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + tt * tt), sn = c * tt;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const double a0 = X[i][p], b0 = X[i][q];
          X[i][p] = c * a0 - sn * b0;
          X[i][q] = sn * a0 + c * b0;
        }
      }
    if (!rotated) break;
  }
  // thin V (normalised columns; dropped singular values zeroed, which leaves the host's sums
  // unchanged) to the V workspace; zform_kernel forms Z from it
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    double nrm = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) nrm += X[i][j] * X[i][j];
    const double sg = sqrt(nrm);
    const bool keep = !((double)(float)sg < 0.0000000000000001);
#pragma unroll
    for (int i = 0; i < N; ++i)
      W.V[((int64_t)i * RM + j) * K + r] = keep && sg > 0 ? X[i][j] / sg : 0.0;
  }
}

// Z = I - V V^T from the V workspace (rows of V: N, columns: R), for robots still active.  V is
// read once into registers (one robot per lane: 1 024 waves for 65 536 robots, one per SIMD, so
// the N*R doubles cost no occupancy); Z is symmetric bit for bit (each entry sums the same
// products V[i][l]*V[j][l] in l order), so the upper triangle is formed and stored twice.
template <int N, int R>
__global__ __launch_bounds__(64) void zform_kernel(Work W) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K || W.state[r] != 0) return;
  double v[N][R];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int l = 0; l < R; ++l) v[i][l] = W.V[((int64_t)i * R + l) * K + r];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = i; j < N; ++j) {
      double sum = 0;
#pragma unroll
      for (int l = 0; l < R; ++l) sum += v[i][l] * v[j][l];
      const float z = (i == j ? 1.f : 0.f) - (float)sum;
      W.Z[((int64_t)i * N + j) * K + r] = z;
      if (j != i) W.Z[((int64_t)j * N + i) * K + r] = z;
    }
}

__global__ void outputs_kernel(Plan P, Work W, float* torques, float* tracking, int32_t* codes) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = W.count;
  if (r >= K) return;
  const int D = P.dof, n = P.dim;
  const int st = W.state[r];
  codes[r] = st == 2 ? 3 : 0;
  if (st == 2) return;
  for (int i = 0; i < D; ++i)
    torques[r * D + i] = ld(W.res, D + i, K, r) + P.h[r * D + i];
  if (tracking)
    for (int i = 0; i < n; ++i) tracking[r * n + i] = ld(W.res, i, K, r);
}

int check(hipError_t e) { return e == hipSuccess ? 0 : -1; }

dim3 grid_for(int64_t K, int bs) { return dim3((unsigned)((K + bs - 1) / bs)); }

}  // namespace

int launch_init(const Plan& P, const Work& W, double* G, double* g0, hipStream_t s) {
  hipLaunchKernelGGL(init_kernel, grid_for(W.count, 256), dim3(256), 0, s, P, W, G, g0,
                     G != nullptr ? 1 : 0);
  return check(hipGetLastError());
}

int launch_build_tasks(const Plan& P, const Work& W, hipStream_t s) {
  hipLaunchKernelGGL(build_tasks_kernel, grid_for(W.count, 256), dim3(256), 0, s, P, W);
  return check(hipGetLastError());
}

template <int N>
bool try_build_level_reg(const Plan& P, const Work& W, int level, double* CE, double* ce0,
                         double* CI, double* ci0, hipStream_t s) {
  if (P.dim != N) return false;
  hipLaunchKernelGGL(build_level_reg_kernel<N>, grid_for(W.count, 64), dim3(64), 0, s, P, W,
                     P.level_row0[level], P.level_rows[level], CE, ce0, CI, ci0);
  return true;
}

template <int N, int R>
bool try_finish_level_reg(const Plan& P, const Work& W, const double* x1, const double* f1,
                          const int32_t* st1, const double* x2, const double* f2,
                          const int32_t* st2, int acc_rows, hipStream_t s) {
  if (P.dim != N || acc_rows != R) return false;
  hipLaunchKernelGGL((finish_level_reg_kernel<N, R>), grid_for(W.count, 64), dim3(64), 0, s, P,
                     W, x1, f1, st1, x2, f2, st2, acc_rows);
  hipLaunchKernelGGL((zform_kernel<N, R>), grid_for(W.count, 64), dim3(64), 0, s, W);
  return true;
}

int launch_build_level(const Plan& P, const Work& W, int level, double* CE, double* ce0,
                       double* CI, double* ci0, hipStream_t s) {
  if (try_build_level_reg<14>(P, W, level, CE, ce0, CI, ci0, s) ||
      try_build_level_reg<12>(P, W, level, CE, ce0, CI, ci0, s) ||
      try_build_level_reg<10>(P, W, level, CE, ce0, CI, ci0, s) ||
      try_build_level_reg<8>(P, W, level, CE, ce0, CI, ci0, s) ||
      try_build_level_reg<6>(P, W, level, CE, ce0, CI, ci0, s))
    return check(hipGetLastError());
  hipLaunchKernelGGL(build_level_kernel, grid_for(W.count, 256), dim3(256), 0, s, P, W,
                     P.level_row0[level], P.level_rows[level], CE, ce0, CI, ci0);
  return check(hipGetLastError());
}

int launch_finish_level(const Plan& P, const Work& W, int level, const double* x1,
                        const double* f1, const int32_t* st1, const double* x2, const double* f2,
                        const int32_t* st2, int acc_rows, hipStream_t s) {
  (void)level;
  // DOF 7 (the reference robot): the stacked row counts of its usual stacks
  if (try_finish_level_reg<14, 10>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s) ||
      try_finish_level_reg<14, 11>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s) ||
      try_finish_level_reg<14, 12>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s) ||
      try_finish_level_reg<14, 7>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s) ||
      try_finish_level_reg<14, 8>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s) ||
      try_finish_level_reg<14, 9>(P, W, x1, f1, st1, x2, f2, st2, acc_rows, s))
    return check(hipGetLastError());
  const int c = P.dim;
  const size_t per = acc_rows > 0 ? ((size_t)acc_rows * c + (acc_rows >= c ? (size_t)c * c : 0)) * 8
                                  : 0;
  int bs = 64;
  while (bs > 1 && per * bs > 64 * 1024) bs /= 2;
  if (per * bs > 160 * 1024) return -2;
  hipLaunchKernelGGL(finish_level_kernel, grid_for(W.count, bs), dim3(bs), per * bs, s, P, W,
                     x1, f1, st1, x2, f2, st2, acc_rows);
  return check(hipGetLastError());
}

int launch_outputs(const Plan& P, const Work& W, float* torques, float* tracking, int32_t* codes,
                   hipStream_t s) {
  hipLaunchKernelGGL(outputs_kernel, grid_for(W.count, 256), dim3(256), 0, s, P, W, torques,
                     tracking, codes);
  return check(hipGetLastError());
}

}  // namespace mgqp_dev

namespace mgqp_dev {

namespace {

// Workspace per (device, stream): cycles enqueued on different streams never share one.
struct CycleWs {
  size_t bytes = 0;
  void* buf = nullptr;
  int64_t qp_count = -1;  // G / g0 initialised for this (count, dim)
  int qp_dim = -1;
  int lim_m = -1, lim_n = -1;  // the constant limits matrix [-I; +I] uploaded for this (m, n)
  size_t lim_off = 0;          // ... at this workspace offset
};
std::mutex g_cws_mu;
std::map<std::pair<int, hipStream_t>, CycleWs> g_cws_map;
thread_local std::string g_cws_err;

int fail(const char* what, hipError_t e, const char** err) {
  g_cws_err = std::string(what) + ": " + hipGetErrorString(e);
  *err = g_cws_err.c_str();
  return -1;
}

}  // namespace

int run_cycle(const Plan& P, int64_t K, const float* Bcumul_host, float* torques, float* tracking,
              int32_t* codes, hipStream_t s, const char** err) {
  if (K <= 0) return 0;
  const int n = P.dim, m = P.nineq;
  int pmax = 0;
  for (int l = 0; l < P.nlevels; ++l) pmax = P.level_rows[l] > pmax ? P.level_rows[l] : pmax;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t fK = (size_t)K;
  // workspace map
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += al(bytes); return o; };
  const size_t oCond = take(fK * P.total_rows * n * 4), oGoal = take(fK * P.total_rows * 4),
               oLim = take(fK * m * 4), oZ = take(fK * n * n * 4), oRes = take(fK * n * 4),
               oU = take(fK * n * 4), oState = take(fK * 4), oB = take((size_t)m * n * 4),
               oV = take(fK * n * n * 8),
               oG = take(fK * n * n * 8), og0 = take(fK * n * 8), oCE = take(fK * n * pmax * 8),
               oce0 = take(fK * pmax * 8), oCI = take(fK * n * m * 8), oci0 = take(fK * m * 8),
               ox1 = take(fK * n * 8), of1 = take(fK * 8), os1 = take(fK * 4),
               ox2 = take(fK * n * 8), of2 = take(fK * 8), os2 = take(fK * 4);
  hipError_t e;
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return fail("hipGetDevice", e, err);
  std::lock_guard<std::mutex> lock(g_cws_mu);
  CycleWs& g_cws = g_cws_map[{dev, s}];
  if (g_cws.bytes < off) {
    if (g_cws.buf) {
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail("hipStreamSynchronize", e, err);
      (void)hipFree(g_cws.buf);
    }
    g_cws.buf = nullptr;
    g_cws.bytes = 0;
    g_cws.qp_count = -1;
    g_cws.lim_m = g_cws.lim_n = -1;
    if ((e = hipMalloc(&g_cws.buf, off)) != hipSuccess) return fail("hipMalloc", e, err);
    g_cws.bytes = off;
  }
  char* b = static_cast<char*>(g_cws.buf);
  Work W;
  W.count = K;
  W.cond = reinterpret_cast<float*>(b + oCond);
  W.goal = reinterpret_cast<float*>(b + oGoal);
  W.limits = reinterpret_cast<float*>(b + oLim);
  W.Z = reinterpret_cast<float*>(b + oZ);
  W.res = reinterpret_cast<float*>(b + oRes);
  W.u = reinterpret_cast<float*>(b + oU);
  W.state = reinterpret_cast<int32_t*>(b + oState);
  W.Bcumul = reinterpret_cast<float*>(b + oB);
  W.V = reinterpret_cast<double*>(b + oV);
  double *G = reinterpret_cast<double*>(b + oG), *g0 = reinterpret_cast<double*>(b + og0),
         *CE = reinterpret_cast<double*>(b + oCE), *ce0 = reinterpret_cast<double*>(b + oce0),
         *CI = reinterpret_cast<double*>(b + oCI), *ci0 = reinterpret_cast<double*>(b + oci0),
         *x1 = reinterpret_cast<double*>(b + ox1), *f1 = reinterpret_cast<double*>(b + of1),
         *x2 = reinterpret_cast<double*>(b + ox2), *f2 = reinterpret_cast<double*>(b + of2);
  int32_t *s1 = reinterpret_cast<int32_t*>(b + os1), *s2 = reinterpret_cast<int32_t*>(b + os2);

  // The limits matrix depends on the DOF only: uploaded once per (m, n) into the workspace, with
  // a synchronous copy after the stream has drained (earlier cycles may still read the old one),
  // so the caller's host buffer is never read after this call returns.
  if (g_cws.lim_m != m || g_cws.lim_n != n || g_cws.lim_off != oB) {
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail("hipStreamSynchronize", e, err);
    if ((e = hipMemcpy(const_cast<float*>(W.Bcumul), Bcumul_host, (size_t)m * n * 4,
                       hipMemcpyHostToDevice)) != hipSuccess)
      return fail("hipMemcpy", e, err);
    g_cws.lim_m = m;
    g_cws.lim_n = n;
    g_cws.lim_off = oB;
  }
  const bool init_qp = !(g_cws.qp_count == K && g_cws.qp_dim == n);
  if (launch_init(P, W, init_qp ? G : nullptr, g0, s)) return fail("init", hipGetLastError(), err);
  g_cws.qp_count = K;
  g_cws.qp_dim = n;
  if (launch_build_tasks(P, W, s)) return fail("build_tasks", hipGetLastError(), err);

  int last = -1;
  for (int l = 0; l < P.nlevels; ++l)
    if (P.level_rows[l] > 0) last = l;
  for (int l = 0; l <= last; ++l) {
    const int p = P.level_rows[l];
    if (p == 0) continue;  // empty level: `continue` at :781
    if (launch_build_level(P, W, l, CE, ce0, CI, ci0, s)) return fail("build_level", hipGetLastError(), err);
    qpgpu_problem_desc d{};
    d.n = n;
    d.p = p;
    d.m = m;
    d.batch = K;
    d.flags = P.solver_flags;
    // one launch gives both the solve with CI and the retry without it (:717-736): the latter
    // is the state after the equality phase (qpgpu_solve_batched_eq)
    const int rc = qpgpu_solve_batched_eq(&d, G, g0, CE, ce0, CI, ci0, x1, f1, s1, nullptr, x2,
                                          f2, s2, s);
    if (rc != QPGPU_SUCCESS) {
      g_cws_err = std::string("qpgpu_solve_batched_eq: ") + qpgpu_last_error();
      *err = g_cws_err.c_str();
      return -3;
    }
    const int acc = l < last ? P.level_row0[l] + p : 0;  // Z after the last level is unused
    const int frc = launch_finish_level(P, W, l, x1, f1, s1, x2, f2, s2, acc, s);
    if (frc == -2) {
      g_cws_err = "stacked task rows too large for the LDS projector";
      *err = g_cws_err.c_str();
      return -2;
    }
    if (frc) return fail("finish_level", hipGetLastError(), err);
  }
  if (launch_outputs(P, W, torques, tracking, codes, s)) return fail("outputs", hipGetLastError(), err);
  return 0;
}

}  // namespace mgqp_dev
