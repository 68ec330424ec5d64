// qp_lane.hip — gfx950 batched Goldfarb–Idnani solver, ONE QP PER LANE (n <= 8).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; operation order
// of the prebuilt libquadprog.a fixed in SURVEY.md §3.2) for 64 independent QPs per wavefront.
// There is no cross-lane communication at all: every lane runs the whole algorithm for its own
// QP, so the serial chains (Givens coefficients, back-substitutions, step lengths) are
// executed once per QP instead of once per lane of a subgroup, which is the dominant cost at
// these sizes.  Per-lane state placement (gfx950: 512 VGPR+AGPR per lane at 1 wave/SIMD,
// 160 KiB LDS per CU):
//   * J (= L^{-T}, n x n, touched by column pairs in every Givens sweep) lives in LDS,
//     lane-interleaved (element (i,j) of lane l at [(i*NM + j)*64 + l]) so every access is a
//     conflict-free ds_read/write_b64 and column indices may be run-time values;
//   * R (upper triangle + first subdiagonal, the only entries the algorithm ever makes
//     non-zero), x, z, d, np, u, r, A and s live in registers with compile-time indices;
//   * G is factored in registers; CE, CI and ci0 are streamed from global memory (L2 / MALL)
//     each time the algorithm reads them: the l1 scan walks CI row by row, which keeps every
//     s[i] accumulating in the reference's j-ascending order.
// IEEE binary64 throughout, no contraction: results are bitwise identical to the CPU
// restatement (oracle/qp_oracle.c), which tests/ check.
#include "qp_common.h"

namespace qpk {

template <typename T>
__device__ __forceinline__ T opq_l(T v) {
  asm("" : "+v"(v));
  return v;
}

template <int N, typename T>
__device__ __forceinline__ T lsel(const T (&v)[N], int i) {
  T r = opq_l(v[0]);
#pragma unroll
  for (int k = 1; k < N; k++) r = (k == i) ? opq_l(v[k]) : r;
  return r;
}

template <int N, typename T>
__device__ __forceinline__ void lput(T (&v)[N], int i, T x) {
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = (k == i) ? x : v[k];
}

// R storage: packed upper triangle (row-major) followed by the first subdiagonal.
template <int NM>
struct RIdx {
  static constexpr int NUP = NM * (NM + 1) / 2;
  static constexpr int SIZE = NUP + NM - 1;
  // compile-time index of R[i][j]; -1 for entries that are always zero
  static constexpr int at(int i, int j) {
    return j >= i ? i * NM - i * (i - 1) / 2 + (j - i) : (i == j + 1 ? NUP + j : -1);
  }
};

template <int NM, int MM, int T>
__global__ void __launch_bounds__(64) qp_lane_kernel(const QpArgs a) {
  static_assert(MM <= 64, "bitmask bookkeeping holds m <= 64");
  using RI = RIdx<NM>;
  __shared__ double Jl[NM * NM * 64];

  const int lane = threadIdx.x;
  const int64_t b = (int64_t)blockIdx.x * 64 + lane;
  if (b >= a.batch) return;  // lanes are fully independent

#define JL(i, j) Jl[((i) * NM + (j)) * 64 + lane]

  const int n = a.n, p = a.p, m = a.m;
  const double inf = dinf();
  // per-QP views: element e of each block is at <base> + e*T (qbase, include/qpgpu.h layouts)
  const double* __restrict__ CIb = a.CI + qbase<T>(b, n * m);
  const double* __restrict__ ci0b = a.ci0 + qbase<T>(b, m);
  const double* __restrict__ CEb = a.CE + qbase<T>(b, n * p);
  const double* __restrict__ ce0b = a.ce0 + qbase<T>(b, p);

  int status = QPGPU_QP_OK;
  double fval = 0.0;
  int iter = 0;
  bool write_x = true;
  double xv[NM];
#pragma unroll
  for (int i = 0; i < NM; i++) xv[i] = 0.0;
  double c1 = 0.0, c2 = 0.0;

  // ---------------------------------------------------------------- setup (registers)
  bool chol_ok = true;
  double bad_sum = 0.0;
  {
    double Gr[NM][NM];
    const double* Gb = a.G + qbase<T>(b, n * n);
#pragma unroll
    for (int i = 0; i < NM; i++)
#pragma unroll
      for (int j = 0; j < NM; j++) Gr[i][j] = (i < n && j < n) ? Gb[(i * n + j) * T] : 0.0;
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) c1 += Gr[i][i];
    // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored
#pragma unroll
    for (int i = 0; i < NM; i++) {
      if (i < n && chol_ok) {
        double sum = Gr[i][i];
#pragma unroll
        for (int k = i - 1; k >= 0; k--) sum -= Gr[i][k] * Gr[i][k];
        if (sum <= 0.0) {
          chol_ok = false;
          bad_sum = sum;
        } else {
          const double dg = sqrt(sum);
          Gr[i][i] = dg;
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < n) {
              double s2 = Gr[i][j];
#pragma unroll
              for (int k = i - 1; k >= 0; k--) s2 -= Gr[i][k] * Gr[j][k];
              Gr[j][i] = s2 / dg;
            }
#pragma unroll
          for (int k = i + 1; k < NM; k++) Gr[i][k] = Gr[k][i];
        }
      }
    }
    if (a.flags & QPGPU_FLAG_WRITE_FACTOR) {
      double* Gw = a.G + qbase<T>(b, n * n);
#pragma unroll
      for (int i = 0; i < NM; i++)
#pragma unroll
        for (int j = 0; j < NM; j++)
          if (i < n && j < n) Gw[(i * n + j) * T] = Gr[i][j];
    }
    if (chol_ok) {
      // J = L^{-T}: row i of J = L^{-1} e_i (forward_elimination); c2 = trace(J)
#pragma unroll
      for (int r = 0; r < NM; r++) {
        if (r < n) {
          double y[NM];
#pragma unroll
          for (int i = 0; i < NM; i++) {
            double v = 0.0;
            if (i < n) {
              v = (i == r) ? 1.0 : 0.0;
#pragma unroll
              for (int j = 0; j < i; j++) v -= Gr[i][j] * y[j];
              v = v / Gr[i][i];
            }
            y[i] = v;
          }
#pragma unroll
          for (int j = 0; j < NM; j++) JL(r, j) = y[j];
          c2 += y[r];
        }
      }
      // cholesky_solve (@.text+0x31a2): x = -G^{-1} g0
      double g0v[NM], y[NM];
      const double* g0b = a.g0 + qbase<T>(b, n);
#pragma unroll
      for (int i = 0; i < NM; i++) g0v[i] = (i < n) ? g0b[i * T] : 0.0;
#pragma unroll
      for (int i = 0; i < NM; i++) {
        double v = 0.0;
        if (i < n) {
          v = g0v[i];
#pragma unroll
          for (int j = 0; j < i; j++) v -= Gr[i][j] * y[j];
          v = v / Gr[i][i];
        }
        y[i] = v;
      }
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        if (i < n) {
          double v = y[i];
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < n) v -= Gr[i][j] * xv[j];
          xv[i] = v / Gr[i][i];
        }
      }
#pragma unroll
      for (int i = 0; i < NM; i++) xv[i] = -xv[i];
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) fval += g0v[i] * xv[i];
      fval = 0.5 * fval;
    }
  }

  if (!chol_ok) {
    status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
    fval = bad_sum;
    write_x = false;
  } else {
    // ---------------------------------------------------------------- state
    double Rv[RI::SIZE];
#pragma unroll
    for (int i = 0; i < RI::SIZE; i++) Rv[i] = 0.0;
    double dv[NM], zv[NM], npv[NM], uv[NM + 1], rv[NM];
    int Av[NM + 1];
#pragma unroll
    for (int i = 0; i < NM; i++) dv[i] = zv[i] = npv[i] = rv[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= NM; i++) {
      uv[i] = 0.0;
      Av[i] = 0;
    }
    double R_norm = 1.0;
    int iq = 0;

    auto compute_d = [&]() {
#pragma unroll
      for (int c = 0; c < NM; c++) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NM; j++)
          if (j < n) s += JL(j, c) * npv[j];
        dv[c] = s;
      }
    };
    auto update_z = [&]() {
#pragma unroll
      for (int r = 0; r < NM; r++) {
        double z = 0.0;
#pragma unroll
        for (int j = 0; j < NM; j++)
          if (j >= iq && j < n) z += JL(r, j) * dv[j];
        zv[r] = z;
      }
    };
    auto update_r = [&]() {
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        if (i < iq) {
          double s = 0.0;
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < iq) s += Rv[RI::at(i, j)] * rv[j];
          rv[i] = (dv[i] - s) / Rv[RI::at(i, i)];
        }
      }
    };
    auto add_constraint = [&]() -> bool {
      if (iq >= n) return false;  // reference UB (p > n); reported as dependent
#pragma unroll
      for (int j = NM - 1; j >= 1; j--) {
        if (j <= n - 1 && j >= iq + 1) {
          double cc = dv[j - 1], ss = dv[j];
          const double h = qp_distance(cc, ss);
          if (!(fabs(h) < kEps)) {
            dv[j] = 0.0;
            ss = ss / h;
            cc = cc / h;
            if (cc < 0.0) {
              cc = -cc;
              ss = -ss;
              dv[j - 1] = -h;
            } else {
              dv[j - 1] = h;
            }
            const double xny = ss / (1.0 + cc);
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < n) {
                const double t1 = JL(k, j - 1), t2 = JL(k, j);
                const double n1 = t1 * cc + t2 * ss;
                JL(k, j - 1) = n1;
                JL(k, j) = xny * (t1 + n1) - t2;
              }
          }
        }
      }
      iq++;
      // R[:iq, iq-1] = d[:iq]
#pragma unroll
      for (int c = 0; c < NM; c++)
#pragma unroll
        for (int i = 0; i <= c; i++) {
          const bool w = (c == iq - 1);
          Rv[RI::at(i, c)] = w ? dv[i] : Rv[RI::at(i, c)];
        }
      const double dd = fabs(lsel<NM>(dv, iq - 1));
      if (dd <= kEps * R_norm) return false;
      R_norm = (R_norm < dd) ? dd : R_norm;
      return true;
    };
    auto delete_constraint = [&](int l) {
      int qq = 0;
      bool found = false;
#pragma unroll
      for (int k = 0; k <= NM; k++)
        if (!found && k >= p && k < iq && Av[k] == l) {
          qq = k;
          found = true;
        }
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i >= qq && i < iq - 1) {
          Av[i] = Av[i + 1];
          uv[i] = uv[i + 1];
        }
      // shift R columns left from qq (only upper + subdiagonal entries exist)
#pragma unroll
      for (int c = 0; c < NM - 1; c++) {
        const bool sh = (c >= qq && c < iq - 1);
#pragma unroll
        for (int r = 0; r <= c + 1 && r < NM; r++) {
          // destination R[r][c] (upper or subdiagonal), source R[r][c+1] (upper)
          Rv[RI::at(r, c)] = sh ? Rv[RI::at(r, c + 1)] : Rv[RI::at(r, c)];
        }
      }
      {
        const int aiq = lsel<NM + 1>(Av, iq);
        const double uiq = lsel<NM + 1>(uv, iq);
        lput<NM + 1>(Av, iq - 1, aiq);
        lput<NM + 1>(uv, iq - 1, uiq);
        lput<NM + 1>(Av, iq, 0);
        lput<NM + 1>(uv, iq, 0.0);
      }
      // R[j][iq-1] = 0 for j < iq
#pragma unroll
      for (int c = 0; c < NM; c++)
#pragma unroll
        for (int r = 0; r <= c + 1 && r < NM; r++) {
          const bool z = (c == iq - 1) && (r < iq);
          Rv[RI::at(r, c)] = z ? 0.0 : Rv[RI::at(r, c)];
        }
      iq--;
      if (iq == 0) return;
#pragma unroll
      for (int j = 0; j < NM - 1; j++) {
        if (j >= qq && j < iq) {
          double cc = Rv[RI::at(j, j)], ss = Rv[RI::at(j + 1, j)];
          const double h = qp_distance(cc, ss);
          if (!(fabs(h) < kEps)) {
            cc = cc / h;
            ss = ss / h;
            Rv[RI::at(j + 1, j)] = 0.0;
            if (cc < 0.0) {
              Rv[RI::at(j, j)] = -h;
              cc = -cc;
              ss = -ss;
            } else {
              Rv[RI::at(j, j)] = h;
            }
            const double xny = ss / (1.0 + cc);
#pragma unroll
            for (int k = j + 1; k < NM; k++)
              if (k < iq) {
                const double t1 = Rv[RI::at(j, k)], t2 = Rv[RI::at(j + 1, k)];
                const double r1 = t1 * cc + t2 * ss;
                Rv[RI::at(j, k)] = r1;
                Rv[RI::at(j + 1, k)] = xny * (t1 + r1) - t2;
              }
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < n) {
                const double t1 = JL(k, j), t2 = JL(k, j + 1);
                const double n1 = t1 * cc + t2 * ss;
                JL(k, j) = n1;
                JL(k, j + 1) = xny * (n1 + t1) - t2;
              }
          }
        }
      }
    };
    auto dot = [&](const double(&u_)[NM], const double(&v_)[NM]) -> double {
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) s += u_[i] * v_[i];
      return s;
    };

    // ---------------------------------------------------------------- equality phase
    bool done = false;
    for (int i = 0; i < p && !done; i++) {
#pragma unroll
      for (int j = 0; j < NM; j++) npv[j] = (j < n) ? CEb[(j * p + i) * T] : 0.0;
      compute_d();
      update_z();
      update_r();
      double t2 = 0.0;
      const double zz = dot(zv, zv);
      const double znp = dot(zv, npv);
      if (fabs(zz) > kEps) t2 = (-dot(npv, xv) - ce0b[i * T]) / znp;
#pragma unroll
      for (int k = 0; k < NM; k++) xv[k] += t2 * zv[k];
      lput<NM + 1>(uv, iq, t2);
#pragma unroll
      for (int k = 0; k < NM; k++)
        if (k < iq) uv[k] -= t2 * rv[k];
      fval += 0.5 * (t2 * t2) * znp;
      lput<NM + 1>(Av, i, -i - 1);
      if (!add_constraint()) {
        status = QPGPU_QP_DEPENDENT;
        done = true;
      }
    }

    // ---------------------------------------------------------------- active-set loop
    if (!done) {
      double sv[MM];
#pragma unroll
      for (int i = 0; i < MM; i++) sv[i] = 0.0;
      double xold[NM], uold[NM + 1];
      int aold[NM + 1];
#pragma unroll
      for (int i = 0; i < NM; i++) xold[i] = 0.0;
#pragma unroll
      for (int i = 0; i <= NM; i++) {
        uold[i] = 0.0;
        aold[i] = 0;
      }
      uint64_t act = 0;   // bit c set <=> iai[c] == -1
      uint64_t excl = 0;  // bit c set <=> iaexcl[c] == false
      int ip = 0, steps = 0;
      double ss = 0.0;
      bool need_scan = true, need_select = true;
      const int max_steps = a.max_steps;
      while (true) {
        if (need_scan) {  // ---- l1
          iter++;
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k >= p && k < iq) act |= 1ull << Av[k];
          // s = CI^T x + ci0, walking CI row by row (each s[i] sums j ascending)
#pragma unroll
          for (int i = 0; i < MM; i++) sv[i] = 0.0;
#pragma unroll
          for (int j = 0; j < NM; j++)
            if (j < n) {
              const double xj = xv[j];
#pragma unroll
              for (int i = 0; i < MM; i++)
                if (i < m) sv[i] += CIb[(j * m + i) * T] * xj;
            }
          double psi = 0.0;
#pragma unroll
          for (int i = 0; i < MM; i++)
            if (i < m) {
              sv[i] += ci0b[i * T];
              psi += (sv[i] < 0.0) ? sv[i] : 0.0;
            }
          excl = 0;
          ss = 0.0;
          ip = 0;
          if (fabs(psi) <= (double)m * kEps * c1 * c2 * 100.0) break;  // optimal
#pragma unroll
          for (int i = 0; i < NM; i++) {
            uold[i] = (i < iq) ? uv[i] : uold[i];
            aold[i] = (i < iq) ? Av[i] : aold[i];
            xold[i] = xv[i];
          }
        }
        if (need_select) {  // ---- l2 (ss deliberately not reset: reference quirk)
#pragma unroll
          for (int i = 0; i < MM; i++)
            if (i < m) {
              const bool elig = !((act >> i) & 1ull) && !((excl >> i) & 1ull);
              const bool take = sv[i] < ss && elig;
              ss = take ? sv[i] : ss;
              ip = take ? i : ip;
            }
          if (ss >= 0.0) break;  // optimal
#pragma unroll
          for (int j = 0; j < NM; j++) npv[j] = (j < n) ? CIb[(j * m + ip) * T] : 0.0;
          lput<NM + 1>(uv, iq, 0.0);
          lput<NM + 1>(Av, iq, ip);
        }
        // ---- l2a
        if (max_steps > 0 && ++steps > max_steps) {
          status = QPGPU_QP_MAX_ITER;
          break;
        }
        compute_d();
        update_z();
        update_r();
        int l = 0;
        double t1 = inf;
#pragma unroll
        for (int k = 0; k < NM; k++)
          if (k >= p && k < iq && rv[k] > 0.0) {
            const double q_ = uv[k] / rv[k];
            const bool take = q_ < t1;
            t1 = take ? q_ : t1;
            l = take ? opq_l(Av[k]) : l;
          }
        const double zz = dot(zv, zv);
        const double znp = dot(zv, npv);
        double t2;
        if (fabs(zz) > kEps) {
          t2 = -lsel<MM>(sv, ip) / znp;
          if (t2 < 0) t2 = inf;  // Takano Akio patch
        } else {
          t2 = inf;
        }
        const double t = (t2 < t1) ? t2 : t1;
        if (t >= inf) {
          status = QPGPU_QP_INFEASIBLE;
          fval = inf;
          break;
        }
        if (t2 >= inf) {  // dual step only
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k < iq) uv[k] -= t * rv[k];
          lput<NM + 1>(uv, iq, lsel<NM + 1>(uv, iq) + t);
          act &= ~(1ull << l);
          delete_constraint(l);
          need_scan = need_select = false;
          continue;
        }
#pragma unroll
        for (int k = 0; k < NM; k++) xv[k] += t * zv[k];
        fval += t * znp * (0.5 * t + lsel<NM + 1>(uv, iq));
#pragma unroll
        for (int k = 0; k < NM; k++)
          if (k < iq) uv[k] -= t * rv[k];
        lput<NM + 1>(uv, iq, lsel<NM + 1>(uv, iq) + t);
        if (fabs(t - t2) < kEps) {  // full step
          if (!add_constraint()) {
            excl |= 1ull << ip;
            delete_constraint(ip);
            act = 0;
#pragma unroll
            for (int i = 0; i < NM; i++)
              if (i >= p && i < iq) {
                Av[i] = aold[i];
                uv[i] = uold[i];
                act |= 1ull << Av[i];
              }
#pragma unroll
            for (int i = 0; i < NM; i++) xv[i] = xold[i];
            need_scan = false;
            need_select = true;
          } else {
            act |= 1ull << ip;
            need_scan = need_select = true;
          }
          continue;
        }
        // partial step: drop l, refresh s[ip]
        act &= ~(1ull << l);
        delete_constraint(l);
        {
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < NM; j++)
            if (j < n) s += CIb[(j * m + ip) * T] * xv[j];
          lput<MM>(sv, ip, s + ci0b[ip * T]);
        }
        need_scan = need_select = false;
      }
    }
  }
#undef JL

  if (write_x) {
    double* xb = a.x + qbase<T>(b, n);
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) xb[i * T] = xv[i];
  }
  a.f[b] = fval;
  a.status[b] = status;
  if (a.iters) a.iters[b] = iter;
}

template <int NM, int MM>
static hipError_t launch_lane(const QpArgs& a, hipStream_t stream) {
  const int64_t blocks = (a.batch + 63) / 64;
  if (a.tile == 64)
    hipLaunchKernelGGL((qp_lane_kernel<NM, MM, 64>), dim3((unsigned)blocks), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL((qp_lane_kernel<NM, MM, 1>), dim3((unsigned)blocks), dim3(64), 0, stream, a);
  return hipGetLastError();
}

struct LaneVariant {
  int nmax, mmax;
  const char* name;
  hipError_t (*launch)(const QpArgs&, hipStream_t);
};

static const LaneVariant kLaneVariants[] = {
    {7, 14, "qp_lane<N=7,M=14>", launch_lane<7, 14>},
    {8, 16, "qp_lane<N=8,M=16>", launch_lane<8, 16>},
};

const LaneVariant* pick_lane(int n, int m) {
  for (const auto& v : kLaneVariants)
    if (n <= v.nmax && m <= v.mmax) return &v;
  return nullptr;
}

}  // namespace qpk

extern "C" hipError_t qpk_launch_lane(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                      const char** name) {
  const qpk::LaneVariant* v = qpk::pick_lane(a->n, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  return v->launch(*a, stream);
}

extern "C" const char* qpk_lane_name(int n, int /*p*/, int m) {
  const qpk::LaneVariant* v = qpk::pick_lane(n, m);
  return v ? v->name : nullptr;
}
