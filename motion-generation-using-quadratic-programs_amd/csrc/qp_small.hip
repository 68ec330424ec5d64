// qp_small.hip — gfx950 batched Goldfarb–Idnani solver for small dense QPs (n <= 16).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; body in the
// prebuilt libquadprog.a, operation order fixed in SURVEY.md §3.2) for a batch of independent
// QPs, one QP per SUBGROUP of S lanes of a 64-lane wavefront (64/S QPs per wave).
//
// Work split inside a subgroup (lane ls = 0..S-1):
//   * rows k = ls + q*S of J (= L^{-T}) live in registers (Jr[q][:]); every Givens rotation of
//     add_constraint / delete_constraint is row-parallel, and update_z is a row-local dot;
//   * inequality columns c = ls + q*S of CI (and ci0) live in registers (CIr[q][:]); the
//     l1 scan s = CI^T x + ci0 is column-local;
//   * compute_d's column sums go through an LDS transpose (P) so each sum keeps the reference
//     order (j ascending); G/L and R live in LDS (R is touched column-wise by add_constraint
//     and row-pair-wise by delete_constraint);
//   * the O(n) serial state (x, z, d, np, u, r, A and every step length) is replicated in all
//     S lanes and computed redundantly — identical values, so every control decision is
//     subgroup-uniform and the subgroup never diverges internally.
// All replicated arrays are indexed with compile-time indices only (fully unrolled loops with
// run-time predicates), so nothing spills to scratch.  Arithmetic is IEEE binary64 with the
// reference's evaluation order and no contraction: results are bitwise identical to the CPU
// restatement (oracle/qp_oracle.c), which tests/ check.
#include "qp_common.h"

namespace qpk {

// Opaque copy of a register value.  Selecting among array elements that are still loads at
// InstCombine time gets rewritten into ONE load through a selected address, which pins the
// array in scratch memory; routing each element through an empty asm keeps it a register.
template <typename T>
__device__ __forceinline__ T opq(T v) {
  asm("" : "+v"(v));
  return v;
}

template <int N, typename T>
__device__ __forceinline__ T sel(const T (&v)[N], int i) {
  // unconditional selects: a conditional form lets the optimiser merge the chain back into
  // a run-time-indexed load, which sends the whole array to scratch.
  T r = opq(v[0]);
#pragma unroll
  for (int k = 1; k < N; k++) r = (k == i) ? opq(v[k]) : r;
  return r;
}

template <int N, typename T>
__device__ __forceinline__ void put(T (&v)[N], int i, T x) {
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = (k == i) ? x : v[k];
}

template <int S, int NM, int MM>
struct SmallCfg {
  static_assert(64 % S == 0, "S must divide 64");
  static_assert(MM <= 64, "bitmask bookkeeping holds m <= 64");
  static constexpr int QPW = 64 / S;            // QPs per wavefront
  static constexpr int RPL = (NM + S - 1) / S;  // J rows per lane
  static constexpr int CPL = (MM + S - 1) / S;  // CI columns per lane
  static constexpr int RS = NM + 1;             // LDS row stride (odd: conflict-free rows)
  static constexpr int OFF_R = 0;
  static constexpr int OFF_P = OFF_R + NM * RS;  // G / L during setup, then compute_d transpose
  static constexpr int OFF_S = OFF_P + NM * RS;  // s[m]
  static constexpr int OFF_D = OFF_S + MM;       // d exchange
  static constexpr int OFF_Z = OFF_D + NM;       // z exchange
  static constexpr int OFF_NP = OFF_Z + NM;      // np exchange
  static constexpr int OFF_XOLD = OFF_NP + NM;
  static constexpr int OFF_UOLD = OFF_XOLD + NM;
  static constexpr int OFF_AOLD = OFF_UOLD + NM + 1;
  static constexpr int RAW = OFF_AOLD + NM + 1;
  static constexpr int REGION = ((RAW + 31) / 32) * 32 + 1;  // odd stride between QPs
  static constexpr int LDS_DOUBLES = QPW * REGION;
};

template <int S, int NM, int MM>
__global__ void __launch_bounds__(64) qp_small_kernel(const QpArgs a) {
  using C = SmallCfg<S, NM, MM>;
  constexpr int RS = C::RS;
  constexpr int RPL = C::RPL;
  constexpr int CPL = C::CPL;
  __shared__ double lds_all[C::LDS_DOUBLES];

  const int lane = threadIdx.x;
  const int sg = lane / S;
  const int ls = lane - sg * S;
  const int64_t b = (int64_t)blockIdx.x * C::QPW + sg;
  if (b >= a.batch) return;  // the whole subgroup leaves together

  double* const Lq = lds_all + sg * C::REGION;
  double* const Rm = Lq + C::OFF_R;
  double* const Pm = Lq + C::OFF_P;
  double* const sb = Lq + C::OFF_S;
  double* const db = Lq + C::OFF_D;
  double* const zb = Lq + C::OFF_Z;
  double* const npb = Lq + C::OFF_NP;
  double* const xold = Lq + C::OFF_XOLD;
  double* const uold = Lq + C::OFF_UOLD;
  double* const aold = Lq + C::OFF_AOLD;

  const int n = a.n, p = a.p, m = a.m;
  const int T = a.tile;  // layout stride (include/qpgpu.h): 1 = QP-major, 64 = TILED64
  const double inf = dinf();
  const int64_t gbase = qbase_rt(b, n * n, T);

  // ---------------------------------------------------------------- loads
  {
    const double* Gb = a.G + gbase;
    for (int e = ls; e < n * n; e += S) {
      const int i = e / n;
      const int j = e - i * n;
      Pm[i * RS + j] = Gb[(int64_t)e * T];
    }
  }
  double CIr[CPL][NM];
  double ci0r[CPL];
  {
    const double* CIb = a.CI + qbase_rt(b, n * m, T);
    const double* ci0b = a.ci0 + qbase_rt(b, m, T);
#pragma unroll
    for (int q = 0; q < CPL; q++) {
      const int c = ls + q * S;
      const bool own = c < m;
#pragma unroll
      for (int j = 0; j < NM; j++) CIr[q][j] = (own && j < n) ? CIb[(int64_t)(j * m + c) * T] : 0.0;
      ci0r[q] = own ? ci0b[(int64_t)c * T] : 0.0;
    }
  }
  double g0v[NM];
#pragma unroll
  for (int i = 0; i < NM; i++) g0v[i] = (i < n) ? a.g0[qbase_rt(b, n, T) + (int64_t)i * T] : 0.0;
  sg_sync();

  int status = QPGPU_QP_OK;
  double fval = 0.0;
  int iter = 0;
  double xv[NM];
#pragma unroll
  for (int i = 0; i < NM; i++) xv[i] = 0.0;
  bool write_x = true;

  // c1 = trace(G) before factorisation
  double c1 = 0.0;
#pragma unroll
  for (int i = 0; i < NM; i++)
    if (i < n) c1 += Pm[i * RS + i];

  // ---------------------------------------------------------------- Cholesky (in LDS)
  // cholesky_decomposition @.text+0x2df0: row-wise, descending-k sums, upper mirrored.
  bool chol_ok = true;
  double bad_sum = 0.0;
  for (int i = 0; i < n; i++) {
    double sum = Pm[i * RS + i];
    for (int k = i - 1; k >= 0; k--) sum -= Pm[i * RS + k] * Pm[i * RS + k];
    if (sum <= 0.0) {
      chol_ok = false;
      bad_sum = sum;
      break;
    }
    const double dg = sqrt(sum);
    for (int j = i + 1 + ls; j < n; j += S) {
      double s2 = Pm[i * RS + j];
      for (int k = i - 1; k >= 0; k--) s2 -= Pm[i * RS + k] * Pm[j * RS + k];
      Pm[j * RS + i] = s2 / dg;
    }
    if (ls == 0) Pm[i * RS + i] = dg;
    sg_sync();
    for (int k = i + 1 + ls; k < n; k += S) Pm[i * RS + k] = Pm[k * RS + i];
    sg_sync();
  }
  if (a.flags & QPGPU_FLAG_WRITE_FACTOR) {
    double* Gb = a.G + gbase;
    for (int e = ls; e < n * n; e += S) {
      const int i = e / n;
      const int j = e - i * n;
      Gb[(int64_t)e * T] = Pm[i * RS + j];
    }
  }

  if (!chol_ok) {
    status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
    fval = bad_sum;
    write_x = false;
    if (a.x_eq && ls == 0) {
      a.f_eq[b] = fval;
      a.st_eq[b] = status;
    }
  } else {
    // ---------------------------------------------------------------- J = L^{-T}
    double Jr[RPL][NM];
#pragma unroll
    for (int q = 0; q < RPL; q++) {
      const int k = ls + q * S;
      double y[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) {
        double v = 0.0;
        if (i < n) {
          v = (i == k) ? 1.0 : 0.0;
#pragma unroll
          for (int j = 0; j < i; j++) v -= Pm[i * RS + j] * y[j];
          v = v / Pm[i * RS + i];
        }
        y[i] = v;
      }
#pragma unroll
      for (int j = 0; j < NM; j++) Jr[q][j] = (k < n) ? y[j] : 0.0;
    }
    // c2 = trace(J), summed in row order
#pragma unroll
    for (int q = 0; q < RPL; q++) {
      const int k = ls + q * S;
      if (k < n) db[k] = sel<NM>(Jr[q], k);
    }
    sg_sync();
    double c2 = 0.0;
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) c2 += db[i];

    // unconstrained minimiser: cholesky_solve (@.text+0x31a2), x = -G^{-1} g0
    {
      double y[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) {
        double v = 0.0;
        if (i < n) {
          v = g0v[i];
#pragma unroll
          for (int j = 0; j < i; j++) v -= Pm[i * RS + j] * y[j];
          v = v / Pm[i * RS + i];
        }
        y[i] = v;
      }
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        if (i < n) {
          double v = y[i];
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < n) v -= Pm[i * RS + j] * xv[j];
          xv[i] = v / Pm[i * RS + i];
        }
      }
#pragma unroll
      for (int i = 0; i < NM; i++) xv[i] = -xv[i];
    }
    fval = 0.0;
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) fval += g0v[i] * xv[i];
    fval = 0.5 * fval;
    sg_sync();  // all reads of L done before P is reused

    // R = 0
    for (int e = ls; e < NM * RS; e += S) Rm[e] = 0.0;
    sg_sync();

    // ---------------------------------------------------------------- replicated state
    double dv[NM], zv[NM], npv[NM], uv[NM + 1], rv[NM];
    int Av[NM + 1];
#pragma unroll
    for (int i = 0; i < NM; i++) dv[i] = zv[i] = npv[i] = rv[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= NM; i++) {
      uv[i] = 0.0;
      Av[i] = 0;
    }
    double npo[RPL];  // np at this lane's rows
    double R_norm = 1.0;
    int iq = 0;

    // compute_d: d[i] = sum_j J[j][i] np[j] (j ascending) via the LDS transpose P
    auto compute_d = [&]() {
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        const int k = ls + q * S;
        if (k < n) {
#pragma unroll
          for (int c = 0; c < NM; c++)
            if (c < n) Pm[k * RS + c] = Jr[q][c] * npo[q];
        }
      }
      sg_sync();
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        const int c = ls + q * S;
        if (c < n) {
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < NM; j++)
            if (j < n) s += Pm[j * RS + c];
          db[c] = s;
        }
      }
      sg_sync();
#pragma unroll
      for (int i = 0; i < NM; i++) dv[i] = (i < n) ? db[i] : 0.0;
      sg_sync();
    };
    // update_z: z[i] = sum_{j>=iq} J[i][j] d[j] (row-local), then all-gathered
    auto update_z = [&]() {
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        const int k = ls + q * S;
        double z = 0.0;
#pragma unroll
        for (int j = 0; j < NM; j++)
          if (j >= iq && j < n) z += Jr[q][j] * dv[j];
        if (k < n) zb[k] = z;
      }
      sg_sync();
#pragma unroll
      for (int i = 0; i < NM; i++) zv[i] = (i < n) ? zb[i] : 0.0;
      sg_sync();
    };
    // update_r: r = R[lo:iq, lo:iq]^{-1} d[lo:iq], back substitution (replicated).  Only the
    // inequality rows (lo = p) are computed: the equality constraints' rows feed only their
    // multipliers u[0..p), which nothing reads (t1, the dual step's drop and the rollback use the
    // inequalities' u; x and f never use u), and r[i] for i >= p does not depend on the rows
    // below.  For the same reason the equality phase runs none.
    auto update_r = [&](int lo) {
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        if (i >= lo && i < iq) {
          double s = 0.0;
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < iq) s += Rm[i * RS + j] * rv[j];
          rv[i] = (dv[i] - s) / Rm[i * RS + i];
        }
      }
    };
    // add_constraint (@.text+0x21fd)
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
            for (int q = 0; q < RPL; q++) {
              const double t1 = Jr[q][j - 1], t2 = Jr[q][j];
              Jr[q][j - 1] = t1 * cc + t2 * ss;
              Jr[q][j] = xny * (t1 + Jr[q][j - 1]) - t2;
            }
          }
        }
      }
      iq++;
      if (ls == 0) {
#pragma unroll
        for (int i = 0; i < NM; i++)
          if (i < iq) Rm[i * RS + iq - 1] = dv[i];
      }
      sg_sync();
      const double dd = fabs(sel<NM>(dv, iq - 1));
      if (dd <= kEps * R_norm) return false;
      R_norm = (R_norm < dd) ? dd : R_norm;
      return true;
    };
    // delete_constraint (@.text+0x26a8)
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
      for (int j = ls; j < n; j += S)
        for (int i = qq; i < iq - 1; i++) Rm[j * RS + i] = Rm[j * RS + i + 1];
      {
        const int aiq = sel<NM + 1>(Av, iq);
        const double uiq = sel<NM + 1>(uv, iq);
        put<NM + 1>(Av, iq - 1, aiq);
        put<NM + 1>(uv, iq - 1, uiq);
        put<NM + 1>(Av, iq, 0);
        put<NM + 1>(uv, iq, 0.0);
      }
      for (int j = ls; j < iq; j += S) Rm[j * RS + iq - 1] = 0.0;
      iq--;
      sg_sync();
      if (iq == 0) return;
#pragma unroll
      for (int j = 0; j < NM - 1; j++) {
        if (j >= qq && j < iq) {
          double cc = Rm[j * RS + j], ss = Rm[(j + 1) * RS + j];
          const double h = qp_distance(cc, ss);
          if (!(fabs(h) < kEps)) {
            cc = cc / h;
            ss = ss / h;
            double nd;
            if (cc < 0.0) {
              nd = -h;
              cc = -cc;
              ss = -ss;
            } else {
              nd = h;
            }
            const double xny = ss / (1.0 + cc);
            for (int k = j + 1 + ls; k < iq; k += S) {
              const double t1 = Rm[j * RS + k], t2 = Rm[(j + 1) * RS + k];
              const double r1 = t1 * cc + t2 * ss;
              Rm[j * RS + k] = r1;
              Rm[(j + 1) * RS + k] = xny * (t1 + r1) - t2;
            }
            if (ls == 0) {
              Rm[(j + 1) * RS + j] = 0.0;
              Rm[j * RS + j] = nd;
            }
#pragma unroll
            for (int q = 0; q < RPL; q++) {
              const double t1 = Jr[q][j], t2 = Jr[q][j + 1];
              Jr[q][j] = t1 * cc + t2 * ss;
              Jr[q][j + 1] = xny * (Jr[q][j] + t1) - t2;
            }
          }
          sg_sync();
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
      const double* CEb = a.CE + qbase_rt(b, n * p, T);
#pragma unroll
      for (int j = 0; j < NM; j++) npv[j] = (j < n) ? CEb[(int64_t)(j * p + i) * T] : 0.0;
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        const int k = ls + q * S;
        npo[q] = (k < n) ? CEb[(int64_t)(k * p + i) * T] : 0.0;
      }
      compute_d();
      update_z();
      double t2 = 0.0;
      const double zz = dot(zv, zv);
      const double znp = dot(zv, npv);
      if (fabs(zz) > kEps) t2 = (-dot(npv, xv) - a.ce0[qbase_rt(b, p, T) + (int64_t)i * T]) / znp;
#pragma unroll
      for (int k = 0; k < NM; k++) xv[k] += t2 * zv[k];
      put<NM + 1>(uv, iq, t2);
      fval += 0.5 * (t2 * t2) * znp;
      put<NM + 1>(Av, i, -i - 1);
      if (!add_constraint()) {
        status = QPGPU_QP_DEPENDENT;
        done = true;
      }
    }
    if (a.x_eq) {  // the m = 0 answer: an empty l1 scan returns right here
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n && (i % S) == ls) a.x_eq[qbase_rt(b, n, T) + (int64_t)i * T] = xv[i];
      if (ls == 0) {
        a.f_eq[b] = fval;
        a.st_eq[b] = status;
      }
    }

    // ---------------------------------------------------------------- active-set loop
    if (!done) {
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
#pragma unroll
          for (int q = 0; q < CPL; q++) {
            const int c = ls + q * S;
            if (c < m) {
              double s = 0.0;
#pragma unroll
              for (int j = 0; j < NM; j++)
                if (j < n) s += CIr[q][j] * xv[j];
              s += ci0r[q];
              sb[c] = s;
            }
          }
          sg_sync();
          excl = 0;
          ss = 0.0;
          ip = 0;
          double psi = 0.0;
#pragma unroll
          for (int i = 0; i < MM; i++)
            if (i < m) {
              const double si = sb[i];
              psi += (si < 0.0) ? si : 0.0;
            }
          if (fabs(psi) <= (double)m * kEps * c1 * c2 * 100.0) break;  // optimal
          if (ls == 0) {
#pragma unroll
            for (int i = 0; i < NM; i++) {
              if (i < iq) {
                uold[i] = uv[i];
                aold[i] = (double)Av[i];
              }
              xold[i] = xv[i];
            }
          }
          sg_sync();
        }
        if (need_select) {  // ---- l2 (ss deliberately not reset: reference quirk)
#pragma unroll
          for (int i = 0; i < MM; i++)
            if (i < m) {
              const double si = sb[i];
              const bool elig = !((act >> i) & 1ull) && !((excl >> i) & 1ull);
              if (si < ss && elig) {
                ss = si;
                ip = i;
              }
            }
          if (ss >= 0.0) break;  // optimal
          if ((ip % S) == ls) {
            const int qs = ip / S;
#pragma unroll
            for (int j = 0; j < NM; j++)
              if (j < n) {
                double v = opq(CIr[0][j]);
#pragma unroll
                for (int q = 1; q < CPL; q++) v = (q == qs) ? opq(CIr[q][j]) : v;
                npb[j] = v;
              }
          }
          sg_sync();
#pragma unroll
          for (int i = 0; i < NM; i++) npv[i] = (i < n) ? npb[i] : 0.0;
#pragma unroll
          for (int q = 0; q < RPL; q++) {
            const int k = ls + q * S;
            npo[q] = (k < n) ? npb[k] : 0.0;
          }
          sg_sync();
          put<NM + 1>(uv, iq, 0.0);
          put<NM + 1>(Av, iq, ip);
        }
        // ---- l2a
        if (max_steps > 0 && ++steps > max_steps) {
          status = QPGPU_QP_MAX_ITER;
          break;
        }
        compute_d();
        update_z();
        update_r(p);
        int l = 0;
        double t1 = inf;
#pragma unroll
        for (int k = 0; k < NM; k++)
          if (k >= p && k < iq && rv[k] > 0.0) {
            const double q_ = uv[k] / rv[k];
            const bool take = q_ < t1;
            t1 = take ? q_ : t1;
            l = take ? opq(Av[k]) : l;
          }
        const double zz = dot(zv, zv);
        const double znp = dot(zv, npv);
        double t2;
        if (fabs(zz) > kEps) {
          t2 = -sb[ip] / znp;
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
            if (k >= p && k < iq) uv[k] -= t * rv[k];
          put<NM + 1>(uv, iq, sel<NM + 1>(uv, iq) + t);
          act &= ~(1ull << l);
          delete_constraint(l);
          need_scan = need_select = false;
          continue;
        }
        // primal and dual step
#pragma unroll
        for (int k = 0; k < NM; k++) xv[k] += t * zv[k];
        fval += t * znp * (0.5 * t + sel<NM + 1>(uv, iq));
#pragma unroll
        for (int k = 0; k < NM; k++)
          if (k >= p && k < iq) uv[k] -= t * rv[k];
        put<NM + 1>(uv, iq, sel<NM + 1>(uv, iq) + t);
        if (fabs(t - t2) < kEps) {  // full step
          if (!add_constraint()) {
            excl |= 1ull << ip;
            delete_constraint(ip);
            act = 0;
#pragma unroll
            for (int i = 0; i < NM; i++)
              if (i >= p && i < iq) {
                Av[i] = (int)aold[i];
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
        if ((ip % S) == ls) {
          const int qs = ip / S;
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < NM; j++)
            if (j < n) {
              double v = opq(CIr[0][j]);
#pragma unroll
              for (int q = 1; q < CPL; q++) v = (q == qs) ? opq(CIr[q][j]) : v;
              s += v * xv[j];
            }
          double c0 = opq(ci0r[0]);
#pragma unroll
          for (int q = 1; q < CPL; q++) c0 = (q == qs) ? opq(ci0r[q]) : c0;
          sb[ip] = s + c0;
        }
        sg_sync();
        need_scan = need_select = false;
      }
    }
  }

  // ---------------------------------------------------------------- outputs
  if (write_x) {
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n && (i % S) == ls) a.x[qbase_rt(b, n, T) + (int64_t)i * T] = xv[i];
  }
  if (ls == 0) {
    a.f[b] = fval;
    a.status[b] = status;
    if (a.iters) a.iters[b] = iter;
  }
}

// ------------------------------------------------------------------------------------------
// launch table
// ------------------------------------------------------------------------------------------
template <int S, int NM, int MM>
static hipError_t launch_small(const QpArgs& a, hipStream_t stream) {
  using C = SmallCfg<S, NM, MM>;
  const int64_t blocks = (a.batch + C::QPW - 1) / C::QPW;
  hipLaunchKernelGGL((qp_small_kernel<S, NM, MM>), dim3((unsigned)blocks), dim3(64), 0, stream,
                     a);
  return hipGetLastError();
}

struct SmallVariant {
  int nmax, mmax;
  const char* name;
  hipError_t (*launch)(const QpArgs&, hipStream_t);
};

static const SmallVariant kSmallVariants[] = {
    {8, 16, "qp_small<S=8,N=8,M=16>", launch_small<8, 8, 16>},
    {8, 32, "qp_small<S=8,N=8,M=32>", launch_small<8, 8, 32>},
    {16, 32, "qp_small<S=16,N=16,M=32>", launch_small<16, 16, 32>},
    {16, 64, "qp_small<S=16,N=16,M=64>", launch_small<16, 16, 64>},
};

const SmallVariant* pick_small(int n, int /*p*/, int m) {
  for (const auto& v : kSmallVariants)
    if (n <= v.nmax && m <= v.mmax) return &v;  // any p: iq never exceeds n
  return nullptr;
}

}  // namespace qpk

// exported to qpgpu_api.cpp (internal linkage boundary of the library)
extern "C" hipError_t qpk_launch_small(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                       const char** name) {
  const qpk::SmallVariant* v = qpk::pick_small(a->n, a->p, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  return v->launch(*a, stream);
}

extern "C" const char* qpk_small_name(int n, int p, int m) {
  const qpk::SmallVariant* v = qpk::pick_small(n, p, m);
  return v ? v->name : nullptr;
}
