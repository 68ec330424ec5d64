// qp_generic.hip — gfx950 batched Goldfarb–Idnani solver for QPs of ANY size (the shapes the
// register / LDS / n <= 256 kernels do not cover: n > 256 or m > 1024).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72, which accepts any
// n, p, m; operation order of the prebuilt libquadprog.a fixed in SURVEY.md §3.2 and restated in
// oracle/qp_oracle.c) for one QP per 256-thread workgroup, with every per-QP array — J, R (the
// factor L during the setup), x, z, d, np, r, u, s, A, iai, iaexcl and the rollback copies — in
// a global workspace sized at run time from (n, m), so the shape has no compile-time bound.
//
// Division of work (every element keeps the reference's operations in the reference's order,
// so results are bitwise identical to the CPU restatement):
//   * thread 0 ("lead") runs the serial chains: the Cholesky pivots, the back-substitutions
//     (cholesky_solve, update_r), the scalar products, the Givens coefficients of
//     add_constraint / delete_constraint and the active-set bookkeeping;
//   * the threads share the independent element loops: the Cholesky column below each pivot,
//     the rows of J = L^-T, compute_d (thread = column of J), update_z (thread = row), the
//     rotations of J's rows (each thread carries its row through the whole sweep), the l1 scan
//     (thread = constraint) and the vector updates.
// J is column-major (J[r][c] at c*n + r), so update_z and the row rotations read and write it
// coalesced across threads.  The kernel is the correctness path for large shapes: it keeps the
// reference's serial dependences rather than restructuring them, and is not tuned.
#include <type_traits>

#include "qp_common.h"

namespace qpk {

constexpr int kGenBS = 256;  // threads per workgroup (one QP)
constexpr int kGU = 8;       // operand loads batched per chunk of a sequential sum (qp_common.h)

// per-QP workspace layout (doubles), from the launch's (n, m)
struct GenLay {
  int64_t J, R, x, z, d, np, r, xo, u, uo, gc, s, ints, flags, per_qp;
};
__host__ __device__ inline GenLay gen_lay(int n, int m) {
  GenLay L;
  const int64_t nn = (int64_t)n * n;
  L.J = 0;
  L.R = nn;
  L.x = 2 * nn;
  L.z = L.x + n;
  L.d = L.z + n;
  L.np = L.d + n;
  L.r = L.np + n;
  L.xo = L.r + n;
  L.u = L.xo + n;
  L.uo = L.u + n + 1;
  L.gc = L.uo + n + 1;  // Givens coefficients: (cc, ss, xny, applied) per rotation, n rotations
  L.s = L.gc + 4 * (int64_t)n;
  L.ints = L.s + m;  // int A[n+1], A_old[n+1], iai[m]
  L.flags = L.ints + (2 * (int64_t)(n + 1) + m + 1) / 2;  // uint8 iaexcl[m]
  L.per_qp = (L.flags + (m + 7) / 8 + 1) | 1;
  return L;
}

struct GenCtl {
  double f, c1, c2, R_norm, ss, t, t1, t2, psi, dg;
  int status, iq, ip, l, iter, steps, phase, ok, qq, ng;
};

enum : int { G_DONE = 0, G_L1 = 1, G_L2 = 2, G_L2A = 3 };

__global__ void __launch_bounds__(kGenBS) qp_generic_kernel(const QpArgs a, double* __restrict__ ws) {
  __shared__ GenCtl c;
  const int tid = threadIdx.x;
  const bool lead = tid == 0;
  const int64_t b = blockIdx.x;
  const int n = a.n, p = a.p, m = a.m, T = a.tile;
  const GenLay Ly = gen_lay(n, m);
  double* const W = ws + b * Ly.per_qp;
  double* const Jm = W + Ly.J;
  double* const Rm = W + Ly.R;
  double* const xv = W + Ly.x;
  double* const zv = W + Ly.z;
  double* const dv = W + Ly.d;
  double* const npv = W + Ly.np;
  double* const rv = W + Ly.r;
  double* const xo = W + Ly.xo;
  double* const uv = W + Ly.u;
  double* const uo = W + Ly.uo;
  double* const gc = W + Ly.gc;
  double* const sv = W + Ly.s;
  int* const Av = reinterpret_cast<int*>(W + Ly.ints);
  int* const Ao = Av + n + 1;
  int* const iai = Ao + n + 1;
  uint8_t* const exc = reinterpret_cast<uint8_t*>(W + Ly.flags);  // iaexcl[i]
#define J_(r_, c_) Jm[(int64_t)(c_) * n + (r_)]
#define R_(i_, j_) Rm[(int64_t)(i_) * n + (j_)]
#define EL(ptr, e) (ptr)[(int64_t)(e) * T]
  const double* Gb = a.G + qbase_rt(b, (int64_t)n * n, T);
  const double* g0b = a.g0 + qbase_rt(b, n, T);
  const double* CEb = a.CE + qbase_rt(b, (int64_t)n * p, T);
  const double* ce0b = a.ce0 + qbase_rt(b, p, T);
  const double* CIb = a.CI + qbase_rt(b, (int64_t)n * m, T);
  const double* ci0b = a.ci0 + qbase_rt(b, m, T);
  const double inf = dinf();
  const int64_t nn = (int64_t)n * n;

  // ---------------------------------------------------------------- setup
  // G -> R (the factor L lives there until J and x are built)
  for (int64_t e = tid; e < nn; e += kGenBS) Rm[e] = EL(Gb, e);
  __syncthreads();
  if (lead) {
    double c1 = 0.0;  // trace(G) before the factorisation
    for (int i = 0; i < n; i++) c1 += R_(i, i);
    c.c1 = c1;
    c.status = QPGPU_QP_OK;
    c.iter = 0;
    c.steps = 0;
  }
  // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored
  for (int i = 0; i < n; i++) {
    if (lead) {
      const double sum = seq_fms_down<kGU>(R_(i, i), 0, i, [&](int k) { return R_(i, k); },
                                           [&](int k) { return R_(i, k); });
      if (sum <= 0.0) {
        c.status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
        c.f = sum;
      } else {
        c.dg = sqrt(sum);
      }
    }
    __syncthreads();
    if (c.status != QPGPU_QP_OK) break;
    const double dg = c.dg;
    for (int j = i + 1 + tid; j < n; j += kGenBS) {
      const double sum = seq_fms_down<kGU>(R_(i, j), 0, i, [&](int k) { return R_(i, k); },
                                           [&](int k) { return R_(j, k); });
      R_(j, i) = sum / dg;
    }
    if (lead) R_(i, i) = dg;
    __syncthreads();
    for (int k = i + 1 + tid; k < n; k += kGenBS) R_(i, k) = R_(k, i);
    __syncthreads();
  }
  if (a.flags & QPGPU_FLAG_WRITE_FACTOR) {  // G <- the reference's G after the call
    double* Gw = a.G + qbase_rt(b, (int64_t)n * n, T);
    for (int64_t e = tid; e < nn; e += kGenBS) EL(Gw, e) = Rm[e];
  }
  const bool chol_ok = c.status == QPGPU_QP_OK;
  if (chol_ok) {
    // J = L^{-T}: row r of J is L^{-1} e_r (forward_elimination, j ascending)
    for (int r = tid; r < n; r += kGenBS)
      for (int i = 0; i < n; i++) {
        const double v = seq_fms_up<kGU>((i == r) ? 1.0 : 0.0, 0, i, [&](int j) { return R_(i, j); },
                                         [&](int j) { return J_(r, j); });
        J_(r, i) = v / R_(i, i);
      }
    __syncthreads();
    if (lead) {
      double c2 = 0.0;
      for (int i = 0; i < n; i++) c2 += J_(i, i);
      c.c2 = c2;
      // cholesky_solve (@.text+0x31a2): forward into d, backward into x, x = -x
      for (int i = 0; i < n; i++) {
        const double v = seq_fms_up<kGU>(EL(g0b, i), 0, i, [&](int j) { return R_(i, j); },
                                         [&](int j) { return dv[j]; });
        dv[i] = v / R_(i, i);
      }
      for (int i = n - 1; i >= 0; i--) {
        const double v = seq_fms_up<kGU>(dv[i], i + 1, n, [&](int j) { return R_(i, j); },
                                         [&](int j) { return xv[j]; });
        xv[i] = v / R_(i, i);
      }
      double f = 0.0;
      for (int i = 0; i < n; i++) {
        xv[i] = -xv[i];
        f += EL(g0b, i) * xv[i];
      }
      c.f = 0.5 * f;
      c.R_norm = 1.0;
      c.iq = 0;
    }
    __syncthreads();
    // R = 0, u = 0, A = 0, d = 0 (the reference's fresh workspace)
    for (int64_t e = tid; e < nn; e += kGenBS) Rm[e] = 0.0;
    for (int i = tid; i <= n; i += kGenBS) {
      uv[i] = 0.0;
      Av[i] = 0;
      if (i < n) dv[i] = 0.0;
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- shared steps
  auto compute_d = [&]() {  // d = J^T np, j ascending (thread = column)
    for (int col = tid; col < n; col += kGenBS)
      dv[col] = seq_fma_up<kGU>(0.0, 0, n, [&](int j) { return J_(j, col); }, [&](int j) { return npv[j]; });
    __syncthreads();
  };
  auto update_z = [&](int iq) {  // z = J[:, iq:] d[iq:] (thread = row)
    for (int r = tid; r < n; r += kGenBS)
      zv[r] = seq_fma_up<kGU>(0.0, iq, n, [&](int j) { return J_(r, j); }, [&](int j) { return dv[j]; });
    __syncthreads();
  };
  // r = R[p:iq, p:iq]^{-1} d[p:iq] (lead): the inequality rows only — the equality constraints'
  // rows feed only their multipliers u[0..p), which nothing reads (t1, the dual step's drop and
  // the rollback use the inequalities' u; x and f never use u), and r[i] for i >= p does not
  // depend on the rows below.  For the same reason the equality phase runs none.
  auto update_r = [&](int iq) {
    if (lead)
      for (int i = iq - 1; i >= p; i--) {
        const double s = seq_fma_up<kGU>(0.0, i + 1, iq, [&](int j) { return R_(i, j); },
                                         [&](int j) { return rv[j]; });
        rv[i] = (dv[i] - s) / R_(i, i);
      }
    __syncthreads();
  };
  auto dot = [&](const double* u_, const double* v_) {
    return seq_fma_up<kGU>(0.0, 0, n, [&](int i) { return u_[i]; }, [&](int i) { return v_[i]; });
  };
  // The recorded rotations applied to every row of J, each thread carrying its rows through the
  // sweep in rotation order (one load and one store per column; a chunk's J entries and
  // coefficients are loaded before its stores).  add_constraint: rotation g maps
  // (J[k][j-1], J[k][j]), j = n-1-g, to (n1, xny (t1 + n1) - t2) and n1 is the next rotation's
  // t2; delete_constraint: rotation g maps (J[k][j], J[k][j+1]), j = qq+g, to
  // (n1, xny (n1 + t1) - t2) and the second is the next rotation's t1.  A skipped rotation
  // (|h| < eps) leaves both columns unchanged.
  auto sweep_add = [&](int ng) {
    for (int k = tid; k < n; k += kGenBS) {
      double carry = J_(k, n - 1);
      for (int gb = 0; gb < ng; gb += kGU) {
        double t1v[kGU], cv[kGU], sw[kGU], xw[kGU];
        bool fw[kGU];
#pragma unroll
        for (int u = 0; u < kGU; u++) {
          const int g = gb + u < ng ? gb + u : ng - 1;
          t1v[u] = J_(k, n - 2 - g);
          cv[u] = gc[4 * g];
          sw[u] = gc[4 * g + 1];
          xw[u] = gc[4 * g + 2];
          fw[u] = gc[4 * g + 3] != 0.0;
        }
#pragma unroll
        for (int u = 0; u < kGU; u++)
          if (gb + u < ng) {
            const double t1 = t1v[u], t2 = carry;
            const double n1 = t1 * cv[u] + t2 * sw[u];
            J_(k, n - 1 - gb - u) = fw[u] ? xw[u] * (t1 + n1) - t2 : t2;
            carry = fw[u] ? n1 : t1;
          }
      }
      J_(k, n - 1 - ng) = carry;
    }
    __syncthreads();
  };
  auto sweep_delete = [&](int ng, int qq) {
    for (int k = tid; k < n; k += kGenBS) {
      double carry = J_(k, qq);
      for (int gb = 0; gb < ng; gb += kGU) {
        double t2v[kGU], cv[kGU], sw[kGU], xw[kGU];
        bool fw[kGU];
#pragma unroll
        for (int u = 0; u < kGU; u++) {
          const int g = gb + u < ng ? gb + u : ng - 1;
          t2v[u] = J_(k, qq + g + 1);
          cv[u] = gc[4 * g];
          sw[u] = gc[4 * g + 1];
          xw[u] = gc[4 * g + 2];
          fw[u] = gc[4 * g + 3] != 0.0;
        }
#pragma unroll
        for (int u = 0; u < kGU; u++)
          if (gb + u < ng) {
            const double t1 = carry, t2 = t2v[u];
            const double n1 = t1 * cv[u] + t2 * sw[u];
            J_(k, qq + gb + u) = fw[u] ? n1 : t1;
            carry = fw[u] ? xw[u] * (n1 + t1) - t2 : t2;
          }
      }
      J_(k, qq + ng) = carry;
    }
    __syncthreads();
  };
  // add_constraint (@.text+0x21fd): the lead runs the d-chain (which reads no J) and records
  // every rotation; the threads then rotate their rows of J; R's new column and the degeneracy
  // test.  Leaves 1 (added) or 0 (degenerate / iq == n) in c.ok.
  auto add_constraint = [&]() {
    const int iq0 = c.iq;
    if (lead) {
      int ng = 0;
      if (iq0 < n)
        for (int j = n - 1; j >= iq0 + 1; j--, ng++) {
          double cc = dv[j - 1], ss = dv[j];
          const double h = qp_distance(cc, ss);
          gc[4 * ng + 3] = 0.0;
          if (fabs(h) < kEps) continue;
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
          gc[4 * ng] = cc;
          gc[4 * ng + 1] = ss;
          gc[4 * ng + 2] = ss / (1.0 + cc);
          gc[4 * ng + 3] = 1.0;
        }
      c.ng = ng;
    }
    __syncthreads();
    if (iq0 < n) sweep_add(c.ng);
    if (iq0 < n)
      for (int i = tid; i <= iq0; i += kGenBS) R_(i, iq0) = dv[i];  // R[:iq, iq-1] = d[:iq]
    __syncthreads();
    if (lead) {
      if (iq0 >= n) {
        c.ok = 0;  // reference UB (p > n): reported as dependent (oracle/qp_oracle.c)
      } else {
        const int iq = iq0 + 1;
        c.iq = iq;
        const double ad = fabs(dv[iq - 1]);
        if (ad <= kEps * c.R_norm) {
          c.ok = 0;
        } else {
          c.R_norm = (c.R_norm < ad) ? ad : c.R_norm;
          c.ok = 1;
        }
      }
    }
    __syncthreads();
  };
  // delete_constraint (@.text+0x26a8) of constraint l
  auto delete_constraint = [&](int l) {
    if (lead) {
      const int iq = c.iq;
      int qq = 0;
      for (int i = p; i < iq; i++)
        if (Av[i] == l) {
          qq = i;
          break;
        }
      for (int i = qq; i < iq - 1; i++) {
        Av[i] = Av[i + 1];
        uv[i] = uv[i + 1];
      }
      Av[iq - 1] = Av[iq];
      uv[iq - 1] = uv[iq];
      Av[iq] = 0;
      uv[iq] = 0.0;
      c.qq = qq;
    }
    __syncthreads();
    {
      const int iq = c.iq, qq = c.qq;
      for (int j = tid; j < n; j += kGenBS) {  // shift R's columns left from qq (row j)
        for (int i = qq; i < iq - 1; i++) R_(j, i) = R_(j, i + 1);
        if (j < iq) R_(j, iq - 1) = 0.0;
      }
    }
    __syncthreads();
    if (lead) {
      const int iq = --c.iq, qq = c.qq;
      int ng = 0;
      if (iq > 0)
        for (int j = qq; j < iq; j++, ng++) {
          double cc = R_(j, j), ss = R_(j + 1, j);
          const double h = qp_distance(cc, ss);
          gc[4 * ng + 3] = 0.0;
          if (fabs(h) < kEps) continue;
          cc = cc / h;
          ss = ss / h;
          R_(j + 1, j) = 0.0;
          if (cc < 0.0) {
            R_(j, j) = -h;
            cc = -cc;
            ss = -ss;
          } else {
            R_(j, j) = h;
          }
          const double xny = ss / (1.0 + cc);
          for (int k = j + 1; k < iq; k++) {
            const double t1 = R_(j, k), t2 = R_(j + 1, k);
            const double r1 = t1 * cc + t2 * ss;
            R_(j, k) = r1;
            R_(j + 1, k) = xny * (t1 + r1) - t2;
          }
          gc[4 * ng] = cc;
          gc[4 * ng + 1] = ss;
          gc[4 * ng + 2] = xny;
          gc[4 * ng + 3] = 1.0;
        }
      c.ng = ng;
    }
    __syncthreads();
    sweep_delete(c.ng, c.qq);
  };

  // ---------------------------------------------------------------- equality phase
  if (chol_ok) {
    for (int i = 0; i < p; i++) {
      for (int j = tid; j < n; j += kGenBS) npv[j] = EL(CEb, (int64_t)j * p + i);
      __syncthreads();
      const int iq = c.iq;
      compute_d();
      update_z(iq);
      if (lead) {
        double t2 = 0.0;
        if (fabs(dot(zv, zv)) > kEps) t2 = (-dot(npv, xv) - EL(ce0b, i)) / dot(zv, npv);
        c.t2 = t2;
        uv[iq] = t2;
        c.f += 0.5 * (t2 * t2) * dot(zv, npv);
        Av[i] = -i - 1;
      }
      __syncthreads();
      {
        const double t2 = c.t2;
        for (int k = tid; k < n; k += kGenBS) xv[k] += t2 * zv[k];
      }
      __syncthreads();
      add_constraint();
      if (!c.ok) {
        if (lead) c.status = QPGPU_QP_DEPENDENT;
        __syncthreads();
        break;
      }
    }
  }
  if (a.x_eq) {  // the m = 0 answer (qpgpu_solve_batched_eq): an empty l1 scan returns here
    if (c.status != QPGPU_QP_NOT_POSITIVE_DEFINITE) {
      double* xb = a.x_eq + qbase_rt(b, n, T);
      for (int i = tid; i < n; i += kGenBS) EL(xb, i) = xv[i];
    }
    if (lead) {
      a.f_eq[b] = c.f;
      a.st_eq[b] = c.status;
    }
  }
  if (lead) c.phase = c.status == QPGPU_QP_OK ? G_L1 : G_DONE;
  for (int i = tid; i < m; i += kGenBS) iai[i] = i;
  __syncthreads();

  // ---------------------------------------------------------------- active-set loop
  const int max_steps = a.max_steps;
  while (c.phase != G_DONE) {
    if (c.phase == G_L1) {
      // ---- l1: s = CI^T x + ci0 (thread = constraint, j ascending), psi in i order (lead)
      if (lead) {
        c.iter++;
        for (int i = p; i < c.iq; i++) iai[Av[i]] = -1;
      }
      for (int i = tid; i < m; i += kGenBS) {
        exc[i] = 1;
        const double c0 = EL(ci0b, i);
        double s = seq_fma_up<kGU>(0.0, 0, n, [&](int j) { return EL(CIb, (int64_t)j * m + i); },
                                   [&](int j) { return xv[j]; });
        s += c0;
        sv[i] = s;
      }
      __syncthreads();
      if (lead) {
        double psi = 0.0;
        for (int i = 0; i < m; i++) psi += (sv[i] < 0.0) ? sv[i] : 0.0;
        c.ss = 0.0;
        c.ip = 0;
        if (fabs(psi) <= (double)m * kEps * c.c1 * c.c2 * 100.0) {
          c.phase = G_DONE;
        } else {
          for (int i = 0; i < c.iq; i++) {
            uo[i] = uv[i];
            Ao[i] = Av[i];
          }
          c.phase = G_L2;
        }
      }
      for (int i = tid; i < n; i += kGenBS) xo[i] = xv[i];  // (unused when optimal)
      __syncthreads();
      continue;
    }
    if (c.phase == G_L2) {
      // ---- l2 (ss deliberately not reset: reference quirk)
      if (lead) {
        double ss = c.ss;
        int ip = c.ip;
        for (int i = 0; i < m; i++)
          if (sv[i] < ss && iai[i] != -1 && exc[i]) {
            ss = sv[i];
            ip = i;
          }
        c.ss = ss;
        c.ip = ip;
        if (ss >= 0.0) {
          c.phase = G_DONE;
        } else {
          uv[c.iq] = 0.0;
          Av[c.iq] = ip;
          c.phase = G_L2A;
        }
      }
      __syncthreads();
      if (c.phase == G_L2A) {
        const int ip = c.ip;
        for (int j = tid; j < n; j += kGenBS) npv[j] = EL(CIb, (int64_t)j * m + ip);
      }
      __syncthreads();
      continue;
    }
    // ---- l2a
    if (lead && max_steps > 0 && ++c.steps > max_steps) {
      c.status = QPGPU_QP_MAX_ITER;
      c.phase = G_DONE;
    }
    __syncthreads();
    if (c.phase == G_DONE) break;
    const int iq = c.iq;
    compute_d();
    update_z(iq);
    update_r(iq);
    if (lead) {
      int l = 0;
      double t1 = inf;
      for (int k = p; k < iq; k++)
        if (rv[k] > 0.0 && uv[k] / rv[k] < t1) {
          t1 = uv[k] / rv[k];
          l = Av[k];
        }
      double t2;
      if (fabs(dot(zv, zv)) > kEps) {
        t2 = -sv[c.ip] / dot(zv, npv);
        if (t2 < 0) t2 = inf;  // Takano Akio patch
      } else {
        t2 = inf;
      }
      const double t = (t2 < t1) ? t2 : t1;
      c.t = t;
      c.t1 = t1;
      c.t2 = t2;
      c.l = l;
      if (t >= inf) {
        c.status = QPGPU_QP_INFEASIBLE;
        c.f = inf;
        c.phase = G_DONE;
      } else if (t2 >= inf) {  // dual step
        for (int k = p; k < iq; k++) uv[k] -= t * rv[k];
        uv[iq] += t;
        iai[l] = l;
        c.ok = 2;
      } else {  // primal and dual step
        c.f += t * dot(zv, npv) * (0.5 * t + uv[iq]);
        for (int k = p; k < iq; k++) uv[k] -= t * rv[k];
        uv[iq] += t;
        c.ok = fabs(t - t2) < kEps ? 3 : 4;
      }
    }
    __syncthreads();
    if (c.phase == G_DONE) break;
    const int kind = c.ok;
    if (kind == 2) {
      delete_constraint(c.l);
      continue;  // l2a
    }
    {
      const double t = c.t;
      for (int k = tid; k < n; k += kGenBS) xv[k] += t * zv[k];
    }
    __syncthreads();
    if (kind == 3) {  // full step
      add_constraint();
      if (!c.ok) {
        const int ip = c.ip;
        if (lead) exc[ip] = 0;
        __syncthreads();
        delete_constraint(ip);
        for (int i = tid; i < m; i += kGenBS) iai[i] = i;
        __syncthreads();
        if (lead)
          for (int i = p; i < c.iq; i++) {
            Av[i] = Ao[i];
            uv[i] = uo[i];
            iai[Av[i]] = -1;
          }
        for (int i = tid; i < n; i += kGenBS) xv[i] = xo[i];
        if (lead) c.phase = G_L2;
      } else {
        if (lead) {
          iai[c.ip] = -1;
          c.phase = G_L1;
        }
      }
      __syncthreads();
      continue;
    }
    // partial step: drop l, refresh s[ip]
    if (lead) iai[c.l] = c.l;
    __syncthreads();
    delete_constraint(c.l);
    if (lead) {
      const int ip = c.ip;
      const double s = seq_fma_up<kGU>(0.0, 0, n, [&](int k) { return EL(CIb, (int64_t)k * m + ip); },
                                       [&](int k) { return xv[k]; });
      sv[ip] = s + EL(ci0b, ip);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- outputs
  if (c.status != QPGPU_QP_NOT_POSITIVE_DEFINITE) {
    double* xb = a.x + qbase_rt(b, n, T);
    for (int i = tid; i < n; i += kGenBS) EL(xb, i) = xv[i];
  }
  if (lead) {
    a.f[b] = c.f;
    a.status[b] = c.status;
    if (a.iters) a.iters[b] = c.iter;
  }
#undef J_
#undef R_
#undef EL
}

}  // namespace qpk

// Largest shape the generic kernel accepts: n*n and the workspace offsets stay within int64 and a
// QP's workspace within 2^34 doubles (128 GiB); int32 element indices of the inputs (n*n, n*m).
// CE offsets (n*p, j*p + i) are computed in int64, so p is not bounded here.
extern "C" int qpk_generic_covers(int n, int m) {
  return n >= 1 && m >= 0 && (int64_t)n * n < ((int64_t)1 << 31) && (int64_t)n * m < ((int64_t)1 << 31);
}
extern "C" int64_t qpk_generic_workspace_bytes(int n, int m, int64_t batch) {
  return qpk::gen_lay(n, m).per_qp * 8 * batch;
}
extern "C" const char* qpk_generic_name(int n, int /*p*/, int m) {
  return qpk_generic_covers(n, m) ? "qp_generic<BS=256,global workspace>" : nullptr;
}
extern "C" hipError_t qpk_launch_generic(const qpk::QpArgs* a, hipStream_t stream, double* ws) {
  if (a->batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(qpk::qp_generic_kernel, dim3((unsigned)a->batch), dim3(qpk::kGenBS), 0, stream, *a, ws);
  return hipGetLastError();
}
