/*
 * qp_oracle.c — CPU restatement of the reference QuadProg++ solve_quadprog().
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *   The product (libqpgpu.so / libquadprog_amd.so) never links or calls it.
 *
 * What it restates.  The reference links a prebuilt static archive,
 * /root/reference/lib/QuadProgpp/libquadprog.a (CMakeLists.txt:95), whose source is not in the
 * repository.  Its interface and contract are the text at include/QuadProgpp/QuadProg++.hh:1-72;
 * its algorithm is Di Gaspero's QuadProg++ (~1.2.x, namespace renamed to ArrayHH), i.e. the
 * Goldfarb–Idnani dual active-set method (Math. Prog. 27 (1983) 1-33).  The operation order
 * below follows SURVEY.md §3.2, which fixed it by reading the archive's disassembly
 * (archive symbol offsets are cited per function as libquadprog.a(QuadProg++.o)@.text+0xNNN).
 * Every floating-point operation is evaluated in the same order with IEEE binary64 and no
 * contraction (build with -ffp-contract=off; x86-64 SSE2 has no FMA without -march).
 *
 * Parity pinning.  The archive may not be executed in this project (it is prebuilt machine
 * code shipped inside the reference), and the reference holds no tests or fixtures
 * (SURVEY.md §4).  The oracle is pinned by (i) the one archive output recorded in SURVEY.md §4
 * (the QuadProg++ demo problem: f = 12, x = [1, 2.0000000000000009]) and (ii) independent
 * KKT-certificate checks in tests/.  DESIGN.md calls this "partially pinned".
 *
 * Divergences, on inputs where the reference has undefined behaviour only:
 *   - n == 0 is rejected (the reference reads b[0]/L[0][0] out of bounds);
 *   - add_constraint() with iq == n reports "dependent" instead of writing R[i][n] out of
 *     bounds (only reachable with p > n);
 *   - an optional cap on active-set steps (max_steps > 0) reports QPGPU_QP_MAX_ITER; the
 *     reference has no cap.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/qpgpu.h"

#define QPO_EPS DBL_EPSILON /* std::numeric_limits<double>::epsilon(), .rodata +0x190 */

/* Operation counts (SURVEY.md §8(d) "Algorithmic flops": the restatement counts the operations
 * it actually executes, per config and seed).  Built into a separate library with -DQPO_COUNT
 * (liboracle_qp_count.so); the timed / parity oracle has no counting code.  Counted are the
 * binary64 operations the reference's evaluation performs: multiplications, additions and
 * subtractions, divisions and square roots (negation, fabs, comparisons and min/max are not
 * arithmetic and are not counted; the reference has no fused multiply-add).  Per thread. */
#ifdef QPO_COUNT
static __thread uint64_t qpo_cnt_mul, qpo_cnt_add, qpo_cnt_div, qpo_cnt_sqrt;
#define CNT(mul, add, div, sq) \
  (qpo_cnt_mul += (uint64_t)(mul), qpo_cnt_add += (uint64_t)(add), qpo_cnt_div += (uint64_t)(div), \
   qpo_cnt_sqrt += (uint64_t)(sq))
void qpo_op_counts(uint64_t out[4]) {
  out[0] = qpo_cnt_mul;
  out[1] = qpo_cnt_add;
  out[2] = qpo_cnt_div;
  out[3] = qpo_cnt_sqrt;
  qpo_cnt_mul = qpo_cnt_add = qpo_cnt_div = qpo_cnt_sqrt = 0;
}
#else
#define CNT(mul, add, div, sq) ((void)0)
#endif

#ifdef QPO_TRACE
void (*qpo_trace_cb)(int n, const double *x) = 0;
#endif

/* distance(a, b): overflow-safe hypot, three branches (weak symbol `distance`). */
static double qpo_distance(double a, double b) {
  double a1 = fabs(a), b1 = fabs(b), t;
  if (a1 > b1) {
    CNT(2, 1, 1, 1);
    t = b1 / a1;
    return a1 * sqrt(1.0 + t * t);
  } else if (b1 > a1) {
    CNT(2, 1, 1, 1);
    t = a1 / b1;
    return b1 * sqrt(1.0 + t * t);
  }
  CNT(1, 0, 0, 0);
  return a1 * 1.4142135623730951; /* a1 * sqrt(2.0), constant at .rodata +0x1e8 */
}

/* scalar_product: left-to-right sum starting at 0.0. */
static double qpo_dot(int n, const double *a, const double *b) {
  double s = 0.0;
  CNT(n, n, 0, 0);
  for (int i = 0; i < n; i++) s += a[i] * b[i];
  return s;
}

/* cholesky_decomposition (@.text+0x2df0): row-wise, descending-k inner sums, then mirror.
 * Returns 0 on success, 1 (and the failing pivot in *bad_sum) when sum <= 0. */
static int qpo_cholesky(int n, double *A, double *bad_sum) {
  for (int i = 0; i < n; i++) {
    for (int j = i; j < n; j++) {
      double sum = A[i * n + j];
      CNT(i, i, i == j ? 0 : 1, i == j ? 1 : 0);
      for (int k = i - 1; k >= 0; k--) sum -= A[i * n + k] * A[j * n + k];
      if (i == j) {
        if (sum <= 0.0) {
          *bad_sum = sum;
          return 1;
        }
        A[i * n + i] = sqrt(sum);
      } else {
        A[j * n + i] = sum / A[i * n + i];
      }
    }
    for (int k = i + 1; k < n; k++) A[i * n + k] = A[k * n + i];
  }
  return 0;
}

/* forward_elimination: L y = b, L lower (row-major n x n). */
static void qpo_forward(int n, const double *L, double *y, const double *b) {
  CNT((int64_t)n * (n - 1) / 2, (int64_t)n * (n - 1) / 2, n, 0);
  y[0] = b[0] / L[0];
  for (int i = 1; i < n; i++) {
    y[i] = b[i];
    for (int j = 0; j < i; j++) y[i] -= L[i * n + j] * y[j];
    y[i] = y[i] / L[i * n + i];
  }
}

/* backward_elimination: U x = y with U = the mirrored upper triangle. */
static void qpo_backward(int n, const double *U, double *x, const double *y) {
  CNT((int64_t)n * (n - 1) / 2, (int64_t)n * (n - 1) / 2, n, 0);
  x[n - 1] = y[n - 1] / U[(n - 1) * n + (n - 1)];
  for (int i = n - 2; i >= 0; i--) {
    x[i] = y[i];
    for (int j = i + 1; j < n; j++) x[i] -= U[i * n + j] * x[j];
    x[i] = x[i] / U[i * n + i];
  }
}

/* compute_d: d = J^T np, column dots with j ascending. */
static void qpo_compute_d(int n, double *d, const double *J, const double *np) {
  CNT((int64_t)n * n, (int64_t)n * n, 0, 0);
  for (int i = 0; i < n; i++) {
    double sum = 0.0;
    for (int j = 0; j < n; j++) sum += J[j * n + i] * np[j];
    d[i] = sum;
  }
}

/* update_z: z = J[:, iq:] d[iq:]. */
static void qpo_update_z(int n, double *z, const double *J, const double *d, int iq) {
  CNT((int64_t)n * (n - iq), (int64_t)n * (n - iq), 0, 0);
  for (int i = 0; i < n; i++) {
    z[i] = 0.0;
    for (int j = iq; j < n; j++) z[i] += J[i * n + j] * d[j];
  }
}

/* update_r: r = R[:iq,:iq]^{-1} d[:iq] (upper back-substitution). */
static void qpo_update_r(int n, const double *R, double *r, const double *d, int iq) {
  for (int i = iq - 1; i >= 0; i--) {
    double sum = 0.0;
    CNT(iq - 1 - i, iq - i, 1, 0);
    for (int j = i + 1; j < iq; j++) sum += R[i * n + j] * r[j];
    r[i] = (d[i] - sum) / R[i * n + i];
  }
}

/* add_constraint (@.text+0x21fd): Givens sweep j = n-1 .. iq+1 zeroing d[j] while rotating
 * columns (j-1, j) of J; then R[:iq, iq-1] = d and the degeneracy test. */
static int qpo_add_constraint(int n, double *R, double *J, double *d, int *iq, double *R_norm) {
  if (*iq >= n) return 0; /* UB in the reference (R[i][n]); see header */
  for (int j = n - 1; j >= *iq + 1; j--) {
    double cc = d[j - 1], ss = d[j];
    double h = qpo_distance(cc, ss);
    if (fabs(h) < QPO_EPS) continue;
    CNT(3 * n, 1 + 3 * n, 3, 0);
    d[j] = 0.0;
    ss = ss / h;
    cc = cc / h;
    if (cc < 0.0) {
      cc = -cc;
      ss = -ss;
      d[j - 1] = -h;
    } else {
      d[j - 1] = h;
    }
    double xny = ss / (1.0 + cc);
    for (int k = 0; k < n; k++) {
      double t1 = J[k * n + j - 1], t2 = J[k * n + j];
      J[k * n + j - 1] = t1 * cc + t2 * ss;
      J[k * n + j] = xny * (t1 + J[k * n + j - 1]) - t2;
    }
  }
  (*iq)++;
  for (int i = 0; i < *iq; i++) R[i * n + *iq - 1] = d[i];
  if (fabs(d[*iq - 1]) <= QPO_EPS * *R_norm) return 0; /* degenerate */
  double ad = fabs(d[*iq - 1]);
  *R_norm = (*R_norm < ad) ? ad : *R_norm; /* std::max<double>(R_norm, |d|) */
  return 1;
}

/* delete_constraint (@.text+0x26a8): drop active constraint l (no "non existing constraint"
 * check in this archive: qq stays 0 if l is absent), shift A/u/R columns, re-triangularise R
 * with Givens on rows (j, j+1) and rotate the same columns of J. */
static void qpo_delete_constraint(int n, double *R, double *J, int *A, double *u, int p, int *iq,
                                  int l) {
  int qq = 0;
  for (int i = p; i < *iq; i++)
    if (A[i] == l) {
      qq = i;
      break;
    }
  for (int i = qq; i < *iq - 1; i++) {
    A[i] = A[i + 1];
    u[i] = u[i + 1];
    for (int j = 0; j < n; j++) R[j * n + i] = R[j * n + i + 1];
  }
  A[*iq - 1] = A[*iq];
  u[*iq - 1] = u[*iq];
  A[*iq] = 0;
  u[*iq] = 0.0;
  for (int j = 0; j < *iq; j++) R[j * n + *iq - 1] = 0.0;
  (*iq)--;
  if (*iq == 0) return;
  for (int j = qq; j < *iq; j++) {
    double cc = R[j * n + j], ss = R[(j + 1) * n + j];
    double h = qpo_distance(cc, ss);
    if (fabs(h) < QPO_EPS) continue;
    CNT(3 * (*iq - j - 1) + 3 * n, 1 + 3 * (*iq - j - 1) + 3 * n, 3, 0);
    cc = cc / h;
    ss = ss / h;
    R[(j + 1) * n + j] = 0.0;
    if (cc < 0.0) {
      R[j * n + j] = -h;
      cc = -cc;
      ss = -ss;
    } else {
      R[j * n + j] = h;
    }
    double xny = ss / (1.0 + cc);
    for (int k = j + 1; k < *iq; k++) {
      double t1 = R[j * n + k], t2 = R[(j + 1) * n + k];
      R[j * n + k] = t1 * cc + t2 * ss;
      R[(j + 1) * n + k] = xny * (t1 + R[j * n + k]) - t2;
    }
    for (int k = 0; k < n; k++) {
      double t1 = J[k * n + j], t2 = J[k * n + j + 1];
      J[k * n + j] = t1 * cc + t2 * ss;
      J[k * n + j + 1] = xny * (J[k * n + j] + t1) - t2;
    }
  }
}

/*
 * qpo_solve — one QP, semantics of solve_quadprog (@.text+0x0).
 * G (n x n, row-major) is overwritten with the Cholesky factor (L mirrored), like the reference.
 * Returns a qpgpu_qp_status; *f gets the reference's return value (or the failing pivot for
 * NOT_POSITIVE_DEFINITE).  *iters = number of l1 passes (the reference's `iter`).
 * max_steps <= 0: no cap (reference behaviour).
 */
int qpo_solve(int n, int p, int m, double *G, const double *g0, const double *CE,
              const double *ce0, const double *CI, const double *ci0, double *x, double *f,
              int *iters, int max_steps) {
  const double inf = INFINITY;
  const int mp = m + p;
  int status = QPGPU_QP_OK;
  *iters = 0;
  if (n <= 0 || p < 0 || m < 0) return -1;

  /* workspace (Vector/Matrix temporaries of the reference, sized as there) */
  size_t nn = (size_t)n * n;
  double *R = (double *)calloc(nn, sizeof(double));
  double *J = (double *)calloc(nn, sizeof(double));
  double *dbl = (double *)calloc((size_t)4 * (mp + 1) + (size_t)5 * n, sizeof(double));
  int *ibuf = (int *)calloc((size_t)3 * (mp + 1), sizeof(int));
  unsigned char *iaexcl = (unsigned char *)calloc((size_t)mp + 1, 1);
  double *s = dbl, *r = s + (mp + 1), *u = r + (mp + 1), *u_old = u + (mp + 1);
  double *z = u_old + (mp + 1), *d = z + n, *np = d + n, *x_old = np + n, *tmp = x_old + n;
  int *A = ibuf, *A_old = A + (mp + 1), *iai = A_old + (mp + 1);

  double f_value, psi, c1, c2, ss, R_norm, t, t1, t2, sum;
  int iq, ip, l, iter = 0, steps = 0;

  /* c1 = trace(G) before factorisation */
  c1 = 0.0;
  CNT(0, n, 0, 0);
  for (int i = 0; i < n; i++) c1 += G[i * n + i];
  {
    double bad;
    if (qpo_cholesky(n, G, &bad)) {
      *f = bad;
      status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
      goto done;
    }
  }
  for (int i = 0; i < n; i++) d[i] = 0.0;
  R_norm = 1.0;
  /* J = L^{-T}: row i of J is L^{-1} e_i; c2 = trace(J) */
  c2 = 0.0;
  for (int i = 0; i < n; i++) {
    d[i] = 1.0;
    qpo_forward(n, G, z, d);
    for (int j = 0; j < n; j++) J[i * n + j] = z[j];
    CNT(0, 1, 0, 0);
    c2 += z[i];
    d[i] = 0.0;
  }
  /* unconstrained minimiser x = -G^{-1} g0 (cholesky_solve @.text+0x31a2) */
  qpo_forward(n, G, tmp, g0);
  qpo_backward(n, G, x, tmp);
  for (int i = 0; i < n; i++) x[i] = -x[i];
  CNT(1, 0, 0, 0);
  f_value = 0.5 * qpo_dot(n, g0, x);

  /* equality constraints */
  iq = 0;
  for (int i = 0; i < p; i++) {
    for (int j = 0; j < n; j++) np[j] = CE[j * p + i];
    qpo_compute_d(n, d, J, np);
    qpo_update_z(n, z, J, d, iq);
    qpo_update_r(n, R, r, d, iq);
    t2 = 0.0;
    if (fabs(qpo_dot(n, z, z)) > QPO_EPS) {
      CNT(0, 1, 1, 0);
      t2 = (-qpo_dot(n, np, x) - ce0[i]) / qpo_dot(n, z, np);
    }
    CNT(n + iq + 3, n + iq + 1, 0, 0);
    for (int k = 0; k < n; k++) x[k] += t2 * z[k];
    u[iq] = t2;
    for (int k = 0; k < iq; k++) u[k] -= t2 * r[k];
    f_value += 0.5 * (t2 * t2) * qpo_dot(n, z, np);
    A[i] = -i - 1;
    if (!qpo_add_constraint(n, R, J, d, &iq, &R_norm)) {
      *f = f_value;
      status = QPGPU_QP_DEPENDENT;
      goto done;
    }
  }

  for (int i = 0; i < m; i++) iai[i] = i;

l1:
  iter++;
#ifdef QPO_TRACE
  /* tools/lazy_scan_sim.py: x at every l1 pass (a separate build; the oracle has no hook) */
  if (qpo_trace_cb) qpo_trace_cb(n, x);
#endif
  for (int i = p; i < iq; i++) {
    ip = A[i];
    iai[ip] = -1;
  }
  ss = 0.0;
  psi = 0.0;
  ip = 0;
  CNT((int64_t)m * n + 4, (int64_t)m * (n + 2), 0, 0);
  for (int i = 0; i < m; i++) {
    iaexcl[i] = 1;
    sum = 0.0;
    for (int j = 0; j < n; j++) sum += CI[j * m + i] * x[j];
    sum += ci0[i];
    s[i] = sum;
    psi += (sum < 0.0) ? sum : 0.0; /* std::min(0.0, sum) */
  }
  if (fabs(psi) <= (double)m * QPO_EPS * c1 * c2 * 100.0) {
    *f = f_value;
    goto done;
  }
  for (int i = 0; i < iq; i++) {
    u_old[i] = u[i];
    A_old[i] = A[i];
  }
  for (int i = 0; i < n; i++) x_old[i] = x[i];

l2:
  for (int i = 0; i < m; i++) {
    if (s[i] < ss && iai[i] != -1 && iaexcl[i]) {
      ss = s[i];
      ip = i;
    }
  }
  if (ss >= 0.0) {
    *f = f_value;
    goto done;
  }
  for (int i = 0; i < n; i++) np[i] = CI[i * m + ip];
  u[iq] = 0.0;
  A[iq] = ip;

l2a:
  if (max_steps > 0 && ++steps > max_steps) {
    *f = f_value;
    status = QPGPU_QP_MAX_ITER;
    goto done;
  }
  qpo_compute_d(n, d, J, np);
  qpo_update_z(n, z, J, d, iq);
  qpo_update_r(n, R, r, d, iq);
  l = 0;
  t1 = inf;
  for (int k = p; k < iq; k++) {
    if (r[k] > 0.0) {
      CNT(0, 0, 1, 0);
      if (u[k] / r[k] < t1) {
        CNT(0, 0, 1, 0);
        t1 = u[k] / r[k];
        l = A[k];
      }
    }
  }
  if (fabs(qpo_dot(n, z, z)) > QPO_EPS) {
    CNT(0, 0, 1, 0);
    t2 = -s[ip] / qpo_dot(n, z, np);
    if (t2 < 0) t2 = inf; /* Takano Akio patch */
  } else {
    t2 = inf;
  }
  t = (t2 < t1) ? t2 : t1; /* std::min(t1, t2) */
  if (t >= inf) {
    *f = inf;
    status = QPGPU_QP_INFEASIBLE;
    goto done;
  }
  if (t2 >= inf) {
    /* dual step only */
    CNT(iq, iq + 1, 0, 0);
    for (int k = 0; k < iq; k++) u[k] -= t * r[k];
    u[iq] += t;
    iai[l] = l;
    qpo_delete_constraint(n, R, J, A, u, p, &iq, l);
    goto l2a;
  }
  /* primal and dual step */
  CNT(n + 3 + iq, n + 2 + iq + 2, 0, 0);
  for (int k = 0; k < n; k++) x[k] += t * z[k];
  f_value += t * qpo_dot(n, z, np) * (0.5 * t + u[iq]);
  for (int k = 0; k < iq; k++) u[k] -= t * r[k];
  u[iq] += t;
  if (fabs(t - t2) < QPO_EPS) {
    /* full step */
    if (!qpo_add_constraint(n, R, J, d, &iq, &R_norm)) {
      iaexcl[ip] = 0;
      qpo_delete_constraint(n, R, J, A, u, p, &iq, ip);
      for (int i = 0; i < m; i++) iai[i] = i;
      for (int i = p; i < iq; i++) {
        A[i] = A_old[i];
        u[i] = u_old[i];
        iai[A[i]] = -1;
      }
      for (int i = 0; i < n; i++) x[i] = x_old[i];
      goto l2;
    } else {
      iai[ip] = -1;
    }
    goto l1;
  }
  /* partial step: drop constraint l */
  iai[l] = l;
  qpo_delete_constraint(n, R, J, A, u, p, &iq, l);
  sum = 0.0;
  CNT(n, n + 1, 0, 0);
  for (int k = 0; k < n; k++) sum += CI[k * m + ip] * x[k];
  s[ip] = sum + ci0[ip];
  goto l2a;

done:
  *iters = iter;
  free(R);
  free(J);
  free(dbl);
  free(ibuf);
  free(iaexcl);
  return status;
}

/* Batched driver over the qpgpu.h layout; `threads` host threads over contiguous shards. */
typedef struct {
  int n, p, m, max_steps, write_factor;
  int64_t b0, b1;
  const double *G, *g0, *CE, *ce0, *CI, *ci0;
  double *x, *f;
  int32_t *status, *iters;
} qpo_job;

static void *qpo_worker(void *arg) {
  qpo_job *j = (qpo_job *)arg;
  const int n = j->n, p = j->p, m = j->m;
  double *Gw = (double *)malloc((size_t)n * n * sizeof(double));
  for (int64_t b = j->b0; b < j->b1; b++) {
    double *Gb = j->write_factor ? (double *)j->G + b * n * n : Gw;
    if (!j->write_factor) memcpy(Gw, j->G + b * n * n, (size_t)n * n * sizeof(double));
    int it = 0;
    int st = qpo_solve(n, p, m, Gb, j->g0 + b * n, j->CE + b * n * p, j->ce0 + b * p,
                       j->CI + b * n * m, j->ci0 + b * m, j->x + b * n, j->f + b, &it,
                       j->max_steps);
    j->status[b] = st;
    if (j->iters) j->iters[b] = it;
  }
  free(Gw);
  return NULL;
}

int qpo_solve_batch(int64_t batch, int n, int p, int m, double *G, const double *g0,
                    const double *CE, const double *ce0, const double *CI, const double *ci0,
                    double *x, double *f, int32_t *status, int32_t *iters, int write_factor,
                    int max_steps, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if ((int64_t)threads > batch) threads = batch > 0 ? (int)batch : 1;
  qpo_job jobs[256];
  pthread_t tid[256];
  for (int t = 0; t < threads; t++) {
    qpo_job *j = &jobs[t];
    j->n = n; j->p = p; j->m = m; j->max_steps = max_steps; j->write_factor = write_factor;
    j->b0 = batch * t / threads;
    j->b1 = batch * (t + 1) / threads;
    j->G = G; j->g0 = g0; j->CE = CE; j->ce0 = ce0; j->CI = CI; j->ci0 = ci0;
    j->x = x; j->f = f; j->status = status; j->iters = iters;
  }
  if (threads == 1) {
    qpo_worker(&jobs[0]);
    return 0;
  }
  for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, qpo_worker, &jobs[t]);
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  return 0;
}
