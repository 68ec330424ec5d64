// TEST HARNESS ONLY — never part of the product.
//
// Provides the two solver entry points the controller calls (the drop-in solve_quadprog and
// qpgpu_solve_batched_host) on top of the CPU oracle (oracle/qp_oracle.c), so that the
// controller's host logic (builder, hierarchy, batching, retry, exception mapping) can be
// tested in the CPU suite.  Linked with the controller sources into
// tests/_build/libmgqp_cpu_harness.so; the shipped libmgqp_amd.so links the GPU libraries and
// has no such path.
#include <cmath>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <vector>

#include "qpgpu.h"
#include "quadprog_amd/QuadProg++.hh"

extern "C" int qpo_solve(int n, int p, int m, double* G, const double* g0, const double* CE,
                         const double* ce0, const double* CI, const double* ci0, double* x,
                         double* f, int* iters, int max_steps);

double solve_quadprog(Matrix<double>& G, Vector<double>& g0, const Matrix<double>& CE,
                      const Vector<double>& ce0, const Matrix<double>& CI,
                      const Vector<double>& ci0, Vector<double>& x) {
  const int n = G.ncols(), p = CE.ncols(), m = CI.ncols();
  std::vector<double> g(n * n), ce(n * p), ci(n * m), xx(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) g[i * n + j] = G[i][j];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < p; ++j) ce[i * p + j] = CE[i][j];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) ci[i * m + j] = CI[i][j];
  double f = 0;
  int it = 0;
  const int st = qpo_solve(n, p, m, g.data(), &g0[0], p ? ce.data() : nullptr,
                           p ? &ce0[0] : nullptr, m ? ci.data() : nullptr, m ? &ci0[0] : nullptr,
                           xx.data(), &f, &it, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) G[i][j] = g[i * n + j];
  x.resize(n);
  for (int i = 0; i < n; ++i) x[i] = xx[i];
  if (st == QPGPU_QP_DEPENDENT) throw std::runtime_error("Constraints are linearly dependent");
  if (st == QPGPU_QP_NOT_POSITIVE_DEFINITE) {
    std::ostringstream os;
    os << "Error in cholesky decomposition, sum: " << f;
    throw std::logic_error(os.str());
  }
  return f;
}

extern "C" {
static const char* g_err = "";
const char* qpgpu_last_error(void) { return g_err; }

int qpgpu_solve_batched_host(const qpgpu_problem_desc* d, double* G, const double* g0,
                             const double* CE, const double* ce0, const double* CI,
                             const double* ci0, double* x, double* f, int32_t* status,
                             int32_t* iters) {
  const int n = d->n, p = d->p, m = d->m;
  for (int64_t b = 0; b < d->batch; ++b) {
    std::vector<double> g(G + b * n * n, G + (b + 1) * n * n);
    int it = 0;
    status[b] = qpo_solve(n, p, m, g.data(), g0 + b * n, p ? CE + b * n * p : nullptr,
                          p ? ce0 + b * p : nullptr, m ? CI + b * n * m : nullptr,
                          m ? ci0 + b * m : nullptr, x + b * n, f + b, &it, 0);
    if (iters) iters[b] = it;
  }
  return QPGPU_SUCCESS;
}
}
