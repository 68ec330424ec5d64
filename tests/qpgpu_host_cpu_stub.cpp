// TEST HARNESS ONLY — never part of the product.
//
// The C-ABI host entry point (include/qpgpu.h qpgpu_solve_batched_host) on top of the CPU
// restatement (oracle/qp_oracle.c), with the product's semantics for what the drop-in and the
// controller rely on (per-QP status, f, x, iters; QPGPU_FLAG_WRITE_FACTOR writes the factor
// into G; x left untouched on NOT_POSITIVE_DEFINITE).  It lets tests/test_sanitizers.py build the
// shipped HOST sources (quadprog_dropin.cpp, mgqp_controller.cpp, mgqp_capi.cpp,
// mgqp_component.cpp, the RTT shim) with ASan + UBSan on a machine without a GPU.
#include <cstddef>
#include <cstdint>
#include <vector>

#include "qpgpu.h"

extern "C" int qpo_solve(int n, int p, int m, double* G, const double* g0, const double* CE,
                         const double* ce0, const double* CI, const double* ci0, double* x,
                         double* f, int* iters, int max_steps);

extern "C" {
const char* qpgpu_last_error(void) { return ""; }

int qpgpu_solve_batched_host(const qpgpu_problem_desc* d, double* G, const double* g0,
                             const double* CE, const double* ce0, const double* CI,
                             const double* ci0, double* x, double* f, int32_t* status,
                             int32_t* iters) {
  if (!d || d->n <= 0 || d->p < 0 || d->m < 0 || d->batch < 0) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->layout != QPGPU_LAYOUT_QP_MAJOR) return QPGPU_ERR_INVALID_ARGUMENT;
  const int n = d->n, p = d->p, m = d->m;
  // the kernels' coverage: any shape up to the generic kernel's indexing limits
  if ((int64_t)n * n >= ((int64_t)1 << 31) || (int64_t)n * m >= ((int64_t)1 << 31))
    return QPGPU_ERR_UNSUPPORTED_SHAPE;
  const bool wf = (d->flags & QPGPU_FLAG_WRITE_FACTOR) != 0;
  std::vector<double> g((std::size_t)n * n), xb((std::size_t)n);
  for (int64_t b = 0; b < d->batch; ++b) {
    double* Gb = G + b * n * n;
    double* gw = Gb;
    if (!wf) {
      g.assign(Gb, Gb + (std::size_t)n * n);
      gw = g.data();
    }
    for (int i = 0; i < n; ++i) xb[i] = x[b * n + i];
    int it = 0;
    const int st = qpo_solve(n, p, m, gw, g0 + b * n, p ? CE + b * n * p : nullptr,
                             p ? ce0 + b * p : nullptr, m ? CI + b * n * m : nullptr,
                             m ? ci0 + b * m : nullptr, xb.data(), f + b, &it,
                             d->max_iter > 0 ? d->max_iter : 1000 + 100 * (n + p + m));
    status[b] = st;
    if (st != QPGPU_QP_NOT_POSITIVE_DEFINITE)
      for (int i = 0; i < n; ++i) x[b * n + i] = xb[i];
    if (iters) iters[b] = it;
  }
  return QPGPU_SUCCESS;
}
}
