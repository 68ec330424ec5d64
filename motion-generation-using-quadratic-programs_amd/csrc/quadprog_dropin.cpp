// quadprog_dropin.cpp — the reference's C++ solver entry point, served by the gfx950 kernels.
//
// Exports  double solve_quadprog(ArrayHH::Matrix<double>&, ArrayHH::Vector<double>&,
//                                const Matrix<double>&, const Vector<double>&,
//                                const Matrix<double>&, const Vector<double>&, Vector<double>&)
// with the reference's mangled name, so linking libquadprog_amd.so in place of
// lib/QuadProgpp/libquadprog.a (reference CMakeLists.txt:95) is the whole integration.
// Callers: reference src/mgqp.cpp:708 and :725.
//
// Reference-visible behaviour reproduced here (reference QuadProg++.hh:27-45):
//   * the five dimension checks, in order, with the archive's message texts, as
//     std::logic_error;
//   * x.resize(n) before solving; G overwritten with the Cholesky factor (L mirrored);
//   * return value f, or +inf when infeasible;
//   * non-positive-definite G: G printed to stdout by print_matrix("A", G), then
//     std::logic_error("Error in cholesky decomposition, sum: <sum>");
//   * dependent equalities: std::runtime_error("Constraints are linearly dependent").
// The solve itself always runs on the GPU through qpgpu_solve_batched_host(); there is no
// CPU solver in this library.
#include <cmath>
#include <iostream>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "QuadProg++.hh"
#include "qpgpu.h"

namespace {

// print_matrix("A", G) as QuadProg++ prints it before the Cholesky exception.
void print_matrix_like_reference(const char* name, const Matrix<double>& A) {
  std::ostringstream s;
  s << name << ": " << std::endl;
  for (unsigned int i = 0; i < A.nrows(); i++) {
    s << " ";
    for (unsigned int j = 0; j < A.ncols(); j++) s << A[i][j] << ", ";
    s << std::endl;
  }
  std::string t = s.str();
  t = t.substr(0, t.size() - 3);  // drop the trailing ", \n"
  std::cout << t << std::endl;
}

[[noreturn]] void throw_api_error(int rc) {
  std::ostringstream os;
  os << "qpgpu: solve failed (code " << rc << ")";
  if (rc == QPGPU_ERR_HIP || rc == QPGPU_ERR_NO_DEVICE) os << ": " << qpgpu_last_error();
  if (rc == QPGPU_ERR_UNSUPPORTED_SHAPE) os << ": no gfx950 kernel covers this (n, p, m)";
  throw std::runtime_error(os.str());
}

}  // namespace

double solve_quadprog(Matrix<double>& G, Vector<double>& g0, const Matrix<double>& CE,
                      const Vector<double>& ce0, const Matrix<double>& CI,
                      const Vector<double>& ci0, Vector<double>& x) {
  std::ostringstream msg;
  const unsigned int n = G.ncols(), p = CE.ncols(), m = CI.ncols();
  if (G.nrows() != n) {
    msg << "The matrix G is not a squared matrix (" << G.nrows() << " x " << G.ncols() << ")";
    throw std::logic_error(msg.str());
  }
  if (CE.nrows() != n) {
    msg << "The matrix CE is incompatible (incorrect number of rows " << CE.nrows()
        << " , expecting " << n << ")";
    throw std::logic_error(msg.str());
  }
  if (ce0.size() != p) {
    msg << "The vector ce0 is incompatible (incorrect dimension " << ce0.size()
        << ", expecting " << p << ")";
    throw std::logic_error(msg.str());
  }
  if (CI.nrows() != n) {
    msg << "The matrix CI is incompatible (incorrect number of rows " << CI.nrows()
        << " , expecting " << n << ")";
    throw std::logic_error(msg.str());
  }
  if (ci0.size() != m) {
    msg << "The vector ci0 is incompatible (incorrect dimension " << ci0.size()
        << ", expecting " << m << ")";
    throw std::logic_error(msg.str());
  }
  x.resize(n);
  if (n == 0) throw std::logic_error("qpgpu: n == 0 is not supported (undefined in QuadProg++)");

  // ArrayHH storage is one contiguous row-major block starting at &M[0][0] (Array.hh:910-919),
  // which is exactly the per-QP layout of include/qpgpu.h, so no repacking is needed.
  double* Gp = &G[0][0];
  const double* CEp = p ? &CE[0][0] : nullptr;
  const double* CIp = m ? &CI[0][0] : nullptr;
  const double* ce0p = p ? &ce0[0] : nullptr;
  const double* ci0p = m ? &ci0[0] : nullptr;

  qpgpu_problem_desc d{};
  d.n = (int32_t)n;
  d.p = (int32_t)p;
  d.m = (int32_t)m;
  d.batch = 1;
  d.flags = QPGPU_FLAG_WRITE_FACTOR;
  double f = 0.0;
  int32_t status = 0, iters = 0;
  const int rc = qpgpu_solve_batched_host(&d, Gp, &g0[0], CEp, ce0p, CIp, ci0p, &x[0], &f,
                                          &status, &iters);
  if (rc != QPGPU_SUCCESS) throw_api_error(rc);
  switch (status) {
    case QPGPU_QP_OK:
      return f;
    case QPGPU_QP_INFEASIBLE:
      return std::numeric_limits<double>::infinity();
    case QPGPU_QP_NOT_POSITIVE_DEFINITE: {
      print_matrix_like_reference("A", G);
      std::ostringstream os;
      os << "Error in cholesky decomposition, sum: " << f;
      throw std::logic_error(os.str());
    }
    case QPGPU_QP_DEPENDENT:
      throw std::runtime_error("Constraints are linearly dependent");
    default:
      throw std::runtime_error("qpgpu: active-set step cap reached (no reference equivalent)");
  }
}
