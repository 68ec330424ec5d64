// quadprog_amd/eigen/QuadProg++.hh — the second drop-in signature of the solver: the
// Eigen-variant API `QuadProgpp::Solver::solve(...) -> Status::Value` of the fork the reference
// vendors in include/QuadProgpp/eigen/QuadProg++.hh:83-118 (sketched at reference
// src/mgqp.cpp:675-693), served by the gfx950 kernels through the C-ABI
// (include/qpgpu.h, qpgpu_solve_batched_host with batch 1).
//
// Header-only: the reference ships this variant as the archive libquadprog_eigen.a, which is
// missing from the reference tree, so there is nothing to link-replace; a caller includes this
// header instead and links libqpgpu.so.
//
// Matrix types (as in the reference header, selected by config.hh):
//   QUADPROGPP_ENABLE_EIGEN defined -> Eigen::Matrix<double, Dynamic, Dynamic, ColMajor> /
//                                      Eigen::Matrix<double, Dynamic, 1, ColMajor>
//   otherwise                       -> QuadProgpp::Matrix<double> / QuadProgpp::Vector<double>
//                                      (eigen/Array.hh: the ArrayHH containers)
//
// Behaviour.  The fork's implementation is not available (missing archive), so its exact
// semantics are UNPINNED; this header follows the contract its own header states
// (eigen/QuadProg++.hh:13-67), its vendored helpers and the QuadProg++ solver it forks:
//   * the problem is min ½xᵀGx + g0ᵀx s.t. CEᵀx + ce0 = 0, CIᵀx + ci0 >= 0 with G n×n,
//     CE n×p, CI n×m, solved by the same Goldfarb–Idnani kernels as solve_quadprog: bit-identical
//     to libquadprog_amd.so for n <= 64, within 1e-10 relative above (the MFMA panel setup).
//     The fork itself factors with Eigen's LLT and inverts U in place
//     (eigen/EigenHelpers.hh:43-99), so its last bits differ from QuadProg++ in any case;
//   * x is resized to n and receives the solution; G is left unchanged (the fork's helper
//     factors a copy, EigenHelpers.hh:48-51 — the legacy header note 3 predates it);
//   * Status::OK when the solve succeeds; Status::FAILURE when the problem is infeasible, G is
//     not positive definite, the equality constraints are linearly dependent or the step cap
//     is hit (no exceptions for numerical failures: that is what the Status return is for);
//     objective() returns the last cost (+inf when infeasible);
//   * inconsistent dimensions throw std::logic_error with solve_quadprog's messages;
//   * a failing C-ABI call (no GPU, unsupported shape) throws std::runtime_error.
#ifndef QUADPROG_AMD_EIGEN_QUADPROGPP_HH
#define QUADPROG_AMD_EIGEN_QUADPROGPP_HH

#include <cstdint>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "config.hh"
#include "qpgpu.h"

#ifdef QUADPROGPP_ENABLE_EIGEN
#include <Eigen/Dense>
#define QPPP_VECTOR(t_Scalar) Eigen::Matrix<t_Scalar, Eigen::Dynamic, 1, Eigen::ColMajor>
#define QPPP_MATRIX(t_Scalar) Eigen::Matrix<t_Scalar, Eigen::Dynamic, Eigen::Dynamic, Eigen::ColMajor>
#else
#include "Array.hh"
#define QPPP_VECTOR(t_Scalar) QuadProgpp::Vector<t_Scalar>
#define QPPP_MATRIX(t_Scalar) QuadProgpp::Matrix<t_Scalar>
#endif

namespace QuadProgpp {

class Status {
 public:
  enum Value { OK = 0, FAILURE = 1 };
};

namespace amd_detail {

// element access / shape for both container families (ArrayHH: M[i][j], nrows(); Eigen and
// any Eigen-like type: M(i, j), rows())
template <class M>
inline auto rows_of(const M& A) -> decltype(A.rows(), 0u) { return (unsigned)A.rows(); }
template <class M>
inline auto cols_of(const M& A) -> decltype(A.cols(), 0u) { return (unsigned)A.cols(); }
template <class M>
inline auto rows_of(const M& A) -> decltype(A.nrows(), 0u) { return A.nrows(); }
template <class M>
inline auto cols_of(const M& A) -> decltype(A.ncols(), 0u) { return A.ncols(); }
template <class M>
inline auto at(M& A, unsigned i, unsigned j) -> decltype(A(i, j)) { return A(i, j); }
template <class M>
inline auto at(M& A, unsigned i, unsigned j) -> decltype(A[i][j]) { return A[i][j]; }

// Reusable host staging: the C-ABI takes row-major per-QP blocks (include/qpgpu.h), the
// Eigen types are column-major, so every matrix is packed element by element.
struct Staging {
  std::vector<double> G, g0, CE, ce0, CI, ci0, x;
};

// Solves one problem; returns the qpgpu per-QP status (QPGPU_QP_*) and the cost in f.
template <class MatG, class VecG, class MatE, class VecE, class MatI, class VecI, class VecX>
int solve_generic(Staging& s, MatG& G, VecG& g0, const MatE& CE, const VecE& ce0,
                  const MatI& CI, const VecI& ci0, VecX& x, double& f) {
  const unsigned n = cols_of(G), p = cols_of(CE), m = cols_of(CI);
  std::ostringstream msg;
  if (rows_of(G) != n) {
    msg << "The matrix G is not a squared matrix (" << rows_of(G) << " x " << cols_of(G) << ")";
    throw std::logic_error(msg.str());
  }
  if (rows_of(CE) != n) {
    msg << "The matrix CE is incompatible (incorrect number of rows " << rows_of(CE)
        << " , expecting " << n << ")";
    throw std::logic_error(msg.str());
  }
  if ((unsigned)ce0.size() != p) {
    msg << "The vector ce0 is incompatible (incorrect dimension " << ce0.size()
        << ", expecting " << p << ")";
    throw std::logic_error(msg.str());
  }
  if (rows_of(CI) != n) {
    msg << "The matrix CI is incompatible (incorrect number of rows " << rows_of(CI)
        << " , expecting " << n << ")";
    throw std::logic_error(msg.str());
  }
  if ((unsigned)ci0.size() != m) {
    msg << "The vector ci0 is incompatible (incorrect dimension " << ci0.size()
        << ", expecting " << m << ")";
    throw std::logic_error(msg.str());
  }
  x.resize(n);
  if (n == 0) throw std::logic_error("qpgpu: n == 0 is not supported (undefined in QuadProg++)");
  s.G.resize((size_t)n * n);
  s.g0.resize(n);
  s.CE.resize((size_t)n * p);
  s.ce0.resize(p);
  s.CI.resize((size_t)n * m);
  s.ci0.resize(m);
  s.x.resize(n);
  for (unsigned i = 0; i < n; i++) {
    for (unsigned j = 0; j < n; j++) s.G[(size_t)i * n + j] = at(G, i, j);
    for (unsigned j = 0; j < p; j++) s.CE[(size_t)i * p + j] = at(CE, i, j);
    for (unsigned j = 0; j < m; j++) s.CI[(size_t)i * m + j] = at(CI, i, j);
    s.g0[i] = g0[i];
  }
  for (unsigned j = 0; j < p; j++) s.ce0[j] = ce0[j];
  for (unsigned j = 0; j < m; j++) s.ci0[j] = ci0[j];

  qpgpu_problem_desc d{};
  d.n = (int32_t)n;
  d.p = (int32_t)p;
  d.m = (int32_t)m;
  d.batch = 1;
  d.flags = 0;  // G is not written back (see the header comment)
  int32_t status = 0, iters = 0;
  f = 0.0;
  const int rc = qpgpu_solve_batched_host(&d, s.G.data(), s.g0.data(), p ? s.CE.data() : nullptr,
                                          p ? s.ce0.data() : nullptr, m ? s.CI.data() : nullptr,
                                          m ? s.ci0.data() : nullptr, s.x.data(), &f, &status,
                                          &iters);
  if (rc != QPGPU_SUCCESS) {
    std::ostringstream os;
    os << "qpgpu: solve failed (code " << rc << ")";
    if (rc == QPGPU_ERR_HIP || rc == QPGPU_ERR_NO_DEVICE) os << ": " << qpgpu_last_error();
    throw std::runtime_error(os.str());
  }
  for (unsigned i = 0; i < n; i++) x[i] = s.x[i];
  if (status == QPGPU_QP_INFEASIBLE) f = std::numeric_limits<double>::infinity();
  return status;
}

}  // namespace amd_detail

class Solver {
 public:
  Solver() : impl(new Implementation) {}
  ~Solver() { delete impl; }
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  Status::Value solve(QPPP_MATRIX(double) & G, QPPP_VECTOR(double) & g0,
                      const QPPP_MATRIX(double) & CE, const QPPP_VECTOR(double) & ce0,
                      const QPPP_MATRIX(double) & CI, const QPPP_VECTOR(double) & ci0,
                      QPPP_VECTOR(double) & x) {
    impl->last_status = amd_detail::solve_generic(impl->staging, G, g0, CE, ce0, CI, ci0, x,
                                                  impl->last_cost);
    return impl->last_status == QPGPU_QP_OK ? Status::OK : Status::FAILURE;
  }

  // not in the reference API: the cost of the last solve (+inf when infeasible; the failing
  // pivot when G was not positive definite) and its qpgpu status (QPGPU_QP_*)
  double objective() const { return impl->last_cost; }
  int detailed_status() const { return impl->last_status; }

 private:
  class Implementation {
   public:
    amd_detail::Staging staging;
    double last_cost = 0.0;
    int last_status = QPGPU_QP_OK;
  };
  Implementation* impl;
};

}  // namespace QuadProgpp

#endif  // QUADPROG_AMD_EIGEN_QUADPROGPP_HH
