// QuadProg++.hh — drop-in declaration of the reference solver entry point.
//
// Same signature, namespace placement and mangled name as the reference
// (include/QuadProgpp/QuadProg++.hh:65-72, global namespace with `using namespace ArrayHH`):
//   _Z14solve_quadprogRN7ArrayHH6MatrixIdEERNS_6VectorIdEERKS1_RKS4_S7_S9_S5_
// Contract (reference QuadProg++.hh:8-45): min 0.5 x'Gx + g0'x  s.t.  CE'x + ce0 = 0,
// CI'x + ci0 >= 0.  Returns the objective, or +inf if infeasible.  G is overwritten with its
// Cholesky factor; x is resized to n.  Throws std::logic_error on dimension mismatch or a
// non-positive-definite G (after printing G to stdout), std::runtime_error("Constraints are
// linearly dependent").
//
// Implemented by libquadprog_amd.so on top of the gfx950 kernels (include/qpgpu.h); every
// call runs on the GPU.
//
// Any n, p, m is solved, as by the reference (QuadProg++.hh:69-72): shapes beyond the specialised
// kernels (n > 256 or m > 1024) run on the generic workspace kernel (qp_generic.hip), bit for bit
// like the others.  Differences from the reference's contract (it has no GPU):
//   * n == 0 throws std::logic_error("qpgpu: n == 0 is not supported (undefined in
//     QuadProg++)"); n*n or n*m at or above 2^31 (an 8 GiB G), beyond the generic kernel's
//     indexing, throws std::runtime_error("qpgpu: solve failed (code 2): no gfx950 kernel covers
//     this (n, p, m)");
//   * no usable GPU: std::runtime_error("qpgpu: solve failed (code 4): ...") (code 3 for another
//     HIP runtime failure, with its message);
//   * the safety cap on active-set steps (1000 + 100 (n + p + m)), which terminating problems
//     never reach: std::runtime_error("qpgpu: active-set step cap reached (no reference
//     equivalent)").
#ifndef QUADPROG_AMD_QUADPROGPP_HH
#define QUADPROG_AMD_QUADPROGPP_HH

#include "Array.hh"

using namespace ArrayHH;

double solve_quadprog(Matrix<double>& G, Vector<double>& g0, const Matrix<double>& CE,
                      const Vector<double>& ce0, const Matrix<double>& CI,
                      const Vector<double>& ci0, Vector<double>& x);

#endif
