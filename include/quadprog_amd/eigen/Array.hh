// quadprog_amd/eigen/Array.hh — QuadProgpp::Vector / QuadProgpp::Matrix for the non-Eigen
// build of eigen/QuadProg++.hh (reference include/QuadProgpp/eigen/Array.hh declares the same
// container interface in namespace QuadProgpp).  They are the ArrayHH containers of
// quadprog_amd/Array.hh under the fork's namespace.
#pragma once

#include "../Array.hh"

namespace QuadProgpp {
template <typename T>
using Vector = ArrayHH::Vector<T>;
template <typename T>
using Matrix = ArrayHH::Matrix<T>;
}  // namespace QuadProgpp
