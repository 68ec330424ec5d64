// quadprog_amd/eigen/config.hh — container selection for eigen/QuadProg++.hh, as the
// reference's include/QuadProgpp/eigen/config.hh does (which enables Eigen).  Eigen is the
// default; define QUADPROGPP_DISABLE_EIGEN to use the ArrayHH containers instead.
#pragma once

#if !defined(QUADPROGPP_DISABLE_EIGEN) && !defined(QUADPROGPP_ENABLE_EIGEN)
#define QUADPROGPP_ENABLE_EIGEN true
#endif
