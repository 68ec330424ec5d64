// qp_lane_p0.hip — the exact lane kernel's p = 0 instantiations (C2: joint-limit QPs with no
// equality constraints) in a translation unit of their own, so that the Makefile can schedule them
// with LLVM's iterative-minreg strategy while qp_lane.hip's other instantiations keep iterative-ilp
// (measured per configuration, profiles/r05_s11).  Same source, same arithmetic: bit-identical
// results (tests/test_gpu_parity.py); qp_lane.hip's launcher calls qpk_launch_lane_p0 for them.
#define QPGPU_LANE_PART 2
#include "qp_lane.hip"
