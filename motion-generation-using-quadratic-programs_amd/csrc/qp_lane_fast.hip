// qp_lane_fast.hip — the lane kernel's QPGPU_FLAG_FAST build: qp_lane.hip compiled with
// QPGPU_LANE_FAST=1 (reciprocal-based divisions, direct rotation lengths) and -ffp-contract=fast
// (Makefile), into its own namespace and entry points (qpk_launch_lane_fast, qpk_lane_name_fast).
// Results are held to north_star's 1e-10 relative, with the same status and l1-pass counts, by
// tests/test_gpu_parity.py (test_fast_*); the default build stays bit-identical to the reference.
#define QPGPU_LANE_FAST 1
#include "qp_lane.hip"
