// mgqp_device.h — device side of the batched controller pipeline.
//
// One control cycle for `count` robots without a host round trip between levels:
//   build_tasks   : every robot's equality rows (cond) and goals for all levels + the level-0
//                   limit vector (src/mgqp.cpp:912-1134), one lane per robot
//   build_level l : CE = (cond_l Z)^T, ce0 = goal_l - cond_l res, CI = (Bcumul Z)^T,
//                   ci0 = bcumul (src/mgqp.cpp:783-793), written as double QP-major blocks
//   solve         : the batched QuadProg++ kernels (qpgpu_solve_batched), with and without CI
//                   (the retry of src/mgqp.cpp:717-736)
//   finish level l: pick the solve, res = last_res + Z u, then the null-space projector of the
//                   stacked rows by one-sided Jacobi in LDS (src/mgqp.cpp:814-862)
//   outputs       : torques = tau + h (src/mgqp.cpp:1146-1152)
// The float/double operation order is the host controller's (mgqp_controller.cpp), so the
// device pipeline reproduces the host-orchestrated batched path bit for bit.
#ifndef MGQP_DEVICE_H
#define MGQP_DEVICE_H

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace mgqp_dev {

constexpr int kMaxDof = 16;
constexpr int kMaxGen = 64;
constexpr int kMaxLevels = 8;

enum GenType : int32_t { GEN_TASK = 0, GEN_JOINT = 1, GEN_DYN = 2 };
enum GenFlags : int32_t { F_POS = 1, F_VEL = 2, F_ACC = 4 };

struct RowGen {  // one addToProblem call of the builder, in the reference's order
  int32_t type, joint, level, flags;
  int32_t row0;  // first row of this generator in the stacked `cond` array
  int32_t rows;
};

struct Plan {
  int32_t dof, ws, dim, ngen, nlevels, total_rows, nineq;
  int32_t level_rows[kMaxLevels], level_row0[kMaxLevels];
  float kTP, kTD, kJP, kJD;
  RowGen gen[kMaxGen];
  // robot-major port arrays (device); task-space ports: [count][ts_len]
  const float* ts[kMaxDof][6];  // desired pos/vel/acc, current pos/vel/acc
  const float* js[kMaxDof][3];  // desired joint pos/vel/acc: [count]
  const float* jac[kMaxDof];    // [count][ws][jac_cols]
  const float* jacd[kMaxDof];
  int32_t ts_len[kMaxDof], jac_cols[kMaxDof];
  const float* angles;  // [count][status_len]
  const float* velocities;
  const float* h;        // [count][dof]
  const float* inertia;  // [count][dof][dof]
  int32_t status_len;
  uint32_t solver_flags;  // QPGPU_FLAG_* of the level solves (host side only)
  // limits configuration (already size-normalised on the host, :1113-1117)
  float accP[kMaxDof], accN[kMaxDof], tP[kMaxDof], tN[kMaxDof], sup[kMaxDof], inf[kMaxDof];
};

// Workspace arrays (all robot-minor "SoA": element e of robot r at [e * count + r]).
struct Work {
  int64_t count;
  float* cond;    // [total_rows * dim][count]
  float* goal;    // [total_rows][count]
  float* limits;  // [nineq][count]
  float* Z;       // [dim * dim][count]
  float* res;     // [dim][count]
  float* u;       // [dim][count]
  int32_t* state; // [count]: 0 active, 1 done (stopped at a level), 2 exception
  double* V;      // [dim * dim][count]: thin right singular vectors of the projector
  const float* Bcumul;  // [nineq][dim] shared by all robots (limitsMatrix, :1083-1085)
};

int launch_build_tasks(const Plan& P, const Work& W, hipStream_t s);
// Writes the level-l QPs (n = dim, p = level_rows[l], m = nineq or 0) into QP-major doubles.
int launch_build_level(const Plan& P, const Work& W, int level, double* CE, double* ce0,
                       double* CI, double* ci0, hipStream_t s);
// acc_rows: number of stacked cond rows (levels <= l with rows) for the projector; 0 = skip.
int launch_finish_level(const Plan& P, const Work& W, int level, const double* x1,
                        const double* f1, const int32_t* st1, const double* x2, const double* f2,
                        const int32_t* st2, int acc_rows, hipStream_t s);
int launch_outputs(const Plan& P, const Work& W, float* torques, float* tracking, int32_t* codes,
                   hipStream_t s);
int launch_init(const Plan& P, const Work& W, double* G, double* g0, hipStream_t s);

// The whole cycle: workspace (grow-only, cached per device), init, builder, every level with a
// solve (solve with CI, solve without CI, finish), outputs.  Bcumul_host: nineq x dim floats.
// Enqueued on `s`; returns 0 or a negative code with *err set.
int run_cycle(const Plan& P, int64_t count, const float* Bcumul_host, float* torques,
              float* tracking, int32_t* codes, hipStream_t s, const char** err);

}  // namespace mgqp_dev

#endif
