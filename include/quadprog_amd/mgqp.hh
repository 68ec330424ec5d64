// mgqp.hh — the motion-generation controller around the solver.
//
// Restates the reference component's QP builder and hierarchy solver without Orocos RTT or Eigen:
//   * MotionGenerationQuadraticProgram::solveNextStep      (reference src/mgqp.cpp:655-749)
//   * MotionGenerationQuadraticProgram::solveNextHierarchy (reference src/mgqp.cpp:751-869)
//   * MotionGenerationQuadraticProgram::updateHook         (reference src/mgqp.cpp:872-1189)
//   * QuadraticProblem / StackOfTasks                      (reference include/mgqp.hpp:30-64)
//   * the RTT operations setDOFsize/setGains/set*Limits/setPriorityLevel (src/mgqp.cpp:89-95,
//     180-570)
// Ports become plain values: every RTT input port is a Port<T> whose `has` flag stands for
// "flow != RTT::NoData"; the output ports are the fields of CycleOutputs.  Eigen's float
// matrices are MatF (row-major float) and VecF (std::vector<float>).  Every QP goes to the
// gfx950 solver: the single-robot path through the drop-in solve_quadprog() (libquadprog_amd),
// the batched path (update_batched) through qpgpu_solve_batched_host(), one launch per level
// and problem shape for all robots at once.
#ifndef QUADPROG_AMD_MGQP_HH
#define QUADPROG_AMD_MGQP_HH

#include <map>
#include <string>
#include <vector>

namespace mgqp_amd {

using VecF = std::vector<float>;

struct MatF {
  int rows = 0, cols = 0;
  std::vector<float> a;  // row-major
  MatF() {}
  MatF(int r, int c, float v = 0.f) : rows(r), cols(c), a((size_t)r * c, v) {}
  float& operator()(int i, int j) { return a[(size_t)i * cols + j]; }
  float operator()(int i, int j) const { return a[(size_t)i * cols + j]; }
  static MatF identity(int n);
};

// include/mgqp.hpp:30-51
struct QuadraticProblem {
  MatF conditions;   // equality rows  A  (A x + a = 0 after the builder's sign convention)
  VecF goal;
  MatF constraints;  // inequality rows B (B x + b >= 0)
  VecF limits;
  int pbDOF = 0;
  int nbConditions() const { return conditions.rows; }
  int rows() const { return conditions.rows; }
  int cols() const { return conditions.cols; }
  int init(int DOFsize);
  int dof() const { return pbDOF; }
};

// include/mgqp.hpp:53-64
struct StackOfTasks {
  int stackSize = 0;
  std::vector<QuadraticProblem> qps;
  std::map<std::string, int> level;
  int init(int nbOfLevels);
  QuadraticProblem* getQP(int lvl) { return &qps[lvl]; }
  int getLevel(const std::string& task) const;
  bool setPriority(const std::string& task, int priorityLevel);
};

template <class T>
struct Port {
  bool has = false;  // false <=> RTT::NoData
  T v{};
  void set(const T& x) { has = true; v = x; }
};

struct JointState {  // rstrt::robot::JointState (angles, velocities)
  VecF angles, velocities;
};

// The per-joint input ports of reference src/mgqp.cpp:904-916 (joint index j = port suffix j+1).
struct JointPorts {
  Port<VecF> desiredTaskSpacePosition, desiredTaskSpaceVelocity, desiredTaskSpaceAcceleration;
  Port<VecF> currentTaskSpacePosition, currentTaskSpaceVelocity, currentTaskSpaceAcceleration;
  Port<float> desiredJointSpacePosition, desiredJointSpaceVelocity, desiredJointSpaceAcceleration;
  Port<MatF> jacobian, jacobianDot;
};

struct CycleInputs {
  Port<JointState> robotstatus;
  Port<VecF> h;
  Port<MatF> inertia;
  std::vector<JointPorts> joints;  // DOFsize entries
};

// Result of one updateHook cycle.  `code` tells which reference exit was taken.
enum CycleCode {
  CYCLE_WRITTEN = 0,       // ports written (src/mgqp.cpp:1165-1176)
  CYCLE_NO_DATA = 1,       // "FAILED, NO DATA, RETURN" (src/mgqp.cpp:879-883)
  CYCLE_NO_JACOBIAN = 2,   // "FAILED, NO JACOBIAN FOR JOINT j RETURN" (src/mgqp.cpp:988-993)
  CYCLE_EXCEPTION = 3,     // solve_quadprog threw (linearly dependent constraints)
};

struct CycleOutputs {
  int code = CYCLE_NO_DATA;
  std::string error;
  VecF torques;   // out_torques_port (tau + h)
  VecF tracking;  // solveNextHierarchy() result [acceleration; torques] before adding h
  VecF jointPosLimitInf, jointPosLimitSup, jointVelLimitInf, jointVelLimitSup, jointAccLimitInf,
      jointAccLimitSup, jointAccDynLimitInf, jointAccDynLimitSup, jointTorqueLimitInf,
      jointTorqueLimitSup;
};

class MotionGenerationQuadraticProgram {
 public:
  MotionGenerationQuadraticProgram();  // src/mgqp.cpp:97-139 defaults

  // RTT operations (src/mgqp.cpp:89-95)
  void setDOFsize(unsigned int DOFsize);
  void setGains(float kp, float kd);
  bool setTorqueLimits(const std::vector<double>& P, const std::vector<double>& N);
  bool setAccelerationLimits(const std::vector<double>& P, const std::vector<double>& N);
  bool setAngularLimits(const std::vector<double>& sup, const std::vector<double>& inf);
  bool setPriorityLevel(const std::string& task, int level);

  // One control cycle (updateHook).  Throws what solve_quadprog throws, like the reference.
  void updateHook(const CycleInputs& in, CycleOutputs& out);

  // Batched cycles: `count` robots with this controller's configuration, each with its own
  // inputs.  The QPs of every level are solved in one GPU launch per problem shape.  A
  // robot whose solve throws in the reference gets code CYCLE_EXCEPTION instead.
  void update_batched(const CycleInputs* in, CycleOutputs* out, long count, int threads = 0);

  // Device-resident batch (include/mgqp_amd.h mgqp_device_batch; `batch` is that struct).
  // Returns 0, CYCLE_NO_DATA / CYCLE_NO_JACOBIAN for a uniform early exit, or throws
  // std::runtime_error / std::length_error.
  int update_device(const void* batch, float* torques, float* tracking, int* codes, void* stream);

  // src/mgqp.cpp:655-749 and 751-869 (they operate on this->stack_of_tasks)
  bool solveNextStep(const MatF& A, const VecF& a, const MatF& B, const VecF& b, VecF* res);
  VecF solveNextHierarchy();

  int DOFsize() const { return DOFsize_; }
  StackOfTasks stack_of_tasks;

 private:
  friend struct BatchRunner;
  int DOFsize_ = 0;
  unsigned WorkspaceDimension = 3;
  float gainTranslationP, gainTranslationD, gainJointP, gainJointD;
  VecF JointTorquesLimitsP, JointTorquesLimitsN, JointAccelerationLimitsP, JointAccelerationLimitsN,
      JointLimitsSup, JointLimitsInf;
};

// Null-space projector of the hierarchy (src/mgqp.cpp:836-862): Z = I - V A V^T with V the thin
// right singular vectors of Acumul and A(k,k) = [sigma_k >= 1e-16].  Exposed for the tests.
MatF nullspace_projector(const MatF& Acumul, int dim);

}  // namespace mgqp_amd

#endif
