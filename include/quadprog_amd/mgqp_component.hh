// mgqp_component.hh — the reference's Orocos component, MotionGenerationQuadraticProgram
// (include/mgqp.hpp:70-241, src/mgqp.cpp), on the RTT surface of rtt/RTT.hh (SURVEY.md §8(f)
// rank 2: "RTT component surface, the shim now").
//
// Same operations (src/mgqp.cpp:89-95), same port names and types created by setDOFsize
// (:180-482), same FlowStatus handling in updateHook (:874-916: any of robotstatus / h /
// inertia without data -> "FAILED, NO DATA, RETURN", nothing written), same output writes
// (:1146-1176), configureHook's connection checks (:142-170) and the factory registration
// (:1270).  The control law itself is mgqp_amd::MotionGenerationQuadraticProgram (mgqp.hh):
// updateHook reads every port into one CycleInputs and runs that controller's updateHook, so the
// port path and the CycleInputs path are the same computation — every QP on the gfx950 solver.
// Eigen::VectorXf / MatrixXf are mgqp_amd::VecF / MatF.
#ifndef QUADPROG_AMD_MGQP_COMPONENT_HH
#define QUADPROG_AMD_MGQP_COMPONENT_HH

#include <string>
#include <vector>

#include "quadprog_amd/mgqp.hh"
#include "quadprog_amd/rtt/RTT.hh"
#include "quadprog_amd/rtt/rstrt.hh"

namespace mgqp_amd {
namespace rtt {

class MotionGenerationQuadraticProgram : public RTT::TaskContext {
 public:
  explicit MotionGenerationQuadraticProgram(const std::string& name);
  ~MotionGenerationQuadraticProgram() override;

  // operations (src/mgqp.cpp:89-95)
  void setDOFsize(unsigned int DOFsize);
  void setGains(float kp, float kd);
  void printCurrentState();
  bool setTorqueLimits(std::vector<double> torquesP, std::vector<double> torquesN);
  bool setAccelerationLimits(std::vector<double> accelerationsP, std::vector<double> accelerationsN);
  bool setAngularLimits(std::vector<double> limitSup, std::vector<double> limitInf);
  bool setPriorityLevel(std::string task, int level);
  // the Eigen-vector forms (mgqp.hpp:86-88)
  bool setTorqueLimitsE(VecF torquesP, VecF torquesN);
  bool setAccelerationLimitsE(VecF accelerationsP, VecF accelerationsN);
  bool setAngularLimitsE(VecF jointsP, VecF jointsN);

  // the controller the ports feed, and the last cycle's outcome (CycleCode; -1 before any)
  mgqp_amd::MotionGenerationQuadraticProgram& controller() { return ctl_; }
  int lastCycleCode() const { return last_code_; }

 protected:
  bool configureHook() override;
  bool startHook() override;
  void updateHook() override;
  void stopHook() override;
  void cleanupHook() override;

 private:
  void removeJointPorts();
  template <class P>
  static void clear(std::vector<P*>& v);

  mgqp_amd::MotionGenerationQuadraticProgram ctl_;
  unsigned int DOFsize_ = 0;
  bool portsPrepared_ = false;
  int last_code_ = -1;

  // per-joint input ports (mgqp.hpp:96-110), index j <-> name suffix j+1
  std::vector<RTT::InputPort<VecF>*> in_desiredTaskSpacePosition_port, in_desiredTaskSpaceVelocity_port,
      in_desiredTaskSpaceAcceleration_port, in_currentTaskSpacePosition_port,
      in_currentTaskSpaceVelocity_port, in_currentTaskSpaceAcceleration_port;
  std::vector<RTT::InputPort<float>*> in_desiredJointSpacePosition_port,
      in_desiredJointSpaceVelocity_port, in_desiredJointSpaceAcceleration_port;
  std::vector<RTT::InputPort<MatF>*> in_jacobian_port, in_jacobianDot_port;
  RTT::InputPort<VecF> in_h_port;
  RTT::InputPort<MatF> in_inertia_port;
  RTT::InputPort<rstrt::robot::JointState> in_robotstatus_port;

  RTT::OutputPort<rstrt::dynamics::JointTorques> out_torques_port;
  RTT::OutputPort<VecF> out_jointPosLimitInf_port, out_jointPosLimitSup_port, out_jointVelLimitInf_port,
      out_jointVelLimitSup_port, out_jointAccLimitInf_port, out_jointAccLimitSup_port,
      out_jointAccDynLimitInf_port, out_jointAccDynLimitSup_port, out_jointTorqueLimitInf_port,
      out_jointTorqueLimitSup_port;

  rstrt::robot::JointState in_robotstatus_var;
  VecF in_h_var;
  MatF in_inertia_var;
  rstrt::dynamics::JointTorques out_torques_var;
  VecF torquesP_, torquesN_, accP_, accN_;  // for printCurrentState
};

}  // namespace rtt
}  // namespace mgqp_amd

#endif
