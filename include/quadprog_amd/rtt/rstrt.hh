// rstrt.hh — the rst-rt message types the reference controller's ports carry
// (include/mgqp.hpp:122-125, src/mgqp.cpp:1148-1176), with Eigen::VectorXf replaced by the
// controller's VecF (rst-rt and Eigen are not installed in this image: SURVEY.md §8(c)).
#ifndef QUADPROG_AMD_RSTRT_HH
#define QUADPROG_AMD_RSTRT_HH

#include "quadprog_amd/mgqp.hh"

namespace rstrt {
namespace robot {
struct JointState {  // in_robotstatus_port: angles, velocities, torques
  JointState() {}
  explicit JointState(int dof) : angles(dof, 0.f), velocities(dof, 0.f), torques(dof, 0.f) {}
  mgqp_amd::VecF angles, velocities, torques;
};
}  // namespace robot
namespace dynamics {
struct JointTorques {  // out_torques_port
  JointTorques() {}
  explicit JointTorques(int dof) : torques(dof, 0.f) {}
  mgqp_amd::VecF torques;
};
}  // namespace dynamics
namespace kinematics {
struct JointAngles {  // q_des (set up by setDOFsize, src/mgqp.cpp:474-475)
  JointAngles() {}
  explicit JointAngles(int dof) : angles(dof, 0.f) {}
  mgqp_amd::VecF angles;
};
struct JointVelocities {
  JointVelocities() {}
  explicit JointVelocities(int dof) : velocities(dof, 0.f) {}
  mgqp_amd::VecF velocities;
};
}  // namespace kinematics
}  // namespace rstrt

#endif
