// The reference component deployed the way ops/mgqp.ops:180-236 deploys it, on the RTT surface
// of include/quadprog_amd/rtt/RTT.hh: loadComponent by type name, operations called by name,
// peers' output ports connected to the controller's ports by name, configure / start, then N
// activity triggers.  Every cycle's out_torques (read through a connected sink port) and the
// limit outputs must equal, bit for bit, a second controller driven through the CycleInputs
// path with the same inputs.  Also: the NoData early exit (src/mgqp.cpp:874-883), OldData
// re-use of the last samples, "no jacobian" exit, configureHook's connection checks,
// setDOFsize's port set, operation signature checks, and the Exception state on a solver throw.
//
// Linked either with the shipped libmgqp_amd.so (GPU: every QP on the gfx950 kernels) or, in the
// CPU suite, with the controller sources + the test-only oracle harness.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "quadprog_amd/mgqp_component.hh"

using mgqp_amd::MatF;
using mgqp_amd::VecF;

static int g_fail = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                          \
    }                                                                    \
  } while (0)

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static float urand(float lo, float hi) {  // SplitMix64 -> [lo, hi)
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return lo + (hi - lo) * (float)((z >> 40) * (1.0 / 16777216.0));
}
static VecF vrand(int n, float lo, float hi) {
  VecF v(n);
  for (auto& x : v) x = urand(lo, hi);
  return v;
}
static MatF mrand(int r, int c, float lo, float hi) {
  MatF m(r, c);
  for (auto& x : m.a) x = urand(lo, hi);
  return m;
}
static bool same_bits(const VecF& a, const VecF& b) {
  return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * 4) == 0);
}

// the deployment's peers: fkin7 (kinematics/dynamics), trajectorygenerator2, singen, and the
// robot's torque input (ops/mgqp.ops:199-236)
struct Fkin : RTT::TaskContext {
  RTT::OutputPort<rstrt::robot::JointState> out_robotstatus_port{"out_robotstatus_port"};
  RTT::OutputPort<VecF> out_coriolisAndGravity_port{"out_coriolisAndGravity_port"};
  RTT::OutputPort<MatF> out_inertia_port{"out_inertia_port"};
  RTT::OutputPort<MatF> out_jacobianTranslation_port{"out_jacobianTranslation_port"};
  RTT::OutputPort<MatF> out_jacobianDotTranslation_port{"out_jacobianDotTranslation_port"};
  RTT::OutputPort<VecF> out_cartPosTranslation_port{"out_cartPosTranslation_port"};
  RTT::OutputPort<VecF> out_cartVelTranslation_port{"out_cartVelTranslation_port"};
  RTT::OutputPort<VecF> out_cartAccTranslation_port{"out_cartAccTranslation_port"};
  explicit Fkin(const std::string& n) : TaskContext(n) {
    for (RTT::base::PortInterface* p :
         std::initializer_list<RTT::base::PortInterface*>{&out_robotstatus_port, &out_coriolisAndGravity_port,
                                                          &out_inertia_port, &out_jacobianTranslation_port,
                                                          &out_jacobianDotTranslation_port, &out_cartPosTranslation_port,
                                                          &out_cartVelTranslation_port, &out_cartAccTranslation_port})
      ports()->addPort(*p);
  }
};
struct Traj : RTT::TaskContext {
  RTT::OutputPort<VecF> pos{"out_desiredTaskSpacePosition_port"}, vel{"out_desiredTaskSpaceVelocity_port"},
      acc{"out_desiredTaskSpaceAcceleration_port"};
  explicit Traj(const std::string& n) : TaskContext(n) {
    ports()->addPort(pos);
    ports()->addPort(vel);
    ports()->addPort(acc);
  }
};
struct Singen : RTT::TaskContext {
  RTT::OutputPort<float> out{"out_sin_port"};
  explicit Singen(const std::string& n) : TaskContext(n) { ports()->addPort(out); }
};
struct Robot : RTT::TaskContext {
  RTT::InputPort<rstrt::dynamics::JointTorques> torques{"full_arm_JointTorqueCtrl"};
  explicit Robot(const std::string& n) : TaskContext(n) { ports()->addPort(torques); }
};

struct CycleData {
  rstrt::robot::JointState rs;
  VecF h, cp, cv, ca, dp, dv, da;
  MatF M, J, Jd;
  float sinv;
};

static CycleData make_cycle(int dof, const VecF& sup, const VecF& inf) {
  CycleData c;
  c.rs = rstrt::robot::JointState(dof);
  for (int j = 0; j < dof; ++j) {  // strictly inside the angle limits (finite log() limits)
    c.rs.angles[j] = inf[j] + (sup[j] - inf[j]) * urand(0.2f, 0.8f);
    c.rs.velocities[j] = urand(-0.5f, 0.5f);
    c.rs.torques[j] = urand(-1.f, 1.f);
  }
  c.h = vrand(dof, -5.f, 5.f);
  MatF A = mrand(dof, dof, -0.3f, 0.3f);
  c.M = MatF(dof, dof);
  for (int i = 0; i < dof; ++i)
    for (int j = 0; j < dof; ++j) {
      float s = i == j ? 1.0f : 0.f;
      for (int k = 0; k < dof; ++k) s += A(k, i) * A(k, j);
      c.M(i, j) = s;
    }
  c.J = mrand(3, dof, -1.f, 1.f);
  c.Jd = mrand(3, dof, -0.1f, 0.1f);
  c.cp = vrand(3, -0.5f, 0.5f);
  c.cv = vrand(3, -0.2f, 0.2f);
  c.ca = vrand(3, -0.1f, 0.1f);
  c.dp = vrand(3, -0.5f, 0.5f);
  c.dv = vrand(3, -0.2f, 0.2f);
  c.da = vrand(3, -0.1f, 0.1f);
  c.sinv = urand(-0.5f, 0.5f);
  return c;
}

// the same cycle as CycleInputs (what the component must build from its ports): joint 7 gets
// the task-space ports, joint 1 the joint-space position (ops/mgqp.ops:228-236)
static mgqp_amd::CycleInputs as_inputs(const CycleData& c, int dof) {
  mgqp_amd::CycleInputs in;
  in.robotstatus.set(mgqp_amd::JointState{c.rs.angles, c.rs.velocities});
  in.h.set(c.h);
  in.inertia.set(c.M);
  in.joints.resize(dof);
  auto& j7 = in.joints[dof - 1];
  j7.jacobian.set(c.J);
  j7.jacobianDot.set(c.Jd);
  j7.currentTaskSpacePosition.set(c.cp);
  j7.currentTaskSpaceVelocity.set(c.cv);
  j7.currentTaskSpaceAcceleration.set(c.ca);
  j7.desiredTaskSpacePosition.set(c.dp);
  j7.desiredTaskSpaceVelocity.set(c.dv);
  j7.desiredTaskSpaceAcceleration.set(c.da);
  in.joints[0].desiredJointSpacePosition.set(c.sinv);
  return in;
}

static void configure_ops(RTT::TaskContext* tc, const VecF& sup, const VecF& inf, int dof) {
  // ops/mgqp.ops:184-197 and :258-263, every call by operation name
  tc->getOperation<void(unsigned int)>("setDOFsize")(dof);
  std::vector<double> tl(dof, 100.0), al(dof, 5.0), s(sup.begin(), sup.end()), i(inf.begin(), inf.end());
  std::vector<double> tln(dof, -100.0), aln(dof, -5.0);
  CHECK(tc->getOperation<bool(std::vector<double>, std::vector<double>)>("setTorqueLimits")(tl, tln));
  CHECK(tc->getOperation<bool(std::vector<double>, std::vector<double>)>("setAccelerationLimits")(al, aln));
  CHECK(tc->getOperation<bool(std::vector<double>, std::vector<double>)>("setAngularLimits")(s, i));
  auto prio = tc->getOperation<bool(std::string, int)>("setPriorityLevel");
  CHECK(prio("in_desiredTaskSpacePosition_" + std::to_string(dof), 0));
  CHECK(prio("in_desiredTaskSpaceVelocity_" + std::to_string(dof), 0));
  CHECK(prio("in_desiredTaskSpaceAcceleration_" + std::to_string(dof), 0));
  CHECK(prio("in_desiredJointSpacePosition_1", 2));
  CHECK(!prio("in_desiredJointSpacePosition_2", 4));  // level > stackSize is refused
}

static void configure_direct(mgqp_amd::MotionGenerationQuadraticProgram& c, const VecF& sup,
                             const VecF& inf, int dof) {
  c.setDOFsize(dof);
  CHECK(c.setTorqueLimits(std::vector<double>(dof, 100.0), std::vector<double>(dof, -100.0)));
  CHECK(c.setAccelerationLimits(std::vector<double>(dof, 5.0), std::vector<double>(dof, -5.0)));
  CHECK(c.setAngularLimits(std::vector<double>(sup.begin(), sup.end()),
                           std::vector<double>(inf.begin(), inf.end())));
  c.setPriorityLevel("in_desiredTaskSpacePosition_" + std::to_string(dof), 0);
  c.setPriorityLevel("in_desiredTaskSpaceVelocity_" + std::to_string(dof), 0);
  c.setPriorityLevel("in_desiredTaskSpaceAcceleration_" + std::to_string(dof), 0);
  c.setPriorityLevel("in_desiredJointSpacePosition_1", 2);
}

int main(int argc, char** argv) {
  const int cycles = argc > 1 ? std::atoi(argv[1]) : 20;
  const int dof = 7;
  const VecF sup = {0.8f, 1.5f, 2.5f, 1.5f, 3.0f, 1.5f, 3.0f};  // ops/mgqp.ops:189
  const VecF inf = {-0.8f, -1.5f, -2.5f, -1.5f, -3.0f, -1.5f, -3.0f};
  const std::string d = std::to_string(dof);

  RTT::Deployer dep;
  CHECK(dep.loadComponent("myTorqueController", "MotionGenerationQuadraticProgram"));
  CHECK(!dep.loadComponent("other", "NoSuchComponent"));
  CHECK(dep.setActivity("myTorqueController", 0.05, 50, 0));
  RTT::TaskContext* tc = dep.getPeer("myTorqueController");
  CHECK(tc && tc->getPeriod() == 0.05);
  auto* comp = dynamic_cast<mgqp_amd::rtt::MotionGenerationQuadraticProgram*>(tc);
  CHECK(comp != nullptr);
  if (!comp) return 1;
  CHECK((tc->getOperationNames() ==
         std::vector<std::string>{"printCurrentState", "setAccelerationLimits", "setAngularLimits",
                                  "setDOFsize", "setGains", "setPriorityLevel", "setTorqueLimits"}));
  bool threw = false;
  try {
    tc->getOperation<void(int)>("setDOFsize");  // wrong signature
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  configure_ops(tc, sup, inf, dof);
  // setDOFsize's port set: 3 + 11*DOF inputs, 11 outputs (src/mgqp.cpp:180-482)
  CHECK((int)tc->ports()->getPortNames().size() == 3 + 11 * dof + 11);
  CHECK(tc->ports()->getPort("in_jacobian_port_" + d) != nullptr);
  // the 10 limit ports by the names the reference registers (src/mgqp.cpp:412-469) and the
  // OCL reporter subscribes to (ops/logData.ops:17-26)
  static const char* kLimitPorts[] = {
      "out_jointPosLimitInf_port",    "out_jointPosLimitSup_port",    "out_jointVelLimitInf_port",
      "out_jointVelLimitSup_port",    "out_jointAccLimitInf_port",    "out_jointAccLimitSup_port",
      "out_jointAccDynLimitInf_port", "out_jointAccDynLimitSup_port", "out_jointTorqueLimitInf_port",
      "out_jointTorqueLimitSup_port"};
  for (const char* nm : kLimitPorts) CHECK(dynamic_cast<RTT::OutputPort<VecF>*>(tc->ports()->getPort(nm)) != nullptr);
  CHECK(tc->ports()->getPort("out_jointAccDynLimitSup") == nullptr);
  CHECK(tc->ports()->getPort("in_jacobian_port_" + std::to_string(dof + 1)) == nullptr);

  Fkin fkin("fkin7");
  Traj traj("trajectorygenerator2");
  Singen sg("singen");
  Robot robot("robot_gazebo");
  for (RTT::TaskContext* p : std::initializer_list<RTT::TaskContext*>{&fkin, &traj, &sg, &robot}) dep.addPeer(p);

  CHECK(!tc->configure());  // nothing connected yet: configureHook refuses
  RTT::ConnPolicy cp;
  // ops/mgqp.ops:214-236, port by port by name
  CHECK(dep.connect("fkin7.out_robotstatus_port", "myTorqueController.in_robotstatus_port", cp));
  CHECK(dep.connect("fkin7.out_coriolisAndGravity_port", "myTorqueController.in_h_port", cp));
  CHECK(dep.connect("fkin7.out_inertia_port", "myTorqueController.in_inertia_port", cp));
  CHECK(dep.connect("fkin7.out_jacobianTranslation_port", "myTorqueController.in_jacobian_port_" + d, cp));
  CHECK(dep.connect("fkin7.out_jacobianDotTranslation_port", "myTorqueController.in_jacobianDot_port_" + d, cp));
  CHECK(dep.connect("fkin7.out_cartPosTranslation_port", "myTorqueController.in_currentTaskSpacePosition_port_" + d, cp));
  CHECK(dep.connect("fkin7.out_cartVelTranslation_port", "myTorqueController.in_currentTaskSpaceVelocity_port_" + d, cp));
  CHECK(dep.connect("fkin7.out_cartAccTranslation_port", "myTorqueController.in_currentTaskSpaceAcceleration_port_" + d, cp));
  CHECK(dep.connect("trajectorygenerator2.out_desiredTaskSpacePosition_port", "myTorqueController.in_desiredTaskSpacePosition_port_" + d, cp));
  CHECK(dep.connect("trajectorygenerator2.out_desiredTaskSpaceVelocity_port", "myTorqueController.in_desiredTaskSpaceVelocity_port_" + d, cp));
  CHECK(dep.connect("trajectorygenerator2.out_desiredTaskSpaceAcceleration_port", "myTorqueController.in_desiredTaskSpaceAcceleration_port_" + d, cp));
  CHECK(dep.connect("singen.out_sin_port", "myTorqueController.in_desiredJointSpacePosition_port_1", cp));
  CHECK(!dep.connect("singen.out_sin_port", "myTorqueController.in_h_port", cp));  // type mismatch
  CHECK(!tc->configure());  // out_torques_port still unconnected
  CHECK(dep.connect("myTorqueController.out_torques_port", "robot_gazebo.full_arm_JointTorqueCtrl", cp));
  // every limit port connected by name, as ops/logData.ops:17-26 reports them
  std::vector<std::unique_ptr<RTT::InputPort<VecF>>> limit_sinks;
  for (const char* nm : kLimitPorts) {
    limit_sinks.emplace_back(new RTT::InputPort<VecF>(std::string("sink_") + nm));
    CHECK(dynamic_cast<RTT::OutputPort<VecF>*>(tc->ports()->getPort(nm))->connectTo(*limit_sinks.back()));
  }
  RTT::InputPort<VecF>& accdyn_sink = *limit_sinks[6];
  CHECK(tc->configure());
  CHECK(tc->start());

  // before any input sample: "FAILED, NO DATA, RETURN", nothing written
  CHECK(tc->update());
  CHECK(comp->lastCycleCode() == mgqp_amd::CYCLE_NO_DATA);
  rstrt::dynamics::JointTorques got;
  CHECK(robot.torques.read(got) == RTT::NoData);

  mgqp_amd::MotionGenerationQuadraticProgram direct;
  configure_direct(direct, sup, inf, dof);

  int written = 0;
  for (int k = 0; k < cycles; ++k) {
    const CycleData c = make_cycle(dof, sup, inf);
    const bool fresh = (k % 3) != 2;  // every third cycle: no new samples -> OldData re-use
    static CycleData last;
    const CycleData& used = fresh ? c : last;
    if (fresh) {
      fkin.out_robotstatus_port.write(c.rs);
      fkin.out_coriolisAndGravity_port.write(c.h);
      fkin.out_inertia_port.write(c.M);
      fkin.out_jacobianTranslation_port.write(c.J);
      fkin.out_jacobianDotTranslation_port.write(c.Jd);
      fkin.out_cartPosTranslation_port.write(c.cp);
      fkin.out_cartVelTranslation_port.write(c.cv);
      fkin.out_cartAccTranslation_port.write(c.ca);
      traj.pos.write(c.dp);
      traj.vel.write(c.dv);
      traj.acc.write(c.da);
      sg.out.write(c.sinv);
      last = c;
    }
    CHECK(tc->update());
    mgqp_amd::CycleOutputs ref;
    direct.updateHook(as_inputs(used, dof), ref);
    CHECK(comp->lastCycleCode() == ref.code);
    if (ref.code != mgqp_amd::CYCLE_WRITTEN) continue;
    const RTT::FlowStatus fs = robot.torques.read(got);
    CHECK(fs == RTT::NewData);
    CHECK(same_bits(got.torques, ref.torques));
    VecF dyn;
    CHECK(accdyn_sink.read(dyn) == RTT::NewData);
    CHECK(same_bits(dyn, ref.jointAccDynLimitInf));
    ++written;
  }
  CHECK(written == cycles);
  CHECK(robot.torques.read(got) == RTT::OldData);  // no new cycle since the last read

  // the jacobian of the task joint disconnected: "FAILED, NO JACOBIAN FOR JOINT 7 RETURN"
  tc->ports()->getPort("in_jacobian_port_" + d)->disconnect();
  CHECK(tc->update());
  CHECK(comp->lastCycleCode() == mgqp_amd::CYCLE_NO_JACOBIAN);

  // a second setDOFsize rebuilds the port set (old connections dropped)
  tc->getOperation<void(unsigned int)>("setDOFsize")(3);
  CHECK((int)tc->ports()->getPortNames().size() == 3 + 11 * 3 + 11);
  CHECK(tc->ports()->getPort("in_jacobian_port_7") == nullptr);
  CHECK(!dynamic_cast<RTT::InputPort<VecF>*>(tc->ports()->getPort("in_h_port"))->connected());
  // the reference's removePort names miss the limit ports' "_port" suffix (src/mgqp.cpp:187-196
  // vs :412-469): they are not removed there, but re-adding them under the same name replaces
  // them through addPort, which disconnects the old registration (RTT 2.x addLocalPort ->
  // removeLocalPort): present, no longer connected
  for (const char* nm : kLimitPorts) {
    CHECK(tc->ports()->getPort(nm) != nullptr);
    CHECK(!dynamic_cast<RTT::OutputPort<VecF>*>(tc->ports()->getPort(nm))->connected());
  }

  // a throwing solve puts the component in the Exception state, like an exception escaping
  // RTT's updateHook: the task joint's jacobian has three identical rows, so level 0's
  // equalities are linearly dependent (solve_quadprog throws, src/mgqp.cpp:708)
  {
    RTT::Deployer d2;
    CHECK(d2.loadComponent("c2", "MotionGenerationQuadraticProgram"));
    RTT::TaskContext* t2 = d2.getPeer("c2");
    t2->getOperation<void(unsigned int)>("setDOFsize")(2);
    CHECK(t2->getOperation<bool(std::string, int)>("setPriorityLevel")("in_desiredTaskSpacePosition_2", 0));
    Fkin f2("f2");
    Traj g2("g2");
    Robot r2("r2");
    d2.addPeer(&f2);
    d2.addPeer(&g2);
    d2.addPeer(&r2);
    CHECK(d2.connect("f2.out_robotstatus_port", "c2.in_robotstatus_port"));
    CHECK(d2.connect("f2.out_coriolisAndGravity_port", "c2.in_h_port"));
    CHECK(d2.connect("f2.out_inertia_port", "c2.in_inertia_port"));
    CHECK(d2.connect("f2.out_jacobianTranslation_port", "c2.in_jacobian_port_2"));
    CHECK(d2.connect("f2.out_jacobianDotTranslation_port", "c2.in_jacobianDot_port_2"));
    CHECK(d2.connect("f2.out_cartPosTranslation_port", "c2.in_currentTaskSpacePosition_port_2"));
    CHECK(d2.connect("g2.out_desiredTaskSpacePosition_port", "c2.in_desiredTaskSpacePosition_port_2"));
    CHECK(d2.connect("c2.out_torques_port", "r2.full_arm_JointTorqueCtrl"));
    CHECK(t2->configure() && t2->start());
    f2.out_robotstatus_port.write(rstrt::robot::JointState(2));
    f2.out_coriolisAndGravity_port.write(VecF(2, 0.f));
    f2.out_inertia_port.write(MatF::identity(2));
    MatF J(3, 2, 0.f);
    for (int r = 0; r < 3; ++r) J(r, 0) = 1.f;
    f2.out_jacobianTranslation_port.write(J);
    f2.out_jacobianDotTranslation_port.write(MatF(3, 2, 0.f));
    f2.out_cartPosTranslation_port.write(VecF{0.f, 0.f, 0.f});
    g2.pos.write(VecF{0.1f, 0.2f, 0.3f});
    CHECK(!t2->update());
    CHECK(t2->getTaskState() == RTT::TaskContext::Exception);
    CHECK(t2->lastException() == "Constraints are linearly dependent");
    CHECK(!t2->update() && t2->recover() && t2->getTaskState() == RTT::TaskContext::Stopped);
    rstrt::dynamics::JointTorques none;
    CHECK(r2.torques.read(none) == RTT::NoData);
  }

  // update_batched: the controller's member stack comes from the last robot that completed its
  // cycle, never from a robot whose solve threw (here the last one: dependent equalities)
  {
    mgqp_amd::MotionGenerationQuadraticProgram bc;
    configure_direct(bc, sup, inf, dof);
    std::vector<mgqp_amd::CycleInputs> ins;
    ins.push_back(as_inputs(make_cycle(dof, sup, inf), dof));
    mgqp_amd::CycleInputs bad = as_inputs(make_cycle(dof, sup, inf), dof);
    MatF J(3, dof, 0.f);
    for (int r = 0; r < 3; ++r) J(r, 0) = 1.f;  // three identical task rows on level 0
    bad.joints[dof - 1].jacobian.set(J);
    ins.push_back(bad);
    std::vector<mgqp_amd::CycleOutputs> outs(2);
    bc.update_batched(ins.data(), outs.data(), 2, 1);
    CHECK(outs[0].code == mgqp_amd::CYCLE_WRITTEN && outs[1].code == mgqp_amd::CYCLE_EXCEPTION);
    mgqp_amd::MotionGenerationQuadraticProgram one;
    configure_direct(one, sup, inf, dof);
    mgqp_amd::CycleOutputs o1;
    one.updateHook(ins[0], o1);
    const auto& a = bc.stack_of_tasks.qps[0];
    const auto& b = one.stack_of_tasks.qps[0];
    CHECK(a.conditions.rows == b.conditions.rows && a.conditions.a == b.conditions.a &&
          a.goal == b.goal && a.limits == b.limits);
  }

  std::printf("%s: %d cycles through ports == CycleInputs path (bitwise), %d failures\n",
              g_fail ? "FAILED" : "OK", written, g_fail);
  return g_fail ? 1 : 0;
}
