// mgqp_capi.cpp — extern "C" wrapper of the controller (include/mgqp_amd.h).
#include <cmath>
#include <cstring>
#include <exception>
#include <limits>
#include <string>
#include <vector>

#include "mgqp_amd.h"
#include "mgqp_ctl.h"
#include "quadprog_amd/mgqp.hh"

using namespace mgqp_amd;


namespace {

thread_local std::string g_err;

VecF vec(const float* p, int n) { return VecF(p, p + n); }

MatF mat(const float* p, int r, int c) {
  MatF M(r, c);
  std::memcpy(M.a.data(), p, sizeof(float) * (size_t)r * c);
  return M;
}

CycleInputs convert(const mgqp_cycle_inputs& in, int DOF) {
  CycleInputs ci;
  if (in.angles && in.velocities) {
    JointState js;
    js.angles = vec(in.angles, in.status_len);
    js.velocities = vec(in.velocities, in.status_len);
    ci.robotstatus.set(js);
  }
  if (in.h) ci.h.set(vec(in.h, DOF));
  if (in.inertia) ci.inertia.set(mat(in.inertia, DOF, DOF));
  ci.joints.resize(DOF);
  for (int j = 0; j < DOF && in.joints; ++j) {
    const mgqp_joint_ports& p = in.joints[j];
    JointPorts& o = ci.joints[j];
    const int L = p.ts_len;
    if (p.desired_ts_position) o.desiredTaskSpacePosition.set(vec(p.desired_ts_position, L));
    if (p.desired_ts_velocity) o.desiredTaskSpaceVelocity.set(vec(p.desired_ts_velocity, L));
    if (p.desired_ts_acceleration)
      o.desiredTaskSpaceAcceleration.set(vec(p.desired_ts_acceleration, L));
    if (p.current_ts_position) o.currentTaskSpacePosition.set(vec(p.current_ts_position, L));
    if (p.current_ts_velocity) o.currentTaskSpaceVelocity.set(vec(p.current_ts_velocity, L));
    if (p.current_ts_acceleration)
      o.currentTaskSpaceAcceleration.set(vec(p.current_ts_acceleration, L));
    if (p.desired_js_position) o.desiredJointSpacePosition.set(*p.desired_js_position);
    if (p.desired_js_velocity) o.desiredJointSpaceVelocity.set(*p.desired_js_velocity);
    if (p.desired_js_acceleration) o.desiredJointSpaceAcceleration.set(*p.desired_js_acceleration);
    if (p.jacobian) o.jacobian.set(mat(p.jacobian, p.jac_rows, p.jac_cols));
    if (p.jacobian_dot) o.jacobianDot.set(mat(p.jacobian_dot, p.jac_rows, p.jac_cols));
  }
  return ci;
}

std::vector<double> dv(const double* p, int n) { return std::vector<double>(p, p + n); }

void put(float* dst, const VecF& v, int DOF) {
  for (int i = 0; i < DOF; ++i)
    dst[i] = i < (int)v.size() ? v[i] : std::numeric_limits<float>::quiet_NaN();
}

}  // namespace

extern "C" {

mgqp_ctl* mgqp_create(void) { return new mgqp_ctl(); }
void mgqp_destroy(mgqp_ctl* c) { delete c; }
void mgqp_set_dof(mgqp_ctl* c, uint32_t dof) { c->c.setDOFsize(dof); }
void mgqp_set_gains(mgqp_ctl* c, float kp, float kd) { c->c.setGains(kp, kd); }
int mgqp_set_torque_limits(mgqp_ctl* c, const double* P, const double* N, int32_t n) {
  return c->c.setTorqueLimits(dv(P, n), dv(N, n));
}
int mgqp_set_acceleration_limits(mgqp_ctl* c, const double* P, const double* N, int32_t n) {
  return c->c.setAccelerationLimits(dv(P, n), dv(N, n));
}
int mgqp_set_angular_limits(mgqp_ctl* c, const double* sup, const double* inf, int32_t n) {
  return c->c.setAngularLimits(dv(sup, n), dv(inf, n));
}
int mgqp_set_priority_level(mgqp_ctl* c, const char* task, int32_t level) {
  return c->c.setPriorityLevel(task, level);
}

int mgqp_update(mgqp_ctl* c, const mgqp_cycle_inputs* in, float* torques, float* tracking,
                float* limits_out) {
  const int DOF = c->c.DOFsize();
  CycleOutputs out;
  try {
    c->c.updateHook(convert(*in, DOF), out);
  } catch (const std::exception& e) {
    g_err = e.what();
    return MGQP_CYCLE_EXCEPTION;
  }
  if (out.code != CYCLE_WRITTEN) {
    g_err = out.error;
    return out.code;
  }
  put(torques, out.torques, DOF);
  if (tracking) put(tracking, out.tracking, 2 * DOF);
  if (limits_out) {
    const VecF* L[10] = {&out.jointPosLimitInf,   &out.jointPosLimitSup,   &out.jointVelLimitInf,
                         &out.jointVelLimitSup,   &out.jointAccLimitInf,   &out.jointAccLimitSup,
                         &out.jointAccDynLimitInf, &out.jointAccDynLimitSup,
                         &out.jointTorqueLimitInf, &out.jointTorqueLimitSup};
    for (int k = 0; k < 10; ++k) put(limits_out + k * DOF, *L[k], DOF);
  }
  return MGQP_CYCLE_WRITTEN;
}

int mgqp_update_batched(mgqp_ctl* c, int64_t count, const mgqp_cycle_inputs* in, float* torques,
                        float* tracking, int32_t* codes, int32_t threads) {
  const int DOF = c->c.DOFsize();
  try {
    std::vector<CycleInputs> ins(count);
    for (int64_t r = 0; r < count; ++r) ins[r] = convert(in[r], DOF);
    std::vector<CycleOutputs> outs(count);
    c->c.update_batched(ins.data(), outs.data(), count, threads);
    for (int64_t r = 0; r < count; ++r) {
      codes[r] = outs[r].code;
      if (outs[r].code != CYCLE_WRITTEN) {
        g_err = outs[r].error;
        continue;
      }
      put(torques + r * DOF, outs[r].torques, DOF);
      if (tracking) put(tracking + r * 2 * DOF, outs[r].tracking, 2 * DOF);
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  return 0;
}

void mgqp_nullspace_projector(const float* A, int32_t rows, int32_t cols, int32_t dim, float* Z) {
  MatF M = mat(A, rows, cols);
  MatF R = nullspace_projector(M, dim);
  std::memcpy(Z, R.a.data(), sizeof(float) * (size_t)dim * dim);
}

const char* mgqp_last_error(void) { return g_err.c_str(); }

void mgqp_capi_set_error(const char* msg) { g_err = msg; }

}  // extern "C"
