// mgqp_device_host.cpp — host half of the device-resident controller cycle: turns the
// controller's configuration and the batch's port presence into a mgqp_dev::Plan (the builder's
// addToProblem sequence of reference src/mgqp.cpp:912-1143, identical for every robot of a batch
// because they share connected ports and priorities), then runs mgqp_dev::run_cycle.
#include <cmath>
#include <stdexcept>
#include <string>

#include "mgqp_amd.h"
#include "mgqp_device.h"
#include "mgqp_ctl.h"
#include "quadprog_amd/mgqp.hh"

namespace mgqp_amd {

namespace {
std::string cat(const char* s, int i) { return std::string(s) + std::to_string(i); }
}  // namespace

int MotionGenerationQuadraticProgram::update_device(const void* batch, float* torques,
                                                    float* tracking, int* codes, void* stream) {
  const mgqp_device_batch& b = *static_cast<const mgqp_device_batch*>(batch);
  const int D = DOFsize_;
  if (D <= 0 || D > mgqp_dev::kMaxDof || D > MGQP_MAX_DOF)
    throw std::length_error("DOFsize outside the device pipeline's range (1..16)");
  if (!b.h || !b.inertia || !b.angles || !b.velocities) return CYCLE_NO_DATA;  // :879-883
  if (b.status_len < D) throw std::length_error("robot status shorter than DOFsize");
  if (stack_of_tasks.stackSize > mgqp_dev::kMaxLevels)
    throw std::length_error("too many priority levels for the device pipeline");

  mgqp_dev::Plan P{};
  P.dof = D;
  P.ws = (int)WorkspaceDimension;
  P.dim = 2 * D;
  P.nlevels = stack_of_tasks.stackSize;
  P.nineq = 4 * D;
  P.kTP = gainTranslationP;
  P.kTD = gainTranslationD;
  P.kJP = gainJointP;
  P.kJD = gainJointD;
  P.angles = b.angles;
  P.velocities = b.velocities;
  P.h = b.h;
  P.inertia = b.inertia;
  P.status_len = b.status_len;
  P.solver_flags = b.solver_flags;

  // generators in the reference's order: joints outer, levels inner, task rows before the
  // joint row; the dynamics rows close level 0 (:1136-1143)
  const char* tsn[3] = {"in_desiredTaskSpacePosition_", "in_desiredTaskSpaceVelocity_",
                        "in_desiredTaskSpaceAcceleration_"};
  const char* jsn[3] = {"in_desiredJointSpacePosition_", "in_desiredJointSpaceVelocity_",
                        "in_desiredJointSpaceAcceleration_"};
  int ng = 0;
  auto add = [&](int type, int joint, int level, int flags, int rows) {
    if (ng >= mgqp_dev::kMaxGen) throw std::length_error("too many task generators");
    P.gen[ng++] = mgqp_dev::RowGen{type, joint, level, flags, 0, rows};
  };
  for (int j = 0; j < D; ++j) {
    for (int k = 0; k < 6; ++k) P.ts[j][k] = b.ts[j][k];
    for (int k = 0; k < 3; ++k) P.js[j][k] = b.js[j][k];
    P.jac[j] = b.jacobian[j];
    P.jacd[j] = b.jacobian_dot[j];
    P.ts_len[j] = b.ts_len[j];
    P.jac_cols[j] = b.jac_cols[j];
    for (int lvl = 0; lvl < stack_of_tasks.stackSize; ++lvl) {
      int tf = 0, jf = 0;
      for (int k = 0; k < 3; ++k)
        if (b.ts[j][k] && b.ts[j][k + 3] && stack_of_tasks.getLevel(cat(tsn[k], j + 1)) == lvl)
          tf |= 1 << k;
      if (tf && (!b.jacobian[j] || !b.jacobian_dot[j])) return CYCLE_NO_JACOBIAN;  // :988-993
      for (int k = 0; k < 3; ++k)
        if (b.js[j][k] && stack_of_tasks.getLevel(cat(jsn[k], j + 1)) == lvl) jf |= 1 << k;
      if (tf) {
        if (b.jac_rows[j] != P.ws || b.ts_len[j] < P.ws || b.jac_cols[j] > 2 * D ||
            b.jac_cols[j] > b.status_len || b.jac_cols[j] <= 0)
          throw std::length_error("jacobian shape does not match the task space / DOF");
        add(mgqp_dev::GEN_TASK, j, lvl, tf, P.ws);
      }
      if (jf) add(mgqp_dev::GEN_JOINT, j, lvl, jf, 1);
    }
  }
  add(mgqp_dev::GEN_DYN, 0, 0, 0, D);
  P.ngen = ng;
  // rows grouped by level (Acumul stacks levels in order), generator order inside a level
  int row = 0;
  for (int l = 0; l < P.nlevels; ++l) {
    P.level_row0[l] = row;
    for (int g = 0; g < ng; ++g)
      if (P.gen[g].level == l) {
        P.gen[g].row0 = row;
        row += P.gen[g].rows;
      }
    P.level_rows[l] = row - P.level_row0[l];
  }
  P.total_rows = row;

  // limits configuration (:1113-1117): wrong-sized vectors read as zeros; the angle limits are
  // replaced on the member like the reference does
  if ((int)JointLimitsSup.size() != D) JointLimitsSup.assign(D, 0.f);
  if ((int)JointLimitsInf.size() != D) JointLimitsInf.assign(D, 0.f);
  for (int i = 0; i < D; ++i) {
    P.accP[i] = (int)JointAccelerationLimitsP.size() == D ? JointAccelerationLimitsP[i] : 0.f;
    P.accN[i] = (int)JointAccelerationLimitsN.size() == D ? JointAccelerationLimitsN[i] : 0.f;
    P.tP[i] = (int)JointTorquesLimitsP.size() == D ? JointTorquesLimitsP[i] : 0.f;
    P.tN[i] = (int)JointTorquesLimitsN.size() == D ? JointTorquesLimitsN[i] : 0.f;
    P.sup[i] = JointLimitsSup[i];
    P.inf[i] = JointLimitsInf[i];
  }
  // limitsMatrix [-I; +I] (:1083-1085)
  std::vector<float> B((size_t)4 * D * 2 * D, 0.f);
  for (int i = 0; i < 2 * D; ++i) {
    B[(size_t)i * 2 * D + i] = -1.f;
    B[(size_t)(2 * D + i) * 2 * D + i] = 1.f;
  }
  const char* err = nullptr;
  const int rc = mgqp_dev::run_cycle(P, b.count, B.data(), torques, tracking,
                                     reinterpret_cast<int32_t*>(codes),
                                     static_cast<hipStream_t>(stream), &err);
  if (rc) throw std::runtime_error(std::string("mgqp device cycle: ") + (err ? err : "error"));
  return 0;
}

}  // namespace mgqp_amd

extern "C" int mgqp_update_device(mgqp_ctl* c, const mgqp_device_batch* b, float* torques,
                                  float* tracking, int32_t* codes, void* stream) {
  try {
    return c->c.update_device(b, torques, tracking, codes, stream);
  } catch (const std::exception& e) {
    mgqp_capi_set_error(e.what());
    return -1;
  }
}
