// mgqp_controller.cpp — the reference component's QP builder and hierarchy solver, with every QP
// solved on the gfx950 kernels.  See include/quadprog_amd/mgqp.hh.
//
// Float arithmetic follows the reference expressions element by element (Eigen::MatrixXf /
// VectorXf there, MatF / VecF here); matrix products accumulate left to right.  Eigen's own
// product kernels and JacobiSVD are not available in this image, so the float glue is "parity
// unpinned" at the last bits; the QP solves inside it are bitwise QuadProg++.
#include "quadprog_amd/mgqp.hh"

#include <algorithm>
#include <cmath>
#include <iostream>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "qpgpu.h"
#include "quadprog_amd/QuadProg++.hh"

namespace mgqp_amd {

MatF MatF::identity(int n) {
  MatF I(n, n, 0.f);
  for (int i = 0; i < n; ++i) I(i, i) = 1.f;
  return I;
}

int QuadraticProblem::init(int DOFsize) {  // include/mgqp.hpp:41-48
  pbDOF = DOFsize;
  conditions = MatF(0, DOFsize);
  goal.clear();
  constraints = MatF(0, DOFsize);
  limits.clear();
  return 0;
}

int StackOfTasks::init(int nbOfLevels) {  // include/mgqp.hpp:58
  stackSize = nbOfLevels;
  qps.resize(stackSize);
  return 0;
}

int StackOfTasks::getLevel(const std::string& task) const {  // include/mgqp.hpp:62
  auto it = level.find(task);
  return it == level.end() ? -1 : it->second;
}

bool StackOfTasks::setPriority(const std::string& task, int priorityLevel) {  // mgqp.hpp:63
  if (priorityLevel >= stackSize) return false;
  level[task] = priorityLevel;
  return true;
}

namespace {

constexpr bool kTryToConverge = true;  // src/mgqp.cpp:20

std::string cat(const char* s, int i) { return std::string(s) + std::to_string(i); }

MatF mul(const MatF& A, const MatF& B) {
  MatF C(A.rows, B.cols, 0.f);
  for (int i = 0; i < A.rows; ++i)
    for (int j = 0; j < B.cols; ++j) {
      float s = 0.f;
      for (int k = 0; k < A.cols; ++k) s += A(i, k) * B(k, j);
      C(i, j) = s;
    }
  return C;
}

VecF mulv(const MatF& A, const VecF& x) {
  VecF y(A.rows, 0.f);
  for (int i = 0; i < A.rows; ++i) {
    float s = 0.f;
    for (int k = 0; k < A.cols; ++k) s += A(i, k) * x[k];
    y[i] = s;
  }
  return y;
}

// matrixAppend (src/mgqp.cpp:574-617): puts b under a; copies b when a is empty; a column
// mismatch is reported and ignored.
void matrixAppend(MatF* a, const MatF& b) {
  if (a->rows == 0) {
    *a = b;
    return;
  }
  if (b.rows == 0) return;
  if (a->cols != b.cols) {
    std::cerr << "DIM ERR - A.size() : (" << a->rows << "x" << a->cols << ")B.size() : ("
              << b.rows << "x" << b.cols << ")\n";
    return;
  }
  a->a.insert(a->a.end(), b.a.begin(), b.a.end());
  a->rows += b.rows;
}

void matrixAppend(VecF* a, const VecF& b) {
  if (a->empty()) {
    *a = b;
    return;
  }
  a->insert(a->end(), b.begin(), b.end());
}

// addToProblem (src/mgqp.cpp:619-648)
void addToProblem(const MatF& conditions, const VecF& goal, QuadraticProblem& problem) {
  if (conditions.cols != problem.dof())
    throw std::length_error(
        "condition matrix number of columns does not match the problem's number of columns");
  if ((size_t)conditions.rows != goal.size())
    throw std::length_error(
        "condition matrix number of rows is different than the goals number of rows");
  matrixAppend(&problem.conditions, conditions);
  matrixAppend(&problem.goal, goal);
}

// One-sided (Hestenes) Jacobi on the columns of X (rows x k, row-major, double).  Returns the
// column norms; X's columns end up mutually orthogonal, W (k x k) accumulates the rotations.
void hestenes(std::vector<double>& X, int rows, int k, std::vector<double>* W) {
  for (int sweep = 0; sweep < 80; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < k - 1; ++p)
      for (int q = p + 1; q < k; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int i = 0; i < rows; ++i) {
          const double xp = X[(size_t)i * k + p], xq = X[(size_t)i * k + q];
          al += xp * xp;
          be += xq * xq;
          ga += xp * xq;
        }
        if (ga == 0.0 || std::fabs(ga) <= 1e-15 * std::sqrt(al * be)) continue;
        rotated = true;
        const double zeta = (be - al) / (2.0 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < rows; ++i) {
          double& xp = X[(size_t)i * k + p];
          double& xq = X[(size_t)i * k + q];
          const double a0 = xp, b0 = xq;
          xp = c * a0 - s * b0;
          xq = s * a0 + c * b0;
        }
        if (W)
          for (int i = 0; i < k; ++i) {
            double& wp = (*W)[(size_t)i * k + p];
            double& wq = (*W)[(size_t)i * k + q];
            const double a0 = wp, b0 = wq;
            wp = c * a0 - s * b0;
            wq = s * a0 + c * b0;
          }
      }
    if (!rotated) break;
  }
}

}  // namespace

// src/mgqp.cpp:836-862.  Thin SVD Acumul = U S V^T (V: dim x min(r, dim)), then
// Z = I - V A V^T with A(k,k) = 1 when sigma_k >= 1e-16 (the reference zeroes A(k,k) below it).
MatF nullspace_projector(const MatF& A, int dim) {
  const int r = A.rows, c = A.cols;
  const int k = std::min(r, c);
  std::vector<double> V((size_t)c * k, 0.0);  // thin right singular vectors (columns)
  std::vector<bool> keep(k, false);
  if (r >= c) {
    std::vector<double> X((size_t)r * c), W((size_t)c * c, 0.0);
    for (size_t i = 0; i < X.size(); ++i) X[i] = A.a[i];
    for (int i = 0; i < c; ++i) W[(size_t)i * c + i] = 1.0;
    hestenes(X, r, c, &W);
    for (int j = 0; j < c; ++j) {
      double nrm = 0;
      for (int i = 0; i < r; ++i) nrm += X[(size_t)i * c + j] * X[(size_t)i * c + j];
      keep[j] = !((double)(float)std::sqrt(nrm) < 0.0000000000000001);
      for (int i = 0; i < c; ++i) V[(size_t)i * k + j] = W[(size_t)i * c + j];
    }
  } else {
    // A^T = V S U^T: Jacobi on the columns of A^T (c x r); its normalised columns are V.
    std::vector<double> X((size_t)c * r);
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < c; ++j) X[(size_t)j * r + i] = A(i, j);
    hestenes(X, c, r, nullptr);
    for (int j = 0; j < r; ++j) {
      double nrm = 0;
      for (int i = 0; i < c; ++i) nrm += X[(size_t)i * r + j] * X[(size_t)i * r + j];
      const double sg = std::sqrt(nrm);
      keep[j] = !((double)(float)sg < 0.0000000000000001);
      if (sg > 0)
        for (int i = 0; i < c; ++i) V[(size_t)i * k + j] = X[(size_t)i * r + j] / sg;
    }
  }
  MatF Z = MatF::identity(dim);
  for (int i = 0; i < c && i < dim; ++i)
    for (int j = 0; j < c && j < dim; ++j) {
      double s = 0;
      for (int l = 0; l < k; ++l)
        if (keep[l]) s += V[(size_t)i * k + l] * V[(size_t)j * k + l];
      Z(i, j) = (i == j ? 1.f : 0.f) - (float)s;
    }
  return Z;
}

MotionGenerationQuadraticProgram::MotionGenerationQuadraticProgram() {
  stack_of_tasks.init(3);  // src/mgqp.cpp:97
  gainTranslationP = 100;  // src/mgqp.cpp:106-110
  gainTranslationD = 25;
  gainJointP = 200;
  gainJointD = 100;
}

void MotionGenerationQuadraticProgram::setDOFsize(unsigned int DOFsize) {
  // src/mgqp.cpp:180-482: (re)creates the per-joint ports; here the port set is implied by
  // CycleInputs::joints.  Output vectors are zero-initialised at DOFsize.
  DOFsize_ = (int)DOFsize;
  WorkspaceDimension = 3;
}

void MotionGenerationQuadraticProgram::setGains(float kp, float kd) {  // src/mgqp.cpp:1208-1212
  gainTranslationP = kp;
  gainTranslationD = kd;
}

static bool set_pair(const std::vector<double>& P, const std::vector<double>& N, int dof,
                     const char* what, VecF* dP, VecF* dN) {
  // src/mgqp.cpp:494-558 (doubleVToEigenV + set*LimitsE)
  if ((int)P.size() != dof || (int)N.size() != dof) {
    std::cerr << "Can't assign " << P.size() << " " << what << " limits to " << dof
              << " joints robot\n";
    return false;
  }
  dP->assign(P.begin(), P.end());
  dN->assign(N.begin(), N.end());
  return true;
}

bool MotionGenerationQuadraticProgram::setTorqueLimits(const std::vector<double>& P,
                                                       const std::vector<double>& N) {
  return set_pair(P, N, DOFsize_, "torque", &JointTorquesLimitsP, &JointTorquesLimitsN);
}
bool MotionGenerationQuadraticProgram::setAccelerationLimits(const std::vector<double>& P,
                                                             const std::vector<double>& N) {
  return set_pair(P, N, DOFsize_, "acceleration", &JointAccelerationLimitsP,
                  &JointAccelerationLimitsN);
}
bool MotionGenerationQuadraticProgram::setAngularLimits(const std::vector<double>& sup,
                                                        const std::vector<double>& inf) {
  return set_pair(sup, inf, DOFsize_, "joint", &JointLimitsSup, &JointLimitsInf);
}

bool MotionGenerationQuadraticProgram::setPriorityLevel(const std::string& task, int level) {
  if (level > stack_of_tasks.stackSize) {  // src/mgqp.cpp:560-569
    std::cerr << "priority level greater than the priority task size" << '\n';
    return false;
  }
  stack_of_tasks.setPriority(task, level);
  return true;
}

// ---------------------------------------------------------------------------------------------
// solveNextStep (src/mgqp.cpp:655-749), single robot: the drop-in solve_quadprog (GPU, batch 1).
bool MotionGenerationQuadraticProgram::solveNextStep(const MatF& A, const VecF& a, const MatF& B,
                                                     const VecF& b, VecF* res) {
  if (A.cols != B.cols) {
    std::cerr << "A and B matrix don't have the same DOF\nA.cols()=" << A.cols
              << " ; B.cols()=" << B.cols << "\n";
    throw std::logic_error("solveNextStep: A.cols() != B.cols()");  // assert at :665
  }
  const int pbDOF = A.cols;
  ArrayHH::Matrix<double> G(pbDOF, pbDOF), CE(A.rows, A.cols), CI(B.rows, B.cols);
  ArrayHH::Vector<double> g0(pbDOF), ce0(a.size()), ci0(b.size()), x(pbDOF);
  for (int i = 0; i < pbDOF; ++i)
    for (int j = 0; j < pbDOF; ++j) G[i][j] = i == j ? 1.0 : 0.0;  // JG = I (:672)
  for (int i = 0; i < A.rows; ++i)
    for (int j = 0; j < A.cols; ++j) CE[i][j] = A(i, j);
  for (int i = 0; i < B.rows; ++i)
    for (int j = 0; j < B.cols; ++j) CI[i][j] = B(i, j);
  for (size_t i = 0; i < a.size(); ++i) ce0[i] = a[i];
  for (size_t i = 0; i < b.size(); ++i) ci0[i] = b[i];
  for (int i = 0; i < pbDOF; ++i) g0[i] = 0.0;

  double sum = solve_quadprog(G, g0, ArrayHH::t(CE), ce0, ArrayHH::t(CI), ci0, x);  // :708
  res->assign(pbDOF, 0.f);
  for (int i = 0; i < pbDOF; ++i) (*res)[i] = (float)x[i];
  if (std::isnan(sum) || sum == std::numeric_limits<double>::infinity()) {
    if (kTryToConverge) {  // :717-736 retry without inequalities
      CI.resize(0, pbDOF);
      ci0.resize(0);
      sum = solve_quadprog(G, g0, ArrayHH::t(CE), ce0, ArrayHH::t(CI), ci0, x);
      for (int i = 0; i < pbDOF; ++i) (*res)[i] = (float)x[i];
      if (std::isnan(sum) || sum == std::numeric_limits<double>::infinity()) {
        res->assign(pbDOF, 0.f);
        return false;
      }
      return true;
    }
    res->assign(pbDOF, 0.f);
    return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// solveNextHierarchy (src/mgqp.cpp:751-869) split into per-level halves so that the batched
// path can solve the QPs of one level for all robots in a single launch.
struct Hier {
  int dim = 0;
  MatF Acumul, Bcumul, Z;
  VecF acumul, bcumul, res, last_res, u;
  bool stepSuccess = true;  // uninitialised in the reference; only read after a solve there
  bool done = false;
  VecF result;

  void begin(int d) {
    dim = d;
    Acumul = MatF(0, d);
    Bcumul = MatF(0, d);
    acumul.clear();
    bcumul.clear();
    last_res.assign(d, 0.f);
    res.assign(d, 0.f);
    u.assign(d, 0.f);
    Z = MatF::identity(d);
    done = false;
  }
  // Stacks this level's inequalities and builds its QP.  Returns 0 (skip the level, `continue`
  // at :781), 1 (solve A,a,B,b), or 2 (no solve at this level but finish() still runs).
  int prepare(const QuadraticProblem& p, MatF& A, VecF& a, MatF& B, VecF& b) {
    matrixAppend(&Bcumul, p.constraints);
    matrixAppend(&bcumul, p.limits);
    last_res = res;
    if (p.conditions.rows == 0 && p.constraints.rows == 0) return 0;
    if (p.conditions.rows > 0 && Bcumul.rows > 0) {  // pb1 (:783) and pb2 (:789)
      A = mul(p.conditions, Z);
      VecF cl = mulv(p.conditions, last_res);
      a.resize(p.goal.size());
      for (size_t i = 0; i < a.size(); ++i) a[i] = p.goal[i] - cl[i];
      B = mul(Bcumul, Z);
      b = bcumul;
      return 1;
    }
    if (p.conditions.rows > 0 && p.constraints.rows == 0 && Bcumul.rows == 0) {  // pb3 (:795)
      A = mul(p.conditions, Z);
      VecF cl = mulv(p.conditions, last_res);
      a.resize(p.goal.size());
      for (size_t i = 0; i < a.size(); ++i) a[i] = p.goal[i] - cl[i];
      B = MatF(1, Z.cols, 0.f);
      b.assign(1, 0.f);
      return 1;
    }
    return 2;
  }
  // :814-867.  Returns false when the hierarchy stops at this level.
  bool finish(const QuadraticProblem& p) {
    if (!stepSuccess) {
      result = last_res;
      done = true;
      return false;
    }
    VecF zu = mulv(Z, u);
    for (int i = 0; i < dim; ++i) res[i] = last_res[i] + zu[i];
    if (p.conditions.rows > 0) {
      matrixAppend(&Acumul, p.conditions);
      matrixAppend(&acumul, p.goal);
      Z = nullspace_projector(Acumul, dim);
    }
    return true;
  }
};

VecF MotionGenerationQuadraticProgram::solveNextHierarchy() {
  Hier h;
  h.begin(2 * DOFsize_);
  for (int lvl = 0; lvl < stack_of_tasks.stackSize; ++lvl) {
    const QuadraticProblem& p = *stack_of_tasks.getQP(lvl);
    MatF A, B;
    VecF a, b;
    const int k = h.prepare(p, A, a, B, b);
    if (k == 0) continue;
    if (k == 1) h.stepSuccess = solveNextStep(A, a, B, b, &h.u);
    if (!h.finish(p)) return h.result;
  }
  return h.res;
}

// ---------------------------------------------------------------------------------------------
// updateHook (src/mgqp.cpp:872-1189), split into the builder (everything before
// solveNextHierarchy) and the output stage, shared by the single and batched paths.
namespace {

struct BuildState {
  VecF accP, accN;  // jointAccelAndAngleLimitP/N (:1113-1124)
};

// Returns CYCLE_WRITTEN when the stack is ready to solve, else the early-exit code.
int build_stack(const CycleInputs& in, int DOF, unsigned WD, float kTP, float kTD, float kJP,
                float kJD, StackOfTasks& sot, VecF& JointAccelerationLimitsP,
                VecF& JointAccelerationLimitsN, VecF& JointTorquesLimitsP,
                VecF& JointTorquesLimitsN, VecF& JointLimitsSup, VecF& JointLimitsInf,
                BuildState& bs, std::string& err) {
  if (!in.h.has || !in.inertia.has || !in.robotstatus.has) {
    err = "FAILED, NO DATA, RETURN";
    return CYCLE_NO_DATA;
  }
  const VecF& angles = in.robotstatus.v.angles;
  const VecF& velocities = in.robotstatus.v.velocities;
  if ((int)angles.size() < DOF || (int)velocities.size() < DOF || (int)in.joints.size() < DOF)
    throw std::length_error("robot status / joint port count smaller than DOFsize");
  for (int i = 0; i < sot.stackSize; ++i) sot.getQP(i)->init(2 * DOF);

  for (int j = 0; j < DOF; ++j) {
    const JointPorts& jp = in.joints[j];
    for (int lvl = 0; lvl < sot.stackSize; ++lvl) {
      QuadraticProblem* prob = sot.getQP(lvl);
      bool taskSpaceOperation = false, jointSpaceOperation = false;
      VecF dP(3, 0.f), cP(3, 0.f), dV(3, 0.f), cV(3, 0.f), dA(3, 0.f), cA(3, 0.f);
      auto head = [&](const VecF& v) {
        if (v.size() < WD) throw std::length_error("task-space port shorter than workspace");
        return VecF(v.begin(), v.begin() + WD);
      };
      if (jp.desiredTaskSpacePosition.has && jp.currentTaskSpacePosition.has &&
          sot.getLevel(cat("in_desiredTaskSpacePosition_", j + 1)) == lvl) {
        dP = head(jp.desiredTaskSpacePosition.v);
        cP = head(jp.currentTaskSpacePosition.v);
        taskSpaceOperation = true;
      }
      if (jp.desiredTaskSpaceVelocity.has && jp.currentTaskSpaceVelocity.has &&
          sot.getLevel(cat("in_desiredTaskSpaceVelocity_", j + 1)) == lvl) {
        dV = head(jp.desiredTaskSpaceVelocity.v);
        cV = head(jp.currentTaskSpaceVelocity.v);
        taskSpaceOperation = true;
      }
      if (jp.desiredTaskSpaceAcceleration.has && jp.currentTaskSpaceAcceleration.has &&
          sot.getLevel(cat("in_desiredTaskSpaceAcceleration_", j + 1)) == lvl) {
        dA = head(jp.desiredTaskSpaceAcceleration.v);
        cA = head(jp.currentTaskSpaceAcceleration.v);
        taskSpaceOperation = true;
      }
      if (taskSpaceOperation && (!jp.jacobian.has || !jp.jacobianDot.has)) {
        err = "FAILED, NO JACOBIAN FOR JOINT " + std::to_string(j + 1) + " RETURN";
        return CYCLE_NO_JACOBIAN;
      }
      float qd = angles[j], qdd = velocities[j], qddd = 0.f;
      if (jp.desiredJointSpacePosition.has &&
          sot.getLevel(cat("in_desiredJointSpacePosition_", j + 1)) == lvl) {
        qd = jp.desiredJointSpacePosition.v;
        jointSpaceOperation = true;
      }
      if (jp.desiredJointSpaceVelocity.has &&
          sot.getLevel(cat("in_desiredJointSpaceVelocity_", j + 1)) == lvl) {
        qdd = jp.desiredJointSpaceVelocity.v;
        jointSpaceOperation = true;
      }
      if (jp.desiredJointSpaceAcceleration.has &&
          sot.getLevel(cat("in_desiredJointSpaceAcceleration_", j + 1)) == lvl) {
        qddd = jp.desiredJointSpaceAcceleration.v;  // read but unused by the builder (:1017-1026)
        jointSpaceOperation = true;
      }
      (void)qddd;

      if (taskSpaceOperation) {  // :1038-1059
        const MatF& J = jp.jacobian.v;
        const MatF& Jd = jp.jacobianDot.v;
        if (J.rows != (int)WD || Jd.rows != J.rows || Jd.cols != J.cols || J.cols > 2 * DOF ||
            J.cols > (int)velocities.size())
          throw std::length_error("jacobian shape does not match the task space / DOF");
        MatF A(J.rows, 2 * DOF, 0.f);
        for (int r = 0; r < J.rows; ++r)
          for (int c = 0; c < J.cols; ++c) A(r, c) = J(r, c);
        VecF a(WD);
        for (unsigned r = 0; r < WD; ++r) {
          float jq = 0.f;  // (in_jacobianDot_var * qDot)(r)
          for (int c = 0; c < Jd.cols; ++c) jq += Jd(r, c) * velocities[c];
          float t = kTP * (dP[r] - cP[r]);
          t = t + kTD * (dV[r] - cV[r]);
          t = t - jq;
          t = t + dA[r];
          t = t - cA[r];
          a[r] = -t;
        }
        addToProblem(A, a, *prob);
      }
      if (jointSpaceOperation) {  // :1060-1070
        MatF A(1, 2 * DOF, 0.f);
        A(0, j) = 1.f;
        VecF a(1);
        a[0] = -(kJP * (qd - angles[j]) + kJD * (qdd - velocities[j]));
        addToProblem(A, a, *prob);
      }
    }
  }

  // inequalities (:1075-1134)
  const int nbInequality = 4 * DOF, half = nbInequality / 2, quarter = nbInequality / 4;
  MatF limitsMatrix(nbInequality, 2 * DOF, 0.f);
  VecF limits(nbInequality, 0.f);
  for (int i = 0; i < half; ++i) {
    limitsMatrix(i, i) = -1.f;
    limitsMatrix(half + i, i) = 1.f;
  }
  bs.accP = (int)JointAccelerationLimitsP.size() != DOF ? VecF(quarter, 0.f) : JointAccelerationLimitsP;
  bs.accN = (int)JointAccelerationLimitsN.size() != DOF ? VecF(quarter, 0.f) : JointAccelerationLimitsN;
  if ((int)JointLimitsSup.size() != DOF) JointLimitsSup.assign(DOF, 0.f);
  if ((int)JointLimitsInf.size() != DOF) JointLimitsInf.assign(DOF, 0.f);
  for (int i = 0; i < (int)bs.accP.size(); ++i) {
    // std::min/std::max on double: NaN in the second argument keeps the first (:1121-1122)
    const double lp = std::log((double)(float)(JointLimitsSup[i] - angles[i]));
    const double ln = -std::log((double)(float)(angles[i] - JointLimitsInf[i]));
    bs.accP[i] = (float)std::min((double)bs.accP[i], lp);
    bs.accN[i] = (float)std::max((double)bs.accN[i], ln);
  }
  const VecF tP = (int)JointTorquesLimitsP.size() != DOF ? VecF(quarter, 0.f) : JointTorquesLimitsP;
  const VecF tN = (int)JointTorquesLimitsN.size() != DOF ? VecF(quarter, 0.f) : JointTorquesLimitsN;
  for (int i = 0; i < quarter; ++i) {
    limits[i] = bs.accP[i];
    limits[quarter + i] = tP[i];
    limits[2 * quarter + i] = -bs.accN[i];
    limits[3 * quarter + i] = -tN[i];
  }
  QuadraticProblem* q0 = sot.getQP(0);
  q0->constraints = limitsMatrix;
  q0->limits = limits;
  // dynamics row [M -I] (:1136-1143)
  const MatF& M = in.inertia.v;
  if (M.rows != DOF || M.cols != DOF) throw std::length_error("inertia matrix is not DOF x DOF");
  MatF A(DOF, 2 * DOF, 0.f);
  for (int r = 0; r < DOF; ++r) {
    for (int c = 0; c < DOF; ++c) A(r, c) = M(r, c);
    A(r, DOF + r) = -1.f;
  }
  addToProblem(A, VecF(DOF, 0.f), *q0);
  return CYCLE_WRITTEN;
}

}  // namespace

namespace {

// Output stage of updateHook (:1146-1176).
void write_outputs(CycleOutputs& out, const VecF& tracking, const VecF& h, int DOF,
                   const VecF& JointLimitsInf, const VecF& JointLimitsSup,
                   const VecF& JointAccelerationLimitsN, const VecF& JointAccelerationLimitsP,
                   const VecF& JointTorquesLimitsN, const VecF& JointTorquesLimitsP,
                   const BuildState& bs) {
  if ((int)h.size() < DOF) throw std::length_error("h port shorter than DOFsize");
  out.tracking = tracking;
  out.torques.assign(DOF, 0.f);
  for (int i = 0; i < DOF; ++i) out.torques[i] = tracking[DOF + i] + h[i];
  out.jointPosLimitInf = JointLimitsInf;
  out.jointPosLimitSup = JointLimitsSup;
  out.jointVelLimitInf.assign(DOF, 0.f);
  out.jointVelLimitSup.assign(DOF, 0.f);
  out.jointAccLimitInf = JointAccelerationLimitsN;
  out.jointAccLimitSup = JointAccelerationLimitsP;
  out.jointAccDynLimitInf = bs.accN;
  out.jointAccDynLimitSup = JointAccelerationLimitsP;  // reference defect kept (:1161)
  out.jointTorqueLimitInf = JointTorquesLimitsN;
  out.jointTorqueLimitSup = JointTorquesLimitsP;
  out.code = CYCLE_WRITTEN;
  out.error.clear();
}

template <class F>
void parallel_for(long count, int threads, F&& fn) {
  if (threads <= 1 || count < 64) {
    for (long i = 0; i < count; ++i) fn(i);
    return;
  }
  std::vector<std::thread> pool;
  const long chunk = (count + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const long b = t * chunk, e = std::min(count, b + chunk);
    if (b >= e) break;
    pool.emplace_back([&fn, b, e] {
      for (long i = b; i < e; ++i) fn(i);
    });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

void MotionGenerationQuadraticProgram::updateHook(const CycleInputs& in, CycleOutputs& out) {
  BuildState bs;
  std::string err;
  const int code = build_stack(in, DOFsize_, WorkspaceDimension, gainTranslationP,
                               gainTranslationD, gainJointP, gainJointD, stack_of_tasks,
                               JointAccelerationLimitsP, JointAccelerationLimitsN,
                               JointTorquesLimitsP, JointTorquesLimitsN, JointLimitsSup,
                               JointLimitsInf, bs, err);
  if (code != CYCLE_WRITTEN) {
    out.code = code;
    out.error = err;
    return;
  }
  const VecF tracking = solveNextHierarchy();
  write_outputs(out, tracking, in.h.v, DOFsize_, JointLimitsInf, JointLimitsSup,
                JointAccelerationLimitsN, JointAccelerationLimitsP, JointTorquesLimitsN,
                JointTorquesLimitsP, bs);
}

// ---------------------------------------------------------------------------------------------
// Batched cycles.  Robots advance through the hierarchy level by level; the QPs of a level are
// grouped by shape (p, m) and each group is one qpgpu_solve_batched_host() call, i.e. one
// kernel launch for all robots.  The retry without inequalities (:717-736) is a second launch
// over the robots whose first solve returned NaN or +inf.
struct BatchRunner {
  struct Robot {
    StackOfTasks sot;
    Hier h;
    BuildState bs;
    int code = CYCLE_NO_DATA;
    std::string err;
    bool active = false;
    int kind = 0;
    MatF A, B;
    VecF a, b;
    double f = 0;
    int32_t status = 0;
  };

  static void solve_group(std::vector<Robot*>& rs, int n, int p, int m, bool drop_ci,
                          int threads, std::vector<std::vector<double>>* xs) {
    const long cnt = (long)rs.size();
    const int mm = drop_ci ? 0 : m;
    std::vector<double> G((size_t)cnt * n * n), g0((size_t)cnt * n, 0.0), CE((size_t)cnt * n * p),
        ce0((size_t)cnt * p), CI((size_t)cnt * n * mm), ci0((size_t)cnt * mm), x((size_t)cnt * n),
        f(cnt);
    std::vector<int32_t> st(cnt);
    parallel_for(cnt, threads, [&](long r) {
      const Robot& R = *rs[r];
      double* Gq = &G[(size_t)r * n * n];
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Gq[i * n + j] = i == j ? 1.0 : 0.0;
      double* CEq = &CE[(size_t)r * n * p];  // CE = t(A): n x p
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < p; ++j) CEq[i * p + j] = R.A(j, i);
      for (int j = 0; j < p; ++j) ce0[(size_t)r * p + j] = R.a[j];
      double* CIq = mm ? &CI[(size_t)r * n * mm] : nullptr;
      for (int i = 0; i < n && mm; ++i)
        for (int j = 0; j < mm; ++j) CIq[i * mm + j] = R.B(j, i);
      for (int j = 0; j < mm; ++j) ci0[(size_t)r * mm + j] = R.b[j];
    });
    qpgpu_problem_desc d{};
    d.n = n;
    d.p = p;
    d.m = mm;
    d.batch = cnt;
    const int rc = qpgpu_solve_batched_host(&d, G.data(), g0.data(), p ? CE.data() : nullptr,
                                            p ? ce0.data() : nullptr, mm ? CI.data() : nullptr,
                                            mm ? ci0.data() : nullptr, x.data(), f.data(),
                                            st.data(), nullptr);
    if (rc != QPGPU_SUCCESS)
      throw std::runtime_error(std::string("qpgpu_solve_batched_host failed: ") +
                               qpgpu_last_error());
    xs->resize(cnt);
    for (long r = 0; r < cnt; ++r) {
      rs[r]->f = f[r];
      rs[r]->status = st[r];
      (*xs)[r].assign(x.begin() + (size_t)r * n, x.begin() + (size_t)(r + 1) * n);
    }
  }
};

void MotionGenerationQuadraticProgram::update_batched(const CycleInputs* in, CycleOutputs* out,
                                                      long count, int threads) {
  if (threads <= 0) threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  std::vector<BatchRunner::Robot> rob(count);
  const int DOF = DOFsize_, dim = 2 * DOF;
  // The builder replaces wrongly sized angle limits with zeros (:1116-1117) on the member;
  // every robot does the same with its copy, and the member is updated once here.
  VecF sup0 = JointLimitsSup, inf0 = JointLimitsInf;
  parallel_for(count, threads, [&](long r) {
    auto& R = rob[r];
    R.sot = stack_of_tasks;
    VecF aP = JointAccelerationLimitsP, aN = JointAccelerationLimitsN, tP = JointTorquesLimitsP,
         tN = JointTorquesLimitsN, sup = sup0, inf = inf0;
    try {
      R.code = build_stack(in[r], DOF, WorkspaceDimension, gainTranslationP, gainTranslationD,
                           gainJointP, gainJointD, R.sot, aP, aN, tP, tN, sup, inf, R.bs, R.err);
    } catch (const std::exception& e) {
      R.code = CYCLE_EXCEPTION;
      R.err = e.what();
    }
    R.active = R.code == CYCLE_WRITTEN;
    if (R.active) R.h.begin(dim);
  });
  if ((int)JointLimitsSup.size() != DOF) JointLimitsSup.assign(DOF, 0.f);
  if ((int)JointLimitsInf.size() != DOF) JointLimitsInf.assign(DOF, 0.f);

  for (int lvl = 0; lvl < stack_of_tasks.stackSize; ++lvl) {
    parallel_for(count, threads, [&](long r) {
      auto& R = rob[r];
      R.kind = R.active ? R.h.prepare(*R.sot.getQP(lvl), R.A, R.a, R.B, R.b) : 0;
    });
    std::map<std::pair<int, int>, std::vector<BatchRunner::Robot*>> groups;
    for (long r = 0; r < count; ++r)
      if (rob[r].kind == 1) groups[{rob[r].A.rows, rob[r].B.rows}].push_back(&rob[r]);
    for (auto& kv : groups) {
      std::vector<std::vector<double>> xs;
      BatchRunner::solve_group(kv.second, dim, kv.first.first, kv.first.second, false, threads,
                               &xs);
      std::vector<BatchRunner::Robot*> retry;
      for (size_t i = 0; i < kv.second.size(); ++i) {
        auto& R = *kv.second[i];
        if (R.status == QPGPU_QP_DEPENDENT || R.status == QPGPU_QP_MAX_ITER) {
          R.active = false;
          R.code = CYCLE_EXCEPTION;
          R.err = R.status == QPGPU_QP_DEPENDENT
                      ? "Constraints are linearly dependent"
                      : "qpgpu: active-set step cap reached (no reference equivalent)";
          continue;
        }
        R.h.u.assign(dim, 0.f);
        for (int j = 0; j < dim; ++j) R.h.u[j] = (float)xs[i][j];
        if (std::isnan(R.f) || R.f == std::numeric_limits<double>::infinity()) retry.push_back(&R);
        else R.h.stepSuccess = true;
      }
      if (!retry.empty()) {
        std::vector<std::vector<double>> xr;
        BatchRunner::solve_group(retry, dim, kv.first.first, kv.first.second, true, threads, &xr);
        for (size_t i = 0; i < retry.size(); ++i) {
          auto& R = *retry[i];
          if (R.status == QPGPU_QP_DEPENDENT || R.status == QPGPU_QP_MAX_ITER) {
            R.active = false;
            R.code = CYCLE_EXCEPTION;
            R.err = R.status == QPGPU_QP_DEPENDENT
                        ? "Constraints are linearly dependent"
                        : "qpgpu: active-set step cap reached (no reference equivalent)";
            continue;
          }
          for (int j = 0; j < dim; ++j) R.h.u[j] = (float)xr[i][j];
          if (std::isnan(R.f) || R.f == std::numeric_limits<double>::infinity()) {
            R.h.u.assign(dim, 0.f);
            R.h.stepSuccess = false;
          } else {
            R.h.stepSuccess = true;
          }
        }
      }
    }
    parallel_for(count, threads, [&](long r) {
      auto& R = rob[r];
      if (!R.active || R.kind == 0) return;
      if (!R.h.finish(*R.sot.getQP(lvl))) R.active = false;  // stops with last_res
    });
  }

  parallel_for(count, threads, [&](long r) {
    auto& R = rob[r];
    CycleOutputs& o = out[r];
    if (R.code != CYCLE_WRITTEN) {
      o.code = R.code;
      o.error = R.err;
      return;
    }
    const VecF tracking = R.h.done ? R.h.result : R.h.res;
    try {
      write_outputs(o, tracking, in[r].h.v, DOF, JointLimitsInf, JointLimitsSup,
                    JointAccelerationLimitsN, JointAccelerationLimitsP, JointTorquesLimitsN,
                    JointTorquesLimitsP, R.bs);
    } catch (const std::exception& e) {
      o.code = CYCLE_EXCEPTION;
      o.error = e.what();
    }
  });
  // the member stack (what solveNextHierarchy() reads) is the last robot's that completed its
  // cycle; a robot whose build or solve threw may hold a half-built stack, so it never leaks
  // into the controller, and with no completed robot the member is left untouched
  for (long r = count - 1; r >= 0; --r)
    if (out[r].code == CYCLE_WRITTEN) {
      stack_of_tasks = rob[r].sot;
      break;
    }
}

}  // namespace mgqp_amd
