/* mgqp_amd.h — C-ABI of the motion-generation controller.
 *
 * Wraps mgqp_amd::MotionGenerationQuadraticProgram (include/quadprog_amd/mgqp.hh) for FFI
 * callers (ctypes in tests/ and bench.py).  Every entry replaces one member of the reference
 * component:
 *   mgqp_set_dof              <- setDOFsize            (reference src/mgqp.cpp:180)
 *   mgqp_set_gains            <- setGains              (src/mgqp.cpp:1208)
 *   mgqp_set_torque_limits    <- setTorqueLimits       (src/mgqp.cpp:494)
 *   mgqp_set_acceleration_limits <- setAccelerationLimits (src/mgqp.cpp:503)
 *   mgqp_set_angular_limits   <- setAngularLimits      (src/mgqp.cpp:512)
 *   mgqp_set_priority_level   <- setPriorityLevel      (src/mgqp.cpp:560)
 *   mgqp_update               <- updateHook            (src/mgqp.cpp:872-1189)
 *   mgqp_update_batched       <- updateHook for `count` robots in one pass (GPU batched solves)
 *   mgqp_nullspace_projector  <- the JacobiSVD null-space block (src/mgqp.cpp:836-862)
 * Input ports are pointers; NULL stands for RTT::NoData.  All matrices are row-major float.
 */
#ifndef MGQP_AMD_H
#define MGQP_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgqp_ctl mgqp_ctl;

typedef struct {
  const float* desired_ts_position;     /* in_desiredTaskSpacePosition_port_j   (ts_len) */
  const float* desired_ts_velocity;     /* in_desiredTaskSpaceVelocity_port_j */
  const float* desired_ts_acceleration; /* in_desiredTaskSpaceAcceleration_port_j */
  const float* current_ts_position;     /* in_currentTaskSpacePosition_port_j */
  const float* current_ts_velocity;     /* in_currentTaskSpaceVelocity_port_j */
  const float* current_ts_acceleration; /* in_currentTaskSpaceAcceleration_port_j */
  const float* desired_js_position;     /* in_desiredJointSpacePosition_port_j   (scalar) */
  const float* desired_js_velocity;     /* in_desiredJointSpaceVelocity_port_j */
  const float* desired_js_acceleration; /* in_desiredJointSpaceAcceleration_port_j */
  const float* jacobian;                /* in_jacobian_port_j     (jac_rows x jac_cols) */
  const float* jacobian_dot;            /* in_jacobianDot_port_j  (jac_rows x jac_cols) */
  int32_t ts_len;
  int32_t jac_rows;
  int32_t jac_cols;
  int32_t reserved;
} mgqp_joint_ports;

typedef struct {
  const float* angles;            /* in_robotstatus_port: angles (status_len) */
  const float* velocities;        /*                      velocities (status_len) */
  const float* h;                 /* in_h_port (DOF) */
  const float* inertia;           /* in_inertia_port (DOF x DOF) */
  const mgqp_joint_ports* joints; /* DOF entries; joint j <-> port suffix j+1 */
  int32_t status_len;
  int32_t reserved;
} mgqp_cycle_inputs;

/* updateHook exit codes */
enum {
  MGQP_CYCLE_WRITTEN = 0,     /* output ports written */
  MGQP_CYCLE_NO_DATA = 1,     /* "FAILED, NO DATA, RETURN" */
  MGQP_CYCLE_NO_JACOBIAN = 2, /* "FAILED, NO JACOBIAN FOR JOINT j RETURN" */
  MGQP_CYCLE_EXCEPTION = 3    /* the reference would throw (message in mgqp_last_error) */
};

mgqp_ctl* mgqp_create(void);
void mgqp_destroy(mgqp_ctl* c);
void mgqp_set_dof(mgqp_ctl* c, uint32_t dof);
void mgqp_set_gains(mgqp_ctl* c, float kp, float kd);
int mgqp_set_torque_limits(mgqp_ctl* c, const double* P, const double* N, int32_t count);
int mgqp_set_acceleration_limits(mgqp_ctl* c, const double* P, const double* N, int32_t count);
int mgqp_set_angular_limits(mgqp_ctl* c, const double* sup, const double* inf, int32_t count);
int mgqp_set_priority_level(mgqp_ctl* c, const char* task, int32_t level);

/* One cycle.  torques: DOF floats (out_torques); tracking: 2*DOF floats (solveNextHierarchy
 * result) or NULL; limits_out: 10*DOF floats (the ten out_joint*Limit* ports in declaration
 * order PosInf, PosSup, VelInf, VelSup, AccInf, AccSup, AccDynInf, AccDynSup, TorqueInf,
 * TorqueSup; entries of unset limits are NaN) or NULL.  Returns an MGQP_CYCLE_* code. */
int mgqp_update(mgqp_ctl* c, const mgqp_cycle_inputs* in, float* torques, float* tracking,
                float* limits_out);

/* `count` robots sharing this controller's configuration: torques count x DOF, tracking
 * count x 2*DOF (or NULL), codes count.  threads <= 0 picks min(16, cores).  Returns 0, or -1
 * when a GPU call failed (mgqp_last_error). */
int mgqp_update_batched(mgqp_ctl* c, int64_t count, const mgqp_cycle_inputs* in, float* torques,
                        float* tracking, int32_t* codes, int32_t threads);

/* Device-resident batch: every pointer is DEVICE memory, robot-major
 * (robot r's block at r * block size).  NULL = RTT::NoData for all robots of the batch. */
#define MGQP_MAX_DOF 16
typedef struct {
  int64_t count;
  const float* angles;      /* [count][status_len] */
  const float* velocities;  /* [count][status_len] */
  const float* h;           /* [count][DOF] */
  const float* inertia;     /* [count][DOF][DOF] */
  const float* ts[MGQP_MAX_DOF][6]; /* joint j: desired pos/vel/acc, current pos/vel/acc [count][ts_len[j]] */
  const float* js[MGQP_MAX_DOF][3]; /* joint j: desired joint pos/vel/acc [count] */
  const float* jacobian[MGQP_MAX_DOF];     /* [count][jac_rows[j]][jac_cols[j]] */
  const float* jacobian_dot[MGQP_MAX_DOF];
  int32_t ts_len[MGQP_MAX_DOF];
  int32_t jac_rows[MGQP_MAX_DOF];
  int32_t jac_cols[MGQP_MAX_DOF];
  int32_t status_len;
  uint32_t solver_flags; /* QPGPU_FLAG_* for the level solves: 0 (bitwise with the host paths) or
                            QPGPU_FLAG_FAST (the wave kernel's fast build: within 1e-10) */
} mgqp_device_batch;

/* One control cycle for `b->count` robots entirely on the GPU: builder, per-level QPs, the
 * batched solver (with the reference's retry without inequalities), null-space projector and
 * outputs, enqueued on `stream` (hipStream_t; NULL = default).  torques [count][DOF],
 * tracking [count][2*DOF] (or NULL), codes [count] are DEVICE arrays; codes get
 * MGQP_CYCLE_WRITTEN or MGQP_CYCLE_EXCEPTION per robot.  Returns 0, MGQP_CYCLE_NO_DATA /
 * MGQP_CYCLE_NO_JACOBIAN when the whole batch exits early like updateHook (nothing written),
 * or -1 on an argument / GPU error (mgqp_last_error).  Bit-identical to mgqp_update_batched. */
int mgqp_update_device(mgqp_ctl* c, const mgqp_device_batch* b, float* torques, float* tracking,
                       int32_t* codes, void* stream);

/* Z = I - V A V^T for Acumul (rows x cols), written as dim x dim. */
void mgqp_nullspace_projector(const float* A, int32_t rows, int32_t cols, int32_t dim, float* Z);

const char* mgqp_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
