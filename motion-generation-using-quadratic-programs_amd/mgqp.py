"""mgqp — Python binding of the motion-generation controller.

ctypes over libmgqp_amd.so (include/mgqp_amd.h).  `Controller` mirrors the reference component's
operations (src/mgqp.cpp:89-95) and its updateHook (src/mgqp.cpp:872-1189); every QP it builds is
solved on the gfx950 kernels (single cycles through the drop-in solve_quadprog, batched cycles
through one qpgpu launch per level and shape).  No CPU solver exists behind it.

Ports: a `Scenario` holds `count` robots' port values as numpy arrays; a port that is not
connected (RTT::NoData) is simply absent from `Scenario.ports`.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmgqp_amd.so")

TS_PORTS = ("desired_ts_position", "desired_ts_velocity", "desired_ts_acceleration",
            "current_ts_position", "current_ts_velocity", "current_ts_acceleration")
JS_PORTS = ("desired_js_position", "desired_js_velocity", "desired_js_acceleration")
JOINT_FIELDS = TS_PORTS + JS_PORTS + ("jacobian", "jacobian_dot")
# reference port-name stems, used by setPriorityLevel (src/mgqp.cpp:946-1018)
PORT_TASK_NAME = {
    "desired_ts_position": "in_desiredTaskSpacePosition_",
    "desired_ts_velocity": "in_desiredTaskSpaceVelocity_",
    "desired_ts_acceleration": "in_desiredTaskSpaceAcceleration_",
    "desired_js_position": "in_desiredJointSpacePosition_",
    "desired_js_velocity": "in_desiredJointSpaceVelocity_",
    "desired_js_acceleration": "in_desiredJointSpaceAcceleration_",
}

CYCLE_WRITTEN, CYCLE_NO_DATA, CYCLE_NO_JACOBIAN, CYCLE_EXCEPTION = 0, 1, 2, 3
LIMIT_PORTS = ("jointPosLimitInf", "jointPosLimitSup", "jointVelLimitInf", "jointVelLimitSup",
               "jointAccLimitInf", "jointAccLimitSup", "jointAccDynLimitInf",
               "jointAccDynLimitSup", "jointTorqueLimitInf", "jointTorqueLimitSup")

# numpy images of the C structs (include/mgqp_amd.h)
JOINT_DTYPE = np.dtype([(f, np.uint64) for f in JOINT_FIELDS] +
                       [("ts_len", np.int32), ("jac_rows", np.int32), ("jac_cols", np.int32),
                        ("reserved", np.int32)])
CYCLE_DTYPE = np.dtype([("angles", np.uint64), ("velocities", np.uint64), ("h", np.uint64),
                        ("inertia", np.uint64), ("joints", np.uint64), ("status_len", np.int32),
                        ("reserved", np.int32)])
assert JOINT_DTYPE.itemsize == 104 and CYCLE_DTYPE.itemsize == 48

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback)")
        _lib = _bind(ctypes.CDLL(LIB_PATH))
    return _lib


def load_library(path: str):
    """Bind another build of the controller C-ABI (the tests' CPU harness uses this)."""
    return _bind(ctypes.CDLL(path))


def _bind(L):
    if True:
        vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
        L.mgqp_create.restype = vp
        L.mgqp_destroy.argtypes = [vp]
        L.mgqp_set_dof.argtypes = [vp, ctypes.c_uint32]
        L.mgqp_set_gains.argtypes = [vp, f32, f32]
        for nm in ("mgqp_set_torque_limits", "mgqp_set_acceleration_limits",
                   "mgqp_set_angular_limits"):
            getattr(L, nm).argtypes = [vp, vp, vp, i32]
            getattr(L, nm).restype = ctypes.c_int
        L.mgqp_set_priority_level.argtypes = [vp, ctypes.c_char_p, i32]
        L.mgqp_set_priority_level.restype = ctypes.c_int
        L.mgqp_update.argtypes = [vp, vp, vp, vp, vp]
        L.mgqp_update.restype = ctypes.c_int
        L.mgqp_update_batched.argtypes = [vp, ctypes.c_int64, vp, vp, vp, vp, i32]
        L.mgqp_update_batched.restype = ctypes.c_int
        L.mgqp_nullspace_projector.argtypes = [vp, i32, i32, i32, vp]
        if hasattr(L, "mgqp_update_device"):
            L.mgqp_update_device.argtypes = [vp, vp, vp, vp, vp, vp]
            L.mgqp_update_device.restype = ctypes.c_int
        L.mgqp_last_error.restype = ctypes.c_char_p
    return L


EXPORTED_SYMBOLS = ("mgqp_create", "mgqp_destroy", "mgqp_set_dof", "mgqp_set_gains",
                    "mgqp_set_torque_limits", "mgqp_set_acceleration_limits",
                    "mgqp_set_angular_limits", "mgqp_set_priority_level", "mgqp_update",
                    "mgqp_update_batched", "mgqp_update_device", "mgqp_nullspace_projector",
                    "mgqp_last_error")

MAX_DOF = 16
_P = ctypes.c_void_p


class DeviceBatchC(ctypes.Structure):
    """include/mgqp_amd.h mgqp_device_batch."""
    _fields_ = [("count", ctypes.c_int64), ("angles", _P), ("velocities", _P), ("h", _P),
                ("inertia", _P), ("ts", (_P * 6) * MAX_DOF), ("js", (_P * 3) * MAX_DOF),
                ("jacobian", _P * MAX_DOF), ("jacobian_dot", _P * MAX_DOF),
                ("ts_len", ctypes.c_int32 * MAX_DOF), ("jac_rows", ctypes.c_int32 * MAX_DOF),
                ("jac_cols", ctypes.c_int32 * MAX_DOF), ("status_len", ctypes.c_int32),
                ("solver_flags", ctypes.c_uint32)]


class DeviceScenario:
    """A Scenario uploaded to HBM (torch tensors, robot-major) plus the C struct pointing at it:
    the input of Controller.update_device (the device-resident cycle)."""

    def __init__(self, sc: Scenario, device="cuda"):
        import torch

        self.dof, self.count = sc.dof, sc.count
        t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)
        self.tensors = {"angles": t(sc.angles), "velocities": t(sc.velocities), "h": t(sc.h),
                        "inertia": t(sc.inertia)}
        self.ports = {k: t(v) for k, v in sc.ports.items()}
        b = DeviceBatchC()
        b.count = sc.count
        ptr = lambda x: None if x is None else x.data_ptr()
        for nm, x in self.tensors.items():
            setattr(b, nm, ptr(x))
        if sc.angles is not None:
            b.status_len = sc.angles.shape[1]
        ts_idx = {nm: i for i, nm in enumerate(TS_PORTS)}
        js_idx = {nm: i for i, nm in enumerate(JS_PORTS)}
        for (j, nm), x in self.ports.items():
            if nm in ts_idx:
                b.ts[j][ts_idx[nm]] = x.data_ptr()
                b.ts_len[j] = x.shape[1]
            elif nm in js_idx:
                b.js[j][js_idx[nm]] = x.data_ptr()
            else:
                (b.jacobian if nm == "jacobian" else b.jacobian_dot)[j] = x.data_ptr()
                b.jac_rows[j], b.jac_cols[j] = x.shape[1], x.shape[2]
        self.c = b


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


@dataclass
class Scenario:
    """Port values of `count` robots (float32, C-contiguous).

    angles/velocities: (count, status_len); h: (count, dof); inertia: (count, dof, dof);
    ports[(joint, name)]: (count, ts_len) for task-space ports, (count,) for joint-space
    scalars, (count, rows, cols) for jacobian / jacobian_dot.  A missing key is RTT::NoData;
    angles/h/inertia set to None are NoData too."""

    dof: int
    count: int
    angles: np.ndarray | None
    velocities: np.ndarray | None
    h: np.ndarray | None
    inertia: np.ndarray | None
    ports: dict = field(default_factory=dict)

    def robot(self, r: int) -> "Scenario":
        sl = slice(r, r + 1)
        pick = lambda a: None if a is None else np.ascontiguousarray(a[sl])
        return Scenario(self.dof, 1, pick(self.angles), pick(self.velocities), pick(self.h),
                        pick(self.inertia), {k: pick(v) for k, v in self.ports.items()})

    def pack(self):
        """Build the mgqp_cycle_inputs / mgqp_joint_ports arrays (vectorised).  Returns
        (cycles, joints, keepalive)."""
        K, D = self.count, self.dof
        keep = []

        def arr(a):
            a = np.ascontiguousarray(a, dtype=np.float32)
            keep.append(a)
            return a

        joints = np.zeros(K * D, dtype=JOINT_DTYPE).reshape(K, D)
        for (j, name), a in self.ports.items():
            a = arr(a)
            stride = a.strides[0]
            joints[name][:, j] = np.uint64(_ptr(a)) + np.arange(K, dtype=np.uint64) * np.uint64(stride)
            if name in TS_PORTS:
                joints["ts_len"][:, j] = a.shape[1]
            if name in ("jacobian", "jacobian_dot"):
                joints["jac_rows"][:, j] = a.shape[1]
                joints["jac_cols"][:, j] = a.shape[2]
        cycles = np.zeros(K, dtype=CYCLE_DTYPE)
        for name in ("angles", "velocities", "h", "inertia"):
            a = getattr(self, name)
            if a is None:
                continue
            a = arr(a)
            cycles[name] = np.uint64(_ptr(a)) + np.arange(K, dtype=np.uint64) * np.uint64(a.strides[0])
        if self.angles is not None:
            cycles["status_len"] = self.angles.shape[1]
        cycles["joints"] = np.uint64(_ptr(joints)) + np.arange(K, dtype=np.uint64) * np.uint64(
            D * JOINT_DTYPE.itemsize)
        keep.append(joints)
        return cycles, joints, keep


class Controller:
    """MotionGenerationQuadraticProgram (reference include/mgqp.hpp:70-241) without RTT."""

    def __init__(self, dof: int, library=None):
        self._L = library if library is not None else lib()
        self._h = self._L.mgqp_create()
        self.dof = dof
        self._L.mgqp_set_dof(self._h, dof)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.mgqp_destroy(self._h)
            self._h = None

    def last_error(self) -> str:
        return self._L.mgqp_last_error().decode()

    def setGains(self, kp: float, kd: float):
        self._L.mgqp_set_gains(self._h, kp, kd)

    def _pair(self, fn, P, N):
        P = np.ascontiguousarray(P, dtype=np.float64)
        N = np.ascontiguousarray(N, dtype=np.float64)
        if P.shape != N.shape:
            raise ValueError("limit vectors differ in size")  # assert at src/mgqp.cpp:497
        return bool(fn(self._h, _ptr(P), _ptr(N), P.size))

    def setTorqueLimits(self, P, N):
        return self._pair(self._L.mgqp_set_torque_limits, P, N)

    def setAccelerationLimits(self, P, N):
        return self._pair(self._L.mgqp_set_acceleration_limits, P, N)

    def setAngularLimits(self, sup, inf):
        return self._pair(self._L.mgqp_set_angular_limits, sup, inf)

    def setPriorityLevel(self, task: str, level: int):
        return bool(self._L.mgqp_set_priority_level(self._h, task.encode(), level))

    def updateHook(self, sc: Scenario):
        """One cycle for robot 0 of `sc`.  Returns (code, torques, tracking, limits dict)."""
        cycles, _, keep = sc.pack()
        D = self.dof
        tq = np.zeros(D, np.float32)
        tr = np.zeros(2 * D, np.float32)
        lim = np.zeros((10, D), np.float32)
        code = self._L.mgqp_update(self._h, _ptr(cycles), _ptr(tq), _ptr(tr), _ptr(lim))
        del keep
        return code, tq, tr, dict(zip(LIMIT_PORTS, lim))

    def update_batched(self, sc: Scenario, threads: int = 0):
        """All robots of `sc`.  Returns (codes, torques (K, dof), tracking (K, 2*dof))."""
        cycles, _, keep = sc.pack()
        K, D = sc.count, self.dof
        tq = np.zeros((K, D), np.float32)
        tr = np.zeros((K, 2 * D), np.float32)
        codes = np.zeros(K, np.int32)
        rc = self._L.mgqp_update_batched(self._h, K, _ptr(cycles), _ptr(tq), _ptr(tr), _ptr(codes),
                                       threads)
        del keep
        if rc != 0:
            raise RuntimeError("mgqp_update_batched: " + self.last_error())
        return codes, tq, tr


def _update_device(self, dsc: "DeviceScenario", out=None, stream=None, fast: bool = False):
    """The device-resident cycle (mgqp_update_device).  Returns (rc, codes, torques, tracking)
    as torch tensors on the scenario's device (enqueued on `stream`, not synchronised).
    fast=True solves the levels with the wave kernel's QPGPU_FLAG_FAST build (1e-10)."""
    import torch

    dsc.c.solver_flags = 0x4 if fast else 0  # QPGPU_FLAG_FAST

    dev = next(iter(dsc.tensors.values())).device
    if out is None:
        out = (torch.empty((dsc.count, self.dof), dtype=torch.float32, device=dev),
               torch.empty((dsc.count, 2 * self.dof), dtype=torch.float32, device=dev),
               torch.empty(dsc.count, dtype=torch.int32, device=dev))
    tq, tr, codes = out
    rc = self._L.mgqp_update_device(self._h, ctypes.addressof(dsc.c), tq.data_ptr(),
                                    tr.data_ptr() if tr is not None else None, codes.data_ptr(),
                                    stream)
    if rc < 0:
        raise RuntimeError("mgqp_update_device: " + self.last_error())
    return rc, codes, tq, tr


Controller.update_device = _update_device


def last_error() -> str:
    return lib().mgqp_last_error().decode()


def nullspace_projector(A, dim: int) -> np.ndarray:
    A = np.ascontiguousarray(A, dtype=np.float32)
    Z = np.zeros((dim, dim), np.float32)
    lib().mgqp_nullspace_projector(_ptr(A), A.shape[0], A.shape[1], dim, _ptr(Z))
    return Z


# --- the reference deployment (ops/mgqp.ops) --------------------------------------------------
OPS_ANGLE_SUP = (0.8, 1.5, 2.5, 1.5, 3.0, 1.5, 3.0)  # ops/mgqp.ops:189
TORQUE_LIMIT, ACCEL_LIMIT = 100, 5                    # ops/mgqp.ops:133-134


def ops_controller(dof: int = 7, library=None) -> Controller:
    """The controller as ops/mgqp.ops:183-195 and :287-293 configure it (DOFsize 7)."""
    c = Controller(dof, library)
    c.setTorqueLimits([TORQUE_LIMIT] * dof, [-TORQUE_LIMIT] * dof)
    c.setAccelerationLimits([ACCEL_LIMIT] * dof, [-ACCEL_LIMIT] * dof)
    sup = OPS_ANGLE_SUP if dof == 7 else (3,) * dof  # `var int AngleLimit = 3.14..` is 3
    c.setAngularLimits(list(sup), [-s for s in sup])
    c.setPriorityLevel(f"in_desiredTaskSpacePosition_{dof}", 0)
    c.setPriorityLevel(f"in_desiredTaskSpaceVelocity_{dof}", 0)
    c.setPriorityLevel(f"in_desiredTaskSpaceAcceleration_{dof}", 0)
    c.setPriorityLevel("in_desiredJointSpacePosition_1", 2)
    return c


def _normal(seed: int, stream: int, shape):
    return np.random.default_rng([seed, stream]).standard_normal(shape).astype(np.float32)


def make_scenario(count: int, seed: int = 2026, dof: int = 7, ws: int = 3) -> Scenario:
    """`count` synthetic robot states wired like ops/mgqp.ops:203-262 for DOFsize 7: the end
    effector (joint `dof`) has task-space position/velocity/acceleration targets, its Jacobian
    and Jacobian derivative; joint 1 follows a sine position target (singen).  Angles stay
    strictly inside the ops angle limits; M is symmetric positive definite."""
    K, D = count, dof
    sup = np.array(OPS_ANGLE_SUP if D == 7 else (3.0,) * D, np.float32)
    u = np.random.default_rng([seed, 0]).uniform(-0.9, 0.9, (K, D)).astype(np.float32)
    angles = (u * sup).astype(np.float32)
    vel = 0.5 * _normal(seed, 1, (K, D))
    B = 0.5 * _normal(seed, 2, (K, D, D))
    M = (B @ np.swapaxes(B, 1, 2) + 0.5 * np.eye(D, dtype=np.float32)).astype(np.float32)
    h = 5.0 * _normal(seed, 3, (K, D))
    J = 0.5 * _normal(seed, 4, (K, ws, D))
    Jd = 0.1 * _normal(seed, 5, (K, ws, D))
    xc = 0.5 * _normal(seed, 6, (K, ws))
    vc = 0.2 * _normal(seed, 7, (K, ws))
    ac = 0.2 * _normal(seed, 8, (K, ws))
    xd = xc + 0.05 * _normal(seed, 9, (K, ws))
    vd = 0.1 * _normal(seed, 10, (K, ws))
    ad = 0.1 * _normal(seed, 11, (K, ws))
    qd1 = (0.5 * np.sin(np.arange(K, dtype=np.float64) * 0.05)).astype(np.float32)
    e = D - 1
    ports = {
        (e, "desired_ts_position"): xd, (e, "desired_ts_velocity"): vd,
        (e, "desired_ts_acceleration"): ad, (e, "current_ts_position"): xc,
        (e, "current_ts_velocity"): vc, (e, "current_ts_acceleration"): ac,
        (e, "jacobian"): J, (e, "jacobian_dot"): Jd, (0, "desired_js_position"): qd1,
    }
    return Scenario(D, K, angles, vel, h, M, ports)
