"""CPU restatement of the reference controller's QP builder and hierarchy.

TEST INFRASTRUCTURE ONLY: used by tests/ as the checker for libmgqp_amd (never by the product).

Follows reference src/mgqp.cpp statement by statement in numpy float32 (the reference uses
Eigen::MatrixXf / VectorXf), with the QP solves done by the bitwise QuadProg++ restatement
(oracle/qp_oracle.c) and the null-space projector by numpy's SVD.  PARITY UNPINNED at the float
level: Eigen (product kernels, JacobiSVD) is absent from this image and the reference has no
fixtures for the controller, so the tests compare with float tolerances.
"""
from __future__ import annotations

import math

import numpy as np

import oracle as qpo

TS = ("position", "velocity", "acceleration")


def _append(a, b):
    """matrixAppend (src/mgqp.cpp:574-617)."""
    if a.shape[0] == 0:
        return b.copy()
    if b.shape[0] == 0:
        return a
    if a.ndim == 2 and a.shape[1] != b.shape[1]:
        return a
    return np.concatenate([a, b]).astype(np.float32)


class OracleController:
    def __init__(self, dof):
        self.dof = dof
        self.levels = {}
        self.stackSize = 3
        self.kTP, self.kTD, self.kJP, self.kJD = np.float32(100), np.float32(25), np.float32(200), np.float32(100)
        self.max_f = 0.0
        self.tP = self.tN = self.aP = self.aN = self.sup = self.inf = np.zeros(0, np.float32)

    def set_limits(self, torque, accel, angles):
        f = lambda v: np.asarray(v, np.float32)
        self.tP, self.tN = f(torque[0]), f(torque[1])
        self.aP, self.aN = f(accel[0]), f(accel[1])
        self.sup, self.inf = f(angles[0]), f(angles[1])

    def _note(self, f):
        if math.isfinite(f):
            self.max_f = max(self.max_f, abs(f))

    @property
    def ill_conditioned(self):
        """True when the last update() had a solve with |f| > 1e8: the level's projected
        constraints were (numerically) dependent and the dual steps blew up, so the result
        depends on the last bits of the float glue (chaotic in the reference as well)."""
        return self.max_f > 1e8

    def level(self, name):
        return self.levels.get(name, -1)

    # solveNextStep (src/mgqp.cpp:655-749)
    def solve_next_step(self, A, a, B, b):
        n = A.shape[1]
        G = np.eye(n)
        g0 = np.zeros(n)
        CE = A.astype(np.float64).T.copy()
        CI = B.astype(np.float64).T.copy().reshape(n, B.shape[0])
        st, f, x, _ = qpo.solve_one(G.copy(), g0, CE, a.astype(np.float64), CI, b.astype(np.float64))
        self._note(f)
        if st == 3:
            raise RuntimeError("Constraints are linearly dependent")
        if math.isnan(f) or f == math.inf:
            st, f, x, _ = qpo.solve_one(np.eye(n), g0, CE, a.astype(np.float64), np.zeros((n, 0)),
                                        np.zeros(0))
            self._note(f)
            if st == 3:
                raise RuntimeError("Constraints are linearly dependent")
            if math.isnan(f) or f == math.inf:
                return False, np.zeros(n, np.float32)
        return True, x.astype(np.float32)

    @staticmethod
    def projector(Acumul, dim):
        """src/mgqp.cpp:836-862 with numpy's thin SVD."""
        _, s, vt = np.linalg.svd(Acumul.astype(np.float64), full_matrices=False)
        V = vt.T
        keep = (s.astype(np.float32) >= 1e-16).astype(np.float64)
        return (np.eye(dim) - (V * keep) @ V.T).astype(np.float32)

    # solveNextHierarchy (src/mgqp.cpp:751-869)
    def hierarchy(self, qps):
        dim = 2 * self.dof
        Acumul = np.zeros((0, dim), np.float32)
        Bcumul = np.zeros((0, dim), np.float32)
        acumul = np.zeros(0, np.float32)
        bcumul = np.zeros(0, np.float32)
        res = np.zeros(dim, np.float32)
        u = np.zeros(dim, np.float32)
        Z = np.eye(dim, dtype=np.float32)
        ok = True
        for cond, goal, cons, lim in qps:
            Bcumul = _append(Bcumul, cons)
            bcumul = _append(bcumul, lim)
            last_res = res
            if cond.shape[0] == 0 and cons.shape[0] == 0:
                continue
            if cond.shape[0] > 0 and Bcumul.shape[0] > 0:
                ok, u = self.solve_next_step(cond @ Z, goal - cond @ last_res, Bcumul @ Z, bcumul)
            elif cond.shape[0] > 0 and cons.shape[0] == 0 and Bcumul.shape[0] == 0:
                ok, u = self.solve_next_step(cond @ Z, goal - cond @ last_res,
                                             np.zeros((1, dim), np.float32), np.zeros(1, np.float32))
            if not ok:
                return last_res
            res = (last_res + Z @ u).astype(np.float32)
            if cond.shape[0] > 0:
                Acumul = _append(Acumul, cond)
                acumul = _append(acumul, goal)
                Z = self.projector(Acumul, dim)
        return res

    # updateHook (src/mgqp.cpp:872-1189); sc is an mgqp.Scenario, robot r
    def update(self, sc, r):
        self.max_f = 0.0
        D = self.dof
        if sc.h is None or sc.inertia is None or sc.angles is None:
            return 1, None, None
        q, qd = sc.angles[r].astype(np.float32), sc.velocities[r].astype(np.float32)
        port = lambda j, nm: None if (j, nm) not in sc.ports else np.asarray(sc.ports[(j, nm)][r], np.float32)
        qps = [[np.zeros((0, 2 * D), np.float32), np.zeros(0, np.float32)] for _ in range(self.stackSize)]
        for j in range(D):
            for lvl in range(self.stackSize):
                ts = False
                vals = {}
                for k, nm in enumerate(TS):
                    d, c = port(j, "desired_ts_" + nm), port(j, "current_ts_" + nm)
                    if d is None or c is None or self.level(f"in_desiredTaskSpace{nm.capitalize()}_{j + 1}") != lvl:
                        vals[nm] = (np.zeros(3, np.float32), np.zeros(3, np.float32))
                    else:
                        vals[nm] = (d[:3], c[:3])
                        ts = True
                if ts and (port(j, "jacobian") is None or port(j, "jacobian_dot") is None):
                    return 2, None, None
                js = False
                qdes, qddes = q[j], qd[j]
                v = port(j, "desired_js_position")
                if v is not None and self.level(f"in_desiredJointSpacePosition_{j + 1}") == lvl:
                    qdes, js = np.float32(v), True
                v = port(j, "desired_js_velocity")
                if v is not None and self.level(f"in_desiredJointSpaceVelocity_{j + 1}") == lvl:
                    qddes, js = np.float32(v), True
                v = port(j, "desired_js_acceleration")
                if v is not None and self.level(f"in_desiredJointSpaceAcceleration_{j + 1}") == lvl:
                    js = True
                if ts:
                    J, Jd = port(j, "jacobian"), port(j, "jacobian_dot")
                    A = np.zeros((J.shape[0], 2 * D), np.float32)
                    A[:, :J.shape[1]] = J
                    (dP, cP), (dV, cV), (dA, cA) = vals["position"], vals["velocity"], vals["acceleration"]
                    a = -(self.kTP * (dP - cP) + self.kTD * (dV - cV) - Jd @ qd[:J.shape[1]] + dA - cA)
                    qps[lvl][0] = _append(qps[lvl][0], A)
                    qps[lvl][1] = _append(qps[lvl][1], a.astype(np.float32))
                if js:
                    A = np.zeros((1, 2 * D), np.float32)
                    A[0, j] = 1
                    a = np.array([-(self.kJP * (qdes - q[j]) + self.kJD * (qddes - qd[j]))], np.float32)
                    qps[lvl][0] = _append(qps[lvl][0], A)
                    qps[lvl][1] = _append(qps[lvl][1], a)
        # inequalities (src/mgqp.cpp:1075-1134)
        lm = np.zeros((4 * D, 2 * D), np.float32)
        lm[:2 * D] = -np.eye(2 * D)
        lm[2 * D:] = np.eye(2 * D)
        z = np.zeros(D, np.float32)
        aP = self.aP.copy() if self.aP.size == D else z.copy()
        aN = self.aN.copy() if self.aN.size == D else z.copy()
        sup = self.sup if self.sup.size == D else z
        inf = self.inf if self.inf.size == D else z
        with np.errstate(invalid="ignore", divide="ignore"):
            for i in range(D):
                lp = math.log(float(np.float32(sup[i] - q[i]))) if sup[i] - q[i] > 0 else (
                    -math.inf if sup[i] - q[i] == 0 else math.nan)
                ln = math.log(float(np.float32(q[i] - inf[i]))) if q[i] - inf[i] > 0 else (
                    -math.inf if q[i] - inf[i] == 0 else math.nan)
                ln = -ln
                aP[i] = np.float32(lp if lp < float(aP[i]) else float(aP[i]))   # std::min
                aN[i] = np.float32(ln if float(aN[i]) < ln else float(aN[i]))   # std::max
        tP = self.tP if self.tP.size == D else z
        tN = self.tN if self.tN.size == D else z
        limits = np.concatenate([aP, tP, -aN, -tN]).astype(np.float32)
        dyn = np.concatenate([sc.inertia[r].astype(np.float32), -np.eye(D, dtype=np.float32)], axis=1)
        qps[0][0] = _append(qps[0][0], dyn)
        qps[0][1] = _append(qps[0][1], np.zeros(D, np.float32))
        levels = []
        for lvl in range(self.stackSize):
            cons = lm if lvl == 0 else np.zeros((0, 2 * D), np.float32)
            lim = limits if lvl == 0 else np.zeros(0, np.float32)
            levels.append((qps[lvl][0], qps[lvl][1], cons, lim))
        tracking = self.hierarchy(levels)
        torques = (tracking[D:] + sc.h[r].astype(np.float32)).astype(np.float32)
        return 0, torques, tracking


def ops_oracle(dof=7):
    """Oracle twin of mgqp.ops_controller()."""
    import mgqp

    o = OracleController(dof)
    sup = np.array(mgqp.OPS_ANGLE_SUP if dof == 7 else (3,) * dof, np.float32)
    o.set_limits(([mgqp.TORQUE_LIMIT] * dof, [-mgqp.TORQUE_LIMIT] * dof),
                 ([mgqp.ACCEL_LIMIT] * dof, [-mgqp.ACCEL_LIMIT] * dof), (sup, -sup))
    for nm in ("Position", "Velocity", "Acceleration"):
        o.levels[f"in_desiredTaskSpace{nm}_{dof}"] = 0
    o.levels["in_desiredJointSpacePosition_1"] = 2
    return o
