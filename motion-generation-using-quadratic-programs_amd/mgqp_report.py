"""mgqp_report — the reference deployment's trajectory log format.

The reference logs closed-loop runs with OCL FileReporting (ops/logData.ops:1-28) into
build/reports.dat, one space-separated row per reporting period, and analyses them with
plotresult.m.  This module writes the same column layout from this framework's controller
cycles, and reads it back the way plotresult.m does, so a run of the GPU controller and a run of
the reference deployment can be compared trajectory against trajectory.

Column layout (ops/logData.ops:8-26 report order; plotresult.m:29-190 reads it with
JOINT_OP = true), for DOF d (7 on the LWR4+):
  1                    time
  3 + 3 + 3            trajectorygenerator2 desired task-space position / velocity / acceleration
  3 + 3 + 3            fkin7 current task-space position / velocity / acceleration
  1                    singen out_sin_port (the joint-1 position target, plotresult's desPosJ1)
  d + d + d            robot_gazebo full_arm_JointFeedback: angles, velocities, torques
  d                    out_torques_port
  10 x d               out_joint{Pos,Vel,Acc,AccDyn,Torque}Limit{Inf,Sup}_port, in the order of
                       mgqp.LIMIT_PORTS
The first line is a header; plotresult.m skips it (dlmread(..., 1, 0)) after collapsing runs of
spaces (plotresult.m:16-23), so its text is informational.

Values that come from simulation peers this framework does not have (Gazebo's measured joint
torques) are written as NaN unless the caller passes them.
"""
from __future__ import annotations

import math

import numpy as np

from mgqp import LIMIT_PORTS

TASK_PORTS = ("desired_ts_position", "desired_ts_velocity", "desired_ts_acceleration",
              "current_ts_position", "current_ts_velocity", "current_ts_acceleration")


def columns(dof: int = 7, ws: int = 3) -> list:
    """Column names in file order."""
    names = ["time"]
    for p in TASK_PORTS:
        names += [f"{p}[{i}]" for i in range(ws)]
    names.append("out_sin")
    for p in ("feedback_angles", "feedback_velocities", "feedback_torques", "out_torques"):
        names += [f"{p}[{j}]" for j in range(dof)]
    for p in LIMIT_PORTS:
        names += [f"out_{p}[{j}]" for j in range(dof)]
    return names


def report_row(t: float, sc, r: int, torques, limits: dict, task_joint: int | None = None,
               feedback_torques=None, ws: int = 3) -> np.ndarray:
    """One row for robot r of Scenario `sc` after a cycle that produced `torques` (dof) and
    `limits` ({LIMIT_PORTS name: (dof,)}, as Controller.updateHook returns them).  The
    reported task is joint `task_joint`'s task-space ports (default: the end effector, as
    trajectorygenerator2 / fkin7 in ops/mgqp.ops); absent ports (RTT::NoData) are NaN."""
    D = sc.dof
    e = D - 1 if task_joint is None else task_joint
    row = [float(t)]
    for p in TASK_PORTS:
        a = sc.ports.get((e, p))
        row += list(np.asarray(a[r], np.float64)[:ws]) if a is not None else [math.nan] * ws
    sin = sc.ports.get((0, "desired_js_position"))
    row.append(float(sin[r]) if sin is not None else math.nan)
    for a in (sc.angles, sc.velocities):
        row += list(np.asarray(a[r], np.float64)[:D]) if a is not None else [math.nan] * D
    row += (list(np.asarray(feedback_torques, np.float64)[:D]) if feedback_torques is not None
            else [math.nan] * D)
    row += list(np.asarray(torques, np.float64)[:D])
    for p in LIMIT_PORTS:
        row += list(np.asarray(limits[p], np.float64)[:D])
    out = np.asarray(row, np.float64)
    assert out.size == len(columns(D, ws))
    return out


def write_reports(path: str, rows, dof: int = 7, ws: int = 3) -> None:
    """Header + one line per row, single-space separated, float32 values printed exactly
    (repr of the float: the controller's ports are float)."""
    with open(path, "w") as f:
        f.write("# " + " ".join(columns(dof, ws)) + "\n")
        for row in rows:
            f.write(" ".join(repr(float(v)) for v in row) + "\n")


def read_reports(path: str, dof: int = 7, ws: int = 3) -> dict:
    """plotresult.m's parse (collapse spaces, skip the header line, numeric matrix), returned
    as {column name: series} plus the matrix under "data"."""
    names = columns(dof, ws)
    rows = []
    with open(path) as f:
        next(f, None)  # header (an empty file has none)
        for lineno, line in enumerate(f, start=2):
            parts = line.split()
            if not parts:
                continue
            if len(parts) != len(names):
                raise ValueError(f"{path}:{lineno}: {len(parts)} columns, expected {len(names)}")
            rows.append([float(v) for v in parts])
    data = np.asarray(rows, np.float64).reshape(len(rows), len(names))
    out = {n: data[:, i] for i, n in enumerate(names)}
    out["data"] = data
    return out


def compare_runs(a: dict, b: dict, names=None) -> dict:
    """Trajectory-level comparison of two read_reports() results over their common rows:
    max |a - b| per column (NaN-aware: columns absent in either run are skipped)."""
    n = min(a["data"].shape[0], b["data"].shape[0])
    res = {}
    for k in names or [c for c in a if c != "data"]:
        x, y = a[k][:n], b[k][:n]
        m = ~(np.isnan(x) | np.isnan(y))
        if m.any():
            res[k] = float(np.max(np.abs(x[m] - y[m])))
    return res
