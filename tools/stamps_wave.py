"""Diagnostic: per-phase s_memtime stamps of the qp_wave kernel (qpgpu_debug_set_stamps).

usage: python tools/stamps_wave.py N P M BATCH   (default C3: 30 6 60 65536)
Needs a library built with the per-phase clocks (SRC=qp_wave tools/ab_build.sh stamps
-DQPGPU_WAVE_STAMPS=1, run with QPGPU_LIB_PATH=_ab/stamps/libqpgpu.so); the product build keeps
only the phase-boundary stamps.  Prints cycles per block for: loads + Cholesky, J = L^-T +
unconstrained solve, equality phase,
active-set loop.  Never used for timing numbers."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))
import qpgpu  # noqa: E402

n, p, m, B = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (30, 6, 60, 65536)))
pr = qpgpu.make_problems("general", n, p, m, 0, B, seed=2026)
db = qpgpu.DeviceBatch(pr, "cuda:0")
blocks = B  # upper bound on blocks (>= QPs / QPs-per-block)
st = torch.zeros(blocks * 18, dtype=torch.int64, device="cuda:0")
fn = qpgpu.LIB.qpgpu_debug_set_stamps
fn.argtypes = [ctypes.c_void_p]
for rep in range(2):
    st.zero_()
    fn(ctypes.c_void_p(st.data_ptr()))
    db.solve(family="wave", fast=os.environ.get("WFAST") == "1")  # WFAST=1: the fast build
    torch.cuda.synchronize()
fn(None)
s = st.cpu().numpy().reshape(blocks, 18).astype(np.int64)
s = s[s[:, 0] != 0]
names = ["loads+cholesky", "J + x0", "equality", "active-set"]
tot = s[:, 4] - s[:, 0]
print(f"({n},{p},{m}) x {B}: {len(s)} blocks; cycles/block mean {tot.mean():.0f} p50 {np.median(tot):.0f} max {tot.max()}")
for k, nm in enumerate(names):
    d = s[:, k + 1] - s[:, k]
    print(f"  {nm:15s} mean {d.mean():10.0f} p50 {np.median(d):10.0f} max {d.max():10d}")
for k, nm in enumerate(["scan", "select", "d/z", "lead step", "add_constraint", "delete"]):
    print(f"    loop {nm:15s} mean {s[:, 8 + k].mean():10.0f}")
det = os.environ.get("WDETAIL", "0")  # the QPGPU_WAVE_STAMPS_DETAIL of the build
lab = {"0": ["eq d/z", "eq update_r", "eq lead t2 + x/u"],
       "1": ["loop update_r", "loop steps", "loop sum iq"],
       "2": ["add: chain+coef", "add: J sweep", "add: R col+test"]}[det]
for k, nm in [(5, lab[0]), (6, lab[1]), (7, lab[2]), (14, "eq add_constraint"),
              (15, "|h| chains (eq + loop)")]:
    print(f"    {nm:20s} mean {s[:, k].mean():10.0f}")
it = db.iters.cpu().numpy()
print("  l1 passes: mean", it.mean(), "max", it.max())
start = s[:, 0] - s[:, 0].min()
print("  block start offsets: p50", np.median(start), "max", start.max(), " end max", (s[:, 4] - s[:, 0].min()).max())
