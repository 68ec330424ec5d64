"""Diagnostic: per-phase s_memtime stamps of the lane kernel (qpgpu_debug_set_stamps).

Runs the bench workload once with stamps on and prints, per phase, cycles per wave
(mean / p50 / p90 / max) plus the wave's l1-pass maximum.  Never used for timing numbers."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))
import qpgpu  # noqa: E402

kind, n, p, m = (sys.argv[1] if len(sys.argv) > 1 else "general"), 7, 6, 14
layout = sys.argv[2] if len(sys.argv) > 2 else "qp_major"
fast = len(sys.argv) > 3 and sys.argv[3] == "fast"
family = sys.argv[4] if len(sys.argv) > 4 else "lane"  # "pair": 32 QPs per wave (qp_pair.hip)
QPW = 32 if family == "pair" else 64
if kind == "box":
    p = 0
B = int(os.environ.get("STAMPS_B", "65536"))  # e.g. 1: one QP (BASELINE config 1 latency)
pr = qpgpu.make_problems(kind, n, p, m, 0, B, seed=2026)
db = qpgpu.DeviceBatch(pr, "cuda:0", layout=layout)
waves = (B + QPW - 1) // QPW
st = torch.zeros(waves * 18, dtype=torch.int64, device="cuda:0")
fn = qpgpu.LIB.qpgpu_debug_set_stamps
fn.argtypes = [ctypes.c_void_p]
for rep in range(3):
    fn(ctypes.c_void_p(st.data_ptr()))
    db.solve(family=family, fast=fast)
    torch.cuda.synchronize()
fn(None)
s = st.cpu().numpy().reshape(waves, 18).astype(np.int64)
itv = db.iters.cpu().numpy()
it = np.pad(itv, (0, max(0, waves * QPW - len(itv))))[: waves * QPW].reshape(waves, QPW)
names = ["loads+setup", "equality", "active-set", "stores"]
tot = s[:, 4] - s[:, 0]
print(f"{kind} {layout}{' fast' if fast else ''} {family}: total cycles/wave mean {tot.mean():.0f} p50 {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max()}")
for k, nm in enumerate(names):
    d = s[:, k + 1] - s[:, k]
    print(f"  {nm:12s} mean {d.mean():9.0f} p50 {np.median(d):9.0f} p90 {np.percentile(d, 90):9.0f} max {d.max():9d}")
asp = s[:, 3] - s[:, 2]
print(f"  in loop: iterations/wave mean {s[:, 7].mean():.2f} max {s[:, 7].max()}; scan {s[:, 5].mean():.0f} "
      f"select {s[:, 6].mean():.0f} l2a+rest {(asp - s[:, 5] - s[:, 6]).mean():.0f} cycles/wave; "
      f"first scan {s[:, 8].mean():.0f}")
if (s[:, 12] > 0).any():  # QPGPU_LANE_STAMPS=2 builds: compute_d + update_z + update_r inside l2a
    print(f"  l2a detail: compute_d + update_z + update_r {s[:, 12].mean():.0f} cycles/wave "
          f"({s[:, 12].mean() / max(1.0, s[:, 7].mean()):.0f} per iteration)")
mx = it.max(axis=1)
print("  l1 passes: lane mean", it.mean(), "wave-max mean", mx.mean(), "max", mx.max())
for v in sorted(set(mx.tolist())):
    sel = mx == v
    print(f"    wave-max {v}: {sel.sum():5d} waves, active-set cycles mean {(s[sel, 3] - s[sel, 2]).mean():.0f}")
if (s[:, 9] > 0).all():
    g = s[:, 9] - s[:, 0]
    print(f"  setup detail: G landed+read {g.mean():.0f}", end="")
    if (s[:, 10] > 0).all():
        print(f", Cholesky + round-B wait {(s[:, 10] - s[:, 9]).mean():.0f}", end="")
        if (s[:, 11] > 0).all():
            print(f", CE -> AGPR {(s[:, 11] - s[:, 10]).mean():.0f}, warm-up + J + solve {(s[:, 1] - s[:, 11]).mean():.0f}", end="")
    print()
# constant 100 MHz clock (slots 16 / 17): shader clock rate and the spread of wave starts / ends
rt0, rt1 = s[:, 16], s[:, 17]
if (rt1 > rt0).all():
    ghz = (s[:, 4] - s[:, 0]) / ((rt1 - rt0) * 10.0)
    t0 = rt0.min()
    st_us, en_us = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0
    print(f"  shader clock GHz: mean {ghz.mean():.3f} min {ghz.min():.3f} max {ghz.max():.3f}")
    print(f"  wave start (us after the first): p50 {np.median(st_us):.2f} p90 {np.percentile(st_us, 90):.2f} max {st_us.max():.2f}")
    print(f"  wave end   (us after the first start): p50 {np.median(en_us):.2f} p90 {np.percentile(en_us, 90):.2f} max {en_us.max():.2f}")
    dur = en_us - st_us
    print(f"  wave duration us: mean {dur.mean():.2f} p50 {np.median(dur):.2f} max {dur.max():.2f}")
    for x in range(8 if waves >= 8 else 0):
        sel = (np.arange(waves) % 8) == x
        print(f"    block%8={x}: start max {st_us[sel].max():.2f} end max {en_us[sel].max():.2f} clock {ghz[sel].mean():.3f}")
