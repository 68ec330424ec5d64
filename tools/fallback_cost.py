"""Diagnostic (GPU): what the QPGPU_FLAG_FAST lane kernel's IEEE fallback costs.

Kernel time of a clean C1 batch against the same batch with one non-finite G per wave, so that
every wave's fast attempt turns invalid in the setup and re-solves with the IEEE forms
(qp_lane.hip, lane_body<..., SAFE>).  Moved out of the parity suite in round 5 (a wall-clock
ratio is not a correctness property).  Usage: python tools/fallback_cost.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import qpgpu  # noqa: E402


def kernel_ms(pr, reps=10):
    db = qpgpu.DeviceBatch(pr, "cuda:0", with_iters=False)
    s = torch.cuda.current_stream()
    go = db.launcher(s, fast=True)
    go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        go()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 65536, seed=31)
    bad = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    bad.G[5::64, 0, 0] = np.nan
    t_clean, t_bad = kernel_ms(pr), kernel_ms(bad)
    print(json.dumps({"kernel": qpgpu.kernel_name(7, 6, 14, fast=True), "clean_ms": t_clean,
                      "every_wave_falls_back_ms": t_bad, "ratio": t_bad / t_clean}))


if __name__ == "__main__":
    main()
