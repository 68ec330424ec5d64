#!/usr/bin/env python3
"""Benchmark of the motion-generation controller cycle.

One step = one updateHook cycle for `--robots` robots configured like ops/mgqp.ops (DOFsize 7:
level 0 = end-effector task + dynamics + 28 limits, level 2 = joint-1 position), i.e. per robot
two (14, 10, 28) + (14, 10, 0) solves, two (14, 1, 28) + (14, 1, 0) solves, the null-space
projector and the float glue.  Legs:
  device : mgqp_update_device, inputs resident in HBM, HIP events around the whole cycle
  host   : mgqp_update_batched (host builder/projector threads + one GPU launch per level/shape)
  cpu    : the same C++ controller with the CPU oracle solver (tests' harness build), 1 thread,
           on a bounded sample — the CPU baseline
Prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"),
                os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mgqp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--host-robots", type=int, default=16384)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    sc = mgqp.make_scenario(args.robots, seed=2026)
    c = mgqp.ops_controller()
    dsc = mgqp.DeviceScenario(sc, "cuda")
    out = None
    for _ in range(args.warmup):
        rc, codes, tq, tr = c.update_device(dsc)
        out = (tq, tr, codes)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        c.update_device(dsc, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    ok = float((out[2] == 0).float().mean().item())
    res = {"metric": "mgqp control cycles/s (DOF 7, 3-level hierarchy, device-resident)",
           "value": args.robots / (ms * 1e-3), "unit": "cycles/s", "robots": args.robots,
           "ms_per_step": ms, "steps": args.steps, "warmup": args.warmup,
           "written_frac": ok, "dtype": "f32 glue + f64 QPs", "data": "synthetic"}

    if not args.no_host:
        hs = mgqp.make_scenario(args.host_robots, seed=2026)
        ch = mgqp.ops_controller()
        ch.update_batched(hs)
        t = time.perf_counter()
        ch.update_batched(hs)
        el = time.perf_counter() - t
        res["host_orchestrated"] = {"value": args.host_robots / el, "unit": "cycles/s",
                                    "robots": args.host_robots,
                                    "threads": min(16, os.cpu_count() or 1)}
    if not args.no_cpu:
        import test_mgqp_host as th

        H = mgqp.load_library(th.build_harness())
        cc = mgqp.ops_controller(library=H)
        chunk = 512
        cs = mgqp.make_scenario(chunk, seed=2026)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            cc.update_batched(cs, threads=1)
            done += chunk
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": done / el, "unit": "cycles/s", "cores": 1, "kind": "port",
                               "sample": f"C++ controller + oracle solver, 1 thread, {done} cycles "
                                         f"of the same scenario in {el:.1f} s"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
