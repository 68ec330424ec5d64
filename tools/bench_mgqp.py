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
    ap.add_argument("--streams", type=int, default=3,
                    help="independent cycles pipelined over this many HIP streams (1 = serialized)")
    ap.add_argument("--wide", action="store_true",
                    help="angle limits +-20 rad and gains (10, 2), as tests/test_gpu_mgqp.py's wide case: "
                         "level-0 QPs are then feasible for part of the robots, so their solves run the "
                         "active-set loop instead of the retry snapshot")
    ap.add_argument("--fast", action="store_true",
                    help="level solves with the wave kernel's QPGPU_FLAG_FAST build (within 1e-10)")
    args = ap.parse_args()

    def configure(ctl):
        if args.wide:
            ctl.setAngularLimits([20.0] * 7, [-20.0] * 7)
            ctl.setGains(10, 2)
        return ctl

    sc = mgqp.make_scenario(args.robots, seed=2026)
    c = configure(mgqp.ops_controller())
    dsc = mgqp.DeviceScenario(sc, "cuda")
    S = max(1, args.streams)
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = []
    for j in range(S):  # one output set per stream (workspaces are per stream in the library)
        with torch.cuda.stream(streams[j]):
            rc, codes, tq, tr = c.update_device(dsc, stream=streams[j].cuda_stream, fast=args.fast)
        outs.append((tq, tr, codes))
    for k in range(args.warmup):
        c.update_device(dsc, out=outs[k % S], stream=streams[k % S].cuda_stream, fast=args.fast)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        c.update_device(dsc, out=outs[k % S], stream=streams[k % S].cuda_stream, fast=args.fast)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    # serialized cycle time (one stream, HIP events)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for _ in range(3):
        c.update_device(dsc, out=outs[0], stream=streams[0].cuda_stream, fast=args.fast)
    e1.record(streams[0])
    torch.cuda.synchronize()
    ms_serial = e0.elapsed_time(e1) / 3
    ok = float((outs[0][2] == 0).float().mean().item())
    same = all(torch.equal(outs[0][0], o[0]) for o in outs[1:])
    res = {"metric": "mgqp control cycles/s (DOF 7, 3-level hierarchy, device-resident)",
           "value": args.robots / (ms * 1e-3), "unit": "cycles/s", "robots": args.robots,
           "ms_per_step": ms, "ms_per_cycle_serialized": ms_serial, "streams": S,
           "streams_outputs_identical": bool(same), "steps": args.steps, "warmup": args.warmup,
           "written_frac": ok, "dtype": "f32 glue + f64 QPs", "data": "synthetic",
           "limits": "wide (+-20 rad, gains 10/2)" if args.wide else "ops/mgqp.ops",
           "level_solves": "fast (QPGPU_FLAG_FAST, 1e-10)" if args.fast else "exact (bitwise)"}

    if not args.no_host:
        hs = mgqp.make_scenario(args.host_robots, seed=2026)
        ch = configure(mgqp.ops_controller())
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
        cc = configure(mgqp.ops_controller(library=H))
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
