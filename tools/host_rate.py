"""PCIe-inclusive rate of the host-pointer entry (qpgpu_solve_batched_host): inputs in host
memory, results back in host memory, one call per batch.
usage: python tools/host_rate.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "motion-generation-using-quadratic-programs_amd"))
import qpgpu  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
out = {}
for cfg, (kind, n, p, m) in {"C1": ("general", 7, 6, 14), "C2": ("box", 7, 0, 14)}.items():
    pr = qpgpu.make_problems(kind, n, p, m, 0, 65536, seed=2026)
    in_bytes = 8 * 65536 * (n * n + n + n * p + p + n * m + m)
    for fast in (False, True):
        qpgpu.solve_batched_host(pr, fast=fast)  # warm-up (allocations, code objects)
        t0 = time.perf_counter()
        for _ in range(reps):
            qpgpu.solve_batched_host(pr, fast=fast)
        dt = (time.perf_counter() - t0) / reps
        out[f"{cfg}{'_fast' if fast else ''}"] = {"ms_per_call": dt * 1e3, "solves_per_s": 65536 / dt,
                                                 "input_bytes": in_bytes,
                                                 "input_gbs": in_bytes / dt / 1e9}
print(json.dumps(out, indent=1))
