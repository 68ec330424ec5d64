"""Kernel time of the C5 batch (4 096 x (256, 0, 512), seed 2026) on the n > 64 paths: the default
(tolerance mode after the MFMA panel setup) and QPGPU_FLAG_EXACT (the reference's operation
order, serial sums), one launch each after one untimed launch, HIP events on the launch stream.
  usage: python tools/c5_exact_cost.py [batch] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd")]
import torch  # noqa: E402

import qpgpu  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["default", "exact"]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
pr = qpgpu.make_problems("general", 256, 0, 512, 0, B, seed=2026)
db = qpgpu.DeviceBatch(pr, dev, with_iters=True)
st = torch.cuda.Stream(dev)
res = {"batch": B}
for mode in modes:
    launch = db.launcher(st, exact=(mode == "exact"))
    t0 = time.time()
    launch()
    torch.cuda.synchronize(dev)
    first = time.time() - t0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record(st)
        for _ in range(reps):
            launch()
        e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    it = db.iters.cpu().numpy()
    res[mode] = {"ms_per_launch": ms, "first_launch_s": first, "solves_per_s": B / ms * 1e3,
                 "mean_l1_passes": float(it.mean())}
    print(mode, json.dumps(res[mode]), flush=True)
print(json.dumps(res))
