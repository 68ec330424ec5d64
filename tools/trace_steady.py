"""Steady-state kernel duration from a rocprofv3 kernel trace: the mean and median duration of
the last K dispatches of every kernel whose name contains PATTERN (the bench's timed steps and
kernel-duration rounds come last; its warm-up launches, while the clocks ramp, come first).
    usage: python tools/trace_steady.py TRACE.csv PATTERN [K]"""
import csv
import statistics
import sys

path, pat = sys.argv[1], sys.argv[2]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
by = {}
for r in csv.DictReader(open(path)):
    if pat in r["Kernel_Name"]:
        by.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for name, v in by.items():
    v.sort()
    d = [(e - s) / 1e3 for s, e in v[-K:]]
    print(f"{name[:70]}: {len(v)} dispatches; last {len(d)}: mean {statistics.mean(d):.2f} us, "
          f"median {statistics.median(d):.2f} us, min {min(d):.2f}, max {max(d):.2f}")
