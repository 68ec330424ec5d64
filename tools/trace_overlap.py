"""Does `value` come from overlapping launches?  Reads a rocprofv3 --kernel-trace CSV of a default
bench run (K timed steps pipelined over 3 streams after W warmup steps) and reports, for the timed
steps' solver dispatches: their average duration, the span from the first start to the last end,
span / K (the pipelined time per step the line's ms_per_step measures), how many dispatches
overlap another one in time, the largest number running at once, and the queues they ran on.

  python tools/trace_overlap.py TRACE.csv KERNEL_SUBSTRING WARMUP STEPS [OUT.json]
The bench's first K + W dispatches of the kernel are the pipelined run (bench.py timed()); the
serialized run, the roofline's kernel-reps and the other arithmetic's launches follow them.
"""
import csv
import json
import sys


def main():
    path, sub, W, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    run = rows[W:W + K]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in run]
    dur = [(e - s) * 1e-3 for s, e, _ in iv]
    span = (max(e for _, e, _ in iv) - min(s for s, _, _ in iv)) * 1e-3
    overlapping = sum(1 for i, (s, e, _) in enumerate(iv)
                      if any(j != i and s < e2 and s2 < e for j, (s2, e2, _) in enumerate(iv)))
    ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
    cur = peak = 0
    for _, d in ev:
        cur += d
        peak = max(peak, cur)
    # time during which two or more of the dispatches run at once
    both = 0
    cur = 0
    last = ev[0][0]
    for t, d in ev:
        if cur >= 2:
            both += t - last
        cur += d
        last = t
    out = {"kernel": run[0]["Kernel_Name"][:120], "dispatches": len(run), "warmup_skipped": W,
           "avg_dispatch_us": sum(dur) / len(dur), "min_dispatch_us": min(dur), "max_dispatch_us": max(dur),
           "span_us": span, "span_per_step_us": span / K, "dispatches_overlapping_another": overlapping,
           "max_concurrent": peak, "time_with_2plus_running_us": both * 1e-3,
           "queues": sorted({q for _, _, q in iv})}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
