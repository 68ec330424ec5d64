"""Summarise rocprofv3 SQ counter CSVs written by tools/gpu_session.sh (per-wave averages)."""
import collections
import csv
import os
import sys

d = sys.argv[1]
for fam in sorted({x.split("_", 1)[1] for x in os.listdir(d) if x.startswith("sq")}):
    tot = collections.defaultdict(list)
    for p in ("sqA", "sqB", "sqC"):
        f = os.path.join(d, f"{p}_{fam}", "c1_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if "qp_" in r["Kernel_Name"]:
                tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in tot.items()}
    w = avg.get("SQ_WAVES", 1.0)
    print(fam, "waves", w)
    for k in sorted(avg):
        if k != "SQ_WAVES":
            print(f"   {k:22s} {avg[k] / w:12.0f} per wave")
