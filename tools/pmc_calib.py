"""FETCH_SIZE / WRITE_SIZE calibration from tools/fetch_probe.hip run under rocprofv3 (one
--pmc pass per counter).  usage: python tools/pmc_calib.py <fetch_dir> <write_dir> [out.json]

Each probe kernel moves a known byte count once from HBM (tools/fetch_probe.hip); the factor is
counter bytes / true bytes for that access pattern (MI355X_MICROARCH.md §HBM: 0.5 for 16-B
coalesced reads; other widths uncalibrated there)."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

NREC, REC = 1 << 18, 1792
READ = {k: NREC * REC for k in ("coalesced_x4", "coalesced_lds", "coalesced_x2", "lane_x4", "lane_x2", "lane_lds",
                                  "lane_touch4")}  # lane_touch4: the lines it touches
WRITE = {"store_lane_x2": NREC * 56, "store_x2": NREC * 8}


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"].split("(")[0].strip()].append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd = sys.argv[1:3]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_calibration.json"
    fe, wr = per_kernel(fd, "FETCH_SIZE"), per_kernel(wd, "WRITE_SIZE")
    res = {"source": "tools/fetch_probe.hip under rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                     "(separate passes); factor = counter bytes / true bytes, median over 3 launches",
           "read": {}, "write": {}}
    for k, b in READ.items():
        v = [x for n, xs in fe.items() if n.endswith(k) for x in xs]
        if v:
            res["read"][k] = {"fetch_kib": statistics.median(v), "true_bytes": b,
                              "factor": statistics.median(v) * 1024 / b}
    for k, b in WRITE.items():
        v = [x for n, xs in wr.items() if n.endswith(k) for x in xs]
        if v:
            res["write"][k] = {"write_kib": statistics.median(v), "true_bytes": b,
                               "factor": statistics.median(v) * 1024 / b}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
