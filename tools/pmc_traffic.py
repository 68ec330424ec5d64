"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM traffic.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <batch> <kernel_name> [out.json]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch from the L2 memory-side request counters (Infinity
Cache hits included, MI355X_MICROARCH.md §HBM).  The read side is divided by the factor that
tools/fetch_probe.hip measured for the solver's access patterns (profiles/pmc_calibration.json:
0.50 for 16-B loads, coalesced or one record per lane, plain or LDS-DMA, and for coalesced 8-B
loads; 0.26 for per-lane 8-B loads, which only the selected-column gathers use, from L2);
WRITE_SIZE is exact for the solver's 8-B stores (factor 1.00).  The md5 of the measured
libqpgpu.so is recorded so bench.py can say which build the figure belongs to.

A solve can be several kernels (C5: the MFMA panel setup, then the active-set loop): the median
per dispatch is taken per kernel name and the step's figure is their sum; the per-kernel
figures are kept under "kernels"."""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys
from collections import defaultdict


def per_kernel(d, counter, fast, pair=False):
    # bench.py also times the other arithmetic build of the lane kernel (other_arithmetic) and
    # the lane-pair kernel (pair_kernel): only the kernels of the measured build count
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if ("qp_pair" in kn) != pair:
                continue
            if r["Counter_Name"] == counter and "qp_" in kn and ("_fast_" in kn) == fast:
                vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, config, batch, kname = sys.argv[1:6]
    out = sys.argv[6] if len(sys.argv) > 6 else "profiles/pmc_traffic.json"
    calib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                         "pmc_calibration.json")
    read_factor = 0.5
    if os.path.exists(calib):
        read_factor = json.load(open(calib))["read"]["lane_x4"]["factor"]
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "motion-generation-using-quadratic-programs_amd", "lib", "libqpgpu.so")
    md5 = hashlib.md5(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None
    fast = "fast" in kname
    pair = "qp_pair" in kname
    fe = per_kernel(fetch_dir, "FETCH_SIZE", fast, pair)
    wr = per_kernel(write_dir, "WRITE_SIZE", fast, pair)
    # the n > 64 default runs the workspace kernel twice per step: the tolerance loop, then the
    # certification's EXACT re-solve, whose workgroups exit at once unless their QP is marked
    #  — the same kernel name with a tiny count; its dispatches are split off
    def split(vals):
        out = {}
        for k, v in vals.items():
            top = max(v) if v else 0.0
            big = [x for x in v if x >= 0.01 * top]
            small = [x for x in v if x < 0.01 * top]
            out[k] = big
            if small and big:
                out[k + " [re-solve launch]"] = small
        return out

    fe, wr = split(fe), split(wr)
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        fk = statistics.median(fe[k]) if fe[k] else 0.0
        wk = statistics.median(wr[k]) if wr[k] else 0.0
        kernels[k] = {"fetch_kib_raw": fk, "write_kib": wk, "dispatches": [len(fe[k]), len(wr[k])],
                      "hbm_bytes_per_launch": (fk / read_factor + wk) * 1024}
    fetch_kib = sum(v["fetch_kib_raw"] for v in kernels.values())
    write_kib = sum(v["write_kib"] for v in kernels.values())
    rec = {
        "fetch_kib_raw": fetch_kib,
        "write_kib": write_kib,
        "hbm_bytes_per_launch_raw": (fetch_kib + write_kib) * 1024,
        "hbm_bytes_per_launch": (fetch_kib / read_factor + write_kib) * 1024,
        "read_factor": read_factor,
        "libqpgpu_md5": md5,
        "kernels": kernels,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median per dispatch "
                  "per kernel, summed over the step's kernels; read side / %.3f (the factor "
                  "tools/fetch_probe.hip measured for 16-B loads, profiles/pmc_calibration.json)" % read_factor,
    }
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[f"{config}:{batch}:{kname}"] = rec
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
