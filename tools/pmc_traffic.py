"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM traffic.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <batch> <kernel_name> [out.json]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch from the L2 memory-side request counters (Infinity
Cache hits included, MI355X_MICROARCH.md §HBM).  On gfx950 FETCH_SIZE under-reports wide
coalesced streaming reads by exactly 2x; this kernel's reads are mixed (LDS-DMA dwordx4 tiles and
per-lane 8-byte loads), so both the raw and the 2x-corrected read figures are recorded and the
corrected one is used as `hbm_bytes_per_launch` (an upper estimate)."""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "qp_" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return vals


fetch_dir, write_dir, config, batch, kname = sys.argv[1:6]
out = sys.argv[6] if len(sys.argv) > 6 else "profiles/pmc_traffic.json"
fe = per_dispatch(fetch_dir, "FETCH_SIZE")
wr = per_dispatch(write_dir, "WRITE_SIZE")
fetch_kib = statistics.median(fe)
write_kib = statistics.median(wr)
rec = {
    "fetch_kib_raw": fetch_kib,
    "write_kib": write_kib,
    "dispatches": [len(fe), len(wr)],
    "hbm_bytes_per_launch_raw": (fetch_kib + write_kib) * 1024,
    "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median per dispatch; "
              f"read side x2 (gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md §HBM)",
}
db = json.load(open(out)) if os.path.exists(out) else {}
db[f"{config}:{batch}:{kname}"] = rec
json.dump(db, open(out, "w"), indent=1)
print(json.dumps(rec))
