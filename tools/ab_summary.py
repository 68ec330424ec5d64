"""Summarise A/B bench logs: python tools/ab_summary.py gpurun_out/TAGa gpurun_out/TAGb ..."""
import glob
import json
import os
import sys

rows = {}
for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
        name = os.path.basename(f)[6:-4]
        try:
            line = [l for l in open(f) if l.startswith("{")][-1]
        except IndexError:
            continue
        r = json.loads(line)["roofline"]
        us = r.get("kernel_us") or (r["bytes_per_launch"] / r["achieved"] / 1e3 if "bytes_per_launch" in r else None)
        rows.setdefault(name, []).append((r["frac"], us))
for k, v in rows.items():
    print(f"{k:24s} " + "  ".join(f"frac {f:.4f}" + (f" ({u:.2f} us)" if u else "") for f, u in v))
