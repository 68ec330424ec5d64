"""One row per bench line: config, kernel, kernel time, HBM / FP64 fractions, traffic ratio,
solves/s, CPU baseline and parity sample.   usage: python tools/line_summary.py LOG..."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d["roofline"]
        h, c = r["hbm"], r.get("compute") or {}
        cb = d.get("cpu_baseline") or {}
        par = cb.get("parity") or {}
        o = d.get("other_arithmetic")
        print(f"{path}: {d['config']['workload'][:3]} {d['config']['kernel']} kernel {h['kernel_ms'] * 1e3:.1f} us "
              f"hbm {h['frac']:.3f} fp64 {c.get('frac', 0):.3f} traffic {h.get('traffic_ratio')} "
              f"value {d['value']:.3g} streams1 {d['value_streams1']:.3g} "
              f"cpu1 {cb.get('value', 0):.3g} cpuN {cb.get('value_threads', cb.get('value_16', 0)) if cb else 0} "
              f"parity {json.dumps(par)[:160]}"
              + (f" | other {o['kernel']} {o['kernel_ms'] * 1e3:.1f} us frac {o['frac']:.3f}" if o else ""))
