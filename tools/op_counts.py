"""Operation counts of the reference's evaluation for every bench config (SURVEY.md §8(d)
"Algorithmic flops": the restatement counts the operations it actually executes, per config and
seed).  The counting build of the CPU restatement (oracle/liboracle_qp_count.so, -DQPO_COUNT)
solves each config's whole bench batch (bench.py's generator, seed 2026) on the host; the
table goes to profiles/op_counts.json, which bench.py reads for its compute-roofline column.
Test infrastructure: bench.py reads the data file, never the oracle, for this column.

usage: python tools/op_counts.py [config ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import qpgpu  # noqa: E402
from bench import CONFIGS, C4_GLOBAL  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "op_counts.json")


def main():
    cfgs = sys.argv[1:] or [c for c in CONFIGS if c != "C4"]
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for cfg in cfgs:
        kind, n, p, m, bdef, _ = CONFIGS[cfg]
        B = bdef or C4_GLOBAL
        seed = 2026
        t0 = time.time()
        tot = {"mul": 0, "add": 0, "div": 0, "sqrt": 0, "flops": 0}
        step = 8192
        for b0 in range(0, B, step):
            pr = qpgpu.make_problems(kind, n, p, m, b0, min(B, b0 + step), seed=seed)
            c = oracle.op_counts(pr, max_steps=1000 + 100 * (n + p + m))
            for k in tot:
                tot[k] += c[k]
        rec = dict(tot, batch=B, seed=seed, per_qp=tot["flops"] / B,
                   div_per_qp=tot["div"] / B, sqrt_per_qp=tot["sqrt"] / B,
                   source="oracle/qp_oracle.c built with -DQPO_COUNT (tools/op_counts.py), the "
                          "whole bench batch; flops = mul + add + div + sqrt, the reference "
                          "evaluation's binary64 operations (no fused multiply-add)")
        db[f"{cfg}:{B}:{seed}"] = rec
        json.dump(db, open(OUT, "w"), indent=1)
        print(cfg, f"{rec['per_qp']:.1f} flops/QP", f"{time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
