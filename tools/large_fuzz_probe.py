"""Per-QP record of the n > 64 default path (the workspace variant's tolerance mode: MFMA panel
setup, tree sums) against the oracle on the FULL fuzz generator (tests/qp_cases.fuzz_case with
large=True, no mild variant): for each seed, the QPs whose status, l1-pass count, x or f differ
from the oracle beyond north_star's plain per-QP 1e-10, with their generator mode.  Test
infrastructure: the oracle is the checker.
  usage: python tools/large_fuzz_probe.py OUT_JSON [seeds...]   (flags: env PROBE_FLAGS=exact|fast)
"""
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"),
                os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
import qp_cases  # noqa: E402
import qpgpu  # noqa: E402


def relerr(a, b):
    d = float(np.abs(a - b).max(initial=0.0))
    s = float(np.abs(b).max(initial=0.0))
    if d == 0.0:
        return 0.0
    return d / s if s > 0 else float("inf")


def main():
    out = sys.argv[1]
    seeds = [int(s) for s in sys.argv[2:]] or list(range(16))
    large = os.environ.get("PROBE_SMALL") is None
    kw = {}
    if os.environ.get("PROBE_FLAGS") == "exact":
        kw["exact"] = True
    summary = {}
    for seed in seeds:
        pr, modes = qp_cases.fuzz_case(seed, large=large)
        prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
        xo, fo, so, io = oracle.solve_batch(prc, max_steps=1000 + 100 * (pr.n + pr.p + pr.m))
        xg, fg, sg, ig = qpgpu.solve_batched_host(pr, layout="tiled64" if seed % 2 else "qp_major", **kw)
        bad = []
        for b in range(pr.batch):
            ok = so[b] == qpgpu.QP_OK and sg[b] == qpgpu.QP_OK
            ex = relerr(xg[b], xo[b]) if ok else 0.0
            ef = relerr(np.array([fg[b]]), np.array([fo[b]])) if ok else 0.0
            if so[b] != sg[b] or io[b] != ig[b] or ex > 1e-10 or ef > 1e-10:
                bad.append({"qp": b, "mode": modes[b], "status": [int(so[b]), int(sg[b])],
                            "iters": [int(io[b]), int(ig[b])], "x_rel": ex, "f_rel": ef,
                            "x_ref_inf": float(np.abs(xo[b]).max(initial=0.0)), "f_ref": float(fo[b])})
                print(f"seed {seed} {bad[-1]}", flush=True)
        summary[seed] = {"shape": [pr.n, pr.p, pr.m, pr.batch], "modes": dict(Counter(modes)),
                         "bad": bad, "bad_modes": dict(Counter(d["mode"] for d in bad))}
        print(f"seed {seed} shape {summary[seed]['shape']} bad {len(bad)} {summary[seed]['bad_modes']}", flush=True)
    tot = Counter()
    for v in summary.values():
        tot.update(v["bad_modes"])
    res = {"flags": kw, "large": large, "seeds": seeds,
           "qps": int(sum(v["shape"][3] for v in summary.values())),
           "bad_total": int(sum(len(v["bad"]) for v in summary.values())), "bad_by_mode": dict(tot),
           "per_seed": summary}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("qps", "bad_total", "bad_by_mode")}))


if __name__ == "__main__":
    main()
