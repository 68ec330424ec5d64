"""Parity of a library build against the oracle at the bench shapes, without requiring bitwise
equality: per config the number of QPs whose status / l1-pass count differ and the largest
relative error of x and f over the QPs both solve (north_star's bar is 1e-10).  For A/B builds
(tools/ab_build.sh) that give up the reference's operation order.  Test infrastructure: the
oracle is only the checker here.
  usage: [QPGPU_LIB_PATH=_ab/<name>/libqpgpu.so] python tools/fast_diag.py [--fast] [config ...]
(--fast: the in-library QPGPU_FLAG_FAST build of the lane kernel)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)

import oracle  # noqa: E402
import qpgpu  # noqa: E402
from bench import CONFIGS  # noqa: E402


def rel(a, b):
    with np.errstate(invalid="ignore"):
        r = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
    return float(np.max(r)) if r.size else 0.0


FAST = "--fast" in sys.argv
cfgs = [a for a in sys.argv[1:] if a != "--fast"]
print("lib", qpgpu.LIB_PATH, "fast" if FAST else "")
for cfg in cfgs or ["C1", "C2"]:
    kind, n, p, m, B, _ = CONFIGS[cfg]
    for seed in (2026, 12345):
        pr = qpgpu.make_problems(kind, n, p, m, 0, B, seed=seed)
        xo, fo, so, io = oracle.solve_batch(pr, max_steps=1000 + 100 * (n + p + m), threads=8)
        xg, fg, sg, ig = qpgpu.solve_batched_host(pr, fast=FAST)
        ok = (so == 0) & (sg == 0)
        print(f"{cfg} seed {seed}: {B} QPs, status differs {int((so != sg).sum())}, l1 passes differ "
              f"{int((io != ig).sum())}, x bitwise-equal {int((xg[ok] == xo[ok]).all(axis=1).sum())}/{int(ok.sum())}, "
              f"max rel x {rel(xg[ok], xo[ok]):.3e} f {rel(fg[ok], fo[ok]):.3e}", flush=True)
