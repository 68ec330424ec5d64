"""Worst QPs of a fast build against the oracle (per-QP relative error), with the exact build's
result on the same QPs: usage python tools/fast_worst.py kind n p m B seed [family]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import qpgpu  # noqa: E402

kind, n, p, m, B, seed = sys.argv[1], *map(int, sys.argv[2:7])
fam = sys.argv[7] if len(sys.argv) > 7 else None
pr = qpgpu.make_problems(kind, n, p, m, 0, B, seed=seed)
xo, fo, so, io = oracle.solve_batch(qpgpu.Problems(n, p, m, pr.G.copy(), *pr.arrays()[1:]), max_steps=1000 + 100 * (n + p + m), threads=8)
xf, ff, sf, itf = qpgpu.solve_batched_host(pr, fast=True, family=fam)
xe, fe, se, ite = qpgpu.solve_batched_host(pr, family=fam)
print("kernel fast:", qpgpu.LIB.qpgpu_kernel_name_flags(n, p, m, qpgpu.FLAG_FAST | qpgpu.FAMILY_FLAGS[fam]).decode())
print("status equal fast/exact:", (sf == so).all(), (se == so).all(), "iters equal:", (itf == io).all(), (ite == io).all())
print("exact bitwise x:", np.array_equal(xe.view(np.uint64), xo.view(np.uint64)))
ok = so == 0
ex, ef = qpgpu.rel_error_per_qp(xf, xo, ff, fo)
ex[~ok] = 0
ef[~ok] = 0
for k in np.argsort(-ex)[:5]:
    print(f"QP {k} (wave {k // 64} lane {k % 64}): ex {ex[k]:.3e} ef {ef[k]:.3e} st {so[k]} it {io[k]}/{itf[k]}")
    print("   x_ref ", np.array2string(xo[k], precision=6))
    print("   x_fast", np.array2string(xf[k], precision=6))
    print("   f", fo[k], ff[k], fe[k])
