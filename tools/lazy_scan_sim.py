"""Simulation of a lazy l1 scan for C5 (DESIGN §6.4 / VERDICT r03 item 6), on the CPU.

The oracle built with -DQPO_TRACE reports x at every l1 pass.  A block of constraints (16
consecutive columns of CI) is skipped at a pass when a rigorous bound proves none of its
constraints is violated: s_i(x) >= s_i(x_e) - ||a_i||_2 ||x - x_e||_2 - margin_i > 0, where x_e is
the x of the block's last evaluation and margin_i covers the rounding of both dot products
(2 gamma_{n+1} (||a_i||_1 ||x||_inf + |ci0_i|)).  Prints the fraction of CI blocks a lazy scan
would still read.  usage: python tools/lazy_scan_sim.py [qps] [block]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))
import qpgpu  # noqa: E402

so = "/tmp/liboracle_qp_trace.so"
subprocess.check_call(["cc", "-O2", "-fPIC", "-std=c11", "-ffp-contract=off", "-DQPO_TRACE", "-shared", "-o", so,
                       os.path.join(ROOT, "oracle", "qp_oracle.c"), "-lm", "-lpthread"])
lib = ctypes.CDLL(so)
CB = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.POINTER(ctypes.c_double))
xs = []
cb = CB(lambda n, x: xs.append(np.ctypeslib.as_array(x, (n,)).copy()))
ctypes.c_void_p.in_dll(lib, "qpo_trace_cb").value = ctypes.cast(cb, ctypes.c_void_p).value

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 3
BLK = int(sys.argv[2]) if len(sys.argv) > 2 else 16
n, p, m = 256, 0, 512
pr = qpgpu.make_problems("general", n, p, m, 0, Q, seed=2026)
u = 2.0 ** -53
gam = (n + 1) * u / (1 - (n + 1) * u)
tot_blocks = tot_eval = 0
for q in range(Q):
    xs.clear()
    G = pr.G[q].copy()
    x = np.zeros(n)
    f = np.zeros(1)
    it = np.zeros(1, dtype=np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.qpo_solve(n, p, m, P(G), P(pr.g0[q]), None, None, P(np.ascontiguousarray(pr.CI[q])), P(pr.ci0[q]),
                  P(x), P(f), P(it), 100000)
    CI, ci0 = pr.CI[q], pr.ci0[q]
    if os.environ.get("LAZY_SORT") == "1":  # constraints stored in the order of their first-scan slack
        order = np.argsort(-(CI.T @ xs[0] + ci0))
        CI, ci0 = CI[:, order], ci0[order]
    a2 = np.linalg.norm(CI, axis=0)
    a1 = np.abs(CI).sum(axis=0)
    nb = (m + BLK - 1) // BLK
    xe = [None] * nb
    se = [None] * nb
    le = [0.0] * nb
    ev = 0
    L = 0.0
    PATH = os.environ.get("LAZY_PATH") == "1"  # bound ||x - x_e|| by the path length since x_e
    for k, xk in enumerate(xs):
        if k:
            L += np.linalg.norm(xk - xs[k - 1])
        s = CI.T @ xk + ci0
        marg = 2 * gam * (a1 * np.abs(xk).max() + np.abs(ci0)) * 1.01
        for b in range(nb):
            sl = slice(b * BLK, min(m, (b + 1) * BLK))
            if xe[b] is not None:
                d = (L - le[b]) * (1 + 1e-12) if PATH else np.linalg.norm(xk - xe[b])
                lb = se[b] - a2[sl] * d - marg[sl]
                if (lb > 0).all():
                    continue
            xe[b], se[b], le[b] = xk, s[sl], L
            ev += 1
    tot_blocks += nb * len(xs)
    tot_eval += ev
    print(f"QP {q}: {len(xs)} l1 passes, blocks read {ev} of {nb * len(xs)} ({ev / (nb * len(xs)):.3f})")
print(f"all: lazy scan reads {tot_eval / tot_blocks:.3f} of the CI blocks (block = {BLK} constraints)")
