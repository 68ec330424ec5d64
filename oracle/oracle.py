"""ctypes binding of the CPU restatement (oracle/qp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker / the timed CPU baseline — never by the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_qp.so")
COUNT_LIB_PATH = os.path.join(HERE, "liboracle_qp_count.so")  # the same code, -DQPO_COUNT


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or not os.path.exists(COUNT_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.qpo_solve.argtypes = [ctypes.c_int] * 3 + [vp] * 9 + [ctypes.c_int]
        L.qpo_solve.restype = ctypes.c_int
        L.qpo_solve_batch.argtypes = [ctypes.c_int64] + [ctypes.c_int] * 3 + [vp] * 10 + [ctypes.c_int] * 3
        L.qpo_solve_batch.restype = ctypes.c_int
        _lib = L
    return _lib


_clib = None


def count_lib():
    global _clib
    if _clib is None:
        build()
        L = ctypes.CDLL(COUNT_LIB_PATH)
        vp = ctypes.c_void_p
        L.qpo_solve_batch.argtypes = [ctypes.c_int64] + [ctypes.c_int] * 3 + [vp] * 10 + [ctypes.c_int] * 3
        L.qpo_solve_batch.restype = ctypes.c_int
        L.qpo_op_counts.argtypes = [vp]
        L.qpo_op_counts.restype = None
        _clib = L
    return _clib


def op_counts(pr, max_steps: int = 0):
    """Binary64 operations the reference's evaluation executes on a qpgpu.Problems batch
    (SURVEY.md §8(d)): the counting build of the restatement solves it on one thread.
    Returns {"mul", "add", "div", "sqrt", "flops", "per_qp"}; flops = mul + add + div + sqrt
    (the reference has no fused multiply-add)."""
    B, n, p, m = pr.batch, pr.n, pr.p, pr.m
    L = count_lib()
    out = np.zeros(4, dtype=np.uint64)
    L.qpo_op_counts(_p(out))  # reset
    G = np.ascontiguousarray(pr.G, dtype=np.float64)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)]
    x = np.zeros((B, n))
    f = np.zeros(B)
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    L.qpo_solve_batch(B, n, p, m, _p(G), *[_p(a) for a in arrs], _p(x), _p(f), _p(st), _p(it), 0,
                      max_steps, 1)
    L.qpo_op_counts(_p(out))
    mul, add, div, sq = (int(v) for v in out)
    flops = mul + add + div + sq
    return {"mul": mul, "add": add, "div": div, "sqrt": sq, "flops": flops, "per_qp": flops / max(1, B)}


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def solve_batch(pr, write_factor: bool = False, max_steps: int = 0, threads: int = 1):
    """Solve a qpgpu.Problems batch on the CPU.  Returns (x, f, status, iters).

    max_steps mirrors the GPU safety cap (0 = none, the reference's behaviour).  With
    write_factor=True pr.G receives the Cholesky factors like the reference's G."""
    B, n, p, m = pr.batch, pr.n, pr.p, pr.m
    G = pr.G if write_factor else np.ascontiguousarray(pr.G, dtype=np.float64)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)]
    x = np.zeros((B, n))
    f = np.zeros(B)
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    lib().qpo_solve_batch(B, n, p, m, _p(G), *[_p(a) for a in arrs], _p(x), _p(f), _p(st), _p(it),
                          1 if write_factor else 0, max_steps, threads)
    return x, f, st, it


def solve_one(G, g0, CE, ce0, CI, ci0, max_steps: int = 0):
    """One QP with reference argument shapes (CE n x p, CI n x m).  G is overwritten.
    Returns (status, f, x, iters)."""
    G = np.ascontiguousarray(G, dtype=np.float64)
    n = G.shape[0]
    CE = np.ascontiguousarray(np.asarray(CE, dtype=np.float64).reshape(n, -1))
    CI = np.ascontiguousarray(np.asarray(CI, dtype=np.float64).reshape(n, -1))
    p, m = CE.shape[1], CI.shape[1]
    g0 = np.ascontiguousarray(g0, dtype=np.float64).reshape(n)
    ce0 = np.ascontiguousarray(ce0, dtype=np.float64).reshape(p)
    ci0 = np.ascontiguousarray(ci0, dtype=np.float64).reshape(m)
    x = np.zeros(n)
    f = np.zeros(1)
    it = np.zeros(1, dtype=np.int32)
    st = lib().qpo_solve(n, p, m, _p(G), _p(g0), _p(CE), _p(ce0), _p(CI), _p(ci0), _p(x), _p(f), _p(it),
                         max_steps)
    return st, float(f[0]), x, int(it[0])
