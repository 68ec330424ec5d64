"""CPU tests of the oracle (oracle/qp_oracle.c): pinned to the reference's golden vector and
independently certified by KKT conditions (it is the checker for every GPU parity test)."""
import json
import os

import numpy as np
import pytest
from scipy.optimize import lsq_linear

import oracle
import qp_cases
import qpgpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_reference_kat_bitwise():
    """The archive's demo output, bit for bit, including the factored G."""
    kat = json.load(open(os.path.join(HERE, "golden", "reference_kat.json")))
    for c in kat["cases"]:
        G = np.array(c["G"])
        st, f, x, it = oracle.solve_one(G, c["g0"], c["CE"], c["ce0"], c["CI"], c["ci0"])
        assert st == qpgpu.QP_OK
        assert f.hex() == c["expect_f_hex"]
        assert [v.hex() for v in x] == c["expect_x_hex"]
        assert [[v.hex() for v in row] for row in G] == c["expect_G_after_hex"]


def kkt_residual(G, g0, CE, ce0, CI, ci0, x, tol_act=1e-7):
    """Independent optimality certificate: stationarity residual with the best non-negative
    multipliers on the (numerically) active inequalities, plus primal feasibility."""
    n = G.shape[0]
    s = CI.T @ x + ci0
    act = np.where(s <= tol_act * (1 + np.abs(ci0)))[0]
    A = np.concatenate([CE, CI[:, act]], axis=1)
    rhs = G @ x + g0
    if A.shape[1] == 0:
        stat = np.linalg.norm(rhs)
    else:
        lb = np.concatenate([np.full(CE.shape[1], -np.inf), np.zeros(len(act))])
        res = lsq_linear(A, rhs, bounds=(lb, np.full(A.shape[1], np.inf)), tol=1e-14, max_iter=2000)
        stat = np.linalg.norm(A @ res.x - rhs)
    eq = np.max(np.abs(CE.T @ x + ce0)) if CE.shape[1] else 0.0
    ineq = max(0.0, -np.min(s)) if CI.shape[1] else 0.0
    scale = 1.0 + np.linalg.norm(g0) + np.linalg.norm(G, 2) * np.linalg.norm(x)
    return stat / scale, eq, ineq


@pytest.mark.parametrize("name,kind,n,p,m", qp_cases.CONFIGS)
def test_oracle_kkt(name, kind, n, p, m):
    B = 24 if n <= 16 else 6
    pr = qp_cases.make(kind, n, p, m, B)
    G0 = pr.G.copy()
    x, f, st, it = oracle.solve_batch(pr)
    assert (st == qpgpu.QP_OK).all(), st
    for b in range(B):
        stat, eq, ineq = kkt_residual(G0[b], pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b], x[b])
        assert stat < 1e-9, (b, stat)
        assert eq < 1e-9 and ineq < 1e-9, (b, eq, ineq)
        fx = 0.5 * x[b] @ G0[b] @ x[b] + pr.g0[b] @ x[b]
        assert abs(fx - f[b]) <= 1e-9 * (1 + abs(fx)), (b, fx, f[b])


def test_oracle_batch_matches_single_and_threads():
    pr = qp_cases.make("general", 7, 6, 14, 64)
    x1, f1, s1, i1 = oracle.solve_batch(pr, threads=1)
    x4, f4, s4, i4 = oracle.solve_batch(pr, threads=4)
    assert np.array_equal(x1, x4) and np.array_equal(f1, f4) and np.array_equal(i1, i4)
    for b in (0, 17, 63):
        st, f, x, it = oracle.solve_one(pr.G[b].copy(), pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b])
        assert f == f1[b] and np.array_equal(x, x1[b]) and it == i1[b]


def test_oracle_edge_statuses():
    want = {"demo": 0, "infeasible": 1, "dependent": 3, "not_pd": 2, "not_pd0": 2, "mgqp_retry": 0,
            "neg_inf_limit": 1, "p_gt_n": 3}
    for name, pr in qp_cases.edge_cases():
        x, f, st, it = oracle.solve_batch(pr, max_steps=5000)
        if name in want:
            assert st[0] == want[name], (name, st)
        assert np.isin(st, [0, 1, 2, 3]).all(), (name, st)


def test_oracle_not_pd_reports_pivot():
    pr = dict(qp_cases.edge_cases())["not_pd"]
    x, f, st, it = oracle.solve_batch(pr)
    assert st[0] == qpgpu.QP_NOT_POSITIVE_DEFINITE
    assert f[0] == 1.0 - 4.0  # second pivot: 1 - 2^2 / 1


def test_oracle_write_factor_is_cholesky():
    pr = qp_cases.make("general", 7, 6, 14, 8)
    G0 = pr.G.copy()
    oracle.solve_batch(pr, write_factor=True)
    for b in range(8):
        L = np.tril(pr.G[b])
        assert np.allclose(L @ L.T, G0[b], rtol=1e-12, atol=1e-10)
        assert np.array_equal(np.triu(pr.G[b]), np.triu(L.T))


def test_max_steps_cap():
    pr = dict(qp_cases.edge_cases())["long_paths"]
    x, f, st, it = oracle.solve_batch(pr, max_steps=1)
    assert (st == qpgpu.QP_MAX_ITER).any()


@pytest.mark.parametrize("seed", range(8))
def test_oracle_fuzz_kkt(seed):
    """The oracle on the fuzz generator's mild cases (tests/test_gpu_fuzz.py): every QP it calls
    solved carries an independent KKT certificate, except on rank-deficient CE: there the
    reference's dependence test (|d_iq| <= eps R_norm: add_constraint @.text+0x21fd of the
    archive, oracle/qp_oracle.c qpo_add_constraint) can miss a column
    that is dependent only up to rounding, and it goes on with a near-singular R, as the oracle
    does.  No generator mode yields a non-positive-definite G."""
    pr, modes = qp_cases.fuzz_case(seed, mild=True)
    G0 = pr.G.copy()
    x, f, st, it = oracle.solve_batch(pr, max_steps=1000 + 100 * (pr.n + pr.p + pr.m))
    for b in [b for b in np.where(st == qpgpu.QP_OK)[0] if modes[b] != "rank_def_ce"][:40]:
        stat, eq, ineq = kkt_residual(G0[b], pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b], x[b])
        sc = 1.0 + np.abs(pr.ci0[b]).max(initial=0.0) + np.abs(pr.ce0[b]).max(initial=0.0)
        assert stat < 1e-7 and eq < 1e-8 * sc and ineq < 1e-8 * sc, (b, stat, eq, ineq)
    assert not (st == qpgpu.QP_NOT_POSITIVE_DEFINITE).any()
