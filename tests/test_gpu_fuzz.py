"""Seeded fuzz parity (tests/qp_cases.fuzz_case): random shapes (n <= 64, p <= n, m <= 4n) routed
to every kernel family, with per-QP data modes the fixed configs do not reach — exact ties in
the most-violated selection (the reference keeps the first strict minimum,
oracle/qp_oracle.c:374), ill-conditioned and badly scaled G, zero / duplicated / contradictory
inequality columns, rank-deficient CE.  The default path is held bit for bit against the oracle
(status, l1 passes, x, f, and the factor written back on the write_factor cases); the fast
builds to their 1e-10 contract on the mild variant of the same generator."""
import numpy as np
import pytest

import qp_cases
from test_gpu_parity import FAMILIES, TOL, assert_parity

pytestmark = pytest.mark.gpu

SEEDS = range(48)


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_parity(gpu, seed, family):
    pr, _ = qp_cases.fuzz_case(seed)
    assert_parity(pr, f"fuzz {seed} {(pr.n, pr.p, pr.m, pr.batch)}", write_factor=seed % 3 == 0,
                  family=family, layout="tiled64" if seed % 2 else "qp_major")


X_FLOOR = 1e-13  # absolute floor for the fast builds' x where the reference's x is rounding noise


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_fast(gpu, seed):
    """The fast builds (QPGPU_FLAG_FAST) on the mild cases, measured in tools/fuzz_probe.py
    (profiles/r05_z2): on every QP except those with a rank-deficient CE, the same status and l1
    passes as the reference; x within 1e-10 of ||x_ref||_inf plus an absolute 1e-13
    (small-integer data whose solution is 0 leaves x_ref at ~1e-16 of rounding noise, where a
    relative measure is meaningless); f within 1e-10 of its terms plus 1e-13 of the
    unconstrained objective's magnitude (f accumulates over the steps, so its rounding floor is
    set by the largest intermediate objective).  A rank-deficient CE is decided by the
    reference's own dependence test (|d_iq| <= eps R_norm) on rounding residue, and when it passes
    the solve continues with a near-singular R: the reference's x there carries no KKT
    certificate (tests/test_oracle.py::test_oracle_fuzz_kkt), and another rounding lands
    elsewhere.  Those QPs are held bitwise by the default path (test_fuzz_parity) only."""
    pr, modes = qp_cases.fuzz_case(seed, mild=True)
    assert_tolerance_contract(pr, modes, f"fast fuzz {seed} {(pr.n, pr.p, pr.m, pr.batch)}", fast=True,
                              layout="tiled64" if seed % 2 else "qp_major")


def assert_tolerance_contract(pr, modes, label, **kw):
    """The documented contract of the non-bitwise arithmetic (test_fuzz_fast's docstring)."""
    import oracle
    import qpgpu

    prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xo, fo, so, io = oracle.solve_batch(prc, max_steps=1000 + 100 * (pr.n + pr.p + pr.m))
    xg, fg, sg, ig = qpgpu.solve_batched_host(pr, **kw)
    held = np.array([md != "rank_def_ce" for md in modes])
    assert np.array_equal(so[held], sg[held]), f"{label}: status differs at {np.where(held & (so != sg))[0]}"
    assert np.array_equal(io[held], ig[held]), f"{label}: l1 passes differ at {np.where(held & (io != ig))[0]}"
    ok = held & (so == qpgpu.QP_OK) & (sg == qpgpu.QP_OK)
    dx = np.abs(xg[ok] - xo[ok]).max(axis=1, initial=0.0)
    nx = np.abs(xo[ok]).max(axis=1, initial=0.0)
    bad = np.where(dx > TOL * nx + X_FLOOR)[0]
    assert not bad.size, f"{label}: x off at {np.where(ok)[0][bad]}: {dx[bad]} vs |x_ref| {nx[bad]}"
    fs = np.maximum(np.abs(fo[ok]), qpgpu.objective_term_scale(pr.G[ok], pr.g0[ok], xo[ok]))
    df = np.abs(fg[ok] - fo[ok])
    f_unc = np.abs([g @ np.linalg.solve(G, g) for G, g in zip(pr.G[ok], pr.g0[ok])])
    badf = np.where(df > TOL * fs + X_FLOOR * (1.0 + f_unc))[0]
    assert not badf.size, f"{label}: f off at {np.where(ok)[0][badf]}: {df[badf]} vs terms {fs[badf]}"


# ---- n in [65, 192]: the workspace variant.  QPGPU_FLAG_EXACT keeps the reference's
# order (bitwise on every mode); the default there is the tolerance mode (MFMA panel setup, tree
# sums), held to the same contract as the fast builds on the mild cases.

@pytest.mark.parametrize("seed", range(16))
def test_fuzz_large_exact(gpu, seed):
    pr, _ = qp_cases.fuzz_case(seed, large=True)
    assert_parity(pr, f"large fuzz {seed} {(pr.n, pr.p, pr.m, pr.batch)}", exact=True,
                  write_factor=seed % 4 == 0, layout="tiled64" if seed % 2 else "qp_major")


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_large_default(gpu, seed):
    pr, modes = qp_cases.fuzz_case(seed, mild=True, large=True)
    assert_tolerance_contract(pr, modes, f"large fuzz default {seed} {(pr.n, pr.p, pr.m, pr.batch)}",
                              layout="tiled64" if seed % 2 else "qp_major")


@pytest.mark.parametrize("seed", range(0, 48, 3))
def test_fuzz_single_calls(gpu, seed):
    """The reference's own call pattern — one solve_quadprog() per QP — through the Python mirror
    of the drop-in (qpgpu.solve_quadprog: the host entry's pinned staging, one H2D, the kernel,
    one D2H): the first QPs of each fuzz case, bitwise against the oracle's single solve (x, f
    and the factor left in G), and the reference's exceptions where it throws."""
    import oracle
    import qpgpu

    pr, modes = qp_cases.fuzz_case(seed)
    for b in range(min(pr.batch, 12)):
        G = pr.G[b].copy()
        Go = pr.G[b].copy()
        st, fo, xo, _ = oracle.solve_one(Go, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b],
                                         max_steps=1000 + 100 * (pr.n + pr.p + pr.m))  # the C-ABI's cap
        label = f"seed {seed} qp {b} ({modes[b]})"
        if st == qpgpu.QP_NOT_POSITIVE_DEFINITE:
            with pytest.raises(ValueError, match="cholesky"):
                qpgpu.solve_quadprog(G, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b])
            continue
        if st == qpgpu.QP_MAX_ITER:  # (the reference has no cap; the mirror raises at it)
            with pytest.raises(RuntimeError, match="step cap"):
                qpgpu.solve_quadprog(G, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b])
            continue
        if st == qpgpu.QP_DEPENDENT:
            with pytest.raises(RuntimeError, match="linearly dependent"):
                qpgpu.solve_quadprog(G, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b])
            continue
        f, x = qpgpu.solve_quadprog(G, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b])
        assert np.float64(f).view(np.uint64) == np.float64(fo).view(np.uint64) or (np.isnan(f) and np.isnan(fo)), label
        assert np.array_equal(np.asarray(x).view(np.uint64), np.asarray(xo).view(np.uint64)), label
        assert np.array_equal(G.view(np.uint64), Go.view(np.uint64)), label
