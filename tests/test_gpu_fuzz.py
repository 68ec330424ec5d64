"""Seeded fuzz parity (tests/qp_cases.fuzz_case): random shapes (n <= 64, p <= n, m <= 4n) routed
to every kernel family, with per-QP data modes the fixed configs do not reach — exact ties in
the most-violated selection (the reference keeps the first strict minimum,
oracle/qp_oracle.c:374), ill-conditioned and badly scaled G, zero / duplicated / contradictory
inequality columns, rank-deficient CE.  The default path is held bit for bit against the oracle
(status, l1 passes, x, f, and the factor written back on the write_factor cases); the fast
builds to their 1e-10 contract on the mild variant of the same generator; the n > 64 default
(tolerance mode + EXACT re-solve of what it cannot certify) to the plain per-QP bar on the full
generator."""
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
# order (bitwise on every mode).  The default there is the tolerance mode (MFMA panel setup, tree
# sums) whose uncertified QPs are re-solved EXACT: held to north_star's PLAIN bar
# on the FULL generator — cond(G) to 1e8, scales to 1e+-40, rank-deficient CE, integer ties,
# duplicated / contradictory columns — with no exclusion: identical status and l1 passes, x and
# f within 1e-10 relative per QP.

@pytest.mark.parametrize("seed", range(16))
def test_fuzz_large_exact(gpu, seed):
    pr, _ = qp_cases.fuzz_case(seed, large=True)
    assert_parity(pr, f"large fuzz {seed} {(pr.n, pr.p, pr.m, pr.batch)}", exact=True,
                  write_factor=seed % 4 == 0, layout="tiled64" if seed % 2 else "qp_major")


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_large_default(gpu, seed):
    pr, modes = qp_cases.fuzz_case(seed, large=True)
    assert_parity(pr, f"large fuzz default {seed} {(pr.n, pr.p, pr.m, pr.batch)} {modes}",
                  layout="tiled64" if seed % 2 else "qp_major")


@pytest.mark.parametrize("seed", range(0, 64, 4))
def test_fuzz_large_certified_part(gpu, seed):
    """The tolerance mode alone (the EXACT re-solve switched off): every QP it certifies meets
    the plain bar by itself, and every QP the plain bar would reject carries a mark — so the
    re-solve, not luck, is what holds the default path to the bar."""
    import oracle
    import qpgpu

    pr, modes = qp_cases.fuzz_case(seed, large=True)
    prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xo, fo, so, io = oracle.solve_batch(prc, max_steps=1000 + 100 * (pr.n + pr.p + pr.m))
    qpgpu.set_resolve(False)
    try:
        xg, fg, sg, ig = qpgpu.solve_batched_host(pr)
    finally:
        qpgpu.set_resolve(True)
    marked = (sg & qpgpu.STATUS_RESOLVE) != 0
    sg = sg & 0xFF
    for b in np.where(~marked)[0]:
        lab = f"seed {seed} qp {b} ({modes[b]}) certified"
        assert so[b] == sg[b] and io[b] == ig[b], lab
        if so[b] == qpgpu.QP_OK:
            ex, ef = qpgpu.rel_error_per_qp(xg[b:b + 1], xo[b:b + 1], fg[b:b + 1], fo[b:b + 1])
            assert ex.max() <= TOL and ef.max() <= TOL, (lab, ex, ef)


def test_large_default_degenerate_after_pending_sweep(gpu):
    """n in [65, 192] on the default flags with duplicated and scaled-
    duplicate inequality columns, so degenerate adds and deletes follow the two-deep deferred J
    sweeps of the tolerance loop (QPGPU_WAVE_TOLLOOP bit 3): the plain per-QP bar, and the
    tolerance mode alone meets it on every QP it certifies."""
    import oracle
    import qpgpu

    n, p, m, B = 120, 3, 240, 6
    pr = qp_cases.make("general", n, p, m, B, seed=4242)
    pr.CI[:, :, 120:200] = pr.CI[:, :, 0:80]
    pr.ci0[:, 120:200] = pr.ci0[:, 0:80] - 1e-3
    pr.CI[:, :, 200:240] = 2.0 * pr.CI[:, :, 40:80]
    pr.ci0[:, 200:240] = 2.0 * pr.ci0[:, 40:80] - 0.5
    pr.g0 *= 5.0  # long active-set paths
    assert_parity(pr, "degenerate adds after pending sweeps")
    prc = qpgpu.Problems(n, p, m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xo, fo, so, io = oracle.solve_batch(prc, max_steps=1000 + 100 * (n + p + m))
    qpgpu.set_resolve(False)
    try:
        xg, fg, sg, ig = qpgpu.solve_batched_host(pr)
    finally:
        qpgpu.set_resolve(True)
    cert = (sg & qpgpu.STATUS_RESOLVE) == 0
    assert np.array_equal((sg & 0xFF)[cert], so[cert]) and np.array_equal(ig[cert], io[cert])
    ok = cert & (so == qpgpu.QP_OK)
    if ok.any():
        ex, ef = qpgpu.rel_error_per_qp(xg[ok], xo[ok], fg[ok], fo[ok])
        assert ex.max() <= TOL and ef.max() <= TOL


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64) if a.dtype == np.float64 else a


def _shadow_ab(pr):
    """The n > 64 default path with the EXACT re-solve off (so every certification mark shows),
    once with the l1 scans filtered through the fp32 copy of CI and once fp64-only; returns both
    results and the shadow path's (scans tried, scans settled)."""
    import qpgpu

    qpgpu.set_resolve(False)
    try:
        qpgpu.shadow_stats(reset=True)
        on = qpgpu.solve_batched_host(pr)
        stats = qpgpu.shadow_stats(reset=True)[:2]
        qpgpu.set_shadow(False)
        off = qpgpu.solve_batched_host(pr)
    finally:
        qpgpu.set_shadow(True)
        qpgpu.set_resolve(True)
    return on, off, stats


@pytest.mark.parametrize("seed", range(0, 64, 2))
def test_large_default_shadow_scan_bitwise(gpu, seed):
    """the l1 scan from the fp32 copy of CI is a filter whose bounds only decide
    which s_i need their fp64 sums — the same products in the same order as the fp64 scan.  On the
    full large fuzz generator (scales to 1e+-40, where fp32 underflows or overflows and the bounds
    must send the scan back to fp64) x, f, the status words with their certification marks and
    the l1 passes are identical bit for bit with and without it."""
    pr, modes = qp_cases.fuzz_case(seed, large=True)
    on, off, (tried, settled) = _shadow_ab(pr)
    for name, a, b in zip(("x", "f", "status", "passes"), on, off):
        assert np.array_equal(_bits(a), _bits(b)), f"seed {seed} {modes}: {name} differs with the fp32 scan"
    assert settled <= tried


def test_c5_shadow_scan_bitwise_and_used(gpu):
    """C5's shape (n = 256, p = 0, m = 512; the bench generator's first 64 QPs): bit-identical
    results with and without the fp32 scan, which settles most of the scans there."""
    import qpgpu

    pr = qpgpu.make_problems("general", 256, 0, 512, 0, 64, seed=2026)
    on, off, (tried, settled) = _shadow_ab(pr)
    for name, a, b in zip(("x", "f", "status", "passes"), on, off):
        assert np.array_equal(_bits(a), _bits(b)), f"C5: {name} differs with the fp32 scan"
    assert tried > 0 and settled >= 0.5 * tried, (tried, settled)


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
