"""The lane-pair kernel (qp_pair.hip: one QP per two lanes, 32 QPs per wave, two waves per SIMD;
QPGPU_FLAG_FAST only, shape (7, 6, 14) QP-major) against the oracle: north_star's 1e-10 relative
per QP on x and f, identical status and l1-pass counts — over the bench batch, partial waves,
and every exit of the algorithm (not positive definite, non-finite data, degenerate adds,
infeasible and dependent QPs, long active-set paths)."""
import numpy as np
import pytest

import qpgpu
from test_gpu_parity import assert_fast_parity

pytestmark = pytest.mark.gpu

PAIR = "pair"


def _c1(b0, b1, seed):
    return qpgpu.make_problems("general", 7, 6, 14, b0, b1, seed=seed)


@pytest.mark.parametrize("seed", [2026, 12345])
def test_pair_full_size(gpu, seed):
    """C1 at the bench size (65 536 QPs)."""
    assert_fast_parity(_c1(0, 65536, seed), f"pair C1 seed {seed}", family=PAIR)


@pytest.mark.parametrize("B", [1, 2, 31, 33, 1001])
def test_pair_partial_waves(gpu, B):
    """Batches that end inside a wave (32 QPs per wave): idle pairs read QP b0 and write nothing."""
    assert_fast_parity(_c1(0, B, 900 + B), f"pair B={B}", family=PAIR)


def _edge_batch():
    pr = _c1(0, 256, 77)
    G, CE, ce0, CI, ci0, g0 = pr.G, pr.CE, pr.ce0, pr.CI, pr.ci0, pr.g0
    G[0, 2, 2] = -1.0e3                       # not positive definite at row 2
    G[1, 3, 4] = G[1, 4, 3] = np.nan          # NaN factor: the wave's fast attempt falls back
    ci0[2, 5] = -np.inf                       # a -inf limit
    ci0[3, 9] = np.nan                        # a NaN limit
    G[4, 1, 1] = 1.0e300                      # a factor outside the fast forms' range
    for qp in range(8, 16):                   # duplicated inequalities: degenerate adds, rollback
        CI[qp, :, 7:] = CI[qp, :, :7]
        ci0[qp, 7:] = ci0[qp, :7] - 1e-3
    for qp in range(16, 24):                  # a . x >= 1 and -a . x >= 1: infeasible
        CI[qp, :, 1] = -CI[qp, :, 0]
        ci0[qp, 0] = ci0[qp, 1] = -1.0
    g0[24:32] *= 30.0                         # long active-set paths
    for qp in range(32, 40):                  # linearly dependent equality constraints
        CE[qp, :, 5] = CE[qp, :, 4]
        ce0[qp, 5] = ce0[qp, 4]
    return pr


def test_pair_edges(gpu):
    pr = _edge_batch()
    assert_fast_parity(pr, "pair edges", family=PAIR)
    # the cases did exercise those exits (statuses as the oracle's, checked above)
    _, _, st, _ = qpgpu.solve_batched_host(pr, fast=True, family=PAIR)
    for want in (qpgpu.QP_NOT_POSITIVE_DEFINITE, qpgpu.QP_INFEASIBLE, qpgpu.QP_DEPENDENT, qpgpu.QP_OK):
        assert (st == want).any(), f"no QP ended with status {want}"


def test_pair_agrees_with_lane_fast(gpu):
    """Same decisions as the single-lane fast build on a full batch; x within 1e-10 of it."""
    pr = _c1(0, 65536, 4242)
    xl, fl, sl, il = qpgpu.solve_batched_host(pr, fast=True, family="lane")
    xp, fp, sp, ip = qpgpu.solve_batched_host(pr, fast=True, family=PAIR)
    assert np.array_equal(sl, sp) and np.array_equal(il, ip)
    ok = sl == qpgpu.QP_OK
    ex, _ = qpgpu.rel_error_per_qp(xp[ok], xl[ok], fp[ok], fl[ok])
    assert float(ex.max()) <= 1e-10


def test_pair_rules(gpu):
    """FORCE_PAIR needs FAST; other shapes, the TILED64 layout and the m = 0 snapshot are not the
    pair kernel's (unsupported shape); the kernel name reports it."""
    assert qpgpu.LIB.qpgpu_kernel_name_flags(7, 6, 14, qpgpu.FLAG_FAST | qpgpu.FLAG_FORCE_PAIR).decode() \
        == "qp_pair_fast<N=7,P=6,M=14>"
    assert qpgpu.LIB.qpgpu_kernel_name_flags(7, 6, 14, qpgpu.FLAG_FORCE_PAIR).decode() == ""
    assert qpgpu.LIB.qpgpu_kernel_name_flags(7, 0, 14, qpgpu.FLAG_FAST | qpgpu.FLAG_FORCE_PAIR).decode() == ""
    pr = _c1(0, 64, 1)
    with pytest.raises(RuntimeError):
        qpgpu.solve_batched_host(pr, family=PAIR)  # without FAST
    with pytest.raises(RuntimeError):
        qpgpu.solve_batched_host(qpgpu.make_problems("general", 7, 5, 14, 0, 64, seed=1), fast=True, family=PAIR)
    with pytest.raises(RuntimeError):
        qpgpu.solve_batched_host(pr, fast=True, family=PAIR, layout="tiled64")


def test_pair_fallback_is_bounded(gpu):
    """One QP with a NaN in G in every wave: every wave's fast attempt stops after the Cholesky
    and re-solves with the IEEE forms — under 2.5x the clean batch's time, results in contract."""
    import torch

    B = 65536
    pr = _c1(0, B, 31)
    bad = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    bad.G[5::32, 0, 0] = np.nan

    def kernel_ms(p_):
        db = qpgpu.DeviceBatch(p_, "cuda:0", with_iters=False)
        s = torch.cuda.current_stream()
        go = db.launcher(s, fast=True, family=PAIR)
        go()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            go()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 10

    t_clean, t_bad = kernel_ms(pr), kernel_ms(bad)
    assert t_bad < 2.5 * t_clean, f"fallback batch {t_bad:.3f} ms vs clean {t_clean:.3f} ms"
    assert_fast_parity(bad.slice(0, 4096), "pair fallback (NaN G in every wave)", family=PAIR)
