"""GPU parity: the gfx950 kernels (through the C-ABI) against the oracle on identical inputs.

Bar (north_star, per QP): status and l1-pass count identical, ||x - x_ref||_inf / ||x_ref||_inf
<= 1e-10 and |f - f_ref| / |f_ref| <= 1e-10 — the PLAIN relative error, asserted for every build
that produces a bench line's `value` — and, for every path that keeps the reference's operation
order, x and f BITWISE identical.  The one tolerance path is the default n > 64 one, whose setup
runs as blocked f64 MFMA (qp_panel.hip): held to the plain 1e-10 on x and f (identical status and
iteration counts), and the same shapes are also checked bitwise with QPGPU_FLAG_EXACT.

The QPGPU_FLAG_FAST builds (opt-in, not a bench line's value since round 5) have a weaker
documented contract, asserted separately below (assert_fast_parity): x within the plain 1e-10,
f within 1e-10 of its terms max(|f_ref|, 0.5|x'Gx| + |g0'x|)."""
import json
import os

import numpy as np
import pytest

import oracle
import qp_cases
import qpgpu

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-10  # north_star: "within 1e-10 relative"


def _relerr(xg, xo, fg, fo, ok, pr=None):
    """north_star's criterion per QP (qpgpu.rel_error_per_qp): the max over the QPs of
    ||x - x_ref||_inf / ||x_ref||_inf (over the `ok` QPs, whose x is defined) and of the plain
    |f - f_ref| / |f_ref| (every QP).  Given `pr` (its original G), also the max of |f - f_ref|
    relative to the objective's terms max(|f_ref|, 0.5 |x^T G x| + |g0^T x|) — the fast builds'
    contract and an extra figure for the failure message."""
    ex, _ = qpgpu.rel_error_per_qp(xg[ok], xo[ok], fg[ok], fo[ok])
    _, efp = qpgpu.rel_error_per_qp(xg, xo, fg, fo)
    mx = lambda a: float(a.max()) if a.size else 0.0
    eft = None
    if pr is not None:
        scale = np.zeros(len(fo))
        scale[ok] = qpgpu.objective_term_scale(pr.G[ok], pr.g0[ok], xo[ok])
        _, ef = qpgpu.rel_error_per_qp(xg, xo, fg, fo, f_scale=scale)
        eft = mx(ef)
    return mx(ex), mx(efp), eft


def _bit_mismatch(a, b, show=6):
    """Elements whose bits differ, as (gpu hex, oracle hex) pairs.  Two NaNs count as equal: IEEE
    754 leaves the sign and payload of a NaN that an invalid operation creates (inf - inf, 0 * inf,
    sqrt(-x)) to the implementation — x86 creates 0xfff8..., gfx950 0x7ff8... — so only the fact
    that a value is NaN is part of the reference behaviour, not its bits."""
    a = np.ascontiguousarray(a, dtype=np.float64).ravel()
    b = np.ascontiguousarray(b, dtype=np.float64).ravel()
    diff = (a.view(np.uint64) != b.view(np.uint64)) & ~(np.isnan(a) & np.isnan(b))
    idx = np.where(diff)[0][:show]
    return [(float(a[i]).hex(), float(b[i]).hex()) for i in idx]


FAMILIES = (None, "lane", "subgroup", "wave")


def covers(family, n, m):
    if family == "lane":
        return n <= 8 and m <= 16
    if family == "subgroup":
        return n <= 16 and m <= 64
    if family == "wave":
        return n <= 256 and m <= 1024
    if family == "generic":
        return True
    return bool(qpgpu.kernel_name(n, 0, m))


def bitwise_expected(n, m, write_factor=False, exact=False):
    """Every path keeps the reference's operation order except the workspace variant's tolerance
    mode (n > 64, or m beyond the LDS variants): MFMA panel setup, then tree-summed compute_d /
    update_z / update_r in the loop (qp_wave.hip, QPGPU_WAVE_TOLLOOP)."""
    return exact or write_factor or "qp_panel" not in qpgpu.kernel_name(n, 0, m)


def assert_parity(pr, label, max_iter=0, write_factor=False, family=None, layout=None, exact=False):
    if not covers(family, pr.n, pr.m):
        pytest.skip(f"family {family} does not cover {(pr.n, pr.p, pr.m)}")
    prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    cap = max_iter if max_iter > 0 else 1000 + 100 * (pr.n + pr.p + pr.m)
    xo, fo, so, io = oracle.solve_batch(prc, write_factor=write_factor, max_steps=cap)
    prg = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xg, fg, sg, ig = qpgpu.solve_batched_host(prg, write_factor=write_factor, max_iter=max_iter,
                                              family=family, layout=layout, exact=exact)
    assert np.array_equal(so, sg), f"{label}: status differs at {np.where(so != sg)[0][:10]}"
    assert np.array_equal(io, ig), f"{label}: iteration count differs at {np.where(io != ig)[0][:10]}"
    ok = so != qpgpu.QP_NOT_POSITIVE_DEFINITE  # x untouched on that exit (reference throws)
    ex, ef, eft = _relerr(xg, xo, fg, fo, ok, pr)
    assert ex <= TOL and ef <= TOL, f"{label}: rel err x {ex:.3e} f {ef:.3e} (f vs its terms {eft:.3e})"
    if not bitwise_expected(pr.n, pr.m, write_factor, exact):
        return so, io
    bx, bf = _bit_mismatch(xg[ok], xo[ok]), _bit_mismatch(fg, fo)
    assert not bx and not bf, (f"{label}: within tolerance but not bitwise (x {ex:.3e}, f {ef:.3e}); "
                               f"x (gpu, oracle) {bx}; f (gpu, oracle) {bf}")
    if write_factor:
        bg = _bit_mismatch(prg.G, prc.G)
        assert not bg, f"{label}: factor differs (gpu, oracle) {bg}"
    return so, io


def test_reference_kat_on_gpu(gpu):
    kat = json.load(open(os.path.join(HERE, "golden", "reference_kat.json")))
    for c in kat["cases"]:
        G = np.array(c["G"])
        f, x = qpgpu.solve_quadprog(G, c["g0"], c["CE"], c["ce0"], c["CI"], c["ci0"])
        assert f.hex() == c["expect_f_hex"]
        assert [v.hex() for v in x] == c["expect_x_hex"]
        assert [[v.hex() for v in row] for row in G] == c["expect_G_after_hex"]


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("name,kind,n,p,m", qp_cases.CONFIGS)
def test_config_parity(gpu, name, kind, n, p, m, family):
    B = 4096 if n <= 16 else 512
    assert_parity(qp_cases.make(kind, n, p, m, B), name, family=family)


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("name,pr", qp_cases.edge_cases(), ids=[c[0] for c in qp_cases.edge_cases()])
def test_edge_parity(gpu, name, pr, family, layout):
    assert_parity(pr, name, write_factor=True, family=family, layout=layout)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("name,kind,n,p,m,B", qp_cases.LARGE_CONFIGS)
def test_large_config_parity(gpu, name, kind, n, p, m, B, exact):
    if exact and n <= 64:
        pytest.skip("n <= 64 is bitwise on the default path already")
    assert_parity(qp_cases.make(kind, n, p, m, B, seed=11), name, exact=exact)


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("n,p,m,B", [(65, 5, 130, 6), (128, 16, 256, 4), (200, 0, 400, 3),
                                       (20, 2, 300, 4), (40, 0, 600, 3), (96, 30, 700, 2)])
@pytest.mark.parametrize("exact", [False, True])
def test_panel_setup_shapes(gpu, n, p, m, B, layout, exact):
    """MFMA panel setup + tolerance-mode loop: sizes on and off the 16-tile grid, with equalities,
    both layouts; n < 32 with m > 256 (workspace variant without the fused d/z pass), n = 40 (the
    fused pass with lanes past n idle), iq past 64 (the tree update_r's second lane group)."""
    assert_parity(qp_cases.make("general", n, p, m, B, seed=n), f"panel n={n}", layout=layout, exact=exact)


def test_panel_setup_not_pd(gpu):
    """A non-positive pivot inside the blocked factorization: same status, f = that pivot."""
    n, m = 100, 10
    pr = qp_cases.make("general", n, 0, m, 3, seed=2)
    pr.G[0, 70, 70] = -5.0e3  # row 70 fails (block 4, column 6)
    pr.G[1, :, :] = np.eye(n)
    pr.G[1, 3, 3] = 0.0       # first block, fourth pivot
    assert_parity(pr, "panel not_pd")


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("write_factor", [False, True])
@pytest.mark.parametrize("n,p,m,B", [(30, 6, 60, 65), (32, 8, 64, 64), (24, 0, 60, 33)])
def test_wave_one_wave_per_simd_edges(gpu, n, p, m, B, write_factor, layout):
    """The qp_wave variant launched at one wave per SIMD (LDS > 20 KiB per block: C3-sized QPs),
    whose Cholesky / J / x0 run in registers across the lanes: failing pivots first, inside and
    last, non-finite G entries (the reference's literal J path), the factor written back, and
    an odd batch (the last wave's second QP is idle)."""
    pr = qp_cases.make("general", n, p, m, B, seed=n + B)
    pr.G[0, 5, 5] = -1.0e3      # fails at pivot 5
    pr.G[1, 0, 0] = -1.0        # fails at pivot 0
    pr.G[2, n - 1, n - 1] = 0.0  # fails (or nearly) at the last pivot
    pr.G[3, 3, 7] = pr.G[3, 7, 3] = np.nan
    pr.G[4, 2, 2] = np.inf
    pr.G[5, 4, 9] = 1.0e300      # huge off-diagonal: overflow in the later pivots
    assert_parity(pr, f"wave edges n={n}", write_factor=write_factor, family="wave", layout=layout)


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("name,kind,n,p,m", qp_cases.CONFIGS)
def test_config_parity_tiled(gpu, name, kind, n, p, m, family):
    B = 1000 if n <= 16 else 200
    assert_parity(qp_cases.make(kind, n, p, m, B, seed=77), name, family=family, layout="tiled64")


@pytest.mark.parametrize("family", FAMILIES)
def test_batch_tail_and_odd_sizes(gpu, family):
    for B in (1, 3, 7, 9, 63, 65, 1001):
        assert_parity(qp_cases.make("general", 7, 6, 14, B, seed=B), f"B={B}", family=family)


@pytest.mark.parametrize("family", FAMILIES)
def test_max_iter_cap_matches(gpu, family):
    pr = dict(qp_cases.edge_cases())["long_paths"]
    st, _ = assert_parity(pr, "cap", max_iter=2, family=family)
    assert (st == qpgpu.QP_MAX_ITER).any()


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("family", FAMILIES)
def test_full_size_c1_parity(gpu, family, layout):
    """BASELINE.json metric config: 65 536 x (7, 6, 14), bitwise against the oracle."""
    assert_parity(qpgpu.make_problems("general", 7, 6, 14, 0, 65536, seed=2026), "C1 full", family=family,
                  layout=layout)


@pytest.mark.parametrize("family", FAMILIES)
def test_full_size_c2_parity(gpu, family):
    assert_parity(qpgpu.make_problems("box", 7, 0, 14, 0, 65536, seed=2026), "C2 full", family=family)


def test_device_api_matches_host_api(gpu):
    import torch

    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 2048, seed=99)
    db = qpgpu.DeviceBatch(pr, "cuda:0")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        db.solve(stream=s)
    s.synchronize()
    x, f, st, it = db.results()
    xh, fh, sh, ih = qpgpu.solve_batched_host(pr)
    assert np.array_equal(x, xh) and np.array_equal(f, fh) and np.array_equal(st, sh)
    # G untouched without the write-factor flag
    assert np.array_equal(db.G.cpu().numpy(), pr.G)


def test_threads_share_one_stream_workspace(gpu):
    """Host threads enqueueing workspace-kernel solves (n > 64) of different sizes on the SAME
    stream (the device's default stream): the grow-only workspace cached per (device, stream)
    must not be freed under a launch another thread has not enqueued yet (qpgpu_api.cpp
    device_workspace holds its lock through the enqueue).  Every thread's batch stays bitwise
    equal to the oracle (EXACT)."""
    import threading

    import torch

    shapes = [(66, 2, 80, 3), (120, 4, 200, 2), (90, 0, 150, 4), (160, 3, 240, 2)]
    cases = []
    for k, (n, p, m, B) in enumerate(shapes):
        pr = qpgpu.make_problems("general", n, p, m, 0, B, seed=500 + k)
        prc = qpgpu.Problems(n, p, m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
        cases.append((qpgpu.DeviceBatch(pr, "cuda:0"), oracle.solve_batch(prc)))
    s = torch.cuda.default_stream(torch.device("cuda:0"))
    errors = []

    def worker(db, reps):
        try:
            for _ in range(reps):
                db.solve(stream=s, exact=True)
        except Exception as exc:  # surfaced in the main thread
            errors.append(exc)

    threads = [threading.Thread(target=worker, args=(db, 6)) for db, _ in cases]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for (db, (xo, fo, so, io)), (n, p, m, B) in zip(cases, shapes):
        x, f, st, it = db.results()
        assert np.array_equal(st, so) and np.array_equal(it, io), (n, p, m)
        assert not _bit_mismatch(x, xo) and not _bit_mismatch(f, fo), (n, p, m)


def test_python_mirror_raises_like_reference(gpu):
    with pytest.raises(RuntimeError, match="Constraints are linearly dependent"):
        qpgpu.solve_quadprog(2 * np.eye(3), np.ones(3), [[1., 1.], [2., 2.], [0., 0.]], [1., 1.],
                             np.zeros((3, 0)), [])
    with pytest.raises(ValueError, match=r"Error in cholesky decomposition, sum: -3"):
        qpgpu.solve_quadprog(np.array([[1., 2.], [2., 1.]]), np.zeros(2), np.zeros((2, 0)), [],
                             [[1.], [0.]], [0.])
    f, x = qpgpu.solve_quadprog(np.eye(2), np.zeros(2), np.zeros((2, 0)), [],
                                [[1., -1.], [0., 0.]], [-1., 0.])
    assert f == float("inf")


def test_device_relayout_roundtrip(gpu):
    import torch

    rng = np.random.default_rng(3)
    for B, E in ((1, 5), (65, 98), (1000, 49), (4096, 33)):
        a = rng.standard_normal((B, E))
        src = torch.from_numpy(a).to("cuda:0")
        t = torch.zeros((B + 63) // 64 * 64 * E, dtype=torch.float64, device="cuda:0")
        qpgpu.relayout(src, t, B, E, True)
        back = torch.zeros_like(src)
        qpgpu.relayout(t, back, B, E, False)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), qpgpu.to_tiled64(a))
        assert np.array_equal(back.cpu().numpy(), a)


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("kind,n,p,m", [("general", 7, 6, 14), ("general", 14, 10, 28),
                                        ("general", 14, 1, 28), ("general", 30, 6, 60),
                                        ("box", 7, 0, 14), ("general", 5, 7, 6)])
def test_eq_snapshot_equals_m0_solve(gpu, family, layout, kind, n, p, m):
    """qpgpu_solve_batched_eq: the m = 0 answer written after the equality phase must equal a
    separate solve with the inequalities dropped (the reference's retry, src/mgqp.cpp:723),
    bit for bit — checked against the oracle."""
    import torch

    if not covers(family, n, m):
        pytest.skip("family does not cover the shape")
    pr = qpgpu.make_problems(kind, n, p, m, 0, 777, seed=5)
    lay = qpgpu.LAYOUTS[layout]
    db = qpgpu.DeviceBatch(pr, "cuda:0", with_iters=True, layout=layout)
    xe = torch.full_like(db.x, float("nan"))
    fe = torch.empty_like(db.f)
    se = torch.empty_like(db.status)
    db.solve(family=family, eq_out=(xe, fe, se))
    torch.cuda.synchronize()
    x, f, st, it = db.results()
    # the full solve is unchanged by the extra outputs
    xo, fo, so, io = oracle.solve_batch(pr, max_steps=1000 + 100 * (n + p + m))
    assert np.array_equal(so, st) and np.array_equal(fo.view(np.uint64), f.view(np.uint64))
    # the snapshot against the oracle's m = 0 solve
    pr0 = qpgpu.Problems(n, p, 0, pr.G.copy(), pr.g0, pr.CE, pr.ce0, np.zeros((pr.batch, n, 0)),
                         np.zeros((pr.batch, 0)))
    x0, f0, s0, _ = oracle.solve_batch(pr0)
    xe = xe.cpu().numpy()
    if lay == qpgpu.LAYOUT_TILED64:
        xe = qpgpu.from_tiled64(xe.reshape(-1), pr.batch, (n,))
    assert np.array_equal(se.cpu().numpy(), s0)
    assert np.array_equal(fe.cpu().numpy().view(np.uint64), f0.view(np.uint64))
    ok = s0 != qpgpu.QP_NOT_POSITIVE_DEFINITE
    assert np.array_equal(xe[ok].view(np.uint64), x0[ok].view(np.uint64))


def test_c4_shard_parity(gpu):
    """One rank's shard of C4 (1 048 576 x (7, 6, 14) over 8 GPUs): the last rank's 131 072 QPs,
    generated from their global indices as bench.py's rank 7 does, bitwise against the oracle."""
    import qpdist

    b0, b1 = qpdist.shard(7, 131072)
    assert_parity(qpgpu.make_problems("general", 7, 6, 14, b0, b1, seed=2026), "C4 shard 7")


@pytest.mark.parametrize("exact", [False, True])
def test_c5_bench_problems_parity(gpu, exact):
    """The bench's own C5 problems (qpgpu.make_problems, seed 2026: ~134 l1 passes per QP, iq
    well past 64), so the tolerance-mode loop (tree sums, fused d/z pass, deferred J sweep,
    DESIGN §5.3) is held to 1e-10 with identical status and pass counts over long active-set
    paths, and EXACT stays bitwise; QPs from the start and the far end of the batch."""
    n, p, m = 256, 0, 512
    for b0 in (0, 4093):
        pr = qpgpu.make_problems("general", n, p, m, b0, b0 + 3, seed=2026)
        so, io = assert_parity(pr, f"C5 bench QPs {b0}..{b0 + 2}", exact=exact)
        assert (so == qpgpu.QP_OK).all() and io.min() > 50, (so, io)


# ---- QPGPU_FLAG_FAST (the lane kernel's fast build): same status and l1-pass counts;
# x within north_star's plain 1e-10; f within 1e-10 of its terms (the fast builds' documented
# contract — the plain |df|/|f| bar needs the reference's own rounding on QPs whose f cancels,
# DESIGN §3.3, which is why no bench line's value comes from these builds)

def assert_fast_parity(pr, label, layout=None, decisions=True, family=None):
    prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xo, fo, so, io = oracle.solve_batch(prc, max_steps=1000 + 100 * (pr.n + pr.p + pr.m),
                                        threads=8 if pr.batch >= 4096 else 1)
    xg, fg, sg, ig = qpgpu.solve_batched_host(pr, fast=True, layout=layout, family=family)
    assert np.array_equal(so, sg), f"{label}: status differs at {np.where(so != sg)[0][:10]}"
    if decisions:
        assert np.array_equal(io, ig), f"{label}: l1-pass count differs at {np.where(io != ig)[0][:10]}"
    ok = so == qpgpu.QP_OK
    sub = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G[ok], pr.g0[ok], pr.CE[ok], pr.ce0[ok], pr.CI[ok], pr.ci0[ok])
    ex, efp, eft = _relerr(xg[ok], xo[ok], fg[ok], fo[ok], np.ones(int(ok.sum()), dtype=bool), sub)
    assert ex <= TOL and eft <= TOL, f"{label}: rel err x {ex:.3e} f vs its terms {eft:.3e} (plain |df|/|f| {efp:.3e})"
    return ex, eft


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("kind,p", [("general", 6), ("box", 0)])
def test_fast_full_size(gpu, kind, p, layout):
    """C1 / C2 at the bench size (65 536 QPs, seeds 2026 and 12345)."""
    for seed in (2026, 12345):
        assert_fast_parity(qpgpu.make_problems(kind, 7, p, 14, 0, 65536, seed=seed), f"fast {kind} {seed}",
                           layout=layout)


@pytest.mark.parametrize("n,p,m", [(7, 3, 14), (8, 2, 16), (5, 1, 9), (3, 0, 6), (8, 0, 16), (7, 6, 10)])
def test_fast_other_lane_shapes(gpu, n, p, m):
    """The generic (run-time p) and the N=8 instantiations of the fast build, odd batch sizes."""
    assert_fast_parity(qpgpu.make_problems("general", n, p, m, 0, 1001, seed=n * 100 + m), f"fast {(n, p, m)}")


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("name,pr", qp_cases.edge_cases(), ids=[c[0] for c in qp_cases.edge_cases()])
def test_fast_edge_cases(gpu, name, pr, layout):
    """Every exit of the algorithm through the fast build: same status; x, f within 1e-10 where the
    QP is solved.  Non-finite data (the -inf / NaN limits) makes the fast forms invalid on those
    lanes, so their waves re-solve with IEEE divisions (lane_body<..., SAFE>) — in both layouts,
    since the re-solve body has its own TILED64 loads and stores."""
    if not covers("lane", pr.n, pr.m):
        pytest.skip("shape outside the lane kernel")
    assert_fast_parity(pr, f"fast {name}", layout=layout)


def test_fast_flag_rules(gpu):
    """FAST does not combine with EXACT or WRITE_FACTOR; outside the lane shapes it is the
    default path (bitwise)."""
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 64, seed=1)
    with pytest.raises(RuntimeError):
        qpgpu.solve_batched_host(pr, fast=True, exact=True)
    with pytest.raises(RuntimeError):
        qpgpu.solve_batched_host(pr, fast=True, write_factor=True)
    assert qpgpu.kernel_name(7, 6, 14, fast=True).startswith("qp_lane_fast")
    assert qpgpu.kernel_name(30, 6, 60, fast=True).startswith("qp_wave_fast")
    # n > 64: the default path (already the 1e-10 tolerance mode) serves FAST as well
    assert qpgpu.kernel_name(100, 5, 200, fast=True) == qpgpu.kernel_name(100, 5, 200)
    big = qp_cases.make("general", 100, 5, 200, 4)
    xf, ff, sf, _ = qpgpu.solve_batched_host(big, fast=True)
    xd, fd, sd, _ = qpgpu.solve_batched_host(big)
    assert np.array_equal(xf.view(np.uint64), xd.view(np.uint64)) and np.array_equal(sf, sd)


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("kind,p", [("general", 6), ("box", 0)])
def test_fast_fallback_parity(gpu, kind, p, layout):
    """Every wave of a full C1 (C2) batch holds one QP whose G is non-finite, so every wave's fast
    attempt turns invalid in the setup and the wave re-solves with the IEEE forms: the results
    still meet the fast contract, in both layouts (the re-solve body's TILED64 x store is its
    own code).  (What the fallback costs in time is measured by tools/fallback_cost.py, not
    asserted in the parity suite.)"""
    B = 65536
    pr = qpgpu.make_problems(kind, 7, p, 14, 0, B, seed=31)
    bad = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    bad.G[5::64, 0, 0] = np.nan
    assert_fast_parity(bad, f"fast fallback {kind} (NaN G in every wave)", layout=layout)


def test_fast_loop_top_exit_regression(gpu):
    """The round-4 wrong-result run (profiles/r04_s2/worst_base.log: qp_lane_fast<N=8,M=16> on
    1 001 QPs of (8, 0, 16), seed 816, x off by up to 4e-2 on 4 QPs) with the
    loop-top exit compiled in: every QP's data is finite and moderate, so no wave takes the
    fallback, and x must stay within the fast contract (measured 4.7e-15 since round 5)."""
    assert qpgpu.kernel_name(8, 0, 16, fast=True) == "qp_lane_fast<N=8,M=16>"
    for layout in ("qp_major", "tiled64"):
        ex, _ = assert_fast_parity(qpgpu.make_problems("general", 8, 0, 16, 0, 1001, seed=816),
                                   f"loop-top regression {layout}", layout=layout)
        assert ex <= 1e-12, ex


# ---- QPGPU_FLAG_FAST for the wave kernel's LDS variants (n <= 64, m <= 256): the
# reference's own QP shapes (mgqp levels n = 14, p in {10, 1}, m = 28; src/mgqp.cpp:708), C3 and
# the other size classes — north_star's 1e-10 relative per QP, identical status and l1 passes

WAVE_FAST_SHAPES = [("general", 14, 10, 28, 4096), ("general", 14, 1, 28, 4096),
                    ("general", 30, 6, 60, 2048), ("box", 16, 0, 32, 1000),
                    ("general", 20, 0, 40, 999), ("general", 32, 3, 128, 300),
                    ("general", 48, 10, 100, 200), ("general", 64, 10, 256, 100),
                    ("box", 64, 0, 128, 64)]


@pytest.mark.parametrize("kind,n,p,m,B", WAVE_FAST_SHAPES)
def test_fast_wave_shapes(gpu, kind, n, p, m, B):
    assert qpgpu.kernel_name(n, p, m, fast=True).startswith("qp_wave_fast")
    assert_fast_parity(qpgpu.make_problems(kind, n, p, m, 0, B, seed=7 * n + m), f"fast wave {(n, p, m)}")


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("p", [10, 1])
def test_fast_wave_mgqp_levels(gpu, p, layout):
    """The reference's per-cycle QP (n = 14, m = 28; level 0 p = 10, level 2 p = 1), both
    layouts, 65 536 QPs (the bench's mgqp batch)."""
    assert_fast_parity(qpgpu.make_problems("general", 14, p, 28, 0, 65536, seed=2026),
                       f"fast mgqp p={p}", layout=layout)


def test_fast_wave_c3_full(gpu):
    """C3 at the bench size: 65 536 x (30, 6, 60), seed 2026."""
    assert_fast_parity(qpgpu.make_problems("general", 30, 6, 60, 0, 65536, seed=2026), "fast C3 full")


@pytest.mark.parametrize("name,pr", qp_cases.edge_cases(), ids=[c[0] for c in qp_cases.edge_cases()])
def test_fast_wave_edge_cases(gpu, name, pr):
    """Every exit of the algorithm through the wave kernel's fast build (forced family): same
    status, x and f within 1e-10 where solved; the non-finite cases take the IEEE fallback."""
    assert_fast_parity(pr, f"fast wave {name}", family="wave")


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("n,p,m,B", [(30, 6, 60, 65), (32, 8, 64, 64), (24, 0, 60, 33), (14, 10, 28, 9)])
def test_fast_wave_fallback_edges(gpu, n, p, m, B, layout):
    """Non-finite and extreme G entries in some QPs of a batch: those waves re-solve with the IEEE
    forms; status, passes and x, f of every QP as the oracle's (within 1e-10)."""
    pr = qp_cases.make("general", n, p, m, B, seed=n + B + 1)
    pr.G[0, 5, 5] = -1.0e3
    pr.G[1, 3, 7] = pr.G[1, 7, 3] = np.nan
    pr.G[2, 2, 2] = np.inf
    pr.G[3, 4, 9] = 1.0e300
    pr.ci0[4, 1] = -np.inf
    assert_fast_parity(pr, f"fast wave fallback n={n} {layout}", layout=layout)


# ---- the generic workspace kernel (qp_generic.hip): any n, p, m, bitwise with the reference's
# operation order — the default for shapes beyond the specialised kernels (n > 256 or m > 1024),
# and forced here on every shape the other families cover too

@pytest.mark.parametrize("name,kind,n,p,m", qp_cases.CONFIGS)
def test_generic_config_parity(gpu, name, kind, n, p, m):
    B = 512 if n <= 16 else 64
    assert_parity(qp_cases.make(kind, n, p, m, B, seed=21), f"generic {name}", write_factor=True,
                  family="generic")


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("name,pr", qp_cases.edge_cases(), ids=[c[0] for c in qp_cases.edge_cases()])
def test_generic_edge_parity(gpu, name, pr, layout):
    assert_parity(pr, f"generic {name}", write_factor=True, family="generic", layout=layout)


def test_generic_cap_and_odd_batches(gpu):
    st, _ = assert_parity(dict(qp_cases.edge_cases())["long_paths"], "generic cap", max_iter=2,
                          family="generic")
    assert (st == qpgpu.QP_MAX_ITER).any()
    for B in (1, 3, 65):
        assert_parity(qp_cases.make("general", 40, 5, 90, B, seed=B), f"generic B={B}", family="generic")


@pytest.mark.parametrize("kind,n,p,m,B", [("general", 300, 10, 1100, 2), ("general", 512, 0, 64, 2),
                                          ("general", 100, 20, 1500, 3), ("box", 260, 0, 520, 2)])
@pytest.mark.parametrize("write_factor", [False, True])
def test_generic_beyond_specialised_shapes(gpu, kind, n, p, m, B, write_factor):
    """Shapes no specialised kernel covers (n > 256 or m > 1024) run on the generic kernel by
    default — the reference's solve_quadprog takes any n, p, m (QuadProg++.hh:69-72) — bitwise
    against the oracle (x, f, status, l1 passes, and the factor left in G)."""
    assert qpgpu.kernel_name(n, p, m).startswith("qp_generic")
    assert_parity(qp_cases.make(kind, n, p, m, B, seed=n + m), f"generic {(n, p, m)}",
                  write_factor=write_factor)


# every size class's largest shape and the first one past it (kernel_name and the default path):
# lane (8, 16), subgroup S=8 (8, 32), wave LDS variants (16, 32) / (32, 128) / (64, 256), the
# workspace variant (256, 1024), then the generic kernel
BOUNDARY_SHAPES = [(8, 2, 16, 130), (8, 2, 17, 130), (9, 2, 16, 130), (8, 0, 32, 70), (8, 0, 33, 70),
                   (16, 3, 32, 40), (17, 3, 32, 40), (32, 4, 128, 20), (33, 4, 128, 20),
                   (64, 5, 256, 6), (65, 5, 256, 4), (256, 4, 1024, 1), (256, 4, 1025, 1),
                   (257, 4, 1024, 1)]


@pytest.mark.parametrize("n,p,m,B", BOUNDARY_SHAPES)
def test_size_class_boundaries(gpu, n, p, m, B):
    """Each kernel family's largest shape and the first shape past it, on the default path:
    bitwise against the oracle where the path keeps the reference's order, within 1e-10 with
    identical status and passes in the n > 64 tolerance mode, and EXACT bitwise everywhere."""
    pr = qp_cases.make("general", n, p, m, B, seed=n * 1000 + m)
    assert qpgpu.kernel_name(n, p, m), (n, p, m)
    assert_parity(pr, f"boundary {(n, p, m)} [{qpgpu.kernel_name(n, p, m)}]")
    if not bitwise_expected(n, m):
        assert_parity(pr, f"boundary {(n, p, m)} EXACT", exact=True)


@pytest.mark.parametrize("layout,B", [("qp_major", 10), ("tiled64", 150)])
def test_generic_sub_batches(gpu, layout, B):
    """The generic kernel over sub-batches (its per-launch workspace capped, qpgpu_api.cpp): with
    the cap lowered to three QPs' workspace, a batch runs as 3-QP launches (QP-major) or 64-QP
    tile launches (TILED64), each with its inputs and outputs offset — bitwise as one launch."""
    import ctypes

    n, p, m = 40, 5, 90
    qpgpu.LIB.qpk_generic_workspace_bytes.restype = ctypes.c_int64
    qpgpu.LIB.qpk_generic_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64]
    per = qpgpu.LIB.qpk_generic_workspace_bytes(n, m, 1)
    setcap = qpgpu.LIB.qpgpu_debug_set_generic_ws_cap
    setcap.argtypes = [ctypes.c_int64]
    setcap(3 * per)
    try:
        assert_parity(qp_cases.make("general", n, p, m, B, seed=B), f"generic sub-batches B={B}",
                      write_factor=True, family="generic", layout=layout)
    finally:
        setcap(0)


@pytest.mark.parametrize("layout,B", [("qp_major", 10), ("tiled64", 150)])
def test_generic_sub_batches_eq(gpu, layout, B):
    """The same sub-batches through qpgpu_solve_batched_eq: each sub-batch's x_eq /
    f_eq / status_eq and iters are offset like x / f / status — the full solve and the m = 0
    snapshot bitwise against the oracle across every sub-batch boundary."""
    import ctypes

    import torch

    n, p, m = 40, 5, 90
    qpgpu.LIB.qpk_generic_workspace_bytes.restype = ctypes.c_int64
    qpgpu.LIB.qpk_generic_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64]
    per = qpgpu.LIB.qpk_generic_workspace_bytes(n, m, 1)
    setcap = qpgpu.LIB.qpgpu_debug_set_generic_ws_cap
    setcap.argtypes = [ctypes.c_int64]
    pr = qp_cases.make("general", n, p, m, B, seed=B + 1)
    db = qpgpu.DeviceBatch(pr, "cuda:0", with_iters=True, layout=layout)
    xe = torch.full_like(db.x, float("nan"))
    fe = torch.full_like(db.f, float("nan"))
    se = torch.full_like(db.status, -7)
    setcap(3 * per)
    try:
        db.solve(family="generic", eq_out=(xe, fe, se))
        torch.cuda.synchronize()
    finally:
        setcap(0)
    x, f, st, it = db.results()
    xo, fo, so, io = oracle.solve_batch(qpgpu.Problems(n, p, m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0),
                                        max_steps=1000 + 100 * (n + p + m))
    assert np.array_equal(so, st) and np.array_equal(io, it)
    assert np.array_equal(fo.view(np.uint64), f.view(np.uint64))
    assert np.array_equal(xo.view(np.uint64), x.view(np.uint64))
    pr0 = qpgpu.Problems(n, p, 0, pr.G.copy(), pr.g0, pr.CE, pr.ce0, np.zeros((B, n, 0)), np.zeros((B, 0)))
    x0, f0, s0, _ = oracle.solve_batch(pr0)
    xe = xe.cpu().numpy()
    if layout == "tiled64":
        xe = qpgpu.from_tiled64(xe.reshape(-1), B, (n,))
    assert np.array_equal(se.cpu().numpy(), s0)
    assert np.array_equal(fe.cpu().numpy().view(np.uint64), f0.view(np.uint64))
    assert np.array_equal(xe.view(np.uint64), x0.view(np.uint64))
