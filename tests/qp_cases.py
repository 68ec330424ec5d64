"""Problem families shared by the CPU and GPU test suites (SURVEY.md §8(d) configs + edge cases
of the reference's contract, QuadProg++.hh:8-45, and the error paths of SURVEY §5)."""
import numpy as np

import qpgpu

# (name, kind, n, p, m) — C1/C4, C2, C3, the two mgqp levels, plus small shapes
CONFIGS = [
    ("C1_general_7_6_14", "general", 7, 6, 14),
    ("C2_box_7_0_14", "box", 7, 0, 14),
    ("mgqp_L0_14_10_28", "general", 14, 10, 28),
    ("mgqp_L2_14_1_28", "general", 14, 1, 28),
    ("C3_general_30_6_60", "general", 30, 6, 60),
    ("general_8_0_16", "general", 8, 0, 16),
    ("general_5_2_30", "general", 5, 2, 30),
    ("box_16_0_32", "box", 16, 0, 32),
    ("general_16_3_64", "general", 16, 3, 64),
    ("general_1_0_2", "general", 1, 0, 2),
    ("general_3_0_0", "general", 3, 0, 0),
    ("general_4_4_0", "general", 4, 4, 0),
]


# shapes only the qp_wave kernels cover (n > 16), with batch sizes the oracle finishes quickly
LARGE_CONFIGS = [
    ("n17_general", "general", 17, 3, 40, 256),
    ("n32_general", "general", 32, 8, 64, 256),
    ("n33_box", "box", 33, 0, 66, 128),
    ("n48_general", "general", 48, 10, 100, 64),
    ("n64_general", "general", 64, 0, 128, 32),
    ("n64_box", "box", 64, 0, 128, 32),
    ("n100_general", "general", 100, 20, 200, 8),
    ("C5_n256_box", "box", 256, 0, 512, 4),
    ("C5_n256_general", "general", 256, 0, 512, 2),
]


def make(kind, n, p, m, B, seed=12345):
    return qpgpu.make_problems(kind, n, p, m, 0, B, seed=seed)


def edge_cases():
    """Small hand-built batches that force every exit of the algorithm."""
    out = []
    # reference demo
    out.append(("demo", qpgpu.Problems(2, 1, 3, np.array([[[4., -2.], [-2., 4.]]]), np.array([[6., 0.]]),
                                       np.array([[[1.], [1.]]]), np.array([[-3.]]),
                                       np.array([[[1., 0., 1.], [0., 1., 1.]]]), np.array([[0., 0., -2.]]))))
    # infeasible: x0 >= 1 and x0 <= 0
    out.append(("infeasible", qpgpu.Problems(2, 0, 2, np.eye(2)[None].copy(), np.zeros((1, 2)),
                                             np.zeros((1, 2, 0)), np.zeros((1, 0)),
                                             np.array([[[1., -1.], [0., 0.]]]), np.array([[-1., 0.]]))))
    # dependent equalities (duplicated column)
    out.append(("dependent", qpgpu.Problems(3, 2, 0, (2 * np.eye(3))[None].copy(), np.ones((1, 3)),
                                            np.array([[[1., 1.], [2., 2.], [0., 0.]]]), np.array([[1., 1.]]),
                                            np.zeros((1, 3, 0)), np.zeros((1, 0)))))
    # G not positive definite
    out.append(("not_pd", qpgpu.Problems(2, 0, 1, np.array([[[1., 2.], [2., 1.]]]), np.zeros((1, 2)),
                                         np.zeros((1, 2, 0)), np.zeros((1, 0)),
                                         np.array([[[1.], [0.]]]), np.array([[0.]]))))
    # G negative on the first pivot
    out.append(("not_pd0", qpgpu.Problems(2, 0, 0, np.array([[[-1., 0.], [0., 1.]]]), np.zeros((1, 2)),
                                          np.zeros((1, 2, 0)), np.zeros((1, 0)),
                                          np.zeros((1, 2, 0)), np.zeros((1, 0)))))
    # mgqp retry shape: identity G, zero g0, equalities only (src/mgqp.cpp:723-725)
    rng = np.random.default_rng(7)
    CE = rng.standard_normal((1, 6, 3))
    out.append(("mgqp_retry", qpgpu.Problems(6, 3, 0, np.eye(6)[None].copy(), np.zeros((1, 6)), CE,
                                             rng.standard_normal((1, 3)), np.zeros((1, 6, 0)), np.zeros((1, 0)))))
    # -inf limit (the "-inf problem.log.txt" chain: log() of a negative joint margin)
    pr = qpgpu.make_problems("box", 7, 0, 14, 0, 1, seed=3)
    pr.ci0[0, 3] = -np.inf
    out.append(("neg_inf_limit", pr))
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 1, seed=4)
    pr.ci0[0, 5] = np.nan
    out.append(("nan_limit", pr))
    # duplicated / near-duplicated inequality columns (degenerate add_constraint -> rollback)
    prs = qpgpu.make_problems("general", 6, 0, 12, 0, 64, seed=5)
    prs.CI[:, :, 6:] = prs.CI[:, :, :6]
    prs.ci0[:, 6:] = prs.ci0[:, :6] - 1e-3
    out.append(("duplicated_ineq", prs))
    prs = qpgpu.make_problems("general", 5, 1, 15, 0, 64, seed=6)
    prs.CI[:, :, 10:] = prs.CI[:, :, :5] * 2.0
    prs.ci0[:, 10:] = prs.ci0[:, :5] * 2.0 - 0.5
    out.append(("scaled_dup_ineq", prs))
    # many strongly violated constraints (long active-set paths)
    prs = qpgpu.make_problems("general", 8, 0, 16, 0, 256, seed=8)
    prs.g0 *= 30.0
    out.append(("long_paths", prs))
    # p > n: reference UB; both implementations report "dependent"
    out.append(("p_gt_n", qpgpu.Problems(2, 3, 0, np.eye(2)[None].copy(), np.zeros((1, 2)),
                                         np.array([[[1., 0., 1.], [0., 1., 1.]]]), np.array([[1., 1., 1.]]),
                                         np.zeros((1, 2, 0)), np.zeros((1, 0)))))
    return out


# ---- seeded fuzz cases (tests/test_gpu_fuzz.py): random shapes across every kernel family and
# per-QP data modes the configs above do not reach — exact ties in the most-violated selection
# (small-integer data), ill-conditioned and badly scaled G, zero / duplicated / contradictory
# constraint columns, rank-deficient CE.  Every QP is drawn from (seed, its index) only.

FUZZ_MODES = ("plain", "ill_conditioned", "scaled", "dup_zero_cols", "contradictory", "rank_def_ce",
              "diag_box", "integer_ties")


def _fuzz_qp(rng, n, p, m, mode, mild):
    A = rng.standard_normal((n, n))
    G = A.T @ A + n * np.eye(n)
    g0 = 10.0 * rng.standard_normal(n)
    xf = 0.1 * rng.standard_normal(n)
    CE = rng.standard_normal((n, p))
    CI = rng.standard_normal((n, m))
    slack = np.abs(rng.standard_normal(m))
    if mode == "ill_conditioned":
        Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
        k = rng.uniform(1.0, 2.0 if mild else 8.0)
        G = (Q * np.logspace(0.0, -k, n)) @ Q.T
        G = 0.5 * (G + G.T)
    elif mode == "scaled":
        s = rng.uniform(-3, 3) if mild else rng.uniform(-40, 40)
        G *= 10.0 ** s
        g0 *= 10.0 ** (s + rng.uniform(-2, 2))
        CI *= 10.0 ** rng.uniform(-3 if mild else -20, 3 if mild else 20)
    elif mode == "dup_zero_cols" and m >= 2:
        for j in rng.choice(m, size=max(1, m // 3), replace=False):
            src = int(rng.integers(m))
            r = int(rng.integers(3))
            CI[:, j] = CI[:, src] * (1.0 if r == 0 else rng.uniform(0.5, 2.0)) if r < 2 else 0.0
    elif mode == "diag_box":
        G = np.diag(rng.uniform(0.1, 10.0, n))
        if m >= 2 * n:
            CI[:, :2 * n] = np.hstack([-np.eye(n), np.eye(n)])
    elif mode == "integer_ties":
        G = np.diag(rng.integers(1, 4, n).astype(float))
        g0 = rng.integers(-4, 5, n).astype(float)
        CE = rng.integers(-1, 2, (n, p)).astype(float)
        CI = rng.integers(-1, 2, (n, m)).astype(float)
        xf = np.zeros(n)
        slack = rng.integers(0, 3, m).astype(float)
    elif mode == "rank_def_ce" and p >= 2:
        CE[:, -1] = CE[:, 0] * rng.choice([1.0, -2.0, 0.5])
    ce0 = -CE.T @ xf
    ci0 = -CI.T @ xf + slack
    if mode == "contradictory" and m >= 2:
        j = int(rng.integers(m - 1))
        CI[:, j + 1] = -CI[:, j]
        ci0[j + 1] = -ci0[j] - rng.uniform(0.0, 1.0)
    if mode == "dup_zero_cols":
        zero = ~CI.any(axis=0)
        ci0[zero] = np.where(rng.random(int(zero.sum())) < 0.5, -1.0, 1.0)
    return G, g0, CE, ce0, CI, ci0


def fuzz_case(seed, mild=False, large=False):
    """A batch of random shape: n in [1, 64], p in [0, n], m in [0, 4n] (capped at 256), 1..300
    QPs, each QP's data mode drawn independently.  mild=True keeps cond(G) <= 1e2 and
    scales within 1e+-6 (the fast builds' 1e-10 contract is relative to a well-posed problem).
    large=True draws n in [65, 192], m in [0, 2n], 1..4 QPs (the workspace variant's shapes).
    Returns (problems, each QP's mode)."""
    rng = np.random.default_rng([20261018 + large, seed])
    if large:
        n = int(rng.integers(65, 193))
        p = int(rng.integers(0, 11))
        m = int(rng.integers(0, 2 * n + 1))
        B = int(rng.integers(1, 5))
    else:
        n = int(rng.choice([int(rng.integers(1, 9)), int(rng.integers(9, 17)), int(rng.integers(17, 65))],
                           p=[0.5, 0.3, 0.2]))
        p = int(rng.integers(0, min(n, 10) + 1))
        m = int(min(256, rng.integers(0, 4 * n + 1)))
        if n <= 8 and rng.random() < 0.5:
            m = min(m, 16)
        B = int(rng.integers(1, 301 if n <= 16 else 65))
    modes = [FUZZ_MODES[int(rng.integers(len(FUZZ_MODES)))] for _ in range(B)]
    qs = [_fuzz_qp(np.random.default_rng([20261018 + large, seed, b]), n, p, m, modes[b], mild) for b in range(B)]
    st = lambda k: np.ascontiguousarray(np.stack([q[k] for q in qs]))
    return qpgpu.Problems(n, p, m, st(0), st(1), st(2), st(3), st(4), st(5)), modes
