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
