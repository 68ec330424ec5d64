"""Runs the C++ drop-in test program (tests/dropin_test.cpp, built by __graft_entry__.build())
against libquadprog_amd.so on the GPU."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_build", "dropin_test")


def test_dropin_program(gpu):
    assert os.path.exists(BIN), "build() did not produce tests/_build/dropin_test"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin_test: OK" in r.stdout
    # the non-PD exception is preceded by print_matrix("A", G) on stdout, as in the reference
    assert "A: " in r.stdout


def test_eigen_api_program(gpu):
    """QuadProgpp::Solver (include/quadprog_amd/eigen/QuadProg++.hh) vs solve_quadprog."""
    b = os.path.join(ROOT, "tests", "_build", "eigen_api_test")
    assert os.path.exists(b), "build() did not produce tests/_build/eigen_api_test"
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "eigen_api_test: OK" in r.stdout


def _write_batch(path, pr):
    import numpy as np

    with open(path, "wb") as fh:
        np.array([pr.batch, pr.n, pr.p, pr.m], dtype=np.int32).tofile(fh)
        for b in range(pr.batch):
            for a in (pr.G[b], pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b]):
                np.ascontiguousarray(a, dtype=np.float64).tofile(fh)


def _parse(out):
    recs = []
    for ln in out.splitlines():
        if ln.startswith("f "):
            tok = ln.split()
            xi, gi = tok.index("x"), tok.index("G")
            recs.append(("ok", float.fromhex(tok[1]), [float.fromhex(t) for t in tok[xi + 1:gi]],
                         [float.fromhex(t) for t in tok[gi + 1:]]))
        elif ln.startswith(("runtime_error", "logic_error")):
            recs.append((ln.split()[0], ln.split(" ", 1)[1]))
    return recs


@pytest.mark.parametrize("kind,n,p,m", [("general", 7, 6, 14), ("box", 7, 0, 14),
                                        ("general", 14, 10, 28), ("general", 30, 6, 60),
                                        ("general", 300, 10, 1100), ("general", 512, 0, 64)])
def test_single_qp_through_cpp_symbol_matches_oracle(gpu, tmp_path, kind, n, p, m):
    """BASELINE config 1: single QPs through the mangled solve_quadprog symbol (ArrayHH
    containers, t() temporaries as src/mgqp.cpp:708 passes them), one call each, bit for bit
    against the oracle: f, x and the Cholesky factor left in G.  The reference takes any size
    (QuadProg++.hh:69-72): (300, 10, 1100) and (512, 0, 64) go through the generic kernel."""
    import numpy as np

    import oracle
    import qpgpu

    pr = qpgpu.make_problems(kind, n, p, m, 0, 48 if n <= 64 else 2, seed=31)
    path = str(tmp_path / "qps.bin")
    _write_batch(path, pr)
    r = subprocess.run([BIN, "--qp", path], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    recs = _parse(r.stdout)
    assert len(recs) == pr.batch
    for b, rec in enumerate(recs):
        G = pr.G[b].copy()
        st, f, x, _ = oracle.solve_one(G, pr.g0[b], pr.CE[b], pr.ce0[b], pr.CI[b], pr.ci0[b],
                                       max_steps=1000 + 100 * (n + p + m))
        if st == qpgpu.QP_DEPENDENT:
            assert rec == ("runtime_error", "Constraints are linearly dependent")
            continue
        assert st in (qpgpu.QP_OK, qpgpu.QP_INFEASIBLE) and rec[0] == "ok", (b, st, rec[:2])
        assert np.float64(rec[1]).view(np.uint64) == np.float64(f).view(np.uint64), b
        assert np.array_equal(np.array(rec[2]).view(np.uint64), x.view(np.uint64)), b
        assert np.array_equal(np.array(rec[3]).view(np.uint64), G.reshape(-1).view(np.uint64)), b


@pytest.mark.parametrize("kind,n,p,m", [("general", 7, 6, 14), ("general", 14, 10, 28)])
def test_eigen_api_matches_oracle(gpu, tmp_path, kind, n, p, m):
    """The Eigen-variant Solver API (include/quadprog_amd/eigen/QuadProg++.hh, reference
    eigen/QuadProg++.hh:101-118) through both container paths, against the oracle bit for bit:
    status, objective and x (the fork itself is unpinned: its archive is missing)."""
    import numpy as np

    import oracle
    import qpgpu

    b = os.path.join(ROOT, "tests", "_build", "eigen_api_test")
    pr = qpgpu.make_problems(kind, n, p, m, 0, 32, seed=8)
    path = str(tmp_path / "qps.bin")
    _write_batch(path, pr)
    r = subprocess.run([b, "--qp", path], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln.split() for ln in r.stdout.splitlines() if ln[:2] in ("A ", "C ")]
    assert len(lines) == 2 * pr.batch
    for q in range(pr.batch):
        st, f, x, _ = oracle.solve_one(pr.G[q].copy(), pr.g0[q], pr.CE[q], pr.ce0[q], pr.CI[q],
                                       pr.ci0[q], max_steps=1000 + 100 * (n + p + m))
        for tok in lines[2 * q: 2 * q + 2]:
            assert int(tok[1]) == st, (q, tok[0])
            assert np.float64(float.fromhex(tok[2])).view(np.uint64) == np.float64(f).view(np.uint64)
            xs = np.array([float.fromhex(t) for t in tok[3:]])
            assert np.array_equal(xs.view(np.uint64), x.view(np.uint64)), (q, tok[0])


def test_single_calls_outputs_fresh(gpu):
    """The zero-copy host entry (the drop-in's path) once returned the previous call's x with the
    new call's status and f (profiles/r06_f6: the outputs then shared the coarse-grained staging
    buffer, whose L2 write-backs the status word could overtake).  3 000 consecutive single
    (7, 6, 14) solves of distinct QPs through the host entry: x, f, status and the factor written
    back bitwise against the oracle every time (a stale x would be the zeros passed in)."""
    import numpy as np

    import oracle
    import qpgpu

    n, p, m, B = 7, 6, 14, 3000
    pr = qpgpu.make_problems("general", n, p, m, 0, B, seed=77)
    prc = qpgpu.Problems(n, p, m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    xo, fo, so, _ = oracle.solve_batch(prc, write_factor=True, max_steps=1000 + 100 * (n + p + m))
    for q in range(B):
        one = qpgpu.Problems(n, p, m, pr.G[q:q + 1].copy(), pr.g0[q:q + 1], pr.CE[q:q + 1], pr.ce0[q:q + 1],
                             pr.CI[q:q + 1], pr.ci0[q:q + 1])
        x, f, st, _ = qpgpu.solve_batched_host(one, write_factor=True)
        assert st[0] == so[q], q
        assert np.float64(f[0]).view(np.uint64) == np.float64(fo[q]).view(np.uint64), q
        assert np.array_equal(x[0].view(np.uint64), xo[q].view(np.uint64)), (q, x[0], xo[q])
        assert np.array_equal(one.G.view(np.uint64), prc.G[q:q + 1].view(np.uint64)), q
