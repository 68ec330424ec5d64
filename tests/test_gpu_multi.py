"""qpgpu_solve_batched_multi (include/qpgpu.h): the batch split into contiguous shards over
several GPUs of one process, each shard's outputs gathered into the caller's buffers — the C++
host's multi-GPU path (north_star).  On the one-GPU box the same device is listed
several times (its shards then run concurrently on separate worker threads and streams); every
result bitwise against the oracle and against one single-device call."""
import os
import subprocess

import numpy as np
import pytest

import oracle
import qpgpu
from test_gpu_dropin import _write_batch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_build", "multi_dev_test")


def _oracle(pr, write_factor=False):
    prc = qpgpu.Problems(pr.n, pr.p, pr.m, pr.G.copy(), pr.g0, pr.CE, pr.ce0, pr.CI, pr.ci0)
    return oracle.solve_batch(prc, write_factor=write_factor, max_steps=1000 + 100 * (pr.n + pr.p + pr.m),
                              threads=8 if pr.batch >= 4096 else 1) + (prc.G,)


def _bitwise(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


@pytest.mark.parametrize("layout", ["qp_major", "tiled64"])
@pytest.mark.parametrize("ndev", [1, 2, 3, 5])
@pytest.mark.parametrize("kind,n,p,m,B", [("general", 7, 6, 14, 4099), ("box", 7, 0, 14, 1000),
                                          ("general", 14, 10, 28, 777), ("general", 30, 6, 60, 130),
                                          ("general", 100, 5, 200, 5)])
def test_multi_device_shards(gpu, kind, n, p, m, B, ndev, layout):
    pr = qpgpu.make_problems(kind, n, p, m, 0, B, seed=n * 7 + ndev)
    xo, fo, so, io, _ = _oracle(pr)
    x, f, st, it = qpgpu.solve_batched_host(pr, layout=layout, devices=[0] * ndev)
    assert np.array_equal(st, so) and np.array_equal(it, io)
    x1, f1, s1, i1 = qpgpu.solve_batched_host(pr, layout=layout)
    assert _bitwise(f, f1) and _bitwise(x, x1) and np.array_equal(st, s1)
    if "qp_panel" in qpgpu.kernel_name(n, p, m):  # the n > 64 default: tolerance mode
        ok = so == qpgpu.QP_OK
        ex, ef = qpgpu.rel_error_per_qp(x[ok], xo[ok], f[ok], fo[ok])
        assert ex.max() <= 1e-10 and ef.max() <= 1e-10
    else:
        assert _bitwise(f, fo) and _bitwise(x, xo)


def test_multi_device_write_factor_and_edges(gpu):
    """The factor written back per shard, and the reference's exits spread over the shards: not
    positive definite, -inf / NaN limits, duplicated inequality columns (degenerate adds)."""
    big = qpgpu.make_problems("general", 7, 6, 14, 0, 300, seed=3)
    big.G[10, 0, 0] = -1.0
    big.G[200, 3, 3] = -50.0
    big.ci0[20, 3] = -np.inf
    big.ci0[120, 5] = np.nan
    big.CI[50:60, :, 7:] = big.CI[50:60, :, :7]
    big.ci0[50:60, 7:] = big.ci0[50:60, :7] - 1e-3
    xo, fo, so, io, Go = _oracle(big, write_factor=True)
    G = big.G.copy()
    pr = qpgpu.Problems(7, 6, 14, G, big.g0, big.CE, big.ce0, big.CI, big.ci0)
    x, f, st, it = qpgpu.solve_batched_host(pr, write_factor=True, devices=[0, 0, 0, 0])
    assert (so == qpgpu.QP_NOT_POSITIVE_DEFINITE).sum() >= 1
    assert np.array_equal(st, so) and np.array_equal(it, io)
    assert _bitwise(np.where(np.isnan(fo), 0, f), np.where(np.isnan(fo), 0, fo))
    ok = so != qpgpu.QP_NOT_POSITIVE_DEFINITE
    assert _bitwise(x[ok], xo[ok]) and _bitwise(G, Go)


def test_multi_device_argument_errors(gpu):
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 10, seed=1)
    for devs in ([], [qpgpu.device_count()], [-1], [0] * 65):
        with pytest.raises(qpgpu.QpgpuError, match="code 1"):
            qpgpu.solve_batched_host(pr, devices=devs)


def test_multi_device_cpp_program(gpu, tmp_path):
    """The C++ host's call (tests/multi_dev_test.cpp: plain C-ABI, no Python): 2 049 C1 QPs over
    the device listed three times, bitwise against the oracle."""
    assert os.path.exists(BIN), "build() did not produce tests/_build/multi_dev_test"
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 2049, seed=77)
    path = tmp_path / "batch.bin"
    _write_batch(str(path), pr)
    r = subprocess.run([BIN, str(path), "0", "0", "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr
    assert "multi_dev_test: OK 2049 QPs over 3 device slots" in r.stdout
    xo, fo, so, io, _ = _oracle(pr)
    recs = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("qp ")]
    assert len(recs) == pr.batch
    for b, t in enumerate(recs):
        assert int(t[1]) == b and int(t[2]) == so[b] and int(t[3]) == io[b]
        assert float.fromhex(t[4]) == fo[b] or (np.isnan(fo[b]) and t[4].endswith("nan"))
        assert [float.fromhex(v) for v in t[6:]] == xo[b].tolist()
