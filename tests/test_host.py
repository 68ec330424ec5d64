"""CPU tests of the host side: C-ABI library surface (loads, exports every declared symbol,
fails loudly without a device), the drop-in's exported C++ symbol, the generator, and the
reference-mirroring argument checks."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import qpgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "qpgpu.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(qpgpu_\w+)\(", src, flags=re.M)))


def test_header_and_exports_agree():
    decl = declared_functions()
    assert set(decl) == set(qpgpu.EXPORTED_SYMBOLS)
    lib = ctypes.CDLL(qpgpu.LIB_PATH)
    for name in decl:
        assert hasattr(lib, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", qpgpu.LIB_PATH]).decode()
    for name in decl:
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_dropin_exports_reference_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", qpgpu.DROPIN_PATH]).decode()
    assert "_Z14solve_quadprogRN7ArrayHH6MatrixIdEERNS_6VectorIdEERKS1_RKS4_S7_S9_S5_" in out


def test_eigen_api_header_builds_and_fails_loudly_without_gpu():
    """QuadProgpp::Solver (reference eigen/QuadProg++.hh:83-118): build() compiled the test
    program against the header; with no device it must abort on the C-ABI error, never solve
    on the CPU."""
    b = os.path.join(ROOT, "tests", "_build", "eigen_api_test")
    assert os.path.exists(b), "build() did not produce tests/_build/eigen_api_test"
    if qpgpu.device_count() > 0:
        pytest.skip("a GPU is visible: covered by tests/test_gpu_dropin.py")
    r = subprocess.run([b], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "qpgpu: solve failed" in r.stderr


def test_kernel_coverage_table():
    assert qpgpu.kernel_name(7, 6, 14) != ""
    assert qpgpu.kernel_name(7, 0, 14) != ""
    assert qpgpu.kernel_name(14, 10, 28) != ""
    assert qpgpu.kernel_name(0, 0, 0) == ""
    assert qpgpu.LIB.qpgpu_abi_version() == 1
    # any size, as the reference (QuadProg++.hh:69-72): beyond the specialised kernels the
    # generic workspace kernel
    for shape in ((300, 10, 1100), (512, 0, 64), (100, 20, 1500), (4000, 0, 8)):
        assert qpgpu.kernel_name(*shape).startswith("qp_generic"), shape
    assert qpgpu.kernel_name(50000, 0, 1) == ""  # n*n >= 2^31: outside even the generic kernel
    g = qpgpu.LIB.qpgpu_kernel_name_flags(7, 6, 14, qpgpu.FLAG_FORCE_GENERIC).decode()
    assert g.startswith("qp_generic")


def test_kernel_name_flags_follow_the_flag_rules():
    """qpgpu_kernel_name_flags names what a launch with those flags runs, and nothing for flag
    combinations the solve entry points reject."""
    nm = lambda f: qpgpu.LIB.qpgpu_kernel_name_flags(7, 6, 14, f).decode()
    assert nm(qpgpu.FLAG_FAST).startswith("qp_lane_fast")
    assert nm(0) == qpgpu.kernel_name(7, 6, 14)
    assert nm(qpgpu.FLAG_FAST | qpgpu.FLAG_EXACT) == ""
    assert nm(qpgpu.FLAG_FAST | qpgpu.FLAG_WRITE_FACTOR) == ""
    assert nm(qpgpu.FLAG_FORCE_LANE | qpgpu.FLAG_FORCE_WAVE) == ""
    assert nm(0x8) == ""
    # the generic family has no fast build: FAST | FORCE_GENERIC launches (and names) the generic
    # kernel, on every shape
    for shape in ((7, 6, 14), (30, 6, 60), (14, 10, 28)):
        g = qpgpu.LIB.qpgpu_kernel_name_flags(*shape, qpgpu.FLAG_FAST | qpgpu.FLAG_FORCE_GENERIC).decode()
        assert g.startswith("qp_generic"), (shape, g)
    # bit 0x1000 (the removed lane-pair family) is an unknown flag now
    assert nm(qpgpu.FLAG_FAST | 0x1000) == ""
    assert "qp_pair" not in open(qpgpu.LIB._name, "rb").read().decode("latin-1")


def test_no_device_fails_loudly():
    if qpgpu.device_count() > 0:
        pytest.skip("a GPU is visible")
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 4)
    with pytest.raises(qpgpu.QpgpuError):
        qpgpu.solve_batched_host(pr)


def test_invalid_arguments():
    d = qpgpu.ProblemDesc(0, 0, 0, 0, 1, 0, 0)
    z = ctypes.c_void_p(0)
    assert qpgpu.LIB.qpgpu_solve_batched(ctypes.byref(d), *([z] * 11)) == qpgpu.ERR_INVALID_ARGUMENT
    d = qpgpu.ProblemDesc(7, 6, 14, 0, 4, 0x80, 0)
    assert qpgpu.LIB.qpgpu_solve_batched(ctypes.byref(d), *([z] * 11)) == qpgpu.ERR_INVALID_ARGUMENT
    d = qpgpu.ProblemDesc(7, 6, 14, 0, 4, 0, 7)  # unknown layout
    assert qpgpu.LIB.qpgpu_solve_batched(ctypes.byref(d), *([z] * 11)) == qpgpu.ERR_INVALID_ARGUMENT
    d = qpgpu.ProblemDesc(7, 6, 14, 0, 0, 0, 0)  # empty batch is a no-op
    assert qpgpu.LIB.qpgpu_solve_batched(ctypes.byref(d), *([z] * 11)) == qpgpu.SUCCESS


def test_generator_is_counter_based():
    a = qpgpu.make_problems("general", 7, 6, 14, 0, 100, seed=2026)
    b = qpgpu.make_problems("general", 7, 6, 14, 40, 60, seed=2026)
    for u, v in zip(a.arrays(), b.arrays()):
        assert np.array_equal(u[40:60], v)
    c = qpgpu.make_problems("general", 7, 6, 14, 0, 100, seed=2027)
    assert not np.array_equal(a.G, c.G)
    # G symmetric positive definite, CI feasible at x_f by construction
    assert np.allclose(a.G, np.swapaxes(a.G, 1, 2))
    assert np.all(np.linalg.eigvalsh(a.G) > 0)


def test_box_generator_layout():
    pr = qpgpu.make_problems("box", 7, 0, 14, 0, 3)
    assert np.array_equal(pr.CI[0], np.concatenate([-np.eye(7), np.eye(7)], axis=1))
    assert np.array_equal(pr.ci0[0], np.ones(14))


def test_algorithmic_bytes():
    # C2 1408, C1/C4 1792, C3 24056, C5 1581064 bytes per QP
    assert qpgpu.algorithmic_bytes_per_qp(7, 0, 14) == 1408
    assert qpgpu.algorithmic_bytes_per_qp(7, 6, 14) == 1792
    assert qpgpu.algorithmic_bytes_per_qp(30, 6, 60) == 24056
    assert qpgpu.algorithmic_bytes_per_qp(256, 0, 512) == 1581064


def test_python_mirror_dimension_errors():
    with pytest.raises(ValueError, match="not a squared matrix"):
        qpgpu.solve_quadprog(np.zeros((2, 3)), np.zeros(3), np.zeros((3, 0)), [], np.zeros((3, 0)), [])
    with pytest.raises(ValueError, match="ce0 is incompatible"):
        qpgpu.solve_quadprog(np.eye(2), np.zeros(2), np.ones((2, 1)), [1.0, 2.0], np.zeros((2, 0)), [])
    with pytest.raises(ValueError, match="ci0 is incompatible"):
        qpgpu.solve_quadprog(np.eye(2), np.zeros(2), np.zeros((2, 0)), [], np.ones((2, 2)), [1.0])


def test_tiled64_roundtrip_host():
    rng = np.random.default_rng(0)
    for B in (1, 63, 64, 65, 200):
        a = rng.standard_normal((B, 7, 3))
        t = qpgpu.to_tiled64(a)
        assert t.size == (B + 63) // 64 * 64 * 21
        # element e of QP b at (b//64)*64*E + e*64 + b%64
        b, e = B - 1, 20
        assert t[(b // 64) * 64 * 21 + e * 64 + b % 64] == a.reshape(B, 21)[b, e]
        assert np.array_equal(qpgpu.from_tiled64(t, B, (7, 3)), a)


def test_library_built_from_the_current_sources():
    """The in-tree libqpgpu.so was linked from the sources in the tree (the Makefile records their
    sha256, qpgpu.build_provenance): a stale library — the round-4 wrong-result run came from one
     — fails here instead of being measured."""
    if os.environ.get("QPGPU_LIB_PATH"):
        pytest.skip("an A/B library is loaded")
    prov = qpgpu.build_provenance()
    assert prov["sources_sha256_at_build"], prov
    assert prov["matches_sources"], f"libqpgpu.so is older than its sources: rebuild ({prov})"
