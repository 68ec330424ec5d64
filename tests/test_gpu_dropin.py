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
