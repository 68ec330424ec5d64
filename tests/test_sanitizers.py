"""ASan + UBSan over the CPU-side code (SURVEY.md §5 "Race detection / sanitizers").

The shipped host sources — the ArrayHH drop-in (quadprog_dropin.cpp), the controller
(mgqp_controller.cpp, mgqp_capi.cpp), the RTT component and shim (mgqp_component.cpp,
include/quadprog_amd/rtt/RTT.hh) — and the CPU restatement (oracle/qp_oracle.c) are compiled
with -fsanitize=address,undefined -fno-sanitize-recover=all and driven by the same test programs
the GPU suite runs (dropin_test, eigen_api_test, rtt_component_test).  The GPU is replaced by
tests/qpgpu_host_cpu_stub.cpp (the C-ABI host entry on the oracle), so this runs in the CPU suite.
Any sanitizer report aborts the program and fails the test.  The HIP kernels themselves are not
covered: GPU sanitizers are not available on this pool."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd", "csrc")
OUT = os.path.join(HERE, "_build", "san")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
INC = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "include", "quadprog_amd")]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _oracle_obj():
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "qp_oracle_san.o")
    subprocess.check_call(["gcc", "-std=c11", "-ffp-contract=off", *SAN, *INC, "-c",
                           os.path.join(ROOT, "oracle", "qp_oracle.c"), "-o", obj])
    return obj


def _build(name, sources):
    exe = os.path.join(OUT, name)
    subprocess.check_call(["g++", "-std=c++17", "-ffp-contract=off", "-pthread", *SAN, *INC, "-o", exe,
                           *sources, os.path.join(HERE, "qpgpu_host_cpu_stub.cpp"), _oracle_obj()])
    return exe


def _run(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=600, env=ENV)
    log = r.stdout[-4000:] + r.stderr[-4000:]
    assert r.returncode == 0, log
    assert "ERROR: AddressSanitizer" not in log and "runtime error:" not in log, log
    return r.stdout


def test_dropin_asan_ubsan():
    exe = _build("dropin_test_san", [os.path.join(HERE, "dropin_test.cpp"),
                                     os.path.join(CSRC, "quadprog_dropin.cpp")])
    out = _run(exe)
    assert "CHECK FAILED" not in out, out[-3000:]


def test_eigen_api_asan_ubsan():
    exe = _build("eigen_api_test_san", ["-DQUADPROGPP_DISABLE_EIGEN", os.path.join(HERE, "eigen_api_test.cpp"),
                                        os.path.join(CSRC, "quadprog_dropin.cpp")])
    out = _run(exe)
    assert "CHECK FAILED" not in out and "FAIL" not in out, out[-3000:]


def test_rtt_component_asan_ubsan():
    exe = _build("rtt_component_test_san", [os.path.join(HERE, "rtt_component_test.cpp"),
                                            os.path.join(CSRC, "mgqp_component.cpp"),
                                            os.path.join(CSRC, "mgqp_controller.cpp"),
                                            os.path.join(CSRC, "mgqp_capi.cpp"),
                                            os.path.join(CSRC, "quadprog_dropin.cpp")])
    out = _run(exe, "20")
    assert "OK: 20 cycles through ports == CycleInputs path (bitwise)" in out, out[-3000:]
