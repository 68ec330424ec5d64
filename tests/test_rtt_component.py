"""The reference component on the RTT surface (reference
src/mgqp.cpp:89-95 operations, :180-482 ports, :874-916 FlowStatus handling, :1270 factory),
deployed and connected by port name as ops/mgqp.ops:180-236 does (tests/rtt_component_test.cpp).

CPU suite: the component + controller sources linked with the test-only oracle harness
(tests/_build/libmgqp_cpu_harness.so).  GPU suite: the binary build() links against the shipped
libmgqp_amd.so, so every QP of every cycle runs on the gfx950 kernels.  Either way every cycle's
out_torques read through a connected port must equal the CycleInputs path bit for bit."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd")


def _run(exe, cycles):
    r = subprocess.run([exe, str(cycles)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"OK: {cycles} cycles through ports == CycleInputs path (bitwise)" in r.stdout
    return r.stdout


def test_rtt_component_cpu_harness():
    import test_mgqp_host

    harness = test_mgqp_host.build_harness()
    exe = os.path.join(HERE, "_build", "rtt_component_test_cpu")
    subprocess.check_call([
        "g++", "-O2", "-std=c++17", "-Wall", "-ffp-contract=off",
        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "include", "quadprog_amd"),
        "-o", exe, os.path.join(HERE, "rtt_component_test.cpp"),
        os.path.join(PKG, "csrc", "mgqp_component.cpp"),
        "-L" + os.path.dirname(harness), "-lmgqp_cpu_harness", "-Wl,-rpath," + os.path.dirname(harness)])
    out = _run(exe, 30)
    assert "FAILED, NO DATA, RETURN" in out and "NO JACOBIAN FOR JOINT 7" in out


@pytest.mark.gpu
def test_rtt_component_gpu(gpu):
    exe = os.path.join(HERE, "_build", "rtt_component_test")
    if not os.path.exists(exe):
        pytest.fail("tests/_build/rtt_component_test missing: run __graft_entry__.build()")
    _run(exe, 40)
