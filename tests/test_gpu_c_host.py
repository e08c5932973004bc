"""The C ABI from a plain C host (tests/native/c_host_check.c): no Python and
no PyTorch between the caller and libdlsim_hip.so — what a non-Python binding
of the reference's aggregate does. Every case is compared
bit for bit with the C oracle inside the program."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "native", "_build", "c_host_check")


def test_c_host_check():
    assert os.path.exists(BIN), "build() compiles tests/native/c_host_check.c"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("c_host_check OK"), r.stdout
    assert r.stdout.count("bit-identical") == 27, r.stdout
    assert "dlsim_device_alloc" in r.stdout, r.stdout
