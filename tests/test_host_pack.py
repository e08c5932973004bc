"""CPU test of the host pack of dlsim_host_wreduce (csrc/host_pack.hpp):
compiled with g++ and run on random tensor sets, chunk sizes and thread
counts, both copy modes; staging bytes must equal the concatenation."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "decentralized-learning-simulator_amd", "csrc")
SRC = os.path.join(ROOT, "tests", "native", "host_pack_check.cpp")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pack") / "host_pack_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-I", CSRC, SRC, "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("mode", ["stream", "memcpy"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pack_matches_concatenation(checker, mode, seed):
    env = dict(os.environ, DLSIM_PACK_COPY=mode)
    r = subprocess.run([checker, str(seed)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr
