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
    env = dict(os.environ, DLSIM_AB="1", DLSIM_PACK_COPY=mode)
    r = subprocess.run([checker, str(seed)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_host_pack_entry_point(threads):
    """dlsim_host_pack through the library (no GPU call): tensors of mixed
    dtypes and sizes at their byte offsets, bytes equal to a plain copy."""
    import torch
    from dasklearn_amd import _native
    g = torch.Generator().manual_seed(threads)
    srcs, offs, off = [], [], 0
    for i in range(60):
        n = int(torch.randint(0, 200_000 if i % 7 == 0 else 3000, (1,), generator=g))
        dt = (torch.float32, torch.bfloat16, torch.float16)[i % 3]
        t = torch.randn(n + 1, generator=g).to(dt)[1:]  # unaligned source
        srcs.append(t)
        offs.append(off)
        off += t.numel() * t.element_size() + (i % 5) * 4
    dst = torch.zeros(off + 16, dtype=torch.uint8)
    _native.host_pack(srcs, offs, dst, threads=threads)
    for t, o in zip(srcs, offs):
        b = t.numel() * t.element_size()
        assert torch.equal(dst[o:o + b], t.contiguous().view(torch.uint8)), o
    with pytest.raises(ValueError):
        _native.host_pack(srcs[:1], [off + 100], dst)
